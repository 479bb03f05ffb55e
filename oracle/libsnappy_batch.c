/*
 * libsnappy_batch.c -- CPU BASELINE HELPER (test/bench infrastructure only, never shipped).
 *
 * Times Google's libsnappy (the C library the reference's own benchmark ccalls,
 * test/libsnappy.jl:5-30 and test/benchmarks.jl) on a batch of independent blocks, OpenMP over
 * blocks.  The library is dlopen'ed at run time (/opt/conda/lib/libsnappy.so.1, snappy 1.1.8 in
 * this image), so nothing links against it and the bench still runs where it is absent.
 * Only bench.py's cpu_baseline leg calls this.
 */
#include <dlfcn.h>
#include <stddef.h>
#include <stdint.h>

typedef int (*snappy_fn)(const char*, size_t, char*, size_t*);

static snappy_fn g_compress, g_uncompress;

/* 0 on success, -1 if the library or its symbols are missing */
int lsb_open(const char* path) {
  void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!h) return -1;
  g_compress = (snappy_fn)dlsym(h, "snappy_compress");
  g_uncompress = (snappy_fn)dlsym(h, "snappy_uncompress");
  return (g_compress && g_uncompress) ? 0 : -1;
}

/* block b: in[in_off[b] .. +in_len[b]) -> out + out_off[b] (capacity out_cap[b]); out_len[b] =
 * bytes written.  Returns the number of blocks whose call failed. */
static int run(snappy_fn f, const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint32_t nblk,
               uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap, uint32_t* out_len, int nthreads) {
  int bad = 0;
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads) reduction(+ : bad)
  for (uint32_t b = 0; b < nblk; ++b) {
    size_t ol = out_cap[b];
    if (f((const char*)in + in_off[b], in_len[b], (char*)out + out_off[b], &ol) != 0) {
      ++bad;
      ol = 0;
    }
    out_len[b] = (uint32_t)ol;
  }
  return bad;
}

int lsb_compress_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint32_t nblk, uint8_t* out,
                       const uint64_t* out_off, const uint32_t* out_cap, uint32_t* out_len, int nthreads) {
  if (!g_compress) return -1;
  return run(g_compress, in, in_off, in_len, nblk, out, out_off, out_cap, out_len, nthreads);
}

int lsb_uncompress_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint32_t nblk,
                         uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap, uint32_t* out_len,
                         int nthreads) {
  if (!g_uncompress) return -1;
  return run(g_uncompress, in, in_off, in_len, nblk, out, out_off, out_cap, out_len, nthreads);
}
