/* Single-buffer C API timing (design tool, GPU box): sm_compress / sm_uncompress of one
 * stream of MiB megabytes from host buffers, the way a Julia caller drives the drop-in.
 *   gcc -O2 -I include -o /tmp/c_single tools/c_single.c -L snappy.jl_amd -lsnappy_mi355x \
 *       -Wl,-rpath,$PWD/snappy.jl_amd && /tmp/c_single tests/golden/testdata/alice29.txt 64
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "snappy_mi355x.h"

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  static char corpus[1 << 21];
  size_t clen = fread(corpus, 1, sizeof(corpus), f);
  fclose(f);
  size_t n = (size_t)atoi(argv[2]) << 20;
  char* in = malloc(n);
  for (size_t i = 0; i < n; i += clen) memcpy(in + i, corpus, i + clen <= n ? clen : n - i);
  size_t cap = sm_max_compressed_length(n);
  char* comp = malloc(cap);
  char* back = malloc(n);
  sm_ctx* ctx = sm_ctx_create(0);
  for (int mode = 1; mode >= 0; --mode) {
    size_t cl = cap, bl = n;
    sm_compress(ctx, in, n, comp, &cl, mode); /* warm */
    double t0 = now();
    cl = cap;
    int st = sm_compress(ctx, in, n, comp, &cl, mode);
    double t1 = now();
    sm_uncompress(ctx, comp, cl, back, &bl);
    double t2 = now();
    bl = n;
    int st2 = sm_uncompress(ctx, comp, cl, back, &bl);
    double t3 = now();
    printf("%s: %zu MiB ratio %.3f  compress %.2f GB/s (st %d)  uncompress %.2f GB/s (st %d, path %d)  ok %d\n",
           mode ? "fast" : "reference", n >> 20, (double)cl / n, n / (t1 - t0) / 1e9, st, n / (t3 - t2) / 1e9, st2,
           sm_ctx_last_path(ctx), bl == n && memcmp(in, back, n) == 0);
  }
  sm_ctx_destroy(ctx);
  return 0;
}
