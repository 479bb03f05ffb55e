/*
 * asan_driver.c -- runs the oracle (snappy_oracle.c) under AddressSanitizer + UBSan
 * (TEST INFRASTRUCTURE ONLY; built by `make asan_driver`, run by tests/test_oracle_asan.py).
 *
 * For every file on the command line: reference- and compat-mode compress into a buffer of
 * exactly smo_max_compressed_length(n) bytes, the round trip into a buffer of exactly n bytes,
 * then a seeded mutation fuzz of the compressed stream (byte flips, truncations, extensions;
 * the reference's corrupted-input cases, test/runtests.jl:62-122, are of these kinds) decoded
 * into a heap buffer of exactly the declared length, and the raw file itself fed to the decoder
 * as if it were compressed.  Every buffer is a separate malloc, so any read or write the
 * restated decoder makes outside its input or output is a sanitizer abort.
 * Exit 0: all round trips exact and no sanitizer report.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "snappy_oracle.h"

static uint64_t rng_state = 0x5EEDull;
static uint64_t rnd(void) {  // splitmix64
  uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* decode `c` (exactly n bytes of its own allocation) into an exact-size output; returns status */
static int decode_exact(const uint8_t* c, size_t n) {
  uint8_t* in = (uint8_t*)malloc(n ? n : 1);
  memcpy(in, c, n);
  size_t want = 0;
  int st = smo_uncompressed_length(in, n, &want);
  if (st == SMO_OK && want <= (64u << 20)) {
    uint8_t* out = (uint8_t*)malloc(want ? want : 1);
    size_t got = 0;
    st = smo_uncompress(in, n, out, want, &got);
    free(out);
  }
  free(in);
  return st;
}

int main(int argc, char** argv) {
  int fuzz = 300, a0 = 1;
  long fails = 0, rejected = 0, decoded = 0;
  if (argc > 2 && strcmp(argv[1], "-n") == 0) {  // mutations per file and mode
    fuzz = atoi(argv[2]);
    a0 = 3;
  }
  for (int a = a0; a < argc; ++a) {
    FILE* f = fopen(argv[a], "rb");
    if (!f) {
      fprintf(stderr, "cannot open %s\n", argv[a]);
      return 2;
    }
    fseek(f, 0, SEEK_END);
    size_t n = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t* raw = (uint8_t*)malloc(n ? n : 1);
    if (fread(raw, 1, n, f) != n) return 2;
    fclose(f);
    (void)(decode_exact(raw, n) == SMO_OK ? ++decoded : ++rejected);  // the file as a stream
    for (int compat = 0; compat < 2; ++compat) {
      size_t cap = smo_max_compressed_length(n), cl = 0;
      uint8_t* comp = (uint8_t*)malloc(cap);
      if (smo_compress(raw, n, comp, &cl, compat) != SMO_OK) ++fails;
      uint8_t* back = (uint8_t*)malloc(n ? n : 1);
      size_t bl = 0;
      if (smo_uncompress(comp, cl, back, n, &bl) != SMO_OK || bl != n || memcmp(back, raw, n) != 0) ++fails;
      free(back);
      for (int k = 0; k < fuzz && cl > 0; ++k) {
        size_t m = cl + 8;
        uint8_t* mut = (uint8_t*)malloc(m);
        memcpy(mut, comp, cl);
        size_t ml = cl;
        switch (rnd() % 3) {
          case 0:  // flip 1..4 bytes
            for (int j = 1 + (int)(rnd() % 4); j > 0; --j) mut[rnd() % cl] ^= (uint8_t)(1 + rnd() % 255);
            break;
          case 1:  // truncate
            ml = (size_t)(rnd() % cl);
            break;
          default:  // extend by 1..8 bytes
            ml = cl + 1 + (size_t)(rnd() % 8);
            for (size_t j = cl; j < ml; ++j) mut[j] = (uint8_t)rnd();
        }
        (void)(decode_exact(mut, ml) == SMO_OK ? ++decoded : ++rejected);
        free(mut);
      }
      free(comp);
    }
    free(raw);
  }
  printf("asan_driver: %d files, %ld mutated/foreign streams decoded, %ld rejected, %ld round-trip failures\n",
         argc - a0, decoded, rejected, fails);
  return fails ? 1 : 0;
}
