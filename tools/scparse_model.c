// CPU model of the round-3 fast compressor's parse (design tool, not product code): compressed
// size of <= 64 KiB blocks when every position gets the exact latest earlier position with the
// same hash as its one candidate (every position inserted in order), and the block is cut into
// S-byte super-chunks, each parsed by the exact greedy walk (copies capped at LCAP bytes and at
// the super-chunk end; literal runs restart at super-chunk starts).
// Build: gcc -O2 -o /tmp/scm tools/scparse_model.c
// Run:   /tmp/scm S hashbits lcap file...   (each file is cut into 64 KiB blocks; prints sizes)
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint32_t ld32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
static uint32_t lit_bytes(uint32_t n) { return n == 0 ? 0 : n + (n <= 60 ? 1 : n <= 256 ? 2 : 3); }
static uint32_t copy_bytes(uint32_t off, uint32_t len) {
  uint32_t b = 0;
  while (len >= 68) { b += 3; len -= 64; }
  if (len > 64) { b += 3; len -= 60; }
  return b + ((len < 12 && off < 2048) ? 2 : 3);
}
static int REFH = 0, DEPTH = 1, PREF8 = 0, TIE2 = 0, PAR = 0, ROW = 0;
static uint32_t hsh(uint32_t w, int bits) {
  if (REFH) return (w * 0x1e35a7bdu) >> (32 - bits);
  return ((((w ^ (w >> 12)) & 0xffffff) * 0x1e35a7u) >> 10) & ((1u << bits) - 1); }
static uint32_t vlen(uint32_t v) { return v < 128 ? 1 : v < 16384 ? 2 : v < (1u << 21) ? 3 : 4; }

static uint64_t block_size(const uint8_t* d, uint32_t n, uint32_t S, int tb, uint32_t lcap, int header) {
  static uint32_t T[1 << 16], prev[65536], prev2[65536], T2[1<<16];
  memset(T, 0, sizeof(uint32_t) << tb); memset(T2, 0, sizeof(uint32_t) << tb);
  for (uint32_t qi = 0; qi < n; ++qi) {
    uint32_t q = qi;
    if (ROW) {  // super-chunk by super-chunk; inside one: position-in-row j, then row (lane) order
      const uint32_t sc = qi / S * S, r = qi - sc, j = r / (S / 16), lane = r % (S / 16);
      q = sc + 16 * lane + j;
    }
    if (q + 4 > n) { prev[q] = prev2[q] = 0; continue; }
    uint32_t h = hsh(ld32(d + q), tb);
    if (PAR) {  // two tables by parity class: exchange own class, read the other
      uint32_t cls = PAR == 1 ? (q & 1) : ((q >> 6) & 1);  // (ROW: q & 1 is the instruction parity)
      uint32_t* Ta = cls ? T2 : T;
      uint32_t* Tb = cls ? T : T2;
      uint32_t a = Ta[h], bb = Tb[h];
      if (PAR == 2 && bb && bb - 1 >= (q & ~63u)) bb = 0;  // (not possible for group classes)
      prev[q] = a > bb ? a : bb;
      prev2[q] = a > bb ? bb : a;
      Ta[h] = q + 1;
      continue;
    }
    prev[q] = T[h];
    prev2[q] = T2[h];
    T2[h] = T[h];
    T[h] = q + 1;
  }
  uint64_t out = header ? vlen(n) : 0;
  for (uint32_t s0 = 0; s0 < n; s0 += S) {
    uint32_t s1 = s0 + S < n ? s0 + S : n, p = s0, ls = s0;
    while (p < s1) {
      uint32_t L = 0, cbest = 0;
      for (int k = 0; k < DEPTH; ++k) {
        uint32_t pv = k ? prev2[p] : prev[p];
        if (p + 4 <= s1 && pv) {
          if (pv - 1 >= p) continue;  // (ROW order: a later position can be in the table)
          uint32_t c = pv - 1, lim = s1 - p < lcap ? s1 - p : lcap, l = 0;
          uint32_t lim8 = PREF8 && lim > (uint32_t)PREF8 ? (uint32_t)PREF8 : lim;
          while (l < lim8 && d[c + l] == d[p + l]) ++l;
          if (l > L || (TIE2 && l == L && l > 0)) { L = l; cbest = pv; }
        }
      }
      if (PREF8 && L == (uint32_t)PREF8) {  // extend the chosen candidate only
        uint32_t c = cbest - 1, lim = s1 - p < lcap ? s1 - p : lcap;
        while (L < lim && d[c + L] == d[p + L]) ++L;
      }
      if (L >= 4) {
        out += lit_bytes(p - ls) + copy_bytes(p - (cbest - 1), L);
        p += L;
        ls = p;
      } else {
        ++p;
      }
    }
    out += lit_bytes(s1 - ls);
  }
  return out;
}

int main(int argc, char** argv) {
  if (argc < 5) return 1;
  uint32_t S = atoi(argv[1]), lcap = atoi(argv[3]);
  int tb = atoi(argv[2]);
  if (getenv("REFH")) REFH = 1;
  if (getenv("TIE2")) TIE2 = 1;
  if (getenv("ROW")) ROW = 1;
  if (getenv("PAR")) PAR = atoi(getenv("PAR"));
  if (getenv("DEPTH")) DEPTH = atoi(getenv("DEPTH"));
  if (getenv("PREF8")) PREF8 = atoi(getenv("PREF8"));
  uint64_t tin = 0, tout = 0;
  for (int f = 4; f < argc; ++f) {
    FILE* fp = fopen(argv[f], "rb");
    if (!fp) return 2;
    fseek(fp, 0, SEEK_END);
    long sz = ftell(fp);
    fseek(fp, 0, SEEK_SET);
    uint8_t* d = malloc(sz + 16);
    if (fread(d, 1, sz, fp) != (size_t)sz) return 3;
    fclose(fp);
    uint64_t out = vlen((uint32_t)sz);
    for (long o = 0; o < sz; o += 65536) {
      uint32_t n = sz - o < 65536 ? (uint32_t)(sz - o) : 65536;
      out += block_size(d + o, n, S, tb, lcap, 0);
    }
    printf("%s %ld %lu\n", argv[f], sz, (unsigned long)out);
    tin += sz;
    tout += out;
    free(d);
  }
  printf("TOTAL %lu %lu %.4f\n", (unsigned long)tin, (unsigned long)tout, (double)tout / tin);
  return 0;
}
