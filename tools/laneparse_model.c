// CPU model of lane-serial parses (design tool, not product code): compressed size of a 64 KiB
// block when the block is cut into C-byte chunks, each parsed greedily by one lane, with
// candidates from
//   mode 0 "exact":    the exact latest earlier position with the same hash (every position
//                      inserted in order: the inserter wave of sm_compress_fast.hip);
//   mode 1 "snapshot": the latest position before the lane's ROUND (K chunks parsed together;
//                      the table is merged with ds_max after each round, so it is exact up to
//                      the round start), plus the lane's own chunk history (exact, private);
//   mode 2 "snapshot + left": mode 1 plus the previous chunk's positions at the same or
//                      smaller in-chunk offset (lockstep lanes: what lane i-1 has inserted).
// Copies are capped at LCAP bytes and end at the chunk end; literal runs merge across chunks.
// Build: gcc -O2 -o /tmp/lpm tools/laneparse_model.c ; run: /tmp/lpm blocks.bin [nblocks]
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint32_t ld32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
static uint32_t lit_bytes(uint32_t n) { return n == 0 ? 0 : n + (n <= 60 ? 1 : n <= 256 ? 2 : 3); }
static uint32_t copy_bytes(uint32_t off, uint32_t len) { return (len < 12 && off < 2048) ? 2 : 3; }  // len <= 64
static uint32_t hsh(uint32_t w, int bits) { return ((((w ^ (w >> 12)) & 0xffffff) * 0x1e35a7u) >> 10) & ((1u << bits) - 1); }

static int LCAP = 64;
static uint32_t ISTR = 1, PSTR = 1, OFFMAX = 65535, NOMERGE = 0;

static uint64_t model(const uint8_t* d, uint32_t n, int mode, uint32_t C, uint32_t K, int tb) {
  const uint32_t tab = 1u << tb;
  uint32_t* T = calloc(tab, 4);      // snapshot (or exact, mode 0)
  uint32_t* prev = malloc(4 * n);    // exact prev (mode 0) / in-chunk prev (modes 1,2)
  uint32_t* H = malloc(4 * n);
  for (uint32_t q = 0; q < n; ++q) H[q] = q + 4 <= n ? hsh(ld32(d + q), tb) : 0xffffffffu;
  if (mode == 0)
    for (uint32_t q = 0; q + 4 <= n; ++q) { prev[q] = T[H[q]]; if (q % ISTR == 0) T[H[q]] = q + 1; }
  uint64_t out = 0;
  uint32_t ls = 0;  // literal run start (block-wide: runs merge across chunks)
  uint32_t nch = (n + C - 1) / C;
  uint32_t* P = calloc(tab, 4);
  for (uint32_t k0 = 0; k0 < nch; k0 += K) {
    for (uint32_t k = k0; k < k0 + K && k < nch; ++k) {
      uint32_t c0 = k * C, ce = c0 + C < n ? c0 + C : n;
      if (mode) {  // own-chunk exact history
        for (uint32_t q = c0; q < ce; ++q) {
          if (H[q] == 0xffffffffu) { prev[q] = 0; continue; }
          prev[q] = P[H[q]] > c0 ? P[H[q]] : 0;
          P[H[q]] = q + 1;
        }
      }
      uint32_t p = c0;
      if (NOMERGE) { out += lit_bytes(c0 - ls); ls = c0; }
      while (p < ce) {
        uint32_t best = 0, bc = 0;
        if (p + 4 <= ce && p % PSTR == 0) {
          uint32_t cands[4];
          int nc = 0;
          cands[nc++] = prev[p];
          if (mode) cands[nc++] = T[H[p]];
          if (mode == 2 && k > k0) {  // previous chunk, positions at in-chunk offset <= mine
            uint32_t best_q = 0;
            for (uint32_t q = c0 - C; q <= p - C; ++q)
              if (H[q] == H[p]) best_q = q + 1;
            cands[nc++] = best_q;
          }
          for (int i = 0; i < nc; ++i) {
            if (!cands[i]) continue;
            uint32_t c = cands[i] - 1;
            if (c >= p || p - c > OFFMAX) continue;
            uint32_t L = 0, lim = ce - p < (uint32_t)LCAP ? ce - p : (uint32_t)LCAP;
            while (L < lim && d[c + L] == d[p + L]) ++L;
            if (L >= 4 && (L > best || (L == best && c > bc))) { best = L; bc = c; }
          }
        }
        if (best) {
          out += lit_bytes(p - ls) + copy_bytes(p - bc, best);
          p += best;
          ls = p;
        } else
          ++p;
      }
    }
    if (mode)  // merge the round into the snapshot (ds_max: the latest position per bucket)
      for (uint32_t q = k0 * C; q < (k0 + K) * C && q < n; ++q)
        if (H[q] != 0xffffffffu && T[H[q]] < q + 1) T[H[q]] = q + 1;
  }
  out += lit_bytes(n - ls) + 3;
  free(T); free(prev); free(H); free(P);
  return out;
}

int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "rb");
  size_t nb = argc > 2 ? (size_t)atoi(argv[2]) : 100;
  uint8_t* buf = malloc(nb * 65536);
  nb = fread(buf, 65536, nb, f);
  fclose(f);
  if (getenv("LCAP")) LCAP = atoi(getenv("LCAP"));
  if (getenv("NOMERGE")) NOMERGE = 1;
  if (getenv("OFFMAX")) OFFMAX = atoi(getenv("OFFMAX"));
  if (getenv("ISTR")) ISTR = atoi(getenv("ISTR"));
  if (getenv("PSTR")) PSTR = atoi(getenv("PSTR"));
  int only0 = getenv("ONLY0") != 0;
  struct { int mode; uint32_t C, K; int tb; } cfg[] = {
      {0, 256, 1, 13}, {0, 128, 1, 13}, {0, 64, 1, 13}, {0, 256, 1, 14}, {0, 128, 1, 14}, {0, 64, 1, 14}, {0, 1 << 16, 1, 13}, {0, 1 << 16, 1, 14},
      {1, 256, 64, 13}, {1, 256, 16, 13}, {1, 128, 64, 13}, {1, 128, 32, 13}, {1, 128, 16, 13}, {1, 64, 64, 13},
      {1, 64, 32, 13}, {1, 64, 16, 13}, {1, 32, 64, 13}, {1, 64, 64, 14}, {1, 128, 32, 14},
      {2, 128, 32, 13}, {2, 64, 64, 13}, {2, 256, 64, 13},
  };
  for (size_t c = 0; c < sizeof(cfg) / sizeof(cfg[0]); ++c) {
    if (only0 && cfg[c].mode) continue;
    uint64_t out = 0;
    for (size_t b = 0; b < nb; ++b) out += model(buf + 65536 * b, 65536, cfg[c].mode, cfg[c].C, cfg[c].K, cfg[c].tb);
    printf("mode %d chunk %5u lanes/round %3u tab 2^%d : ratio %.4f\n", cfg[c].mode, cfg[c].C, cfg[c].K, cfg[c].tb,
           (double)out / (nb * 65536.0));
    fflush(stdout);
  }
  return 0;
}
