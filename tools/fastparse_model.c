// CPU model of the fast-mode parse (design tool, not product code): estimates the
// compressed size of the chunked, round-based parse of sm_compress_fast.hip for different
// chunk sizes, table sizes and candidate policies, on 64 KiB blocks of a file.
// Build: gcc -O2 -o /tmp/fpm tools/fastparse_model.c ; run: /tmp/fpm file...
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint32_t ld32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }

static uint32_t lit_bytes(uint32_t n) { return n == 0 ? 0 : n + (n <= 60 ? 1 : n <= 256 ? 2 : 3); }
static uint32_t copy_bytes(uint32_t off, uint32_t len) {
  if (len < 12) return off < 2048 ? 2 : 3;
  uint32_t b = 0;
  while (len >= 68) { b += 3; len -= 64; }
  if (len > 64) { b += 3; len -= 60; }
  return b + ((len < 12 && off < 2048) ? 2 : 3);
}

// policy: 0 = first-chance only (prior rounds), 1 = second chance else first, 2 = best of both,
//         3 = exact latest-earlier (ideal table)
static int g_nbr = 0, g_first = 0, g_skip = 0, g_nonempty = 0, g_pbits = 8, g_intrap = 0;  // probe the private tables of g_nbr previous chunks

static uint64_t model_block(const uint8_t* d, uint32_t n, uint32_t chunk, uint32_t waves, uint32_t tab,
                            int policy, int exact_intrachunk) {
  uint32_t* T = calloc(tab, 4);
  uint32_t* Tprev = calloc(tab, 4);
  uint32_t* cand1 = malloc(sizeof(uint32_t) * (n + 1));
  uint32_t* cand2 = malloc(sizeof(uint32_t) * (n + 1));
  uint64_t out = 3;
  uint32_t nch = (n + chunk - 1) / chunk, rounds = (nch + waves - 1) / waves;
  for (uint32_t r = 0; r < rounds; ++r) {
    uint32_t r0 = r * waves * chunk, r1 = r0 + waves * chunk; if (r1 > n) r1 = n;
    memcpy(Tprev, T, tab * 4);
    // exact sequential inserts for policy 3 / intra-chunk
    for (uint32_t q = r0; q < r1; ++q) {
      if (q + 4 > n) { cand1[q] = cand2[q] = 0; continue; }
      uint32_t h = (uint32_t)(((uint64_t)(ld32(d + q) * 0x1e35a7bdu) * tab) >> 32);
      cand1[q] = Tprev[h];
      uint32_t cq = T[h];  // latest earlier (sequential) -- used by policy 3 and intra-chunk
      cand2[q] = cq;
      T[h] = q + 1;
    }
    // private tables (8-bit hash) of the round's chunks: max position per bucket
    uint32_t P[64][256];
    for (uint32_t k = r * waves; k < (r + 1) * waves && k < nch; ++k) {
      uint32_t c0 = k * chunk, ce = c0 + chunk < n ? c0 + chunk : n;
      memset(P[k - r * waves], 0, sizeof(P[0]));
      for (uint32_t q = c0; q + 4 <= n && q < ce; ++q) P[k - r * waves][(ld32(d + q) * 0x1e35a7bdu) >> (32 - g_pbits)] = q + 1;
    }
    // second-chance table = max after round (T now)
    for (uint32_t k = r * waves; k < (r + 1) * waves && k < nch; ++k) {
      uint32_t c0 = k * chunk, ce = c0 + chunk < n ? c0 + chunk : n;
      uint32_t p = c0, ls = c0;
      while (p < ce) {
        uint32_t best = 0, bc = 0;
        if (p + 4 <= ce) {
          uint32_t cands[3]; int nc = 0;
          uint32_t h = (uint32_t)(((uint64_t)(ld32(d + p) * 0x1e35a7bdu) * tab) >> 32);
          uint32_t sc = T[h];
          uint32_t exact = cand2[p];
          if (policy == 3) cands[nc++] = exact;
          else {
            if (policy >= 1 && sc && sc - 1 < p) cands[nc++] = sc;
            if (policy == 0 || policy == 2 || nc == 0) cands[nc++] = cand1[p];
            if (g_intrap) {  // the kernel's A: latest earlier chunk position with the same private hash
              uint32_t best_q = 0, hp = (ld32(d + p) * 0x1e35a7bdu) >> (32 - g_pbits);
              for (uint32_t q = c0; q < p; ++q)
                if (q + 4 <= n && ((ld32(d + q) * 0x1e35a7bdu) >> (32 - g_pbits)) == hp) best_q = q + 1;
              if (best_q) cands[nc++] = best_q;
            } else if (exact_intrachunk && exact && exact - 1 >= c0) cands[nc++] = exact;
          }
          uint32_t nb[64]; int nn = 0, have = 0;
          for (int i = 0; i < nc; ++i)
            if (cands[i] && cands[i] - 1 < p && ld32(d + cands[i] - 1) == ld32(d + p)) have = 1;
          for (int m = 1; m <= g_nbr && !(g_skip && have) && (int)(k - r * waves) - m >= 0; ++m) {
            uint32_t v = P[k - r * waves - m][(ld32(d + p) * 0x1e35a7bdu) >> (32 - g_pbits)];
            if (g_nonempty) {  // take the nearest non-empty entry, verified or not
              if (!v) continue;
              nb[nn++] = v;
              break;
            }
            if (g_first && !(v && v - 1 < p && ld32(d + v - 1) == ld32(d + p))) continue;
            nb[nn++] = v;
            if (g_first) break;
          }
          for (int i = 0; i < nc + nn; ++i) {
            uint32_t cv = i < nc ? cands[i] : nb[i - nc];
            if (!cv) continue;
            uint32_t c = cv - 1;
            if (c >= p) continue;
            uint32_t L = 0;
            while (p + L < ce && d[c + L] == d[p + L]) ++L;
            if (L >= 4 && L > best) { best = L; bc = c; }
          }
        }
        if (best) {
          out += lit_bytes(p - ls) + copy_bytes(p - bc, best);
          p += best; ls = p;
        } else ++p;
      }
      out += lit_bytes(ce - ls);
    }
  }
  free(T); free(Tprev); free(cand1); free(cand2);
  return out;
}

int main(int argc, char** argv) {
  size_t total = 0, cap = 1 << 24;
  uint8_t* buf = malloc(cap);
  for (int i = 1; i < argc; ++i) {
    FILE* f = fopen(argv[i], "rb");
    total += fread(buf + total, 1, cap - total, f);
    fclose(f);
  }
  if (getenv("NBR")) g_nbr = atoi(getenv("NBR"));  // e.g. NBR=4 FIRST=1 (nearest verified only)
  if (getenv("FIRST")) g_first = 1;
  if (getenv("SKIP")) g_skip = 1;                   // probe only positions without a verified A/B
  if (getenv("NONEMPTY")) g_nonempty = 1;           // nearest non-empty neighbour entry only
  if (getenv("PBITS")) g_pbits = atoi(getenv("PBITS"));  // private (per-chunk) table hash bits
  if (getenv("INTRAP")) g_intrap = 1;               // intra-chunk candidate from the private table
  struct { uint32_t chunk, waves, tab; int pol, intra; } cfg[] = {
      {256, 4, 16384, 2, 1}, {256, 8, 16384, 2, 1}, {128, 8, 16384, 2, 1}, {256, 8, 16384, 1, 1},
      {256, 4, 12288, 2, 1}, {256, 8, 12288, 2, 1}, {256, 4, 8192, 2, 1}, {256, 8, 8192, 2, 1},
      {512, 8, 16384, 2, 1}, {256, 16, 16384, 2, 1}, {256, 8, 16384, 0, 1},
      {128, 16, 16384, 2, 1}, {64, 16, 16384, 2, 1}, {64, 32, 16384, 2, 1}, {128, 8, 16384, 3, 1},
      {128, 16, 16384, 0, 1}, {128, 16, 16384, 1, 1}, {128, 16, 16384, 0, 0}, {128, 16, 16384, 2, 0},
  };
  for (size_t c = 0; c < sizeof(cfg) / sizeof(cfg[0]); ++c) {
    uint64_t out = 0, in = 0;
    for (size_t o = 0; o + 65536 <= total; o += 65536) {
      out += model_block(buf + o, 65536, cfg[c].chunk, cfg[c].waves, cfg[c].tab, cfg[c].pol, cfg[c].intra);
      in += 65536;
    }
    printf("chunk %5u waves %u tab %5u policy %d intra %d : ratio %.4f\n", cfg[c].chunk, cfg[c].waves, cfg[c].tab,
           cfg[c].pol, cfg[c].intra, (double)out / in);
  }
  return 0;
}
