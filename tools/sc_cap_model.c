// CPU model of the fast compressor's walks with a cap on resynchronisation walks (design tool, not
// product code).  Candidates as the kernel picks them (two slots by group parity; the more recent
// 4-byte match unless it is nearer than FAR = 256 bytes and the older matches), rows of 16
// positions per lane, 1 KiB super-chunks, the first walk from every row start, resynchronisation
// rounds whose rewalks stop after KCAP length computations (KCAP=0: no cap, the kernel): a lane
// that has not met its old path by then keeps its old tokens from that position on (the bytes
// between become literals).  Prints the SIMT iterations of both phases and the stream size
// against the uncapped parse.
// Build: gcc -O2 -w -o /tmp/cm tools/sc_cap_model.c    Run: KCAP=2 /tmp/cm file...
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static uint32_t ld32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
static uint32_t cand[65536];
static uint8_t match[65536];
static uint32_t Lp[65536];  // recorded length code per visited position
static int KCAP;
static long n_sc, it1, rsit, rsr;
static uint64_t out_bytes;
static uint32_t lit_bytes(uint32_t n) { return n == 0 ? 0 : n + (n <= 60 ? 1 : (n <= 256 ? 2 : 3)); }
static uint32_t copy_bytes(uint32_t off, uint32_t L) {
  uint32_t k = L >= 68 ? (L - 4) >> 6 : 0, R0 = L - 64 * k, x = R0 > 64, R = R0 - 60 * x;
  return 3 * (k + x) + ((R < 12 && off < 2048) ? 2 : 3);
}
static const uint8_t* B;
static uint32_t sce_g;
static uint32_t enc_at(uint32_t q) {
  uint32_t c = cand[q], l = 0;
  while (l < 16 && B[c + l] == B[q + l]) ++l;
  uint32_t av = sce_g - q;
  uint32_t e = (l == 16 && av > 16) ? 17 : (l < av ? l : av);
  Lp[q] = e;
  return e;
}
static uint32_t full_len(uint32_t q) {  // the token's length (extended when 17)
  uint32_t L = Lp[q];
  if (L == 17) {
    uint32_t c = cand[q];
    L = 16;
    uint32_t cap = sce_g - q < 255 ? sce_g - q : 255;
    while (L < cap && B[c + L] == B[q + L]) ++L;
  }
  return L;
}
int main(int argc, char** argv) {
  if (getenv("KCAP")) KCAP = atoi(getenv("KCAP"));
  for (int f = 1; f < argc; ++f) {
    FILE* fp = fopen(argv[f], "rb");
    fseek(fp, 0, SEEK_END);
    long sz = ftell(fp);
    fseek(fp, 0, SEEK_SET);
    uint8_t* d = calloc(sz + 64, 1);
    if (fread(d, 1, sz, fp) != (size_t)sz) return 2;
    fclose(fp);
    for (long o = 0; o < sz; o += 65536) {
      uint32_t n = sz - o < 65536 ? sz - o : 65536;
      const uint8_t* b = d + o;
      B = b;
      static uint32_t T[8192];
      memset(T, 0, sizeof T);
      for (uint32_t q = 0; q < n; ++q) {
        match[q] = 0;
        if (q + 4 > n) continue;
        const uint32_t w = ld32(b + q), h = (w * 0x1e35a7bdu) >> 19, par = (q >> 6) & 1;
        const uint32_t own = par ? T[h] >> 16 : T[h] & 0xffff, oth = par ? T[h] & 0xffff : T[h] >> 16;
        T[h] = par ? (T[h] & 0xffff) | ((q + 1) << 16) : (T[h] & 0xffff0000u) | (q + 1);
        const uint32_t c1 = own > oth ? own : oth, c2 = own > oth ? oth : own;
        const uint32_t sce = (q / 1024 + 1) * 1024 < n ? (q / 1024 + 1) * 1024 : n;
        if (q + 4 > sce) continue;
        const int m1 = c1 && c1 - 1 < q && ld32(b + c1 - 1) == w, m2 = c2 && c2 - 1 < q && ld32(b + c2 - 1) == w;
        if (!m1 && !m2) continue;
        match[q] = 1;
        cand[q] = (m2 && (!m1 || q - (c1 - 1) < 256)) ? c2 - 1 : c1 - 1;
      }
      for (uint32_t sc0 = 0; sc0 < n; sc0 += 1024) {
        const uint32_t sce = sc0 + 1024 < n ? sc0 + 1024 : n;
        sce_g = sce;
        n_sc++;
        uint32_t mask[64], S[64], E[64], P[64];
        for (int l = 0; l < 64; ++l) {
          uint32_t c0 = sc0 + 16 * l;
          mask[l] = 0;
          for (int i = 0; i < 16; ++i)
            if (c0 + i < sce && match[c0 + i]) mask[l] |= 1u << i;
        }
        // one walk: from row position sr, stop on `stop` bits (merge) or after cap lengths
        // returns steps; sets path, mpos (merge or cut position, 16 none), cut flag
        auto int walk(int l, uint32_t sr, uint32_t stop, int cap, uint32_t* path, uint32_t* mpos, int* cut);
        int walk(int l, uint32_t sr, uint32_t stop, int cap, uint32_t* path, uint32_t* mpos, int* cut) {
          const uint32_t c0 = sc0 + 16 * l;
          const uint32_t m0 = sr < 16 ? mask[l] >> sr : 0;
          uint32_t i = m0 ? sr + __builtin_ctz(m0) : 16;
          *path = 0;
          *mpos = 16;
          *cut = 0;
          int steps = 0;
          while (i < 16) {
            if ((stop >> i) & 1) {
              *mpos = i;
              break;
            }
            if (cap && steps == cap) {
              *mpos = i;
              *cut = 1;
              break;
            }
            *path |= 1u << i;
            const uint32_t e = enc_at(c0 + i);
            steps++;
            const uint32_t t = i + (e < 16 ? e : 16);
            const uint32_t m = mask[l] >> t;
            i = m ? t + __builtin_ctz(m) : 16;
          }
          return steps;
        }
        auto uint32_t lane_end(int l, uint32_t Pl);
        uint32_t lane_end(int l, uint32_t Pl) {  // the last token's end if it leaves the row, else the row end
          const uint32_t c0 = sc0 + 16 * l, ce = c0 < sce ? (c0 + 16 < sce ? c0 + 16 : sce) : c0;
          if (!Pl) return ce;
          const uint32_t last = 31 - __builtin_clz(Pl);
          const uint32_t L = full_len(c0 + last);
          return c0 + last + L > ce ? c0 + last + L : ce;
        }
        int mx = 0;
        for (int l = 0; l < 64; ++l) {
          const uint32_t c0 = sc0 + 16 * l;
          S[l] = c0;
          if (c0 < sce) {
            uint32_t mp;
            int ct;
            int st = walk(l, 0, 0, 0, &P[l], &mp, &ct);
            if (st > mx) mx = st;
            E[l] = lane_end(l, P[l]);
          } else {
            P[l] = 0;
            E[l] = c0;
          }
        }
        it1 += mx;
        for (;;) {
          uint32_t sn[64];
          int chg = 0;
          for (int l = 0; l < 64; ++l) {
            sn[l] = l ? E[l - 1] : sc0;
            chg += sn[l] != S[l];
          }
          if (!chg) break;
          rsr++;
          int mxs = 0;
          uint32_t NE[64];
          for (int l = 0; l < 64; ++l) {
            NE[l] = E[l];
            if (sn[l] == S[l]) continue;
            const uint32_t c0 = sc0 + 16 * l, ce = c0 < sce ? (c0 + 16 < sce ? c0 + 16 : sce) : c0;
            S[l] = sn[l];
            if (sn[l] >= ce) {
              P[l] = 0;
              NE[l] = sn[l];
              continue;
            }
            uint32_t nP, mp;
            int ct;
            const int st = walk(l, sn[l] - c0, P[l], KCAP, &nP, &mp, &ct);
            if (st > mxs) mxs = st;
            if (mp == 16) P[l] = nP;
            else P[l] = nP | (P[l] & ~((1u << mp) - 1));  // merged, or cut: the old tokens from mp on
            NE[l] = lane_end(l, P[l]);
          }
          for (int l = 0; l < 64; ++l) E[l] = NE[l];
          rsit += mxs;
        }
        // the super-chunk's output: tokens in lane order, literal runs between them (merged)
        uint32_t p = sc0, run = 0;
        uint64_t ob = 0;
        for (int l = 0; l < 64; ++l) {
          const uint32_t c0 = sc0 + 16 * l;
          for (uint32_t pm = P[l]; pm; pm &= pm - 1) {
            const uint32_t q = c0 + __builtin_ctz(pm);
            if (q < p) continue;  // (a token covered by an earlier lane's copy: never kept)
            run += q - p;
            ob += lit_bytes(run);
            run = 0;
            const uint32_t L = full_len(q);
            ob += copy_bytes(q - cand[q], L);
            p = q + L;
          }
        }
        if (p < sce) run += sce - p;
        ob += lit_bytes(run);
        out_bytes += ob;
      }
    }
    free(d);
  }
  printf("KCAP %d: first walk %.2f, resync rounds %.2f, resync iterations %.2f per super-chunk; output %lu B\n", KCAP,
         (double)it1 / n_sc, (double)rsr / n_sc, (double)rsit / n_sc, (unsigned long)out_bytes);
  return 0;
}
