// CPU model of the fast compressor's stream SIZE (design tool, not product code): the kernel's
// per-position candidates (k_compress_sc section B/C: a 13-bit table of two u16 slots, group parity
// picks the slot, the more recent 4-byte match unless it is nearer than FAR and the older matches),
// then the exact greedy parse of each 1 KiB super-chunk (what the lane walks + resynchronisation
// compute: copies up to 255 bytes that stop at the super-chunk end, positions without 4 bytes
// before the super-chunk end start no copy), literal runs merged inside a super-chunk only, and the
// block-level fallback to one literal.  Variants (environment):
//   FARMAX=x   ... and the older one is nearer than x
//   BLK=b      fragment bytes (64 KiB)
//   LONGNEAR=1 the FAR rule, but a near recent candidate against the older by 16-byte lengths
//   MARGIN=m   (LONG16) a near (< FAR) recent candidate only when longer than the older by >= m
//   TBITS=b    hash table of 2^b buckets (kernel: 13)
//   FAR=d      the older candidate when the recent one is nearer than d (kernel: 256)
//   LONGEST=1  of the two 4-byte-matching candidates, the one with the longer match (ties: recent)
//   LONG8=1    ... the longer by an 8-byte compare only (ties and both >= 8: the FAR rule)
//   LONG16=1   ... by a 16-byte compare (the dense mode)
//   XSC=1      copies may run past the super-chunk end (to the block end)
//   MERGE=1    literal runs merged across super-chunks
//   SCS=n      super-chunk bytes (1024)
//   HASH=1     the full-rate hash of round 5: ((w ^ (w >> 15)) * 0x9e3779 as u24 x u24) >> (32 - b)
//   POS0=1     slots hold positions (not position + 1): an empty slot is candidate 0 (verified)
//   SPARSE=1   only even positions are hashed and inserted; an odd position q - 1 takes the even
//              q's candidate c as c - 1 when the byte before it matches (a 5-byte match)
// Prints per file: the model's size, the size the reference's parse gives (the oracle), the ratio.
// Build: gcc -O2 -o /tmp/rm tools/ratio_model.c -L oracle -loracle_snappy -Wl,-rpath,$PWD/oracle
// Run:   [FAR=256] /tmp/rm tests/golden/testdata/{alice29.txt,...}
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint32_t ld32(const uint8_t* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
static int hashmode = 0, pos0 = 0, sparse = 0;
static int farmax = 1 << 30, blk = 65536, longnear = 0, margin = 0, tbits = 13, far_d = 256, longest = 0, long8 = 0, long16 = 0, xsc = 0, merge = 0, scs = 1024;

static uint32_t lit_bytes(uint32_t n) { return n == 0 ? 0 : n + (n <= 60 ? 1 : (n <= 256 ? 2 : (n <= 65536 ? 3 : 4))); }
static uint64_t n_copies = 0, n_near = 0, n_both = 0, n_need = 0;
static uint8_t g_both[65536], g_need[65536];
static uint32_t copy_bytes(uint32_t off, uint32_t L) {
  ++n_copies;
  n_near += off < 256;
  uint32_t k = L >= 68 ? (L - 4) >> 6 : 0, R0 = L - 64 * k, x = R0 > 64, R = R0 - 60 * x;
  return 3 * (k + x) + ((R < 12 && off < 2048) ? 2 : 3);
}
static uint32_t mlen(const uint8_t* b, uint32_t p, uint32_t q, uint32_t lim) {
  uint32_t l = 0;
  while (q + l < lim && b[p + l] == b[q + l]) ++l;
  return l;
}

// one block (fragment) of n <= 65536 bytes: stream bytes without the varint header
static uint64_t block_bytes(const uint8_t* b, uint32_t n) {
  static uint32_t T[8192];
  static uint32_t cand[65536];
  static uint8_t has[65536];
  memset(T, 0, sizeof T);
  for (uint32_t q = 0; q < n; ++q) has[q] = 0;
  for (uint32_t q = 0; q < n; ++q) {
    if (q + 4 > n) continue;
    if (sparse && (q & 1)) continue;
    const uint32_t w = ld32(b + q);
    uint32_t h;
    if (hashmode == 1) h = (((w ^ (w >> 15)) & 0xffffffu) * 0x9e3779u) >> (32 - tbits);
    else if (hashmode == 2) h = ((w & 0xffffffu) * 0x9e3779u + (w >> 24) * 0x7a3c9bu) >> (32 - tbits);
    else if (hashmode == 3) h = (((w & 0xffffffu) * 0x1e35a7u) ^ ((w >> 8) * 0x9e3779u)) >> (32 - tbits);
    else if (hashmode == 4) h = ((w & 0xffffffu) * 0x1e35a7u + (w >> 8) * 0x2545f5u) >> (32 - tbits);
    else if (hashmode == 5) h = (uint32_t)(((uint64_t)(w & 0xffffffu) * 0x9e3779u + (uint64_t)((w >> 8) & 0xffffffu) * 0x1e35a7u) >> 32) & ((1u << tbits) - 1);
    else h = (w * 0x1e35a7bdu) >> (32 - tbits);
    const uint32_t par = (q >> 6) & 1;
    const uint32_t own = par ? T[h] >> 16 : T[h] & 0xffff, oth = par ? T[h] & 0xffff : T[h] >> 16;
    const uint32_t qv = pos0 ? q : q + 1;
    T[h] = par ? (T[h] & 0xffff) | (qv << 16) : (T[h] & 0xffff0000u) | qv;
    const uint32_t c1 = own > oth ? own : oth, c2 = own > oth ? oth : own;
    const uint32_t p1 = pos0 ? c1 : c1 - 1, p2 = pos0 ? c2 : c2 - 1;
    const int m1 = (pos0 ? p1 < q : c1 != 0) && ld32(b + p1) == w, m2 = (pos0 ? p2 < q : c2 != 0) && ld32(b + p2) == w;
    if (!m1 && !m2) continue;
    int use2 = m2 && (!m1 || (q - p1 < (uint32_t)far_d && q - p2 < (uint32_t)farmax));
    if (longnear && m1 && m2 && q - p1 < (uint32_t)far_d) {  // only a near recent one is compared
      const uint32_t lim = q + 16 < n ? q + 16 : n;
      const uint32_t l1 = mlen(b, p1, q, lim), l2 = mlen(b, p2, q, lim);
      use2 = l2 >= l1;
    } else if (longnear) {
    } else if (m1 && m2 && (longest || long8 || long16)) {
      const uint32_t cap = long16 ? 16 : 8;
      const uint32_t lim = (long8 || long16) ? (q + cap < n ? q + cap : n) : n;
      const uint32_t l1 = mlen(b, p1, q, lim), l2 = mlen(b, p2, q, lim);
      if (margin && q - p1 < (uint32_t)far_d)  // a near recent one only when longer by >= margin
        use2 = !(l1 >= l2 + (uint32_t)margin);
      else if (l1 != l2)
        use2 = l2 > l1;
      else if (longest) use2 = 0;
    }
    has[q] = 1;
    cand[q] = use2 ? p2 : p1;
    if (sparse && q > 0 && cand[q] > 0 && b[cand[q] - 1] == b[q - 1]) {
      has[q - 1] = 1;
      cand[q - 1] = cand[q] - 1;
    }
    g_both[q] = m1 && m2;
    {
      const uint32_t lim16 = q + 16 < n ? q + 16 : n;
      g_need[q] = m1 && m2 && (mlen(b, p1, q, lim16) < 16 || q - p1 < (uint32_t)far_d);
    }
  }
  uint64_t out = 0;
  uint32_t run = 0;  // pending literal run
  for (uint32_t s0 = 0; s0 < n; s0 += scs) {
    const uint32_t se = s0 + scs < n ? s0 + scs : n;
    const uint32_t lim = xsc ? n : se;
    uint32_t p = s0 > 0 && xsc ? p : s0;
    if (!merge && run) {
      out += lit_bytes(run);
      run = 0;
    }
    while (p < se) {
      if (has[p] && p + 4 <= lim) {
        uint32_t L = mlen(b, cand[p], p, lim);
        if (L > 255) L = 255;
        if (L >= 4) {
          n_both += g_both[p];
          n_need += g_need[p];
          out += lit_bytes(run);
          run = 0;
          out += copy_bytes(p - cand[p], L);
          p += L;
          continue;
        }
      }
      ++run;
      ++p;
    }
    if (xsc && p > se) {
      // (the next super-chunk starts where this copy ended)
      s0 = p - scs;  // loop adds scs back
      if (p >= n) break;
      // restart at p: emulate by continuing the outer loop with s0 + scs == p
    }
  }
  out += lit_bytes(run);
  const uint64_t lit = lit_bytes(n);
  return out > lit ? lit : out;
}

#include "../oracle/snappy_oracle.h"

static uint32_t vlen(uint32_t v) { return v < 128 ? 1 : v < 16384 ? 2 : v < (1u << 21) ? 3 : v < (1u << 28) ? 4 : 5; }

int main(int argc, char** argv) {
  if (getenv("FAR")) far_d = atoi(getenv("FAR"));
  if (getenv("TBITS")) tbits = atoi(getenv("TBITS"));
  if (getenv("MARGIN")) margin = atoi(getenv("MARGIN"));
  if (getenv("LONGNEAR")) longnear = atoi(getenv("LONGNEAR"));
  if (getenv("BLK")) blk = atoi(getenv("BLK"));
  if (getenv("FARMAX")) farmax = atoi(getenv("FARMAX"));
  if (getenv("LONGEST")) longest = atoi(getenv("LONGEST"));
  if (getenv("LONG8")) long8 = atoi(getenv("LONG8"));
  if (getenv("LONG16")) long16 = atoi(getenv("LONG16"));
  if (getenv("XSC")) xsc = atoi(getenv("XSC"));
  if (getenv("MERGE")) merge = atoi(getenv("MERGE"));
  if (getenv("SCS")) scs = atoi(getenv("SCS"));
  if (getenv("HASH")) hashmode = atoi(getenv("HASH"));
  if (getenv("POS0")) pos0 = atoi(getenv("POS0"));
  if (getenv("SPARSE")) sparse = atoi(getenv("SPARSE"));
  double worst = 0, tot_m = 0, tot_r = 0;
  for (int f = 1; f < argc; ++f) {
    FILE* fp = fopen(argv[f], "rb");
    if (!fp) continue;
    fseek(fp, 0, SEEK_END);
    long sz = ftell(fp);
    fseek(fp, 0, SEEK_SET);
    uint8_t* b = malloc(sz + 64);
    uint8_t* o = malloc(sz + sz / 6 + 64);
    if (fread(b, 1, sz, fp) != (size_t)sz) return 1;
    fclose(fp);
    memset(b + sz, 0, 64);
    uint64_t m = vlen((uint32_t)sz);
    for (long off = 0; off < sz; off += blk) m += block_bytes(b + off, (uint32_t)(sz - off < blk ? sz - off : blk));
    size_t r = 0;
    if (smo_compress(b, sz, o, &r, 0) != 0) return 1;
    const double q = (double)m / r;
    if (q > worst) worst = q;
    tot_m += m;
    tot_r += r;
    const char* nm = strrchr(argv[f], '/');
    printf("%-20s %9ld  ref %9zu  model %9lu (%.4f)\n", nm ? nm + 1 : argv[f], sz, r, (unsigned long)m, q);
    free(b);
    free(o);
  }
  printf("worst %.4f  total %.4f  copies %lu near(<256) %.3f both %.3f need %.3f\n", worst, tot_m / tot_r, (unsigned long)n_copies, (double)n_near / n_copies, (double)n_both / n_copies, (double)n_need / n_copies);
  return 0;
}
