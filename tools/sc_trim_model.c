// CPU model of the fast compressor's parse (design tool, not product code): the kernel's candidates
// and first walks (tools/sc_resync_model.c), then ways of joining the rows of a super-chunk, each
// printed as stream bytes (literal runs merged inside a super-chunk, as the kernel does):
//  resync:    a lane whose true start (the previous lane's end) differs walks again from there, in
//             rounds until no start changes (the round-3 kernel before SC_MONO; RCAP=k caps the
//             rounds and trims the rest);
//  trim:      every lane keeps its first walk; its start is the running max of the earlier lanes'
//             ends, tokens ending at or before it are dropped, the one it falls inside starts there
//             instead (same offset, shorter; below 4 bytes its bytes become literals); trim+fill and
//             resync1 are two ways of filling the gaps a trim opens;
//  monotone:  the kernel's SC_MONO: one rewalk round from the running max of the first walks' ends
//             (a rewalk that does not merge keeps the old last token when it ends later), then the
//             trim; MCAP=k rounds; SHORTCP=1 keeps 1..3-byte remainders that end past the row as
//             copies; HYBRID=1 runs the full rounds for super-chunks where a covered lane keeps a
//             token (long repeats), as the kernel does.
//  OLDER=1 / FARD=d: candidate-choice experiments (the older candidate always / when the recent one
//             is nearer than d).  CLIPK=k: first-walk overhangs of 1..k bytes clipped.
// Build: gcc -O2 -w -o /tmp/tm tools/sc_trim_model.c     Run: [ENV=..] /tmp/tm file...
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static uint32_t ld32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
static uint32_t T[8192], T2[8192], cand[65536];
static uint8_t match[65536];
static const uint8_t* b;
static uint32_t sc0, sce, clipK = 0; static int hybrid = 0, mo_fallback = 0; static uint64_t n_fb = 0; static int mcap = 1, shortcp = 0; static uint64_t n_shortcp = 0; static uint64_t n_mlens = 0, n_mrounds = 0, n_keep = 0; static int farD = 0, older = 0, rcap = 1000, noclip = 0; static uint64_t n_ftrim = 0;
static uint64_t n_lens_rs = 0, n_rounds = 0, n_clipped = 0;
static uint32_t lenAt(uint32_t q) {  // the kernel's length byte (17: extend)
  uint32_t c = cand[q], l = 0;
  while (l < 16 && b[c + l] == b[q + l]) ++l;
  uint32_t av = sce - q;
  return (l == 16 && av > 16) ? 17 : (l < av ? l : av);
}
static uint32_t extend(uint32_t q) {
  uint32_t c = cand[q], L = 16, cap = sce - q < 255 ? sce - q : 255;
  while (L < cap && b[c + L] == b[q + L]) ++L;
  return L;
}
static uint32_t copy_bytes(uint32_t off, uint32_t L) {
  if (L < 4) return 3;
  uint32_t k = L >= 68 ? (L - 4) >> 6 : 0, R0 = L - 64 * k, x = R0 > 64, R = R0 - 60 * x;
  return 3 * (k + x) + ((R < 12 && off < 2048) ? 2 : 3);
}
static uint32_t lit_bytes(uint32_t n) { return n == 0 ? 0 : n + (n <= 60 ? 1 : (n <= 256 ? 2 : 3)); }
typedef struct { uint32_t q, L, off; } Tok;
// stream bytes of a super-chunk's token list (sorted, non-overlapping)
static uint64_t sc_bytes(const Tok* t, int nt) {
  uint64_t s = 0;
  uint32_t p = sc0;
  for (int i = 0; i < nt; ++i) { s += lit_bytes(t[i].q - p) + copy_bytes(t[i].off, t[i].L); p = t[i].q + t[i].L; }
  return s + lit_bytes(sce - p);
}
// one walk of lane l from row position sr until it leaves the row or meets a bit of stop
static void walk(uint32_t l, uint32_t sr, uint32_t stop, uint32_t mask, uint32_t* path, uint32_t* mpos, uint32_t* pend,
                 uint32_t* Lr) {
  uint32_t c0 = sc0 + 16 * l, ce = c0 < sce ? (c0 + 16 < sce ? c0 + 16 : sce) : c0;
  uint32_t m0 = sr < 16 ? mask >> sr : 0, i = m0 ? sr + __builtin_ctz(m0) : 16, last = 16, lastL = 0;
  *path = 0; *mpos = 16;
  while (i < 16) {
    if ((stop >> i) & 1) { *mpos = i; break; }
    *path |= 1u << i; last = i;
    uint32_t enc = lenAt(c0 + i);
    Lr[i] = enc; lastL = enc; if (stop) n_lens_rs++;
    uint32_t t = i + (enc < 16 ? enc : 16), m = mask >> t;
    i = m ? t + __builtin_ctz(m) : 16;
  }
  *pend = ce;
  if (last < 16 && last + (lastL < 16 ? lastL : 16) >= 16) {
    uint32_t L = lastL == 17 ? extend(c0 + last) : lastL;
    if (lastL == 17) Lr[last] = L;
    *pend = c0 + last + L;
    if (clipK && sr == 0 && stop == 0 && *pend > ce && *pend - ce <= clipK) {  // (first walks only)
      n_clipped++;
      uint32_t L2 = ce - c0 - last;
      if (L2 >= 4) Lr[last] = L2; else *path &= ~(1u << last);
      *pend = ce;
    }
  }
}
int main(int argc, char** argv) {
  if (getenv("HYBRID")) hybrid = 1;
  if (getenv("SHORTCP")) shortcp = 1;
  if (getenv("MCAP")) mcap = atoi(getenv("MCAP"));
  if (getenv("FARD")) farD = atoi(getenv("FARD"));
  if (getenv("OLDER")) older = 1;
  if (getenv("NOCLIP")) noclip = 1;
  if (getenv("RCAP")) rcap = atoi(getenv("RCAP"));
  if (getenv("CLIPK")) clipK = atoi(getenv("CLIPK"));
  uint64_t tot_mo = 0, n_cp = 0, n_small = 0, n_tail = 0, tot_r1 = 0, n_rw1 = 0, n_clip = 0, tot_tf = 0, n_fill = 0, tot_in = 0, tot_rs = 0, tot_tr = 0, n_trim = 0, n_drop = 0, n_short = 0;
  for (int f = 1; f < argc; ++f) {
    FILE* fp = fopen(argv[f], "rb");
    fseek(fp, 0, SEEK_END); long sz = ftell(fp); fseek(fp, 0, SEEK_SET);
    uint8_t* d = calloc(sz + 64, 1);
    if (fread(d, 1, sz, fp) != (size_t)sz) return 2;
    fclose(fp);
    uint64_t f_rs = 0, f_tr = 0, f_tf = 0, f_r1 = 0, f_mo = 0;
    for (long o = 0; o < sz; o += 65536) {
      uint32_t n = sz - o < 65536 ? sz - o : 65536;
      b = d + o;
      memset(T, 0, sizeof T); memset(T2, 0, sizeof T2);
      for (uint32_t q = 0; q < n; ++q) {
        match[q] = 0;
        if (q + 4 > n) continue;
        uint32_t h = (ld32(b + q) * 0x1e35a7bdu) >> 19, cls = (q >> 6) & 1;
        uint32_t *Ta = cls ? T2 : T, *Tb = cls ? T : T2, a = Ta[h], bb = Tb[h];
        uint32_t c1 = a > bb ? a : bb, c2 = a > bb ? bb : a;
        Ta[h] = q + 1;
        uint32_t e = (q / 1024 + 1) * 1024; if (e > n) e = n;
        int ok1 = q + 4 <= e && c1 && c1 - 1 < q, ok2 = q + 4 <= e && c2 && c2 - 1 < q;
        if (older) { uint32_t t = c1; c1 = c2; c2 = t; int tk = ok1; ok1 = ok2; ok2 = tk; }
        if (farD && ok1 && ok2 && q - (c1 - 1) < (uint32_t)farD && ld32(b + c2 - 1) == ld32(b + q)) { uint32_t t = c1; c1 = c2; c2 = t; }
        if (ok1 && ld32(b + c1 - 1) == ld32(b + q)) { match[q] = 1; cand[q] = c1 - 1; }
        else if (ok2 && ld32(b + c2 - 1) == ld32(b + q)) { match[q] = 1; cand[q] = c2 - 1; }
      }
      for (sc0 = 0; sc0 < n; sc0 += 1024) {
        sce = sc0 + 1024 < n ? sc0 + 1024 : n;
        uint32_t mask[64], P[64], E[64], S[64], L1[64][16], P1[64], E1[64];
        for (int l = 0; l < 64; ++l) {
          uint32_t c0 = sc0 + 16 * l; mask[l] = 0;
          for (int i = 0; i < 16; ++i) if (c0 + i < sce && match[c0 + i]) mask[l] |= 1u << i;
        }
        for (int l = 0; l < 64; ++l) {
          uint32_t c0 = sc0 + 16 * l, mp;
          S[l] = c0;
          if (c0 < sce) walk(l, 0, 0, mask[l], &P[l], &mp, &E[l], L1[l]); else { P[l] = 0; E[l] = c0; }
          P1[l] = P[l]; E1[l] = E[l];
        }
        // ---- trim ----
        Tok tt[1100]; int nt = 0;
        uint32_t run = sc0;  // max end of earlier lanes
        for (int l = 0; l < 64; ++l) {
          uint32_t c0 = sc0 + 16 * l;
          if (c0 >= sce) break;
          uint32_t s = run > c0 ? run : c0;
          for (uint32_t pm = P1[l]; pm; pm &= pm - 1) {
            uint32_t i = __builtin_ctz(pm), q = c0 + i, L = L1[l][i];
            if (q + L <= s) { n_drop++; continue; }
            if (q < s) {
              n_trim++;
              uint32_t L2 = q + L - s;
              if (L2 < 4) { n_short++; continue; }
              tt[nt++] = (Tok){s, L2, q - cand[q]};
            } else {
              tt[nt++] = (Tok){q, L, q - cand[q]};
            }
          }
          if (E1[l] > run) run = E1[l];
        }
        f_tr += sc_bytes(tt, nt);
        // ---- trim + fill: the gap a trim opens ([s, next kept token) or [s, the lane's end)) takes
        // greedy matches clipped at the gap's end (no lane's end moves: no cascade) ----
        nt = 0; run = sc0;
        for (int l = 0; l < 64; ++l) {
          uint32_t c0 = sc0 + 16 * l;
          if (c0 >= sce) break;
          uint32_t s = run > c0 ? run : c0, ce = c0 + 16 < sce ? c0 + 16 : sce;
          uint32_t lend = E1[l] > s ? E1[l] : s;
          int first = nt, filled = 0;
          Tok kept[8]; int nk = 0;
          for (uint32_t pm = P1[l]; pm; pm &= pm - 1) {
            uint32_t i = __builtin_ctz(pm), q = c0 + i, L = L1[l][i];
            if (q + L <= s) continue;
            if (q < s) { uint32_t L2 = q + L - s; if (L2 < 4) continue; kept[nk++] = (Tok){s, L2, q - cand[q]}; }
            else kept[nk++] = (Tok){q, L, q - cand[q]};
          }
          // fill [s, gap end) when s is not a kept token's start
          if (s < ce && !(nk && kept[0].q == s)) {
            uint32_t ge = nk ? kept[0].q : lend, j = s;
            while (j < ge && j < ce) {
              if (!match[j]) { ++j; continue; }
              uint32_t L = 0, c = cand[j], cap = ge - j;
              while (L < cap && L < 255 && b[c + L] == b[j + L]) ++L;
              if (L >= 4) { tt[nt++] = (Tok){j, L, j - c}; j += L; n_fill++; } else ++j;
            }
          }
          for (int k = 0; k < nk; ++k) tt[nt++] = kept[k];
          (void)first; (void)filled;
          if (E1[l] > run) run = E1[l];
        }
        f_tf += sc_bytes(tt, nt);
        // ---- one resync round, clipped: a lane whose start s = the running max of earlier first-walk
        // ends differs from its row start walks again from s (stopping where it meets its old path);
        // a new last token may not end past the lane's old end max(E1, s) (clipped there) ----
        nt = 0; run = sc0;
        for (int l = 0; l < 64; ++l) {
          uint32_t c0 = sc0 + 16 * l;
          if (c0 >= sce) break;
          uint32_t s = run > c0 ? run : c0, ce = c0 + 16 < sce ? c0 + 16 : sce;
          uint32_t lend = E1[l] > s ? E1[l] : s;
          uint32_t Lr[16]; memcpy(Lr, L1[l], sizeof Lr);
          uint32_t Pn = P1[l];
          Tok extra = {0, 0, 0};
          // the old last token, as a tail piece from position x to lend (when it straddles x)
          #define OLDTAIL(x) { if (P1[l]) { uint32_t ob = 31 - __builtin_clz(P1[l]), oq = c0 + ob; \
              if (oq < (x) && oq + L1[l][ob] == lend && lend >= (x) + 4) { extra = (Tok){(x), lend - (x), oq - cand[oq]}; n_tail++; } } }
          if (s != c0) {
            if (s >= ce) { Pn = 0; OLDTAIL(s) }
            else {
              uint32_t nP, mp, ne;
              walk(l, s - c0, P1[l], mask[l], &nP, &mp, &ne, Lr);
              n_rw1++;
              Pn = mp == 16 ? nP : (nP | (P1[l] & ~((1u << mp) - 1)));
              if (mp == 16) {
                uint32_t nend = ne;
                if (nP && !noclip) { uint32_t lastb = 31 - __builtin_clz(nP); if (c0 + lastb + Lr[lastb] > lend) { n_clip++; uint32_t L2 = lend - c0 - lastb; if (L2 < 4) { Pn &= ~(1u << lastb); nend = c0 + lastb; } else { Lr[lastb] = L2; nend = lend; } } }
                if (nend < lend) OLDTAIL(nend > s ? nend : s)
              }
            }
          }
          for (uint32_t pm = Pn; pm; pm &= pm - 1) { uint32_t i = __builtin_ctz(pm); tt[nt++] = (Tok){c0 + i, Lr[i], c0 + i - cand[c0 + i]}; }
          if (extra.L) tt[nt++] = extra;
          if (E1[l] > run) run = E1[l];
        }
        if (noclip) {  // the final trim against the running max of the token ends (a rewalk may end later)
          Tok t2[1100]; int n2 = 0; uint32_t mx = sc0;
          for (int k = 0; k < nt; ++k) {
            Tok t = tt[k];
            if (t.q + t.L <= mx) continue;
            if (t.q < mx) { if (t.q + t.L - mx < 4) { continue; } t.L = t.q + t.L - mx; t.q = mx; n_ftrim++; }
            t2[n2++] = t; mx = t.q + t.L;
          }
          memcpy(tt, t2, n2 * sizeof(Tok)); nt = n2;
        }
        f_r1 += sc_bytes(tt, nt);
        // ---- monotone: rounds of rewalks from s = max(c0, running max of earlier ends); a lane that
        // does not merge keeps its old last token when that ends later (ends never decrease); after
        // mcap rounds, a final in-order trim of every lane's tokens against the running max ----
        {
          uint32_t MP[64], ME[64], ML[64][16], MS[64], oxl[64];
          for (int l = 0; l < 64; ++l) { MP[l] = P1[l]; ME[l] = E1[l]; MS[l] = sc0 + 16 * l; memcpy(ML[l], L1[l], sizeof ML[l]); }
          for (int rr = 0; rr < mcap; ++rr) {
            uint32_t run2 = sc0, NS[64]; int chg = 0;
            for (int l = 0; l < 64; ++l) { uint32_t c0 = sc0 + 16 * l; NS[l] = run2 > c0 ? run2 : c0; if (ME[l] > run2) run2 = ME[l]; }
            for (int l = 0; l < 64; ++l) {
              uint32_t c0 = sc0 + 16 * l, ce = c0 < sce ? (c0 + 16 < sce ? c0 + 16 : sce) : c0;
              if (NS[l] == MS[l]) continue;
              chg++;
              MS[l] = NS[l];
              if (NS[l] >= ce) continue;  // covered: trimmed at the end
              uint32_t nP, mp, ne, Lr[16];
              memcpy(Lr, ML[l], sizeof Lr);
              walk(l, NS[l] - c0, MP[l], mask[l], &nP, &mp, &ne, Lr);
              n_mlens++;
              if (mp == 16) {
                uint32_t np = nP;
                if (MP[l]) { uint32_t ob = 31 - __builtin_clz(MP[l]); if (c0 + ob + ML[l][ob] > ne && __builtin_popcount(nP) < 4 && !(nP >> ob & 1)) { np |= 1u << ob; ne = c0 + ob + ML[l][ob]; Lr[ob] = ML[l][ob]; n_keep++; } }
                MP[l] = np; ME[l] = ne > ME[l] ? ne : ME[l];
              } else MP[l] = nP | (MP[l] & ~((1u << mp) - 1));
              memcpy(ML[l], Lr, sizeof Lr);
            }
            if (!chg) break;
            n_mrounds++;
          }
          nt = 0;
          uint32_t cur = sc0;
          int bad = 0;
          for (int l = 0; l < 64; ++l) {
            uint32_t c0 = sc0 + 16 * l;
            if (c0 >= sce) break;
            uint32_t ce0 = c0 + 16 < sce ? c0 + 16 : sce;
            int covered = cur >= ce0;
            int nbefore = nt;
            for (uint32_t pm = MP[l]; pm; pm &= pm - 1) {
              uint32_t i = __builtin_ctz(pm), q = c0 + i, L = ML[l][i];
              if (q + L <= cur) continue;
              uint32_t ce = c0 + 16 < sce ? c0 + 16 : sce;
              if (q < cur) { if (q + L - cur < 4 && (q + L <= ce || !shortcp)) continue; if (q + L - cur < 4) n_shortcp++; tt[nt++] = (Tok){cur, q + L - cur, q - cand[q]}; }
              else tt[nt++] = (Tok){q, L, q - cand[q]};
              cur = q + L;
            }
            if (covered && nt > nbefore) bad = 1;
          }
          if (hybrid && bad) { n_fb++; f_mo += 0; mo_fallback = 1; } else { mo_fallback = 0; f_mo += sc_bytes(tt, nt); }
        }
        // ---- resync ----
        for (int rr = 0; rr < rcap; ++rr) {
          uint32_t sn[64], NE[64]; int chg = 0;
          for (int l = 0; l < 64; ++l) { sn[l] = l ? E[l - 1] : sc0; if (sn[l] != S[l]) chg++; }
          if (!chg) break;
          n_rounds++;
          for (int l = 0; l < 64; ++l) {
            NE[l] = E[l];
            if (sn[l] == S[l]) continue;
            uint32_t c0 = sc0 + 16 * l, ce = c0 < sce ? (c0 + 16 < sce ? c0 + 16 : sce) : c0;
            S[l] = sn[l];
            if (sn[l] >= ce) { P[l] = 0; NE[l] = sn[l]; continue; }
            uint32_t nP, mp, ne;
            walk(l, sn[l] - c0, P[l], mask[l], &nP, &mp, &ne, L1[l]);
            if (mp == 16) { P[l] = nP; NE[l] = ne; } else P[l] = nP | (P[l] & ~((1u << mp) - 1));
          }
          for (int l = 0; l < 64; ++l) E[l] = NE[l];
        }
        nt = 0; run = sc0;
        for (int l = 0; l < 64; ++l) {  // (after rcap rounds: trim against the running max of the ends)
          uint32_t c0 = sc0 + 16 * l;
          if (c0 >= sce) break;
          uint32_t s = run > S[l] ? run : S[l];
          for (uint32_t pm = P[l]; pm; pm &= pm - 1) {
            uint32_t i = __builtin_ctz(pm), q = c0 + i, L = L1[l][i];
            if (q + L <= s) continue;
            if (q < s) { if (q + L - s >= 4) tt[nt++] = (Tok){s, q + L - s, q - cand[q]}; }
            else tt[nt++] = (Tok){q, L, q - cand[q]};
          }
          if (E[l] > run) run = E[l];
        }
        f_rs += sc_bytes(tt, nt);
        if (mo_fallback) f_mo += sc_bytes(tt, nt);
        for (int k = 0; k < nt; ++k) { n_cp++; if (tt[k].off < 256) n_small++; }
      }
    }
 printf("%-20s monotone %.4f (%.4fx)\n", argv[f], (double)f_mo / sz, (double)f_mo / f_rs); tot_mo += f_mo;
    printf("%-20s %8ld  resync %.4f  trim %.4f (%.4fx)  trim+fill %.4f (%.4fx) resync1 %.4f (%.4fx)\n", argv[f], sz, (double)f_rs / sz,
           (double)f_tr / sz, (double)f_tr / f_rs, (double)f_tf / sz, (double)f_tf / f_rs, (double)f_r1 / sz, (double)f_r1 / f_rs);
    tot_in += sz; tot_rs += f_rs; tot_tr += f_tr; tot_tf += f_tf; tot_r1 += f_r1;
    free(d);
  }
  printf("monotone: %.4f (%.4fx), %.3f rounds/sc, %.2f rewalks/sc, kept %llu short copies %llu fallbacks %.4f/sc\n", (double)tot_mo / tot_in, (double)tot_mo / tot_rs, n_mrounds / (tot_in / 1024.0), n_mlens / (tot_in / 1024.0), (unsigned long long)n_keep, (unsigned long long)n_shortcp, n_fb / (tot_in / 1024.0));
  printf("copies %llu, offset < 256: %.3f\n", (unsigned long long)n_cp, (double)n_small / n_cp);
  printf("resync: %.3f rounds/sc, %.2f lengths/sc (stop-walks), first-walk clips %llu\n", (double)n_rounds / (tot_in / 1024.0), (double)n_lens_rs / (tot_in / 1024.0), (unsigned long long)n_clipped);
  printf("resync1 %.4f (%.4fx), rewalks %llu clipped %llu tails %llu ftrim %llu\n", (double)tot_r1 / tot_in, (double)tot_r1 / tot_rs, (unsigned long long)n_rw1, (unsigned long long)n_clip, (unsigned long long)n_tail, (unsigned long long)n_ftrim);
  printf("trim+fill %.4f (%.4fx), fills %llu\n", (double)tot_tf / tot_in, (double)tot_tf / tot_rs, (unsigned long long)n_fill);
  printf("total %llu: resync %.4f trim %.4f (%.4fx); trimmed %llu (short %llu) dropped %llu\n", (unsigned long long)tot_in,
         (double)tot_rs / tot_in, (double)tot_tr / tot_in, (double)tot_tr / tot_rs, (unsigned long long)n_trim,
         (unsigned long long)n_short, (unsigned long long)n_drop);
}
