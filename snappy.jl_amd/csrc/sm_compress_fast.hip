// sm_compress_fast.hip -- "fast mode" batched snappy compression for gfx950 (MI355X).
//
// Produces a valid snappy stream per <= 64 KiB block (decodes bit-exactly under Snappy.jl's
// uncompress, src/internal.jl:411-466) with a wave-parallel parse instead of the reference's
// serial greedy loop (internal.jl:127-250).
//
// One workgroup of 16 waves per block, in two roles:
//  * the INSERTER (wave 15) walks the block's positions in order, 64 per instruction, through
//    a hash table with ds_wrxchg_rtn_b32.  A wave's LDS instructions execute in order and the
//    conflicting lanes of one instruction in ascending lane order, so the value each position
//    gets back is exactly the sequential one: the latest and the second-latest earlier
//    position with the same hash (a table entry holds both: the exchange puts the new position
//    in the low half and a ds_write_b16 moves the old latest into the high half).  Correctness
//    never depends on that order -- every candidate is verified -- only the ratio does.  The
//    candidates go to a per-round LDS ring, one round ahead of the parse.
//  * 15 PARSE waves.  The block is cut into kChunk-byte chunks whose parse never crosses the
//    chunk end (copies are truncated there, literal runs end there), so the chunks of a round
//    are parsed independently: in round r parse wave w owns chunk slots w and w + 15 (fast
//    mode; slot w in dense mode), kChunk/64 positions per lane (q = c0 + 64j + lane).  Per
//    chunk: verify the chain candidates of every position (8 bytes) and extend the matches
//    that fill that window (compacted into full waves of jobs, copies capped at 64 bytes),
//    greedy parse by pointer doubling (J_k = J_{k-1} o J_{k-1}), token sizes in closed form and
//    a DPP scan, then (after the round barrier) the round layout over the round's chunks --
//    literal runs that cross chunk boundaries are merged -- and the emission: token lanes
//    write tag bytes, position lanes scatter literal bytes.
// One barrier per round (chunk infos are double-buffered); the parse waves step their issue
// priority down through a round so they cross it together.  Output is deterministic.
#include <stdlib.h>

#include <type_traits>

#include "sm_device.h"
#include "sm_internal.h"

#ifndef SM_ABLATE  // diagnostic builds only: 1 no emit, 2 no matches, 4 inserter only, 8 no extension past 8 bytes,
                   // 16 no global stores in the emission
#define SM_ABLATE 0
#endif

namespace sm {

constexpr uint32_t kScreenTodo = 0xfffffffeu;  // out_len mark of k_literal_screen: the parse compresses this block

#if SM_STAMP
__device__ unsigned long long g_stamp_c[12];
__device__ unsigned long long g_stamp_w[16];  // barrier wait per wave index
#endif
STAMP_MACROS(12)

#ifndef SM_FAST_CHUNK
#define SM_FAST_CHUNK 256
#endif
constexpr uint32_t kChunk = SM_FAST_CHUNK;     // bytes per chunk: 128 or 256
static_assert(kChunk == 128 || kChunk == 256, "chunk size");
constexpr int kP = kChunk / 64;                // positions per lane
// Hash table: 8 K u32 buckets, 32 KiB (the ring and the jump tables of 256-byte chunks need
// the rest of the LDS); a bucket holds (second-latest+1) << 16 | (latest+1), the high half
// only in depth 2 (SM_MODE_FAST_DENSE).  A 16 K-bucket u16 table updated with
// ds_mskor_rtn_b32 (masked exchange of one half) fits the same 32 KiB: depth 1 then gives
// ratio 0.578 instead of 0.598 on the bench text but runs 7% slower (more copies to parse).
constexpr uint32_t kTabBits = 13;
constexpr uint32_t kTabBytes = 4u << kTabBits;
constexpr uint32_t kWavesPerBlock = 16;
constexpr uint32_t kPW = kWavesPerBlock - 1;  // parse waves; wave kPW is the inserter
constexpr uint32_t kThreads = 64 * kWavesPerBlock;
// J0..J_{kLevels-1}: a chunk holds <= kChunk/4 copies, so its walk takes < kChunk/4 steps
constexpr uint32_t kLevels = kChunk == 256 ? 6 : 5;
// the chain's end marker: the chunk end (128 fits a byte); for 256-byte chunks position 255,
// which is never a match (a match needs 4 bytes), so "the first match at or after x" never
// names it and it maps to itself at every level
constexpr uint32_t kEnd = kChunk == 256 ? 255 : kChunk;
constexpr uint32_t kRow = kChunk + 8;         // a jump-table row (8-B aligned)
// levels built: for 256-byte chunks J0..J4 (16 steps); a chain longer than 32 elements
// (element 31 is a copy) finishes with two more J4 steps instead of a J5 level (4.15 ->
// 4.11 ms on the bench text; building J0..J3 or J0..J2 and stepping more: within noise)
#ifndef SM_FAST_BUILT
#define SM_FAST_BUILT 5
#endif
constexpr uint32_t kBuilt = kChunk == 256 ? SM_FAST_BUILT : kLevels;

// Longest copy the parse takes (0: to the chunk end).  64 is emit_copy!'s own piece size, so a
// longer match costs the same bytes as 64-byte copies chained through the next positions'
// candidates; capping bounds the extension loop at four steps (text: 4.13 -> 4.09 ms, ratio
// 0.5977 -> 0.5978; 128 gains nothing).
#ifndef SM_FAST_LCAP
#define SM_FAST_LCAP 64
#endif
constexpr bool kShortCopies = SM_FAST_LCAP != 0 && SM_FAST_LCAP <= 64;  // one piece per copy
#ifndef SM_FAST_XCOMPACT
#define SM_FAST_XCOMPACT 1
#endif
constexpr bool kXCompact = SM_FAST_XCOMPACT && kChunk == 256;  // extension jobs compacted (below)
constexpr uint32_t kVW = 8;  // bytes the verification compares (16: equal time, round 2)

// literal tag bytes for a run of len bytes (0 = no run): emit_literal! (internal.jl:271-284)
__device__ inline uint32_t lit_tag_bytes(uint32_t len) { return len == 0 ? 0u : (len <= 60 ? 1u : (len <= 256 ? 2u : 3u)); }

// literal tag of `ts` bytes (lit_tag_bytes(len)) for a run of len bytes at dst[o]
__device__ inline void put_lit_tag(uint8_t* dst, uint32_t o, uint32_t ts, uint32_t len) {
  if (ts == 1) {
    dst[o] = (uint8_t)((len - 1) << 2);
  } else if (ts >= 2) {
    dst[o] = (uint8_t)((58 + ts) << 2);  // 60: one length byte, 61: two
    dst[o + 1] = (uint8_t)(len - 1);
    if (ts == 3) dst[o + 2] = (uint8_t)((len - 1) >> 8);
  }
}

// emit_copy! byte count (internal.jl:306-329), closed form
__device__ inline uint32_t copy_bytes_cf(uint32_t off, uint32_t L) {
  if (kShortCopies) return (L < 12 && off < 2048) ? 2 : 3;
  uint32_t k = L >= 68 ? ((L - 68) >> 6) + 1 : 0;
  uint32_t R = L - (k << 6);
  uint32_t e = R > 64 ? 1 : 0;
  R -= 60 * e;
  return 3 * (k + e) + ((R < 12 && off < 2048) ? 2 : 3);
}

// emit_copy! bytes (internal.jl:289-329): 64-byte pieces while L >= 68, a 60 if L > 64, then
// the rest as copy-1 (L < 12, off < 2048) or copy-2
__device__ inline void put_copy_cf(uint8_t* dst, uint32_t o, uint32_t off, uint32_t L) {
  const uint8_t lo = (uint8_t)off, hi = (uint8_t)(off >> 8);
  if (kShortCopies) {  // L <= 64: one copy-1 or copy-2 (emit_copy_upto_64!, internal.jl:289-304)
    const bool c1 = L < 12 && off < 2048;
    dst[o] = (uint8_t)(c1 ? 1 + ((L - 4) << 2) + ((off >> 3) & 0xe0) : 2 + ((L - 1) << 2));
    dst[o + 1] = lo;
    if (!c1) dst[o + 2] = hi;
    return;
  }
  while (L >= 68) {
    dst[o] = (uint8_t)(2 + (63 << 2));
    dst[o + 1] = lo;
    dst[o + 2] = hi;
    o += 3;
    L -= 64;
  }
  if (L > 64) {
    dst[o] = (uint8_t)(2 + (59 << 2));
    dst[o + 1] = lo;
    dst[o + 2] = hi;
    o += 3;
    L -= 60;
  }
  if (L < 12 && off < 2048) {
    dst[o] = (uint8_t)(1 + ((L - 4) << 2) + ((off >> 3) & 0xe0));
    dst[o + 1] = lo;
  } else {
    dst[o] = (uint8_t)(2 + ((L - 1) << 2));
    dst[o + 1] = lo;
    dst[o + 2] = hi;
  }
}

#ifndef SM_FAST_PRIO
#define SM_FAST_PRIO 3
#endif
// Parse waves step their priority down through a round (2 for the previous round's emission,
// 1 for the first chunk, 0 for the second): the SIMD issues oldest-first among equal
// priorities, so without it the youngest parse wave of each SIMD finishes the round last,
// alone; with it the waves move through the round together (text: 4.29 -> 4.18 ms).
#ifndef SM_FAST_PPRIO
#define SM_FAST_PPRIO 1
#endif

// Fast-mode hash of the 4 bytes at a position: full-rate 24-bit multiply (v_mul_u32_u24) of
// the word folded to 24 bits, bits 10.. of the product (the reference's 32-bit multiply,
// internal.jl:94, is quarter rate; fast mode only needs a good spread -- ratio 0.5545 against
// 0.5538 with the reference hash in tools/fastparse_model.c terms).
template <uint32_t kBits>
__device__ inline uint32_t fast_hash(uint32_t w) {
  uint32_t p;  // the compiler widens a masked 24-bit product to v_mul_lo_u32: issue it directly
  asm("v_mul_u32_u24 %0, %1, %2" : "=v"(p) : "s"(0x1e35a7u), "v"(w ^ (w >> 12)));
  return (p >> 10) & ((1u << kBits) - 1);
}

// Round geometry per mode.  SM_MODE_FAST (depth 1) keeps u16 candidates and gives each parse
// wave two chunks per round (30 chunks, 7680 positions: half the rounds, so half the barrier
// tails and round layouts per byte); SM_MODE_FAST_DENSE (depth 2) keeps u32 candidate pairs,
// which leave LDS for one chunk per wave (15 chunks, 3840 positions).  Both rings are 30 KiB.
template <int D>
struct Cfg {
#ifndef SM_FAST_LASTINS  // 1: the inserter parses the final round's chunk slot kPW (see the round loop)
#define SM_FAST_LASTINS 1
#endif
#ifndef SM_FAST_CPW
#define SM_FAST_CPW 2
#endif
  static constexpr int kCPW = D == 1 ? SM_FAST_CPW : 1;  // chunks per parse wave per round
  static constexpr uint32_t kSlots = kPW * kCPW;         // chunks per round
  static constexpr uint32_t kRoundPos = kSlots * kChunk; // positions per round
  typedef typename std::conditional<D == 1, uint16_t, uint32_t>::type Cand;
  static constexpr uint32_t kRingBytes = 2 * kRoundPos * sizeof(Cand);
};

// Hashes of one group of 64 positions [base, base + 64) (base a multiple of 64) into hr[lane]:
// the words come from aligned dwords (one ds_read2), so reads past n stay inside the LDS
// allocation (the table follows the block).  Positions without 4 bytes hash garbage: the
// inserter still inserts them (no exec masks), which is harmless -- they are the block's last
// positions, so no valid position is ever handed one of them as a candidate (later positions
// are all invalid too, and within one exchange the lower lanes go first).
template <typename Cand>
__device__ inline void hash_group(const uint8_t* data, Cand* hr, uint32_t base, uint32_t lane) {
  const uint32_t* dw = reinterpret_cast<const uint32_t*>(data + base) + (lane >> 2);
  hr[lane] = (Cand)fast_hash<kTabBits>(__builtin_amdgcn_alignbyte(dw[1], dw[0], lane & 3u));
}

// Inserter: positions [r0, r0 + kRoundPos) in order.  ring[i] holds the hash of position r0 + i
// (written by the parse waves, hash_group) and receives its candidates: the old table entry.
// The inserter's own work is three LDS instructions per 64 positions (read the hashes, exchange,
// write the candidates), kG groups per step so the round trips overlap; the hashing is the
// parse waves' (it was 80% of this single wave's issue slots, the floor under every round).
template <int D>
__device__ inline void insert_round(uint32_t* T, typename Cfg<D>::Cand* ring, uint32_t r0, uint32_t n, uint32_t lane) {
#ifndef SM_FAST_KG
#define SM_FAST_KG 6
#endif
  constexpr int kG = SM_FAST_KG;
  constexpr uint32_t kRP = Cfg<D>::kRoundPos;
  static_assert((kRP / 64) % kG == 0, "insert step");
  if (r0 >= n) return;
  // only groups whose chunk exists have hashes in the ring (a short last round stops at n)
  const uint32_t ngroups = min((n - r0 + 63) >> 6, kRP / 64);
  auto step = [&](uint32_t g0, uint32_t (&h)[kG], bool guarded) {
    const uint32_t pos1 = r0 + 64 * g0 + lane + 1;
    uint32_t old[kG], hn[kG];
#pragma unroll
    for (int i = 0; i < kG; ++i)
      if (!guarded || g0 + i < ngroups)
        old[i] = __hip_atomic_exchange(&T[h[i]], pos1 + 64 * i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    // the next step's hashes, behind this step's exchanges
#pragma unroll
    for (int i = 0; i < kG; ++i)
      if (g0 + kG + i < ngroups) hn[i] = ring[64 * (g0 + kG + i) + lane];
#pragma unroll
    for (int i = 0; i < kG; ++i) {
      if (!guarded || g0 + i < ngroups) {
        // the old latest becomes the second-latest (the new entry's high half)
        if (D > 1) reinterpret_cast<uint16_t*>(&T[h[i]])[1] = (uint16_t)old[i];  // (dense only)
        ring[64 * (g0 + i) + lane] = (typename Cfg<D>::Cand)old[i];
      }
    }
#pragma unroll
    for (int i = 0; i < kG; ++i) h[i] = hn[i];
  };
  uint32_t h[kG];
#pragma unroll
  for (int i = 0; i < kG; ++i)
    if ((uint32_t)i < ngroups) h[i] = ring[64 * i + lane];
  uint32_t g0 = 0;
  for (; g0 + kG <= ngroups; g0 += kG) step(g0, h, false);  // full steps: no exec or scalar guards
  if (g0 < ngroups) step(g0, h, true);
}

// A parsed chunk, held in registers from its parse to its emission after the round barrier.
struct ChunkTok {
  uint32_t c0, ce;           // the chunk's positions [c0, ce); ce == c0: no chunk
  uint32_t ta, tb;           // token in lane t: copy position | length << 16; offset
  uint32_t ntok, incl, sz;   // tokens; inclusive scan of token sizes; this lane's token size
  uint32_t litlen, littag, ls;  // the token's literal run: length, tag bytes, start
  uint64_t ts[kP];           // copy-start bitmask of the chunk's positions
};

// Parse of chunk [c0, ce) (ce > c0); returns the chunk info word for the round layout:
// unmerged size | leading literal piece << 11 | trailing literal piece << 20 | no copies at all
// << 29.  cvin[j]: the ring candidates of position c0 + 64j + lane, u16 halves of position + 1
// (0: none); kDepth halves are verified.
template <int kDepth>
__device__ inline uint32_t parse_chunk(const uint8_t* data, const uint32_t (&cvin)[kP], uint8_t* jt, uint64_t* tsw,
                                       uint32_t c0, uint32_t ce, uint32_t n, uint32_t lane, ChunkTok& t) {
  t.c0 = c0;
  t.ce = ce;
  t.ta = t.tb = t.ntok = t.incl = t.sz = t.litlen = t.littag = t.ls = 0;
#pragma unroll
  for (int j = 0; j < kP; ++j) t.ts[j] = 0;
  // (a) candidates: the latest (and second-latest) earlier position with the same hash,
  // verified and extended 8 bytes at a time; the longest wins (ties: the latest).
  uint32_t Ls[kP], offs[kP];
  // every group's ring entry and word first, then branch-free verification: every lane reads
  // its candidate's 8 bytes (an invalid candidate reads its own position), so the LDS round
  // trips overlap and no exec-mask branches are needed (text: 3.92 -> 3.87 ms)
  uint32_t cvs[kP];
  uint64_t wqs[kP];
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    const uint32_t q = c0 + 64 * j + lane;
    cvs[j] = cvin[j];
    wqs[j] = lds_ld64(data, q < n ? q : 0);  // the 8 bytes at q
  }
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    const uint32_t q = c0 + 64 * j + lane;
    const bool can = q + 4 <= ce;
    uint32_t L = 0, c = q;
#pragma unroll
    for (int i = 0; i < kDepth; ++i) {
      const uint32_t p = (cvs[j] >> (16 * i)) & 0xffffu;  // position + 1, 0 = none
      const bool ok = can && p != 0 && p - 1 < q;
      const uint64_t x = lds_ld64(data, ok ? p - 1 : q) ^ wqs[j];
      const uint32_t l = x ? (uint32_t)(__builtin_ctzll(x) >> 3) : 8u;
      if (ok && l >= 4 && l > L) {
        L = l;
        c = p - 1;
      }
    }
    Ls[j] = min(L, ce - q);
    offs[j] = q - c;
  }
  // finish matches that filled the 8-byte window: 16 bytes per lane per step
  auto ext_step = [&](uint32_t q, uint32_t off, uint32_t lim, uint32_t& L, bool& more) {
    // five aligned dwords per side, four funnel shifts each
    const uint32_t avail = lim - L;
    const uint32_t a = q - off + L, b = q + L;
    const uint32_t* wa = reinterpret_cast<const uint32_t*>(data + (a & ~3u));
    const uint32_t* wb = reinterpret_cast<const uint32_t*>(data + (b & ~3u));
    const uint32_t sa = a & 3u, sb = b & 3u;
    uint32_t x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      x[k] = __builtin_amdgcn_alignbyte(wa[k + 1], wa[k], sa) ^ __builtin_amdgcn_alignbyte(wb[k + 1], wb[k], sb);
    const uint64_t lo = ((uint64_t)x[1] << 32) | x[0], hi = ((uint64_t)x[3] << 32) | x[2];
    const uint32_t fb = lo ? (uint32_t)(__builtin_ctzll(lo) >> 3) : (hi ? 8u + (uint32_t)(__builtin_ctzll(hi) >> 3) : 16u);
    L += min(fb, avail);
    more = fb == 16 && avail > 16;
  };
  auto ext_lim = [&](uint32_t q) { return SM_FAST_LCAP ? min(ce - q, (uint32_t)SM_FAST_LCAP) : ce - q; };
  if (kXCompact) {
    // The extensions of all four position groups are compacted into one list first (ballot
    // prefix into a per-wave LDS scratch: jump-table rows 1-4, free until the doubling), so
    // the step loop runs over full waves of jobs instead of four partly idle groups; the
    // lengths come back through row 5.
    uint32_t* jl = reinterpret_cast<uint32_t*>(jt + kRow);
    uint8_t* lr = jt + 5 * kRow;
    uint64_t JM[kP];
    uint32_t nj = 0;
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      const uint32_t q = c0 + 64 * j + lane;
      const bool need = !(SM_ABLATE & 8) && Ls[j] >= kVW && Ls[j] < ext_lim(q);  // then Ls[j] == kVW
      JM[j] = ballot(need);
      if (need)
        jl[nj + __builtin_amdgcn_mbcnt_hi((uint32_t)(JM[j] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)JM[j], 0u))] =
            (64 * j + lane) | (offs[j] << 8);
      nj += (uint32_t)__builtin_popcountll(JM[j]);
    }
    if (nj) {
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      for (uint32_t r0 = 0; r0 < nj; r0 += 64) {
        const bool act = r0 + lane < nj;
        const uint32_t d = jl[act ? r0 + lane : 0];
        const uint32_t pos = d & 0xffu, q = c0 + pos;
        const uint32_t lim = ext_lim(q);
        uint32_t L = kVW;
        bool more = act;
        while (ballot(more)) {
          if (more) ext_step(q, d >> 8, lim, L, more);
        }
        if (act) lr[pos] = (uint8_t)L;
      }
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
#pragma unroll
      for (int j = 0; j < kP; ++j)
        if ((JM[j] >> lane) & 1u) Ls[j] = lr[64 * j + lane];
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
    }
  } else {
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      const uint32_t q = c0 + 64 * j + lane;
      uint32_t L = Ls[j];
      const uint32_t lim = ext_lim(q);
      bool more = !(SM_ABLATE & 8) && L >= kVW && L < lim;
      while (ballot(more)) {
        if (more) ext_step(q, offs[j], lim, L, more);
      }
      Ls[j] = L;
    }
  }
  if (SM_ABLATE & 2) {
#pragma unroll
    for (int j = 0; j < kP; ++j) Ls[j] = 0;
  }
  // Greedy parse by pointer doubling (no serial loop) over the chunk's positions.  J0 skips
  // literal runs: J0[r] = the first match position >= r + L(r) (L = 0 for a non-match), else
  // kEnd, so the greedy walk from 0 steps only between copies; J_k = J_{k-1} o J_{k-1}.  Chain
  // element t of the chunk is then computed directly in lane t from the jump tables.  No
  // copies at all (incompressible): no parse.
  uint64_t M[kP];
  uint64_t any = 0;
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    M[j] = ballot(Ls[j] != 0);
    any |= M[j];
  }
  uint32_t nmatch = 0, last_end = 0;
  if (any) {
    // F[i]: the first match position in words > i (kEnd: none)
    uint32_t F[kP];
    F[kP - 1] = kEnd;
#pragma unroll
    for (int i = kP - 2; i >= 0; --i) F[i] = M[i + 1] ? 64u * (i + 1) + ctz64(M[i + 1]) : F[i + 1];
    uint32_t jv[kP];
    // NM[x] = the first match position >= x, for this lane's positions (register j is word
    // j of the masks, so no select); J0[r] = NM[r + L(r)]: NM goes to row 0, the match
    // positions gather NM at r + L (all reads issued before the row is overwritten; entry
    // kChunk holds kEnd) and store their J0.
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      const uint32_t rr = 64 * j + lane;
      const uint64_t m = M[j] >> lane;
      jv[j] = m ? rr + ctz64(m) : F[j];
      jt[rr] = (uint8_t)jv[j];
    }
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    uint32_t g[kP];
#pragma unroll
    for (int j = 0; j < kP; ++j) g[j] = jt[64 * j + lane + Ls[j]];  // L = 0: NM[r] itself
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      jv[j] = g[j];
      jt[64 * j + lane] = (uint8_t)jv[j];  // unchanged where L = 0
    }
#pragma unroll
    for (int kk = 1; kk < (int)kBuilt; ++kk) {
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
#pragma unroll
      for (int j = 0; j < kP; ++j) {
        jv[j] = jt[(kk - 1) * kRow + jv[j]];
        jt[kk * kRow + 64 * j + lane] = (uint8_t)jv[j];
      }
    }
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    // chain element t (lane t < kChunk/4) from position 0: J_k for every set bit k of t.
    // Only element 0 can be a non-match (J0 jumps to match positions), the rest are the
    // copies; past the last copy the chain sits at kEnd (no match).
    uint32_t c = 0;
#pragma unroll
    for (int kk = 0; kk < (int)kBuilt; ++kk) {
      const uint32_t tt = jt[kk * kRow + c];
      c = ((lane >> kk) & 1u) ? tt : c;
    }
    // lane t >= S = 2^kBuilt holds element t mod S: the lanes >= kS advance S steps (two
    // applications of the last level) while element kS - 1 is a copy, else they are past
    // the chain's end
#pragma unroll
    for (uint32_t kS = 1u << kBuilt; kS < 64; kS += 1u << kBuilt) {
      if (readlane(c, kS - 1) < kEnd) {
        if (lane >= kS) {
          c = jt[(kBuilt - 1) * kRow + c];
          c = jt[(kBuilt - 1) * kRow + c];
        }
      } else {
        c = lane >= kS ? kEnd : c;
        break;
      }
    }
    // the match at c is held by lane c mod 64 (register c / 64): full-wave shuffles of
    // length | offset << 9
    const uint32_t ci = c & 63u, cj = c >> 6;
    uint32_t vc = 0;
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      const uint32_t v = __shfl(Ls[j] | (offs[j] << 9), ci, 64);
      vc = cj == (uint32_t)j ? v : vc;
    }
    const uint32_t Lc = c < kEnd ? vc & 0x1ffu : 0u;
    const bool istok = lane < kChunk / 4 && Lc != 0;
    const uint64_t tm = ballot(istok);
    nmatch = (uint32_t)__builtin_popcountll(tm);
    const uint32_t sh = (uint32_t)(tm & 1u) ^ 1u;  // tokens start at lane 1 if 0 is no match
    if (nmatch) last_end = readlane(c + Lc, nmatch - 1 + sh);
    // token: position | length << 16; offset
    const uint32_t tav = __shfl(c | (Lc << 16), lane + sh, 64), tbv = __shfl(vc >> 9, lane + sh, 64);
    if (nmatch) {
      t.ta = tav;
      t.tb = tbv;
    }
    // copy-start bitmask (position p of the chunk) for the literal scatter
    if (lane < kP) tsw[lane] = 0;
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (istok)
      __hip_atomic_fetch_or(&tsw[c >> 6], 1ull << (c & 63u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
#pragma unroll
    for (int j = 0; j < kP; ++j) t.ts[j] = tsw[j];
    __atomic_signal_fence(__ATOMIC_SEQ_CST);  // the next chunk's jump tables follow these reads
  }
  t.ntok = nmatch;
  if (last_end < ce - c0) {  // trailing literal run: a token without a copy
    const bool me = lane == t.ntok;
    t.ta = me ? ce - c0 : t.ta;
    t.tb = me ? 0u : t.tb;
    ++t.ntok;
  }
  const uint32_t tq = c0 + (t.ta & 0xffff), tL = t.ta >> 16;
  const uint32_t end = tq + tL;
  const uint32_t prev_end = __builtin_amdgcn_update_dpp(0u, end, 0x138, 0xf, 0xf, false);  // wave_shr:1
  t.ls = lane == 0 ? c0 : prev_end;
  {  // selects, not a branch: lanes past the tokens get zeros
    const bool tok = lane < t.ntok;
    t.litlen = tok ? tq - t.ls : 0u;
    t.littag = lit_tag_bytes(t.litlen);
    t.sz = tok ? t.littag + t.litlen + (tL ? copy_bytes_cf(t.tb, tL) : 0u) : 0u;
  }
  t.incl = scan_dpp(t.sz);
  const uint32_t trail = ce - c0 - last_end;
  return readlane(t.incl, t.ntok - 1) | (readlane(t.litlen, 0) << 11) | (trail << 20) | ((nmatch == 0) << 29);
}

// Emission of a parsed chunk at output offset o0 (its place in the round): token lanes write
// tag bytes, position lanes scatter literal bytes.  mycont: the chunk's leading literal
// continues the previous chunk's run (its tag is dropped); myrun: the chunk's trailing run
// spans later chunks and its tag encodes that whole length.
__device__ inline void emit_chunk(uint8_t* dst, const uint8_t* data, const ChunkTok& t, uint32_t o0, uint32_t mycont,
                                  uint32_t myrun, uint32_t lane) {
  const uint32_t rm = mycont ? readlane(t.littag, 0) : 0u;  // leading tag removed
  const uint32_t tq = t.c0 + (t.ta & 0xffff), tL = t.ta >> 16;
  const uint32_t o = o0 + t.incl - t.sz - (lane > 0 ? rm : 0u);
  uint32_t mytag = (lane == 0 && mycont) ? 0u : t.littag, tagv = t.litlen;
  if (myrun && lane == t.ntok - 1) {  // the run's trailing token
    mytag = lit_tag_bytes(myrun);
    tagv = myrun;
  }
  const bool st_on = !(SM_ABLATE & 16) || dst == nullptr;  // ablation 16: no global stores (kept computation)
  if (lane < t.ntok && st_on) {
    put_lit_tag(dst, o, mytag, tagv);
    if (tL) put_copy_cf(dst, o + mytag + t.litlen, t.tb, tL);
  }
  const uint32_t delta = o + mytag - t.ls;  // output - input position of the run (mod 2^32)
  const uint32_t end = tq + tL;
  // all LDS reads (the literal bytes, the shuffles) of the four position groups are issued
  // before the first store, so their round trips overlap
  uint32_t below = 0, cnt[kP], pend[kP], dl[kP], v[kP];
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    v[j] = data[t.c0 + 64 * j + lane];  // inside the block area even past ce (not stored then)
    cnt[j] = below + __builtin_amdgcn_mbcnt_hi((uint32_t)(t.ts[j] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)t.ts[j], 0u));
    cnt[j] += (uint32_t)(t.ts[j] >> lane) & 1u;  // tokens whose copy starts at or before x
    below += __builtin_popcountll(t.ts[j]);
  }
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    pend[j] = __shfl(end, cnt[j] ? cnt[j] - 1 : 0, 64);
    dl[j] = __shfl(delta, cnt[j], 64);
  }
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    const uint32_t x = t.c0 + 64 * j + lane;
    // one mask (bitwise, so the compiler does not split it into nested branches)
    const bool lit = (x < t.ce) & ((cnt[j] == 0) | (x >= pend[j]));
    if (lit && st_on) dst[x + dl[j]] = (uint8_t)v[j];  // 32-bit offset: saddr store
  }
}

// Round layout, lane-parallel over the round's chunk slots (lane u = slot u): a literal run
// that crosses chunk boundaries inside the round is emitted once, with one tag for its total
// length in the chunk where it starts (runs restart at round boundaries).
//   cont_in[u]: chunk u's leading literal piece continues chunk u-1's trailing piece (no tag)
//   mid[u]:     chunk u is all literal and continues a run (no tag of its own)
//   start[u]:   chunk u's trailing piece starts a run; if cont_in[u+1] the run spans chunks
//               and its tag encodes the run length up to the end of the last piece.
struct RoundLayout {
  uint32_t inclm, Smv, contv, runv, total;
};
template <uint32_t kSlots>
__device__ inline RoundLayout round_layout(const uint32_t* cinfo, uint32_t r, uint32_t n, uint32_t lane) {
  uint32_t inclm, Smv, contv, runv, total;
  const uint32_t info = lane < kSlots ? cinfo[lane] : 0u;
  const uint32_t S = info & 0x7ffu, lead = (info >> 11) & 0x1ffu, trl = (info >> 20) & 0x1ffu;
  const bool nocp = (info >> 29) & 1u;
  const uint32_t trl_prev = __builtin_amdgcn_update_dpp(0u, trl, 0x138, 0xf, 0xf, false);  // wave_shr:1
  const bool cont_in = lane > 0 && lane < kSlots && trl_prev > 0 && lead > 0;
  const bool mid = nocp && cont_in;
  const bool start = trl > 0 && !mid;
  const bool cont_next = __builtin_amdgcn_update_dpp(0u, (uint32_t)cont_in, 0x130, 0xf, 0xf, false) != 0;  // wave_shl:1
  const uint32_t cu = (r * kSlots + lane) * kChunk;                      // chunk start
  const uint32_t ceu = min(cu + kChunk, n);
  // the run ending in chunk u ends at cu + lead; a run starting in chunk v ends in the
  // first later chunk whose piece ends it (suffix min over lanes)
  const bool ends = cont_in && !(mid && cont_next);
  uint32_t nxt = ends ? lane : 0xffu;
  if (kSlots < 16) {  // one DPP row
    nxt = min(nxt, (uint32_t)__builtin_amdgcn_update_dpp(0xffu, nxt, 0x101, 0xf, 0xf, false));  // row_shl:1
    nxt = min(nxt, (uint32_t)__builtin_amdgcn_update_dpp(0xffu, nxt, 0x102, 0xf, 0xf, false));  // row_shl:2
    nxt = min(nxt, (uint32_t)__builtin_amdgcn_update_dpp(0xffu, nxt, 0x104, 0xf, 0xf, false));  // row_shl:4
    nxt = min(nxt, (uint32_t)__builtin_amdgcn_update_dpp(0xffu, nxt, 0x108, 0xf, 0xf, false));  // row_shl:8
  } else {
#pragma unroll
    for (uint32_t d = 1; d < kSlots; d <<= 1) {
      const uint32_t o2 = __shfl_down(nxt, d, 64);
      nxt = (lane + d < kSlots && o2 < nxt) ? o2 : nxt;
    }
  }
  nxt = __builtin_amdgcn_update_dpp(0xffu, nxt, 0x130, 0xf, 0xf, false);                       // first end after u
  const uint32_t endpos = __shfl(cu + lead, nxt & 63u, 64);
  const uint32_t runlen = (start && cont_next) ? endpos - (ceu - trl) : 0u;
  const uint32_t Sm = S - (cont_in ? lit_tag_bytes(lead) : 0u) +
                      (runlen ? lit_tag_bytes(runlen) - lit_tag_bytes(trl) : 0u);
  inclm = scan_dpp(lane < kSlots ? Sm : 0u);
  total = readlane(inclm, kSlots - 1);
  Smv = Sm;
  contv = cont_in;
  runv = runlen;
  return RoundLayout{inclm, Smv, contv, runv, total};
}

template <int D>
constexpr size_t fast_lds() {
  return kBlockSize + kTabBytes + Cfg<D>::kRingBytes + 4 * 64 + kWavesPerBlock * kLevels * kRow + kWavesPerBlock * 8 * kP;
}
static_assert(fast_lds<1>() <= 160 * 1024 && fast_lds<2>() <= 160 * 1024, "fast compressor LDS exceeds a CU");

template <int kDepth>
__global__ __launch_bounds__(kThreads) void k_compress_fast(CompressArgs a) {
  typedef Cfg<kDepth> C;
  typedef typename C::Cand Cand;
  constexpr uint32_t kSlots = C::kSlots, kRP = C::kRoundPos;
  // static LDS: every address is a link-time constant (a dynamic allocation's base costs a
  // v_add of its relocated 0 on every access)
  __shared__ __attribute__((aligned(16))) uint8_t smem[fast_lds<kDepth>()];
  // The block sits at LDS offset 0, so a chain candidate (a position) is its own byte address;
  // the table follows it (a bucket's address is one v_lshl_add).
  uint8_t* data = smem;                                                     // 64 KiB block
  uint32_t* T = reinterpret_cast<uint32_t*>(smem + kBlockSize);             // hash table
  Cand* ring = reinterpret_cast<Cand*>(smem + kBlockSize + kTabBytes);      // 2 x kRoundPos candidates
  uint32_t* csize = reinterpret_cast<uint32_t*>(ring + 2 * kRP);            // 2 x 32 chunk infos
  const uint32_t tid = threadIdx.x;
  const uint32_t wave = uniform(tid >> 6);
  const uint32_t lane = tid & 63;
  const bool inserter = wave == kPW;
  // per-wave jump tables and copy-start bitmasks (the inserter's are used in the final round)
  uint8_t* jt = reinterpret_cast<uint8_t*>(csize + 64) + wave * kLevels * kRow;
  uint64_t* tsw = reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(csize + 64) + kWavesPerBlock * kLevels * kRow) +
                  wave * kP;

  const uint32_t b = blockIdx.x;
  if (a.screened && a.out_len[b] != kScreenTodo) return;  // emitted as one literal by k_literal_screen
  const uint32_t n = a.in_len[b];
  const uint8_t* src = a.in + a.in_off[b];
  uint8_t* dst = a.out + a.out_off[b];
  if (n > kBlockSize) {
    if (tid == 0) a.out_len[b] = 0xffffffffu;
    return;
  }

  // stage the block: all 16 B loads of a thread in flight when aligned
  if (((uintptr_t)src & 15) == 0) {
    const uint4* s16 = reinterpret_cast<const uint4*>(src);
    uint4* d16 = reinterpret_cast<uint4*>(data);
    const uint32_t n16 = n >> 4;
    if (n16 == kBlockSize / 16) {
      constexpr int kLoads = kBlockSize / 16 / kThreads;
      uint4 v[kLoads];
#pragma unroll
      for (int i = 0; i < kLoads; ++i) v[i] = s16[tid + i * kThreads];
#pragma unroll
      for (int i = 0; i < kLoads; ++i) d16[tid + i * kThreads] = v[i];
    } else {
      for (uint32_t k = tid; k < n16; k += kThreads) d16[k] = s16[k];
      for (uint32_t k = (n & ~15u) + tid; k < n; k += kThreads) data[k] = src[k];
    }
  } else {
    for (uint32_t k = tid; k < n; k += kThreads) data[k] = src[k];
  }
  {
    const uint4 z = make_uint4(0, 0, 0, 0);
    uint4* t16 = reinterpret_cast<uint4*>(T);
    for (uint32_t k = tid; k < kTabBytes / 16; k += kThreads) t16[k] = z;  // 0 = no position
  }
  if (kEnd == kChunk && lane < kLevels) jt[lane * kRow + kChunk] = (uint8_t)kChunk;
  if (lane == 0) jt[kChunk] = (uint8_t)kEnd;  // NM past the chunk: no match
  uint32_t op = 0;
  if (a.header) {
    uint32_t nb = varint_len(n);
    if (tid < nb) dst[tid] = (uint8_t)(((n >> (7 * tid)) & 0x7f) | (tid + 1 < nb ? 0x80 : 0));
    op = nb;
  }
  __syncthreads();

  const uint32_t nchunks = (n + kChunk - 1) / kChunk;
  const uint32_t rounds = (nchunks + kSlots - 1) / kSlots;
  // hashes of rounds 0 and 1 (the ring's two halves) by every wave; later rounds' hashes are
  // written by the parse waves into the slots whose candidates they have just read
  for (uint32_t g = wave; g < 2 * kRP / 64 && 64 * g < n; g += kWavesPerBlock) hash_group(data, ring + 64 * g, 64 * g, lane);
  __syncthreads();
  // the inserter shares a SIMD with three parse waves and gates every round: issue it first
  if (inserter && SM_FAST_PRIO) __builtin_amdgcn_s_setprio(SM_FAST_PRIO);
  if (inserter) insert_round<kDepth>(T, ring, 0, n, lane);
  __syncthreads();

  STAMP_DECL
  for (uint32_t r = 0; r < rounds; ++r) {
#if SM_FAST_XBAR
    __syncthreads();
#endif
    uint32_t* cinfo = csize + (r & 1) * 32;
    ChunkTok tk[C::kCPW];
    // The final round has nothing left to insert.  A full 64 KiB block's final round holds 16
    // chunks (256 = 8 x 30 + 16), so without help parse wave 0 takes slots 0 and 15 and the
    // round lasts as long as a full one; the idle inserter parses slot kPW instead, and the
    // round takes one chunk's time.  Wave 0 hands it the output offset (csize[63] is spare:
    // chunk infos use csize[0..kSlots) of each half) before the round's barrier.
    const bool ins_parse = SM_FAST_LASTINS && kSlots > kPW && r + 1 == rounds;
    if (ins_parse && wave == 0 && lane == 0) csize[63] = op;
    if (inserter && !ins_parse) {
      insert_round<kDepth>(T, ring + ((r + 1) & 1) * kRP, (r + 1) * kRP, n, lane);
      STAMP(8)
      STAMP_COUNT(10, 1)
    } else {
      // parse wave w owns the round's chunk slots w, w + 15, ...
#pragma unroll
      for (int u = 0; u < C::kCPW; ++u) {
        const uint32_t slot = inserter ? kPW : wave + kPW * u;
        const bool mine = inserter ? u == 0 : !(ins_parse && slot == kPW);
        const uint32_t k = r * kSlots + slot;
        const uint32_t c0 = k * kChunk;
        if (SM_FAST_PPRIO && u == 0 && !inserter) __builtin_amdgcn_s_setprio(1);
        if (SM_FAST_PPRIO && u == 1 && !inserter) __builtin_amdgcn_s_setprio(0);
        if (!mine) {
          tk[u].c0 = tk[u].ce = c0;  // parsed (and its chunk info written) by the other wave
        } else if (k < nchunks && (SM_ABLATE & 4)) {  // diagnostic: hashes only (the inserter needs them)
          Cand* cr = ring + (r & 1) * kRP + slot * kChunk;
          if (k + 2 * kSlots < nchunks) {
#pragma unroll
            for (int j = 0; j < kP; ++j) hash_group(data, cr + 64 * j, c0 + 2 * kRP + 64 * j, lane);
          }
          tk[u].c0 = tk[u].ce = c0;
          if (lane == 0) cinfo[slot] = 0;
        } else if (k < nchunks) {
          STAMP_COUNT(11, 1)
          Cand* cr = ring + (r & 1) * kRP + slot * kChunk;
          uint32_t cv[kP];
#pragma unroll
          for (int j = 0; j < kP; ++j) cv[j] = cr[64 * j + lane];
          // the same slot of round r + 2 (this ring half's next use): its hashes, in place
          // (the reads above are this lane's, and a wave's LDS instructions run in order)
          if (k + 2 * kSlots < nchunks) {
#pragma unroll
            for (int j = 0; j < kP; ++j) hash_group(data, cr + 64 * j, c0 + 2 * kRP + 64 * j, lane);
          }
          const uint32_t info = parse_chunk<kDepth>(data, cv, jt, tsw, c0, min(c0 + kChunk, n), n, lane, tk[u]);
          if (lane == 0) cinfo[slot] = info;
        } else {
          tk[u].c0 = tk[u].ce = c0;
          if (lane == 0) cinfo[slot] = 0;
        }
      }
      STAMP(3)
    }
    __syncthreads();  // the round's chunk infos; the next round's candidates
    if (inserter && !ins_parse) {
      STAMP(9)
      continue;
    }
    if (inserter) op = csize[63];
    STAMP(4)
    if (SM_FAST_PPRIO) __builtin_amdgcn_s_setprio(2);

    // (c) round layout (round_layout), then the emission
    const RoundLayout lay = round_layout<kSlots>(cinfo, r, n, lane);
    const uint32_t inclm = lay.inclm, Smv = lay.Smv, contv = lay.contv, runv = lay.runv, total = lay.total;
    STAMP(5)
    if (!(SM_ABLATE & 1)) {
#pragma unroll
      for (int u = 0; u < C::kCPW; ++u) {
        const uint32_t slot = inserter ? kPW : wave + kPW * u;
        if (tk[u].ce > tk[u].c0)
          emit_chunk(dst, data, tk[u], op + readlane(inclm - Smv, slot), readlane(contv, slot), readlane(runv, slot), lane);
      }
    }
    STAMP(6)
    op += total;
  }
  STAMP(7)
  STAMP_FLUSH(g_stamp_c)
#if SM_STAMP
  if (lane == 0) atomicAdd(&g_stamp_w[wave], (unsigned long long)(inserter ? st_acc[9] : st_acc[4]));
#endif
  if (tid == 0) a.out_len[b] = op;
}

#if SM_STAMP
extern "C" int sm_debug_stamps_c(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamp_c), sizeof(g_stamp_c)) != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out + 12, HIP_SYMBOL(g_stamp_w), sizeof(g_stamp_w)) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_c), z, sizeof(g_stamp_c)) != hipSuccess) return -1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_w), z, sizeof(g_stamp_w)) != hipSuccess) return -1;
  }
  return 0;
}
#endif



// ---- incompressible screen ---------------------------------------------------------------
// Before the parse, one light workgroup per block looks for repeated content anywhere in the block
// through content-defined anchors: the positions whose 4-byte word hashes into the top 1/64 of the
// hash range (the reference's multiply, internal.jl:94).  Repeated content repeats its anchors at
// any distance, so a block counts the anchors whose word an earlier-inserted anchor already had
// (an LDS table of 4 K words, exchanged).  Text and structured data count hundreds; random,
// compressed and encrypted data count ~0.  The first 8 KiB go first (text decides there); the rest
// of the block is read only when they show no repeats.  Below kScrMin the block is emitted here as
// ONE literal (header, emit_literal! tag, the bytes: internal.jl:271-284 -- the reference's own
// output for random 64 KiB blocks is also one 65,542-B literal) from the registers that read it,
// with aligned 16-B stores: an incompressible block is read once and written once.  The parse
// kernel then skips it.  This is the batch analogue of the reference's skip heuristic
// (internal.jl:162-175).  The bet only costs ratio, never validity: a literal encodes any bytes,
// and a block with fewer than kScrMin repeated anchors has ~kScrMin x 64 B of repeats at most.
constexpr uint32_t kScrMin = 8;           // repeated anchors that make a block "compressible"
constexpr uint32_t kScrMinLen = 8192;     // smaller blocks always take the parse
constexpr uint32_t kScrThreads = 512;
constexpr uint32_t kScrPieces = kBlockSize / 16 / kScrThreads;  // 16-B pieces per thread (8)
constexpr uint32_t kScrFirst = 1;                               // pieces of the first pass (8 KiB)
constexpr uint32_t kScrTabBits = 12;
constexpr uint32_t kScrEmpty = 0xffffffffu;  // its hash is no anchor, so no anchor word equals it
static_assert(((kScrEmpty * kHashMul) >> 26) != 0, "the empty mark must not be an anchor word");

// 16 bytes of src at o (any alignment of src), zero past n
__device__ inline uint4 scr_load16(const uint8_t* src, uint32_t o, uint32_t n, bool aligned) {
  if (aligned && o + 16 <= n) return *reinterpret_cast<const uint4*>(src + o);
  uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
  for (uint32_t k = 0; k < 16; ++k)
    if (o + k < n) w[k >> 2] |= (uint32_t)src[o + k] << (8 * (k & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// repeated anchors among the 16 positions of a piece v (bytes [o, o + 16)), nv = the next piece
// (valid = its first 3 bytes are real: the positions 13..15 have their 4 bytes)
__device__ inline uint32_t scr_anchors(uint32_t* tab, uint4 v, uint4 nv, uint32_t o, uint32_t n, bool nvalid) {
  const uint32_t x[5] = {v.x, v.y, v.z, v.w, nv.x};
  uint32_t rep = 0;
#pragma unroll
  for (uint32_t j = 0; j < 16; ++j) {
    const uint32_t w = (j & 3) ? __builtin_amdgcn_alignbyte(x[(j >> 2) + 1], x[j >> 2], j & 3) : x[j >> 2];
    const uint32_t h = w * kHashMul;
    const bool ok = o + j + 4 <= n && (j < 13 || nvalid);
    if (ok && (h >> 26) == 0) {
      const uint32_t old = atomicExch(&tab[(h >> 14) & ((1u << kScrTabBits) - 1)], w);
      rep += old == w ? 1u : 0u;
    }
  }
  return rep;
}

__global__ __launch_bounds__(kScrThreads) void k_literal_screen(CompressArgs a) {
  __shared__ uint32_t tab[1u << kScrTabBits];
  __shared__ uint32_t cnt[2];
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const uint32_t b = blockIdx.x;
  const uint32_t n = a.in_len[b];
  const uint8_t* src = a.in + a.in_off[b];
  uint8_t* dst = a.out + a.out_off[b];
  if (n < kScrMinLen || n > kBlockSize) {
    if (tid == 0) a.out_len[b] = kScreenTodo;
    return;
  }
  const bool aligned = ((uintptr_t)src & 15) == 0;
  for (uint32_t k = tid; k < (1u << kScrTabBits); k += kScrThreads) tab[k] = kScrEmpty;
  if (tid < 2) cnt[tid] = 0;
  uint4 v[kScrPieces];
#pragma unroll
  for (uint32_t i = 0; i < kScrPieces; ++i) v[i] = make_uint4(0, 0, 0, 0);
  // piece i of thread t: bytes [16 (t + 512 i), +16); lane + 1 holds the next piece (a wave's last
  // lane: its positions 13..15 are skipped -- 3 of every 1,024)
  auto pass = [&](uint32_t i0, uint32_t i1, uint32_t slot) {
#pragma unroll
    for (uint32_t i = i0; i < i1; ++i) v[i] = scr_load16(src, 16 * (tid + kScrThreads * i), n, aligned);
    __syncthreads();  // (the table is initialised)
    uint32_t rep = 0;
#pragma unroll
    for (uint32_t i = i0; i < i1; ++i) {
      uint4 nv;
      nv.x = __builtin_amdgcn_update_dpp(0u, v[i].x, 0x130, 0xf, 0xf, false);  // wave_shl:1
      rep += scr_anchors(tab, v[i], nv, 16 * (tid + kScrThreads * i), n, lane < 63);
    }
    rep = __builtin_amdgcn_readlane(scan_dpp(rep), 63);
    if (lane == 0 && rep) atomicAdd(&cnt[slot], rep);
    __syncthreads();
  };
  pass(0, kScrFirst, 0);
  if (cnt[0] >= kScrMin) {  // text and structured data decide on their first 8 KiB
    if (tid == 0) a.out_len[b] = kScreenTodo;
    return;
  }
  if (n > 16 * kScrThreads * kScrFirst) pass(kScrFirst, kScrPieces, 1);
  if (cnt[0] + cnt[1] >= kScrMin) {
    if (tid == 0) a.out_len[b] = kScreenTodo;
    return;
  }
  // literal-only stream from the registers: D[j] = src[j - h] for j >= h.  Piece p (source bytes
  // [16p, 16p + 16)) makes the aligned output unit that starts m bytes into it, m = -(ad + h) mod
  // 16, from its bytes and the next piece's (lane + 1; a wave's last lane reloads it).  The partial
  // units at either end are written byte by byte.
  const uint32_t hv0 = a.header ? varint_len(n) : 0u;
  const uint32_t h = hv0 + literal_tag_bytes(n);
  const uint32_t ad = (uint32_t)((uintptr_t)dst & 15);
  const uint32_t m = (16u - ((ad + h) & 15u)) & 15u;
  uint4* d16 = reinterpret_cast<uint4*>(dst - ad);
  const uint32_t u_of_p0 = (m + ad + h) >> 4;  // the unit of piece 0
  const uint32_t dw = m >> 2, bs = m & 3u;
#pragma unroll
  for (uint32_t i = 0; i < kScrPieces; ++i) {
    const uint32_t p = tid + kScrThreads * i;
    const bool full = 16 * p + m + 16 <= n;
    uint4 nv;
    nv.x = __builtin_amdgcn_update_dpp(0u, v[i].x, 0x130, 0xf, 0xf, false);
    nv.y = __builtin_amdgcn_update_dpp(0u, v[i].y, 0x130, 0xf, 0xf, false);
    nv.z = __builtin_amdgcn_update_dpp(0u, v[i].z, 0x130, 0xf, 0xf, false);
    nv.w = __builtin_amdgcn_update_dpp(0u, v[i].w, 0x130, 0xf, 0xf, false);
    if (lane == 63 && full && m != 0) nv = scr_load16(src, 16 * (p + 1), n, aligned);
    if (full) {
      const uint32_t x[8] = {v[i].x, v[i].y, v[i].z, v[i].w, nv.x, nv.y, nv.z, nv.w};
      uint32_t r[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) {  // x[dw + k], selects (no dynamic register indexing)
        uint32_t t = x[k];
#pragma unroll
        for (int d = 1; d < 4; ++d) t = dw == (uint32_t)d ? x[k + d] : t;
        r[k] = t;
      }
      d16[u_of_p0 + p] = make_uint4(__builtin_amdgcn_alignbyte(r[1], r[0], bs), __builtin_amdgcn_alignbyte(r[2], r[1], bs),
                                    __builtin_amdgcn_alignbyte(r[3], r[2], bs), __builtin_amdgcn_alignbyte(r[4], r[3], bs));
    }
  }
  // the head: header + source bytes [0, m); the tail: source bytes past the last full unit
  const uint32_t nfull = n >= m + 16 ? (n - m) / 16 : 0u;
  const uint32_t headEnd = h + min(m, n);             // D bytes [0, headEnd)
  const uint32_t tailBeg = nfull ? h + m + 16 * nfull : headEnd;  // D bytes [tailBeg, h + n)
  const uint32_t nh = headEnd, nt = h + n - tailBeg;
  for (uint32_t j = tid; j < nh + nt; j += kScrThreads) {
    const uint32_t jj = j < nh ? j : tailBeg + (j - nh);
    uint8_t c;
    if (jj < hv0) {
      c = (uint8_t)(((n >> (7 * jj)) & 0x7f) | (jj + 1 < hv0 ? 0x80 : 0));
    } else if (jj < h) {  // emit_literal! tag: 60..63 << 2 then len-1 little-endian
      const uint32_t tb = h - hv0, k = jj - hv0;
      c = tb == 1 ? (uint8_t)((n - 1) << 2) : (k == 0 ? (uint8_t)((58 + tb) << 2) : (uint8_t)((n - 1) >> (8 * (k - 1))));
    } else {
      c = src[jj - h];
    }
    dst[jj] = c;
  }
  if (tid == 0) a.out_len[b] = h + n;
}

template <int D>
static hipError_t launch_depth(const CompressArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_compress_fast<D>, dim3(a.nblk), dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

// mode 1 (SM_MODE_FAST): one chain candidate per position; mode 2 (SM_MODE_FAST_DENSE): two.
// The screen runs first; the parse kernel compresses the blocks it marks kScreenTodo.
hipError_t launch_compress_fast(const CompressArgs& a0, int mode, hipStream_t s) {
  CompressArgs a = a0;
  a.screened = 1;
  hipLaunchKernelGGL(k_literal_screen, dim3(a.nblk), dim3(kScrThreads), 0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  static const int old = [] {
    const char* v = getenv("SM_FAST_OLD");
    return v ? atoi(v) : 0;
  }();
  if (!old) return launch_compress_sc(a, mode, s);
  return mode == 2 ? launch_depth<2>(a, s) : launch_depth<1>(a, s);
}

}  // namespace sm
