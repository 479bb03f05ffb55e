// sm_compress_fast.hip -- "fast mode" batched snappy compression for gfx950 (MI355X).
//
// Produces a valid snappy stream per <= 64 KiB block (decodes bit-exactly under Snappy.jl's
// uncompress, src/internal.jl:411-466) with a wave-parallel parse instead of the reference's
// serial greedy loop (internal.jl:127-250).
//
// One workgroup of W = 16 waves per block (four per SIMD, to hide the chain of LDS round
// trips); the block is staged once in LDS (64 KiB) beside a shared 16 K-entry latest-position
// table (u32, 64 KiB), a 128-entry u64 private table per wave (16 KiB) and 5-level parse jump
// tables (10 KiB): 154 KiB, one block per CU.  The block is cut into 128-byte chunks whose
// parse never crosses the chunk end (copies are truncated there, literal runs end there), so
// the chunks of a round are parsed independently: in round r wave w owns chunk W*r+w, two
// positions per lane (q = c0 + 64*j + lane).  Per chunk:
//  1. (a) insert every position into the shared table with ds_max_u32 (order-independent ->
//     deterministic) and into the wave's private table with ds_max_rtn_u32, whose return is
//     the latest EARLIER position of the chunk with the same 7-bit hash (lanes of one
//     instruction are serialised in ascending order on gfx950; verified, see tools/probe_lds);
//  2. (b) two candidates per position: A = that intra-chunk position, else the shared
//     table after the round (if it is an earlier position); B = the shared table as of the
//     previous round.  Both verified (4 bytes) and extended 16 bytes branch-free with unaligned
//     ds_read_b64; the longer one wins;
//  3. greedy parse by pointer doubling over the chunk (J_k = J_{k-1} o J_{k-1}, binary
//     descent); the visited copies are compacted into token lanes; sizes in closed form,
//     DPP wave scan, chunk sizes exchanged through LDS -> exact output offsets;
//  4. (c) token lanes write tag bytes; position lanes scatter literal bytes.
// Two barriers per round.  Output is deterministic (no order-dependent table state).
#include "sm_device.h"
#include "sm_internal.h"

#ifndef SM_ABLATE  // diagnostic builds only (tools/ablate.sh): 1 no emit, 2 no matches, 4 no inserts
#define SM_ABLATE 0
#endif

namespace sm {

#if SM_STAMP
__device__ unsigned long long g_stamp_c[12];
#endif
STAMP_MACROS(12)

constexpr uint32_t kFTabBits = 14;
constexpr uint32_t kFTab = 1u << kFTabBits;   // shared table entries
constexpr uint32_t kPrivBits = 7;
constexpr uint32_t kPriv = 1u << kPrivBits;   // private (intra-chunk) table entries per wave
// A private entry is u64 (pos+1) << 32 | the 4 bytes at pos: ds_max still orders by position,
// and a candidate taken from it is verified in registers, with no data read.
constexpr uint32_t kChunk = 128;
#ifndef SM_FAST_WAVES
#define SM_FAST_WAVES 16
#endif
constexpr uint32_t kWavesPerBlock = SM_FAST_WAVES;  // 16: four waves per SIMD hide the LDS latency chain
constexpr uint32_t kThreads = 64 * kWavesPerBlock;
constexpr uint32_t kLevels = 5;              // J0..J4: the copy-to-copy walk of a chunk takes <= 31 steps
constexpr uint32_t kRow = kChunk + 8;        // a jump-table row (8-B aligned); entry kChunk, the chunk end, is its own image
constexpr uint32_t kEager = 16;               // bytes compared per candidate before the long-match loop
#ifndef SM_FAST_NBR
#define SM_FAST_NBR 6
#endif
constexpr uint32_t kNbr = SM_FAST_NBR;       // earlier chunks of the round probed for candidate C

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
  uint32_t k = L >= 68 ? ((L - 68) >> 6) + 1 : 0;
  uint32_t R = L - (k << 6);
  uint32_t e = R > 64 ? 1 : 0;
  R -= 60 * e;
  return 3 * (k + e) + ((R < 12 && off < 2048) ? 2 : 3);
}

// emit_copy! bytes (internal.jl:289-329) for L <= 128 (at most one 64-piece)
__device__ inline void put_copy_cf(uint8_t* dst, uint32_t o, uint32_t off, uint32_t L) {
  const uint8_t lo = (uint8_t)off, hi = (uint8_t)(off >> 8);
  if (L >= 68) {
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

__global__ __launch_bounds__(kThreads) void k_compress_fast(CompressArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* data = smem;                                                       // 64 KiB block
  uint32_t* T = reinterpret_cast<uint32_t*>(smem + kBlockSize);               // shared table
  const uint32_t tid = threadIdx.x;
  const uint32_t wave = uniform(tid >> 6);
  const uint32_t lane = tid & 63;
  uint64_t* P = reinterpret_cast<uint64_t*>(T + kFTab) + wave * kPriv;       // private table
  uint32_t* csize = T + kFTab + 2 * kWavesPerBlock * kPriv;                   // per-wave chunk sizes
  uint8_t* jt = reinterpret_cast<uint8_t*>(csize + kWavesPerBlock) + wave * kLevels * kRow;  // parse jump tables

  const uint32_t b = blockIdx.x;
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
    // shared table: 0 = empty; private entries: position field 0 (empty, below every insert)
    // and an all-ones word, so a probe matches an empty entry only for the word 0xffffffff
    // and then yields the rejected position 0xffffffff
    const uint4 z = make_uint4(0, 0, 0, 0), e = make_uint4(0xffffffffu, 0, 0xffffffffu, 0);
    uint4* t16 = reinterpret_cast<uint4*>(T);
    for (uint32_t k = tid; k < kFTab / 4; k += kThreads) t16[k] = z;
    for (uint32_t k = kFTab / 4 + tid; k < (kFTab + 2 * kWavesPerBlock * kPriv) / 4; k += kThreads) t16[k] = e;
  }
  if (lane < kLevels) jt[lane * kRow + kChunk] = (uint8_t)kChunk;
  uint32_t op = 0;
  if (a.header) {
    uint32_t nb = varint_len(n);
    if (tid < nb) dst[tid] = (uint8_t)(((n >> (7 * tid)) & 0x7f) | (tid + 1 < nb ? 0x80 : 0));
    op = nb;
  }
  __syncthreads();

  const uint32_t nchunks = (n + kChunk - 1) / kChunk;
  const uint32_t rounds = (nchunks + kWavesPerBlock - 1) / kWavesPerBlock;

  uint64_t w[2];  // the 8 bytes at each position
  uint32_t t1[2];
  {
    const uint32_t c0 = wave * kChunk;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      uint32_t q = c0 + 64 * j + lane;
      w[j] = lds_ld64(data, q < n ? q : 0);
      t1[j] = 0;
    }
  }

  STAMP_DECL
  for (uint32_t r = 0; r < rounds; ++r) {
    STAMP_COUNT(11, 1)
    const uint32_t k = r * kWavesPerBlock + wave;
    const bool active = k < nchunks;
    const uint32_t c0 = k * kChunk;
    const uint32_t ce = active ? min(c0 + kChunk, n) : c0;

    // (a) inserts
    uint64_t pin[2] = {0, 0};
    if (active && !(SM_ABLATE & 4)) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint32_t q = c0 + 64 * j + lane;
        const uint32_t hm = (uint32_t)w[j] * kHashMul;
        if (q + 4 <= n) {
          __hip_atomic_fetch_max(&T[hm >> (32 - kFTabBits)], q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          pin[j] = __hip_atomic_fetch_max(&P[hm >> (32 - kPrivBits)], ((uint64_t)(q + 1) << 32) | (uint32_t)w[j],
                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
    }
    STAMP(0)
    __syncthreads();  // B1
    STAMP(1)

    // (b) candidates, verify, extend, walk, sizes
    uint32_t ta = 0, tb = 0, ntok = 0, incl = 0, sz = 0, litlen = 0, littag = 0, ls = 0;
    uint64_t ts0 = 0, ts1 = 0;
    if (active) {
      // Candidates per position: A = the latest earlier position of the chunk with the same
      // 7-bit hash (ds_max_rtn above), B = the shared table as of the previous round, C = the
      // nearest earlier chunk of this round (waves wave-1..wave-kNbr) whose private table holds
      // a 4-byte match (the positions the round-lagged shared table misses).  The longest
      // match wins (ties: A, B, C).
      uint32_t Ls[2], offs[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint32_t q = c0 + 64 * j + lane;
        const bool can = q + 4 <= ce;
        const uint64_t wq = w[j];
        const uint32_t pa = (uint32_t)(pin[j] >> 32);
        const bool oka = pa > c0 && (uint32_t)pin[j] == (uint32_t)wq;  // an earlier chunk position
        const uint32_t ca = oka ? pa - 1 : q;
        const uint32_t cb = t1[j] != 0 ? t1[j] - 1 : q;
        uint32_t cc = q;
        if (kNbr) {
          // wave w-m's table; for m > w the index wraps to a later chunk of the round, whose
          // positions fail cc < q below and whose older entries are genuine earlier matches
          const uint32_t hp = ((uint32_t)wq * kHashMul) >> (32 - kPrivBits);
          const uint64_t* P0 = reinterpret_cast<const uint64_t*>(T + kFTab);
          uint64_t v[kNbr ? kNbr : 1];
#pragma unroll
          for (uint32_t m = 1; m <= kNbr; ++m) v[m - 1] = P0[((wave - m) & (kWavesPerBlock - 1)) * kPriv + hp];
#pragma unroll
          for (int m = (int)kNbr; m >= 1; --m)
            cc = (uint32_t)v[m - 1] == (uint32_t)wq ? (uint32_t)(v[m - 1] >> 32) - 1 : cc;
        }
        // verify 4 bytes, then grow to 8 and 16; every read is masked to the lanes still
        // matching (an LDS access costs by its active lanes)
        const uint32_t cand[3] = {ca, cb, cc};
        uint32_t len[3];
        len[0] = (can && oka) ? 4u : 0u;                                   // verified by its entry
        len[1] = (can && cb < q && cb != ca && lds_ld32(data, cb) == (uint32_t)wq) ? 4u : 0u;
        len[2] = (can && cc < q && cc != ca && cc != cb) ? 4u : 0u;  // verified by the probe
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          if (len[i]) {
            const uint32_t x = lds_ld32(data, cand[i] + 4) ^ (uint32_t)(wq >> 32);
            len[i] = x ? 4 + ((uint32_t)__builtin_ctz(x) >> 3) : 8u;
          }
        }
        if (len[0] == 8 || len[1] == 8 || len[2] == 8) {
          const uint64_t wq2 = lds_ld64(data, q + 8);
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            if (len[i] == 8) {
              const uint64_t x = lds_ld64(data, cand[i] + 8) ^ wq2;
              len[i] = x ? 8 + (uint32_t)(__builtin_ctzll(x) >> 3) : 16u;
            }
          }
        }
        uint32_t L = len[0], c = ca;
#pragma unroll
        for (int i = 1; i < 3; ++i) {
          c = len[i] > L ? cand[i] : c;
          L = len[i] > L ? len[i] : L;
        }
        L = min(L, ce - q);
        Ls[j] = (SM_ABLATE & 2) ? 0u : L;
        offs[j] = q - c;
      }
      STAMP(2)
      // finish matches that filled the eager window: 8 bytes per lane per step
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint32_t q = c0 + 64 * j + lane;
        uint32_t L = Ls[j];
        bool more = L >= kEager && q + L < ce;
        while (ballot(more)) {
          if (more) {
            const uint32_t avail = ce - q - L;
            const uint64_t x = lds_ld64(data, q - offs[j] + L) ^ lds_ld64(data, q + L);
            const uint32_t fb = x ? (uint32_t)(__builtin_ctzll(x) >> 3) : 8u;
            L += min(fb, avail);
            more = fb == 8 && avail > 8;
          }
        }
        Ls[j] = L;
      }
      STAMP(3)
      // Greedy parse by pointer doubling (no serial loop) over the chunk's 128 positions.
      // J0 skips literal runs: J0[r] = the first match position >= r + L(r) (L = 0 for a
      // non-match), else the chunk end, so the greedy walk from 0 steps only between copies
      // (<= 32 copies of >= 4 bytes: 31 steps); J_k = J_{k-1} o J_{k-1}, k < 5.  Copy t of the
      // chunk is then computed directly in lane t from the jump tables.
      // no copies at all (incompressible): skip the parse
      const uint64_t M0 = ballot(Ls[0] != 0), M1 = ballot(Ls[1] != 0);
      uint32_t nmatch = 0, last_end = 0;
      if (M0 | M1) {
        uint32_t jv[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const uint32_t r = 64 * j + lane;
          const uint32_t x = r + Ls[j];  // <= 128: copies end inside the chunk
          const uint64_t m0 = x < 64 ? M0 >> x : 0;
          const uint64_t m1 = x < 64 ? M1 : (x < 128 ? M1 >> (x - 64) : 0);
          const uint32_t b1 = x < 64 ? 64u : x;
          jv[j] = m0 ? x + (uint32_t)__builtin_ctzll(m0) : (m1 ? b1 + (uint32_t)__builtin_ctzll(m1) : kChunk);
          jt[r] = (uint8_t)jv[j];
        }
#pragma unroll
        for (int k = 1; k < (int)kLevels; ++k) {
          __atomic_signal_fence(__ATOMIC_SEQ_CST);
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            jv[j] = jt[(k - 1) * kRow + jv[j]];
            jt[k * kRow + 64 * j + lane] = (uint8_t)jv[j];
          }
        }
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        // chain element t (lane t < 32) from position 0: J_k for every set bit k of t.  Only
        // element 0 can be a non-match (J0 jumps to match positions), the rest are the copies.
        uint32_t c = 0;
#pragma unroll
        for (int k = 0; k < (int)kLevels; ++k) {
          const uint32_t t = jt[k * kRow + c];
          c = ((lane >> k) & 1u) ? t : c;
        }
        // the match at c is held by lane c mod 64 (register c / 64): full-wave shuffles
        const uint32_t ci = c & 63u;
        const uint32_t l0 = __shfl(Ls[0], ci, 64), l1 = __shfl(Ls[1], ci, 64);
        const uint32_t o0 = __shfl(offs[0], ci, 64), o1 = __shfl(offs[1], ci, 64);
        const uint32_t Lc = c < 64 ? l0 : (c < kChunk ? l1 : 0u);
        const uint32_t oc = c < 64 ? o0 : o1;
        const bool istok = lane < 32 && Lc != 0;
        const uint64_t tm = ballot(istok);
        nmatch = (uint32_t)__builtin_popcountll(tm);
        const uint32_t sh = (uint32_t)(tm & 1u) ^ 1u;  // tokens start at lane 1 if 0 is no match
        const uint32_t tav = __shfl(c | (Lc << 16), lane + sh, 64), tbv = __shfl(oc, lane + sh, 64);
        if (nmatch) {
          ta = tav;
          tb = tbv;
          last_end = readlane(c + Lc, nmatch - 1 + sh);
        }
        // copy-start bitmask (position p of the chunk) for the literal scatter
        uint64_t* tsw = reinterpret_cast<uint64_t*>(jt);
        if (lane == 0) tsw[0] = tsw[1] = 0;
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        if (istok)
          __hip_atomic_fetch_or(&tsw[c >> 6], 1ull << (c & 63u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        ts0 = tsw[0];
        ts1 = tsw[1];
      }
      STAMP(4)
      ntok = nmatch;
      if (last_end < ce - c0) {  // trailing literal run: a token without a copy
        const bool me = lane == ntok;
        ta = me ? ce - c0 : ta;
        tb = me ? 0u : tb;
        ++ntok;
      }
      const uint32_t tq = c0 + (ta & 0xffff), tL = ta >> 16;
      const uint32_t end = tq + tL;
      const uint32_t prev_end = __shfl_up(end, 1, 64);
      ls = lane == 0 ? c0 : prev_end;
      if (lane < ntok) {
        litlen = tq - ls;
        littag = lit_tag_bytes(litlen);
        sz = littag + litlen + (tL ? copy_bytes_cf(tb, tL) : 0);
      }
      incl = scan_dpp(sz);
      // chunk info for the round layout: unmerged size | leading literal piece | trailing
      // literal piece | no copies at all
      const uint32_t trail = ce - c0 - last_end;
      if (lane == 0)
        csize[wave] = readlane(incl, ntok - 1) | (readlane(litlen, 0) << 11) | (trail << 19) | ((nmatch == 0) << 27);
    } else {
      if (lane == 0) csize[wave] = 0;
    }

    STAMP(5)
    // next round: words and first-chance candidates (table as of this round)
    uint64_t wn[2];
    uint32_t t1n[2];
    {
      const uint32_t k2 = k + kWavesPerBlock;
      const uint32_t c2 = k2 * kChunk;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint32_t q = c2 + 64 * j + lane;
        wn[j] = lds_ld64(data, q < n ? q : 0);
        t1n[j] = k2 < nchunks ? T[((uint32_t)wn[j] * kHashMul) >> (32 - kFTabBits)] : 0;
      }
    }
    STAMP(6)
    __syncthreads();  // B2
    STAMP(7)

    // (c) round layout, lane-parallel over the round's chunks (lane u = chunk u): a literal
    // run that crosses chunk boundaries inside the round is emitted once, with one tag for
    // its total length in the chunk where it starts (runs restart at round boundaries).
    //   cont_in[u]: chunk u's leading literal piece continues chunk u-1's trailing piece (no tag)
    //   mid[u]:     chunk u is all literal and continues a run (no tag of its own)
    //   start[u]:   chunk u's trailing piece starts a run; if cont_in[u+1] the run spans chunks
    //               and its tag encodes the run length up to the end of the last piece.
    uint32_t myb, mycont, myrun, total;
    {
      const uint32_t info = lane < kWavesPerBlock ? csize[lane] : 0u;
      const uint32_t S = info & 0x7ffu, lead = (info >> 11) & 0xffu, trl = (info >> 19) & 0xffu;
      const bool nocp = (info >> 27) & 1u;
      const uint32_t trl_prev = __shfl_up(trl, 1, 64);
      const bool cont_in = lane > 0 && lane < kWavesPerBlock && trl_prev > 0 && lead > 0;
      const bool mid = nocp && cont_in;
      const bool start = trl > 0 && !mid;
      const bool cont_next = __shfl_down((uint32_t)cont_in, 1, 64) != 0 && lane + 1 < kWavesPerBlock;
      const uint32_t cu = (r * kWavesPerBlock + lane) * kChunk;              // chunk start
      const uint32_t ceu = min(cu + kChunk, n);
      // the run ending in chunk u ends at cu + lead; a run starting in chunk v ends in the
      // first later chunk whose piece ends it (suffix min over lanes)
      const bool ends = cont_in && !(mid && cont_next);
      uint32_t nxt = ends ? lane : 0xffu;
#pragma unroll
      for (uint32_t d = 1; d < kWavesPerBlock; d <<= 1) {
        const uint32_t o2 = __shfl_down(nxt, d, 64);
        nxt = (lane + d < kWavesPerBlock && o2 < nxt) ? o2 : nxt;
      }
      nxt = __shfl_down(nxt, 1, 64);                                         // first end after u
      const uint32_t endpos = __shfl(cu + lead, nxt & 63u, 64);
      const uint32_t runlen = (start && cont_next) ? endpos - (ceu - trl) : 0u;
      const uint32_t Sm = S - (cont_in ? lit_tag_bytes(lead) : 0u) +
                          (runlen ? lit_tag_bytes(runlen) - lit_tag_bytes(trl) : 0u);
      const uint32_t inclm = scan_dpp(lane < kWavesPerBlock ? Sm : 0u);
      total = readlane(inclm, kWavesPerBlock - 1);
      myb = readlane(inclm - Sm, wave);
      mycont = readlane((uint32_t)cont_in, wave);
      myrun = readlane(runlen, wave);
    }
    STAMP(8)
    if (active && !(SM_ABLATE & 1)) {
      const uint32_t rm = mycont ? readlane(littag, 0) : 0u;                 // leading tag removed
      const uint32_t tq = c0 + (ta & 0xffff), tL = ta >> 16;
      const uint32_t o = op + myb + incl - sz - (lane > 0 ? rm : 0u);
      uint32_t mytag = (lane == 0 && mycont) ? 0u : littag, tagv = litlen;
      if (myrun && lane == ntok - 1) {                                       // the run's trailing token
        mytag = lit_tag_bytes(myrun);
        tagv = myrun;
      }
      if (lane < ntok) {
        put_lit_tag(dst, o, mytag, tagv);
        if (tL) put_copy_cf(dst, o + mytag + litlen, tb, tL);
      }
      const int32_t delta = (int32_t)(o + mytag) - (int32_t)ls;
      const uint32_t end = tq + tL;
      uint32_t below = 0;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint64_t ts = j == 0 ? ts0 : ts1;
        const uint32_t x = c0 + 64 * j + lane;
        uint32_t cnt = below + __builtin_amdgcn_mbcnt_hi((uint32_t)(ts >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ts, 0u));
        cnt += (uint32_t)(ts >> lane) & 1u;  // tokens whose copy starts at or before x
        const uint32_t pend = __shfl(end, cnt ? cnt - 1 : 0, 64);
        const int32_t dl = __shfl(delta, cnt, 64);
        if (x < ce && (cnt == 0 || x >= pend)) dst[(int32_t)x + dl] = (uint8_t)w[j];
        below += __builtin_popcountll(ts);
      }
    }
    STAMP(9)
    op += total;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      w[j] = wn[j];
      t1[j] = t1n[j];
    }
  }
  STAMP(10)
  STAMP_FLUSH(g_stamp_c)
  if (tid == 0) a.out_len[b] = op;
}

#if SM_STAMP
extern "C" int sm_debug_stamps_c(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamp_c), sizeof(g_stamp_c)) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[12] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_c), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

constexpr size_t kFastLds =
    kBlockSize + 4 * (kFTab + 2 * kWavesPerBlock * kPriv + kWavesPerBlock) + kWavesPerBlock * kLevels * kRow;
static_assert(kFastLds <= 160 * 1024, "fast compressor LDS exceeds a CU");

hipError_t launch_compress_fast(const CompressArgs& a, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)k_compress_fast, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)kFastLds);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(k_compress_fast, dim3(a.nblk), dim3(kThreads), kFastLds, s, a);
  return hipGetLastError();
}

}  // namespace sm
