// sm_compress_fast.hip -- "fast mode" batched snappy compression for gfx950 (MI355X).
//
// Produces a valid snappy stream per <= 64 KiB block (decodes bit-exactly under Snappy.jl's
// uncompress, src/internal.jl:411-466) with a wave-parallel parse instead of the reference's
// serial greedy loop (internal.jl:127-250).
//
// One workgroup of 8 waves per block; the block is staged once in LDS (64 KiB) beside a
// shared 16 K-entry latest-position table (u32, 64 KiB) and a 256-entry private table per
// wave (8 KiB): 136 KiB, one block per CU.  The block is cut into 128-byte chunks whose parse
// never crosses the chunk end (copies are truncated there, literal runs end there), so the
// chunks of a round are parsed independently: in round r wave w owns chunk 8r+w, two
// positions per lane (q = c0 + 64*j + lane).  Per chunk:
//  1. (a) insert every position into the shared table with ds_max_u32 (order-independent ->
//     deterministic) and into the wave's private table with ds_max_rtn_u32, whose return is
//     the latest EARLIER position of the chunk with the same 8-bit hash (lanes of one
//     instruction are serialised in ascending order on gfx950; verified, see tools/probe_lds);
//  2. (b) two candidates per position: A = that intra-chunk position, else the shared
//     table after the round (if it is an earlier position); B = the shared table as of the
//     previous round.  Both verified (4 bytes) and extended 16 bytes branch-free with unaligned
//     ds_read_b64; the longer one wins;
//  3. greedy walk over the two match ballots in SALU (s_ff1 + one v_readlane per copy);
//     tokens land in lanes; sizes in closed form, DPP wave scan, chunk sizes exchanged
//     through LDS -> exact output offsets;
//  4. (c) token lanes write tag bytes; position lanes scatter literal bytes.
// Two barriers per round.  Output is deterministic (no order-dependent table state).
#include "sm_device.h"
#include "sm_internal.h"

#ifndef SM_ABLATE  // diagnostic builds only (tools/ablate.sh): 1 no emit, 2 no matches, 4 no inserts
#define SM_ABLATE 0
#endif

namespace sm {

constexpr uint32_t kFTabBits = 14;
constexpr uint32_t kFTab = 1u << kFTabBits;   // shared table entries
constexpr uint32_t kPrivBits = 8;
constexpr uint32_t kPriv = 1u << kPrivBits;   // private (intra-chunk) table entries per wave
constexpr uint32_t kChunk = 128;
constexpr uint32_t kWavesPerBlock = 8;
constexpr uint32_t kThreads = 64 * kWavesPerBlock;
constexpr uint32_t kEager = 16;               // bytes compared past the first 4 before the wave takes over

typedef uint16_t __attribute__((aligned(1))) fu16u;
typedef uint32_t __attribute__((aligned(1))) fu32u;
typedef uint64_t __attribute__((aligned(1))) fu64u;

__device__ inline uint32_t ld32u(const uint8_t* p) { return *reinterpret_cast<const fu32u*>(p); }
__device__ inline uint64_t ld64u(const uint8_t* p) { return *reinterpret_cast<const fu64u*>(p); }

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

// match length of lds[i1..] vs lds[i2..] capped at avail, whole wave (512 B per round)
__device__ inline uint32_t wave_match_len8(const uint8_t* lds, uint32_t i1, uint32_t i2, uint32_t avail,
                                           uint32_t lane) {
  uint32_t base = 0;
  for (;;) {
    uint32_t off = base + 8 * lane;
    uint32_t res;
    bool stop;
    if (off >= avail) {
      res = avail;
      stop = true;
    } else {
      uint64_t x = ld64u(lds + i1 + off) ^ ld64u(lds + i2 + off);
      uint32_t fb = x ? (uint32_t)(__builtin_ctzll(x) >> 3) : 8u;
      res = min(off + fb, avail);
      stop = (fb < 8) || (off + 8 >= avail);
    }
    uint64_t m = ballot(stop);
    if (m) return readlane(res, ctz64(m));
    base += 8 * kWave;
  }
}

// bytes matching past the first 4 (0..kEager), branch-free
__device__ inline uint32_t ext16(const uint8_t* d, uint32_t c, uint32_t q) {
  uint64_t x0 = ld64u(d + c + 4) ^ ld64u(d + q + 4);
  uint64_t x1 = ld64u(d + c + 12) ^ ld64u(d + q + 12);
  uint32_t e0 = (uint32_t)(__builtin_ctzll(x0 | (1ull << 63)) >> 3);  // 0..7, or 7 if equal
  uint32_t e1 = (uint32_t)(__builtin_ctzll(x1 | (1ull << 63)) >> 3);
  return x0 ? e0 : (x1 ? 8 + e1 : 16);
}

__global__ __launch_bounds__(512) void k_compress_fast(CompressArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* data = smem;                                                       // 64 KiB block
  uint32_t* T = reinterpret_cast<uint32_t*>(smem + kBlockSize);               // shared table
  const uint32_t tid = threadIdx.x;
  const uint32_t wave = uniform(tid >> 6);
  const uint32_t lane = tid & 63;
  uint32_t* P = T + kFTab + wave * kPriv;                                     // private table
  uint32_t* csize = T + kFTab + kWavesPerBlock * kPriv;                       // per-wave chunk sizes
  uint8_t* jt = reinterpret_cast<uint8_t*>(csize + kWavesPerBlock) + wave * 8 * kChunk;  // parse jump tables

  const uint32_t b = blockIdx.x;
  const uint32_t n = a.in_len[b];
  const uint8_t* src = a.in + a.in_off[b];
  uint8_t* dst = a.out + a.out_off[b];
  if (n > kBlockSize) {
    if (tid == 0) a.out_len[b] = 0xffffffffu;
    return;
  }

  // stage the block: 8 x 16 B per thread in flight when aligned
  if (((uintptr_t)src & 15) == 0) {
    const uint4* s16 = reinterpret_cast<const uint4*>(src);
    uint4* d16 = reinterpret_cast<uint4*>(data);
    const uint32_t n16 = n >> 4;
    if (n16 == kBlockSize / 16) {
      uint4 v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = s16[tid + i * kThreads];
#pragma unroll
      for (int i = 0; i < 8; ++i) d16[tid + i * kThreads] = v[i];
    } else {
      for (uint32_t k = tid; k < n16; k += kThreads) d16[k] = s16[k];
      for (uint32_t k = (n & ~15u) + tid; k < n; k += kThreads) data[k] = src[k];
    }
  } else {
    for (uint32_t k = tid; k < n; k += kThreads) data[k] = src[k];
  }
  {
    uint4 z = make_uint4(0, 0, 0, 0);
    uint4* t16 = reinterpret_cast<uint4*>(T);
    for (uint32_t k = tid; k < (kFTab + kWavesPerBlock * kPriv) / 4; k += kThreads) t16[k] = z;
  }
  uint32_t op = 0;
  if (a.header) {
    uint32_t nb = varint_len(n);
    if (tid < nb) dst[tid] = (uint8_t)(((n >> (7 * tid)) & 0x7f) | (tid + 1 < nb ? 0x80 : 0));
    op = nb;
  }
  __syncthreads();

  const uint32_t nchunks = (n + kChunk - 1) / kChunk;
  const uint32_t rounds = (nchunks + kWavesPerBlock - 1) / kWavesPerBlock;

  uint32_t w[2], t1[2];
  {
    const uint32_t c0 = wave * kChunk;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      uint32_t q = c0 + 64 * j + lane;
      w[j] = ld32u(data + (q < n ? q : 0));
      t1[j] = 0;
    }
  }

  for (uint32_t r = 0; r < rounds; ++r) {
    const uint32_t k = r * kWavesPerBlock + wave;
    const bool active = k < nchunks;
    const uint32_t c0 = k * kChunk;
    const uint32_t ce = active ? min(c0 + kChunk, n) : c0;

    // (a) inserts
    uint32_t pin[2] = {0, 0};
    if (active && !(SM_ABLATE & 4)) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint32_t q = c0 + 64 * j + lane;
        const uint32_t hm = w[j] * kHashMul;
        if (q + 4 <= n) {
          __hip_atomic_fetch_max(&T[hm >> (32 - kFTabBits)], q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          pin[j] = __hip_atomic_fetch_max(&P[hm >> (32 - kPrivBits)], q + 1, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
    }
    __syncthreads();  // B1

    // (b) candidates, verify, extend, walk, sizes
    uint32_t ta = 0, tb = 0, ntok = 0, incl = 0, sz = 0, litlen = 0, littag = 0, ls = 0;
    uint64_t ts0 = 0, ts1 = 0;
    if (active) {
      uint32_t Ls[2], offs[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint32_t q = c0 + 64 * j + lane;
        const bool can = q + 4 <= ce;
        const uint32_t cap = can ? ce - q - 4 : 0;
        const uint32_t t2 = T[(w[j] * kHashMul) >> (32 - kFTabBits)];
        uint32_t ca = pin[j] > c0 ? pin[j] - 1 : ((t2 != 0 && t2 - 1 < q) ? t2 - 1 : q);
        uint32_t cb = t1[j] != 0 ? t1[j] - 1 : q;
        const bool oka = can && ca < q && ld32u(data + ca) == w[j];
        const bool okb = can && cb < q && cb != ca && ld32u(data + cb) == w[j];
        const uint32_t la = oka ? 4 + min(ext16(data, ca, q), cap) : 0;
        const uint32_t lb = okb ? 4 + min(ext16(data, cb, q), cap) : 0;
        const bool useb = lb > la;
        Ls[j] = (SM_ABLATE & 2) ? 0u : (useb ? lb : la);
        offs[j] = q - (useb ? cb : ca);
      }
      // finish matches that filled the eager window: 8 bytes per lane per step
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint32_t q = c0 + 64 * j + lane;
        uint32_t L = Ls[j];
        bool more = L >= 4 + kEager && q + L < ce;
        while (ballot(more)) {
          if (more) {
            const uint32_t avail = ce - q - L;
            const uint64_t x = ld64u(data + q - offs[j] + L) ^ ld64u(data + q + L);
            const uint32_t fb = x ? (uint32_t)(__builtin_ctzll(x) >> 3) : 8u;
            L += min(fb, avail);
            more = fb == 8 && avail > 8;
          }
        }
        Ls[j] = L;
      }
      // Greedy parse by pointer doubling (no serial loop): J0[r] = r + max(L(r), 1) over the
      // chunk's 128 positions, J_k = J_{k-1} o J_{k-1}; position r is visited by the greedy
      // walk from 0 iff the binary descent along J_7..J_0 (largest visited position <= r)
      // lands on r.  Visited match positions are the copies.
      uint32_t cur[2] = {0xffffu, 0xffffu};  // no copies at all (incompressible): skip the parse
      if (ballot(Ls[0] != 0 || Ls[1] != 0)) {
        uint32_t jv[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const uint32_t r = 64 * j + lane;
          jv[j] = r + max(Ls[j], 1u);  // <= 255
          jt[r] = (uint8_t)jv[j];
        }
#pragma unroll
        for (int k = 1; k < 8; ++k) {
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            jv[j] = jv[j] < kChunk ? jt[(k - 1) * kChunk + jv[j]] : jv[j];
            jt[k * kChunk + 64 * j + lane] = (uint8_t)jv[j];
          }
        }
        cur[0] = cur[1] = 0;
#pragma unroll
        for (int k = 7; k >= 0; --k) {
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const uint32_t t = jt[k * kChunk + cur[j]];
            cur[j] = t <= 64u * j + lane ? t : cur[j];
          }
        }
      }
      const bool tok0 = cur[0] == lane && Ls[0] != 0;
      const bool tok1 = cur[1] == 64 + lane && Ls[1] != 0;
      ts0 = ballot(tok0);
      ts1 = ballot(tok1);
      const uint32_t n0 = __builtin_popcountll(ts0);
      const uint32_t nmatch = n0 + __builtin_popcountll(ts1);
      uint32_t last_end = 0;
      if (nmatch) {  // end of the last copy (highest token position)
        const uint32_t j = ts1 ? 1u : 0u;
        const uint64_t m = ts1 ? ts1 : ts0;
        const uint32_t l = 63 - (uint32_t)__builtin_clzll(m);
        last_end = 64 * j + l + readlane(j ? Ls[1] : Ls[0], l);
      }
      // compact the copies into lanes 0..nmatch-1 (slots reuse J level 0..3, no longer read)
      uint2* slots = reinterpret_cast<uint2*>(jt);
      if (tok0) slots[__builtin_amdgcn_mbcnt_hi((uint32_t)(ts0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ts0, 0u))] =
          make_uint2(lane | (Ls[0] << 16), offs[0]);
      if (tok1) slots[n0 + __builtin_amdgcn_mbcnt_hi((uint32_t)(ts1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ts1, 0u))] =
          make_uint2((64 + lane) | (Ls[1] << 16), offs[1]);
      if (lane < nmatch) {
        const uint2 sv = slots[lane];
        ta = sv.x;
        tb = sv.y;
      }
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
        littag = litlen == 0 ? 0 : (litlen <= 60 ? 1 : 2);
        sz = littag + litlen + (tL ? copy_bytes_cf(tb, tL) : 0);
      }
      incl = scan_dpp(sz);
      if (lane == 0) csize[wave] = readlane(incl, ntok - 1);
    } else {
      if (lane == 0) csize[wave] = 0;
    }

    // next round: words and first-chance candidates (table as of this round)
    uint32_t wn[2], t1n[2];
    {
      const uint32_t k2 = k + kWavesPerBlock;
      const uint32_t c2 = k2 * kChunk;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint32_t q = c2 + 64 * j + lane;
        wn[j] = ld32u(data + (q < n ? q : 0));
        t1n[j] = k2 < nchunks ? T[(wn[j] * kHashMul) >> (32 - kFTabBits)] : 0;
      }
    }
    __syncthreads();  // B2

    // (c) emit at the exact output offset
    uint32_t before = 0, total = 0;
#pragma unroll
    for (uint32_t v = 0; v < kWavesPerBlock; ++v) {
      const uint32_t s = csize[v];
      before += v < wave ? s : 0;
      total += s;
    }
    if (active && !(SM_ABLATE & 1)) {
      const uint32_t o = op + before + incl - sz;
      const uint32_t tq = c0 + (ta & 0xffff), tL = ta >> 16;
      if (lane < ntok) {
        if (littag == 1) {
          dst[o] = (uint8_t)((litlen - 1) << 2);
        } else if (littag == 2) {
          dst[o] = (uint8_t)(60 << 2);
          dst[o + 1] = (uint8_t)(litlen - 1);
        }
        if (tL) put_copy_cf(dst, o + littag + litlen, tb, tL);
      }
      const int32_t delta = (int32_t)(o + littag) - (int32_t)ls;
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
    op += total;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      w[j] = wn[j];
      t1[j] = t1n[j];
    }
  }
  if (tid == 0) a.out_len[b] = op;
}

constexpr size_t kFastLds =
    kBlockSize + 4 * (kFTab + kWavesPerBlock * kPriv + kWavesPerBlock) + kWavesPerBlock * 8 * kChunk;

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
