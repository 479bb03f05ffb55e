// sm_compress_lanes.hip -- SM_MODE_FAST batched snappy compression for gfx950 (MI355X):
// exact candidates from an in-order inserter kernel, then a LANE-SERIAL greedy parse.
//
// Produces a valid snappy stream per <= 64 KiB block (decodes bit-exactly under Snappy.jl's
// uncompress, src/internal.jl:411-466); the reference's serial loop (internal.jl:127-250) is
// restated as two kernels per sub-batch of blocks:
//
//  k_prev_insert (one wave per block, 5 blocks per CU: a 32 KiB table each)
//    walks the block's positions in order, 64 per LDS instruction, through a 16 K-bucket table of
//    u16 positions (14-bit hash; a bucket is half a dword, exchanged with ds_mskor_rtn_b32).  A
//    wave's LDS instructions execute in order and the conflicting lanes of one instruction in
//    ascending lane order, so every position gets back exactly the sequential answer -- the
//    latest earlier position with the same hash -- which goes to a per-position scratch array
//    prev[] in device memory (2 B per input byte, coalesced).  Correctness never depends on that
//    order (every candidate is verified); only the ratio does.
//
//  k_compress_lanes (one 512-lane workgroup per block, 2 per CU: the block in LDS)
//    cuts the block into 128-byte chunks, one per LANE, and each lane parses its chunk greedily
//    and serially, like the reference, from prev[]: a step probes four positions at once (their
//    candidates verified 8 bytes at a time against the block in LDS), takes the first match or
//    moves on by four; a match that fills the 8 bytes is extended 16 bytes per step up to 64
//    (emit_copy!'s piece size) or the chunk end.  Copies never cross a chunk end and literal runs
//    restart at chunk starts, so the chunks are independent.  A lane writes its tokens straight
//    into a staging slot of the block's own output region (literal runs capped at 60 bytes, so
//    a run's one tag byte is reserved when it starts), then the workgroup scans the chunk sizes
//    and every lane moves its chunk to its final place.
//
// Why: the wave-parallel parse of sm_compress_fast.hip (k_compress_fast<1>) spends ~3.6
// instructions per input byte on doubling tables, shuffles and scans to reproduce a serial
// greedy walk; a lane walking its own chunk spends ~0.5, and the inserter, freed from sharing
// a workgroup with the block, runs on five blocks per CU.
#include "sm_device.h"
#include "sm_internal.h"

namespace sm {

constexpr uint32_t kPvBits = 14;                      // inserter hash bits: 16 K u16 buckets, 32 KiB
constexpr uint32_t kPvG = 4;                          // exchanges per inserter step (one asm statement)
constexpr uint32_t kLChunk = 128;                     // positions per lane
constexpr uint32_t kLThreads = kBlockSize / kLChunk;  // 512 lanes: a full block
constexpr uint32_t kLStride = 134;                    // staging bytes per chunk: <= 131 of output + 3 of overhang
constexpr uint32_t kLCap = 64;                        // longest copy: emit_copy!'s piece (internal.jl:289-304)
constexpr uint32_t kLRun = 57;                        // a literal run is closed once it reaches this (<= 60 after a step)

// fast-mode hash: a full-rate 24-bit multiply of the word folded to 24 bits (the compiler widens a
// masked product to the quarter-rate v_mul_lo_u32, so it is issued directly)
__device__ inline uint32_t pv_hash(uint32_t w) {
  uint32_t p;
  asm("v_mul_u32_u24 %0, %1, %2" : "=v"(p) : "s"(0x1e35a7u), "v"(w ^ (w >> 12)));
  return (p >> 10) & ((1u << kPvBits) - 1);
}

typedef uint32_t __attribute__((aligned(1))) lu32u;
typedef uint64_t __attribute__((aligned(1))) lu64u;
typedef uint4 __attribute__((aligned(1))) lu128u;

// ---- k_prev_insert ------------------------------------------------------------------------
// The block streams through two 4 KiB LDS buffers (coalesced 16-B loads, one batch ahead: a
// batch's 64 groups of exchanges hide the next batch's HBM latency); each position's word is
// then two aligned LDS dwords and a funnel shift.
constexpr uint32_t kPvBatch = 4096;

// 16 bytes of the block at off (unaligned global load; the block's end is never crossed)
__device__ inline uint4 load16_clip(const uint8_t* src, uint32_t off, uint32_t n) {
  if (off + 16 <= n) return *reinterpret_cast<const lu128u*>(src + off);
  uint32_t w[4] = {0, 0, 0, 0};
  for (uint32_t k = 0; k < 16 && off + k < n; ++k) w[k >> 2] |= (uint32_t)src[off + k] << (8 * (k & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

__global__ __launch_bounds__(64) void k_prev_insert(CompressArgs a, uint32_t b0) {
  __shared__ __attribute__((aligned(16))) uint32_t T[1u << (kPvBits - 1)];  // bucket h: half (h & 1) of T[h >> 1]
  __shared__ __attribute__((aligned(16))) uint8_t stg[2][kPvBatch + 16];     // batch i (+ the next 16 bytes)
  const uint32_t lane = threadIdx.x, b = b0 + blockIdx.x;
  if (a.screened && a.out_len[b] != kScreenTodo) return;
  const uint32_t n = a.in_len[b];
  if (n > kBlockSize) return;
  const uint8_t* src = a.in + a.in_off[b];
  uint16_t* pv = a.prev + (size_t)blockIdx.x * kBlockSize;
  for (uint32_t k = lane; k < sizeof(T) / 16; k += 64) reinterpret_cast<uint4*>(T)[k] = make_uint4(0, 0, 0, 0);
  const uint32_t nbat = (n + kPvBatch - 1) / kPvBatch;
  uint4 r[5];  // lane's 16-B pieces of a batch: 1 KiB apart, lane 0's fifth = the next batch's first 16 B
  auto load = [&](uint32_t i) {
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) r[j] = load16_clip(src, kPvBatch * i + 16 * lane + 1024 * j, n);
    r[4] = lane == 0 ? load16_clip(src, kPvBatch * (i + 1), n) : make_uint4(0, 0, 0, 0);
  };
  auto put = [&](uint32_t i) {
    uint4* d = reinterpret_cast<uint4*>(stg[i & 1]);
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) d[lane + 64 * j] = r[j];
    if (lane == 0) d[kPvBatch / 16] = r[4];
  };
  load(0);
  put(0);
  if (nbat > 1) load(1);
  for (uint32_t i = 0; i < nbat; ++i) {
    const uint8_t* sb = stg[i & 1];
    const uint32_t q0 = kPvBatch * i;
    for (uint32_t g0 = 0; g0 < kPvBatch / 64 && q0 + 64 * g0 < n; g0 += kPvG) {
      uint32_t la[kPvG], mk[kPvG], vv[kPvG], sh[kPvG], old[kPvG];
#pragma unroll
      for (uint32_t k = 0; k < kPvG; ++k) {
        const uint32_t rel = 64 * (g0 + k) + lane, q = q0 + rel;
        const uint32_t* dw = reinterpret_cast<const uint32_t*>(sb + 64 * (g0 + k)) + (lane >> 2);
        const uint32_t h = pv_hash(__builtin_amdgcn_alignbyte(dw[1], dw[0], lane & 3u));
        const bool v = q + 4 <= n;
        sh[k] = (h & 1u) << 4;
        la[k] = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint32_t*)(&T[h >> 1]));
        mk[k] = v ? 0xffffu << sh[k] : 0u;  // mask 0: memory unchanged
        vv[k] = v ? (q + 1) << sh[k] : 0u;
      }
      // D = (D & ~mask) | value with the old dword back; the exchanges and their wait are ONE
      // asm statement (early-clobber results), so no result register is touched before it lands
      static_assert(kPvG == 4, "the asm issues four exchanges");
      asm volatile(
          "ds_mskor_rtn_b32 %0, %4, %8, %12\n"
          "ds_mskor_rtn_b32 %1, %5, %9, %13\n"
          "ds_mskor_rtn_b32 %2, %6, %10, %14\n"
          "ds_mskor_rtn_b32 %3, %7, %11, %15\n"
          "s_waitcnt lgkmcnt(0)"
          : "=&v"(old[0]), "=&v"(old[1]), "=&v"(old[2]), "=&v"(old[3])
          : "v"(la[0]), "v"(la[1]), "v"(la[2]), "v"(la[3]), "v"(mk[0]), "v"(mk[1]), "v"(mk[2]), "v"(mk[3]),
            "v"(vv[0]), "v"(vv[1]), "v"(vv[2]), "v"(vv[3])
          : "memory");
#pragma unroll
      for (uint32_t k = 0; k < kPvG; ++k) {
        const uint32_t q = q0 + 64 * (g0 + k) + lane;
        if (q < n) pv[q] = (uint16_t)(old[k] >> sh[k]);
      }
    }
    if (i + 1 < nbat) {
      put(i + 1);
      if (i + 2 < nbat) load(i + 2);
    }
  }
}

// ---- k_compress_lanes ---------------------------------------------------------------------
// copy tag bytes for (off, L), L in 4..64: copy-1 (L < 12, off < 2048) or copy-2
// (emit_copy_upto_64!, internal.jl:289-304); packed little-endian, and the tag's size
__device__ inline uint32_t copy_tag(uint32_t off, uint32_t L, uint32_t& sz) {
  const bool c1 = L < 12 && off < 2048;
  sz = c1 ? 2u : 3u;
  return c1 ? (1u + ((L - 4) << 2) + ((off >> 3) & 0xe0u)) | ((off & 0xffu) << 8)
            : (2u + ((L - 1) << 2)) | ((off & 0xffffu) << 8);
}

__global__ __launch_bounds__(kLThreads, 4) void k_compress_lanes(CompressArgs a, uint32_t b0) {
  __shared__ __attribute__((aligned(16))) uint8_t data[kBlockSize + 64];
  __shared__ uint32_t wsum[kLThreads / 64];
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const uint32_t b = b0 + blockIdx.x;
  if (a.screened && a.out_len[b] != kScreenTodo) return;  // emitted as one literal by k_literal_screen
  const uint32_t n = a.in_len[b];
  const uint8_t* src = a.in + a.in_off[b];
  uint8_t* dst = a.out + a.out_off[b];
  if (n > kBlockSize) {
    if (tid == 0) a.out_len[b] = 0xffffffffu;
    return;
  }
  // stage the block (aligned: all 16-B loads of a thread in flight)
  if (((uintptr_t)src & 15) == 0) {
    const uint4* s16 = reinterpret_cast<const uint4*>(src);
    uint4* d16 = reinterpret_cast<uint4*>(data);
    const uint32_t n16 = n >> 4;
    if (n16 == kBlockSize / 16) {
      constexpr int kLoads = kBlockSize / 16 / kLThreads;
      uint4 v[kLoads];
#pragma unroll
      for (int i = 0; i < kLoads; ++i) v[i] = s16[tid + i * kLThreads];
#pragma unroll
      for (int i = 0; i < kLoads; ++i) d16[tid + i * kLThreads] = v[i];
    } else {
      for (uint32_t k = tid; k < n16; k += kLThreads) d16[k] = s16[k];
      for (uint32_t k = (n & ~15u) + tid; k < n; k += kLThreads) data[k] = src[k];
    }
  } else {
    for (uint32_t k = tid; k < n; k += kLThreads) data[k] = src[k];
  }
  if (tid < 64) data[n + tid] = 0;  // reads past the block see zeros (never part of a match: lengths stop at ce)
  const uint32_t hdr = a.header ? varint_len(n) : 0u;
  if (tid < hdr) dst[tid] = (uint8_t)(((n >> (7 * tid)) & 0x7f) | (tid + 1 < hdr ? 0x80 : 0));
  __syncthreads();

  const uint16_t* pv = a.prev + (size_t)blockIdx.x * kBlockSize;
  const uint32_t c0 = tid * kLChunk, ce = min(c0 + kLChunk, n);
  const uint32_t ost = hdr + tid * kLStride;  // this chunk's staging slot in the output region
  uint32_t p = c0, o = ost, otag = 0, run = 0;
  bool act = c0 < n, ext = false;
  uint32_t cq = 0, coff = 0, cL = 0, clim = 0;
  while (ballot(act)) {
    bool emit = false;
    if (act && !ext) {
      // probe positions p .. p+3: the candidates (prev[], u16 position + 1, 0 = none) and the
      // bytes at p .. p+10 (four aligned dwords, funnel-shifted)
      const uint64_t pr = *reinterpret_cast<const lu64u*>(pv + p);
      const uint32_t* dw = reinterpret_cast<const uint32_t*>(data + (p & ~3u));
      const uint32_t s = p & 3u;
      const uint32_t d0 = dw[0], d1 = dw[1], d2 = dw[2], d3 = dw[3];
      const uint32_t W0 = __builtin_amdgcn_alignbyte(d1, d0, s), W1 = __builtin_amdgcn_alignbyte(d2, d1, s),
                     W2 = __builtin_amdgcn_alignbyte(d3, d2, s);
      uint32_t first = 4, fl = 0, fc = 0;
#pragma unroll
      for (int i = 3; i >= 0; --i) {  // descending: the lowest matching i wins
        const uint32_t q = p + i;
        const uint32_t cv = (uint32_t)(pr >> (16 * i)) & 0xffffu;
        const bool ok = cv != 0 && cv - 1 < q && q + 4 <= ce;
        const uint32_t lo = i == 0 ? W0 : __builtin_amdgcn_alignbyte(W1, W0, i);
        const uint32_t hi = i == 0 ? W1 : __builtin_amdgcn_alignbyte(W2, W1, i);
        const uint64_t x = lds_ld64(data, ok ? cv - 1 : 0) ^ (((uint64_t)hi << 32) | lo);
        const uint32_t l = x ? (uint32_t)(__builtin_ctzll(x) >> 3) : 8u;
        if (ok && l >= 4) {
          first = i;
          fl = l;
          fc = cv - 1;
        }
      }
      // literal bytes p .. p+first-1 (those inside the chunk): appended to the open run
      const uint32_t nlit = min(first, ce - p);
      if (nlit) {
        if (run == 0) {
          otag = o;  // the run's tag byte, written when it closes
          ++o;
        }
        *reinterpret_cast<lu32u*>(dst + o) = W0;  // 4 bytes; the ones past the run are overwritten later
        o += nlit;
        run += nlit;
      }
      if (first < 4) {
        if (run) {
          dst[otag] = (uint8_t)((run - 1) << 2);
          run = 0;
        }
        cq = p + first;
        coff = cq - fc;
        clim = min(kLCap, ce - cq);
        cL = min(fl, clim);
        ext = cL == 8 && clim > 8;
        emit = !ext;
      } else {
        p = min(p + 4, ce);
        if (run >= kLRun) {
          dst[otag] = (uint8_t)((run - 1) << 2);
          run = 0;
        }
      }
    } else if (act) {
      // extend the copy at cq: 16 bytes a step
      const uint32_t x0 = cq + cL, y0 = x0 - coff;
      const uint32_t* wx = reinterpret_cast<const uint32_t*>(data + (x0 & ~3u));
      const uint32_t* wy = reinterpret_cast<const uint32_t*>(data + (y0 & ~3u));
      const uint32_t sx = x0 & 3u, sy = y0 & 3u;
      uint32_t x[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        x[k] = __builtin_amdgcn_alignbyte(wx[k + 1], wx[k], sx) ^ __builtin_amdgcn_alignbyte(wy[k + 1], wy[k], sy);
      const uint64_t lo = ((uint64_t)x[1] << 32) | x[0], hi = ((uint64_t)x[3] << 32) | x[2];
      const uint32_t fb = lo ? (uint32_t)(__builtin_ctzll(lo) >> 3) : (hi ? 8u + (uint32_t)(__builtin_ctzll(hi) >> 3) : 16u);
      cL += min(fb, clim - cL);
      emit = fb < 16 || cL >= clim;
      ext = !emit;
    }
    if (emit) {
      uint32_t tsz;
      *reinterpret_cast<lu32u*>(dst + o) = copy_tag(coff, cL, tsz);
      o += tsz;
      p = cq + cL;
    }
    if (act && !ext && p >= ce) {
      if (run) dst[otag] = (uint8_t)((run - 1) << 2);
      act = false;
    }
  }

  // chunk sizes -> final offsets (a block scan), then every lane moves its chunk there: all the
  // staged bytes are read before any is overwritten (the wait + barrier)
  const uint32_t S = o - ost;
  const uint32_t incl = scan_dpp(S);
  if (lane == 63) wsum[wave] = incl;
  __threadfence_block();  // this lane's staging stores have landed
  uint4 v[(kLStride + 15) / 16];
#pragma unroll
  for (uint32_t i = 0; i < (kLStride + 15) / 16; ++i)
    v[i] = 16 * i < S ? *reinterpret_cast<const lu128u*>(dst + ost + 16 * i) : make_uint4(0, 0, 0, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  uint32_t base = hdr;
  for (uint32_t w = 0; w < wave; ++w) base += wsum[w];
  const uint32_t P = base + incl - S;
#pragma unroll
  for (uint32_t i = 0; i < (kLStride + 15) / 16; ++i) {
    const uint32_t at = 16 * i;
    if (at + 16 <= S) {
      *reinterpret_cast<lu128u*>(dst + P + at) = v[i];
    } else if (at < S) {  // the tail: exact bytes (the next chunk starts right after)
      const uint32_t r = S - at;
      const uint32_t wv[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k) {
        if (4 * k + 4 <= r) {
          *reinterpret_cast<lu32u*>(dst + P + at + 4 * k) = wv[k];
        } else if (4 * k < r) {
#pragma unroll
          for (uint32_t e = 0; e < 3; ++e)
            if (4 * k + e < r) dst[P + at + 4 * k + e] = (uint8_t)(wv[k] >> (8 * e));
        }
      }
    }
  }
  if (tid == kLThreads - 1) a.out_len[b] = P + S;  // the last lane: base + its inclusive sum
}

hipError_t launch_compress_lanes(const CompressArgs& a, uint32_t sub, hipStream_t s) {
  for (uint32_t b0 = 0; b0 < a.nblk; b0 += sub) {
    const uint32_t nb = min(sub, a.nblk - b0);
    hipLaunchKernelGGL(k_prev_insert, dim3(nb), dim3(64), 0, s, a, b0);
    hipLaunchKernelGGL(k_compress_lanes, dim3(nb), dim3(kLThreads), 0, s, a, b0);
  }
  return hipGetLastError();
}

}  // namespace sm
