// sm_compress_lanes.hip -- SM_MODE_FAST batched snappy compression for gfx950 (MI355X):
// exact candidates from an in-order inserter kernel, then a LANE-SERIAL greedy parse.
//
// Produces a valid snappy stream per <= 64 KiB block (decodes bit-exactly under Snappy.jl's
// uncompress, src/internal.jl:411-466); the reference's serial loop (internal.jl:127-250) is
// restated as two kernels per sub-batch of blocks:
//
//  k_prev_insert (one wave per block, four blocks per CU: a 32 KiB table + a 4 KiB stage each)
//    walks the block's positions in order, 64 per LDS instruction, through a 16 K-bucket table of
//    u16 positions (14-bit hash; a bucket is half a dword, exchanged with ds_mskor_rtn_b32).  A
//    wave's LDS instructions execute in order and the conflicting lanes of one instruction in
//    ascending lane order, so every position gets back exactly the sequential answer -- the
//    latest earlier position with the same hash -- which goes to a per-position scratch array
//    prev[] in device memory (2 B per input byte, coalesced).  Correctness never depends on that
//    order (every candidate is verified); only the ratio does.
//
//  k_compress_lanes (one 256-lane workgroup per block and CU: the block and a pass's prev[] in LDS)
//    cuts the block into 128-byte chunks, one per LANE, in two passes of 256 chunks.  A pass's
//    prev[] (64 KiB) is copied into LDS with coalesced loads; each lane then parses its chunk
//    greedily and serially, like the reference: a step probes four positions at once (their
//    candidates verified 8 bytes at a time against the block in LDS), takes the first match or
//    moves on by four; a match that fills the 8 bytes is extended 16 bytes per step up to 64
//    (emit_copy!'s piece size) or the chunk end.  Copies never cross a chunk end and literal runs
//    restart at chunk starts, so the chunks are independent.  The lane writes its tokens over the
//    prev[] entries it has already read (its output never overtakes its reads: a step consumes >= 4
//    positions = 8 bytes of prev[] and writes at most a few more bytes than it consumes); literal
//    runs are capped at 60 bytes, so a run's one tag byte is reserved when it starts.  A scan of
//    the chunk sizes then places every chunk, and each lane stores its chunk with 16-byte stores.
//    All per-lane traffic is LDS; global memory sees only coalesced block, prev[] and output I/O.
#include "sm_device.h"
#include "sm_internal.h"

namespace sm {

constexpr uint32_t kPvBits = 14;    // inserter hash bits: 16 K u16 buckets, 32 KiB
constexpr uint32_t kPvG = 4;        // exchanges per inserter step (one asm statement)
constexpr uint32_t kPvBatch = 4096;  // inserter staging batch
constexpr uint32_t kLChunk = 64;    // positions per lane
constexpr uint32_t kLLanes = 512;   // lanes (chunks) per pass: 32 KiB of positions
constexpr uint32_t kLSlice = 2 * kLChunk;  // LDS bytes per lane: its chunk's prev[], then its output
constexpr uint32_t kLPitch = kLSlice + 4;  // slice pitch: an odd number of dwords, so lanes at equal offsets hit distinct banks
constexpr uint32_t kLCap = 64;      // longest copy: emit_copy!'s piece (internal.jl:289-304)
static_assert(kLChunk <= 64, "a run between two copies of a chunk must fit a one-byte tag (<= 60)");

// fast-mode hash: a full-rate 24-bit multiply of the word folded to 24 bits (the compiler widens a
// masked product to the quarter-rate v_mul_lo_u32, so it is issued directly)
__device__ inline uint32_t pv_hash(uint32_t w) {
  uint32_t p;
  asm("v_mul_u32_u24 %0, %1, %2" : "=v"(p) : "s"(0x1e35a7u), "v"(w ^ (w >> 12)));
  return (p >> 10) & ((1u << kPvBits) - 1);
}

typedef uint4 __attribute__((aligned(1))) lu128u;
typedef uint32_t __attribute__((aligned(1))) lu32u;

// 16 bytes of the block at off (unaligned global load; the block's end is never crossed)
__device__ inline uint4 load16_clip(const uint8_t* src, uint32_t off, uint32_t n) {
  if (off + 16 <= n) return *reinterpret_cast<const lu128u*>(src + off);
  uint32_t w[4] = {0, 0, 0, 0};
  for (uint32_t k = 0; k < 16 && off + k < n; ++k) w[k >> 2] |= (uint32_t)src[off + k] << (8 * (k & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// ---- k_prev_insert ------------------------------------------------------------------------
// The block streams through a 4 KiB LDS stage: the next batch's coalesced 16-B loads are issued
// when a batch starts, so its 64 groups of exchanges hide their HBM latency.  Within a batch the
// next step's words are read before this step's exchanges, so the two LDS round trips overlap.
__global__ __launch_bounds__(64) void k_prev_insert(CompressArgs a, uint32_t b0) {
  __shared__ __attribute__((aligned(16))) uint32_t T[1u << (kPvBits - 1)];  // bucket h: half (h & 1) of T[h >> 1]
  __shared__ __attribute__((aligned(16))) uint8_t stg[kPvBatch + 16];        // batch i (+ the next 16 bytes)
  const uint32_t lane = threadIdx.x, b = b0 + blockIdx.x;
  if (a.screened && a.out_len[b] != kScreenTodo) return;
  const uint32_t n = a.in_len[b];
  if (n > kBlockSize) return;
  const uint8_t* src = a.in + a.in_off[b];
  uint16_t* pv = a.prev + (size_t)blockIdx.x * kBlockSize;
  for (uint32_t k = lane; k < sizeof(T) / 16; k += 64) reinterpret_cast<uint4*>(T)[k] = make_uint4(0, 0, 0, 0);
  const uint32_t nbat = (n + kPvBatch - 1) / kPvBatch;
  uint4 r[5];  // the lane's 16-B pieces of a batch, 1 KiB apart; lane 0's fifth = the next batch's first 16 B
  auto load = [&](uint32_t i) {
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) r[j] = load16_clip(src, kPvBatch * i + 16 * lane + 1024 * j, n);
    r[4] = lane == 0 ? load16_clip(src, kPvBatch * (i + 1), n) : make_uint4(0, 0, 0, 0);
  };
  auto put = [&]() {
    uint4* d = reinterpret_cast<uint4*>(stg);
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) d[lane + 64 * j] = r[j];
    if (lane == 0) d[kPvBatch / 16] = r[4];
  };
  // the word of position 64 g + lane of the stage (two aligned dwords, a funnel shift)
  auto word = [&](uint32_t g) {
    const uint32_t* dw = reinterpret_cast<const uint32_t*>(stg + 64 * g) + (lane >> 2);
    return __builtin_amdgcn_alignbyte(dw[1], dw[0], lane & 3u);
  };
  // one step = kPvG groups: hashes and exchange operands of step s + 1 are computed while step s's
  // exchanges are in flight (issued by one asm statement, waited for by a second that names
  // their results -- the ISA between the two never touches those registers)
  struct Ops {
    uint32_t la[kPvG], mk[kPvG], vv[kPvG], sh[kPvG];
  };
  auto prep = [&](uint32_t q0, uint32_t g0, const uint32_t (&w)[kPvG], Ops& o) {
#pragma unroll
    for (uint32_t k = 0; k < kPvG; ++k) {
      const uint32_t q = q0 + 64 * (g0 + k) + lane;
      const uint32_t h = pv_hash(w[k]);
      const bool v = q + 4 <= n;  // (positions without 4 bytes, and past the block: mask 0)
      o.sh[k] = (h & 1u) << 4;
      o.la[k] = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint32_t*)(&T[h >> 1]));
      o.mk[k] = v ? 0xffffu << o.sh[k] : 0u;  // mask 0: memory unchanged
      o.vv[k] = v ? (q + 1) << o.sh[k] : 0u;
    }
  };
  load(0);
  put();
  for (uint32_t i = 0; i < nbat; ++i) {
    if (i + 1 < nbat) load(i + 1);  // in flight during this batch's exchanges
    const uint32_t q0 = kPvBatch * i;
    const uint32_t ng = min(kPvBatch, n - q0 + 63) >> 6;  // groups of this batch
    uint32_t wa[kPvG], wb[kPvG];
#pragma unroll
    for (uint32_t k = 0; k < kPvG; ++k) {
      wa[k] = word(k);
      wb[k] = word(kPvG + k);
    }
    Ops cur, nxt;
    prep(q0, 0, wa, cur);
    for (uint32_t g0 = 0; g0 < ng; g0 += kPvG) {
      uint32_t old[kPvG];
      static_assert(kPvG == 4, "the asm issues four exchanges");
      // D = (D & ~mask) | value, the old dword back
      asm volatile(
          "ds_mskor_rtn_b32 %0, %4, %8, %12\n"
          "ds_mskor_rtn_b32 %1, %5, %9, %13\n"
          "ds_mskor_rtn_b32 %2, %6, %10, %14\n"
          "ds_mskor_rtn_b32 %3, %7, %11, %15"
          : "=&v"(old[0]), "=&v"(old[1]), "=&v"(old[2]), "=&v"(old[3])
          : "v"(cur.la[0]), "v"(cur.la[1]), "v"(cur.la[2]), "v"(cur.la[3]), "v"(cur.mk[0]), "v"(cur.mk[1]),
            "v"(cur.mk[2]), "v"(cur.mk[3]), "v"(cur.vv[0]), "v"(cur.vv[1]), "v"(cur.vv[2]), "v"(cur.vv[3])
          : "memory");
#pragma unroll
      for (uint32_t k = 0; k < kPvG; ++k) wa[k] = word(min(g0 + 2 * kPvG + k, kPvBatch / 64 - 1));  // two steps ahead
      prep(q0, g0 + kPvG, wb, nxt);
      // the wait names the next step's operands too, so their VALU is issued before it
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(old[0]), "+v"(old[1]), "+v"(old[2]), "+v"(old[3]), "+v"(nxt.la[0]), "+v"(nxt.la[1]),
                     "+v"(nxt.la[2]), "+v"(nxt.la[3]), "+v"(nxt.mk[0]), "+v"(nxt.mk[1]), "+v"(nxt.mk[2]), "+v"(nxt.mk[3]),
                     "+v"(nxt.vv[0]), "+v"(nxt.vv[1]), "+v"(nxt.vv[2]), "+v"(nxt.vv[3])
                   :
                   : "memory");
#pragma unroll
      for (uint32_t k = 0; k < kPvG; ++k) {
        const uint32_t q = q0 + 64 * (g0 + k) + lane;
        if (q < n) pv[q] = (uint16_t)(old[k] >> cur.sh[k]);
      }
      cur = nxt;
#pragma unroll
      for (uint32_t k = 0; k < kPvG; ++k) wb[k] = wa[k];
    }
    if (i + 1 < nbat) put();  // (a wave's LDS accesses run in order: the batch's reads are done)
  }
}
static_assert((kPvBatch / 64) % kPvG == 0, "a batch is whole steps");

// ---- k_compress_lanes ---------------------------------------------------------------------
// cnt bytes of an LDS slice (4-byte aligned) from byte s0 to global g: 16-B pieces assembled from
// five aligned dwords, unaligned 16-B stores, an exact tail (the next chunk's bytes follow)
__device__ inline void copy_out(uint8_t* g, const uint8_t* sl4, uint32_t s0, uint32_t cnt) {
  for (uint32_t at = 0; at < cnt; at += 16) {
    const uint32_t x = s0 + at;
    const uint32_t* w = reinterpret_cast<const uint32_t*>(sl4 + (x & ~3u));
    const uint32_t sh = x & 3u;
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
    const uint32_t v[4] = {__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                           __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh)};
    if (at + 16 <= cnt) {
      *reinterpret_cast<lu128u*>(g + at) = make_uint4(v[0], v[1], v[2], v[3]);
    } else {
      const uint32_t r = cnt - at;
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k) {
        if (4 * k + 4 <= r) {
          *reinterpret_cast<lu32u*>(g + at + 4 * k) = v[k];
        } else if (4 * k < r) {
#pragma unroll
          for (uint32_t e = 0; e < 3; ++e)
            if (4 * k + e < r) g[at + 4 * k + e] = (uint8_t)(v[k] >> (8 * e));
        }
      }
    }
  }
}

// copy tag bytes for (off, L), L in 4..64: copy-1 (L < 12, off < 2048) or copy-2
// (emit_copy_upto_64!, internal.jl:289-304); packed little-endian, and the tag's size
__device__ inline uint32_t copy_tag(uint32_t off, uint32_t L, uint32_t& sz) {
  const bool c1 = L < 12 && off < 2048;
  sz = c1 ? 2u : 3u;
  return c1 ? (1u + ((L - 4) << 2) + ((off >> 3) & 0xe0u)) | ((off & 0xffu) << 8)
            : (2u + ((L - 1) << 2)) | ((off & 0xffffu) << 8);
}

__global__ __launch_bounds__(kLLanes, 1) void k_compress_lanes(CompressArgs a, uint32_t b0) {
  __shared__ __attribute__((aligned(16))) uint8_t data[kBlockSize + 64];
  __shared__ __attribute__((aligned(16))) uint8_t sl[kLLanes * kLPitch + 16];  // per-lane prev[] / output
  __shared__ uint32_t wsum[kLLanes / 64];
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
      constexpr int kLoads = kBlockSize / 16 / kLLanes;
      uint4 v[kLoads];
#pragma unroll
      for (int i = 0; i < kLoads; ++i) v[i] = s16[tid + i * kLLanes];
#pragma unroll
      for (int i = 0; i < kLoads; ++i) d16[tid + i * kLLanes] = v[i];
    } else {
      for (uint32_t k = tid; k < n16; k += kLLanes) d16[k] = s16[k];
      for (uint32_t k = (n & ~15u) + tid; k < n; k += kLLanes) data[k] = src[k];
    }
  } else {
    for (uint32_t k = tid; k < n; k += kLLanes) data[k] = src[k];
  }
  if (tid < 64) data[n + tid] = 0;  // reads past the block see zeros (lengths stop at the chunk end anyway)
  const uint32_t hdr = a.header ? varint_len(n) : 0u;
  if (tid < hdr) dst[tid] = (uint8_t)(((n >> (7 * tid)) & 0x7f) | (tid + 1 < hdr ? 0x80 : 0));
  const uint16_t* pvg = a.prev + (size_t)blockIdx.x * kBlockSize;
  uint8_t* my = sl + kLPitch * tid;  // this lane's slice
  uint32_t op = hdr;                 // output bytes placed so far

  for (uint32_t c0p = 0; c0p < n; c0p += kLLanes * kLChunk) {
    // the pass's prev[] (positions [c0p, c0p + 32 K)) into the slices: coalesced 16-B loads
    {
      const uint32_t np = min(kLLanes * kLChunk, n - c0p);
      const uint4* s16 = reinterpret_cast<const uint4*>(pvg + c0p);
      const uint32_t n16 = (2 * np + 15) >> 4;  // (entries past n are never used: reading them is harmless)
      for (uint32_t k = tid; k < n16; k += kLLanes) {
        const uint4 v = s16[k];  // piece k: lane k / (kLSlice / 16), at 16 (k mod kLSlice / 16) in its slice
        uint32_t* d = reinterpret_cast<uint32_t*>(sl + kLPitch * (k / (kLSlice / 16)) + 16 * (k % (kLSlice / 16)));
        d[0] = v.x;
        d[1] = v.y;
        d[2] = v.z;
        d[3] = v.w;
      }
    }
    __syncthreads();  // (also: the block staging above, and the previous pass's stores from the slices)
    const uint32_t c0 = c0p + tid * kLChunk, ce = min(c0 + kLChunk, n);
    uint32_t p = c0, o = 0, otag = 0, run = 0;
    uint32_t lead = 0, ncopy = 0;  // the leading literal run (its tag byte stays open); copies so far
    bool act = c0 < n, ext = false;
    uint32_t cq = 0, coff = 0, cL = 0, clim = 0;
    auto put_bytes = [&](uint32_t at, uint32_t v, uint32_t cnt) {  // cnt (<= 4) low bytes of v at my[at]
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k)
        if (k < cnt) my[at + k] = (uint8_t)(v >> (8 * k));
    };
    while (ballot(act)) {
      bool emit = false;
      if (act && !ext) {
        // probe positions p .. p+3: their candidates (prev[], u16 position + 1, 0 = none: read
        // before this step's output bytes are written over them) and the bytes at p .. p+10
        const uint64_t pr = lds_ld64(my, 2 * (p - c0));
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
          put_bytes(o, W0, nlit);
          o += nlit;
          run += nlit;
        }
        if (first < 4) {
          if (run) {
            if (ncopy) {  // an internal run (<= 56 bytes): its tag now
              my[otag] = (uint8_t)((run - 1) << 2);
            } else {      // the leading run: its tag is the copy-out's (it may continue the previous chunk's run)
              lead = run;
            }
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
        put_bytes(o, copy_tag(coff, cL, tsz), tsz);
        o += tsz;
        p = cq + cL;
        ++ncopy;
      }
      if (act && !ext && p >= ce) act = false;  // an open run here is the trailing run (run bytes, tag at otag)
    }
    // Literal runs that cross chunk boundaries are merged (within a wave's 64 chunks; they restart
    // at wave boundaries), as the reference's single greedy walk would emit them: chunk k's
    // trailing run continues into k+1's leading run, through chunks that are all literal.
    //   cont: this chunk's leading run continues the previous chunk's trailing run (tag dropped)
    //   mid:  the chunk is all literal and continues a run (no tag at all)
    //   start: the chunk's trailing run starts a run; its tag encodes the run's whole length
    const bool allit = c0 < n && ncopy == 0;
    const uint32_t len = c0 < n ? ce - c0 : 0u;
    if (allit) lead = len;  // (its one run: leading and trailing, tag byte at 0)
    const uint32_t trail = run;
    const uint32_t trail_prev = __builtin_amdgcn_update_dpp(0u, trail, 0x138, 0xf, 0xf, false);  // wave_shr:1
    const bool cont = lead > 0 && trail_prev > 0;
    const bool mid = allit && cont;
    const bool start = trail > 0 && !mid;
    if (lead > 0 && !cont && !allit) my[0] = (uint8_t)((lead - 1) << 2);  // a leading run of its own (<= 60)
    // run length for a start: trail + the leads of the following chunks up to the first non-mid one
    const uint32_t C = scan_dpp(cont ? lead : 0u);  // inclusive
    uint32_t f = mid ? 64u : lane;                   // first non-mid lane at or after each lane (suffix min)
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t o2 = __shfl_down(f, d, 64);
      f = lane + d < 64 ? min(f, o2) : f;
    }
    const uint32_t fn = __shfl_down(f, 1, 64);  // first non-mid lane after this one
    const uint32_t Cf = __shfl(C, lane < 63 ? min(fn, 63u) : 63u, 64);
    const uint32_t runlen = start ? trail + (lane < 63 ? Cf : C) - C : 0u;
    const uint32_t tsz = start ? (runlen <= 60 ? 1u : (runlen <= 256 ? 2u : 3u)) : 0u;
    const uint32_t a0 = cont ? 1u : 0u;             // first staged byte written
    const uint32_t aend = start ? otag : o;          // segment A: staged [a0, aend)
    const uint32_t S = (aend - a0) + (start ? tsz + (o - otag - 1) : 0u);
    const uint32_t incl = scan_dpp(S);
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t base = op, tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < kLLanes / 64; ++w) {
      base += w < wave ? wsum[w] : 0u;
      tot += wsum[w];
    }
    const uint32_t P = base + incl - S;
    copy_out(dst + P, my, a0, aend - a0);
    if (start) {
      const uint32_t q = P + (aend - a0), l1 = runlen - 1;
      if (tsz == 1) {
        dst[q] = (uint8_t)(l1 << 2);
      } else {  // emit_literal! (internal.jl:271-284): 60 or 61 << 2, then len-1 little-endian
        dst[q] = (uint8_t)((58 + tsz) << 2);
        dst[q + 1] = (uint8_t)l1;
        if (tsz == 3) dst[q + 2] = (uint8_t)(l1 >> 8);
      }
      copy_out(dst + q + tsz, my, otag + 1, o - otag - 1);
    }
    op += tot;
    __syncthreads();  // the slices' reads are done before the next pass's prev[] lands in them
  }
  if (tid == 0) a.out_len[b] = op;
}

hipError_t launch_compress_lanes(const CompressArgs& a, uint32_t sub, hipStream_t s) {
  for (uint32_t b0 = 0; b0 < a.nblk; b0 += sub) {
    const uint32_t nb = min(sub, a.nblk - b0);
    hipLaunchKernelGGL(k_prev_insert, dim3(nb), dim3(64), 0, s, a, b0);
    hipLaunchKernelGGL(k_compress_lanes, dim3(nb), dim3(kLLanes), 0, s, a, b0);
  }
  return hipGetLastError();
}

}  // namespace sm
