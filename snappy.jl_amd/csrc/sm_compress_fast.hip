// sm_compress_fast.hip -- the incompressible screen that runs before the fast-mode compressor
// (k_compress_sc, sm_compress_sc.hip), and the fast-mode launch.
//
// The screen emits a block with no repeated content as ONE literal (the reference's own output for
// such a block, src/internal.jl:271-284) and marks every other block for the parse.  The round-1/2
// parse kernel that used to live here (k_compress_fast) was replaced by k_compress_sc in round 3
// and removed in round 4.
#include "sm_device.h"
#include "sm_internal.h"

namespace sm {

constexpr uint32_t kScreenTodo = 0xfffffffeu;  // out_len mark of k_literal_screen: the parse compresses this block

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
constexpr uint32_t kScrAnchorDiv = 256;   // fewer than one anchor per 256 bytes scanned: not random (expected: 1 per 64)
#ifndef SM_SCR_THREADS
#define SM_SCR_THREADS 512
#endif
#ifndef SM_SCR_FIRST
#define SM_SCR_FIRST 1
#endif
constexpr uint32_t kScrThreads = SM_SCR_THREADS;
constexpr uint32_t kScrPieces = kBlockSize / 16 / kScrThreads;  // 16-B pieces per thread (8)
constexpr uint32_t kScrFirst = SM_SCR_FIRST;                    // pieces of the first pass (8 KiB)
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
__device__ inline uint32_t scr_anchors(uint32_t* tab, uint4 v, uint4 nv, uint32_t o, uint32_t n, bool nvalid,
                                       uint32_t& anc) {
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
      ++anc;
    }
  }
  return rep;
}

__global__ __launch_bounds__(kScrThreads) void k_literal_screen(CompressArgs a) {
  __shared__ uint32_t tab[1u << kScrTabBits];
  __shared__ uint32_t cnt[4];  // repeated anchors (first pass, rest), anchors (first pass, rest)
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const uint32_t b = blockIdx.x;
  uint32_t n;
  uint64_t ioff, ooff;
  if (a.plan_n) {  // a single-buffer input: this block's fragment-table entry is the screen's to write
    ioff = (uint64_t)b * kBlockSize;
    n = (uint32_t)min((uint64_t)kBlockSize, a.plan_n - ioff);
    ooff = (uint64_t)b * a.plan_slot;
    if (tid == 0) {
      const_cast<uint64_t*>(a.in_off)[b] = ioff;
      const_cast<uint32_t*>(a.in_len)[b] = n;
      const_cast<uint64_t*>(a.out_off)[b] = ooff;
    }
  } else {
    n = a.in_len[b];
    ioff = a.in_off[b];
    ooff = a.out_off[b];
  }
  const uint8_t* src = a.in + ioff;
  uint8_t* dst = a.out + ooff;
  if (a.in_host && n <= kBlockSize) {  // the upload folded in: this block's bytes to the device copy
    src = a.in_host + ioff;
    uint8_t* const d = const_cast<uint8_t*>(a.in) + ioff;
    const bool al = (((uintptr_t)src | (uintptr_t)d) & 15) == 0;
    const uint32_t n16 = al ? n >> 4 : 0u;
    for (uint32_t k = tid; k < n16; k += kScrThreads)
      reinterpret_cast<uint4*>(d)[k] = reinterpret_cast<const uint4*>(src)[k];
    for (uint32_t k = 16 * n16 + tid; k < n; k += kScrThreads) d[k] = src[k];
  }
  if (n < kScrMinLen || n > kBlockSize) {
    if (tid == 0) a.out_len[b] = kScreenTodo;
    return;
  }
  const bool aligned = ((uintptr_t)src & 15) == 0;
  for (uint32_t k = tid; k < (1u << kScrTabBits); k += kScrThreads) tab[k] = kScrEmpty;
  if (tid < 4) cnt[tid] = 0;
  uint4 v[kScrPieces];
#pragma unroll
  for (uint32_t i = 0; i < kScrPieces; ++i) v[i] = make_uint4(0, 0, 0, 0);
  // piece i of thread t: bytes [16 (t + 512 i), +16); lane + 1 holds the next piece (a wave's last
  // lane: its positions 13..15 are skipped -- 3 of every 1,024)
  auto pass = [&](uint32_t i0, uint32_t i1, uint32_t slot) {
#pragma unroll
    for (uint32_t i = i0; i < i1; ++i) v[i] = scr_load16(src, 16 * (tid + kScrThreads * i), n, aligned);
    __syncthreads();  // (the table is initialised)
    uint32_t rep = 0, anc = 0;
#pragma unroll
    for (uint32_t i = i0; i < i1; ++i) {
      uint4 nv;
      nv.x = __builtin_amdgcn_update_dpp(0u, v[i].x, 0x130, 0xf, 0xf, false);  // wave_shl:1
      rep += scr_anchors(tab, v[i], nv, 16 * (tid + kScrThreads * i), n, lane < 63, anc);
    }
    rep = __builtin_amdgcn_readlane(scan_dpp(rep), 63);
    anc = __builtin_amdgcn_readlane(scan_dpp(anc), 63);
    if (lane == 0 && rep) atomicAdd(&cnt[slot], rep);
    if (lane == 0 && anc) atomicAdd(&cnt[2 + slot], anc);
    __syncthreads();
  };
  pass(0, kScrFirst, 0);
  if (cnt[0] >= kScrMin) {  // text and structured data decide on their first 8 KiB
    if (tid == 0) a.out_len[b] = kScreenTodo;
    return;
  }
  if (n > 16 * kScrThreads * kScrFirst) pass(kScrFirst, kScrPieces, 1);
  // Too few anchors for the bytes scanned (random data has one per 64 positions: ~1,024 in a
  // block) means few distinct words -- a constant run or a short period, whose words may all miss
  // the anchor range -- not random data: that block goes to the parse too (a constant 64 KiB
  // block was one 65,542-byte literal, against the reference's 3,077 bytes).
  const uint32_t scanned = min(n, n > 16 * kScrThreads * kScrFirst ? kBlockSize : 16 * kScrThreads * kScrFirst);
  if (cnt[0] + cnt[1] >= kScrMin || (cnt[2] + cnt[3]) * kScrAnchorDiv < scanned) {
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


// modes 1 (SM_MODE_FAST) and 2 (SM_MODE_FAST_DENSE): the screen first, then the super-chunk parse
// (k_compress_sc) of the blocks it marked kScreenTodo.
hipError_t launch_compress_fast(const CompressArgs& a0, int mode, hipStream_t s) {
  CompressArgs a = a0;
  a.screened = 1;
  hipLaunchKernelGGL(k_literal_screen, dim3(a.nblk), dim3(kScrThreads), 0, s, a);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_compress_sc(a, mode, s);
}

// the screen, then the parse in parts (k_compress_sc_span)
hipError_t launch_compress_span(const CompressArgs& a0, int mode, const ScSpan& sp, hipStream_t s) {
  if (mode != 1 && mode != 2) return hipErrorInvalidValue;
  CompressArgs a = a0;
  a.screened = 1;
  hipLaunchKernelGGL(k_literal_screen, dim3(a.nblk), dim3(kScrThreads), 0, s, a);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_compress_sc_span(a, mode, sp, s);
}

}  // namespace sm
