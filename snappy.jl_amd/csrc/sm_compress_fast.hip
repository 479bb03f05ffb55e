// sm_compress_fast.hip -- "fast mode" batched snappy compression for gfx950 (MI355X).
//
// Produces a valid snappy stream per 64 KiB block (decodes bit-exactly under Snappy.jl's
// uncompress, src/internal.jl:411-466) without the reference's serial greedy loop.
//
// Work decomposition: one workgroup of 4 waves per block, the block staged once in LDS
// (64 KiB) next to a shared latest-position hash table (4088 x u32).  80 KiB per workgroup,
// so two blocks (8 waves) are resident per CU.  The block is cut into 256-byte chunks; a
// chunk's parse never crosses its end (copies are truncated at the chunk boundary and
// literal runs end there), so chunks are parsed independently: in round r wave w owns chunk
// 4r+w.  Per chunk:
//   1. hash all 256 positions (4 per lane, position = c0 + 64*j + lane);
//   2. candidates: the table as of the previous round (read before this round's updates),
//      or -- second chance -- the table after this round's atomicMax updates when that
//      entry is an EARLIER position (deterministic: max is order-independent);
//   3. verify the 4 bytes and extend (unaligned ds_read_b64 compares, 16 B eagerly);
//   4. greedy walk over the 4 match ballots (scalar: s_ff1 + v_readlane per copy), tokens
//      written into lanes with a lane-select;
//   5. per-token sizes, wave prefix sum, chunk sizes exchanged through LDS -> exact output
//      offsets; tag bytes written by token lanes, literal bytes scattered by position lanes.
// Two barriers per round: [updates] B1 [2nd-chance, verify, extend, walk, size, next-round
// lookups] B2 [emit].
#include "sm_device.h"
#include "sm_internal.h"

namespace sm {

constexpr uint32_t kFTab = 4088;   // table entries: 64 KiB + 4088*4 + 16 <= 80 KiB
constexpr uint32_t kChunk = 256;
constexpr uint32_t kWavesPerBlock = 4;
constexpr uint32_t kEagerExt = 16;  // bytes compared per lane before deferring to the wave

typedef uint32_t __attribute__((aligned(1))) u32u;
typedef uint64_t __attribute__((aligned(1))) u64u;

__device__ inline uint32_t ld32u(const uint8_t* p) { return *reinterpret_cast<const u32u*>(p); }
__device__ inline uint64_t ld64u(const uint8_t* p) { return *reinterpret_cast<const u64u*>(p); }

__device__ inline uint32_t ftab_index(uint32_t w) { return __umulhi(w * kHashMul, kFTab); }

// copy tags for (offset, len), len <= 256 here; internal.jl:289-329 encoding
__device__ inline void store_copy_tags(uint8_t* dst, uint32_t o, uint32_t offset, uint32_t len) {
  while (len >= 68) {
    dst[o] = (uint8_t)(2 + (63 << 2));
    dst[o + 1] = (uint8_t)offset;
    dst[o + 2] = (uint8_t)(offset >> 8);
    o += 3;
    len -= 64;
  }
  if (len > 64) {
    dst[o] = (uint8_t)(2 + (59 << 2));
    dst[o + 1] = (uint8_t)offset;
    dst[o + 2] = (uint8_t)(offset >> 8);
    o += 3;
    len -= 60;
  }
  if (len < 12 && offset < 2048) {
    dst[o] = (uint8_t)(1 + ((len - 4) << 2) + ((offset >> 3) & 0xe0));
    dst[o + 1] = (uint8_t)offset;
  } else {
    dst[o] = (uint8_t)(2 + ((len - 1) << 2));
    dst[o + 1] = (uint8_t)offset;
    dst[o + 2] = (uint8_t)(offset >> 8);
  }
}

// match length of lds[i1..] vs lds[i2..] capped at avail (<= 512 per round), whole wave
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
      res = off + fb;
      if (res > avail) res = avail;
      stop = (fb < 8) || (off + 8 >= avail);
    }
    uint64_t m = ballot(stop);
    if (m) return readlane(res, ctz64(m));
    base += 8 * kWave;
  }
}

__global__ __launch_bounds__(256) void k_compress_fast(CompressArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[kBlockSize + 4 * kFTab + 16];
  uint8_t* data = smem;
  uint32_t* T = reinterpret_cast<uint32_t*>(smem + kBlockSize);
  uint32_t* csize = T + kFTab;  // per-wave chunk output size of the current round

  const uint32_t b = blockIdx.x;
  const uint32_t tid = threadIdx.x;
  const uint32_t wave = uniform(tid >> 6);  // readfirstlane: lets the walk compile to SALU
  const uint32_t lane = tid & 63;
  const uint32_t n = a.in_len[b];
  const uint8_t* src = a.in + a.in_off[b];
  uint8_t* dst = a.out + a.out_off[b];
  if (n > kBlockSize) {
    if (tid == 0) a.out_len[b] = 0xffffffffu;
    return;
  }

  // stage the block (16 B per thread when aligned) and clear the table
  if (((uintptr_t)src & 15) == 0) {
    const uint4* s16 = reinterpret_cast<const uint4*>(src);
    uint4* d16 = reinterpret_cast<uint4*>(data);
    for (uint32_t k = tid; k < (n >> 4); k += 256) d16[k] = s16[k];
    for (uint32_t k = (n & ~15u) + tid; k < n; k += 256) data[k] = src[k];
  } else {
    for (uint32_t k = tid; k < n; k += 256) data[k] = src[k];
  }
  for (uint32_t k = tid; k < kFTab; k += 256) T[k] = 0;

  uint32_t op = 0;
  if (a.header) {
    uint32_t nb = varint_len(n);
    if (tid < nb) dst[tid] = (uint8_t)(((n >> (7 * tid)) & 0x7f) | (tid + 1 < nb ? 0x80 : 0));
    op = nb;
  }
  __syncthreads();

  const uint32_t nchunks = (n + kChunk - 1) / kChunk;
  const uint32_t rounds = (nchunks + kWavesPerBlock - 1) / kWavesPerBlock;

  uint32_t w[4], h[4], t1[4];
  {
    const uint32_t c0 = wave * kChunk;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint32_t q = c0 + 64 * j + lane;
      w[j] = ld32u(data + (q < n ? q : 0));
      h[j] = ftab_index(w[j]);
      t1[j] = 0;
    }
  }

  for (uint32_t r = 0; r < rounds; ++r) {
    const uint32_t k = r * kWavesPerBlock + wave;
    const bool active = k < nchunks;
    const uint32_t c0 = k * kChunk;
    const uint32_t ce = active ? min(c0 + kChunk, n) : c0;

    // (a) insert this chunk's positions
    if (active) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t q = c0 + 64 * j + lane;
        if (q + 4 <= n) __hip_atomic_fetch_max(&T[h[j]], q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    __syncthreads();  // B1

    // (b) candidates, verify, extend, walk, size
    uint32_t ml[4], cand[4];
    uint64_t mask[4];
    uint64_t ts[4] = {0, 0, 0, 0};
    uint32_t tm = 0, tL = 0, td = 0;  // token (lane t): copy start, copy length, offset
    uint32_t ntok = 0;
    uint32_t incl = 0, sz = 0, litlen = 0, littag = 0, ls = 0;
    if (active) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t q = c0 + 64 * j + lane;
        bool can = q + 4 <= ce;
        uint32_t t2 = T[h[j]];
        uint32_t c = (t2 != 0 && t2 - 1 < q) ? t2 - 1 : t1[j] - 1u;
        bool ok = can && c < q && ld32u(data + c) == w[j];
        uint32_t len = 0;
        if (ok) {
          uint32_t cap = ce - q - 4;
          uint32_t e = 0;
          for (;;) {
            uint64_t x = ld64u(data + c + 4 + e) ^ ld64u(data + q + 4 + e);
            if (x) {
              e += (uint32_t)(__builtin_ctzll(x) >> 3);
              break;
            }
            e += 8;
            if (e >= kEagerExt || e >= cap) break;
          }
          len = 4 + (e < cap ? e : cap);
        }
        ml[j] = len;
        cand[j] = c;
        mask[j] = ballot(ok);
      }
      // greedy walk (wave-uniform scalar code)
      uint32_t p = c0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t s0 = c0 + 64 * j;
        for (;;) {
          if (p >= s0 + 64) break;
          uint32_t rel = p > s0 ? p - s0 : 0;
          uint64_t mm = mask[j] >> rel;
          if (!mm) break;
          uint32_t l = rel + ctz64(mm);
          uint32_t q = s0 + l;
          uint32_t L = readlane(ml[j], l);
          uint32_t c = readlane(cand[j], l);
          if (L >= 4 + kEagerExt && q + L < ce) L += wave_match_len8(data, c + L, q + L, ce - q - L, lane);
          const bool me = lane == ntok;  // token ntok lives in lane ntok
          tm = me ? q : tm;
          tL = me ? L : tL;
          td = me ? q - c : td;
          ts[j] |= 1ull << l;
          ++ntok;
          p = q + L;
        }
      }
      if (p < ce) {  // trailing literal run of the chunk: a token with no copy
        const bool me = lane == ntok;
        tm = me ? ce : tm;
        tL = me ? 0u : tL;
        ++ntok;
      }
      // sizes and offsets (token t in lane t)
      uint32_t end = tm + tL;
      uint32_t prev_end = __shfl_up(end, 1, 64);
      ls = lane == 0 ? c0 : prev_end;
      if (lane < ntok) {
        litlen = tm - ls;
        littag = litlen == 0 ? 0 : (litlen <= 60 ? 1 : 2);
        sz = littag + litlen + (tL ? copy_tag_bytes(td, tL) : 0);
      }
      incl = wave_incl_scan(sz, lane);
      if (lane == 0) csize[wave] = ntok ? readlane(incl, ntok - 1) : 0;
    } else {
      if (lane == 0) csize[wave] = 0;
    }

    // next round's words, hashes and first-chance candidates (table as of this round)
    uint32_t wn[4], hn[4], t1n[4];
    {
      const uint32_t k2 = k + kWavesPerBlock;
      const uint32_t c2 = k2 * kChunk;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t q = c2 + 64 * j + lane;
        wn[j] = ld32u(data + (q < n ? q : 0));
        hn[j] = ftab_index(wn[j]);
        t1n[j] = (k2 < nchunks) ? T[hn[j]] : 0;
      }
    }
    __syncthreads();  // B2

    // (c) emit at the exact output offset
    uint32_t before = 0, total = 0;
#pragma unroll
    for (uint32_t v = 0; v < kWavesPerBlock; ++v) {
      uint32_t s = csize[v];
      before += (v < wave) ? s : 0;
      total += s;
    }
    if (active) {
      const uint32_t base = op + before;
      uint32_t o = base + incl - sz;
      if (lane < ntok) {
        if (littag == 1) {
          dst[o] = (uint8_t)((litlen - 1) << 2);
        } else if (littag == 2) {
          dst[o] = (uint8_t)(60 << 2);
          dst[o + 1] = (uint8_t)(litlen - 1);
        }
        if (tL) store_copy_tags(dst, o + littag + litlen, td, tL);
      }
      // literal bytes: position lanes scatter into their token's literal run
      const int32_t delta = (int32_t)(o + littag) - (int32_t)ls;  // valid in token lanes
      const uint32_t end = tm + tL;
      uint32_t below = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t x = c0 + 64 * j + lane;
        uint32_t cnt = below + __builtin_amdgcn_mbcnt_hi((uint32_t)(ts[j] >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)ts[j], 0u));
        cnt += (uint32_t)(ts[j] >> lane) & 1u;  // tokens with copy start <= x
        uint32_t pend = __shfl(end, cnt ? cnt - 1 : 0, 64);
        int32_t dl = __shfl(delta, cnt, 64);
        bool lit = x < ce && (cnt == 0 || x >= pend);
        if (lit) dst[(int32_t)x + dl] = (uint8_t)w[j];
        below += __builtin_popcountll(ts[j]);
      }
    }
    op += total;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      w[j] = wn[j];
      h[j] = hn[j];
      t1[j] = t1n[j];
    }
  }
  if (tid == 0) a.out_len[b] = op;
}

hipError_t launch_compress_fast(const CompressArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_compress_fast, dim3(a.nblk), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace sm
