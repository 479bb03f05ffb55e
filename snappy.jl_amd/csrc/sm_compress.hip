// sm_compress.hip -- batched 64 KiB-block snappy compression for gfx950 (MI355X).
//
// Two kernels, one wavefront (64 lanes) per block, block staged in LDS:
//
//  k_compress_exact  -- "reference mode": byte-identical to Snappy.jl's compress
//                       (src/internal.jl:127-250 incl. quirks Q1/Q3, src/Snappy.jl:20-36 incl.
//                       Q2).  The greedy parse is inherently serial (the u16 hash table at
//                       internal.jl:189-193 carries state between probes), so it runs as
//                       wave-uniform scalar code; the wave parallelises what is parallel:
//                       block staging, table reset, find_match_length (256 B compared per
//                       LDS round, internal.jl:343-387) and literal copies.
//
//  k_compress_fast   -- "fast mode", see sm_compress_fast.hip.
//
// Data layout in HBM: input blocks at in[in_off[b]], outputs at out[out_off[b]] (caller
// reserves max_compressed_length(len)+5 per block, i.e. fixed slots), out_len[b] = bytes.
#include "sm_device.h"
#include "sm_internal.h"

namespace sm {

#if SM_STAMP
__device__ unsigned long long g_stamp_x[8];
#endif
STAMP_MACROS(8)

constexpr uint32_t kLdsPad = 64;  // readable slack after the block for lds_ld32 / wave compares

// ---- output emission (global memory, wave-uniform op) -------------------------------

__device__ inline uint32_t emit_varint(uint8_t* dst, uint32_t op, uint32_t v, uint32_t lane) {
  uint32_t nb = varint_len(v);
  if (lane < nb) dst[op + lane] = (uint8_t)(((v >> (7 * lane)) & 0x7f) | (lane + 1 < nb ? 0x80 : 0));
  return op + nb;
}

// internal.jl:252-287.  ref_q3: one-byte tag only for len < 60 (Snappy.jl); else len-1 < 60.
__device__ inline uint32_t emit_literal_g(uint8_t* dst, uint32_t op, const uint8_t* lds, uint32_t start,
                                          uint32_t len, uint32_t lane, bool ref_q3) {
  uint32_t n = len - 1;
  bool one = ref_q3 ? (len < 60) : (n < 60);
  if (one) {
    if (lane == 0) dst[op] = (uint8_t)(n << 2);
    op += 1;
  } else {
    uint32_t count = n < 256 ? 1 : n < 65536 ? 2 : n < (1u << 24) ? 3 : 4;
    if (lane == 0) dst[op] = (uint8_t)((59 + count) << 2);
    if (lane >= 1 && lane <= count) dst[op + lane] = (uint8_t)(n >> (8 * (lane - 1)));
    op += 1 + count;
  }
  wave_copy_lds_to_global(dst + op, lds, start, len, lane);
  return op + len;
}

// internal.jl:289-304 (single lane)
__device__ inline uint32_t put_copy_upto_64(uint8_t* dst, uint32_t op, uint32_t offset, uint32_t len) {
  if (len < 12 && offset < 2048) {
    dst[op] = (uint8_t)(1 + ((len - 4) << 2) + ((offset >> 3) & 0xe0));
    dst[op + 1] = (uint8_t)offset;
    return op + 2;
  }
  dst[op] = (uint8_t)(2 + ((len - 1) << 2));
  dst[op + 1] = (uint8_t)offset;
  dst[op + 2] = (uint8_t)(offset >> 8);
  return op + 3;
}

// internal.jl:306-329 (single lane)
__device__ inline uint32_t put_copy(uint8_t* dst, uint32_t op, uint32_t offset, uint32_t len) {
  if (len < 12) return put_copy_upto_64(dst, op, offset, len);
  while (len >= 68) { op = put_copy_upto_64(dst, op, offset, 64); len -= 64; }
  if (len > 64) { op = put_copy_upto_64(dst, op, offset, 60); len -= 60; }
  return put_copy_upto_64(dst, op, offset, len);
}

__device__ inline uint32_t emit_copy_g(uint8_t* dst, uint32_t op, uint32_t offset, uint32_t len, uint32_t lane) {
  if (lane == 0) put_copy(dst, op, offset, len);
  return op + copy_tag_bytes(offset, len);
}

__device__ inline uint32_t uld32(const uint8_t* lds, uint32_t pos) { return uniform(lds_ld32(lds, pos)); }

// ---- reference mode ------------------------------------------------------------------
//
// Batched exact probes.  After every copy the reference's literal search probes positions
// p0 + D[k], D[0] = 0, D[k+1] = D[k] + (skip_k >> 5), skip_0 = 32, skip_{k+1} = skip_k +
// (skip_k >> 5) (internal.jl:162-175): a fixed sequence, so 64 probes go in one step, lane j =
// probe k0 + j.  Probe k runs only if p0 + D[k+1] <= ip_limit (:175, checked before the probe).
// Its candidate is the table entry as of just before it (:190), i.e. the latest earlier
// insert with its hash.  Inserted positions only ever increase within a fragment (probes, then
// ip-1 and ip after a copy, :228-235), so the table holds pos+1 (0 = never written, read as
// candidate 0 exactly like the reference's 0xffff refill, Snappy.jl:30 / internal.jl:190) and
// ds_max_rtn_u32 gives every lane its exact sequential candidate: conflicting lanes of one
// instruction are serviced in ascending lane order on gfx950 (tools/probe_lds.hip; the
// byte-parity tests pin it).  The first lane whose candidate matches is the reference's
// match; the inserts of later lanes never happened sequentially and are undone exactly: for
// each hash, the first later lane's return value is the entry's correct value.

constexpr uint32_t kMaxProbes = 320;  // D[k] > 65536 for k >= ~250: a search never gets further

__global__ __launch_bounds__(64) void k_compress_exact(CompressArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t sdata[kBlockSize + kLdsPad];
  __shared__ __attribute__((aligned(16))) uint32_t stab[kMaxHashTableSize];  // pos + 1, 0 = empty
  __shared__ uint32_t sD[kMaxProbes + 1];                                     // probe offsets

  const uint32_t b = blockIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t n = a.in_len[b];
  const uint8_t* src = a.in + a.in_off[b];
  uint8_t* dst = a.out + a.out_off[b];
  if (n > kBlockSize) {  // batch contract violated: refuse instead of overrunning LDS
    if (lane == 0) a.out_len[b] = 0xffffffffu;
    return;
  }

  wave_load_global_to_lds(sdata, src, n, lane);
  if (lane < kLdsPad) sdata[n + lane] = 0;
  const uint32_t tsize = a.table_size ? a.table_size : hashtable_size(n);      // Snappy.jl:27 (Q2)
  const uint32_t shift = 32 - (31 - __builtin_clz(tsize));                     // internal.jl:128
  for (uint32_t k = lane; k < tsize; k += kWave) stab[k] = 0;                  // Snappy.jl:30
  if (lane == 0) {
    uint32_t d = 0, skip = 32;
    for (uint32_t k = 0; k <= kMaxProbes; ++k) {
      sD[k] = d;
      const uint32_t step = skip >> 5;                                         // :170-172
      skip += step;
      d = min(d + step, 0x20000u);
    }
  }
  __syncthreads();

  uint32_t op = a.header ? emit_varint(dst, 0, n, lane) : 0;                   // Snappy.jl:26
  if (n == 0) {
    if (lane == 0) a.out_len[b] = op;
    return;
  }
  const uint32_t e = n - 1;                  // inclusive end (ip_end)
  const int32_t ip_limit = (int32_t)n - 16;  // internal.jl:131, Q1: 1-based ip_end-15
  uint32_t ip = 0, next_emit = 0, cand = 0;

  STAMP_DECL
  if (n >= kInputMarginBytes) {                                                // internal.jl:133
    for (;;) {
      STAMP(4)
      ip += 1;                                                                 // :163
      // literal search, 64 probes per step (:167-194)
      const uint32_t p0 = ip;
      bool found = false;
      for (uint32_t k0 = 0; k0 < kMaxProbes; k0 += kWave) {
        const uint32_t p = p0 + sD[k0 + lane];
        const bool valid = (int32_t)(p0 + sD[k0 + lane + 1]) <= ip_limit;     // :175
        const uint32_t cur = valid ? lds_ld32(sdata, p) : 0u;
        const uint32_t h = hash32(cur, shift);
        uint32_t r = 0;
        if (valid) r = __hip_atomic_fetch_max(&stab[h], p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t c = r ? r - 1 : 0u;                                     // :190
        const bool hit = valid && lds_ld32(sdata, c) == cur;                   // :193
        const uint64_t hm = ballot(hit);
        if (hm) {
          const uint32_t j = ctz64(hm);
          const uint32_t pj = readlane(p, j);
          if (valid && lane > j && r <= pj + 1) stab[h] = r;                   // undo later probes
          ip = pj;
          cand = readlane(c, j);
          found = true;
          break;
        }
        if (ballot(valid) != ~0ull) break;                                     // :175 -> remainder
      }
      STAMP(0)
      if (!found) goto emit_remainder;
      op = emit_literal_g(dst, op, sdata, next_emit, ip - next_emit, lane, true);   // :200
      STAMP(1)
      for (;;) {                                                               // :211-239
        STAMP_COUNT(6, 1)
        uint32_t avail = e - (ip + 4) + 1;
        uint32_t matched = 4 + wave_match_length(sdata, cand + 4, ip + 4, avail, lane);  // :216
        STAMP(2)
        op = emit_copy_g(dst, op, ip - cand, matched, lane);                   // :217
        ip += matched;
        next_emit = ip;
        if ((int32_t)ip >= ip_limit) goto emit_remainder;                      // :222
        uint32_t prev_hash = hash32(uld32(sdata, ip - 1), shift);              // :228
        uint32_t input_bytes = uld32(sdata, ip);
        uint32_t cur_hash = hash32(input_bytes, shift);
        if (lane == 0) stab[prev_hash] = ip;                                   // :233 (pos ip-1)
        const uint32_t rv = uniform(stab[cur_hash]);                           // :234
        cand = rv ? rv - 1 : 0u;
        if (lane == 0) stab[cur_hash] = ip + 1;                                // :235 (pos ip)
        if (input_bytes != uld32(sdata, cand)) {                               // :238
          STAMP(3)
          break;
        }
        STAMP(3)
      }
    }
  }
emit_remainder:
  if (next_emit <= e) op = emit_literal_g(dst, op, sdata, next_emit, e - next_emit + 1, lane, true);  // :244-248
  STAMP(5)
  STAMP_FLUSH(g_stamp_x)
  if (lane == 0) a.out_len[b] = op;
}

// ---- gather (single-stream assembly) ---------------------------------------------------

__global__ __launch_bounds__(256) void k_gather(const uint8_t* __restrict__ src, const uint64_t* src_off,
                                                 const uint32_t* len, const uint64_t* dst_off,
                                                 uint8_t* __restrict__ dst) {
  const uint32_t b = blockIdx.x;
  const uint8_t* s = src + src_off[b];
  uint8_t* d = dst + dst_off[b];
  const uint32_t n = len[b];
  for (uint32_t k = threadIdx.x; k < n; k += blockDim.x) d[k] = s[k];
}

#if SM_STAMP
extern "C" int sm_debug_stamps_x(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamp_x), sizeof(g_stamp_x)) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[8] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_x), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

hipError_t launch_compress(const CompressArgs& a, int mode, hipStream_t s) {
  if (a.nblk == 0) return hipSuccess;
  if (mode != 0) return launch_compress_fast(a, mode, s);
  hipLaunchKernelGGL(k_compress_exact, dim3(a.nblk), dim3(64), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_gather(const uint8_t* src, const uint64_t* src_off, const uint32_t* len,
                         const uint64_t* dst_off, uint8_t* dst, uint32_t nblk, hipStream_t s) {
  if (nblk == 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather, dim3(nblk), dim3(256), 0, s, src, src_off, len, dst_off, dst);
  return hipGetLastError();
}

}  // namespace sm
