// sm_compress.hip -- batched 64 KiB-block snappy compression for gfx950 (MI355X).
//
//  k_compress_exact  -- "reference mode": byte-identical to Snappy.jl's compress
//                       (src/internal.jl:127-250 incl. quirks Q1/Q3, src/Snappy.jl:20-36 incl.
//                       Q2).  The greedy parse is serial, so one wave runs it per block as
//                       wave-uniform code; five blocks share a CU (the block is read from HBM,
//                       only the 32 KiB table is in LDS).  See "reference mode" below.
//
//  k_compress_fast   -- "fast mode", see sm_compress_fast.hip.
//
// Data layout in HBM: input blocks at in[in_off[b]], outputs at out[out_off[b]] (caller
// reserves max_compressed_length(len)+5 per block, i.e. fixed slots), out_len[b] = bytes.
#include <type_traits>

#include "sm_device.h"
#include "sm_internal.h"

namespace sm {


// ---- output emission (global memory, wave-uniform op) -------------------------------

__device__ inline uint32_t emit_varint(uint8_t* dst, uint32_t op, uint32_t v, uint32_t lane) {
  uint32_t nb = varint_len(v);
  if (lane < nb) dst[op + lane] = (uint8_t)(((v >> (7 * lane)) & 0x7f) | (lane + 1 < nb ? 0x80 : 0));
  return op + nb;
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

// ---- reference mode ------------------------------------------------------------------
//
// The reference's greedy parse (internal.jl:127-250) is serial: the hash table carries state
// from probe to probe (:189-193), and skip and limit depend on it.  One wave runs it per block
// as wave-uniform code.  The kernel's speed is therefore how many parses run at once per CU,
// times how short each parse's dependency chain is:
//
//  * Five parses per CU.  The block is read in place from HBM through a buffer resource
//    (range-checked to exactly the block; its lines stay in L2), and the only LDS is the
//    32 KiB table of 16 K u16 positions (0 = empty = candidate 0, as the reference's 0xffff
//    fill reads, Snappy.jl:30, internal.jl:190-191).
//    Staging the block in LDS instead fits one parse per CU (2.3-2.8 GB/s measured).
//  * Batched exact probes.  After every copy the literal search probes positions p0 + D[k],
//    D[0] = 0, D[k+1] = D[k] + (skip_k >> 5), skip_0 = 32, skip_{k+1} = skip_k + (skip_k >> 5)
//    (:162-175): a fixed sequence, so 64 probes go in one step, lane j = probe k0 + j.  Probe k
//    runs only if p0 + D[k+1] <= ip_limit (:175, checked before the probe).  Its candidate is
//    the table entry as of just before it (:190).  Each lane exchanges its half-dword entry
//    with ds_mskor_rtn_b32; the lanes of one LDS instruction are serviced in ascending lane
//    order on gfx950 (tools/probe_lds.hip; the byte-parity tests pin it), so every lane gets
//    its exact sequential candidate.  The first lane whose candidate matches is the
//    reference's match; the inserts of later lanes never happened sequentially and are undone
//    exactly: for each hash, the first later lane's returned entry is the correct value.
//  * Fused verification.  A copy step compares 256 bytes at cand and ip in one round; bytes
//    [0, 4) are the reference's verification (:238), the rest find_match_length (:216).  The
//    words at ip-1 and ip for the next step's hashes (:228-231) come out of the same round's
//    registers (two readlanes), not from another load.
//  * Deferred emission.  A copy is a token (position, offset, length) written into lane
//    (copy index mod 64); every 64 copies the wave emits them together: sizes, a DPP scan for
//    the output offsets, then each lane writes its literal run (the bytes since the previous
//    copy; runs over 64 bytes by the whole wave) and its copy tags.  The bytes equal the
//    reference's in-line emission (:200, :217), which depends only on the token sequence.

constexpr uint32_t kMaxProbes = 320;  // D[k] > 65536 for k >= ~250: a search never gets further
constexpr uint32_t kProbeSteps = kMaxProbes / kWave;
constexpr uint32_t kTabBytes = 2 * kMaxHashTableSize;

// The block in HBM through a raw buffer resource over exactly [0, n): a dword load at offset o
// returns 0 when o + 4 > n (the whole dword), and unaligned dword loads are served (both
// measured on gfx950, tools/probes/buffer_range.hip).  word(pos) therefore loads at
// min(pos, n - 4) and shifts, so the bytes below n are exact and the bytes past it read 0
// (the zero slack the reference's find_match_length never compares) -- and no load touches
// memory past the block.  A position at or past n (a shift of 32 or more) gives 0 explicitly:
// such a shift is undefined in C++, and the hardware's v_lshrrev would mask it to 5 bits.
struct BlockBytes {
  __amdgpu_buffer_rsrc_t r;
  uint32_t nm4;  // n - 4 (word() is used only when n >= 15)
  __device__ uint32_t word(uint32_t pos) const {
    const uint32_t pc = min(pos, nm4), sh = pos - pc;  // sh: 0..3 below n, >= 4 at or past n
    const uint32_t w = __builtin_amdgcn_raw_buffer_load_b32(r, (int)pc, 0, 0);
    return sh < 4 ? w >> (sh << 3) : 0u;
  }
  __device__ uint32_t byte(uint32_t pos) const { return __builtin_amdgcn_raw_buffer_load_b8(r, (int)pos, 0, 0); }
};

// The block staged in LDS (one parse per CU, for single calls and small batches): the same bytes
// as BlockBytes -- exact below n, 0 at and past n (the staging zeroes 32 bytes past n, and a
// position past n is clamped to n) -- at LDS latency instead of L2/HBM latency on the parse's
// dependency chain (a lone 64 KiB fragment's parse is that chain: ~2 loads per probe step).
struct LdsBytes {
  const uint8_t* blk;
  uint32_t n;
  __device__ uint32_t word(uint32_t pos) const { return lds_ld32(blk, min(pos, n)); }
  __device__ uint32_t byte(uint32_t pos) const { return blk[min(pos, n)]; }
};
constexpr uint32_t kLdsBlockPad = 32;

// Table entry h is half (h & 1) of dword h >> 1 and holds a position, 0 when never written.
// The reference stores pos - 1 with 0xffff = empty and reads candidate (entry + 1) mod 2^16
// (Snappy.jl:30, internal.jl:190-191): the same candidates, position 0 and "empty" alike
// giving 0, without the decode on the parse's chain.  The probe's exchange and its wait are
// one asm statement with an early-clobber result, so the compiler cannot copy the result
// register before the data lands.  Returns the entry's old value (the candidate).
__device__ inline uint32_t tab_probe(uint32_t* t, uint32_t h, uint32_t p) {
  const uint32_t sh = (h & 1u) << 4;
  const uint32_t addr = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint32_t*)(&t[h >> 1]));
  const uint32_t mk = 0xffffu << sh, v = p << sh;
  uint32_t old;
  asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(old)
               : "v"(addr), "v"(mk), "v"(v)
               : "memory");
  return (old >> sh) & 0xffffu;
}

// wave-cooperative copy of len block bytes from s to global memory (16-byte stores in the body)
template <class B>
__device__ inline void copy_to_global(const B& S, uint8_t* __restrict__ g, uint32_t s, uint32_t len,
                                      uint32_t lane) {
  uint32_t head = (uint32_t)((16 - ((uintptr_t)g & 15)) & 15);
  if (head > len) head = len;
  if (lane < head) g[lane] = (uint8_t)S.byte(s + lane);
  g += head; s += head; len -= head;
  const uint32_t n16 = len >> 4;
  uint4* g16 = reinterpret_cast<uint4*>(g);
  // four 16-byte units per lane per step, all loads issued before the stores (a whole
  // incompressible block is one literal: 64 steps of one load round trip each otherwise)
  constexpr uint32_t kU = 4;
  for (uint32_t k0 = lane; k0 < n16; k0 += kU * kWave) {
    uint4 v[kU];
#pragma unroll
    for (uint32_t i = 0; i < kU; ++i) {
      const uint32_t p = s + 16 * (k0 + i * kWave);
      if (k0 + i * kWave < n16) v[i] = make_uint4(S.word(p), S.word(p + 4), S.word(p + 8), S.word(p + 12));
    }
#pragma unroll
    for (uint32_t i = 0; i < kU; ++i)
      if (k0 + i * kWave < n16) g16[k0 + i * kWave] = v[i];
  }
  const uint32_t done = n16 << 4;
  if (lane < len - done) g[done + lane] = (uint8_t)S.byte(s + done + lane);
}

// internal.jl:252-287, whole wave.  Q3: the one-byte tag only for len < 60.
template <class B>
__device__ inline uint32_t emit_literal_w(const B& S, uint8_t* dst, uint32_t op, uint32_t start,
                                          uint32_t len, uint32_t lane) {
  const uint32_t n = len - 1;
  if (len < 60) {
    if (lane == 0) dst[op] = (uint8_t)(n << 2);
    op += 1;
  } else {
    const uint32_t count = n < 256 ? 1 : n < 65536 ? 2 : n < (1u << 24) ? 3 : 4;
    if (lane == 0) dst[op] = (uint8_t)((59 + count) << 2);
    if (lane >= 1 && lane <= count) dst[op + lane] = (uint8_t)(n >> (8 * (lane - 1)));
    op += 1 + count;
  }
  copy_to_global(S, dst + op, start, len, lane);
  return op + len;
}

// Emission of ntok (<= 64) queued copies: lane t holds copy t (tk = position | offset << 16,
// tl = length), preceded by its literal run from the previous copy's end (`base` for t = 0).
// Returns the new output offset; base becomes the last copy's end.
template <class B>
__device__ uint32_t flush_copies(const B& S, uint8_t* __restrict__ dst, uint32_t op, uint32_t& base,
                                 uint32_t ntok, uint32_t tk, uint32_t tl, uint32_t lane) {
  const bool act = lane < ntok;
  const uint32_t pos = tk & 0xffffu, off = tk >> 16;
  const uint32_t end = pos + tl;
  const uint32_t pend = __shfl_up(end, 1, kWave);
  const uint32_t ls = lane == 0 ? base : pend;
  const uint32_t ll = act ? pos - ls : 0u;
  // literal tag bytes, Q3 (:271-284); a run is < 65536 bytes here
  const uint32_t lt = ll == 0 ? 0u : ll < 60 ? 1u : ll <= 256 ? 2u : 3u;
  const uint32_t ct = act ? copy_tag_bytes(off, tl) : 0u;
  const uint32_t sz = lt + ll + ct;
  const uint32_t inc = scan_dpp(sz);
  const uint32_t o = op + inc - sz;
  const uint32_t lo = o + lt;
  if (lt == 1) dst[o] = (uint8_t)((ll - 1) << 2);
  if (lt > 1) {
    const uint32_t n1 = ll - 1;
    dst[o] = (uint8_t)((58 + lt) << 2);
    dst[o + 1] = (uint8_t)n1;
    if (lt > 2) dst[o + 2] = (uint8_t)(n1 >> 8);
  }
  for (uint32_t i = 0;; i += 4) {  // runs up to 64 bytes: lane-private, four bytes a step
    const bool go = ll <= 64 && i < ll;
    if (!ballot(go)) break;
    if (go) {
      const uint32_t w = S.word(ls + i), r = ll - i;
      uint8_t* q = dst + lo + i;
      q[0] = (uint8_t)w;
      if (r > 1) q[1] = (uint8_t)(w >> 8);
      if (r > 2) q[2] = (uint8_t)(w >> 16);
      if (r > 3) q[3] = (uint8_t)(w >> 24);
    }
  }
  for (uint64_t lm = ballot(ll > 64); lm; lm &= lm - 1) {  // longer runs: the whole wave
    const uint32_t t = ctz64(lm);
    copy_to_global(S, dst + readlane(lo, t), readlane(ls, t), readlane(ll, t), lane);
  }
  if (act) put_copy(dst, lo + ll, off, tl);
  base = readlane(end, ntok - 1);
  return op + readlane(inc, kWave - 1);
}

// lane l of old := v (v and l wave-uniform; no builtin for v_writelane_b32 in this compiler)
__device__ inline uint32_t writelane(uint32_t v, uint32_t l, uint32_t old) {
  asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(old) : "s"(v), "{m0}"(l));
  return old;
}

// kLds = false: the block read in place from HBM (BlockBytes), five parses per CU -- batches;
// kLds = true: the block staged in LDS (LdsBytes), one parse per CU -- at most one block per CU
// (single calls: alice29.txt's 64 KiB fragments 4.95 ms -> see DESIGN.md section 3.1).  The
// parse below is the same code for both, so the bytes are identical.
template <bool kLds>
__global__ __launch_bounds__(64) void k_compress_exact(CompressArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t stab[kTabBytes / 4];
  __shared__ __attribute__((aligned(16))) uint8_t sblk[kLds ? kBlockSize + kLdsBlockPad : 16];

  const uint32_t b = blockIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t n = a.in_len[b];
  uint8_t* dst = a.out + a.out_off[b];
  if (n > kBlockSize) {  // batch contract violated: refuse (positions are 16-bit)
    if (lane == 0) a.out_len[b] = 0xffffffffu;
    return;
  }
  std::conditional_t<kLds, LdsBytes, BlockBytes> S;
  if constexpr (kLds) {
    const uint8_t* src = a.in + a.in_off[b];
    wave_load_global_to_lds(sblk, src, n, lane);
    for (uint32_t k = n + lane; k < n + kLdsBlockPad; k += kWave) sblk[k] = 0;  // zeros past the block
    S.blk = sblk;
    S.n = n;
  } else {
    S.r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.in + a.in_off[b]), (short)0, (int)n, 0x00020000);
    S.nm4 = n - 4;
  }
  const uint32_t tsize = a.table_size ? a.table_size : hashtable_size(n);      // Snappy.jl:27 (Q2)
  const uint32_t shift = 32 - (31 - __builtin_clz(tsize));                     // internal.jl:128
  for (uint32_t k = lane; k < tsize / 2; k += kWave) stab[k] = 0;              // Snappy.jl:30
  // probe offsets D[64 i + lane] and D[64 i + lane + 1] (:170-172), in registers
  uint32_t Dk[kProbeSteps] = {}, Dn[kProbeSteps] = {};
  {
    uint32_t d = 0, skip = 32;
#pragma unroll
    for (uint32_t i = 0; i < kProbeSteps; ++i) {
      for (uint32_t l = 0; l < kWave; ++l) {
        Dk[i] = writelane(d, l, Dk[i]);
        if (l) Dn[i] = writelane(d, l - 1, Dn[i]);
        else if (i) Dn[i - 1] = writelane(d, kWave - 1, Dn[i - 1]);
        const uint32_t step = skip >> 5;
        skip += step;
        d = min(d + step, 0x20000u);
      }
    }
    Dn[kProbeSteps - 1] = writelane(d, kWave - 1, Dn[kProbeSteps - 1]);
  }
  __syncthreads();

  uint32_t op = a.header ? emit_varint(dst, 0, n, lane) : 0;                   // Snappy.jl:26
  if (n == 0) {
    if (lane == 0) a.out_len[b] = op;
    return;
  }
  const uint32_t e = n - 1;                  // inclusive end (ip_end)
  const int32_t ip_limit = (int32_t)n - 16;  // internal.jl:131, Q1: 1-based ip_end-15
  uint32_t ip = 0, next_emit = 0, base = 0, ntok = 0, tk = 0, tl = 0;

  if (n >= kInputMarginBytes) {                                                // internal.jl:133
    for (;;) {
      ip += 1;                                                                 // :163
      // literal search, 64 probes per step (:167-194)
      const uint32_t p0 = ip;
      // the step that ends the search: its lanes' position, hash, old entry and validity
      uint32_t p = 0, h = 0, raw = 0;
      bool valid = false;
      uint64_t hm = 0;
#pragma unroll
      for (uint32_t i = 0; i < kProbeSteps; ++i) {
        p = p0 + Dk[i];
        valid = (int32_t)(p0 + Dn[i]) <= ip_limit;                             // :175
        const uint32_t cur = S.word(p);
        h = hash32(cur, shift);
        raw = 0;
        if (__builtin_expect(valid, 1)) raw = tab_probe(stab, h, p);                                // :190 (raw = candidate)
        // (raw < p: a candidate is an earlier position.  The ascending lane order makes that so on
        // gfx950; the compare makes a different order a missed match, never a wrapped offset)
        hm = ballot(valid && raw < p && S.word(raw) == cur);                   // :193
        if (hm || ballot(valid) != ~0ull) break;                               // a match, or :175
      }
      const bool found = hm != 0;
      uint32_t cand = 0;
      if (__builtin_expect(found, 1)) {
        const uint32_t j = ctz64(hm);
        const uint32_t pj = readlane(p, j);
        if (valid && lane > j && raw <= pj)                                    // undo later probes
          reinterpret_cast<uint16_t*>(stab)[h] = (uint16_t)raw;
        ip = pj;
        cand = readlane(raw, j);
      }
      if (__builtin_expect(!found, 0)) break;                                  // -> remainder
      for (;;) {                                                               // :211-239
        // bytes [0, 4) of a round are the verification (:238; known equal after a probe hit),
        // the rest find_match_length (:216).  Reads past the block return 0 and are capped.
        const uint32_t avail = n - ip;
        // first mismatching byte of a lane's word, 4 if none (ffbl(0) = ~0)
        auto fbyte = [](uint32_t x) {
          uint32_t r;
          asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
          return min(r >> 3, 4u);
        };
        uint32_t A = S.word(ip + 4 * lane);
        uint32_t fb = fbyte(A ^ S.word(cand + 4 * lane));
        // lanes whose word reaches the end (4 lane + 4 >= avail) stop the round too
        const uint64_t lim0 = avail > 4 * kWave ? 0ull : ~0ull << ((avail - 1) >> 2);
        uint64_t m = ballot(fb < 4) | lim0;
        uint32_t f, rb = 0;
        if (__builtin_expect(m != 0, 1)) {
          f = min(readlane(4 * lane + fb, ctz64(m)), avail);
        } else {
          for (;;) {  // matches of 256 bytes and more
            rb += 4 * kWave;
            const uint32_t off = rb + 4 * lane;
            fb = fbyte(S.word(ip + off) ^ S.word(cand + off));
            m = ballot(fb < 4 || off + 4 >= avail);
            if (__builtin_expect(m != 0, 1)) {
              f = min(readlane(off + fb, ctz64(m)), avail);
              break;
            }
          }
        }
        // :238; cand >= ip (a later position, only if the table's insert order broke) fails as a
        // verification does: the guard the lane-order assumption lacked
        if (__builtin_expect(f < 4 || cand >= ip, 0)) break;
        // The next candidate first (:228-235, one lane: insert ip-1, read and replace the entry
        // for ip), so the bookkeeping below runs under its LDS round trip.  Past ip_limit the
        // inserts are never read: the parse ends there.
        const uint32_t ipn = ip + f;                                           // :217-220
        uint32_t wp, wc;
        if (__builtin_expect(rb == 0 && f <= 4 * kWave - 4, 1)) {  // words at ipn-1, ipn: lanes (f-1)/4, +1
          const uint32_t k = (f - 1) >> 2, r8 = ((f - 1) & 3u) << 3;
          const uint64_t w = ((uint64_t)readlane(A, k + 1) << 32) | readlane(A, k);
          wp = (uint32_t)(w >> r8);
          wc = (uint32_t)(w >> (r8 + 8));
        } else {
          wp = uniform(S.word(ipn - 1));
          wc = uniform(S.word(ipn));
        }
        // (every lane stores the same value at the same address: one lane's store, no exec mask)
        uint16_t* u = reinterpret_cast<uint16_t*>(stab);
        u[hash32(wp, shift)] = (uint16_t)(ipn - 1);
        const uint32_t h2 = hash32(wc, shift);
        const uint32_t raw = u[h2];
        u[h2] = (uint16_t)ipn;
        tk = writelane(ip | ((ip - cand) << 16), ntok, tk);
        tl = writelane(f, ntok, tl);
        ++ntok;
        ip = ipn;
        next_emit = ip;
        if (__builtin_expect(ntok == kWave, 0)) {
          op = flush_copies(S, dst, op, base, ntok, tk, tl, lane);
          ntok = 0;
        }
        if (__builtin_expect((int32_t)ip >= ip_limit, 0)) break;               // :222
        cand = readlane(raw, 0);
      }
      if (__builtin_expect((int32_t)ip >= ip_limit, 0)) break;                 // :222 -> remainder
    }
  }
  if (ntok) op = flush_copies(S, dst, op, base, ntok, tk, tl, lane);
  if (next_emit <= e) op = emit_literal_w(S, dst, op, next_emit, e - next_emit + 1, lane);  // :244-248
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

// ---- the single-buffer call's device-side bookkeeping (sm_compress, small inputs) ----------
// Fragment f of the input is [64 KiB f, +64 KiB) and compresses into slot f (fixed pitch).
__global__ __launch_bounds__(256) void k_frag_plan(uint64_t n, uint32_t nfrag, uint64_t slot, uint64_t* in_off,
                                                   uint32_t* in_len, uint64_t* out_off) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= nfrag) return;
  const uint64_t b = (uint64_t)f * kBlockSize;
  in_off[f] = b;
  in_len[f] = (uint32_t)min((uint64_t)kBlockSize, n - b);
  out_off[f] = (uint64_t)f * slot;
}

// n bytes from s8 (16-byte aligned) to g (any alignment) by the workgroup's part y of ny:
// aligned 16-byte stores of byte-shifted units, the partial units at both ends by bytes (part 0;
// they share a 16-byte unit with the neighbouring pieces)
__device__ __attribute__((always_inline)) inline void gather_unit(const uint8_t* __restrict__ s8, uint32_t n,
                                                                 uint8_t* __restrict__ g, uint32_t y, uint32_t ny) {
  const uint4* s16 = reinterpret_cast<const uint4*>(s8);
  const uint32_t ad = (uint32_t)((uintptr_t)g & 15);
  const uint32_t u0 = ad ? 1u : 0u, u1 = (n + ad) >> 4;  // whole units [u0, u1); unit u = bytes [16u - ad, +16)
  uint4* const g16 = reinterpret_cast<uint4*>(g - ad);
  const uint32_t sb = (16 - ad) & 15, dw = sb >> 2, bs = sb & 3;
  const uint32_t stride = blockDim.x * ny;
  for (uint32_t u = u0 + y * blockDim.x + threadIdx.x; u < u1; u += stride) {
    const uint32_t j = 16 * u - ad;
    const uint4 A = s16[j >> 4], B = s16[(j >> 4) + 1];
    const uint32_t x[8] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w};
    uint32_t r5[5];
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      uint32_t vv = x[q];
#pragma unroll
      for (int dd = 1; dd < 4; ++dd) vv = dw == (uint32_t)dd ? x[q + dd] : vv;
      r5[q] = vv;
    }
    g16[u] = make_uint4(__builtin_amdgcn_alignbyte(r5[1], r5[0], bs), __builtin_amdgcn_alignbyte(r5[2], r5[1], bs),
                        __builtin_amdgcn_alignbyte(r5[3], r5[2], bs), __builtin_amdgcn_alignbyte(r5[4], r5[3], bs));
  }
  if (y == 0) {
    const uint32_t nh = min(u0 ? 16 - ad : 0u, n);
    const uint32_t tb = max(16 * u1 > ad ? 16 * u1 - ad : 0u, nh);
    if (threadIdx.x < nh + (n - tb)) {
      const uint32_t jj = threadIdx.x < nh ? threadIdx.x : tb + (threadIdx.x - nh);
      g[jj] = s8[jj];
    }
  }
}

// Fragment b's len[b] bytes from src + src_off[b] (16-byte aligned) to dst + (the lengths of
// fragments 0..b-1, one lane each: nfrag <= 64) at any alignment: aligned 16-byte stores of
// byte-shifted units, the partial units at both ends by bytes (they share a 16-byte unit with the
// neighbouring fragments); blockIdx.y strides the units.  tot[0] = the sum, tot[1] = 1 when a
// length is an error mark or over its fragment's bound (never expected): then nothing is copied.
__global__ __launch_bounds__(256) void k_gather16(const uint8_t* __restrict__ src, const uint64_t* src_off,
                                                  const uint32_t* len, const uint32_t* in_len, uint32_t nfrag,
                                                  uint64_t* tot, uint8_t* __restrict__ dst) {
  __shared__ uint32_t sh[2];
  const uint32_t b = blockIdx.x;
  if (threadIdx.x < kWave) {
    const uint32_t l = threadIdx.x;
    const uint32_t L = l < nfrag ? len[l] : 0u;
    const bool bad = l < nfrag && (uint64_t)L > 32 + (uint64_t)in_len[l] + in_len[l] / 6;
    const uint32_t before = scan_dpp(l < b ? L : 0u);  // (lanes < b: their lengths; < 2^17 each)
    const uint32_t all = scan_dpp(bad ? 0u : L);
    const bool anybad = ballot(bad) != 0;
    if (l == 63) {
      sh[0] = before;
      sh[1] = anybad;
      if (b == 0 && blockIdx.y == 0) {
        tot[0] = all;
        tot[1] = anybad;
      }
    }
  }
  __syncthreads();
  if (sh[1]) return;
  gather_unit(src + src_off[b], len[b], dst + sh[0], blockIdx.y, gridDim.y);
}

// k_gather16 for the parts of k_compress_sc_span: unit u = part u % parts of block u / parts (one
// thread each: nblk * parts <= 256, parts a power of 2 <= 64, so a block's parts are lanes of one
// wave, summed by butterfly), at src + out_off[block] + part pitch.  A block whose parts sum to more
// than one literal of the block is written as that literal instead (emit_literal!,
// internal.jl:271-284: the whole-block parse's fallback, k_compress_sc's writer), from the input.
// tot[0] = the total; tot[1] = 1 on an error mark (nothing is copied).
__global__ __launch_bounds__(256) void k_gather_parts(const uint8_t* __restrict__ src, const uint64_t* out_off,
                                                      ScSpan sp, const uint8_t* __restrict__ in,
                                                      const uint64_t* in_off, const uint32_t* in_len, uint32_t nunit,
                                                      uint64_t* tot, uint8_t* __restrict__ dst) {
  __shared__ uint32_t wsum[4], ex[256], eff[256], code;
  const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint32_t L = t < nunit ? sp.part_len[t] : 0u;
  const uint32_t nb = t < nunit ? in_len[t / sp.parts] : 0u;
  const uint32_t lit = nb ? literal_tag_bytes(nb) + nb : 0u;
  // error marks (>= 0xfff00000), and any part longer than its pitch (it would run into the next
  // part's slot): a part's output is at most span * kSpanSlot = pitch bytes; part 0 may instead be
  // a screened block's literal (its varint header, tag and bytes)
  const uint32_t bound = (t % sp.parts == 0) ? max((uint32_t)sp.pitch, lit + 5u) : (uint32_t)sp.pitch;
  const bool big = t < nunit && L > bound;
  const uint32_t Lv = big ? 0u : L;
  uint32_t sum = Lv;  // the block's parts
  for (uint32_t d = 1; d < sp.parts; d <<= 1) sum += (uint32_t)__shfl_xor((int)sum, (int)d, 64);
  const bool over = t < nunit && nb && sum > lit;
  const uint32_t E = over ? (t % sp.parts == 0 ? lit : 0u) : Lv;  // this unit's bytes in the stream
  const uint32_t inc = scan_dpp(E);
  const uint64_t anybig = ballot(big);
  if (t == 0) code = 0;
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  if (lane == 0 && anybig) code = 1;
  uint32_t pre = 0;
  for (uint32_t k = 0; k < w; ++k) pre += wsum[k];
  ex[t] = pre + inc - E;
  eff[t] = over ? 1u : 0u;
  __syncthreads();
  const uint32_t u = blockIdx.x;
  if (u == 0 && blockIdx.y == 0 && t == 0) {
    tot[0] = (uint64_t)wsum[0] + wsum[1] + wsum[2] + wsum[3];
    tot[1] = code;
  }
  if (code) return;
  const uint32_t b = u / sp.parts, j = u % sp.parts;
  uint8_t* const g = dst + ex[u];
  if (!eff[u]) {
    gather_unit(src + out_off[b] + (uint64_t)j * sp.pitch, sp.part_len[u], g, blockIdx.y, gridDim.y);
  } else if (j == 0) {  // the block as one literal: its tag, then its bytes
    const uint32_t n = in_len[b], tb = literal_tag_bytes(n);
    if (blockIdx.y == 0 && t < tb) {
      const uint32_t n1 = n - 1;
      g[t] = tb == 1 ? (uint8_t)(n1 << 2) : (t == 0 ? (uint8_t)((58 + tb) << 2) : (uint8_t)(n1 >> (8 * (t - 1))));
    }
    gather_unit(in + in_off[b], n, g + tb, blockIdx.y, gridDim.y);
  }
}

// ---- a sharded stream's fragments at their places in it (Snappy.jl:29-35) ----------
// Fragment b (len[b] bytes at src + src_off[b]) to dst + (dst_off[b] - base): dst_off[b] is the
// fragment's offset in the whole stream (the all-gathered exclusive scan behind the varint
// header), base = 0 with the header (dst is the stream from its first byte and varint(total) is
// written there) or dst_off[0] without it (dst is the caller's byte range from its first
// fragment).  loc_off[b] (optional) receives dst_off[b] - base.  A length that is an error mark,
// or a fragment that would end past cap, copies nothing and sets *status = SM_ERR_DEVICE
// (optional; never cleared here).  blockIdx.y strides the fragment's 16-byte units.
__global__ __launch_bounds__(256) void k_place(const uint8_t* __restrict__ src, const uint64_t* src_off,
                                               const uint32_t* len, const uint64_t* dst_off, uint32_t nfrag,
                                               uint64_t total, int header, uint64_t cap, uint8_t* __restrict__ dst,
                                               uint64_t* loc_off, int32_t* status) {
  const uint32_t b = blockIdx.x;
  if (header && b == 0 && blockIdx.y == 0) {  // varint(total), src/varint.jl:46-69
    const uint32_t hv = varint_len((uint32_t)total);
    if (threadIdx.x < hv && threadIdx.x < cap)
      dst[threadIdx.x] = (uint8_t)((((uint32_t)total >> (7 * threadIdx.x)) & 0x7f) | (threadIdx.x + 1 < hv ? 0x80 : 0));
  }
  if (b >= nfrag) return;  // (an empty stream: the header alone)
  const uint64_t base = header ? 0ull : dst_off[0];
  const uint32_t n = len[b];
  const uint64_t at = dst_off[b] - base;  // (a mark earlier in the scan wraps this past cap)
  const bool bad = n >= kOutLenError || at > cap || cap - at < n;
  if (blockIdx.y == 0 && threadIdx.x == 0) {
    if (loc_off) loc_off[b] = at;
    if (bad && status) *status = kErrDevice;
  }
  if (bad) return;
  const uint8_t* const s = src + src_off[b];
  if (((uintptr_t)s & 15) == 0) {
    gather_unit(s, n, dst + at, blockIdx.y, gridDim.y);
  } else {
    for (uint32_t k = blockIdx.y * blockDim.x + threadIdx.x; k < n; k += blockDim.x * gridDim.y) dst[at + k] = s[k];
  }
}

hipError_t launch_place(const uint8_t* src, const uint64_t* src_off, const uint32_t* len, const uint64_t* dst_off,
                        uint32_t nfrag, uint64_t total, int header, uint64_t cap, uint8_t* dst, uint64_t* loc_off,
                        int32_t* status, hipStream_t s) {
  if (nfrag == 0 && !header) return hipSuccess;
  hipLaunchKernelGGL(k_place, dim3(max(nfrag, 1u), 4), dim3(256), 0, s, src, src_off, len, dst_off, nfrag, total, header,
                     cap, dst, loc_off, status);
  return hipGetLastError();
}

hipError_t launch_frag_plan(uint64_t n, uint32_t nfrag, uint64_t slot, uint64_t* in_off, uint32_t* in_len,
                            uint64_t* out_off, hipStream_t s) {
  hipLaunchKernelGGL(k_frag_plan, dim3((nfrag + 255) / 256), dim3(256), 0, s, n, nfrag, slot, in_off, in_len, out_off);
  return hipGetLastError();
}

hipError_t launch_parts_gather(const uint8_t* src, const uint64_t* out_off, const ScSpan& sp, const uint8_t* in,
                               const uint64_t* in_off, const uint32_t* in_len, uint32_t nblk, uint64_t* tot,
                               uint8_t* dst, hipStream_t s) {
  const uint32_t nunit = nblk * sp.parts;
  if (nblk == 0 || sp.parts == 0 || sp.parts > kWave || (sp.parts & (sp.parts - 1)) || nunit > 256)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_gather_parts, dim3(nunit, 4), dim3(256), 0, s, src, out_off, sp, in, in_off, in_len, nunit,
                     tot, dst);
  return hipGetLastError();
}

hipError_t launch_frag_gather(const uint8_t* src, const uint64_t* src_off, const uint32_t* out_len,
                              const uint32_t* in_len, uint32_t nfrag, uint64_t* tot, uint8_t* dst, hipStream_t s) {
  if (nfrag == 0 || nfrag > kWave) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_gather16, dim3(nfrag, 4), dim3(256), 0, s, src, src_off, out_len, in_len, nfrag, tot, dst);
  return hipGetLastError();
}


// the current device's CU count (cached per device)
static uint32_t cu_count() {
  static uint32_t cache[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  uint32_t ncu = __atomic_load_n(&cache[dev], __ATOMIC_RELAXED);
  if (!ncu) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    ncu = (uint32_t)v;
    __atomic_store_n(&cache[dev], ncu, __ATOMIC_RELAXED);
  }
  return ncu;
}

hipError_t launch_compress(const CompressArgs& a, int mode, hipStream_t s) {
  if (a.nblk == 0) return hipSuccess;
  if (mode != 0) return launch_compress_fast(a, mode, s);
  // at most one block per CU: each parse gets a CU and reads its block from LDS; more: five
  // parses per CU reading their blocks in place (the LDS holds one staged block)
  if (a.nblk <= cu_count())
    hipLaunchKernelGGL(k_compress_exact<true>, dim3(a.nblk), dim3(64), 0, s, a);
  else
    hipLaunchKernelGGL(k_compress_exact<false>, dim3(a.nblk), dim3(64), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_gather(const uint8_t* src, const uint64_t* src_off, const uint32_t* len,
                         const uint64_t* dst_off, uint8_t* dst, uint32_t nblk, hipStream_t s) {
  if (nblk == 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather, dim3(nblk), dim3(256), 0, s, src, src_off, len, dst_off, dst);
  return hipGetLastError();
}

}  // namespace sm
