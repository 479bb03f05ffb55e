// sm_device.h -- snappy raw-format constants and CDNA4 wave primitives shared by the
// gfx950 kernels.  Format rules follow /root/reference/src/internal.jl:15-85 and
// src/varint.jl; nothing here is transcribed from the reference's tables (CHAR_TABLE is
// derived from the tag rules in sm_char_entry()).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sm {

constexpr uint32_t kBlockSize = 65536;        // internal.jl:31
constexpr uint32_t kInputMarginBytes = 15;    // internal.jl:32
constexpr uint32_t kMaxHashTableSize = 16384; // internal.jl:33
constexpr uint32_t kHashMul = 0x1e35a7bdu;    // internal.jl:94
constexpr int kWave = 64;

// status codes (mirror include/snappy_mi355x.h)
enum : int32_t {
  kOk = 0,
  kInvalidInput = 1,
  kBufferTooSmall = 2,
  kErrInputTooLarge = 16,
  kErrInvalid = 17,
  kErrVarint = 18,
  kErrCopyOffset = 19,
  kErrCopyLength = 20,
  kErrLiteral = 21,
  kErrDevice = 32,  // SM_ERR_DEVICE: a block length that is a compressor error mark (>= kOutLenError)
  kErrCross = 64,  // internal: a fragment's copy reads another fragment (never returned by the ABI)
};

__host__ __device__ inline uint32_t max_compressed_length(uint32_t n) { return 32 + n + n / 6; }

// SM_OUT_LEN_ERROR: a compressor's error mark in d_out_len (include/snappy_mi355x.h).  A device
// decoder handed such a length (a caller passing comp_len straight on) reports kErrDevice without
// reading the slot: the mark is an error, never a stream length (Snappy.jl:50 raises, never decodes).
constexpr uint32_t kOutLenError = 0xfff00000u;

// internal.jl:107-113
__host__ __device__ inline uint32_t hashtable_size(uint64_t n) {
  uint32_t ht = 256;
  while (ht < kMaxHashTableSize && ht < n) ht <<= 1;
  return ht;
}

// internal.jl:35-46 layout: bits 0-7 length, 8-10 copy offset>>8, 11-13 extra bytes.
__host__ __device__ inline uint32_t char_entry(uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  // branch-free on the device: the kind-switch compiles to a divergent branch tree that a wave of
  // mixed tags runs every arm of (exec masks, ~16 SALU); these are selects on the same values
  const uint32_t kind = c & 3, hi = c >> 2;
  const uint32_t tlc = __builtin_amdgcn_perm(0u, 0x04020100u, kind);  // copy tag bytes 1/2/4 (kind 0: 0)
  const uint32_t lit = hi < 60 ? hi + 1 : (((hi - 59) << 11) | 1);
  const uint32_t cp1 = (1u << 11) | ((c >> 5) << 8) | (4 + (hi & 7));
  const uint32_t cpx = (tlc << 11) | (hi + 1);
  return kind == 0 ? lit : (kind == 1 ? cp1 : cpx);
#else
  uint32_t kind = c & 3, hi = c >> 2;
  if (kind == 0) return hi < 60 ? hi + 1 : (((hi - 59) << 11) | 1);
  if (kind == 1) return (1u << 11) | ((c >> 5) << 8) | (4 + ((c >> 2) & 7));
  if (kind == 2) return (2u << 11) | (hi + 1);
  return (4u << 11) | (hi + 1);
#endif
}

__host__ __device__ inline uint32_t varint_len(uint32_t v) {
  return v < (1u << 7) ? 1 : v < (1u << 14) ? 2 : v < (1u << 21) ? 3 : v < (1u << 28) ? 4 : 5;
}

// bytes of the literal tag for a run of len (>0) bytes (internal.jl:271-284)
__host__ __device__ inline uint32_t literal_tag_bytes(uint32_t len) {
  uint32_t n = len - 1;
  return n < 60 ? 1 : n < 256 ? 2 : n < 65536 ? 3 : n < (1u << 24) ? 4 : 5;
}

// bytes emit_copy! (internal.jl:306-329) produces for (offset, len)
__host__ __device__ inline uint32_t copy_tag_bytes(uint32_t offset, uint32_t len) {
  if (len < 12) return (offset < 2048) ? 2 : 3;
  uint32_t b = 0;
  while (len >= 68) { b += 3; len -= 64; }
  if (len > 64) { b += 3; len -= 60; }
  return b + ((len < 12 && offset < 2048) ? 2 : 3);
}

// ---- wave primitives -------------------------------------------------------------

__device__ inline uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

__device__ inline uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// the lane predicate of an SGPR lane mask (free: the mask is the predicate)
__device__ inline bool inverse_ballot(uint64_t m) { return __builtin_amdgcn_inverse_ballot_w64(m); }

__device__ inline uint32_t uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ inline uint32_t readlane(uint32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }

__device__ inline uint32_t ctz64(uint64_t m) { return (uint32_t)__builtin_ctzll(m); }

// inclusive wave-wide prefix sum (64 lanes)
__device__ inline uint32_t wave_incl_scan(uint32_t v, uint32_t lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t t = __shfl_up(v, d, 64);
    if (lane >= (uint32_t)d) v += t;
  }
  return v;
}

// inclusive wave-64 scan with DPP (row_shr 1/2/4/8 within rows, row_bcast 15/31 across)
__device__ inline uint32_t scan_dpp(uint32_t v) {
  v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);
  return v;
}

// Unaligned little-endian loads from an LDS byte array, built from aligned dword reads +
// v_alignbyte_b32.  A misaligned ds_read_b32/b64 is serviced one lane per LDS cycle (~64
// cycles per wave-instruction) against 2-8 aligned and ~15 for this form on random
// addresses (tools/lds_bench.hip, measured on MI355X).
// the LDS byte address of a pointer into a __shared__ array
__device__ inline uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// lds_ld32: the array must have >= 4 readable bytes past pos+3.
__device__ inline uint32_t lds_ld32(const uint8_t* lds, uint32_t pos) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(lds + (pos & ~3u));
  uint32_t lo = w[0], hi = w[1];
  return __builtin_amdgcn_alignbyte(hi, lo, pos);  // (v_alignbyte_b32 shifts by 8 * S2[1:0]: no & 3)
}

// lds_ld64: >= 4 readable bytes past pos+7.
__device__ inline uint64_t lds_ld64(const uint8_t* lds, uint32_t pos) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(lds + (pos & ~3u));
  const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], sh = pos;  // (alignbyte: S2[1:0] only)
  return ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32) | __builtin_amdgcn_alignbyte(w1, w0, sh);
}

__device__ inline uint32_t hash32(uint32_t bytes, uint32_t shift) { return (bytes * kHashMul) >> shift; }

// Wave-cooperative copy of len bytes from an LDS byte array (at s) to global memory.
// 16-byte-aligned stores for the body; byte stores for the unaligned head/tail.
__device__ inline void wave_copy_lds_to_global(uint8_t* __restrict__ g, const uint8_t* lds, uint32_t s,
                                               uint32_t len, uint32_t lane) {
  uint32_t head = (uint32_t)((16 - ((uintptr_t)g & 15)) & 15);
  if (head > len) head = len;
  if (lane < head) g[lane] = lds[s + lane];
  g += head; s += head; len -= head;
  uint32_t n16 = len >> 4;
  uint4* g16 = reinterpret_cast<uint4*>(g);
  for (uint32_t k = lane; k < n16; k += kWave) {
    uint32_t p = s + 16 * k;
    uint4 v;
    v.x = lds_ld32(lds, p);
    v.y = lds_ld32(lds, p + 4);
    v.z = lds_ld32(lds, p + 8);
    v.w = lds_ld32(lds, p + 12);
    g16[k] = v;
  }
  uint32_t done = n16 << 4;
  if (lane < len - done) g[done + lane] = lds[s + done + lane];
}

// Wave-cooperative global->LDS load of len bytes (block staging).  lds must be 16-B
// aligned; src may have any alignment.
__device__ inline void wave_load_global_to_lds(uint8_t* lds, const uint8_t* __restrict__ src, uint32_t len,
                                               uint32_t lane) {
  if (((uintptr_t)src & 15) == 0) {
    const uint4* s16 = reinterpret_cast<const uint4*>(src);
    uint4* d16 = reinterpret_cast<uint4*>(lds);
    uint32_t n16 = len >> 4;
    for (uint32_t k = lane; k < n16; k += kWave) d16[k] = s16[k];
    for (uint32_t k = (n16 << 4) + lane; k < len; k += kWave) lds[k] = src[k];
  } else if (((uintptr_t)src & 3) == 0) {
    const uint32_t* s4 = reinterpret_cast<const uint32_t*>(src);
    uint32_t* d4 = reinterpret_cast<uint32_t*>(lds);
    uint32_t n4 = len >> 2;
    for (uint32_t k = lane; k < n4; k += kWave) d4[k] = s4[k];
    for (uint32_t k = (n4 << 2) + lane; k < len; k += kWave) lds[k] = src[k];
  } else {
    for (uint32_t k = lane; k < len; k += kWave) lds[k] = src[k];
  }
}

// first i (relative) at which a[i1+i] != a[i2+i], capped at avail; LDS-resident bytes.
// One wave round compares 256 bytes (4 per lane).  Reads stay below i2+avail+3 (clamped).
__device__ inline uint32_t wave_match_length(const uint8_t* lds, uint32_t i1, uint32_t i2, uint32_t avail,
                                             uint32_t lane) {
  uint32_t base = 0;
  for (;;) {
    uint32_t off = base + 4 * lane;
    uint32_t res;
    bool stop;
    if (off >= avail) {
      res = avail; stop = true;
    } else {
      uint32_t x = lds_ld32(lds, i1 + off) ^ lds_ld32(lds, i2 + off);
      uint32_t fb = x ? (uint32_t)(__builtin_ctz(x) >> 3) : 4u;
      res = off + fb;
      if (res > avail) res = avail;
      stop = (fb < 4) || (off + 4 >= avail);
    }
    uint64_t m = ballot(stop);
    if (m) return readlane(res, ctz64(m));
    base += 4 * kWave;
  }
}

}  // namespace sm
