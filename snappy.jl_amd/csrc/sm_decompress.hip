// sm_decompress.hip -- batched snappy decompression for gfx950 (MI355X).
//
// One wavefront per compressed stream.  Accept/reject semantics are Snappy.jl's
// (src/internal.jl:411-527, src/Snappy.jl:46-52), including its leniencies:
//   * `while ip < endof(input)` (internal.jl:416): a tag on the last byte is never parsed;
//   * the 4-byte lookahead is zero-padded past the end (internal.jl:426-430);
//   * literal length is len + trailer in UInt32 arithmetic (wraps);
//   * copy offset check `op-1 <= offset-1` with unsigned wrap (internal.jl:499);
//   * the copy-length check is skipped on the 2x8-byte fast path (internal.jl:500-505).
// The first error in stream order wins, as the reference throws at the first one.
//
// Tag walk: the wave keeps a 256-byte window of the compressed stream in VGPRs (4 B/lane)
// and reads tag bytes with v_readlane (wave-uniform scalar walk).  Each tag's bytes are then
// moved wave-wide: literals global->output, copies output->output with RLE handled as
// src = op - offset + (k mod offset), which is the byte the reference's sequential
// incremental_copy_slow! (internal.jl:477-481) would read.
// Output: staged in LDS when the declared length is <= 64 KiB (every block the compressor
// produces), then written with 16-B stores; longer streams decode straight into HBM.
#include "sm_device.h"
#include "sm_internal.h"

namespace sm {

struct Window {
  uint32_t w;      // 4 bytes per lane, little-endian
  uint32_t base;   // stream position of lane 0 byte 0
};

__device__ inline void win_load(Window& win, const uint8_t* __restrict__ in, uint32_t N, uint32_t pos, uint32_t lane) {
  uint32_t p = pos + 4 * lane;
  uint32_t v = 0;
  if (p + 3 < N && (((uintptr_t)(in + p)) & 3) == 0) {
    v = *reinterpret_cast<const uint32_t*>(in + p);
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) v |= (p + k < N ? (uint32_t)in[p + k] : 0u) << (8 * k);
  }
  win.w = v;
  win.base = pos;
}

// 4 bytes at stream position pos (zero past N), window must cover pos..pos+7
__device__ inline uint32_t win_ld32(const Window& win, uint32_t pos) {
  uint32_t rel = pos - win.base;
  uint32_t lo = readlane(win.w, rel >> 2);
  uint32_t hi = readlane(win.w, (rel >> 2) + 1);
  return __builtin_amdgcn_alignbyte(hi, lo, rel & 3);
}

template <bool kLds>
__device__ inline int32_t decode_stream(const uint8_t* __restrict__ in, uint32_t N, uint32_t ip, uint32_t size,
                                        uint8_t* out, uint32_t lane) {
  Window win;
  win_load(win, in, N, ip, lane);
  uint32_t op = 0;
  while ((int64_t)ip < (int64_t)N - 1) {                                 // internal.jl:416
    if (ip - win.base > 4 * kWave - 8) win_load(win, in, N, ip, lane);
    uint32_t c = win_ld32(win, ip) & 0xff;
    uint32_t tag = win_ld32(win, ip + 1);                                // :426-430 (zeros past N)
    ip += 1;
    uint32_t entry = char_entry(c);                                      // :435-439
    uint32_t len = entry & 0xff;
    uint32_t taglen = entry >> 11;
    uint32_t trailer = taglen >= 4 ? tag : (tag & ((1u << (8 * taglen)) - 1u));
    ip += taglen;
    if (c & 3) {                                                         // :458-460 copy
      uint32_t offset = (entry & 0x700) + trailer;
      int64_t avail_out = (int64_t)size - op;
      if ((int64_t)op <= (int64_t)(uint32_t)(offset - 1u)) return kErrCopyOffset;   // :499
      if (!(len <= 16 && offset >= 8 && avail_out >= 16) && avail_out < (int64_t)len)
        return kErrCopyLength;                                           // :505
      if (lane < len) {
        uint32_t k = lane;
        uint32_t sidx = op - offset + (offset >= len ? k : k % offset);
        if (kLds) {
          out[op + k] = out[sidx];
        } else {
          volatile uint8_t* vo = out;
          vo[op + k] = vo[sidx];
        }
      }
      if (!kLds) __threadfence_block();
      op += len;
    } else {                                                             // :461-462 literal
      uint32_t litlen = len + trailer;                                   // UInt32 wrap
      int64_t avail_out = (int64_t)size - op;
      int64_t avail_in = (int64_t)N - ip;
      if (avail_out < (int64_t)litlen || avail_in < (int64_t)litlen) return kErrLiteral;  // :518
      for (uint32_t k = lane; k < litlen; k += kWave) {
        if (kLds) out[op + k] = in[ip + k];
        else ((volatile uint8_t*)out)[op + k] = in[ip + k];
      }
      if (!kLds) __threadfence_block();
      op += litlen;
      ip += litlen;
    }
  }
  if (op != size) return kErrInvalid;                                    // Snappy.jl:50
  return kOk;
}

__global__ __launch_bounds__(64) void k_decompress(DecompressArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t sout[kBlockSize + 64];
  const uint32_t b = blockIdx.x;
  const uint32_t lane = lane_id();
  const uint8_t* in = a.in + a.in_off[b];
  const uint32_t N = a.in_len[b];
  uint8_t* dst = a.out + a.out_off[b];
  const uint32_t cap = a.out_cap[b];

  // varint32 header (varint.jl:12-37)
  uint32_t hb = (lane < 5 && lane < N) ? in[lane] : 0;
  int32_t st = kErrVarint;
  uint32_t size = 0, ip = 0;
  for (uint32_t i = 0; i < 5; ++i) {
    if (i >= N) break;
    uint32_t bt = readlane(hb, i);
    if (i < 4) {
      size |= (bt & 0x7f) << (7 * i);
      if (bt < 0x80) { st = kOk; ip = i + 1; break; }
    } else {
      size |= (bt & 0x7f) << 28;
      if (bt < 0x10) { st = kOk; ip = 5; }
    }
  }
  if (st == kOk && size > cap) st = kBufferTooSmall;
  if (st == kOk) {
    if (size <= kBlockSize) {
      st = decode_stream<true>(in, N, ip, size, sout, lane);
      if (st == kOk) {
        __syncthreads();
        wave_copy_lds_to_global(dst, sout, 0, size, lane);
      }
    } else {
      st = decode_stream<false>(in, N, ip, size, dst, lane);
    }
  }
  if (lane == 0) {
    a.status[b] = st;
    a.out_len[b] = st == kOk ? size : 0;
  }
}

hipError_t launch_decompress(const DecompressArgs& a, int /*large*/, hipStream_t s) {
  if (a.nblk == 0) return hipSuccess;
  hipLaunchKernelGGL(k_decompress, dim3(a.nblk), dim3(64), 0, s, a);
  return hipGetLastError();
}

}  // namespace sm
