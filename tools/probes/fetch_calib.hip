// FETCH_SIZE calibration for the decoder's access shapes (design probe, GPU box; VERDICT round 5
// item 2: "calibrate FETCH_SIZE for the decoder's 16-byte gathers with a probe of known byte count").
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/probes/fetch_calib tools/probes/fetch_calib.hip
//   rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d DIR -o p -- tools/probes/fetch_calib
//
// Every kernel reads a known set of bytes from a 1 GiB buffer (past the 256 MiB Infinity Cache,
// cold: the buffer is rewritten between kernels) and reports nothing but a checksum:
//  k_stream16  -- 16 B per lane, coalesced, the whole 1 GiB (the guide's calibrated case: raw
//                 FETCH = 1/2 of the bytes);
//  k_stream4   -- 4 B per lane, coalesced (the decoder's ring / prefetch loads), the whole 1 GiB;
//  k_gather16  -- 16 B per lane as two unaligned 8-byte loads at random 16-B-unaligned
//                 addresses (a far copy source's piece), 2^22 of them;
//  k_gather64  -- 64 contiguous bytes per 4 lanes (a 64-byte copy source), 2^22 of them.
// The host prints the bytes each kernel asked for and the lines (128 B) they touch, so the
// profile's FETCH_SIZE per kernel divides into bytes-per-request and lines-per-request factors.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

typedef uint64_t __attribute__((aligned(1))) u64u;

__global__ void k_fill(uint32_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = (uint32_t)i * 2654435761u + seed;
}

__global__ void k_stream16(const uint4* p, size_t n16, uint32_t* sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;  // (never: keeps the loads)
}

__global__ void k_stream4(const uint32_t* p, size_t n4, uint32_t* sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
    acc ^= p[i];
  if (acc == 0x12345678u) sink[0] = acc;
}

__device__ inline uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  return x;
}

// request r: 16 bytes at a random byte offset (any alignment) below n - 16
__global__ void k_gather16(const uint8_t* p, size_t n, uint32_t nreq, uint32_t* sink) {
  uint64_t acc = 0;
  for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < nreq; r += gridDim.x * blockDim.x) {
    const uint64_t o = mix(r + 1) % (n - 16);
    const u64u* g = reinterpret_cast<const u64u*>(p + o);
    acc ^= g[0] ^ g[1];
  }
  if (acc == 0x12345678u) sink[0] = (uint32_t)acc;
}

// request r: 64 contiguous bytes at a random byte offset, 16 B per lane by 4 lanes
__global__ void k_gather64(const uint8_t* p, size_t n, uint32_t nreq, uint32_t* sink) {
  uint64_t acc = 0;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  for (uint32_t q = t; q < 4 * nreq; q += gridDim.x * blockDim.x) {
    const uint32_t r = q >> 2, k = q & 3;
    const uint64_t o = mix(r + 1) % (n - 64);
    const u64u* g = reinterpret_cast<const u64u*>(p + o + 16 * k);
    acc ^= g[0] ^ g[1];
  }
  if (acc == 0x12345678u) sink[0] = (uint32_t)acc;
}

static uint64_t mix_h(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  return x;
}

int main() {
  const size_t n = (size_t)1 << 30;
  const uint32_t nreq = 1u << 22;
  uint8_t* p = nullptr;
  uint32_t* sink = nullptr;
  CK(hipMalloc(&p, n));
  CK(hipMalloc(&sink, 64));
  auto refill = [&](uint32_t seed) -> int {
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint32_t*>(p), n / 4, seed);
    CK(hipDeviceSynchronize());
    return 0;
  };
  if (refill(1)) return 1;
  hipLaunchKernelGGL(k_stream16, dim3(8192), dim3(256), 0, 0, reinterpret_cast<const uint4*>(p), n / 16, sink);
  CK(hipDeviceSynchronize());
  if (refill(2)) return 1;
  hipLaunchKernelGGL(k_stream4, dim3(8192), dim3(256), 0, 0, reinterpret_cast<const uint32_t*>(p), n / 4, sink);
  CK(hipDeviceSynchronize());
  if (refill(3)) return 1;
  hipLaunchKernelGGL(k_gather16, dim3(4096), dim3(256), 0, 0, p, n, nreq, sink);
  CK(hipDeviceSynchronize());
  if (refill(4)) return 1;
  hipLaunchKernelGGL(k_gather64, dim3(4096), dim3(256), 0, 0, p, n, nreq, sink);
  CK(hipDeviceSynchronize());
  // the lines each gather kernel touches (128-B lines; distinct over the whole kernel)
  uint64_t l16 = 0, l64 = 0;
  {
    // lines per request, summed (requests almost never share a line in 1 GiB: 2^22 of 2^23 lines
    // would, so count distinct lines by a bitmap)
    const size_t nl = n / 128;
    uint8_t* seen16 = (uint8_t*)calloc(nl / 8 + 1, 1);
    uint8_t* seen64 = (uint8_t*)calloc(nl / 8 + 1, 1);
    for (uint32_t r = 0; r < nreq; ++r) {
      const uint64_t o16 = mix_h(r + 1) % (n - 16);
      for (uint64_t L = o16 / 128; L <= (o16 + 15) / 128; ++L)
        if (!(seen16[L >> 3] & (1u << (L & 7)))) { seen16[L >> 3] |= (uint8_t)(1u << (L & 7)); ++l16; }
      const uint64_t o64 = mix_h(r + 1) % (n - 64);
      for (uint64_t L = o64 / 128; L <= (o64 + 63) / 128; ++L)
        if (!(seen64[L >> 3] & (1u << (L & 7)))) { seen64[L >> 3] |= (uint8_t)(1u << (L & 7)); ++l64; }
    }
    free(seen16);
    free(seen64);
  }
  printf("k_stream16: %zu bytes requested (16 B/lane coalesced)\n", n);
  printf("k_stream4:  %zu bytes requested (4 B/lane coalesced)\n", n);
  printf("k_gather16: %u requests of 16 B = %llu bytes; %llu distinct 128-B lines\n", nreq,
         (unsigned long long)nreq * 16, (unsigned long long)l16);
  printf("k_gather64: %u requests of 64 B = %llu bytes; %llu distinct 128-B lines\n", nreq,
         (unsigned long long)nreq * 64, (unsigned long long)l64);
  CK(hipFree(p));
  CK(hipFree(sink));
  return 0;
}
