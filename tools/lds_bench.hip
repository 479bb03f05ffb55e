// LDS access-cost microbenchmark (design tool): cycles per wave-instruction of 4- and 8-byte
// LDS reads by address pattern -- sequential / random, aligned / byte-misaligned -- with
// 16 waves per CU (the fast compressor's shape).  Build + run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/lds_bench tools/lds_bench.hip && /tmp/lds_bench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t __attribute__((aligned(1))) u32u;
typedef uint64_t __attribute__((aligned(1))) u64u;

constexpr int kIters = 512;

template <int W, int PAT>
__global__ __launch_bounds__(1024) void k(uint32_t* out, uint32_t seed) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[65536 + 64];
  for (uint32_t i = threadIdx.x; i < (65536 + 64) / 4; i += 1024) reinterpret_cast<uint32_t*>(lds)[i] = i * 2654435761u;
  __syncthreads();
  uint32_t x = seed ^ (threadIdx.x * 0x9E3779B9u) ^ blockIdx.x;
  uint32_t acc = 0;
  const uint32_t lane = threadIdx.x & 63;
  for (int it = 0; it < kIters; ++it) {
    x = x * 1664525u + 1013904223u;  // per-lane LCG
    uint32_t a;
    if (PAT == 0) a = ((it * 64 + lane) * W) & 0xffff;                       // sequential, aligned
    else if (PAT == 1) a = ((it * 64 + lane) * W + 1) & 0xffff;              // sequential, misaligned
    else if (PAT == 2) a = (x >> 16) & ~(uint32_t)(W - 1);                   // random, aligned
    else if (PAT == 3) a = (x >> 16);                                         // random, byte address
    else if (PAT == 4) a = ((x >> 16) & ~3u) | 1;                             // random, 4-aligned+1
    else if (PAT == 5) a = ((x >> 16) & ~7u) | 4;                             // random, 4 mod 8
    else a = (x >> 16) & ~3u;                                                 // random, 4-aligned
    a ^= acc & 0;  // keep loads independent of acc
    if (W == 1) acc += lds[a];
    else if (W == 4) acc += *reinterpret_cast<const u32u*>(lds + a);
    else if (W == 16) {
      const uint4 v = *reinterpret_cast<const uint4*>(lds + (a & ~15u));
      acc += v.x ^ v.y ^ v.z ^ v.w;
    } else if (W == 2) {  // two aligned dwords (ds_read2_b32) + funnel shift = a misaligned 4-byte read
      const uint32_t* dw = reinterpret_cast<const uint32_t*>(lds);
      const uint32_t i = a >> 2;
      acc += __builtin_amdgcn_alignbyte(dw[i + 1], dw[i], a & 3);
    } else if (W == 3) {  // 4-aligned ds_read_b64 + funnel shift
      typedef uint64_t __attribute__((aligned(4))) u64a4;
      const uint64_t v = *reinterpret_cast<const u64a4*>(lds + (a & ~3u));
      acc += __builtin_amdgcn_alignbyte((uint32_t)(v >> 32), (uint32_t)v, a & 3);
    } else {
      const uint64_t v = *reinterpret_cast<const u64u*>(lds + a);
      acc += (uint32_t)v ^ (uint32_t)(v >> 32);
    }
  }
  out[blockIdx.x * 1024 + threadIdx.x] = acc;
}

template <int PAT>
__global__ __launch_bounds__(1024) void kg(const uint8_t* g, uint32_t* out, uint32_t seed) {
  uint32_t x = seed ^ (threadIdx.x * 0x9E3779B9u) ^ blockIdx.x;
  uint32_t acc = 0;
  const uint32_t lane = threadIdx.x & 63;
  const uint8_t* base = g + (size_t)blockIdx.x * 65536;
  for (int it = 0; it < kIters / 8; ++it) {
    x = x * 1664525u + 1013904223u;
    uint32_t a;
    if (PAT == 0) a = ((it * 64 + lane) * 8) & 0xffff;
    else if (PAT == 1) a = ((it * 64 + lane) * 8 + 3) & 0xffff;
    else if (PAT == 2) a = (x >> 16) & ~7u;
    else a = (x >> 16);
    const uint64_t v = *reinterpret_cast<const u64u*>(base + a);
    acc += (uint32_t)v ^ (uint32_t)(v >> 32);
  }
  out[blockIdx.x * 1024 + threadIdx.x] = acc;
}

template <int PAT>
void runG(const uint8_t* g, uint32_t* d, const char* name) {
  const int blocks = 256 * 8;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  kg<PAT><<<blocks, 1024>>>(g, d, 1);
  hipEventRecord(e0);
  kg<PAT><<<blocks, 1024>>>(g, d, 2);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double winst = (double)blocks * 16 * (kIters / 8) / 256.0;
  printf("%-28s %8.3f ms  %6.2f CU-cycles per wave-load (L2-resident 128 MiB)\n", name, ms, ms * 1e-3 * 2.4e9 / winst);
}

template <int W, int PAT>
float run(uint32_t* d, const char* name) {
  const int blocks = 256 * 8;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k<W, PAT><<<blocks, 1024>>>(d, 1);
  hipEventRecord(e0);
  k<W, PAT><<<blocks, 1024>>>(d, 2);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  // cycles per wave-instruction per CU: time * 2.4 GHz / (wave-instructions per CU)
  const double winst = (double)blocks * 16 * kIters / 256.0;
  printf("%-28s %8.3f ms  %6.2f CU-cycles per wave-read\n", name, ms, ms * 1e-3 * 2.4e9 / winst);
  return ms;
}

int main() {
  uint32_t* d;
  hipMalloc(&d, 256 * 8 * 1024 * 4);
  run<4, 0>(d, "b32 sequential aligned");
  run<4, 1>(d, "b32 sequential misaligned");
  run<4, 2>(d, "b32 random aligned");
  run<4, 3>(d, "b32 random byte-addr");
  run<4, 4>(d, "b32 random 4k+1");
  run<8, 0>(d, "b64 sequential aligned");
  run<8, 1>(d, "b64 sequential misaligned");
  run<8, 2>(d, "b64 random aligned");
  run<8, 3>(d, "b64 random byte-addr");
  run<8, 4>(d, "b64 random 4k+1");
  run<8, 5>(d, "b64 random 4 mod 8");
  run<16, 2>(d, "b128 random 16-aligned");
  run<2, 3>(d, "read2_b32+alignbyte random");
  run<3, 3>(d, "b64@4-aligned+alignbyte rnd");
  run<2, 1>(d, "read2_b32+alignbyte seq");
  run<3, 1>(d, "b64@4-aligned+alignbyte seq");
  run<1, 3>(d, "u8 random");
  run<1, 0>(d, "u8 sequential");
  uint8_t* g;
  hipMalloc(&g, (size_t)256 * 8 * 65536 + 64);
  hipMemset(g, 1, (size_t)256 * 8 * 65536 + 64);
  runG<0>(g, d, "global b64 seq aligned");
  runG<1>(g, d, "global b64 seq misaligned");
  runG<2>(g, d, "global b64 random aligned");
  runG<3>(g, d, "global b64 random byte-addr");
  hipFree(g);
  hipFree(d);
  return 0;
}
