// Design probe (not product code): are unaligned ds_read_b32 / b64 / b128 served correctly on
// gfx950 (the byte address need not be a multiple of the access size), and what do they cost
// against aligned reads and against the five-dword + alignbyte composition the compressor uses?
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/ldsu lds_unaligned.hip && /tmp/ldsu
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ inline uint8_t pat(uint32_t i) { return (uint8_t)(i * 131u + (i >> 8) * 7u + 3u); }

// correctness: every lane reads at byte offset 5 * lane + s (s = 0..15) with each width
__global__ void k_check(uint32_t* err) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[4096];
  const uint32_t l = threadIdx.x;
  for (uint32_t i = l; i < 4096; i += 64) buf[i] = pat(i);
  __syncthreads();
  uint32_t bad = 0;
  for (uint32_t s = 0; s < 16; ++s) {
    const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)(buf + 5 * l + s);
    uint32_t v32;
    u32x2 v64;
    u32x4 v128;
    asm volatile("ds_read_b32 %0, %3\n ds_read_b64 %1, %3\n ds_read_b128 %2, %3\n s_waitcnt lgkmcnt(0)"
                 : "=v"(v32), "=v"(v64), "=v"(v128) : "v"(a) : "memory");
    const uint32_t p = 5 * l + s;
    uint32_t e[4] = {0, 0, 0, 0};
    for (int k = 0; k < 16; ++k) e[k >> 2] |= (uint32_t)pat(p + k) << (8 * (k & 3));
    bad += (v32 != e[0]);
    bad += (v64.x != e[0]) + (v64.y != e[1]);
    bad += (v128.x != e[0]) + (v128.y != e[1]) + (v128.z != e[2]) + (v128.w != e[3]);
  }
  atomicAdd(err, bad);
}

// throughput: kIt rounds of 8 independent reads per wave at per-lane addresses from `mode`:
// 0 aligned b128 at 16 * lane, 1 unaligned b128 at 16 * lane + 1, 2 unaligned b128 at a
// pseudo-random byte per lane, 3 the five-dword composition (5 x b32 + 4 alignbyte) at the same
// random bytes, 4 aligned b32 at 4 * lane, 5 unaligned b32 at the random bytes, 6 b32 pair +
// alignbyte at the random bytes, 7 unaligned b64 at the random bytes
template <int M>
__global__ __launch_bounds__(1024) void k_rate(uint32_t* out, int iters) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[65536 + 64];
  const uint32_t t = threadIdx.x, l = t & 63;
  for (uint32_t i = t; i < (65536 + 64) / 4; i += 1024) reinterpret_cast<uint32_t*>(buf)[i] = i * 2654435761u;
  __syncthreads();
  const uint32_t base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)buf;
  uint32_t x = (t * 2654435761u) >> 16;
  uint32_t acc = 0;
  for (int it = 0; it < iters; ++it) {
    uint32_t a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      x = x * 1664525u + 1013904223u;
      const uint32_t r = (x >> 8) & 0xffffu;
      a[j] = M == 0 ? base + 16 * l + 1024 * j : (M == 1 ? base + 16 * l + 1 + 1024 * j : (M == 4 ? base + 4 * l + 256 * j : base + r));
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (M <= 2) {
        u32x4 v;
        asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a[j]) : "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        acc ^= v.x + v.y + v.z + v.w;
      } else if (M == 3) {
        uint32_t w0, w1, w2, w3, w4;
        const uint32_t aa = a[j] & ~3u, s = a[j] & 3u;
        asm volatile("ds_read_b32 %0, %5\n ds_read_b32 %1, %5 offset:4\n ds_read_b32 %2, %5 offset:8\n"
                     " ds_read_b32 %3, %5 offset:12\n ds_read_b32 %4, %5 offset:16\n s_waitcnt lgkmcnt(0)"
                     : "=v"(w0), "=v"(w1), "=v"(w2), "=v"(w3), "=v"(w4) : "v"(aa) : "memory");
        acc ^= __builtin_amdgcn_alignbyte(w1, w0, s) + __builtin_amdgcn_alignbyte(w2, w1, s) +
               __builtin_amdgcn_alignbyte(w3, w2, s) + __builtin_amdgcn_alignbyte(w4, w3, s);
      } else if (M == 4 || M == 5) {
        uint32_t v;
        asm volatile("ds_read_b32 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a[j]) : "memory");
        acc ^= v;
      } else if (M == 6) {
        uint32_t w0, w1;
        const uint32_t aa = a[j] & ~3u, s = a[j] & 3u;
        asm volatile("ds_read_b32 %0, %2\n ds_read_b32 %1, %2 offset:4\n s_waitcnt lgkmcnt(0)"
                     : "=v"(w0), "=v"(w1) : "v"(aa) : "memory");
        acc ^= __builtin_amdgcn_alignbyte(w1, w0, s);
      } else {
        u32x2 v;
        asm volatile("ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a[j]) : "memory");
        acc ^= v.x + v.y;
      }
    }
  }
  out[blockIdx.x * 1024 + t] = acc;
}

template <int M>
static float run(uint32_t* d, int ncu, int iters) {
  hipLaunchKernelGGL(k_rate<M>, dim3(ncu), dim3(1024), 0, 0, d, iters);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k_rate<M>, dim3(ncu), dim3(1024), 0, 0, d, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  uint32_t* d;
  (void)hipMalloc(&d, 64u << 20);
  (void)hipMemset(d, 0, 4);
  hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, d);
  uint32_t bad = 0;
  (void)hipMemcpy(&bad, d, 4, hipMemcpyDeviceToHost);
  printf("unaligned ds_read_b32/b64/b128 mismatches: %u of %u\n", bad, 64u * 16u * 7u);
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const int iters = 2000;
  const char* names[8] = {"b128 aligned, conflict-free", "b128 +1 byte, lane stride 16", "b128 random byte",
                          "5 x b32 + 4 alignbyte, random byte", "b32 aligned, conflict-free", "b32 random byte",
                          "2 x b32 + alignbyte, random byte", "b64 random byte"};
  float ms[8] = {run<0>(d, ncu, iters), run<1>(d, ncu, iters), run<2>(d, ncu, iters), run<3>(d, ncu, iters),
                 run<4>(d, ncu, iters), run<5>(d, ncu, iters), run<6>(d, ncu, iters), run<7>(d, ncu, iters)};
  for (int m = 0; m < 8; ++m) {
    const double per = ms[m] * 1e-3 * 2.4e9 / (16.0 * iters * 8);  // CU cycles per wave-read (16 waves per CU)
    printf("%-40s %.3f ms  %.2f CU-cycles per wave-instruction\n", names[m], ms[m], per);
  }
  return 0;
}
