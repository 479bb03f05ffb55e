// LDS atomic / scatter-write cost microbenchmark (design tool): CU-cycles per wave-instruction
// of random-address LDS atomics and sub-dword writes into a 16 K-entry u32 table, with 1 wave
// per workgroup (the fast compressor's single inserter wave) and with 16 waves.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/lds_atomic_bench tools/lds_atomic_bench.hip && /tmp/lds_atomic_bench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kIters = 1024;

template <int OP>
__global__ void k(uint32_t* out, uint32_t seed) {
  __shared__ __attribute__((aligned(16))) uint32_t T[16384];
  for (uint32_t i = threadIdx.x; i < 16384; i += blockDim.x) T[i] = i;
  __syncthreads();
  uint32_t x = seed ^ (threadIdx.x * 0x9E3779B9u) ^ blockIdx.x;
  uint32_t acc = 0;
  for (int it = 0; it < kIters; ++it) {
    x = x * 1664525u + 1013904223u;
    const uint32_t h = x >> 18;  // random bucket
    if (OP == 0) acc += __hip_atomic_exchange(&T[h], it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else if (OP == 1) reinterpret_cast<uint16_t*>(&T[h])[1] = (uint16_t)it;
    else if (OP == 2) T[h] = it;
    else if (OP == 3) acc += __hip_atomic_fetch_max(&T[h], (uint32_t)it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else if (OP == 4) __hip_atomic_fetch_max(&T[h], (uint32_t)it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else if (OP == 5) acc += T[h];
    else if (OP == 6) {  // exchange then the dependent high-half write (the inserter's pair)
      const uint32_t o = __hip_atomic_exchange(&T[h], it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      reinterpret_cast<uint16_t*>(&T[h])[1] = (uint16_t)o;
      acc += o;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int OP>
void run(uint32_t* d, const char* name) {
  for (int waves : {1, 4, 16}) {
    const int blocks = 256 * (waves == 1 ? 1 : 2);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    k<OP><<<blocks, 64 * waves>>>(d, 1);
    hipEventRecord(e0);
    k<OP><<<blocks, 64 * waves>>>(d, 2);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    // wave-instructions per CU (64 KiB of LDS per block: at most 2 blocks per CU)
    const double winst = (double)blocks * waves * kIters / 256.0;
    printf("%-34s waves/block %2d: %7.2f CU-cycles per wave-instruction\n", name, waves, ms * 1e-3 * 2.4e9 / winst);
  }
}

int main() {
  uint32_t* d;
  hipMalloc(&d, 256 * 8 * 1024 * 4);
  run<0>(d, "ds_wrxchg_rtn_b32 random");
  run<1>(d, "ds_write_b16 (hi) random");
  run<2>(d, "ds_write_b32 random");
  run<3>(d, "ds_max_rtn_u32 random");
  run<4>(d, "ds_max_u32 random");
  run<5>(d, "ds_read_b32 random");
  run<6>(d, "wrxchg + dependent write_b16");
  hipFree(d);
  return 0;
}
