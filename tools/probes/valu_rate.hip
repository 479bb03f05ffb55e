// VALU issue rate probe (design tool): integer VALU wave-instructions per cycle per SIMD with W waves
// per SIMD, 8 independent dependency chains per wave.  hipcc --offload-arch=gfx950 -O3 -o /tmp/vr valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int OP>
__global__ void k(uint32_t* out, int iters) {
  uint32_t a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = threadIdx.x * (j + 1) + blockIdx.x;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[j]) : "v"(a[(j + 1) & 7]));
        if (OP == 1) asm volatile("v_alignbyte_b32 %0, %0, %1, 1" : "+v"(a[j]) : "v"(a[(j + 1) & 7]));
        if (OP == 2) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[j]) : "v"(a[(j + 1) & 7]));
      }
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) s ^= a[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t* d;
  hipMalloc(&d, 64u << 20);
  const int iters = 2000;
  for (int op = 0; op < 3; ++op) {
    for (int w : {1, 2, 4, 8}) {  // waves per SIMD: workgroups of 256 threads (one wave per SIMD), w per CU
      dim3 grid(ncu * w), block(256);
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      auto launch = [&]() {
        if (op == 0) hipLaunchKernelGGL(k<0>, grid, block, 0, 0, d, iters);
        if (op == 1) hipLaunchKernelGGL(k<1>, grid, block, 0, 0, d, iters);
        if (op == 2) hipLaunchKernelGGL(k<2>, grid, block, 0, 0, d, iters);
      };
      launch();
      hipDeviceSynchronize();
      hipEventRecord(e0);
      launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double instr_per_simd = (double)w * iters * 16 * 8;  // wave-instructions per SIMD
      const double cycles = ms * 1e-3 * 2.4e9;                    // at 2.4 GHz (approximate)
      printf("op %d (%s) waves/SIMD %d: %.3f ms, %.2f cycles per wave-instruction per SIMD\n", op,
             op == 0 ? "v_add_u32" : op == 1 ? "v_alignbyte" : "v_cndmask", w, ms, cycles / instr_per_simd);
    }
  }
  return 0;
}
