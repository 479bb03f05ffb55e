// VALU issue rate probe (design tool): integer VALU wave-instructions per cycle per SIMD with W waves
// per SIMD, 8 independent dependency chains per wave.  hipcc --offload-arch=gfx950 -O3 -o /tmp/vr valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <utility>

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
        if (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[j]) : "v"(a[(j + 1) & 7]) : "s4", "s5");
        if (OP == 1) asm volatile("v_alignbyte_b32 %0, %0, %1, 1" : "+v"(a[j]) : "v"(a[(j + 1) & 7]) : "s4", "s5");
        if (OP == 2) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[4:5]" : "+v"(a[j]) : "v"(a[(j + 1) & 7]) : "s4", "s5");
        if (OP == 3) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[j]) : "v"(a[(j + 1) & 7]) : "s4", "s5");
        if (OP == 4) asm volatile("v_lshlrev_b32 %0, 3, %1" : "+v"(a[j]) : "v"(a[(j + 1) & 7]) : "s4", "s5");
        if (OP == 5) asm volatile("v_bfe_u32 %0, %0, %1, 8" : "+v"(a[j]) : "v"(a[(j + 1) & 7]) : "s4", "s5");
        if (OP == 6) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[j]) : "v"(a[(j + 1) & 7]) : "s4", "s5");
        if (OP == 7) asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(a[j]) : "v"(a[(j + 1) & 7]) : "s4", "s5");
        if (OP == 8) asm volatile("v_min_u32 %0, %0, %1" : "+v"(a[j]) : "v"(a[(j + 1) & 7]) : "s4", "s5");
        if (OP == 9) asm volatile("v_ffbl_b32 %0, %1" : "+v"(a[j]) : "v"(a[(j + 1) & 7]) : "s4", "s5");
        if (OP == 10) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(a[j]) : "v"(a[(j + 1) & 7]) : "s4", "s5");
        if (OP == 11) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[j]) : "v"(a[(j + 1) & 7]) : "s4", "s5");
        if (OP == 12) asm volatile("v_cmp_gt_u32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[j]) : "v"(a[(j + 1) & 7]) : "s4", "s5", "vcc");
        if (OP == 13) asm volatile("v_lshrrev_b64 v[20:21], 3, v[20:21]" : : : "v20", "v21");
      }
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) s ^= a[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

static const char* kNames[] = {"v_add_u32", "v_alignbyte", "v_cndmask_e64", "v_xor", "v_lshlrev", "v_bfe_u32", "v_mul_u32_u24", "v_lshl_add", "v_min_u32", "v_ffbl", "v_perm", "v_mul_lo_u32", "v_cmp+cndmask", "v_lshrrev_b64"};
constexpr int kOps = 14;

template <int OP>
static void launch(dim3 g, dim3 b, uint32_t* d, int iters) { hipLaunchKernelGGL(k<OP>, g, b, 0, 0, d, iters); }
template <int... I>
static void launch_op(int op, dim3 g, dim3 b, uint32_t* d, int iters, std::integer_sequence<int, I...>) {
  ((op == I ? launch<I>(g, b, d, iters) : void()), ...);
}

int main() {
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t* d;
  (void)hipMalloc(&d, 64u << 20);
  const int iters = 1000;
  for (int op = 0; op < kOps; ++op) {
    for (int w : {1, 4}) {  // waves per SIMD: workgroups of 256 threads (one wave per SIMD), w per CU
      dim3 grid(ncu * w), block(256);
      hipEvent_t e0, e1;
      (void)hipEventCreate(&e0);
      (void)hipEventCreate(&e1);
      launch_op(op, grid, block, d, iters, std::make_integer_sequence<int, kOps>{});
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(e0);
      launch_op(op, grid, block, d, iters, std::make_integer_sequence<int, kOps>{});
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      const double instr_per_simd = (double)w * iters * 16 * 8;  // wave-instructions per SIMD
      const double cycles = ms * 1e-3 * 2.4e9;                    // at 2.4 GHz (approximate)
      printf("%-16s waves/SIMD %d: %.3f ms, %.2f cycles per wave-instruction per SIMD\n", kNames[op], w, ms,
             cycles / instr_per_simd);
    }
  }
  return 0;
}
