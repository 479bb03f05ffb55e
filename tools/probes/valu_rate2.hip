// VALU issue rate probe, round 6 (design tool): cycles per wave-instruction per SIMD for the
// integer VALU forms the codec kernels use, with 4 waves per SIMD (16 per CU), 8 independent
// chains per wave.  hipcc --offload-arch=gfx950 -O3 -o tools/probes/valu_rate2 tools/probes/valu_rate2.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <utility>

#define OPS(X)                                                                          \
  X(0, "v_add_u32 e32", "v_add_u32 %0, %0, %1")                                         \
  X(1, "v_sub_u32 e32", "v_sub_u32 %0, %0, %1")                                         \
  X(2, "v_and_b32 e32", "v_and_b32 %0, %0, %1")                                         \
  X(3, "v_or_b32 e32", "v_or_b32 %0, %0, %1")                                           \
  X(4, "v_xor_b32 e32", "v_xor_b32 %0, %0, %1")                                         \
  X(5, "v_mov_b32", "v_mov_b32 %0, %1")                                                 \
  X(6, "v_cndmask e32 vcc", "v_cndmask_b32 %0, %0, %1, vcc")                            \
  X(7, "v_cndmask e64 sgpr", "v_cndmask_b32_e64 %0, %0, %1, s[4:5]")                    \
  X(8, "v_alignbyte", "v_alignbyte_b32 %0, %0, %1, 1")                                  \
  X(9, "v_alignbyte vsh", "v_alignbyte_b32 %0, %0, %1, %1")                             \
  X(10, "v_lshlrev e32", "v_lshlrev_b32 %0, 3, %1")                                     \
  X(11, "v_lshrrev e32", "v_lshrrev_b32 %0, 3, %1")                                     \
  X(12, "v_lshlrev e32 vv", "v_lshlrev_b32 %0, %1, %0")                                 \
  X(13, "v_min_u32 e32", "v_min_u32 %0, %0, %1")                                        \
  X(14, "v_max_u32 e32", "v_max_u32 %0, %0, %1")                                        \
  X(15, "v_bfe_u32", "v_bfe_u32 %0, %0, %1, 8")                                         \
  X(16, "v_ffbl_b32", "v_ffbl_b32 %0, %1")                                              \
  X(17, "v_perm_b32", "v_perm_b32 %0, %0, %1, %1")                                      \
  X(18, "v_add3_u32", "v_add3_u32 %0, %0, %1, %1")                                      \
  X(19, "v_or3_b32", "v_or3_b32 %0, %0, %1, %1")                                        \
  X(20, "v_lshl_or_b32", "v_lshl_or_b32 %0, %0, 2, %1")                                 \
  X(21, "v_and_or_b32", "v_and_or_b32 %0, %0, %1, %1")                                  \
  X(22, "v_lshl_add_u32", "v_lshl_add_u32 %0, %0, 2, %1")                               \
  X(23, "v_bitop3_b32", "v_bitop3_b32 %0, %0, %1, %1 bitop3:0x80")                      \
  X(24, "v_bfi_b32", "v_bfi_b32 %0, %0, %1, %1")                                        \
  X(25, "v_cmp_lt e32 (vcc)", "v_cmp_lt_u32 vcc, %0, %1")                               \
  X(26, "v_cmp_lt e64 (sgpr)", "v_cmp_lt_u32_e64 s[6:7], %0, %1")                       \
  X(27, "v_mul_u32_u24", "v_mul_u32_u24 %0, %0, %1")                                    \
  X(28, "v_mul_lo_u32", "v_mul_lo_u32 %0, %0, %1")                                      \
  X(29, "v_add_u32 e64", "v_add_u32_e64 %0, %0, %1")                                    \
  X(30, "v_xad_u32", "v_xad_u32 %0, %0, %1, %1")                                        \
  X(31, "v_mov_b32 dpp shr1", "v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf") \
  X(32, "v_add_u32 dpp shr1", "v_add_u32_dpp %0, %1, %0 row_shr:1 row_mask:0xf bank_mask:0xf") \
  X(33, "v_lshrrev_b64", "v_lshrrev_b64 v[20:21], 3, v[20:21]")                         \
  X(34, "v_sub_u32 e64 sgpr", "v_sub_u32_e64 %0, s8, %0")                               \
  X(35, "v_pk_add_u16", "v_pk_add_u16 %0, %0, %1")                                      \
  X(36, "v_add_u16 e32", "v_add_u16 %0, %0, %1")                                        \
  X(37, "v_min3_u32", "v_min3_u32 %0, %0, %1, %1")                                      \
  X(38, "v_med3_u32", "v_med3_u32 %0, %0, %1, %1")                                      \
  X(39, "v_not_b32", "v_not_b32 %0, %1")

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, int iters) {
  uint32_t a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = threadIdx.x * (j + 1) + blockIdx.x;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
#define X(n, name, text) \
  if (OP == n) asm volatile(text : "+v"(a[j]) : "v"(a[(j + 1) & 7]) : "s4", "s5", "s6", "s7", "s8", "vcc", "v20", "v21");
        OPS(X)
#undef X
      }
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) s ^= a[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

#define X(n, name, text) name,
static const char* kNames[] = {OPS(X)};
#undef X
constexpr int kOps = sizeof(kNames) / sizeof(kNames[0]);

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
  const int iters = 2000;
  // the reference: v_add_u32 e32 at 4 waves per SIMD; everything relative to it
  double ref = 0;
  for (int op = 0; op < kOps; ++op) {
    const int w = 4;  // workgroups of 256 threads (one wave per SIMD), w per CU
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
    const double instr_per_simd = (double)w * iters * 16 * 8;
    const double cyc = ms * 1e-3 * 2.4e9 / instr_per_simd;
    if (op == 0) ref = cyc;
    printf("%-22s %.3f ms  %.2f cycles/wave-instr per SIMD (2.4 GHz)  x%.2f of v_add_u32\n", kNames[op], ms, cyc,
           cyc / ref);
  }
  return 0;
}
