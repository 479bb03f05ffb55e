// Diagnostic probe (not product code): unaligned LDS dword/qword reads and the lane order of
// conflicting ds_max_rtn_u32 within one instruction, on gfx950.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void k(uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[1024];
  __shared__ uint32_t tab[64];
  int l = threadIdx.x;
  for (int i = l; i < 1024; i += 64) buf[i] = (uint8_t)(i * 7 + 3);
  if (l < 64) tab[l] = 0;
  __syncthreads();
  // unaligned 32-bit and 64-bit reads at byte offset 3*l+1
  uint32_t pos = 3 * l + 1;
  uint32_t v32;
  uint64_t v64;
  typedef uint32_t __attribute__((aligned(1))) u32u;
  typedef uint64_t __attribute__((aligned(1))) u64u;
  v32 = *(const u32u*)(buf + pos);
  v64 = *(const u64u*)(buf + pos);
  uint32_t e32 = 0; uint64_t e64 = 0;
  for (int k2 = 0; k2 < 4; ++k2) e32 |= (uint32_t)(uint8_t)((pos + k2) * 7 + 3) << (8 * k2);
  for (int k2 = 0; k2 < 8; ++k2) e64 |= (uint64_t)(uint8_t)((pos + k2) * 7 + 3) << (8 * k2);
  out[l] = (v32 == e32);
  out[64 + l] = (v64 == e64);
  // conflicting atomic max with return: all lanes -> 4 addresses, value = lane+1
  uint32_t r = atomicMax(&tab[l & 3], (uint32_t)(l + 1));
  out[128 + l] = r;
}

int main() {
  uint32_t* d; hipMalloc(&d, 192 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  uint32_t h[192]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int ok32 = 0, ok64 = 0;
  for (int i = 0; i < 64; ++i) { ok32 += h[i]; ok64 += h[64 + i]; }
  printf("unaligned ds_read_b32 correct lanes: %d/64, ds_read_b64: %d/64\n", ok32, ok64);
  int ordered = 1;
  for (int i = 0; i < 64; ++i) { uint32_t expect = (i >= 4) ? (uint32_t)(i - 4 + 1) : 0; if (h[128 + i] != expect) ordered = 0; }
  printf("ds_max_rtn lane-ascending: %d; first lanes:", ordered);
  for (int i = 0; i < 16; ++i) printf(" %u", h[128 + i]);
  printf("\n");
  return 0;
}
