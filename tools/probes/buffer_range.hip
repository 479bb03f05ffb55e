// Buffer-resource probe (design tool, GPU box): what a raw buffer dword load returns at and past
// num_records (6 here), from an aligned and from a misaligned base.  Measured on gfx950: a load
// at offset o returns 0 when o + 4 > num_records (the whole dword), and unaligned loads are
// served -- the basis of the reference-mode compressor's exact block bounds (sm_compress.hip).
//   hipcc --offload-arch=gfx950 -O2 -o /tmp/buffer_range tools/probes/buffer_range.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
__global__ void k(const uint8_t* src, uint32_t* out) {
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 6, 0x00020000);
  int t = threadIdx.x;  // offsets 0..11
  out[t] = __builtin_amdgcn_raw_buffer_load_b32(r, t, 0, 0);
  __amdgpu_buffer_rsrc_t r2 = __builtin_amdgcn_make_buffer_rsrc((void*)(src + 1), (short)0, 6, 0x00020000);
  out[16 + t] = __builtin_amdgcn_raw_buffer_load_b32(r2, t, 0, 0);
}
int main() {
  uint8_t h[64]; for (int i = 0; i < 64; ++i) h[i] = i + 1;
  uint8_t* d; uint32_t* o; hipMalloc(&d, 64); hipMalloc(&o, 128);
  hipMemcpy(d, h, 64, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, 1, 12, 0, 0, d, o);
  uint32_t ho[32]; hipMemcpy(ho, o, 128, hipMemcpyDeviceToHost);
  for (int i = 0; i < 12; ++i) printf("base+0 off %2d: %08x   base+1 off %2d: %08x\n", i, ho[i], i, ho[16 + i]);
  return 0;
}
