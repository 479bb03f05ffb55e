// Design probe (not product code): does one wave's global atomic exchange to a shared address
// service its lanes in ascending lane order on gfx950 (as ds_mskor_rtn_b32 does in the LDS), and
// what does a dependent exchange round cost?
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/gx global_xchg_order.hip && /tmp/gx
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

__global__ void k_order(uint32_t* T, uint32_t* ret, int groups) {
  const uint32_t l = threadIdx.x;
  // lanes in `groups` sets share an address: lane l -> address l % groups
  const uint32_t a = l % groups;
  ret[l] = atomicExch(&T[a], l + 1);
}

__global__ void k_chain(uint32_t* T, uint32_t* out, int iters) {
  uint32_t v = threadIdx.x;
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) v = atomicExch(&T[(v * 2654435761u >> 16) & 16383], v + 1) + i;
  long long t1 = clock64();
  if (threadIdx.x == 0) out[0] = (uint32_t)((t1 - t0) / iters);
  out[1 + threadIdx.x] = v;
}

__global__ void k_chain_lds(uint32_t* out, int iters) {
  __shared__ uint32_t T[16384];
  for (int i = threadIdx.x; i < 16384; i += 64) T[i] = 0;
  __syncthreads();
  uint32_t v = threadIdx.x;
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) v = atomicExch(&T[(v * 2654435761u >> 16) & 16383], v + 1) + i;
  long long t1 = clock64();
  if (threadIdx.x == 0) out[0] = (uint32_t)((t1 - t0) / iters);
  out[1 + threadIdx.x] = v;
}

int main() {
  uint32_t *T, *ret;
  (void)hipMalloc(&T, 1 << 20);
  (void)hipMalloc(&ret, 4096);
  int bad = 0, trials = 0;
  for (int groups = 1; groups <= 8; groups *= 2) {
    for (int rep = 0; rep < 50; ++rep) {
      (void)hipMemset(T, 0, 64);
      hipLaunchKernelGGL(k_order, dim3(1), dim3(64), 0, 0, T, ret, groups);
      uint32_t h[64];
      (void)hipMemcpy(h, ret, 256, hipMemcpyDeviceToHost);
      for (int l = 0; l < 64; ++l) {
        const uint32_t want = l >= groups ? (uint32_t)(l - groups + 1) : 0u;  // ascending lane order
        bad += h[l] != want;
      }
      ++trials;
    }
  }
  printf("global atomicExch, lanes sharing addresses: %d of %d lane results differ from ascending lane order\n", bad,
         trials * 64);
  (void)hipMemset(T, 0, 1 << 16);
  hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, 0, T, ret, 2000);
  uint32_t c;
  (void)hipMemcpy(&c, ret, 4, hipMemcpyDeviceToHost);
  printf("dependent global atomicExch round (one wave, L2-resident table): %u clock64 ticks\n", c);
  hipLaunchKernelGGL(k_chain_lds, dim3(1), dim3(64), 0, 0, ret, 2000);
  (void)hipMemcpy(&c, ret, 4, hipMemcpyDeviceToHost);
  printf("dependent LDS atomicExch round (one wave): %u clock64 ticks\n", c);
  return 0;
}
