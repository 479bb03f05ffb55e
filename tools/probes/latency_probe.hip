// Single-call latency floor (design tool, GPU box): what one small sm_uncompress / sm_compress
// call can cost at best, per ingredient.  Medians of 200 repetitions, microseconds.
//   hipcc --offload-arch=gfx950 -O2 -o /tmp/latency_probe tools/probes/latency_probe.hip && /tmp/latency_probe
// Ingredients: launch + synchronize (one kernel, a chain of six, the chain as a hipGraph), host
// waits (hipStreamSynchronize vs spinning on a flag the last kernel stores to pinned memory),
// and moving N bytes each way: pageable hipMemcpyAsync, memcpy + DMA through registered
// (pinned) memory, and a kernel reading / writing the pinned memory directly over PCIe.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                            \
    }                                                                     \
  } while (0)

__global__ void k_empty(int* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1;
}

// grid-stride 16-byte copy; src or dst may be host-mapped pinned memory
__global__ void k_copy16(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

// the last kernel of a call publishes completion to a pinned host word (vector store + release)
__global__ void k_flag(volatile unsigned* flag, unsigned v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    __threadfence_system();
    flag[0] = v;
  }
}

static double med(const std::function<void()>& f, int n = 200) {
  f();
  f();
  std::vector<double> t(n);
  for (int i = 0; i < n; ++i) {
    auto a = std::chrono::steady_clock::now();
    f();
    t[i] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
  }
  std::sort(t.begin(), t.end());
  return t[n / 2];
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int* d_int;
  CK(hipMalloc(&d_int, 64));
  const size_t maxn = 1 << 20;
  uint8_t *d_a, *d_b;
  CK(hipMalloc(&d_a, maxn));
  CK(hipMalloc(&d_b, maxn));
  std::vector<uint8_t> page_in(maxn, 1), page_out(maxn);
  // registered pinned staging (what sm_ctx's HostBuf does) and a hipHostMalloc'd one
  void* reg = nullptr;
  if (posix_memalign(&reg, 4096, maxn)) return 1;
  CK(hipHostRegister(reg, maxn, hipHostRegisterMapped));
  void* reg_dev = nullptr;
  CK(hipHostGetDevicePointer(&reg_dev, reg, 0));
  void* hm = nullptr;
  CK(hipHostMalloc(&hm, maxn, hipHostMallocMapped));
  void* hm_dev = nullptr;
  CK(hipHostGetDevicePointer(&hm_dev, hm, 0));
  unsigned* flag = nullptr;
  CK(hipHostMalloc((void**)&flag, 64, hipHostMallocMapped | hipHostMallocCoherent));
  unsigned* flag_dev = nullptr;
  CK(hipHostGetDevicePointer((void**)&flag_dev, flag, 0));

  printf("launch + wait:\n");
  printf("  1 kernel + hipStreamSynchronize        %7.1f\n",
         med([&] { k_empty<<<1, 64, 0, s>>>(d_int); CK(hipStreamSynchronize(s)); }));
  printf("  6 kernels + hipStreamSynchronize       %7.1f\n", med([&] {
           for (int i = 0; i < 6; ++i) k_empty<<<1, 64, 0, s>>>(d_int);
           CK(hipStreamSynchronize(s));
         }));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
  for (int i = 0; i < 6; ++i) k_empty<<<1, 64, 0, s>>>(d_int);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  printf("  6 kernels as a hipGraph + sync         %7.1f\n",
         med([&] { CK(hipGraphLaunch(ge, s)); CK(hipStreamSynchronize(s)); }));
  unsigned seq = 0;
  printf("  1 kernel + spin on a pinned flag       %7.1f\n", med([&] {
           ++seq;
           k_flag<<<1, 64, 0, s>>>(flag_dev, seq);
           while (__atomic_load_n(&flag[0], __ATOMIC_ACQUIRE) != seq) {
           }
         }));
  printf("  6 kernels + spin on a pinned flag      %7.1f\n", med([&] {
           ++seq;
           for (int i = 0; i < 5; ++i) k_empty<<<1, 64, 0, s>>>(d_int);
           k_flag<<<1, 64, 0, s>>>(flag_dev, seq);
           while (__atomic_load_n(&flag[0], __ATOMIC_ACQUIRE) != seq) {
           }
         }));
  CK(hipStreamSynchronize(s));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  printf("  1 kernel + event record + event sync   %7.1f\n", med([&] {
           k_empty<<<1, 64, 0, s>>>(d_int);
           CK(hipEventRecord(ev, s));
           CK(hipEventSynchronize(ev));
         }));

  // a call's small control words: from / to the stack (pageable) or a pinned block
  uint32_t word[4] = {1, 2, 3, 4};
  printf("control words (16 B):\n");
  printf("  kernel + H2D stack + sync              %7.1f\n", med([&] {
           CK(hipMemcpyAsync(d_int, word, 16, hipMemcpyHostToDevice, s));
           k_empty<<<1, 64, 0, s>>>(d_int);
           CK(hipStreamSynchronize(s));
         }));
  printf("  kernel + H2D pinned + sync             %7.1f\n", med([&] {
           memcpy(hm, word, 16);
           CK(hipMemcpyAsync(d_int, hm, 16, hipMemcpyHostToDevice, s));
           k_empty<<<1, 64, 0, s>>>(d_int);
           CK(hipStreamSynchronize(s));
         }));
  printf("  kernel + D2H stack + sync              %7.1f\n", med([&] {
           k_empty<<<1, 64, 0, s>>>(d_int);
           CK(hipMemcpyAsync(word, d_int, 16, hipMemcpyDeviceToHost, s));
           CK(hipStreamSynchronize(s));
         }));
  printf("  kernel + D2H pinned + sync             %7.1f\n", med([&] {
           k_empty<<<1, 64, 0, s>>>(d_int);
           CK(hipMemcpyAsync(hm, d_int, 16, hipMemcpyDeviceToHost, s));
           CK(hipStreamSynchronize(s));
         }));
  printf("  kernel + 2x D2H stack + 64K D2H pageable + sync %7.1f\n", med([&] {
           k_empty<<<1, 64, 0, s>>>(d_int);
           CK(hipMemcpyAsync(word, d_int, 4, hipMemcpyDeviceToHost, s));
           CK(hipMemcpyAsync(word + 1, d_int + 1, 4, hipMemcpyDeviceToHost, s));
           CK(hipMemcpyAsync(page_out.data(), d_b, 65536, hipMemcpyDeviceToHost, s));
           CK(hipStreamSynchronize(s));
         }));
  printf("  kernel + 64K D2H pinned (words in it) + sync + memcpy %7.1f\n", med([&] {
           k_empty<<<1, 64, 0, s>>>(d_int);
           CK(hipMemcpyAsync(reg, d_b, 65536 + 16, hipMemcpyDeviceToHost, s));
           CK(hipStreamSynchronize(s));
           memcpy(page_out.data(), reg, 65536);
         }));

  printf("  kernel + 64K D2H pageable + sync       %7.1f\n", med([&] {
           k_empty<<<1, 64, 0, s>>>(d_int);
           CK(hipMemcpyAsync(page_out.data(), d_b, 65536, hipMemcpyDeviceToHost, s));
           CK(hipStreamSynchronize(s));
         }));
  printf("  kernel + 4B D2H stack + 64K D2H pageable + sync %7.1f\n", med([&] {
           k_empty<<<1, 64, 0, s>>>(d_int);
           CK(hipMemcpyAsync(word, d_int, 4, hipMemcpyDeviceToHost, s));
           CK(hipMemcpyAsync(page_out.data(), d_b, 65536, hipMemcpyDeviceToHost, s));
           CK(hipStreamSynchronize(s));
         }));
  printf("  4B D2H stack + 64K D2H pageable + sync %7.1f\n", med([&] {
           CK(hipMemcpyAsync(word, d_int, 4, hipMemcpyDeviceToHost, s));
           CK(hipMemcpyAsync(page_out.data(), d_b, 65536, hipMemcpyDeviceToHost, s));
           CK(hipStreamSynchronize(s));
         }));
  printf("  kernel + 64K D2H pinned + sync         %7.1f\n", med([&] {
           k_empty<<<1, 64, 0, s>>>(d_int);
           CK(hipMemcpyAsync(reg, d_b, 65536, hipMemcpyDeviceToHost, s));
           CK(hipStreamSynchronize(s));
         }));
  printf("  kernel + 65552 B D2H pinned + sync     %7.1f\n", med([&] {
           k_empty<<<1, 64, 0, s>>>(d_int);
           CK(hipMemcpyAsync(reg, d_b, 65552, hipMemcpyDeviceToHost, s));
           CK(hipStreamSynchronize(s));
         }));
  printf("  65552 B D2H pinned + sync              %7.1f\n", med([&] {
           CK(hipMemcpyAsync(reg, d_b, 65552, hipMemcpyDeviceToHost, s));
           CK(hipStreamSynchronize(s));
         }));
  printf("  kernel + 16K D2H pinned + sync         %7.1f\n", med([&] {
           k_empty<<<1, 64, 0, s>>>(d_int);
           CK(hipMemcpyAsync(reg, d_b, 16384, hipMemcpyDeviceToHost, s));
           CK(hipStreamSynchronize(s));
         }));
  printf("  kernel + 100000 B D2H pinned + sync    %7.1f\n", med([&] {
           k_empty<<<1, 64, 0, s>>>(d_int);
           CK(hipMemcpyAsync(reg, d_b, 100000, hipMemcpyDeviceToHost, s));
           CK(hipStreamSynchronize(s));
         }));
  printf("  kernel + 100000 B D2H pageable + sync  %7.1f\n", med([&] {
           k_empty<<<1, 64, 0, s>>>(d_int);
           CK(hipMemcpyAsync(page_out.data(), d_b, 100000, hipMemcpyDeviceToHost, s));
           CK(hipStreamSynchronize(s));
         }));

  printf("call shapes (23 KB in, 100 KB out):\n");
  printf("  path-4 shape: H2D pageable, 6 kernels, 40B D2H stack, D2H pageable, sync %7.1f\n", med([&] {
           CK(hipMemcpyAsync(d_a, page_in.data(), 23000, hipMemcpyHostToDevice, s));
           for (int i = 0; i < 6; ++i) k_empty<<<1, 64, 0, s>>>(d_int);
           CK(hipMemcpyAsync(word, d_int, 16, hipMemcpyDeviceToHost, s));
           CK(hipMemcpyAsync(page_out.data(), d_b, 100000, hipMemcpyDeviceToHost, s));
           CK(hipStreamSynchronize(s));
         }));
  printf("  path-0 shape: H2D, 2x8B H2D, kernel, 2x4B D2H, sync, D2H, sync %7.1f\n", med([&] {
           CK(hipMemcpyAsync(d_a, page_in.data(), 23000, hipMemcpyHostToDevice, s));
           CK(hipMemcpyAsync(d_int, word, 8, hipMemcpyHostToDevice, s));
           CK(hipMemcpyAsync(d_int + 2, word, 8, hipMemcpyHostToDevice, s));
           k_empty<<<1, 64, 0, s>>>(d_int);
           CK(hipMemcpyAsync(word, d_int, 4, hipMemcpyDeviceToHost, s));
           CK(hipMemcpyAsync(word + 1, d_int, 4, hipMemcpyDeviceToHost, s));
           CK(hipStreamSynchronize(s));
           CK(hipMemcpyAsync(page_out.data(), d_b, 100000, hipMemcpyDeviceToHost, s));
           CK(hipStreamSynchronize(s));
         }));
  printf("  kernels only: memcpy in, copy kernel, 6 kernels, kernel out, sync, memcpy %7.1f\n", med([&] {
           memcpy(reg, page_in.data(), 23008);
           k_copy16<<<6, 256, 0, s>>>((const uint4*)reg_dev, (uint4*)d_a, 23008 / 16);
           for (int i = 0; i < 6; ++i) k_empty<<<1, 64, 0, s>>>(d_int);
           k_copy16<<<25, 256, 0, s>>>((const uint4*)d_b, (uint4*)reg_dev, 100000 / 16);
           CK(hipStreamSynchronize(s));
           memcpy(page_out.data(), reg, 100000);
         }));
  printf("  H2D pinned DMA, 6 kernels, kernel out, sync, memcpy %7.1f\n", med([&] {
           memcpy(reg, page_in.data(), 23008);
           CK(hipMemcpyAsync(d_a, reg, 23008, hipMemcpyHostToDevice, s));
           for (int i = 0; i < 6; ++i) k_empty<<<1, 64, 0, s>>>(d_int);
           k_copy16<<<25, 256, 0, s>>>((const uint4*)d_b, (uint4*)reg_dev, 100000 / 16);
           CK(hipStreamSynchronize(s));
           memcpy(page_out.data(), reg, 100000);
         }));

  for (size_t n : {(size_t)4096, (size_t)65536, (size_t)262144, (size_t)1 << 20}) {
    const size_t n16 = n / 16;
    const unsigned grid = (unsigned)std::min<size_t>(1024, (n16 + 255) / 256);
    printf("%zu bytes:\n", n);
    printf("  H2D pageable memcpyAsync + sync        %7.1f\n", med([&] {
             CK(hipMemcpyAsync(d_a, page_in.data(), n, hipMemcpyHostToDevice, s));
             CK(hipStreamSynchronize(s));
           }));
    printf("  H2D memcpy->registered + DMA + sync    %7.1f\n", med([&] {
             memcpy(reg, page_in.data(), n);
             CK(hipMemcpyAsync(d_a, reg, n, hipMemcpyHostToDevice, s));
             CK(hipStreamSynchronize(s));
           }));
    printf("  H2D memcpy->registered + kernel + sync %7.1f\n", med([&] {
             memcpy(reg, page_in.data(), n);
             k_copy16<<<grid, 256, 0, s>>>((const uint4*)reg_dev, (uint4*)d_a, n16);
             CK(hipStreamSynchronize(s));
           }));
    printf("  H2D memcpy->hostmalloc + kernel + sync %7.1f\n", med([&] {
             memcpy(hm, page_in.data(), n);
             k_copy16<<<grid, 256, 0, s>>>((const uint4*)hm_dev, (uint4*)d_a, n16);
             CK(hipStreamSynchronize(s));
           }));
    printf("  D2H pageable memcpyAsync + sync        %7.1f\n", med([&] {
             CK(hipMemcpyAsync(page_out.data(), d_b, n, hipMemcpyDeviceToHost, s));
             CK(hipStreamSynchronize(s));
           }));
    printf("  D2H DMA->registered + sync + memcpy    %7.1f\n", med([&] {
             CK(hipMemcpyAsync(reg, d_b, n, hipMemcpyDeviceToHost, s));
             CK(hipStreamSynchronize(s));
             memcpy(page_out.data(), reg, n);
           }));
    printf("  D2H kernel->registered + sync + memcpy %7.1f\n", med([&] {
             k_copy16<<<grid, 256, 0, s>>>((const uint4*)d_b, (uint4*)reg_dev, n16);
             CK(hipStreamSynchronize(s));
             memcpy(page_out.data(), reg, n);
           }));
    printf("  D2H kernel->hostmalloc + sync + memcpy %7.1f\n", med([&] {
             k_copy16<<<grid, 256, 0, s>>>((const uint4*)d_b, (uint4*)hm_dev, n16);
             CK(hipStreamSynchronize(s));
             memcpy(page_out.data(), hm, n);
           }));
    printf("  round trip: pageable H2D, 6 kernels, pageable D2H %7.1f\n", med([&] {
             CK(hipMemcpyAsync(d_a, page_in.data(), n, hipMemcpyHostToDevice, s));
             for (int i = 0; i < 6; ++i) k_empty<<<1, 64, 0, s>>>(d_int);
             CK(hipMemcpyAsync(page_out.data(), d_b, n, hipMemcpyDeviceToHost, s));
             CK(hipStreamSynchronize(s));
           }));
    printf("  round trip: kernel in, 6 kernels, kernel out, one sync %7.1f\n", med([&] {
             memcpy(reg, page_in.data(), n);
             k_copy16<<<grid, 256, 0, s>>>((const uint4*)reg_dev, (uint4*)d_a, n16);
             for (int i = 0; i < 6; ++i) k_empty<<<1, 64, 0, s>>>(d_int);
             k_copy16<<<grid, 256, 0, s>>>((const uint4*)d_b, (uint4*)reg_dev, n16);
             CK(hipStreamSynchronize(s));
             memcpy(page_out.data(), reg, n);
           }));
  }
  CK(hipStreamSynchronize(s));
  CK(hipHostUnregister(reg));
  free(reg);
  CK(hipHostFree(hm));
  CK(hipHostFree(flag));
  printf("done\n");
  return 0;
}
