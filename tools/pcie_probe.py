"""PCIe probe (design tool, GPU box): D2H of a 644 MiB device buffer into pageable host memory by
hipMemcpy, hipMemcpyAsync + sync, and after hipHostRegister (with the registration's cost), plus
CPU read speed of hipHostMalloc'd vs registered memory."""
import ctypes
import time

import numpy as np
import torch

hip = ctypes.CDLL("libamdhip64.so")
n = 675282944
dev = torch.device("cuda", 0)
d = torch.empty(n, dtype=torch.uint8, device=dev)
d.fill_(7)
torch.cuda.synchronize()
dp = ctypes.c_void_p(d.data_ptr())
back = np.zeros(n, dtype=np.uint8)
back[:] = 1
bp = ctypes.c_void_p(back.ctypes.data)
D2H, H2D = 2, 1


def best(fn, reps=3):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter(); fn(); ts.append(time.perf_counter() - t0)
    return min(ts)


x = best(lambda: hip.hipMemcpy(bp, dp, ctypes.c_size_t(n), D2H)); print("hipMemcpy D2H pageable   %.1f GB/s" % (n / x / 1e9))
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
x = best(lambda: (hip.hipMemcpyAsync(bp, dp, ctypes.c_size_t(n), D2H, s), hip.hipStreamSynchronize(s)))
print("hipMemcpyAsync D2H pageable %.1f GB/s" % (n / x / 1e9))
x = best(lambda: hip.hipMemcpy(dp, bp, ctypes.c_size_t(n), H2D)); print("hipMemcpy H2D pageable   %.1f GB/s" % (n / x / 1e9))
t0 = time.perf_counter(); r = hip.hipHostRegister(bp, ctypes.c_size_t(n), 0); t1 = time.perf_counter()
print("hipHostRegister 644 MiB: rc %d, %.2f ms" % (r, (t1 - t0) * 1e3))
x = best(lambda: (hip.hipMemcpyAsync(bp, dp, ctypes.c_size_t(n), D2H, s), hip.hipStreamSynchronize(s)))
print("registered D2H %.1f GB/s" % (n / x / 1e9))
t0 = time.perf_counter(); hip.hipHostUnregister(bp); t1 = time.perf_counter()
print("hipHostUnregister: %.2f ms" % ((t1 - t0) * 1e3))
# CPU reads
m = 64 << 20
hp = ctypes.c_void_p()
hip.hipHostMalloc(ctypes.byref(hp), ctypes.c_size_t(m), 0)
arr = np.ctypeslib.as_array((ctypes.c_uint8 * m).from_address(hp.value))
arr[:] = 3
x = best(lambda: int(arr[::256].sum())); print("CPU strided read hipHostMalloc(default): %.2f ms per 256K reads" % (x * 1e3))
reg = np.ones(m, dtype=np.uint8)
hip.hipHostRegister(ctypes.c_void_p(reg.ctypes.data), ctypes.c_size_t(m), 0)
x = best(lambda: int(reg[::256].sum())); print("CPU strided read registered: %.2f ms per 256K reads" % (x * 1e3))
x = best(lambda: np.copyto(back[:m], arr)); print("CPU copy from hipHostMalloc: %.1f GB/s" % (m / x / 1e9))
x = best(lambda: np.copyto(back[:m], reg)); print("CPU copy from registered: %.1f GB/s" % (m / x / 1e9))
