"""Pageable duplex probe (design tool, GPU box): a pageable H2D and a pageable D2H from two host
threads at once (hipMemcpyAsync on two streams), against each alone."""
import ctypes
import threading
import time

import numpy as np
import torch

hip = ctypes.CDLL("libamdhip64.so")
dev = torch.device("cuda", 0)
n1, n2 = 675282944, 298570842
d1 = torch.empty(n1, dtype=torch.uint8, device=dev)
d2 = torch.empty(n2, dtype=torch.uint8, device=dev)
h1 = np.ones(n1, dtype=np.uint8)
h2 = np.ones(n2, dtype=np.uint8)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def up():
    hip.hipMemcpyAsync(ctypes.c_void_p(d1.data_ptr()), ctypes.c_void_p(h1.ctypes.data), ctypes.c_size_t(n1), 1,
                       ctypes.c_void_p(s1.cuda_stream))
    hip.hipStreamSynchronize(ctypes.c_void_p(s1.cuda_stream))


def down():
    hip.hipMemcpyAsync(ctypes.c_void_p(h2.ctypes.data), ctypes.c_void_p(d2.data_ptr()), ctypes.c_size_t(n2), 2,
                       ctypes.c_void_p(s2.cuda_stream))
    hip.hipStreamSynchronize(ctypes.c_void_p(s2.cuda_stream))


def best(fn, reps=3):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter(); fn(); ts.append(time.perf_counter() - t0)
    return min(ts) * 1e3


def both():
    t = threading.Thread(target=down)
    t.start()
    up()
    t.join()


print("H2D alone %.2f ms, D2H alone %.2f ms, both (two threads) %.2f ms" % (best(up), best(down), best(both)))
