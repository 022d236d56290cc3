"""Cost of hipHostRegister on a large pageable buffer, and H2D rates from
pageable vs registered memory (one 1 GiB hipMemcpy each)."""
import ctypes
import time

import numpy as np
import torch

hip = ctypes.CDLL("libamdhip64.so")
torch.cuda.init()
GiB = 1 << 30
for size in (1 * GiB, 10 * GiB):
    a = np.empty(size, dtype=np.uint8)
    a[::4096] = 1  # fault the pages in
    p = a.ctypes.data
    t0 = time.perf_counter()
    rc = hip.hipHostRegister(ctypes.c_void_p(p), ctypes.c_size_t(size), 0)
    t1 = time.perf_counter()
    print("register %d GiB: rc=%d %.2f ms" % (size // GiB, rc, (t1 - t0) * 1e3), flush=True)
    d = torch.empty(GiB, dtype=torch.uint8, device="cuda")
    for name in ("registered", "unregistered"):
        if name == "unregistered":
            t2 = time.perf_counter()
            rc2 = hip.hipHostUnregister(ctypes.c_void_p(p))
            print("unregister: rc=%d %.2f ms" % (rc2, (time.perf_counter() - t2) * 1e3))
        best = 1e9
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            hip.hipMemcpy(ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(p), ctypes.c_size_t(GiB), 1)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        print("  H2D 1 GiB from %s: %.1f GB/s" % (name, GiB / best / 1e9), flush=True)
    del a, d
