"""Streaming MD5 class (qsmd5_ctx) rate: 64 MiB fed in 1 MiB and 64 KiB host
pieces, and as one 64 MiB device update; digest checked against the oracle."""
import ctypes
import sys
import time

sys.path.insert(0, "qsfs-fuse_amd")
sys.path.insert(0, "tests")
import qsmd5  # noqa: E402
from oracle_util import lcg_bytes, md5_ref  # noqa: E402

L = 64 << 20
data = lcg_bytes(99, L)
want = md5_ref(data, L)
lib = qsmd5.lib()
lib.qsmd5_init(0)
for piece in (1 << 20, 64 << 10):
    h = qsmd5.MD5()
    t0 = time.perf_counter()
    base = ctypes.addressof(data)
    for off in range(0, L, piece):
        h.update((base + off, piece))
    d = h.finalize().digest()
    dt = time.perf_counter() - t0
    print("ctx %d KiB pieces: %.1f ms, %.3f GiB/s, %s" % (piece >> 10, dt * 1e3, L / dt / (1 << 30),
                                                          "ok" if d == want else "FAIL"), flush=True)
