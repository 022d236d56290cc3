import ctypes, sys, time
sys.path.insert(0, "qsfs-fuse_amd"); sys.path.insert(0, "tests")
t0 = time.perf_counter()
import qsmd5
lib = qsmd5.lib()
t1 = time.perf_counter()
from oracle_util import lcg_bytes
data = lcg_bytes(12345, 10 << 20)
t2 = time.perf_counter(); rc = lib.qsmd5_init(0); t3 = time.perf_counter()
print("load %.1f ms, init %.1f ms (rc %d)" % ((t1 - t0) * 1e3, (t3 - t2) * 1e3, rc))
for i in range(3):
    a = time.perf_counter(); d = qsmd5.hash_one((ctypes.addressof(data), 10 << 20)); b = time.perf_counter()
    print("call %d: %.1f ms %s" % (i, (b - a) * 1e3, d.hex()))
