import ctypes, statistics, sys, time
sys.path.insert(0, "qsfs-fuse_amd"); sys.path.insert(0, "tests")
import qsmd5
from oracle_util import lcg_bytes, md5_ref
qsmd5.lib().qsmd5_init(0)
for L in (1, 1024, 65536, 1 << 20):
    data = lcg_bytes(7, L)
    want = md5_ref(data, L)
    ts = []
    for i in range(30):
        t0 = time.perf_counter()
        d = qsmd5.hash_one((ctypes.addressof(data), L))
        ts.append(time.perf_counter() - t0)
        assert d == want
    ts = ts[5:]
    print("hash_one %8d B: median %.1f us, min %.1f us" % (L, statistics.median(ts) * 1e6, min(ts) * 1e6), flush=True)
