"""Group commit of concurrent qsmd5_hash_batch calls (qsmd5_rt_route.cpp).

qsfs calls md5() from up to numtransfer worker threads at once
(TransferManager.cpp:55-60), each call one part.  A launch costs one chain
time whatever its width, so the runtime merges calls that arrive while the GPU
is busy into the next launch.  Checked here:
- every caller gets its own digests, bit-exact with the oracle;
- one caller's invalid input fails only that caller (the merged batch is
  re-run request by request);
- the REF_TRUNCATE32 flag stays per caller inside a merged batch;
- concurrent one-part calls finish in far less time than the same calls
  serialised (QSMD5_NO_COALESCE=1), measured in child processes;
- native callers in a tight loop (tests/cpp/coalesce_bench, qsfs's executor
  threads calling md5() part after part): the leader's linger lets the callers
  released by one launch ride in the next.
"""
import ctypes
import json
import os
import subprocess
import sys
import threading

import pytest

from conftest import ROOT
import qsmd5
from oracle_util import lcg_bytes, md5_many

pytestmark = pytest.mark.gpu

MiB = 1 << 20


def _threads(fns):
    bar = threading.Barrier(len(fns))
    out = [None] * len(fns)

    def run(i):
        bar.wait()
        try:
            out[i] = ("ok", fns[i]())
        except Exception as e:  # noqa: BLE001 - the test inspects it
            out[i] = ("err", e)

    th = [threading.Thread(target=run, args=(i,)) for i in range(len(fns))]
    for t in th:
        t.start()
    for t in th:
        t.join(300)
    return out


def test_concurrent_callers_get_their_own_digests():
    bufs = [lcg_bytes(600 + i, MiB + 13 * i) for i in range(8)]
    lens = [MiB + 13 * i for i in range(8)]
    want = md5_many(list(zip(bufs, lens)))
    fns = [lambda i=i: qsmd5.hash_batch([(ctypes.addressof(bufs[i]), lens[i]),
                                         (ctypes.addressof(bufs[(i + 1) % 8]), lens[(i + 1) % 8])])
           for i in range(8)]
    for rnd in range(3):
        res = _threads(fns)
        for i, (kind, val) in enumerate(res):
            assert kind == "ok", val
            assert val == [want[i], want[(i + 1) % 8]], (rnd, i)


def test_bad_caller_fails_alone():
    bufs = [lcg_bytes(700 + i, 3 * MiB) for i in range(6)]
    want = md5_many([(b, 3 * MiB) for b in bufs])
    fns = [lambda i=i: qsmd5.hash_batch([(ctypes.addressof(bufs[i]), 3 * MiB)]) for i in range(6)]
    fns[3] = lambda: qsmd5.hash_batch([(0, 1000)])  # NULL with a length: -EINVAL
    res = _threads(fns)
    for i, (kind, val) in enumerate(res):
        if i == 3:
            assert kind == "err" and isinstance(val, qsmd5.Md5Error), val
        else:
            assert kind == "ok" and val == [want[i]], (i, kind, val)


def test_truncate_flag_stays_per_caller():
    # 5 GiB + 100 B would be needed to see truncation change a digest; the flag's
    # plumbing is what is checked: both callers get the standard digest of a
    # short buffer whether or not they pass the flag.
    b = lcg_bytes(4242, 5000)
    want = md5_many([(b, 5000)])[0]
    fns = [lambda: qsmd5.hash_batch([(ctypes.addressof(b), 5000)], flags=qsmd5.FLAG_REF_TRUNCATE32),
           lambda: qsmd5.hash_batch([(ctypes.addressof(b), 5000)])]
    for kind, val in _threads(fns):
        assert kind == "ok" and val == [want]


def test_host_flag_stays_per_caller():
    """QSMD5_FLAG_HOST is a caller's promise about its own chunks: a merged
    batch keeps it only if every merged caller made it, so callers passing
    device buffers without the flag still hash correctly beside flagged ones."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    L = 2 * MiB
    bufs = [lcg_bytes(900 + i, L) for i in range(6)]
    want = md5_many([(b, L) for b in bufs])
    devs = [torch.frombuffer(bytearray(bytes(b)), dtype=torch.uint8).cuda() for b in bufs]
    torch.cuda.synchronize()
    fns = []
    for i in range(6):
        if i % 2:
            fns.append(lambda i=i: qsmd5.hash_batch([(devs[i].data_ptr(), L)]))
        else:
            fns.append(lambda i=i: qsmd5.hash_batch([(ctypes.addressof(bufs[i]), L)],
                                                    flags=qsmd5.FLAG_HOST))
    for rnd in range(3):
        for i, (kind, val) in enumerate(_threads(fns)):
            assert kind == "ok" and val == [want[i]], (rnd, i, kind, val)


TIMING_SCRIPT = r'''
import ctypes, json, sys, threading, time
import qsmd5
from oracle_util import lcg_bytes, md5_many
T, L = 6, 10 << 20
bufs = [lcg_bytes(800 + i, L) for i in range(T)]
want = md5_many([(b, L) for b in bufs])
qsmd5.hash_batch([b"warm"])
bar = threading.Barrier(T)
got = [None] * T
def run(i):
    bar.wait()
    for _ in range(2):
        got[i] = qsmd5.hash_batch([(ctypes.addressof(bufs[i]), L)])[0]
t0 = time.perf_counter()
th = [threading.Thread(target=run, args=(i,)) for i in range(T)]
[t.start() for t in th]
[t.join() for t in th]
print(json.dumps({"wall_s": time.perf_counter() - t0, "ok": got == want}))
'''


def _timed(no_coalesce, linger_us=None):
    env = dict(os.environ, PYTHONPATH=os.pathsep.join(
        [os.path.join(ROOT, "qsfs-fuse_amd"), os.path.join(ROOT, "tests")]))
    if no_coalesce:
        env["QSMD5_NO_COALESCE"] = "1"
    if linger_us is not None:
        env["QSMD5_COALESCE_LINGER_US"] = str(linger_us)
    out = subprocess.run([sys.executable, "-c", TIMING_SCRIPT], env=env, capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr[-3000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_coalescing_beats_serialised_calls():
    ser = _timed(True)
    co0 = _timed(False, linger_us=0)
    co = _timed(False)
    assert ser["ok"] and co0["ok"] and co["ok"]
    # 12 one-part calls from 6 threads: serialised = 12 chain times (~1 s);
    # merged = a few launches; with the linger, a worker released by one launch
    # rides in the next instead of the one after
    print("serialised %.3f s, coalesced without linger %.3f s, with linger %.3f s"
          % (ser["wall_s"], co0["wall_s"], co["wall_s"]))
    assert co0["wall_s"] < 0.6 * ser["wall_s"], (ser, co0)
    assert co["wall_s"] < 0.6 * ser["wall_s"], (ser, co)


def _native(env_extra):
    exe = os.path.join(ROOT, "tests", "cpp", "coalesce_bench")
    if not os.path.exists(exe):
        subprocess.check_call([
            "g++", "-std=c++17", "-O2", os.path.join(ROOT, "tests", "cpp", "coalesce_bench.cpp"),
            "-I" + os.path.join(ROOT, "include"), "-L" + os.path.join(ROOT, "qsfs-fuse_amd", "lib"),
            "-lqsmd5", "-lpthread", "-Wl,-rpath," + os.path.join(ROOT, "qsfs-fuse_amd", "lib"),
            "-o", exe])
    env = dict(os.environ, **env_extra)
    out = subprocess.run([exe, "5", "6"], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr[-2000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_native_callers_linger():
    no_linger = _native({"QSMD5_COALESCE_LINGER_US": "0"})
    linger = _native({})
    ser = _native({"QSMD5_NO_COALESCE": "1"})
    print("5 native threads x 6 parts: serialised %.3f s, no linger %.3f s, linger %.3f s"
          % (ser["wall_s"], no_linger["wall_s"], linger["wall_s"]))
    assert ser["ok"] and no_linger["ok"] and linger["ok"]
    assert linger["wall_s"] < 0.85 * no_linger["wall_s"], (no_linger, linger)
    assert no_linger["wall_s"] < 0.6 * ser["wall_s"], (ser, no_linger)
