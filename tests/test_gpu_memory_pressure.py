"""A GPU short of memory ("Digest failure must not be silent. A GPU
error must fall back to CPU MD5 (same digest)").

qsfs shares the card with whatever else runs on the node.  Here another
tenant -- torch, in the same process -- holds all but ~256 MiB of HBM, and a
host batch of 64 x 10 MiB parts is routed to the GPU (one CPU thread priced:
the GPU is the faster estimate; whole-chunk staging, so the ring needs
regions of >= 512 MiB).  The runtime's staging ring cannot be allocated:
under auto routing the batch is re-hashed on the CPU with identical digests,
counted as a fallback, and the GPU is NOT marked lost (memory pressure is not
a dead context); forced onto the GPU the call fails loudly
with -ENOMEM.  Once the memory is back, the next batch runs on the GPU again.
Runs in a child process so the hog and the runtime state die with it."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

SCRIPT = r"""
import ctypes, errno, json, sys
import torch
import qsmd5
from oracle_util import lcg_bytes, md5_many
MiB = 1 << 20
out = {}
assert torch.cuda.is_available()
torch.cuda.set_device(0)
assert qsmd5.lib().qsmd5_init(0) == 0
bufs = [lcg_bytes(900 + i, 10 * MiB) for i in range(64)]
chunks = [(ctypes.addressof(b), 10 * MiB) for b in bufs]
want = md5_many(chunks)
out["route"] = qsmd5.route([10 * MiB] * 64)
# the other tenant: all but ~256 MiB of what is free
free, total = torch.cuda.mem_get_info()
hog, size = None, free - 256 * MiB
while hog is None and size > 0:
    try:
        hog = torch.empty(size, dtype=torch.uint8, device="cuda")
    except RuntimeError:
        size -= 1024 * MiB
out["hog_gib"] = round(size / 2**30, 1)
out["free_after_hog_mib"] = torch.cuda.mem_get_info()[0] // MiB
s0 = qsmd5.stats()
got = qsmd5.hash_batch(chunks)
out["auto_digests_ok"] = got == want
out["auto_backend"] = qsmd5.last_backend()
s1 = qsmd5.stats()
out["fallbacks"] = s1["fallbacks"] - s0["fallbacks"]
out["gpu_lost"] = s1["gpu_lost"]
try:
    qsmd5.hash_batch(chunks, flags=qsmd5.FLAG_GPU_ONLY)
    out["forced_rc"] = 0
except qsmd5.Md5Error as e:
    out["forced_rc"] = e.code
del hog
torch.cuda.empty_cache()
out["free_after_release_mib"] = torch.cuda.mem_get_info()[0] // MiB
s2 = qsmd5.stats()
got = qsmd5.hash_batch(chunks)
out["after_digests_ok"] = got == want
out["after_backend"] = qsmd5.last_backend()
out["after_fallbacks"] = qsmd5.stats()["fallbacks"] - s2["fallbacks"]
out["after_route"] = qsmd5.route([10 * MiB] * 64)
out["last_error"] = qsmd5.lib().qsmd5_last_error().decode() if hasattr(qsmd5.lib().qsmd5_last_error(), "decode") else str(qsmd5.lib().qsmd5_last_error())
out["rates"] = qsmd5.rates() if hasattr(qsmd5, "rates") else None
print(json.dumps(out))
"""


def test_gpu_out_of_memory_falls_back_to_the_cpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    # whole-chunk staging (QSMD5_COLUMN_BYTES=0): the ring then needs >= 512 MiB
    # regions, which cannot fit in the ~256 MiB the hog leaves
    env = dict(os.environ, QSMD5_BACKEND="auto", QSMD5_CPU_THREADS="1", QSMD5_COLUMN_BYTES="0",
               QSMD5_ROUTE_LANES="0",  # the scalar model: the batch prices to the GPU
               PYTHONPATH=os.pathsep.join([os.path.join(ROOT, "qsfs-fuse_amd"), os.path.join(ROOT, "tests")]))
    env.pop("QSMD5_INJECT_GPU_FAULT", None)
    out = subprocess.run([sys.executable, "-c", SCRIPT], env=env, capture_output=True, text=True,
                         timeout=240)
    assert out.returncode == 0, out.stdout + out.stderr[-3000:]
    r = json.loads(out.stdout.strip().splitlines()[-1])
    print(r)
    import qsmd5
    assert r["route"] == qsmd5.BACKEND_GPU, r
    assert r["free_after_hog_mib"] < 512, r  # the ring for 640 MiB of parts cannot fit
    assert r["auto_digests_ok"] and r["auto_backend"] == qsmd5.BACKEND_CPU, r
    assert r["fallbacks"] == 1 and r["gpu_lost"] == 0, r
    assert r["forced_rc"] == -12, r  # -ENOMEM, loud
    assert r["after_digests_ok"] and r["after_backend"] == qsmd5.BACKEND_GPU, r


def test_a_stale_hip_error_on_the_thread_does_not_fail_a_launch():
    """The launchers return hipGetLastError() after a launch, which reports the
    last failure of ANY HIP call on the thread.  A caller whose own earlier HIP
    call failed (here an impossible hipMalloc through the same HIP runtime the
    library uses) must still get its batch hashed on the GPU, not a bogus
    launch failure (the memory-pressure test above first showed it: after an
    out-of-memory fallback, every later GPU batch on that thread failed)."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ctypes
    import qsmd5
    from oracle_util import lcg_bytes, md5_many
    assert qsmd5.lib().qsmd5_init(0) == 0
    # every HIP runtime mapped in THIS process (with torch imported first,
    # libqsmd5.so's soname resolves to torch's bundled copy): each is left
    # with a stale error on this thread
    hip_paths = sorted({ln.split()[-1] for ln in open("/proc/self/maps")
                        if ln.split() and "libamdhip64.so" in ln.split()[-1]})
    assert hip_paths, "no HIP runtime mapped"
    for path in hip_paths:
        hip = ctypes.CDLL(path)
        p = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 60)) != 0
    bufs = [lcg_bytes(1300 + i, (1 << 20) + 7 * i) for i in range(8)]
    chunks = [(ctypes.addressof(b), len(b)) for b in bufs]
    assert qsmd5.hash_batch(chunks, flags=qsmd5.FLAG_GPU_ONLY) == md5_many(chunks)
    assert qsmd5.last_backend() == qsmd5.BACKEND_GPU
