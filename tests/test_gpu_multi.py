"""In-process multi-GPU sharding of the C-ABI (SURVEY.md §8b "multi-GPU
sharding is internal", §8e).

A qsfs daemon is one process, so the drop-in cannot use one process per GPU:
`QSMD5_DEVICES` binds several GPUs inside libqsmd5 and `qsmd5_hash_batch`
splits a batch over them.  Host chunks go in contiguous, byte-balanced ranges
(`QSMD5_SHARD_BYTES` per extra GPU), device chunks run on the GPU that holds
them, one thread per GPU, and digests are scattered back by index.

The GPU box has one MI355X, so the shards run as two contexts on GPU 0
(`QSMD5_DEVICES=0,0`: separate streams, scratch and staging rings, one thread
each).  That exercises the split, the threads, the scatter and the error
paths.  Every digest is checked against the oracle.  Each case runs in a child
process: the runtime binds its GPUs once per process.
"""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

PY = sys.executable
BASE_ENV = dict(os.environ, PYTHONPATH=os.pathsep.join(
    [os.path.join(ROOT, "qsfs-fuse_amd"), os.path.join(ROOT, "tests")]))

SHARD_SCRIPT = r'''
import ctypes, sys
import torch
import qsmd5
from oracle_util import lcg_bytes, md5_many

MiB = 1 << 20
# host (pageable) chunks: 40 x ~1 MiB, ragged lengths, unaligned ends
lens = [MiB + 37 * i + (i % 5) for i in range(40)]
bufs = [lcg_bytes(900 + i, L) for i, L in enumerate(lens)]
want = md5_many([(b, L) for b, L in zip(bufs, lens)])
host = [(ctypes.addressof(b), L) for b, L in zip(bufs, lens)]
got = qsmd5.hash_batch(host)
assert got == want, "host shards differ from the oracle"

# pinned host chunks (the qsfs pool, SURVEY §8f row 2) inside one big buffer
n, L = 24, 3 * MiB + 11
p = qsmd5.alloc_pinned(n * (L + 5))
try:
    raw = (ctypes.c_uint8 * (n * (L + 5))).from_address(p)
    for i in range(n):
        ctypes.memmove(p + i * (L + 5), lcg_bytes(77 + i, L), L)
    pins = [(p + i * (L + 5), L) for i in range(n)]
    got = qsmd5.hash_batch(pins)
    assert got == md5_many([(p + i * (L + 5), L) for i in range(n)]), "pinned shards differ"
finally:
    qsmd5.free_pinned(p)

# mixed: device chunks on GPU 0 interleaved with host chunks, plus empties
dev = torch.empty(8 * 2 * MiB, dtype=torch.uint8, device="cuda:0")
qsmd5.synth_fill_lcg(dev.data_ptr(), 2 * MiB, 2 * MiB - 3, 4242, 8)
torch.cuda.synchronize()
dev_host = dev.cpu().numpy()
mixed, ref = [], []
for i in range(8):
    mixed.append((dev.data_ptr() + i * 2 * MiB, 2 * MiB - 3))
    ref.append((dev_host.ctypes.data + i * 2 * MiB, 2 * MiB - 3))
    mixed.append(host[i])
    ref.append(host[i])
mixed.append(b"")
ref.append((0, 0))
got = qsmd5.hash_batch(mixed)
assert got == md5_many(ref), "mixed shards differ"
print("shard-ok")
'''


def _run(script, **env):
    e = dict(BASE_ENV, **env)
    return subprocess.run([PY, "-c", script], env=e, capture_output=True, text=True, timeout=300)


@pytest.mark.parametrize("devices", ["0,0", "0,0,0,0"])
def test_contexts_shard_and_match_oracle(devices):
    """Two contexts, and four (the node's shard threads rehearsed on one
    card): every context takes a shard of some batch, each runs the
    host-ordered staging pipeline on its own streams, every digest matches."""
    out = _run(SHARD_SCRIPT, QSMD5_DEVICES=devices, QSMD5_SHARD_BYTES=str(8 << 20),
               QSMD5_TRACE="1")
    assert out.returncode == 0, out.stdout + out.stderr[-4000:]
    assert "shard-ok" in out.stdout
    # the split really happened: every context took chunks in some batch
    shards = [l for l in out.stderr.splitlines() if l.startswith("qsmd5 shard:")]
    for c in range(len(devices.split(","))):
        assert any("context %d (GPU 0) takes" % c in l and not l.endswith("takes 0 chunks")
                   for l in shards), "\n".join(shards)


def test_small_batch_stays_on_one_gpu():
    script = r'''
import qsmd5
assert qsmd5.md5("abc") == "900150983cd24fb0d6963f7d28e17f72"
assert qsmd5.hash_batch([b"x" * 1000, b""])[1].hex() == "d41d8cd98f00b204e9800998ecf8427e"
print("small-ok")
'''
    out = _run(script, QSMD5_DEVICES="0,0", QSMD5_TRACE="1")  # default 4 GiB per extra GPU
    assert out.returncode == 0, out.stdout + out.stderr[-4000:]
    shards = [l for l in out.stderr.splitlines() if l.startswith("qsmd5 shard:")]
    assert shards and all(l.endswith("takes 0 chunks") for l in shards if "context 1" in l)


def test_all_devices_on_one_gpu_box():
    script = r'''
import qsmd5
assert qsmd5.md5("message digest") == "f96b697d7cb7938d525a2f31aaf161d0"
print("all-ok")
'''
    out = _run(script, QSMD5_DEVICES="all")
    assert out.returncode == 0, out.stdout + out.stderr[-4000:]


@pytest.mark.parametrize("spec,errno_name", [("63", "ENODEV"), ("0,zz", "EINVAL"), ("", None)])
def test_bad_device_lists(spec, errno_name):
    script = r'''
import errno, sys
import qsmd5
rc = qsmd5.lib().qsmd5_init(0)
print("rc", rc)
want = sys.argv[1]
sys.exit(0 if (rc == 0 if want == "None" else rc == -getattr(errno, want)) else 1)
'''
    e = dict(BASE_ENV, QSMD5_DEVICES=spec)
    out = subprocess.run([PY, "-c", script, str(errno_name)], env=e, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr[-2000:]


def test_part_count_beyond_one_gpu_shards():
    """North star: shard "only when one file's part count exceeds a single
    GPU's batch".  40 000 small host parts (4 MB, far below QSMD5_SHARD_BYTES)
    exceed one GPU's 32 768 resident chains, so both contexts take a shard."""
    script = r'''
import ctypes
import qsmd5
from oracle_util import lcg_bytes, md5_many
n, L = 40000, 100
buf = lcg_bytes(31, n * L)
chunks = [(ctypes.addressof(buf) + i * L, L - (i % 3)) for i in range(n)]
assert qsmd5.hash_batch(chunks) == md5_many(chunks)
print("parts-ok")
'''
    out = _run(script, QSMD5_DEVICES="0,0", QSMD5_TRACE="1")
    assert out.returncode == 0, out.stdout + out.stderr[-4000:]
    assert "parts-ok" in out.stdout
    shards = [l for l in out.stderr.splitlines() if l.startswith("qsmd5 shard:")]
    assert any("context 1 (GPU 0) takes" in l and not l.endswith("takes 0 chunks") for l in shards), \
        "\n".join(shards)


def test_concurrent_read_jobs_spread_over_bound_gpus():
    """Pull-driven batches (qsmd5_hash_read) from four threads at once, with
    two bound contexts (QSMD5_DEVICES=0,0) and one read slot each: the jobs
    go to the context with the fewest in flight, so both take some, and every
    digest equals the oracle's."""
    script = r'''
import ctypes, threading
import qsmd5
from oracle_util import lcg_bytes, md5_many
MiB = 1 << 20
jobs = []
for j in range(4):
    lens = [MiB + 4099 * i for i in range(24)]
    bufs = [lcg_bytes(3000 + 100 * j + i, L) for i, L in enumerate(lens)]
    jobs.append({"lens": lens, "bufs": bufs})
def reader(bufs):
    def read(chunk, off, n, dst):
        ctypes.memmove(dst, ctypes.addressof(bufs[chunk]) + off, n)
        return n
    return read
def work(job):
    job["got"] = qsmd5.hash_read(job["lens"], reader(job["bufs"]), staging_bytes=4 * MiB,
                                 flags=qsmd5.FLAG_GPU_ONLY)
th = [threading.Thread(target=work, args=(job,)) for job in jobs]
for t in th: t.start()
for t in th: t.join()
for job in jobs:
    assert job["got"] == md5_many([(b, L) for b, L in zip(job["bufs"], job["lens"])])
print("read-spread-ok")
'''
    out = _run(script, QSMD5_DEVICES="0,0", QSMD5_TRACE="1", QSMD5_READ_SLOTS="1")
    assert out.returncode == 0 and "read-spread-ok" in out.stdout, out.stdout + out.stderr[-4000:]
    ctx = [l.split("context ")[1].split()[0] for l in out.stderr.splitlines() if l.startswith("qsmd5 read: job")]
    assert len(ctx) == 4 and set(ctx) == {"0", "1"}, ctx
