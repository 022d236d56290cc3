"""BASELINE config 5 on the MI355X: one 100 GB object as 10 000 x 10 MiB parts.

The reference hashes such an object part by part, serially, in
QSTransferManager::DoMultiPartUpload (/root/reference/src/client/
QSTransferManager.cpp:602-673) through File::Flush (src/data/File.cpp:639-644).
Here bench_config5.py shards the parts over ranks (contiguous ranges,
qsmd5.parallel.shard_range), hashes each rank's range in one batch on the
gfx950 kernels, all-gathers the 16-byte digests and checks every one of them
against tests/golden/batch_10MiB.json (produced by the reference's own
MD5.cpp).  Each case is launched by torch.distributed.run in fresh child
processes: the pytest process never hands its GPU state to a rank.

  device, RCCL, 1 rank      10 000 parts (97.7 GiB) resident in HBM, ONE launch
  host,   RCCL, 1 rank      >= 2 000 parts in pinned host memory (sized to the
                            box's free memory), qsmd5_hash_batch_ex(FLAG_HOST):
                            H2D columns + hash + D2H, digest all-gather inside
  device, gloo, 2 ranks     both ranks share the one card (5 000 parts each):
                            the multi-rank flow and parity, not a scaling number
"""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

PY = sys.executable
PARTS = 10000
L = 10 << 20


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _host_parts():
    """Parts for the host leg: at least 2 000 (19.5 GiB pinned), at most 4 000
    (39 GiB: page-locking takes a while), within half of the memory this box
    has free."""
    avail = None
    try:
        for line in open("/proc/meminfo"):
            if line.startswith("MemAvailable:"):
                avail = int(line.split()[1]) * 1024
    except OSError:
        pass
    try:
        cap = open("/sys/fs/cgroup/memory.max").read().strip()
        if cap != "max":
            avail = min(avail or int(cap), int(cap))
    except (OSError, ValueError):
        pass
    if avail is None:
        return 2000
    return max(2000, min(4000, int(avail * 0.5) // L // 1000 * 1000))


def _run(nproc, extra, timeout=900):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", QSMD5_BACKEND="gpu")
    cmd = [PY, "-u", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % nproc,
           "--master-addr=127.0.0.1", "--master-port=%d" % _free_port(),
           os.path.join(ROOT, "bench_config5.py"), "--reps", "2"] + extra
    # the ranks' progress lines go straight to stderr (seen live under pytest -s)
    out = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, text=True, timeout=timeout, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-3000:]
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    print("\n".join(json.dumps(x) for x in lines))
    return lines


def _check(r, n, world, resident, collective):
    assert r["config"] == 5 and r["resident"] == resident and r["n_gpus"] == world
    assert r["parity"] == "ok: %d/%d == reference golden" % (n, n)
    assert sum(r["parts_per_rank"]) == n and len(r["parts_per_rank"]) == world
    assert r["collective"].startswith(collective)
    st = r["backend_stats"]
    assert st["cpu_batches"] == 0 and st["gpu_lost"] == 0, st  # the gfx950 kernels hashed it


def test_config5_device_resident_10000_parts_one_launch_rccl():
    (r,) = _run(1, ["--resident", "device", "--parts", str(PARTS)])
    _check(r, PARTS, 1, "device", "RCCL")
    # one launch of 10 000 chains takes about one 10 MiB chain time (~0.08 s)
    assert r["seconds"] < 1.0, r


def test_config5_host_resident_pinned_rccl():
    n = _host_parts()
    (r,) = _run(1, ["--resident", "host", "--parts", str(n)])
    _check(r, n, 1, "host", "RCCL")
    assert r["backend_stats"]["gpu_batches"] >= 1


def test_config5_two_ranks_share_one_gpu_gloo():
    (r,) = _run(2, ["--resident", "device", "--parts", str(PARTS), "--dist-backend", "gloo"])
    _check(r, PARTS, 2, "device", "gloo")
    assert r["parts_per_rank"] == [PARTS // 2, PARTS // 2]
