"""The DoMultiPartUpload flow with the batch pre-hash on the MI355X
(QSTransferManager.cpp:602-673).

tests/cpp/multipart_harness builds a file held in many separately allocated
pages, slices it as PrepareUpload does, gathers each wave of parts into pool
buffers (File::ReadNoLoad, File.cpp:308-375), hashes the wave with ONE
qsmd5_hash_batch_ex(QSMD5_FLAG_HOST) through qsfs-fuse_amd/host/qsfs_multipart.hpp
and hands each part's hex digest on.  Every digest is checked against the
reference-produced golden table.
"""
import json
import os

import pytest

from conftest import GOLDEN, ROOT
from multipart_util import run

torch = pytest.importorskip("torch")
MiB = 1 << 20


@pytest.fixture(scope="module")
def gold():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return json.load(open(os.path.join(GOLDEN, "batch_10MiB.json")))["md5"]


@pytest.mark.gpu
@pytest.mark.parametrize("slab", [False, True], ids=["buffer_each", "one_slab"])
@pytest.mark.parametrize("pinned", [False, True], ids=["pageable_pool", "pinned_pool"])
def test_whole_file_wave_on_the_gpu(gold, pinned, slab):
    """A pool as large as the file: one wave, one GPU batch of 512 parts, from
    pool buffers allocated one by one (as ResourceManager does) or carved from
    one slab (qsmd5::BufferSlab), pageable or pinned."""
    args = ["--aligned", "--size=%d" % (512 * 10 * MiB), "--pool=512", "--repeat=3", "--no-pipeline"]
    args += (["--pinned"] if pinned else []) + (["--slab"] if slab else [])
    r = run(args, "gpu")
    assert r["parts"] == 512 and r["waves"] == 1 and r["gpu_waves"] == 1
    assert r["md5"] == gold[:512]
    first, warm = r["hash_s_runs"][0], min(r["hash_s_runs"][1:])
    print("512 x 10 MiB paged file, %s pool, %s: gather %.3f s; hash first pass %.3f s "
          "(%.1f GiB/s), reused pool %.3f s (%.1f GiB/s)"
          % ("pinned" if pinned else "pageable", "one slab" if slab else "buffer each",
             r["gather_s"], first, 5.0 / first, warm, 5.0 / warm))


@pytest.mark.gpu
@pytest.mark.cpu_backend
def test_default_pool_routes_waves_by_size(gold):
    """auto: qsfs's default pool (5 x 10 MiB buffers, 50 MiB heap) gives waves
    below the GPU break-even, hashed on the CPU; a 64-buffer pool's waves go to
    the gfx950 kernels under the scalar model (QSMD5_ROUTE_LANES=0) and to the
    CPU's AVX-512 lanes, ~3x faster on this host, under the default lane
    pricing.  Same golden digests every way."""
    small = run(["--aligned", "--size=%d" % (64 * 10 * MiB), "--pool=5", "--no-pipeline"], "auto")
    assert small["waves"] == 13 and small["cpu_waves"] == 13 and small["gpu_waves"] == 0
    big = run(["--aligned", "--size=%d" % (128 * 10 * MiB), "--pool=64", "--no-pipeline"], "auto",
              extra_env={"QSMD5_ROUTE_LANES": "0"})
    assert big["waves"] == 2 and big["gpu_waves"] == 2
    lanes = run(["--aligned", "--size=%d" % (128 * 10 * MiB), "--pool=64", "--no-pipeline"], "auto")
    if "avx512f" in open("/proc/cpuinfo").read():
        assert lanes["cpu_waves"] == 2, lanes
    assert lanes["md5"] == gold[:128]
    assert small["md5"] == gold[:64] and big["md5"] == gold[:128]
    print("64 parts, pool 5 (CPU waves): hash %.3f s; 128 parts, pool 64 (GPU waves): hash %.3f s"
          % (small["hash_s"], big["hash_s"]))


@pytest.mark.gpu
def test_registered_pageable_pool(gold):
    """qsfs's own pageable buffers, registered once (qsmd5_register_host, as
    at daemon start-up): no first-touch page locking, and the separate buffers'
    rows go through the gather kernel."""
    r = run(["--aligned", "--size=%d" % (512 * 10 * MiB), "--pool=512", "--register", "--repeat=2",
             "--no-pipeline"], "gpu")
    assert r["registered"] and r["gpu_waves"] == 1
    assert r["md5"] == gold[:512]
    first, warm = r["hash_s_runs"]
    print("512 x 10 MiB, 512 registered pageable buffers: register %.3f s once; hash first pass "
          "%.3f s (%.1f GiB/s), reused %.3f s (%.1f GiB/s)"
          % (r["register_s"], first, 5.0 / first, warm, 5.0 / warm))


@pytest.mark.gpu
@pytest.mark.parametrize("pool_kind", ["pinned", "register"])
def test_pool_refilled_between_waves(gold, pool_kind):
    """qsfs refills the same transfer buffers for every wave.  A pool of 64
    buffers for 128 parts: each buffer is filled with part k, hashed through
    the gather kernel (it reads pinned / registered host memory over PCIe via
    device pointers), then refilled with part k + 64 and read again.  Stale
    host data served from a GPU-side cache would repeat wave 1's digests in
    wave 2; every digest must be part k's own."""
    flag = "--pinned" if pool_kind == "pinned" else "--register"
    r = run(["--aligned", "--size=%d" % (128 * 10 * MiB), "--pool=64", flag, "--repeat=2", "--no-pipeline"], "gpu",
            extra_env={"QSMD5_TRACE": "1"})
    assert r["parts"] == 128 and r["waves"] == 2 and r["gpu_waves"] == 2
    assert r["md5"] == gold[:128]
    assert len(set(r["md5"])) == 128  # no wave-2 digest repeats a wave-1 one
    gathered = [int(ln.split(" regions, ")[1].split()[0]) for ln in r["_stderr"].splitlines()
                if ln.startswith("qsmd5 trace:") and "gathered rows" in ln]
    assert len(gathered) == 4 and min(gathered) >= 64, gathered  # 2 passes x 2 waves, every row


@pytest.mark.gpu
@pytest.mark.parametrize("wait", ["auto", "spin"])
def test_gpu_waves_leave_the_host_cores_free(gold, wait):
    """A GPU wave is one ~85 ms chain; the caller used to spin through it and
    the column pipeline's stream waits kept a HIP thread polling too (~2 host
    cores per wave, profiles/r04_route_sweep_before_hostorder.jsonl).  With the
    host-ordered staging and sleep-poll waits (QSMD5_WAIT=auto), 8 waves of 8
    pinned 10 MiB parts cost the host little beyond the harness's own gather;
    QSMD5_WAIT=spin still hashes correctly (and spins the caller)."""
    r = run(["--aligned", "--size=%d" % (64 * 10 * MiB), "--pool=8", "--pinned", "--slab",
             "--no-pipeline", "--repeat=2"], "gpu", extra_env={"QSMD5_WAIT": wait})
    assert r["md5"] == gold[:64] and r["gpu_waves"] == 8
    hashing_cpu = r["cpu_s_runs"][-1] - r["gather_s"]
    print("QSMD5_WAIT=%s: wall %.3f s, host CPU beyond the gather %.3f s, busy threads %s"
          % (wait, r["wall_s_runs"][-1], hashing_cpu, r["busy_threads"]))
    if wait == "auto":
        assert hashing_cpu < 0.15 * r["wall_s_runs"][-1], r
    else:
        assert hashing_cpu > 0.5 * r["hash_s"], r  # the spin is real: the test would see a regression


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [[], ["--async=2"], ["--cancel-after=9"]], ids=["sync", "async", "cancel"])
def test_concurrent_files_gpu_waves(gold, mode):
    """Four files flushed at once through one pinned 32-buffer slab pool, every
    wave forced onto the GPU, the next wave of each file prepared on its helper
    thread while its current one uploads: waves of different files meet in the
    runtime's group commit and share launches.  No deadlock, every digest
    golden (cancelled: the first 9 of each file), every buffer back."""
    r = run(["--aligned", "--size=%d" % (32 * 10 * MiB), "--pool=32", "--pinned", "--slab", "--files=4",
             "--upload-ms=2", "--deadlock-s=60"] + mode, "gpu")
    want = 9 if "--cancel-after=9" in mode else 32
    assert r["deadlock"] is False and r["error"] == "", r
    assert r["pool_free_after"] == 32 and r["gpu_waves"] >= 4 and r["cpu_waves"] == 0, r
    for m in r["md5_files"]:
        assert m[:want] == gold[:want] and not any(m[want:]), m


@pytest.mark.gpu
def test_reference_loop_beside_the_staged_binding():
    """the flush loop the binding replaces, timed beside it
    on the same file -- QSTransferManager::DoMultiPartUpload with -m as the
    reference runs it (Acquire, ReadNoLoad, the reference's own
    md5(shared_ptr<iostream>) from oracle/_ref, upload; serial on the flushing
    thread) against qsmd5::upload_parts_staged, 128 x 10 MiB at -n 5, uploads
    that return at once.  Both golden; the binding is faster."""
    if not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libref_md5.so")):
        pytest.skip("oracle/_ref not built")
    gold = json.load(open(os.path.join(GOLDEN, "batch_10MiB.json")))["md5"]
    base = ["--aligned", "--size=%d" % (128 * 10 * MiB), "--pool=5"]
    ref = run(base + ["--reference-loop"], "auto", timeout=600)
    stg = run(base + ["--pinned", "--staged", "--repeat=2"], "gpu", timeout=600)
    assert ref["md5"] == gold[:128] and stg["md5"] == gold[:128]
    rw, sw = ref["seconds"], min(stg["wall_s_runs"])
    print("128 x 10 MiB, -n 5: reference loop %.3f s (md5 %.3f s, reads %.3f s, %.2f CPU-s); "
          "staged binding %.3f s (%.2f CPU-s): %.1fx" % (rw, ref["hash_s"], ref["loop_read_s"],
                                                        ref["cpu_s_runs"][0], sw, stg["cpu_s_runs"][-1], rw / sw))
    assert sw < rw
