"""The DoMultiPartUpload flow with the batch pre-hash on
the CPU backend: tests/cpp/multipart_harness gathers parts from a paged file
into pool buffers (File::ReadNoLoad), hashes each pool-size wave with one
qsmd5_hash_batch_ex call, and hands the hex digests on per part.  Here the
library's CPU backend hashes (QSMD5_BACKEND=cpu); tests/test_gpu_multipart.py
runs the same flow on the MI355X.  Digests are checked against the
reference-produced golden table, or the oracle for unaligned files."""
import ctypes
import json
import os

import pytest

from conftest import GOLDEN, ROOT
import subprocess

from multipart_util import build_tsan, run, run_raw
from oracle_util import lcg_bytes, md5_many

MiB = 1 << 20


def test_aligned_parts_match_golden():
    gold = json.load(open(os.path.join(GOLDEN, "batch_10MiB.json")))["md5"]
    r = run(["--aligned", "--size=%d" % (12 * 10 * MiB), "--pool=5", "--no-pipeline"], "cpu")
    assert r["parts"] == 12 and r["waves"] == 3 and r["cpu_waves"] == 3
    assert r["md5"] == gold[:12]


def test_prepare_upload_slicing_and_ragged_tail():
    """25 MiB + 3 B and 21 MiB files: PrepareUpload's [10, 10, 5] and averaged
    [10, 5.5, 5.5] MiB parts (QSTransferManager.cpp:517-542), gathered from
    pages that straddle part boundaries."""
    for size, seed in ((25 * MiB + 3, 31), (21 * MiB, 32), (100 * MiB + 12345, 33)):
        r = run(["--size=%d" % size, "--seed=%d" % seed, "--pool=2"], "cpu")
        data = lcg_bytes(seed, size)
        base, off, want = ctypes.addressof(data), 0, []
        for L in r["part_sizes"]:
            want.append((base + off, L))
            off += L
        assert off == size
        assert r["md5"] == [d.hex() for d in md5_many(want)], size


@pytest.mark.parametrize("mode", ["sync", "sync_no_pipeline", "async_executor"])
def test_concurrent_files_share_a_blocking_pool(mode):
    """four files of 12 parts flush at once from four
    threads through ONE blocking 5-buffer pool (ResourceManager::Acquire
    blocks, ResourceManager.cpp:53-67), with a simulated 2 ms upload per part:
    on the caller's thread (the reference's sync path), or on a 3-thread
    executor whose completion handler releases the buffer (its async path,
    QSTransferManager.cpp:654-659).  A wave only ever blocks for its first
    buffer while holding none, so no deadlock (the harness's watchdog would
    exit 3), and every part of every file matches the golden table."""
    gold = json.load(open(os.path.join(GOLDEN, "batch_10MiB.json")))["md5"]
    args = ["--aligned", "--size=%d" % (12 * 10 * MiB), "--pool=5", "--files=4", "--upload-ms=2",
            "--deadlock-s=10"]
    if mode == "sync_no_pipeline":
        args.append("--no-pipeline")
    if mode == "async_executor":
        args.append("--async=3")
    r = run(args, "cpu", timeout=120)
    assert r["deadlock"] is False and r["files"] == 4 and r["parts"] == 12
    assert r["widest_wave"] <= 5 and r["waves"] >= 4 * 3
    for f, got in enumerate(r["md5_files"]):
        assert got == gold[:12], f


def test_hold_and_wait_flow_deadlocks():
    """The negative control for the test above: the flow round 3's
    INTEGRATION.md sketched -- blocking Acquire per part of a 4-part wave
    before hashing it -- under the same four files and 5-buffer pool holds
    buffers while it waits for more, and the harness's watchdog finds every
    uploader blocked with no buffer free (exit 3)."""
    out = run_raw(["--aligned", "--size=%d" % (12 * 10 * MiB), "--pool=5", "--files=4",
                   "--naive-wave=4", "--deadlock-s=3"], "cpu", timeout=120)
    assert out.returncode == 3, out.stdout + out.stderr
    r = json.loads(out.stdout.splitlines()[-1])
    assert r["deadlock"] is True and r["free"] == 0 and r["waiting"] >= 2


def test_pipeline_hides_hashing_behind_upload():
    """with the pipeline, the next wave is gathered and
    hashed on a helper thread while this thread uploads (20 ms per part
    simulated), so the uploader hardly waits for hashing (wait_s); without it
    every wave's gather + hash sits between uploads.  Same golden digests."""
    gold = json.load(open(os.path.join(GOLDEN, "batch_10MiB.json")))["md5"]
    base = ["--aligned", "--size=%d" % (24 * 10 * MiB), "--pool=8", "--upload-ms=20"]
    serial = run(base + ["--no-pipeline"], "cpu", timeout=120)
    piped = run(base, "cpu", timeout=120)
    assert serial["md5"] == gold[:24] and piped["md5"] == gold[:24]
    # the first wave is hashed before any upload can start, in both
    first = piped["seconds"] - piped["upload_s"] - piped["wait_s"]
    print("serial: wall %.3f s, upload %.3f s, waiting for hashes %.3f s; pipelined: wall %.3f s, "
          "upload %.3f s, waiting %.3f s (first wave %.3f s)"
          % (serial["seconds"], serial["upload_s"], serial["wait_s"], piped["seconds"],
             piped["upload_s"], piped["wait_s"], first))
    assert piped["wait_s"] < 0.3 * serial["wait_s"], (piped, serial)
    assert piped["seconds"] < serial["seconds"]


@pytest.mark.parametrize("mode", [[], ["--async=3"], ["--no-pipeline"], ["--max-wave=2"],
                                  ["--cancel-after=5"], ["--cancel-after=5", "--async=3"],
                                  ["--check-throws-after=5", "--async=3"]],
                         ids=["sync", "async", "no_pipeline", "max_wave_2", "cancel", "cancel_async",
                              "check_throws_async"])
def test_concurrent_files_under_tsan(mode):
    """The drop-in header's threads -- the pipeline's helper thread preparing
    the next wave, the shared pool, the executor's completion handler
    releasing buffers -- under ThreadSanitizer, four files at once through
    one 5-buffer pool: no report, every digest golden."""
    exe = build_tsan()
    gold = json.load(open(os.path.join(GOLDEN, "batch_10MiB.json")))["md5"]
    # the HIP/HSA suppressions: on a GPU box the harness's qsmd5_init starts the
    # uninstrumented HIP runtime even with QSMD5_BACKEND=cpu
    env = dict(os.environ, QSMD5_BACKEND="cpu", TSAN_OPTIONS="halt_on_error=0:exitcode=66:suppressions="
               + os.path.join(ROOT, "tests", "cpp", "tsan_hip.supp"))
    out = subprocess.run(["setarch", "x86_64", "-R", exe, "--aligned", "--size=%d" % (12 * 10 * MiB),
                          "--pool=5", "--files=4", "--upload-ms=2", "--deadlock-s=20"] + mode,
                         env=env, capture_output=True, text=True, timeout=300)
    assert "WARNING: ThreadSanitizer" not in out.stderr, out.stderr[-8000:]
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads(out.stdout)
    want = 5 if ("--cancel-after=5" in mode or "--check-throws-after=5" in mode) else 12
    assert r["deadlock"] is False and r["pool_free_after"] == 5, r
    assert all(m[:want] == gold[:want] and not any(m[want:]) for m in r["md5_files"]), r["md5_files"]


@pytest.mark.parametrize("fault,mode,want_uploaded", [
    ("--short-read-part=9", [], None),
    ("--short-read-part=9", ["--no-pipeline"], 8),
    ("--short-read-part=1", [], 0),
    ("--fail-upload-part=7", [], 6),
    ("--fail-upload-part=7", ["--async=2"], 6),
    ("--short-read-part=20", ["--async=3"], None),
    ("--check-throws-after=5", [], 5),            # the cancel check itself throws mid-wave
    ("--check-throws-after=5", ["--async=2"], 5),
])
def test_failures_stop_the_upload_and_return_every_buffer(fault, mode, want_uploaded):
    """A short read (File::ReadNoLoad found a hole) or a failed upload stops
    the file's upload, as the reference does (QSTransferManager.cpp:611-643):
    no part at or after the failing one is handed on, the parts before the
    failing wave keep their golden digests, and every buffer -- the wave's,
    the one in upload, the one the helper thread was preparing -- is back in
    the shared pool afterwards (pool_free_after == pool)."""
    gold = json.load(open(os.path.join(GOLDEN, "batch_10MiB.json")))["md5"]
    args = ["--aligned", "--size=%d" % (20 * 10 * MiB), "--pool=4", "--upload-ms=1", fault] + mode
    out = run_raw(args, "cpu", timeout=120)
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads(out.stdout)
    bad = int(fault.split("=")[1])  # the first part that must not go out (1-based)
    if fault.startswith("--check-throws-after="):
        bad += 1  # N parts went out, the check before part N + 1 threw
    assert r["error"], r
    assert r["pool_free_after"] == 4, r
    done = [i for i, h in enumerate(r["md5"]) if h]
    assert all(i < bad - 1 for i in done), done           # nothing at or after the failing part
    assert done == list(range(len(done)))                 # a prefix of the file, in order
    assert [r["md5"][i] for i in done] == gold[:len(done)]
    if want_uploaded is not None:
        assert r["uploaded"] == want_uploaded, r


@pytest.mark.parametrize("after,mode", [(0, []), (1, []), (7, []), (7, ["--no-pipeline"]), (7, ["--async=2"]),
                                        (3, ["--files=3"]), (19, []), (20, [])],
                         ids=["before_first", "after_1", "after_7", "after_7_no_pipeline", "after_7_async",
                              "three_files", "after_19", "after_all"])
def test_cancel_stops_the_upload_and_returns_every_buffer(after, mode):
    """The transfer's cancel flag (TransferHandle::ShouldContinue, asked by
    the reference before each part, QSTransferManager.cpp:608 and 646): once
    it says stop, no further part is handed to the upload, the call returns
    normally with stats.stopped and stats.uploaded == the parts handed on
    (the caller marks the rest failed, :669-671), and every buffer -- the
    wave's, the one the helper thread was preparing -- is back in the pool."""
    gold = json.load(open(os.path.join(GOLDEN, "batch_10MiB.json")))["md5"]
    args = ["--aligned", "--size=%d" % (20 * 10 * MiB), "--pool=4", "--upload-ms=1",
            "--cancel-after=%d" % after] + mode
    out = run_raw(args, "cpu", timeout=120)
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads(out.stdout)
    files = r["files"]
    assert r["error"] == "" and r["deadlock"] is False, r
    assert r["pool_free_after"] == 4, r
    want = min(after, 20)
    assert r["stats_uploaded"] == want * files and r["uploaded"] == want * files, r
    # the last part handed on ends the loop before anyone asks again
    assert r["stopped"] == (files if after < 20 else 0), r
    for m in r["md5_files"]:
        assert m[:want] == gold[:want] and not any(m[want:]), m


# ---- the pool-free pre-hash (--staged) -------------------------

@pytest.mark.parametrize("extra", [[], ["--no-pipeline"], ["--wave-parts=5"],
                                   ["--wave-parts=5", "--async=3"], ["--staging=1000000"]])
def test_staged_prehash_matches_golden(extra):
    """qsmd5::upload_parts_staged: every part of a 24-part file pre-hashed by
    qsmd5_hash_read straight from the pages (no pool buffer), then the
    reference's one-buffer-at-a-time loop at qsfs's default -n 5.  Waves of 5
    parts pipelined on the helper thread, the async executor, and a 1 MB
    budget (rows of 64 KiB, many groups) give the same golden digests, and
    every pool buffer comes back."""
    gold = json.load(open(os.path.join(GOLDEN, "batch_10MiB.json")))["md5"]
    r = run(["--aligned", "--size=%d" % (24 * 10 * MiB), "--pool=5", "--staged"] + extra, "cpu")
    assert r["staged"] is True and r["parts"] == 24 and r["uploaded"] == 24
    assert r["md5"] == gold[:24]
    assert r["pool_free_after"] == 5
    want_waves = 5 if "--wave-parts=5" in extra else 1
    assert r["waves"] == want_waves and r["widest_wave"] == (5 if want_waves == 5 else 24)


@pytest.mark.parametrize("extra,waves", [(["--wave-parts=8", "--first-wave=2"], [2, 4, 8, 8, 2]),
                                         (["--wave-parts=8", "--first-wave=2", "--no-pipeline"], [8, 8, 8]),
                                         (["--wave-parts=64", "--first-wave=3"], [3, 6, 12, 3])])
def test_staged_wave_ramp(extra, waves):
    """StagedOptions::first_wave_parts: with the pipeline, the first wave is
    small and each next one doubles up to wave_parts (the first upload waits
    for a CPU-sized wave, every larger wave is pre-hashed while the smaller one
    uploads); without the pipeline the ramp is off.  Same golden digests."""
    gold = json.load(open(os.path.join(GOLDEN, "batch_10MiB.json")))["md5"]
    r = run(["--aligned", "--size=%d" % (24 * 10 * MiB), "--pool=5", "--staged", "--upload-ms=1"] + extra, "cpu")
    assert r["md5"] == gold[:24] and r["uploaded"] == 24 and r["pool_free_after"] == 5
    assert r["waves"] == len(waves) and r["widest_wave"] == max(waves), (r["waves"], r["widest_wave"])


def test_staged_ragged_file_matches_oracle():
    for size, seed in ((25 * MiB + 3, 41), (100 * MiB + 12345, 42)):
        r = run(["--size=%d" % size, "--seed=%d" % seed, "--pool=2", "--staged",
                 "--staging=%d" % (4 * MiB)], "cpu")
        data = lcg_bytes(seed, size)
        base, off, want = ctypes.addressof(data), 0, []
        for L in r["part_sizes"]:
            want.append((base + off, L))
            off += L
        assert r["md5"] == [d.hex() for d in md5_many(want)], size


def test_staged_concurrent_files_share_a_blocking_pool():
    """Four files flushing at once through one 5-buffer blocking pool: the
    pre-hash holds no buffer and the upload loop holds one at a time while it
    holds none, so there is no hold-and-wait to deadlock on."""
    gold = json.load(open(os.path.join(GOLDEN, "batch_10MiB.json")))["md5"]
    r = run(["--aligned", "--size=%d" % (12 * 10 * MiB), "--pool=5", "--files=4", "--upload-ms=2",
             "--deadlock-s=10", "--staged", "--wave-parts=4", "--async=3"], "cpu", timeout=120)
    assert r["deadlock"] is False
    for f, got in enumerate(r["md5_files"]):
        assert got == gold[:12], f


@pytest.mark.parametrize("fault,upload_expected", [("--short-read-part=7", 0),
                                                   ("--fail-upload-part=7", 6)])
def test_staged_faults_stop_the_upload_and_return_every_buffer(fault, upload_expected):
    """A short read inside part 7 fails the whole-file pre-hash before any
    part is uploaded (the reference stops at its first short read,
    QSTransferManager.cpp:625-643, after uploading the parts before it; here
    no part goes out unhashed); a failing upload of part 7 stops after 6."""
    out = run_raw(["--aligned", "--size=%d" % (12 * 10 * MiB), "--pool=5", "--staged", fault], "cpu")
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    r = json.loads(out.stdout)
    assert r["uploaded"] == upload_expected and r["pool_free_after"] == 5
    assert ("short read" in r["error"]) == ("short-read" in fault)


def test_staged_cancel_stops_between_parts():
    r = run(["--aligned", "--size=%d" % (12 * 10 * MiB), "--pool=5", "--staged", "--wave-parts=4",
             "--cancel-after=6"], "cpu")
    assert r["stopped"] == 1 and r["uploaded"] == 6 and r["stats_uploaded"] == 6
    assert r["pool_free_after"] == 5


def test_busy_cores_lower_the_cpu_efficiency():
    """VERDICT r04 item 3's load, as scripts/r05_route_sweep.sh sets it up: the
    harness held to 2 cores (--cpus=2) with 2 spinning threads of other work on
    them (--load=2).  The CPU backend's waves then take longer than priced, and
    qsmd5_get_cpu_efficiency (the factor auto routing divides CPU estimates by)
    reads well below 1; on the same cores without the load it stays near 1.
    Every digest stays golden."""
    gold = json.load(open(os.path.join(GOLDEN, "batch_10MiB.json")))["md5"]
    base = ["--aligned", "--size=%d" % (16 * 10 * MiB), "--pool=8", "--no-pipeline", "--repeat=2",
            "--cpus=2"]
    env = {"QSMD5_CPU_THREADS": "2", "QSMD5_CPU_EFF_DECAY_S": "1000"}
    idle = run(base + ["--load=0"], "cpu", extra_env=env)
    busy = run(base + ["--load=2"], "cpu", extra_env=env)
    assert idle["md5"] == gold[:16] and busy["md5"] == gold[:16]
    assert busy["cpus"] == 2 and busy["load_threads"] == 2
    assert busy["cpu_efficiency"] < 0.75, busy["cpu_efficiency"]
    assert busy["cpu_efficiency"] < idle["cpu_efficiency"] - 0.2, (idle["cpu_efficiency"], busy["cpu_efficiency"])


# ---- round 6: the reference's own loop beside the staged binding, read-ahead ------

REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref_md5.so")


@pytest.mark.skipif(not os.path.exists(REF_SO), reason="oracle/_ref not built (oracle/build_ref.sh)")
@pytest.mark.parametrize("mode", [[], ["--async=5"]])
def test_reference_loop_matches_golden(mode):
    """--reference-loop: QSTransferManager::DoMultiPartUpload
    with -m as the reference runs it -- Acquire, ReadNoLoad, the reference's own
    md5(shared_ptr<iostream>) from oracle/_ref (MD5.cpp compiled in place; the
    baseline, test infrastructure), upload -- on the flushing thread or on the
    executor.  Its digests are the golden table's, so the staged binding and
    the loop it replaces are timed on the same bytes."""
    gold = json.load(open(os.path.join(GOLDEN, "batch_10MiB.json")))["md5"]
    r = run(["--aligned", "--size=%d" % (12 * 10 * MiB), "--pool=5", "--reference-loop", "--upload-ms=1"] + mode,
            "cpu")
    assert r["reference_loop"] is True and r["md5"] == gold[:12] and r["uploaded"] == 12
    assert r["pool_free_after"] == 5 and r["hash_s"] > 0
    if not mode:  # serial: every part's md5 on this thread, between its read and its upload
        assert r["seconds"] >= r["hash_s"] + r["loop_read_s"]


@pytest.mark.parametrize("extra", [[], ["--wave-parts=5", "--first-wave=2"]])
def test_staged_read_ahead_matches_golden(extra):
    """StagedOptions::read_ahead: while a part uploads,
    the next part is read into a buffer the pool has free (try_acquire),
    wherever the last upload took longer than the last read.  With 20 ms
    uploads nearly every part after the first is read ahead; with uploads
    that return at once none is (nothing to hide behind).  The digests stay
    golden and every buffer comes back; --no-read-ahead is the reference's
    one-buffer loop exactly."""
    gold = json.load(open(os.path.join(GOLDEN, "batch_10MiB.json")))["md5"]
    base = ["--aligned", "--size=%d" % (16 * 10 * MiB), "--pool=5", "--staged"] + extra
    on = run(base + ["--upload-ms=20"], "cpu")
    off = run(base + ["--upload-ms=20", "--no-read-ahead"], "cpu")
    fast = run(base + ["--upload-ms=0"], "cpu")
    for r in (on, off, fast):
        assert r["md5"] == gold[:16] and r["uploaded"] == 16 and r["pool_free_after"] == 5
    assert off["read_ahead"] == 0 and fast["read_ahead"] == 0
    assert on["read_ahead"] >= 16 - 2 * on["waves"] - 1, on["read_ahead"]


def test_staged_read_ahead_faults_return_every_buffer():
    """A short read that the read-ahead hits, and a failing upload while a part
    is being read ahead: the upload stops, nothing leaks."""
    for fault, want in (("--short-read-part=7", 0), ("--fail-upload-part=7", 6)):
        out = run_raw(["--aligned", "--size=%d" % (12 * 10 * MiB), "--pool=5", "--staged", "--wave-parts=12",
                       "--upload-ms=20", fault], "cpu")
        assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
        r = json.loads(out.stdout)
        assert r["uploaded"] == want and r["pool_free_after"] == 5, (fault, r["uploaded"])


def _nested_read_exe(tmp_path):
    exe = str(tmp_path / "nested_read")
    subprocess.check_call([
        "g++", "-std=c++17", "-O2", os.path.join(ROOT, "tests", "cpp", "nested_read.cpp"),
        "-I" + os.path.join(ROOT, "include"), "-L" + os.path.join(ROOT, "qsfs-fuse_amd", "lib"), "-lqsmd5",
        "-lpthread", "-Wl,-rpath," + os.path.join(ROOT, "qsfs-fuse_amd", "lib"), "-o", exe])
    return exe


@pytest.mark.parametrize("args", [["shutdown", "cpu"], ["nested-read", "cpu", "auto"],
                                  ["nested-read", "cpu", "cpu"]])
def test_read_callbacks_call_back_into_the_library(tmp_path, args):
    """read callbacks that call qsmd5 entry points.  With
    QSMD5_FLAG_READ_PARALLEL the callbacks also run on the library's reader
    threads; one of them starts qsmd5_shutdown and then calls qsmd5_hash_one
    while the shutdown is pending.  A reader thread's call is a nested call
    (its depth is raised), so it does not wait at the shutdown gate: the
    outer call finishes and the shutdown then gets through.  (Round 5's
    reader threads deadlocked here: outer call, reader thread and shutdown
    waiting on each other.)  Nested qsmd5_hash_read calls hash right too."""
    out = subprocess.run([_nested_read_exe(tmp_path)] + args, capture_output=True, text=True, timeout=120,
                         env=dict(os.environ, QSMD5_BACKEND="auto"))
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert out.returncode == 0 and r["deadlock"] is False and r["digests_ok"], out.stdout + out.stderr
    if args[0] == "shutdown":
        assert r["reader_thread_reads"] > 0 and r["shutdown_rc"] == 0
    else:
        assert r["nested_ok"] == r["nested_calls"] > 0


def test_backends_alternate_per_pass_in_one_process():
    """--backends=cpu,auto: the harness sets QSMD5_BACKEND before each pass
    (the library reads it at each call), so backends can be compared in one
    process; every pass hands on the same golden digests."""
    gold = json.load(open(os.path.join(GOLDEN, "batch_10MiB.json")))["md5"]
    r = run(["--aligned", "--size=%d" % (8 * 10 * MiB), "--pool=5", "--staged", "--repeat=4",
             "--backends=cpu,auto"], "cpu", extra_env={"QSMD5_TRACE": "1"})
    assert r["md5"] == gold[:8] and r["pass_mismatch"] == 0
    reasons = [json.loads(l.split("qsmd5 read trace: ", 1)[1])["reason"] for l in r["_stderr"].splitlines()
               if "qsmd5 read trace: " in l]
    assert len(reasons) == 4 and reasons[0] == reasons[2] == "forced" and reasons[1] != "forced", reasons


@pytest.mark.parametrize("mode", [[], ["--wave-parts=4", "--first-wave=2"], ["--async=3"], ["--cancel-after=5"]],
                         ids=["whole", "ramp", "async", "cancel"])
def test_staged_concurrent_files_under_tsan(mode):
    """The staged binding's threads under ThreadSanitizer (round 6): the
    pre-hash helper, the upload loop's read-ahead thread, the shared pool and
    the executor's handler, four files at once through one 5-buffer pool with
    uploads slow enough (30 ms) that the read-ahead runs (not with the
    executor, whose upload() returns at once).  No report, every digest
    golden, every buffer back."""
    exe = build_tsan()
    gold = json.load(open(os.path.join(GOLDEN, "batch_10MiB.json")))["md5"]
    env = dict(os.environ, QSMD5_BACKEND="cpu", TSAN_OPTIONS="halt_on_error=0:exitcode=66:suppressions="
               + os.path.join(ROOT, "tests", "cpp", "tsan_hip.supp"))
    out = subprocess.run(["setarch", "x86_64", "-R", exe, "--aligned", "--size=%d" % (8 * 10 * MiB),
                          "--pool=5", "--files=4", "--upload-ms=30", "--deadlock-s=30", "--staged"] + mode,
                         env=env, capture_output=True, text=True, timeout=300)
    assert "WARNING: ThreadSanitizer" not in out.stderr, out.stderr[-8000:]
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads(out.stdout)
    want = 5 if "--cancel-after=5" in mode else 8
    assert r["deadlock"] is False and r["pool_free_after"] == 5, r
    assert all(m[:want] == gold[:want] and not any(m[want:]) for m in r["md5_files"]), r["md5_files"]
    if "--cancel-after=5" not in mode and "--async=3" not in mode:  # an executor's upload() returns at once
        assert r["read_ahead"] > 0, r["read_ahead"]
