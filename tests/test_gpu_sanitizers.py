"""Host-sanitizer runs of the runtime under concurrent callers (SURVEY.md §5:
"run the CPU path under -fsanitize=thread; the C-ABI must be reentrant").

scripts/build_sanitized.sh builds tests/cpp/race_stress.cpp against the
runtime's host code instrumented with ThreadSanitizer, and with
AddressSanitizer + UBSan (the gfx950 kernels are the product object; GPU
sanitizers are not available on the pool).  Each binary races qsmd5_init,
hash_one (group commit), ragged batches, the streaming context and the pinned
pool from several threads and checks every digest against the oracle.  A
sanitizer report fails the test even when every digest matched.

QSMD5_DEVICES=0,0 binds two contexts to the box's one GPU, so the batch
splitter's per-device threads (qsmd5_rt_staging.cpp run_sharded, in-process sharding) run
under the sanitizer too; a 1 MiB QSMD5_SHARD_BYTES makes even these small
batches split, and QSMD5_MAPS_AFTER=2 sends the classifier to its
/proc/self/maps cache from the second pageable query.
"""
import os
import re
import signal
import subprocess
import threading
import time

import pytest

from conftest import ROOT

SAN = os.path.join(ROOT, "qsfs-fuse_amd", "lib", "san")
REPORT_MARKERS = ("WARNING: ThreadSanitizer", "ERROR: AddressSanitizer", "runtime error:",
                  "ERROR: LeakSanitizer")


SYMBOLIZER = "/opt/rocm/llvm/bin/llvm-symbolizer"


class _Result:
    def __init__(self, returncode, stdout, stderr):
        self.returncode, self.stdout, self.stderr = returncode, stdout, stderr


def _diagnose(pid, err):
    """Where a sanitizer child that took a deadly signal is: the faulting pc and
    address resolved against the child's own /proc/<pid>/maps (library, offset,
    symbol), and what each of its threads is blocked in.  Read while the child
    is still alive, so the layout is the one the fault happened in."""
    lines = []
    try:
        with open("/proc/%d/maps" % pid) as f:
            maps = [ln.split() for ln in f]
    except OSError as e:
        return "no maps: %s" % e
    def find(addr):
        for m in maps:
            lo, hi = (int(x, 16) for x in m[0].split("-"))
            if lo <= addr < hi:
                return lo, m[5] if len(m) > 5 else "[anon]"
        return None, None
    for what, pat in (("pc", r"\(pc (0x[0-9a-f]+)"), ("address", r"on unknown address (0x[0-9a-f]+)")):
        for hx in re.findall(pat, err):
            a = int(hx, 16)
            lo, path = find(a)
            if path is None:
                lines.append("%s %s: not mapped now" % (what, hx))
                continue
            base = min(int(m[0].split("-")[0], 16) for m in maps if len(m) > 5 and m[5] == path)
            rel = a - base
            sym = ""
            if what == "pc" and path.startswith("/") and os.path.exists(SYMBOLIZER):
                try:
                    sym = subprocess.run([SYMBOLIZER, "--obj=" + path, hex(rel)], capture_output=True,
                                         text=True, timeout=20).stdout.strip().replace("\n", " @ ")
                except (OSError, subprocess.SubprocessError) as e:
                    sym = "symbolizer: %s" % e
            lines.append("%s %s: %s + %s %s" % (what, hx, path, hex(rel), sym))
    try:
        for tid in sorted(os.listdir("/proc/%d/task" % pid), key=int):
            d = "/proc/%d/task/%s/" % (pid, tid)
            def rd(name):
                try:
                    with open(d + name) as f:
                        return f.read().strip()
                except OSError:
                    return "?"
            lines.append("thread %s %-16s state %s wchan %s" % (tid, rd("comm"), rd("stat").split(") ")[-1][:1],
                                                                rd("wchan")))
    except OSError:
        pass
    return "\n".join(lines)


def _watch(cmd, env, timeout=110, grace=15):
    """subprocess.run with a watchdog: a child that reports a deadly signal
    (a sanitizer's DEADLYSIGNAL) but does not exit within `grace` seconds, or
    runs past `timeout`, is diagnosed (_diagnose) and killed with its process
    group, and the test fails at once with its output -- one bad child costs
    seconds, not the suite (round 3: a SEGV'd child hung to the 110 s limit)."""
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         start_new_session=True)
    bufs = {"out": [], "err": []}
    readers = [threading.Thread(target=lambda f=f, k=k: bufs[k].extend(iter(f.readline, "")), daemon=True)
               for f, k in ((p.stdout, "out"), (p.stderr, "err"))]
    for r in readers:
        r.start()
    t0 = time.monotonic()
    deadly_at = None
    while p.poll() is None:
        now = time.monotonic()
        if deadly_at is None and any("DEADLYSIGNAL" in ln for ln in list(bufs["err"])):
            deadly_at = now
        if (deadly_at is not None and now - deadly_at > grace) or now - t0 > timeout:
            err = "".join(bufs["err"])
            diag = _diagnose(p.pid, err)
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except OSError:
                pass
            p.wait()
            for r in readers:
                r.join(5)
            why = "took a deadly signal and did not exit within %d s" % grace if deadly_at is not None \
                else "ran past %d s" % timeout
            pytest.fail("%s %s; killed.\n--- diagnosis ---\n%s\n--- stderr ---\n%s\n--- stdout ---\n%s" % (
                os.path.basename(cmd[0]), why, diag, "".join(bufs["err"])[-6000:], "".join(bufs["out"])[-2000:]))
        time.sleep(0.1)
    for r in readers:
        r.join(10)
    return _Result(p.returncode, "".join(bufs["out"]), "".join(bufs["err"]))


def _run(variant, devices, threads=6, rounds=12, max_len=3 << 20, extra=(), expect_clean=True,
         backend="gpu", inject=None, cpu_threads=None):
    exe = os.path.join(SAN, "race_stress_" + variant)
    if not os.path.exists(exe):
        pytest.fail("%s missing: run scripts/build_sanitized.sh (built by __graft_entry__.build())" % exe)
    env = dict(os.environ)
    env["QSMD5_BACKEND"] = backend
    env.pop("QSMD5_INJECT_GPU_FAULT", None)
    if inject:
        env["QSMD5_INJECT_GPU_FAULT"] = inject
    env.pop("QSMD5_CPU_THREADS", None)
    env.pop("QSMD5_SPLIT", None)
    env.pop("QSMD5_LOG", None)
    if cpu_threads:
        env["QSMD5_CPU_THREADS"] = str(cpu_threads)
    if backend == "auto":
        env["QSMD5_LOG"] = "1"  # the routing decisions, checked below
        env["QSMD5_ROUTE_LANES"] = "0"  # the scalar model, under which ragged batches split
    env.pop("QSMD5_DEVICES", None)
    if devices:
        env["QSMD5_DEVICES"] = devices
        env["QSMD5_SHARD_BYTES"] = str(1 << 20)  # split even these small batches
        env["QSMD5_MAPS_AFTER"] = "2"            # and read /proc/self/maps early
    # leak checking would report HIP runtime allocations that live until exit
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=0:exitcode=23"
    env["TSAN_OPTIONS"] = ("halt_on_error=0:exitcode=66:second_deadlock_stack=1:print_suppressions=1:"
                           "suppressions=" + os.path.join(ROOT, "tests", "cpp", "tsan_hip.supp"))
    out = _watch([exe, str(threads), str(rounds), str(max_len)] + list(extra), env)
    text = out.stdout + out.stderr
    if not expect_clean:
        return out.returncode, text
    for m in REPORT_MARKERS:
        at = text.find(m)
        assert at < 0, text[max(0, at - 200):at + 8000]
    assert out.returncode == 0, text[-6000:]
    assert "race_stress ok" in out.stdout, text[-3000:]
    sup = [ln for ln in out.stderr.splitlines() if "suppression" in ln.lower() or ln.strip().startswith(("race:", "called_from_lib:"))]
    routes = sorted({ln for ln in out.stderr.splitlines() if ln.startswith("qsmd5: backend=")
                     for ln in [ln.split(" chunks=")[0]]})
    return out.stdout + "\n".join(sup + routes)


@pytest.mark.gpu
@pytest.mark.parametrize("devices", ["", "0,0"])
def test_race_stress_tsan(devices):
    print(_run("tsan", devices))


@pytest.mark.gpu
@pytest.mark.parametrize("devices", ["", "0,0"])
def test_race_stress_asan_ubsan(devices):
    print(_run("asan", devices))


@pytest.mark.gpu
@pytest.mark.cpu_backend
@pytest.mark.parametrize("variant", ["tsan", "asan"])
@pytest.mark.parametrize("inject", [None, "1"], ids=["routed", "gpu_fault_fallback"])
def test_race_stress_auto_backend(variant, inject):
    """QSMD5_BACKEND=auto: small calls and streams route to the library's CPU
    MD5 (its helper threads included) while larger batches take the GPU, and
    ragged batches split between the two (one CPU thread, so that the
    stress's small batches already favour the GPU); with an injected GPU fault
    every GPU call falls back to the CPU.  Both under the sanitizers, every
    digest against the oracle."""
    out = _run(variant, "", backend="auto", inject=inject, cpu_threads=1)
    print(out)
    assert "backend=gpu+cpu reason=split" in out, out[-3000:]
    assert "backend=cpu reason=size" in out, out[-3000:]


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["tsan", "asan"])
def test_race_stress_small_buffers(variant):
    """The negative control's sizes (64 KiB buffers) without the planted race:
    every case's chunks stay inside the worker's buffer (race_stress.cpp
    in_buf aborts otherwise), under both sanitizers.  Round 3's control built
    128-256 KiB chunks from a 64 KiB buffer and hashed unmapped memory."""
    print(_run(variant, "", threads=4, rounds=10, max_len=1 << 16))


@pytest.mark.gpu
def test_tsan_negative_control_reports_planted_race():
    """The suppressions silence only the uninstrumented HIP/HSA runtimes: a
    race planted in instrumented code (race_stress.cpp `racy`) is reported."""
    rc, text = _run("tsan", "", threads=4, rounds=4, max_len=1 << 16, extra=["racy"],
                    expect_clean=False)
    assert "WARNING: ThreadSanitizer: data race" in text, text[-3000:]
    assert "race_stress.cpp" in text and "worker" in text, text[-3000:]
    assert rc == 66, rc  # TSAN_OPTIONS exitcode: the report fails the run


@pytest.mark.gpu
@pytest.mark.cpu_backend
@pytest.mark.parametrize("variant", ["tsan", "asan"])
@pytest.mark.parametrize("args,slots", [(["shutdown", "gpu"], "4"), (["nested-read", "gpu", "auto"], "1"),
                                        (["nested-read", "gpu", "gpu"], "1")],
                         ids=["parallel_readers_shutdown", "nested_auto", "nested_gpu_edeadlk"])
def test_nested_read_callbacks_under_sanitizers(variant, args, slots):
    """tests/cpp/nested_read.cpp over the instrumented runtime (round 6,
    ADVICE r05): the outer pull-driven batch on the GPU, its read callbacks on
    the calling thread and the reader crew calling back into the library --
    qsmd5_hash_one while a shutdown is pending, or a nested qsmd5_hash_read
    (CPU under auto; -EDEADLK when forced onto the GPU's only, busy slot).
    No deadlock, every digest right, no sanitizer report."""
    exe = os.path.join(SAN, "nested_read_" + variant)
    if not os.path.exists(exe):
        pytest.fail("%s missing: run scripts/build_sanitized.sh" % exe)
    env = dict(os.environ, QSMD5_BACKEND="auto", QSMD5_READ_SLOTS=slots,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:exitcode=23",
               TSAN_OPTIONS="halt_on_error=0:exitcode=66:second_deadlock_stack=1:suppressions=" +
               os.path.join(ROOT, "tests", "cpp", "tsan_hip.supp"))
    out = _watch([exe] + args, env)
    text = out.stdout + out.stderr
    for m in REPORT_MARKERS:
        at = text.find(m)
        assert at < 0, text[max(0, at - 200):at + 8000]
    assert out.returncode == 0 and '"deadlock": false' in out.stdout, text[-4000:]

