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
splitter's per-device threads (qsmd5_runtime.cpp, in-process sharding) run
under the sanitizer too; a 1 MiB QSMD5_SHARD_BYTES makes even these small
batches split, and QSMD5_MAPS_AFTER=2 sends the classifier to its
/proc/self/maps cache from the second pageable query.
"""
import os
import subprocess

import pytest

from conftest import ROOT

SAN = os.path.join(ROOT, "qsfs-fuse_amd", "lib", "san")
REPORT_MARKERS = ("WARNING: ThreadSanitizer", "ERROR: AddressSanitizer", "runtime error:",
                  "ERROR: LeakSanitizer")


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
    env.pop("QSMD5_DEVICES", None)
    if devices:
        env["QSMD5_DEVICES"] = devices
        env["QSMD5_SHARD_BYTES"] = str(1 << 20)  # split even these small batches
        env["QSMD5_MAPS_AFTER"] = "2"            # and read /proc/self/maps early
    # leak checking would report HIP runtime allocations that live until exit
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=0:exitcode=23"
    env["TSAN_OPTIONS"] = ("halt_on_error=0:exitcode=66:second_deadlock_stack=1:print_suppressions=1:"
                           "suppressions=" + os.path.join(ROOT, "tests", "cpp", "tsan_hip.supp"))
    out = subprocess.run([exe, str(threads), str(rounds), str(max_len)] + list(extra), env=env,
                         capture_output=True, text=True, timeout=110)
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
def test_tsan_negative_control_reports_planted_race():
    """The suppressions silence only the uninstrumented HIP/HSA runtimes: a
    race planted in instrumented code (race_stress.cpp `racy`) is reported."""
    rc, text = _run("tsan", "", threads=4, rounds=4, max_len=1 << 16, extra=["racy"],
                    expect_clean=False)
    assert "WARNING: ThreadSanitizer: data race" in text, text[-3000:]
    assert "race_stress.cpp" in text and "worker" in text, text[-3000:]
    assert rc == 66, rc  # TSAN_OPTIONS exitcode: the report fails the run
