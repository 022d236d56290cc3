"""CPU check of the host-sanitizer builds (scripts/build_sanitized.sh, run by
__graft_entry__.build()): both binaries exist, start under their sanitizer
runtimes with the HIP runtime loaded, and without a GPU stop with "no GPU"
(exit 2) before any hashing.  The stress itself is tests/test_gpu_sanitizers.py."""
import os
import subprocess

import pytest

from conftest import ROOT

SAN = os.path.join(ROOT, "qsfs-fuse_amd", "lib", "san")
# The same suppressions as tests/test_gpu_sanitizers.py: on a machine with a
# GPU even QSMD5_BACKEND=cpu starts the uninstrumented HIP/HSA runtimes
# (qsmd5_device_count), whose own threads TSan would otherwise report.
TSAN = ("halt_on_error=0:exitcode=66:suppressions=" + os.path.join(ROOT, "tests", "cpp", "tsan_hip.supp"))


@pytest.mark.parametrize("variant", ["tsan", "asan"])
def test_sanitized_binary_starts(variant):
    exe = os.path.join(SAN, "race_stress_" + variant)
    assert os.path.exists(exe), "run __graft_entry__.build() (scripts/build_sanitized.sh)"
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", TSAN_OPTIONS=TSAN)
    out = subprocess.run([exe, "2", "1", "4096"], env=env, capture_output=True, text=True,
                         timeout=120)
    text = out.stdout + out.stderr
    assert "Sanitizer" not in text, text[-3000:]
    if out.returncode == 2:
        assert "no GPU" in text, text
    else:  # a GPU is visible: the short stress must then pass
        assert out.returncode == 0 and "race_stress ok" in out.stdout, text[-3000:]


@pytest.mark.parametrize("groups", ["1", "2"], ids=["16_lanes", "32_lanes"])
@pytest.mark.parametrize("variant", ["tsan", "asan"])
def test_race_stress_cpu_backend(variant, groups):
    """The same stress with the library's CPU backend and no GPU
    (QSMD5_BACKEND=cpu): six threads racing every entry point -- hash_one,
    ragged batches over the backend's worker threads and 16- or 32-lane
    multi-buffer cores, streaming contexts copied mid-stream, shutdown and
    re-init -- under ThreadSanitizer, and under AddressSanitizer + UBSan.
    Every digest is checked against the oracle inside the binary."""
    exe = os.path.join(SAN, "race_stress_" + variant)
    env = dict(os.environ, QSMD5_BACKEND="cpu", QSMD5_CPU_THREADS="4", QSMD5_CPU_MB_GROUPS=groups,
               ASAN_OPTIONS="detect_leaks=0", TSAN_OPTIONS=TSAN)
    out = subprocess.run(["setarch", "x86_64", "-R", exe, "6", "16"], env=env,
                         capture_output=True, text=True, timeout=300)
    text = out.stdout + out.stderr
    if out.returncode == 2 and "no GPU" in text:
        pytest.skip("binary predates the CPU mode")
    assert "Sanitizer" not in text and "runtime error" not in text, text[-4000:]
    assert out.returncode == 0 and "race_stress ok" in out.stdout, text[-3000:]


def test_tsan_negative_control_cpu_backend():
    """The planted unsynchronised counter is reported by the TSan build on the
    CPU backend too: the check above would see a race."""
    exe = os.path.join(SAN, "race_stress_tsan")
    env = dict(os.environ, QSMD5_BACKEND="cpu", TSAN_OPTIONS=TSAN)
    out = subprocess.run(["setarch", "x86_64", "-R", exe, "4", "4", "65536", "racy"], env=env,
                         capture_output=True, text=True, timeout=300)
    assert "WARNING: ThreadSanitizer: data race" in out.stderr, (out.stdout + out.stderr)[-3000:]
    assert out.returncode == 66


@pytest.mark.parametrize("variant", ["tsan", "asan"])
@pytest.mark.parametrize("args", [["shutdown", "cpu"], ["shutdown", "auto"], ["nested-read", "cpu", "auto"]],
                         ids=["parallel_readers_shutdown_cpu", "parallel_readers_shutdown_auto", "nested_read"])
def test_nested_read_callbacks_cpu_backend(variant, args):
    """tests/cpp/nested_read.cpp (round 6) over the runtime built
    with ThreadSanitizer, and with AddressSanitizer + UBSan, on the library's
    CPU path: the window's rows read by the reader crew, whose callbacks call
    qsmd5_hash_one while a shutdown is pending, or nested qsmd5_hash_read
    calls.  No deadlock, every digest right, no sanitizer report."""
    exe = os.path.join(SAN, "nested_read_" + variant)
    assert os.path.exists(exe), "run __graft_entry__.build() (scripts/build_sanitized.sh)"
    env = dict(os.environ, QSMD5_BACKEND="auto", ASAN_OPTIONS="detect_leaks=0", TSAN_OPTIONS=TSAN)
    out = subprocess.run(["setarch", "x86_64", "-R", exe] + args, env=env, capture_output=True, text=True,
                         timeout=300)
    text = out.stdout + out.stderr
    assert "Sanitizer" not in text and "runtime error" not in text, text[-4000:]
    assert out.returncode == 0 and '"deadlock": false' in out.stdout, text[-3000:]

