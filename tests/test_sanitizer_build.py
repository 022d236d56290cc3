"""CPU check of the host-sanitizer builds (scripts/build_sanitized.sh, run by
__graft_entry__.build()): both binaries exist, start under their sanitizer
runtimes with the HIP runtime loaded, and without a GPU stop with "no GPU"
(exit 2) before any hashing.  The stress itself is tests/test_gpu_sanitizers.py."""
import os
import subprocess

import pytest

from conftest import ROOT

SAN = os.path.join(ROOT, "qsfs-fuse_amd", "lib", "san")


@pytest.mark.parametrize("variant", ["tsan", "asan"])
def test_sanitized_binary_starts(variant):
    exe = os.path.join(SAN, "race_stress_" + variant)
    assert os.path.exists(exe), "run __graft_entry__.build() (scripts/build_sanitized.sh)"
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", TSAN_OPTIONS="exitcode=66")
    out = subprocess.run([exe, "2", "1", "4096"], env=env, capture_output=True, text=True,
                         timeout=120)
    text = out.stdout + out.stderr
    assert "Sanitizer" not in text, text[-3000:]
    if out.returncode == 2:
        assert "no GPU" in text, text
    else:  # a GPU is visible: the short stress must then pass
        assert out.returncode == 0 and "race_stress ok" in out.stdout, text[-3000:]
