"""CPU test of the VMA rule behind the runtime's pointer classifier
(qsfs-fuse_amd/csrc/qsmd5_vma.h): which /proc/self/maps entries may be
remembered as host memory so that later chunks inside them skip the HIP
pointer query.  Device memory must never qualify (tests/cpp/test_vma.cpp)."""
import os
import subprocess

from conftest import ROOT


def test_host_vma_rule(tmp_path):
    exe = str(tmp_path / "test_vma")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-Werror",
                           os.path.join(ROOT, "tests", "cpp", "test_vma.cpp"), "-o", exe])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("vma ok"), out.stdout
