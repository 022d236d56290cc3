"""CPU test of the host-staging plan (qsfs-fuse_amd/csrc/qsmd5_plan.h).

The plan decides how host-resident chunks are cut into groups, columns and
ring regions before any H2D copy (qsmd5_rt_staging.cpp run_batch).  The GPU
column tests check digests end to end; this test checks the plan's
invariants directly on the CPU over ~1 700 length mixes, ring sizes, slice
targets and column widths (tests/cpp/test_plan.cpp): every byte of every
chunk staged exactly once, each slice fitting its region, and so on.
"""
import os
import subprocess

from conftest import ROOT


def test_host_staging_plan_invariants(tmp_path):
    exe = str(tmp_path / "test_plan")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-Werror",
                           os.path.join(ROOT, "tests", "cpp", "test_plan.cpp"), "-o", exe])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("plan ok"), out.stdout
