"""Runs tests/cpp/multipart_harness (the DoMultiPartUpload flow with the batch
pre-hash) and returns its JSON report."""
import json
import os
import subprocess

from conftest import ROOT

HARNESS = os.path.join(ROOT, "tests", "cpp", "multipart_harness")


def newest_source():
    """The harness is rebuilt when it or any header it compiles in changed."""
    paths = [os.path.join(ROOT, "tests", "cpp", "multipart_harness.cpp"),
             os.path.join(ROOT, "qsfs-fuse_amd", "host", "qsfs_multipart.hpp"),
             os.path.join(ROOT, "qsfs-fuse_amd", "host", "qsfs_md5.hpp"),
             os.path.join(ROOT, "include", "qsmd5.h")]
    return max(os.path.getmtime(p) for p in paths)


def build():
    src = os.path.join(ROOT, "tests", "cpp", "multipart_harness.cpp")
    if not os.path.exists(HARNESS) or os.path.getmtime(HARNESS) < newest_source():
        subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", src,
                               "-I" + os.path.join(ROOT, "include"),
                               "-L" + os.path.join(ROOT, "qsfs-fuse_amd", "lib"), "-lqsmd5",
                               "-lpthread", "-ldl", "-Wl,-rpath,$ORIGIN/../../qsfs-fuse_amd/lib", "-o", HARNESS])


def run_raw(args, backend, timeout=300, extra_env=None):
    build()
    env = dict(os.environ, QSMD5_BACKEND=backend)
    env.update(extra_env or {})
    return subprocess.run([HARNESS] + list(args), env=env, capture_output=True, text=True,
                          timeout=timeout)


def run(args, backend, timeout=300, extra_env=None):
    out = run_raw(args, backend, timeout, extra_env)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    r = json.loads(out.stdout)
    r["_stderr"] = out.stderr
    return r


HARNESS_TSAN = os.path.join(ROOT, "tests", "cpp", "multipart_harness_tsan")


def build_tsan():
    """The harness and the drop-in header (qsfs_multipart.hpp: helper thread,
    pool, executor handoff) under ThreadSanitizer; libqsmd5 itself is not
    instrumented (its own threads are covered by test_gpu_sanitizers.py)."""
    src = os.path.join(ROOT, "tests", "cpp", "multipart_harness.cpp")
    if not os.path.exists(HARNESS_TSAN) or os.path.getmtime(HARNESS_TSAN) < newest_source():
        subprocess.check_call(["/opt/rocm/llvm/bin/clang++", "-std=c++17", "-O1", "-g",
                               "-fsanitize=thread", src, "-I" + os.path.join(ROOT, "include"),
                               "-L" + os.path.join(ROOT, "qsfs-fuse_amd", "lib"), "-lqsmd5",
                               "-lpthread", "-ldl", "-Wl,-rpath," + os.path.join(ROOT, "qsfs-fuse_amd", "lib"),
                               "-o", HARNESS_TSAN])
    return HARNESS_TSAN
