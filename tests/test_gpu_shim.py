"""The C++ drop-in (qsfs-fuse_amd/host/qsfs_md5.hpp) on the GPU.

tests/cpp/test_shim.cpp uses the reference-shaped interface -- global
md5(std::string), md5(shared_ptr<iostream>) over a qsfs StreamBuf-style view,
class MD5 -- and prints one digest per case; each is checked here against
hashlib / the oracle.  The binary also asserts the reference's stream side
effects (read position reset to 0, MD5.cpp:343-346) and loud failure.
"""
import hashlib
import os
import subprocess

import pytest

from conftest import ROOT
from oracle_util import lcg_bytes

BIN = os.path.join(ROOT, "tests", "cpp", "test_shim")


def build_shim():
    subprocess.check_call([
        "g++", "-std=c++17", "-O2", os.path.join(ROOT, "tests", "cpp", "test_shim.cpp"),
        "-I" + os.path.join(ROOT, "include"), "-L" + os.path.join(ROOT, "qsfs-fuse_amd", "lib"),
        "-lqsmd5", "-Wl,-rpath," + os.path.join(ROOT, "qsfs-fuse_amd", "lib"), "-o", BIN])


def check_shim_output(out):
    assert out.returncode == 0, out.stdout + out.stderr
    got = dict(line.split() for line in out.stdout.strip().splitlines() if not line.startswith("parts_"))
    h = lambda b: hashlib.md5(b).hexdigest()
    assert got["str_empty"] == h(b"")
    assert got["str_abc"] == h(b"abc")
    assert got["str_literal"] == h(b"message digest")
    import base64
    assert got["content_md5_abc"] == base64.b64encode(hashlib.md5(b"abc").digest()).decode()
    for L in (0, 2, 55, 64, 10485760):
        assert got["view_%d" % L] == h(bytes(lcg_bytes(12345, L + 100))[:L]), L
    assert got["streamtest_read1"] == h(b"01")
    assert got["stringstream_100000q"] == h(b"q" * 100000)
    assert got["class_pieces"] == h(bytes(lcg_bytes(4242, 200000)))
    assert got["class_ctor_abc"] == h(b"abc")
    for i in range(6):
        assert got["batch_%d" % i] == h(bytes(lcg_bytes(500 + i, 1000 * i * i + 3 * i + 1))[:1000 * i * i + 3 * i])
    MiB = 1 << 20
    rows = [l.split() for l in out.stdout.splitlines() if l.startswith("parts_")]
    for fsz, sizes in ((25 * MiB + 3, [10 * MiB, 10 * MiB, 5 * MiB + 3]),
                       (21 * MiB, [10 * MiB, 11 * MiB // 2, 11 * MiB - 11 * MiB // 2])):
        mine = [r for r in rows if r[0].startswith("parts_%d_" % fsz)]
        assert [int(r[2]) for r in mine] == sizes, mine
        data = bytes(lcg_bytes(777, fsz))
        for r in mine:
            off, sz = int(r[1]), int(r[2])
            assert r[3] == h(data[off:off + sz]), r
    d = bytes(lcg_bytes(31337, 5000))
    assert got["copy_b"] == h(d)
    assert got["copy_a"] == h(d[:100] + b"x")
    assert got["copy_c"] == h(d + b"y")
    assert got["failures"] == "0"


def shim_binary():
    src = os.path.join(ROOT, "tests", "cpp", "test_shim.cpp")
    hdr = os.path.join(ROOT, "qsfs-fuse_amd", "host", "qsfs_md5.hpp")
    if not os.path.exists(BIN) or os.path.getmtime(BIN) < max(os.path.getmtime(src), os.path.getmtime(hdr)):
        build_shim()
    return BIN


@pytest.mark.gpu
def test_cpp_dropin_shim():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    check_shim_output(subprocess.run([shim_binary()], capture_output=True, text=True, timeout=300))


def test_cpp_dropin_shim_cpu_backend():
    """The same drop-in program with the library's CPU backend (QSMD5_BACKEND=cpu,
    no GPU needed): the C++ surface, the stream side effects and the class's
    copy semantics hold whichever backend hashes."""
    env = dict(os.environ, QSMD5_BACKEND="cpu")
    check_shim_output(subprocess.run([shim_binary()], capture_output=True, text=True, timeout=300, env=env))
