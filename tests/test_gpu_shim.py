"""The C++ drop-in (qsfs-fuse_amd/host/qsfs_md5.hpp) on the GPU.

tests/cpp/test_shim.cpp uses the reference-shaped interface -- global
md5(std::string), md5(shared_ptr<iostream>) over a qsfs StreamBuf-style view,
class MD5 -- and prints one digest per case.  Each is checked against the
reference's own output where a committed fixture holds those bytes
(tests/golden/*.json, made by the reference's MD5.cpp: rfc1321, lcg_lengths,
stream_pieces) and against the pinned oracle (oracle/md5_oracle.c, itself
checked against every fixture by tests/test_oracle.py) for the rest
(no hashlib in a -m gpu assertion).  The binary also
asserts the reference's stream side effects (read position reset to 0,
MD5.cpp:343-346) and loud failure.
"""
import base64
import json
import os
import subprocess

import pytest

from conftest import ROOT
from oracle_util import lcg_bytes, md5_ref

BIN = os.path.join(ROOT, "tests", "cpp", "test_shim")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def build_shim():
    subprocess.check_call([
        "g++", "-std=c++17", "-O2", os.path.join(ROOT, "tests", "cpp", "test_shim.cpp"),
        "-I" + os.path.join(ROOT, "include"), "-L" + os.path.join(ROOT, "qsfs-fuse_amd", "lib"),
        "-lqsmd5", "-Wl,-rpath," + os.path.join(ROOT, "qsfs-fuse_amd", "lib"), "-o", BIN])


def _golden():
    """Reference-produced digests: RFC 1321 texts, LCG(12345) prefixes by length,
    the 200 000-byte LCG(4242) stream of the MD5 class cases."""
    rfc = {c["text"]: c["md5"] for c in json.load(open(os.path.join(GOLDEN, "rfc1321.json")))["cases"]}
    lcg = json.load(open(os.path.join(GOLDEN, "lcg_lengths.json")))
    assert lcg["generator"] == "lcg" and lcg["seed"] == 12345
    by_len = {c["len"]: c["md5"] for c in lcg["cases"]}
    sp = json.load(open(os.path.join(GOLDEN, "stream_pieces.json")))
    assert sp["seed"] == 4242 and sp["len"] == 200000
    whole = sp["cases"][0]
    assert whole["cuts"] == [200000]
    return rfc, by_len, whole["md5"]


def check_shim_output(out):
    assert out.returncode == 0, out.stdout + out.stderr
    got = dict(line.split() for line in out.stdout.strip().splitlines() if not line.startswith("parts_"))
    rfc, by_len, pieces_md5 = _golden()
    o = lambda b: md5_ref(b).hex()  # the pinned oracle, for bytes no fixture holds
    assert got["str_empty"] == rfc[""]
    assert got["str_abc"] == rfc["abc"]
    assert got["str_literal"] == rfc["message digest"]
    assert got["content_md5_abc"] == base64.b64encode(bytes.fromhex(rfc["abc"])).decode()
    for L in (0, 2, 55, 64, 10485760):  # view_L = the first L bytes of LCG(12345)
        assert got["view_%d" % L] == by_len[L], L
    assert got["streamtest_read1"] == o(b"01")
    assert got["stringstream_100000q"] == o(b"q" * 100000)
    assert got["class_pieces"] == pieces_md5
    assert got["class_ctor_abc"] == rfc["abc"]
    for i in range(6):
        assert got["batch_%d" % i] == o(bytes(lcg_bytes(500 + i, 1000 * i * i + 3 * i + 1))[:1000 * i * i + 3 * i])
    MiB = 1 << 20
    rows = [l.split() for l in out.stdout.splitlines() if l.startswith("parts_")]
    for fsz, sizes in ((25 * MiB + 3, [10 * MiB, 10 * MiB, 5 * MiB + 3]),
                       (21 * MiB, [10 * MiB, 11 * MiB // 2, 11 * MiB - 11 * MiB // 2])):
        mine = [r for r in rows if r[0].startswith("parts_%d_" % fsz)]
        assert [int(r[2]) for r in mine] == sizes, mine
        data = bytes(lcg_bytes(777, fsz))
        for r in mine:
            off, sz = int(r[1]), int(r[2])
            assert r[3] == o(data[off:off + sz]), r
    d = bytes(lcg_bytes(31337, 5000))
    assert got["copy_b"] == o(d)
    assert got["copy_a"] == o(d[:100] + b"x")
    assert got["copy_c"] == o(d + b"y")
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
