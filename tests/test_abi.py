"""Host-side checks of the C-ABI library (no GPU needed).

- libqsmd5.so loads and exports every function include/qsmd5.h declares;
- qsmd5_hex reproduces MD5::hexdigest (MD5.cpp:317-325);
- qsmd5_plan_parts reproduces QSTransferManager::PrepareUpload slicing
  (QSTransferManager.cpp:475-550), checked against the worked examples in
  SURVEY.md §8(a) and a direct restatement of the reference's arithmetic;
- without a GPU every hashing entry point fails loudly with -ENODEV (no CPU
  fallback exists in the product path).
"""
import ctypes
import errno
import os
import random
import re
import subprocess

import pytest

import qsmd5
from conftest import ROOT

MiB = 1 << 20
GiB = 1 << 30


def declared_functions():
    text = open(os.path.join(ROOT, "include", "qsmd5.h")).read()
    return sorted(set(re.findall(r"QSMD5_API\s+[\w\s\*]+?\b(qsmd5_\w+)\s*\(", text)))


def test_header_declares_expected_surface():
    names = declared_functions()
    for must in ["qsmd5_init", "qsmd5_hash_one", "qsmd5_hash_batch", "qsmd5_hash_batch_device_async",
                 "qsmd5_hex", "qsmd5_ctx_create", "qsmd5_ctx_update", "qsmd5_ctx_final",
                 "qsmd5_ctx_destroy", "qsmd5_alloc_pinned", "qsmd5_free_pinned",
                 "qsmd5_plan_parts", "qsmd5_hash_parts"]:
        assert must in names


def test_library_exports_every_declared_symbol():
    so = qsmd5.lib_path()
    L = ctypes.CDLL(so)
    for name in declared_functions():
        assert hasattr(L, name), name
    out = subprocess.check_output(["nm", "-D", "--defined-only", so]).decode()
    exported = set(re.findall(r" T (\w+)", out))
    assert set(declared_functions()) == {s for s in exported if s.startswith("qsmd5_")}
    # nothing but the C-ABI leaks (kernel stubs and launchers stay hidden)
    assert not [s for s in exported if "device_stub" in s or "launch_" in s]


def test_flags_match_header():
    """The binding's FLAG_* constants are the header's QSMD5_FLAG_* values."""
    text = open(os.path.join(ROOT, "include", "qsmd5.h")).read()
    flags = dict(re.findall(r"#define QSMD5_FLAG_(\w+)\s+(\d+)", text))
    assert set(flags) >= {"NONE", "REF_TRUNCATE32", "ALIGNED16", "HOST"}
    for name, val in flags.items():
        if name != "NONE":
            assert getattr(qsmd5, "FLAG_" + name) == int(val), name
    vals = [int(v) for k, v in flags.items() if k != "NONE"]
    assert all(v & (v - 1) == 0 for v in vals) and len(set(vals)) == len(vals)  # distinct bits


def test_abi_version():
    assert qsmd5.lib().qsmd5_abi_version() == 1


def test_hex_matches_reference_format():
    rng = random.Random(3)
    for _ in range(100):
        d = bytes(rng.getrandbits(8) for _ in range(16))
        assert qsmd5.hexdigest(d) == "".join("%02x" % b for b in d)
    assert qsmd5.hexdigest(b"\x00" * 16) == "0" * 32
    assert qsmd5.hexdigest(b"\xff" * 16) == "f" * 32


def test_base64_content_md5_header():
    """RFC 1864 header form, checked against Python's base64 and RFC 1864's own
    example digest (MD5 of "Check Integrity!" = Q2hlY2sgSW50ZWdyaXR5IQ==)."""
    import base64
    rng = random.Random(4)
    for _ in range(200):
        d = bytes(rng.getrandbits(8) for _ in range(16))
        assert qsmd5.content_md5(d) == base64.b64encode(d).decode()
    assert qsmd5.content_md5(b"Check Integrity!") == "Q2hlY2sgSW50ZWdyaXR5IQ=="
    # the digest of "" (RFC 1321 A.5) in header form
    assert qsmd5.content_md5(bytes.fromhex("d41d8cd98f00b204e9800998ecf8427e")) == \
        "1B2M2Y8AsgTpgAmY7PhCfg=="


def prepare_upload_restated(total, buf, min_part, threshold):
    """Direct restatement of QSTransferManager::PrepareUpload (QSTransferManager.cpp:492-546)."""
    if total < threshold:
        return [(1, 0, total)]
    part_count = -(-total // buf)  # ceil(total / buf), exact for integers
    last = total - (part_count - 1) * buf
    avg = last < min_part
    count = part_count - 1 if avg else part_count
    parts = [(i, (i - 1) * buf, buf) for i in range(1, count)]
    if not avg:
        parts.append((part_count, (part_count - 1) * buf, last))
    else:
        sz1 = (last + buf) // 2
        sz2 = last + buf - sz1
        parts.append((count, (count - 1) * buf, sz1))
        parts.append((part_count, (count - 1) * buf + sz1, sz2))
    return parts


def plan(total, **kw):
    return [p.astuple() for p in qsmd5.plan_parts(total, **kw)]


def test_plan_parts_survey_examples():
    # 25 MiB -> [10,10,5]; 21 MiB -> [10, 5.5, 5.5]; 100 GiB -> 10240 x 10 MiB
    assert [s for _, _, s in plan(25 * MiB)] == [10 * MiB, 10 * MiB, 5 * MiB]
    p21 = plan(21 * MiB)
    assert [s for _, _, s in p21] == [10 * MiB, 11 * MiB // 2, 11 * MiB // 2]
    assert [n for n, _, _ in p21] == [1, 2, 3]
    p100 = plan(100 * GiB)
    assert len(p100) == 10240 and all(s == 10 * MiB for _, _, s in p100)
    assert plan(19 * MiB) == [(1, 0, 19 * MiB)]  # below the 20 MiB threshold: PutObject
    assert plan(0) == [(1, 0, 0)]
    # odd remainder: the averaged pair must not lose the last byte
    p = plan(20 * MiB + 3)
    assert sum(s for _, _, s in p) == 20 * MiB + 3


def test_plan_parts_matches_restatement_random():
    rng = random.Random(11)
    for _ in range(400):
        buf = rng.choice([1, 2, 4, 8, 10, 16, 32, 64]) * MiB
        total = rng.choice([rng.randrange(0, 200 * MiB), rng.randrange(0, 8 * GiB),
                            20 * MiB + rng.randrange(-3, 4)])
        want = prepare_upload_restated(total, buf, 4 * MiB, 20 * MiB)
        got = plan(total, buf_size=buf)
        if want and want[0][0] == 0:  # degenerate averaging with a single part
            continue
        assert got == want, (total, buf)
        assert sum(s for _, _, s in got) == total
        off = 0
        for _, o, s in got:
            assert o == off
            off += s


def test_plan_parts_range_begin_and_capacity():
    p = plan(25 * MiB, range_begin=1000)
    assert [o for _, o, _ in p] == [1000, 1000 + 10 * MiB, 1000 + 20 * MiB]
    L = qsmd5.lib()
    need = ctypes.c_size_t()
    arr = (qsmd5.Part * 1)()
    rc = L.qsmd5_plan_parts(25 * MiB, 10 * MiB, 4 * MiB, 20 * MiB, 0, arr, 1, ctypes.byref(need))
    assert rc == -errno.EINVAL and need.value == 3
    assert L.qsmd5_plan_parts(5, 0, 0, 0, 0, None, 0, ctypes.byref(need)) == -errno.EINVAL


def test_plan_parts_refuses_more_than_uint16_part_ids():
    """The reference's Part id is uint16_t (TransferHandle.h:50; map key :45):
    a 70 000-part plan would wrap at part 65 536 and collide with part 1.
    qsmd5_plan_parts refuses it with -EINVAL and the count; 65 535 parts, the
    most the reference can number, plan exactly as the restatement says."""
    L = qsmd5.lib()
    need = ctypes.c_size_t()
    total = 70000 * MiB  # 70 000 parts of 1 MiB (qsfs -b 1)
    rc = L.qsmd5_plan_parts(total, MiB, 4 * MiB, 20 * MiB, 0, None, 0, ctypes.byref(need))
    assert rc == -errno.EINVAL and need.value == 70000
    assert b"uint16_t" in L.qsmd5_last_error()
    with pytest.raises(qsmd5.Md5Error):
        qsmd5.plan_parts(total, buf_size=MiB)
    edge = 65535 * MiB
    got = plan(edge, buf_size=MiB)
    assert got == prepare_upload_restated(edge, MiB, 4 * MiB, 20 * MiB)
    assert len(got) == 65535 and got[-1][0] == 65535
    with pytest.raises(qsmd5.Md5Error):
        qsmd5.plan_parts(edge + 1, buf_size=MiB)  # 65 536 parts (the averaged tail keeps the id)


def test_shutdown_idempotent_without_gpu():
    """qsmd5_shutdown with nothing to release returns 0, twice; without a GPU
    an init after it fails with -ENODEV again (the failed state was reset)."""
    L = qsmd5.lib()
    assert L.qsmd5_shutdown() == 0
    assert L.qsmd5_shutdown() == 0
    if qsmd5.device_count() == 0:
        assert L.qsmd5_init(0) == -errno.ENODEV
        assert L.qsmd5_shutdown() == 0
        assert L.qsmd5_init(0) == -errno.ENODEV


def test_kernel_choice_policy_host_only(monkeypatch):
    """The kernel selection is host logic (no GPU): latency kernel up to 16 384
    chunks, its 64 KiB-ring form up to 32 768, then the coalesced kernel for
    16-B-aligned chunks or the one-wave kernel; QSMD5_KERNEL overrides."""
    monkeypatch.delenv("QSMD5_KERNEL", raising=False)
    A = qsmd5.FLAG_ALIGNED16
    assert [qsmd5.kernel_choice(n) for n in (1, 512, 16384, 16385, 32768, 32769)] == [1, 1, 1, 3, 3, 0]
    assert qsmd5.kernel_choice(32769, A) == 2 and qsmd5.kernel_choice(512, A) == 1
    for name, want, want_aligned in (("pc", 1, 1), ("pc2", 3, 3), ("v1", 0, 0), ("coal", 0, 2)):
        monkeypatch.setenv("QSMD5_KERNEL", name)
        assert qsmd5.kernel_choice(100) == want and qsmd5.kernel_choice(100, A) == want_aligned


def test_strerror():
    L = qsmd5.lib()
    assert L.qsmd5_strerror(0) == b"success"
    assert L.qsmd5_strerror(-errno.ENODEV) == b"no usable GPU"


def test_no_gpu_fails_loudly():
    if qsmd5.device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(qsmd5.Md5Error) as e:
        qsmd5.hash_one(b"abc")
    assert e.value.code == -errno.ENODEV
    with pytest.raises(qsmd5.Md5Error):
        qsmd5.hash_batch([b"abc", b"def"])
    with pytest.raises(qsmd5.Md5Error):
        qsmd5.MD5("abc")


def test_etag_matching_rules():
    """Single-part ETag = the MD5 hex, optionally quoted; multipart ETags are refused."""
    import hashlib
    d = hashlib.md5(b"qsfs").digest()
    h = d.hex()
    assert qsmd5.etag_matches(d, h)
    assert qsmd5.etag_matches(d, '"%s"' % h)
    assert qsmd5.etag_matches(d, h.upper())
    assert not qsmd5.etag_matches(d, "0" * 32)
    for bad in ["", '""', h[:31], h + "0", '"%s-3"' % h, "g" * 32, "%s-12" % h[:29]]:
        with pytest.raises(qsmd5.Md5Error) as e:
            qsmd5.etag_matches(d, bad)
        assert e.value.code == -errno.EINVAL


BOOST = "/root/reference/third_party/boost_1_49_0"


@pytest.mark.skipif(not os.path.isdir(BOOST), reason="reference boost headers not present")
def test_dropin_compiles_with_boost_shared_ptr(tmp_path):
    """qsfs passes boost::shared_ptr<std::iostream>; the drop-in template must take it."""
    src = os.path.join(ROOT, "tests", "cpp", "compile_boost_shim.cpp")
    subprocess.check_call(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Wextra", "-w",
                           "-I" + BOOST, src])


def test_integration_maps_every_entry_point():
    """INTEGRATION.md §0 names every function the header declares (and what it
    replaces in the reference); `name`, `_ex` is the table's shorthand."""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    table = text[text.index("## 0. Entry-point map"):text.index("## 1. Build and link")]
    missing = []
    for name in declared_functions():
        short = name[:-3] if name.endswith("_ex") else None
        if "`%s`" % name in table:
            continue
        if short and "`%s`, `_ex`" % short in table:
            continue
        missing.append(name)
    assert not missing, missing
