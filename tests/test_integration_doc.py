"""INTEGRATION.md §3's DoMultiPartUpload binding compiles and works as printed.

The §3 code block that starts with `#include "qsfs_multipart.hpp"` is cut in
two: the pool adapter (namespace scope) and the loop that replaces the
reference's part loop (QSTransferManager.cpp:602-673).  Both are compiled,
unedited but for one line -- the loop's `parts` vector, which the snippet says
comes "from handle->GetQueuedParts(), in part order", is initialised from the
harness's plan -- into tests/cpp/integration_doctest.cpp, whose test doubles
give them the interfaces they name.  Runs on the library's CPU backend: every
part handed on must carry the MD5 of its bytes, every part not sent (the
transfer cancelled) must be marked failed, and the pool must be full again."""
import json
import os
import re
import subprocess

import pytest

from conftest import ROOT

MiB = 1 << 20


def snippet_pieces():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text[text.index("## 3. Batch pre-hash"):text.index("## 4. ")]
    blocks = re.findall(r"```cpp\n(.*?)```", sec, re.S)
    block = [b for b in blocks if b.startswith('#include "qsfs_multipart.hpp"')]
    assert len(block) == 1, "INTEGRATION.md §3 must hold exactly one binding block"
    block = block[0]
    cut = block.index("// QSTransferManager::DoMultiPartUpload, replacing the part loop")
    adapter, loop = block[:cut], block[cut:]
    parts_line = re.findall(r"^std::vector<qsmd5_part> parts;.*$", loop, re.M)
    assert len(parts_line) == 1, loop
    loop = loop.replace(parts_line[0], "std::vector<qsmd5_part> parts = queued;  // " + parts_line[0])
    return adapter, loop


@pytest.fixture(scope="module")
def doctest_exe(tmp_path_factory):
    d = tmp_path_factory.mktemp("integration_doc")
    adapter, loop = snippet_pieces()
    (d / "adapter.inc").write_text(adapter)
    (d / "loop.inc").write_text(loop)
    exe = str(d / "integration_doctest")
    subprocess.check_call([
        "g++", "-std=c++17", "-O1", "-Wall", "-Wno-unused-variable",
        '-DINTEGRATION_ADAPTER="%s"' % (d / "adapter.inc"), '-DINTEGRATION_LOOP="%s"' % (d / "loop.inc"),
        os.path.join(ROOT, "tests", "cpp", "integration_doctest.cpp"),
        "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "qsfs-fuse_amd", "host"),
        "-L" + os.path.join(ROOT, "qsfs-fuse_amd", "lib"), "-lqsmd5", "-lpthread",
        "-Wl,-rpath," + os.path.join(ROOT, "qsfs-fuse_amd", "lib"), "-o", exe])
    return exe


@pytest.mark.parametrize("flush", ["async", "sync"])
@pytest.mark.parametrize("cancel_after", [-1, 0, 1, 7, 12, 100],
                         ids=["whole_file", "cancelled_first", "after_1", "after_7", "after_12", "never"])
def test_binding_as_printed(doctest_exe, cancel_after, flush):
    """async: File::Flush handed the upload to the executor (no lock held);
    sync: the flushing thread holds the file's lock through the upload
    (single-thread mode, File::Truncate) and the binding must not read from
    its helper thread.  12 x 4 MiB + 1234 B: 13 parts, the last two averaged
    (PrepareUpload, :517-542); 66 parts at 2 MiB, more than one wave."""
    env = dict(os.environ, QSMD5_BACKEND="cpu")
    for fsz, psz, nparts in ((12 * 4 * MiB + 1234, 4 * MiB, 13), (132 * MiB, 2 * MiB, 66)):
        out = subprocess.run([doctest_exe, str(fsz), str(psz), "5", str(cancel_after), flush],
                             env=env, capture_output=True, text=True, timeout=120)
        assert out.returncode == 0, out.stdout + out.stderr[-3000:]
        r = json.loads(out.stdout.strip().splitlines()[-1])
        sent = nparts if cancel_after < 0 else min(nparts, cancel_after)
        assert r == {"parts": nparts, "sent": sent, "failed": nparts - sent, "pool_free": 5, "bad": 0,
                     "deadlock": False}, r


@pytest.mark.parametrize("flush", ["async", "sync"])
def test_write_during_the_upload_rehashes_the_part(doctest_exe, flush):
    """Another descriptor writes the part after the next to go out once 2
    parts went out (part 4 of the first wave of 4, pre-hashed before the
    uploads began; the next one may already be read ahead): the stored
    digest of that part no longer matches its bytes, so the
    binding (source_changed over File's write counter) re-hashes it from its
    buffer; every Content-MD5 the SDK gets is the MD5 of the bytes it gets."""
    env = dict(os.environ, QSMD5_BACKEND="cpu")
    out = subprocess.run([doctest_exe, str(132 * MiB), str(2 * MiB), "5", "-1", flush, "2"],
                         env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr[-3000:]
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["sent"] == 66 and r["bad"] == 0, r


def test_write_during_the_upload_negative_control(tmp_path):
    """The same binding with its source_changed line taken out: the part
    written mid-upload goes out with the pre-hash's stale digest, and the
    doctest sees it (exit 1)."""
    adapter, loop = snippet_pieces()
    lines = [ln for ln in loop.splitlines() if ln.startswith("opt.source_changed")]
    assert len(lines) == 1, loop
    (tmp_path / "adapter.inc").write_text(adapter)
    (tmp_path / "loop.inc").write_text(loop.replace(lines[0], "// " + lines[0]))
    exe = str(tmp_path / "integration_doctest_nc")
    subprocess.check_call([
        "g++", "-std=c++17", "-O1", "-Wall", "-Wno-unused-variable", "-Wno-unused-but-set-variable",
        '-DINTEGRATION_ADAPTER="%s"' % (tmp_path / "adapter.inc"), '-DINTEGRATION_LOOP="%s"' % (tmp_path / "loop.inc"),
        os.path.join(ROOT, "tests", "cpp", "integration_doctest.cpp"),
        "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "qsfs-fuse_amd", "host"),
        "-L" + os.path.join(ROOT, "qsfs-fuse_amd", "lib"), "-lqsmd5", "-lpthread",
        "-Wl,-rpath," + os.path.join(ROOT, "qsfs-fuse_amd", "lib"), "-o", exe])
    env = dict(os.environ, QSMD5_BACKEND="cpu")
    out = subprocess.run([exe, str(132 * MiB), str(2 * MiB), "5", "-1", "async", "2"],
                         env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 1 and "MD5 of the bytes sent" in out.stderr, (out.returncode, out.stderr[-2000:])


def test_sync_flush_without_the_flag_deadlocks(doctest_exe):
    """The negative control: the flushing thread holds the file's lock, as
    File::Flush's synchronous branch does, but the binding is not told -- its
    pipeline's helper thread blocks in ReadNoLoad while the flushing thread
    waits for it.  The doctest's watchdog reports the deadlock (exit 3)."""
    env = dict(os.environ, QSMD5_BACKEND="cpu")
    out = subprocess.run([doctest_exe, str(132 * MiB), str(2 * MiB), "5", "-1", "sync_unflagged"],
                         env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 3 and '"deadlock": true' in out.stdout, (out.returncode, out.stdout)


def test_log_sink_binding_as_printed(tmp_path):
    """INTEGRATION.md §2's log sink (qsmd5_set_log_callback into qsfs's
    DebugInfo / DebugWarning / DebugError) compiles as printed, and a hashing
    call's backend line reaches DebugInfo (CPU backend, no GPU needed)."""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text[text.index("**The backend in qsfs's own log**"):text.index("## 3. Batch pre-hash")]
    block = re.findall(r"```cpp\n(.*?)```", sec, re.S)[0]
    lines = [ln for ln in block.splitlines() if not ln.startswith("#include")]
    reg = [ln for ln in lines if ln.startswith("qsmd5_set_log_callback(")]
    assert len(reg) == 1, block
    fn = "\n".join(ln for ln in lines if ln not in reg)
    (tmp_path / "fn.inc").write_text(fn + "\n")
    (tmp_path / "reg.inc").write_text(reg[0] + "\n")
    exe = str(tmp_path / "log_doctest")
    subprocess.check_call([
        "g++", "-std=c++17", "-O1", "-Wall",
        '-DLOG_SINK_FUNCTION="%s"' % (tmp_path / "fn.inc"), '-DLOG_SINK_REGISTRATION="%s"' % (tmp_path / "reg.inc"),
        os.path.join(ROOT, "tests", "cpp", "integration_log_doctest.cpp"),
        "-I" + os.path.join(ROOT, "include"), "-L" + os.path.join(ROOT, "qsfs-fuse_amd", "lib"), "-lqsmd5",
        "-Wl,-rpath," + os.path.join(ROOT, "qsfs-fuse_amd", "lib"), "-o", exe])
    env = dict(os.environ, QSMD5_BACKEND="cpu")
    out = subprocess.run([exe], env=env, capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    assert "I qsmd5: backend=cpu reason=forced chunks=1 bytes=3" in out.stdout.splitlines(), out.stdout
    assert out.stderr == "", out.stderr  # the sink takes every line
