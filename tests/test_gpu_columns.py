"""Column-pipelined staging of host-resident batches (qsmd5_rt_staging.cpp run_batch,
qsmd5_column_pc_kernel) on an MI355X.

A host batch is cut into columns of W bytes per chunk; each column is one H2D
transfer plus one launch that resumes every chain from its parked state.  These
tests force tiny and odd column widths (QSMD5_COLUMN_BYTES) so that every chunk
crosses many column boundaries, chunks end inside, at and just past a column,
groups shrink column by column, and both copy forms run (one 2-D copy for a
run of equal parts at a constant stride, per-chunk copies otherwise).  Every
digest is checked bit-exactly against the reference-generated fixtures or the
CPU oracle.
"""
import ctypes
import os

import pytest

import qsmd5
from oracle_util import lcg_bytes, md5_many, md5_ref

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu
MiB = 1 << 20


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert qsmd5.lib().qsmd5_init(0) == 0
    yield
    os.environ.pop("QSMD5_COLUMN_BYTES", None)


@pytest.fixture
def columns():
    def set_width(w):
        if w is None:
            os.environ.pop("QSMD5_COLUMN_BYTES", None)
        else:
            os.environ["QSMD5_COLUMN_BYTES"] = str(w)
    yield set_width
    os.environ.pop("QSMD5_COLUMN_BYTES", None)


def hexes(ds):
    return [d.hex() for d in ds]


@pytest.mark.parametrize("width,maxlen", [(64, 8192), (192, 16384), (4096, MiB + 1),
                                          (65536 + 64, 64 * MiB), (MiB, 64 * MiB)])
def test_lcg_lengths_forced_columns(golden, columns, width, maxlen):
    """Every padding edge (lengths around 55/56/64, up to `maxlen`) with the
    message split at `width`-byte column boundaries; overlapping chunks (all at
    the same base) take the per-chunk copy path."""
    g = golden("lcg_lengths.json")
    cases = [c for c in g["cases"] if c["len"] <= maxlen]
    data = lcg_bytes(12345, max(c["len"] for c in cases))
    base = ctypes.addressof(data)
    columns(width)
    got = qsmd5.hash_batch([(base, c["len"]) for c in cases])
    assert hexes(got) == [c["md5"] for c in cases]


@pytest.mark.parametrize("width", [64, 4096, 3 * 65536])
@pytest.mark.parametrize("pinned", [False, True])
def test_file_parts_two_d_runs(columns, width, pinned):
    """A file's upload parts (equal parts at a constant stride, short last part):
    one 2-D copy per column for the run, a plain copy for the last part.  The
    file starts at an odd address, so the host rows are unaligned."""
    size = 37 * 65536 + 4321
    part = 65536 * 2 + 640
    src = bytes(lcg_bytes(99, size))
    if pinned:
        p = qsmd5.alloc_pinned(size + 8)
        keep = None
    else:
        keep = ctypes.create_string_buffer(size + 8)
        p = ctypes.addressof(keep)
    try:
        base = p + 3
        ctypes.memmove(base, src, size)
        chunks = [(base + o, min(part, size - o)) for o in range(0, size, part)]
        want = [md5_ref(src[o:o + L]) for o, L in ((c[0] - base, c[1]) for c in chunks)]
        columns(width)
        assert qsmd5.hash_batch(chunks) == want
    finally:
        if pinned:
            qsmd5.free_pinned(p)


def test_ragged_host_forced_columns(golden, columns):
    """The reference-generated ragged batch (659 chunks, 0 B .. 63.65 MiB) from
    pinned host memory with 1 MiB columns: the active prefix of the group
    shrinks column by column down to the single longest chunk."""
    g = golden("ragged.json")
    lens = g["lengths"]
    offs, pos = [], 0
    for L in lens:
        offs.append(pos)
        pos += (L + 255) & ~255
    t = torch.empty(pos + 256, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for i, (o, L) in enumerate(zip(offs, lens)):
        qsmd5.synth_fill_lcg(t.data_ptr() + o, 0, L, 7000 + i, 1, s)
    torch.cuda.synchronize()
    p = qsmd5.alloc_pinned(pos + 256)
    try:
        host = torch.from_numpy(
            __import__("numpy").ctypeslib.as_array((ctypes.c_uint8 * (pos + 256)).from_address(p)))
        host.copy_(t.cpu())
        del t
        columns(MiB)
        got = qsmd5.hash_batch([(p + o, L) for o, L in zip(offs, lens)])
        assert hexes(got) == g["md5"]
        columns(0)  # whole-chunk row slices, same answer
        assert hexes(qsmd5.hash_batch([(p + o, L) for o, L in zip(offs, lens)])) == g["md5"]
    finally:
        qsmd5.free_pinned(p)


def test_mixed_device_and_host_with_columns(columns):
    """Device chunks (one launch) and column-staged host chunks in one batch."""
    host = lcg_bytes(5, 3 * MiB)
    hb = ctypes.addressof(host)
    dev = torch.frombuffer(bytearray(bytes(host)), dtype=torch.uint8).cuda()
    spans = [(0, 3 * MiB), (7, 2 * MiB + 13), (64, 64), (100, 0), (1, 1234567), (5, 55)]
    chunks, ref = [], []
    for i, (o, L) in enumerate(spans):
        on_dev = i % 2 == 1
        chunks.append(((dev.data_ptr() if on_dev else hb) + o, L))
        ref.append((hb + o, L))
    columns(4096 + 64)
    assert qsmd5.hash_batch(chunks) == md5_many(ref)


def test_pinned_batch_automatic_columns(golden, columns):
    """The planner's own choice: 96 x 10 MiB pinned (960 MiB) gets ~5 MiB
    columns; every digest vs the reference-generated fixture."""
    columns(None)
    g = golden("batch_10MiB.json")
    n, L = 96, g["len"]
    p = qsmd5.alloc_pinned(n * L)
    try:
        t = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        qsmd5.synth_fill_lcg(t.data_ptr(), L, L, 12345, n, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        ctypes.memmove(p, bytes(t.cpu().numpy()), n * L)
        del t
        got = qsmd5.hash_batch([(p + i * L, L) for i in range(n)])
        assert hexes(got) == g["md5"][:n]
        # scattered (reversed) order: no constant stride, per-chunk copies
        got = qsmd5.hash_batch([(p + (n - 1 - i) * L, L) for i in range(n)])
        assert hexes(got) == g["md5"][:n][::-1]
    finally:
        qsmd5.free_pinned(p)


def test_config3_pinned_4096_columns(golden, columns):
    """BASELINE config 3 in full: 4096 x 10 MiB (40 GiB) in pinned host memory,
    automatic columns, all 4096 digests vs the fixture."""
    import numpy as np
    columns(None)
    g = golden("batch_10MiB.json")
    n, L = 4096, g["len"]
    p = qsmd5.alloc_pinned(n * L)
    try:
        host = np.ctypeslib.as_array((ctypes.c_uint8 * (n * L)).from_address(p))
        step = 256
        buf = torch.empty(step * L, dtype=torch.uint8, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        for k in range(0, n, step):
            qsmd5.synth_fill_lcg(buf.data_ptr(), L, L, 12345 + k, step, s)
            torch.from_numpy(host[k * L:(k + step) * L]).copy_(buf)
        torch.cuda.synchronize()
        del buf
        got = qsmd5.hash_batch([(p + i * L, L) for i in range(n)])
        assert hexes(got) == g["md5"][:n]
    finally:
        qsmd5.free_pinned(p)


def test_columns_beyond_one_resident_round(columns):
    """A host batch of > 16 384 chunks cut into columns runs the column kernel
    with the 64 KiB ring (two workgroups per CU, qsmd5_column_pc2_kernel)."""
    import random
    rng = random.Random(17)
    n = 18000
    data = lcg_bytes(99, 2 * MiB)
    base = ctypes.addressof(data)
    spans = [(rng.randrange(0, MiB), rng.randrange(0, 3000)) for _ in range(n)]
    want = md5_many([(base + o, L) for o, L in spans])
    columns(1024)
    assert qsmd5.hash_batch([(base + o, L) for o, L in spans]) == want
