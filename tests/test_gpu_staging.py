"""Host staging across allocations: the GPUTEST_r01 illegal-memory-access case.

Round 1's driver run faulted the GPU in test_gpu_fuzz seed 0: equal-length
host chunks sitting in two different allocations (a pinned pool and a pageable
numpy pool) were sent as ONE hipMemcpy2DAsync whose source span ran from the
first allocation through unmapped memory into the second.  With a pinned first
row HIP reads that span by DMA, and the bytes between the allocations faulted.

The runtime now forms a 2-D copy only when the whole span lies inside one
allocation or mapping (qsmd5_plan.h plan_copy_runs; CPU-tested by
tests/cpp/test_plan.cpp).  These tests rebuild the failing shape on purpose,
deterministically: a pageable mapping placed at a chosen address above or
below a pinned buffer, with an unmapped gap between, so equal-length chunks in
the two sit at a constant positive stride across the gap.  Every digest is
checked against the oracle.
"""
import ctypes
import mmap
import os

import numpy as np
import pytest

import qsmd5
from oracle_util import md5_many

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

SIZE = 32 << 20
GAP = 2 << 20
LENGTHS = [55, 88, 4095, 4096, (256 << 10) + 7, 1 << 20]

_libc = ctypes.CDLL(None, use_errno=True)
_libc.mmap.restype = ctypes.c_void_p
_libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                       ctypes.c_long]
_libc.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
_libc.mprotect.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
MAP_FIXED_NOREPLACE = 0x100000
MAP_FAILED = ctypes.c_void_p(-1).value


def _map_at(addr, size):
    """Anonymous pageable mapping at exactly `addr`, or None."""
    p = _libc.mmap(addr, size, mmap.PROT_READ | mmap.PROT_WRITE,
                   mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS | MAP_FIXED_NOREPLACE, -1, 0)
    if p in (None, MAP_FAILED):
        return None
    if p != addr:  # an old kernel took it as a hint only
        _libc.munmap(p, size)
        return None
    return p


def _pageable_near(pinned, above):
    """A pageable mapping next to `pinned` with >= GAP unmapped bytes between."""
    # HIP packs its own mappings around pinned buffers and may reserve a large
    # range next to them: search densely up to 1 GiB away, then at doubling
    # distances up to 512 GiB (a 2-D run needs a stride below 2^40)
    offs = [SIZE + GAP * k for k in range(1, 512)] + [1 << j for j in range(31, 40)]
    for off in offs:
        addr = pinned + off if above else pinned - off
        addr &= ~(mmap.PAGESIZE - 1)
        if addr <= 0:
            continue
        p = _map_at(addr, SIZE)
        if p is not None:
            return p
    pytest.skip("no free address range next to the pinned buffer")


def _fill(ptr, seed):
    a = np.ctypeslib.as_array((ctypes.c_uint8 * SIZE).from_address(ptr))
    a[:] = np.random.default_rng(seed).integers(0, 256, size=SIZE, dtype=np.uint8)
    return a


@pytest.fixture
def pinned():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert qsmd5.lib().qsmd5_init(0) == 0
    p = qsmd5.alloc_pinned(SIZE)
    _fill(p, 1)
    yield p
    qsmd5.free_pinned(p)


def _pairs(lo, hi, L, off=1000):
    """Equal-length chunks whose lane order (by length, then address) has a
    constant stride that runs from the `lo` allocation across the unmapped gap
    into `hi`: rows at lo+off + k*D, D = (hi - lo) / 2, k = 0..3 (rows 0-1 in
    lo, rows 2-3 in hi).  A 2-D copy of all four rows would read the gap; the
    runtime must cut the run where `lo` ends.  Falls back to the two-row pair
    when the allocations are too far apart for the progression."""
    D = (hi - lo) // 2
    if off + D + L <= SIZE and (hi - lo) % 2 == 0:
        return [(lo + off + k * D, L) for k in range(4)]
    return [(lo + off, L), (hi + off, L)]


def _check(chunks, flags=0, column=None):
    if column is None:
        os.environ.pop("QSMD5_COLUMN_BYTES", None)
    else:
        os.environ["QSMD5_COLUMN_BYTES"] = str(column)
    try:
        got = qsmd5.hash_batch(chunks, flags=flags)
    finally:
        os.environ.pop("QSMD5_COLUMN_BYTES", None)
    assert got == md5_many(chunks)


@pytest.mark.parametrize("above", [True, False], ids=["pageable_above", "pageable_below"])
@pytest.mark.parametrize("flags", [0, qsmd5.FLAG_HOST], ids=["classified", "flag_host"])
def test_pinned_and_pageable_equal_lengths(pinned, above, flags):
    pg = _pageable_near(pinned, above)
    try:
        _fill(pg, 2)
        lo, hi = (pinned, pg) if above else (pg, pinned)
        for L in LENGTHS:
            chunks = [(lo + 1000, L), (hi + 1000, L)]  # the seed-0 pair
            _check(chunks, flags)
            _check(_pairs(lo, hi, L), flags)
            # column-staged: every column of the pair is a cross-allocation run
            _check(_pairs(lo, hi, L), flags, column=1024)
    finally:
        _libc.munmap(pg, SIZE)


def test_two_pinned_pools(pinned):
    other = qsmd5.alloc_pinned(SIZE)
    try:
        _fill(other, 3)
        lo, hi = sorted([pinned, other])
        for L in LENGTHS:
            _check(_pairs(lo, hi, L))
            _check(_pairs(lo, hi, L), qsmd5.FLAG_HOST, column=4160)
    finally:
        qsmd5.free_pinned(other)


def test_two_pageable_mappings_with_a_gap(pinned):
    """Two pageable mappings with an unmapped hole between them, carved out of
    one reservation so the layout does not depend on the address space (the
    four-row progression of _pairs always fits here)."""
    span = 2 * SIZE + GAP
    res = _libc.mmap(None, span, 0,  # PROT_NONE
                     mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS, -1, 0)
    assert res not in (None, MAP_FAILED)
    a, b = res, res + SIZE + GAP
    try:
        assert _libc.munmap(res + SIZE, GAP) == 0  # the hole
        for p in (a, b):
            assert _libc.mprotect(p, SIZE, mmap.PROT_READ | mmap.PROT_WRITE) == 0
        _fill(a, 4)
        _fill(b, 5)
        for L in LENGTHS:
            _check(_pairs(a, b, L))
            _check(_pairs(a, b, L), qsmd5.FLAG_HOST, column=1024)
    finally:
        _libc.munmap(a, SIZE)
        _libc.munmap(b, SIZE)


def test_file_parts_in_one_buffer_still_one_run(pinned):
    """The fast path stays: a file's equal parts in one pinned buffer (a single
    allocation) still go as 2-D runs and hash correctly, whole and in columns."""
    L = (1 << 20) + 64
    chunks = [(pinned + i * L, L) for i in range(SIZE // L)]
    _check(chunks)
    _check(chunks, column=256 << 10)


@pytest.mark.parametrize("gather", ["1", "0"])
@pytest.mark.parametrize("column", [None, 1024, 4160])
def test_gather_kernel_rows_from_pinned_buffers(pinned, gather, column, monkeypatch):
    """Rows that cannot share a 2-D copy and sit in pinned memory are read by
    qsmd5_gather_kernel (one launch per slice; QSMD5_GATHER=0 sends them back
    to one DMA copy each).  16-B-aligned starts with every tail length 0..15,
    rows shorter than 16 B, and separate pinned allocations."""
    monkeypatch.setenv("QSMD5_GATHER", gather)
    others = [qsmd5.alloc_pinned(1 << 20) for _ in range(3)]
    try:
        for i, o in enumerate(others):
            _fill_n(o, 1 << 20, 10 + i)
        chunks = []
        for i, L in enumerate([1, 15, 16, 17, 31, 4096 + 5, 65536 + 15, 300000 + 7]):
            base = others[i % 3] if i % 2 else pinned
            chunks.append((base + 16 * (1 + 7 * i), L))  # 16-B aligned, irregular spacing
        chunks += [(o + 16 * 5, 200003) for o in others]  # equal lengths, separate allocations
        _check(chunks, column=column)
    finally:
        for o in others:
            qsmd5.free_pinned(o)


def _fill_n(ptr, n, seed):
    a = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(ptr))
    a[:] = np.random.default_rng(seed).integers(0, 256, size=n, dtype=np.uint8)


def test_gather_from_registered_pageable_buffers(pinned):
    """Pageable buffers registered with qsmd5_register_host are HIP-known host
    memory: rows in separate registered buffers take the gather kernel."""
    bufs = [np.zeros(SIZE // 4, dtype=np.uint8) for _ in range(3)]
    for i, b in enumerate(bufs):
        b[:] = np.random.default_rng(40 + i).integers(0, 256, size=b.size, dtype=np.uint8)
        qsmd5.register_host(b.ctypes.data, b.nbytes)
    try:
        L = (1 << 20) + 9
        chunks = [(b.ctypes.data + 16 * k, L) for k in range(2) for b in bufs]
        _check(chunks)
        _check(chunks, column=4160)
    finally:
        for b in bufs:
            qsmd5.unregister_host(b.ctypes.data)


def test_register_buffers_sharing_a_page():
    """Registration covers whole 4 KiB pages.  Adjacent heap
    buffers share a boundary page; a pool registers them one by one.  Either
    both registrations succeed and both buffers hash correctly through the
    gather path, or the second fails with -EINVAL naming the shared page --
    never a generic -EIO.  A second range starting in the first page of a
    registered one, or the same pointer twice, is -EINVAL."""
    import errno
    blk = np.zeros(6 * 4096, dtype=np.uint8)
    blk[:] = np.random.default_rng(77).integers(0, 256, size=blk.size, dtype=np.uint8)
    base = (blk.ctypes.data + 4095) & ~4095
    a, la = base + 96, 2 * 4096 - 96 - 1000      # ends inside page 1
    b, lb = a + la, 2 * 4096 + 1000 - 16          # starts in page 1, right after a
    qsmd5.register_host(a, la)
    try:
        with pytest.raises(qsmd5.Md5Error) as e:
            qsmd5.register_host(base + 8, 16)     # starts in a's first page
        assert e.value.code == -errno.EINVAL
        with pytest.raises(qsmd5.Md5Error) as e:
            qsmd5.register_host(a, 16)            # the same pointer twice
        assert e.value.code == -errno.EINVAL
        try:
            qsmd5.register_host(b, lb)
            b_ok = True
        except qsmd5.Md5Error as e2:
            assert e2.code == -errno.EINVAL and "shares a page" in str(e2)
            b_ok = False
        print("shared-page registration accepted by HIP: %s" % b_ok)
        _check([(a, la), (b, lb)] if b_ok else [(a, la)])
        if b_ok:
            qsmd5.unregister_host(b)
    finally:
        qsmd5.unregister_host(a)


@pytest.mark.parametrize("column", [None, 1024])
def test_shared_page_survives_unregistering_its_first_owner(column):
    """two registrations share a boundary page; the FIRST one (a)
    is unregistered while the second (b) is still registered, and b -- whose
    first page is the shared one -- is then hashed through the gather kernel
    (a 16-B-aligned row in a registered allocation of its own) against the
    oracle, before b is unregistered too.  A page unpinned or unmapped with a
    would fault the gather kernel or hash stale bytes here."""
    blk = np.zeros(128 * 4096, dtype=np.uint8)
    blk[:] = np.random.default_rng(78).integers(0, 256, size=blk.size, dtype=np.uint8)
    base = (blk.ctypes.data + 4095) & ~4095
    a, la = base + 96, 2 * 4096 - 96 - 1024       # ends inside page 1, at a 16-B boundary
    b, lb = a + la, 100 * 4096 + 1000             # starts in page 1, right after a; with the
    #                                               other rows > 256 KiB: staged, not inline
    assert b % 16 == 0
    qsmd5.register_host(a, la)
    try:
        qsmd5.register_host(b, lb)
    except qsmd5.Md5Error as e:
        qsmd5.unregister_host(a)
        pytest.skip("HIP refused the shared-page registration (-EINVAL path): %s" % e)
    a_done = False
    try:
        qsmd5.unregister_host(a)
        a_done = True
        other = qsmd5.alloc_pinned(1 << 16)       # a second row in its own allocation
        try:
            _fill_n(other, 1 << 16, 79)
            chunks = [(b, lb), (other, 5000), (b + 16, lb - 16)]
            for _ in range(2):
                _check(chunks, column=column)
            blk[b - base:b - base + 64] ^= 0x5a  # the shared page changes: no stale copy
            _check(chunks, column=column)
        finally:
            qsmd5.free_pinned(other)
    finally:
        qsmd5.unregister_host(b)
        if not a_done:
            qsmd5.unregister_host(a)
