"""qsmd5_hash_read -- the pull-driven batch behind the multipart pre-hash --
on the library's CPU backend (no GPU needed).

The library asks the caller's read(chunk, offset, length, dst) for each
chunk's bytes in column windows (qsmd5_plan.h plan_read) and folds every
window into that chunk's running MD5.  Checked here: digests against the
reference-produced fixtures and the pinned oracle over every padding edge,
empty chunks, groups and columns forced by a tiny staging budget; the read
contract (each chunk's windows in increasing offset order, every byte asked
for exactly once, nothing past the chunk); a short read fails the call with
-EIO as the reference's upload stops (QSTransferManager.cpp:625-643); and
the reader's exception reaches the caller.  The GPU path of the same entry
point is tests/test_gpu_read.py.
"""
import ctypes
import random

import pytest

import qsmd5
from oracle_util import lcg_bytes, md5_many

CPU = qsmd5.FLAG_CPU_ONLY
MiB = 1 << 20


class Recorder(object):
    """A reader over in-memory buffers that records every call."""

    def __init__(self, bufs, lens):
        self.bufs, self.lens, self.calls = bufs, lens, []

    def __call__(self, chunk, offset, length, dst):
        self.calls.append((chunk, offset, length))
        if offset + length > self.lens[chunk]:
            return 0
        ctypes.memmove(dst, ctypes.addressof(self.bufs[chunk]) + offset, length)
        return length

    def check_contract(self):
        seen = {}
        for c, off, length in self.calls:
            assert length > 0
            assert off == seen.get(c, 0), "chunk %d: window at %d, expected %d" % (c, off, seen.get(c, 0))
            seen[c] = off + length
        for c, L in enumerate(self.lens):
            assert seen.get(c, 0) == L, "chunk %d: %d of %d bytes read" % (c, seen.get(c, 0), L)


def _case(lens, staging, seed=7):
    bufs = [lcg_bytes(seed + i, L) for i, L in enumerate(lens)]
    rec = Recorder(bufs, lens)
    got = qsmd5.hash_read(lens, rec, staging_bytes=staging, flags=CPU)
    want = md5_many([(b, L) for b, L in zip(bufs, lens)])
    assert got == want
    rec.check_contract()
    return rec


def test_read_lcg_lengths_match_reference(golden):
    """Every padding edge 0..200 B and the longer lengths of the fixture, each
    the first L bytes of LCG(12345), through windows of a 1 MiB budget."""
    g = golden("lcg_lengths.json")
    cases = [c for c in g["cases"] if c["len"] <= 16 * MiB]
    lens = [c["len"] for c in cases]
    src = lcg_bytes(12345, max(lens))
    rec = Recorder([src] * len(lens), lens)
    got = qsmd5.hash_read(lens, rec, staging_bytes=1 * MiB, flags=CPU)
    assert [d.hex() for d in got] == [c["md5"] for c in cases]
    rec.check_contract()


def test_read_file_parts_match_batch_fixture(golden):
    """Parts of a file whose part i is LCG(12345 + i): the first 24 digests of
    batch_10MiB.json, read through a 64 MiB budget (10 columns per part)."""
    want = golden("batch_10MiB.json")["md5"][:24]
    L = 10 * MiB
    lens = [L] * 24
    bufs = [lcg_bytes(12345 + i, L) for i in range(24)]
    rec = Recorder(bufs, lens)
    got = qsmd5.hash_read(lens, rec, staging_bytes=64 * MiB, flags=CPU)
    assert [d.hex() for d in got] == want
    rec.check_contract()


@pytest.mark.parametrize("staging", [0, 1, 200000, 1 * MiB, 16 * MiB])
def test_read_ragged_groups_and_columns(staging):
    """Ragged lengths (empty, sub-block, block edges, multi-MiB) in caller
    order unrelated to length; tiny budgets force many groups of few rows."""
    rng = random.Random(staging + 3)
    lens = [0, 1, 55, 56, 63, 64, 65, 119, 120, 128, 4096, 3 * MiB + 5, 0, 2 * MiB]
    lens += [rng.randrange(0, 3 * MiB) for _ in range(40)]
    rng.shuffle(lens)
    _case(lens, staging)


def test_read_short_read_fails_with_eio():
    L = 3 * MiB
    bufs = [lcg_bytes(1, L), lcg_bytes(2, L)]

    def short(chunk, offset, length, dst):
        ctypes.memmove(dst, ctypes.addressof(bufs[chunk]) + offset, length)
        return length - 1 if chunk == 1 else length  # ReadNoLoad found a hole

    with pytest.raises(qsmd5.Md5Error) as e:
        qsmd5.hash_read([L, L], short, flags=CPU)
    assert e.value.code == -5  # -EIO
    assert "short read of chunk 1" in str(e.value)


def test_read_reader_exception_reaches_the_caller():
    def boom(chunk, offset, length, dst):
        raise KeyError("page gone")

    with pytest.raises(KeyError):
        qsmd5.hash_read([100, 200], boom, flags=CPU)


def test_read_argument_errors():
    L = qsmd5.lib()
    out = (ctypes.c_uint8 * 16)()
    lens = (ctypes.c_uint64 * 1)(5)
    assert L.qsmd5_hash_read(lens, 1, qsmd5.READ_FN(), None, 0, out, CPU) == -22  # NULL read
    assert L.qsmd5_hash_read(lens, 0, qsmd5.READ_FN(), None, 0, out, CPU) == 0    # nothing to do
    big = (ctypes.c_uint64 * 1)(1 << 38)
    assert L.qsmd5_hash_read(big, 1, qsmd5.READ_FN(lambda *a: 0), None, 0, out, CPU) == -22
    assert L.qsmd5_hash_read(lens, 1, qsmd5.READ_FN(lambda *a: 0), None, 0, out,
                             qsmd5.FLAG_CPU_ONLY | qsmd5.FLAG_GPU_ONLY) == -22


def test_read_auto_mode_without_gpu_falls_back(monkeypatch):
    """QSMD5_BACKEND=auto on a box without a GPU: a file of 64 x 1 MiB parts
    prices to the GPU, whose initialisation fails; the batch is read again from
    the start and hashed on the CPU, same digests."""
    if qsmd5.device_count() > 0:
        pytest.skip("a GPU is present: the fallback is exercised by the GPU suite")
    monkeypatch.setenv("QSMD5_BACKEND", "auto")
    monkeypatch.setenv("QSMD5_GPU_CHAIN_GIBS", "100")  # price the GPU as the faster
    lens = [1 * MiB] * 64
    bufs = [lcg_bytes(900 + i, L) for i, L in enumerate(lens)]
    rec = Recorder(bufs, lens)
    got = qsmd5.hash_read(lens, rec)
    assert got == md5_many([(b, L) for b, L in zip(bufs, lens)])
    assert qsmd5.last_backend() == qsmd5.BACKEND_CPU


@pytest.mark.parametrize("threads", ["1", "2", "4"])
@pytest.mark.parametrize("staging", [256 << 10, 4 * MiB, 0])
def test_read_lanes_and_scalar_agree(monkeypatch, threads, staging):
    """Round 5: with AVX-512 the CPU backend runs each window 16 rows at a time
    per thread in the vector lanes (md5_mb16_blocks continues every row's
    chunk state over its whole blocks; a final column's tail goes through the
    running context).  Lanes (QSMD5_CPU_MB=1) and scalar rows (=0) give the
    oracle's digests on ragged lengths, at 1, 2 and 4 threads and budgets
    that force many groups, and keep the read contract."""
    monkeypatch.setenv("QSMD5_CPU_THREADS", threads)
    rng = random.Random(int(threads) * 31 + staging)
    lens = [0, 1, 63, 64, 65, 127, 128, 4096, 65536, 65537, MiB, 2 * MiB + 63]
    lens += [rng.randrange(0, 2 * MiB) for _ in range(60)]
    rng.shuffle(lens)
    for mb in ("1", "0"):
        monkeypatch.setenv("QSMD5_CPU_MB", mb)
        _case(lens, staging, seed=400 + int(threads))


def test_read_routing_compares_wall_times(monkeypatch):
    """Auto routes a pull-driven batch by its wall time on each backend:
    the reads and the hashing overlap window by window, so it is about
    max(the caller's reads, the hashing), plus on the GPU the last window's
    copy and column kernel (round 6).  With reads priced fast
    (QSMD5_READ_GIBS=50), 8 x 10 MiB prices to the CPU lanes (~23 ms) against
    one GPU chain (~85 ms); with reads priced slow (0.5 GiB/s) and narrow
    windows (a 2 MiB budget: 128 KiB columns, a ~1 ms GPU tail) both backends
    are read-bound and the GPU is within 5% of the CPU, which routes it to
    the GPU (whose hashing leaves the host's cores free) -- here, without a
    GPU, that attempt falls back to the CPU.  With the default budget the
    10 MiB columns leave no overlap (one window: read it all, then an 85 ms
    chain) and the CPU wins.  The log carries the decision."""
    if qsmd5.device_count() > 0:
        pytest.skip("GPU present: the slow-read case would really run on it")
    if "avx512f" not in open("/proc/cpuinfo").read():
        pytest.skip("host without AVX-512F: the lanes are never priced")
    for k, v in (("QSMD5_BACKEND", "auto"), ("QSMD5_CPU_THREADS", "4"), ("QSMD5_GPU_CHAIN_GIBS", "0.119"),
                 ("QSMD5_CPU_LOAD_FEEDBACK", "0"), ("QSMD5_ROUTE_LANES", "1")):
        monkeypatch.setenv(k, v)
    lines = []
    qsmd5.set_log_callback(lambda level, text: lines.append(text))
    try:
        lens = [10 * MiB] * 8
        bufs = [lcg_bytes(77 + i, L) for i, L in enumerate(lens)]
        want_md5 = md5_many([(b, L) for b, L in zip(bufs, lens)])
        for gibs, staging, want in (("50", 0, "backend=cpu reason=size"), ("0.5", 2 * MiB, "backend=gpu reason=size"),
                                    ("0.5", 0, "backend=cpu reason=size")):
            monkeypatch.setenv("QSMD5_READ_GIBS", gibs)
            del lines[:]
            assert qsmd5.hash_read(lens, Recorder(bufs, lens), staging_bytes=staging) == want_md5  # auto
            assert any(want in l and "(read)" in l for l in lines), (gibs, staging, lines)
    finally:
        qsmd5.set_log_callback(None)


@pytest.mark.parametrize("readers", ["1", "3", "8"])
def test_read_parallel_flag(monkeypatch, readers):
    """QSMD5_FLAG_READ_PARALLEL (round 5): the library may call read from
    QSMD5_READ_THREADS threads at once, for different chunks of a window.
    Same digests, every chunk's windows still in order and every byte read
    once; a short read on any thread still fails the call with -EIO."""
    monkeypatch.setenv("QSMD5_READ_THREADS", readers)
    rng = random.Random(int(readers))
    lens = [rng.choice([0, 1, 64, 65, 4096, 1 << 20, 3 * MiB + 7]) for _ in range(40)]
    bufs = [lcg_bytes(900 + i, L) for i, L in enumerate(lens)]
    rec = Recorder(bufs, lens)
    got = qsmd5.hash_read(lens, rec, staging_bytes=1 << 20, flags=CPU | qsmd5.FLAG_READ_PARALLEL)
    assert got == md5_many([(b, L) for b, L in zip(bufs, lens)])
    rec.check_contract()
    bad = Recorder(bufs, lens)
    bad.lens = list(lens)
    bad.lens[lens.index(3 * MiB + 7)] = MiB  # the reader says this chunk ends early
    with pytest.raises(qsmd5.Md5Error) as e:
        qsmd5.hash_read(lens, bad, staging_bytes=1 << 20, flags=CPU | qsmd5.FLAG_READ_PARALLEL)
    assert e.value.code == -5  # -EIO
    assert "short read of chunk %d" % lens.index(3 * MiB + 7) in str(e.value)
