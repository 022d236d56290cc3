"""The DoMultiPartUpload flow with the batch pre-hash on
the CPU backend: tests/cpp/multipart_harness gathers parts from a paged file
into pool buffers (File::ReadNoLoad), hashes each pool-size wave with one
qsmd5_hash_batch_ex call, and hands the hex digests on per part.  Here the
library's CPU backend hashes (QSMD5_BACKEND=cpu); tests/test_gpu_multipart.py
runs the same flow on the MI355X.  Digests are checked against the
reference-produced golden table, or the oracle for unaligned files."""
import ctypes
import json
import os

from conftest import GOLDEN
from multipart_util import run
from oracle_util import lcg_bytes, md5_many

MiB = 1 << 20


def test_aligned_parts_match_golden():
    gold = json.load(open(os.path.join(GOLDEN, "batch_10MiB.json")))["md5"]
    r = run(["--aligned", "--size=%d" % (12 * 10 * MiB), "--pool=5"], "cpu")
    assert r["parts"] == 12 and r["waves"] == 3 and r["cpu_waves"] == 3
    assert r["md5"] == gold[:12]


def test_prepare_upload_slicing_and_ragged_tail():
    """25 MiB + 3 B and 21 MiB files: PrepareUpload's [10, 10, 5] and averaged
    [10, 5.5, 5.5] MiB parts (QSTransferManager.cpp:517-542), gathered from
    pages that straddle part boundaries."""
    for size, seed in ((25 * MiB + 3, 31), (21 * MiB, 32), (100 * MiB + 12345, 33)):
        r = run(["--size=%d" % size, "--seed=%d" % seed, "--pool=2"], "cpu")
        data = lcg_bytes(seed, size)
        base, off, want = ctypes.addressof(data), 0, []
        for L in r["part_sizes"]:
            want.append((base + off, L))
            off += L
        assert off == size
        assert r["md5"] == [d.hex() for d in md5_many(want)], size
