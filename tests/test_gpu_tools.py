"""qsmd5sum: the batch caller end to end on the GPU.

Files are sliced like QSTransferManager::PrepareUpload and hashed in one
call: mapped, through qsmd5_hash_batch, or pulled with pread through
qsmd5_hash_read (--read); every printed digest is checked against the pinned
oracle on the same byte range.
"""
import os
import subprocess
import tempfile

import pytest

import qsmd5
from conftest import ROOT
from oracle_util import lcg_bytes, md5_ref

pytestmark = pytest.mark.gpu
MiB = 1 << 20
TOOL = os.path.join(ROOT, "qsfs-fuse_amd", "bin", "qsmd5sum")


@pytest.mark.parametrize("mode", [[], ["--read"], ["--read", "--staging", "1"]],
                         ids=["mapped", "pulled", "pulled_1MiB_staging"])
def test_qsmd5sum_parts_match_oracle(mode):
    """Mapped files in one qsmd5_hash_batch, or (--read, round 5) every part
    pulled with pread through qsmd5_hash_read's bounded staging."""
    if not os.path.exists(TOOL):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "qsfs-fuse_amd")])
    sizes = [0, 5, 19 * MiB, 20 * MiB, 21 * MiB + 3, 25 * MiB, 64 * MiB + 1]
    with tempfile.TemporaryDirectory() as td:
        paths, blobs = [], []
        for i, sz in enumerate(sizes):
            b = bytes(lcg_bytes(500 + i, sz))[:sz]
            p = os.path.join(td, "f%d" % i)
            with open(p, "wb") as f:
                f.write(b)
            paths.append(p)
            blobs.append(b)
        out = subprocess.run([TOOL] + mode + paths, capture_output=True, text=True, timeout=300)
        assert out.returncode == 0, out.stderr
        lines = out.stdout.strip().splitlines()
        want = []
        for p, b in zip(paths, blobs):
            parts = qsmd5.plan_parts(len(b))
            if len(parts) == 1 and len(b) < 20 * MiB:
                want.append("%s  %s" % (md5_ref(b).hex(), p))
            else:
                for q in parts:
                    want.append("%s  %s#%d %d %d" % (
                        md5_ref(b[q.offset:q.offset + q.size]).hex(), p,
                        q.part_number, q.offset, q.size))
        assert lines == want
        # -b 1: 1 MiB parts (the -b option of qsfs, Parser.cpp:167)
        out = subprocess.run([TOOL, "-b", "1", "--parts"] + mode + [paths[5]], capture_output=True,
                             text=True, timeout=300)
        assert out.returncode == 0, out.stderr
        assert len(out.stdout.strip().splitlines()) == 25
