"""Randomised batches through qsmd5_hash_batch_ex, every digest against the oracle.

Each seeded batch mixes lengths (0 B .. ~2 MiB, log-uniform, padding edges
included), memory kinds (device, pinned host, pageable host), byte offsets,
duplicates, and the runtime's knobs drawn per batch:
- QSMD5_COLUMN_BYTES: automatic, whole chunks, or a forced width;
- QSMD5_KERNEL: automatic or forced;
- QSMD5_MAPS_AFTER: VMA classification on early or off;
- QSMD5_FLAG_HOST: when every chunk is host memory;
- QSMD5_GATHER / QSMD5_GATHER_GROUPS: the gather kernel for lone pinned rows,
  on, off, or with 1..16 workgroups;
- QSMD5_PC_LANES and QSMD5_LOAD_NT: lanes per latency-kernel workgroup and nt
  producer loads;
- QSMD5_STAGING_BYTES / QSMD5_SLICE_BYTES: a staging ring of one or a few
  regions and small slices, so that slices reuse regions behind the kernels
  that last read them (the host-ordered pipeline's waits).
Host chunks come from two separate pinned pools, a pageable pool and a
pageable pool registered with qsmd5_register_host.
This drives the paths the fixed tests pin one at a time: the inline small-batch
path, single- and multi-slice staging, column kernels, the classifier's range
caches and 2-D copy runs.
"""
import ctypes
import os
import random

import numpy as np
import pytest

import qsmd5
from oracle_util import md5_many

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

POOL = 24 << 20
# QSMD5_FUZZ_SEEDS widens the sweep for a one-off soak (the suite runs 64 + 16)
N_BATCH = int(os.environ.get("QSMD5_FUZZ_SEEDS", "64"))
N_STREAM = max(16, N_BATCH // 4)
EDGES = [0, 1, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128, 4095, 4096, 4097]
KNOBS = ("QSMD5_COLUMN_BYTES", "QSMD5_KERNEL", "QSMD5_MAPS_AFTER", "QSMD5_GATHER",
         "QSMD5_GATHER_GROUPS", "QSMD5_PC_LANES", "QSMD5_LOAD_NT", "QSMD5_STAGING_BYTES",
         "QSMD5_SLICE_BYTES")


@pytest.fixture(scope="module")
def pools():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert qsmd5.lib().qsmd5_init(0) == 0
    rng = np.random.default_rng(2024)
    host = rng.integers(0, 256, size=POOL, dtype=np.uint8)
    dev = torch.from_numpy(host.copy()).cuda()
    pp = qsmd5.alloc_pinned(POOL)
    pinned = np.ctypeslib.as_array((ctypes.c_uint8 * POOL).from_address(pp))
    pinned[:] = host
    pp2 = qsmd5.alloc_pinned(POOL)
    pinned2 = np.ctypeslib.as_array((ctypes.c_uint8 * POOL).from_address(pp2))
    pinned2[:] = host
    reg = host.copy()
    qsmd5.register_host(reg.ctypes.data, POOL)
    torch.cuda.synchronize()
    yield {"host": host, "dev": dev, "pinned": pinned, "pinned2": pinned2, "reg": reg}
    qsmd5.unregister_host(reg.ctypes.data)
    qsmd5.free_pinned(pp)
    qsmd5.free_pinned(pp2)
    for k in KNOBS:
        os.environ.pop(k, None)


def _length(rng):
    if rng.random() < 0.2:
        return rng.choice(EDGES)
    return int(2 ** rng.uniform(0, 21)) + rng.randrange(97)


@pytest.mark.parametrize("seed", range(N_BATCH))
def test_random_batches(pools, seed):
    rng = random.Random(seed)
    n = rng.choice([1, 2, 3, 17, 64, 65, 200, 300])
    kinds = rng.choice([["dev"], ["pinned"], ["host"], ["pinned", "host"], ["dev", "pinned", "host"],
                        ["pinned", "pinned2"], ["pinned", "pinned2", "reg"], ["reg", "host"],
                        ["dev", "pinned2", "reg", "host"]])
    chunks, refs = [], []
    for _ in range(n):
        L = _length(rng)
        off = rng.randrange(POOL - L)
        k = rng.choice(kinds)
        if k == "dev":
            ptr = pools["dev"].data_ptr() + off
        else:
            ptr = pools[k].ctypes.data + off
        chunks.append((ptr if L else 0, L))
        refs.append((pools["host"].ctypes.data + off, L))
    if n > 2 and rng.random() < 0.3:  # duplicates
        chunks += chunks[:2]
        refs += refs[:2]
    env = {
        "QSMD5_COLUMN_BYTES": rng.choice([None, None, "0", "1024", "4160", str(256 << 10)]),
        "QSMD5_KERNEL": rng.choice([None, None, "pc", "pc2", "v1", "coal"]),
        "QSMD5_MAPS_AFTER": rng.choice([None, "1", "100000000"]),
        "QSMD5_GATHER": rng.choice([None, None, "0"]),
        "QSMD5_GATHER_GROUPS": rng.choice([None, "1", "3", "16"]),
        "QSMD5_PC_LANES": rng.choice([None, None, "16", "32", "48"]),
        "QSMD5_LOAD_NT": rng.choice([None, None, "1"]),
        # a ring of one or a few regions: slices wait for the kernel that
        # last used their region (the host-ordered pipeline's reuse path)
        "QSMD5_STAGING_BYTES": rng.choice([None, None, None, "1", str(1 << 20), str(8 << 20)]),
        "QSMD5_SLICE_BYTES": rng.choice([None, None, "65536", str(1 << 20)]),
    }
    for k, v in env.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    flags = qsmd5.FLAG_HOST if "dev" not in kinds and rng.random() < 0.5 else 0
    got = qsmd5.hash_batch(chunks, flags=flags)
    want = md5_many(refs)
    assert got == want, (seed, n, kinds, env, flags,
                         [i for i, (a, b) in enumerate(zip(got, want)) if a != b][:5])


@pytest.mark.parametrize("seed", range(N_STREAM))
def test_random_stream_updates(pools, seed):
    """The MD5 class (qsmd5_ctx): random pieces from host and device memory, so
    the host-side tail and the one-lane column launches meet every split."""
    rng = random.Random(1000 + seed)
    start = rng.randrange(4096)
    pos, pieces = start, []
    for _ in range(rng.randrange(1, 40)):
        L = rng.choice([0, 1, 63, 64, 65, 127, rng.randrange(1, 5000), rng.randrange(1, 300000)])
        if pos + L > POOL:
            break
        pieces.append((pos, L, rng.choice(["host", "pinned", "dev"])))
        pos += L
    h = qsmd5.MD5()
    for off, L, k in pieces:
        base = pools["dev"].data_ptr() if k == "dev" else pools[k].ctypes.data
        h.update((base + off if L else 0, L))
    want = md5_many([(pools["host"].ctypes.data + start, pos - start)])[0]
    assert h.finalize().digest() == want, (seed, [(L, k) for _, L, k in pieces])


N_READ = max(16, N_BATCH // 4)


@pytest.mark.parametrize("seed", range(N_READ))
def test_random_read_batches(pools, seed):
    """Pull-driven batches (qsmd5_hash_read, round 5): random lengths (edges,
    0 B .. ~2 MiB), random chunk counts and staging budgets from 64 KiB (one
    row of a window per chunk, many groups) to 64 MiB, read from the pinned,
    registered or pageable pool, sometimes from several threads at once (the
    read slots).  Every digest against the oracle on the same bytes."""
    import threading
    rng = random.Random(5000 + seed)
    jobs = []
    for _ in range(rng.choice([1, 1, 2, 3, 6])):
        n = rng.choice([1, 2, 17, 64, 65, 200])
        kind = rng.choice(["pinned", "reg", "host"])
        lens, offs = [], []
        for _ in range(n):
            L = _length(rng)
            lens.append(L)
            offs.append(rng.randrange(POOL - L))
        jobs.append({"lens": lens, "offs": offs, "kind": kind,
                     "staging": rng.choice([0, 64 << 10, 1 << 20, 4 << 20, 64 << 20])})

    def run(job):
        base = pools[job["kind"]].ctypes.data

        def read(chunk, off, length, dst):
            ctypes.memmove(dst, base + job["offs"][chunk] + off, length)
            return length
        try:
            job["got"] = qsmd5.hash_read(job["lens"], read, staging_bytes=job["staging"],
                                         flags=qsmd5.FLAG_GPU_ONLY)
        except Exception as e:  # reported below
            job["err"] = repr(e)

    th = [threading.Thread(target=run, args=(j,)) for j in jobs]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    for j in jobs:
        assert "err" not in j, (seed, j["err"])
        want = md5_many([(pools["host"].ctypes.data + o, L) for o, L in zip(j["offs"], j["lens"])])
        assert j["got"] == want, (seed, len(j["lens"]), j["staging"], j["kind"])
