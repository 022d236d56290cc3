"""Multi-rank sharding + digest gather (qsmd5.parallel) over gloo on CPU.

The GPU path shards a file's parts across ranks (one process per GPU) and
all-gathers the 16-byte digests (RCCL over xGMI on MI355X).  Here two CPU
ranks run the same code over gloo; the per-rank hashing uses the oracle as a
stand-in for the kernel (no GPU in this container), and the gathered table is
checked against the reference-produced golden digests.
"""
import json
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN

MiB = 1 << 20


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, n, out_path):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.join(os.path.dirname(here), "qsfs-fuse_amd")]
    from oracle_util import lcg_bytes, md5_many
    from qsmd5.parallel import gather_digests, shard_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b, e = shard_range(n, rank, world)
    bufs = [lcg_bytes(12345 + i, 10 * MiB) for i in range(b, e)]
    digs = md5_many([(x, 10 * MiB) for x in bufs], threads=2)
    local = torch.tensor([list(d) for d in digs], dtype=torch.uint8).reshape(-1, 16)
    full = gather_digests(local, n)
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump([bytes(r.tolist()).hex() for r in full], f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 37), (2, 1), (3, 8)])
def test_gather_digests_gloo(world, n):
    want = json.load(open(os.path.join(GOLDEN, "batch_10MiB.json")))["md5"][:n]
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "digests.json")
        mp.spawn(_rank_main, args=(world, _free_port(), n, out), nprocs=world, join=True)
        got = json.load(open(out))
    assert got == want


def test_shard_range_partition():
    from qsmd5.parallel import shard_range
    for n in [0, 1, 7, 512, 10000]:
        for world in [1, 2, 3, 8]:
            spans = [shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (b0, e0), (b1, e1) in zip(spans, spans[1:]):
                assert e0 == b1
            sizes = [e - b for b, e in spans]
            assert max(sizes) - min(sizes) <= 1
