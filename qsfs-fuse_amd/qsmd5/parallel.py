"""Multi-GPU sharding of a file's parts.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI on
MI355X; "gloo" on CPU for tests).  Parts are independent MD5 chains, so the
only exchange is the digest gather at the end: 16 bytes per part, e.g.
160 KB for a 100 GB object of 10 000 x 10 MiB parts.  Part p goes to the rank
whose contiguous range holds it, so each rank reads (or H2D-copies) one
contiguous byte range of the object.
"""
import torch
import torch.distributed as dist


def shard_range(n, rank, world):
    """[begin, end) of the parts rank `rank` hashes out of n (contiguous, balanced)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    return (rank * n) // world, ((rank + 1) * n) // world


def gather_digests(local, n, group=None):
    """All-gather every rank's [m_r, 16] uint8 digests into the full [n, 16] table.

    Ranks hold contiguous shards from shard_range, so the gathered table is in
    part order.  Shards differ in size by at most one; they are padded to the
    largest for the collective and trimmed after.
    """
    world = dist.get_world_size(group)
    sizes = [shard_range(n, r, world) for r in range(world)]
    m_max = max(e - b for b, e in sizes)
    if local.dim() != 2 or local.shape[1] != 16:
        raise ValueError("local digests must be [m, 16]")
    pad = torch.zeros((m_max, 16), dtype=torch.uint8, device=local.device)
    pad[: local.shape[0]] = local
    if dist.get_backend(group) == "gloo":
        # gloo (CPU tests, single-GPU rehearsals) gathers host tensors
        pad_h = pad.cpu()
        parts = [torch.empty_like(pad_h) for _ in range(world)]
        dist.all_gather(parts, pad_h, group=group)
        out = torch.cat(parts, 0).to(local.device)
    else:
        out = torch.empty((world * m_max, 16), dtype=torch.uint8, device=local.device)
        dist.all_gather_into_tensor(out, pad, group=group)
    rows = [out[r * m_max: r * m_max + (e - b)] for r, (b, e) in enumerate(sizes)]
    return torch.cat(rows, 0)
