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


def group_report(parts_local, device=None, group=None):
    """What the process group itself says about a multi-rank run: its backend
    and size (dist.get_backend / get_world_size, not the launcher's
    environment) and, all-gathered from every rank, that rank's GPU (ordinal
    and PCI domain:bus:device; -1 on CPU ranks) and the parts it hashed.  A
    scaling line carrying this shows RCCL saw N ranks on N distinct GPUs."""
    world = dist.get_world_size(group)
    backend = dist.get_backend(group)
    ordinal, pci = -1, (-1, -1, -1)
    if device is not None and getattr(device, "type", "cpu") == "cuda":
        ordinal = device.index if device.index is not None else torch.cuda.current_device()
        p = torch.cuda.get_device_properties(ordinal)
        pci = (getattr(p, "pci_domain_id", -1), getattr(p, "pci_bus_id", -1),
               getattr(p, "pci_device_id", -1))
    mine = torch.tensor([dist.get_rank(group), ordinal, pci[0], pci[1], pci[2], int(parts_local)],
                        dtype=torch.int64)
    if backend == "gloo":
        rows = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(rows, mine, group=group)
    else:
        mine = mine.to(device)
        out = torch.empty((world, mine.numel()), dtype=torch.int64, device=device)
        dist.all_gather_into_tensor(out, mine.reshape(1, -1), group=group)
        rows = list(out.cpu())
    ranks = []
    for r in rows:
        rank, dev, dom, bus, slot, parts = (int(x) for x in r.tolist())
        ranks.append({"rank": rank, "device": dev,
                      "pci": "%04x:%02x:%02x" % (dom, bus, slot) if bus >= 0 else None,
                      "parts": parts})
    pcis = {x["pci"] for x in ranks if x["pci"]}
    return {"backend": backend, "world_size": world, "ranks": ranks,
            "distinct_gpus": len(pcis)}
