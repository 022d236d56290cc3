#!/usr/bin/env python3
"""Where does pinned host memory land relative to the GPU's NUMA node?
(config5_host reads each rank's shard over its own GPU's PCIe link; SURVEY.md
§8e asks for NUMA-local pinned memory.)  Prints the GPU's NUMA node (sysfs),
this process's CPU affinity, and the NUMA node of pages of a 1 GiB buffer from
qsmd5_alloc_pinned (hipHostMalloc default flags), by move_pages(2) query."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "qsfs-fuse_amd"))


def page_nodes(base, size, samples=64):
    libc = ctypes.CDLL(None, use_errno=True)
    page = os.sysconf("SC_PAGE_SIZE")
    addrs = [(base + (size * k) // samples) & ~(page - 1) for k in range(samples)]
    pages = (ctypes.c_void_p * samples)(*addrs)
    status = (ctypes.c_int * samples)()
    rc = libc.syscall(279, 0, samples, pages, None, status, 0)  # SYS_move_pages, x86_64
    if rc != 0:
        return {"error": os.strerror(ctypes.get_errno())}
    hist = {}
    for s in status:
        hist[str(s)] = hist.get(str(s), 0) + 1
    return hist


def main():
    import torch
    import qsmd5
    dev = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(dev)
    p = torch.cuda.get_device_properties(dev)
    bdf = "%04x:%02x:%02x.0" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
    node = None
    try:
        node = int(open("/sys/bus/pci/devices/%s/numa_node" % bdf).read())
    except OSError as e:
        node = str(e)
    nodes_online = open("/sys/devices/system/node/online").read().strip()
    out = {"gpu_bdf": bdf, "gpu_numa_node": node, "nodes_online": nodes_online,
           "affinity_cpus": len(os.sched_getaffinity(0))}
    qsmd5.lib().qsmd5_init(0)
    size = 1 << 30
    base = qsmd5.alloc_pinned(size)
    out["pinned_page_nodes"] = page_nodes(base, size)
    qsmd5.free_pinned(base)
    # The same from a thread running on the other node's CPUs under a memory
    # policy that prefers the other node: does HIP place pinned memory near the
    # GPU itself, or follow the caller's placement?
    other = 1 - node if isinstance(node, int) and node in (0, 1) else None
    if other is not None and os.path.exists("/sys/devices/system/node/node%d/cpulist" % other):
        cpus = set()
        for part in open("/sys/devices/system/node/node%d/cpulist" % other).read().strip().split(","):
            a, _, b = part.partition("-")
            cpus.update(range(int(a), int(b or a) + 1))
        os.sched_setaffinity(0, cpus & os.sched_getaffinity(0) or cpus)
        libc = ctypes.CDLL(None, use_errno=True)
        mask = ctypes.c_ulong(1 << other)
        rc = libc.syscall(238, 1, ctypes.byref(mask), 64)  # set_mempolicy(MPOL_PREFERRED)
        out["other_node"] = other
        out["set_mempolicy_rc"] = rc
        base = qsmd5.alloc_pinned(size)
        out["pinned_page_nodes_from_other_node"] = page_nodes(base, size)
        qsmd5.free_pinned(base)
        buf = ctypes.create_string_buffer(size)  # plain malloc'd and touched: the policy's node
        out["malloc_page_nodes_from_other_node"] = page_nodes(ctypes.addressof(buf), size)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
