#!/usr/bin/env python3
"""bench.py -- qsfs MD5 chunk-hashing path on MI355X (BASELINE.json metric).

Workload (BASELINE config 2): per GPU, a batch of 512 chunks
of 10 MiB (10 485 760 B), device-resident in HBM, chunk i = LCG(12345 + i)
(generated on the device before timing).  One step = one pass
of the hot path over the batch: qsmd5_hash_batch_device_async (the gfx950
kernel) producing all 512 digests, plus, for N > 1 GPUs, the RCCL all-gather
of the 16-byte digests (rank r holds parts [512 r, 512 (r+1)) of the job).

  python bench.py --gpus N --steps K --warmup W

prints ONE JSON line (rank 0) with value = whole-job GiB/s hashed, the
roofline of the dominant kernel (HIP events on the launch stream) and the CPU
baseline (the reference's own md5() built from /root/reference into
oracle/_ref, or the oracle port if that build is absent) timed on this host's
cores over the same 512 chunks -- which also re-checks every GPU digest
against the reference on the box.  Digests are checked against the committed
golden fixture (tests/golden/batch_10MiB.json) every run.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "qsfs-fuse_amd"))

from qsmd5.launch import launched, spawn_ranks  # noqa: E402  (no torch, no HIP)

MiB = 1 << 20
CHUNK = 10 * MiB
BATCH = 512
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
METRIC = "GiB/s MD5-hashed, device-resident 10 MB chunks, batch=512; % HBM-read peak"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _host_topology():
    """CPU model, sockets, physical cores, logical CPUs, affinity and cgroup quota."""
    model, phys, sockets = "unknown", set(), set()
    try:
        pid = None
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "model name" and model == "unknown":
                model = v
            elif k == "physical id":
                pid = v
                sockets.add(v)
            elif k == "core id":
                phys.add((pid, v))
    except OSError:
        pass
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        quota = None if q == "max" else round(int(q) / int(period), 2)
    except (OSError, ValueError):
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    return {"cpu_model": model, "sockets": len(sockets) or None,
            "physical_cores": len(phys) or None, "logical_cpus": os.cpu_count() or 0,
            "affinity_cpus": affinity, "cgroup_cpu_quota": quota}


def cpu_baseline(host_chunks, gpu_hex, gpu_value):
    """Time the reference md5() (or the oracle port) on this host's cores over
    the chunks: 1 thread (as deployed: one file's parts hashed serially,
    File.cpp:639-644), 5 (qsfs numtransfer default), 16 (this box's CPU share)
    and every logical CPU the host shows.  Both reference call forms are timed:
    md5(std::string) (MD5.cpp:335-339) and the call site's md5(iostream)
    (MD5.cpp:341-349, two extra copies)."""
    n = len(host_chunks)
    ptrs = (ctypes.c_void_p * n)(*host_chunks)
    lens = (ctypes.c_uint64 * n)(*([CHUNK] * n))
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libref_md5.so")
    if os.path.exists(ref_so):
        R = ctypes.CDLL(ref_so)
        R.ref_md5_prepare.restype = ctypes.c_void_p
        R.ref_md5_prepare.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        R.ref_md5_run.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        R.ref_md5_release.argtypes = [ctypes.c_void_p]

        def run(k, thr, iostream=0):
            h = R.ref_md5_prepare(ptrs, lens, k)
            out = (ctypes.c_char * (33 * k))()
            t0 = time.perf_counter()
            R.ref_md5_run(h, out, thr, iostream)
            dt = time.perf_counter() - t0
            R.ref_md5_release(h)
            raw = bytes(out)
            return dt, [raw[33 * i:33 * i + 32].decode() for i in range(k)]
        kind, what = "reference", "reference md5() from src/base/MD5.cpp (-O2)"
    else:
        O = ctypes.CDLL(os.path.join(ROOT, "oracle", "libmd5_oracle.so"))
        O.oracle_md5_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                       ctypes.c_void_p, ctypes.c_int]

        def run(k, thr, iostream=0):
            out = (ctypes.c_uint8 * (16 * k))()
            t0 = time.perf_counter()
            O.oracle_md5_batch(ptrs, lens, k, out, thr)
            dt = time.perf_counter() - t0
            raw = bytes(out)
            return dt, [raw[16 * i:16 * i + 16].hex() for i in range(k)]
        kind, what = "port", "oracle/md5_oracle.c (-O3)"
    topo = _host_topology()
    nproc = min(256, topo["logical_cpus"] or 1)
    gib = lambda k: k * CHUNK / float(1 << 30)
    by_threads, by_threads_iostream, samples = {}, {}, {}
    ref_hex = None
    for thr, k in ((1, 16), (5, 40), (16, 128), (nproc, n)):
        k = min(k, n)
        run(min(thr, k), thr)  # wake the cores first (idle CPUs start slow)
        passes = [run(k, thr) for _ in range(2)]
        dt = min(p[0] for p in passes)  # best of 2: thread start-up skew, not hashing
        by_threads[str(thr)] = round(gib(k) / dt, 3)
        samples[str(thr)] = k
        if k == n:
            ref_hex = passes[0][1]
    for thr, k in ((1, 16), (nproc, n)):
        k = min(k, n)
        run(min(thr, k), thr, 1)
        dt = min(run(k, thr, 1)[0] for _ in range(2))
        by_threads_iostream[str(thr)] = round(gib(k) / dt, 3)
    all_core = by_threads[str(nproc)]
    agree = ref_hex == gpu_hex
    quota = topo["cgroup_cpu_quota"]
    # The best measured rate is the baseline; `cores` is its thread count.  A
    # cgroup CPU quota below the host's CPU count caps what these threads get,
    # so the whole host's rate is also estimated from the 1-thread rate (the
    # threads scale linearly up to the quota: see by_threads).
    best_thr = max(by_threads, key=lambda t: by_threads[t])
    phys = topo["physical_cores"] or nproc
    host_est = round(by_threads["1"] * phys, 1)
    quota_bound = quota is not None and quota < nproc
    cpu_best = max(by_threads[best_thr], host_est)
    return {
        "value": by_threads[best_thr], "unit": "GiB/s", "cores": int(best_thr), "kind": kind,
        "sample": "%s, md5(std::string) form, over the same 10 MiB chunks: %s threads on "
                  "%s chunks (best of 2 passes after a warm-up); value = the best of these, "
                  "%s threads on %d chunks (cores = that thread count). Host: %s, %s sockets, "
                  "%s physical cores, %d logical CPUs, cgroup CPU quota %s" % (
                      what, "/".join(by_threads), "/".join(str(samples[t]) for t in by_threads),
                      best_thr, samples[best_thr], topo["cpu_model"], topo["sockets"],
                      topo["physical_cores"], topo["logical_cpus"],
                      quota if quota is not None else "none"),
        "agrees_with_gpu": agree,
        "by_threads": by_threads,
        "by_threads_iostream": by_threads_iostream,
        "host": topo,
        "cpu_vs_gpu": {
            "gpu_GiBps": gpu_value, "cpu_all_threads_measured_GiBps": all_core,
            "cpu_1_thread_GiBps": by_threads["1"],
            "measured_threads_quota_bound": quota_bound,
            "whole_host_estimate_GiBps": host_est,
            "whole_host_estimate_rule": "1-thread rate x %d physical cores (SMT not counted)" % phys,
            "faster_at_this_batch": "cpu (whole host, %s)" % (
                "estimated: the measured threads are held to a %.0f-CPU quota" % quota
                if quota_bound else "measured") if cpu_best > gpu_value else "gpu",
            "note": "at batch=512 the GPU job is 512 serial MD5 chains, one per chunk, each "
                    "~0.12 GiB/s on a GPU lane against ~0.8 GiB/s on a host core, so a host "
                    "with more than ~75 free cores hashes the same 512 chains faster; the GPU "
                    "leaves those cores to qsfs and outruns any host once a batch holds "
                    "thousands of chains (config 5: 10 000 parts in one launch)"},
    }


def _traffic_from_profiles():
    """HBM bytes per launch of the headline kernel from the newest committed PMC
    summary for this workload (profiles/<round>_*traffic.json)."""
    pdir = os.path.join(ROOT, "profiles")
    found = None
    if os.path.isdir(pdir):
        for f in sorted(os.listdir(pdir)):  # round-prefixed names: the last match is the newest
            if not f.endswith("traffic.json"):
                continue
            try:
                d = json.load(open(os.path.join(pdir, f)))
            except (OSError, ValueError):
                continue
            if isinstance(d, dict) and d.get("workload") == "batch512x10MiB":
                found = d.get("hbm_read_bytes_per_launch")
    return found


def _clock_evidence():
    """The headline kernel's effective clock from the newest committed clock
    log (profiles/<round>_effective_clock.log: GRBM_GUI_ACTIVE / 8 XCDs / wall
    per dispatch, scripts/summarize_clock.py), with the file it came from.
    Read from the committed profile, not measured in this run."""
    import re
    pdir = os.path.join(ROOT, "profiles")
    logs = sorted(f for f in os.listdir(pdir) if f.endswith("effective_clock.log")) if os.path.isdir(pdir) else []
    for f in reversed(logs):
        ghz = []
        for line in open(os.path.join(pdir, f)):
            if line.strip() == "" and ghz:
                break  # the headline section is the first one
            m = re.search(r"qsmd5_batch_pc64_kernel\s.*->\s*([0-9.]+) GHz", line)
            if m:
                ghz.append(float(m.group(1)))
        if ghz:
            return ("the kernel ran at %.3f-%.3f GHz over %d dispatches of this workload: GRBM_GUI_ACTIVE / "
                    "8 XCDs / wall (profiles/%s, a committed PMC pass, not this run), so the 2.4 GHz cycle "
                    "count above is the kernel's own" % (min(ghz), max(ghz), len(ghz), f))
    return "not measured (no profiles/*_effective_clock.log)"


def _host_mem_available():
    """Bytes of host memory this node can still give (MemAvailable, capped by
    the cgroup limit), or None."""
    avail = None
    try:
        for line in open("/proc/meminfo"):
            if line.startswith("MemAvailable:"):
                avail = int(line.split()[1]) * 1024
    except (OSError, ValueError):
        pass
    for cap_f, used_f in (("/sys/fs/cgroup/memory.max", "/sys/fs/cgroup/memory.current"),  # v2
                          ("/sys/fs/cgroup/memory/memory.limit_in_bytes",            # v1
                           "/sys/fs/cgroup/memory/memory.usage_in_bytes")):
        try:
            cap = open(cap_f).read().strip()
            if cap == "max" or int(cap) >= 1 << 60:  # v1 writes ~2^63 for "no limit"
                continue
            left = int(cap) - int(open(used_f).read().strip())
            avail = left if avail is None else min(avail, left)
        except (OSError, ValueError):
            pass
    return avail


def config5_host_leg(args, rank, world, dev, cpu=False):
    """BASELINE config 5 from host memory, the case that scales with GPUs
    (SURVEY.md §8e): ONE object of 10 000 x 10 MiB parts,
    part p = LCG(12345 + p).  Rank r holds its contiguous part range
    shard_range(n, r, world) in its own pinned host memory and hashes it with
    qsmd5_hash_batch_ex(QSMD5_FLAG_HOST) over its own GPU's PCIe link; the
    16-byte digests are all-gathered (RCCL) inside the timed region.  Strong
    scaling: the object is fixed, so value = object bytes / max-over-ranks
    time.  The reference hashes the same parts one after another on one core
    (QSTransferManager.cpp:602-673, File.cpp:639-644).

    The object is 97.7 GiB of host memory on the node; when the node has less
    than 1/0.6 of that free, the part count is cut to fit and the line says so.
    """
    import torch
    import torch.distributed as dist
    from bench_config5 import HostShard, L as PART
    from qsmd5.parallel import group_report

    dist_on = dist.is_initialized()
    want = args.config5_parts
    n = want
    if dist_on:
        dist.barrier()  # every rank reads free memory before any allocates
    avail = _host_mem_available()
    if avail is not None:
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
        nodes = max(1, world // max(1, local_world))
        fit = int(avail * 0.6) // PART * nodes
        n = min(want, max(world, fit))  # cut to fit, but never below a part per rank
    if dist_on:
        t = torch.tensor([n], dtype=torch.int64, device="cpu" if cpu or
                         dist.get_backend() == "gloo" else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        n = int(t.item())
    # The shard's pinned allocation can fail where the free-memory reading was
    # optimistic (another tenant, a limit not visible here): then every rank
    # skips the key together, and the headline line is still printed.
    shard, err = None, ""
    try:
        shard = HostShard(n, rank, world, dev, cpu_rehearsal=cpu)
    except Exception as e:  # qsmd5.Md5Error (-ENOMEM), torch OOM
        err = "rank %d: %s" % (rank, e)
        log("config5_host: %s" % err)
    if dist_on:
        ok_t = torch.tensor([0 if shard is None else 1], dtype=torch.int64,
                            device="cpu" if cpu or dist.get_backend() == "gloo" else dev)
        dist.all_reduce(ok_t, op=dist.ReduceOp.MIN)
        all_ok = bool(ok_t.item())
    else:
        all_ok = shard is not None
    if not all_ok:
        if shard is not None:
            shard.close()
        return {"skipped": "a rank could not hold its shard of %d parts in pinned host memory%s"
                           % (n, (": " + err) if err else "")}, True
    sync = (lambda: None) if cpu else torch.cuda.synchronize
    reps = max(1, args.config5_reps)
    with shard:  # the pinned shard is freed whatever happens below
        for _ in range(args.config5_warmup):
            shard.step()
        if dist_on:
            dist.barrier()
        sync()
        t0 = time.perf_counter()
        table = None
        for _ in range(reps):
            table = shard.step()
        sync()
        if dist_on:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if dist_on:
            tt = torch.tensor([elapsed], dtype=torch.float64,
                              device="cpu" if cpu or dist.get_backend() == "gloo" else dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            elapsed = float(tt.item())
        pg = group_report(shard.m, None if cpu else dev) if dist_on else None
        path = shard.path
        m_local = shard.m
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "batch_10MiB.json")))["md5"]
    got = [bytes(r).hex() for r in table.cpu().numpy()]
    ok = n <= len(gold) and got == gold[:n]
    per_pass = elapsed / reps
    value = n * PART / float(1 << 30) / per_pass
    out = {
        "workload": "BASELINE config 5 from host memory: one object of %d x 10 MiB parts "
                    "(%.1f GiB), contiguous part range per rank in that rank's pinned host "
                    "memory, qsmd5_hash_batch_ex(QSMD5_FLAG_HOST) over its own GPU link, "
                    "16-B digest all-gather inside the timed region" % (n, n * PART / 2.0 ** 30),
        "value": round(value, 3), "unit": "GiB/s", "scaling": "strong", "n_gpus": world,
        "parts": n, "parts_per_rank": [x["parts"] for x in pg["ranks"]] if pg else [m_local],
        "seconds_per_pass": round(per_pass, 4), "passes": reps, "warmup": args.config5_warmup,
        "per_gpu_GiBps": round(value / world, 3),
        "collective": ("RCCL all_gather_into_tensor (16 B per part)"
                       if dist_on and dist.get_backend() == "nccl" else
                       "gloo all_gather (host)" if dist_on else "none (one rank)"),
        "process_group": pg,
        "path": path,
        "parity": "ok: %d/%d digests == reference golden" % (n, n) if ok else "FAIL",
    }
    if n != want:
        out["reduced_from"] = want
        out["reduced_because"] = "node host memory: %.1f GiB free" % ((avail or 0) / 2.0 ** 30)
    return out, ok


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=BATCH, help="chunks per GPU (default 512)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-always", action="store_true",
                    help="init the process group and gather digests even at world size 1 "
                         "(exercises the RCCL path on a 1-GPU box)")
    ap.add_argument("--rehearse-gloo", action="store_true",
                    help="N>1 rehearsal on a 1-GPU box: every rank on cuda:0, gloo digest gather")
    ap.add_argument("--config5-parts", type=int, default=10000,
                    help="parts of the config5_host object (10 MiB each; default the 100 GB object)")
    ap.add_argument("--config5-reps", type=int, default=3, help="timed passes of config5_host")
    ap.add_argument("--config5-warmup", type=int, default=1, help="untimed passes of config5_host")
    ap.add_argument("--no-config5", action="store_true", help="skip the config5_host key")
    ap.add_argument("--cpu-rehearsal", action="store_true",
                    help="no GPU: run only the config5_host leg on CPU ranks over gloo (numpy "
                         "parts, libqsmd5's CPU backend) and print its JSON line")
    args = ap.parse_args()

    if args.gpus > 1 and not launched():
        # A bare `bench.py --gpus N` (the driver's command): form the N ranks here,
        # one fresh process per GPU, before anything touches a GPU.
        log("bench.py: no launcher environment; starting %d rank processes" % args.gpus)
        return spawn_ranks(os.path.abspath(__file__), sys.argv[1:], args.gpus)
    if args.cpu_rehearsal:
        return cpu_rehearsal(args)

    # The bench measures the gfx950 kernels only: no CPU routing or fallback.
    os.environ["QSMD5_BACKEND"] = "gpu"
    import torch
    import torch.distributed as dist
    import qsmd5
    from qsmd5.parallel import gather_digests, group_report

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("note: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (args.gpus, world))
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU (it measures the gfx950 kernels)")
    if args.rehearse_gloo:
        local = 0
    elif local >= torch.cuda.device_count():
        raise SystemExit("rank %d has no GPU of its own (%d visible); --rehearse-gloo runs every "
                         "rank on cuda:0" % (rank, torch.cuda.device_count()))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    distributed = world > 1 or args.dist_always
    if distributed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        if args.rehearse_gloo:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        # from here the group, not the launcher's environment, says how many
        # ranks there are
        world, rank = dist.get_world_size(), dist.get_rank()
    rc = qsmd5.lib().qsmd5_init(0)
    if rc != 0:
        raise SystemExit("qsmd5_init failed: %d" % rc)

    B, L = args.batch, CHUNK
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    # --- synthetic device-resident input: chunk j of the job = LCG(12345 + j) --------
    data = torch.empty(B * L, dtype=torch.uint8, device=dev)
    seed0 = 12345 + rank * B
    qsmd5.synth_fill_lcg(data.data_ptr(), L, L, seed0, B, sp)
    desc = torch.empty((B, 2), dtype=torch.int64)
    desc[:, 0] = data.data_ptr() + torch.arange(B, dtype=torch.int64) * L
    desc[:, 1] = L
    desc = desc.to(dev)
    # Two digest tables, alternated by step: the timed steps write into tables
    # zeroed after the warm-up, and parity checks the first and the last timed
    # step's own output, so a timed launch that did no work cannot pass on the
    # warm-up's digests.
    digs = [torch.zeros((B, 16), dtype=torch.uint8, device=dev) for _ in range(2)]
    torch.cuda.synchronize()
    kernel = {0: "one-wave (qsmd5_batch_kernel)", 1: "producer/consumer (qsmd5_batch_pc64_kernel)",
              2: "coalesced (qsmd5_batch_coal_kernel)",
              3: "producer/consumer, 64 KiB ring (qsmd5_batch_pc2_kernel)"}[qsmd5.kernel_choice(B)]

    def step(k, ev=None):
        dig = digs[k & 1]
        if ev is not None:
            ev[0].record(stream)
        qsmd5.hash_device(desc.data_ptr(), dig.data_ptr(), B, stream=sp)
        if ev is not None:
            ev[1].record(stream)
        if distributed:
            return gather_digests(dig, B * world)
        return dig

    for k in range(args.warmup):
        step(k)
    for d in digs:  # the timed steps start from zeroed tables
        d.zero_()
    torch.cuda.synchronize()
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps)]
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    first = out = None
    for k in range(args.steps):
        out = step(k, events[k])
        if k == 0:
            first = out  # a reference: for N > 1 the gather's own tensor, else digs[0]
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if distributed:
        tt = torch.tensor([elapsed], dtype=torch.float64,
                          device="cpu" if args.rehearse_gloo else dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    kernel_ms = [a.elapsed_time(b) for a, b in events]
    kavg_ms = sum(kernel_ms) / len(kernel_ms)

    # --- parity: every digest of the job against the reference-produced fixture -------
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "batch_10MiB.json")))["md5"]
    table = out
    got_hex = [bytes(r).hex() for r in table.cpu().numpy()]
    first_hex = [bytes(r).hex() for r in first.cpu().numpy()]
    ntot = B * world
    parity_ok = ntot <= len(gold) and got_hex[:ntot] == gold[:ntot] and first_hex[:ntot] == gold[:ntot]
    if rank == 0 and not parity_ok:
        bad = [i for i in range(min(ntot, len(gold))) if got_hex[i] != gold[i]]
        log("PARITY FAILURE: %d of %d digests differ (first %s)" % (len(bad), ntot, bad[:5]))

    pg = group_report(B, dev) if distributed else None
    job_bytes = float(ntot) * L
    value = job_bytes / (1 << 30) / elapsed * args.steps
    ms_per_step = elapsed / args.steps * 1e3
    achieved_gbs = B * L / (kavg_ms * 1e-3) / 1e9
    result = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic: LCG(12345+i) chunks generated on device, resident in HBM",
        "config": {"workload": "batch=%d x 10 MiB chunks per GPU, device-resident "
                               "(BASELINE config 2)" % B,
                   "global_batch": ntot, "chunk_bytes": L,
                   "parallelism": "part-shard x%d + RCCL digest all-gather" % world
                   if world > 1 else "single GPU", "kernel": kernel},
        "roofline": {"bound": "hbm", "achieved": round(achieved_gbs, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved_gbs / HBM_PEAK_GBS, 5),
                     "traffic": _traffic_from_profiles(),
                     "kernel_ms_avg": round(kavg_ms, 3),
                     "algorithmic_bytes_per_launch": B * L},
        # the stream-parallelism ceiling beside % of HBM peak.  A chunk
        # is one serial chain of 64 MD5 steps per 64-B block, each step 4 dependent
        # VALU (bitop3, add3, alignbit, add).  Measured on gfx950 with one wave alone
        # on its SIMD (ubench chaincost, profiles/r02_chaincost.log): the steps from
        # registers take 1045 cycles per block; fed from the LDS ring (16
        # ds_read_b128 per block, the shipped graded phase-start wait) 1133
        # (profiles/r03_chaincost.log).  The ceiling uses the register floor, at the
        # 2.4 GHz the chip holds with a few CUs busy.
        "stream_ceiling": {
            "chains": ntot // world, "floor_cycles_per_block": 1045.0,
            "lds_fed_floor_cycles_per_block": 1133.0,
            "GBps": round(B * 64 * 2.4e9 / 1045.0 / 1e9, 2),
            "frac": round(achieved_gbs / (B * 64 * 2.4e9 / 1045.0 / 1e9), 4),
            "note": "achieved / (B x per-chain issue floor): how close the kernel is to what "
                    "B serial MD5 chains allow on one GPU; the floor has no operand "
                    "traffic at all, so 1045 / 1133 = 0.922 is the most an LDS-fed chain "
                    "can reach"},
        "per_chain": {"GiBps": round(B * L / (1 << 30) / (kavg_ms * 1e-3) / B, 4),
                      "cycles_per_64B_block_at_2p4GHz": round(kavg_ms * 1e-3 * 2.4e9 / (L / 64), 1),
                      "note": "MD5 is a serial chain per chunk; at batch=512 the job rate is "
                              "512 x the per-chain rate (SURVEY.md §0 item 5)",
                      "clock_evidence": _clock_evidence()},
        "parity": "ok: %d/%d digests == reference golden" % (ntot, ntot) if parity_ok else "FAIL",
        "process_group": pg,
        "cpu_baseline": None,
    }
    if world > 1:
        result["launcher"] = ("bench.py: %d child processes, one per GPU" % world
                              if os.environ.get("QSMD5_SPAWNED_BY") == "bench" else
                              "external (torch.distributed.run or equivalent)")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        host = data.cpu().numpy()
        chunks = [host[i * L:(i + 1) * L].ctypes.data for i in range(B)]
        cb = cpu_baseline(chunks, got_hex[:B], round(value, 3))
        result["cpu_baseline"] = cb
        if not cb["agrees_with_gpu"]:
            result["parity"] = "FAIL (cpu reference disagrees)"
        del host
    del data, desc, digs, out, first, table
    torch.cuda.empty_cache()
    c5_ok = True
    if not args.no_config5:
        # the host-resident object, strong-scaled over the ranks (extra key; the
        # headline above is unchanged)
        result["config5_host"], c5_ok = config5_host_leg(args, rank, world, dev)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if distributed:
        dist.destroy_process_group()
    return 0 if parity_ok and c5_ok else 3


def cpu_rehearsal(args):
    """The config5_host leg on CPU ranks over gloo (tests/test_bench_gloo.py):
    sharding, the digest gather, max-over-ranks timing and parity without a GPU."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29517")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    world, rank = dist.get_world_size(), dist.get_rank()
    c5, ok = config5_host_leg(args, rank, world, torch.device("cpu"), cpu=True)
    if rank == 0:
        print(json.dumps({"rehearsal": "cpu ranks over gloo, libqsmd5 CPU backend (no GPU; not "
                                       "a measurement)", "n_gpus": world, "config5_host": c5}),
              flush=True)
    dist.destroy_process_group()
    return 0 if ok else 3


if __name__ == "__main__":
    sys.exit(main())
