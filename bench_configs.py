#!/usr/bin/env python3
"""bench_configs.py -- the other BASELINE.json configs (bench.py runs config 2).

  1  1 x 10 MiB KAT on the reference CPU path (plumbing) + the same chunk on the GPU
  3  4096 x 10 MiB in pinned host memory: end-to-end host -> digest through
     qsmd5_hash_batch (H2D slices overlapped with hashing, D2H of digests)
  4  ragged batch 8 KiB..64 MiB (tests/golden/ragged.json, ~4 GiB) + the -b
     bufsize sweep {1,2,4,8,10,16,32,64} MiB, device-resident
  5  10 000 x 10 MiB (97.7 GiB) on ONE GPU, device-resident (the per-GPU share at
     N GPUs is 10000/N; the 8-GPU run is the driver's bench.py --gpus 8)
  sat  kernel-quality line: enough independent chains to need the HBM roofline
     (131072 x 64 KiB and x 256 KiB, coalesced kernel)
Further lines, on request:
  3p / 3cmp / 3cols  config 3 from pageable memory; pinned vs pageable at equal
     sizes; 64 / 1024 / 4096 parts (column-width sweeps via QSMD5_COLUMN_BYTES)
  5h   config 5 host-resident (10000 x 10 MiB from pinned memory)
  small  1 M x 1 KiB objects from pageable (with and without QSMD5_FLAG_HOST)
     and pinned memory
  pool   512 pool buffers passed in pool order and shuffled
  tiny   device-resident 1 M x 1 KiB, 1 M x 4 KiB, 512 K x 16 KiB
  satpad saturation at exact power-of-two strides vs padded
  satsweep / sat64 / sat256  the coalesced kernel at 131072 x {16..256} KiB, or one
     of the two sat lines alone (scripts/r05_sat_attrib.sh: PMC passes per size)

Every digest is checked against the reference-produced golden fixtures where
they exist.  One JSON object per config on stdout.
Usage: python bench_configs.py [--configs 1,3,4,5,sat] [--reps 3]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
# These lines measure the gfx950 kernels: no size routing to the CPU MD5.
os.environ.setdefault("QSMD5_BACKEND", "gpu")
sys.path.insert(0, os.path.join(ROOT, "qsfs-fuse_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
MiB = 1 << 20
GiB = 1 << 30
HBM_PEAK_GBS = 8000.0


def gold(name):
    return json.load(open(os.path.join(ROOT, "tests", "golden", name)))


def emit(d):
    print(json.dumps(d), flush=True)


def timed(fn, reps):
    import torch
    best, out = None, None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None or dt < best else best
    return best, out


def config1():
    import qsmd5
    from oracle_util import lcg_bytes, md5_ref
    data = lcg_bytes(12345, 10 * MiB)
    want = "302bec822b27cea263612fb3f76fa34b"
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libref_md5.so")
    cpu_kind, cpu_hex = "port", md5_ref(data, 10 * MiB).hex()
    if os.path.exists(ref_so):
        R = ctypes.CDLL(ref_so)
        R.ref_md5_string.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_char_p]
        out = ctypes.create_string_buffer(33)
        t0 = time.perf_counter()
        R.ref_md5_string(ctypes.addressof(data), 10 * MiB, out)
        cpu_s = time.perf_counter() - t0
        cpu_kind, cpu_hex = "reference", out.value.decode()
    else:
        t0 = time.perf_counter()
        md5_ref(data, 10 * MiB)
        cpu_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    g = qsmd5.hash_one((ctypes.addressof(data), 10 * MiB)).hex()
    gpu_s = time.perf_counter() - t0
    emit({"config": 1, "workload": "1 x 10 MiB LCG(12345) KAT", "expected": want,
          "cpu": {"kind": cpu_kind, "md5": cpu_hex, "ms": round(cpu_s * 1e3, 2)},
          "gpu_hash_one": {"md5": g, "ms_incl_h2d_and_launch": round(gpu_s * 1e3, 2)},
          "parity": "ok" if cpu_hex == want == g else "FAIL",
          "note": "a single chunk is one serial MD5 chain: the GPU lane is slower than a "
                  "CPU core here; batches are what the GPU path is for"})


def config3(reps, n=4096, label=""):
    import numpy as np
    import torch
    import qsmd5
    L = 10 * MiB
    g = gold("batch_10MiB.json")["md5"][:n]
    p = qsmd5.alloc_pinned(n * L)
    try:
        host = np.ctypeslib.as_array((ctypes.c_uint8 * (n * L)).from_address(p))
        step = 256
        buf = torch.empty(step * L, dtype=torch.uint8, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        for k in range(0, n, step):
            m = min(step, n - k)
            qsmd5.synth_fill_lcg(buf.data_ptr(), L, L, 12345 + k, m, s)
            torch.from_numpy(host[k * L:(k + m) * L]).copy_(buf[:m * L])
        torch.cuda.synchronize()
        del buf
        chunks = [(p + i * L, L) for i in range(n)]
        dt, digs = timed(lambda: qsmd5.hash_batch(chunks), reps)
        wall, kern = qsmd5.last_timing()
        ok = [d.hex() for d in digs] == g
        emit({"config": 3, "workload": "%d x 10 MiB in pinned host memory, end-to-end "
                                       "(H2D + hash + D2H digests)%s" % (n, label),
              "value": round(n * L / GiB / dt, 3), "unit": "GiB/s", "seconds": round(dt, 4),
              "last_call_wall_ms": round(wall, 2), "last_call_kernel_window_ms": round(kern, 2),
              "parity": "ok: %d/%d == reference golden" % (n, n) if ok else "FAIL"})
    finally:
        qsmd5.free_pinned(p)


def config3_pageable(reps, n=1024):
    """Config 3's flow from ordinary pageable host memory: what qsfs has today,
    its ResourceManager buffers being plain vector<char> (ResourceManager.cpp:53-77),
    not the pinned pool of SURVEY.md §8f row 2."""
    import numpy as np
    import torch
    import qsmd5
    L = 10 * MiB
    g = gold("batch_10MiB.json")["md5"][:n]
    host = np.empty(n * L, dtype=np.uint8)
    step = 256
    buf = torch.empty(step * L, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for k in range(0, n, step):
        m = min(step, n - k)
        qsmd5.synth_fill_lcg(buf.data_ptr(), L, L, 12345 + k, m, s)
        torch.from_numpy(host[k * L:(k + m) * L]).copy_(buf[:m * L])
    torch.cuda.synchronize()
    del buf
    base = host.ctypes.data
    chunks = [(base + i * L, L) for i in range(n)]
    dt, digs = timed(lambda: qsmd5.hash_batch(chunks), reps)
    wall, kern = qsmd5.last_timing()
    ok = [d.hex() for d in digs] == g
    emit({"config": "3-pageable", "workload": "%d x 10 MiB in PAGEABLE host memory, end-to-end "
                                              "(H2D + hash + D2H digests)" % n,
          "value": round(n * L / GiB / dt, 3), "unit": "GiB/s", "seconds": round(dt, 4),
          "last_call_wall_ms": round(wall, 2), "last_call_kernel_window_ms": round(kern, 2),
          "parity": "ok: %d/%d == reference golden" % (n, n) if ok else "FAIL"})
    del host


def many_small(reps, n=1 << 20, L=1024):
    """Many small objects (qsfs uploads every file below 20 MiB as one PutObject
    with its own Content-MD5, QSClient.cpp:437-458): n chunks of L bytes in one
    host buffer, one batch.  Reports the wall time and the kernel window, so the
    host-side cost per chunk (classification, sort, descriptors) is visible.
    Run for pageable host memory with and without QSMD5_FLAG_HOST (the caller
    vouches that every chunk is host memory: no per-chunk pointer query), and
    for pinned host memory (the runtime's range cache answers after one query)."""
    import numpy as np
    import qsmd5
    from oracle_util import md5_many
    Lb = qsmd5.lib()
    for mem, flags in (("pageable", 0), ("pageable", qsmd5.FLAG_HOST), ("pinned", 0)):
        if mem == "pinned":
            pp = qsmd5.alloc_pinned(n * L)
            host = np.ctypeslib.as_array((ctypes.c_uint8 * (n * L)).from_address(pp))
        else:
            host = np.empty(n * L, dtype=np.uint8)
        rng = np.random.default_rng(5)
        host[:] = rng.integers(0, 256, size=n * L, dtype=np.uint8)
        desc = np.empty((n, 2), dtype=np.uint64)
        desc[:, 0] = host.ctypes.data + np.arange(n, dtype=np.uint64) * L
        desc[:, 1] = L
        out = np.empty((n, 16), dtype=np.uint8)

        def run():
            rc = Lb.qsmd5_hash_batch_ex(
                ctypes.cast(desc.ctypes.data, ctypes.POINTER(qsmd5.qsmd5_chunk)), n,
                ctypes.cast(out.ctypes.data, ctypes.POINTER(ctypes.c_uint8)), flags)
            assert rc == 0, rc
            return out

        dt, _ = timed(run, reps)
        wall, kern = qsmd5.last_timing()
        sample = list(range(0, n, n // 64))
        want = md5_many([(host.ctypes.data + i * L, L) for i in sample])
        ok = [bytes(out[i]) for i in sample] == want
        emit({"config": "many-small", "workload": "%d x %d B objects in one %s host buffer, one batch%s"
                                                 % (n, L, mem, ", QSMD5_FLAG_HOST" if flags else ""),
              "objects_per_s": round(n / dt), "GiBps": round(n * L / GiB / dt, 3),
              "seconds": round(dt, 4), "last_call_wall_ms": round(wall, 2),
              "last_call_kernel_window_ms": round(kern, 2),
              "host_us_per_chunk": round((wall - kern) * 1e3 / n, 3),
              "parity": "ok (64 sampled vs oracle)" if ok else "FAIL"})
        del host
        if mem == "pinned":
            qsmd5.free_pinned(pp)


def config4(reps):
    import torch
    import qsmd5
    gr = gold("ragged.json")
    lens = gr["lengths"]
    offs, pos = [], 0
    for L in lens:
        offs.append(pos)
        pos += (L + 255) & ~255
    t = torch.empty(pos + 256, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for i, (o, L) in enumerate(zip(offs, lens)):
        qsmd5.synth_fill_lcg(t.data_ptr() + o, 0, L, 7000 + i, 1, s)
    torch.cuda.synchronize()
    chunks = [(t.data_ptr() + o, L) for o, L in zip(offs, lens)]
    dt, digs = timed(lambda: qsmd5.hash_batch(chunks), reps)
    ok = [d.hex() for d in digs] == gr["md5"]
    tot = sum(lens)
    emit({"config": 4, "workload": "ragged: %d chunks, 0 B..64 MiB (log-uniform 8 KiB-64 MiB, "
                                   "seed 7) = %.2f GiB, device-resident" % (len(lens), tot / GiB),
          "value": round(tot / GiB / dt, 3), "unit": "GiB/s", "seconds": round(dt, 4),
          "longest_chunk_MiB": round(max(lens) / MiB, 2),
          "chain_bound_s": "wall >= longest chunk / per-chain rate",
          "parity": "ok: %d/%d == reference golden" % (len(lens), len(lens)) if ok else "FAIL"})
    del t
    sweep = []
    extra = [int(x) for x in os.environ.get("QSMD5_SWEEP_EXTRA_MIB", "").split(",") if x]
    for sw in gr["sweep"] + [{"mib": m, "seed0": 900000 + m, "md5": None} for m in extra]:
        L = sw["mib"] * MiB
        nb = 512
        tt = torch.empty(nb * L, dtype=torch.uint8, device="cuda")
        qsmd5.synth_fill_lcg(tt.data_ptr(), L, L, sw["seed0"], nb, s)
        torch.cuda.synchronize()
        ch = [(tt.data_ptr() + i * L, L) for i in range(nb)]
        dt, digs = timed(lambda: qsmd5.hash_batch(ch), reps)
        if sw["md5"] is None:  # extra sizes: no golden; the first 8 against the oracle
            from oracle_util import md5_many
            host = tt[:8 * L].cpu().numpy()
            ok = digs[:8] == md5_many([(host.ctypes.data + i * L, L) for i in range(8)])
            del host
        else:
            ok = [d.hex() for d in digs[:len(sw["md5"])]] == sw["md5"]
        sweep.append({"bufsize_MiB": sw["mib"], "batch": nb, "GiBps": round(nb * L / GiB / dt, 3),
                      "ms": round(dt * 1e3, 3), "parity": "ok" if ok else "FAIL"})
        del tt
    emit({"config": "4-sweep", "workload": "-b bufsize sweep, 512 chunks each, device-resident, "
                                           "synchronous qsmd5_hash_batch", "results": sweep})


def config4_split(reps):
    """Config 4 under QSMD5_BACKEND=auto, where a ragged batch splits: its
    longest chunks go to the CPU threads (QSMD5_CPU_THREADS, default 4) while
    the GPU hashes the rest.  Device-resident and pageable host-resident, each
    against the same batch on the GPU alone (QSMD5_FLAG_GPU_ONLY)."""
    import numpy as np
    import torch
    import qsmd5
    gr = gold("ragged.json")
    lens = gr["lengths"]
    offs, pos = [], 0
    for L in lens:
        offs.append(pos)
        pos += (L + 255) & ~255
    t = torch.empty(pos + 256, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for i, (o, L) in enumerate(zip(offs, lens)):
        qsmd5.synth_fill_lcg(t.data_ptr() + o, 0, L, 7000 + i, 1, s)
    torch.cuda.synchronize()
    host = t.cpu().numpy()
    tot = sum(lens)
    prev = os.environ.get("QSMD5_BACKEND")
    os.environ["QSMD5_BACKEND"] = "auto"
    try:
        for where, base in (("device-resident", t.data_ptr()), ("pageable host", host.ctypes.data)):
            chunks = [(base + o, L) for o, L in zip(offs, lens)]
            res = {}
            for mode, flags in (("split", 0), ("gpu_only", qsmd5.FLAG_GPU_ONLY)):
                dt, digs = timed(lambda: qsmd5.hash_batch(chunks, flags=flags), reps)
                res[mode] = (dt, [d.hex() for d in digs] == gr["md5"], qsmd5.last_backend())
            emit({"config": "4-split", "workload": "ragged: %d chunks, 0 B..64 MiB = %.2f GiB, %s, "
                                                   "QSMD5_BACKEND=auto" % (len(lens), tot / GiB, where),
                  "cpu_threads": int(os.environ.get("QSMD5_CPU_THREADS", "4")),
                  "split": {"GiBps": round(tot / GiB / res["split"][0], 3),
                            "seconds": round(res["split"][0], 4),
                            "backend": {1: "gpu", 2: "cpu", 3: "gpu+cpu"}.get(res["split"][2])},
                  "gpu_only": {"GiBps": round(tot / GiB / res["gpu_only"][0], 3),
                               "seconds": round(res["gpu_only"][0], 4)},
                  "parity": "ok: %d/%d == reference golden, both modes" % (len(lens), len(lens))
                  if res["split"][1] and res["gpu_only"][1] else "FAIL"})
    finally:
        if prev is None:
            os.environ.pop("QSMD5_BACKEND", None)
        else:
            os.environ["QSMD5_BACKEND"] = prev
    del t, host


def config5(reps, n=10000):
    import torch
    import qsmd5
    L = 10 * MiB
    g = gold("batch_10MiB.json")["md5"][:n]
    t = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    qsmd5.synth_fill_lcg(t.data_ptr(), L, L, 12345, n, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    chunks = [(t.data_ptr() + i * L, L) for i in range(n)]
    dt, digs = timed(lambda: qsmd5.hash_batch(chunks), reps)
    ok = [d.hex() for d in digs] == g
    emit({"config": 5, "workload": "%d x 10 MiB (%.1f GiB) device-resident on one GPU" % (
        n, n * L / GiB), "value": round(n * L / GiB / dt, 3), "unit": "GiB/s",
        "seconds": round(dt, 4), "kernel": "pc" if qsmd5.kernel_choice(n) == 1 else "v1",
        "parity": "ok: %d/%d == reference golden" % (n, n) if ok else "FAIL"})
    del t


def pool(reps, n=512):
    """Pooled part buffers handed out in any order: n x 10 MiB device buffers cut
    from one allocation at an exact 10 MiB stride, passed to qsmd5_hash_batch in
    pool order and in a shuffled order (a buffer pool's free list).  The runtime
    orders equal-length lanes by address, so both run at the same rate."""
    import random
    import torch
    import qsmd5
    L = 10 * MiB
    g = gold("batch_10MiB.json")["md5"][:n]
    t = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    qsmd5.synth_fill_lcg(t.data_ptr(), L, L, 12345, n, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    perm = list(range(n))
    random.Random(5).shuffle(perm)
    res = {}
    for name, order in (("pool order", list(range(n))), ("shuffled", perm)):
        chunks = [(t.data_ptr() + i * L, L) for i in order]
        dt, digs = timed(lambda: qsmd5.hash_batch(chunks), reps)
        ok = [d.hex() for d in digs] == [g[i] for i in order]
        res[name] = {"GiBps": round(n * L / GiB / dt, 3), "ms": round(dt * 1e3, 3),
                     "parity": "ok" if ok else "FAIL"}
    emit({"config": "pool", "workload": "%d x 10 MiB device buffers at an exact 10 MiB stride, "
                                        "synchronous qsmd5_hash_batch" % n, "results": res})
    del t


def saturation(reps, L=64 * 1024, pad=4352, n=131072, warm_s=0.5):
    """Throughput regime: 131072 independent chains (one wave per 64, 8 waves per
    CU = one resident round), where the coalesced kernel runs instead of the
    latency kernel.  Reports the median and best of >= 10 launches, timed after
    >= warm_s seconds of untimed launches: the chip raises its clock over the
    first tens of ms of load (1.6 -> 1.9 GHz in the per-wave stamps,
    profiles/r05_stamps.jsonl), and without this warm-up a 10-launch series of
    short launches is timed mostly inside that ramp (round 5)."""
    import torch
    import qsmd5
    from oracle_util import md5_many
    S = L + pad  # skewed stride: lanes walk in lockstep, avoid one-channel strides
    t = torch.empty(n * S, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    qsmd5.synth_fill_lcg(t.data_ptr(), S, L, 5, n, s.cuda_stream)
    desc = torch.empty((n, 2), dtype=torch.int64)
    desc[:, 0] = t.data_ptr() + torch.arange(n, dtype=torch.int64) * S
    desc[:, 1] = L
    desc = desc.cuda()
    dig = torch.zeros((n, 16), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    import time
    t_warm, warm = time.time(), 0
    while time.time() - t_warm < warm_s:
        for _ in range(4):
            qsmd5.hash_device(desc.data_ptr(), dig.data_ptr(), n, stream=s.cuda_stream,
                              flags=qsmd5.FLAG_ALIGNED16)
        warm += 4
        torch.cuda.synchronize()
    reps = max(reps, 10)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps + 1)]
    for a, b in ev:
        a.record(s)
        qsmd5.hash_device(desc.data_ptr(), dig.data_ptr(), n, stream=s.cuda_stream,
                          flags=qsmd5.FLAG_ALIGNED16)
        b.record(s)
    torch.cuda.synchronize()
    times = sorted(a.elapsed_time(b) for a, b in ev[1:])
    med, best = times[len(times) // 2], times[0]
    host = t[:64 * S].cpu().numpy()
    want = md5_many([(host.ctypes.data + i * S, L) for i in range(64)])
    ok = [bytes(r) for r in dig[:64].cpu().numpy()] == want
    gbs = n * L / (med * 1e-3) / 1e9
    emit({"config": "saturation", "workload": "%d x %d KiB device-resident, stride +%d B (kernel %s)" % (
        n, L // 1024, pad, ["v1", "pc", "coal", "pc2"][qsmd5.kernel_choice(n, qsmd5.FLAG_ALIGNED16)]),
        "GiBps": round(n * L / GiB / (med * 1e-3), 1), "GBps": round(gbs, 1),
        "frac_of_hbm_peak": round(gbs / HBM_PEAK_GBS, 4), "kernel_ms_median": round(med, 3),
        "kernel_ms_best": round(best, 3), "launches": reps, "warmup_launches": warm,
        "best_frac_of_hbm_peak": round(n * L / (best * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        "parity": "ok (64 sampled chunks vs oracle)" if ok else "FAIL"})
    del t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="1,3,4,5,sat")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    import qsmd5
    torch.cuda.set_device(0)
    assert qsmd5.lib().qsmd5_init(0) == 0
    for c in args.configs.split(","):
        c = c.strip()
        if c == "1":
            config1()
        elif c == "3":
            config3(args.reps)
        elif c == "small":
            many_small(args.reps)
        elif c == "5h":
            config3(args.reps, n=10000, label=" -- BASELINE config 5 host-resident (97.7 GiB)")
        elif c == "3cmp":  # pinned vs pageable at equal sizes
            for n in (1024, 4096):
                config3(args.reps, n=n)
                config3_pageable(args.reps, n=n)
        elif c == "3cols":  # host batches across sizes, for column-width sweeps
            for n in (64, 1024, 4096):
                config3_pageable(args.reps, n=n)
        elif c == "3p":
            config3_pageable(args.reps)
        elif c == "4":
            config4(args.reps)
        elif c == "4split":
            config4_split(args.reps)
        elif c == "5":
            config5(args.reps)
        elif c == "satpad":  # exact power-of-two strides vs the padded default
            for L in (64 * 1024, 256 * 1024):
                for pad in (0, 4352):
                    saturation(args.reps, L=L, pad=pad)
                    torch.cuda.empty_cache()
        elif c == "tiny":  # device-resident tiny chunks: the per-chain fixed cost
            for L, n in ((1024, 1 << 20), (4096, 1 << 20), (16384, 1 << 19)):
                saturation(args.reps, L=L, pad=0, n=n)
                torch.cuda.empty_cache()
        elif c == "satsweep":  # round 5: the coalesced kernel's rate against chunk length
            for kib in (16, 32, 64, 128, 256):
                saturation(args.reps, L=kib * 1024)
                torch.cuda.empty_cache()
        elif c == "sat64":
            saturation(args.reps)
        elif c == "sat256":
            saturation(args.reps, L=256 * 1024)
        elif c == "pool":
            pool(args.reps)
        elif c == "sat":
            saturation(args.reps)
            torch.cuda.empty_cache()
            saturation(args.reps, L=256 * 1024)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
