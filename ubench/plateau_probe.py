#!/usr/bin/env python3
"""ubench/plateau_probe.py -- where does the >= 32 MiB part plateau come from?

Device-resident batches of 512 equal parts through qsmd5_hash_batch (latency
kernel), GiB/s best of 3, digests of 8 parts checked against the oracle.
Layouts separate the suspects: part length, the stride between parts, the size
of the allocation they sit in, and one allocation per part.
  python ubench/plateau_probe.py [case ...]
Test/measurement infrastructure, not product code.
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "qsfs-fuse_amd"), os.path.join(ROOT, "tests")]
os.environ.setdefault("QSMD5_BACKEND", "gpu")
MiB, GiB = 1 << 20, 1 << 30
N = 512


def run(name, part, stride, alloc_bytes=None, separate=False, reps=3, n=None):
    global N
    N = n or 512
    import torch
    import qsmd5
    from oracle_util import md5_many
    s = torch.cuda.current_stream().cuda_stream
    bufs = []
    if separate:
        bufs = [torch.empty(part, dtype=torch.uint8, device="cuda") for _ in range(N)]
        ptrs = [b.data_ptr() for b in bufs]
        for i, p in enumerate(ptrs):
            qsmd5.synth_fill_lcg(p, part, part, 5000 + i, 1, s)
    else:
        total = alloc_bytes or (N - 1) * stride + part
        t = torch.empty(total, dtype=torch.uint8, device="cuda")
        bufs = [t]
        ptrs = [t.data_ptr() + i * stride for i in range(N)]
        qsmd5.synth_fill_lcg(t.data_ptr(), stride, part, 5000, N, s)
    torch.cuda.synchronize()
    chunks = [(p, part) for p in ptrs]
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        digs = qsmd5.hash_batch(chunks)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    host = [torch.empty(0)] * 0
    sample = []
    for i in range(8):
        h = (bufs[i] if separate else bufs[0][i * stride:i * stride + part]).cpu().numpy()
        host.append(h)
        sample.append((h.ctypes.data, part))
    ok = digs[:8] == md5_many(sample)
    print(json.dumps({"case": name, "parts": N, "tag": os.environ.get("QSMD5_PROBE_TAG", ""), "part_MiB": part / MiB, "stride_MiB": stride / MiB,
                      "alloc_GiB": round((alloc_bytes or ((N - 1) * stride + part)) / GiB, 2)
                      if not separate else "one per part",
                      "GiBps": round(N * part / GiB / best, 3), "ms": round(best * 1e3, 2),
                      "parity": "ok" if ok else "FAIL"}), flush=True)
    del bufs, host
    torch.cuda.empty_cache()


CASES = {
    "p32_s32": lambda: run("32 MiB parts, 32 MiB stride, 16 GiB alloc", 32 * MiB, 32 * MiB),
    "p32_sep": lambda: run("32 MiB parts, one allocation each", 32 * MiB, 32 * MiB, separate=True),
    "p32_s32k": lambda: run("32 MiB parts, 32 MiB + 16 KiB stride", 32 * MiB, 32 * MiB + 16384),
    "p24_s24": lambda: run("24 MiB parts, 24 MiB stride", 24 * MiB, 24 * MiB),
    "p24_s24_big": lambda: run("24 MiB parts, 24 MiB stride, in a 32 GiB alloc", 24 * MiB, 24 * MiB,
                               alloc_bytes=32 * GiB),
    "p24_s32": lambda: run("24 MiB parts, 32 MiB stride", 24 * MiB, 32 * MiB),
    "p10_s32": lambda: run("10 MiB parts, 32 MiB stride", 10 * MiB, 32 * MiB),
    "p10_s10_big": lambda: run("10 MiB parts, 10 MiB stride, in a 32 GiB alloc", 10 * MiB, 10 * MiB,
                               alloc_bytes=32 * GiB),
    "p64_sep": lambda: run("64 MiB parts, one allocation each", 64 * MiB, 64 * MiB, separate=True),
    "p64_s64": lambda: run("64 MiB parts, 64 MiB stride", 64 * MiB, 64 * MiB),
}

if __name__ == "__main__":
    # QSMD5_SKEW_BLOCKS is read once per process: "skew:<blocks>" re-runs the
    # given cases in a child process with that start skew (0 = off)
    import subprocess
    args = sys.argv[1:]
    if args and args[0].startswith("skew:"):
        for sk in args[0][5:].split(","):
            env = dict(os.environ, QSMD5_SKEW_BLOCKS=sk, QSMD5_PROBE_TAG="skew=%s" % sk)
            r = subprocess.run([sys.executable, __file__] + args[1:], env=env)
            if r.returncode:
                sys.exit(r.returncode)
        sys.exit(0)
    import torch
    import qsmd5
    assert torch.cuda.is_available()
    assert qsmd5.lib().qsmd5_init(0) == 0
    for c in (args or list(CASES)):
        if c in CASES:
            CASES[c]()
        else:  # "p<part MiB>+<pad bytes>[x<parts>]": parts at a stride of part + pad
            spec, _, nparts = c[1:].partition("x")
            part, pad = spec.split("+")
            run("%s x %s MiB parts, +%s B stride pad" % (nparts or 512, part, pad), int(part) * MiB,
                int(part) * MiB + int(pad), n=int(nparts) if nparts else None)
