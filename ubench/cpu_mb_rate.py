"""CPU backend rate, scalar (QSMD5_CPU_MB=0) against the AVX-512 multi-buffer
path (16 messages per thread), on this host: equal parts at an exact stride,
a ragged set and BASELINE config 4's 659 lengths (pageable host), 1 and 4 threads, every digest checked against the oracle."""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, time, json
sys.path.insert(0, %r); sys.path.insert(0, %r)
import numpy as np
import qsmd5
from oracle_util import md5_many
rng = np.random.default_rng(1)
RAGGED = json.load(open(%r))["lengths"]
out = []
for name, lens in (("16 x 10 MiB", [10 << 20] * 16), ("64 x 10 MiB", [10 << 20] * 64),
                   ("256 x 1 MiB", [1 << 20] * 256),
                   ("ragged 200, 8 KiB-16 MiB", [int(x) for x in np.exp(rng.uniform(np.log(8192), np.log(16 << 20), 200))]),
                   ("config 4 lengths: 659 chunks, 0 B-64 MiB", RAGGED)):
    offs, pos = [], 0
    for L in lens:
        offs.append(pos); pos += L
    big = np.frombuffer(rng.bytes(pos), dtype=np.uint8)
    ch = [(big.ctypes.data + o, L) for o, L in zip(offs, lens)]
    got = qsmd5.hash_batch(ch, flags=qsmd5.FLAG_CPU_ONLY)
    ok = got == md5_many(ch)
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter(); qsmd5.hash_batch(ch, flags=qsmd5.FLAG_CPU_ONLY)
        best = min(best, time.perf_counter() - t0)
    out.append({"batch": name, "GiBps": round(sum(lens) / 2**30 / best, 3), "ms": round(best * 1e3, 2), "parity": ok})
print(json.dumps(out))
''' % (os.path.join(ROOT, "qsfs-fuse_amd"), os.path.join(ROOT, "tests"),
       os.path.join(ROOT, "tests", "golden", "ragged.json"))

for mb in ("0", "1"):
    for thr in ("1", "4"):
        env = dict(os.environ, QSMD5_CPU_MB=mb, QSMD5_CPU_THREADS=thr)
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True,
                           timeout=600)
        if r.returncode:
            sys.exit(r.stderr[-2000:])
        print('{"path": "%s", "threads": %s, "results": %s}'
              % ("multi-buffer" if mb == "1" else "scalar", thr, r.stdout.strip()), flush=True)
