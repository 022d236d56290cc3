"""Process-level behaviour of the GPU path on an MI355X.

- init after fork: qsfs daemonises inside fuse_main() and starts its threads in
  qsfs_init afterwards (Operations.cpp:1520-1549, Mounter.cpp:90-95); the
  library initialises lazily, so a child forked before any GPU use hashes
  correctly, and so does the parent afterwards;
- several processes hashing on one GPU at once (qsfs instances per mount);
- the N>1 bench flow (sharding, digest gather, max-over-ranks timing, one
  JSON line) rehearsed with 2 ranks on the one GPU over gloo.
Each case runs in child processes, never in the (GPU-initialised) pytest
process itself.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

PY = sys.executable
ENV = dict(os.environ, PYTHONPATH=os.pathsep.join(
    [os.path.join(ROOT, "qsfs-fuse_amd"), os.path.join(ROOT, "tests")]))

FORK_SCRIPT = r'''
import os, sys
import qsmd5
L = qsmd5.lib()          # library loaded, no HIP call yet
pid = os.fork()
if pid == 0:             # the daemon side of fuse_main's fork
    try:
        ok = qsmd5.md5("abc") == "900150983cd24fb0d6963f7d28e17f72"
        ok = ok and qsmd5.hash_batch([b"x" * 1000, b""])[1].hex() == "d41d8cd98f00b204e9800998ecf8427e"
    except Exception as e:
        print("child error", e, file=sys.stderr)
        ok = False
    os._exit(0 if ok else 3)
_, st = os.waitpid(pid, 0)
child_ok = os.WIFEXITED(st) and os.WEXITSTATUS(st) == 0
parent_ok = qsmd5.md5("message digest") == "f96b697d7cb7938d525a2f31aaf161d0"
print("child_ok=%s parent_ok=%s" % (child_ok, parent_ok))
sys.exit(0 if child_ok and parent_ok else 1)
'''

SHUTDOWN_SCRIPT = r'''
import ctypes, os, sys
import qsmd5
from oracle_util import md5_ref  # the pinned oracle (tests/test_oracle.py)
buf = bytearray(os.urandom((3 << 20) + 5))
view = (ctypes.c_uint8 * len(buf)).from_buffer(buf)
addr = ctypes.addressof(view)
want = [md5_ref(bytes(buf)), md5_ref(bytes(buf[7:1000007]))]
chunks = [(addr, len(buf)), (addr + 7, 1000000)]
for cycle in range(3):
    qsmd5.register_host(addr, len(buf))          # (re)initialises the runtime
    p = qsmd5.alloc_pinned(1 << 20)
    ctypes.memmove(p, addr, 1 << 20)
    got = qsmd5.hash_batch(chunks + [(p, 1 << 20)])
    assert got[:2] == want and got[2] == md5_ref(bytes(buf[:1 << 20])), cycle
    qsmd5.free_pinned(p)
    if cycle == 2:
        qsmd5.unregister_host(addr)              # the caller's own unregister, then
    qsmd5.shutdown()                             # shutdown releases what is left
    qsmd5.shutdown()                             # idempotent
st = qsmd5.stats()
assert st["cpu_batches"] == 0 and st["gpu_batches"] == 3, st
print("shutdown cycles ok")
'''

FORK_AFTER_INIT_SCRIPT = r'''
import os, sys, signal
import qsmd5
L = qsmd5.lib()
assert L.qsmd5_init(0) == 0                       # parent initialised the GPU runtime
assert qsmd5.hash_batch([b"abc"], flags=qsmd5.FLAG_GPU_ONLY)[0].hex() == "900150983cd24fb0d6963f7d28e17f72"
pid = os.fork()
if pid == 0:   # must not touch the parent's HIP state
    signal.alarm(60)
    try:
        ok = L.qsmd5_init(0) == qsmd5.ENODEV
        try:
            qsmd5.hash_batch([b"abc"], flags=qsmd5.FLAG_GPU_ONLY)
            ok = False
        except qsmd5.Md5Error as e:
            ok = ok and e.code == qsmd5.ENODEV
        ok = ok and qsmd5.md5("message digest") == "f96b697d7cb7938d525a2f31aaf161d0"
        ok = ok and qsmd5.last_backend() == qsmd5.BACKEND_CPU and qsmd5.device_count() == 0
        ok = ok and L.qsmd5_shutdown() == 0       # drops the handles without a HIP call
    except Exception as e:
        print("child error", e, file=sys.stderr)
        ok = False
    os._exit(0 if ok else 3)
_, st = os.waitpid(pid, 0)
child_ok = os.WIFEXITED(st) and os.WEXITSTATUS(st) == 0
parent_ok = qsmd5.hash_batch([b"a"], flags=qsmd5.FLAG_GPU_ONLY)[0].hex() == "0cc175b9c0f1b6a831c399e269772661"
print("child_ok=%s parent_ok=%s" % (child_ok, parent_ok))
sys.exit(0 if child_ok and parent_ok else 1)
'''

FORK_AFTER_SHUTDOWN_SCRIPT = r'''
import os, sys, signal
import qsmd5
L = qsmd5.lib()
assert L.qsmd5_init(0) == 0
assert qsmd5.hash_batch([b"abc"], flags=qsmd5.FLAG_GPU_ONLY)[0].hex() == "900150983cd24fb0d6963f7d28e17f72"
assert L.qsmd5_shutdown() == 0                    # state back to "not initialised" ...
inits = qsmd5.stats()["inits"]
assert inits == 1, qsmd5.stats()
pid = os.fork()                                   # ... and only then the fork
if pid == 0:
    signal.alarm(60)
    try:
        ok = L.qsmd5_init(0) == qsmd5.ENODEV
        try:
            qsmd5.hash_batch([b"abc"], flags=qsmd5.FLAG_GPU_ONLY)
            ok = False
        except qsmd5.Md5Error as e:
            ok = ok and e.code == qsmd5.ENODEV
        ok = ok and qsmd5.md5("message digest") == "f96b697d7cb7938d525a2f31aaf161d0"
        ok = ok and L.qsmd5_shutdown() == 0 and L.qsmd5_init(0) == qsmd5.ENODEV
        st = qsmd5.stats()
        ok = ok and st["inits"] == inits          # no HIP initialisation ran in the child
        if not ok:
            print("child stats", st, file=sys.stderr)
    except Exception as e:
        print("child error", e, file=sys.stderr)
        ok = False
    os._exit(0 if ok else 3)
_, st = os.waitpid(pid, 0)
child_ok = os.WIFEXITED(st) and os.WEXITSTATUS(st) == 0
parent_ok = qsmd5.hash_batch([b"a"], flags=qsmd5.FLAG_GPU_ONLY)[0].hex() == "0cc175b9c0f1b6a831c399e269772661"
parent_ok = parent_ok and qsmd5.stats()["inits"] == 2     # the parent re-initialised
print("child_ok=%s parent_ok=%s" % (child_ok, parent_ok))
sys.exit(0 if child_ok and parent_ok else 1)
'''

LOG_SINK_GPU_SCRIPT = r'''
import ctypes, sys
import qsmd5
got = []
qsmd5.set_log_callback(lambda level, msg: got.append((level, msg)))
bufs = [(ctypes.c_uint8 * (1 << 20))() for _ in range(64)]
qsmd5.hash_batch([(ctypes.addressof(b), 1 << 20) for b in bufs], flags=qsmd5.FLAG_GPU_ONLY)
qsmd5.hash_batch([b"abc"], flags=qsmd5.FLAG_CPU_ONLY)
for level, msg in got:
    print("%d|%s" % (level, msg))
'''

WORKER_SCRIPT = r'''
import sys, ctypes
import qsmd5
from oracle_util import lcg_bytes, md5_many
seed = int(sys.argv[1])
bufs = [lcg_bytes(seed * 100 + i, (1 << 20) + 37 * i) for i in range(24)]
want = md5_many([(b, (1 << 20) + 37 * i) for i, b in enumerate(bufs)])
for _ in range(3):
    got = qsmd5.hash_batch([(ctypes.addressof(b), (1 << 20) + 37 * i) for i, b in enumerate(bufs)])
    if got != want:
        sys.exit(2)
print("worker", seed, "ok")
'''


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_init_after_fork():
    out = subprocess.run([PY, "-c", FORK_SCRIPT], env=ENV, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "child_ok=True parent_ok=True" in out.stdout


@pytest.mark.parametrize("devices", ["", "0,0"])
def test_shutdown_releases_and_reinitialises(devices):
    """qsmd5_shutdown (a daemon's exit path): three cycles of register a
    pageable buffer + pinned pool + batch + shutdown; each later call
    re-initialises, a registration released by shutdown can be made again,
    and every digest matches the oracle.  "0,0" binds two contexts to the GPU."""
    env = dict(ENV)
    env.pop("QSMD5_DEVICES", None)
    if devices:
        env["QSMD5_DEVICES"] = devices
    out = subprocess.run([PY, "-c", SHUTDOWN_SCRIPT], env=env, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "shutdown cycles ok" in out.stdout


@pytest.mark.cpu_backend
def test_fork_after_init_child_hashes_on_cpu():
    """A child forked after the runtime initialised cannot use the parent's
    HIP state: init and a GPU-only batch fail with -ENODEV without a HIP
    call, auto routing hashes on the CPU, and the parent keeps its GPU."""
    env = dict(ENV, QSMD5_BACKEND="auto")
    out = subprocess.run([PY, "-c", FORK_AFTER_INIT_SCRIPT], env=env, capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "child_ok=True parent_ok=True" in out.stdout


@pytest.mark.cpu_backend
def test_fork_after_shutdown_child_makes_no_hip_call():
    """a child forked after the parent initialised AND shut the
    runtime down still makes no HIP call: qsmd5_init, a GPU-only batch and a
    re-init after the child's own shutdown return -ENODEV, the process's
    initialisation count (qsmd5_stats.inits) stays where the fork left it,
    and auto routing hashes on the CPU."""
    env = dict(ENV, QSMD5_BACKEND="auto")
    out = subprocess.run([PY, "-c", FORK_AFTER_SHUTDOWN_SCRIPT], env=env, capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "child_ok=True parent_ok=True" in out.stdout


@pytest.mark.cpu_backend
def test_log_callback_names_the_bound_gpu_and_backends():
    """qsmd5_set_log_callback on the MI355X: the GPU bound
    at initialisation (gfx950, its CU count) and each call's backend, reason,
    chunk count and bytes reach the host's logger at LogLevel Info, and
    nothing of it reaches stderr."""
    env = dict(ENV, QSMD5_BACKEND="auto")
    out = subprocess.run([PY, "-c", LOG_SINK_GPU_SCRIPT], env=env, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    lines = [ln.split("|", 1) for ln in out.stdout.splitlines() if "|" in ln]
    assert any(lvl == "0" and m.startswith("qsmd5: bound GPU") and "gfx950" in m for lvl, m in lines), lines
    assert ["0", "qsmd5: backend=gpu reason=forced chunks=64 bytes=67108864"] in lines, lines
    assert ["0", "qsmd5: backend=cpu reason=forced chunks=1 bytes=3"] in lines, lines
    assert "qsmd5:" not in out.stderr, out.stderr


def test_concurrent_processes_one_gpu():
    procs = [subprocess.Popen([PY, "-c", WORKER_SCRIPT, str(k)], env=ENV,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for k in range(3)]
    for p in procs:
        o, e = p.communicate(timeout=300)
        assert p.returncode == 0, o + e


def test_bench_two_rank_rehearsal():
    cmd = [PY, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--batch", "64", "--rehearse-gloo", "--config5-parts", "40", "--config5-reps", "1"]
    out = subprocess.run(cmd, env=ENV, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["config"]["global_batch"] == 128
    assert r["parity"].startswith("ok: 128/128")
    assert r["cpu_baseline"] is None and r["scaling"] == "weak"
    c5 = r["config5_host"]
    assert c5["parts_per_rank"] == [20, 20] and c5["parity"] == "ok: 40/40 digests == reference golden"
    pg = r["process_group"]  # the group's own account: two gloo ranks sharing one card
    assert pg["backend"] == "gloo" and pg["world_size"] == 2 and pg["distinct_gpus"] == 1
    assert [x["parts"] for x in pg["ranks"]] == [64, 64] and {x["device"] for x in pg["ranks"]} == {0}


def test_bench_rehearsal_rank_without_parts():
    """Three ranks share the card over gloo and the config5_host object has
    only two parts: rank 0 holds none (an empty pinned shard, no launch, an
    empty digest block in the gather), and every digest still arrives."""
    cmd = [PY, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "3",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "3", "--steps", "1", "--warmup", "1",
           "--batch", "16", "--rehearse-gloo", "--config5-parts", "2", "--config5-reps", "1",
           "--config5-warmup", "0"]
    out = subprocess.run(cmd, env=ENV, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 3 and r["parity"].startswith("ok: 48/48")
    c5 = r["config5_host"]
    assert c5["parts"] == 2 and c5["parts_per_rank"] == [0, 1, 1]
    assert c5["parity"] == "ok: 2/2 digests == reference golden"


def test_bench_rccl_path_world_one():
    """The RCCL path of bench.py (nccl process group bound to the device,
    all_gather_into_tensor of the digests, all_reduce MAX of the time) run at
    world size 1 under torch.distributed.run: what every rank does on the
    driver's 8-GPU node, minus the peers."""
    cmd = [PY, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "2", "--warmup", "1",
           "--batch", "64", "--dist-always", "--no-cpu-baseline", "--config5-parts", "32",
           "--config5-reps", "1"]
    out = subprocess.run(cmd, env=ENV, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 1 and r["config"]["global_batch"] == 64
    assert r["parity"].startswith("ok: 64/64")
    c5 = r["config5_host"]
    assert c5["collective"].startswith("RCCL") and c5["parity"] == "ok: 32/32 digests == reference golden"
    for pg in (r["process_group"], c5["process_group"]):  # RCCL's own world, over its own GPU
        assert pg["backend"] == "nccl" and pg["world_size"] == 1 and pg["distinct_gpus"] == 1
        assert pg["ranks"][0]["pci"] is not None
    assert r["process_group"]["ranks"][0]["parts"] == 64 and c5["process_group"]["ranks"][0]["parts"] == 32


def _bare_env():
    """The driver's environment for `python bench.py --gpus N`: no launcher variables."""
    env = dict(ENV)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def test_bench_forms_two_ranks_itself_on_the_card():
    """`bench.py --gpus 2 --rehearse-gloo` with no launcher in front (VERDICT r04
    item 1): bench.py starts both rank processes itself; they share the box's
    one card over gloo and the group reports two ranks."""
    cmd = [PY, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--batch", "64", "--rehearse-gloo", "--config5-parts", "40", "--config5-reps", "1"]
    out = subprocess.run(cmd, env=_bare_env(), capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["parity"].startswith("ok: 128/128")
    assert r["launcher"] == "bench.py: 2 child processes, one per GPU"
    pg = r["process_group"]
    assert pg["world_size"] == 2 and [x["rank"] for x in pg["ranks"]] == [0, 1]
    assert r["config5_host"]["parts_per_rank"] == [20, 20]


def test_bench_parity_checks_the_timed_steps_own_digests():
    """the digest tables are zeroed after the warm-up and
    the first and last timed steps write to different tables, so parity holds
    only if the timed launches themselves produced every digest."""
    cmd = [PY, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1", "--no-config5",
           "--no-cpu-baseline"]
    out = subprocess.run(cmd, env=_bare_env(), capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 1 and r["parity"] == "ok: 512/512 digests == reference golden"
    assert "launcher" not in r  # the N = 1 line keeps BENCH_r03's keys
