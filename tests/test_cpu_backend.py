"""The library's CPU backend (qsfs-fuse_amd/csrc/md5_cpu.h) and the routing
around it, on the CPU (no GPU needed).

SURVEY.md §8b: "The backend is chosen by size: CPU below a threshold, GPU
above" and "GPU failure falls back to CPU and returns the same digest"; §5:
an env knob selects auto/cpu/gpu and the backend is logged.  This CPU MD5 is
product code inside libqsmd5.so, so before it may answer for the GPU it is
pinned here against every committed golden fixture (produced by the
reference's own MD5.cpp, tests/golden/make_golden.py), exactly as the oracle
is in test_oracle.py.  The oracle itself is only the fixture generator's
restatement: libqsmd5.so never links or loads it (checked below).

Everything here goes through the C-ABI with QSMD5_FLAG_CPU_ONLY or
QSMD5_BACKEND=cpu/auto; without a GPU, auto mode takes the fallback path.
"""
import ctypes
import errno
import os
import random
import subprocess

import pytest

import qsmd5
from conftest import ROOT
from oracle_util import lcg_bytes, md5_many

CPU = qsmd5.FLAG_CPU_ONLY
MiB = 1 << 20


def _hex_all(chunks, flags=CPU):
    return [d.hex() for d in qsmd5.hash_batch(chunks, flags=flags)]


def test_rfc1321(golden):
    for c in golden("rfc1321.json")["cases"]:
        assert _hex_all([c["text"].encode()]) == [c["md5"]]


def test_lcg_lengths_all_padding_edges(golden):
    g = golden("lcg_lengths.json")
    big = max(c["len"] for c in g["cases"])
    data = lcg_bytes(g["seed"], big)
    addr = ctypes.addressof(data)
    got = _hex_all([(addr, c["len"]) for c in g["cases"]])
    assert got == [c["md5"] for c in g["cases"]]
    # unaligned starts: the same bytes at offsets 1..7 hash the same
    for off in range(1, 8):
        buf = (ctypes.c_uint8 * (4096 + 8))()
        ctypes.memmove(ctypes.addressof(buf) + off, addr, 4096)
        assert _hex_all([(ctypes.addressof(buf) + off, 4096)]) == \
            [c["md5"] for c in g["cases"] if c["len"] == 4096]


def test_stream_pieces_class(golden, monkeypatch):
    """The MD5 class (qsmd5_ctx) under QSMD5_BACKEND=cpu, update() in pieces."""
    monkeypatch.setenv("QSMD5_BACKEND", "cpu")
    g = golden("stream_pieces.json")
    data = lcg_bytes(g["seed"], g["len"])
    base = ctypes.addressof(data)
    for case in g["cases"]:
        h = qsmd5.MD5()
        off = 0
        for cut in case["cuts"]:
            h.update((base + off, cut))
            off += cut
        assert h.finalize().hexdigest() == case["md5"], case["cuts"][:4]
        assert h.hexdigest() == case["md5"]
        # the reference's update() after finalize() leaves the digest as it was
        h.update(b"more bytes")
        assert h.finalize().hexdigest() == case["md5"]


def test_md5_copy_forks_the_state(monkeypatch):
    """qsmd5_ctx_copy on a CPU context: the reference MD5's value semantics."""
    monkeypatch.setenv("QSMD5_BACKEND", "cpu")
    from md5_copy_cases import run_copy_cases
    run_copy_cases(qsmd5, lambda d, off, n: d[off:off + n])


def test_ragged_and_sweep(golden):
    g = golden("ragged.json")
    bufs = [lcg_bytes(7000 + i, L) for i, L in enumerate(g["lengths"])]
    assert _hex_all([(ctypes.addressof(b), L) for b, L in zip(bufs, g["lengths"])]) == g["md5"]
    del bufs
    for s in g["sweep"]:
        L = s["mib"] << 20
        bufs = [lcg_bytes(s["seed0"] + i, L) for i in range(len(s["md5"]))]
        assert _hex_all([(ctypes.addressof(b), L) for b in bufs]) == s["md5"], s["mib"]


def test_batch_10mib_prefix(golden):
    g = golden("batch_10MiB.json")
    bufs = [lcg_bytes(12345 + i, g["len"]) for i in range(24)]
    assert _hex_all([(ctypes.addressof(b), g["len"]) for b in bufs]) == g["md5"][:24]


def test_truncate32(golden):
    """>= 4 GiB: full RFC 1321 length by default; QSMD5_FLAG_REF_TRUNCATE32
    reproduces the reference's 32-bit size_type (MD5.h:53, MD5.cpp:106)."""
    g = golden("truncate32.json")
    data = lcg_bytes(g["seed"], g["len"])
    a = ctypes.addressof(data)
    assert _hex_all([(a, g["len"])]) == [g["full_md5"]]
    assert _hex_all([(a, g["len"])], CPU | qsmd5.FLAG_REF_TRUNCATE32) == [g["reference_md5"]]


def test_auto_mode_without_gpu_falls_back(monkeypatch):
    """No GPU here: auto mode still returns the digest (the fallback path) and
    says so; forced GPU fails loudly with -ENODEV."""
    if qsmd5.device_count() > 0:
        pytest.skip("GPU present")
    monkeypatch.setenv("QSMD5_BACKEND", "auto")
    monkeypatch.setenv("QSMD5_ROUTE_LANES", "0")  # the scalar model: 40 x 256 KiB prices to the GPU
    big = lcg_bytes(12345, 10 << 20)
    many = [(ctypes.addressof(big) + i * (256 << 10), 256 << 10) for i in range(40)]
    before = qsmd5.stats()
    assert qsmd5.route([256 << 10] * 40) == qsmd5.BACKEND_GPU  # GPU would be picked ...
    got = qsmd5.hash_batch(many)  # ... fails (no device), and the CPU answers
    assert got == qsmd5.hash_batch(many, flags=CPU)
    assert qsmd5.last_backend() == qsmd5.BACKEND_CPU
    after = qsmd5.stats()
    assert after["fallbacks"] == before["fallbacks"] + 1
    assert qsmd5.md5("abc") == "900150983cd24fb0d6963f7d28e17f72"  # routed by size
    with pytest.raises(qsmd5.Md5Error) as e:
        qsmd5.hash_batch(many, flags=qsmd5.FLAG_GPU_ONLY)
    assert e.value.code == -errno.ENODEV
    with pytest.raises(qsmd5.Md5Error) as e:
        qsmd5.hash_batch([b"x"], flags=qsmd5.FLAG_GPU_ONLY | CPU)
    assert e.value.code == -errno.EINVAL


def test_bad_backend_name(monkeypatch):
    monkeypatch.setenv("QSMD5_BACKEND", "fpga")
    with pytest.raises(qsmd5.Md5Error) as e:
        qsmd5.hash_one(b"abc")
    assert e.value.code == -errno.EINVAL


def test_routing_rule(monkeypatch):
    """Size routing (qsmd5_route): a lone part of any size goes to the CPU (the
    unchanged per-part md5() call site, QSClient.cpp:369-371); whole files'
    parts and large object batches go to the GPU; the break-even moves with
    QSMD5_CPU_THREADS as the cost model says."""
    monkeypatch.delenv("QSMD5_CPU_THREADS", raising=False)
    monkeypatch.setenv("QSMD5_ROUTE_LANES", "0")  # scalar chains (the lanes: test_lane_priced_*)
    monkeypatch.setenv("QSMD5_CPU_LOAD_FEEDBACK", "0")  # the idle-host model exactly
    # the rule at the reference rates (the host's own rates: the test below)
    monkeypatch.setenv("QSMD5_CPU_GIBS", "0.7")
    monkeypatch.setenv("QSMD5_GPU_CHAIN_GIBS", "0.119")
    C, G = qsmd5.BACKEND_CPU, qsmd5.BACKEND_GPU
    MiB = 1 << 20
    for L in (0, 1, 1024, 10 * MiB, 64 * MiB, 4 << 30):
        assert qsmd5.route([L]) == C, L
    assert qsmd5.route([10 * MiB] * 512) == G  # BASELINE config 2
    assert qsmd5.route([10 * MiB] * 10000) == G  # config 5
    assert qsmd5.route([1024] * (1 << 20)) == G  # many small objects

    def break_even(L, lo=1, hi=1 << 16):
        while hi - lo > 1:
            mid = (lo + hi) // 2
            lo, hi = (mid, hi) if qsmd5.route([L] * mid) == C else (lo, mid)
        return hi  # first batch size that goes to the GPU

    n4 = break_even(10 * MiB)
    assert 15 <= n4 <= 40, n4
    monkeypatch.setenv("QSMD5_CPU_THREADS", "1")
    n1 = break_even(10 * MiB)
    assert n1 < n4 and 4 <= n1 <= 10, n1
    # routing is monotone in the batch size for equal parts
    monkeypatch.delenv("QSMD5_CPU_THREADS")
    seq = [qsmd5.route([MiB] * n) for n in range(1, 200)]
    assert seq == sorted(seq, key=lambda b: b == G)


def _predicted_break_even(r, S):
    """First n for which equal host parts of S bytes go to the GPU, by the cost
    model of qsmd5_rt_route.cpp ("backend routing") at rates r."""
    GiB = float(1 << 30)
    T, rc, g, K = r["cpu_threads"], r["cpu_chain_gibs"], r["gpu_chain_gibs"], r["link_gibs"]
    for n in range(1, 1 << 16):
        cpu = 1e3 * (max(S / rc, n * S / (T * rc)) + 0.0 / r["d2h_gibs"]) / GiB
        gpu = r["gpu_call_ms"] + 1e3 * (S / g + n * S / K) / GiB
        if not cpu < gpu:
            return n
    return None


def test_routing_prices_this_hosts_measured_rates(monkeypatch):
    """the CPU rates are timed on this host at the first
    routing decision (qsmd5_get_rates), and the break-even batch moves exactly
    as the cost model predicts when the CPU rate is forced slower or faster
    (QSMD5_CPU_GIBS) or the GPU chain faster (QSMD5_GPU_CHAIN_GIBS)."""
    for k in ("QSMD5_CPU_GIBS", "QSMD5_GPU_CHAIN_GIBS", "QSMD5_LINK_GIBS", "QSMD5_CPU_THREADS"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("QSMD5_ROUTE_LANES", "0")  # the scalar model this test restates
    monkeypatch.setenv("QSMD5_CPU_LOAD_FEEDBACK", "0")
    MiB = 1 << 20
    r = qsmd5.rates()
    assert r["source"] & qsmd5.RATE_CPU_MEASURED and not r["source"] & qsmd5.RATE_CPU_ENV
    assert 0.05 < r["cpu_chain_gibs"] < 10, r
    if "avx512f" in open("/proc/cpuinfo").read():
        assert r["cpu_lane_thread_gibs"] > 2 * r["cpu_chain_gibs"], r  # 16 lanes in one thread
    if qsmd5.device_count() == 0:
        assert r["gpu_chain_gibs"] == 0.119 and not r["source"] & qsmd5.RATE_GPU_MEASURED

    def break_even(L):
        lo, hi = 0, 1 << 16
        while hi - lo > 1:
            mid = (lo + hi) // 2
            lo, hi = (mid, hi) if qsmd5.route([L] * mid) == qsmd5.BACKEND_CPU else (lo, mid)
        return hi

    S = 10 * MiB
    seen = {}
    for cpu in (None, "0.35", "0.7", "1.4"):
        if cpu is None:
            monkeypatch.delenv("QSMD5_CPU_GIBS", raising=False)
        else:
            monkeypatch.setenv("QSMD5_CPU_GIBS", cpu)
        rr = qsmd5.rates()
        if cpu is not None:
            assert rr["cpu_chain_gibs"] == float(cpu) and rr["source"] & qsmd5.RATE_CPU_ENV
        seen[cpu] = break_even(S)
        assert seen[cpu] == _predicted_break_even(rr, S), (cpu, rr)
    assert seen["0.35"] < seen["0.7"] < seen["1.4"]
    assert (seen["0.35"], seen["0.7"], seen["1.4"]) == (13, 25, 53)  # the worked numbers, DESIGN §1
    # a faster GPU chain halves the CPU's share
    monkeypatch.setenv("QSMD5_CPU_GIBS", "0.7")
    monkeypatch.setenv("QSMD5_GPU_CHAIN_GIBS", "0.238")
    rr = qsmd5.rates()
    assert rr["source"] & qsmd5.RATE_GPU_ENV
    assert break_even(S) == _predicted_break_even(rr, S) < seen["0.7"]


def _config4_lengths():
    """BASELINE config 4's shape: 659 chunks, log-uniform 8 KiB-64 MiB."""
    rng = random.Random(7)
    return [int(2 ** rng.uniform(13, 26)) for _ in range(659)]


def test_split_routing_rule(monkeypatch):
    """Ragged batches split: the longest host chunks go to the CPU threads while
    the GPU hashes the rest (qsmd5_route -> BACKEND_SPLIT).  Equal parts and
    many small objects never split; QSMD5_SPLIT=0 turns it off."""
    monkeypatch.delenv("QSMD5_CPU_THREADS", raising=False)
    monkeypatch.setenv("QSMD5_ROUTE_LANES", "0")
    monkeypatch.setenv("QSMD5_CPU_LOAD_FEEDBACK", "0")
    monkeypatch.setenv("QSMD5_CPU_GIBS", "0.7")
    monkeypatch.setenv("QSMD5_GPU_CHAIN_GIBS", "0.119")
    monkeypatch.delenv("QSMD5_SPLIT", raising=False)
    MiB = 1 << 20
    S, G = qsmd5.BACKEND_SPLIT, qsmd5.BACKEND_GPU
    lens = _config4_lengths()
    assert qsmd5.route(lens) == S
    assert qsmd5.route([10 * MiB] * 512) == G
    assert qsmd5.route([10 * MiB] * 512 + [64 * MiB]) == S  # one long straggler
    assert qsmd5.route([1024] * (1 << 16) + [4096]) == G  # the link, not a chain, sets the time
    monkeypatch.setenv("QSMD5_SPLIT", "0")
    assert qsmd5.route(lens) == G
    assert qsmd5.route([10 * MiB] * 512 + [64 * MiB]) == G


def test_split_batch_digests_on_cpu_only_box(monkeypatch):
    """Without a GPU a split batch still returns every digest (its GPU share
    falls back to the CPU) and matches the oracle chunk by chunk."""
    if qsmd5.device_count() > 0:
        pytest.skip("a GPU is visible: routing prices this host's measured rates and the "
                    "batch need not split (the GPU suite covers split batches)")
    monkeypatch.setenv("QSMD5_BACKEND", "auto")
    monkeypatch.setenv("QSMD5_ROUTE_LANES", "0")
    monkeypatch.setenv("QSMD5_CPU_THREADS", "1")  # a small batch that still favours the GPU
    monkeypatch.delenv("QSMD5_SPLIT", raising=False)
    MiB = 1 << 20
    lens = [MiB + 7, 64, 0, MiB, 999] * 10 + [4 * MiB + 3, 3 * MiB]
    assert qsmd5.route(lens) == qsmd5.BACKEND_SPLIT
    bufs = [lcg_bytes(700 + i, L) for i, L in enumerate(lens)]
    chunks = [(ctypes.addressof(b) if L else 0, L) for b, L in zip(bufs, lens)]
    s0 = qsmd5.stats()
    assert qsmd5.hash_batch(chunks) == md5_many(chunks)
    assert qsmd5.last_backend() == qsmd5.BACKEND_CPU
    assert qsmd5.stats()["fallbacks"] == s0["fallbacks"] + 1


def test_log_names_the_backend(tmp_path):
    """QSMD5_LOG=1 logs each call's backend, reason and size."""
    code = ("import sys; sys.path.insert(0, %r); import qsmd5; "
            "qsmd5.hash_batch([b'abc'] * 3, flags=qsmd5.FLAG_CPU_ONLY)"
            % os.path.join(ROOT, "qsfs-fuse_amd"))
    env = dict(os.environ, QSMD5_LOG="1")
    out = subprocess.run(["python", "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "qsmd5: backend=cpu reason=forced chunks=3 bytes=9" in out.stderr


LOG_SINK_SCRIPT = r'''
import ctypes, sys
import qsmd5
got = []
qsmd5.set_log_callback(lambda level, msg: got.append((level, msg)))
qsmd5.hash_batch([b"abc"] * 3, flags=qsmd5.FLAG_CPU_ONLY)
if qsmd5.device_count() == 0:     # auto routing picks the GPU, which is absent here: fallback
    big = (ctypes.c_uint8 * (10 << 20))()
    qsmd5.hash_batch([(ctypes.addressof(big) + i * (256 << 10), 256 << 10) for i in range(40)])
qsmd5.set_log_callback(None)
qsmd5.hash_batch([b"x"], flags=qsmd5.FLAG_CPU_ONLY)   # not seen by the removed sink
for level, msg in got:
    print("%d|%s" % (level, msg))
'''


def test_log_callback_carries_backend_without_stderr():
    """VERDICT r03 item 5 / SURVEY.md §5: qsmd5_set_log_callback hands each
    call's backend, reason and size to the host's logger (qsfs: DebugInfo via
    LogMacros.h) at LogLevel Info, and a GPU that cannot be used at Warn --
    with nothing on stderr, even under QSMD5_LOG=1.  Removing the sink
    restores stderr."""
    env = dict(os.environ, QSMD5_LOG="1", QSMD5_BACKEND="auto", QSMD5_ROUTE_LANES="0",
               PYTHONPATH=os.path.join(ROOT, "qsfs-fuse_amd"))
    out = subprocess.run(["python", "-c", LOG_SINK_SCRIPT], env=env, capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr
    lines = [ln.split("|", 1) for ln in out.stdout.splitlines() if "|" in ln]
    assert ["0", "qsmd5: backend=cpu reason=forced chunks=3 bytes=9"] in lines, out.stdout
    # the removed sink saw nothing more; the default stderr logging is back
    assert not any("chunks=1 bytes=1" in m for _, m in lines), out.stdout
    assert "qsmd5: backend=cpu reason=forced chunks=1 bytes=1" in out.stderr
    assert "chunks=3" not in out.stderr and "GPU" not in out.stderr, out.stderr
    if qsmd5.device_count() == 0:
        levels = {lvl for lvl, m in lines if "GPU" in m}
        assert "1" in levels, out.stdout  # the unusable GPU and the fallback: LOG_WARN
        assert any(m.startswith("qsmd5: backend=cpu reason=fallback chunks=40") for _, m in lines), out.stdout


SINK_SWAP_SCRIPT = r'''
import gc, threading
import qsmd5
stop = threading.Event()
errors = []
def hasher():
    try:
        while not stop.is_set():
            qsmd5.hash_batch([b"abc"] * 4, flags=qsmd5.FLAG_CPU_ONLY)  # logs through the sink
    except Exception as e:
        errors.append(e)
threads = [threading.Thread(target=hasher) for _ in range(3)]
for t in threads:
    t.start()
seen = [0]
for k in range(400):
    qsmd5.set_log_callback(lambda level, msg, k=k: seen.__setitem__(0, seen[0] + 1))
    if k % 50 == 0:
        qsmd5.set_log_callback(None)
    gc.collect()  # a replaced thunk freed here would be called by a hashing thread
stop.set()
for t in threads:
    t.join()
assert not errors, errors
print("swaps ok, %d messages" % seen[0])
'''


def test_log_sink_swaps_while_threads_hash():
    """a replaced sink may still be running on another thread (the
    library never frees it), so the binding keeps every ctypes thunk it ever
    installed; 400 swaps under three hashing threads, with a garbage
    collection after each, must not crash."""
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "qsfs-fuse_amd"))
    out = subprocess.run(["python", "-c", SINK_SWAP_SCRIPT], env=env, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "swaps ok" in out.stdout


def test_product_library_does_not_carry_the_oracle():
    """The CPU backend is the library's own code: libqsmd5.so neither links
    the oracle nor exports or contains its symbols."""
    so = qsmd5.lib_path()
    needed = subprocess.run(["readelf", "-d", so], capture_output=True, text=True).stdout
    assert "md5_oracle" not in needed and "ref_md5" not in needed
    syms = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True).stdout
    assert "oracle_" not in syms and "ref_md5" not in syms
    allsyms = subprocess.run(["nm", so], capture_output=True, text=True).stdout
    assert "oracle_md5" not in allsyms


def test_multibuffer_and_scalar_paths_agree():
    """Every CPU path against the oracle, each in its own process: the AVX-512
    multi-buffer lanes (md5_cpu_mb.cpp, when the host has AVX-512F) in one
    16-lane group per thread and in two interleaved groups (32 lanes,
    QSMD5_CPU_MB_GROUPS=2: 200 chunks on 3 threads fill them), and the scalar
    chain (QSMD5_CPU_MB=0).  Ragged lengths 0..3 MiB at odd offsets, so
    lanes run out at different blocks and are refilled mid-batch, plus tails
    on every side of the 56-byte padding edge."""
    script = r'''
import ctypes, random, sys
sys.path.insert(0, %r); sys.path.insert(0, %r)
import qsmd5
from oracle_util import md5_many
rng = random.Random(77)
lens = [rng.choice([0, 1, 55, 56, 63, 64, 65, 119, 120]) for _ in range(40)]
lens += [rng.randrange(0, 3 << 20) for _ in range(160)]
buf = ctypes.create_string_buffer(bytes(rng.getrandbits(8) for _ in range(1 << 16)) * 80)
chunks, pos = [], 3
for L in lens:
    chunks.append((ctypes.addressof(buf) + pos, L))
    pos = (pos + L + 7) %% (len(buf) - (3 << 20) - 8)
got = qsmd5.hash_batch(chunks, flags=qsmd5.FLAG_CPU_ONLY)
assert got == md5_many(chunks), "CPU backend digests differ from the oracle"
print("ok", len(chunks))
''' % (os.path.join(ROOT, "qsfs-fuse_amd"), os.path.join(ROOT, "tests"))
    for mb, groups in (("1", "1"), ("1", "2"), ("0", "1")):  # 16 lanes, 32 lanes, scalar
        env = dict(os.environ, QSMD5_CPU_MB=mb, QSMD5_CPU_THREADS="3", QSMD5_CPU_MB_GROUPS=groups)
        out = subprocess.run([os.sys.executable, "-c", script], env=env, capture_output=True,
                             text=True, timeout=300)
        assert out.returncode == 0 and out.stdout.startswith("ok"), (mb, out.stdout + out.stderr[-2000:])


def test_lane_priced_routing_is_the_default(monkeypatch, golden):
    """Round 5: the multi-buffer lanes are priced for host
    batches by default -- BASELINE config 4's lengths and 64 x 10 MiB stay on
    the CPU, 512 x 10 MiB at one thread still takes the GPU.  QSMD5_ROUTE_LANES=0
    restores the scalar model (split / GPU)."""
    if "avx512f" not in open("/proc/cpuinfo").read():
        pytest.skip("host without AVX-512F: the lanes are never priced")
    G, C, S = qsmd5.BACKEND_GPU, qsmd5.BACKEND_CPU, qsmd5.BACKEND_SPLIT
    lens = golden("ragged.json")["lengths"]
    monkeypatch.setenv("QSMD5_CPU_THREADS", "4")
    monkeypatch.setenv("QSMD5_CPU_LOAD_FEEDBACK", "0")
    monkeypatch.setenv("QSMD5_ROUTE_LANES", "0")
    assert qsmd5.route(lens) == S
    assert qsmd5.route([10 * MiB] * 64) == G
    monkeypatch.delenv("QSMD5_ROUTE_LANES")
    assert qsmd5.route(lens) == C
    assert qsmd5.route([10 * MiB] * 64) == C
    # 512 x 10 MiB is a GPU batch for one CPU thread's lanes on any host; at 4
    # threads a fast AVX-512 host's lanes can outrun the link (the MI355X box's
    # EPYC does, 5 GiB at ~37 GiB/s), which the router then rightly prices
    monkeypatch.setenv("QSMD5_CPU_THREADS", "1")
    assert qsmd5.route([10 * MiB] * 512) == G
    monkeypatch.setenv("QSMD5_CPU_THREADS", "4")
    assert qsmd5.route([10 * MiB]) == C  # a lone part: scalar, as before
    monkeypatch.setenv("QSMD5_CPU_MB", "0")  # no lanes, nothing to price
    assert qsmd5.route(lens) == S


def test_cpu_load_feedback_moves_batches_to_the_gpu(monkeypatch):
    """CPU batches timed slower than priced (a host whose
    cores are busy) lower qsmd5_get_cpu_efficiency, and auto routing then
    prices the CPU that much slower: a batch on the CPU side of the idle
    break-even moves to the GPU.  Here the load is simulated by pricing the
    CPU 8x faster than it runs (QSMD5_CPU_GIBS), so its batches take ~8x their
    estimate; the value relaxes back to 1 when no CPU batch runs
    (QSMD5_CPU_EFF_DECAY_S)."""
    monkeypatch.setenv("QSMD5_ROUTE_LANES", "0")
    monkeypatch.setenv("QSMD5_CPU_MB", "0")  # scalar chains, the rate QSMD5_CPU_GIBS prices
    monkeypatch.setenv("QSMD5_CPU_THREADS", "1")
    monkeypatch.setenv("QSMD5_GPU_CHAIN_GIBS", "0.119")
    monkeypatch.setenv("QSMD5_CPU_LOAD_FEEDBACK", "1")
    monkeypatch.setenv("QSMD5_CPU_EFF_DECAY_S", "1000")
    real = qsmd5.rates()["cpu_chain_gibs"]
    monkeypatch.setenv("QSMD5_CPU_GIBS", "%.4f" % (8 * real))
    n = next(k for k in range(1, 400) if qsmd5.route([MiB] * (k + 1)) == qsmd5.BACKEND_GPU)
    assert qsmd5.route([MiB] * n) == qsmd5.BACKEND_CPU  # n: the largest CPU batch of 1 MiB parts
    data = lcg_bytes(5, 4 * MiB)
    for _ in range(3):  # three slow CPU batches, priced at >= 2 ms each
        qsmd5.hash_batch([(ctypes.addressof(data), 4 * MiB)] * 8, flags=CPU)
    eff = qsmd5.cpu_efficiency()
    assert eff < 0.5, eff
    assert qsmd5.route([MiB] * n) == qsmd5.BACKEND_GPU
    monkeypatch.setenv("QSMD5_CPU_LOAD_FEEDBACK", "0")  # off: the idle-host model again
    assert qsmd5.cpu_efficiency() == 1.0 and qsmd5.route([MiB] * n) == qsmd5.BACKEND_CPU
    monkeypatch.setenv("QSMD5_CPU_LOAD_FEEDBACK", "1")
    monkeypatch.setenv("QSMD5_CPU_EFF_DECAY_S", "0")  # decay "now": the sample has aged out
    import time
    time.sleep(0.01)
    assert qsmd5.cpu_efficiency() > 0.99


def test_shutdown_not_starved_by_overlapping_calls(tmp_path):
    """six threads hash back to back so that some call always holds
    the runtime's call lock; qsmd5_shutdown must still get through (the gate
    in CallScope holds new calls back while it is pending) and the threads'
    later calls must work.  Before the gate it waited until the hashers were
    stopped (20 s, the program's watchdog)."""
    exe = str(tmp_path / "shutdown_starvation")
    subprocess.check_call([
        "g++", "-std=c++17", "-O2", os.path.join(ROOT, "tests", "cpp", "shutdown_starvation.cpp"),
        "-I" + os.path.join(ROOT, "include"), "-L" + os.path.join(ROOT, "qsfs-fuse_amd", "lib"), "-lqsmd5",
        "-lpthread", "-Wl,-rpath," + os.path.join(ROOT, "qsfs-fuse_amd", "lib"), "-o", exe])
    out = subprocess.run([exe, "6"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    import json
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert not r["starved"] and r["shutdown_s"] < 5.0 and r["calls_after"] > 0


def test_background_flag_without_a_gpu_routes_as_usual(monkeypatch):
    """QSMD5_FLAG_BACKGROUND (round 5): a batch whose latency the caller
    hides goes to the GPU whenever one is usable; without one it is routed
    as any batch (a lone part to the CPU), and hashes right."""
    if qsmd5.device_count() > 0:
        pytest.skip("GPU present (tests/test_gpu_routing.py covers the GPU side)")
    monkeypatch.setenv("QSMD5_BACKEND", "auto")
    data = lcg_bytes(31, 3 * MiB)
    assert qsmd5.route([3 * MiB], flags=qsmd5.FLAG_BACKGROUND) == qsmd5.BACKEND_CPU
    got = qsmd5.hash_batch([(ctypes.addressof(data), 3 * MiB)], flags=qsmd5.FLAG_BACKGROUND)
    assert got == md5_many([(data, 3 * MiB)])
