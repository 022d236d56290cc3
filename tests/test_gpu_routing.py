"""Backend routing and GPU-failure fallback on the MI355X.

QSMD5_BACKEND=auto sends a batch to the CPU when the CPU's estimated time is
the lower (a lone part, a few parts) and to the gfx950 kernels above the
break-even; a GPU failure falls back to the library's CPU MD5 and returns the
same digest; a lost GPU context sends every later call to the CPU.  Failures
are injected with QSMD5_INJECT_GPU_FAULT (no real fault is provoked on the
box).  Every digest is checked against the oracle.
"""
import ctypes
import json
import os
import statistics
import subprocess
import sys
import time

import pytest

import qsmd5
from conftest import ROOT
from oracle_util import lcg_bytes, md5_many

torch = pytest.importorskip("torch")
pytestmark = [pytest.mark.gpu, pytest.mark.cpu_backend]

MiB = 1 << 20


@pytest.fixture
def auto(monkeypatch):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.setenv("QSMD5_BACKEND", "auto")
    monkeypatch.delenv("QSMD5_INJECT_GPU_FAULT", raising=False)
    # the scalar idle-host model these tests restate (lanes and load feedback:
    # test_lane_priced_* below, tests/test_cpu_backend.py)
    monkeypatch.setenv("QSMD5_ROUTE_LANES", "0")
    monkeypatch.setenv("QSMD5_CPU_LOAD_FEEDBACK", "0")
    assert qsmd5.lib().qsmd5_init(0) == 0


def _batch(n, L, seed=500):
    bufs = [lcg_bytes(seed + i, L) for i in range(n)]
    return bufs, [(ctypes.addressof(b), L) for b in bufs]


def test_break_even_batches_take_the_gpu(auto):
    _, chunks = _batch(64, MiB)
    assert qsmd5.route([MiB] * 64) == qsmd5.BACKEND_GPU
    s0 = qsmd5.stats()
    assert qsmd5.hash_batch(chunks) == md5_many(chunks)
    assert qsmd5.last_backend() == qsmd5.BACKEND_GPU
    assert qsmd5.stats()["gpu_batches"] == s0["gpu_batches"] + 1


def test_lone_part_goes_to_the_cpu_and_beats_the_reference(auto):
    """The unchanged per-part call site (QSClient.cpp:369-371 -> md5(iostream),
    MD5.cpp:341-349) on one 10 MiB part: routed to the CPU, and no slower than
    the reference's md5(iostream) on this host (oracle/_ref, when built)."""
    data = lcg_bytes(12345, 10 * MiB)
    addr = ctypes.addressof(data)
    times = []
    for _ in range(5):
        t0 = time.perf_counter()
        d = qsmd5.hash_one((addr, 10 * MiB))
        times.append(time.perf_counter() - t0)
        assert qsmd5.last_backend() == qsmd5.BACKEND_CPU
    assert d.hex() == "302bec822b27cea263612fb3f76fa34b"
    ours = statistics.median(times)
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libref_md5.so")
    if not os.path.exists(ref_so):
        pytest.skip("reference build absent; ours %.1f ms" % (ours * 1e3))
    R = ctypes.CDLL(ref_so)
    R.ref_md5_iostream.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_char_p]
    rt = []
    out = ctypes.create_string_buffer(33)
    for _ in range(5):
        t0 = time.perf_counter()
        R.ref_md5_iostream(addr, 10 * MiB, out)
        rt.append(time.perf_counter() - t0)
    ref = statistics.median(rt)
    print("lone 10 MiB part: library %.2f ms (CPU route), reference md5(iostream) %.2f ms"
          % (ours * 1e3, ref * 1e3))
    assert out.value.decode() == "302bec822b27cea263612fb3f76fa34b"
    assert ours <= ref * 1.05


def test_cpu_backend_reads_long_device_chunks_in_pieces(auto):
    """The CPU backend reads a device chunk back through an 8 MiB host buffer:
    chunks of 8 MiB - 1 .. 19 MiB + 13 B, ragged ends, against the oracle."""
    lens = [8 * MiB - 1, 8 * MiB, 8 * MiB + 1, 19 * MiB + 13]
    offs = [0]
    for L in lens[:-1]:
        offs.append(offs[-1] + L + 3)  # odd starts too
    dev = torch.empty(offs[-1] + lens[-1], dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for k, (o, L) in enumerate(zip(offs, lens)):
        qsmd5.synth_fill_lcg(dev.data_ptr() + o, L, L, 950 + k, 1, s)
    torch.cuda.synchronize()
    dhost = dev.cpu().numpy()
    want = md5_many([(dhost.ctypes.data + o, L) for o, L in zip(offs, lens)])
    got = qsmd5.hash_batch([(dev.data_ptr() + o, L) for o, L in zip(offs, lens)],
                           flags=qsmd5.FLAG_CPU_ONLY)
    assert got == want
    assert qsmd5.last_backend() == qsmd5.BACKEND_CPU


def test_injected_gpu_fault_falls_back_with_identical_digests(auto, monkeypatch):
    host_bufs, host = _batch(48, MiB)
    dev = torch.empty(16 * MiB, dtype=torch.uint8, device="cuda")
    qsmd5.synth_fill_lcg(dev.data_ptr(), MiB, MiB, 900, 16, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    dchunks = [(dev.data_ptr() + i * MiB, MiB) for i in range(16)]
    dhost = dev.cpu().numpy()
    want = md5_many(host) + md5_many([(dhost.ctypes.data + i * MiB, MiB) for i in range(16)])
    monkeypatch.setenv("QSMD5_INJECT_GPU_FAULT", "1")
    s0 = qsmd5.stats()
    assert qsmd5.hash_batch(host + dchunks) == want  # device chunks come back by D2H
    assert qsmd5.last_backend() == qsmd5.BACKEND_CPU
    s1 = qsmd5.stats()
    assert s1["fallbacks"] == s0["fallbacks"] + 1 and not s1["gpu_lost"]
    # forced GPU: the failure is returned, never a digest
    with pytest.raises(qsmd5.Md5Error):
        qsmd5.hash_batch(host, flags=qsmd5.FLAG_GPU_ONLY)
    monkeypatch.delenv("QSMD5_INJECT_GPU_FAULT")
    assert qsmd5.hash_batch(host + dchunks) == want  # a transient failure: the GPU again
    assert qsmd5.last_backend() == qsmd5.BACKEND_GPU


_STICKY = r"""
import ctypes, sys
sys.path[:0] = [%(pkg)r, %(tests)r]
import torch, qsmd5
from oracle_util import lcg_bytes, md5_many
bufs = [lcg_bytes(77 + i, 1 << 20) for i in range(64)]
chunks = [(ctypes.addressof(b), 1 << 20) for b in bufs]
want = md5_many(chunks)
import os
os.environ["QSMD5_INJECT_GPU_FAULT"] = "sticky"
assert qsmd5.hash_batch(chunks) == want
del os.environ["QSMD5_INJECT_GPU_FAULT"]
st = qsmd5.stats()
assert st["gpu_lost"] == 1 and st["fallbacks"] == 1, st
assert qsmd5.hash_batch(chunks) == want  # GPU lost: straight to the CPU
assert qsmd5.last_backend() == qsmd5.BACKEND_CPU
assert qsmd5.stats()["fallbacks"] == 1
dev = torch.zeros(4096, dtype=torch.uint8, device="cuda")
try:
    qsmd5.hash_batch([dev])
    raise SystemExit("a device chunk was hashed after the context was lost")
except qsmd5.Md5Error as e:
    assert e.code == -5, e
print("STICKY_OK")
"""


def test_lost_gpu_context_sends_every_later_call_to_the_cpu(auto):
    code = _STICKY % {"pkg": os.path.join(ROOT, "qsfs-fuse_amd"), "tests": os.path.join(ROOT, "tests")}
    env = dict(os.environ, QSMD5_BACKEND="auto")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                         timeout=240)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "STICKY_OK" in out.stdout
    assert "qsmd5: GPU context lost" in out.stderr  # logged once
    assert out.stderr.count("qsmd5: GPU context lost") == 1


def test_streaming_class_in_auto_mode_reads_device_pieces(auto):
    """Under auto the MD5 class hashes on the CPU (one stream = one chain);
    device pieces are copied back first.  Same digest as the oracle."""
    L = 3 * MiB + 17
    dev = torch.empty(L, dtype=torch.uint8, device="cuda")
    qsmd5.synth_fill_lcg(dev.data_ptr(), L, L, 4242, 1, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    host = dev.cpu().numpy()
    h = qsmd5.MD5()
    cuts = [1, 63, 64, 65, MiB, 2 * MiB - 193 + 17]
    off = 0
    for i, c in enumerate(cuts):
        src = dev.data_ptr() if i % 2 else host.ctypes.data
        h.update((src + off, c))
        off += c
    assert off == L
    assert h.finalize().digest() == md5_many([(host.ctypes.data, L)])[0]


def _ragged_host(seed=31):
    """60 chunks of ~1-3 MiB and two of 16 MiB + a few bytes (host, pageable)."""
    import random
    rng = random.Random(seed)
    lens = [MiB + rng.randrange(2 * MiB) for _ in range(60)] + [16 * MiB + 5, 16 * MiB + 77]
    rng.shuffle(lens)
    bufs = [lcg_bytes(seed * 1000 + i, L) for i, L in enumerate(lens)]
    return lens, bufs, [(ctypes.addressof(b), L) for b, L in zip(bufs, lens)]


def test_split_ragged_host_batch(auto, monkeypatch):
    """A ragged batch splits: its two long chunks go to the CPU threads while
    the GPU hashes the other 60; every digest equals the oracle's."""
    monkeypatch.setenv("QSMD5_CPU_THREADS", "1")
    lens, _bufs, chunks = _ragged_host()
    assert qsmd5.route(lens) == qsmd5.BACKEND_SPLIT
    s0 = qsmd5.stats()
    assert qsmd5.hash_batch(chunks) == md5_many(chunks)
    assert qsmd5.last_backend() == qsmd5.BACKEND_SPLIT
    s1 = qsmd5.stats()
    assert s1["gpu_batches"] == s0["gpu_batches"] + 1 and s1["cpu_batches"] == s0["cpu_batches"] + 1
    took = s1["cpu_chunks"] - s0["cpu_chunks"]
    assert 2 <= took < len(lens) and s1["gpu_chunks"] - s0["gpu_chunks"] == len(lens) - took
    monkeypatch.setenv("QSMD5_SPLIT", "0")
    assert qsmd5.hash_batch(chunks) == md5_many(chunks)
    assert qsmd5.last_backend() == qsmd5.BACKEND_GPU


def test_split_batch_gpu_fault_falls_back(auto, monkeypatch):
    monkeypatch.setenv("QSMD5_CPU_THREADS", "1")
    lens, _bufs, chunks = _ragged_host(seed=32)
    monkeypatch.setenv("QSMD5_INJECT_GPU_FAULT", "1")
    s0 = qsmd5.stats()
    assert qsmd5.hash_batch(chunks) == md5_many(chunks)
    assert qsmd5.last_backend() == qsmd5.BACKEND_CPU
    s1 = qsmd5.stats()
    assert s1["fallbacks"] == s0["fallbacks"] + 1 and not s1["gpu_lost"]


def test_split_config4_device_resident(auto, golden):
    """BASELINE config 4 (659 device-resident chunks, 0 B-64 MiB) under auto
    routing: the longest chunks are read back and hashed by the CPU threads
    while the GPU runs the rest; all 659 digests equal the reference's."""
    gr = golden("ragged.json")
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
    t0 = time.perf_counter()
    digs = qsmd5.hash_batch(chunks)
    split_s = time.perf_counter() - t0
    assert [d.hex() for d in digs] == gr["md5"]
    assert qsmd5.last_backend() == qsmd5.BACKEND_SPLIT
    t0 = time.perf_counter()
    assert [d.hex() for d in qsmd5.hash_batch(chunks, flags=qsmd5.FLAG_GPU_ONLY)] == gr["md5"]
    gpu_s = time.perf_counter() - t0
    print("config 4 device-resident: split %.3f s, GPU only %.3f s" % (split_s, gpu_s))


def test_lane_priced_routing_keeps_host_batch_on_cpu(auto, monkeypatch):
    """Lanes priced (the default since round 5) on the box's host CPU: a
    ragged host batch (62 chunks, 1-16 MiB) stays on the CPU's multi-buffer
    lanes instead of splitting, and every digest equals the oracle's; with
    QSMD5_ROUTE_LANES=0 it splits as before."""
    if "avx512f" not in open("/proc/cpuinfo").read():
        pytest.skip("host without AVX-512F: the lanes are never priced")
    monkeypatch.setenv("QSMD5_CPU_THREADS", "1")  # one thread: the scalar model splits
    lens, _bufs, chunks = _ragged_host(seed=33)
    monkeypatch.setenv("QSMD5_ROUTE_LANES", "1")
    assert qsmd5.route(lens) == qsmd5.BACKEND_CPU
    s0 = qsmd5.stats()
    assert qsmd5.hash_batch(chunks) == md5_many(chunks)
    assert qsmd5.last_backend() == qsmd5.BACKEND_CPU
    s1 = qsmd5.stats()
    assert s1["gpu_batches"] == s0["gpu_batches"] and s1["cpu_chunks"] - s0["cpu_chunks"] == len(lens)
    monkeypatch.setenv("QSMD5_ROUTE_LANES", "0")
    assert qsmd5.route(lens) == qsmd5.BACKEND_SPLIT


def test_device_chunks_pay_their_read_back_in_routing(auto):
    """a device-resident chunk priced for the CPU carries its D2H
    read-back, and costs the GPU no link time.  n equal 10 MiB chunks where
    the model (at this host's measured rates, qsmd5_get_rates) sends host
    memory to the CPU but device memory to the GPU: qsmd5_route agrees with
    real pointers, and the device batch then runs on the gfx950 kernels."""
    GiB = float(1 << 30)
    S = 10 * MiB
    r = qsmd5.rates()
    T, rc, g, K, D = (r["cpu_threads"], r["cpu_chain_gibs"], r["gpu_chain_gibs"], r["link_gibs"],
                      r["d2h_gibs"])

    def cpu_ms(n, dev):
        return 1e3 * (max(S / rc, n * S / (T * rc)) + (n * S / D if dev else 0)) / GiB

    def gpu_ms(n, dev):
        return r["gpu_call_ms"] + 1e3 * (S / g + (0 if dev else n * S / K)) / GiB

    ns = [n for n in range(2, 200) if cpu_ms(n, False) < gpu_ms(n, False) and
          not cpu_ms(n, True) < gpu_ms(n, True)]
    if not ns:
        pytest.skip("no batch size separates host from device at these rates: %s" % r)
    n = ns[len(ns) // 2]
    dev = torch.empty(n * S, dtype=torch.uint8, device="cuda")
    qsmd5.synth_fill_lcg(dev.data_ptr(), S, S, 12345, n, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    arr = (qsmd5.qsmd5_chunk * n)()
    for i in range(n):
        arr[i].ptr, arr[i].len = dev.data_ptr() + i * S, S
    assert qsmd5.lib().qsmd5_route(arr, n, 0) == qsmd5.BACKEND_GPU, (n, r)
    assert qsmd5.route([S] * n) == qsmd5.BACKEND_CPU, (n, r)  # the same sizes as host memory
    got = qsmd5.hash_batch([(dev.data_ptr() + i * S, S) for i in range(n)])
    assert qsmd5.last_backend() == qsmd5.BACKEND_GPU
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "batch_10MiB.json")))["md5"]
    assert [d.hex() for d in got] == gold[:n]
    print("n=%d device 10 MiB chunks: GPU; as host memory: CPU; rates %s" % (n, r))


def test_background_batches_take_the_gpu(auto):
    """QSMD5_FLAG_BACKGROUND (round 5): a lone part, and a pull-driven batch of
    8 parts -- both the CPU's on speed -- go to the GPU when the caller says
    their latency is hidden (the staged pre-hash's later waves), with the
    oracle's digests; without the flag they stay on the CPU."""
    MiB = 1 << 20
    data = lcg_bytes(41, 8 * MiB)
    one = [(ctypes.addressof(data), 8 * MiB)]
    assert qsmd5.route([8 * MiB]) == qsmd5.BACKEND_CPU
    assert qsmd5.route([8 * MiB], flags=qsmd5.FLAG_BACKGROUND) == qsmd5.BACKEND_GPU
    want = md5_many(one)
    assert qsmd5.hash_batch(one, flags=qsmd5.FLAG_BACKGROUND) == want
    assert qsmd5.last_backend() == qsmd5.BACKEND_GPU
    assert qsmd5.hash_batch(one) == want and qsmd5.last_backend() == qsmd5.BACKEND_CPU
    lens = [MiB] * 8

    def read(chunk, off, n, dst):
        ctypes.memmove(dst, ctypes.addressof(data) + chunk * MiB + off, n)
        return n
    want8 = md5_many([(ctypes.addressof(data) + i * MiB, MiB) for i in range(8)])
    assert qsmd5.hash_read(lens, read, flags=qsmd5.FLAG_BACKGROUND) == want8
    assert qsmd5.last_backend() == qsmd5.BACKEND_GPU
