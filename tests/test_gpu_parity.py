"""Parity of the HIP path (through the C-ABI, libqsmd5.so) on an MI355X.

Every digest is compared bit-exactly with the golden fixtures produced by the
reference's own MD5.cpp (tests/golden/) or, for inputs the fixtures do not
hold, with the CPU oracle on the same bytes.  Covers both kernels, host
(pageable and pinned) and device memory, unaligned pointers, every padding
edge, ragged batches, the streaming MD5 class, the part planner + batch
pre-hash, >= 4 GiB lengths, concurrency and error behaviour.
"""
import ctypes
import errno
import os
import threading

import pytest

import qsmd5
from oracle_util import lcg_bytes, md5_many, md5_ref

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu
MiB = 1 << 20


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert qsmd5.lib().qsmd5_init(0) == 0
    yield
    os.environ.pop("QSMD5_KERNEL", None)


@pytest.fixture(params=["pc", "pc2", "v1", "coal"])
def kernel(request):
    os.environ["QSMD5_KERNEL"] = request.param
    yield request.param
    os.environ.pop("QSMD5_KERNEL", None)


def dev_lcg(seed, n, nchunks=1, stride=None):
    """Device tensor filled by the GPU LCG generator (qsmd5_synth_fill_lcg)."""
    stride = stride or n
    t = torch.empty(max(stride * nchunks, 1), dtype=torch.uint8, device="cuda")
    qsmd5.synth_fill_lcg(t.data_ptr(), stride, n, seed, nchunks,
                         torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return t


def hexes(ds):
    return [d.hex() for d in ds]


def test_rfc1321(golden):
    for c in golden("rfc1321.json")["cases"]:
        assert qsmd5.md5(c["text"]) == c["md5"]


def test_lcg_lengths_host(golden, kernel):
    g = golden("lcg_lengths.json")
    big = max(c["len"] for c in g["cases"])
    data = lcg_bytes(12345, big)
    base = ctypes.addressof(data)
    got = qsmd5.hash_batch([(base, c["len"]) for c in g["cases"]])
    assert hexes(got) == [c["md5"] for c in g["cases"]]


def test_lcg_lengths_device(golden, kernel):
    g = golden("lcg_lengths.json")
    big = max(c["len"] for c in g["cases"])
    t = dev_lcg(12345, big)
    assert bytes(t[:64].cpu().numpy()) == bytes(lcg_bytes(12345, 64))  # generator parity
    got = qsmd5.hash_batch([(t.data_ptr(), c["len"]) for c in g["cases"]])
    assert hexes(got) == [c["md5"] for c in g["cases"]]


def test_generator_matches_oracle():
    for seed, n in [(1, 1), (2, 1023), (3, 1025), (12345, 3 * MiB + 7)]:
        t = dev_lcg(seed, n)
        assert bytes(t[:n].cpu().numpy()) == bytes(lcg_bytes(seed, n))[:n]


def test_unaligned_device_pointers(kernel):
    n = 1 << 20
    t = dev_lcg(777, n)
    host = bytes(t.cpu().numpy())
    lens = [0, 1, 3, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128, 129, 4096, 8191, 65537, 300001]
    chunks, want = [], []
    for off in range(8):
        for L in lens:
            o = off * 4099 + off
            chunks.append((t.data_ptr() + o, L))
            want.append(md5_ref(host[o:o + L]))
    assert qsmd5.hash_batch(chunks) == want


def test_unaligned_host_pointers(kernel):
    data = lcg_bytes(4321, 1 << 20)
    base = ctypes.addressof(data)
    raw = bytes(data)
    chunks, want = [], []
    for off in range(1, 8):
        for L in [0, 1, 63, 64, 65, 1000, 100003]:
            chunks.append((base + off, L))
            want.append(md5_ref(raw[off:off + L]))
    assert qsmd5.hash_batch(chunks) == want


def test_ragged_batch_device(golden):
    g = golden("ragged.json")
    lens = g["lengths"]
    offs, pos = [], 0
    for L in lens:
        offs.append(pos)
        pos += (L + 255) & ~255
    t = torch.empty(pos + 256, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for i, (o, L) in enumerate(zip(offs, lens)):
        qsmd5.synth_fill_lcg(t.data_ptr() + o, 0, L, 7000 + i, 1, s)
    torch.cuda.synchronize()
    got = qsmd5.hash_batch([(t.data_ptr() + o, L) for o, L in zip(offs, lens)])
    assert hexes(got) == g["md5"]


def test_bufsize_sweep_device(golden):
    for sw in golden("ragged.json")["sweep"]:
        L = sw["mib"] * MiB
        n = len(sw["md5"])
        t = dev_lcg(sw["seed0"], L, nchunks=n)
        got = qsmd5.hash_batch([(t.data_ptr() + i * L, L) for i in range(n)])
        assert hexes(got) == sw["md5"], sw["mib"]


def test_start_skew_wave_mixed_lengths():
    """A wave whose longest chunk is >= 32 MiB runs with per-lane start skew
    (pc_body): lanes with tiny, empty, unaligned and multi-block chunks in the
    same wave must still hash exactly their own bytes."""
    big = 32 * MiB + 77
    lens = [big, 32 * MiB, 0, 1, 55, 56, 63, 64, 65, 127, 128, 1000, 4096 + 3, 65536 + 9,
            3 * MiB + 1] + [1 + 97 * i for i in range(40)]
    offs, pos = [], 0
    for i, L in enumerate(lens):
        pos += 1 + (i % 7)  # unaligned starts
        offs.append(pos)
        pos += L
    t = torch.empty(pos + 256, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    qsmd5.synth_fill_lcg(t.data_ptr(), 0, pos + 256, 31337, 1, s)
    torch.cuda.synchronize()
    raw = t.cpu().numpy()
    want = md5_many([(raw.ctypes.data + o, L) for o, L in zip(offs, lens)])
    got = qsmd5.hash_batch([(t.data_ptr() + o, L) for o, L in zip(offs, lens)])
    assert got == want


@pytest.mark.parametrize("lanes,nt", [("1", "0"), ("7", "0"), ("32", "1"), ("63", "0")])
def test_latency_kernel_lanes_and_cache_policy(lanes, nt, monkeypatch):
    """QSMD5_PC_LANES: chains per workgroup of the latency kernel (the runtime
    picks 32 for parts >= 32 MiB, pc_lanes_for); QSMD5_LOAD_NT: the producer's
    cache policy.  Odd lane counts leave the tail lanes of every workgroup and
    a partial last workgroup idle; every chunk must still hash its own bytes."""
    monkeypatch.setenv("QSMD5_PC_LANES", lanes)
    monkeypatch.setenv("QSMD5_LOAD_NT", nt)
    monkeypatch.setenv("QSMD5_KERNEL", "pc")
    lens = [0, 1, 55, 64, 65, 4096 + 3, 300001] + [1 + 977 * i for i in range(143)]
    offs, pos = [], 0
    for i, L in enumerate(lens):
        pos += 1 + (i % 5)
        offs.append(pos)
        pos += L
    t = dev_lcg(4711, pos + 64)
    raw = t.cpu().numpy()
    want = md5_many([(raw.ctypes.data + o, L) for o, L in zip(offs, lens)])
    assert qsmd5.hash_batch([(t.data_ptr() + o, L) for o, L in zip(offs, lens)]) == want


def test_long_parts_run_at_half_a_wave_per_cu():
    """Parts >= 32 MiB take the 32-lanes-per-workgroup launch (pc_lanes_for):
    40 x 33 MiB (+ 3 B) device parts against the oracle."""
    L, n = 33 * MiB + 3, 40
    t = dev_lcg(8080, L, nchunks=n, stride=L + 13)
    raw = t.cpu().numpy()
    want = md5_many([(raw.ctypes.data + i * (L + 13), L) for i in range(n)])
    assert qsmd5.hash_batch([(t.data_ptr() + i * (L + 13), L) for i in range(n)]) == want


def _device_batch(n, L, seed0):
    t = dev_lcg(seed0, L, nchunks=n)
    desc = torch.empty((n, 2), dtype=torch.int64)
    desc[:, 0] = t.data_ptr() + torch.arange(n, dtype=torch.int64) * L
    desc[:, 1] = L
    return t, desc.cuda()


def test_batch512_device_resident_async(golden):
    """BASELINE config 2: 512 x 10 MiB device-resident, all 512 digests."""
    g = golden("batch_10MiB.json")
    n, L = 512, g["len"]
    t, desc = _device_batch(n, L, 12345)
    dig = torch.zeros((n, 16), dtype=torch.uint8, device="cuda")
    qsmd5.hash_device(desc.data_ptr(), dig.data_ptr(), n,
                      stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = [bytes(r) for r in dig.cpu().numpy()]
    assert hexes(got) == g["md5"][:n]


def test_batch4096_device_resident(golden):
    """Config 3 shape (4096 x 10 MiB) device-resident: every digest vs the fixture."""
    g = golden("batch_10MiB.json")
    n, L = 4096, g["len"]
    t, desc = _device_batch(n, L, 12345)
    got = qsmd5.hash_batch([(t.data_ptr() + i * L, L) for i in range(n)])
    assert hexes(got) == g["md5"][:n]
    del t


def test_pool_buffers_in_any_order(golden):
    """Pool buffers handed over in shuffled order (a buffer pool's free list):
    digests land in caller order, and the runtime's address ordering of
    equal-length lanes keeps the rate of the pool order (without it, 50.8 vs
    59.3 GiB/s: profiles/r01_config_pool.jsonl)."""
    import random
    import time
    g = golden("batch_10MiB.json")
    n, L = 512, g["len"]
    t, _ = _device_batch(n, L, 12345)
    perm = list(range(n))
    random.Random(5).shuffle(perm)
    # duplicates and a zero-length chunk mixed in: ties on address, empty lanes
    order = perm + [perm[0], perm[1]]
    chunks = [(t.data_ptr() + i * L, L) for i in order] + [(t.data_ptr(), 0)]
    got = qsmd5.hash_batch(chunks)
    assert hexes(got) == [g["md5"][i] for i in order] + [md5_ref(b"").hex()]

    def rate(order):  # best of 3 timed calls after a warm-up: one slow call is noise
        ch = [(t.data_ptr() + i * L, L) for i in order]
        qsmd5.hash_batch(ch)
        best = float("inf")
        for _ in range(3):
            t0 = time.perf_counter()
            qsmd5.hash_batch(ch)
            best = min(best, time.perf_counter() - t0)
        return 1.0 / best
    in_order, shuffled = rate(range(n)), rate(perm)
    print("pool order %.1f GiB/s, shuffled %.1f GiB/s" % (in_order * 5, shuffled * 5))
    assert shuffled > 0.93 * in_order, (in_order, shuffled)
    del t


def test_classifier_many_allocations_and_host_flag():
    """The runtime remembers the exact range of each HIP allocation it has seen,
    and the VMA of each pageable pointer (8 ranges in all).  Here more device
    and pinned allocations than that are mixed with pageable buffers in shuffled
    order, with the VMA cache on (QSMD5_MAPS_AFTER lowered) and off.  Chunks end on an
    allocation's last byte.  Every chunk must still be classified right.
    QSMD5_FLAG_HOST on the host-only subset gives the same digests without the
    pointer queries."""
    import random
    rng = random.Random(11)
    items, keep = [], []
    for i in range(10):  # pinned: distinct hipHostMalloc ranges
        L = 65536 + 37 * i
        p = qsmd5.alloc_pinned(L)
        keep.append(p)
        data = bytes(lcg_bytes(900 + i, L))
        ctypes.memmove(p, data, L)
        items += [("host", (p, L), md5_ref(data)), ("host", (p + L - 1000, 1000), md5_ref(data[-1000:]))]
    tensors = []
    for i in range(12):  # device: >= 10 MiB each, so torch gives each its own hipMalloc
        L = (10 << 20) + 4097 * i
        t = dev_lcg(950 + i, L)
        tensors.append(t)
        data = t.cpu().numpy().tobytes()
        items += [("dev", (t.data_ptr(), L), md5_ref(data)),
                  ("dev", (t.data_ptr() + L - 777, 777), md5_ref(data[-777:]))]
    pageable = []
    for i in range(5):
        L = 300000 + 11 * i
        b = lcg_bytes(990 + i, L)
        pageable.append(b)
        items.append(("host", (ctypes.addressof(b), L), md5_ref(bytes(b))))
    items.append(("host", (0, 0), md5_ref(b"")))
    # many pageable chunks: with QSMD5_MAPS_AFTER lowered below, the runtime
    # also reads /proc/self/maps and remembers the VMAs of pageable pointers
    for j in range(300):
        b = pageable[j % 5]
        off = (j * 997) % (len(b) - 2000)
        items.append(("host", (ctypes.addressof(b) + off, 1500), md5_ref(bytes(b)[off:off + 1500])))
    for j in range(60):
        t = tensors[j % 12]
        off = (j * 65537) % (t.numel() - 5000)
        items.append(("dev", (t.data_ptr() + off, 4000),
                      md5_ref(t[off:off + 4000].cpu().numpy().tobytes())))
    try:
        for rnd, after in enumerate(("16", "16", None)):
            if after:
                os.environ["QSMD5_MAPS_AFTER"] = after
            else:
                os.environ.pop("QSMD5_MAPS_AFTER", None)
            rng.shuffle(items)
            got = qsmd5.hash_batch([c for _, c, _ in items])
            assert got == [w for _, _, w in items], rnd
        host = [(c, w) for k, c, w in items if k == "host"]
        got = qsmd5.hash_batch([c for c, _ in host], flags=qsmd5.FLAG_HOST)
        assert got == [w for _, w in host]
    finally:
        os.environ.pop("QSMD5_MAPS_AFTER", None)
        for p in keep:
            qsmd5.free_pinned(p)


def test_batch_pinned_host(golden):
    g = golden("batch_10MiB.json")
    n, L = 96, g["len"]
    p = qsmd5.alloc_pinned(n * L)
    try:
        t = dev_lcg(12345, L, nchunks=n)
        ctypes.memmove(p, bytes(t.cpu().numpy()), n * L)
        del t
        got = qsmd5.hash_batch([(p + i * L, L) for i in range(n)])
        assert hexes(got) == g["md5"][:n]
    finally:
        qsmd5.free_pinned(p)


def test_stream_pieces_class(golden):
    g = golden("stream_pieces.json")
    raw = bytes(lcg_bytes(g["seed"], g["len"]))
    dev = torch.frombuffer(bytearray(raw), dtype=torch.uint8).cuda()
    for case in g["cases"]:
        m = qsmd5.MD5()
        assert m.hexdigest() == ""
        off = 0
        for cut in case["cuts"]:
            m.update(raw[off:off + cut])
            off += cut
        assert m.finalize().hexdigest() == case["md5"]
        # the same pieces from device memory
        m2 = qsmd5.MD5()
        off = 0
        for cut in case["cuts"]:
            m2.update(dev[off:off + cut])
            off += cut
        assert m2.finalize().hexdigest() == case["md5"]
    assert qsmd5.MD5("abc").hexdigest() == "900150983cd24fb0d6963f7d28e17f72"


def test_md5_copy_forks_the_state_on_gpu():
    """qsmd5_ctx_copy on a GPU context (QSMD5_BACKEND=gpu: the chaining state
    lives in device memory and is copied device to device), from host pieces
    and from device pieces."""
    from md5_copy_cases import run_copy_cases
    run_copy_cases(qsmd5, lambda d, off, n: d[off:off + n])
    dev = {}

    def dev_piece(d, off, n):
        if id(d) not in dev:
            dev[id(d)] = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda()
        return dev[id(d)][off:off + n]
    run_copy_cases(qsmd5, dev_piece)


def test_md5_stream_mirror():
    import io
    s = io.BytesIO(b"0123456789" * 1000)
    s.seek(17)
    h = qsmd5.md5_stream(s)
    assert h == md5_ref(b"0123456789" * 1000).hex() and s.tell() == 0


def test_plan_and_hash_parts_host_and_device():
    size = 100 * MiB + 12345  # 10 full parts + averaged pair
    data = lcg_bytes(31337, size)
    parts = qsmd5.plan_parts(size)
    assert len(parts) == 11
    raw = memoryview(data)
    want = md5_many([(ctypes.addressof(data) + p.offset, p.size) for p in parts])
    assert qsmd5.hash_parts(data, parts) == want
    dev = dev_lcg(31337, size)
    assert qsmd5.hash_parts(dev, parts) == want
    del raw


def test_length_over_4gib_truncation_flag(golden):
    """>= 4 GiB: full RFC 1321 by default; the reference's 32-bit truncation on request."""
    g = golden("truncate32.json")
    L = g["len"]
    t = dev_lcg(g["seed"], L)
    full = qsmd5.hash_batch([(t.data_ptr(), L)])[0]
    trunc = qsmd5.hash_batch([(t.data_ptr(), L)], flags=1)[0]
    assert full.hex() == g["full_md5"]
    assert trunc.hex() == g["reference_md5"]
    del t


def test_concurrent_callers():
    data = [lcg_bytes(900 + i, 3 * MiB + i) for i in range(8)]
    want = [md5_ref(d) for d in data]
    errs = []

    def worker(k):
        try:
            for _ in range(3):
                got = qsmd5.hash_batch(data[k:] + data[:k])
                assert got == want[k:] + want[:k]
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)

    th = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs, errs


def test_errors_and_empty():
    L = qsmd5.lib()
    out = (ctypes.c_uint8 * 16)()
    assert L.qsmd5_hash_one(None, 5, out) == -errno.EINVAL
    assert L.qsmd5_hash_one(ctypes.c_void_p(1), 1 << 38, out) == -errno.EINVAL
    assert L.qsmd5_hash_one(None, 0, out) == 0
    assert bytes(out).hex() == "d41d8cd98f00b204e9800998ecf8427e"
    assert qsmd5.hash_batch([]) == []
    assert L.qsmd5_hash_batch(None, 0, None) == 0


def test_kernel_choice_policy():
    os.environ.pop("QSMD5_KERNEL", None)
    A = qsmd5.FLAG_ALIGNED16
    assert qsmd5.kernel_choice(512) == 1 and qsmd5.kernel_choice(512, A) == 1
    assert qsmd5.kernel_choice(16384) == 1
    assert qsmd5.kernel_choice(16385) == 3 and qsmd5.kernel_choice(16385, A) == 3
    assert qsmd5.kernel_choice(32768) == 3
    assert qsmd5.kernel_choice(32769) == 0
    assert qsmd5.kernel_choice(32769, A) == 2


def test_coalesced_kernel_ragged_aligned(kernel):
    """All three kernels on one ragged, 16-B-aligned device batch (lengths 0..~1 MiB)."""
    import random
    rng = random.Random(21)
    lens = [0, 1, 63, 64, 65, 127, 128, 129, 191, 192, 255, 256] + \
        [rng.randrange(0, 1 << 20) for _ in range(200)]
    offs, pos = [], 0
    for L in lens:
        offs.append(pos)
        pos += ((L + 15) & ~15) + 16 * rng.randrange(0, 5)
    t = dev_lcg(99, pos + 64)
    host = bytes(t.cpu().numpy())
    hb = (ctypes.c_uint8 * len(host)).from_buffer_copy(host)
    want = md5_many([(ctypes.addressof(hb) + o, L) for o, L in zip(offs, lens)])
    got = qsmd5.hash_batch([(t.data_ptr() + o, L) for o, L in zip(offs, lens)])
    assert got == want


@pytest.mark.parametrize("n,kind", [(20000, 3), (40000, 2)])
def test_device_async_large_batches(n, kind):
    """16 385..32 768 chunks go to the 64 KiB-ring latency kernel, more (with
    QSMD5_FLAG_ALIGNED16) to the coalesced kernel."""
    os.environ.pop("QSMD5_KERNEL", None)
    L = 4096 + 64 + 7
    S = 8192 + 16
    t = dev_lcg(3, L, nchunks=n, stride=S)
    desc = torch.empty((n, 2), dtype=torch.int64)
    desc[:, 0] = t.data_ptr() + torch.arange(n, dtype=torch.int64) * S
    desc[:, 1] = L
    desc = desc.cuda()
    dig = torch.zeros((n, 16), dtype=torch.uint8, device="cuda")
    assert qsmd5.kernel_choice(n, qsmd5.FLAG_ALIGNED16) == kind
    qsmd5.hash_device(desc.data_ptr(), dig.data_ptr(), n,
                      stream=torch.cuda.current_stream().cuda_stream, flags=qsmd5.FLAG_ALIGNED16)
    torch.cuda.synchronize()
    host = t.cpu().numpy()
    sample = list(range(0, n, 97)) + [n - 1]
    want = md5_many([(host.ctypes.data + i * S, L) for i in sample])
    got = [bytes(dig[i].cpu().numpy()) for i in sample]
    assert got == want


def test_verify_etag_download_buffer():
    data = bytes(lcg_bytes(55, 3 * MiB + 17))
    etag = '"%s"' % md5_ref(data).hex()  # the pinned oracle
    assert qsmd5.verify_etag(data, etag)
    dev = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    assert qsmd5.verify_etag(dev, etag)
    assert not qsmd5.verify_etag(data[:-1], etag)
    with pytest.raises(qsmd5.Md5Error):
        qsmd5.verify_etag(data, etag[:-2] + '-2"')


@pytest.mark.parametrize("n", [17000, 33000])
def test_large_batches_select_throughput_kernels(n):
    """> 16 384 chunks through the synchronous API: staged host chunks and
    unaligned device chunks (17 000: 64 KiB-ring latency kernel; 33 000:
    coalesced kernel for the staged chunks, one-wave kernel for the unaligned)."""
    os.environ.pop("QSMD5_KERNEL", None)
    import random
    rng = random.Random(8)
    host = lcg_bytes(71, 4 << 20)
    base = ctypes.addressof(host)
    spans = [(rng.randrange(0, (4 << 20) - 5000), rng.randrange(0, 5000)) for _ in range(n)]
    want = md5_many([(base + o, L) for o, L in spans])
    assert qsmd5.hash_batch([(base + o, L) for o, L in spans]) == want
    dev = torch.frombuffer(bytearray(bytes(host)), dtype=torch.uint8).cuda()
    odd = [(o | 1, L) for o, L in spans]
    want_odd = md5_many([(base + o, L) for o, L in odd])
    assert qsmd5.hash_batch([(dev.data_ptr() + o, L) for o, L in odd]) == want_odd


def test_one_long_chain_past_the_two_second_poll():
    """One 1 GiB chunk is one serial chain of ~8.5 s on a GPU lane: the
    synchronous call sleeps through most of its estimate and then polls, every
    1 ms once the batch runs 2 s past its start (wait_stream).  Device- and
    host-resident (pinned), digest == oracle, and the caller's thread is not
    spinning meanwhile (its CPU time stays a small part of the wall time)."""
    import resource
    import time
    L = 1 << 30
    data = lcg_bytes(4711, L)
    want = md5_ref(data, L)
    dev = torch.frombuffer(data, dtype=torch.uint8).cuda()
    torch.cuda.synchronize()
    for src in ("device", "pinned"):
        if src == "device":
            chunk = dev
        else:
            p = qsmd5.alloc_pinned(L)
            ctypes.memmove(p, ctypes.addressof(data), L)
            chunk = (p, L)
        c0 = resource.getrusage(resource.RUSAGE_THREAD)
        t0 = time.time()
        got = qsmd5.hash_batch([chunk], flags=qsmd5.FLAG_GPU_ONLY)
        wall = time.time() - t0
        c1 = resource.getrusage(resource.RUSAGE_THREAD)
        cpu = (c1.ru_utime - c0.ru_utime) + (c1.ru_stime - c0.ru_stime)
        if src == "pinned":
            qsmd5.free_pinned(p)
        print("%s: 1 GiB chain %.2f s wall, %.3f s of the caller's CPU" % (src, wall, cpu))
        assert got == [want], src
        # device: one launch, the caller sleeps and polls; pinned: 4096 column
        # launches ordered by the host, which wakes per column (a spinning
        # caller would show cpu ~ wall)
        assert wall > 2.0 and cpu < (0.2 if src == "device" else 0.5) * wall, (src, wall, cpu)


def test_device_chunk_past_its_allocation_is_refused(monkeypatch):
    """A device chunk whose length runs past the end of its HIP allocation
    would send the kernel -- or the CPU backend's read-back copy -- out of
    bounds (a GPU memory fault, not a wrong digest): the batch is refused with
    -EINVAL before any launch or copy, forced onto the GPU, forced onto the
    CPU, and under auto routing (which sends one small chunk to the CPU).  The
    same allocation hashed to its last byte is fine.  The 64 MiB buffer is a
    hipMalloc of its own, made through the HIP runtime libqsmd5.so uses (a
    torch tensor may sit inside a larger cached segment, whose end is further
    out)."""
    MiB = 1 << 20
    size, tail = 64 * MiB, 8192
    paths = sorted({ln.split()[-1] for ln in open("/proc/self/maps")
                    if ln.split() and "libamdhip64.so" in ln.split()[-1]})
    if len(paths) != 1:
        pytest.skip("not exactly one HIP runtime mapped: %s" % paths)
    hip = ctypes.CDLL(paths[0])
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    p = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(p), size) == 0
    try:
        assert hip.hipMemset(p, 0, size) == 0 and hip.hipDeviceSynchronize() == 0
        base = p.value
        ok = qsmd5.hash_batch([(base + size - tail, tail)], flags=qsmd5.FLAG_GPU_ONLY)
        assert ok == [md5_ref(bytes(tail))]
        monkeypatch.setenv("QSMD5_BACKEND", "auto")
        for flags in (qsmd5.FLAG_GPU_ONLY, qsmd5.FLAG_CPU_ONLY, 0):
            with pytest.raises(qsmd5.Md5Error) as e:
                qsmd5.hash_batch([(base + size - tail, tail + 4096)], flags=flags)
            assert e.value.code == -errno.EINVAL, flags
            assert "runs past the end of its allocation" in str(e.value), str(e.value)
        # the MD5 class (a CPU context under auto, a GPU one forced): the piece
        # is refused, the context is left as it was and hashes on
        for backend in ("auto", "gpu"):
            monkeypatch.setenv("QSMD5_BACKEND", backend)
            m = qsmd5.MD5()
            m.update(b"abc")
            with pytest.raises(qsmd5.Md5Error) as e:
                m.update((base + size - tail, tail + 4096))
            assert e.value.code == -errno.EINVAL, backend
            m.update((base + size - tail, tail))
            assert m.finalize().hexdigest() == md5_ref(b"abc" + bytes(tail)).hex(), backend
    finally:
        hip.hipFree(p)
