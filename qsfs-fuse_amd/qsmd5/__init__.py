"""qsmd5 -- Python binding of the MI355X MD5 chunk-hashing path (include/qsmd5.h).

Thin ctypes layer over ``qsfs-fuse_amd/lib/libqsmd5.so``; tests, bench.py and
__graft_entry__ use it.  It mirrors the reference interface names:

  md5(data) -> str              std::string md5(const std::string)   MD5.cpp:335-339
  md5_stream(stream) -> str     std::string md5(shared_ptr<iostream>) MD5.cpp:341-349
  MD5().update(b).finalize().hexdigest()   class MD5                MD5.h:51-93

plus the batch entry points the reference lacks (hash_batch, hash_parts,
hash_device).  If the library is missing this module raises on first use
(``lib()``).  The library picks the backend per call (QSMD5_BACKEND =
auto | gpu | cpu, or FLAG_GPU_ONLY / FLAG_CPU_ONLY): under "gpu" every hash
runs on the gfx950 kernels and, without a GPU, raises ``Md5Error`` with
-ENODEV; under "auto" small calls and GPU failures are hashed by the
library's own CPU MD5 (``stats()`` / ``last_backend()`` say which ran).
"""
import ctypes
import errno
import os

__all__ = [
    "Md5Error", "lib", "lib_path", "shutdown", "hexdigest", "md5", "md5_stream", "MD5", "hash_batch",
    "hash_one", "hash_device", "hash_parts", "plan_parts", "kernel_choice", "device_count",
    "alloc_pinned", "free_pinned", "hash_read", "buffer_reader", "register_host", "unregister_host", "synth_fill_lcg", "last_timing", "Part", "etag_matches",
    "verify_etag", "FLAG_REF_TRUNCATE32", "FLAG_ALIGNED16", "FLAG_HOST", "FLAG_GPU_ONLY", "FLAG_BACKGROUND", "FLAG_READ_PARALLEL",
    "FLAG_CPU_ONLY", "stats", "rates", "cpu_efficiency", "last_backend", "route", "BACKEND_GPU", "BACKEND_CPU", "BACKEND_SPLIT",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG_ROOT = os.path.dirname(_HERE)


def lib_path():
    return os.environ.get("QSMD5_LIB", os.path.join(_PKG_ROOT, "lib", "libqsmd5.so"))


class Md5Error(RuntimeError):
    def __init__(self, code, what):
        self.code = code
        super().__init__("%s failed: %d (%s)" % (what, code, _detail(code)))


class qsmd5_chunk(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("len", ctypes.c_uint64)]


class Stats(ctypes.Structure):
    """qsmd5_stats: process-wide backend counters."""
    _fields_ = [("gpu_batches", ctypes.c_uint64), ("cpu_batches", ctypes.c_uint64),
                ("fallbacks", ctypes.c_uint64), ("gpu_chunks", ctypes.c_uint64),
                ("cpu_chunks", ctypes.c_uint64), ("gpu_lost", ctypes.c_int),
                ("inits", ctypes.c_int)]

    def asdict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class Rates(ctypes.Structure):
    """qsmd5_rates: what auto routing prices a batch with (GiB/s)."""
    _fields_ = [("cpu_chain_gibs", ctypes.c_double), ("cpu_lane_thread_gibs", ctypes.c_double),
                ("gpu_chain_gibs", ctypes.c_double), ("link_gibs", ctypes.c_double),
                ("d2h_gibs", ctypes.c_double), ("gpu_call_ms", ctypes.c_double),
                ("cpu_threads", ctypes.c_int), ("source", ctypes.c_int)]

    def asdict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class Part(ctypes.Structure):
    """qsmd5_part: one multipart-upload part (QSTransferManager.cpp:475-550)."""
    _fields_ = [("part_number", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
                ("offset", ctypes.c_uint64), ("size", ctypes.c_uint64)]

    def __repr__(self):
        return "Part(%d, off=%d, size=%d)" % (self.part_number, self.offset, self.size)

    def astuple(self):
        return (self.part_number, self.offset, self.size)


_lib = None

# qsmd5_read_fn: uint64_t (*)(void* user, size_t chunk, uint64_t offset, uint64_t len, void* dst)
READ_FN = ctypes.CFUNCTYPE(ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64,
                           ctypes.c_uint64, ctypes.c_void_p)

# qsmd5_log_fn: void (*)(int level, const char* msg, void* user)
LOG_FN = ctypes.CFUNCTYPE(None, ctypes.c_int, ctypes.c_char_p, ctypes.c_void_p)
LOG_INFO, LOG_WARN, LOG_ERROR = 0, 1, 2  # qsfs LogLevel::Value (base/LogLevel.h:27)
# Every ctypes callback ever installed, for the life of the process: the
# library never frees a replaced sink because another thread may have loaded it
# and be about to call it (qsmd5_rt_device.cpp), so the code it points at must
# not be freed either.  A few hundred bytes per installed sink.
_log_keep = []


def lib():
    """Load libqsmd5.so (raises OSError loudly if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    path = lib_path()
    if not os.path.exists(path):
        raise OSError("libqsmd5.so not built at %s (run __graft_entry__.build())" % path)
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so.7.
    # Loading torch first lets libqsmd5's NEEDED libamdhip64.so.7 bind to that
    # copy instead of pulling /opt/rocm's in beside it (two runtimes in one
    # process leave torch without devices).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(path)
    c_u8p = ctypes.POINTER(ctypes.c_uint8)
    sig = {
        "qsmd5_init": (ctypes.c_int, [ctypes.c_int]),
        "qsmd5_shutdown": (ctypes.c_int, []),
        "qsmd5_abi_version": (ctypes.c_int, []),
        "qsmd5_device_count": (ctypes.c_int, []),
        "qsmd5_strerror": (ctypes.c_char_p, [ctypes.c_int]),
        "qsmd5_last_error": (ctypes.c_char_p, []),
        "qsmd5_hash_one": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, c_u8p]),
        "qsmd5_hash_batch": (ctypes.c_int, [ctypes.POINTER(qsmd5_chunk), ctypes.c_size_t, c_u8p]),
        "qsmd5_hash_batch_ex": (ctypes.c_int, [ctypes.POINTER(qsmd5_chunk), ctypes.c_size_t,
                                               c_u8p, ctypes.c_int]),
        "qsmd5_hash_batch_device_async": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p,
                                                         ctypes.c_size_t, ctypes.c_void_p,
                                                         ctypes.c_void_p]),
        "qsmd5_kernel_choice": (ctypes.c_int, [ctypes.c_size_t]),
        "qsmd5_kernel_choice_ex": (ctypes.c_int, [ctypes.c_size_t, ctypes.c_int]),
        "qsmd5_hash_batch_device_async_ex": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p,
                                                            ctypes.c_size_t, ctypes.c_void_p,
                                                            ctypes.c_void_p, ctypes.c_int]),
        "qsmd5_hex": (None, [c_u8p, ctypes.c_char_p]),
        "qsmd5_base64": (None, [c_u8p, ctypes.c_char_p]),
        "qsmd5_ctx_create": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p)]),
        "qsmd5_ctx_update": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]),
        "qsmd5_ctx_final": (ctypes.c_int, [ctypes.c_void_p, c_u8p]),
        "qsmd5_ctx_destroy": (None, [ctypes.c_void_p]),
        "qsmd5_ctx_copy": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]),
        "qsmd5_alloc_pinned": (ctypes.c_int, [ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]),
        "qsmd5_free_pinned": (ctypes.c_int, [ctypes.c_void_p]),
        "qsmd5_register_host": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t]),
        "qsmd5_unregister_host": (ctypes.c_int, [ctypes.c_void_p]),
        "qsmd5_plan_parts": (ctypes.c_int, [ctypes.c_uint64] * 5 + [
            ctypes.POINTER(Part), ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]),
        "qsmd5_hash_parts": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Part), ctypes.c_size_t,
                                            c_u8p]),
        "qsmd5_etag_matches": (ctypes.c_int, [c_u8p, ctypes.c_char_p]),
        "qsmd5_verify_etag": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_char_p]),
        "qsmd5_last_backend": (ctypes.c_int, []),
        "qsmd5_route": (ctypes.c_int, [ctypes.POINTER(qsmd5_chunk), ctypes.c_size_t, ctypes.c_int]),
        "qsmd5_get_stats": (ctypes.c_int, [ctypes.POINTER(Stats)]),
        "qsmd5_get_rates": (ctypes.c_int, [ctypes.POINTER(Rates)]),
        "qsmd5_last_timing": (ctypes.c_int, [ctypes.POINTER(ctypes.c_double),
                                             ctypes.POINTER(ctypes.c_double)]),
        "qsmd5_synth_fill_lcg": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                                ctypes.c_uint32, ctypes.c_uint32,
                                                ctypes.c_void_p]),
        "qsmd5_set_log_callback": (ctypes.c_int, [LOG_FN, ctypes.c_void_p]),
        "qsmd5_get_cpu_efficiency": (ctypes.c_int, [ctypes.POINTER(ctypes.c_double)]),
        "qsmd5_hash_read": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t, READ_FN,
                                           ctypes.c_void_p, ctypes.c_uint64, c_u8p, ctypes.c_int]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def _detail(code):
    try:
        L = lib()
        return "%s; %s" % (L.qsmd5_strerror(code).decode(), L.qsmd5_last_error().decode())
    except OSError:
        return os.strerror(-code) if code < 0 else str(code)


def _check(rc, what):
    if rc != 0:
        raise Md5Error(rc, what)


def device_count():
    return lib().qsmd5_device_count()


def shutdown():
    """qsmd5_shutdown: release the runtime's GPU resources (idempotent; a later
    call initialises afresh)."""
    _check(lib().qsmd5_shutdown(), "qsmd5_shutdown")


def set_log_callback(fn):
    """qsmd5_set_log_callback: route the library's messages to fn(level, text)
    (level LOG_INFO / LOG_WARN / LOG_ERROR) instead of stderr; None restores
    the default.  fn runs on the thread that made the qsmd5 call."""
    if fn is None:
        _check(lib().qsmd5_set_log_callback(LOG_FN(), None), "qsmd5_set_log_callback")
        return
    cb = LOG_FN(lambda level, msg, _user: fn(level, msg.decode(errors="replace")))
    _log_keep.append(cb)  # before the library can call it; never dropped (see _log_keep)
    _check(lib().qsmd5_set_log_callback(cb, None), "qsmd5_set_log_callback")


def kernel_choice(n, flags=0):
    return lib().qsmd5_kernel_choice_ex(n, flags)


FLAG_REF_TRUNCATE32 = 1
FLAG_ALIGNED16 = 2
FLAG_HOST = 4  # every chunk is host memory: skip the per-chunk pointer query
FLAG_GPU_ONLY = 8  # gfx950 kernels only: no CPU routing or fallback
FLAG_CPU_ONLY = 16  # the library's CPU MD5 only
FLAG_BACKGROUND = 32  # latency hidden by the caller: the GPU whenever one is usable (auto)
FLAG_READ_PARALLEL = 64  # hash_read: read may run on several library threads at once
BACKEND_GPU = 1
BACKEND_CPU = 2
BACKEND_SPLIT = 3  # both at once: the longest host chunks on the CPU, the rest on the GPU


def stats():
    """Process-wide backend counters (qsmd5_get_stats) as a dict."""
    st = Stats()
    _check(lib().qsmd5_get_stats(ctypes.byref(st)), "qsmd5_get_stats")
    return st.asdict()


RATE_CPU_MEASURED, RATE_CPU_ENV, RATE_GPU_MEASURED, RATE_GPU_ENV = 1, 2, 4, 8


def rates():
    """qsmd5_get_rates as a dict: the rates auto routing uses on this host."""
    r = Rates()
    _check(lib().qsmd5_get_rates(ctypes.byref(r)), "qsmd5_get_rates")
    return r.asdict()


def cpu_efficiency():
    """qsmd5_get_cpu_efficiency: the share of its priced rate the CPU backend
    got lately (1.0 on an idle host); auto routing divides CPU estimates by it."""
    v = ctypes.c_double()
    _check(lib().qsmd5_get_cpu_efficiency(ctypes.byref(v)), "qsmd5_get_cpu_efficiency")
    return v.value


def route(lengths, flags=0):
    """Backend (BACKEND_CPU / BACKEND_GPU / BACKEND_SPLIT) that
    QSMD5_BACKEND=auto picks for a batch of host chunks of these lengths (host
    logic; no data is read, the pointers are placeholders)."""
    n = len(lengths)
    arr = (qsmd5_chunk * max(n, 1))()
    for i, L in enumerate(lengths):
        arr[i].ptr = 1 if L else 0
        arr[i].len = L
    return lib().qsmd5_route(arr, n, flags | FLAG_HOST)


def last_backend():
    """BACKEND_GPU / BACKEND_CPU / BACKEND_SPLIT of this thread's last hashing
    call (0: none)."""
    return lib().qsmd5_last_backend()


def hexdigest(digest):
    """16 raw bytes -> 32 lowercase hex chars via qsmd5_hex (MD5.cpp:317-325)."""
    d = (ctypes.c_uint8 * 16).from_buffer_copy(bytes(digest))
    out = ctypes.create_string_buffer(33)
    lib().qsmd5_hex(d, out)
    return out.value.decode()


def content_md5(digest):
    """16 raw bytes -> RFC 1864 Content-MD5 header value (base64, 24 chars)."""
    d = (ctypes.c_uint8 * 16).from_buffer_copy(bytes(digest))
    out = ctypes.create_string_buffer(25)
    lib().qsmd5_base64(d, out)
    return out.value.decode()


# ---- buffers -------------------------------------------------------------------------

def _as_chunk(buf, keep):
    """(ptr, len) of bytes/bytearray/memoryview/numpy/torch tensor (any device)."""
    try:
        import torch  # noqa: F401
        if isinstance(buf, torch.Tensor):
            if not buf.is_contiguous():
                raise ValueError("tensor must be contiguous")
            return buf.data_ptr(), buf.numel() * buf.element_size()
    except ImportError:
        pass
    if isinstance(buf, tuple) and len(buf) == 2:  # raw (ptr, len)
        return int(buf[0]), int(buf[1])
    if isinstance(buf, bytes):
        cb = ctypes.c_char_p(buf)
        keep.append(cb)
        return ctypes.cast(cb, ctypes.c_void_p).value, len(buf)
    mv = memoryview(buf)
    if not mv.contiguous:
        raise ValueError("buffer must be contiguous")
    n = mv.nbytes
    if n == 0:
        return 0, 0
    if mv.readonly:
        # read-only views (e.g. slices of bytes): borrow without copying
        import numpy as np
        a = np.frombuffer(mv, dtype=np.uint8)
        keep.append(a)
        return a.ctypes.data, n
    c = (ctypes.c_uint8 * n).from_buffer(mv)
    keep.append(c)
    return ctypes.addressof(c), n


def hash_batch(buffers, flags=0):
    """MD5 of every buffer (host or device), one batch -> list of 16-byte digests."""
    bufs = list(buffers)
    n = len(bufs)
    if n == 0:
        return []
    keep = []
    arr = (qsmd5_chunk * n)()
    for i, b in enumerate(bufs):
        p, L = _as_chunk(b, keep)
        arr[i].ptr = p
        arr[i].len = L
    out = (ctypes.c_uint8 * (16 * n))()
    _check(lib().qsmd5_hash_batch_ex(arr, n, out, flags), "qsmd5_hash_batch")
    raw = bytes(out)
    return [raw[16 * i:16 * i + 16] for i in range(n)]


def hash_one(buf):
    keep = []
    p, L = _as_chunk(buf, keep)
    out = (ctypes.c_uint8 * 16)()
    _check(lib().qsmd5_hash_one(p, L, out), "qsmd5_hash_one")
    return bytes(out)


def md5(data):
    """Mirror of the reference free function md5(std::string) -> lowercase hex."""
    if isinstance(data, str):
        data = data.encode("latin-1")
    return hexdigest(hash_one(data))


def md5_stream(stream):
    """Mirror of md5(shared_ptr<iostream>) (MD5.cpp:341-349): hash the stream's
    bytes from position 0 to its end and leave the read position at 0."""
    stream.seek(0)
    data = stream.read()
    stream.seek(0)
    if isinstance(data, str):
        data = data.encode("latin-1")
    return md5(data)


def hash_device(chunks_dev, digests_dev, n, order_dev=None, stream=0, flags=0):
    """Enqueue qsmd5_hash_batch_device_async_ex.  chunks_dev: device pointer to n
    qsmd5_chunk records (int64 pairs); digests_dev: device pointer to [n,16] uint8."""
    _check(lib().qsmd5_hash_batch_device_async_ex(
        ctypes.c_void_p(int(chunks_dev)), ctypes.c_void_p(int(order_dev or 0)), n,
        ctypes.c_void_p(int(digests_dev)), ctypes.c_void_p(int(stream or 0)), flags),
        "qsmd5_hash_batch_device_async")


def plan_parts(file_size, buf_size=10 << 20, min_part=4 << 20, threshold=20 << 20,
               range_begin=0):
    """QSTransferManager::PrepareUpload slicing -> list of Part."""
    L = lib()
    need = ctypes.c_size_t(0)
    _check(L.qsmd5_plan_parts(file_size, buf_size, min_part, threshold, range_begin, None, 0,
                              ctypes.byref(need)), "qsmd5_plan_parts")
    arr = (Part * max(need.value, 1))()
    _check(L.qsmd5_plan_parts(file_size, buf_size, min_part, threshold, range_begin, arr,
                              need.value, ctypes.byref(need)), "qsmd5_plan_parts")
    return [arr[i] for i in range(need.value)]


def hash_parts(file_buf, parts):
    """Batch pre-hash of all parts of one file buffer (host or device)."""
    keep = []
    p, _ = _as_chunk(file_buf, keep)
    n = len(parts)
    if n == 0:
        return []
    arr = (Part * n)(*parts)
    out = (ctypes.c_uint8 * (16 * n))()
    _check(lib().qsmd5_hash_parts(p, arr, n, out), "qsmd5_hash_parts")
    raw = bytes(out)
    return [raw[16 * i:16 * i + 16] for i in range(n)]


def hash_read(lens, read, staging_bytes=0, flags=0):
    """qsmd5_hash_read: MD5 of n chunks the library pulls in column windows
    through ``read(chunk, offset, length, dst_address) -> bytes copied`` (the
    File::ReadNoLoad form), staging at most ``staging_bytes`` (0: default).
    Returns the list of 16-byte digests.  An exception in ``read`` fails the
    call and is re-raised here."""
    lens = [int(x) for x in lens]
    n = len(lens)
    if n == 0:
        return []
    arr = (ctypes.c_uint64 * n)(*lens)
    errors = []

    def thunk(_user, chunk, offset, length, dst):
        if errors:
            return 0
        try:
            return int(read(chunk, offset, length, dst))
        except BaseException as e:  # noqa: B902 -- carried to the caller below
            errors.append(e)
            return 0  # a short read: the library stops and returns -EIO

    cb = READ_FN(thunk)  # alive for the whole call: the library calls it only inside it
    out = (ctypes.c_uint8 * (16 * n))()
    rc = lib().qsmd5_hash_read(arr, n, cb, None, staging_bytes, out, flags)
    if errors:
        raise errors[0]
    _check(rc, "qsmd5_hash_read")
    raw = bytes(out)
    return [raw[16 * i:16 * i + 16] for i in range(n)]


def buffer_reader(chunks):
    """A read callback over in-memory chunks [(address, length), ...]: copies
    the asked window with ctypes.memmove."""
    def read(chunk, offset, length, dst):
        addr, L = chunks[chunk]
        if offset + length > L:
            return 0
        ctypes.memmove(dst, addr + offset, length)
        return length
    return read


class MD5(object):
    """Mirror of the reference class MD5 (MD5.h:51-93) over qsmd5_ctx."""

    def __init__(self, text=None):
        self._ctx = ctypes.c_void_p()
        _check(lib().qsmd5_ctx_create(ctypes.byref(self._ctx)), "qsmd5_ctx_create")
        self._digest = None
        if text is not None:
            self.update(text)
            self.finalize()

    def update(self, data):
        # after finalize() the reference's update leaves the digest as it was
        # (MD5.cpp:240-269, 284-312): a no-op here too
        if self._digest is not None:
            return self
        if isinstance(data, str):
            data = data.encode("latin-1")
        keep = []
        p, L = _as_chunk(data, keep)
        _check(lib().qsmd5_ctx_update(self._ctx, p, L), "qsmd5_ctx_update")
        return self

    def copy(self):
        """An independent copy with the running state (the reference class is a
        value type, MD5.h:51-93); as hashlib's copy()."""
        other = MD5.__new__(MD5)
        other._ctx = ctypes.c_void_p()
        _check(lib().qsmd5_ctx_copy(self._ctx, ctypes.byref(other._ctx)), "qsmd5_ctx_copy")
        other._digest = self._digest
        return other

    __copy__ = copy

    def finalize(self):
        if self._digest is None:
            out = (ctypes.c_uint8 * 16)()
            _check(lib().qsmd5_ctx_final(self._ctx, out), "qsmd5_ctx_final")
            self._digest = bytes(out)
        return self

    def digest(self):
        return self._digest

    def hexdigest(self):
        # MD5::hexdigest returns "" before finalize (MD5.cpp:318)
        return hexdigest(self._digest) if self._digest is not None else ""

    def __del__(self):
        try:
            if self._ctx:
                lib().qsmd5_ctx_destroy(self._ctx)
                self._ctx = ctypes.c_void_p()
        except Exception:
            pass


def etag_matches(digest, etag):
    """qsmd5_etag_matches: True/False, or raises Md5Error(-EINVAL) for a
    multipart / malformed ETag."""
    d = (ctypes.c_uint8 * 16).from_buffer_copy(bytes(digest))
    rc = lib().qsmd5_etag_matches(d, etag.encode() if isinstance(etag, str) else etag)
    if rc < 0:
        raise Md5Error(rc, "qsmd5_etag_matches")
    return rc == 1


def verify_etag(buf, etag):
    """Hash a downloaded buffer (host or device) on the GPU and compare with its ETag."""
    keep = []
    p, L = _as_chunk(buf, keep)
    rc = lib().qsmd5_verify_etag(p, L, etag.encode() if isinstance(etag, str) else etag)
    if rc < 0:
        raise Md5Error(rc, "qsmd5_verify_etag")
    return rc == 1


def alloc_pinned(nbytes):
    p = ctypes.c_void_p()
    _check(lib().qsmd5_alloc_pinned(nbytes, ctypes.byref(p)), "qsmd5_alloc_pinned")
    return p.value


def free_pinned(ptr):
    _check(lib().qsmd5_free_pinned(ctypes.c_void_p(ptr)), "qsmd5_free_pinned")


def register_host(ptr, nbytes):
    _check(lib().qsmd5_register_host(ctypes.c_void_p(ptr), nbytes), "qsmd5_register_host")


def unregister_host(ptr):
    _check(lib().qsmd5_unregister_host(ctypes.c_void_p(ptr)), "qsmd5_unregister_host")


def synth_fill_lcg(base_ptr, stride, length, seed0, nchunks, stream=0):
    _check(lib().qsmd5_synth_fill_lcg(ctypes.c_void_p(base_ptr), stride, length, seed0, nchunks,
                                      ctypes.c_void_p(int(stream or 0))), "qsmd5_synth_fill_lcg")


def last_timing():
    w, k = ctypes.c_double(), ctypes.c_double()
    lib().qsmd5_last_timing(ctypes.byref(w), ctypes.byref(k))
    return w.value, k.value


ENODEV = -errno.ENODEV
