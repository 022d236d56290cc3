"""ctypes access to the CPU oracle (oracle/md5_oracle.c) for tests only.

The oracle is the checker, never the thing under test: tests compare the HIP
path (through libqsmd5.so) with it and with the golden fixtures.
"""
import ctypes
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_o = None


def oracle():
    global _o
    if _o is None:
        L = ctypes.CDLL(os.path.join(ROOT, "oracle", "libmd5_oracle.so"))
        L.oracle_md5.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        L.oracle_md5_reference_string.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        L.oracle_lcg_fill.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32]
        L.oracle_md5_update.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
        L.oracle_md5_init.argtypes = [ctypes.c_void_p]
        L.oracle_md5_final.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_md5_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                       ctypes.c_void_p, ctypes.c_int]
        _o = L
    return _o


def lcg_bytes(seed, n):
    """LCG test data as a ctypes buffer (n bytes, mutable)."""
    buf = (ctypes.c_uint8 * max(n, 1))()
    oracle().oracle_lcg_fill(buf, n, seed & 0xffffffff)
    return buf


def md5_ref(data, n=None):
    """Oracle MD5 (full 64-bit length) of a bytes-like / ctypes buffer."""
    if n is None:
        n = len(data) if not isinstance(data, ctypes.Array) else ctypes.sizeof(data)
    out = (ctypes.c_uint8 * 16)()
    if isinstance(data, (bytes, bytearray)):
        data = (ctypes.c_uint8 * max(n, 1)).from_buffer_copy(bytes(data) or b"\0")
    oracle().oracle_md5(data, n, out)
    return bytes(out)


def md5_ref_truncating(data, n):
    """The reference md5(std::string) semantics: len mod 2^32 bytes."""
    out = (ctypes.c_uint8 * 16)()
    oracle().oracle_md5_reference_string(data, n, out)
    return bytes(out)


def md5_many(bufs_and_lens, threads=8):
    """Oracle digests of many (ctypes buffer or address, len) pairs on host threads."""
    n = len(bufs_and_lens)
    ptrs = (ctypes.c_void_p * n)()
    lens = (ctypes.c_uint64 * n)()
    for i, (b, L) in enumerate(bufs_and_lens):
        ptrs[i] = b if isinstance(b, int) else ctypes.addressof(b)
        lens[i] = L
    out = (ctypes.c_uint8 * (16 * n))()
    oracle().oracle_md5_batch(ptrs, lens, n, out, threads)
    raw = bytes(out)
    return [raw[16 * i:16 * i + 16] for i in range(n)]


class OracleCtx(object):
    """Streaming oracle (MD5::update semantics, 32-bit piece lengths)."""

    def __init__(self):
        self.buf = (ctypes.c_uint8 * 256)()
        oracle().oracle_md5_init(self.buf)

    def update(self, addr, n):
        oracle().oracle_md5_update(self.buf, addr, n)

    def final(self):
        out = (ctypes.c_uint8 * 16)()
        oracle().oracle_md5_final(self.buf, out)
        return bytes(out)
