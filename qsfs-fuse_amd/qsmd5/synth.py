"""Synthetic part data on the host: the SURVEY.md §8c LCG in numpy.

x <- x * 1103515245 + 12345 (mod 2^32), applied before each byte; byte =
(x >> 16) & 0xff; x0 = seed.  The same generator runs on the device as
qsmd5_synth_fill_lcg (md5_kernels.hip); this host form feeds the CPU
rehearsals of the multi-rank benches, where no device exists.  Blocks of
4096 bytes advance together by the generator's 4096-step jump.
"""
import numpy as np

_A, _C, _M = 1103515245, 12345, 1 << 32
_BLOCK = 4096


def _block_coeffs():
    """x_{k+1} = A_k x0 + C_k (mod 2^32) for k < _BLOCK, and the full jump."""
    a = np.empty(_BLOCK, dtype=np.uint64)
    c = np.empty(_BLOCK, dtype=np.uint64)
    ak, ck = 1, 0
    for k in range(_BLOCK):
        ak, ck = (ak * _A) % _M, (ck * _A + _C) % _M
        a[k], c[k] = ak, ck
    return a, c, ak, ck


_COEFFS = None


def lcg_fill(seed, n):
    """n bytes of LCG(seed) as a numpy uint8 array."""
    global _COEFFS
    if _COEFFS is None:
        _COEFFS = _block_coeffs()
    a, c, ja, jc = _COEFFS
    out = np.empty(((n + _BLOCK - 1) // _BLOCK) * _BLOCK, dtype=np.uint8)
    x0 = seed % _M
    mask = np.uint64(_M - 1)
    for b in range(0, out.size, _BLOCK):
        xs = (a * np.uint64(x0) + c) & mask
        out[b:b + _BLOCK] = ((xs >> np.uint64(16)) & np.uint64(0xff)).astype(np.uint8)
        x0 = (ja * x0 + jc) % _M
    return out[:n]
