#!/usr/bin/env python3
"""Generate the committed golden fixtures from the REFERENCE's own MD5.

Runs in the build container only (needs oracle/_ref/libref_md5.so, built by
oracle/build_ref.sh from /root/reference/src/base/MD5.cpp).  Every digest in
tests/golden/*.json is produced by the reference's md5(std::string)
(MD5.cpp:335-339) and, where noted, cross-checked against its
md5(shared_ptr<iostream>) form (MD5.cpp:341-349) and Python hashlib.

Data is never committed -- only (generator, seed, length) -> digest triples.
Generator "lcg" (SURVEY.md §8c): x <- x*1103515245 + 12345 (mod 2^32) before
each byte, byte = (x >> 16) & 0xff, x0 = seed.  It is produced here by
oracle_lcg_fill (oracle/md5_oracle.c) and on the GPU by qsmd5_synth_fill_lcg.

Usage: python tests/golden/make_golden.py [--skip-big]
"""
import argparse
import concurrent.futures as cf
import ctypes
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
MiB = 1 << 20

RFC1321 = [
    ("", "d41d8cd98f00b204e9800998ecf8427e"),
    ("a", "0cc175b9c0f1b6a831c399e269772661"),
    ("abc", "900150983cd24fb0d6963f7d28e17f72"),
    ("message digest", "f96b697d7cb7938d525a2f31aaf161d0"),
    ("abcdefghijklmnopqrstuvwxyz", "c3fcd3d76192e4007dfb496cca67e13b"),
    ("ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789",
     "d174ab98d277d9f5a5611c2c9f419d9f"),
    ("1234567890" * 8, "57edf4a22be3c955ac49da2e2107b67a"),
]

LCG_LENGTHS = sorted(set(
    list(range(0, 201)) +
    [255, 256, 257, 511, 512, 513, 1000, 1023, 1024, 1025, 4095, 4096, 4097, 8191, 8192,
     65535, 65536, 65537, 1048575, 1048576, 1048577, 4194304, 5767168,
     10485759, 10485760, 10485761, 67108864]))

SWEEP_MIB = [1, 2, 4, 8, 10, 16, 32, 64]


def load():
    ref = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libref_md5.so"))
    orc = ctypes.CDLL(os.path.join(ROOT, "oracle", "libmd5_oracle.so"))
    ref.ref_md5_string.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    ref.ref_md5_iostream.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    ref.ref_md5_pieces.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint32),
                                   ctypes.c_size_t, ctypes.c_char_p]
    orc.oracle_lcg_fill.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32]
    return ref, orc


def lcg(orc, seed, n):
    buf = ctypes.create_string_buffer(max(n, 1))
    orc.oracle_lcg_fill(buf, n, seed & 0xffffffff)
    return buf, n


def ref_hex(ref, buf, n, iostream=False):
    out = ctypes.create_string_buffer(33)
    (ref.ref_md5_iostream if iostream else ref.ref_md5_string)(buf, n, out)
    return out.value.decode()


def det_lengths(seed, lo, hi, total):
    """Deterministic log-uniform lengths in [lo, hi] (own 64-bit LCG, no numpy)."""
    import math
    x = seed
    out, acc = [], 0
    while acc < total:
        x = (x * 6364136223846793005 + 1442695040888963407) & ((1 << 64) - 1)
        u = (x >> 11) / float(1 << 53)
        L = int(round(math.exp(math.log(lo) + u * (math.log(hi) - math.log(lo)))))
        L = max(lo, min(hi, L))
        out.append(L)
        acc += L
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-big", action="store_true", help="skip 4096x10MiB and 4GiB+ fixtures")
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 4)
    args = ap.parse_args()
    ref, orc = load()

    # 1. RFC 1321 appendix A.5
    rfc = []
    for text, want in RFC1321:
        b = text.encode()
        got = ref_hex(ref, b, len(b))
        assert got == want == hashlib.md5(b).hexdigest(), (text, got, want)
        rfc.append({"text": text, "md5": got})
    json.dump({"source": "RFC 1321 A.5, digests by reference md5(std::string)", "cases": rfc},
              open(os.path.join(HERE, "rfc1321.json"), "w"), indent=1)

    # 2. LCG(12345) at edge lengths -- both reference call forms + hashlib.
    cases = []
    for L in LCG_LENGTHS:
        buf, n = lcg(orc, 12345, L)
        a = ref_hex(ref, buf, n)
        b = ref_hex(ref, buf, n, iostream=True)
        c = hashlib.md5(buf.raw[:n]).hexdigest()
        assert a == b == c, (L, a, b, c)
        cases.append({"len": L, "md5": a})
    json.dump({"generator": "lcg", "seed": 12345, "source": "reference md5(std::string) == "
               "md5(shared_ptr<iostream>) == hashlib", "cases": cases},
              open(os.path.join(HERE, "lcg_lengths.json"), "w"), indent=0)

    # 3. Streaming class API: MD5::update in pieces then finalize().
    pieces = []
    buf, n = lcg(orc, 4242, 200000)
    cut_sets = [[200000], [1] * 100 + [199900], [63, 1, 64, 65, 199807], [55, 9, 100000, 99936],
                [4096] * 48 + [3392], [0, 7, 0, 199993], [130000, 70000]]
    for cuts in cut_sets:
        assert sum(cuts) == n
        arr = (ctypes.c_uint32 * len(cuts))(*cuts)
        out = ctypes.create_string_buffer(33)
        ref.ref_md5_pieces(buf, arr, len(cuts), out)
        assert out.value.decode() == hashlib.md5(buf.raw[:n]).hexdigest()
        pieces.append({"cuts": cuts, "md5": out.value.decode()})
    json.dump({"generator": "lcg", "seed": 4242, "len": n, "source": "reference MD5 class "
               "update()*+finalize()", "cases": pieces},
              open(os.path.join(HERE, "stream_pieces.json"), "w"), indent=0)

    def hash_seed(seed, L):
        b, n = lcg(orc, seed, L)
        return ref_hex(ref, b, n)

    pool = cf.ThreadPoolExecutor(args.threads)

    # 4. Ragged batch (config 4): log-uniform lengths in [8 KiB, 64 MiB], seed 7,
    #    ~4 GiB, plus edge lengths; chunk i uses LCG seed 7000 + i.
    edges = [0, 1, 3, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128, 8191, 8192, 8193]
    lens = edges + det_lengths(7, 8 * 1024, 64 * MiB, 4 << 30)
    ragged = list(pool.map(lambda i: hash_seed(7000 + i, lens[i]), range(len(lens))))
    # Bufsize sweep (-b MiB, Parser.cpp:167): 8 chunks per size, seed 100000*S + i.
    sweep = []
    for S in SWEEP_MIB:
        d = list(pool.map(lambda i: hash_seed(100000 * S + i, S * MiB), range(8)))
        sweep.append({"mib": S, "seed0": 100000 * S, "md5": d})
    json.dump({"generator": "lcg", "seed_rule": "chunk i: 7000 + i", "lengths": lens,
               "md5": ragged, "sweep": sweep, "source": "reference md5(std::string)"},
              open(os.path.join(HERE, "ragged.json"), "w"), indent=0)

    # 5. Uniform 10 MiB batches (configs 2, 3 and 5): chunk i = LCG(12345 + i).
    count = 512 if args.skip_big else 10000
    digs = list(pool.map(lambda i: hash_seed(12345 + i, 10 * MiB), range(count)))
    json.dump({"generator": "lcg", "seed_rule": "chunk i: 12345 + i", "len": 10 * MiB,
               "md5": digs, "source": "reference md5(std::string)"},
              open(os.path.join(HERE, "batch_10MiB.json"), "w"))

    # 6. Length >= 4 GiB: the reference hashes only len mod 2^32 bytes.
    if not args.skip_big:
        L = (1 << 32) + 1000
        buf, n = lcg(orc, 99, L)
        trunc = ref_hex(ref, buf, n)
        full = hashlib.md5(memoryview(buf)[:n]).hexdigest()
        assert trunc == hashlib.md5(buf.raw[:1000]).hexdigest()
        json.dump({"generator": "lcg", "seed": 99, "len": L, "reference_md5": trunc,
                   "full_md5": full, "source": "reference md5(std::string) (truncating) and "
                   "hashlib (full RFC 1321)"},
                  open(os.path.join(HERE, "truncate32.json"), "w"), indent=1)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    sys.exit(main())
