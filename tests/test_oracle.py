"""The CPU oracle (oracle/md5_oracle.c) against the golden fixtures.

The fixtures were produced by the reference's own MD5.cpp compiled in place
(oracle/build_ref.sh, tests/golden/make_golden.py); this pins the oracle
before it is trusted as the checker for the HIP path.
"""
import ctypes
import hashlib
import os
import random

import pytest

from conftest import ROOT
from oracle_util import OracleCtx, lcg_bytes, md5_many, md5_ref, md5_ref_truncating

RFC_LITERAL = {  # RFC 1321 appendix A.5, independent of any build
    "": "d41d8cd98f00b204e9800998ecf8427e",
    "abc": "900150983cd24fb0d6963f7d28e17f72",
    "message digest": "f96b697d7cb7938d525a2f31aaf161d0",
}


def test_rfc1321_vectors(golden):
    cases = golden("rfc1321.json")["cases"]
    assert len(cases) == 7
    for c in cases:
        b = c["text"].encode()
        assert md5_ref(b).hex() == c["md5"]
        if c["text"] in RFC_LITERAL:
            assert c["md5"] == RFC_LITERAL[c["text"]]


def test_lcg_generator_matches_survey_definition():
    x, out = 777, bytearray()
    for _ in range(1000):
        x = (x * 1103515245 + 12345) & 0xffffffff
        out.append((x >> 16) & 0xff)
    assert bytes(lcg_bytes(777, 1000)) == bytes(out)


def test_lcg_lengths(golden):
    g = golden("lcg_lengths.json")
    assert g["seed"] == 12345
    big = max(c["len"] for c in g["cases"])
    data = lcg_bytes(12345, big)  # prefixes of one stream are the shorter cases
    addr = ctypes.addressof(data)
    got = md5_many([(addr, c["len"]) for c in g["cases"]])
    for c, d in zip(g["cases"], got):
        assert d.hex() == c["md5"], c["len"]
    # the SURVEY §8c headline value
    assert {c["len"]: c["md5"] for c in g["cases"]}[10485760] == "302bec822b27cea263612fb3f76fa34b"


def test_streaming_pieces(golden):
    g = golden("stream_pieces.json")
    data = lcg_bytes(g["seed"], g["len"])
    base = ctypes.addressof(data)
    for case in g["cases"]:
        ctx = OracleCtx()
        off = 0
        for cut in case["cuts"]:
            ctx.update(base + off, cut)
            off += cut
        assert ctx.final().hex() == case["md5"], case["cuts"][:4]


def test_ragged_and_sweep(golden):
    g = golden("ragged.json")
    bufs = [lcg_bytes(7000 + i, L) for i, L in enumerate(g["lengths"])]
    got = md5_many([(b, L) for b, L in zip(bufs, g["lengths"])], threads=os.cpu_count() or 4)
    assert [d.hex() for d in got] == g["md5"]
    del bufs
    for s in g["sweep"]:
        L = s["mib"] << 20
        bufs = [lcg_bytes(s["seed0"] + i, L) for i in range(len(s["md5"]))]
        got = md5_many([(b, L) for b in bufs])
        assert [d.hex() for d in got] == s["md5"], s["mib"]


def test_batch_10mib_prefix(golden):
    g = golden("batch_10MiB.json")
    assert len(g["md5"]) == 10000
    n = 48
    bufs = [lcg_bytes(12345 + i, g["len"]) for i in range(n)]
    got = md5_many([(b, g["len"]) for b in bufs], threads=os.cpu_count() or 4)
    assert [d.hex() for d in got] == g["md5"][:n]


def test_against_hashlib_random():
    rng = random.Random(1)
    for _ in range(200):
        n = rng.choice([rng.randrange(0, 300), rng.randrange(0, 1 << 16)])
        b = bytes(rng.getrandbits(8) for _ in range(n)) if n < 4096 else os.urandom(n)
        assert md5_ref(b) == hashlib.md5(b).digest()


def test_truncate32_semantics(golden):
    """Reference md5(std::string) hashes only len mod 2^32 bytes (MD5.h:53, MD5.cpp:106)."""
    g = golden("truncate32.json")
    L = g["len"]
    assert L > (1 << 32)
    data = lcg_bytes(g["seed"], L)
    assert md5_ref_truncating(data, L).hex() == g["reference_md5"]
    assert md5_ref(data, L).hex() == g["full_md5"]


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libref_md5.so")),
                    reason="reference build not present (only in the build container)")
def test_oracle_vs_reference_build():
    ref = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libref_md5.so"))
    ref.ref_md5_iostream.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    rng = random.Random(5)
    for _ in range(100):
        n = rng.randrange(0, 5000)
        b = os.urandom(n)
        out = ctypes.create_string_buffer(33)
        ref.ref_md5_iostream(b, n, out)
        assert out.value.decode() == md5_ref(b).hex()
