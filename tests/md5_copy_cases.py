"""Copy semantics of the MD5 class (qsmd5_ctx_copy), shared by the CPU-backend
and GPU tests.  The reference MD5 (MD5.h:51-93) is a value type: a copy taken
mid-stream carries the running state -- the 64-bit count, the buffered tail
(MD5::buffer, MD5.h:79) and the chaining state -- and then hashes on by
itself, and operator<< takes it by value (MD5.h:61)."""
from oracle_util import lcg_bytes, md5_ref


def run_copy_cases(qsmd5, piece):
    """piece(data, off, n) -> what MD5.update() takes for data[off:off+n]
    (host bytes, a (ptr, len) pair or a device tensor slice)."""
    data = bytes(lcg_bytes(8675309, 300000))
    ref = lambda b: md5_ref(b).hex()
    # (prefix, suffix of the copy, suffix of the original): copies taken at an
    # empty state, inside a block (tail pending), on a block boundary, deep
    # into the stream, and suffixes that cross blocks or stay in the tail
    for pre, a_more, b_more in ((0, 0, 1), (0, 64, 3), (5, 59, 60), (64, 0, 128), (100, 200000, 7),
                                (131072, 1, 100000), (299999, 1, 0)):
        m = qsmd5.MD5()
        m.update(piece(data, 0, pre))
        c = m.copy()
        c.update(piece(data, pre, a_more))
        m.update(piece(data, pre + 10, b_more))  # different bytes: the two must not share state
        assert c.finalize().hexdigest() == ref(data[:pre + a_more]), (pre, a_more)
        assert m.finalize().hexdigest() == ref(data[:pre] + data[pre + 10:pre + 10 + b_more]), (pre, b_more)
    # a copy of a finalised context is finalised with the same digest; a
    # copy of a copy; the original stays usable after its copy is gone
    m = qsmd5.MD5()
    m.update(piece(data, 0, 1000))
    c = m.copy()
    cc = c.copy()
    del c
    m.update(piece(data, 1000, 24))
    assert m.finalize().hexdigest() == ref(data[:1024])
    done = m.copy()
    assert done.hexdigest() == ref(data[:1024])
    done.update(piece(data, 0, 5))  # after finalize: a no-op, as the reference
    assert done.finalize().hexdigest() == ref(data[:1024])
    cc.update(piece(data, 1000, 5000))
    assert cc.finalize().hexdigest() == ref(data[:6000])
