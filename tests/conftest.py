"""pytest configuration: the `gpu` marker, import paths, shared fixtures.

`-m "not gpu"` tests run on any CPU box: the oracle against the golden
fixtures, host-only C-ABI logic (hex, part planning), the exported-symbol
check of libqsmd5.so, and the multi-rank digest gather over gloo.
`-m gpu` tests are the parity tests proper: every digest through the C-ABI on
an MI355X against the committed golden fixtures (produced by the reference's
own MD5.cpp) and the oracle.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "qsfs-fuse_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")

# Parity tests measure the gfx950 kernels, never the library's CPU backend:
# every test (and every subprocess it starts) runs with QSMD5_BACKEND=gpu
# unless it sets the backend itself, and the `gpu_only_backend` fixture below
# fails any -m gpu test during which the CPU backend hashed anything.
os.environ["QSMD5_BACKEND"] = "gpu"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "cpu_backend: exercises the library's CPU routing/fallback")


# Host-sanitizer runs (test_gpu_sanitizers.py) are the slowest GPU tests and
# the only ones that run uninstrumented vendor runtimes under TSan/ASan.  They
# go last, so that under `-x` a failure there can never leave a parity test
# unrun (round 3: a sanitizer child stopped the suite with 17 tests behind it).
# The memory-pressure test (another tenant holding nearly all HBM) goes just
# before them, for the same reason: it depends on the box's free memory.
LAST_FILES = ("test_gpu_memory_pressure.py", "test_gpu_sanitizers.py")


def pytest_collection_modifyitems(session, config, items):
    def rank(it):
        name = os.path.basename(str(it.fspath))
        return LAST_FILES.index(name) + 1 if name in LAST_FILES else 0
    items.sort(key=rank)  # stable


def _ensure_built():
    """Build oracle/ and libqsmd5.so in place if a fresh checkout lacks them."""
    oracle_so = os.path.join(ROOT, "oracle", "libmd5_oracle.so")
    lib_so = os.path.join(ROOT, "qsfs-fuse_amd", "lib", "libqsmd5.so")
    if not os.path.exists(oracle_so):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "libmd5_oracle.so"])
    if not os.path.exists(lib_so):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "qsfs-fuse_amd"), "-j4"])


_ensure_built()


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden():
    return load_golden


@pytest.fixture(autouse=True)
def gpu_only_backend(request):
    """In -m gpu tests, the CPU backend must not have hashed a single call
    (tests of the routing and fallback opt out with @pytest.mark.cpu_backend)."""
    if request.node.get_closest_marker("gpu") is None or \
            request.node.get_closest_marker("cpu_backend") is not None:
        yield
        return
    import qsmd5
    before = qsmd5.stats()["cpu_batches"]
    yield
    after = qsmd5.stats()["cpu_batches"]
    assert after == before, "the CPU backend hashed %d call(s) in a GPU parity test" % (after - before)
