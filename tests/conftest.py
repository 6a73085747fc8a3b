import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mos-networking-stack_amd")
for p in (os.path.join(ROOT, "tests"), PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (MI355X); runs the HIP path")


def _ensure_built():
    """Build the oracle and libmosrx.so in-tree if missing (cross-compiles without a GPU)."""
    if not os.path.exists(os.path.join(ROOT, "oracle", "libmosrx_oracle.so")):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    if not os.path.exists(os.path.join(PKG, "libmosrx.so")):
        subprocess.check_call(["make", "-s", "-C", PKG])


_ensure_built()


@pytest.fixture(scope="session")
def gpu_ctx():
    import mosrx
    ctx = mosrx.Context(0)
    yield ctx
    ctx.close()
