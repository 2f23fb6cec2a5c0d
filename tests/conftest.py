import os
import sys

import pytest

# The library's streaming pipeline gives every lane its own HIP stream and
# caps its depth at the process's hardware queues - 1 (GPU_MAX_HW_QUEUES,
# HIP's default 4): the tests run it at the depth bench.py uses.  Set before
# HIP initialises (the torch import below).
os.environ["GPU_MAX_HW_QUEUES"] = "16"

# torch's bundled HIP runtime has the same soname (libamdhip64.so.7) as the
# system one libjxg.so links; importing torch first makes the process use a
# single HIP runtime.
try:
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the CPU suite
    torch = None

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "jpeg-xl-lossy-image-compression-thesis_amd")
ORACLE_DIR = os.path.join(ROOT, "oracle")
for p in (PKG_DIR, ORACLE_DIR, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


@pytest.fixture(scope="session")
def oracle():
    import oracle_ffi

    oracle_ffi.build()
    return oracle_ffi


@pytest.fixture(scope="session")
def decoder():
    import jxl_decode

    return jxl_decode


@pytest.fixture(scope="session")
def jxg_mod():
    import jxg

    jxg.load()
    return jxg
