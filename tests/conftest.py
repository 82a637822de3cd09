import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session", autouse=True)
def _native_built():
    """Build the in-tree native libraries once if they are missing (hipcc
    cross-compiles without a GPU)."""
    from oneccl_amd import build as b
    need = [b.LIB / "libmi_reduce.so", b.LIB / "libccl_comp_hip.so", ROOT / "oracle" / "lib" / "libcomp_oracle.so"]
    if not all(p.exists() for p in need) and os.environ.get("MI_SKIP_BUILD") != "1":
        b.build_mi_reduce()
        b.build_shim()
        b.build_oracle()
    yield
