import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def built():
    from gobpfld_amd import build as B
    B.build_all()
    return True


@pytest.fixture(scope="session")
def oracle_lib(built):
    from gobpfld_amd import _native as N
    return N.Lib(ROOT / "oracle" / "liboracle.so", "orc_")


@pytest.fixture(scope="session")
def hostsim_lib(built):
    from gobpfld_amd import _native as N
    return N.Lib(ROOT / "tests" / "hostsim" / "libxdpemu_hostsim.so", "xe_")


@pytest.fixture(scope="session")
def gpu_lib(built):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU is visible")
    from gobpfld_amd import _native as N
    return N.product()
