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


@pytest.fixture(scope="session", autouse=True)
def _kernel_cache(request):
    """GPU sessions: build every per-program kernel the suite uses in worker processes, in the
    background, into a session kernel cache (gobpfld_amd/kcache.py; hiprtc compiles one kernel at a time
    per process). Tests start at once and load their kernels from the cache when it has them; a test
    that gets there first compiles its own, exactly as without the cache."""
    if not any(item.get_closest_marker("gpu") for item in request.session.items):
        yield None
        return
    import tempfile
    import threading
    import torch
    if not torch.cuda.is_available():
        yield None
        return
    from gobpfld_amd import _native as N
    from gobpfld_amd import build as B
    from gobpfld_amd import kcache
    from kernel_cases import gpu_cases
    from parity import kernel_sources
    B.build_all()
    lib = N.product()
    d = kcache.enable(lib, tempfile.mkdtemp(prefix="xe-kernels-"))
    sources = kernel_sources(lib, gpu_cases())
    t = threading.Thread(target=kcache.fill, args=(sources, d), daemon=True)
    t.start()
    yield d
