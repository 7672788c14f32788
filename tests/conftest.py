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
    import os
    from gobpfld_amd import build as B
    if os.environ.get("XE_SKIP_PRODUCT_BUILD"):  # local CPU iteration: the hipcc build takes minutes
        B.build_oracle()
        B.build_hostsim()
        return True
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
    """GPU sessions: the per-program kernels the suite uses come from the package's ahead-of-time kernel
    cache (gobpfld_amd/kernels, filled by build() on a CPU machine: gobpfld_amd/aot.py). Whatever it
    misses (a source changed since) is built in the background by worker processes while the tests run;
    a test that gets there first compiles its own kernel, exactly as without a cache."""
    if not any(item.get_closest_marker("gpu") for item in request.session.items):
        yield None
        return
    import threading
    import torch
    if not torch.cuda.is_available():
        yield None
        return
    import os
    from gobpfld_amd import _native as N
    from gobpfld_amd import aot, kcache
    from gobpfld_amd import build as B
    if not os.environ.get("XE_SKIP_PRODUCT_BUILD"):  # (a rebuild on the GPU box would take minutes)
        B.build_all()
    d = kcache.enable(N.product(), aot.KERNEL_DIR)

    def fill():
        kcache.fill(aot.test_sources(), d)

    t = threading.Thread(target=fill, daemon=True)
    t.start()
    yield d


# ---- kernel compiles inside GPU tests (xe_kernel_cache_stats): a test that builds a per-program kernel
# itself instead of loading it from the ahead-of-time cache (gobpfld_amd/aot.py) is named with the
# seconds it spent, in the terminal summary
_COMPILES: list[tuple[str, int, float]] = []
_GPU_RAN = [False]


def _kernel_stats():
    import ctypes as C
    from gobpfld_amd import _native as N
    lib = N._product
    if lib is None or not lib.has("kernel_cache_stats"):
        return None
    h, c, s = C.c_uint64(), C.c_uint64(), C.c_double()
    lib.kernel_cache_stats(C.byref(h), C.byref(c), C.byref(s))
    return h.value, c.value, s.value


@pytest.hookimpl(hookwrapper=True)
def pytest_runtest_call(item):
    before = _kernel_stats() if item.get_closest_marker("gpu") else None
    _GPU_RAN[0] = _GPU_RAN[0] or before is not None
    yield
    if before is None:
        return
    after = _kernel_stats()
    if after and after[1] > before[1]:
        _COMPILES.append((item.nodeid, after[1] - before[1], after[2] - before[2]))


def pytest_terminal_summary(terminalreporter):
    st = _kernel_stats() if _GPU_RAN[0] else None
    if st is None:
        return
    tr = terminalreporter
    tr.section("per-program kernels")
    tr.write_line(f"loaded from the cache: {st[0]}; compiled in-process: {st[1]} ({st[2]:.1f} s)")
    for nodeid, n, s in sorted(_COMPILES, key=lambda x: -x[2])[:20]:
        tr.write_line(f"  {s:8.1f} s  {n:3d} kernel(s)  {nodeid}")
