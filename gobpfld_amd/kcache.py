"""Parallel builds of per-program kernels through the on-disk kernel cache (include/xdpemu.h
xe_set_kernel_cache / xe_kernel_source / xe_compile_kernel_source).

hiprtc compiles one kernel at a time per process (about a second each for a classifier), so a host that
loads many programs — a test suite, a server starting with a set of XDP programs — compiles them in
worker processes instead: the generated sources go to a pool, every worker writes its code object into
the cache directory, and the VMs' own builds (xe_prepare, or their first batch) then load them from
there. Workers need no GPU; they only load the library and call its compile entry point.

    kcache.enable(lib, "/tmp/xe-kernels")
    sources = [s for vm in vms for s in vm.kernel_sources()]
    kcache.fill(sources, "/tmp/xe-kernels")
    for vm in vms: vm.prepare()           # cache hits
"""
from __future__ import annotations

import ctypes as C
import os

_worker_lib = None


def _worker_init(lib_path: str) -> None:
    global _worker_lib
    import atexit
    import shutil
    import tempfile
    # Concurrent hiprtc processes must not share comgr's scratch space: with a common TMPDIR their
    # temporary files collide (workers died of SIGBUS / hung after a few compiles), and comgr's own code
    # cache (~/.cache/comgr) is not safe for concurrent writers either. Each worker gets a private
    # scratch directory and no comgr cache (it fills ours).
    scratch = tempfile.mkdtemp(prefix="xe-kc-")
    os.environ["TMPDIR"] = scratch
    os.environ["AMD_COMGR_CACHE"] = "0"
    tempfile.tempdir = scratch
    atexit.register(shutil.rmtree, scratch, True)
    _worker_lib = C.CDLL(lib_path)
    fn = _worker_lib.xe_compile_kernel_source
    fn.restype = C.c_int
    fn.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p, C.c_size_t]


def _worker_compile(job: tuple[str, str, str]) -> tuple[str, float]:
    import time
    src, arch, d = job
    err = C.create_string_buffer(4096)
    t0 = time.perf_counter()
    rc = _worker_lib.xe_compile_kernel_source(src.encode(), arch.encode(), d.encode(), err, 4096)
    return ("" if rc == 0 else (err.value.decode(errors="replace") or "compile failed")), time.perf_counter() - t0


def enable(lib, cache_dir: str | os.PathLike) -> str:
    """Point the process's per-program kernel builds at `cache_dir` (created if missing)."""
    d = os.fspath(cache_dir)
    os.makedirs(d, exist_ok=True)
    lib.set_kernel_cache(d.encode())
    return d


def default_workers() -> int:
    """Worker processes for this host: the CPUs this process may use, at most 16 (a GPU box's share)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def code_object_name(src: str, arch: str = "gfx950", lib_path: str | os.PathLike | None = None) -> str:
    """File name of the code object `src` compiles to in a cache directory (no device needed)."""
    from . import _native as N
    lib = N.Lib(lib_path or N.product_path(), "xe_")
    buf = C.create_string_buffer(128)
    if lib.kernel_object_name(src.encode(), arch.encode(), buf, len(buf)) != 0:
        raise RuntimeError("xe_kernel_object_name failed")
    return buf.value.decode()


def fill(sources, cache_dir: str | os.PathLike, arch: str = "gfx950", workers: int | None = None,
         lib_path: str | os.PathLike | None = None) -> list[str]:
    """Compile every distinct source into `cache_dir` with a pool of worker processes; returns the
    error texts of the sources that failed (their VMs fall back as their own build would)."""
    from concurrent.futures import ProcessPoolExecutor
    import multiprocessing as mp
    from . import _native as N
    uniq = list(dict.fromkeys(sources))
    if not uniq:
        return []
    d = os.fspath(cache_dir)
    os.makedirs(d, exist_ok=True)
    path = os.fspath(lib_path or N.product_path())
    n = min(workers or default_workers(), len(uniq))
    with ProcessPoolExecutor(max_workers=n, mp_context=mp.get_context("spawn"), initializer=_worker_init,
                             initargs=(path,)) as ex:
        res = list(ex.map(_worker_compile, [(s, arch, d) for s in uniq]))
    global last_times
    last_times = [(t, s) for (_, t), s in zip(res, uniq)]
    return [e for e, _ in res if e]


last_times: list[tuple[float, str]] = []  # (seconds, source) of the last fill's compiles (cache hits ~0 s)
