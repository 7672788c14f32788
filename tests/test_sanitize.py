"""ASan/UBSan builds of the oracle and of the host simulation of the device logic: both are
compiled with -fsanitize=address,undefined (no recovery), a sanitized C++ driver runs every KAT, a
slice of the differential fuzzer and the BASELINE configs at small sizes through both and compares
every observable (tests/sanitize/san_driver.cpp). A sanitizer report fails the test. The host simulation is
built with XE_HOSTSIM_POISON: device allocations start as 0xA5 garbage (hipMalloc does not clear) and the
simulated lane's registers as zero, so logic that reads what it never wrote shows up here rather than as a
device fault that depends on what an earlier kernel left in memory."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
SAN = ROOT / "tests" / "sanitize"
OUT = SAN / "_build"
FLAGS = ["-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
         "-fno-omit-frame-pointer"]


def _build(target: Path, cmd: list[str], sources: list[Path]) -> Path:
    if target.exists() and all(s.stat().st_mtime <= target.stat().st_mtime for s in sources):
        return target
    tmp = target.with_suffix(target.suffix + f".{os.getpid()}.tmp")
    r = subprocess.run(cmd + ["-o", str(tmp)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    os.replace(tmp, target)
    return target


@pytest.mark.slow
def test_sanitized_oracle_and_hostsim_agree(tmp_path):
    cxx = shutil.which("g++")
    if not cxx:
        pytest.skip("g++ missing")
    OUT.mkdir(exist_ok=True)
    csrc = ROOT / "gobpfld_amd" / "csrc"
    hdrs = sorted(csrc.glob("*.h")) + [ROOT / "include" / "xdpemu.h", ROOT / "include" / "xdpemu_io.h"]
    orc = _build(OUT / "liboracle_san.so", [cxx, *FLAGS, "-fPIC", "-shared", str(ROOT / "oracle" / "oracle.cpp")],
                 [ROOT / "oracle" / "oracle.cpp", ROOT / "oracle" / "oracle.h", *hdrs])
    sim_src = [csrc / "xe_runtime.cpp", csrc / "xe_io.cpp", csrc / "xe_multi.cpp", csrc / "xe_jit.cpp"]
    sim = _build(OUT / "libxdpemu_hostsim_san.so",
                 [cxx, *FLAGS, "-fPIC", "-shared", "-DXE_HOSTSIM", "-DXE_HOSTSIM_POISON", *map(str, sim_src), "-pthread"], sim_src + hdrs)
    drv = _build(OUT / "san_driver", [cxx, *FLAGS, str(SAN / "san_driver.cpp"), "-ldl"], [SAN / "san_driver.cpp"])
    import importlib.util
    spec = importlib.util.spec_from_file_location("san_cases", SAN / "cases.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    write = mod.write
    cases = tmp_path / "cases.bin"
    n = write(cases)
    env = dict(os.environ)
    # the driver links the sanitizer runtimes itself; an unrelated preload ahead of them is tolerated
    env["ASAN_OPTIONS"] = "verify_asan_link_order=0:detect_leaks=1:abort_on_error=1"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    r = subprocess.run([str(drv), str(orc), str(sim), str(cases)], capture_output=True, text=True, env=env,
                       timeout=900)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert f"{n} cases, 0 mismatches" in r.stdout, r.stdout
