"""Native build of the emulator (no cmake; hipcc/g++ directly, outputs in-tree).

Targets
  gobpfld_amd/libxdpemu.so          product: gfx950 kernels + host runtime + C ABI (hipcc)
  oracle/liboracle.so               test infrastructure: CPU restatement of emulator/ (g++)
  tests/hostsim/libxdpemu_hostsim.so test-only: the device interpreter logic compiled for the host
                                     (wave size 1) so CPU tests can exercise it; never used by the
                                     product path.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "gobpfld_amd" / "csrc"
LIB = ROOT / "gobpfld_amd" / "libxdpemu.so"
ORACLE_LIB = ROOT / "oracle" / "liboracle.so"
HOSTSIM_LIB = ROOT / "tests" / "hostsim" / "libxdpemu_hostsim.so"

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("XE_OFFLOAD_ARCH", "gfx950")


def _newer(target: Path, sources: list[Path]) -> bool:
    if not target.exists():
        return False
    t = target.stat().st_mtime
    return all(s.stat().st_mtime <= t for s in sources)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise RuntimeError(f"build failed: {cmd[0]} (exit {r.returncode})")


def _sources() -> list[Path]:
    return sorted(CSRC.glob("*.h")) + sorted(CSRC.glob("*.hip")) + sorted(CSRC.glob("*.cpp")) + [
        ROOT / "include" / "xdpemu.h"
    ]


def build_product(force: bool = False) -> Path:
    srcs = _sources()
    if not force and _newer(LIB, srcs):
        return LIB
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [
        HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
        "-Wno-unused-result", "-Wno-unused-command-line-argument",
        str(CSRC / "xe_kernel.hip"), str(CSRC / "xe_runtime.cpp"),
        "-o", str(tmp),
    ]
    _run(cmd)
    os.replace(tmp, LIB)
    return LIB


def build_oracle(force: bool = False) -> Path:
    srcs = [ROOT / "oracle" / "oracle.cpp", ROOT / "oracle" / "oracle.h", ROOT / "include" / "xdpemu.h"]
    if not force and _newer(ORACLE_LIB, srcs):
        return ORACLE_LIB
    cxx = shutil.which("g++") or "g++"
    tmp = ORACLE_LIB.with_suffix(".so.tmp")
    _run([cxx, "-O2", "-std=c++17", "-fPIC", "-shared", str(srcs[0]), "-o", str(tmp)])
    os.replace(tmp, ORACLE_LIB)
    return ORACLE_LIB


def build_hostsim(force: bool = False) -> Path:
    srcs = _sources()
    if not force and _newer(HOSTSIM_LIB, srcs):
        return HOSTSIM_LIB
    HOSTSIM_LIB.parent.mkdir(parents=True, exist_ok=True)
    cxx = shutil.which("g++") or "g++"
    tmp = HOSTSIM_LIB.with_suffix(".so.tmp")
    _run([cxx, "-O2", "-std=c++17", "-fPIC", "-shared", "-DXE_HOSTSIM", str(CSRC / "xe_runtime.cpp"), "-o", str(tmp)])
    os.replace(tmp, HOSTSIM_LIB)
    return HOSTSIM_LIB


def build_all(force: bool = False) -> None:
    build_oracle(force)
    build_hostsim(force)
    build_product(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
    print("built", LIB, ORACLE_LIB, HOSTSIM_LIB)
