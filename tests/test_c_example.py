"""The C ABI from plain C (examples/xdp_batch.c, the shape of the cgo binding in INTEGRATION.md):
compiled and linked against gobpfld_amd/libxdpemu.so on the CPU; run on the GPU (-m gpu)."""
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.fixture(scope="module")
def example_bin(built, tmp_path_factory):
    out = tmp_path_factory.mktemp("cex") / "xdp_batch"
    lib = ROOT / "gobpfld_amd"
    r = subprocess.run(["gcc", "-O2", "-Wall", "-Werror", "-I", str(ROOT / "include"), str(ROOT / "examples" / "xdp_batch.c"),
                        "-L", str(lib), "-lxdpemu", f"-Wl,-rpath,{lib}", "-o", str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return out


def test_c_example_builds_against_the_abi(example_bin):
    assert example_bin.exists()


@pytest.mark.gpu
def test_c_example_runs_on_device(example_bin):
    r = subprocess.run([str(example_bin), "30000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "packets=30000 pass=30000 counts=11000,10000,10007" in r.stdout


def test_c_example_runs_on_hostsim(built, tmp_path):
    """The same C program linked against the host simulation build (CPU): the InitialData image
    (ArrayMap.Init translation) and the batch run through the C ABI, without a GPU."""
    sim = ROOT / "tests" / "hostsim"
    lnk = tmp_path / "libxdpemu.so"
    lnk.symlink_to(sim / "libxdpemu_hostsim.so")
    out = tmp_path / "xdp_batch_sim"
    r = subprocess.run(["gcc", "-O2", "-Wall", "-Werror", "-I", str(ROOT / "include"), str(ROOT / "examples" / "xdp_batch.c"),
                        "-L", str(tmp_path), "-lxdpemu", f"-Wl,-rpath,{tmp_path}", "-o", str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(out), "3000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "packets=3000 pass=3000 counts=2000,1000,1007" in r.stdout
