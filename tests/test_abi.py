"""The C-ABI library (gobpfld_amd/libxdpemu.so) loads and exports every symbol include/xdpemu.h
declares; no compute calls (this runs without a GPU)."""
import ctypes as C
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _declared(header="xdpemu.h"):
    text = (ROOT / "include" / header).read_text()
    return sorted(set(re.findall(r"\b(xe_[a-z_0-9]+)\s*\(", text)))


def _all_declared():
    return sorted(s for h in sorted(p.name for p in (ROOT / "include").glob("*.h")) for s in _declared(h))


def test_header_symbol_list_is_complete():
    from gobpfld_amd import _native as N
    assert sorted(N.HEADER_SYMBOLS) == _declared()
    assert sorted(N.IO_HEADER_SYMBOLS) == _declared("xdpemu_io.h")


def test_product_exports_every_header_symbol(built):
    lib = C.CDLL(str(ROOT / "gobpfld_amd" / "libxdpemu.so"))
    missing = [s for s in _all_declared() if not hasattr(lib, s)]
    assert not missing


def test_product_version_and_settings(built):
    from gobpfld_amd import _native as N
    lib = N.product()
    assert lib.version().decode().startswith("xdpemu")
    st = N.Settings()
    assert lib.default_settings(C.byref(st)) == 0
    assert st.stack_frame_size == 256 and st.max_stack_frames == 8


def test_hostsim_exports_every_header_symbol(built):
    lib = C.CDLL(str(ROOT / "tests" / "hostsim" / "libxdpemu_hostsim.so"))
    assert not [s for s in _all_declared() if not hasattr(lib, s)]
