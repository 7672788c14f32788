"""Ahead-of-time kernels (gobpfld_amd/aot.py) and the packet-read window of the per-program kernels.

CPU: the host build generates the per-program kernel sources without a GPU, and the generator's
packet-offset interval analysis (xe_jit.cpp packet_read_range) gives each config the header window it
reads (C2 parses Ethernet / VLAN / the L3 protocol byte, C3-C5 the IPv4 5-tuple).
GPU: the product library, given the same VM, generates byte-identical sources — so a kernel cache built
on a machine without a GPU is what the device loads."""
import re

import pytest

from parity import config_case


def _case(name):
    prog, maps, entries, _, _ = config_case(name, 16, 4096)
    from gobpfld_amd.emulator import Settings
    return (prog, maps, entries, Settings())


def _window(src):
    lo = re.search(r"#define XE_HDR_LO (\d+)", src)
    hi = re.search(r"#define XE_HDR_HI (\d+)", src)
    return (int(lo.group(1)), int(hi.group(1))) if lo and hi else None


# [lo, hi): the packet bytes each config's program can read (l3 offset 14 or 18 with a VLAN tag)
WINDOWS = {"c1": (0, 0), "c2": (12, 28), "c3": (12, 42), "c4": (12, 42), "c5": (12, 42)}


@pytest.mark.parametrize("name", sorted(WINDOWS))
def test_window_from_packet_read_range(hostsim_lib, name):
    from gobpfld_amd import aot
    srcs = aot.sources([_case(name)], lib=hostsim_lib)
    assert srcs, "no kernel source generated"
    assert _window(srcs[0]) == WINDOWS[name]
    assert "#define XE_HDR_LO_PROVEN 1" in srcs[0]  # every read is at or above XE_HDR_LO


def test_unbounded_packet_pointer_keeps_full_window(hostsim_lib):
    """A packet pointer spilled to the stack and reloaded has no known offset: the whole 64-byte window."""
    from gobpfld_amd import aot
    from gobpfld_amd.asm import Asm
    from gobpfld_amd.emulator import Settings
    a = Asm()
    a.ldx(4, 6, 1, 0).stx(8, 10, -8, 6).ldx(8, 7, 10, -8).ldx(1, 0, 7, 30).exit()
    srcs = aot.sources([(a.assemble(), [], None, Settings())], lib=hostsim_lib)
    assert _window(srcs[0]) is None


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c2", "c3learn", "c5", "bpf2bpf"])
def test_host_generated_sources_equal_device_sources(gpu_lib, hostsim_lib, name):
    from gobpfld_amd import aot
    case = _case(name)
    assert aot.sources([case], lib=hostsim_lib) == aot.sources([case], lib=gpu_lib)
    assert len(aot.sources([case], lib=hostsim_lib, variants=(2,))) == 1  # the verdict-only variant
