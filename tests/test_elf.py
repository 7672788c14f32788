"""ELF loading + relocation to VM indices (gobpfld_amd/elf.py), on synthetic objects
of clang's shape (tests/elfgen.py): the loader's output, then the loaded programs run through the
oracle, the host simulation of the device logic and (-m gpu) the HIP product."""
import struct

import numpy as np
import pytest

from elfgen import R_BPF_64_32, R_BPF_64_64, build_elf
from gobpfld_amd import elf as E
from gobpfld_amd.asm import JEQ, Asm
from gobpfld_amd.emulator import VM, Settings
from parity import assert_same, packets

XDP_PASS = 2


def stats_object():
    """basic03_map_counter shape: an ARRAY of per-action counters, lookup + lock xadd."""
    a = Asm()
    a.st(4, 10, -4, XDP_PASS)
    a.ld_imm64(1, 0)                       # r1 = &xdp_stats_map (relocated)
    a.mov64(2, src=10).add64(2, -4)
    a.call(1)
    a.jmp(JEQ, 0, "out", imm=0)
    a.mov64(1, 1).xadd(8, 0, 0, 1)
    a.label("out").mov64(0, XDP_PASS).exit()
    insns = a.assemble()
    elf = build_elf({"xdp": (insns, [("xdp_stats1_func", 0, len(insns) * 8)])},
                    maps=[("xdp_stats_map", 2, 4, 8, 5, 0)],
                    relocs={"xdp": [(8, "xdp_stats_map", R_BPF_64_64)]})
    want = Asm()
    want.st(4, 10, -4, XDP_PASS).ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    want.jmp(JEQ, 0, "out", imm=0).mov64(1, 1).xadd(8, 0, 0, 1).label("out").mov64(0, XDP_PASS).exit()
    return elf, want.assemble()


def rodata_object():
    """Global data: r0 = *(u32 *)(.rodata + 4) through BPF_PSEUDO_MAP_FD_VALUE."""
    a = Asm()
    a.ld_imm64(1, 4)                       # .rodata + 4 (offset in imm, REL addend)
    a.ldx(4, 0, 1, 0).exit()
    insns = a.assemble()
    rodata = struct.pack("<III", 7, 0xC0FFEE, 9)
    elf = build_elf({"xdp": (insns, [("read_ro", 0, len(insns) * 8)])}, rodata=rodata, bss=16,
                    relocs={"xdp": [(0, ".rodata", R_BPF_64_64)]})
    return elf


def call_object():
    """bpf-to-bpf: the program calls a .text function (R_BPF_64_32 call relocation)."""
    a = Asm()
    a.mov64(1, 5)
    a.emit(0x85, 0, 1, 0, -1)              # call .text+0 (BPF_PSEUDO_CALL, imm = target - 1)
    a.exit()
    insns = a.assemble()
    t = Asm()
    t.mov64(0, src=1).alu64(0x20, 0, imm=3).exit()   # r0 = r1 * 3
    elf = build_elf({"xdp": (insns, [("caller", 0, len(insns) * 8)])}, text=t.assemble(),
                    relocs={"xdp": [(8, ".text", R_BPF_64_32)]})
    return elf


def _run(lib, obj, prog, n=64, size=64):
    vm = VM(Settings(), lib=lib)
    _, idx = E.load_into_vm(vm, obj, prog)
    umem, descs = packets(n, size, seed=11)
    mem = umem.copy()
    r = vm.run_batch(mem, descs, want_regs=True)
    dumps = [vm.map_dump(m) for m in idx.values()]
    vm.close()
    return r, dumps, mem


def test_parse_maps_programs_and_relocation():
    data, want = stats_object()
    obj = E.parse_elf(data)
    assert obj.license == "GPL"
    assert list(obj.maps) == ["xdp_stats_map"]
    d, init = obj.maps["xdp_stats_map"]
    assert (d.type, d.key_size, d.value_size, d.max_entries) == (2, 4, 8, 5) and init is None
    assert list(obj.programs) == ["xdp_stats1_func"]
    assert obj.programs["xdp_stats1_func"].map_refs == {"xdp_stats_map": [8]}
    assert obj.relocated("xdp_stats1_func") == want


def test_global_data_relocation():
    obj = E.parse_elf(rodata_object())
    assert list(obj.maps) == ["rodata", "bss"]                    # declaration order: .rodata, .data, .bss
    d, init = obj.maps["rodata"]
    assert (d.type, d.key_size, d.value_size, d.max_entries) == (2, 4, 12, 1) and len(init) == 12
    assert obj.maps["bss"][1] is None and obj.maps["bss"][0].value_size == 16
    raw = obj.relocated("read_ro")
    op, regs, off, imm = struct.unpack("<BBhi", struct.pack("<Q", raw[0]))
    assert (op, regs >> 4, imm) == (0x18, 2, 1)                    # src = BPF_PSEUDO_MAP_FD_VALUE, map 1
    assert struct.unpack("<BBhi", struct.pack("<Q", raw[1]))[3] == 4  # offset moved to the second slot


def test_text_call_relocation():
    obj = E.parse_elf(call_object())
    raw = obj.relocated("caller")
    assert len(raw) == 3 + 3                                       # .text appended (elf.go:643-648)
    op, regs, off, imm = struct.unpack("<BBhi", struct.pack("<Q", raw[1]))
    assert (op, regs >> 4, imm) == (0x85, 1, 1)                    # 3 + (-1) - 1: lands on slot 3


def test_rejects_non_bpf_and_bad_reloc():
    with pytest.raises(E.ElfError, match="machine type"):
        E.parse_elf(build_elf({"xdp": ([0x95], [("f", 0, 8)])}, machine=62))
    with pytest.raises(E.ElfError, match="not an ELF"):
        E.parse_elf(b"\0" * 64)


def test_elf_programs_oracle_known_answers(oracle_lib):
    data, _ = stats_object()
    r, dumps, _ = _run(oracle_lib, E.parse_elf(data), "xdp_stats1_func")
    assert (r.results["status"] == 0).all() and (r.verdicts == XDP_PASS).all()
    counters = np.frombuffer(dumps[0], dtype=np.uint64)
    assert counters[XDP_PASS] == 64 and counters.sum() == 64
    r, _, _ = _run(oracle_lib, E.parse_elf(rodata_object()), "read_ro")
    assert (r.results["status"] == 0).all() and (r.results["r0"] == 0xC0FFEE).all()
    r, _, _ = _run(oracle_lib, E.parse_elf(call_object()), "caller")
    assert (r.results["status"] == 0).all() and (r.results["r0"] == 15).all()


def _obj(which):
    return {"stats": lambda: stats_object()[0], "rodata": rodata_object, "call": call_object}[which]()


@pytest.mark.parametrize("which", ["stats", "rodata", "call"])
def test_elf_programs_hostsim_equal_oracle(oracle_lib, hostsim_lib, which):
    data = _obj(which)
    obj = E.parse_elf(data)
    prog = next(iter(obj.programs))
    assert_same(_run(hostsim_lib, obj, prog), _run(oracle_lib, obj, prog), f"elf {which}")


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["stats", "rodata", "call"])
def test_elf_programs_device_equal_oracle(gpu_lib, oracle_lib, which):
    data = _obj(which)
    obj = E.parse_elf(data)
    prog = next(iter(obj.programs))
    assert_same(_run(gpu_lib, obj, prog, n=4096), _run(oracle_lib, obj, prog, n=4096), f"elf {which} (device)")
