"""The reference's own example programs, run through the emulator.

Both are xdp-tutorial's basic03-map-counter as gobpfld ships it, written two ways:
  * cmd/examples/xdp_stats_assembly/main.go:52-77 — clang-style assembly text (ebpf.AssemblyToInstructions);
  * cmd/examples/xdp_stats_instructions/main.go:33-124 — ebpf.Instruction literals (ebpf.MustEncode).
Each is transcribed here as data in this repository's own encoders (tests/asm_text.py for the text form, the
label-free offsets written out; gobpfld_amd.asm for the literals), with the loader's map relocation applied as
program_abstract.go:84-113 does for MapFDLocations = {"xdp_stats_map": [8 * 4]}: the LD_IMM64 at slot 4 gets
src = BPF_PSEUDO_MAP_FD and imm = the map (the VM's map index 1, emulator/inst_load.go:36-63). The map is the
examples' xdp_stats_map: ARRAY, key 4, value 8, MaxEntries 5.

CPU: the two transcriptions encode to the same program, and the oracle runs it over the C2 packet stream to
what the program means — every packet XDP_PASS, xdp_stats_map[XDP_PASS] counting them. GPU: the device equals
the oracle on every observable over the C2 stream, on both engines.
"""
import numpy as np
import pytest

from asm_text import encode
from gobpfld_amd import workloads as W
from gobpfld_amd.asm import Asm, JEQ, XDP_ABORTED, XDP_PASS
from gobpfld_amd.emulator import ENGINE_INTERP, ENGINE_JIT, MAP_ARRAY, MapDef, Settings
from parity import assert_same, run_one

STATS_MAP = (MapDef(MAP_ARRAY, 4, 8, 5), None)

# xdp_stats_assembly/main.go:52-77 in tests/asm_text.py's syntax (`goto return` is +3 from slot 8)
ASM_TEXT = """
r1 = 2
*(u32 *)(r10 - 4) = r1
r2 = r10
r2 += -4
r1 = 0 ll
call 1#bpf_map_lookup_elem
r1 = 0
if r0 == 0 goto +3
r1 = 1
lock *(u64 *)(r0 + 0) += r1
r1 = 2
r0 = r1
exit
"""

MAP_FD_SLOT = 4  # MapFDLocations: uint64(ebpf.BPFInstSize) * 4


def relocate(prog: list[int], map_idx: int = 1) -> list[int]:
    """program_abstract.go:84-113 for one map location: src := BPF_PSEUDO_MAP_FD (1), imm := the map."""
    p = list(prog)
    w = p[MAP_FD_SLOT]
    assert w & 0xFF == 0x18, "the relocated slot must be an LD_IMM64"
    w = (w & ~(0xF << 12)) | (1 << 12)
    w = (w & 0xFFFFFFFF) | (map_idx << 32)
    p[MAP_FD_SLOT] = w
    return p


def from_text() -> list[int]:
    return relocate(encode(ASM_TEXT))


def from_literals() -> list[int]:
    """xdp_stats_instructions/main.go:57-124, literal by literal."""
    a = Asm()
    a.mov64(1, XDP_PASS)                 # Mov64{Dest: R1, Value: XDP_PASS}
    a.stx(4, 10, -4, 1)                  # StoreMemoryRegister{Size: W, Dest: R10, Offset: -4, Src: R1}
    a.mov64(2, src=10)                   # Mov64Register{Dest: R2, Src: R10}
    a.add64(2, -4)                       # Add64{Dest: R2, Value: -4}
    a.ld_imm64(1, 0)                     # LoadConstant64bit{Dest: R1} + Nop (the loader fills it in)
    a.call(1)                            # CallHelper{Function: 1}
    a.mov64(1, XDP_ABORTED)              # Mov64{Dest: R1, Value: XDP_ABORTED}
    a.jmp(JEQ, 0, "lbl0", imm=0)         # JumpEqual{Dest: R0, Offset: 3, Value: 0}
    a.mov64(1, 1)                        # Mov64{Dest: R1, Value: 1}
    a.xadd(8, 0, 0, 1)                   # AtomicAdd{Size: DW, Dest: R0, Src: R1}
    a.mov64(1, XDP_PASS)                 # Mov64{Dest: R1, Value: XDP_PASS}
    a.label("lbl0")
    a.mov64(0, src=1)                    # Mov64Register{Dest: R0, Src: R1}
    a.exit()                             # Exit{}
    return relocate(a.assemble())


def test_transcriptions_agree():
    t, lit = from_text(), from_literals()
    assert len(t) == 14 and t == lit


@pytest.mark.parametrize("form", ["assembly", "instructions"])
def test_example_on_oracle(oracle_lib, form):
    prog = from_text() if form == "assembly" else from_literals()
    n = 4096
    umem, descs = W.build_batch("c2", 0, n)
    r, dumps, _ = run_one(oracle_lib, prog, [STATS_MAP], umem, descs)
    assert (r.results["status"] == 0).all() and (r.verdicts == XDP_PASS).all()
    counts = np.frombuffer(dumps[0], dtype=np.uint64)
    assert counts.tolist() == [0, 0, n, 0, 0]  # xdp_stats_map[XDP_PASS] == packets processed
    assert r.stats["steps"] == 14 * n  # every slot runs, the LD_IMM64 filler as a Nop (ebpf/decode.go:34)


@pytest.mark.gpu
@pytest.mark.parametrize("engine", [ENGINE_INTERP, ENGINE_JIT], ids=["interp", "jit"])
@pytest.mark.parametrize("form", ["assembly", "instructions"])
def test_example_device_equals_oracle(gpu_lib, oracle_lib, form, engine):
    prog = from_text() if form == "assembly" else from_literals()
    umem, descs = W.build_batch("c2", 0, 65536)
    a = run_one(gpu_lib, prog, [STATS_MAP], umem, descs, settings=Settings(engine=engine))
    b = run_one(oracle_lib, prog, [STATS_MAP], umem, descs)
    assert_same(a, b, f"{form} example")
    assert a[0].stats["engine_used"] == engine and a[0].stats["mode_used"] == 1
