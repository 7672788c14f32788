"""LRU_HASH values with a nil backing (maps_hash_lru.go:93-161: Update stores what ReadRange of the
value pointer gives; an unreadable range leaves the value without bytes). The device reads a value's
length word only once the map holds such a value (header word 4, xe_interp.h bmem_resolve); these
batches put one there mid-batch and read it and its neighbours afterwards, against the oracle."""
import numpy as np
import pytest

from gobpfld_amd.asm import JEQ, Asm
from gobpfld_amd.emulator import MAP_LRU_HASH, MODE_SEQUENTIAL, MapDef, Settings
from parity import assert_same, packets, run_one


def _program():
    """key = packet byte 0 (& 3). Byte 1 == 1: update the key with an 8-byte value read from fp-4 (4
    bytes inside the frame: an unreadable range, a nil-backed value); otherwise update it from fp-16
    when absent. Then look the key up and load 8 bytes from the value (R0), or 0xFFFF on a miss."""
    a = Asm()
    a.ldx(4, 6, 1, 0)
    a.ldx(1, 7, 6, 0)
    a.ldx(1, 8, 6, 1)
    a.alu64(0x50, 7, imm=3).stx(4, 10, -4, 7)
    a.st(8, 10, -16, 5)
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -4)
    a.jmp(JEQ, 8, "nil", imm=1)
    a.call(1).jmp(JEQ, 0, "ins", imm=0).ja("look")
    a.label("ins")
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -4).mov64(3, src=10).add64(3, -16).mov64(4, 0).call(2).ja("look")
    a.label("nil")
    a.mov64(3, src=10).add64(3, -4).mov64(4, 0).call(2)
    a.label("look")
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.jmp(JEQ, 0, "miss", imm=0)
    a.ldx(8, 0, 0, 0).exit()
    a.label("miss").mov64(0, 0xFFFF).exit()
    return a.assemble()


def _case(lib, oracle_lib, mode):
    maps = [(MapDef(MAP_LRU_HASH, 4, 8, 16), None)]
    umem, descs = packets(600, 64, seed=9)
    pk = umem.reshape(-1)
    # byte 1 == 1 on a few packets after the start: those keys become nil-backed
    for d in descs[:600]:
        pk[int(d["addr"]) + 1] = 0
    for i in (150, 151, 400):
        pk[int(descs[i]["addr"]) + 1] = 1
    s = Settings(mode=mode)
    a = run_one(lib, _program(), maps, umem, descs, settings=s)
    b = run_one(oracle_lib, _program(), maps, umem, descs)
    assert_same(a, b, f"nil-backed LRU values (mode {mode})")


@pytest.mark.parametrize("mode", [0, MODE_SEQUENTIAL], ids=["auto", "seq"])
def test_lru_nil_value_hostsim(hostsim_lib, oracle_lib, mode):
    _case(hostsim_lib, oracle_lib, mode)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, MODE_SEQUENTIAL], ids=["auto", "seq"])
def test_lru_nil_value_device(gpu_lib, oracle_lib, mode):
    _case(gpu_lib, oracle_lib, mode)
