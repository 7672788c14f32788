"""Hash maps above 4M entries. The reference's only capacity rule is `len(m.Values)+1 > MaxEntries`
(emulator/maps_hash.go:84-89); a Go map has no size ceiling. On the device a table of more than 2^23 slots
is a "big map" (xe_internal.h XE_H_BIG): its value handles carry the slot's high bits in the map field, so
slots up to 2^26 stay one 32-bit handle — MaxEntries up to 16,777,216 at half load, up to 2^25 above it
(xe_runtime.cpp hash_cap). The tables here put most entries past slot 2^23: lookups, in-place adds,
inserts and register records (the map index of a value pointer) equal the oracle's. Beyond 2^25 entries,
or a big map past the 31st map, the map is refused (XE_ERR_UNSUPPORTED)."""
import numpy as np
import pytest

from gobpfld_amd.asm import JEQ, Asm, XDP_DROP, XDP_PASS
from gobpfld_amd.emulator import MAP_HASH, EmulatorError, MapDef, Settings, VM
from parity import assert_same, packets, run_one

AND = 0x50
BIG = 3_000_000


def prog_learn_u16():
    """HASH(4 B -> u64) keyed by bytes 0-1 (& 0xffff): hit -> += 1, PASS; miss -> insert 1, DROP."""
    a = Asm()
    a.ldx(4, 6, 1, 0).ldx(2, 8, 6, 0)
    a.stx(4, 10, -4, 8).ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.jmp(JEQ, 0, "ins", imm=0)
    a.mov64(1, 1).xadd(8, 0, 0, 1).mov64(0, XDP_PASS).exit()
    a.label("ins")
    a.st(8, 10, -16, 1)
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -4).mov64(3, src=10).add64(3, -16).mov64(4, 0).call(2)
    a.mov64(0, XDP_DROP).exit()
    return a.assemble()


def _entries():
    return {0: [(np.uint32(k).tobytes(), np.uint64(7).tobytes()) for k in range(0, 65536, 3)]}


SIZES = {"3M": BIG, "16M": 1 << 24, "32M": 1 << 25}


def _case(lib_a, oracle_lib, n, max_entries=BIG, settings=None, regs=True):
    maps = [(MapDef(MAP_HASH, 4, 8, max_entries), None)]
    umem, descs = packets(n, 64, seed=41)
    a = run_one(lib_a, prog_learn_u16(), maps, umem, descs, entries=_entries(), regs=regs, settings=settings)
    b = run_one(oracle_lib, prog_learn_u16(), maps, umem, descs, entries=_entries(), regs=regs)
    assert_same(a, b, f"{max_entries}-entry map")


@pytest.mark.parametrize("size", ["3M", "16M"])
def test_large_map_hostsim(oracle_lib, hostsim_lib, size):
    _case(hostsim_lib, oracle_lib, 3000, SIZES[size])


def test_too_large_map_refused(hostsim_lib):
    vm = VM(Settings(), lib=hostsim_lib)
    with pytest.raises(EmulatorError):
        vm.add_map(MapDef(MAP_HASH, 4, 8, (1 << 25) + 1))
    vm.close()


def test_big_map_index_limits(hostsim_lib):
    """A big map must be among the first 31 maps, and a VM with one holds at most 31 maps."""
    vm = VM(Settings(), lib=hostsim_lib)
    for _ in range(31):
        vm.add_map(MapDef(MAP_HASH, 4, 8, 16))
    with pytest.raises(EmulatorError):
        vm.add_map(MapDef(MAP_HASH, 4, 8, 1 << 24))
    vm.close()
    vm = VM(Settings(), lib=hostsim_lib)
    vm.add_map(MapDef(MAP_HASH, 4, 8, 1 << 24))
    for _ in range(30):
        vm.add_map(MapDef(MAP_HASH, 4, 8, 16))
    with pytest.raises(EmulatorError):
        vm.add_map(MapDef(MAP_HASH, 4, 8, 16))
    vm.close()


@pytest.mark.gpu
@pytest.mark.parametrize("engine", [1, 2], ids=["interp", "jit"])
@pytest.mark.parametrize("size", ["3M", "16M", "32M"])
def test_large_map_device(gpu_lib, oracle_lib, engine, size):
    _case(gpu_lib, oracle_lib, 60000, SIZES[size], Settings(engine=engine))
