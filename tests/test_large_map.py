"""Hash maps above 2M entries (xe_runtime.cpp hash_cap): the device table is the largest one a value
handle can address (2^22 slots) once 2 x MaxEntries no longer fits, so MaxEntries up to 4,194,304 is
accepted; probes run longer above half load, results stay the reference's (emulator/maps_hash.go:65-123
capacity check included). Larger maps are still refused (XE_ERR_UNSUPPORTED)."""
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


def _case(lib_a, oracle_lib, n, settings=None):
    maps = [(MapDef(MAP_HASH, 4, 8, BIG), None)]
    umem, descs = packets(n, 64, seed=41)
    a = run_one(lib_a, prog_learn_u16(), maps, umem, descs, entries=_entries(), regs=False, settings=settings)
    b = run_one(oracle_lib, prog_learn_u16(), maps, umem, descs, entries=_entries(), regs=False)
    assert_same(a, b, "3M-entry map")


def test_large_map_hostsim(oracle_lib, hostsim_lib):
    _case(hostsim_lib, oracle_lib, 3000)


def test_too_large_map_refused(hostsim_lib):
    vm = VM(Settings(), lib=hostsim_lib)
    with pytest.raises(EmulatorError):
        vm.add_map(MapDef(MAP_HASH, 4, 8, (1 << 22) + 1))
    vm.close()


@pytest.mark.gpu
@pytest.mark.parametrize("engine", [1, 2], ids=["interp", "jit"])
def test_large_map_device(gpu_lib, oracle_lib, engine):
    _case(gpu_lib, oracle_lib, 60000, Settings(engine=engine))
