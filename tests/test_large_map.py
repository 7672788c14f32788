"""Hash maps above 4M entries. The reference's only capacity rule is `len(m.Values)+1 > MaxEntries`
(emulator/maps_hash.go:84-89); a Go map has no size ceiling. On the device a table of more than 2^23 slots
is a "big map" (xe_internal.h XE_H_BIG): the 32 map-field values 32..63 of a value handle are shared out
among a VM's big maps, each taking ceil(slots / 2^23) of them, so up to 2^28 slots over all big maps stay
one 32-bit handle: one table of up to 2^27 slots (MaxEntries up to 2^27, xe_runtime.cpp hash_cap) with
others beside it. The tables here put most entries past slot 2^23: lookups, in-place adds, inserts and
register records (the map index of a value pointer) equal the oracle's; one test holds 4.2M live entries
and fills the map to MaxEntries, so inserts past it return E2BIG in packet order. Beyond 2^27 entries, more
fields than there are, or a big map past the 31st map, the map is refused (XE_ERR_UNSUPPORTED)."""
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


SIZES = {"3M": BIG, "16M": 1 << 24, "32M": 1 << 25, "64M": 1 << 26, "128M": 1 << 27}


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
    from gobpfld_amd.emulator import MAP_LRU_HASH
    vm = VM(Settings(), lib=hostsim_lib)
    with pytest.raises(EmulatorError):
        vm.add_map(MapDef(MAP_HASH, 4, 8, (1 << 27) + 1))
    with pytest.raises(EmulatorError):
        vm.add_map(MapDef(MAP_LRU_HASH, 4, 8, (1 << 26) + 1))
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
@pytest.mark.parametrize("size", ["3M", "16M", "32M", "128M"])
def test_large_map_device(gpu_lib, oracle_lib, engine, size):
    _case(gpu_lib, oracle_lib, 60000, SIZES[size], Settings(engine=engine))


@pytest.mark.gpu
def test_big_maps_share_the_handle_fields(gpu_lib):
    """2^26 entries (2^27 slots: 17 fields) + 2^25 (2^26 slots: 9) + 2^24 (2^25 slots: 5) = 31 of the 32
    fields; a fourth big map (2^23 entries: 3 fields) does not fit and is refused, a small map still is
    not big and fits."""
    vm = VM(Settings(), lib=gpu_lib)
    for e in (1 << 26, 1 << 25, 1 << 24):
        vm.add_map(MapDef(MAP_HASH, 4, 8, e))
    with pytest.raises(EmulatorError):
        vm.add_map(MapDef(MAP_HASH, 4, 8, 1 << 23))
    vm.add_map(MapDef(MAP_HASH, 4, 8, 1 << 20))
    vm.close()


LIVE_MAX = 4_200_000  # MaxEntries: more than 4,194,304 live entries


def prog_learn_u32():
    """HASH(4 B -> u64) keyed by packet bytes 0-3: hit -> += 1, R0 = PASS; miss -> insert 1, R0 = the
    update's result (0, or E2BIG = -7 once the map holds MaxEntries: maps_hash.go:84-89)."""
    a = Asm()
    a.ldx(4, 6, 1, 0).ldx(4, 8, 6, 0)
    a.stx(4, 10, -4, 8).ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.jmp(JEQ, 0, "ins", imm=0)
    a.mov64(1, 1).xadd(8, 0, 0, 1).mov64(0, XDP_PASS).exit()
    a.label("ins")
    a.st(8, 10, -16, 1)
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -4).mov64(3, src=10).add64(3, -16).mov64(4, 0).call(2)
    a.exit()
    return a.assemble()


def _live_case(lib, n=100_000, room=1000):
    """A HASH map of MaxEntries LIVE_MAX holding LIVE_MAX - room entries; a batch of lookups of live keys
    and inserts of 3 x room distinct new keys: the first `room` (in packet order) are inserted, the rest
    return E2BIG. -> (results, count, (keys, values) of the entries whose keys the batch touched)."""
    from gobpfld_amd.emulator import VM as _VM
    live = LIVE_MAX - room
    vm = _VM(Settings(), lib=lib)
    m = vm.add_map(MapDef(MAP_HASH, 4, 8, LIVE_MAX))
    keys = (np.arange(live, dtype=np.uint64) * 2654435761 % (1 << 32)).astype(np.uint32)
    vm.map_update_batch(m, keys.view(np.uint8).reshape(-1, 4), np.full(live, 7, np.uint64).view(np.uint8).reshape(-1, 8))
    vm.set_entrypoint(vm.add_raw_program(prog_learn_u32()))
    rng = np.random.default_rng(5)
    pk = keys[rng.integers(0, live, size=n)]
    new = rng.random(n) < 0.1
    fresh = (np.arange(3 * room, dtype=np.uint32) * 2 + 1)  # odd keys: never in the preload (even multiples)
    fresh = fresh[~np.isin(fresh, keys)]
    pk[new] = fresh[rng.integers(0, len(fresh), size=int(new.sum()))]
    umem, descs = packets(n, 64, seed=3)
    umem.reshape(n, 64)[:, :4] = pk.view(np.uint8).reshape(n, 4)
    r = vm.run_batch(umem, descs)
    touched = np.unique(pk)
    vals = [vm.map_lookup(m, int(k).to_bytes(4, "little")) for k in touched]
    out = (r.results.copy(), vm.map_count(m), vals, r.stats["mode_used"])
    vm.close()
    return out


def _check_live(a, b):
    assert (a[0] == b[0]).all(), "results differ"
    assert a[1] == b[1] == LIVE_MAX, (a[1], b[1])
    assert a[2] == b[2], "entries differ"
    assert (b[0]["r0"] == -7).sum() > 0  # the capacity rule was reached inside the batch


def test_live_4m_entries_hostsim(hostsim_lib, oracle_lib):
    _check_live(_live_case(hostsim_lib), _live_case(oracle_lib))


@pytest.mark.gpu
def test_live_4m_entries_device(gpu_lib, oracle_lib):
    _check_live(_live_case(gpu_lib), _live_case(oracle_lib))
