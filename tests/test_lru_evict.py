"""LRU evictions in a keyed batch (xe_interp.h keyed_evict_item; reference: emulator/maps_hash_lru.go:93-161,
eviction at :114-119, delete at :163-183).

A learning batch into a full LRU_HASH map evicts: in packet order the j-th insert of a new key past the
map's room deletes the UsageList's tail at that moment. When no packet of the batch touches the E oldest
values of the batch's start, that tail is the j-th oldest of them, so the device runs the batch on the
keyed path (mode KEYED) with those victims; when some packet looks one of them up, or writes it, the
batch must replay in order (mode SEQUENTIAL). Either way results, the UsageList and the entries equal
the oracle's sequential VM."""
from __future__ import annotations

import numpy as np
import pytest

from gobpfld_amd.emulator import MAP_LRU_HASH, MODE_KEYED, MODE_SEQUENTIAL, MapDef, Settings

MAX = 64


def _program():
    """packet = [op u32][key u32]: op 0 looks the key up (R0 = value or 0xFFFF), op 1 updates it to 7
    (R0 = the helper's result)."""
    from gobpfld_amd.asm import JEQ, Asm
    a = Asm()
    a.ldx(4, 6, 1, 0)
    a.ldx(4, 7, 6, 0)
    a.ldx(4, 1, 6, 4).stx(4, 10, -4, 1)
    a.st(4, 10, -8, 7)
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -4)
    a.jmp(JEQ, 7, "lookup", imm=0)
    a.mov64(3, src=10).add64(3, -8).mov64(4, 0).call(2).exit()
    a.label("lookup").call(1)
    a.jmp(JEQ, 0, "miss", imm=0)
    a.ldx(4, 0, 0, 0).exit()
    a.label("miss").mov64(0, 0xFFFF).exit()
    return a.assemble()


def _batch(ops, keys):
    from gobpfld_amd._native import np_dtypes
    n = len(keys)
    pk = np.zeros((n, 2), dtype="<u4")
    pk[:, 0] = ops
    pk[:, 1] = keys
    descs = np.zeros(n, dtype=np_dtypes()[0])
    descs["addr"] = np.arange(n) * 8
    descs["len"] = 8
    return pk.view(np.uint8).reshape(-1).copy(), descs


def _vm_setup(vm, prog, max_entries, live):
    """An LRU_HASH(4, 4, max_entries) holding keys 0..live-1 (key k updated k-th: key 0 is the oldest)
    and `prog` as the entrypoint (tests/kernel_cases.py builds the same VMs' kernels ahead of time)."""
    m = vm.add_map(MapDef(MAP_LRU_HASH, 4, 4, max_entries))
    for k in range(live):
        vm.map_update(m, int(k).to_bytes(4, "little"), int(1000 + k).to_bytes(4, "little"))
    vm.set_entrypoint(vm.add_raw_program(prog))
    return m


def _vm(lib, live):
    from gobpfld_amd.emulator import VM
    vm = VM(Settings(), lib=lib)
    return vm, _vm_setup(vm, _program(), MAX, live)


def _learning_batch(n, seed, touch_oldest=False, live=MAX):
    """Lookups and updates of the newest half of the live keys, and inserts of new keys 1000+ (each new
    key inserted by several packets); with touch_oldest, one packet looks up the oldest key."""
    rng = np.random.default_rng(seed)
    ops = (rng.random(n) < 0.5).astype(np.uint32)
    keys = rng.integers(live // 2, live, size=n).astype(np.uint32)
    new = rng.random(n) < 0.3
    ops[new] = 1
    keys[new] = 1000 + rng.integers(0, max(1, n // 20), size=int(new.sum()))
    if touch_oldest:
        ops[n // 2], keys[n // 2] = 0, 0
    return _batch(ops, keys)


def _run(lib, batches, live=MAX):
    vm, m = _vm(lib, live)
    out = []
    for umem, descs in batches:
        r = vm.run_batch(umem, descs)
        keys, vals = vm.map_dump(m)
        out.append((r.results.copy(), r.stats["mode_used"], vm.map_lru_order(m), bytes(np.asarray(keys)), bytes(np.asarray(vals))))
    vm.close()
    return out


def _check(got, want, modes):
    for i, ((ra, ma, ua, ka, va), (rb, _, ub, kb, vb)) in enumerate(zip(got, want)):
        assert (ra == rb).all(), f"batch {i}: results differ"
        assert ua == ub, f"batch {i}: UsageList differs"
        assert ka == kb and va == vb, f"batch {i}: entries differ"
        if modes[i] is not None:
            assert ma == modes[i], f"batch {i}: mode {ma}, want {modes[i]}"


CASES = {
    # full map, inserts past its room: the oldest values go, in the order of their inserts
    "evicting": (lambda: [_learning_batch(400, 1)], [MODE_KEYED]),
    # two batches in a row on one VM (the second evicts the first's survivors in stamp order)
    "two_batches": (lambda: [_learning_batch(300, 2), _learning_batch(300, 3)], [MODE_KEYED, MODE_KEYED]),
    # a packet looks a victim up: the batch replays in order
    "victim_touched": (lambda: [_learning_batch(400, 4, touch_oldest=True)], [MODE_SEQUENTIAL]),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_lru_evictions_hostsim(hostsim_lib, oracle_lib, case):
    make, modes = CASES[case]
    batches = make()
    _check(_run(hostsim_lib, batches), _run(oracle_lib, batches), modes)


def test_lru_room_then_evictions_hostsim(hostsim_lib, oracle_lib):
    """A map with room for some of the batch's new keys: the first inserts fill it, the rest evict."""
    batches = [_learning_batch(400, 5, live=MAX - 10)]
    _check(_run(hostsim_lib, batches, live=MAX - 10), _run(oracle_lib, batches, live=MAX - 10), [MODE_KEYED])


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(CASES))
def test_lru_evictions_device(gpu_lib, oracle_lib, case):
    make, modes = CASES[case]
    batches = make()
    _check(_run(gpu_lib, batches), _run(oracle_lib, batches), modes)


def _grow_case(lib, max_entries=5000, n=7000):
    """A full LRU map (max_entries live) and a batch of n inserts of new keys on the one-lane path: every
    insert evicts, and the value pool runs out of room past the first few thousand inserts, so the replay
    starts over from its rollback point with a larger pool."""
    from gobpfld_amd.emulator import VM, MODE_SEQUENTIAL
    vm = VM(Settings(mode=MODE_SEQUENTIAL), lib=lib)
    m = vm.add_map(MapDef(MAP_LRU_HASH, 4, 4, max_entries))
    keys = np.arange(max_entries, dtype=np.uint32)
    vm.map_update_batch(m, keys.view(np.uint8).reshape(-1, 4), (keys + 1).view(np.uint8).reshape(-1, 4))
    vm.set_entrypoint(vm.add_raw_program(_program()))
    umem, descs = _batch(np.ones(n, dtype=np.uint32), 100000 + np.arange(n, dtype=np.uint32))
    r = vm.run_batch(umem, descs)
    out = (r.results.copy(), vm.map_lru_order(m), vm.map_count(m))
    vm.close()
    return out


def test_lru_replay_pool_growth_hostsim(hostsim_lib, oracle_lib):
    a, b = _grow_case(hostsim_lib), _grow_case(oracle_lib)
    assert (a[0] == b[0]).all() and a[1] == b[1] and a[2] == b[2] == 5000


@pytest.mark.gpu
def test_lru_replay_pool_growth_device(gpu_lib, oracle_lib):
    a, b = _grow_case(gpu_lib), _grow_case(oracle_lib)
    assert (a[0] == b[0]).all() and a[1] == b[1] and a[2] == b[2] == 5000


def _churn_case(lib, batches=3, n=40000):
    """The one-lane replay's order log (xe_interp.h lru_log_push), in packet order: a small LRU map under
    lookups and updates — touches that outnumber the log's room (16,384 entries for this map) with no
    eviction to clear it (compactions), then evictions that skip the dead entries of values touched again
    since; the log seeded again from the stamps for each batch."""
    from gobpfld_amd.emulator import VM
    vm = VM(Settings(mode=MODE_SEQUENTIAL), lib=lib)
    m = vm.add_map(MapDef(MAP_LRU_HASH, 4, 4, MAX))
    vm.set_entrypoint(vm.add_raw_program(_program()))
    rng = np.random.default_rng(77)
    out = []
    for b in range(batches):
        ops = (rng.random(n) < 0.08).astype(np.uint32)  # few inserts: the pool keeps its first size
        # the first 3/4 of each batch over half the map's room in keys (no evictions: the log fills up
        # and compacts), the rest over four times its room (evictions skip the log's dead entries)
        keys = rng.zipf(1.3, size=n).astype(np.uint32) % (MAX // 2)
        keys[3 * n // 4:] = rng.integers(0, 4 * MAX, size=n - 3 * n // 4)
        r = vm.run_batch(*_batch(ops, keys))
        k, v = vm.map_dump(m)
        out.append((r.results.copy(), r.stats["mode_used"], vm.map_lru_order(m), bytes(np.asarray(k)), bytes(np.asarray(v))))
    vm.close()
    return out


def test_lru_order_log_churn_hostsim(hostsim_lib, oracle_lib):
    _check(_churn_case(hostsim_lib), _churn_case(oracle_lib), [MODE_SEQUENTIAL] * 3)


@pytest.mark.gpu
def test_lru_order_log_churn_device(gpu_lib, oracle_lib):
    _check(_churn_case(gpu_lib), _churn_case(oracle_lib), [MODE_SEQUENTIAL] * 3)


def _program_imm():
    """As _program, plus op 2: an update whose value register is an IMM (r3 = 0). The reference
    (maps_hash_lru.go:113-119, then :134-137) evicts the UsageList's tail of a full map for a new key
    first and only then returns errMapValNoPtr (R0 = -14): the map shrinks by one."""
    from gobpfld_amd.asm import JEQ, Asm
    a = Asm()
    a.ldx(4, 6, 1, 0)
    a.ldx(4, 7, 6, 0)
    a.ldx(4, 1, 6, 4).stx(4, 10, -4, 1)
    a.st(4, 10, -8, 7)
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -4)
    a.jmp(JEQ, 7, "lookup", imm=0)
    a.jmp(JEQ, 7, "immval", imm=2)
    a.mov64(3, src=10).add64(3, -8).mov64(4, 0).call(2).exit()
    a.label("immval").mov64(3, 0).mov64(4, 0).call(2).exit()
    a.label("lookup").call(1)
    a.jmp(JEQ, 0, "miss", imm=0)
    a.ldx(4, 0, 0, 0).exit()
    a.label("miss").mov64(0, 0xFFFF).exit()
    return a.assemble()


def _imm_case(lib, max_entries, n, seed, mix=False, settings=None):
    """A full LRU map (max_entries live keys), a batch of lookups of existing keys and one update of a new
    key with an IMM value register; with mix, some pointer-valued updates of live keys as well."""
    from gobpfld_amd.emulator import VM
    vm = VM(settings or Settings(), lib=lib)
    m = _vm_setup(vm, _program_imm(), max_entries, max_entries)
    rng = np.random.default_rng(seed)
    ops = np.zeros(n, dtype=np.uint32)
    keys = rng.integers(max_entries // 2, max_entries, size=n).astype(np.uint32)
    if mix:
        upd = rng.random(n) < 0.2
        ops[upd] = 1
    ops[n // 3], keys[n // 3] = 2, 5000 + seed
    out = []
    for _ in range(2):  # a second batch on the same VM sees the first's final map
        r = vm.run_batch(*_batch(ops, keys))
        k, v = vm.map_dump(m)
        out.append((r.results.copy(), r.stats["mode_used"], vm.map_lru_order(m), bytes(np.asarray(k)), bytes(np.asarray(v))))
    count = vm.map_count(m)
    vm.close()
    return out, count


IMM_CASES = {"full8": (8, 64, 1, False), "full64": (64, 400, 2, False), "full64_mixed": (64, 400, 3, True)}


@pytest.mark.parametrize("case", sorted(IMM_CASES))
def test_lru_imm_value_update_evicts_hostsim(hostsim_lib, oracle_lib, case):
    mx, n, seed, mix = IMM_CASES[case]
    (got, gc), (want, wc) = _imm_case(hostsim_lib, mx, n, seed, mix), _imm_case(oracle_lib, mx, n, seed, mix)
    assert wc == mx - 1  # the first batch evicts one value and inserts none; the second finds room
    _check(got, want, [None, None])
    assert gc == wc


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(IMM_CASES))
def test_lru_imm_value_update_evicts_device(gpu_lib, oracle_lib, case):
    mx, n, seed, mix = IMM_CASES[case]
    (got, gc), (want, wc) = _imm_case(gpu_lib, mx, n, seed, mix), _imm_case(oracle_lib, mx, n, seed, mix)
    assert wc == mx - 1
    _check(got, want, [None, None])
    assert gc == wc


def _reuse_case(lib, batches=3, n=20000):
    """A full LRU_HASH(4, 4, 64) on the one-lane path and batches that each insert n new keys: every
    insert evicts. The replay hands an evicted value id to a later packet's insert (xe_interp.h
    lru_free_push / lru_free_pop), so the value pool keeps its size over the stream; before, every insert
    took a fresh id and the pool grew (by rebuilds with 4x the room) towards the ids value handles can
    name. Results, UsageList and entries equal the oracle's after every batch."""
    from gobpfld_amd.emulator import VM
    vm = VM(Settings(mode=MODE_SEQUENTIAL), lib=lib)
    m = _vm_setup(vm, _program(), MAX, MAX)
    out, sizes = [], []
    for b in range(batches):
        ops = np.ones(n, dtype=np.uint32)
        keys = (100000 + b * n + np.arange(n)).astype(np.uint32)
        keys[::7] = keys[::7] - 3  # some keys inserted again a few packets later (a fresh insert: evicted since)
        r = vm.run_batch(*_batch(ops, keys))
        k, v = vm.map_dump(m)
        out.append((r.results.copy(), r.stats["mode_used"], vm.map_lru_order(m), bytes(np.asarray(k)), bytes(np.asarray(v))))
        sizes.append(vm.map_pool(m) if lib.has("debug_map_pool") else None)
    vm.close()
    return out, sizes


def test_lru_replay_reuses_evicted_ids_hostsim(hostsim_lib, oracle_lib):
    (got, sizes), (want, _) = _reuse_case(hostsim_lib), _reuse_case(oracle_lib)
    _check(got, want, [MODE_SEQUENTIAL] * 3)
    assert len({r for r, _ in sizes}) == 1 and sizes[-1][1] < 2 * MAX + 16, sizes  # no growth, ids reused


@pytest.mark.gpu
def test_lru_replay_reuses_evicted_ids_device(gpu_lib, oracle_lib):
    (got, sizes), (want, _) = _reuse_case(gpu_lib), _reuse_case(oracle_lib)
    _check(got, want, [MODE_SEQUENTIAL] * 3)
    assert len({r for r, _ in sizes}) == 1 and sizes[-1][1] < 2 * MAX + 16, sizes
