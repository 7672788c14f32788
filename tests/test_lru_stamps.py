"""LRU stamps (xe_interp.h lru_stamp): a value's place in the UsageList as a number — run epoch << 48,
then packet << 16 | touch within a concurrent run, or the one lane's touch counter within an in-order
run. The UsageList the reference keeps (emulator/maps_hash_lru.go:51-68 promote, :93-161 update with
the eviction at :114-119) must come out of them unchanged:

  * across the renumbering the runtime does before the 16-bit epoch wraps (xe_runtime.cpp
    lru_renumber; reached with xe_debug_set_lru_epoch instead of 65,535 runs): batches of lookups
    (concurrent touches), updates of live keys and evicting inserts (the in-order lane) before and
    after it, against the oracle after every batch — on the host simulation and on the MI355X;
  * in a batch of more than 2^24 packets (gpu): packets past 2^24 used to carry into the epoch bits,
    so the next run's touches sorted below them. The expected UsageList is derived from the packets
    (last touch first, untouched keys after in their earlier order)."""
from __future__ import annotations

import numpy as np
import pytest

from gobpfld_amd.emulator import MAP_LRU_HASH, MapDef, Settings

KEYS = 48
MAX_ENTRIES = 40


def _program():
    """packet = [op u32][key u32]: op 0 looks the key up (R0 = value or 0xFFFF), op 1 updates it
    (R0 = the helper's result; a new key past MaxEntries evicts the tail)."""
    from gobpfld_amd.asm import JEQ, JNE, Asm
    a = Asm()
    a.ldx(4, 6, 1, 0)                       # r6 = ctx->data
    a.ldx(4, 7, 6, 0)                       # op
    a.ldx(4, 1, 6, 4).stx(4, 10, -4, 1)     # key -> fp-4
    a.st(4, 10, -8, 7)                      # value 7 -> fp-8
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
    d_desc, _, _ = np_dtypes()
    n = len(keys)
    pk = np.zeros((n, 2), dtype="<u4")
    pk[:, 0] = ops
    pk[:, 1] = keys
    descs = np.zeros(n, dtype=d_desc)
    descs["addr"] = np.arange(n) * 8
    descs["len"] = 8
    return pk.view(np.uint8).reshape(-1).copy(), descs


def _batches(seed=3):
    """lookup-only batches (concurrent touches) and batches with updates / evicting inserts"""
    rng = np.random.default_rng(seed)
    out = []
    for b in range(8):
        n = 300 + 37 * b
        keys = rng.integers(0, KEYS, size=n)
        ops = np.zeros(n, dtype=np.uint32) if b % 3 != 2 else (rng.random(n) < 0.2).astype(np.uint32)
        out.append(_batch(ops, keys))
    return out


def _vm(lib, epoch=None):
    from gobpfld_amd.emulator import VM
    vm = VM(Settings(), lib=lib)
    m = vm.add_map(MapDef(MAP_LRU_HASH, 4, 4, MAX_ENTRIES))
    for k in range(0, KEYS, 2):  # 24 live keys, most recent last
        vm.map_update(m, int(k).to_bytes(4, "little"), int(100 + k).to_bytes(4, "little"))
    vm.set_entrypoint(vm.add_raw_program(_program()))
    if epoch is not None:
        vm.set_lru_epoch(epoch)
    return vm, m


def _run_stream(lib, epoch):
    vm, m = _vm(lib, epoch)
    seen = []
    for umem, descs in _batches():
        r = vm.run_batch(umem, descs)
        seen.append((r.results.copy(), vm.map_lru_order(m), vm.map_dump(m)))
    vm.close()
    return seen


def _compare(got, want):
    for i, ((ra, ua, da), (rb, ub, db)) in enumerate(zip(got, want)):
        assert (ra == rb).all(), f"batch {i}: results differ"
        assert ua == ub, f"batch {i}: UsageList differs"
        assert all(np.array_equal(x, y) for x, y in zip(da, db)), f"batch {i}: entries differ"


@pytest.mark.parametrize("epoch", [0, 0xfffd, 0xffff])
def test_renumber_keeps_usage_list_hostsim(hostsim_lib, oracle_lib, epoch):
    _compare(_run_stream(hostsim_lib, epoch), _run_stream(oracle_lib, None))


@pytest.mark.gpu
@pytest.mark.parametrize("epoch", [0, 0xfffd])
def test_renumber_keeps_usage_list_device(gpu_lib, oracle_lib, epoch):
    _compare(_run_stream(gpu_lib, epoch), _run_stream(oracle_lib, None))


def test_lru_epoch_setter_bounds(hostsim_lib):
    vm, _ = _vm(hostsim_lib)
    with pytest.raises(RuntimeError):
        vm.set_lru_epoch(0x10000)
    vm.close()


def _expected_order(initial, keys_touched):
    """UsageList after lookups of `keys_touched` in order (a hit promotes to the front, misses change
    nothing): the hit keys by their last touch, latest first, then the untouched ones as they were."""
    keys_touched = np.asarray(keys_touched)
    last = {}
    for k in initial:
        idx = np.flatnonzero(keys_touched == k)
        if len(idx):
            last[k] = int(idx[-1])
    return sorted(last, key=lambda k: -last[k]) + [k for k in initial if k not in last]


@pytest.mark.gpu
def test_batch_past_2_24_packets_device(gpu_lib):
    """17,825,792 lookups (2^24 + 2^20): the stamps of packets past 2^24 stay below the next run's."""
    n = (1 << 24) + (1 << 20)
    vm, m = _vm(gpu_lib)
    initial = [int.from_bytes(k, "little") for k in vm.map_lru_order(m)]
    rng = np.random.default_rng(11)
    keys = rng.integers(0, KEYS, size=n).astype(np.uint32)
    keys[(1 << 24):] = keys[(1 << 24):] % 8 * 2  # the tail of the batch ends on live keys 0, 2, .., 14
    umem, descs = _batch(np.zeros(n, dtype=np.uint32), keys)
    r = vm.run_batch(umem, descs)
    assert r.stats["mode_used"] != 2, "expected a concurrent run, not the in-order lane"
    exp1 = _expected_order(initial, keys)
    assert [int.from_bytes(k, "little") for k in vm.map_lru_order(m)] == exp1
    # a short second run: its touches are newer than every touch of the long one
    umem2, descs2 = _batch(np.zeros(2, dtype=np.uint32), np.array([40, 30], dtype=np.uint32))
    vm.run_batch(umem2, descs2)
    assert [int.from_bytes(k, "little") for k in vm.map_lru_order(m)] == _expected_order(exp1, [40, 30])
    vm.close()


def _loop_program():
    """packet = [key_a u32][loops u32][key_b u32]: looks key_a up `loops` times, then key_b once — more
    touches in one packet than a 16-bit touch number holds (the in-order lane's counter has no such limit)"""
    from gobpfld_amd.asm import JEQ, JNE, Asm
    a = Asm()
    a.ldx(4, 6, 1, 0)
    a.ldx(4, 1, 6, 0).stx(4, 10, -4, 1)     # key_a -> fp-4
    a.ldx(4, 1, 6, 8).stx(4, 10, -8, 1)     # key_b -> fp-8
    a.ldx(4, 8, 6, 4)                       # r8 = loops
    a.jmp(JEQ, 8, "last", imm=0)
    a.label("loop")
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.add64(8, -1)
    a.jmp(JNE, 8, "loop", imm=0)
    a.label("last")
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -8).call(1)
    a.mov64(0, 2).exit()
    return a.assemble()


@pytest.mark.parametrize("which", ["hostsim", pytest.param("gpu", marks=pytest.mark.gpu)])
def test_packet_with_70000_touches(request, oracle_lib, which):
    lib = request.getfixturevalue("hostsim_lib" if which == "hostsim" else "gpu_lib")
    prog = _loop_program()
    orders = []
    for L in (lib, oracle_lib):
        from gobpfld_amd.emulator import VM
        vm = VM(Settings(), lib=L)
        m = vm.add_map(MapDef(MAP_LRU_HASH, 4, 4, MAX_ENTRIES))
        for k in range(0, KEYS, 2):
            vm.map_update(m, int(k).to_bytes(4, "little"), int(100 + k).to_bytes(4, "little"))
        vm.set_entrypoint(vm.add_raw_program(prog))
        got = []
        for rows in ([(4, 70000, 6), (8, 0, 10)], [(12, 0, 14)]):  # the second batch: concurrent touches
            pk = np.array(rows, dtype="<u4")
            umem = pk.view(np.uint8).reshape(-1).copy()
            from gobpfld_amd._native import np_dtypes
            descs = np.zeros(len(rows), dtype=np_dtypes()[0])
            descs["addr"] = np.arange(len(rows)) * 12
            descs["len"] = 12
            r = vm.run_batch(umem, descs)
            got.append((r.results.copy(), vm.map_lru_order(m)))
        orders.append(got)
        vm.close()
    (a, b) = orders
    for (ra, ua), (rb, ub) in zip(a, b):
        assert (ra == rb).all()
        assert ua == ub
    assert [int.from_bytes(k, "little") for k in b[0][1]][:3] == [10, 6, 4]


def test_lookups_past_capacity_stay_concurrent_hostsim(hostsim_lib, oracle_lib):
    """A batch that only looks keys up (present and absent ones: 48 keys against MaxEntries 40 and 24
    live) inserts nothing, so the keyed path's capacity bound (live + keys a packet inserts) holds and
    the batch runs concurrently — it used to count every touched key and replay on one lane."""
    rng = np.random.default_rng(5)
    n = 4096
    keys = rng.integers(0, KEYS, size=n).astype(np.uint32)
    umem, descs = _batch(np.zeros(n, dtype=np.uint32), keys)
    out = []
    for lib in (hostsim_lib, oracle_lib):
        vm, m = _vm(lib)
        r = vm.run_batch(umem, descs)
        out.append((r, vm.map_lru_order(m)))
        vm.close()
    (a, ua), (b, ub) = out
    assert (a.results == b.results).all() and ua == ub
    assert a.stats["mode_used"] != 2, a.stats
