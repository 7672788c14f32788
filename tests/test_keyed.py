"""Keyed ordered execution (xe_internal.h XE_MODE_SPEC / XE_MODE_CHAIN; xe_runtime.cpp keyed).

Programs that write map entries — an in-program insert (bpf_map_update_elem), a plain store into a map
value, an ARRAY update — are order-dependent: the reference runs the packets one after another
(emulator/vm.go:110-173 per packet, emulator/helper_functions.go:76-101 MapUpdateElement,
emulator/maps_hash.go:65-123 HashMap.Update, emulator/inst_store.go:20-99). Instead of replaying such a
batch on one lane, the device runs it as chains: packets that touch a key some packet writes are
joined per key (connected components), each chain runs in packet order on one lane, everything else in
parallel. The result must equal the oracle's sequential VM bit for bit, and a batch whose packets leave
the schedule the SPEC pass predicted (or whose inserts could hit the map's capacity) must still come out
exact through the one-lane replay.
"""
import numpy as np
import pytest

from gobpfld_amd import workloads as W
from gobpfld_amd.asm import JEQ, JGT, Asm, XDP_DROP, XDP_PASS
from gobpfld_amd.emulator import (MAP_ARRAY, MAP_HASH, MODE_KEYED, MODE_PARALLEL, MODE_SEQUENTIAL, VM, MapDef,
                                  Settings)
from parity import assert_same, config_case, packets, run_one

LSH, OR, AND = 0x60, 0x40, 0x50


def _key_byte(a, dst, byte, mask):
    a.ldx(4, 6, 1, 0).ldx(1, dst, 6, byte).alu64(AND, dst, mask)


def prog_last_len():
    """Preloaded HASH(4 B key = byte 0 & 31 -> {u64 pkts, u64 last}): hit -> pkts += 1 (atomic) and
    last = byte 2 (a plain store: last writer wins, order-dependent)."""
    a = Asm()
    _key_byte(a, 8, 0, 31)
    a.ldx(1, 9, 6, 2)
    a.stx(4, 10, -4, 8).ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.jmp(JEQ, 0, "out", imm=0)
    a.mov64(1, 1).xadd(8, 0, 0, 1)
    a.stx(8, 0, 8, 9)
    a.label("out").mov64(0, XDP_PASS).exit()
    return a.assemble()


def prog_rate_limit():
    """ARRAY(8 x u64) keyed by byte 0 & 7: count < 40 -> count += 1, PASS; else DROP. The loaded count
    decides the verdict, so the update is a true read-modify-write (not lifted)."""
    a = Asm()
    _key_byte(a, 8, 0, 7)
    a.stx(4, 10, -4, 8).ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.jmp(JEQ, 0, "drop", imm=0)
    a.ldx(8, 1, 0, 0)
    a.jmp(JGT, 1, "drop", imm=39)
    a.add64(1, 1).stx(8, 0, 0, 1)
    a.mov64(0, XDP_PASS).exit()
    a.label("drop").mov64(0, XDP_DROP).exit()
    return a.assemble()


def prog_two_keys():
    """HASH(4 B -> u64) learning counters for two keys per packet: (byte 0 & 15) and 16 + (byte 0 & 15).
    A miss inserts 1, a hit adds 1. Each packet joins the chains of both its keys (union-find): 16
    chains of two keys each."""
    a = Asm()
    a.ldx(4, 6, 1, 0)
    for k, (byte, base) in enumerate(((0, 0), (0, 16))):
        a.ldx(1, 8, 6, byte).alu64(AND, 8, 15).add64(8, base)
        a.stx(4, 10, -4, 8).ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
        a.jmp(JEQ, 0, f"ins{k}", imm=0)
        a.mov64(1, 1).xadd(8, 0, 0, 1).ja(f"next{k}")
        a.label(f"ins{k}")
        a.st(8, 10, -16, 1)
        a.ld_map(1, 1).mov64(2, src=10).add64(2, -4).mov64(3, src=10).add64(3, -16).mov64(4, 0).call(2)
        a.label(f"next{k}")
    a.mov64(0, XDP_PASS).exit()
    return a.assemble()


def prog_escape():
    """HASH(4 B -> u64) keyed by byte 0 & 7: miss -> insert, then look the key up again; found -> ARRAY
    map 2 element 5 := 1 (a store through the looked-up value). The SPEC pass holds the insert back, so its second lookup
    misses and it never predicts the ARRAY write: the chain pass must notice and replay in order."""
    a = Asm()
    _key_byte(a, 8, 0, 7)
    a.stx(4, 10, -4, 8).ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.jmp(JEQ, 0, "ins", imm=0)
    a.ja("out")
    a.label("ins")
    a.st(8, 10, -16, 7)
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -4).mov64(3, src=10).add64(3, -16).mov64(4, 0).call(2)
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.jmp(JEQ, 0, "out", imm=0)
    a.st(4, 10, -8, 5)
    a.ld_map(1, 2).mov64(2, src=10).add64(2, -8).call(1)
    a.jmp(JEQ, 0, "out", imm=0)
    a.st(8, 0, 0, 1)                        # *(u64 *)&array[5] = 1: a write nothing predicted
    a.label("out").mov64(0, XDP_PASS).exit()
    return a.assemble()


def prog_first_seen():
    """HASH(4 B -> u64): key A = byte 0 & 7; on a miss insert A and a second key B = 100 + (byte 0 & 63)
    (8 Bs per A: 8 chains). The SPEC pass sees every A absent, so it reserves every B; in packet order
    only the first packet of each A inserts its B. The unused reservations stay behind as tombstones."""
    a = Asm()
    _key_byte(a, 8, 0, 7)
    a.ldx(1, 9, 6, 0).alu64(AND, 9, 63).add64(9, 100)
    a.stx(4, 10, -4, 8).ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.jmp(JEQ, 0, "ins", imm=0)
    a.mov64(1, 1).xadd(8, 0, 0, 1).ja("out")
    a.label("ins")
    a.st(8, 10, -16, 1)
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -4).mov64(3, src=10).add64(3, -16).mov64(4, 0).call(2)
    a.stx(4, 10, -8, 9)
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -8).mov64(3, src=10).add64(3, -16).mov64(4, 0).call(2)
    a.label("out").mov64(0, XDP_PASS).exit()
    return a.assemble()


def prog_many_keys():
    """ARRAY(16384 x u64): element (bytes 0-1 & 0x3fff) := byte 2 (a plain store). Thousands of distinct
    written keys: more than the first keyed batch's D table holds, so the path retries with room for
    one key per packet."""
    a = Asm()
    a.ldx(4, 6, 1, 0).ldx(2, 8, 6, 0).alu64(AND, 8, 0x3FFF).ldx(1, 9, 6, 2)
    a.stx(4, 10, -4, 8).ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.jmp(JEQ, 0, "out", imm=0)
    a.stx(8, 0, 0, 9)
    a.label("out").mov64(0, XDP_PASS).exit()
    return a.assemble()


def prog_learn_in_call():
    """prog_two_keys' learning step for key (byte 0 & 15) inside a bpf-to-bpf call (the general lane
    model, emulator/inst_call_bpf.go:18-44), and the packet's byte 3 := 0x5a (a packet write)."""
    a = Asm()
    a.ldx(4, 6, 1, 0)
    a.mov64(2, 0x5A).stx(1, 6, 3, 2)
    a.ldx(1, 8, 6, 0).alu64(AND, 8, 15)
    a.stx(4, 10, -4, 8)
    a.mov64(1, src=10).add64(1, -4)
    a.call_bpf("learn")
    a.mov64(0, XDP_PASS).exit()
    a.label("learn")                        # r1 = key pointer (caller's frame)
    a.mov64(6, src=1)
    a.ld_map(1, 1).mov64(2, src=6).call(1)
    a.jmp(JEQ, 0, "ins", imm=0)
    a.mov64(1, 1).xadd(8, 0, 0, 1).mov64(0, 0).exit()
    a.label("ins")
    a.st(8, 10, -8, 1)
    a.ld_map(1, 1).mov64(2, src=6).mov64(3, src=10).add64(3, -8).mov64(4, 0).call(2)
    a.mov64(0, 0).exit()
    return a.assemble()


def _last_len_maps():
    entries = {0: [(np.uint32(k).tobytes(), bytes(16)) for k in range(0, 32, 2)]}  # even keys preloaded
    return [(MapDef(MAP_HASH, 4, 16, 64), None)], entries


CASES = {
    "last_len": lambda: (prog_last_len(), *_last_len_maps()),
    "rate_limit": lambda: (prog_rate_limit(), [(MapDef(MAP_ARRAY, 4, 8, 8), None)], None),
    "two_keys": lambda: (prog_two_keys(), [(MapDef(MAP_HASH, 4, 8, 64), None)], None),
}


def _check(lib_a, oracle_lib, prog, maps, entries, umem, descs, want_mode, what, settings=None):
    a = run_one(lib_a, prog, maps, umem, descs, entries=entries, regs=False, settings=settings)
    b = run_one(oracle_lib, prog, maps, umem, descs, entries=entries, regs=False)
    assert_same(a, b, what)
    assert a[0].stats["mode_used"] == want_mode, (what, a[0].stats)
    return a


@pytest.mark.parametrize("case", sorted(CASES))
def test_keyed_hostsim(oracle_lib, hostsim_lib, case):
    prog, maps, entries = CASES[case]()
    umem, descs = packets(3000, 64, seed=21)
    _check(hostsim_lib, oracle_lib, prog, maps, entries, umem, descs, MODE_KEYED, case)


def test_keyed_d_table_retry_hostsim(oracle_lib, hostsim_lib):
    umem, descs = packets(12000, 64, seed=25)
    _check(hostsim_lib, oracle_lib, prog_many_keys(), [(MapDef(MAP_ARRAY, 4, 8, 16384), None)], None, umem, descs,
           MODE_KEYED, "many_keys")


def test_keyed_hot_key_replays_hostsim(oracle_lib, hostsim_lib):
    """Every packet reads and writes one ARRAY element: one chain of the whole batch, which goes to the
    staged one-lane replay instead (exact either way)."""
    umem, descs = packets(3000, 64, seed=27, fill=3)  # byte 0 & 7 = 3 for every packet
    _check(hostsim_lib, oracle_lib, prog_rate_limit(), [(MapDef(MAP_ARRAY, 4, 8, 8), None)], None, umem, descs,
           MODE_SEQUENTIAL, "hot key")


def test_keyed_call_and_packet_write_hostsim(oracle_lib, hostsim_lib):
    umem, descs = packets(2500, 64, seed=28)
    _check(hostsim_lib, oracle_lib, prog_learn_in_call(), [(MapDef(MAP_HASH, 4, 8, 64), None)], None, umem, descs,
           MODE_KEYED, "call + packet write")


@pytest.mark.parametrize("case", ["last_len", "two_keys"])
def test_keyed_register_records_hostsim(oracle_lib, hostsim_lib, case):
    """With R0-R9 records requested (no read-modify-write lifting), every chain packet's record too."""
    prog, maps, entries = CASES[case]()
    umem, descs = packets(2000, 64, seed=29)
    a = run_one(hostsim_lib, prog, maps, umem, descs, entries=entries, regs=True)
    b = run_one(oracle_lib, prog, maps, umem, descs, entries=entries, regs=True)
    assert_same(a, b, case)
    assert a[0].stats["mode_used"] == MODE_KEYED


def test_keyed_escape_hostsim(oracle_lib, hostsim_lib):
    umem, descs = packets(2000, 64, seed=22)
    maps = [(MapDef(MAP_HASH, 4, 8, 64), None), (MapDef(MAP_ARRAY, 4, 8, 8), None)]
    _check(hostsim_lib, oracle_lib, prog_escape(), maps, None, umem, descs, MODE_SEQUENTIAL, "escape")


def test_keyed_root_cycle_replays_hostsim(oracle_lib, hostsim_lib, monkeypatch):
    """A D table whose parents form a cycle (injected after the D step: XE_HOSTSIM_DCYCLE, host-simulation
    build only) must not give chains from a partial root: keyed_root flags it and the batch replays in
    order, exact."""
    monkeypatch.setenv("XE_HOSTSIM_DCYCLE", "1")
    prog, maps, entries = CASES["two_keys"]()
    umem, descs = packets(3000, 64, seed=21)
    _check(hostsim_lib, oracle_lib, prog, maps, entries, umem, descs, MODE_SEQUENTIAL, "root cycle")


def test_c3learn_hostsim(oracle_lib, hostsim_lib):
    prog, maps, entries, umem, descs = config_case("c3learn", 8192, flows_cap=4096)
    _check(hostsim_lib, oracle_lib, prog, maps, entries, umem, descs, MODE_KEYED, "c3learn")


def test_c3learn_capacity_hostsim(oracle_lib, hostsim_lib):
    """Inserts that can reach max_entries depend on packet order: the one-lane replay, still exact
    (some learning updates fail with E2BIG exactly where the reference's do)."""
    prog, _, entries, umem, descs = config_case("c3learn", 4096, flows_cap=512)
    maps = [(MapDef(MAP_HASH, 16, 16, 600), None)]
    a = _check(hostsim_lib, oracle_lib, prog, maps, entries, umem, descs, MODE_SEQUENTIAL, "capacity")
    assert len(a[1][0][0]) == 600


def _batches(lib, prog, maps, entries, batches, settings=None):
    vm = VM(settings or Settings(), lib=lib)
    idx = []
    for i, (mdef, init) in enumerate(maps):
        m = vm.add_map(mdef, init)
        idx.append(m)
        for k, v in (entries or {}).get(i, []):
            vm.map_update(m, k, v)
    vm.set_entrypoint(vm.add_raw_program(prog))
    out = []
    for umem, descs in batches:
        mem = umem.copy()
        r = vm.run_batch(mem, descs)
        out.append((r.results.copy(), r.verdicts.copy(), r.stats["mode_used"]))
    dumps = [vm.map_dump(m) for m in idx]
    vm.close()
    return out, dumps


def _tombstones(lib, oracle_lib, n):
    """Batch, host lookups / dump (the host mirror drops the tombstones and re-uploads), batch again."""
    prog = prog_first_seen()
    out = []
    for L in (lib, oracle_lib):
        vm = VM(Settings(), lib=L)
        m = vm.add_map(MapDef(MAP_HASH, 4, 8, 256))
        vm.set_entrypoint(vm.add_raw_program(prog))
        res = []
        for seed in (31, 32):
            umem, descs = packets(n, 64, seed=seed)
            r = vm.run_batch(umem, descs)
            res.append((r.results.copy(), r.stats["mode_used"]))
            keys, vals = vm.map_dump(m)
            look = [vm.map_lookup(m, np.uint32(k).tobytes()) for k in (0, 3, 100, 150, 163, 99)]
            res.append((keys.copy(), vals.copy(), look))
        vm.close()
        out.append(res)
    a, b = out
    assert a[0][1] == MODE_KEYED and a[2][1] == MODE_PARALLEL  # batch 2: every A is known, nothing is written
    for x, y in zip(a, b):
        for u, v in zip(x, y):
            if isinstance(u, np.ndarray):
                assert np.array_equal(u, v)
            elif isinstance(u, list):
                assert [None if q is None else bytes(q) for q in u] == [None if q is None else bytes(q) for q in v]


def test_keyed_tombstones_hostsim(oracle_lib, hostsim_lib):
    _tombstones(hostsim_lib, oracle_lib, 2000)


def test_keyed_batches_hostsim(oracle_lib, hostsim_lib):
    """Consecutive learning batches: the second and third start straight from the SPEC pass (the VM
    remembers that its last batch wrote map entries); the map state carries over exactly."""
    prog, maps, entries, _, _ = config_case("c3learn", 16, flows_cap=2048)
    batches = [W.build_batch("c3learn", k * 3000, 3000) for k in range(3)]
    a, da = _batches(hostsim_lib, prog, maps, entries, batches)
    b, db = _batches(oracle_lib, prog, maps, entries, batches)
    for k, ((ra, va, mode), (rb, vb, _)) in enumerate(zip(a, b)):
        assert np.array_equal(ra, rb) and np.array_equal(va, vb), k
        assert mode == MODE_KEYED, (k, mode)
    assert np.array_equal(da[0][0], db[0][0]) and np.array_equal(da[0][1], db[0][1])


# ------------------------------------------------------------------ MI355X
@pytest.mark.gpu
@pytest.mark.parametrize("engine", [1, 2], ids=["interp", "jit"])
@pytest.mark.parametrize("case", sorted(CASES))
def test_keyed_device(gpu_lib, oracle_lib, case, engine):
    prog, maps, entries = CASES[case]()
    umem, descs = packets(100000, 64, seed=23)
    _check(gpu_lib, oracle_lib, prog, maps, entries, umem, descs, MODE_KEYED, case, Settings(engine=engine))


@pytest.mark.gpu
@pytest.mark.parametrize("engine", [1, 2], ids=["interp", "jit"])
def test_keyed_escape_device(gpu_lib, oracle_lib, engine):
    umem, descs = packets(20000, 64, seed=24)
    maps = [(MapDef(MAP_HASH, 4, 8, 64), None), (MapDef(MAP_ARRAY, 4, 8, 8), None)]
    _check(gpu_lib, oracle_lib, prog_escape(), maps, None, umem, descs, MODE_SEQUENTIAL, "escape", Settings(engine=engine))


@pytest.mark.gpu
@pytest.mark.parametrize("engine", [1, 2], ids=["interp", "jit"])
def test_c3learn_device(gpu_lib, oracle_lib, engine):
    prog, maps, entries, umem, descs = config_case("c3learn", 1 << 18)
    _check(gpu_lib, oracle_lib, prog, maps, entries, umem, descs, MODE_KEYED, "c3learn", Settings(engine=engine))


@pytest.mark.gpu
def test_c3learn_capacity_device(gpu_lib, oracle_lib):
    prog, _, entries, umem, descs = config_case("c3learn", 20000, flows_cap=2048)
    maps = [(MapDef(MAP_HASH, 16, 16, 2300), None)]
    _check(gpu_lib, oracle_lib, prog, maps, entries, umem, descs, MODE_SEQUENTIAL, "capacity")


@pytest.mark.gpu
def test_keyed_batches_device(gpu_lib, oracle_lib):
    prog, maps, entries, _, _ = config_case("c3learn", 16)
    batches = [W.build_batch("c3learn", k * 100000, 100000) for k in range(3)]
    a, da = _batches(gpu_lib, prog, maps, entries, batches)
    b, db = _batches(oracle_lib, prog, maps, entries, batches)
    for k, ((ra, va, mode), (rb, vb, _)) in enumerate(zip(a, b)):
        assert np.array_equal(ra, rb) and np.array_equal(va, vb), k
        assert mode == MODE_KEYED, (k, mode)
    assert np.array_equal(da[0][0], db[0][0]) and np.array_equal(da[0][1], db[0][1])


@pytest.mark.gpu
def test_keyed_tombstones_device(gpu_lib, oracle_lib):
    _tombstones(gpu_lib, oracle_lib, 50000)


@pytest.mark.gpu
def test_keyed_d_table_retry_device(gpu_lib, oracle_lib):
    umem, descs = packets(60000, 64, seed=26)
    _check(gpu_lib, oracle_lib, prog_many_keys(), [(MapDef(MAP_ARRAY, 4, 8, 16384), None)], None, umem, descs,
           MODE_KEYED, "many_keys")


@pytest.mark.gpu
@pytest.mark.parametrize("engine", [1, 0], ids=["interp", "auto"])
def test_keyed_call_and_packet_write_device(gpu_lib, oracle_lib, engine):
    umem, descs = packets(50000, 64, seed=30)
    _check(gpu_lib, oracle_lib, prog_learn_in_call(), [(MapDef(MAP_HASH, 4, 8, 64), None)], None, umem, descs,
           MODE_KEYED, "call + packet write", Settings(engine=engine))


@pytest.mark.gpu
@pytest.mark.parametrize("engine", [1, 2], ids=["interp", "jit"])
@pytest.mark.parametrize("case", ["last_len", "two_keys"])
def test_keyed_register_records_device(gpu_lib, oracle_lib, case, engine):
    prog, maps, entries = CASES[case]()
    umem, descs = packets(40000, 64, seed=31)
    a = run_one(gpu_lib, prog, maps, umem, descs, entries=entries, regs=True, settings=Settings(engine=engine))
    b = run_one(oracle_lib, prog, maps, umem, descs, entries=entries, regs=True)
    assert_same(a, b, case)
    assert a[0].stats["mode_used"] == MODE_KEYED
