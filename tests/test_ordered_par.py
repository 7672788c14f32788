"""Ordered maps in parallel: QUEUE / STACK pushes and PERF_EVENT_ARRAY outputs run in parallel lanes and
are put into packet order afterwards (xe_interp.h list_push_par, xe_runtime.cpp ordered_finalize); LRU_HASH
lookups record each value's last touch and the UsageList is rebuilt from it (xe_runtime.cpp lru_finalize:
in the reference every Lookup promotes, emulator/maps_hash_lru.go:51-91, so the final list is the touched
keys by last touch, ahead of the untouched ones in their old order).

The reference appends in its packet-by-packet loop (emulator/vm.go:110-173): QueueMap/StackMap.Push
(emulator/maps_queue.go:60-77, maps_stack.go:60-77) and PerfEventArray.Push
(emulator/maps_perf_event_array.go:101-115) are unbounded Go appends, so a batch of appends commutes up
to the order of the list — which is packet order, and call order within a packet. Every case runs
against the oracle's single VM (results, register records, the lists in order) and must report
mode_used PARALLEL; a batch that also pops replays in order (mode SEQUENTIAL) and still matches."""
import numpy as np
import pytest

from gobpfld_amd.asm import JEQ, JGT, JNE, Asm
from gobpfld_amd.emulator import (MAP_LRU_HASH, MAP_PERF_EVENT_ARRAY, MAP_QUEUE, MAP_STACK, MODE_KEYED, MODE_PARALLEL,
                                  MODE_SEGMENTS, MODE_SEQUENTIAL, MapDef)
from parity import assert_same, packets, run_one


def _head(a, need):
    a.ldx(4, 6, 1, 0).ldx(4, 7, 1, 4)
    a.mov64(2, src=6).add64(2, need)
    a.jmp(JGT, 2, "out", src=7)


def prog_push(pop=False):
    """push u64 packet[0:8]; when packet[8] is odd also push packet[8:16]; pop: when packet[9] == 0
    pop one element first (order-dependent)."""
    a = Asm()
    _head(a, 16)
    if pop:
        a.ldx(1, 4, 6, 9).jmp(JNE, 4, "nopop", imm=0)
        a.ld_map(1, 1).mov64(2, src=10).add64(2, -24).call(88)
        a.label("nopop")
    a.ldx(8, 3, 6, 0).stx(8, 10, -8, 3)
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -8).mov64(3, 0).call(87)
    a.ldx(1, 4, 6, 8).alu64(0x50, 4, 1)          # r4 &= 1 (AND)
    a.jmp(JEQ, 4, "out", imm=0)
    a.ldx(8, 3, 6, 8).stx(8, 10, -16, 3)
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -16).mov64(3, 0).call(87)
    a.label("out").mov64(0, 2).exit()
    return a.assemble()


def prog_perf():
    """output packet[0 : 1 + packet[10] % 16] as an event; when packet[11] % 4 == 0 output packet[16:24]
    as a second one."""
    a = Asm()
    _head(a, 32)
    a.ldx(1, 5, 6, 10).alu64(0x50, 5, 15).add64(5, 1)
    a.ld_map(2, 1).mov64(4, src=6).mov64(3, 0).call(25)
    a.ldx(1, 4, 6, 11).alu64(0x50, 4, 3)
    a.jmp(JNE, 4, "out", imm=0)
    a.ld_map(2, 1).mov64(4, src=6).add64(4, 16).mov64(5, 8).mov64(3, 0).call(25)
    a.label("out").mov64(0, 2).exit()
    return a.assemble()


def prog_lru(update=False):
    """key = packet[0] % 64: look it up in an LRU_HASH (a hit promotes it) and add 1 to the value;
    update: a miss inserts the key (an order-dependent write: eviction order)."""
    a = Asm()
    _head(a, 16)
    a.ldx(1, 3, 6, 0).alu64(0x50, 3, 63).stx(4, 10, -4, 3)
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.jmp(JEQ, 0, "miss", imm=0)
    a.mov64(1, 1).xadd(8, 0, 0, 1)
    a.ja("out")
    a.label("miss")
    if update:
        a.st(8, 10, -16, 7).ld_map(1, 1).mov64(2, src=10).add64(2, -4).mov64(3, src=10).add64(3, -16)
        a.mov64(4, 0).call(2)
    a.label("out").mov64(0, 2).exit()
    return a.assemble()


def prog_lru_queue():
    """LRU learning as prog_lru(update=True), and every packet also pushes its first byte onto a QUEUE
    (map 2): appends from both keyed passes, put in packet order afterwards."""
    a = Asm()
    _head(a, 16)
    a.ldx(1, 3, 6, 0).stx(8, 10, -24, 3)
    a.ld_map(1, 2).mov64(2, src=10).add64(2, -24).mov64(3, 0).call(87)
    a.ldx(1, 3, 6, 0).alu64(0x50, 3, 63).stx(4, 10, -4, 3)
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.jmp(JEQ, 0, "miss", imm=0)
    a.mov64(1, 1).xadd(8, 0, 0, 1)
    a.ja("out")
    a.label("miss")
    a.st(8, 10, -16, 7).ld_map(1, 1).mov64(2, src=10).add64(2, -4).mov64(3, src=10).add64(3, -16)
    a.mov64(4, 0).call(2)
    a.label("out").mov64(0, 2).exit()
    return a.assemble()


def prog_consume(push=True, peek=None, two_pops=False):
    """A work queue: when packet[9] is even pop one element (the count pass ranks the pops in packet
    order); a popped element's value (or 7 when the list was empty) goes into R8 and the verdict; push:
    then push packet[0:8]; peek "first" / "after": peek at the front (helper 89) before the pop (the
    count pass then cannot rank the pops: in order) or after it, and add the value; two_pops: pop twice
    (the second pop replays the batch in order)."""
    a = Asm()
    _head(a, 16)
    a.mov64(8, 7)

    def do_peek(tag):
        a.ld_map(1, 1).mov64(2, src=10).add64(2, -32).call(89)
        a.jmp(JNE, 0, "nopeek" + tag, imm=0)
        a.ldx(8, 5, 2, 0).alu64(0x00, 8, src=5)
        a.label("nopeek" + tag)

    if peek == "first":
        do_peek("0")
    a.ldx(1, 4, 6, 9).alu64(0x50, 4, 1).jmp(JNE, 4, "nopop", imm=0)
    for k in range(2 if two_pops else 1):
        a.ld_map(1, 1).mov64(2, src=10).add64(2, -24).call(88)
    a.ldx(8, 3, 10, -24)
    a.jmp(JEQ, 3, "nopop", imm=0)                # IMM 0: the list was empty (a pointer never equals 0)
    a.ldx(8, 4, 3, 0).alu64(0x00, 8, src=4)      # r8 += element value
    a.label("nopop")
    if peek == "after":
        do_peek("1")
    if push:
        a.ldx(8, 3, 6, 0).stx(8, 10, -8, 3)
        a.ld_map(1, 1).mov64(2, src=10).add64(2, -8).mov64(3, 0).call(87)
    a.label("out").mov64(0, src=8).alu64(0x50, 0, 3).exit()   # verdict = r8 & 3
    return a.assemble()


def prog_two_lists():
    """Pops from two lists in one batch (round 6: a rank slot per list): when packet[9] is even pop the
    QUEUE (map 1), when packet[10] is even pop the STACK (map 2); the popped values (or 7 for an empty
    list) go into R8 and the verdict."""
    a = Asm()
    _head(a, 16)
    a.mov64(8, 7)
    for m, byte, tag in ((1, 9, "q"), (2, 10, "s")):
        a.ldx(1, 4, 6, byte).alu64(0x50, 4, 1).jmp(JNE, 4, "no" + tag, imm=0)
        a.st(8, 10, -24, 0)
        a.ld_map(1, m).mov64(2, src=10).add64(2, -24).call(88)
        a.ldx(8, 3, 10, -24)
        a.jmp(JEQ, 3, "no" + tag, imm=0)
        a.ldx(8, 5, 3, 0).alu64(0x00, 8, src=5)
        a.label("no" + tag)
    a.label("out").mov64(0, src=8).alu64(0x50, 0, 3).exit()   # (_head jumps to "out" for a short packet)
    return a.assemble()


def prog_peek():
    """Reads only: peek at the front and look up element packet[1] % 64 by index (helper 1 on a queue);
    then push packet[0:8] — the reads sit inside the start contents, so the pushes do not move them."""
    a = Asm()
    _head(a, 16)
    a.mov64(8, 0)
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -32).call(89)
    a.jmp(JNE, 0, "nopeek", imm=0)
    a.ldx(8, 8, 2, 0)
    a.label("nopeek")
    a.ldx(1, 3, 6, 1).alu64(0x50, 3, 63).stx(4, 10, -4, 3)
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.jmp(JEQ, 0, "push", imm=0)
    a.ldx(8, 4, 0, 0).alu64(0x00, 8, src=4)
    a.label("push")
    a.ldx(8, 3, 6, 0).stx(8, 10, -16, 3)
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -16).mov64(3, 0).call(87)
    a.label("out").mov64(0, src=8).alu64(0x50, 0, 3).exit()
    return a.assemble()


LRU = (MapDef(MAP_LRU_HASH, 4, 8, 64), None)
LRU_ROOMY = (MapDef(MAP_LRU_HASH, 4, 8, 128), None)  # every key of the stream fits: no eviction
LRU_PRELOAD = {0: [(k.to_bytes(4, "little"), (1000 * k).to_bytes(8, "little")) for k in range(0, 96, 2)]}
QUEUE = (MapDef(MAP_QUEUE, 0, 8, 16), None)
STACK = (MapDef(MAP_STACK, 0, 8, 16), None)
PERF = (MapDef(MAP_PERF_EVENT_ARRAY, 4, 4, 8), None)
PRELOAD = {0: [(None, (0xAB00 + i).to_bytes(8, "little")) for i in range(3)]}  # userspace pushes first
QUEUE_BIG = (MapDef(MAP_QUEUE, 0, 8, 1 << 20), None)
LISTQ = (MapDef(MAP_QUEUE, 0, 8, 16384), None)
LISTS = (MapDef(MAP_STACK, 0, 8, 16384), None)
LIST_PRELOAD = {0: [(None, (0xC000 + i).to_bytes(8, "little")) for i in range(3072)]}  # more than the pops
LIST_SHORT = {0: [(None, (0xC000 + i).to_bytes(8, "little")) for i in range(40)]}    # fewer than the pops

CASES = {
    "queue": (prog_push, QUEUE, PRELOAD, MODE_PARALLEL),
    "stack": (prog_push, STACK, PRELOAD, MODE_PARALLEL),
    "perf": (prog_perf, PERF, None, MODE_PARALLEL),
    # a rare pop that runs past the 3 preloaded elements after earlier pushes: packet-order segments
    "queue_pop": (lambda: prog_push(pop=True), QUEUE, PRELOAD, MODE_SEGMENTS),
    "lru_lookup": (prog_lru, LRU, LRU_PRELOAD, MODE_PARALLEL),
    "lru_update": (lambda: prog_lru(update=True), LRU, LRU_PRELOAD, MODE_SEQUENTIAL),
    # LRU learning without eviction: the keyed path (misses insert, later packets of the key hit it)
    "lru_learn": (lambda: prog_lru(update=True), LRU_ROOMY, LRU_PRELOAD, MODE_KEYED),
    "lru_learn_queue": (prog_lru_queue, LRU_ROOMY, LRU_PRELOAD, MODE_KEYED),
    # pops / peeks in parallel (xe_interp.h list_pos): the count pass ranks each packet's pop
    "queue_consume": (prog_consume, LISTQ, LIST_PRELOAD, MODE_PARALLEL),
    "queue_consume_peek": (lambda: prog_consume(peek="after"), LISTQ, LIST_PRELOAD, MODE_PARALLEL),
    "stack_consume_peek": (lambda: prog_consume(peek="after", push=False), LISTS, LIST_PRELOAD, MODE_PARALLEL),
    # a peek before the pop: the count pass stops at the peek, the ranked pass finds the pop, and the pass
    # runs again ranked by the pops it observed (round 6)
    "queue_peek_then_pop": (lambda: prog_consume(peek="first"), LISTQ, LIST_PRELOAD, MODE_PARALLEL),
    "stack_consume": (lambda: prog_consume(push=False), LISTS, LIST_PRELOAD, MODE_PARALLEL),
    "queue_drained_no_push": (lambda: prog_consume(push=False), LISTQ, LIST_SHORT, MODE_PARALLEL),
    # two pops in one packet: each packet's pops counted, ranked by the count (round 6)
    "queue_two_pops": (lambda: prog_consume(two_pops=True), LISTQ, LIST_PRELOAD, MODE_PARALLEL),
    # a pop past the start contents after earlier pushes: the packets before the first such pop run in
    # parallel, the rest as a batch of its own that starts with their pushes (packet-order segments, round 6)
    "queue_drained_push": (prog_consume, LISTQ, LIST_SHORT, MODE_SEGMENTS),
    # ... and what must still replay in order: stack pops interleaved with pushes from the first packets on
    "stack_consume_push": (prog_consume, LISTS, LIST_PRELOAD, MODE_SEQUENTIAL),
    "queue_peek_only": (prog_peek, LISTQ, LIST_PRELOAD, MODE_PARALLEL),
    # pops from a queue and a stack in one batch: one rank slot per list (round 6)
    "two_lists_pop": (prog_two_lists, LISTQ, {0: LIST_PRELOAD[0], 1: LIST_PRELOAD[0]}, MODE_PARALLEL),
}


def case_maps(name):
    """The maps a case runs with (its own, and the appends' QUEUE of lru_learn_queue)."""
    extra = {"lru_learn_queue": [QUEUE_BIG], "two_lists_pop": [LISTS]}
    return [CASES[name][1]] + extra.get(name, [])


def _run(lib, name, n, seed=11):
    build, mdef, entries, _ = CASES[name]
    umem, descs = packets(n, 64, seed=seed)
    return run_one(lib, build(), case_maps(name), umem, descs, entries=entries)


@pytest.mark.parametrize("name", sorted(CASES))
def test_appends_hostsim_equal_oracle(oracle_lib, hostsim_lib, name):
    got = _run(hostsim_lib, name, 1024)
    assert_same(got, _run(oracle_lib, name, 1024), name)
    assert got[0].stats["mode_used"] == CASES[name][3]


@pytest.mark.parametrize("name", ["queue", "perf", "lru_learn_queue"])
def test_appends_hostsim_past_device_room(oracle_lib, hostsim_lib, name):
    """More appends than the device room a run starts with (xe_runtime.cpp ord_slack, 4096 elements /
    events): the pass counts every attempted append, ordered_grow resizes the device lists and the pass
    (the parallel one, or the keyed path's SPEC pass) runs once more — still the reference's list, still
    the case's mode."""
    got = _run(hostsim_lib, name, 6144)
    assert_same(got, _run(oracle_lib, name, 6144), name)
    assert got[0].stats["mode_used"] == CASES[name][3]


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_appends_device_equal_oracle(gpu_lib, oracle_lib, name):
    # the list cases pop about every other packet: 4096 packets stay inside their 3072 preloaded elements
    # (2048 where a popping packet pops twice; past the preloaded elements a batch replays in order)
    n = 4096 if name in ("queue_pop", "lru_update") or CASES[name][1] in (LISTQ, LISTS) else 262144
    n = 2048 if name == "queue_two_pops" else n
    got = _run(gpu_lib, name, n)
    assert_same(got, _run(oracle_lib, name, n), name)
    assert got[0].stats["mode_used"] == CASES[name][3]


@pytest.mark.gpu
def test_perf_appends_device_two_batches(gpu_lib, oracle_lib):
    """Two batches into one VM: the second batch's events follow the first's (the parallel order keys
    restart per batch; the list keeps growing past the device room it started with)."""
    from gobpfld_amd.emulator import VM, Settings
    outs = []
    for lib in (gpu_lib, oracle_lib):
        vm = VM(Settings(), lib=lib)
        m = vm.add_map(PERF[0])
        vm.set_entrypoint(vm.add_raw_program(prog_perf()))
        modes = []
        for seed in (3, 4):
            umem, descs = packets(131072, 64, seed=seed)
            r = vm.run_batch(umem, descs)
            modes.append(r.stats["mode_used"])
        outs.append((vm.map_dump(m), modes))
        vm.close()
    (gd, gm), (od, _) = outs
    assert gm == [MODE_PARALLEL, MODE_PARALLEL]
    assert len(gd) == len(od) and gd == od


def _c3lru_run(lib, n, mode=None, name="c3lru", batches=1):
    """C3-LRU (workloads: C3-learn over an LRU_HASH flow table; "c3lrufull": the table full, so learning
    evicts) on one VM over `batches` consecutive batches of n packets: the last batch's results and
    statistics, the table and its UsageList."""
    from gobpfld_amd import workloads as W
    from gobpfld_amd.emulator import VM, Settings
    vm = VM(Settings() if mode is None else Settings(mode=mode), lib=lib)
    W.setup_vm(vm, name)
    for b in range(batches):
        umem, descs = W.build_batch(name, b * n, n)
        r = vm.run_batch(umem, descs)
    k, v = vm.map_dump(1)
    usage = vm.map_lru_order(1)
    vm.close()
    return r, k, v, usage


def _same_c3lru(a, b):
    ra, ka, va, ua = a
    rb, kb, vb, ub = b
    bad = np.nonzero(ra.results != rb.results)[0]
    assert len(bad) == 0, f"{len(bad)} results differ, first at {bad[0] if len(bad) else -1}"
    assert (ra.verdicts == rb.verdicts).all()
    assert np.array_equal(ka, kb) and np.array_equal(va, vb), "LRU flow table differs"
    assert ua == ub, "UsageList differs"
    assert ra.stats["steps"] == rb.stats["steps"]


def test_c3lru_hostsim_keyed_equals_oracle(oracle_lib, hostsim_lib):
    """An LRU flow table that learns (maps_hash_lru.go:93-161): the keyed path's result, UsageList
    included, is the reference's packet-by-packet one."""
    got = _c3lru_run(hostsim_lib, 20000)
    _same_c3lru(got, _c3lru_run(oracle_lib, 20000))
    assert got[0].stats["mode_used"] == MODE_KEYED
    assert len(got[1]) > 65536  # it learned flows


@pytest.mark.gpu
def test_c3lru_device_keyed_equals_oracle(gpu_lib, oracle_lib):
    """C3-LRU at the bench's keyed batch (4,194,304 IMIX packets, ~256K flows learned into a 1M-entry
    LRU_HASH) through the keyed path against one sequential oracle VM: results, verdicts, table, UsageList."""
    n = 4 * 1024 * 1024
    got = _c3lru_run(gpu_lib, n)
    assert got[0].stats["mode_used"] == MODE_KEYED, got[0].stats
    _same_c3lru(got, _c3lru_run(oracle_lib, n))


@pytest.mark.gpu
def test_c3lrufull_device_keyed_equals_oracle(gpu_lib, oracle_lib):
    """C3-LRU-full: a full 1M-entry LRU flow table learning ~205K new flows from 4,194,304 IMIX packets, so
    every learned flow evicts the least recently used entry (maps_hash_lru.go:114-119) — on the keyed path
    with its evictions planned (xe_interp.h keyed_evict_item), against one sequential oracle VM: results,
    verdicts, table and UsageList; then a second batch on the same VM (the steady state)."""
    n = 4 * 1024 * 1024
    got = _c3lru_run(gpu_lib, n, name="c3lrufull")
    assert got[0].stats["mode_used"] == MODE_KEYED, got[0].stats
    assert len(got[1]) == 1 << 20  # still full: every insert evicted one
    _same_c3lru(got, _c3lru_run(oracle_lib, n, name="c3lrufull"))


@pytest.mark.gpu
def test_c3lrufull_two_batches_device(gpu_lib, oracle_lib):
    n = 1 << 20
    got = _c3lru_run(gpu_lib, n, name="c3lrufull", batches=2)
    assert got[0].stats["mode_used"] == MODE_KEYED, got[0].stats
    _same_c3lru(got, _c3lru_run(oracle_lib, n, name="c3lrufull", batches=2))


def _lru_mixed_stream(lib, n=512):
    """Batches that alternate the LRU paths: lookups only (parallel: stamps), learning inserts (keyed
    chains), updates that evict (the one-lane replay: it needs the links rebuilt from the stamps). The
    UsageList and the values after every batch are compared with the oracle's single VM."""
    from gobpfld_amd.emulator import VM, Settings
    vm = VM(Settings(), lib=lib)
    m = vm.add_map(MapDef(MAP_LRU_HASH, 4, 8, 56))  # 48 preloaded: a batch that learns past 8 keys evicts
    for k, v in LRU_PRELOAD[0]:
        vm.map_update(m, k, v)
    progs = {"lookup": vm.add_raw_program(prog_lru()), "learn": vm.add_raw_program(prog_lru(update=True))}
    out = []
    # (after a replay the next 8 batches replay too: the back-off, xe_runtime.cpp kKeyedBackoff)
    for b, kind in enumerate(["lookup", "learn"] + ["lookup"] * 10 + ["learn"] + ["lookup"] * 10):
        umem, descs = packets(n, 64, seed=100 + b)
        vm.set_entrypoint(progs[kind])
        r = vm.run_batch(umem, descs, want_regs=True)
        out.append((r.results.copy(), vm.map_lru_order(m), vm.map_dump(m), r.stats["mode_used"]))
    vm.close()
    return out


def test_lru_stamps_across_paths_hostsim(oracle_lib, hostsim_lib):
    got, want = _lru_mixed_stream(hostsim_lib), _lru_mixed_stream(oracle_lib)
    for b, (g, w) in enumerate(zip(got, want)):
        assert (g[0] == w[0]).all(), f"batch {b}: results"
        assert g[1] == w[1], f"batch {b}: UsageList"
        assert np.array_equal(g[2][0], w[2][0]) and np.array_equal(g[2][1], w[2][1]), f"batch {b}: entries"
    modes = [g[3] for g in got]
    assert modes[0] == MODE_PARALLEL and modes[1] == MODE_SEQUENTIAL and modes[11] == MODE_PARALLEL, modes


@pytest.mark.gpu
def test_lru_stamps_across_paths_device(gpu_lib, oracle_lib):
    got, want = _lru_mixed_stream(gpu_lib, 4096), _lru_mixed_stream(oracle_lib, 4096)
    for b, (g, w) in enumerate(zip(got, want)):
        assert (g[0] == w[0]).all(), f"batch {b}: results"
        assert g[1] == w[1], f"batch {b}: UsageList"
        assert np.array_equal(g[2][0], w[2][0]) and np.array_equal(g[2][1], w[2][1]), f"batch {b}: entries"
