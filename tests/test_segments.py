"""Packet-order segments (xe_runtime.cpp run_segments, XE_MODE_SEGMENTS): a batch whose only order
dependence is a QUEUE / STACK position that may have depended on a push of an earlier packet (a pop past
the start contents after pushes) runs its packets before the first such position in parallel, exactly,
and the rest as a batch of its own whose start contents hold their pushes — cut again where needed.

In the reference the batch is one packet-by-packet loop (emulator/vm.go:110-173) over QueueMap.Push /
Pop (emulator/maps_queue.go:60-91) and StackMap (maps_stack.go:60-90); segments are that loop's order
kept at the cuts, so every observable must equal the oracle's single VM: results, register records,
verdicts, the lists in order, LRU entries and UsageList, over streams of batches on one VM."""
import numpy as np
import pytest

from gobpfld_amd.asm import JEQ, JGT, JNE, Asm
from gobpfld_amd.emulator import MAP_LRU_HASH, MAP_QUEUE, MAP_STACK, MODE_SEGMENTS, MODE_SEQUENTIAL, MapDef, Settings
from parity import assert_same, packets
from test_fuzz_ordered import run_stream

SHORT = [(None, (0xC000 + i).to_bytes(8, "little")) for i in range(40)]  # fewer than a batch's pops
LRU_PRE = [(k.to_bytes(4, "little"), (1000 * k).to_bytes(8, "little")) for k in range(0, 96, 2)]


def prog_work_queue(lru: bool, pop_mod: int = 2, pushes: int = 1, key_from_pop: bool = False):
    """A work queue (map 2) beside an optional LRU_HASH flow table (map 1): lru: look packet[0] % 64 up
    (a hit promotes it and adds 1 to its value); when packet[9] % pop_mod == 0 pop the queue (the popped
    value, or 7 when it was empty, goes into R8 and the verdict); then push packet[0:8] `pushes` times.
    key_from_pop: the popped value % 64 is also looked up in the LRU map (a promotion that depends on what
    the pop returned: a pass that got a position wrong touched other keys, which the cut must undo)."""
    a = Asm()
    a.ldx(4, 6, 1, 0).ldx(4, 7, 1, 4)
    a.mov64(2, src=6).add64(2, 16)
    a.jmp(JGT, 2, "out", src=7)  # shorter than 16 bytes
    a.mov64(8, 7)
    if lru:
        a.ldx(1, 3, 6, 0).alu64(0x50, 3, 63).stx(4, 10, -4, 3)
        a.ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
        a.jmp(JEQ, 0, "nohit", imm=0)
        a.mov64(1, 1).xadd(8, 0, 0, 1)
        a.label("nohit")
    a.ldx(1, 4, 6, 9).alu64(0x90, 4, pop_mod).jmp(JNE, 4, "nopop", imm=0)  # MOD
    a.ld_map(1, 2).mov64(2, src=10).add64(2, -24).call(88)
    a.ldx(8, 3, 10, -24)
    a.jmp(JEQ, 3, "nopop", imm=0)
    a.ldx(8, 4, 3, 0).alu64(0x00, 8, src=4)
    if key_from_pop:
        a.alu64(0x50, 4, 63).stx(4, 10, -12, 4)
        a.ld_map(1, 1).mov64(2, src=10).add64(2, -12).call(1)
    a.label("nopop")
    for k in range(pushes):
        a.ldx(8, 3, 6, 8 * k).stx(8, 10, -8, 3)
        a.ld_map(1, 2).mov64(2, src=10).add64(2, -8).mov64(3, 0).call(87)
    a.label("out").mov64(0, src=8).alu64(0x50, 0, 3).exit()
    return a.assemble()


def _case(name):
    lrumap = (MapDef(MAP_LRU_HASH, 4, 8, 64), None)
    q = (MapDef(MAP_QUEUE, 0, 8, 1 << 16), None)
    if name == "queue":
        return prog_work_queue(False), [lrumap, q], {1: SHORT}
    if name == "queue_lru":
        return prog_work_queue(True), [lrumap, q], {0: LRU_PRE, 1: SHORT}
    if name == "queue_drain_fast":  # pops on 2 of 3 packets, one push each: the queue drains, cut often
        return prog_work_queue(False, pop_mod=3, pushes=1), [lrumap, q], {1: SHORT}
    if name == "queue_two_pushes":
        return prog_work_queue(True, pushes=2), [lrumap, q], {0: LRU_PRE, 1: SHORT}
    if name == "queue_pop_key":
        return prog_work_queue(True, key_from_pop=True), [lrumap, q], {0: LRU_PRE, 1: SHORT}
    raise KeyError(name)


CASES = ["queue", "queue_lru", "queue_drain_fast", "queue_two_pushes", "queue_pop_key"]


def _stream(lib, name, n, nb=3):
    prog, maps, entries = _case(name)
    batches = [packets(n, 64, seed=31 + 7 * b) for b in range(nb)]
    return run_stream(lib, prog, maps, entries, Settings(), batches)


@pytest.mark.parametrize("n", [1024, 8192])
@pytest.mark.parametrize("name", CASES)
def test_segments_hostsim_equal_oracle(oracle_lib, hostsim_lib, name, n):
    got, want = _stream(hostsim_lib, name, n), _stream(oracle_lib, name, n)
    for b, ((ga, gm), (wa, _)) in enumerate(zip(got, want)):
        assert_same(ga, wa, f"{name} batch {b}")
    # the first batch runs past the 40 preloaded elements after pushes: segments (the drained variant
    # may find a cut too early for one and replay in order instead)
    assert got[0][1] in ((MODE_SEGMENTS, MODE_SEQUENTIAL) if name == "queue_drain_fast" else (MODE_SEGMENTS,)), got[0][1]


def test_stack_after_push_still_in_order(oracle_lib, hostsim_lib):
    """Stack pops interleaved with pushes from the first packets on: no cut of 64 packets or more, the
    batch replays in order (and equals the oracle)."""
    prog = prog_work_queue(False)
    maps = [(MapDef(MAP_LRU_HASH, 4, 8, 64), None), (MapDef(MAP_STACK, 0, 8, 1 << 16), None)]
    batches = [packets(2048, 64, seed=5)]
    got = run_stream(hostsim_lib, prog, maps, {1: SHORT}, Settings(), batches)
    want = run_stream(oracle_lib, prog, maps, {1: SHORT}, Settings(), batches)
    assert_same(got[0][0], want[0][0], "stack")
    assert got[0][1] == MODE_SEQUENTIAL


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_segments_device_equal_oracle(gpu_lib, oracle_lib, name):
    n = 16384  # (two pushes per packet stay inside the queue's 65536 entries)
    got, want = _stream(gpu_lib, name, n, nb=2), _stream(oracle_lib, name, n, nb=2)
    for b, ((ga, gm), (wa, _)) in enumerate(zip(got, want)):
        assert_same(ga, wa, f"{name} batch {b}")
    assert got[0][1] in ((MODE_SEGMENTS, MODE_SEQUENTIAL) if name == "queue_drain_fast" else (MODE_SEGMENTS,)), got[0][1]


def test_segments_async_stream_hostsim(hostsim_lib, oracle_lib):
    """Pipelined batches (xe_run_batch_device_async): a batch that must be cut is completed through the
    synchronous path, as segments, in submission order with the batches queued behind it."""
    from parity import _dump, setup_one
    prog, maps, entries = _case("queue_lru")
    bs = [packets(2048, 64, seed=51 + b) for b in range(4)]
    want = run_stream(oracle_lib, prog, maps, entries, Settings(), bs)
    vm, idx = setup_one(hostsim_lib, prog, maps, Settings(), entries)
    keep, handles = [], []
    for u, d in bs:
        u = u.copy()
        v = np.zeros(len(d), dtype=np.uint32)
        keep.append((u, v))
        handles.append(vm.run_batch_device_async(u.ctypes.data, u.nbytes, d.ctypes.data, len(d), d_verdicts=v.ctypes.data))
    sts = [h.stats() for h in handles]
    dumps = [_dump(vm, m) for m in idx]
    vm.close()
    for b, ((r, _, _), _) in enumerate(want):
        assert (keep[b][1] == r.verdicts).all(), f"batch {b}"
    wd = want[-1][0][1]
    assert dumps[1] == wd[1], "queue contents"
    assert all(np.array_equal(dumps[0][k], wd[0][k]) if isinstance(dumps[0][k], np.ndarray) else dumps[0][k] == wd[0][k]
               for k in dumps[0]), "LRU map"
    assert sts[0]["mode_used"] == MODE_SEGMENTS
