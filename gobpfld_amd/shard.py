"""Multi-GPU shard exchange, one process per GPU over torch.distributed.

Every rank runs its own contiguous packet shard (rank k holds the packets after those of ranks < k)
on a map replica with identical initial contents and slot layout. The reference processes all of
those packets in one loop, in order (emulator/vm.go:110-173 per packet), so after the runs the ranks
make their maps equal to that single-VM result:

* all ranks all-gather their footprint records (xe_footprint: flags, per-map read / add masks and add
  widths) and apply the same check (xe_shard_check, one implementation in the library). When it
  passes — no ordered path anywhere, no rank read a field an earlier rank added to, one aligned add
  width per map — init + the sum of the per-map deltas is exact: one all-reduce per map, in lanes of
  the add width (a narrow counter wraps at its own width; u16 lanes travel as u32 containers);
* otherwise the shards are replayed in order: rank k imports the whole map state rank k-1 ended
  with (xe_map_state_export / _import over a broadcast) and runs its shard again; the last state then
  goes to every rank.

Backend "nccl" is RCCL over xGMI on MI355X; "gloo" for the CPU tests. The single-process form of the
same protocol is xe_run_batch_multi (include/xdpemu.h)."""
from __future__ import annotations

import numpy as np


def _bufs(vm, maps, device, attr, size_of):
    import torch
    cache = getattr(vm, attr, None)
    if cache is None:
        cache = {}
        setattr(vm, attr, cache)
    grew = False
    for m in maps:
        need = size_of(m)
        if m not in cache or cache[m].numel() < need:
            cache[m] = torch.zeros(need, dtype=torch.uint8, device=device)
            grew = True
    if grew:
        _collective_done(device)  # the zero fill (torch's stream) lands before the library writes
    return cache


def _gather_check(vm, dist, device):
    import torch
    world = dist.get_world_size()
    fp = vm.footprint()
    t = torch.from_numpy(fp.view(np.int64).copy()).to(device)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    fps = np.concatenate([p.cpu().numpy() for p in parts]).view(np.uint64)  # .cpu() waits for the gather
    return vm.shard_check(fps, world)


def _collective_done(device) -> None:
    """The library's launches run on the stream it is given — or, for stream 0, on the VM's own stream,
    which is not torch's default stream (whose handle is also 0). A collective's result is only ordered
    before work on torch's current stream, so the host waits for it before the library reads it."""
    import torch
    dev = torch.device(device)
    if dev.type == "cuda":
        torch.cuda.current_stream(dev).synchronize()


def _sum_deltas(vm, maps, dist, lanes, device, stream) -> None:
    """init + the sum of every rank's per-map delta, one all-reduce per map in lanes of the add width."""
    import torch
    vbytes = {m: vm.map_values_bytes(m) for m in maps}
    bufs = _bufs(vm, maps, device, "_shard_delta_bufs", lambda m: 2 * vbytes[m])
    for m in maps:
        lane = lanes[m - 1]
        if lane == 0:  # no adds on any rank: nothing to exchange
            continue
        buf = bufs[m]
        vm.map_delta(m, buf.data_ptr(), stream=stream, lane=lane)
        if lane == 8:
            dist.all_reduce(buf[: vbytes[m]].view(torch.int64))
        elif lane == 1:
            dist.all_reduce(buf[: vbytes[m]])
        else:  # 4, and 2 (u32 containers, twice the region)
            dist.all_reduce(buf[: vbytes[m] * (2 if lane == 2 else 1)].view(torch.int32))
        _collective_done(device)
        vm.map_apply_delta(m, buf.data_ptr(), stream=stream, lane=lane)


def _mover(vm, maps, dist, device, stream):
    """move(src, import_on): rank src's whole map state to the ranks import_on(rank) selects. The image
    size is the source's (ordered maps serialise their current contents, so it varies): broadcast first."""
    import torch
    rank = dist.get_rank()

    def move(src: int, import_on) -> None:
        for m in maps:
            size = torch.tensor([vm.map_state_bytes(m) if rank == src else 0], dtype=torch.int64, device=device)
            dist.broadcast(size, src=src)
            nb = int(size.item())  # (.item() waits for the broadcast)
            b = _bufs(vm, [m], device, "_shard_state_bufs", lambda _m: nb)[m][:nb]
            if rank == src:
                vm.map_state_export(m, b.data_ptr(), stream=stream)
            dist.broadcast(b, src=src)
            _collective_done(device)
            if import_on(rank) and rank != src:
                vm.map_state_import(m, b.data_ptr(), stream=stream)
    return move


def exchange_shards(vm, maps, dist, rerun, device="cpu", stream: int = 0) -> dict:
    """After this rank's run: make every rank's maps (and, on replay, its results) exact.

    rerun(): runs this rank's shard again from its original packet bytes (called on replay only).
    Returns {"exact_sum": bool, "lanes": [...]}."""
    rank, world = dist.get_rank(), dist.get_world_size()
    ok, lanes = _gather_check(vm, dist, device)
    if ok:
        _sum_deltas(vm, maps, dist, lanes, device, stream)
        return {"exact_sum": True, "lanes": list(lanes)}
    move = _mover(vm, maps, dist, device, stream)
    for k in range(1, world):
        move(k - 1, lambda r, k=k: r == k)
        if rank == k:
            rerun()
    move(world - 1, lambda r: True)
    return {"exact_sum": False, "lanes": list(lanes)}


class ShardEpoch:
    """Many batches per exchange (xe_epoch_begin / include/xdpemu.h): every rank runs its shard of a
    stream of batches on its own map replica — synchronous or pipelined — and the ranks reconcile
    once at the end of the epoch instead of after every batch.

    The reference order is batch after batch, shards in rank order within a batch. The exchange is
    the per-batch one over the epoch's ORed footprints, with the stricter epoch check (no rank read a
    field any other rank added to); otherwise every rank goes back to the map state at the epoch's
    start and the batches are replayed in that order: batch s of rank k runs on the state batch s of
    rank k - 1 (or batch s - 1 of the last rank) ended with, moved over a broadcast.

    reruns (exchange): one callable per batch of the epoch, in order, each running this rank's shard
    of that batch synchronously from its original packet bytes."""

    def __init__(self, vm, maps, dist, device="cpu", stream: int = 0):
        self.vm, self.maps, self.dist, self.device, self.stream = vm, list(maps), dist, device, stream
        self.base = None

    def begin(self) -> None:
        vm = self.vm
        vm.epoch_begin(self.stream)
        sbytes = {m: vm.map_state_bytes(m) for m in self.maps}
        self.base = _bufs(vm, self.maps, self.device, "_shard_epoch_base", lambda m: sbytes[m])
        for m in self.maps:
            vm.map_state_export(m, self.base[m].data_ptr(), stream=self.stream)

    def exchange(self, reruns) -> dict:
        vm, dist = self.vm, self.dist
        rank, world = dist.get_rank(), dist.get_world_size()
        ok, lanes = _gather_check(vm, dist, self.device)
        if ok:
            _sum_deltas(vm, self.maps, dist, lanes, self.device, self.stream)
            vm.epoch_end()
            return {"exact_sum": True, "lanes": list(lanes), "batches": len(reruns)}
        vm.epoch_end()
        for m in self.maps:  # every rank back to the epoch's start
            vm.map_state_import(m, self.base[m].data_ptr(), stream=self.stream)
        move = _mover(vm, self.maps, dist, self.device, self.stream)
        holder = None
        for rerun in reruns:
            for k in range(world):
                if holder is not None and holder != k:
                    move(holder, lambda r, k=k: r == k)
                if rank == k:
                    rerun()
                holder = k
        if holder is not None:
            move(holder, lambda r: True)
        return {"exact_sum": False, "lanes": list(lanes), "batches": len(reruns)}
