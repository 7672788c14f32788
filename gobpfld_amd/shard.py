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
    for m in maps:
        need = size_of(m)
        if m not in cache or cache[m].numel() < need:
            cache[m] = torch.zeros(need, dtype=torch.uint8, device=device)
    return cache


def exchange_shards(vm, maps, dist, rerun, device="cpu", stream: int = 0) -> dict:
    """After this rank's run: make every rank's maps (and, on replay, its results) exact.

    rerun(): runs this rank's shard again from its original packet bytes (called on replay only).
    Returns {"exact_sum": bool, "lanes": [...]}."""
    import torch
    rank, world = dist.get_rank(), dist.get_world_size()
    fp = vm.footprint()
    t = torch.from_numpy(fp.view(np.int64).copy()).to(device)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    fps = np.concatenate([p.cpu().numpy() for p in parts]).view(np.uint64)
    ok, lanes = vm.shard_check(fps, world)
    if ok:
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
            vm.map_apply_delta(m, buf.data_ptr(), stream=stream, lane=lane)
        return {"exact_sum": True, "lanes": list(lanes)}
    sbytes = {m: vm.map_state_bytes(m) for m in maps}
    sbufs = _bufs(vm, maps, device, "_shard_state_bufs", lambda m: sbytes[m])

    def move(src: int, import_on) -> None:
        for m in maps:
            b = sbufs[m][: sbytes[m]]
            if rank == src:
                vm.map_state_export(m, b.data_ptr(), stream=stream)
            dist.broadcast(b, src=src)
            if import_on(rank) and rank != src:
                vm.map_state_import(m, b.data_ptr(), stream=stream)

    for k in range(1, world):
        move(k - 1, lambda r, k=k: r == k)
        if rank == k:
            rerun()
    move(world - 1, lambda r: True)
    return {"exact_sum": False, "lanes": list(lanes)}
