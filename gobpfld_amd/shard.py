"""Multi-GPU shard exchange: one all-reduce of map-value deltas per run.

Every rank runs its own contiguous packet shard on a map replica with identical initial contents.
After a run, each counter map's delta (values - run-start snapshot) is summed over the ranks and
added back, so every replica ends with init + the adds of all shards. The sum is taken in lanes of
the width of the map adds (a narrow counter wraps at its own width; a u64 word sum would carry
across fields): ranks first agree on the lane (MAX of the widths they saw; 0 = no adds anywhere).
Backend "nccl" is RCCL over xGMI on MI355X; "gloo" for the CPU tests."""
from __future__ import annotations


def allreduce_map_deltas(vm, maps, bufs: dict, dist, stream: int = 0) -> None:
    """bufs[m]: uint8 tensor of vm.map_values_bytes(m) bytes, on the device of the VM's backend."""
    import torch
    dev = next(iter(bufs.values())).device if bufs else "cpu"
    lanes = torch.tensor([vm.map_delta_lane(m) for m in maps], dtype=torch.int32, device=dev)
    dist.all_reduce(lanes, op=dist.ReduceOp.MAX)
    for m, lane in zip(maps, lanes.tolist()):
        if lane == 0:  # no adds on any rank: nothing to exchange
            continue
        buf = bufs[m]
        vm.map_delta(m, buf.data_ptr(), stream=stream, lane=lane)
        if lane == 8:
            dist.all_reduce(buf.view(torch.int64))
        elif lane == 4:
            dist.all_reduce(buf.view(torch.int32))
        elif lane == 1:
            dist.all_reduce(buf)
        else:  # no 16-bit integer reduction in RCCL: widen, sum, wrap back to 16 bits
            t = buf.view(torch.int16).to(torch.int32)
            dist.all_reduce(t)
            buf.view(torch.int16).copy_(t.to(torch.int16))
        vm.map_apply_delta(m, buf.data_ptr(), stream=stream, lane=lane)
