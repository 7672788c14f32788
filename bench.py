#!/usr/bin/env python3
"""Benchmark: device-resident Mpkt/s of XDP-emulator verdicts (BASELINE.json metric).

Default workload (N=1) = BASELINE configs[1], "C2": ~40-insn L2/L3 classifier over 16,777,216 x 64 B
synthetic packets with per-proto ARRAY counters. A step = one pass of the batch through the emulator
(a pipelined xe_run_batch_device_async: the per-program kernel, then the one-block epilogue with the
device-side commutativity check; --sync: xe_run_batch_device) with packets, descriptors and the
verdict buffer already resident in HBM.

N > 1: one process per GPU (torchrun; `--gpus N` without torchrun starts the same ranks as children),
every rank runs its own 16M-packet shard (weak scaling) and the timed steps form one shard epoch whose
map deltas are all-reduced over RCCL (or replayed in order) inside the timed region — the same code
path for N = 1..8. After the timed region every rank checks its verdicts and its map against truth
derived from the generated headers (`verified`). The default line also carries BASELINE configs[4]
as the `c5` side line (33.5M packets per GPU, per-flow HASH counters, the per-flow delta exchange
timed separately, verified the same way). Prints ONE JSON line (rank 0) with roofline and
cpu_baseline objects.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5] [--packets P]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0
WORKLOADS = {
    "c1": "C1: 3-insn XDP_PASS (r0 = 2; r0 += 0; exit), 64 B packets, no maps",
    "c2": "C2 (BASELINE configs[1]): ~40-insn L2/L3 parse->PASS/DROP classifier, per-proto ARRAY counters",
    "c3": "C3: 5-tuple HASH lookup -> REDIRECT + hit counter, 64K flows, IMIX 64/576/1500 B",
    "c4": "C4: ~200-insn JEQ/JGT ACL (48 rules), 1500 B packets, lane-divergence stress",
    "c4f": "C4 in AF_XDP frames: the C4 ACL over 1500 B packets in 2-KiB UMEM chunks after the 256-byte XDP headroom",
    "c5": "C5: C2 parse + per-flow HASH counters {pkts, bytes}, 1M flows, 64 B packets",
    "c3learn": "C3-learn: C3 whose misses (10%, 262,144 new flows) insert the flow (bpf_map_update_elem, BPF_ANY): "
               "map-entry writes, order-dependent; IMIX 64/576/1500 B",
    "c3lru": "C3-LRU: C3-learn over an LRU_HASH flow table (1M entries, 64K preloaded; every lookup hit and update "
             "promotes, misses insert; no eviction): keyed chains with the UsageList relinked by last touch",
    "c3lrufull": "C3-LRU-full: C3-learn over a full LRU_HASH flow table (1M entries: 983,040 stale flows, then the 64K "
                 "hot ones most recent); every learned flow evicts the least recently used entry",
    "c2rmw": "C2-RMW: C2 with the per-proto counter bumped by a plain load/add/store (value->packets++ without "
             "an atomic): the ordered read-modify-write, run in parallel through lift_rmw",
    "bpf2bpf": "bpf2bpf: call-heavy analogue of the reference's cmd/examples/bpf_to_bpf/src/xdp.c — Ethernet / IPv4 "
               "parse and two bpf-to-bpf calls per packet into a stats sub-program (lookup, lifted {pkts, bytes} "
               "adds), 3 HASH maps, 64 B packets",
}  # MI355X_MICROARCH.md: 8.0 TB/s HBM3E spec peak


def alg_bytes_per_packet(name: str, sizes: np.ndarray) -> np.ndarray:
    """16 B descriptor + min(len, 64) header window + 4 B verdict (C2-C5); C1 reads no
    packet bytes, so 16 + 4."""
    if name == "c1":
        return np.full(sizes.shape, 20, dtype=np.int64)
    return 16 + np.minimum(sizes, 64) + 4


ALG_DESC = {"c1": "16 desc + 4 verdict (program reads no packet bytes)"}


PROFILE_ROUNDS = ("r6", "r5", "r4", "r3")  # committed PMC passes, newest first (a newer round's file supersedes)


def _profile(name: str, kind: str, n: int) -> tuple[dict | None, str | None]:
    """profiles/<round>/<config>_<kind>.json of this exact workload and batch size (newest round first)."""
    for rnd in PROFILE_ROUNDS:
        f = ROOT / "profiles" / rnd / f"{name}_{kind}.json"
        if f.exists():
            d = json.loads(f.read_text())
            if d.get("workload") == name and int(d.get("packets", -1)) == n:
                return d, str(f.relative_to(ROOT))
            return None, None
    return None, None


def pmc_traffic(name: str, n: int) -> tuple[float | None, str | None]:
    """HBM bytes per launch from the committed rocprofv3 PMC passes of this workload (2 x FETCH_SIZE +
    WRITE_SIZE, MI355X_MICROARCH.md; profiles/<round>/<config>_traffic.json), when one exists for this exact
    batch size; else (None, None)."""
    d, src = _profile(name, "traffic", n)
    return (None, None) if d is None else (float(d["hbm_bytes_per_launch"]), src)


def sq_issue(name: str, n: int, kernel_s: float | None = None) -> dict:
    """Issue-slot use of the emulator kernel from the committed SQ counter pass of this workload
    (profiles/<round>/<config>_sq_counters.json): wave-instructions per launch against one VALU and one
    SALU issue per CU per clock (256 CUs x 2.4 GHz) over the live average kernel time. Replaces the old
    eBPF-instructions-per-lane 'issue_frac', which counted emulated instructions, not machine issue."""
    d, src = _profile(name, "sq_counters", n)
    if d is None or not kernel_s:
        return {"sq_issue": None}
    slots = 256 * 2.4e9 * kernel_s
    pl = d["per_launch"]
    return {"sq_issue": {"valu_frac": round(pl["SQ_INSTS_VALU"] / slots, 4), "salu_frac": round(pl["SQ_INSTS_SALU"] / slots, 4),
                         "valu_per_chunk": d["per_64_packet_chunk"]["SQ_INSTS_VALU"],
                         "salu_per_chunk": d["per_64_packet_chunk"]["SQ_INSTS_SALU"],
                         "wait_frac": round(pl["SQ_WAIT_INST_ANY"] / max(1, pl["SQ_WAVE_CYCLES"]), 4), "source": src}}


def _oracle_prep(name: str, start: int, n: int):
    """A private oracle VM loaded with `name` and the host batch of packets [start, start+n)."""
    from gobpfld_amd import _native as N
    from gobpfld_amd import workloads as W
    from gobpfld_amd.emulator import VM, Settings
    vm = VM(Settings(), lib=N.Lib(ROOT / "oracle" / "liboracle.so", "orc_"))
    W.setup_vm(vm, name)
    umem, descs = W.build_batch(name, start, n)
    return vm, umem, descs


def _oracle_run(job) -> float:
    """insns/pkt of one prepared shard (ctypes releases the GIL: threads run in parallel)."""
    vm, umem, descs = job
    r = vm.run_batch(umem, descs)
    vm.close()
    return r.stats["steps"] / max(1, len(descs))


def _oracle_rate(name: str, start: int, n: int) -> tuple[float, float]:
    job = _oracle_prep(name, start, n)
    t0 = time.perf_counter()
    ipp = _oracle_run(job)
    return time.perf_counter() - t0, ipp


def host_cpu_info() -> dict:
    """The host the CPU baseline runs on: `nproc` (all CPUs of the machine), the CPUs this process may
    run on (sched_getaffinity), the per-job CPU share the GPU pool grants (OMP_NUM_THREADS on the box,
    16 per GPU; a pool of more threads than the share only oversubscribes it) and the lscpu model."""
    ncpu = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = ncpu
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = min(aff, share) if share > 0 else aff
    return {"nproc": ncpu, "affinity_cpus": aff, "job_cpu_share": share or None, "usable_cpus": max(1, usable),
            "cpu_model": model}


def cpu_baseline(name: str, n_sample: int, target_s: float = 12.0, threads: int = 0) -> dict:
    """The oracle (C++ restatement of emulator/) timed on a bounded prefix of the workload: one thread,
    then `threads` threads, each a private VM over a contiguous shard (valid: the configs' map
    effects commute), wall clock over the whole sample.

    n_sample = 0 calibrates on a 20k-packet prefix and sizes the sample for ~target_s seconds."""
    from concurrent.futures import ThreadPoolExecutor
    from gobpfld_amd import build as B
    B.build_oracle()
    host = host_cpu_info()
    threads = threads or host["usable_cpus"]
    cal_dt, _ = _oracle_rate(name, 0, 20_000)
    r1 = 20_000 / cal_dt
    n1 = n_sample or int(min(max(r1 * target_s / 2, 50_000), 8_000_000))
    dt1, ipp = _oracle_rate(name, 0, n1)
    nt = n_sample or int(min(max(r1 * threads * target_s / 2, 50_000), 32_000_000))
    per = (nt + threads - 1) // threads
    with ThreadPoolExecutor(threads) as ex:
        jobs = list(ex.map(lambda k: _oracle_prep(name, k * per, per), range(threads)))
        t0 = time.perf_counter()
        list(ex.map(_oracle_run, jobs))
        dtt = time.perf_counter() - t0
    return {"value": round(per * threads / dtt / 1e6, 4), "unit": "Mpkt/s", "cores": threads, "kind": "port",
            "host": host,
            "single_thread_value": round(n1 / dt1 / 1e6, 4),
            "sample": f"{per * threads} packets of {name} on {threads} threads (private VMs on contiguous shards, "
                      f"{dtt:.2f} s wall) and the first {n1} packets on 1 thread ({dt1:.2f} s) through "
                      f"oracle/liboracle.so (C++ restatement of gobpfld emulator/, per-packet Reset/Run harness); "
                      f"{ipp:.1f} insns/pkt"}


def e2e_baseline(vm, umem: np.ndarray, descs: np.ndarray, iters: int = 3) -> dict:
    """End-to-end rate: packets start and end in host memory. Pinned host UMEM + descriptors ->
    hipMemcpyAsync H2D -> emulator kernel -> D2H verdicts (+ packet bytes when the program can write
    them) through xe_run_batch_host. Never `value`; reported beside it."""
    import torch
    n = len(descs)
    pu = torch.from_numpy(umem).pin_memory()
    pd = torch.from_numpy(descs.view(np.uint8)).pin_memory()
    pv = torch.empty(n, dtype=torch.int32).pin_memory()
    args = (pu.data_ptr(), pu.numel(), pd.data_ptr(), n, pv.data_ptr())
    vm.run_batch_host_ptrs(*args)  # warm-up (device staging buffers)
    t0 = time.perf_counter()
    for _ in range(iters):
        st = vm.run_batch_host_ptrs(*args)
    dt = (time.perf_counter() - t0) / iters
    h2d = pu.numel() + pd.numel()
    return {"value": round(n / dt / 1e6, 3), "unit": "Mpkt/s", "ms_per_batch": round(dt * 1e3, 3),
            "device_ms_per_batch": round(st["total_ms"], 3), "h2d_bytes_per_packet": round(h2d / n, 2),
            "d2h_bytes_per_packet": 4, "packets": n,
            "path": "pinned host UMEM + descriptors -> H2D -> kernel -> D2H verdicts (xe_run_batch_host)"}


def ordered_paths(d_umem, d_desc, n: int, dev, stream, seq_sample: int = 65536) -> dict:
    """C2-RMW (C2 with `value->packets++` as a plain load/add/store) on the C2 batch: the lifted
    parallel path over all n packets (lift_rmw), and, for scale, the one-lane ordered replay the
    same program takes without lifting (MODE_SEQUENTIAL) on the first `seq_sample` packets."""
    import torch
    from gobpfld_amd import workloads as W
    from gobpfld_amd.emulator import MODE_SEQUENTIAL, VM, Settings
    d_ver = torch.zeros(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)
    out = {"program": WORKLOADS["c2rmw"]}
    for key, mode, cnt, reps in (("lifted_parallel", 0, n, 5), ("sequential_one_lane", MODE_SEQUENTIAL, seq_sample, 1)):
        vm = VM(Settings(device=dev.index or 0, mode=mode))
        W.setup_vm(vm, "c2rmw")
        run = lambda: vm.run_batch_device(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), cnt,
                                          d_verdicts=d_ver.data_ptr(), stream=stream)
        run()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ks = []
        for _ in range(reps):
            st = run()
            ks.append(st["kernel_ms"])
        torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t0) / reps
        out[key] = {"value": round(cnt / dt / 1e6, 3), "unit": "Mpkt/s", "packets": cnt, "ms_per_batch": round(dt * 1e3, 4),
                    "avg_kernel_ms": round(float(np.mean(ks)), 4), "mode_used": st["mode_used"], "conflict": st["conflict"]}
        vm.close()
    return out


def keyed_paths(dev, stream, n: int, batches: int = 5, seq_sample: int = 65536, name: str = "c3learn") -> dict:
    """C3-learn (C3 with flow learning: a miss inserts the flow with bpf_map_update_elem), "c3lru" (the same
    over an LRU_HASH flow table with room for every flow) or "c3lrufull" (the LRU table full: every learned
    flow evicts the least recently used entry) as a steady stream: one VM, map upload and kernel builds
    first (a 0-packet run, then one warm-up batch), then `batches` consecutive batches of n packets
    (packets [k n, (k+1) n)) timed back to back, each on the keyed ordered execution path (SPEC pass,
    chains per written key, xe_internal.h) as the VM's state carries over. For scale, the one-lane in-order
    replay (MODE_SEQUENTIAL) of the first `seq_sample` packets on a fresh VM."""
    import torch
    from gobpfld_amd import workloads as W
    from gobpfld_amd.emulator import MODE_SEQUENTIAL, VM, Settings
    bufs = [device_batch(name, k * n, n, dev) for k in range(batches + 1)]
    d_ver = torch.zeros(n, dtype=torch.int32, device=dev)
    _dsync(dev)
    out = {"program": WORKLOADS[name]}
    vm = VM(Settings(device=dev.index or 0))
    W.setup_vm(vm, name)
    run = lambda b, cnt, v=vm: v.run_batch_device(b[0].data_ptr(), b[0].numel(), b[1].data_ptr(), cnt,
                                                  d_verdicts=d_ver.data_ptr(), stream=stream)
    run(bufs[0], 0)       # upload
    run(bufs[0], n)       # warm-up batch (packets [0, n)): kernels, the keyed tables' sizes
    _dsync(dev)
    sts = []
    t0 = time.perf_counter()
    for k in range(1, batches + 1):
        sts.append(run(bufs[k], n))
    _dsync(dev)
    dt = time.perf_counter() - t0
    entries = vm.map_count(1) if hasattr(vm, "map_count") else None
    vm.close()
    out["keyed"] = {"value": round(batches * n / dt / 1e6, 3), "unit": "Mpkt/s", "packets_per_batch": n,
                    "batches": batches, "ms_per_batch": round(dt / batches * 1e3, 3),
                    "device_ms": [round(st["kernel_ms"], 3) for st in sts],
                    "mode_used": [st["mode_used"] for st in sts], "grid_blocks": sts[-1]["grid_blocks"],
                    "entries_after": entries,
                    "what": f"a stream of {batches} consecutive batches on one VM after one warm-up batch (steady state)"}
    # the one-lane replay, for scale
    vm = VM(Settings(device=dev.index or 0, mode=MODE_SEQUENTIAL))
    W.setup_vm(vm, name)
    run(bufs[0], 0, vm)
    _dsync(dev)
    t0 = time.perf_counter()
    st = run(bufs[0], seq_sample, vm)
    _dsync(dev)
    dt = time.perf_counter() - t0
    vm.close()
    out["sequential_one_lane"] = {"value": round(seq_sample / dt / 1e6, 3), "unit": "Mpkt/s", "packets": seq_sample,
                                  "ms_per_batch": round(dt * 1e3, 3), "device_ms": round(st["kernel_ms"], 3),
                                  "mode_used": [st["mode_used"]]}
    del bufs
    torch.cuda.empty_cache()
    return out


def _rccl_version() -> str | None:
    try:
        import torch
        v = torch.cuda.nccl.version()
        return ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
    except Exception:  # noqa: BLE001 - informational only
        return None


def relaunch_ranks(gpus: int) -> int:
    """`bench.py --gpus N` started without torchrun: the same one-process-per-GPU run the driver launches
    (python -m torch.distributed.run ... bench.py), started as a child before anything touches the GPU,
    so N=1..8 go through one code path (pipelined batches per rank, one shard epoch per timed region)."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(ROOT / "bench.py")] + sys.argv[1:]
    return subprocess.call(cmd, env=dict(os.environ, MASTER_ADDR="127.0.0.1"))


# ---------------------------------------------------------------- self-verification (header-derived truth)
def _c2_truth(idx: np.ndarray):
    """C2 from the generated headers (no emulator involved): verdict per packet, per-proto counts."""
    from gobpfld_amd import workloads as W
    h = W.headers_c2(idx, 64).astype(np.int64)
    et = (h[:, 12] << 8) | h[:, 13]
    vlan = et == 0x8100
    et = np.where(vlan, (h[:, 16] << 8) | h[:, 17], et)
    l3 = np.where(vlan, 18, 14)
    rows = np.arange(len(idx))
    proto = np.where(et == 0x0800, h[rows, l3 + 9], np.where(et == 0x86DD, h[rows, l3 + 6], -1))
    verdict = np.where(np.isin(proto, [1, 6, 17]), 2, 1).astype(np.uint32)
    return verdict, np.bincount(proto[proto >= 0], minlength=256).astype(np.int64)


def _c4_truth(idx: np.ndarray) -> np.ndarray:
    """First match over the 48 ACL rules on the header bytes the program reads (workloads.prog_c4)."""
    from gobpfld_amd import workloads as W
    h = W.headers_c4(idx, 64)
    h64 = h.astype(np.uint64)
    ipv4 = (h[:, 12] == 0x08) & (h[:, 13] == 0x00)
    saddr = h64[:, 26] | (h64[:, 27] << 8) | (h64[:, 28] << 16) | (h64[:, 29] << 24)
    proto, dport = h64[:, 23], h64[:, 36] | (h64[:, 37] << 8)
    verdict = np.full(len(h), 1, dtype=np.uint32)
    open_ = ipv4.copy()
    for s_le, p, dmax, action in W.acl_rules():
        m = open_ & (saddr == np.uint64(s_le)) & (proto == np.uint64(p)) & (dport <= np.uint64(dmax))
        verdict[m] = action
        open_ &= ~m
    return verdict


def shard_truth(name: str, start: int, n: int):
    """Expected verdicts of packets [start, start + n) and the map effect of one run over them, derived
    from the generated headers with numpy (SURVEY §8d workloads; independent of the emulator):
    (verdicts u32[n], delta int64 array or None). None for workloads without such a truth."""
    from gobpfld_amd import workloads as W
    idx = np.arange(start, start + n, dtype=np.uint64)
    if name == "c1":
        return np.full(n, 2, np.uint32), None
    if name in ("c2", "c2rmw"):  # C2-RMW: the same counters, bumped by a (lifted) load / add / store
        return _c2_truth(idx)
    if name in ("c4", "c4f"):
        return _c4_truth(idx), None
    if name == "c3":
        r0 = W.rng_stream(3, idx, 0)
        hit = (W.rng_stream(3, idx, 2) % np.uint64(10)) != 0
        fid = W.zipf_ranks((r0 >> np.uint64(11)).astype(np.float64) / float(1 << 53), W.C3_FLOWS)
        return np.where(hit, 4, 2).astype(np.uint32), np.bincount(fid[hit], minlength=W.C3_FLOWS).astype(np.int64)
    if name == "c5":
        fid = W.rng_stream(5, idx, 0) % np.uint64(W.C5_FLOWS + W.C5_FLOWS // 16)
        hit = fid < np.uint64(W.C5_FLOWS)
        return np.full(n, 2, np.uint32), np.bincount(fid[hit].astype(np.int64), minlength=W.C5_FLOWS).astype(np.int64)
    return None, None


def expected_map(name: str, total: np.ndarray):
    """The map after runs whose summed per-run effects are `total` (init + total), in xe_map_dump form."""
    from gobpfld_amd import workloads as W
    if name in ("c2", "c2rmw"):
        return total.astype(np.uint64).tobytes()
    if name in ("c3", "c5"):
        keys, vals0 = W.c3_map_entries() if name == "c3" else W.c5_map_entries()
        vals = vals0.view(np.uint64).reshape(-1, 2).copy()
        if name == "c3":
            vals[:, 1] += total.astype(np.uint64)            # {flow_id, hits}
        else:
            vals[:, 0] += total.astype(np.uint64)            # {pkts, bytes} of 64-byte packets
            vals[:, 1] += total.astype(np.uint64) * np.uint64(64)
        o = np.lexsort(keys.T[::-1])                         # xe_map_dump order: key bytes, memcmp
        return keys[o], vals[o]
    return None


def verify(name: str, vm, start: int, n: int, runs: int, d_ver, dist, world: int, dev) -> dict:
    """After the timed region: this rank's last verdicts against the truth of its shard, and its map against
    init + runs x the sum over every rank's shard (the single VM over all shards, in order: the per-epoch
    exchange must have made every replica exactly that). Every rank checks; `verified` is their AND."""
    import torch
    t0 = time.perf_counter()
    want_v, delta = shard_truth(name, start, n)
    if want_v is None:
        return {"verified": None, "what": "no header-derived truth for this workload"}
    ok_v = bool((d_ver.cpu().numpy().view(np.uint32) == want_v).all())
    ok_m = True
    if delta is not None:
        t = torch.from_numpy(delta * runs).to(dev)
        if world > 1:
            dist.all_reduce(t)
        exp = expected_map(name, t.cpu().numpy())
        got = vm.map_dump(1)
        if isinstance(exp, bytes):
            ok_m = got == exp
        else:
            k, v = got
            ok_m = (np.array_equal(np.asarray(k).reshape(exp[0].shape), exp[0]) and
                    np.array_equal(np.frombuffer(np.asarray(v).tobytes(), np.uint64).reshape(-1, 2), exp[1]))
    flag = torch.tensor([int(ok_v and ok_m)], dtype=torch.int32, device=dev)
    if world > 1:
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return {"verified": bool(flag.item()), "verdicts_ok_rank0": ok_v, "map_ok_rank0": ok_m if delta is not None else None,
            "what": f"every rank: last verdicts == header truth of its shard; map == init + {runs} runs x sum over "
                    f"{world} shard(s) of the header-derived per-run effect", "check_s": round(time.perf_counter() - t0, 2)}


def _dsync(dev) -> None:
    """torch.cuda.synchronize on a GPU device; nothing on the CPU (the gloo tests drive run_epochs with
    host-simulation VMs over CPU tensors)."""
    import torch
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def run_epochs(vm, epoch, dist, world, dev, d_umem, d_desc, n, d_ver, stream, warmup: int, steps: int, pipelined=True):
    """Warm-up epoch, then the timed epoch: `steps` pipelined batches and (N > 1) the shard exchange (one
    RCCL all-reduce per map, or the in-order replay), all inside the timed region. Returns the timed
    batches' stats, elapsed max over ranks, the exchange's share of it and its outcome."""
    import torch
    exchanges = {"exact_sum": 0, "replayed": 0}

    def sync_run():
        return vm.run_batch_device(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), n, d_verdicts=d_ver.data_ptr(),
                                   stream=stream)

    def epoch_of(k: int):
        if epoch is not None:
            epoch.begin()
        if pipelined:
            hs = [vm.run_batch_device_async(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), n,
                                            d_verdicts=d_ver.data_ptr(), stream=stream) for _ in range(k)]
            vm.sync()
            sts = [h.stats() for h in hs]
        else:
            sts = [sync_run() for _ in range(k)]
        t_x = time.perf_counter()
        if epoch is not None:
            _dsync(dev)
            t_x = time.perf_counter()
            x = epoch.exchange([sync_run] * k)
            exchanges["exact_sum" if x["exact_sum"] else "replayed"] += 1
        return sts, t_x

    epoch_of(warmup)
    _dsync(dev)
    if world > 1:
        dist.barrier()
    _dsync(dev)
    t0 = time.perf_counter()
    sts, t_x = epoch_of(steps)
    _dsync(dev)
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    _dsync(dev)
    t2 = time.perf_counter()
    t = torch.tensor([t2 - t0, t1 - t_x], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return sts, float(t[0].item()), float(t[1].item()), exchanges


def device_batch(name: str, start: int, n: int, dev):
    """The batch of packets [start, start + n) resident in HBM: (d_umem, d_desc, descs). Fixed-size packets
    back to back (C4's 16,777,216 x 1500 B = 25 GB) are laid out on the device — zeroed UMEM, then the
    64-byte header rows copied into their packets' first bytes — instead of building the UMEM on the host
    (the same bytes as workloads.build_batch: bytes past the header window are zero)."""
    import torch
    from gobpfld_amd import workloads as W
    from gobpfld_amd._native import np_dtypes
    cfg = W.CONFIGS[name]
    if isinstance(cfg["pkt"], int) and cfg["pkt"] >= 64 and not cfg.get("frame"):
        size = int(cfg["pkt"])
        idx = np.arange(start, start + n, dtype=np.uint64)
        d_umem = torch.zeros(n * size, dtype=torch.uint8, device=dev)
        d_umem.view(n, size)[:, :64].copy_(torch.from_numpy(W.headers(name, idx, 64)))
        descs = np.zeros(n, dtype=np_dtypes()[0])
        descs["addr"] = np.arange(n, dtype=np.int64) * size
        descs["len"] = size
    elif cfg["pkt"] == "imix" and not cfg.get("frame"):
        # mixed sizes, all >= 64 B: the header rows go to their packets' offsets on the device, 1M at a time
        idx = np.arange(start, start + n, dtype=np.uint64)
        sizes = W.packet_sizes(name, idx)
        assert sizes.min() >= 64
        offs, total = W.packet_offsets(name, sizes)
        d_umem = torch.zeros(max(total, 1), dtype=torch.uint8, device=dev)
        cols = torch.arange(64, dtype=torch.int64, device=dev)
        for c0 in range(0, n, 1 << 20):
            c1 = min(n, c0 + (1 << 20))
            h = torch.from_numpy(W.headers(name, idx[c0:c1], 64)).to(dev)
            pos = torch.from_numpy(offs[c0:c1]).to(dev)[:, None] + cols
            d_umem[pos.reshape(-1)] = h.reshape(-1)
        descs = np.zeros(n, dtype=np_dtypes()[0])
        descs["addr"] = offs
        descs["len"] = sizes
    else:
        umem, descs = W.build_batch(name, start, n)
        d_umem = torch.from_numpy(umem).to(dev)
        del umem
    d_desc = torch.from_numpy(descs.view(np.uint8)).to(dev)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    return d_umem, d_desc, descs


def side_line(name: str, n: int, steps: int, rank: int, world: int, dev, stream, dist) -> dict:
    """A BASELINE config beside the default line, timed and verified the way the main line is: `n`
    packets per GPU, one warm-up batch, then `steps` pipelined batches per rank and (N > 1) the shard
    exchange, timed separately; the kernel's roofline from the batches' HIP-event kernel times.
      c5 = configs[4]: 33,554,432 x 64 B per GPU, per-flow HASH counters {pkts, bytes} (1M flows); the
           exchange is one RCCL all-reduce of the per-flow deltas;
      c4 = configs[3]: 16,777,216 x 1500 B per GPU, the ~200-insn JEQ/JGT ACL (the 1500 B half of the
           metric); no map, so the exchange reconciles nothing;
      c3 = configs[2]: 16,777,216 IMIX packets per GPU, 5-tuple HASH -> flow id, XDP_REDIRECT, per-flow
           hit counters (64K flows, Zipf); checked against the header-derived truth like the others."""
    import torch
    from gobpfld_amd import workloads as W
    from gobpfld_amd.emulator import VM, Settings
    from gobpfld_amd.shard import ShardEpoch
    start = rank * n
    d_umem, d_desc, descs = device_batch(name, start, n, dev)
    d_ver = torch.zeros(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)
    vm = VM(Settings(device=dev.index or 0))
    W.setup_vm(vm, name)
    epoch = ShardEpoch(vm, list(vm.map_defs), dist, device=dev, stream=stream) if world > 1 else None
    sts, elapsed, x_s, exchanges = run_epochs(vm, epoch, dist, world, dev, d_umem, d_desc, n, d_ver, stream,
                                              1, steps)
    ver = verify(name, vm, start, n, 1 + steps, d_ver, dist, world, dev)
    vbytes = vm.map_values_bytes(1) if vm.map_defs else 0
    vm.close()
    del d_umem, d_desc, d_ver
    torch.cuda.empty_cache()
    kms = [st["kernel_ms"] for st in sts]
    k_s = float(np.mean(kms)) / 1e3
    sizes = descs["len"].astype(np.int64)
    alg = float(alg_bytes_per_packet(name, sizes).sum())
    traffic, traffic_src = pmc_traffic(name, n)
    full = float((16 + sizes + 4).sum())  # the full-packet variant for 1500 B packets
    roof = {"bound": "hbm", "achieved": round(alg / k_s / 1e9, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(alg / k_s / 1e9 / HBM_PEAK_GBS, 5), "traffic": None if traffic is None else int(traffic),
            "traffic_source": traffic_src, "kernel": "xe_jit_kernel", "avg_kernel_ms": round(k_s * 1e3, 4),
            "alg_bytes_per_launch": int(alg), "alg_bytes_per_packet": "16 desc + min(len,64) header + 4 verdict",
            **sq_issue(name, n, k_s)}
    if name == "c4":
        # what the same kernel time would be in GB/s if every packet byte were read (the ACL reads bytes
        # 12-42 only): a throughput equivalent for 1500 B packets, not a roofline fraction
        roof["full_packet_bytes_per_launch"] = int(full)
        roof["full_packet_equivalent_gbs"] = round(full / k_s / 1e9, 1)
    return {"workload": WORKLOADS[name], "packets_per_gpu": n, "n_gpus": world, "steps": steps,
            "value": round(n * world * steps / elapsed / 1e6, 3), "unit": "Mpkt/s",
            "ms_per_step": round(elapsed / steps * 1e3, 4), "avg_kernel_ms": round(k_s * 1e3, 4),
            "roofline": roof,
            "exchange_ms": round(x_s * 1e3, 4) if world > 1 else None,
            "exchange": dict(exchanges, delta_bytes_per_gpu=vbytes, per="epoch of the timed steps") if world > 1 else None,
            "mode": sorted({st["mode_used"] for st in sts}), **ver}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--packets", type=int, default=0, help="packets per GPU (default: the config's)")
    ap.add_argument("--cpu-sample", type=int, default=0, help="oracle baseline sample (0 = auto)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--engine", default="auto", choices=["auto", "interp", "jit"])
    ap.add_argument("--mode", default="auto", choices=["auto", "sequential"],
                    help="sequential: every batch on the one-lane in-order path (profiling the replay)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-memory (PCIe-inclusive) measurement")
    ap.add_argument("--no-ordered", action="store_true", help="skip the C2-RMW ordered-path lines (C2 only)")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 side line (C2 only)")
    ap.add_argument("--no-c4", action="store_true", help="skip the C4 (1500 B) side line (C2 only)")
    ap.add_argument("--c4-packets", type=int, default=16 * 1024 * 1024, help="C4 side line: packets per GPU")
    ap.add_argument("--c4-steps", type=int, default=10)
    ap.add_argument("--no-verify", action="store_true", help="skip the post-run self-check")
    ap.add_argument("--c5-packets", type=int, default=32 * 1024 * 1024, help="C5 side line: packets per GPU")
    ap.add_argument("--c5-steps", type=int, default=8)
    ap.add_argument("--no-c3", action="store_true", help="skip the C3 (IMIX, 5-tuple HASH) side line (C2 only)")
    ap.add_argument("--c3-packets", type=int, default=16 * 1024 * 1024, help="C3 side line: packets per GPU")
    ap.add_argument("--c3-steps", type=int, default=10)
    ap.add_argument("--sync", action="store_true", help="one synchronous xe_run_batch_device per step (no pipelining)")
    ap.add_argument("--keyed-packets", type=int, default=4 * 1024 * 1024,
                    help="C3-learn batch of the keyed ordered-execution line (C2 runs only)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1 and args.gpus > 1 and "RANK" not in os.environ:
        sys.exit(relaunch_ranks(args.gpus))

    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N-rank path on one GPU (scripts/rehearse_multi.sh): every rank on one device,
    # the exchange over gloo (RCCL refuses two ranks on one GPU); timings from such a run mean nothing
    if os.environ.get("XE_BENCH_REHEARSE"):
        local = 0
    if world > 1:
        dist.init_process_group("gloo" if os.environ.get("XE_BENCH_REHEARSE") else "nccl", init_method="env://")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from gobpfld_amd import workloads as W
    from gobpfld_amd.emulator import VM, Settings
    from gobpfld_amd.shard import ShardEpoch

    name = args.config
    n = args.packets or (W.CONFIGS[name]["n"] // (8 if name == "c5" else 1))  # C5: 33,554,432 per GPU
    start = rank * n

    # ---- inputs resident in HBM (synthetic packets; shard = contiguous packet index range)
    umem, descs = W.build_batch(name, start, n)
    sizes = descs["len"].astype(np.int64)
    d_umem = torch.from_numpy(umem).to(dev)
    d_desc = torch.from_numpy(descs.view(np.uint8)).to(dev)
    d_ver = torch.zeros(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)  # torch's stream vs the library's: the buffers are complete before any batch

    engine = {"auto": 0, "interp": 1, "jit": 2}[args.engine]
    from gobpfld_amd.emulator import MODE_AUTO, MODE_SEQUENTIAL
    vm = VM(Settings(device=local, engine=engine, mode=MODE_SEQUENTIAL if args.mode == "sequential" else MODE_AUTO))
    W.setup_vm(vm, name)
    stream = torch.cuda.current_stream(dev).cuda_stream
    # A stream of batches through the pipelined entry point (each batch's conflict check runs on the
    # device; xe_sync completes and, if needed, replays them — all inside the timed region). N > 1:
    # the batches of a call form one shard epoch, reconciled once at its end (footprint check, one
    # RCCL all-reduce per map, or the exact in-order replay) inside the timed region.
    epoch = ShardEpoch(vm, list(vm.map_defs), dist, device=dev, stream=stream) if world > 1 else None
    sts, elapsed, x_s, exchanges = run_epochs(vm, epoch, dist, world, dev, d_umem, d_desc, n, d_ver, stream,
                                              args.warmup, args.steps, pipelined=not args.sync)
    kernel_ms, mode, conflicts, steps_retired, status_ok, engines, grid = [], set(), 0, 0, 0, set(), 0
    for st in sts:
        kernel_ms.append(st["kernel_ms"])
        mode.add(st["mode_used"])
        engines.add({1: "interp", 2: "jit"}.get(st["engine_used"], "?"))
        conflicts += st["conflict"]
        steps_retired += st["steps"]
        status_ok += st["status_count"][0]
        grid = st["grid_blocks"]
    # self-check outside the timed region, before anything else runs on this VM
    check = None if args.no_verify else verify(name, vm, start, n, args.warmup + args.steps, d_ver, dist, world, dev)

    total_pkts = n * world * args.steps
    value = total_pkts / elapsed / 1e6
    avg_kernel_s = float(np.mean(kernel_ms)) / 1e3
    bytes_per_launch = float(alg_bytes_per_packet(name, sizes).sum())
    achieved_gbs = bytes_per_launch / avg_kernel_s / 1e9
    insns_per_pkt = steps_retired / max(1, n * args.steps)
    traffic, traffic_src = pmc_traffic(name, n)

    e2e = None
    if rank == 0 and not args.no_e2e:
        e2e = e2e_baseline(vm, umem, descs)
    del umem
    c5 = c4 = c3 = None
    if name == "c2" and not args.no_c3:
        c3 = side_line("c3", args.c3_packets, args.c3_steps, rank, world, dev, stream, dist)
    if name == "c2" and not args.no_c5:
        c5 = side_line("c5", args.c5_packets, args.c5_steps, rank, world, dev, stream, dist)
    if name == "c2" and not args.no_c4:
        c4 = side_line("c4", args.c4_packets, args.c4_steps, rank, world, dev, stream, dist)
    ordered = None
    if rank == 0 and name == "c2" and not args.no_ordered:
        ordered = ordered_paths(d_umem, d_desc, n, dev, stream)
        ordered["keyed_c3learn"] = keyed_paths(dev, stream, args.keyed_packets)
        ordered["keyed_c3lru"] = keyed_paths(dev, stream, args.keyed_packets, name="c3lru")
        ordered["keyed_c3lrufull"] = keyed_paths(dev, stream, args.keyed_packets, name="c3lrufull")
    # what the exchange ran over: the process group's backend and the rank count it saw (N > 1), and
    # RCCL's version; the C5 side line's per-flow delta exchange (time and bytes per GPU) beside it
    comm = {"backend": dist.get_backend() if world > 1 else None,
            "world": dist.get_world_size() if world > 1 else 1,
            "rccl_version": _rccl_version(),
            "c5_exchange_ms": c5["exchange_ms"] if c5 else None,
            "c5_delta_bytes_per_gpu": (c5["exchange"] or {}).get("delta_bytes_per_gpu") if c5 else None,
            "main_exchange_ms": round(x_s * 1e3, 4) if world > 1 else None,
            "main_exchanges": dict(exchanges) if world > 1 else None}
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline:
            cpu = cpu_baseline(name, args.cpu_sample)
        hw = {"c2": "64B", "c3": "IMIX 64/576/1500B", "c4": "1500B", "c4f": "1500B in 2 KiB frames", "c5": "64B"}.get(name, "64B")
        out = {
            "metric": "Mpkt/s device-resident XDP-emulator verdicts, 64B and 1500B batches",
            "value": round(value, 3),
            "unit": "Mpkt/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (deterministic splitmix64 packets, SURVEY §8d)",
            "config": {"workload": WORKLOADS[name],
                       "packets_per_gpu": n, "packet_size": hw,
                       "parallelism": f"dp{world} (packet shards, one process per GPU)",
                       "insns_per_packet": round(insns_per_pkt, 2), "mode": sorted(mode),
                       "engine": sorted(engines),
                       "conflicts": conflicts, "ok_packets_per_step": status_ok // max(1, args.steps),
                       "shard_exchanges": dict(exchanges, per="epoch of the timed steps",
                                               exchange_ms=round(x_s * 1e3, 4)) if world > 1 else None,
                       "batches": "pipelined (xe_run_batch_device_async, depth 3, device-side conflict check)"
                                  if not args.sync else "synchronous (xe_run_batch_device)",
                       "grid": grid},
            "verified": None if check is None else check["verified"],
            "verification": check,
            "roofline": {"bound": "hbm", "achieved": round(achieved_gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved_gbs / HBM_PEAK_GBS, 5),
                         "traffic": None if traffic is None else int(traffic), "traffic_source": traffic_src,
                         "kernel": "xe_jit_kernel" if engines == {"jit"} else "xe_interp_kernel", "avg_kernel_ms": round(avg_kernel_s * 1e3, 4),
                         "kernel_ms_steps": [round(k, 4) for k in kernel_ms],
                         "alg_bytes_per_launch": int(bytes_per_launch),
                         "alg_bytes_per_packet": ALG_DESC.get(name, "16 desc + min(len,64) header + 4 verdict"),
                         **sq_issue(name, n, avg_kernel_s)},
            "cpu_baseline": cpu,
            "e2e": e2e,
            "comm": comm,
            "c5": c5,
            "c4": c4,
            "c3": c3,
            "ordered": ordered,
        }
        print(json.dumps(out), flush=True)
    vm.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
