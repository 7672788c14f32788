#!/usr/bin/env python3
"""Benchmark: device-resident Mpkt/s of XDP-emulator verdicts (BASELINE.json metric).

Default workload (N=1) = BASELINE configs[1], "C2": ~40-insn L2/L3 classifier over 16,777,216 x 64 B
synthetic packets with per-proto ARRAY counters. A step = one pass of the batch through the emulator
(a pipelined xe_run_batch_device_async: the per-program kernel, then the one-block epilogue with the
device-side commutativity check; --sync: xe_run_batch_device) with packets, descriptors and the
verdict buffer already resident in HBM. For N>1 (torchrun, one rank per GPU) every rank runs its own
16M-packet shard (weak scaling); the timed steps form one shard epoch whose counter map deltas are
all-reduced over RCCL (or replayed in order) inside the timed region. Prints ONE JSON line (rank 0)
with roofline and cpu_baseline objects.

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
    "c5": "C5: C2 parse + per-flow HASH counters {pkts, bytes}, 1M flows, 64 B packets",
    "c3learn": "C3-learn: C3 whose misses (10%, 262,144 new flows) insert the flow (bpf_map_update_elem, BPF_ANY): "
               "map-entry writes, order-dependent; IMIX 64/576/1500 B",
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
ISSUE_PEAK = 256 * 64 * 2.4e9  # lane-ops/s: 256 CU x 64 lanes/clk x 2.4 GHz (SURVEY §8d issue roofline)


def pmc_traffic(name: str, n: int) -> tuple[float | None, str | None]:
    """HBM bytes per launch from the committed rocprofv3 PMC passes of this workload (2 x FETCH_SIZE +
    WRITE_SIZE, MI355X_MICROARCH.md; profiles/r3/<config>_traffic.json, made by scripts/traffic_r3.py),
    when one exists for this exact batch size; else (None, None)."""
    for rnd in ("r3", "r2/final"):  # newest committed PMC passes first
        f = ROOT / "profiles" / rnd / f"{name}_traffic.json"
        if f.exists():
            break
    else:
        return None, None
    d = json.loads(f.read_text())
    if d.get("workload") != name or int(d.get("packets", -1)) != n:
        return None, None
    return float(d["hbm_bytes_per_launch"]), str(f.relative_to(ROOT))


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


def keyed_paths(dev, stream, n: int, reps: int = 3, seq_sample: int = 65536) -> dict:
    """C3-learn (C3 with flow learning: a miss inserts the flow with bpf_map_update_elem) on fresh map
    state each run: the keyed ordered execution over all n packets (SPEC pass, chains per written key,
    xe_internal.h) and, for scale, the one-lane in-order replay (MODE_SEQUENTIAL) on the first
    `seq_sample` packets. Map upload and kernel compilation stay outside the timed region (a 0-packet
    run first); the first run of each path is a warm-up."""
    import torch
    from gobpfld_amd import workloads as W
    from gobpfld_amd.emulator import MODE_SEQUENTIAL, VM, Settings
    umem, descs = W.build_batch("c3learn", 0, n)
    d_umem = torch.from_numpy(umem).to(dev)
    d_desc = torch.from_numpy(descs.view(np.uint8)).to(dev)
    d_ver = torch.zeros(n, dtype=torch.int32, device=dev)
    del umem
    out = {"program": WORKLOADS["c3learn"]}
    for key, mode, cnt, r in (("keyed", 0, n, reps), ("sequential_one_lane", MODE_SEQUENTIAL, seq_sample, 1)):
        times, ks, modes, grids = [], [], set(), 0
        for k in range(r + 1):
            vm = VM(Settings(device=dev.index or 0, mode=mode))
            W.setup_vm(vm, "c3learn")
            vm.run_batch_device(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), 0, stream=stream)  # upload
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            st = vm.run_batch_device(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), cnt,
                                     d_verdicts=d_ver.data_ptr(), stream=stream)
            torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t0
            if k:
                times.append(dt)
                ks.append(st["kernel_ms"])
                modes.add(st["mode_used"])
                grids = st["grid_blocks"]
            vm.close()
        dt = float(np.median(times))
        out[key] = {"value": round(cnt / dt / 1e6, 3), "unit": "Mpkt/s", "packets": cnt, "ms_per_batch": round(dt * 1e3, 3),
                    "device_ms": round(float(np.median(ks)), 3), "mode_used": sorted(modes), "grid_blocks": grids,
                    "runs": len(times)}
    return out


def single_process_multi(args, name: str, n: int) -> None:
    """`bench.py --gpus N` without torchrun: one process drives N GPUs through the C ABI
    (xe_multi_create / xe_run_batch_multi: concurrent shards, RCCL delta all-reduce or in-order
    replay), the path a Go host uses through the FFI alone. Same JSON line as the torchrun form."""
    import torch
    from gobpfld_amd import workloads as W
    from gobpfld_amd.emulator import Multi, VM, Settings
    G = args.gpus
    engine = {"auto": 0, "interp": 1, "jit": 2}[args.engine]
    vms, bufs, sizes = [], [], None
    for k in range(G):
        dev = torch.device("cuda", k)
        umem, descs = W.build_batch(name, k * n, n)
        if k == 0:
            sizes = descs["len"].astype(np.int64)
        bufs.append((torch.from_numpy(umem).to(dev), torch.from_numpy(descs.view(np.uint8)).to(dev),
                     torch.zeros(n, dtype=torch.int32, device=dev)))
        vm = VM(Settings(device=k, engine=engine))
        W.setup_vm(vm, name)
        vms.append(vm)
    mu = Multi(vms)
    args_run = ([u.data_ptr() for u, _, _ in bufs], [u.numel() for u, _, _ in bufs], [d.data_ptr() for _, d, _ in bufs],
                [n] * G)
    for _ in range(args.warmup):
        mu.run(*args_run, d_verdicts=[v.data_ptr() for _, _, v in bufs])
    for k in range(G):
        torch.cuda.synchronize(k)
    kernel_ms, replays, steps_retired = [], 0, 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sts, rep = mu.run(*args_run, d_verdicts=[v.data_ptr() for _, _, v in bufs])
        kernel_ms.append(sts[0]["kernel_ms"])
        steps_retired += sts[0]["steps"]
        replays += int(rep)
    for k in range(G):
        torch.cuda.synchronize(k)
    elapsed = time.perf_counter() - t0
    value = n * G * args.steps / elapsed / 1e6
    avg_kernel_s = float(np.mean(kernel_ms)) / 1e3
    achieved = float(alg_bytes_per_packet(name, sizes).sum()) / avg_kernel_s / 1e9
    traffic, traffic_src = pmc_traffic(name, n)
    cpu = None if args.no_cpu_baseline else cpu_baseline(name, args.cpu_sample)
    print(json.dumps({
        "metric": "Mpkt/s device-resident XDP-emulator verdicts, 64B and 1500B batches", "value": round(value, 3),
        "unit": "Mpkt/s", "n_gpus": G, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int64", "data": "synthetic (deterministic splitmix64 packets, SURVEY §8d)",
        "config": {"workload": WORKLOADS[name], "packets_per_gpu": n, "parallelism": f"dp{G} (one process, xe_run_batch_multi)",
                   "insns_per_packet": round(steps_retired / max(1, n * args.steps), 2), "in_order_replays": replays,
                   "batches": "synchronous xe_run_batch_multi: every step runs the shards and reconciles the maps "
                              "(RCCL delta all-reduce or in-order replay) — an exchange per step, unlike the "
                              "torchrun form's one exchange per epoch of pipelined batches"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None if traffic is None else int(traffic),
                     "traffic_source": traffic_src, "avg_kernel_ms": round(avg_kernel_s * 1e3, 4),
                     "kernel": "device 0 emulator kernel"},
        "cpu_baseline": cpu}), flush=True)
    mu.close()
    for v in vms:
        v.close()


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
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-memory (PCIe-inclusive) measurement")
    ap.add_argument("--no-ordered", action="store_true", help="skip the C2-RMW ordered-path lines (C2 only)")
    ap.add_argument("--sync", action="store_true", help="one synchronous xe_run_batch_device per step (no pipelining)")
    ap.add_argument("--keyed-packets", type=int, default=4 * 1024 * 1024,
                    help="C3-learn batch of the keyed ordered-execution line (C2 runs only)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1 and args.gpus > 1:
        from gobpfld_amd import workloads as W
        n1 = args.packets or (W.CONFIGS[args.config]["n"] // (8 if args.config == "c5" else 1))
        return single_process_multi(args, args.config, n1)
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
    n = args.packets or (W.CONFIGS[name]["n"] // (8 if name == "c5" else 1))
    if name == "c5" and not args.packets:
        n = W.CONFIGS["c5"]["n"] // 8  # 33,554,432 per GPU
    start = rank * n

    # ---- inputs resident in HBM (synthetic packets; shard = contiguous packet index range)
    umem, descs = W.build_batch(name, start, n)
    sizes = descs["len"].astype(np.int64)
    d_umem = torch.from_numpy(umem).to(dev)
    d_desc = torch.from_numpy(descs.view(np.uint8)).to(dev)
    d_ver = torch.zeros(n, dtype=torch.int32, device=dev)

    engine = {"auto": 0, "interp": 1, "jit": 2}[args.engine]
    vm = VM(Settings(device=local, engine=engine))
    W.setup_vm(vm, name)
    maps = list(vm.map_defs)
    stream = torch.cuda.current_stream(dev).cuda_stream
    exchanges = {"exact_sum": 0, "replayed": 0}

    def run() -> dict:
        return vm.run_batch_device(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), n,
                                   d_verdicts=d_ver.data_ptr(), stream=stream)

    # A stream of batches through the pipelined entry point (each batch's conflict check runs on the
    # device; xe_sync completes and, if needed, replays them — all inside the timed region). N > 1:
    # the batches of a call form one shard epoch, reconciled once at its end (footprint check, one
    # RCCL all-reduce per map, or the exact in-order replay) inside the timed region.
    pipelined = not args.sync
    epoch = ShardEpoch(vm, maps, dist, device=dev, stream=stream) if world > 1 else None

    def steps(k: int) -> list[dict]:
        if epoch is not None:
            epoch.begin()
        if pipelined:
            hs = [vm.run_batch_device_async(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), n,
                                            d_verdicts=d_ver.data_ptr(), stream=stream) for _ in range(k)]
            vm.sync()
            sts = [h.stats() for h in hs]
        else:
            sts = [run() for _ in range(k)]
        if epoch is not None:
            x = epoch.exchange([run] * k)
            exchanges["exact_sum" if x["exact_sum"] else "replayed"] += 1
        return sts

    steps(args.warmup)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    kernel_ms, mode, conflicts, steps_retired, status_ok, engines, grid = [], set(), 0, 0, 0, set(), 0
    t0 = time.perf_counter()
    sts = steps(args.steps)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    for st in sts:
        kernel_ms.append(st["kernel_ms"])
        mode.add(st["mode_used"])
        engines.add({1: "interp", 2: "jit"}.get(st["engine_used"], "?"))
        conflicts += st["conflict"]
        steps_retired += st["steps"]
        status_ok += st["status_count"][0]
        grid = st["grid_blocks"]
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

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
    ordered = None
    if rank == 0 and name == "c2" and not args.no_ordered:
        ordered = ordered_paths(d_umem, d_desc, n, dev, stream)
        ordered["keyed_c3learn"] = keyed_paths(dev, stream, args.keyed_packets)
    del umem
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline:
            cpu = cpu_baseline(name, args.cpu_sample)
        hw = {"c2": "64B", "c3": "IMIX 64/576/1500B", "c4": "1500B", "c5": "64B"}.get(name, "64B")
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
                       "packets_per_gpu": n, "packet_size": hw, "parallelism": f"dp{world} (packet shards)",
                       "insns_per_packet": round(insns_per_pkt, 2), "mode": sorted(mode),
                       "engine": sorted(engines),
                       "conflicts": conflicts, "ok_packets_per_step": status_ok // max(1, args.steps),
                       "shard_exchanges": dict(exchanges, per="epoch of the timed steps") if world > 1 else None,
                       "batches": "pipelined (xe_run_batch_device_async, depth 3, device-side conflict check)"
                                  if pipelined else "synchronous (xe_run_batch_device)",
                       "grid": grid},
            "roofline": {"bound": "hbm", "achieved": round(achieved_gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved_gbs / HBM_PEAK_GBS, 5),
                         "traffic": None if traffic is None else int(traffic), "traffic_source": traffic_src,
                         "kernel": "xe_jit_kernel" if engines == {"jit"} else "xe_interp_kernel", "avg_kernel_ms": round(avg_kernel_s * 1e3, 4),
                         "kernel_ms_steps": [round(k, 4) for k in kernel_ms],
                         "alg_bytes_per_launch": int(bytes_per_launch),
                         "alg_bytes_per_packet": ALG_DESC.get(name, "16 desc + min(len,64) header + 4 verdict"),
                         "issue_frac": round(insns_per_pkt * n / avg_kernel_s / ISSUE_PEAK, 5)},
            "cpu_baseline": cpu,
            "e2e": e2e,
            "ordered": ordered,
        }
        print(json.dumps(out), flush=True)
    vm.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
