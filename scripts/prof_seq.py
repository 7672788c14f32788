#!/usr/bin/env python3
"""The one-lane in-order replay alone, for profiling (rocprofv3 --kernel-trace / --pmc): `config` in
MODE_SEQUENTIAL over the first `packets` packets of its bench batch, one warm-up run and `reps` timed
runs; prints kernel_ms per run. The dispatch's VGPR / SGPR counts in a kernel trace tell the scalar
replay variant (xe_jit.cpp XE_JV_SEQ) from the plain kernel.
  python scripts/prof_seq.py c2rmw [packets] [reps]"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    import torch
    from gobpfld_amd import workloads as W
    from gobpfld_amd.emulator import MODE_SEQUENTIAL, VM, Settings
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    B = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(B)
    name = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    dev = torch.device("cuda", 0)
    d_umem, d_desc, _ = B.device_batch(name, 0, n, dev)
    d_ver = torch.zeros(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    vm = VM(Settings(device=0, mode=MODE_SEQUENTIAL))
    W.setup_vm(vm, name)
    stream = torch.cuda.current_stream(dev).cuda_stream
    for k in range(reps + 1):
        t0 = time.perf_counter()
        st = vm.run_batch_device(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), n, d_verdicts=d_ver.data_ptr(), stream=stream)
        torch.cuda.synchronize()
        print(f"{name} run {k}: {st['kernel_ms']:.3f} ms kernel, {1e3 * (time.perf_counter() - t0):.1f} ms wall, "
              f"{n / st['kernel_ms'] / 1e3:.3f} Mpkt/s, mode {st['mode_used']}", flush=True)
    vm.close()


if __name__ == "__main__":
    main()
