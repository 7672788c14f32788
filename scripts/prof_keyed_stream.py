#!/usr/bin/env python3
"""Host-side marks (XE_HOST_TIMING, tuning build) of a stream of keyed batches on one VM: where the wall
time of a steady keyed batch goes. python scripts/prof_keyed_stream.py <config> [batches] [packets]"""
import importlib.util
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
B = importlib.util.module_from_spec(spec)
spec.loader.exec_module(B)


def main():
    import torch
    from gobpfld_amd import workloads as W
    from gobpfld_amd.emulator import VM, Settings
    name = sys.argv[1]
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 4 * 1024 * 1024
    dev = torch.device("cuda", 0)
    bufs = [B.device_batch(name, k * n, n, dev) for k in range(nb)]
    d_ver = torch.zeros(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    vm = VM(Settings(device=0))
    W.setup_vm(vm, name)
    stream = torch.cuda.current_stream(dev).cuda_stream
    for k in range(nb):
        b = bufs[k]
        t0 = time.perf_counter()
        st = vm.run_batch_device(b[0].data_ptr(), b[0].numel(), b[1].data_ptr(), n, d_verdicts=d_ver.data_ptr(), stream=stream)
        torch.cuda.synchronize()
        print(f"batch {k}: {1e3 * (time.perf_counter() - t0):.1f} ms wall, {st['kernel_ms']:.3f} ms device, mode {st['mode_used']}",
              file=sys.stderr, flush=True)
    vm.close()


if __name__ == "__main__":
    main()
