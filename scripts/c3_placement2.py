#!/usr/bin/env python3
"""C3 run-to-run modes, second experiment: which map buffer's placement decides the kernel time?

Run with the tuning library (XE_LIB=gobpfld_amd/libxdpemu_tuning.so XE_PRINT_ALLOC=1): every run
prints the device addresses of each map's values, slot records and replicas to stderr. Each trial
re-creates the VM behind a spacer allocation of a different size, so the map buffers land elsewhere,
and prints the kernel ms of 4 runs (stdout, one JSON line per trial). Correlating the two logs names
the buffer (and its address bits) that separates the fast and slow modes.
"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gobpfld_amd import workloads as W  # noqa: E402
from gobpfld_amd.emulator import VM, Settings  # noqa: E402


def main() -> None:
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16 * 1024 * 1024
    trials = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    dev = torch.device("cuda", 0)
    umem, descs = W.build_batch("c3", 0, n)
    d_umem = torch.from_numpy(umem).to(dev)
    d_desc = torch.from_numpy(descs.view(np.uint8)).to(dev)
    d_ver = torch.zeros(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    torch.cuda.synchronize()
    for t in range(trials):
        spacer = torch.empty(int((t * 7919 % 13 + 1) * (3 << 22)), dtype=torch.uint8, device=dev)
        vm = VM(Settings(device=0))
        W.setup_vm(vm, "c3")
        print(json.dumps({"trial": t, "spacer_mb": spacer.numel() >> 20}), file=sys.stderr, flush=True)
        ms = []
        for _ in range(5):
            st = vm.run_batch_device(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), n,
                                     d_verdicts=d_ver.data_ptr(), stream=stream)
            ms.append(round(st["kernel_ms"], 4))
        print(json.dumps({"trial": t, "kernel_ms": ms[1:]}), flush=True)
        vm.close()
        del spacer
        torch.cuda.empty_cache()


if __name__ == "__main__":
    t0 = time.time()
    main()
    print(json.dumps({"elapsed_s": round(time.time() - t0, 1)}))
