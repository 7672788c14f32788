#!/usr/bin/env python3
"""C3 run-to-run bimodality: which allocation decides the kernel time?

In ONE process: the C3 kernel time over several trials where either
  * the VM (hash slot records, values, replicas, aux) is re-created — new map allocations — or
  * the packet buffer (UMEM, ~6.5 GB of IMIX frames) is re-allocated (the old block released first,
    so the caching allocator cannot hand the same one back),
while the other stays. Prints one JSON line per trial: what changed and the kernel ms of 4 runs.
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
    trials = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    dev = torch.device("cuda", 0)
    umem, descs = W.build_batch("c3", 0, n)
    h_umem = torch.from_numpy(umem)
    d_desc = torch.from_numpy(descs.view(np.uint8)).to(dev)
    d_ver = torch.zeros(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def new_umem():
        t = h_umem.to(dev)
        torch.cuda.synchronize()
        return t

    def new_vm():
        vm = VM(Settings(device=0))
        W.setup_vm(vm, "c3")
        return vm

    def times(vm, d_umem):
        out = []
        for _ in range(5):
            st = vm.run_batch_device(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), n,
                                     d_verdicts=d_ver.data_ptr(), stream=stream)
            out.append(round(st["kernel_ms"], 4))
        return out[1:]

    d_umem = new_umem()
    vm = new_vm()
    print(json.dumps({"trial": 0, "changed": "start", "umem_ptr": hex(d_umem.data_ptr()), "kernel_ms": times(vm, d_umem)}),
          flush=True)
    for t in range(1, trials + 1):
        vm.close()
        vm = new_vm()
        print(json.dumps({"trial": t, "changed": "vm", "kernel_ms": times(vm, d_umem)}), flush=True)
        del d_umem
        torch.cuda.empty_cache()
        # keep a spacer so the next UMEM block lands at another address
        spacer = torch.empty(int((t * 37 % 11 + 1) * (1 << 28)), dtype=torch.uint8, device=dev)
        d_umem = new_umem()
        del spacer
        print(json.dumps({"trial": t, "changed": "umem", "umem_ptr": hex(d_umem.data_ptr()),
                          "kernel_ms": times(vm, d_umem)}), flush=True)
    vm.close()


if __name__ == "__main__":
    t0 = time.time()
    main()
    print(json.dumps({"elapsed_s": round(time.time() - t0, 1)}))
