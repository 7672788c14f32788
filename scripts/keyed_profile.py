"""Keyed ordered execution on C3-learn (fresh map state per run): per-run wall time and the stats
line, for `rocprofv3 --kernel-trace --stats -- python scripts/keyed_profile.py` (which kernel of the
SPEC pass / build / parallel pass / chains costs what).

usage: python scripts/keyed_profile.py [packets] [runs]
"""
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from gobpfld_amd import workloads as W  # noqa: E402
from gobpfld_amd.emulator import VM, Settings  # noqa: E402


def main() -> None:
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4 << 20
    runs = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    dev = torch.device("cuda", 0)
    umem, descs = W.build_batch("c3learn", 0, n)
    d_umem = torch.from_numpy(umem).to(dev)
    d_desc = torch.from_numpy(descs.view(np.uint8)).to(dev)
    d_ver = torch.zeros(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    for k in range(runs):
        vm = VM(Settings(device=0))
        W.setup_vm(vm, "c3learn")
        vm.run_batch_device(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), 0, stream=stream)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        st = vm.run_batch_device(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), n, d_verdicts=d_ver.data_ptr(),
                                 stream=stream)
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        print(json.dumps({"run": k, "ms": round(dt * 1e3, 3), "mpkts": round(n / dt / 1e6, 1), "mode_used": st["mode_used"],
                          "device_ms": round(st["kernel_ms"], 3), "grid": st["grid_blocks"]}), flush=True)
        vm.close()


if __name__ == "__main__":
    main()
