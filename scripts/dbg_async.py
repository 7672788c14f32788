"""Debug: the first pipelined batch of tests/test_async.py step by step (engine given on argv)."""
import faulthandler
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
faulthandler.enable()
import torch  # noqa: E402
from gobpfld_amd.emulator import MAP_ARRAY, VM, MapDef, Settings  # noqa: E402
from test_async import batches, prog_mixed  # noqa: E402

engine = int(sys.argv[1]) if len(sys.argv) > 1 else 0
vm = VM(Settings(engine=engine))
m = vm.add_map(MapDef(MAP_ARRAY, 4, 16, 8))
vm.set_entrypoint(vm.add_raw_program(prog_mixed()))
print("setup", flush=True)
vm.prepare()
print("prepared", flush=True)
(u, d), = batches(1, 4096, set())
du = torch.from_numpy(u).cuda()
dd = torch.from_numpy(d.view(np.uint8)).cuda()
dv = torch.zeros(len(d), dtype=torch.int32, device="cuda")
st = vm.run_batch_device(du.data_ptr(), du.numel(), dd.data_ptr(), len(d), d_verdicts=dv.data_ptr())
print("sync batch", st, flush=True)
h = vm.run_batch_device_async(du.data_ptr(), du.numel(), dd.data_ptr(), len(d), d_verdicts=dv.data_ptr())
print("queued", flush=True)
print("async", h.stats(), flush=True)
