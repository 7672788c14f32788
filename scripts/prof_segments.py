"""Round 6: a work queue whose pops reach elements pushed earlier in the same batch (tests/test_segments.py
prog_work_queue: 40 preloaded elements, a pop on half the packets, a push on every packet), run as
packet-order segments (XE_MODE_AUTO -> XE_MODE_SEGMENTS) against the one-lane in-order replay
(Settings(mode=SEQUENTIAL)) on the same batch; both checked against each other (verdicts, queue contents).

    python scripts/prof_segments.py [packets]   ->  one JSON line
"""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from gobpfld_amd.emulator import MODE_SEQUENTIAL, Settings  # noqa: E402
from parity import _dump, packets, setup_one  # noqa: E402
from test_segments import _case  # noqa: E402


def run(mode, n, name):
    import torch
    prog, maps, entries = _case(name)
    umem, descs = packets(n, 64, seed=77)
    vm, idx = setup_one(None, prog, maps, Settings(mode=mode), entries)
    vm.prepare()
    d_umem = torch.from_numpy(umem).cuda()
    d_desc = torch.from_numpy(descs.view(np.uint8)).cuda()
    d_ver = torch.zeros(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    st = vm.run_batch_device(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), n, d_verdicts=d_ver.data_ptr())
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    out = (d_ver.cpu().numpy().copy(), [_dump(vm, m) for m in idx])
    vm.close()
    return st, wall, out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    res = {"what": __doc__.strip().splitlines()[0], "packets": n, "runs": {}}
    outs = {}
    for name in ("queue", "queue_lru"):
        for label, mode in (("auto", 0), ("sequential", MODE_SEQUENTIAL)):
            n_run = n if label == "auto" else min(n, 65536)  # the replay at 65,536 packets (its rate is flat)
            run(mode, min(n_run, 65536), name)  # warm-up: the verdict-only kernel compiled, the maps placed
            st, wall, out = run(mode, n_run, name)
            res["runs"][f"{name}/{label}"] = {"packets": n_run, "mode_used": st["mode_used"], "wall_ms": round(wall * 1e3, 2),
                                              "kernel_ms": round(st["kernel_ms"], 2),
                                              "mpkts": round(n_run / wall / 1e6, 3)}
            outs[(name, label)] = (n_run, out)
            print(name, label, res["runs"][f"{name}/{label}"], file=sys.stderr, flush=True)
    # the same batch prefix through both paths agrees (verdicts of the first 65,536 packets)
    for name in ("queue", "queue_lru"):
        (na, (va, _)), (ns, (vs, _)) = outs[(name, "auto")], outs[(name, "sequential")]
        res["runs"][f"{name}/agree_first_{ns}"] = bool((va[:ns] == vs).all()) if na >= ns else None
    print(json.dumps(res))


if __name__ == "__main__":
    main()
