"""Capture-file ingestion rate: a C2 batch written as a pcap, streamed through
gobpfld_amd.xsk.run_pcap (native pack into pinned staging, H2D overlapped, device run).
One JSON line: packets, seconds, Mpkt/s from the file, device kernel ms."""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from gobpfld_amd import workloads as W  # noqa: E402
from gobpfld_amd import xsk as X  # noqa: E402
from gobpfld_amd.emulator import VM, Settings  # noqa: E402


def write_fixed(path, umem, descs):
    """pcap of the batch, vectorised (every record built with numpy, no per-packet Python)."""
    n = len(descs)
    lens = descs["len"].astype(np.int64)
    rec = 16 + lens
    offs = np.zeros(n + 1, np.int64)
    offs[1:] = np.cumsum(rec)
    out = np.zeros(24 + int(offs[-1]), np.uint8)
    out[:24] = np.frombuffer(np.array([0xA1B2C3D4, 0x00040002, 0, 0, 65535, 1], "<u4").tobytes(), np.uint8)
    hdr = np.zeros((n, 4), "<u4")
    hdr[:, 0] = np.arange(n) // 1_000_000
    hdr[:, 1] = np.arange(n) % 1_000_000
    hdr[:, 2] = lens
    hdr[:, 3] = lens
    hb = hdr.view(np.uint8).reshape(n, 16)
    base = 24 + offs[:-1]
    out[(base[:, None] + np.arange(16)).ravel()] = hb.ravel()
    for L in np.unique(lens):  # packets of one length at a time
        sel = np.nonzero(lens == L)[0]
        src = descs["addr"][sel].astype(np.int64)[:, None] + np.arange(L)
        out[(base[sel, None] + 16 + np.arange(L)).ravel()] = umem[src.ravel()]
    out.tofile(path)


ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--packets", type=int, default=1 << 22)
ap.add_argument("--batch", type=int, default=1 << 20)
ap.add_argument("--repeat", type=int, default=3)
a = ap.parse_args()
path = Path(os.environ.get("TMPDIR", "/tmp")) / f"xe_{a.config}.pcap"
umem, descs = W.build_batch(a.config, 0, a.packets)
t = time.perf_counter()
write_fixed(path, umem, descs)
wt = time.perf_counter() - t
vm = VM(Settings())
W.setup_vm(vm, a.config)
pc = X.PcapFile(path)
best = None
for _ in range(a.repeat):
    pc.rewind()
    r = X.run_pcap(vm, pc, batch=a.batch, staging_bytes=a.batch * 1600)
    if best is None or r.seconds < best.seconds:
        best = r
print(json.dumps({"config": a.config, "packets": best.packets, "batches": best.batches, "seconds": round(best.seconds, 4),
                  "mpps_from_pcap": round(best.mpps, 2), "device_ms": round(best.device_ms, 3),
                  "file_bytes": path.stat().st_size, "status_ok": best.status_count[0], "write_s": round(wt, 2)}))
pc.close()
vm.close()
path.unlink()
