#!/usr/bin/env python3
"""Where a keyed C3-LRU batch spends its device time: bench.py keyed_paths("c3lru") (4M packets, fresh
maps, two runs after a warm-up) with a short one-lane sample, under rocprofv3 --kernel-trace --stats.

  rocprofv3 --kernel-trace --stats -d OUT -o run --output-format csv -- python3 scripts/prof_c3lru.py
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
stream = torch.cuda.current_stream(dev).cuda_stream
r = bench.keyed_paths(dev, stream, 4 * 1024 * 1024, reps=2, seq_sample=1024, name="c3lru")
print(json.dumps({k: v for k, v in r.items() if k != "program"}), flush=True)
