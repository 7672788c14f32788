"""Kernel timeline of the last N dispatches in a rocprofv3 rocpd database (rocprofv3 -d DIR -o run):
start offset, duration, grid and register / LDS use per dispatch.

usage: python scripts/rocpd_timeline.py DIR [N]
"""
import glob
import sqlite3
import sys

db = glob.glob(f"{sys.argv[1]}/**/*.db", recursive=True)[0]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 45
rows = list(sqlite3.connect(db).execute(
    "select name, start, end, duration, grid_x, vgpr_count, lds_size from kernels order by start"))[-n:]
t0 = rows[0][1]
for name, start, _, dur, grid, vgpr, lds in rows:
    print(f"{(start - t0) / 1e3:10.1f} us  dur {dur / 1e3:8.1f} us  grid {grid:8d} vgpr {vgpr:3d} lds {lds:6d}  {name[:64]}")
