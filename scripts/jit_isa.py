#!/usr/bin/env python3
"""Offline ISA inspection of the JIT kernel for a config (CPU only): writes the generated source,
compiles it with hipcc for gfx950 (-S), and prints resource usage + instruction-class counts.

  python scripts/jit_isa.py c2 [-DXE_PEND_MODE=2 ...]
  python scripts/jit_isa.py c3learn --keyed     (the keyed variant: XE_MODE_SPEC / XE_MODE_CHAIN)
"""
import ctypes as C
import re
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from gobpfld_amd import workloads as W  # noqa: E402
from gobpfld_amd._native import PRODUCT_LIB  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c2"
defs = [a for a in sys.argv[2:] if a != "--keyed"]
keyed = "--keyed" in sys.argv[2:]
lib = C.CDLL(str(PRODUCT_LIB))
lib.xe_translate_uops.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]
lib.xe_jit_source.argtypes = [C.c_void_p, C.c_size_t, C.c_char_p, C.c_size_t]
lib.xe_jit_source_geom.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_uint32, C.c_char_p, C.c_size_t]
raw = np.ascontiguousarray(np.asarray(W.CONFIGS[name]["program"](), dtype=np.uint64))
u = np.zeros(len(raw) * 16, dtype=np.uint8)
n = lib.xe_translate_uops(raw.ctypes.data, len(raw), u.ctypes.data, len(raw))
buf = C.create_string_buffer(1 << 22)
# the config's real map geometry (kind, key, value, max entries, cap, key words, replicas)
geom = []
for mdef, _ in W.workload_maps(name):
    if mdef.type in (1, 5):  # HASH / PERCPU_HASH
        cap = 16
        while cap < 2 * mdef.max_entries:
            cap <<= 1
        geom += [2, mdef.key_size, mdef.value_size, mdef.max_entries, cap, (mdef.key_size + 7) // 8, 1]
    else:
        geom += [1, mdef.key_size, mdef.value_size, mdef.max_entries, 0, 0, 16]
g = np.asarray(geom, dtype=np.uint32)
lib.xe_jit_source_geom(u.ctypes.data, n, g.ctypes.data, len(geom) // 7, buf, len(buf))
src = buf.value.decode()
if keyed:
    src = src.replace("#define XE_KEYED 0", "#define XE_KEYED 1")
out = Path("/tmp") / f"xe_jit_{name}{'_keyed' if keyed else ''}"
out.mkdir(exist_ok=True)
(out / "k.hip").write_text('#include <hip/hip_runtime.h>\n' + src)
cmd = ["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "--cuda-device-only", "-S", "-std=c++17",
       "-I", str(ROOT / "gobpfld_amd" / "csrc"), "-Wno-unused-label", "-Wno-unused-variable", *defs,
       "-o", str(out / "k.s"), str(out / "k.hip")]
subprocess.run(cmd, check=True)
asm = (out / "k.s").read_text()
body = asm.split("xe_jit_kernel")[1] if "xe_jit_kernel" in asm else asm
for key in ["vgpr_count", "sgpr_count", "private_segment_fixed_size", "group_segment_fixed_size"]:
    m = re.search(r"\.%s:\s+(\d+)" % key, asm)
    print(f"{key}: {m.group(1) if m else '?'}")
ins = re.findall(r"^\s+([a-z_0-9]+)\s", asm, re.M)
cls = {}
for i in ins:
    k = i.split("_")[0]
    if i.startswith(("global_", "flat_", "scratch_", "buffer_", "ds_")):
        k = i.split("_")[0] + ("_atomic" if "atomic" in i else "")
    cls[k] = cls.get(k, 0) + 1
print("instructions:", len(ins))
print({k: v for k, v in sorted(cls.items(), key=lambda x: -x[1]) if v > 20 or k in ("flat", "flat_atomic", "scratch", "ds", "ds_atomic")})
print("asm:", out / "k.s")
