"""Case file for the sanitizer harness (tests/sanitize/san_driver.cpp).

Writes every KAT (tests/kats.py), a slice of the differential fuzzer's programs (tests/fuzz.py) and the
BASELINE configs at small sizes as one little-endian binary file that the ASan/UBSan builds of the oracle
and of the host-simulation library both run; the driver compares them bit for bit.

  magic "XECASES1", u32 ncases, then per case:
    u32 len + name; u64 max_steps; u32 mode
    u32 nprogs; per program: u32 n, u64 insns[n]
    u32 nmaps;  per map: u32 type, key_size, value_size, max_entries, flags; u32 init_len + bytes;
                u32 nentries; per entry: u8 push, key (key_size bytes unless push), value (value_size)
    u32 npkts; u64 umem_len + bytes; descs (16 B each: u64 addr, u32 len, u32 options)
"""
from __future__ import annotations

import struct
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
sys.path.insert(0, str(HERE.parent.parent))


def _case(name, program, maps, entries, umem, descs, settings=None):
    progs = program if program and isinstance(program[0], list) else [program]
    out = [struct.pack("<I", len(name)), name.encode()]
    out.append(struct.pack("<QI", settings.max_steps if settings else 1 << 20, settings.mode if settings else 0))
    out.append(struct.pack("<I", len(progs)))
    for p in progs:
        arr = np.asarray(p, dtype=np.uint64)
        out += [struct.pack("<I", len(arr)), arr.astype("<u8").tobytes()]
    out.append(struct.pack("<I", len(maps)))
    for i, (mdef, init) in enumerate(maps):
        out.append(struct.pack("<5I", mdef.type, mdef.key_size, mdef.value_size, mdef.max_entries, mdef.flags))
        init = bytes(init or b"")
        out += [struct.pack("<I", len(init)), init]
        ents = (entries or {}).get(i, [])
        out.append(struct.pack("<I", len(ents)))
        for k, v in ents:
            if k is None:
                out += [b"\1", bytes(v).ljust(mdef.value_size, b"\0")[: mdef.value_size]]
            else:
                out += [b"\0", bytes(k).ljust(mdef.key_size, b"\0")[: mdef.key_size],
                        bytes(v).ljust(mdef.value_size, b"\0")[: mdef.value_size]]
    descs = np.ascontiguousarray(descs)
    out.append(struct.pack("<IQ", len(descs), umem.size))
    out += [umem.astype(np.uint8).tobytes(), descs.tobytes()]
    return b"".join(out)


def build_cases() -> list[bytes]:
    from fuzz import gen_program
    from kats import KATS
    from parity import config_case, packets
    from test_fuzz_cpu import fuzz_packets
    cases = []
    for k in KATS:
        umem, descs = packets(4, k["pkt"], seed=7)
        cases.append(_case("kat:" + k["name"], k["program"], k["maps"], k["entries"], umem, descs))
    for seed in range(0, 480, 4):
        prog, maps, entries, settings = gen_program(seed)
        umem, descs = fuzz_packets(seed)
        cases.append(_case(f"fuzz:{seed}", prog, maps, entries, umem, descs, settings))
    for name in ("c1", "c2", "c3", "c4", "c5", "c3learn"):
        prog, maps, entries, umem, descs = config_case(name, 256, flows_cap=512)
        cases.append(_case("config:" + name, prog, maps, entries, umem, descs))
    return cases


def write(path: Path) -> int:
    cases = build_cases()
    path.write_bytes(b"XECASES1" + struct.pack("<I", len(cases)) + b"".join(cases))
    return len(cases)


if __name__ == "__main__":
    print(write(Path(sys.argv[1] if len(sys.argv) > 1 else "/tmp/xe_cases.bin")), "cases")
