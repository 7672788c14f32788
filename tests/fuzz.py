"""Random-program generator for differential tests (oracle vs host simulation vs device).

Programs are raw eBPF slots biased toward the emulator's interesting paths: typed registers and
pointer arithmetic (ctx/packet/stack/map-value pointers), ValueMemory aliasing on the stack,
packet loads/stores, map helpers with stack keys, atomics, 32/64-bit ALU with edge immediates,
signed/unsigned jumps (forward, plus occasional back edges under a step budget), and illegal
registers / out-of-range jump targets that end in VM errors. Every run is deterministic in `seed`.
"""
from __future__ import annotations

import numpy as np

from gobpfld_amd.asm import (ADD, ALU, ALU64, AND, ARSH, ATOMIC, CALL, DIV, DW, EXIT, JEQ, JGE,
                             JGT, JMP, JMP32, JNE, JSGE, JSGT, JSLE, JSLT, LDX, LSH, MEM, MOD, MOV,
                             MUL, NEG, OR, RSH, ST, STX, SUB, XOR, B, H, K, W, X, raw)
from gobpfld_amd.emulator import MAP_ARRAY, MAP_HASH, MapDef, Settings

SIZES = [B, H, W, DW]
ALU_OPS = [ADD, SUB, MUL, DIV, OR, AND, LSH, RSH, MOD, XOR, MOV, ARSH]
JMP_OPS = [JEQ, JGT, JGE, JNE, JSGT, JSGE, JSLT, JSLE]
EDGE_IMMS = [0, 1, -1, 2, 7, 8, 14, 23, 31, 32, 63, 64, 0x7FFFFFFF, -0x80000000, 0xFF, 0xFFFF]

MAPS = [
    (MapDef(MAP_ARRAY, 4, 8, 16), None),
    (MapDef(MAP_HASH, 16, 16, 64), None),
    (MapDef(MAP_ARRAY, 4, 16, 4), None),
]


def _entries(rng):
    ents = {1: []}
    for _ in range(int(rng.integers(0, 12))):
        k = rng.integers(0, 4, size=16, dtype=np.uint8).tobytes()
        v = rng.integers(0, 256, size=16, dtype=np.uint8).tobytes()
        ents[1].append((k, v))
    return ents


def _reg(rng, allow_bad=True):
    """R0-R9 mostly; R10 (readable only through Copy, registers.go:90-114) and R11+ rarely."""
    r = int(rng.integers(0, 10))
    x = rng.random()
    if allow_bad and x < 0.025:
        r = 10
    elif allow_bad and x < 0.03:
        r = 11 + int(rng.integers(0, 5))
    return r


def gen_program(seed: int, length: int = 48):
    """-> (raw slots, maps, entries, settings)"""
    rng = np.random.default_rng(seed)
    p: list[int] = []
    # prologue: packet pointers, a stack key, a map lookup with a null check
    p += [raw(LDX | MEM | W, 2, 1, 0), raw(LDX | MEM | W, 3, 1, 4), raw(ALU64 | MOV | X, 6, 1)]
    if rng.random() < 0.7:
        p += [raw(ST | MEM | W, 10, 0, -4, int(rng.integers(0, 20))),
              raw(ST | MEM | W, 10, 0, -16, int(rng.integers(0, 3))),
              raw(ST | MEM | W, 10, 0, -12, 0), raw(ST | MEM | DW, 10, 0, -8, 0)]
        m = int(rng.integers(1, 4))
        key_off = -16 if m == 2 else -4
        p += [raw(0x18, 1, 1, 0, m), raw(0, 0, 0, 0, 0), raw(ALU64 | MOV | X, 2, 10),
              raw(ALU64 | ADD | K, 2, 0, 0, key_off), raw(JMP | CALL, 0, 0, 0, 1), raw(ALU64 | MOV | X, 7, 0)]
        p += [raw(JMP | JEQ | K, 0, 0, 2, 0), raw(LDX | MEM | DW, 8, 0, 0), raw(ALU64 | MOV | X, 9, 0)]
        # restore the packet pointers clobbered by the call (R1-R5 are caller-saved)
        p += [raw(LDX | MEM | W, 2, 6, 0), raw(LDX | MEM | W, 3, 6, 4)]
    body_start = len(p)
    n = int(rng.integers(length // 2, length))
    back_edges = rng.random() < 0.2
    for i in range(n):
        pc = len(p)
        c = rng.random()
        if c < 0.22:  # ALU
            op = ALU_OPS[int(rng.integers(len(ALU_OPS)))]
            cls = ALU64 if rng.random() < 0.7 else ALU
            if rng.random() < 0.5:
                imm = EDGE_IMMS[int(rng.integers(len(EDGE_IMMS)))] if rng.random() < 0.6 else int(rng.integers(-100, 100))
                p.append(raw(cls | op | K, _reg(rng), 0, 0, imm))
            else:
                p.append(raw(cls | op | X, _reg(rng), _reg(rng)))
        elif c < 0.27:
            p.append(raw((ALU64 if rng.random() < 0.5 else ALU) | NEG, _reg(rng)))
        elif c < 0.30:
            p.append(raw(ALU | 0xD0 | (X if rng.random() < 0.5 else K), _reg(rng), 0, 0,
                         [16, 32, 64][int(rng.integers(3))]))
        elif c < 0.40:  # pointer arithmetic on a packet/stack pointer
            d = [2, 10, 6, 7, 8][int(rng.integers(5))] if rng.random() < 0.8 else _reg(rng)
            dst = int(rng.integers(0, 10))
            p += [raw(ALU64 | MOV | X, dst, d), raw(ALU64 | ADD | K, dst, 0, 0, int(rng.integers(-24, 70)))]
        elif c < 0.55:  # loads
            s = SIZES[int(rng.integers(4))]
            src = [2, 10, 6, 7, 0][int(rng.integers(5))] if rng.random() < 0.7 else _reg(rng)
            off = int(rng.integers(-8, 48)) if src != 10 else -int(rng.integers(1, 40))
            p.append(raw(LDX | MEM | s, _reg(rng), src, off))
        elif c < 0.68:  # stores
            s = SIZES[int(rng.integers(4))]
            dst = [2, 10, 7, 0][int(rng.integers(4))] if rng.random() < 0.8 else _reg(rng)
            off = int(rng.integers(-8, 64)) if dst != 10 else -int(rng.integers(1, 40))
            if rng.random() < 0.5:
                p.append(raw(ST | MEM | s, dst, 0, off, int(rng.integers(-300, 300))))
            else:
                p.append(raw(STX | MEM | s, dst, _reg(rng), off))
        elif c < 0.72:  # atomics (ADD only translates; fetch form sometimes)
            s = DW if rng.random() < 0.5 else W
            dst = [7, 10, 2][int(rng.integers(3))]
            off = -8 if dst == 10 else int(rng.integers(0, 16))
            p.append(raw(STX | ATOMIC | s, dst, _reg(rng), off, 1 if rng.random() < 0.3 else 0))
        elif c < 0.88:  # conditional jumps
            op = JMP_OPS[int(rng.integers(len(JMP_OPS)))]
            cls = JMP if rng.random() < 0.7 else JMP32
            if back_edges and rng.random() < 0.25:
                off = -int(rng.integers(1, max(2, pc - body_start + 1)))
            else:
                off = int(rng.integers(0, 12))
            if rng.random() < 0.5:
                p.append(raw(cls | op | K, _reg(rng), 0, off, EDGE_IMMS[int(rng.integers(len(EDGE_IMMS)))]))
            else:
                p.append(raw(cls | op | X, _reg(rng), _reg(rng), off))
        elif c < 0.92:  # helpers (lookup/update/delete/smp-id, and an unknown id)
            h = [1, 2, 3, 14, 8, 1][int(rng.integers(6))]
            m = int(rng.integers(1, 4))
            p += [raw(0x18, 1, 1, 0, m), raw(0, 0, 0, 0, 0), raw(ALU64 | MOV | X, 2, 10),
                  raw(ALU64 | ADD | K, 2, 0, 0, -16 if m == 2 else -4)]
            if h == 2:
                p += [raw(ALU64 | MOV | X, 3, 10), raw(ALU64 | ADD | K, 3, 0, 0, -32),
                      raw(ST | MEM | DW, 10, 0, -32, int(rng.integers(0, 9))), raw(ST | MEM | DW, 10, 0, -24, 1),
                      raw(ALU64 | MOV | K, 4, 0, 0, int(rng.integers(0, 3)))]
            p.append(raw(JMP | CALL, 0, 0, 0, h))
        elif c < 0.94:
            p += [raw(0x18, _reg(rng, False), 0, 0, int(rng.integers(-2**31, 2**31))), raw(0, 0, 0, 0, int(rng.integers(-2**31, 2**31)))]
        elif c < 0.96:
            p.append(raw(JMP | 0x00, 0, 0, int(rng.integers(0, 6))))  # ja
        else:
            p.append(raw(ALU64 | MOV | K, 0, 0, 0, int(rng.integers(0, 5))))
            p.append(raw(JMP | EXIT))
    p.append(raw(ALU64 | MOV | K, 0, 0, 0, 2))
    p.append(raw(JMP | EXIT))
    # occasionally a target past the end (BAD_PC fallthrough) is left in by the jumps above
    settings = Settings(max_steps=int(rng.integers(200, 2000)) if back_edges else 0)
    return p, list(MAPS), _entries(rng), settings
