"""Test-only text -> raw encoder for the instruction text format of ebpf/asm_test.bpfasm.

Independent of the reference's assembler (ebpf/asm.go): it maps each line of the fixture to the
8-byte encoding its String() form denotes (opcodes per ebpf/ebpf.go and ebpf/decode.go), so that
`decode_text(encode(file)) == file` restates TestDecodeEncodeSymmetry (ebpf/asm_test.go:16-49)
against our oracle's decoder.
"""
from __future__ import annotations

import re

SIZES = {"u32": 0x00, "u16": 0x08, "u8": 0x10, "u64": 0x18}
ALU = {"+=": 0x00, "-=": 0x10, "*=": 0x20, "/=": 0x30, "|=": 0x40, "&=": 0x50, "<<=": 0x60,
       ">>=": 0x70, "%=": 0x90, "^=": 0xa0, "=": 0xb0, "s>>=": 0xc0}
JMP = {"==": 0x10, ">": 0x20, ">=": 0x30, "&": 0x40, "!=": 0x50, "s>": 0x60, "s>=": 0x70,
       "<": 0xa0, "<=": 0xb0, "s<": 0xc0, "s<=": 0xd0}
ATOMIC = {"+=": 0x00, "-=": 0x10, "&=": 0x50, "|=": 0x40, "^=": 0xa0}


def raw(op: int, dst: int = 0, src: int = 0, off: int = 0, imm: int = 0) -> int:
    return (op & 0xff) | (dst & 0xf) << 8 | (src & 0xf) << 12 | (off & 0xffff) << 16 | (imm & 0xffffffff) << 32


def _off(sign: str, val: str) -> int:
    return -int(val) if sign == "-" else int(val)


def encode_line(line: str) -> list[int]:
    s = line.strip()
    R = r"([rw])(\d+)"
    if s == "exit":
        return [raw(0x95)]
    if s == "nop":
        return []  # second slot of the preceding LD_IMM64 (decode.go:34 emits it as Nop)
    if m := re.fullmatch(r"r(\d+) = (\d+) ll", s):
        v = int(m[2])
        return [raw(0x18, int(m[1]), imm=v & 0xffffffff), raw(0, imm=v >> 32)]
    if m := re.fullmatch(r"goto ([+-]\d+)", s):
        return [raw(0x05, off=int(m[1]))]
    if m := re.fullmatch(r"call (\d+)#\w*", s):
        return [raw(0x85, imm=int(m[1]))]
    if m := re.fullmatch(r"call ([+-]\d+)", s):
        return [raw(0x85, src=1, imm=int(m[1]))]
    if m := re.fullmatch(r"if " + R + r" (\S+) (?:" + R + r"|(-?\d+)) goto ([+-]\d+)", s):
        cls = 0x05 if m[1] == "r" else 0x06
        if m[4] is not None:
            return [raw(cls | JMP[m[3]] | 0x08, int(m[2]), int(m[5]), off=int(m[7]))]
        return [raw(cls | JMP[m[3]], int(m[2]), off=int(m[7]), imm=int(m[6]))]
    if m := re.fullmatch(r"r(\d+) = (be|le)(\d+) r\d+", s):
        return [raw(0x04 | 0xd0 | (0x08 if m[2] == "be" else 0), int(m[1]), imm=int(m[3]))]
    if m := re.fullmatch(R + r" = -[rw]\d+", s):
        return [raw((0x07 if m[1] == "r" else 0x04) | 0x80, int(m[2]))]
    if m := re.fullmatch(r"r(\d+) = \*\((u\d+) \*\)\(r(\d+) ([+-]) (\d+)\)", s):
        return [raw(0x61 | SIZES[m[2]], int(m[1]), int(m[3]), off=_off(m[4], m[5]))]
    if m := re.fullmatch(r"\*\((u\d+) \*\)\(r(\d+) ([+-]) (\d+)\) = r(\d+)", s):
        return [raw(0x63 | SIZES[m[1]], int(m[2]), int(m[5]), off=_off(m[3], m[4]))]
    if m := re.fullmatch(r"\*\((u\d+) \*\)\(r(\d+) ([+-]) (\d+)\) = (-?\d+)", s):
        return [raw(0x62 | SIZES[m[1]], int(m[2]), off=_off(m[3], m[4]), imm=int(m[5]))]
    if m := re.fullmatch(r"lock \*\((u\d+) \*\)\(r(\d+) ([+-]) (\d+)\) (\S+) [rw](\d+)", s):
        return [raw(0xc3 | SIZES[m[1]], int(m[2]), int(m[6]), off=_off(m[3], m[4]), imm=ATOMIC[m[5]])]
    if m := re.fullmatch(r"([rw])(\d+) = xchg\(r(\d+) ([+-]) (\d+), [rw]\d+\)", s):
        size = 0x18 if m[1] == "r" else 0x00
        return [raw(0xc3 | size, int(m[3]), int(m[2]), off=_off(m[4], m[5]), imm=0xe1)]
    if m := re.fullmatch(r"([rw])0 = cmpxchg\(r(\d+) ([+-]) (\d+), [rw]0, [rw](\d+)\)", s):
        size = 0x18 if m[1] == "r" else 0x00
        return [raw(0xc3 | size, int(m[2]), int(m[5]), off=_off(m[3], m[4]), imm=0xf1)]
    if m := re.fullmatch(r"r0 = ntohl\(\((u\d+)\) \(\(\(struct sk_buff \*\) r6\)->data\[(-?\d+)\]\)\)", s):
        return [raw(0x20 | SIZES[m[1]], imm=int(m[2]))]
    if m := re.fullmatch(r"r0 = ntohl\(\((u\d+)\) \(\(\(struct sk_buff \*\) r6\)->data\[r(\d+) ([+-]) (\d+)\]\)\)", s):
        return [raw(0x40 | SIZES[m[1]], src=int(m[2]), imm=_off(m[3], m[4]))]
    if m := re.fullmatch(R + r" (\S+) (?:" + R + r"|(-?\d+))", s):
        cls = 0x07 if m[1] == "r" else 0x04
        if m[4] is not None:
            return [raw(cls | ALU[m[3]] | 0x08, int(m[2]), int(m[5]))]
        return [raw(cls | ALU[m[3]], int(m[2]), imm=int(m[6]))]
    raise ValueError(f"unparsed line: {line!r}")


def encode(text: str) -> list[int]:
    out: list[int] = []
    for line in text.splitlines():
        if line.strip():
            out += encode_line(line)
    return out
