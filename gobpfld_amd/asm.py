"""Minimal eBPF encoder with labels, for building programs without a clang toolchain.

Encodes ebpf.RawInstruction (ebpf/ebpf.go:46-56): op u8 | regs u8 (dst low nibble, src high
nibble) | off i16 | imm i32, little endian, one u64 per slot. Opcode constants follow
ebpf/ebpf.go:207-342. Jump offsets are resolved from labels (target = pc + off + 1).
"""
from __future__ import annotations

# classes
LD, LDX, ST, STX, ALU, JMP, JMP32, ALU64 = range(8)
K, X = 0x00, 0x08
# sizes
W, H, B, DW = 0x00, 0x08, 0x10, 0x18
SIZE = {4: W, 2: H, 1: B, 8: DW}
# ALU ops
ADD, SUB, MUL, DIV, OR, AND, LSH, RSH, NEG, MOD, XOR, MOV, ARSH, END = (
    0x00, 0x10, 0x20, 0x30, 0x40, 0x50, 0x60, 0x70, 0x80, 0x90, 0xA0, 0xB0, 0xC0, 0xD0)
# JMP ops
JA, JEQ, JGT, JGE, JSET, JNE, JSGT, JSGE, CALL, CALLX, EXIT, JLT, JLE, JSLT, JSLE = (
    0x00, 0x10, 0x20, 0x30, 0x40, 0x50, 0x60, 0x70, 0x80, 0x88, 0x90, 0xA0, 0xB0, 0xC0, 0xD0)
MEM, ATOMIC = 0x60, 0xC0
# XDP verdicts (ebpf/ebpf.go:329-341)
XDP_ABORTED, XDP_DROP, XDP_PASS, XDP_TX, XDP_REDIRECT = range(5)


def raw(op: int, dst: int = 0, src: int = 0, off: int = 0, imm: int = 0) -> int:
    return ((op & 0xFF) | ((dst & 0xF) << 8) | ((src & 0xF) << 12) | ((off & 0xFFFF) << 16)
            | ((imm & 0xFFFFFFFF) << 32))


class Asm:
    """Program builder. Methods append one (or two, for LD_IMM64) slots; labels resolve jumps."""

    def __init__(self) -> None:
        self.slots: list[tuple] = []  # (op, dst, src, off_or_label, imm)
        self.labels: dict[str, int] = {}

    # -- plumbing
    def emit(self, op, dst=0, src=0, off=0, imm=0):
        self.slots.append((op, dst, src, off, imm))
        return self

    def label(self, name: str):
        if name in self.labels:
            raise ValueError(f"duplicate label {name}")
        self.labels[name] = len(self.slots)
        return self

    def __len__(self) -> int:
        return len(self.slots)

    def assemble(self) -> list[int]:
        out = []
        for pc, (op, dst, src, off, imm) in enumerate(self.slots):
            if isinstance(off, str):
                off = self.labels[off] - pc - 1
            if isinstance(imm, str):  # bpf-to-bpf call: the relative target is in imm
                imm = self.labels[imm] - pc - 1
            if not -32768 <= off <= 32767:
                raise ValueError("jump offset out of range")
            out.append(raw(op, dst, src, off, imm))
        return out

    # -- ALU
    def alu64(self, op, dst, imm=None, src=None):
        return self.emit(ALU64 | (X if src is not None else K) | op, dst, src or 0, 0, imm or 0)

    def alu32(self, op, dst, imm=None, src=None):
        return self.emit(ALU | (X if src is not None else K) | op, dst, src or 0, 0, imm or 0)

    def mov64(self, dst, imm=None, src=None):
        return self.alu64(MOV, dst, imm, src)

    def mov32(self, dst, imm=None, src=None):
        return self.alu32(MOV, dst, imm, src)

    def add64(self, dst, imm=None, src=None):
        return self.alu64(ADD, dst, imm, src)

    def sub64(self, dst, imm=None, src=None):
        return self.alu64(SUB, dst, imm, src)

    def neg64(self, dst):
        return self.emit(ALU64 | NEG, dst)

    def neg32(self, dst):
        return self.emit(ALU | NEG, dst)

    def end(self, dst, bits, to_be: bool):
        return self.emit(ALU | END | (X if to_be else K), dst, 0, 0, bits)

    def ld_imm64(self, dst, value, src=0):
        value &= (1 << 64) - 1
        self.emit(LD | DW, dst, src, 0, value & 0xFFFFFFFF)
        return self.emit(0, 0, 0, 0, value >> 32)

    def ld_map(self, dst, map_idx):  # BPF_PSEUDO_MAP_FD relocated to the VM map index
        self.emit(LD | DW, dst, 1, 0, map_idx)
        return self.emit(0, 0, 0, 0, 0)

    def ld_map_value(self, dst, map_idx, off=0):  # BPF_PSEUDO_MAP_FD_VALUE
        self.emit(LD | DW, dst, 2, 0, map_idx)
        return self.emit(0, 0, 0, 0, off)

    # -- memory
    def ldx(self, size, dst, src, off):
        return self.emit(LDX | MEM | SIZE[size], dst, src, off)

    def st(self, size, dst, off, imm):
        return self.emit(ST | MEM | SIZE[size], dst, 0, off, imm)

    def stx(self, size, dst, off, src):
        return self.emit(STX | MEM | SIZE[size], dst, src, off)

    def xadd(self, size, dst, off, src, fetch=False):
        return self.emit(STX | ATOMIC | SIZE[size], dst, src, off, 0x01 if fetch else 0x00)

    # -- jumps
    def ja(self, target):
        return self.emit(JMP | JA, 0, 0, target)

    def jmp(self, op, dst, target, imm=None, src=None, wide=True):
        cls = JMP if wide else JMP32
        return self.emit(cls | (X if src is not None else K) | op, dst, src or 0, target, imm or 0)

    def call(self, helper):
        return self.emit(JMP | CALL, 0, 0, 0, helper)

    def call_bpf(self, target):  # BPF_PSEUDO_CALL (src = 1): PC += imm (emulator/inst_call_bpf.go:41)
        return self.emit(JMP | CALL, 0, 1, 0, target)

    def exit(self):
        return self.emit(JMP | EXIT)
