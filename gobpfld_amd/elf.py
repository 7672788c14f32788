"""eBPF ELF object loading and relocation to VM indices.

Restates the parts of gobpfld's `LoadProgramFromELF` (elf.go:74-111) that feed the emulator:
  * sections (elf.go:129-152): PROGBITS program sections with SHF_EXECINSTR (parseProgram,
    elf.go:315-401; `.text` is kept aside as the sub-program pool), `maps` / `.maps` 20-byte map
    definitions named by their symbols (parseMaps, elf.go:445-514), `.data` / `.rodata` / `.bss` as
    single-entry ARRAY maps (dataToMap, elf.go:405-442), `license`;
  * relocation tables `.rel<section>` of 16-byte Rel64 entries (parseRelocationTables,
    elf.go:218-258; AbsoluteOffset, elf.go:1005-1016);
  * linking (linkAndRelocate, elf.go:518-848): `.text` appended to a program that calls into it, call
    immediates rewritten, map references collected per program;
  * the map-reference rewrite of BPFProgram load (program_abstract.go:84-113), with VM map indices in
    place of kernel fds: `src = BPF_PSEUDO_MAP_FD (1), imm = index`, or for global data
    `src = BPF_PSEUDO_MAP_FD_VALUE (2), imm = index` and the data offset moved to the second slot.

Map indices follow the harness contract: maps are added to the VM in declaration
order — the `maps` section by offset, then `.rodata`, `.data`, `.bss` — as indices 1..M.
BTF is not parsed (the emulator does not use it).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field

from .emulator import MapDef

EM_BPF = 247
SHT_PROGBITS, SHT_SYMTAB, SHT_NOBITS, SHT_REL = 1, 2, 8, 9
SHF_ALLOC, SHF_EXECINSTR = 0x2, 0x4
R_BPF_NONE, R_BPF_64_64, R_BPF_64_32 = 0, 1, 10
BPF_PSEUDO_MAP_FD, BPF_PSEUDO_MAP_FD_VALUE = 1, 2
MAP_DEF_SIZE = 20  # bpfMapDefSize
DATA_SECTIONS = (".rodata", ".data", ".bss")


class ElfError(ValueError):
    pass


@dataclass
class Section:
    index: int
    name: str
    type: int
    flags: int
    data: bytes
    size: int


@dataclass
class Symbol:
    name: str
    info: int
    shndx: int
    value: int
    size: int

    @property
    def bind(self) -> int:
        return self.info >> 4

    @property
    def type(self) -> int:
        return self.info & 0xF


@dataclass
class ElfProgram:
    name: str
    section: str
    offset: int                      # byte offset of the program in its section
    size: int
    insns: list[int]                 # raw 64-bit instructions (little endian encoding)
    map_refs: dict[str, list[int]] = field(default_factory=dict)  # map name -> byte offsets (MapFDLocations)


@dataclass
class ElfObject:
    license: str
    maps: dict[str, tuple[MapDef, bytes | None]]   # in declaration order
    programs: dict[str, ElfProgram]

    def map_order(self) -> list[str]:
        return list(self.maps)

    def relocated(self, prog: str, indices: dict[str, int] | None = None) -> list[int]:
        """Program `prog` with every map reference rewritten to a VM map index
        (program_abstract.go:98-113; the kernel fd becomes the 1-based VM index)."""
        p = self.programs[prog]
        idx = indices or {name: i + 1 for i, name in enumerate(self.maps)}
        insns = list(p.insns)
        for name, offs in p.map_refs.items():
            if name not in idx:
                raise ElfError(f"program requires unknown map '{name}'")
            for off in offs:
                k = off // 8
                if k + 1 >= len(insns):
                    raise ElfError(f"map reference at {off} is not an LD_IMM64")
                op, regs, o16, imm = _split(insns[k])
                src = regs >> 4
                if src == BPF_PSEUDO_MAP_FD_VALUE:
                    # the offset into the data section moves to the second slot (program_abstract.go:105-108)
                    op2, regs2, off2, _ = _split(insns[k + 1])
                    insns[k + 1] = _join(op2, regs2, off2, imm)
                else:
                    regs = (regs & 0x0F) | (BPF_PSEUDO_MAP_FD << 4)
                insns[k] = _join(op, regs, o16, idx[name])
        return insns


def _split(x: int) -> tuple[int, int, int, int]:
    op, regs, off, imm = struct.unpack("<BBhi", struct.pack("<Q", x))
    return op, regs, off, imm


def _join(op: int, regs: int, off: int, imm: int) -> int:
    return struct.unpack("<Q", struct.pack("<BBhi", op & 0xFF, regs & 0xFF, off, imm))[0]


def _cstr(b: bytes, off: int) -> str:
    end = b.find(b"\0", off)
    return b[off:end if end >= 0 else len(b)].decode("utf-8", "replace")


def parse_elf(data: bytes) -> ElfObject:
    """LoadProgramFromELF (elf.go:74-111) without BTF, returning maps and relocatable programs."""
    if data[:4] != b"\x7fELF":
        raise ElfError("not an ELF file")
    if data[4] != 2:
        raise ElfError("elf file class is not 64 bit")               # elf.go:84-86
    if data[5] != 1:
        raise ElfError("only little-endian eBPF objects are supported")
    (e_type, e_machine, _v, _entry, _phoff, e_shoff, _flags, _ehsize, _phentsize, _phnum, e_shentsize, e_shnum,
     e_shstrndx) = struct.unpack_from("<HHIQQQIHHHHHH", data, 16)
    if e_machine != EM_BPF:
        raise ElfError(f"elf file machine type is not BPF, machine type: {e_machine}")  # elf.go:80-82
    raw = []
    for i in range(e_shnum):
        (name, stype, flags, _addr, off, size, link, info, _align, entsize) = struct.unpack_from(
            "<IIQQQQIIQQ", data, e_shoff + i * e_shentsize)
        raw.append((name, stype, flags, off, size, link, info, entsize))
    shstr = data[raw[e_shstrndx][3]:raw[e_shstrndx][3] + raw[e_shstrndx][4]]
    sections = []
    for i, (name, stype, flags, off, size, link, info, entsize) in enumerate(raw):
        body = b"" if stype == SHT_NOBITS else data[off:off + size]
        sections.append(Section(i, _cstr(shstr, name), stype, flags, body, size))
    # symbols (debug/elf Symbols(): the null symbol is dropped, so index k maps to k-1)
    symbols: list[Symbol] = []
    for i, (name, stype, flags, off, size, link, info, entsize) in enumerate(raw):
        if stype != SHT_SYMTAB:
            continue
        strtab = sections[link].data
        for k in range(1, size // 24):
            sname, sinfo, _other, shndx, value, ssize = struct.unpack_from("<IBBHQQ", data, off + k * 24)
            symbols.append(Symbol(_cstr(strtab, sname), sinfo, shndx, value, ssize))

    license = "Unknown"
    abstract_maps: dict[str, tuple[MapDef, bytes | None]] = {}
    data_maps: dict[str, tuple[MapDef, bytes | None]] = {}
    text: list[int] = []
    programs: dict[str, ElfProgram] = {}
    rel_tables: dict[str, list[tuple[int, int, Symbol]]] = {}

    for sec in sections:                                           # parseElf, elf.go:129-152
        if sec.type == SHT_PROGBITS or sec.name == ".bss":
            if sec.name == "license":
                license = _cstr(sec.data, 0)
            elif sec.name in ("maps", ".maps"):                    # parseMaps, elf.go:445-514
                if not sec.flags & SHF_ALLOC:
                    raise ElfError("maps section has no ALLOC flag")
                for i in range(0, len(sec.data), MAP_DEF_SIZE):
                    t, ks, vs, me, fl = struct.unpack_from("<IIIII", sec.data, i)
                    name = next((s.name for s in symbols if s.shndx == sec.index and s.value == i), "")
                    if not name:
                        raise ElfError(f"unable to find name in symbol table for map at index {i} in section "
                                       f"'{sec.name}'")
                    abstract_maps[name] = (MapDef(t, ks, vs, me, fl), None)
            elif sec.name in DATA_SECTIONS:                         # dataToMap, elf.go:405-442
                init = None if sec.name == ".bss" else bytes(sec.data)
                data_maps[sec.name[1:]] = (MapDef(2, 4, sec.size, 1, 0), init)
            elif sec.name in (".BTF", ".BTF.ext"):
                pass
            elif sec.flags & SHF_EXECINSTR:                          # parseProgram, elf.go:315-401
                if len(sec.data) % 8:
                    raise ElfError("elf section is incorrect size for BPF program, should be divisible by 8")
                insns = list(struct.unpack(f"<{len(sec.data) // 8}Q", sec.data))
                if sec.name == ".text":
                    text = insns
                    continue
                for s in symbols:
                    if s.shndx != sec.index or s.bind != 1 or s.type != 2:  # STB_GLOBAL, STT_FUNC
                        continue
                    start, end = s.value // 8, (s.value + s.size) // 8
                    programs[s.name] = ElfProgram(s.name, sec.name, s.value, s.size, insns[start:end])
        elif sec.type == SHT_REL:                                    # parseRelocationTables, elf.go:218-258
            if len(sec.data) % 16:
                raise ElfError(f"size of relocation table '{sec.name}' not devisable by 16")
            entries = []
            for i in range(0, len(sec.data), 16):
                r_off, r_info = struct.unpack_from("<QQ", sec.data, i)
                symnum, rtype = r_info >> 32, r_info & 0xFFFFFFFF
                if symnum == 0 or symnum > len(symbols):
                    raise ElfError(f"symbol number in relocation table '{sec.name}' does not exist in symbol table")
                entries.append((r_off, rtype, symbols[symnum - 1]))
            rel_tables[sec.name] = entries

    maps = dict(abstract_maps)
    for name in ("rodata", "data", "bss"):
        if name in data_maps:
            maps[name] = data_maps[name]

    def abs_off(off: int, rtype: int) -> int:                          # AbsoluteOffset, elf.go:1005-1016
        if rtype in (R_BPF_64_64, R_BPF_NONE):
            return off
        if rtype == R_BPF_64_32:
            return off & 0xFFFFFFFF
        raise ElfError(f"reloc type not implemented: '{rtype}'")

    for prog in programs.values():                                    # linkAndRelocate, elf.go:603-845
        table = rel_tables.get(".rel" + prog.section)
        if table is None:
            continue
        txt_off = -1
        if text:
            uses_txt = any(0 <= abs_off(o, t) - prog.offset < prog.size and sections[sym.shndx].name == ".text"
                           for o, t, sym in table)
            if uses_txt:
                txt_off = len(prog.insns)
                prog.insns = prog.insns + list(text)
        for o, t, sym in table:
            sec = sections[sym.shndx]
            prog_off = abs_off(o, t) - prog.offset
            if prog_off < 0 or prog_off >= prog.size:
                continue
            if sec.name == ".text":
                if txt_off == -1:
                    raise ElfError("unable to relocate .text entry since it is empty")
                k = prog_off // 8
                op, regs, off16, imm = _split(prog.insns[k])
                prog.insns[k] = _join(op, regs, off16, _i32(txt_off + imm - prog_off // 8))
                continue
            global_data = sec.name in DATA_SECTIONS
            if sec.name in ("maps", ".maps") or global_data:
                name = sec.name[1:] if global_data else sym.name
                if global_data:
                    k = prog_off // 8
                    op, regs, off16, imm = _split(prog.insns[k])
                    prog.insns[k] = _join(op, (regs & 0x0F) | (BPF_PSEUDO_MAP_FD_VALUE << 4), off16, imm)
                if name not in maps:
                    raise ElfError(f"program references undefined map named '{name}'")
                prog.map_refs.setdefault(name, []).append(prog_off)
        if txt_off != -1:
            for o, t, sym in rel_tables.get(".rel.text", []):
                sec = sections[sym.shndx]
                a = abs_off(o, t)
                if sec.name == ".text":
                    k = txt_off + a // 8
                    op, regs, off16, imm = _split(prog.insns[k])
                    prog.insns[k] = _join(op, regs, off16, _i32(txt_off + imm - a // 8))
                elif sec.name == "maps":
                    if sym.name not in maps:
                        raise ElfError(f"program .text references undefined map named '{sym.name}'")
                    prog.map_refs.setdefault(sym.name, []).append(a + txt_off * 8)
    return ElfObject(license, maps, programs)


def _i32(v: int) -> int:
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v >> 31 else v


def load_into_vm(vm, obj: ElfObject, program: str) -> tuple[int, dict[str, int]]:
    """Add the object's maps (declaration order) and `program` (relocated) to an emulator VM and make
    it the entrypoint. Returns (program index, map name -> VM index)."""
    indices = {}
    for name, (mdef, init) in obj.maps.items():
        indices[name] = vm.add_map(mdef, init)
    prog = vm.add_raw_program(obj.relocated(program, indices))
    vm.set_entrypoint(prog)
    return prog, indices
