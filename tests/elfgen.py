"""Synthetic eBPF ELF objects for the loader tests (the reference's own clang-built objects are
prebuilt code and are not loaded here; these have the same shape: clang's section names, 20-byte
`maps` definitions named by symbols, `.rel<section>` REL tables with R_BPF_64_64 map references and
R_BPF_64_32 sub-program calls, `.data`/`.rodata`/`.bss` global data, a `license` section)."""
from __future__ import annotations

import struct

SHT_NULL, SHT_PROGBITS, SHT_SYMTAB, SHT_STRTAB, SHT_NOBITS, SHT_REL = 0, 1, 2, 3, 8, 9
SHF_WRITE, SHF_ALLOC, SHF_EXECINSTR = 1, 2, 4
STB_LOCAL, STB_GLOBAL = 0, 1
STT_NOTYPE, STT_OBJECT, STT_FUNC, STT_SECTION = 0, 1, 2, 3
R_BPF_64_64, R_BPF_64_32 = 1, 10


def build_elf(progs: dict[str, tuple[list[int], list[tuple[str, int, int]]]],
              maps: list[tuple[str, int, int, int, int, int]] = (),
              text: list[int] | None = None,
              data: bytes | None = None, rodata: bytes | None = None, bss: int | None = None,
              relocs: dict[str, list[tuple[int, str, int]]] | None = None,
              license: bytes = b"GPL\0", machine: int = 247) -> bytes:
    """progs: section -> (instructions, [(function symbol, byte offset, byte size)]);
    maps: [(name, type, key_size, value_size, max_entries, flags)];
    relocs: section -> [(byte offset, symbol name, type)]; symbol names are map names, `.text`,
    `.data`, `.rodata`, `.bss` (section symbols)."""
    relocs = relocs or {}
    secs: list[dict] = [dict(name="", type=SHT_NULL, flags=0, data=b"", size=0, link=0, info=0, entsize=0, align=0)]

    def add(name, stype, flags, body, size=None, entsize=0, align=8):
        secs.append(dict(name=name, type=stype, flags=flags, data=body, size=len(body) if size is None else size,
                         link=0, info=0, entsize=entsize, align=align))
        return len(secs) - 1

    idx = {}
    for name, (insns, _) in progs.items():
        idx[name] = add(name, SHT_PROGBITS, SHF_ALLOC | SHF_EXECINSTR, struct.pack(f"<{len(insns)}Q", *insns))
    if text is not None:
        idx[".text"] = add(".text", SHT_PROGBITS, SHF_ALLOC | SHF_EXECINSTR, struct.pack(f"<{len(text)}Q", *text))
    if maps:
        body = b"".join(struct.pack("<IIIII", *m[1:]) for m in maps)
        idx["maps"] = add("maps", SHT_PROGBITS, SHF_ALLOC | SHF_WRITE, body, align=4)
    if data is not None:
        idx[".data"] = add(".data", SHT_PROGBITS, SHF_ALLOC | SHF_WRITE, data)
    if rodata is not None:
        idx[".rodata"] = add(".rodata", SHT_PROGBITS, SHF_ALLOC, rodata)
    if bss is not None:
        idx[".bss"] = add(".bss", SHT_NOBITS, SHF_ALLOC | SHF_WRITE, b"", size=bss)
    add("license", SHT_PROGBITS, SHF_ALLOC | SHF_WRITE, license, align=1)

    # symbols: null, section symbols, map objects, functions
    strtab = bytearray(b"\0")

    def sname(s):
        off = len(strtab)
        strtab.extend(s.encode() + b"\0")
        return off

    syms = [(0, 0, 0, 0, 0, 0)]
    symidx = {}
    for sec in (".text", ".data", ".rodata", ".bss"):
        if sec in idx:
            symidx[sec] = len(syms)
            syms.append((0, (STB_LOCAL << 4) | STT_SECTION, 0, idx[sec], 0, 0))
    for k, m in enumerate(maps):
        symidx[m[0]] = len(syms)
        syms.append((sname(m[0]), (STB_GLOBAL << 4) | STT_OBJECT, 0, idx["maps"], k * 20, 20))
    for name, (_, funcs) in progs.items():
        for fname, off, size in funcs:
            symidx[fname] = len(syms)
            syms.append((sname(fname), (STB_GLOBAL << 4) | STT_FUNC, 0, idx[name], off, size))

    for sec, entries in relocs.items():
        body = b"".join(struct.pack("<QQ", off, (symidx[sym] << 32) | rtype) for off, sym, rtype in entries)
        r = add(".rel" + sec, SHT_REL, 0, body, entsize=16)
        secs[r]["info"] = idx[sec]
    symtab = add(".symtab", SHT_SYMTAB, 0, b"".join(struct.pack("<IBBHQQ", *s) for s in syms), entsize=24)
    strsec = add(".strtab", SHT_STRTAB, 0, bytes(strtab), align=1)
    secs[symtab]["link"] = strsec
    secs[symtab]["info"] = 1
    for s in secs:
        if s["type"] == SHT_REL:
            s["link"] = symtab
    shstr = bytearray(b"\0")
    names = []
    for s in secs:
        names.append(len(shstr) if s["name"] else 0)
        if s["name"]:
            shstr.extend(s["name"].encode() + b"\0")
    shname_off = len(shstr)
    shstr.extend(b".shstrtab\0")
    secs.append(dict(name=".shstrtab", type=SHT_STRTAB, flags=0, data=bytes(shstr), size=len(shstr), link=0, info=0,
                     entsize=0, align=1))
    names.append(shname_off)

    out = bytearray(64)
    offs = []
    for s in secs:
        while len(out) % 8:
            out.append(0)
        offs.append(len(out))
        out.extend(s["data"])
    while len(out) % 8:
        out.append(0)
    shoff = len(out)
    for s, nm, off in zip(secs, names, offs):
        out.extend(struct.pack("<IIQQQQIIQQ", nm, s["type"], s["flags"], 0, off, s["size"], s["link"], s["info"],
                               s["align"], s["entsize"]))
    hdr = b"\x7fELF" + bytes([2, 1, 1, 0]) + bytes(8)
    hdr += struct.pack("<HHIQQQIHHHHHH", 1, machine, 1, 0, 0, shoff, 0, 64, 0, 0, 64, len(secs), len(secs) - 1)
    out[:64] = hdr
    return bytes(out)
