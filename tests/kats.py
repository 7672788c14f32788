"""Known-answer tests derived from the reference source.

The reference has no VM execution tests, so each KAT encodes one quirk of the Go emulator with the
answer read off the cited line. The oracle must produce `expect`; the device must equal the oracle.
"""
from __future__ import annotations

from gobpfld_amd.asm import (ADD, ARSH, DIV, JEQ, JGT, JNE, JSGE, JSGT, JSLE, JSLT, LSH, MOD, MUL,
                             RSH, SUB, XOR, Asm, AND, OR)
from gobpfld_amd.emulator import (MAP_ARRAY, MAP_HASH, MAP_LRU_HASH, MAP_PERF_EVENT_ARRAY, MAP_PROG_ARRAY, MAP_QUEUE,
                                  MAP_STACK, MapDef)

OK, VMERR, PANIC, BUDGET, UNSUP = 0, 1, 2, 3, 4
E_NO_PROGRAM = 1
E_BAD_REG, E_ASSIGN_REG, E_READONLY, E_DIV0, E_NONPTR_LOAD, E_NONPTR_STORE = 2, 3, 4, 5, 6, 7
E_OOB, E_NONCONTIG, E_UNINIT, E_BAD_PC, E_NOT_IMPL, E_NO_HELPER, E_NO_MAP, E_MAP_NOT_PTR = 8, 9, 10, 11, 12, 13, 14, 15
IN_HELPER = 0x80
P_NIL_DEREF, P_NEG_SHIFT, P_DIV0, P_INDEX, P_NIL_MAP = 1, 2, 3, 4, 5
ARRAY8 = (MapDef(MAP_ARRAY, 4, 8, 16), None)
HASH16 = (MapDef(MAP_HASH, 16, 16, 64), None)


def _u64(v):
    return v & ((1 << 64) - 1)


def _s64(v):
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >> 63 else v


KATS: list[dict] = []


def kat(name, expect=None, maps=(), entries=None, pkt=64, cite="", extra=()):
    """extra: more programs (Asm builders) added after the entrypoint, as VM programs 2, 3, ..."""
    def deco(fn):
        a = Asm()
        fn(a)
        progs = [a.assemble()]
        for f in extra:
            b = Asm()
            f(b)
            progs.append(b.assemble())
        KATS.append(dict(name=name, program=progs if extra else progs[0], maps=list(maps), entries=entries or {},
                         expect=expect, pkt=pkt, cite=cite))
        return fn
    return deco


# ---- ALU (Appendix A §A)
@kat("add32_sign_extends", (OK, _s64(0xFFFFFFFF80000000)), cite="emulator/inst_add.go:26")
def _(a):
    a.mov32(0, 0x7FFFFFFF).alu32(ADD, 0, 1).exit()


@kat("sub32_reg_sign_extends", (OK, -1), cite="emulator/inst_sub.go:81")
def _(a):
    a.mov64(0, 0).mov64(1, 1).alu32(SUB, 0, src=1).exit()


@kat("mul64_wraps", (OK, _s64(0x7FFFFFFFFFFFFFFF * 3)), cite="emulator/inst_mul.go:111")
def _(a):
    a.ld_imm64(0, 0x7FFFFFFFFFFFFFFF).mov64(1, 3).alu64(MUL, 0, src=1).exit()


@kat("div64_signed", (OK, -3), cite="emulator/inst_div.go:62")
def _(a):
    a.mov64(0, -7).alu64(DIV, 0, 2).exit()


@kat("div32_minint_by_minus1", (OK, _s64(0xFFFFFFFF80000000)), cite="emulator/inst_div.go:33")
def _(a):
    a.mov32(0, -2147483648).alu32(DIV, 0, -1).exit()


@kat("mod64_by_minus1_is_zero", (OK, 0), cite="emulator/inst_mod.go:62")
def _(a):
    a.ld_imm64(0, 1 << 63).alu64(MOD, 0, -1).exit()


@kat("div_imm_zero_vmerr", (VMERR, E_DIV0), cite="emulator/inst_div.go:29")
def _(a):
    a.mov64(0, 5).alu64(DIV, 0, 0).exit()


@kat("div32_reg_trunc_zero_panics", (PANIC, P_DIV0), cite="emulator/inst_div.go:92-96")
def _(a):
    a.mov64(0, 5).ld_imm64(1, 1 << 32).alu32(DIV, 0, src=1).exit()


@kat("mod_reg_zero_vmerr", (VMERR, E_DIV0), cite="emulator/inst_mod.go:126")
def _(a):
    a.mov64(0, 5).mov64(1, 0).alu64(MOD, 0, src=1).exit()


@kat("lsh32_zero_extends", (OK, 0x80000000), cite="emulator/inst_lsh.go:26")
def _(a):
    a.mov64(0, 1).alu32(LSH, 0, 31).exit()


@kat("lsh64_ge_width_is_zero", (OK, 0), cite="emulator/inst_lsh.go:51 (Go: shift >= width -> 0)")
def _(a):
    a.mov64(0, 1).alu64(LSH, 0, 64).exit()


@kat("lsh_negative_count_panics", (PANIC, P_NEG_SHIFT), cite="emulator/inst_lsh.go:111")
def _(a):
    a.mov64(0, 1).mov64(1, -1).alu64(LSH, 0, src=1).exit()


@kat("rsh32_logical", (OK, 0x7FFFFFFF), cite="emulator/inst_rsh.go:26")
def _(a):
    a.mov64(0, -1).alu32(RSH, 0, 1).exit()


@kat("arsh32_sign_extends", (OK, -1), cite="emulator/inst_arsh.go:26")
def _(a):
    a.mov32(0, -2).alu32(ARSH, 0, 40).exit()


@kat("neg32", (OK, _s64(0xFFFFFFFF80000000)), cite="emulator/inst_neg.go:26")
def _(a):
    a.mov32(0, -2147483648).neg32(0).exit()


@kat("end_to_le_swaps", (OK, 0x3412), cite="emulator/inst_end.go:27-30 (inverted vs Linux)")
def _(a):
    a.mov64(0, 0x1234).end(0, 16, to_be=False).exit()


@kat("end_to_be_truncates", (OK, 0x22334455), cite="emulator/inst_end.go:155-160")
def _(a):
    a.ld_imm64(0, 0x1122334455).end(0, 32, to_be=True).exit()


@kat("end64_to_le_swaps", (OK, _s64(0x0807060504030201)), cite="emulator/inst_end.go:89-98")
def _(a):
    a.ld_imm64(0, 0x0102030405060708).end(0, 64, to_be=False).exit()


@kat("mov32_reg_copies_full_64", (OK, _s64(0x1122334455667788)), cite="emulator/inst_mov.go:62-68")
def _(a):
    a.ld_imm64(3, 0x1122334455667788).mov32(0, src=3).exit()


@kat("lddw_inplace_keeps_pointer_kind", (OK, 1), cite="emulator/inst_load.go:65 (in-place Assign on R1 = ctx ptr)")
def _(a):
    a.ld_imm64(1, 5).mov64(0, 1).jmp(JEQ, 1, "t", imm=5).exit()   # R1 is still a MemoryPtr: not taken
    a.label("t").mov64(0, 2).exit()


@kat("xor_and_or_mix", (OK, ((0x0F0F ^ 0xFF) & 0x3C) | 0x100), cite="emulator/inst_{xor,and,or}.go:51")
def _(a):
    a.mov64(0, 0x0F0F).alu64(XOR, 0, 0xFF).alu64(AND, 0, 0x3C).alu64(OR, 0, 0x100).exit()


# ---- jumps (Appendix A §J)
@kat("jslt_is_le", (OK, 1), cite="emulator/inst_jslt.go:48")
def _(a):
    a.mov64(1, 5).mov64(0, 0).jmp(JSLT, 1, "t", imm=5).exit().label("t").mov64(0, 1).exit()


@kat("jgt_imm_sign_extended_unsigned", (OK, 0), cite="emulator/inst_jgt.go:48")
def _(a):
    a.mov64(1, 5).mov64(0, 0).jmp(JGT, 1, "t", imm=-1).exit().label("t").mov64(0, 1).exit()


@kat("jsgt32_and_jsge", (OK, 3), cite="emulator/inst_jsgt.go:24, inst_jsge.go:24")
def _(a):
    a.mov64(0, 0).ld_imm64(3, 0x1FFFFFFFF).jmp(JSGT, 3, "x", imm=0, wide=False).add64(0, 1)
    a.label("x").jmp(JSGE, 3, "y", imm=-1, wide=False).exit().label("y").add64(0, 2).exit()


@kat("jeq_imm_never_on_pointer", (OK, 7), cite="emulator/inst_jeq.go:48, inst_jne.go:48")
def _(a):
    a.ldx(4, 2, 1, 0)              # r2 = ctx->data (MemoryPtr, value 0)
    a.mov64(0, 0)
    a.jmp(JEQ, 2, "bad", imm=0)    # never taken on a pointer
    a.add64(0, 3)
    a.jmp(JNE, 2, "good", imm=0)   # always taken on a pointer
    a.label("bad").mov64(0, 99).exit()
    a.label("good").add64(0, 4).exit()


@kat("jreg_type_mismatch", (OK, 1), cite="emulator/inst.go:254-258, inst_jne.go:77,106")
def _(a):
    a.ldx(4, 2, 1, 0).mov64(3, 0).mov64(0, 0)
    a.jmp(JEQ, 2, "bad", src=3)    # MemoryPtr vs IMM: not taken even though values are equal
    a.jmp(JNE, 2, "good", src=3)   # kinds differ: taken
    a.label("bad").mov64(0, 99).exit()
    a.label("good").mov64(0, 1).exit()


@kat("jsle32_reg", (OK, 1), cite="emulator/inst_jsle.go:77")
def _(a):
    a.mov64(0, 0).mov64(1, -1).mov64(2, 1).jmp(JSLE, 1, "t", src=2, wide=False).exit()
    a.label("t").mov64(0, 1).exit()


@kat("fallthrough_bad_pc", (VMERR, E_BAD_PC), cite="emulator/vm.go:162-167")
def _(a):
    a.mov64(0, 1).mov64(0, 2)


@kat("jump_past_end_bad_pc", (VMERR, E_BAD_PC), cite="emulator/vm.go:162-167")
def _(a):
    a.mov64(0, 1).emit(0x05, 0, 0, 5).exit()


@kat("jump_negative_panics", (PANIC, P_INDEX), cite="emulator/vm.go:143")
def _(a):
    a.mov64(0, 1).emit(0x05, 0, 0, -3).exit()


@kat("budget_exhausted", (BUDGET, None), cite="emulator/vm.go:117-134 (no budget in Go)")
def _(a):
    a.mov64(0, 0).label("l").add64(0, 1).ja("l").exit()


# ---- registers (§R)
@kat("get_r10_fails", (VMERR, E_BAD_REG), cite="emulator/registers.go:91-116")
def _(a):
    a.mov64(0, 0).add64(0, src=10).exit()


@kat("mov_r10_copies_frame_pointer", (OK, -8), cite="emulator/registers.go:84-85,283-292")
def _(a):
    a.mov64(0, src=10).add64(0, -8).exit()


@kat("stx_r10_src_fails", (VMERR, E_BAD_REG), cite="emulator/inst_store.go:65")
def _(a):
    a.stx(8, 10, -8, 10).mov64(0, 0).exit()


@kat("assign_r10_fails", (VMERR, E_ASSIGN_REG), cite="emulator/registers.go:145")
def _(a):
    a.mov64(10, 1).exit()


@kat("add_pointer_src_makes_pointer", (OK, 14), cite="emulator/inst_add.go:131-147")
def _(a):
    a.ldx(4, 2, 1, 0).mov64(3, 14).add64(3, src=2)   # r3 = IMM + ptr -> MemoryPtr
    a.ldx(1, 4, 3, 0)                                  # loads through r3 prove it is a pointer
    a.mov64(0, src=3).exit()


@kat("ctx_alias_inplace", (OK, 14), cite="emulator/memory.go:37-52, inst_load.go:112")
def _(a):
    a.ldx(4, 2, 1, 0)            # r2 aliases ctx->data object
    a.add64(2, 14)               # in place: mutates the ctx object
    a.ldx(4, 3, 1, 0)            # reload sees data + 14
    a.mov64(0, src=3).exit()


@kat("stack_alias_two_regs", (OK, 11), cite="emulator/memory.go:37-52")
def _(a):
    a.mov64(1, 5).stx(8, 10, -8, 1)
    a.ldx(8, 2, 10, -8).ldx(8, 3, 10, -8)   # both alias the same stored object
    a.add64(2, 6)                            # r3 sees it too
    a.mov64(0, src=3).exit()


@kat("atomic_on_stack_object_updates_alias", (OK, 15), cite="emulator/inst_atomic.go:44-59")
def _(a):
    a.mov64(1, 5).stx(8, 10, -8, 1)
    a.ldx(8, 2, 10, -8)
    a.mov64(3, 10).xadd(8, 10, -8, 3)        # object += 10 in place
    a.mov64(0, src=2).exit()


@kat("ldx_uninit_stack", (VMERR, E_UNINIT), cite="emulator/memory.go:48-50")
def _(a):
    a.ldx(8, 0, 10, -8).exit()


@kat("ldx_noncontiguous", (VMERR, E_NONCONTIG), cite="emulator/memory.go:40-46")
def _(a):
    a.st(4, 10, -8, 1).st(4, 10, -4, 2).ldx(8, 0, 10, -8).exit()


@kat("ldx_partial_returns_full_object", (OK, _s64(0x1122334455667788)), cite="emulator/memory.go:32-53")
def _(a):
    a.ld_imm64(1, 0x1122334455667788).stx(8, 10, -8, 1).ldx(1, 0, 10, -6).exit()


@kat("stack_oob", (VMERR, E_OOB), cite="emulator/memory.go:98-100")
def _(a):
    a.st(8, 10, 0, 1).mov64(0, 0).exit()


@kat("load_via_imm_fails", (VMERR, E_NONPTR_LOAD), cite="emulator/inst_load.go:103-105")
def _(a):
    a.mov64(2, 0).ldx(4, 0, 2, 0).exit()


@kat("store_via_imm_fails", (VMERR, E_NONPTR_STORE), cite="emulator/inst_store.go:41-43")
def _(a):
    a.mov64(2, 0).st(4, 2, 0, 1).mov64(0, 0).exit()


@kat("packet_read_le_and_write", (OK, 0x0201), cite="emulator/memory.go:135-210")
def _(a):
    a.ldx(4, 2, 1, 0)
    a.st(2, 2, 10, 0x0201)        # write packet bytes 10..11
    a.ldx(2, 0, 2, 10).exit()


@kat("packet_oob", (VMERR, E_OOB), cite="emulator/memory.go:136-138")
def _(a):
    a.ldx(4, 2, 1, 0).ldx(4, 0, 2, 62).exit()


@kat("data_end_minus_data_is_pointer", (OK, 64), cite="emulator/inst_sub.go:111 (no pointer edge for sub)")
def _(a):
    a.ldx(4, 2, 1, 0).ldx(4, 3, 1, 4).sub64(3, src=2)
    a.mov64(0, 0).jmp(JEQ, 3, "bad", imm=64)         # still a MemoryPtr: imm compare not taken
    a.mov64(0, src=3).exit().label("bad").mov64(0, 99).exit()


@kat("ctx_ifindex", (OK, 1), cite="xdp_md.ingress_ifindex (harness, SURVEY Appendix B)")
def _(a):
    a.ldx(4, 0, 1, 12).exit()


@kat("lddw_const_inplace", (OK, _s64(0xDEADBEEF00C0FFEE)), cite="emulator/inst_load.go:65")
def _(a):
    a.ld_imm64(0, 0xDEADBEEF00C0FFEE).exit()


# ---- helpers & maps (§C, §MA)
@kat("helper_unknown", (VMERR, E_NO_HELPER), cite="emulator/inst_call_helper.go:26-28")
def _(a):
    a.call(4).mov64(0, 0).exit()


@kat("helper_delete_errors", (VMERR, E_NOT_IMPL | IN_HELPER), maps=[ARRAY8], cite="helper_functions.go:104-106")
def _(a):
    a.call(3).mov64(0, 0).exit()


@kat("helper_pid_tgid", (OK, (1234 << 32) + 5678), cite="helper_functions.go:213-216")
def _(a):
    a.call(14).exit()


@kat("lookup_bad_map_index_r0_zero", (OK, 0), maps=[ARRAY8], cite="helper_functions.go:123-127")
def _(a):
    a.mov64(0, 9).mov64(1, 5).call(1).exit()


@kat("lookup_key_not_pointer_efault", (OK, -14), maps=[ARRAY8], cite="maps_array.go:66-69, helper_functions.go:57-60")
def _(a):
    a.ld_map(1, 1).mov64(2, 0).call(1).exit()


@kat("array_lookup_and_xadd", (OK, 2), maps=[ARRAY8], cite="maps_array.go:65-87, inst_atomic.go")
def _(a):
    a.st(4, 10, -4, 3)
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.mov64(1, 2).xadd(8, 0, 0, 1)
    a.ldx(8, 0, 0, 0).exit()


@kat("array_lookup_out_of_range_null", (OK, 0), maps=[ARRAY8], cite="maps_array.go:79-84")
def _(a):
    a.st(4, 10, -4, 16).ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1).exit()


@kat("array_lookup_uninit_key_panics", (PANIC, P_NIL_DEREF), maps=[ARRAY8], cite="maps_array.go:71-75")
def _(a):
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1).exit()


@kat("array_update_stack_value_efault", (OK, -14), maps=[ARRAY8], cite="maps_array.go:97-100")
def _(a):
    a.st(4, 10, -4, 1).st(8, 10, -16, 7)
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -4).mov64(3, src=10).add64(3, -16).mov64(4, 0).call(2).exit()


@kat("array_update_from_packet_ordered", (OK, 0), maps=[ARRAY8], cite="maps_array.go:89-131 (key/value *MemoryPtr)")
def _(a):
    a.ldx(4, 2, 1, 0).mov64(3, src=2)           # key = packet bytes 0..3 (masked below), value = packet
    a.st(4, 2, 0, 2)                            # packet[0..3] = 2 -> key 2
    a.ld_map(1, 1).mov64(4, 0).call(2).exit()


@kat("lddw_map_value", (OK, 0x55), maps=[(MapDef(MAP_ARRAY, 4, 8, 4), bytes(range(0x50, 0x70)))],
     cite="emulator/inst_load.go:36-63")
def _(a):
    a.ld_map_value(2, 1, 5).ldx(1, 0, 2, 0).exit()


@kat("lddw_map_value_nil_map_panics", (PANIC, P_NIL_MAP), maps=[ARRAY8], cite="emulator/inst_load.go:43-44")
def _(a):
    a.ld_map_value(2, 0, 0).mov64(0, 0).exit()


@kat("lddw_map_value_no_map", (VMERR, E_NO_MAP), maps=[ARRAY8], cite="emulator/inst_load.go:39-41")
def _(a):
    a.ld_map_value(2, 7, 0).mov64(0, 0).exit()


def _hash_entries():
    k = bytes([1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16])
    return {0: [(k, (41).to_bytes(8, "little") + bytes(8))]}


@kat("hash_lookup_hit", (OK, 42), maps=[HASH16], entries=_hash_entries(), cite="maps_hash.go:44-63")
def _(a):
    a.ld_imm64(3, 0x0807060504030201).stx(8, 10, -16, 3)
    a.ld_imm64(3, 0x100F0E0D0C0B0A09).stx(8, 10, -8, 3)
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -16).call(1)
    a.jmp(JEQ, 0, "miss", imm=0)
    a.mov64(1, 1).xadd(8, 0, 0, 1).ldx(8, 0, 0, 0).exit()
    a.label("miss").mov64(0, -1).exit()


@kat("hash_key_readrange_rounding", (OK, -1), maps=[HASH16], entries=_hash_entries(),
     cite="emulator/memory.go:55-95 (a 3-byte run is widened to 4 bytes)")
def _(a):
    a.ld_imm64(3, 0x0807060504030201).stx(8, 10, -16, 3)
    a.ld_imm64(3, 0x100F0E0D0C0B0A09).stx(8, 10, -8, 3)
    a.st(1, 10, -13, 4)          # breaks the first object's run: bytes 0..2 | 3 | 4..7
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -16).call(1)
    a.jmp(JEQ, 0, "miss", imm=0)
    a.mov64(0, 1).exit()
    a.label("miss").mov64(0, -1).exit()


@kat("hash_update_inserts_ordered", (OK, 0), maps=[HASH16], cite="maps_hash.go:65-123")
def _(a):
    a.ldx(4, 2, 1, 0)
    a.ld_map(1, 1).mov64(3, src=2).add64(3, 16).mov64(4, 0).call(2).exit()   # key = pkt[0:16], value = pkt[16:32]


@kat("hash_update_then_lookup_sees_value", (OK, 0x1817161514131211), maps=[HASH16],
     cite="maps_hash.go:65-123, 44-63")
def _(a):
    a.ldx(4, 6, 1, 0)
    a.ld_imm64(3, 0x1817161514131211).stx(8, 6, 16, 3)
    a.ld_map(1, 1).mov64(2, src=6).mov64(3, src=6).add64(3, 16).mov64(4, 0).call(2)
    a.ld_map(1, 1).mov64(2, src=6).call(1)
    a.ldx(8, 0, 0, 0).exit()


@kat("nonatomic_rmw_on_map_value_ordered", (OK, None), maps=[ARRAY8], cite="inst_load.go + inst_store.go on map memory")
def _(a):
    a.st(4, 10, -4, 0).ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.jmp(JEQ, 0, "out", imm=0)
    a.ldx(8, 1, 0, 0).mov64(6, src=1).add64(1, 1).stx(8, 0, 0, 1)   # counter++ (read-modify-write)
    a.mov64(0, src=6).exit()
    a.label("out").mov64(0, -1).exit()


@kat("ordered_replay_restores_packet", (OK, None), maps=[ARRAY8],
     cite="packet write (inst_store.go on ByteMemory) in an order-dependent batch: written once")
def _(a):
    a.ldx(4, 2, 1, 0)                                                  # r2 = data
    a.ldx(4, 3, 2, 4).add64(3, 7).stx(4, 2, 4, 3)                      # pkt[4..8] += 7
    a.st(4, 10, -4, 0).ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.jmp(JEQ, 0, "out", imm=0)
    a.ldx(8, 1, 0, 0).mov64(6, src=1).add64(1, 1).stx(8, 0, 0, 1)    # counter++ (conflict)
    a.mov64(0, src=6).exit()
    a.label("out").mov64(0, -1).exit()


@kat("mixed_width_xadd_ordered", (OK, None),
     maps=[(MapDef(MAP_ARRAY, 4, 8, 16), (0xFFFFFFFE).to_bytes(8, "little") + bytes(120))],
     cite="inst_atomic.go:44-59: a 4-byte add truncates at byte 3, an 8-byte add carries: order-dependent")
def _(a):
    a.st(4, 10, -4, 0).ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.jmp(JEQ, 0, "out", imm=0)
    a.mov64(1, 1).xadd(8, 0, 0, 1).xadd(4, 0, 0, 1).mov64(0, 2).exit()
    a.label("out").mov64(0, -1).exit()


@kat("xadd_then_read_conflict", (OK, None), maps=[ARRAY8], cite="atomic and read of the same bytes: order-dependent")
def _(a):
    a.st(4, 10, -4, 1).ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.jmp(JEQ, 0, "out", imm=0)
    a.mov64(1, 1).xadd(8, 0, 0, 1).ldx(8, 0, 0, 0).exit()
    a.label("out").mov64(0, -1).exit()


@kat("unaligned_xadd_on_array", (OK, 0), maps=[(MapDef(MAP_ARRAY, 4, 16, 4), None)],
     cite="inst_atomic.go:44-59 (any alignment; carry confined to the field)")
def _(a):
    a.st(4, 10, -4, 2).ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.jmp(JEQ, 0, "out", imm=0)
    a.ld_imm64(1, 0x00FF00FF00FF01FF).xadd(8, 0, 3, 1).mov64(1, 0x1FF).xadd(2, 0, 1, 1)
    a.mov64(1, 0x7FFFFFFF).xadd(4, 0, 9, 1)
    a.label("out").mov64(0, 0).exit()


@kat("tail_call_bad_map_index_efault", (OK, -14), maps=[ARRAY8], cite="helper_functions.go:135-139 (R2 = IMM 0 after Reset)")
def _(a):
    a.call(12).exit()


@kat("ld_abs_not_implemented", (VMERR, E_NOT_IMPL), cite="emulator/inst_load.go:146-148")
def _(a):
    a.emit(0x20, 0, 0, 0, 12).exit()


@kat("callx_dispatch", (OK, (1234 << 32) + 5678), cite="emulator/inst_call_helper.go:49-71")
def _(a):
    a.mov64(3, 14).emit(0x8D, 0, 0, 0, 3).exit()


# ---- ValueMemory objects beyond the fields model's 57 (emulator/memory.go:97-107: every stored byte
# may hold its own object; the device's general model keeps them in its arena)
@kat("capacity_64_byte_stores", (OK, 63), cite="emulator/memory.go:97-107 (64 live objects on the stack)")
def _(a):
    for i in range(64):
        a.st(1, 10, -(i + 1), i)
    a.ldx(1, 0, 10, -64).exit()


@kat("capacity_ctx_and_stack", (OK, 23 * 256 + 39), cite="emulator/memory.go:97-107 (24 ctx + 40 stack objects)")
def _(a):
    for i in range(24):
        a.st(1, 1, i, i)
    for i in range(40):
        a.st(1, 10, -(i + 1), i)
    a.ldx(1, 2, 1, 23).ldx(1, 3, 10, -40).mov64(0, src=2).alu64(MUL, 0, 256).add64(0, src=3).exit()


@kat("capacity_loop_256_objects", (OK, 7 * 256 + 255), cite="emulator/memory.go:97-107 (a loop fills the frame)")
def _(a):
    a.mov64(2, 0)
    a.label("loop").mov64(3, src=10).add64(3, -256).add64(3, src=2).stx(1, 3, 0, 2)
    a.add64(2, 1).jmp(JNE, 2, "loop", imm=256)
    a.ldx(1, 0, 10, -256).alu64(MUL, 0, 256).ldx(1, 4, 10, -1).add64(0, src=4)
    a.mov64(5, 7).alu64(MUL, 5, 256).add64(0, src=5).exit()


# ---- bpf-to-bpf calls (emulator/inst_call_bpf.go:18-44, emulator/inst_exit.go:22-48)
@kat("callbpf_basic", (OK, 11), cite="inst_call_bpf.go:41 (PC += imm), inst_exit.go:33-37")
def _(a):
    a.mov64(1, 5).call_bpf("sub").add64(0, 1).exit()
    a.label("sub").mov64(0, src=1).alu64(MUL, 0, 2).exit()


@kat("callbpf_own_stack_frame", (OK, 111), cite="inst_call_bpf.go:23-39 (R10 := next frame, wiped)")
def _(a):
    a.st(8, 10, -8, 111).call_bpf("sub").ldx(8, 0, 10, -8).exit()
    a.label("sub").st(8, 10, -8, 222).mov64(0, 0).exit()


@kat("callbpf_r6_clone_sees_old_stack", (OK, 5 * 16 + 9), cite="registers.go:44-60,294-303 (R6-R9 deep clones)")
def _(a):
    a.st(8, 10, -8, 5).mov64(6, src=10).add64(6, -8).mov64(1, src=10).add64(1, -8)
    a.call_bpf("sub")
    a.ldx(8, 2, 6, 0).ldx(8, 3, 10, -8).mov64(0, src=2).alu64(MUL, 0, 16).add64(0, src=3).exit()
    a.label("sub").st(8, 1, 0, 9).mov64(0, 0).exit()


@kat("callbpf_r7_clone_of_packet", (OK, None), cite="registers.go:233-240 + memory.go:212-219 (packet bytes copied)")
def _(a):
    a.mov64(8, src=1).ldx(4, 7, 1, 0).mov64(1, src=7).call_bpf("sub")
    a.ldx(1, 2, 7, 0).ldx(4, 3, 8, 0).ldx(1, 3, 3, 0).mov64(0, src=2).alu64(MUL, 0, 256).add64(0, src=3).exit()
    a.label("sub").mov64(6, src=1).st(1, 1, 0, 0xAB).mov64(0, 0).exit()


@kat("callbpf_r6_clone_of_map_value", (OK, None), maps=[ARRAY8], cite="registers.go:233-240 (the array memory is copied)")
def _(a):
    a.st(4, 10, -4, 1).ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.jmp(JEQ, 0, "out", imm=0)
    a.mov64(6, src=0).mov64(1, src=0).call_bpf("sub")
    a.ldx(8, 2, 6, 0).mov64(0, src=2).exit()
    a.label("out").mov64(0, -1).exit()
    a.label("sub").mov64(2, 5).stx(8, 1, 0, 2).mov64(0, 0).exit()


@kat("callbpf_frame_overflow_panics", (PANIC, P_INDEX), cite="inst_call_bpf.go:23-28 (&StackFrames[8])")
def _(a):
    a.call_bpf("sub").exit()
    a.label("sub").call_bpf("sub").exit()


@kat("callbpf_depth_7_ok", (OK, 7), cite="inst_call_bpf.go:23-28 (frames 1..7 exist)")
def _(a):
    a.mov64(0, 0).call_bpf("f1").exit()
    for k in range(1, 8):
        a.label(f"f{k}").add64(0, 1)
        if k < 7:
            a.call_bpf(f"f{k + 1}")
        a.exit()


# ---- tail calls (emulator/helper_functions.go:133-210)
PROGS = (MapDef(MAP_PROG_ARRAY, 4, 4, 4), None)


def _prog_table(*idx):
    """PROG_ARRAY contents as host-side updates (AbstractMapToVM gives PROG_ARRAY no InitialData)."""
    return {0: [(int(k).to_bytes(4, "little"), int(i).to_bytes(4, "little")) for k, i in enumerate(idx)]}


def _tail(a, key=0, after=99):
    a.ld_map(2, 1).mov64(3, key).call(12).mov64(0, after).exit()


@kat("tail_call_runs_target", (OK, 42), maps=[PROGS], entries=_prog_table(2),
     cite="helper_functions.go:198-208", extra=[lambda b: b.mov64(0, 42).exit()])
def _(a):
    _tail(a)


@kat("tail_call_keeps_registers_and_stack", (OK, 7 + 100), maps=[PROGS], entries=_prog_table(2),
     cite="helper_functions.go:203-205 (no Reset)",
     extra=[lambda b: b.ldx(8, 0, 10, -8).add64(0, src=6).exit()])
def _(a):
    a.st(8, 10, -8, 7).mov64(6, 100)
    _tail(a)


@kat("tail_call_off_by_one_no_program", (VMERR, E_NO_PROGRAM), maps=[PROGS], entries=_prog_table(3),
     cite="helper_functions.go:189 (len(Programs) < idx lets idx == len through)", extra=[lambda b: b.mov64(0, 1).exit()])
def _(a):
    _tail(a)


@kat("tail_call_index_too_large_efault", (OK, -14), maps=[PROGS], entries=_prog_table(4),
     cite="helper_functions.go:189-192", extra=[lambda b: b.mov64(0, 1).exit()])
def _(a):
    a.ld_map(2, 1).mov64(3, 0).call(12).exit()


@kat("tail_call_zero_index_vmerr", (VMERR, E_NO_PROGRAM | IN_HELPER), maps=[PROGS], entries=_prog_table(0),
     cite="helper_functions.go:194-196")
def _(a):
    _tail(a)


@kat("tail_call_key_beyond_array", (VMERR, 16 | IN_HELPER), maps=[PROGS], entries=_prog_table(2),
     cite="helper_functions.go:178-181 (Lookup returned IMM 0)", extra=[lambda b: b.mov64(0, 1).exit()])
def _(a):
    _tail(a, key=9)


@kat("tail_call_not_prog_array_efault", (OK, -14), maps=[ARRAY8], cite="helper_functions.go:143-146")
def _(a):
    a.ld_map(2, 1).mov64(3, 0).call(12).exit()


# ---- LRU hash (emulator/maps_hash_lru.go)
LRU2 = (MapDef(MAP_LRU_HASH, 4, 8, 2), None)


def _lru_update(a, key, val):
    a.st(4, 10, -4, key).st(8, 10, -16, val).ld_map(1, 1).mov64(2, src=10).add64(2, -4)
    a.mov64(3, src=10).add64(3, -16).mov64(4, 0).call(2)


def _lru_lookup(a, key):
    a.st(4, 10, -4, key).ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)


@kat("lru_evicts_least_recently_used", (OK, 20), maps=[LRU2], cite="maps_hash_lru.go:114-119")
def _(a):
    _lru_update(a, 1, 10)
    _lru_update(a, 2, 20)
    _lru_lookup(a, 1)   # 1 becomes most recent: 2 is now the LRU
    _lru_update(a, 3, 30)  # evicts 2
    _lru_lookup(a, 2)
    a.mov64(6, src=0)
    _lru_lookup(a, 1)
    a.ldx(8, 0, 0, 0).add64(0, 10)   # r0 = 10 + 10
    a.exit()


@kat("lru_update_non_pointer_value_still_evicts", (OK, -14), maps=[(MapDef(MAP_LRU_HASH, 4, 8, 1), None)],
     cite="maps_hash_lru.go:114-137 (eviction precedes the value check)")
def _(a):
    _lru_update(a, 1, 10)
    a.st(4, 10, -4, 2).ld_map(1, 1).mov64(2, src=10).add64(2, -4).mov64(3, 0).mov64(4, 0).call(2).exit()


# ---- queue / stack (emulator/maps_queue.go, maps_stack.go; helper_functions.go:255-374)
Q8 = (MapDef(MAP_QUEUE, 0, 8, 16), None)
S8 = (MapDef(MAP_STACK, 0, 8, 16), None)


def _push(a, val):
    a.st(8, 10, -8, val).ld_map(1, 1).mov64(2, src=10).add64(2, -8).call(87)


def _pop_deref(a):
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -24).call(88)
    a.ldx(8, 3, 10, -24).ldx(8, 0, 3, 0).exit()   # the popped MemoryPtr object, then its bytes


@kat("queue_pop_is_fifo", (OK, 5), maps=[Q8], cite="maps_queue.go:79-91, helper_functions.go:311-324")
def _(a):
    _push(a, 5)
    _push(a, 6)
    _push(a, 7)
    _pop_deref(a)


@kat("stack_pop_is_lifo", (OK, 7), maps=[S8], cite="maps_stack.go:79-90")
def _(a):
    _push(a, 5)
    _push(a, 6)
    _push(a, 7)
    _pop_deref(a)


@kat("queue_lookup_by_index", (OK, 6), maps=[Q8], cite="maps_queue.go:39-58")
def _(a):
    _push(a, 5)
    _push(a, 6)
    a.st(4, 10, -4, 1).ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1).ldx(8, 0, 0, 0).exit()


@kat("queue_lookup_out_of_range_e2big", (OK, -7), maps=[Q8], cite="maps_queue.go:50-52")
def _(a):
    a.st(4, 10, -4, 3).ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1).exit()


@kat("peek_empty_queue_e2big_and_nil_r2", (OK, -7), maps=[Q8], cite="helper_functions.go:356-371 (R2 := nil)")
def _(a):
    a.ld_map(1, 1).call(89).exit()


@kat("nil_register_use_panics", (PANIC, P_NIL_DEREF), maps=[Q8], cite="helper_functions.go:371 then registers.go Copy")
def _(a):
    a.ld_map(1, 1).call(89).mov64(0, src=2).exit()


@kat("peek_queue_front", (OK, 5), maps=[Q8], entries={0: [(None, (5).to_bytes(8, "little")), (None, (6).to_bytes(8, "little"))]},
     cite="helper_functions.go:345-372 (R2 := pointer to Values[0])")
def _(a):
    a.ld_map(1, 1).call(89).ldx(8, 0, 2, 0).exit()


@kat("push_on_array_map_vmerr", (VMERR, 16 | IN_HELPER), maps=[ARRAY8], cite="maps.go:76-78 (push not available)")
def _(a):
    _push(a, 1)
    a.exit()


@kat("pop_empty_writes_imm_zero", (OK, 0), maps=[Q8], cite="maps_queue.go:80-82 + helper_functions.go:311-324")
def _(a):
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -8).call(88).ldx(8, 0, 10, -8).exit()


# ---- perf event output (emulator/helper_functions.go:219-252, maps_perf_event_array.go:101-115)
PERF = (MapDef(MAP_PERF_EVENT_ARRAY, 4, 4, 8), None)


@kat("perf_output_appends_event", (OK, 0), maps=[PERF], cite="helper_functions.go:219-252")
def _(a):
    a.st(8, 10, -8, 0x1234).ld_map(2, 1).mov64(4, src=10).add64(4, -8).mov64(5, 8).call(25).exit()


@kat("perf_output_stack_run_widened_panics", (PANIC, P_INDEX), maps=[PERF],
     cite="memory.go:69-91 (a 6-byte read of an 8-byte object widens to 8: r[i:i+8] past 6)")
def _(a):
    a.st(8, 10, -8, 0x1234).ld_map(2, 1).mov64(4, src=10).add64(4, -8).mov64(5, 6).call(25).exit()


@kat("perf_output_from_packet", (OK, 0), maps=[PERF], cite="maps_perf_event_array.go:101-115 (ReadRange of R4)")
def _(a):
    a.ldx(4, 4, 1, 0).ld_map(2, 1).mov64(5, 20).call(25).exit()


@kat("perf_output_negative_size_panics", (PANIC, 6), maps=[PERF], cite="memory.go:181 make([]byte, negative)")
def _(a):
    a.ldx(4, 4, 1, 0).ld_map(2, 1).mov64(5, -1).call(25).exit()


@kat("perf_lookup_shares_event", (OK, 0x34), maps=[PERF], cite="maps_perf_event_array.go:45-65")
def _(a):
    a.st(8, 10, -8, 0x1234).ld_map(2, 1).mov64(4, src=10).add64(4, -8).mov64(5, 8).call(25)
    a.st(4, 10, -12, 0).ld_map(1, 1).mov64(2, src=10).add64(2, -12).call(1).ldx(1, 0, 0, 0).exit()
