"""Known-answer tests derived from the reference source.

The reference has no VM execution tests, so each KAT encodes one quirk of the Go emulator with the
answer read off the cited line. The oracle must produce `expect`; the device must equal the oracle.
"""
from __future__ import annotations

from gobpfld_amd.asm import (ADD, ARSH, DIV, JEQ, JGT, JNE, JSGE, JSGT, JSLE, JSLT, LSH, MOD, MUL,
                             RSH, SUB, XOR, Asm, AND, OR)
from gobpfld_amd.emulator import MAP_ARRAY, MAP_HASH, MapDef

OK, VMERR, PANIC, BUDGET, UNSUP = 0, 1, 2, 3, 4
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


def kat(name, expect=None, maps=(), entries=None, pkt=64, cite=""):
    def deco(fn):
        a = Asm()
        fn(a)
        KATS.append(dict(name=name, program=a.assemble(), maps=list(maps), entries=entries or {},
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


@kat("tail_call_unsupported", (UNSUP, None), maps=[ARRAY8], cite="helper_functions.go:133-210 (out of scope)")
def _(a):
    a.call(12).mov64(0, 0).exit()


@kat("ld_abs_not_implemented", (VMERR, E_NOT_IMPL), cite="emulator/inst_load.go:146-148")
def _(a):
    a.emit(0x20, 0, 0, 0, 12).exit()


@kat("callx_dispatch", (OK, (1234 << 32) + 5678), cite="emulator/inst_call_helper.go:49-71")
def _(a):
    a.mov64(3, 14).emit(0x8D, 0, 0, 0, 3).exit()
