"""Rule chains (xe_jit.cpp rule_chain_at / emit_rule_dispatch): a first-match chain of N >= 8 rules, each
"JNE rX, K -> next rule", further tests against immediates, then JA to its action, is compiled to a
hashed dispatch on rX instead of a walk over every rule. The reference walks the rules one instruction at
a time (emulator/vm.go:117-173, inst_jeq.go / inst_jgt.go / inst_jne.go), so the dispatch must pick the
same rule and retire the same steps: one per rule before the exit, the tests of every rule whose K
matched up to the one that failed, and the exit rule's tests and JA. Compared with the oracle per packet
(result, R0-R9 and the packet's step count in the register record) and, for the verdict-only variant,
the batch's step total and status histogram. Cases: C4's shape with keys shared by several rules, 64-bit
keys including negative ones (sign-extended immediates), a dispatch register that holds a pointer for some
packets (every JNE taken), one and three further tests per rule."""
import numpy as np
import pytest

from gobpfld_amd.asm import JEQ, JGE, JGT, JNE, JSGE, JSGT, JSLE, JSLT, Asm
from gobpfld_amd.emulator import ENGINE_JIT, VM, Settings
from parity import assert_same, run_one


def _rules(kind):
    rng = np.random.default_rng({"dups": 1, "wide": 2, "ptr": 3, "one": 4, "three": 5}[kind])
    rules = []
    for k in range(24):
        key = {"dups": 0x0A000001 + (k // 3), "wide": -(k // 2 + 1) * 0x01000001, "ptr": 0x0A000001 + k,
               "one": 0x0A000001 + (k % 10), "three": 0x0A000001 + (k // 4)}[kind]
        rules.append((int(key), int(rng.choice([6, 17, 1])), int(rng.integers(1000, 60000)),
                      int(rng.integers(-5, 5)), k % 2))
    return rules


def prog_rules(kind):
    """r6 = data; 32-byte bound; r8 = u32 packet[0] (u64 packet[0:8] for "wide"), r9 = u8 packet[8],
    r5 = u16 packet[10], r4 = u64 packet[16]; then 24 rules; default verdict 7; a rule's action: verdict
    2 (even rules) or 1 (odd). "ptr": r8 holds the packet pointer on packets whose byte 12 is odd."""
    a = Asm()
    a.ldx(4, 6, 1, 0).ldx(4, 7, 1, 4)
    a.mov64(2, src=6).add64(2, 32)
    a.jmp(JGT, 2, "short", src=7)
    a.ldx(8 if kind == "wide" else 4, 8, 6, 0)
    a.ldx(1, 9, 6, 8)
    a.ldx(2, 5, 6, 10)
    a.ldx(8, 4, 6, 16)
    if kind == "ptr":
        a.ldx(1, 3, 6, 12).alu64(0x50, 3, 1)
        a.jmp(JEQ, 3, "r0", imm=0)
        a.mov64(8, src=6)
    for k, (key, proto, dmax, lo, act) in enumerate(_rules(kind)):
        nxt = f"r{k + 1}"
        a.label(f"r{k}")
        if kind == "wide":
            a.jmp(JNE, 8, nxt, imm=key)
        else:
            a.jmp(JNE, 8, nxt, imm=key if key < 2**31 else key - 2**32, wide=False)
        if kind != "one":
            a.jmp(JNE, 9, nxt, imm=proto)
        a.jmp(JGT, 5, nxt, imm=dmax)
        if kind == "three":
            a.jmp(JSGE, 4, nxt, imm=lo)
        a.ja("act1" if act else "act2")
    a.label("r24").mov64(0, 7).exit()
    a.label("act1").mov64(0, 1).exit()
    a.label("act2").mov64(0, 2).exit()
    a.label("short").mov64(0, 0).exit()
    return a.assemble()


def batch(kind, n, seed=9):
    """n packets of 40 bytes (a few of 24: short), keys from the rules on 3 of 4, fields random."""
    from gobpfld_amd._native import np_dtypes
    d_desc, _, _ = np_dtypes()
    rng = np.random.default_rng(seed)
    rules = _rules(kind)
    umem = rng.integers(0, 256, size=n * 40, dtype=np.uint8).reshape(n, 40)
    pick = rng.integers(0, len(rules), size=n)
    hit = rng.random(n) < 0.75
    for i in np.nonzero(hit)[0]:
        key, proto, dmax, lo, _ = rules[pick[i]]
        umem[i, 0:8] = np.frombuffer(int(key & (2**64 - 1)).to_bytes(8, "little"), np.uint8)
        if rng.random() < 0.7:
            umem[i, 8] = proto
            v = int(rng.integers(0, dmax + 1))
            umem[i, 10:12] = np.frombuffer(v.to_bytes(2, "little"), np.uint8)
    descs = np.zeros(n, dtype=d_desc)
    descs["addr"] = np.arange(n) * 40
    descs["len"] = np.where(rng.random(n) < 0.02, 24, 40)
    return umem.reshape(-1).copy(), descs


KINDS = ["dups", "wide", "ptr", "one", "three"]


def test_rule_chain_is_compiled():
    """The generator finds the chain in every case (its dispatch is in the kernel source)."""
    from gobpfld_amd import aot
    for kind in KINDS:
        src = aot.sources([(prog_rules(kind), [], None, Settings(engine=ENGINE_JIT))], variants=(0,))
        assert src and "rule chain: 24 rules on r8" in src[0], kind


def test_rule_programs_hostsim_equal_oracle(hostsim_lib, oracle_lib):
    """The programs themselves on the host simulation (the interpreter's walk): the oracle agrees."""
    for kind in KINDS:
        umem, descs = batch(kind, 2048)
        assert_same(run_one(hostsim_lib, prog_rules(kind), [], umem, descs),
                    run_one(oracle_lib, prog_rules(kind), [], umem, descs), kind)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", KINDS)
def test_rule_chain_device_equals_oracle(gpu_lib, oracle_lib, kind):
    umem, descs = batch(kind, 65536)
    got = run_one(gpu_lib, prog_rules(kind), [], umem, descs, settings=Settings(engine=ENGINE_JIT))
    assert_same(got, run_one(oracle_lib, prog_rules(kind), [], umem, descs), kind)
    assert got[0].stats["engine_used"] == ENGINE_JIT


@pytest.mark.gpu
@pytest.mark.parametrize("kind", KINDS)
def test_rule_chain_verdict_only_steps(gpu_lib, oracle_lib, kind):
    import torch
    n = 65536
    umem, descs = batch(kind, n, seed=21)
    ro = run_one(oracle_lib, prog_rules(kind), [], umem, descs)[0]
    vm = VM(Settings(engine=ENGINE_JIT), lib=gpu_lib)
    vm.set_entrypoint(vm.add_raw_program(prog_rules(kind)))
    vm.prepare()
    d_umem = torch.from_numpy(umem.copy()).cuda()
    d_desc = torch.from_numpy(descs.view(np.uint8)).cuda()
    d_ver = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = vm.run_batch_device(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), n, d_verdicts=d_ver.data_ptr())
    torch.cuda.synchronize()
    vm.close()
    assert (d_ver.cpu().numpy().view(np.uint32) == ro.verdicts).all()
    assert st["steps"] == ro.stats["steps"]
    assert list(st["status_count"][:8]) == list(np.bincount(ro.results["status"], minlength=8)[:8])


# ---- random rule chains: the dispatch's choices against the oracle's walk over many shapes
# (the reference has no JSET / JLT / JLE instruction: emulator/ decodes them and stops, xe_runtime.cpp)
EXTRA_OPS = [JNE, JEQ, JGT, JGE, JSGT, JSGE, JSLT, JSLE]
FIELDS = {9: (8, 1), 5: (10, 2), 4: (16, 8), 3: (24, 4)}  # register: (packet offset, bytes)


def random_rules(seed):
    """(wide, extra-test shape [(register, op, wide)], rules [(key, [imm per extra test], verdict)])"""
    rng = np.random.default_rng(1000 + seed)
    wide = bool(rng.random() < 0.5)
    shape = [(int(rng.choice(list(FIELDS))), int(rng.choice(EXTRA_OPS)), bool(rng.random() < 0.5))
             for _ in range(int(rng.integers(0, 4)))]
    pool = [int(x) for x in rng.integers(-2**31, 2**31, size=int(rng.integers(3, 20)))]
    rules = []
    lo = max(8, 33 // (1 + len(shape)) + 1)  # (the block form: more than 32 conditional jumps)
    for _ in range(int(rng.integers(lo, max(lo, 40) + 1))):
        key = int(rng.choice(pool))
        imms = [int(rng.integers(-300, 70000)) if rng.random() < 0.8 else int(rng.integers(-2**31, 2**31))
                for _ in shape]
        rules.append((key, imms, int(rng.integers(1, 4))))
    return wide, shape, rules


def prog_random(seed):
    wide, shape, rules = random_rules(seed)
    a = Asm()
    a.ldx(4, 6, 1, 0).ldx(4, 7, 1, 4)
    a.mov64(2, src=6).add64(2, 32)
    a.jmp(JGT, 2, "short", src=7)
    a.ldx(8 if wide else 4, 8, 6, 0)
    for reg, (off, size) in FIELDS.items():
        a.ldx(size, reg, 6, off)
    for k, (key, imms, verdict) in enumerate(rules):
        nxt = f"r{k + 1}"
        a.label(f"r{k}")
        a.jmp(JNE, 8, nxt, imm=key, wide=wide)
        for (reg, op, w), imm in zip(shape, imms):
            a.jmp(op, reg, nxt, imm=imm, wide=w)
        a.ja(f"v{verdict}")
    a.label(f"r{len(rules)}").mov64(0, 7).exit()
    for v in (1, 2, 3):
        a.label(f"v{v}").mov64(0, v).exit()
    a.label("short").mov64(0, 0).exit()
    return a.assemble()


def random_batch(seed, n):
    from gobpfld_amd._native import np_dtypes
    d_desc, _, _ = np_dtypes()
    wide, shape, rules = random_rules(seed)
    rng = np.random.default_rng(2000 + seed)
    umem = rng.integers(0, 256, size=(n, 40), dtype=np.uint8)
    for i in range(n):
        if rng.random() < 0.8:
            key, imms, _ = rules[int(rng.integers(0, len(rules)))]
            umem[i, 0:8] = np.frombuffer(int(key & (2**64 - 1)).to_bytes(8, "little"), np.uint8)
            for (reg, op, w), imm in zip(shape, imms):
                if rng.random() < 0.5:  # the field near the rule's immediate
                    off, size = FIELDS[reg]
                    v = (imm + int(rng.integers(-2, 3))) & ((1 << (8 * size)) - 1)
                    umem[i, off:off + size] = np.frombuffer(v.to_bytes(size, "little"), np.uint8)
    descs = np.zeros(n, dtype=d_desc)
    descs["addr"] = np.arange(n) * 40
    descs["len"] = 40
    return umem.reshape(-1).copy(), descs


RANDOM_SEEDS = range(16)


def test_random_chains_compile_as_dispatch():
    from gobpfld_amd import aot
    srcs = aot.sources([(prog_random(s), [], None, Settings(engine=ENGINE_JIT)) for s in RANDOM_SEEDS], variants=(0,))
    assert sum("rule chain:" in x for x in srcs) == len(RANDOM_SEEDS), [("rule chain:" in x) for x in srcs]


def test_random_chains_hostsim_equal_oracle(hostsim_lib, oracle_lib):
    for seed in RANDOM_SEEDS:
        umem, descs = random_batch(seed, 512)
        assert_same(run_one(hostsim_lib, prog_random(seed), [], umem, descs),
                    run_one(oracle_lib, prog_random(seed), [], umem, descs), f"seed {seed}")


@pytest.mark.gpu
def test_random_chains_device_equal_oracle(gpu_lib, oracle_lib):
    """16 random chains (8-40 rules, 32- or 64-bit keys with repeats, 0-3 further tests of any jump op and
    width) on the per-program kernels: results, registers and per-packet steps equal the oracle's walk."""
    for seed in RANDOM_SEEDS:
        umem, descs = random_batch(seed, 8192)
        got = run_one(gpu_lib, prog_random(seed), [], umem, descs, settings=Settings(engine=ENGINE_JIT))
        assert_same(got, run_one(oracle_lib, prog_random(seed), [], umem, descs), f"seed {seed}")
        assert got[0].stats["engine_used"] == ENGINE_JIT
