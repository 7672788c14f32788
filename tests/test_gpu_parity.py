"""GPU parity: the HIP product (gobpfld_amd/libxdpemu.so on gfx950) against the CPU oracle.

Bit-exact comparison of per-packet status/code/pc/R0, the R0..R9 parity records, packet bytes and
final map contents, on the KATs, the five BASELINE configs at reduced size, random programs, and
size-independent properties of the full-size C2 batch.
"""
import numpy as np
import pytest

from gobpfld_amd import workloads as W
from gobpfld_amd.emulator import EmulatorError, ENGINE_INTERP, ENGINE_JIT, MODE_KEYED, MODE_PARALLEL, MODE_SEQUENTIAL, VM, Settings
from kats import KATS
from parity import assert_same, config_case, packets, run_one

pytestmark = pytest.mark.gpu
ENGINES = [ENGINE_INTERP, ENGINE_JIT]
ENGINE_IDS = ["interp", "jit"]
FUZZ_COUNTS = {ENGINE_INTERP: 240, ENGINE_JIT: 48}
CONFIGS = [("c1", 1024, None), ("c2", 65536, None), ("c3", 30000, 8192), ("c4", 8192, None), ("c5", 30000, 8192)]


@pytest.mark.parametrize("engine", ENGINES, ids=ENGINE_IDS)
@pytest.mark.parametrize("k", KATS, ids=[k["name"] for k in KATS])
def test_kat_device_equals_oracle(gpu_lib, oracle_lib, k, engine):
    umem, descs = packets(64, k["pkt"], seed=7)
    # every KAT runs on both engines: calls, tail calls, indirect helpers and the ordered maps take the
    # per-program kernel's dynamic form (xe_jit.cpp generate_dynamic)
    a = run_one(gpu_lib, k["program"], k["maps"], umem, descs, entries=k["entries"], settings=Settings(engine=engine))
    assert a[0].stats["engine_used"] == engine
    b = run_one(oracle_lib, k["program"], k["maps"], umem, descs, entries=k["entries"])
    assert_same(a, b, k["name"])


@pytest.mark.parametrize("engine", ENGINES, ids=ENGINE_IDS)
@pytest.mark.parametrize("name,n,cap", CONFIGS)
def test_config_device_equals_oracle(gpu_lib, oracle_lib, name, n, cap, engine):
    prog, maps, entries, umem, descs = config_case(name, n, cap)
    a = run_one(gpu_lib, prog, maps, umem, descs, entries=entries, settings=Settings(engine=engine))
    assert a[0].stats["engine_used"] == engine
    b = run_one(oracle_lib, prog, maps, umem, descs, entries=entries)
    assert_same(a, b, name)
    assert a[0].stats["mode_used"] == MODE_PARALLEL, "commutative config must run in parallel mode"


@pytest.mark.parametrize("engine", ENGINES, ids=ENGINE_IDS)
def test_sequential_mode_equals_oracle(gpu_lib, oracle_lib, engine):
    prog, maps, entries, umem, descs = config_case("c2", 2048)
    a = run_one(gpu_lib, prog, maps, umem, descs, entries=entries, settings=Settings(mode=MODE_SEQUENTIAL, engine=engine))
    b = run_one(oracle_lib, prog, maps, umem, descs, entries=entries)
    assert_same(a, b, "c2 sequential")
    assert a[0].stats["mode_used"] == MODE_SEQUENTIAL


@pytest.mark.parametrize("engine", ENGINES, ids=ENGINE_IDS)
def test_ordered_program_falls_back(gpu_lib, oracle_lib, engine):
    k = next(k for k in KATS if k["name"] == "nonatomic_rmw_on_map_value_ordered")
    umem, descs = packets(3000, 64, seed=3)
    a = run_one(gpu_lib, k["program"], k["maps"], umem, descs, settings=Settings(engine=engine))
    b = run_one(oracle_lib, k["program"], k["maps"], umem, descs)
    assert_same(a, b, "ordered rmw")
    # one key written by every packet: a single chain holding the whole batch, which the staged
    # one-lane replay runs faster than a chain lane (xe_runtime.cpp keyed: XE_KS_CLONG)
    assert a[0].stats["conflict"] == 1 and a[0].stats["mode_used"] == MODE_SEQUENTIAL
    # packet i saw counter value i: the exact sequential order
    assert (a[0].results["r0"] == np.arange(3000)).all()


@pytest.mark.parametrize("name", ["c2", "c3", "c4", "c5"])
def test_device_resident_api_verdicts_only(gpu_lib, oracle_lib, name):
    """Device-resident batch asking for verdicts only: the per-program kernel's verdict-only variant
    (no result / register records) against the oracle — verdicts, the final map, retired steps."""
    import torch
    n = 1 << 18 if name == "c2" else 1 << 16
    umem, descs = W.build_batch(name, 0, n)
    vm = VM(Settings(), lib=gpu_lib)
    W.setup_vm(vm, name)
    d_umem = torch.from_numpy(umem).cuda()
    d_desc = torch.from_numpy(descs.view(np.uint8)).cuda()
    d_ver = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = vm.run_batch_device(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), n, d_verdicts=d_ver.data_ptr())
    torch.cuda.synchronize()
    ver = d_ver.cpu().numpy().view(np.uint32)
    dev_map = vm.map_dump(1) if name != "c4" else None  # C4 has no map
    vm.close()
    ov = VM(Settings(), lib=oracle_lib)
    W.setup_vm(ov, name)
    r = ov.run_batch(umem.copy(), descs)
    assert (ver == r.verdicts).all()
    if dev_map is not None:
        om = ov.map_dump(1)
        assert (np.array_equal(dev_map[0], om[0]) and np.array_equal(dev_map[1], om[1])) if isinstance(om, tuple) else dev_map == om
    assert st["steps"] == r.stats["steps"]
    assert st["engine_used"] == 2  # the per-program kernel


def _c2_expected(idx):
    """Independent expectation of C2 from the generated headers (no emulator involved)."""
    h = W.headers_c2(idx, 64).astype(np.int64)
    et = (h[:, 12] << 8) | h[:, 13]
    vlan = et == 0x8100
    et = np.where(vlan, (h[:, 16] << 8) | h[:, 17], et)
    l3 = np.where(vlan, 18, 14)
    rows = np.arange(len(idx))
    proto = np.where(et == 0x0800, h[rows, l3 + 9], np.where(et == 0x86DD, h[rows, l3 + 6], -1))
    counted = proto >= 0
    verdict = np.where(np.isin(proto, [1, 6, 17]), 2, 1)
    counts = np.bincount(proto[counted], minlength=256)
    return verdict, counts


def test_c2_full_size_properties(gpu_lib):
    """16M x 64 B C2 batch: verdict histogram and per-proto counters equal the header-derived truth."""
    import torch
    n = 16 * 1024 * 1024
    umem, descs = W.build_batch("c2", 0, n)
    vm = VM(Settings(), lib=gpu_lib)
    W.setup_vm(vm, "c2")
    d_umem = torch.from_numpy(umem).cuda()
    d_desc = torch.from_numpy(descs.view(np.uint8)).cuda()
    d_ver = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = vm.run_batch_device(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), n, d_verdicts=d_ver.data_ptr())
    torch.cuda.synchronize()
    assert st["status_count"][0] == n and st["conflict"] == 0
    verdict, counts = _c2_expected(np.arange(n, dtype=np.uint64))
    ver = d_ver.cpu().numpy().view(np.uint32)
    assert (ver == verdict).all()
    got = np.frombuffer(vm.map_dump(1), dtype=np.uint64)
    assert (got == counts).all()
    # a second identical run doubles every counter (idempotent verdicts, commutative counters)
    vm.run_batch_device(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), n, d_verdicts=d_ver.data_ptr())
    torch.cuda.synchronize()
    assert (np.frombuffer(vm.map_dump(1), dtype=np.uint64) == 2 * counts).all()
    vm.close()


@pytest.mark.parametrize("engine,count", list(FUZZ_COUNTS.items()), ids=ENGINE_IDS)
def test_fuzz_device_equals_oracle(gpu_lib, oracle_lib, engine, count):
    """Random programs (tests/fuzz.py): device == oracle on every observable, per engine."""
    from fuzz import gen_program
    from test_fuzz_cpu import fuzz_packets
    for seed in range(count):
        prog, maps, entries, settings = gen_program(seed, 24 + seed % 64)
        umem, descs = fuzz_packets(seed, 64)
        settings.engine = engine
        b = run_one(oracle_lib, prog, maps, umem, descs, entries=entries, settings=settings)
        a = run_one(gpu_lib, prog, maps, umem, descs, entries=entries, settings=settings)
        assert a[0].stats["engine_used"] == engine
        assert_same(a, b, f"fuzz seed {seed}")


@pytest.mark.parametrize("engine", ENGINES, ids=ENGINE_IDS)
def test_bpf2bpf_calls_device_equals_oracle(gpu_lib, oracle_lib, engine):
    """The call-heavy analogue of cmd/examples/bpf_to_bpf/src/xdp.c (workloads.prog_bpf2bpf: two
    bpf-to-bpf calls per packet, lifted `stats->pkts++` inside the callee) on both engines: results,
    verdicts and the three stats maps equal the oracle, and the batch stays parallel (lifted adds in the
    callee). With register records the loaded values must be exact, so that batch replays in order."""
    prog, maps, entries, umem, descs = config_case("bpf2bpf", 65536)
    a = run_one(gpu_lib, prog, maps, umem, descs, entries=entries, regs=False, settings=Settings(engine=engine))
    b = run_one(oracle_lib, prog, maps, umem, descs, entries=entries, regs=False)
    assert_same(a, b, "bpf2bpf")
    assert a[0].stats["engine_used"] == engine and a[0].stats["mode_used"] == MODE_PARALLEL, a[0].stats
    umem, descs = umem[: 4096 * 64], descs[:4096]
    a = run_one(gpu_lib, prog, maps, umem, descs, entries=entries, regs=True, settings=Settings(engine=engine))
    b = run_one(oracle_lib, prog, maps, umem, descs, entries=entries, regs=True)
    assert_same(a, b, "bpf2bpf regs")
