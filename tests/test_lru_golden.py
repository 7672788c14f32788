"""LRU_HASH pinned by the reference's own test (emulator/maps_hash_lru_test.go:11-124), restated as the
fixture tests/golden/lru_hash_vectors.json (tests/golden/make_lru_vectors.py writes it).

Two forms of the same op sequence:
  * userspace map ops (Map.Update / Map.Lookup, maps_hash_lru.go:70-161) through the C ABI;
  * a BPF program, one packet per op, calling bpf_map_update_elem / bpf_map_lookup_elem, so the
    device's sequential ordered-map path replays the sequence inside one batch.
Both end with the UsageList [6, 2, 1, 5, 4] and key 3 evicted, on the oracle, the host-simulation
build of the device code and (gpu) the MI355X."""
import json
import os

import numpy as np
import pytest

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "lru_hash_vectors.json")))
u32 = lambda x: int(x).to_bytes(4, "little")


def _map(vm):
    from gobpfld_amd.emulator import MapDef
    m = GOLD["map"]
    return vm.add_map(MapDef(m["type"], m["key_size"], m["value_size"], m["max_entries"]))


def _check_final(vm, mi):
    assert [int.from_bytes(k, "little") for k in vm.map_lru_order(mi)] == GOLD["expect_usage"]
    for k in range(1, 7):  # only evicted keys: a hit would promote and change the order checked above
        if str(k) not in GOLD["expect_entries"]:
            assert vm.map_lookup(mi, u32(k)) is None, f"key {k} should have been evicted"


def _host_ops(lib):
    from gobpfld_amd.emulator import VM, Settings
    vm = VM(Settings(), lib=lib)
    mi = _map(vm)
    for op in GOLD["ops"]:
        if op[0] == "update":
            vm.map_update(mi, u32(op[1]), u32(op[2]))
        else:
            assert vm.map_lookup(mi, u32(op[1])) == u32(10 + op[1])
    _check_final(vm, mi)
    keys, vals = vm.map_dump(mi)
    got = {int.from_bytes(bytes(k), "little"): int.from_bytes(bytes(v), "little") for k, v in zip(keys, vals)}
    assert got == {int(k): v for k, v in GOLD["expect_entries"].items()}
    vm.close()


def test_lru_userspace_ops_oracle(oracle_lib):
    _host_ops(oracle_lib)


def test_lru_userspace_ops_hostsim(hostsim_lib):
    _host_ops(hostsim_lib)


@pytest.mark.gpu
def test_lru_userspace_ops_device(gpu_lib):
    _host_ops(gpu_lib)


def _program(mi):
    """Packet = [op u32][key u32][value u32]; op 0 updates (returns the helper's r0), op 1 looks up
    (returns the value or 0xFFFF)."""
    from gobpfld_amd.asm import JEQ, JNE, Asm
    a = Asm()
    a.ldx(4, 6, 1, 0)                       # r6 = ctx->data
    a.ldx(4, 7, 6, 0)                       # op
    a.ldx(4, 1, 6, 4).stx(4, 10, -4, 1)     # key  -> fp-4
    a.ldx(4, 1, 6, 8).stx(4, 10, -8, 1)     # value -> fp-8
    a.ld_map(1, mi).mov64(2, src=10).add64(2, -4)
    a.jmp(JNE, 7, "lookup", imm=0)
    a.mov64(3, src=10).add64(3, -8).mov64(4, 0).call(2).exit()
    a.label("lookup").call(1)
    a.jmp(JEQ, 0, "miss", imm=0)
    a.ldx(4, 0, 0, 0).exit()
    a.label("miss").mov64(0, 0xFFFF).exit()
    return a.assemble()


def _packets():
    from gobpfld_amd._native import np_dtypes
    d_desc, _, _ = np_dtypes()
    ops = GOLD["ops"]
    umem = np.zeros(len(ops) * 64, dtype=np.uint8)
    descs = np.zeros(len(ops), dtype=d_desc)
    for i, op in enumerate(ops):
        rec = [0 if op[0] == "update" else 1, op[1], op[2] if op[0] == "update" else 0]
        umem[i * 64:i * 64 + 12] = np.array(rec, dtype="<u4").view(np.uint8)
    descs["addr"] = np.arange(len(ops)) * 64
    descs["len"] = 64
    return umem, descs


EXPECT_R0 = [0, 0, 0, 0, 0, 11, 12, 0]


def _vm(lib, device=None):
    from gobpfld_amd.emulator import VM, Settings
    vm = VM(Settings() if device is None else Settings(device=device), lib=lib)
    mi = _map(vm)
    vm.set_entrypoint(vm.add_raw_program(_program(mi)))
    return vm, mi


@pytest.mark.parametrize("which", ["oracle", "hostsim"])
def test_lru_program_cpu(oracle_lib, hostsim_lib, which):
    vm, mi = _vm(oracle_lib if which == "oracle" else hostsim_lib)
    umem, descs = _packets()
    if which == "oracle":
        r0 = vm.run_batch(umem, descs).verdicts
    else:
        r0 = np.zeros(len(descs), dtype=np.uint32)
        vm.run_batch_device(umem.ctypes.data, umem.size, descs.ctypes.data, len(descs), d_verdicts=r0.ctypes.data)
    assert list(r0) == EXPECT_R0
    _check_final(vm, mi)
    vm.close()


@pytest.mark.gpu
def test_lru_program_device(gpu_lib):
    import torch
    vm, mi = _vm(gpu_lib, device=0)
    umem, descs = _packets()
    du = torch.from_numpy(umem).cuda()
    dd = torch.from_numpy(descs.view(np.uint8)).cuda()
    dv = torch.zeros(len(descs), dtype=torch.int32, device="cuda")
    vm.run_batch_device(du.data_ptr(), du.numel(), dd.data_ptr(), len(descs), d_verdicts=dv.data_ptr())
    torch.cuda.synchronize()
    assert list(dv.cpu().numpy().view(np.uint32)) == EXPECT_R0
    _check_final(vm, mi)
    vm.close()
