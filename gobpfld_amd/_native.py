"""ctypes binding of the C ABI declared in include/xdpemu.h.

The same binding drives three libraries with identical signatures: the product
(gobpfld_amd/libxdpemu.so, prefix ``xe_``), and — in tests only — the CPU oracle
(oracle/liboracle.so, prefix ``orc_``) and the host simulation of the device logic.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PRODUCT_LIB = ROOT / "gobpfld_amd" / "libxdpemu.so"
TUNING_LIB = ROOT / "gobpfld_amd" / "libxdpemu_tuning.so"  # -DXE_TUNING debug build (scripts/ A/B runs)


def product_path() -> Path:
    """The product library, or — only when XE_LIB names it — the tuning build of the same sources
    (`python -m gobpfld_amd.build --tuning`). Nothing else may stand in for the product: XE_LIB naming
    any other file (the host simulation, the oracle, a stray copy) is an error, not a silent swap."""
    import os
    env = os.environ.get("XE_LIB")
    if not env:
        return PRODUCT_LIB
    p = Path(env).resolve()
    if p not in (PRODUCT_LIB.resolve(), TUNING_LIB.resolve()):
        raise RuntimeError(f"XE_LIB={env}: only {PRODUCT_LIB.name} or {TUNING_LIB.name} may serve as the product library")
    return p


class Desc(C.Structure):  # xsk.go:695-701
    _fields_ = [("addr", C.c_uint64), ("len", C.c_uint32), ("options", C.c_uint32)]


class Result(C.Structure):
    _fields_ = [("status", C.c_uint8), ("r0_kind", C.c_uint8), ("code", C.c_uint16),
                ("pc", C.c_uint32), ("r0", C.c_int64)]


class Regs(C.Structure):
    _fields_ = [("val", C.c_int64 * 10), ("kind", C.c_uint8 * 10), ("region", C.c_uint8 * 10),
                ("map", C.c_uint8 * 10), ("pad", C.c_uint8 * 2), ("steps", C.c_uint32)]


class MapDef(C.Structure):  # map_definition.go:15-27
    _fields_ = [("type", C.c_uint32), ("key_size", C.c_uint32), ("value_size", C.c_uint32),
                ("max_entries", C.c_uint32), ("flags", C.c_uint32)]


class Settings(C.Structure):  # emulator/vm.go:282-296 + device knobs
    _fields_ = [("stack_frame_size", C.c_int32), ("max_stack_frames", C.c_int32),
                ("max_steps", C.c_uint64), ("ingress_ifindex", C.c_uint32),
                ("rx_queue_index", C.c_uint32), ("device", C.c_int32), ("mode", C.c_uint32),
                ("engine", C.c_uint32)]


class PcapInfo(C.Structure):  # include/xdpemu_io.h
    _fields_ = [("linktype", C.c_uint32), ("snaplen", C.c_uint32), ("nanosecond", C.c_uint32),
                ("swapped", C.c_uint32), ("first_record", C.c_uint64)]


class TraceRec(C.Structure):  # xe_trace_rec: one Step's VM.String (emulator/vm.go:248-270)
    _fields_ = [("packet", C.c_uint32), ("step", C.c_uint32), ("pc", C.c_int32), ("pi", C.c_int32),
                ("sf", C.c_uint32), ("kind", C.c_uint8 * 11), ("pad", C.c_uint8), ("val", C.c_int64 * 11)]


# xe_helper_fn: int fn(void* user, uint32_t packet, const int64_t args[5], const uint8_t kinds[5], int64_t* r0)
HELPER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_uint32, C.POINTER(C.c_int64), C.POINTER(C.c_uint8),
                        C.POINTER(C.c_int64))


class BatchStats(C.Structure):
    _fields_ = [("packets", C.c_uint64), ("steps", C.c_uint64), ("status_count", C.c_uint64 * 8),
                ("mode_used", C.c_uint32), ("conflict", C.c_uint32), ("kernel_ms", C.c_float),
                ("total_ms", C.c_float), ("engine_used", C.c_uint32), ("grid_blocks", C.c_uint32)]


# numpy dtypes matching the structs (for zero-copy batch buffers)
def np_dtypes():
    import numpy as np
    desc = np.dtype([("addr", "<u8"), ("len", "<u4"), ("options", "<u4")])
    result = np.dtype([("status", "u1"), ("r0_kind", "u1"), ("code", "<u2"), ("pc", "<u4"), ("r0", "<i8")])
    regs = np.dtype([("val", "<i8", (10,)), ("kind", "u1", (10,)), ("region", "u1", (10,)),
                     ("map", "u1", (10,)), ("pad", "u1", (2,)), ("steps", "<u4")], align=True)
    assert desc.itemsize == 16 and result.itemsize == 16 and regs.itemsize == C.sizeof(Regs)
    return desc, result, regs


def np_trace_dtype():
    import numpy as np
    t = np.dtype([("packet", "<u4"), ("step", "<u4"), ("pc", "<i4"), ("pi", "<i4"), ("sf", "<u4"),
                  ("kind", "u1", (11,)), ("pad", "u1"), ("val", "<i8", (11,))], align=True)
    assert t.itemsize == C.sizeof(TraceRec) == 120
    return t


P = C.c_void_p
_SIGS = {
    "default_settings": (C.c_int, [P]),
    "create": (C.c_int, [P, C.POINTER(P)]),
    "destroy": (None, [P]),
    "last_error": (C.c_char_p, [P]),
    "add_raw_program": (C.c_int, [P, P, C.c_uint32, C.POINTER(C.c_int32)]),
    "set_entrypoint": (C.c_int, [P, C.c_int32]),
    "add_map": (C.c_int, [P, P, P, C.c_size_t, C.POINTER(C.c_int32)]),
    "map_lookup": (C.c_int, [P, C.c_int32, P, P]),
    "map_update": (C.c_int, [P, C.c_int32, P, P]),
    "map_delete": (C.c_int, [P, C.c_int32, P]),
    "map_update_batch": (C.c_int, [P, C.c_int32, P, P, C.c_uint64]),
    "map_count": (C.c_int, [P, C.c_int32, C.POINTER(C.c_uint64)]),
    "map_dump": (C.c_int, [P, C.c_int32, P, P, C.c_uint64, C.POINTER(C.c_uint64)]),
    "map_dump_list": (C.c_int, [P, C.c_int32, P, C.c_uint64, P, C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "map_lru_order": (C.c_int, [P, C.c_int32, P, C.c_uint64, C.POINTER(C.c_uint64)]),
    "map_push": (C.c_int, [P, C.c_int32, P]),
    "run_batch": (C.c_int, [P, P, C.c_uint64, P, C.c_uint32, P, P, P, P]),  # oracle form
    "run_batch_host": (C.c_int, [P, P, C.c_uint64, P, C.c_uint32, P, P, P, P]),
    "run_batch_device": (C.c_int, [P, P, C.c_uint64, P, C.c_uint32, P, P, P, P, P]),
    "run_batch_device_async": (C.c_int, [P, P, C.c_uint64, P, C.c_uint32, P, P, P, P, P]),
    "sync": (C.c_int, [P]),
    "cancel": (C.c_int, [P, C.POINTER(C.c_uint32)]),
    "trace_config": (C.c_int, [P, P, C.c_uint32, C.c_uint32]),
    "trace_read": (C.c_int, [P, C.c_uint32, P, C.c_uint32, C.POINTER(C.c_uint32)]),
    "set_helper": (C.c_int, [P, C.c_uint32, HELPER_FN, P]),
    "reset_helper": (C.c_int, [P, C.c_uint32]),
    "prepare": (C.c_int, [P]),
    "debug_set_schedule": (C.c_int, [P, C.c_uint32]),
    "debug_set_lru_epoch": (C.c_int, [P, C.c_uint64]),
    "debug_map_pool": (C.c_int, [P, C.c_int32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "set_kernel_cache": (C.c_int, [C.c_char_p]),
    "kernel_source": (C.c_int, [P, C.c_int, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "compile_kernel_source": (C.c_int, [C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p, C.c_size_t]),
    "kernel_object_name": (C.c_int, [C.c_char_p, C.c_char_p, C.c_char_p, C.c_size_t]),
    "kernel_cache_stats": (C.c_int, [C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_double)]),
    "map_values_bytes": (C.c_int, [P, C.c_int32, C.POINTER(C.c_uint64)]),
    "map_delta": (C.c_int, [P, C.c_int32, C.c_uint32, P, P]),
    "map_apply_delta": (C.c_int, [P, C.c_int32, C.c_uint32, P, P]),
    "map_delta_lane": (C.c_int, [P, C.c_int32, C.POINTER(C.c_uint32)]),
    "footprint": (C.c_int, [P, C.POINTER(C.c_uint64), C.c_uint32, C.POINTER(C.c_uint32)]),
    "shard_check": (C.c_int, [P, C.c_uint32, C.c_uint32, P]),
    "epoch_begin": (C.c_int, [P, P]),
    "epoch_end": (C.c_int, [P]),
    "map_state_bytes": (C.c_int, [P, C.c_int32, C.POINTER(C.c_uint64)]),
    "map_state_export": (C.c_int, [P, C.c_int32, P, P]),
    "map_state_import": (C.c_int, [P, C.c_int32, P, P]),
    "multi_create": (C.c_int, [P, C.c_uint32, C.POINTER(P)]),
    "multi_destroy": (None, [P]),
    "multi_last_error": (C.c_char_p, [P]),
    "run_batch_multi": (C.c_int, [P, P, P, P, P, P, P, P, P]),
    "version": (C.c_char_p, []),
    "device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "decode_names": (C.c_int, [P, C.c_uint32, C.c_char_p, C.c_size_t]),
    # include/xdpemu_io.h
    "pcap_header": (C.c_int, [P, C.c_uint64, P]),
    "pcap_count": (C.c_int, [P, C.c_uint64, P, C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "pcap_fill": (C.c_int, [P, C.c_uint64, P, C.POINTER(C.c_uint64), P, C.c_uint64, C.c_uint32, C.c_uint32, P,
                            C.c_uint64, C.c_uint32, P, P, P, C.POINTER(C.c_uint32)]),
    "pcap_pack": (C.c_int, [P, C.c_uint64, P, C.POINTER(C.c_uint64), P, C.c_uint64, C.c_uint32, C.c_uint32,
                            C.c_uint32, P, P, P, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)]),
}

# every symbol include/xdpemu.h declares (checked by tests/test_abi.py)
HEADER_SYMBOLS = [
    "xe_default_settings", "xe_create", "xe_destroy", "xe_last_error", "xe_add_raw_program",
    "xe_set_entrypoint", "xe_add_map", "xe_map_lookup", "xe_map_update", "xe_map_delete",
    "xe_map_count", "xe_map_dump", "xe_map_dump_list", "xe_map_lru_order", "xe_map_push", "xe_map_update_batch", "xe_run_batch_device", "xe_run_batch_host",
    "xe_run_batch_device_async", "xe_sync", "xe_prepare", "xe_map_values_bytes", "xe_map_delta", "xe_map_apply_delta", "xe_map_delta_lane", "xe_footprint", "xe_version",
    "xe_device_count", "xe_shard_check", "xe_epoch_begin", "xe_epoch_end", "xe_map_state_bytes", "xe_map_state_export",
    "xe_map_state_import",
    "xe_multi_create", "xe_multi_destroy", "xe_run_batch_multi", "xe_multi_last_error", "xe_debug_set_schedule",
    "xe_debug_set_lru_epoch", "xe_debug_map_pool",
    "xe_set_kernel_cache", "xe_kernel_source", "xe_compile_kernel_source", "xe_kernel_object_name",
    "xe_kernel_cache_stats",
    "xe_cancel", "xe_trace_config", "xe_trace_read", "xe_set_helper", "xe_reset_helper",
]
IO_HEADER_SYMBOLS = ["xe_pcap_header", "xe_pcap_count", "xe_pcap_fill", "xe_pcap_pack"]  # include/xdpemu_io.h


class Lib:
    """A loaded emulator library exposing the xdpemu.h calls without their prefix."""

    def __init__(self, path: Path | str, prefix: str = "xe_"):
        self.path = Path(path)
        if not self.path.exists():
            raise FileNotFoundError(
                f"{self.path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        self.dll = C.CDLL(str(self.path))
        self.prefix = prefix
        for name, (res, args) in _SIGS.items():
            fn = getattr(self.dll, prefix + name, None)
            if fn is None:
                continue
            fn.restype = res
            fn.argtypes = args
            setattr(self, name, fn)

    def has(self, name: str) -> bool:
        return hasattr(self, name)


_product: Lib | None = None


def product() -> Lib:
    """The HIP product library. Raises if it is not built — there is no CPU fallback."""
    global _product
    if _product is None:
        try:  # torch bundles its own HIP runtime: have it loaded first so the process holds one
            import torch  # noqa: F401
        except ImportError:
            pass
        _product = Lib(product_path(), "xe_")
        # the package's ahead-of-time kernel cache (gobpfld_amd/aot.py), when it was built
        kdir = ROOT / "gobpfld_amd" / "kernels"
        if kdir.is_dir() and _product.has("set_kernel_cache"):
            _product.set_kernel_cache(str(kdir).encode())
    return _product
