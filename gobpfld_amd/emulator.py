"""Host-side mirror of gobpfld's `emulator` package API over the MI355X device emulator.

    vm = VM(Settings())                      # emulator.NewVM            (emulator/vm.go:30-48)
    prog = vm.add_raw_program(insns)         # VM.AddRawProgram          (emulator/vm.go:61-73)
    m = vm.add_map(MapDef(...), initial)     # VM.AddMap/AddAbstractMap  (emulator/vm.go:75-98)
    vm.set_entrypoint(prog)                  # VM.SetEntrypoint          (emulator/vm.go:100-108)
    res = vm.run_batch(umem, descs)          # Reset + R1=ctx + Run per packet (vm.go:110-246)
    vm.map_dump(m)                           # final map state (Map.Keys + Lookup)

Errors raise EmulatorError carrying the library's message (the Go API returns `error`).
Per-packet failures never raise: they are reported in the result's `status`.
The product library is the HIP one; passing another `lib` is for tests only.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _native as N

STATUS = {0: "OK", 1: "VMERR", 2: "PANIC", 3: "BUDGET", 4: "UNSUPPORTED"}
MAP_HASH, MAP_ARRAY, MAP_PROG_ARRAY, MAP_PERF_EVENT_ARRAY, MAP_PERCPU_HASH, MAP_PERCPU_ARRAY = 1, 2, 3, 4, 5, 6
MAP_LRU_HASH, MAP_LRU_PERCPU_HASH, MAP_ARRAY_OF_MAPS, MAP_HASH_OF_MAPS, MAP_QUEUE, MAP_STACK = 9, 10, 12, 13, 22, 23
ARRAY_TYPES = (MAP_ARRAY, MAP_PERCPU_ARRAY, MAP_PROG_ARRAY, MAP_ARRAY_OF_MAPS)
HASH_TYPES = (MAP_HASH, MAP_PERCPU_HASH, MAP_HASH_OF_MAPS, MAP_LRU_HASH, MAP_LRU_PERCPU_HASH)
LIST_TYPES = (MAP_QUEUE, MAP_STACK, MAP_PERF_EVENT_ARRAY)
MODE_AUTO, MODE_PARALLEL, MODE_SEQUENTIAL, MODE_KEYED = 0, 1, 2, 3  # MODE_KEYED: mode_used only
MODE_CANCELLED = 4  # mode_used of a pipelined batch VM.cancel dropped
MODE_SEGMENTS = 5  # mode_used: packet-order segments, each in parallel (a list position after an earlier push)
E_HOST_HELPER, E_IN_HELPER = 17, 0x80
ENGINE_AUTO, ENGINE_INTERP, ENGINE_JIT = 0, 1, 2


class EmulatorError(RuntimeError):
    def __init__(self, rc: int, msg: str):
        super().__init__(f"{msg} (rc={rc})")
        self.rc = rc


@dataclass
class MapDef:
    type: int
    key_size: int
    value_size: int
    max_entries: int
    flags: int = 0


@dataclass
class Settings:
    max_steps: int = 1 << 20
    ingress_ifindex: int = 1
    rx_queue_index: int = 0
    device: int = 0
    mode: int = MODE_AUTO
    engine: int = 0  # ENGINE_AUTO


@dataclass
class BatchResult:
    results: np.ndarray        # structured (status, r0_kind, code, pc, r0)
    verdicts: np.ndarray       # uint32(R0)
    regs: np.ndarray | None    # structured parity records or None
    stats: dict


def initial_image(d: MapDef, data: dict) -> bytes | None:
    """AbstractMap.InitialData ({int key: bytes value}, map_abstract.go:33) as the flat image xe_add_map
    takes, copied the way ArrayMap.Init does (emulator/maps_array.go:19-44): value k lands at
    k*ValueSize and runs on into later entries when longer (keys applied in ascending order; Go's map
    order is random and only matters for overlapping copies). Only ARRAY / PERCPU_ARRAY receive
    InitialData (AbstractMapToVM, emulator/maps.go:101-108); other types get None."""
    if data is None or d.type not in (MAP_ARRAY, MAP_PERCPU_ARRAY):
        return None
    size = d.value_size * d.max_entries
    img = bytearray(size)
    for k in sorted(data):
        if not isinstance(k, int):
            raise TypeError("the key type of the initial data must be an int")
        v = bytes(data[k])
        off = k * d.value_size
        if k < 0 or off > size:
            raise ValueError(f"initial data key {k} outside the map")
        img[off:off + len(v)] = v[: size - off]
    return bytes(img)


def _wrap64(v: int) -> int:
    """a Python int as the int64 R0 a helper returns (two's complement wrap)"""
    v = int(v) & ((1 << 64) - 1)
    return v - (1 << 64) if v >> 63 else v


def _stats_dict(s: N.BatchStats) -> dict:
    return {"packets": s.packets, "steps": s.steps, "status_count": list(s.status_count),
            "mode_used": s.mode_used, "conflict": s.conflict, "kernel_ms": s.kernel_ms,
            "total_ms": s.total_ms, "engine_used": s.engine_used, "grid_blocks": s.grid_blocks}


class PendingBatch:
    """A batch queued by VM.run_batch_device_async; owns the statistics record the library fills."""

    def __init__(self, vm: "VM", st: N.BatchStats):
        self.vm, self._st = vm, st

    def stats(self) -> dict:
        self.vm.sync()
        return _stats_dict(self._st)


class VM:
    def __init__(self, settings: Settings | None = None, lib: N.Lib | None = None):
        self.lib = lib or N.product()
        s = settings or Settings()
        cs = N.Settings()
        self.lib.default_settings(C.byref(cs)) if self.lib.has("default_settings") else None
        cs.stack_frame_size, cs.max_stack_frames = 256, 8
        cs.max_steps, cs.ingress_ifindex, cs.rx_queue_index = s.max_steps, s.ingress_ifindex, s.rx_queue_index
        cs.device, cs.mode, cs.engine = s.device, s.mode, s.engine
        self.settings = s
        h = C.c_void_p()
        rc = self.lib.create(C.byref(cs), C.byref(h))
        if rc:
            raise EmulatorError(rc, "create VM")
        self.h = h
        self.map_defs: dict[int, MapDef] = {}
        self._pending: list = []  # pipelined batches whose statistics the library still writes
        self._helpers: dict[int, object] = {}  # ctypes callbacks of the host helpers (kept alive)

    def close(self) -> None:
        if self.h:
            self.lib.destroy(self.h)
            self.h = None
            self._pending.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc: int, what: str) -> None:
        if rc < 0:
            raise EmulatorError(rc, f"{what}: {self.lib.last_error(self.h).decode(errors='replace')}")

    # ---- programs / maps
    def add_raw_program(self, insns) -> int:
        arr = np.ascontiguousarray(np.asarray(insns, dtype=np.uint64))
        idx = C.c_int32()
        self._check(self.lib.add_raw_program(self.h, arr.ctypes.data, len(arr), C.byref(idx)), "add raw program")
        return idx.value

    def set_entrypoint(self, idx: int) -> None:
        self._check(self.lib.set_entrypoint(self.h, idx), "set entrypoint")

    def add_map(self, d: MapDef, initial: bytes | np.ndarray | dict | None = None) -> int:
        """AddAbstractMap; `initial` is a flat image or an InitialData dict (initial_image)."""
        if isinstance(initial, dict):
            initial = initial_image(d, initial)
        md = N.MapDef(d.type, d.key_size, d.value_size, d.max_entries, d.flags)
        buf = None if initial is None else np.frombuffer(bytes(initial), dtype=np.uint8)
        idx = C.c_int32()
        self._check(self.lib.add_map(self.h, C.byref(md), None if buf is None else buf.ctypes.data,
                                     0 if buf is None else len(buf), C.byref(idx)), "add map")
        self.map_defs[idx.value] = d
        return idx.value

    def map_update(self, m: int, key: bytes, value: bytes) -> None:
        d = self.map_defs[m]
        k = bytes(key).ljust(max(d.key_size, 4), b"\0")
        v = bytes(value).ljust(d.value_size, b"\0")
        self._check(self.lib.map_update(self.h, m, k, v), "map update")

    def map_update_batch(self, m: int, keys: np.ndarray, values: np.ndarray) -> None:
        """Bulk update: keys (n, key_size) and values (n, value_size) uint8 arrays."""
        d = self.map_defs[m]
        ks = d.key_size if d.type in HASH_TYPES else 4
        k = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1, ks)
        v = np.ascontiguousarray(values, dtype=np.uint8).reshape(-1, d.value_size)
        assert len(k) == len(v)
        self._check(self.lib.map_update_batch(self.h, m, k.ctypes.data, v.ctypes.data, len(k)), "map update batch")

    def map_lookup(self, m: int, key: bytes) -> bytes | None:
        d = self.map_defs[m]
        k = bytes(key).ljust(max(d.key_size, 4), b"\0")
        out = C.create_string_buffer(max(d.value_size, 1))
        rc = self.lib.map_lookup(self.h, m, k, out)
        self._check(rc, "map lookup")
        return out.raw[: d.value_size] if rc == 1 else None

    def map_delete(self, m: int, key: bytes) -> None:
        d = self.map_defs[m]
        self._check(self.lib.map_delete(self.h, m, bytes(key).ljust(max(d.key_size, 4), b"\0")), "map delete")

    def map_dump(self, m: int):
        """ARRAY -> raw bytes (ValueSize*MaxEntries); HASH / LRU_HASH -> (keys[n,ks], values[n,vs]) sorted
        by key; QUEUE / STACK / PERF_EVENT_ARRAY -> list of records (bytes) in list order."""
        d = self.map_defs[m]
        if d.type in LIST_TYPES:
            return self.map_dump_list(m)
        cnt = C.c_uint64()
        self._check(self.lib.map_dump(self.h, m, None, None, 0, C.byref(cnt)), "map dump")
        n = cnt.value
        if d.type in ARRAY_TYPES:
            raw = np.zeros(d.value_size * d.max_entries, dtype=np.uint8)
            self._check(self.lib.map_dump(self.h, m, raw.ctypes.data, None, n, C.byref(cnt)), "map dump")
            return raw.tobytes()
        keys = np.zeros((n, d.key_size), dtype=np.uint8)
        vals = np.zeros((n, d.value_size), dtype=np.uint8)
        self._check(self.lib.map_dump(self.h, m, keys.ctypes.data if n else None,
                                      vals.ctypes.data if n else None, n, C.byref(cnt)), "map dump")
        return keys, vals

    def map_dump_list(self, m: int) -> list[bytes]:
        """QUEUE / STACK / PERF_EVENT_ARRAY records in the order of the Go Values / Events slice."""
        cnt, nb = C.c_uint64(), C.c_uint64()
        self._check(self.lib.map_dump_list(self.h, m, None, 0, None, 0, C.byref(cnt), C.byref(nb)), "map dump list")
        data = np.zeros(max(1, nb.value), dtype=np.uint8)
        lens = np.zeros(max(1, cnt.value), dtype=np.uint32)
        self._check(self.lib.map_dump_list(self.h, m, data.ctypes.data, nb.value, lens.ctypes.data, cnt.value,
                                           C.byref(cnt), C.byref(nb)), "map dump list")
        out, off = [], 0
        for ln in lens[: cnt.value]:
            out.append(data[off: off + int(ln)].tobytes())
            off += int(ln)
        return out

    def map_lru_order(self, m: int) -> list[bytes]:
        """LRU_HASH UsageList keys, most recently used first (maps_hash_lru.go:21-24)."""
        d = self.map_defs[m]
        cnt = C.c_uint64()
        self._check(self.lib.map_lru_order(self.h, m, None, 0, C.byref(cnt)), "map lru order")
        keys = np.zeros((max(1, cnt.value), d.key_size), dtype=np.uint8)
        self._check(self.lib.map_lru_order(self.h, m, keys.ctypes.data, cnt.value, C.byref(cnt)), "map lru order")
        return [keys[i].tobytes() for i in range(cnt.value)]

    def map_push(self, m: int, value: bytes) -> None:
        """QueueMap/StackMap.Push of one value_size element from userspace."""
        d = self.map_defs[m]
        self._check(self.lib.map_push(self.h, m, bytes(value).ljust(d.value_size, b"\0")), "map push")

    def map_count(self, m: int) -> int:
        """xe_map_count: the map's live entries (HASH / LRU_HASH), elements (QUEUE / STACK) or events."""
        n = C.c_uint64(0)
        self._check(self.lib.map_count(self.h, m, C.byref(n)), "map count")
        return int(n.value)

    def map_values_bytes(self, m: int) -> int:
        b = C.c_uint64()
        self._check(self.lib.map_values_bytes(self.h, m, C.byref(b)), "map values bytes")
        return b.value

    # ---- running
    def run_batch(self, umem: np.ndarray, descs: np.ndarray, want_regs: bool = False) -> BatchResult:
        """Host-memory batch (end-to-end form). `umem` (uint8) receives packet writes."""
        d_desc, d_res, d_regs = N.np_dtypes()
        assert umem.dtype == np.uint8 and umem.flags.c_contiguous
        descs = np.ascontiguousarray(descs, dtype=d_desc)
        n = len(descs)
        res = np.zeros(n, dtype=d_res)
        ver = np.zeros(n, dtype=np.uint32)
        regs = np.zeros(n, dtype=d_regs) if want_regs else None
        st = N.BatchStats()
        fn = self.lib.run_batch_host if self.lib.has("run_batch_host") else self.lib.run_batch
        rc = fn(self.h, umem.ctypes.data if umem.size else None, umem.size, descs.ctypes.data if n else None, n,
                res.ctypes.data if n else None, ver.ctypes.data if n else None,
                regs.ctypes.data if (regs is not None and n) else None, C.byref(st))
        self._check(rc, "run batch")
        return BatchResult(res, ver, regs, _stats_dict(st))

    def run_batch_host_ptrs(self, umem: int, umem_len: int, desc: int, n: int, verdicts: int = 0,
                            results: int = 0) -> dict:
        """Host-memory batch over caller-owned (ideally pinned) buffers given as addresses."""
        st = N.BatchStats()
        rc = self.lib.run_batch_host(self.h, umem or None, umem_len, desc or None, n, results or None,
                                     verdicts or None, None, C.byref(st))
        self._check(rc, "run batch (host pointers)")
        return _stats_dict(st)

    def run_batch_device(self, d_umem: int, umem_len: int, d_desc: int, n: int, d_results: int = 0,
                         d_verdicts: int = 0, d_regs: int = 0, stream: int = 0) -> dict:
        """Device-resident batch: all pointers are device addresses (e.g. torch tensor .data_ptr())."""
        st = N.BatchStats()
        rc = self.lib.run_batch_device(self.h, d_umem or None, umem_len, d_desc or None, n, d_results or None,
                                       d_verdicts or None, d_regs or None, stream or None, C.byref(st))
        self._check(rc, "run batch (device)")
        return _stats_dict(st)

    def run_batch_device_async(self, d_umem: int, umem_len: int, d_desc: int, n: int, d_results: int = 0,
                               d_verdicts: int = 0, d_regs: int = 0, stream: int = 0) -> "PendingBatch":
        """Pipelined device-resident batch (xe_run_batch_device_async): queued behind the batches in
        flight on the same stream; the result equals run_batch_device in submission order. The returned
        handle's .stats() completes the pipeline (xe_sync) and gives this batch's statistics."""
        st = N.BatchStats()
        rc = self.lib.run_batch_device_async(self.h, d_umem or None, umem_len, d_desc or None, n, d_results or None,
                                             d_verdicts or None, d_regs or None, stream or None, C.byref(st))
        self._check(rc, "run batch (device, pipelined)")
        pb = PendingBatch(self, st)
        self._pending.append(pb)
        return pb

    def prepare(self) -> None:
        """xe_prepare: compile the per-program kernel (and its keyed variant) for the current program and
        map geometry now instead of in the first batch. Releases the GIL (ctypes), so several VMs can
        prepare from a thread pool and their kernels compile concurrently. No-op on libraries without it."""
        if self.lib.has("prepare"):
            self._check(self.lib.prepare(self.h), "prepare")

    def kernel_sources(self, variants=(0, 1, 2)) -> list[str]:
        """Sources of the per-program kernels xe_prepare would build (0: the kernel, 1: its keyed variant
        when the program may write map entries, 2: its verdict-only variant); [] when the VM runs the
        interpreter."""
        out = []
        for variant in variants:
            n = C.c_size_t()
            rc = self.lib.kernel_source(self.h, variant, None, 0, C.byref(n))
            if rc == -95:  # XE_ERR_UNSUPPORTED
                continue
            self._check(rc, "kernel source")
            buf = C.create_string_buffer(n.value + 1)
            self._check(self.lib.kernel_source(self.h, variant, buf, n.value + 1, C.byref(n)), "kernel source")
            out.append(buf.value.decode())
        return out

    def set_schedule(self, sched: int) -> None:
        """xe_debug_set_schedule: permute the chunk -> wave schedule of later parallel passes (0 = default)."""
        self._check(self.lib.debug_set_schedule(self.h, sched), "set schedule")

    def set_lru_epoch(self, epoch: int) -> None:
        """xe_debug_set_lru_epoch: the run counter of the LRU stamps (tests reach its renumbering)."""
        self._check(self.lib.debug_set_lru_epoch(self.h, epoch), "set LRU epoch")

    def map_pool(self, m: int) -> tuple[int, int]:
        """xe_debug_map_pool: (room, next fresh id) of an ordered map's device value pool."""
        room, nxt = C.c_uint64(), C.c_uint64()
        self._check(self.lib.debug_map_pool(self.h, m, C.byref(room), C.byref(nxt)), "map pool")
        return room.value, nxt.value

    def sync(self) -> None:
        """Complete every pipelined batch (in-order replays included)."""
        rc = self.lib.sync(self.h)
        self._pending.clear()
        self._check(rc, "sync")

    def cancel(self) -> int:
        """xe_cancel (RunContext's cancellation, emulator/vm.go:117-134): drop every pipelined batch not
        completed yet; the maps return to the state before the oldest of them. Returns how many."""
        k = C.c_uint32()
        rc = self.lib.cancel(self.h, C.byref(k))
        self._pending.clear()
        self._check(rc, "cancel")
        return k.value

    # ---- Step / VM.String: per-packet instruction trace
    def trace(self, packets, max_steps: int = 256) -> None:
        """xe_trace_config: record the first max_steps Steps of each listed packet of every batch
        ([] turns it off)."""
        arr = np.ascontiguousarray(np.asarray(list(packets), dtype=np.uint32))
        self._check(self.lib.trace_config(self.h, arr.ctypes.data if len(arr) else None, len(arr),
                                          max_steps if len(arr) else 0), "trace config")

    def trace_read(self, packet: int) -> np.ndarray:
        """The Step records of `packet` in the last batch (N.np_trace_dtype(): pc, pi, sf, kind[11], val[11])."""
        n = C.c_uint32()
        self._check(self.lib.trace_read(self.h, packet, None, 0, C.byref(n)), "trace read")
        out = np.zeros(n.value, dtype=N.np_trace_dtype())
        if n.value:
            self._check(self.lib.trace_read(self.h, packet, out.ctypes.data, n.value, C.byref(n)), "trace read")
        return out

    # ---- the helper table (VM.HelperFunctions)
    def set_helper(self, hid: int, fn) -> None:
        """Replace helper `hid` (emulator/helper_functions.go:17 HelperFunc): fn(packet, args[5], kinds[5])
        returns R0 (an int) or raises to abort the packet (XE_E_HOST_HELPER); fn=None makes the entry nil."""
        if fn is None:
            self._check(self.lib.set_helper(self.h, hid, N.HELPER_FN(), None), "set helper")
            self._helpers.pop(hid, None)
            return

        def tramp(_user, packet, args, kinds, r0):
            try:
                r0[0] = _wrap64(fn(int(packet), [args[i] for i in range(5)], [kinds[i] for i in range(5)]))
                return 0
            except Exception:
                return 1

        cb = N.HELPER_FN(tramp)
        self._check(self.lib.set_helper(self.h, hid, cb, None), "set helper")
        self._helpers[hid] = cb

    def reset_helper(self, hid: int) -> None:
        """Entry `hid` back to LinuxHelperFunctions' (the built-in helper or nil)."""
        self._check(self.lib.reset_helper(self.h, hid), "reset helper")
        self._helpers.pop(hid, None)

    # ---- multi-GPU shard support
    def map_delta(self, m: int, d_out: int, stream: int = 0, lane: int = 0) -> None:
        self._check(self.lib.map_delta(self.h, m, lane, d_out, stream or None), "map delta")

    def map_delta_lane(self, m: int) -> int:
        """Lane width in bytes of map_delta / map_apply_delta (the width of the last run's map adds)."""
        v = C.c_uint32()
        self._check(self.lib.map_delta_lane(self.h, m, C.byref(v)), "map delta lane")
        return v.value

    def map_apply_delta(self, m: int, d_in: int, stream: int = 0, lane: int = 0) -> None:
        self._check(self.lib.map_apply_delta(self.h, m, lane, d_in, stream or None), "map apply delta")

    def epoch_begin(self, stream: int = 0) -> None:
        """xe_epoch_begin: later map deltas / footprints cover every batch from here (a shard epoch)."""
        self._check(self.lib.epoch_begin(self.h, stream or None), "epoch begin")

    def epoch_end(self) -> None:
        self._check(self.lib.epoch_end(self.h), "epoch end")

    def footprint(self) -> np.ndarray:
        """xe_footprint record of the last run (or of the open shard epoch): [flags, (read, add, widths) per map]."""
        nw = C.c_uint32()
        self._check(self.lib.footprint(self.h, None, 0, C.byref(nw)), "footprint")
        out = np.zeros(nw.value, dtype=np.uint64)
        self._check(self.lib.footprint(self.h, out.ctypes.data_as(C.POINTER(C.c_uint64)), nw.value, C.byref(nw)),
                    "footprint")
        return out

    def shard_check(self, fps: np.ndarray, nshards: int) -> tuple[bool, list[int]]:
        """xe_shard_check over the concatenated footprint records of the shards, in shard order."""
        fps = np.ascontiguousarray(fps, dtype=np.uint64)
        nw = len(fps) // nshards
        lanes = np.zeros(max(1, (nw - 1) // 3), dtype=np.uint32)
        rc = self.lib.shard_check(fps.ctypes.data, nshards, nw, lanes.ctypes.data)
        self._check(rc, "shard check")
        return rc == 1, [int(x) for x in lanes]

    def map_state_bytes(self, m: int) -> int:
        b = C.c_uint64()
        self._check(self.lib.map_state_bytes(self.h, m, C.byref(b)), "map state bytes")
        return b.value

    def map_state_export(self, m: int, d_out: int, stream: int = 0) -> None:
        self._check(self.lib.map_state_export(self.h, m, d_out, stream or None), "map state export")

    def map_state_import(self, m: int, d_in: int, stream: int = 0) -> None:
        self._check(self.lib.map_state_import(self.h, m, d_in, stream or None), "map state import")


class Multi:
    """One process driving N devices (xe_multi_create / xe_run_batch_multi): vms[k] on its own device
    (or sharing one, in tests), set up identically by the caller."""

    def __init__(self, vms: list[VM]):
        self.vms = vms
        self.lib = vms[0].lib
        arr = (C.c_void_p * len(vms))(*[v.h.value for v in vms])
        h = C.c_void_p()
        rc = self.lib.multi_create(arr, len(vms), C.byref(h))
        if rc:
            raise EmulatorError(rc, "multi create")
        self.h = h

    def close(self) -> None:
        if self.h:
            self.lib.multi_destroy(self.h)
            self.h = None

    def run(self, d_umem: list[int], umem_len: list[int], d_desc: list[int], n: list[int],
            d_results: list[int] | None = None, d_verdicts: list[int] | None = None) -> tuple[list[dict], bool]:
        """Run shard k = (d_umem[k], d_desc[k], n[k]) on vms[k]; maps end equal to the single-VM result."""
        G = len(self.vms)
        ptrs = lambda xs: (C.c_void_p * G)(*[x or None for x in xs])
        sts = (N.BatchStats * G)()
        rep = C.c_uint32()
        rc = self.lib.run_batch_multi(self.h, ptrs(d_umem), (C.c_uint64 * G)(*umem_len), ptrs(d_desc),
                                      (C.c_uint32 * G)(*n), ptrs(d_results) if d_results else None,
                                      ptrs(d_verdicts) if d_verdicts else None, sts, C.byref(rep))
        if rc:
            raise EmulatorError(rc, "run batch multi: " + self.lib.multi_last_error(self.h).decode(errors="replace"))
        return [_stats_dict(s) for s in sts], bool(rep.value)
