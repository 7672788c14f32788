"""Packet ingestion for the end-to-end path: capture files and AF_XDP-shaped
UMEM frames, descriptor rings and fill/completion rings, feeding batches to the device emulator.

The reference's host input format is the XSK one (xsk.go): a UMEM of FrameCount x FrameSize bytes,
16-byte `xdp_desc {addr, len, options}` descriptors (xsk.go:695-701), producer/consumer rings whose
indices wrap as u32 and that count as full one slot early (xsk.go:513-606), fill-ring frames
0..rxCount-2 handed to the kernel at start (xsk.go:1026-1031), tx frames after the rx half
(xsk.go:860-935). This module restates that layout; the NIC side is a capture file:

    pc = PcapFile("trace.pcap")
    q = XSKQueue(XSKSettings(FrameSize=2048, FrameCount=8192))
    n = q.receive(pc, 4096)                 # fill-ring frames <- records, rx descriptors posted
    desc = q.rx.dequeue_many(n)             # what an XDP program in front of the socket sees
    res = vm.run_batch(q.umem, desc)        # or run_pcap(vm, pc) for the streaming device path

`run_pcap` is the throughput form: records are packed back to back into pinned staging buffers by
native code (xe_pcap_pack, only packet bytes cross PCIe), copied on a side stream while the
previous batch runs, and run with `xe_run_batch_device`.
"""
from __future__ import annotations

import ctypes as C
import mmap
import struct
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field
from pathlib import Path

import numpy as np

from . import _native as N

LINKTYPE_ETHERNET = 1
XDP_ABORTED, XDP_DROP, XDP_PASS, XDP_TX, XDP_REDIRECT = 0, 1, 2, 3, 4


class XSKError(ValueError):
    pass


class RingFull(RuntimeError):
    """errBufferFull (xsk.go:583)."""


# ---------------------------------------------------------------- capture files
class PcapFile:
    """A classic libpcap capture (us or ns timestamps, either byte order), memory-mapped."""

    def __init__(self, src: str | Path | bytes | np.ndarray, lib: N.Lib | None = None):
        self.lib = lib or N.product()
        self._mm = None
        if isinstance(src, (str, Path)):
            with open(src, "rb") as fh:
                size = Path(src).stat().st_size
                self._mm = mmap.mmap(fh.fileno(), size, prot=mmap.PROT_READ) if size else None
            self.data = np.frombuffer(self._mm, dtype=np.uint8) if self._mm else np.zeros(0, np.uint8)
        else:
            self.data = np.frombuffer(bytes(src), dtype=np.uint8) if isinstance(src, bytes) else src
        self.info = N.PcapInfo()
        rc = self.lib.pcap_header(self._ptr, self.data.size, C.byref(self.info))
        if rc:
            raise XSKError(f"not a classic pcap capture (rc={rc})")
        if self.info.linktype != LINKTYPE_ETHERNET:
            raise XSKError(f"link type {self.info.linktype}: XDP programs see Ethernet frames (1)")
        self.offset = self.info.first_record

    @property
    def _ptr(self) -> int:
        return self.data.ctypes.data if self.data.size else 0

    def count(self) -> tuple[int, int]:
        """(records, captured bytes) from the current offset."""
        n, b = C.c_uint64(), C.c_uint64()
        self.lib.pcap_count(self._ptr, self.data.size, C.byref(self.info), self.offset, C.byref(n), C.byref(b))
        return n.value, b.value

    def rewind(self) -> None:
        self.offset = self.info.first_record

    def fill(self, umem: np.ndarray, frame_size: int, headroom: int, frames: np.ndarray, want_meta=False):
        """Records into the given frame start addresses (xe_pcap_fill); returns descriptors
        (and, with want_meta, wire lengths and ns timestamps)."""
        frames = np.ascontiguousarray(frames, dtype=np.uint64)
        d_desc = N.np_dtypes()[0]
        desc = np.zeros(len(frames), dtype=d_desc)
        olen = np.zeros(len(frames), np.uint32) if want_meta else None
        ts = np.zeros(len(frames), np.uint64) if want_meta else None
        off, got = C.c_uint64(self.offset), C.c_uint32()
        rc = self.lib.pcap_fill(self._ptr, self.data.size, C.byref(self.info), C.byref(off),
                                umem.ctypes.data if umem.size else None, umem.size, frame_size, headroom,
                                frames.ctypes.data if len(frames) else None, 0, len(frames),
                                desc.ctypes.data if len(frames) else None,
                                olen.ctypes.data if want_meta and len(frames) else None,
                                ts.ctypes.data if want_meta and len(frames) else None, C.byref(got))
        self.offset = off.value
        if rc:
            raise XSKError(f"pcap fill: a frame lies outside the UMEM (rc={rc})")
        k = got.value
        return (desc[:k], olen[:k], ts[:k]) if want_meta else desc[:k]

    def pack(self, buf: np.ndarray, desc: np.ndarray, align: int = 64, max_len: int = 0) -> tuple[int, int]:
        """Records back to back into buf (xe_pcap_pack); returns (records, bytes used)."""
        off, got, used = C.c_uint64(self.offset), C.c_uint32(), C.c_uint64()
        rc = self.lib.pcap_pack(self._ptr, self.data.size, C.byref(self.info), C.byref(off), buf.ctypes.data, buf.size,
                                align, max_len, len(desc), desc.ctypes.data, None, None, C.byref(got), C.byref(used))
        if rc:
            raise XSKError(f"pcap pack (rc={rc})")
        self.offset = off.value
        return got.value, used.value

    def close(self) -> None:
        self.data = np.zeros(0, np.uint8)
        if self._mm is not None:
            self._mm.close()
            self._mm = None


def write_pcap(path: str | Path | None, packets, ts_ns=None, nanosecond: bool = False, big_endian: bool = False,
               snaplen: int = 65535, wire_len=None) -> bytes:
    """A classic pcap capture of `packets` (bytes-likes). Returns the bytes; writes them if path."""
    e = ">" if big_endian else "<"
    out = [struct.pack(e + "IHHiIII", 0xA1B23C4D if nanosecond else 0xA1B2C3D4, 2, 4, 0, 0, snaplen,
                       LINKTYPE_ETHERNET)]
    for i, p in enumerate(packets):
        p = bytes(p)
        t = int(ts_ns[i]) if ts_ns is not None else i * 1000
        frac = t % 1_000_000_000 if nanosecond else (t % 1_000_000_000) // 1000
        wl = int(wire_len[i]) if wire_len is not None else len(p)
        out.append(struct.pack(e + "IIII", t // 1_000_000_000, frac, len(p), wl))
        out.append(p)
    data = b"".join(out)
    if path is not None:
        Path(path).write_bytes(data)
    return data


# ---------------------------------------------------------------- XSK layout
@dataclass
class XSKSettings:
    """XSKSettings (xsk.go:720-757), the fields that shape the UMEM and rings."""
    FrameSize: int = 4096
    FrameCount: int = 4096
    Headroom: int = 0
    DisableTx: bool = False
    DisableRx: bool = False

    def validated(self) -> "XSKSettings":
        """NewXSKSocket's checks and defaults (xsk.go:797-822)."""
        s = XSKSettings(self.FrameSize or 4096, self.FrameCount or 4096, self.Headroom, self.DisableTx, self.DisableRx)
        if s.FrameCount <= 0 or s.FrameCount & (s.FrameCount - 1):
            raise XSKError("frame count must be a power of 2")
        if s.FrameSize not in (2048, 4096):
            raise XSKError("frame size must be 2048 or 4096")
        if s.DisableTx and s.DisableRx:
            raise XSKError("tx and rx can't both be disabled")
        if not 0 <= s.Headroom < s.FrameSize:
            raise XSKError("headroom must leave room in the frame")
        return s

    def counts(self) -> tuple[int, int]:
        """(rxCount, txCount): half each unless one side is disabled (xsk.go:860-870)."""
        if self.DisableTx:
            return self.FrameCount, 0
        if self.DisableRx:
            return 0, self.FrameCount
        return self.FrameCount // 2, self.FrameCount // 2


def addr_to_frame_start(addr, frame_size: int):
    """addrToFrameStart (xsk.go:504-506): strip the headroom off a ring address."""
    return (np.asarray(addr, dtype=np.uint64) // np.uint64(frame_size)) * np.uint64(frame_size)


class _Ring:
    """Producer/consumer ring of elem_count (a power of 2) slots; u32 indices that wrap, full at
    elem_count - 1 entries (xsk.go:513-606)."""

    def __init__(self, elem_count: int, dtype):
        if elem_count <= 0 or elem_count & (elem_count - 1):
            raise XSKError("ring size must be a power of 2")
        self.elem_count = elem_count
        self.ring = np.zeros(elem_count, dtype=dtype)
        self.producer = 0
        self.consumer = 0

    def __len__(self) -> int:
        return (self.producer - self.consumer) & 0xFFFFFFFF

    def free(self) -> int:
        return self.elem_count - 1 - len(self)

    def enqueue(self, item) -> None:
        if len(self) == self.elem_count - 1:
            raise RingFull("ring buffer is full")
        self.ring[self.producer & (self.elem_count - 1)] = item
        self.producer = (self.producer + 1) & 0xFFFFFFFF

    def dequeue(self):
        if len(self) == 0:
            return None
        item = self.ring[self.consumer & (self.elem_count - 1)].copy()
        self.consumer = (self.consumer + 1) & 0xFFFFFFFF
        return item

    def enqueue_many(self, items: np.ndarray) -> None:
        items = np.asarray(items, dtype=self.ring.dtype)
        if len(items) > self.free():
            raise RingFull("ring buffer is full")
        idx = (self.producer + np.arange(len(items), dtype=np.uint64)) & np.uint64(self.elem_count - 1)
        self.ring[idx] = items
        self.producer = (self.producer + len(items)) & 0xFFFFFFFF

    def dequeue_many(self, n: int) -> np.ndarray:
        n = min(n, len(self))
        idx = (self.consumer + np.arange(n, dtype=np.uint64)) & np.uint64(self.elem_count - 1)
        out = self.ring[idx].copy()
        self.consumer = (self.consumer + n) & 0xFFFFFFFF
        return out


class DescRing(_Ring):
    """xskDescRing (rx / tx): 16-byte descriptors."""

    def __init__(self, elem_count: int):
        super().__init__(elem_count, N.np_dtypes()[0])


class AddrRing(_Ring):
    """xskAddrRing (fill / completion): u64 UMEM addresses."""

    def __init__(self, elem_count: int):
        super().__init__(elem_count, np.uint64)


class XSKQueue:
    """One socket's UMEM and rings, with a capture file in the NIC's place: `receive` takes frames
    from the fill ring, writes records into them and posts rx descriptors, as the kernel does."""

    def __init__(self, settings: XSKSettings | None = None):
        s = (settings or XSKSettings()).validated()
        self.settings = s
        self.rx_count, self.tx_count = s.counts()
        self.umem = np.zeros(s.FrameSize * s.FrameCount, dtype=np.uint8)
        self.rx = DescRing(max(self.rx_count, 1))
        self.fill = AddrRing(max(self.rx_count, 1))
        self.tx = DescRing(max(self.tx_count, 1))
        self.completion = AddrRing(max(self.tx_count, 1))
        # every rx frame but one goes to the kernel (xsk.go:1026-1031); tx frames follow the rx half
        self.fill.enqueue_many(np.arange(max(self.rx_count - 1, 0), dtype=np.uint64) * np.uint64(s.FrameSize))
        self.tx_free = list(np.uint64(self.rx_count * s.FrameSize) + np.arange(self.tx_count, dtype=np.uint64)
                            * np.uint64(s.FrameSize))

    def receive(self, pcap: PcapFile, max_packets: int) -> int:
        """Kernel rx: up to max_packets records into fill-ring frames, rx descriptors posted."""
        n = min(max_packets, len(self.fill), self.rx.free())
        if n <= 0:
            return 0
        frames = self.fill.ring[(self.fill.consumer + np.arange(n, dtype=np.uint64)) & np.uint64(self.fill.elem_count - 1)]
        desc = pcap.fill(self.umem, self.settings.FrameSize, self.settings.Headroom, frames)
        self.fill.dequeue_many(len(desc))
        self.rx.enqueue_many(desc)
        return len(desc)

    def recycle(self, desc: np.ndarray) -> None:
        """Frames read from rx go back to the fill ring at their frame start (xsk.go:1174)."""
        self.fill.enqueue_many(addr_to_frame_start(desc["addr"], self.settings.FrameSize))

    def transmit(self, desc: np.ndarray) -> None:
        """Frames the program bounced (XDP_TX) are copied into tx frames and posted on the tx ring;
        the NIC side completes them at once (completion ring -> free tx frames)."""
        fs = self.settings.FrameSize
        for d in desc:
            if not self.tx_free:
                raise RingFull("no free tx frame")
            a = int(self.tx_free.pop(0))
            src = int(d["addr"])
            self.umem[a:a + int(d["len"])] = self.umem[src:src + int(d["len"])]
            self.tx.enqueue((a, d["len"], 0))
        for d in self.tx.dequeue_many(len(self.tx)):
            self.completion.enqueue(d["addr"])
        for a in self.completion.dequeue_many(len(self.completion)):
            self.tx_free.append(addr_to_frame_start(a, fs))


# ---------------------------------------------------------------- streaming device path
@dataclass
class PcapRun:
    packets: int = 0
    batches: int = 0
    seconds: float = 0.0
    device_ms: float = 0.0
    verdict_count: dict = field(default_factory=dict)  # R0 value -> packets (status OK)
    status_count: list = field(default_factory=lambda: [0] * 8)
    verdicts: np.ndarray | None = None

    @property
    def mpps(self) -> float:
        return self.packets / self.seconds / 1e6 if self.seconds else 0.0


def run_pcap(vm, pcap: PcapFile, batch: int = 1 << 20, staging_bytes: int | None = None, align: int = 64,
             keep_verdicts: bool = False) -> PcapRun:
    """Stream a capture through the device emulator: native packing into two pinned staging
    buffers, H2D on a side stream overlapped with the previous batch's kernel, verdicts back.
    `vm` is a gobpfld_amd.emulator.VM on the product library."""
    import torch

    d_desc_t = N.np_dtypes()[0]
    staging_bytes = staging_bytes or batch * 1600
    h_buf = [torch.empty(staging_bytes, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    h_desc = [torch.empty(batch * 16, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    d_buf = [torch.empty(staging_bytes, dtype=torch.uint8, device="cuda") for _ in range(2)]
    d_desc = [torch.empty(batch * 16, dtype=torch.uint8, device="cuda") for _ in range(2)]
    d_ver = [torch.empty(batch, dtype=torch.int32, device="cuda") for _ in range(2)]
    h2d, comp = torch.cuda.Stream(), torch.cuda.Stream()
    out = PcapRun()
    kept = []

    def parse(i):
        desc = h_desc[i].numpy().view(d_desc_t)
        return pcap.pack(h_buf[i].numpy(), desc, align=align)

    def upload(i, n, used):
        with torch.cuda.stream(h2d):
            d_buf[i][:used].copy_(h_buf[i][:used], non_blocking=True)
            d_desc[i][:n * 16].copy_(h_desc[i][:n * 16], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(h2d)
        return ev

    def run(i, n, used, ev):
        comp.wait_event(ev)
        st = vm.run_batch_device(d_buf[i].data_ptr(), max(used, 1), d_desc[i].data_ptr(), n,
                                 d_verdicts=d_ver[i].data_ptr(), stream=comp.cuda_stream)
        with torch.cuda.stream(comp):
            v = d_ver[i][:n].cpu()
        return st, v

    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with ThreadPoolExecutor(2) as pool:
        n, used = parse(0)
        if n == 0 and pcap.count()[0]:
            raise XSKError("staging buffer smaller than one record")
        ev = upload(0, n, used) if n else None
        k = 0
        while n:
            nxt = pool.submit(parse, (k + 1) % 2)
            fut = pool.submit(run, k % 2, n, used, ev)
            n2, used2 = nxt.result()
            # the other staging/device pair is free: its batch (k - 1) finished before run(k) began
            ev2 = upload((k + 1) % 2, n2, used2) if n2 else None
            st, v = fut.result()
            out.packets += n
            out.batches += 1
            out.device_ms += st["kernel_ms"]
            out.status_count = [a + b for a, b in zip(out.status_count, st["status_count"])]
            vals, cnt = np.unique(v.numpy().view(np.uint32), return_counts=True)
            for a, b in zip(vals.tolist(), cnt.tolist()):
                out.verdict_count[a] = out.verdict_count.get(a, 0) + b
            if keep_verdicts:
                kept.append(v.numpy().view(np.uint32).copy())
            n, used, ev = n2, used2, ev2
            k += 1
    torch.cuda.synchronize()
    if pcap.count()[0]:
        raise XSKError("a record does not fit in an empty staging buffer (raise staging_bytes)")
    out.seconds = time.perf_counter() - t0
    if keep_verdicts:
        out.verdicts = np.concatenate(kept) if kept else np.zeros(0, np.uint32)
    return out
