/*
 * xdpemu_io.h — packet ingestion for the end-to-end path: capture files into
 * AF_XDP-shaped UMEM frames and 16-byte descriptors (the layout xe_run_batch_* consume).
 *
 * The reference's host input format is the AF_XDP UMEM of FrameCount x FrameSize bytes plus
 * `struct xdp_desc {u64 addr; u32 len; u32 options;}` descriptors (xsk.go:695-701, XSKSettings
 * xsk.go:720-757); its rx path hands the program a frame at `addr` (frame start + headroom). These
 * calls fill exactly that layout from a classic libpcap capture (magic 0xa1b2c3d4 microsecond or
 * 0xa1b23c4d nanosecond timestamps, either byte order) held in memory (e.g. an mmap of the file).
 * Host-only code: no device calls, usable without a GPU.
 */
#ifndef XDPEMU_IO_H
#define XDPEMU_IO_H

#include "xdpemu.h"

#ifdef __cplusplus
extern "C" {
#endif

#define XE_ERR_FORMAT (-103) /* not a classic pcap capture / truncated header */

typedef struct xe_pcap_info {
    uint32_t linktype;     /* LINKTYPE_* (1 = Ethernet, the only one an XDP program sees)   */
    uint32_t snaplen;
    uint32_t nanosecond;   /* 1: timestamps are ns, 0: us                                   */
    uint32_t swapped;      /* 1: the file was written big-endian                            */
    uint64_t first_record; /* byte offset of the first record header (24)                   */
} xe_pcap_info;

/* Validate the global header. Returns XE_OK or XE_ERR_FORMAT. */
int xe_pcap_header(const uint8_t* file, uint64_t file_len, xe_pcap_info* info);

/* Count the complete records from *offset on (a truncated final record is not counted); *bytes
 * receives the captured bytes of the counted records. Returns XE_OK. */
int xe_pcap_count(const uint8_t* file, uint64_t file_len, const xe_pcap_info* info, uint64_t offset,
                  uint64_t* records, uint64_t* bytes);

/* Copy up to `max` records, from *offset on, into UMEM frames: record k goes to the frame starting at
 * UMEM byte address frame_addr[k] (frame_addr NULL: the frames first_frame, first_frame + 1, ...
 * in order), its bytes at frame start + headroom, cut to frame_size - headroom.
 * desc[k] = {frame start + headroom, copied bytes, 0} (the rx descriptor the kernel would post);
 * orig_len[k] (optional) = the record's wire length, ts_ns[k] (optional) = its timestamp in ns.
 * *offset advances past the copied records; *filled = records copied. A truncated final record
 * stops the copy (it stays unread). Returns XE_OK, XE_ERR_INVAL (a frame outside the UMEM,
 * frame_size <= headroom). */
int xe_pcap_fill(const uint8_t* file, uint64_t file_len, const xe_pcap_info* info, uint64_t* offset,
                 uint8_t* umem, uint64_t umem_len, uint32_t frame_size, uint32_t headroom,
                 const uint64_t* frame_addr, uint64_t first_frame, uint32_t max, xe_desc* desc,
                 uint32_t* orig_len, uint64_t* ts_ns, uint32_t* filled);

/* Staging form for the device path: copy up to `max` records, from *offset on, back to back into
 * buf, each starting at a multiple of `align` (a power of two, >= 16), cut to `max_len` bytes
 * (0: no cut); desc[k] = {offset in buf, copied bytes, 0}. Only the packet bytes cross PCIe, not
 * whole frames. Stops before a record that does not fit in buf_len. *used = bytes of buf used.
 * Same offset / filled / orig_len / ts_ns contract as xe_pcap_fill. */
int xe_pcap_pack(const uint8_t* file, uint64_t file_len, const xe_pcap_info* info, uint64_t* offset,
                 uint8_t* buf, uint64_t buf_len, uint32_t align, uint32_t max_len, uint32_t max,
                 xe_desc* desc, uint32_t* orig_len, uint64_t* ts_ns, uint32_t* filled, uint64_t* used);

#ifdef __cplusplus
}
#endif
#endif /* XDPEMU_IO_H */
