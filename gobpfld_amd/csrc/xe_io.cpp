// Capture files -> AF_XDP-shaped UMEM frames + rx descriptors (include/xdpemu_io.h).
// Host-only; the layout it produces is the reference's XSK one (xsk.go:695-757): frame starts are
// multiples of FrameSize, the descriptor points at frame start + headroom (the kernel's rx address,
// which addrToFrameStart, xsk.go:504-506, rounds back down when the frame is recycled).
#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/xdpemu_io.h"

namespace {

constexpr uint32_t kMagicUs = 0xa1b2c3d4u, kMagicNs = 0xa1b23c4du;
constexpr uint64_t kGlobalHeader = 24, kRecordHeader = 16;
constexpr uint64_t kPrefetch = 16384;  // bytes of the capture prefetched ahead of the record walk

inline uint32_t rd32(const uint8_t* p, bool swapped) {
  uint32_t v;
  memcpy(&v, p, 4);
  return swapped ? __builtin_bswap32(v) : v;
}

struct Record {
  uint32_t ts_sec, ts_frac, caplen, wirelen;
};

// The record header at `off` if the whole record lies inside the file.
inline bool record_at(const uint8_t* f, uint64_t len, bool sw, uint64_t off, Record& r) {
  if (off > len || len - off < kRecordHeader) return false;
  r.ts_sec = rd32(f + off, sw);
  r.ts_frac = rd32(f + off + 4, sw);
  r.caplen = rd32(f + off + 8, sw);
  r.wirelen = rd32(f + off + 12, sw);
  return len - off - kRecordHeader >= r.caplen;
}

}  // namespace

extern "C" int xe_pcap_header(const uint8_t* f, uint64_t len, xe_pcap_info* info) {
  if (!f || !info || len < kGlobalHeader) return XE_ERR_FORMAT;
  uint32_t m;
  memcpy(&m, f, 4);
  bool sw = false, ns = false;
  if (m == kMagicUs) {
  } else if (m == kMagicNs) {
    ns = true;
  } else if (m == __builtin_bswap32(kMagicUs)) {
    sw = true;
  } else if (m == __builtin_bswap32(kMagicNs)) {
    sw = ns = true;
  } else {
    return XE_ERR_FORMAT;
  }
  info->swapped = sw;
  info->nanosecond = ns;
  info->snaplen = rd32(f + 16, sw);
  info->linktype = rd32(f + 20, sw) & 0x0fffffffu;  // upper bits: FCS length flags
  info->first_record = kGlobalHeader;
  return XE_OK;
}

extern "C" int xe_pcap_count(const uint8_t* f, uint64_t len, const xe_pcap_info* info, uint64_t off,
                             uint64_t* records, uint64_t* bytes) {
  if (!f || !info) return XE_ERR_INVAL;
  uint64_t n = 0, b = 0;
  Record r;
  while (record_at(f, len, info->swapped, off, r)) {
    n++;
    b += r.caplen;
    off += kRecordHeader + r.caplen;
  }
  if (records) *records = n;
  if (bytes) *bytes = b;
  return XE_OK;
}

inline uint64_t ts_of(const Record& r, const xe_pcap_info* info) {
  return uint64_t(r.ts_sec) * 1000000000ull + (info->nanosecond ? r.ts_frac : uint64_t(r.ts_frac) * 1000u);
}

extern "C" int xe_pcap_fill(const uint8_t* f, uint64_t len, const xe_pcap_info* info, uint64_t* offset,
                            uint8_t* umem, uint64_t umem_len, uint32_t frame_size, uint32_t headroom,
                            const uint64_t* frame_addr, uint64_t first_frame, uint32_t max, xe_desc* desc,
                            uint32_t* orig_len, uint64_t* ts_ns, uint32_t* filled) {
  if (filled) *filled = 0;
  if (!f || !info || !offset || !desc || !filled || (max && !umem) || frame_size <= headroom) return XE_ERR_INVAL;
  const uint64_t room = frame_size - headroom;
  uint64_t off = *offset;
  uint32_t k = 0;
  Record r;
  for (; k < max && record_at(f, len, info->swapped, off, r); k++) {
    const uint64_t frame = frame_addr ? frame_addr[k] : (first_frame + k) * uint64_t(frame_size);
    if (frame % frame_size || frame > umem_len || umem_len - frame < frame_size) {
      *offset = off;
      *filled = k;
      return XE_ERR_INVAL;
    }
    const uint64_t n = r.caplen < room ? r.caplen : room;
    memcpy(umem + frame + headroom, f + off + kRecordHeader, n);
    desc[k].addr = frame + headroom;
    desc[k].len = uint32_t(n);
    desc[k].options = 0;
    if (orig_len) orig_len[k] = r.wirelen;
    if (ts_ns) ts_ns[k] = ts_of(r, info);
    off += kRecordHeader + r.caplen;
  }
  *offset = off;
  *filled = k;
  return XE_OK;
}

// Two passes: the record walk (sequential: each header gives the next offset) lays out the
// descriptors and remembers where each record's bytes are; the copies then run on several threads.
extern "C" int xe_pcap_pack(const uint8_t* f, uint64_t len, const xe_pcap_info* info, uint64_t* offset, uint8_t* buf,
                            uint64_t buf_len, uint32_t align, uint32_t max_len, uint32_t max, xe_desc* desc,
                            uint32_t* orig_len, uint64_t* ts_ns, uint32_t* filled, uint64_t* used) {
  if (filled) *filled = 0;
  if (used) *used = 0;
  if (!f || !info || !offset || !desc || !filled || !used || (max && !buf) || align < 16 || (align & (align - 1)))
    return XE_ERR_INVAL;
  uint64_t off = *offset, at = 0;
  uint32_t k = 0;
  std::vector<uint64_t> src;
  src.reserve(std::min<uint32_t>(max, 1u << 20));
  Record r;
  uint64_t pf = off;  // the walk is a dependent chain of header loads: stream the file in ahead of it
  for (; k < max && record_at(f, len, info->swapped, off, r); k++) {
    const uint64_t n = max_len && r.caplen > max_len ? max_len : r.caplen;
    if (at > buf_len || buf_len - at < n) break;
    for (const uint64_t want = std::min(len, off + kPrefetch); pf < want; pf += 64) __builtin_prefetch(f + pf);
    src.push_back(off + kRecordHeader);
    desc[k].addr = at;
    desc[k].len = uint32_t(n);
    desc[k].options = 0;
    if (orig_len) orig_len[k] = r.wirelen;
    if (ts_ns) ts_ns[k] = ts_of(r, info);
    off += kRecordHeader + r.caplen;
    at += (n + align - 1) & ~uint64_t(align - 1);
  }
  auto copy = [&](uint32_t lo, uint32_t hi) {
    for (uint32_t i = lo; i < hi; i++) memcpy(buf + desc[i].addr, f + src[i], desc[i].len);
  };
  const uint32_t hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const uint32_t nt = k >= (1u << 15) ? hw : 1u;
  if (nt == 1) {
    copy(0, k);
  } else {
    std::vector<std::thread> pool;
    for (uint32_t t = 0; t < nt; t++) pool.emplace_back(copy, uint32_t(uint64_t(k) * t / nt), uint32_t(uint64_t(k) * (t + 1) / nt));
    for (auto& th : pool) th.join();
  }
  *offset = off;
  *filled = k;
  *used = at < buf_len ? at : buf_len;
  return XE_OK;
}
