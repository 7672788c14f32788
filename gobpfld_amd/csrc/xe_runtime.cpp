// xe_runtime.cpp — host runtime and C ABI (include/xdpemu.h) of the batched eBPF/XDP emulator.
//
// * decoder + translator: raw eBPF -> 16-byte micro-ops, reproducing ebpf.Decode's accept/reject
//   table (ebpf/decode.go:8-917) and emulator.Translate's (emulator/inst.go:21-238); register-number
//   errors that the reference would raise deterministically at run time become U_FAIL micro-ops.
// * maps: ARRAY and HASH realised as device-resident tables (host mirror for userspace access).
// * batch runs: parallel kernel, footprint/ordered-write verification, exact sequential fallback.
//
// Built twice: with hipcc into gobpfld_amd/libxdpemu.so (the product), and with g++ -DXE_HOSTSIM
// into tests/hostsim/ (CPU-only test build of the same logic; never loaded by the product).
#include "xe_internal.h"

#include <algorithm>
#include <map>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <array>
#include <thread>
#include <vector>

#ifdef XE_HOSTSIM
// the host simulation runs the one-lane replay's runahead too (seq_packets): every packet runs once with
// its shared writes stopped before it runs for real, so the CPU tests see any effect that leaks from it
#define XE_SEQ_PEEK 1
#include "xe_interp.h"
typedef void* xe_stream_t;
#else
#include <hip/hip_runtime_api.h>
typedef hipStream_t xe_stream_t;
extern "C" int xe_launch_interp(const XeParams* P, uint32_t blocks, uint32_t threads, hipStream_t s);
extern "C" int xe_launch_delta(const void* cur, const void* snap, void* out, uint64_t bytes, uint32_t lane, hipStream_t s);
extern "C" int xe_launch_apply_delta(void* cur, const void* snap, const void* delta, uint64_t bytes, uint32_t lane,
                                     hipStream_t s);
extern "C" int xe_launch_rep_fold(void* vals, void* rep, uint64_t stride_words, uint32_t nrep, uint64_t nwords,
                                  const void* recs, uint32_t rwords, uint32_t vsize, uint32_t cap, const void* lim, hipStream_t s);
extern "C" int xe_launch_delta_sum(void* acc, const void* in, uint64_t bytes, uint32_t lane, hipStream_t s);
extern "C" int xe_launch_prologue(const void* const* src, void* const* dst, const uint64_t* words, uint32_t nseg,
                                  void* zero, uint64_t zero_words, hipStream_t s);
extern "C" int xe_launch_tail(const XeTailArgs* A, hipStream_t s);
extern "C" int xe_launch_desc_overlap(const void* desc, uint32_t n, uint64_t umem_len, void* scratch, size_t* scratch_bytes,
                                      uint32_t* flag, hipStream_t s);
extern "C" void* xe_jit_get(const XeUop* const* progs, const uint32_t* lens, uint32_t nprogs, int32_t entry, int device,
                            const XeDevMap* maps, uint32_t nmaps, bool* cyclic, bool* general, const char** err, int keyed, uint64_t* maxpath);
extern "C" int xe_launch_keyed(const XeKeyed* K, const XeDevMap* maps, uint8_t* skip, uint32_t step, uint32_t items,
                               hipStream_t s);
extern "C" int xe_launch_keyed_sort(const XeKeyed* K, uint32_t n, uint32_t end_bit, void* scratch, size_t* bytes, hipStream_t s);
extern "C" int xe_launch_keyed_esort(const XeKeyed* K, void* scratch, size_t* bytes, hipStream_t s);
extern "C" int xe_launch_append(const XeAppendArgs* A, uint32_t end_bit, void* scratch, size_t* bytes, hipStream_t s);
extern "C" int xe_launch_keyed_scan(const XeKeyed* K, uint32_t n, void* scratch, size_t* bytes, hipStream_t s);
extern "C" int xe_launch_pop(const uint32_t* src, uint32_t* dst, uint32_t n, uint32_t mode, uint32_t arg, XePopSlots sl,
                             uint32_t* flag, hipStream_t s);
extern "C" int xe_launch_lru_relink(uint64_t* tag, uint32_t pool, uint32_t cnt, uint32_t* link, uint64_t* hdr, void* scratch,
                                    size_t* bytes, int renumber, hipStream_t s);
extern "C" int xe_launch_lru_tag_fold(uint64_t* tag, uint64_t* rep, uint32_t pool, uint32_t r, const uint64_t* hdr, hipStream_t s);
extern "C" int xe_launch_lru_log(const uint64_t* tag, uint32_t pool, const uint32_t* order, const uint64_t* hdr, uint64_t* log,
                                 hipStream_t s);
extern "C" int xe_jit_launch(void* fn, const XeParams* P, uint32_t blocks, uint32_t threads, hipStream_t s);
extern "C" int xe_jit_occupancy(void* fn, uint32_t nmaps);
extern "C" int xe_interp_occupancy(uint32_t nmaps);
#endif

// the kernel generator (xe_jit.cpp; in the host simulation too: sources only, no compiles)
extern "C" int xe_jit_may_write_entries(const XeUop* prog, size_t n);
extern "C" size_t xe_jit_source_for(const XeUop* const* progs, const uint32_t* lens, uint32_t nprogs, int32_t entry,
                                    const XeDevMap* maps, uint32_t nmaps, int keyed, char* buf, size_t buflen);

#define XE_FRAME_SIZE 256  // DefaultVMSettings().StackFrameSize (emulator/vm.go:291-296)

namespace {

// ------------------------------------------------------------------ backend
#ifdef XE_HOSTSIM
#ifdef XE_HOSTSIM_POISON  // (sanitizer build) device memory starts as garbage, as hipMalloc's may
int dev_alloc(void** p, size_t n) {
  n = n ? n : 8;
  *p = malloc(n);
  if (*p) memset(*p, 0xA5, n);
  return *p ? 0 : -1;
}
#else
int dev_alloc(void** p, size_t n) { *p = calloc(n ? n : 8, 1); return *p ? 0 : -1; }
#endif
void dev_free(void* p) { free(p); }
int h2d(void* d, const void* h, size_t n, xe_stream_t) { memcpy(d, h, n); return 0; }
int d2h(void* h, const void* d, size_t n, xe_stream_t) { memcpy(h, d, n); return 0; }
int d2d(void* d, const void* s, size_t n, xe_stream_t) { memmove(d, s, n); return 0; }
int dmemset(void* d, int v, size_t n, xe_stream_t) { memset(d, v, n); return 0; }
int dsync(xe_stream_t) { return 0; }
int launch_interp(const XeParams* P, uint32_t, uint32_t, xe_stream_t) {
  XeLane L;
#ifdef XE_HOSTSIM_POISON  // registers a kernel never wrote: zero, the value a fresh VGPR often holds
  memset(static_cast<void*>(&L), 0, sizeof L);
#endif
  static thread_local uint8_t hdrbuf[XE_HDR_WAVE_BYTES + 16];  // one per host thread (xe_multi runs shards concurrently)
  L.hdrbuf = hdrbuf;
  XePend pend;
  stage_maps(L, *P, nullptr);
  wave_state_init(L, *P, 0, &pend);
  if (P->mode == XE_MODE_PARALLEL || P->mode == XE_MODE_SPEC) {
    parallel_packets(L, *P, 0, 1, [&](uint32_t i, bool valid) { run_staged(L, *P, i, valid); });
  } else if (P->mode == XE_MODE_CHAIN) {
    chain_packets(L, *P, 0, 1, [&](uint32_t i, bool valid) { run_staged(L, *P, i, valid); });
  } else {
    seq_packets(L, *P, [&](uint32_t i, bool valid) { run_staged(L, *P, i, valid); },
                [&](bool valid) { run_staged(L, *P, 0, valid, false); });
  }
  flush_wave_state(L, *P);
  return 0;
}
int launch_jit(void*, const XeParams* P, uint32_t b, uint32_t t, xe_stream_t s) { return launch_interp(P, b, t, s); }
template <class T, class C = T>
void lanes_sub(const void* a, const void* b, void* o, uint64_t n) {
  for (uint64_t i = 0; i < n; i++) ((C*)o)[i] = C(T(((const T*)a)[i] - ((const T*)b)[i]));
}
template <class T, class C = T>
void lanes_add(const void* snap, const void* d, void* o, uint64_t n) {
  for (uint64_t i = 0; i < n; i++) ((T*)o)[i] = T(((const T*)snap)[i] + T(((const C*)d)[i]));
}
template <class C>
void lanes_acc(void* acc, const void* in, uint64_t n) {
  for (uint64_t i = 0; i < n; i++) ((C*)acc)[i] = C(((C*)acc)[i] + ((const C*)in)[i]);
}
int launch_delta(const void* cur, const void* snap, void* out, uint64_t bytes, uint32_t lane, xe_stream_t) {
  switch (lane) {
    case 1: lanes_sub<uint8_t>(cur, snap, out, bytes); break;
    case 2: lanes_sub<uint16_t, uint32_t>(cur, snap, out, bytes / 2); break;
    case 4: lanes_sub<uint32_t>(cur, snap, out, bytes / 4); break;
    default: lanes_sub<uint64_t>(cur, snap, out, bytes / 8); break;
  }
  return 0;
}
int launch_apply_delta(void* cur, const void* snap, const void* delta, uint64_t bytes, uint32_t lane, xe_stream_t) {
  switch (lane) {
    case 1: lanes_add<uint8_t>(snap, delta, cur, bytes); break;
    case 2: lanes_add<uint16_t, uint32_t>(snap, delta, cur, bytes / 2); break;
    case 4: lanes_add<uint32_t>(snap, delta, cur, bytes / 4); break;
    default: lanes_add<uint64_t>(snap, delta, cur, bytes / 8); break;
  }
  return 0;
}
int launch_delta_sum(void* acc, const void* in, uint64_t bytes, uint32_t lane, xe_stream_t) {
  switch (lane) {
    case 1: lanes_acc<uint8_t>(acc, in, bytes); break;
    case 2: case 4: lanes_acc<uint32_t>(acc, in, bytes / lane); break;
    default: lanes_acc<uint64_t>(acc, in, bytes / 8); break;
  }
  return 0;
}
int launch_prologue(const void* const* src, void* const* dst, const uint64_t* words, uint32_t nseg, void* zero, uint64_t zw,
                    xe_stream_t) {
  if (zw) memset(zero, 0, zw * 8);
  for (uint32_t g = 0; g < nseg; g++) memcpy(dst[g], src[g], words[g] * 8);
  return 0;
}
int launch_rep_fold(void* vals, void* rep, uint64_t sw, uint32_t nrep, uint64_t nw, const void* recs, uint32_t rwords,
                    uint32_t vsize, uint32_t cap, const void* lim, xe_stream_t) {
  uint64_t* v = (uint64_t*)vals;
  uint64_t* r = (uint64_t*)rep;
  const uint64_t* rc = (const uint64_t*)recs;
  if (lim) nw = std::min<uint64_t>(nw, (((const uint64_t*)lim)[3] * vsize + 7) / 8);
  for (uint64_t i = 0; i < nw; i++) {
    if (rc) {  // xe_kernel.hip xe_rep_fold_kernel: only the words of slots that hold or held an entry
      const uint64_t s0 = 8 * i / vsize, s1 = (8 * i + 7) / vsize;
      if (!((s0 <= cap && rc[s0 * rwords]) || (s1 != s0 && s1 <= cap && rc[s1 * rwords]))) continue;
    }
    for (uint32_t k = 0; k < nrep; k++) { v[i] += r[k * sw + i]; r[k * sw + i] = 0; }
  }
  return 0;
}
int launch_tail(const XeTailArgs* A, xe_stream_t) {  // xe_kernel.hip xe_tail_kernel, one thread
  unsigned long long orw[257] = {};
  const bool poisoned = *A->poison != 0;
  for (uint32_t i = 0; i < A->aux_words; i++) {
    const unsigned long long v = A->aux[i];
    A->aux[i] = 0;
    A->host_aux[i] = v;
    if (i == 0) orw[256] = v;
    else if (i >= 16) orw[(i - 16) % A->rep_words] |= v;
  }
  const bool replay = !poisoned && xe_replay_decision(uint32_t(orw[256]), orw, A->rep_words, A->nmaps, A->mode);
  A->host_aux[XE_AUX_DECISION] = replay ? 1ull : 0ull;
  if (replay) *A->poison = 1u;
  if (poisoned) return 0;
  for (uint32_t f = 0; f < A->ntail; f++) {
    const XeTailMap& T = A->tail[f];
    for (uint64_t i = 0; i < T.words; i++) {
      unsigned long long s = 0;
      for (uint32_t k = 0; k < T.nrep; k++) { s += T.rep[k * T.stride_words + i]; T.rep[k * T.stride_words + i] = 0; }
      T.vals[i] += s;
      T.snap[i] = T.vals[i];
    }
  }
  return 0;
}
int host_alloc(void** p, size_t n) { *p = calloc(n ? n : 8, 1); return *p ? 0 : -1; }
void host_free(void* p) { free(p); }
int host_device_ptr(void** d, void* h) { *d = h; return 0; }
int host_alloc_coherent(void** p, size_t n) { return host_alloc(p, n); }
// host helpers: the simulated kernel ran on this thread and called them in place
int serve_hostcalls(XeHostCall*, xe_stream_t) { return 0; }
// xe_cancel: the simulated batches are complete when their call returns
int poison_async(uint32_t* d, xe_stream_t*) { *d = 2; return 0; }
void stream_destroy(xe_stream_t) {}
int launch_desc_overlap(const void* desc, uint32_t n, uint64_t umem_len, void* scratch, size_t* bytes, uint32_t* flag,
                        xe_stream_t) {  // xe_kernel.hip xe_launch_desc_overlap
  if (!scratch) { *bytes = 8; return 0; }
  std::vector<std::pair<uint64_t, uint32_t>> r;
  const xe_desc* d = (const xe_desc*)desc;
  for (uint32_t i = 0; i < n; i++) {
    uint32_t l = d[i].len;
    if (d[i].addr > umem_len || uint64_t(l) > umem_len - d[i].addr) l = 0;
    if (l) r.emplace_back(d[i].addr, l);
  }
  std::sort(r.begin(), r.end());
  *flag = 0;
  for (size_t i = 0; i + 1 < r.size(); i++)
    if (r[i].first + r[i].second > r[i + 1].first) *flag = 1;
  return 0;
}
int launch_keyed(const XeKeyed* K, const XeDevMap* maps, uint8_t* skip, uint32_t step, uint32_t items, xe_stream_t) {
  if (step == XE_KS_COUNT) {  // xe_kernel.hip xe_keyed_count_kernel
    for (uint32_t x = 0; x < K->dcap; x++)
      if (K->dkid[x]) {
        K->dcount[K->dkid[x] >> 58]++;
        if (K->dkey[uint64_t(x) * K->kw] & XE_KEY_VALID) K->dins[K->dkid[x] >> 58]++;
      }
    return 0;
  }
  for (uint32_t i = 0; i < items; i++) keyed_step(*K, maps, skip, step, i);  // xe_kernel.hip xe_keyed_kernel
  if (step == XE_KS_DSET && getenv("XE_HOSTSIM_DCYCLE")) {
    // test-only fault injection: a parent cycle between D's first two keys, the state a corrupted D table
    // leaves — keyed_root must send the batch to the replay instead of returning a partial root
    uint32_t a = K->dcap, b = K->dcap;
    for (uint32_t x = 0; x < K->dcap && b == K->dcap; x++)
      if (K->dkid[x]) (a == K->dcap ? a : b) = x;
    if (b != K->dcap) { K->dcomp[a] = b; K->dcomp[b] = a; }
  }
  return 0;
}
int launch_keyed_sort(const XeKeyed* K, uint32_t n, uint32_t, void* scratch, size_t* bytes, xe_stream_t) {
  if (!scratch) { *bytes = 8; return 0; }
  std::vector<std::pair<uint32_t, uint32_t>> v(n);
  for (uint32_t i = 0; i < n; i++) v[i] = {K->ckey[i], K->iota[i]};
  std::stable_sort(v.begin(), v.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  for (uint32_t i = 0; i < n; i++) { K->okey[i] = v[i].first; K->order[i] = v[i].second; }
  return 0;
}
int launch_keyed_esort(const XeKeyed* K, void* scratch, size_t* bytes, xe_stream_t) {  // xe_launch_keyed_esort
  if (!scratch) { *bytes = 8; return 0; }
  std::vector<std::pair<uint64_t, uint32_t>> v(K->dcap);
  for (uint32_t i = 0; i < K->dcap; i++) v[i] = {K->ekey[i], K->eval[i]};
  std::stable_sort(v.begin(), v.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  for (uint32_t i = 0; i < K->dcap; i++) { K->ekey2[i] = v[i].first; K->eval2[i] = v[i].second; }
  return 0;
}
int launch_lru_relink(uint64_t* tag, uint32_t pool, uint32_t cnt, uint32_t* link, uint64_t* hdr, void* scratch,
                      size_t* bytes, int renumber, xe_stream_t) {  // xe_kernel.hip xe_launch_lru_relink
  // scratch as on the device: sorted stamps, value ids in, value ids out (lru_sorted_ids)
  if (!scratch) { *bytes = size_t(pool) * 16 + 256; return 0; }
  std::vector<uint32_t> v(pool);
  for (uint32_t i = 0; i < pool; i++) v[i] = i;
  std::stable_sort(v.begin(), v.end(), [&](uint32_t a, uint32_t b) { return tag[a] > tag[b]; });
  uint32_t* vout = (uint32_t*)((uint8_t*)scratch + size_t(pool) * 8) + pool;
  for (uint32_t i = 0; i < pool; i++) vout[i] = v[i];
  if (renumber == 2) return 0;  // the order only
  for (uint32_t i = 0; i < cnt && i < pool; i++) {
    if (renumber) tag[v[i]] = cnt - i;
    link[4 * uint64_t(v[i])] = i ? v[i - 1] : XE_NONE;
    link[4 * uint64_t(v[i]) + 1] = i + 1 < cnt ? v[i + 1] : XE_NONE;
  }
  hdr[0] = cnt ? v[0] : XE_NONE;
  hdr[1] = cnt ? v[cnt - 1] : XE_NONE;
  return 0;
}
int launch_lru_tag_fold(uint64_t* tag, uint64_t* rep, uint32_t pool, uint32_t r, const uint64_t* hdr, xe_stream_t) {  // xe_lru_tag_fold_kernel
  for (uint64_t v = 0; v < std::min<uint64_t>(pool, hdr[3]); v++)
    for (uint32_t k = 0; k < r; k++) {
      uint64_t& x = rep[k * uint64_t(pool) + v];
      if (x > tag[v]) tag[v] = x;
      x = 0;
    }
  return 0;
}
int launch_lru_log(const uint64_t* tag, uint32_t, const uint32_t* order, const uint64_t* hdr, uint64_t* log, xe_stream_t) {
  const uint64_t cnt = hdr[2];  // xe_kernel.hip xe_lru_log_kernel: oldest first
  for (uint64_t i = 0; i < cnt; i++) {
    const uint32_t v = order[cnt - 1 - i];
    log[8 + 2 * i] = tag[v];
    log[9 + 2 * i] = v;
  }
  log[0] = 0;
  log[1] = cnt;
  log[2] = log[3] = XE_NONE;  // no freed value ids (xe_interp.h lru_free_push)
  return 0;
}
int launch_keyed_scan(const XeKeyed* K, uint32_t n, void* scratch, size_t* bytes, xe_stream_t) {
  if (!scratch) { *bytes = 8; return 0; }
  uint32_t acc = 0;
  for (uint32_t i = 0; i < n; i++) { K->ckey[i] = acc; acc += K->iota[i]; }
  return 0;
}
int launch_pop(const uint32_t* src, uint32_t* dst, uint32_t n, uint32_t mode, uint32_t arg, XePopSlots sl, uint32_t* flag,
               xe_stream_t) {  // xe_kernel.hip xe_pop_kernel
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t v = src[i];
    if (mode == 0) dst[i] = v ? 1u << (8u * (sl.slot[(v - 1u) & 63u] & 3u)) : 0u;
    else if (mode == 1) dst[i] = (v >> (8u * arg)) & 0xffu;
    else if (v != dst[i]) *flag = 1u;
  }
  return 0;
}
int launch_append(const XeAppendArgs* A, uint32_t, void* scratch, size_t* bytes, xe_stream_t) {
  if (!scratch) { *bytes = 8; return 0; }
  std::vector<std::pair<uint64_t, uint32_t>> v(A->k);
  for (uint32_t j = 0; j < A->k; j++) v[j] = {A->tag[A->base + j], uint32_t(A->base + j)};
  std::stable_sort(v.begin(), v.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  std::vector<uint64_t> rec;
  if (A->perf) rec.assign(A->rec + 2 * A->base, A->rec + 2 * (A->base + A->k));
  for (uint32_t j = 0; j < A->k; j++) {
    const uint32_t id = v[j].second;
    if (A->perf) {
      A->rec[2 * (A->base + j)] = rec[2 * (id - A->base)];
      A->rec[2 * (A->base + j) + 1] = rec[2 * (id - A->base) + 1];
    } else {
      A->link[A->stack ? A->cnt0 + j : (A->head + A->cnt0 + j) % A->list_cap] = id;
    }
  }
  return 0;
}
struct Timer {
  std::chrono::steady_clock::time_point t;
  void rec(xe_stream_t) { t = std::chrono::steady_clock::now(); }
  static float ms(const Timer& a, const Timer& b) { return std::chrono::duration<float, std::milli>(b.t - a.t).count(); }
  int wait() { return 0; }
  void init() {}
  void fini() {}
};
int set_device(int) { return 0; }
int blocks_per_cu(void*, uint32_t) { return 1; }
int cu_count(int) { return 1; }
#else
int dev_alloc(void** p, size_t n) { return hipMalloc(p, n ? n : 8) == hipSuccess ? 0 : -1; }
void dev_free(void* p) { if (p) (void)hipFree(p); }
int h2d(void* d, const void* h, size_t n, xe_stream_t s) { return hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s) == hipSuccess ? 0 : -1; }
int d2h(void* h, const void* d, size_t n, xe_stream_t s) { return hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, s) == hipSuccess ? 0 : -1; }
int d2d(void* d, const void* src, size_t n, xe_stream_t s) { return hipMemcpyAsync(d, src, n, hipMemcpyDeviceToDevice, s) == hipSuccess ? 0 : -1; }
int dmemset(void* d, int v, size_t n, xe_stream_t s) { return hipMemsetAsync(d, v, n, s) == hipSuccess ? 0 : -1; }
int dsync(xe_stream_t s) { return hipStreamSynchronize(s) == hipSuccess ? 0 : -1; }
int launch_interp(const XeParams* P, uint32_t b, uint32_t t, xe_stream_t s) { return xe_launch_interp(P, b, t, s); }
int launch_jit(void* fn, const XeParams* P, uint32_t b, uint32_t t, xe_stream_t s) { return xe_jit_launch(fn, P, b, t, s); }
int launch_delta(const void* c, const void* sn, void* o, uint64_t b, uint32_t lane, xe_stream_t s) {
  return xe_launch_delta(c, sn, o, b, lane, s);
}
int launch_apply_delta(void* c, const void* sn, const void* d, uint64_t b, uint32_t lane, xe_stream_t s) {
  return xe_launch_apply_delta(c, sn, d, b, lane, s);
}
int launch_rep_fold(void* v, void* r, uint64_t sw, uint32_t nrep, uint64_t nw, const void* recs, uint32_t rwords, uint32_t vsize,
                    uint32_t cap, const void* lim, xe_stream_t s) {
  return xe_launch_rep_fold(v, r, sw, nrep, nw, recs, rwords, vsize, cap, lim, s);
}
int launch_delta_sum(void* acc, const void* in, uint64_t bytes, uint32_t lane, xe_stream_t s) {
  return xe_launch_delta_sum(acc, in, bytes, lane, s);
}
int launch_prologue(const void* const* src, void* const* dst, const uint64_t* words, uint32_t nseg, void* zero, uint64_t zw,
                    xe_stream_t s) {
  return xe_launch_prologue(src, dst, words, nseg, zero, zw, s);
}
int host_alloc(void** p, size_t n) { return hipHostMalloc(p, n ? n : 8, hipHostMallocDefault) == hipSuccess ? 0 : -1; }
int launch_keyed(const XeKeyed* K, const XeDevMap* maps, uint8_t* skip, uint32_t step, uint32_t items, xe_stream_t s) {
  return xe_launch_keyed(K, maps, skip, step, items, s);
}
int launch_keyed_esort(const XeKeyed* K, void* scratch, size_t* bytes, xe_stream_t s) {
  return xe_launch_keyed_esort(K, scratch, bytes, s);
}
int launch_keyed_sort(const XeKeyed* K, uint32_t n, uint32_t end_bit, void* scratch, size_t* bytes, xe_stream_t s) {
  return xe_launch_keyed_sort(K, n, end_bit, scratch, bytes, s);
}
int launch_append(const XeAppendArgs* A, uint32_t end_bit, void* scratch, size_t* bytes, xe_stream_t s) {
  return xe_launch_append(A, end_bit, scratch, bytes, s);
}
int launch_pop(const uint32_t* src, uint32_t* dst, uint32_t n, uint32_t mode, uint32_t arg, XePopSlots sl, uint32_t* flag,
               xe_stream_t s) {
  return xe_launch_pop(src, dst, n, mode, arg, sl, flag, s);
}
int launch_keyed_scan(const XeKeyed* K, uint32_t n, void* scratch, size_t* bytes, xe_stream_t s) {
  return xe_launch_keyed_scan(K, n, scratch, bytes, s);
}
void host_free(void* p) { if (p) (void)hipHostFree(p); }
int launch_lru_relink(uint64_t* tag, uint32_t pool, uint32_t cnt, uint32_t* link, uint64_t* hdr, void* scratch,
                      size_t* bytes, int renumber, xe_stream_t s) {
  return xe_launch_lru_relink(tag, pool, cnt, link, hdr, scratch, bytes, renumber, s);
}
int launch_lru_tag_fold(uint64_t* tag, uint64_t* rep, uint32_t pool, uint32_t r, const uint64_t* hdr, xe_stream_t s) {
  return xe_launch_lru_tag_fold(tag, rep, pool, r, hdr, s);
}
int launch_lru_log(const uint64_t* tag, uint32_t pool, const uint32_t* order, const uint64_t* hdr, uint64_t* log, xe_stream_t s) {
  return xe_launch_lru_log(tag, pool, order, hdr, log, s);
}
int launch_tail(const XeTailArgs* A, xe_stream_t s) { return xe_launch_tail(A, s); }
int launch_desc_overlap(const void* desc, uint32_t n, uint64_t umem_len, void* scratch, size_t* bytes, uint32_t* flag,
                        xe_stream_t s) {
  return xe_launch_desc_overlap(desc, n, umem_len, scratch, bytes, flag, s);
}
// device-visible address of pinned host memory (hipHostMalloc default: mapped, coherent)
int host_device_ptr(void** d, void* h) { return hipHostGetDevicePointer(d, h, 0) == hipSuccess ? 0 : -1; }
// pinned host memory the device polls with system-scope atomics (the host helper mailbox)
int host_alloc_coherent(void** p, size_t n) {
  if (hipHostMalloc(p, n ? n : 8, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return -1;
  memset(*p, 0, n);
  return 0;
}
// Host helpers (xe_set_helper): until the batch's stream is idle, answer the one-lane replay's requests
// in the mailbox (the lane waits for ack == req), calling the registered function on this thread.
int serve_hostcalls(XeHostCall* H, xe_stream_t s) {
  for (;;) {
    const uint32_t req = __atomic_load_n(&H->req, __ATOMIC_ACQUIRE);
    if (req != __atomic_load_n(&H->ack, __ATOMIC_RELAXED)) {
      const uint32_t id = H->id;
      int64_t a[5];
      uint8_t k[5];
      for (int r = 0; r < 5; r++) { a[r] = H->args[r]; k[r] = H->kinds[r]; }
      int64_t r0 = 0;
      const int err = (id < 192 && H->fn[id]) ? H->fn[id](H->user[id], H->packet, a, k, &r0) : 1;
      H->r0 = r0;
      H->err = err ? 1 : 0;
      __atomic_store_n(&H->ack, req, __ATOMIC_RELEASE);
      continue;
    }
    const hipError_t q = hipStreamQuery(s);
    if (q == hipSuccess) return 0;
    if (q != hipErrorNotReady) return -1;
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}
// xe_cancel: mark the pipelined batches poisoned from a stream of its own, so the batches still queued
// behind the running one see it at their first wave (the VM's stream would run the write after them)
int poison_async(uint32_t* d, xe_stream_t* cs) {
  if (!*cs && hipStreamCreateWithFlags(cs, hipStreamNonBlocking) != hipSuccess) return -1;
  if (hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d), 2u, 1, *cs) != hipSuccess) return -1;
  return hipStreamSynchronize(*cs) == hipSuccess ? 0 : -1;
}
void stream_destroy(xe_stream_t s) { if (s) (void)hipStreamDestroy(s); }
struct Timer {
  hipEvent_t e = nullptr;
  void init() { if (!e) (void)hipEventCreate(&e); }
  void fini() { if (e) (void)hipEventDestroy(e); e = nullptr; }
  void rec(xe_stream_t s) { init(); (void)hipEventRecord(e, s); }
  int wait() { return hipEventSynchronize(e) == hipSuccess ? 0 : -1; }
  static float ms(const Timer& a, const Timer& b) { float m = 0; (void)hipEventElapsedTime(&m, a.e, b.e); return m; }
};
int set_device(int d) { return hipSetDevice(d) == hipSuccess ? 0 : -1; }
// resident 256-thread blocks per CU of the kernel that will run (0 = unknown)
int blocks_per_cu(void* jit, uint32_t nmaps) { return jit ? xe_jit_occupancy(jit, nmaps) : xe_interp_occupancy(nmaps); }
int cu_count(int dev) {
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  return n;
}
#endif

// ------------------------------------------------------------------ decoder + translator
int size_log2(uint8_t sizecode) {  // ebpf.Size: W=0x00, H=0x08, B=0x10, DW=0x18 (ebpf/ebpf.go:106-116)
  switch (sizecode) { case 0x00: return 2; case 0x08: return 1; case 0x10: return 0; default: return 3; }
}

XeUop fail_uop(int code) { XeUop u{}; u.cls = U_FAIL; u.imm = code; return u; }

// Returns XE_OK, XE_ERR_DECODE or XE_ERR_TRANSLATE.
int translate(const uint64_t* raw, uint32_t n, std::vector<XeUop>& out, std::string& err) {
  out.assign(n, XeUop{});
  for (uint32_t i = 0; i < n; i++) {
    const uint64_t r = raw[i];
    const uint8_t op = uint8_t(r);
    const uint8_t dst = uint8_t(r >> 8) & 0x0f, src = uint8_t(r >> 12) & 0x0f;
    const int16_t off = int16_t(uint16_t(r >> 16));
    const int32_t imm = int32_t(uint32_t(r >> 32));
    const uint8_t cls = op & 7;
    XeUop u{};
    bool decoded = true, translated = true;

    if (op == 0x18) {  // LD_IMM64 (ebpf/decode.go:21-36) + its Nop filler slot
      if (i + 1 >= n) { err = "decode: load double word imm op code found but not enough instructions"; return XE_ERR_DECODE; }
      if (dst > 9) u = fail_uop(XE_E_BAD_REG);  // Registers.Get(dst) first, inst_load.go:22-25
      else { u.cls = U_LDIMM64; u.dst = dst; u.src = src; u.imm = imm; u.x = uint32_t(raw[i + 1] >> 32); }
      out[i] = u;
      out[i + 1] = XeUop{}; out[i + 1].cls = U_NOP;
      i++;
      continue;
    }
    switch (op) {
      case 0x20: case 0x28: case 0x30: case 0x38:  // LD ABS / IND: translate, fail at run time
      case 0x40: case 0x48: case 0x50: case 0x58:
        u = fail_uop(XE_E_NOT_IMPL);
        break;
      case 0x61: case 0x69: case 0x71: case 0x79:  // LDX (inst_load.go:84-118)
        if (src > 10) { u = fail_uop(XE_E_BAD_REG); break; }
        u.cls = U_LDX; u.src = src; u.tgt = off; u.fl = uint8_t(size_log2(op ^ 0x61) << 4);
        if (dst > 9) u.fl |= UF_BADDST; else u.dst = dst;
        break;
      case 0x62: case 0x6a: case 0x72: case 0x7a:  // ST (inst_store.go:20-51)
        if (dst > 10) { u = fail_uop(XE_E_BAD_REG); break; }
        u.cls = U_ST; u.dst = dst; u.imm = imm; u.tgt = off; u.fl = uint8_t(size_log2(op ^ 0x62) << 4);
        break;
      case 0x63: case 0x6b: case 0x73: case 0x7b:  // STX (inst_store.go:64-99)
        if (src > 9 || dst > 10) { u = fail_uop(XE_E_BAD_REG); break; }
        u.cls = U_STX; u.dst = dst; u.src = src; u.tgt = off; u.fl = uint8_t(size_log2(op ^ 0x63) << 4);
        break;
      case 0xc3: case 0xcb: case 0xd3: case 0xdb: {  // atomics (decode.go:124-184)
        bool known = imm == 0x00 || imm == 0x01 || imm == 0x10 || imm == 0x11 || imm == 0x50 || imm == 0x51 ||
                     imm == 0x40 || imm == 0x41 || imm == 0xa0 || imm == 0xa1 || imm == 0xe1 || imm == 0xf1;
        if (!known) { decoded = false; break; }
        if (imm != 0x00 && imm != 0x01) { translated = false; break; }  // only AtomicAdd (inst.go:52-53)
        if (dst > 10) { u = fail_uop(XE_E_BAD_REG); break; }
        u.cls = U_ATOMIC; u.dst = dst; u.tgt = off; u.fl = uint8_t(size_log2(op ^ 0xc3) << 4);
        if (src > 9) u.fl |= UF_BADSRC; else u.src = src;
        break;
      }
      default:
        if (cls == 0x04 || cls == 0x07) {  // ALU / ALU64 (decode.go:186-540)
          const uint8_t aop = op & 0xf0;
          const bool x = op & 0x08, wide = cls == 0x07;
          if (aop == 0x80) {  // NEG: K form only
            if (x) { decoded = false; break; }
            if (dst > 9) { u = fail_uop(XE_E_BAD_REG); break; }
            u.cls = U_NEG; u.dst = dst; u.fl = wide ? UF_WIDE : 0;
          } else if (aop == 0xd0) {  // END: ALU class, imm 16/32/64
            if (wide || !(imm == 16 || imm == 32 || imm == 64)) { decoded = false; break; }
            if (dst > 9) { u = fail_uop(XE_E_BAD_REG); break; }
            u.cls = U_END; u.dst = dst; u.imm = imm; u.x = x ? 8 : 0;
          } else if (aop == 0xe0 || aop == 0xf0) {
            decoded = false;
          } else if (aop == 0xb0) {  // MOV (inst_mov.go)
            if (!x) {
              if (dst > 9) { u = fail_uop(XE_E_ASSIGN_REG); break; }
              u.cls = U_MOVI; u.dst = dst; u.imm = imm;
            } else {
              if (src > 10) { u = fail_uop(XE_E_BAD_REG); break; }
              if (dst > 9) { u = fail_uop(XE_E_ASSIGN_REG); break; }
              u.cls = U_MOVR; u.dst = dst; u.src = src;
            }
            u.fl = wide ? UF_WIDE : 0;
          } else {
            if (dst > 9 || (x && src > 9)) { u = fail_uop(XE_E_BAD_REG); break; }
            u.cls = U_ALU; u.dst = dst; u.src = x ? src : 0; u.imm = imm; u.x = aop;
            u.fl = uint8_t((wide ? UF_WIDE : 0) | (x ? UF_REG : 0));
          }
        } else if (cls == 0x05 || cls == 0x06) {  // JMP / JMP32 (decode.go:544-902)
          const uint8_t jop = op & 0xf0;
          const bool x = op & 0x08;
          if (op == 0x05) { u.cls = U_JA; u.tgt = int32_t(i) + off; break; }
          if (op == 0x85) {
            if (src == 1) { u.cls = U_CALLBPF; u.imm = imm; }  // ebpf.PSEUDO_CALL
            else { u.cls = U_HELPER; u.imm = imm; }
            break;
          }
          if (op == 0x8d) {  // CALLX: helper id in register Register(imm) (uint8 truncation)
            uint8_t reg = uint8_t(imm);
            if (reg > 9) { u = fail_uop(XE_E_BAD_REG); break; }
            u.cls = U_CALLX; u.dst = reg;
            break;
          }
          if (op == 0x95) { u.cls = U_EXIT; break; }
          switch (jop) {
            case 0x10: case 0x20: case 0x30: case 0x50: case 0x60: case 0x70: case 0xc0: case 0xd0:
              if (dst > 9 || (x && src > 9)) { u = fail_uop(XE_E_BAD_REG); break; }
              u.cls = U_JMP; u.dst = dst; u.src = x ? src : 0; u.imm = imm; u.x = jop;
              u.tgt = int32_t(i) + off;
              u.fl = uint8_t((cls == 0x05 ? UF_WIDE : 0) | (x ? UF_REG : 0));
              break;
            case 0x40: case 0xa0: case 0xb0: translated = false; break;  // JSET / JLT / JLE
            default: decoded = false;
          }
        } else {
          decoded = false;
        }
    }
    if (!decoded) {
      char b[200];
      snprintf(b, sizeof b, "decode: unable to decode raw instruction, inst: %u, op: %2x, imm: %8x", i, op, uint32_t(imm));
      err = b;
      return XE_ERR_DECODE;
    }
    if (!translated) {
      char b[200];
      snprintf(b, sizeof b, "add program: translate: can't translate instruction at %u (op %2x)", i, op);
      err = b;
      // the reference decodes the whole program before translating (vm.go:61-73): finish decoding
      std::vector<XeUop> rest;
      std::string e2;
      if (i + 1 < n) {
        int rc = translate(raw + i + 1, n - i - 1, rest, e2);
        if (rc == XE_ERR_DECODE) { err = e2; return XE_ERR_DECODE; }
      }
      return XE_ERR_TRANSLATE;
    }
    out[i] = u;
  }
  return XE_OK;
}

// Read-modify-write lifting. `ldx rX, [rB+o]; add/sub rX, K|rY; stx [rB+o], rX` with rX dead after the
// store changes map memory exactly as an atomic add of +-K (mod 2^width) would: the only thing the
// lane keeps from the loaded value is the stored sum. Marking the pair UF_LIFT lets a parallel lane
// skip the read footprint and add instead of store (uop_ldx / uop_store), so `value->count++` written
// without an atomic runs in parallel instead of conflicting into the ordered replay. Programs with tail
// calls or indirect helper calls are left alone (their register flow leaves the program). bpf-to-bpf
// calls are followed: a call flows into its callee and, when the callee returns, on to the next slot
// (emulator/inst_call_bpf.go:18-44, inst_exit.go:22-48). The call keeps R6..R9 (it clones them for the
// return), an Exit returns R0..R5 to whichever call site is live. The stx carries the addend:
// imm = K, x = (rY + 1 or 0) | 0x100 when subtracting.
void lift_rmw(std::vector<XeUop>& p) {
  const size_t n = p.size();
  for (const XeUop& u : p)
    if (u.cls == U_CALLX || (u.cls == U_HELPER && u.imm == 12)) return;
  std::vector<bool> target(n + 1, false);
  auto mark = [&](int64_t t) { if (t >= 0 && size_t(t) <= n) target[size_t(t)] = true; };
  for (size_t k = 0; k < n; k++) {
    const XeUop& u = p[k];
    if (u.cls == U_JA || u.cls == U_JMP) mark(int64_t(u.tgt) + 1);
    if (u.cls == U_CALLBPF) { mark(int64_t(k) + u.imm + 1); mark(int64_t(k) + 1); }
  }
  // backward liveness over R0..R10 (bit r); exit reads R0 (and, inside a call, what the return sites
  // read of R0..R5), helpers read R1..R5 and define nothing
  std::vector<uint16_t> live(n + 1, 0);
  auto bit = [](int r) { return uint16_t(r >= 0 && r <= 10 ? 1u << r : 0u); };
  uint16_t ret_live = 0;
  for (bool changed = true; changed;) {
    changed = false;
    for (size_t k = 0; k < n; k++)
      if (p[k].cls == U_CALLBPF && k + 1 < n && (live[k + 1] & 0x3f & ~ret_live)) { ret_live |= live[k + 1] & 0x3f; changed = true; }
    for (size_t k = n; k-- > 0;) {
      const XeUop& u = p[k];
      auto at = [&](int64_t t) -> uint16_t { return t >= 0 && size_t(t) < n ? live[size_t(t)] : 0; };
      uint16_t out = 0, use = 0, def = 0;
      switch (u.cls) {
        case U_EXIT: case U_FAIL: break;
        case U_JA: out = at(int64_t(u.tgt) + 1); break;
        case U_JMP: out = uint16_t(at(int64_t(u.tgt) + 1) | at(int64_t(k) + 1)); break;
        case U_CALLBPF: out = uint16_t(at(int64_t(k) + u.imm + 1) | at(int64_t(k) + 1)); break;
        default: out = at(int64_t(k) + 1); break;
      }
      switch (u.cls) {
        case U_EXIT: use = uint16_t(bit(0) | ret_live); break;
        case U_CALLBPF: use = 0x3c0; break;  // R6..R9 are cloned for the return
        case U_ALU: use = uint16_t(bit(u.dst) | ((u.fl & UF_REG) ? bit(u.src) : 0)); def = bit(u.dst); break;
        case U_MOVI: case U_LDIMM64: def = bit(u.dst); break;
        case U_MOVR: use = bit(u.src); def = bit(u.dst); break;
        case U_NEG: case U_END: use = def = bit(u.dst); break;
        case U_LDX: use = bit(u.src); if (!(u.fl & UF_BADDST)) def = bit(u.dst); break;
        case U_ST: use = bit(u.dst); break;
        case U_STX: case U_ATOMIC: use = uint16_t(bit(u.dst) | bit(u.src)); break;
        case U_JMP: use = uint16_t(bit(u.dst) | ((u.fl & UF_REG) ? bit(u.src) : 0)); break;
        case U_HELPER: use = 0x3e; break;
        default: break;
      }
      const uint16_t in = uint16_t(use | (out & ~def));
      if (in != live[k]) { live[k] = in; changed = true; }
    }
  }
  for (size_t k = 0; k + 2 < n; k++) {
    XeUop &l = p[k], &a = p[k + 1], &s = p[k + 2];
    if (l.cls != U_LDX || (l.fl & UF_BADDST) || a.cls != U_ALU || s.cls != U_STX) continue;
    const int w = uop_size(l);
    const int rx = l.dst, rb = l.src;
    if ((w != 4 && w != 8) || rx == rb || target[k + 1] || target[k + 2]) continue;
    if (a.dst != rx || (a.x != 0x00 && a.x != 0x10) || ((a.fl & UF_REG) && a.src == rx) || (w == 8 && !(a.fl & UF_WIDE))) continue;
    if (s.dst != rb || s.src != rx || s.tgt != l.tgt || uop_size(s) != w) continue;
    if (k + 3 < n && (live[k + 3] & bit(rx))) continue;
    l.fl |= UF_LIFT;
    s.fl |= UF_LIFT;
    s.imm = (a.fl & UF_REG) ? 0 : a.imm;
    s.x = ((a.fl & UF_REG) ? uint32_t(a.src) + 1u : 0u) | (a.x == 0x10 ? 0x100u : 0u);
  }
}

// ------------------------------------------------------------------ maps
uint32_t next_pow2(uint64_t v) {
  uint32_t p = 16;
  while (p < v) p <<= 1;
  return p;
}

// Slot count of a device hash table: a power of two >= 2 x MaxEntries (at most half full), or, above
// kHashCapMax, kHashCapMax itself (probes run longer above half load; every entry still has a slot:
// MaxEntries <= cap). kHashCapMax + 1 slots take 17 of the 32 big-map handle fields (xe_internal.h
// XE_H_BIG), so one such table leaves room for other big maps beside it.
constexpr uint64_t kHashCapMax = 1ull << 27;
uint64_t hash_cap(uint64_t max_entries) {
  uint64_t mult = 2;
  if (const char* e = xe_tuning_env("XE_HASH_CAPX")) mult = uint64_t(std::max(2, atoi(e)));  // A/B: sparser tables
  uint64_t cap = next_pow2(max_entries * mult);
  if (cap > kHashCapMax && max_entries <= kHashCapMax) cap = kHashCapMax;
  return cap;
}
// big-map handle fields (2^23 slots each, xe_internal.h XE_H_BIG) that n slots / value ids need
uint32_t big_fields(uint64_t n) { return uint32_t((n + (1ull << XE_H_SLOT_BITS) - 1) >> XE_H_SLOT_BITS); }

constexpr uint32_t kAsyncDepth = 3;
constexpr uint32_t kKeyedBackoff = 8;  // order-dependent batches that skip the keyed path after a refusal  // pipelined batches in flight per VM (xe_run_batch_device_async)

struct HostMap {
  xe_map_def def{};
  uint32_t dkind = XE_DM_NONE;
  uint32_t cap = 0, kwords = 0;
  uint32_t big = 0;  // HASH / LRU_HASH past the 23-bit handle slot field: 1 + its first big-map field (XE_H_BIG)
  uint32_t big_nf = 0;  // ... and the number of fields it holds
  // LRU_HASH: the most value ids the pool may have (value handles: 2^23 for a map that is not big, its
  // fields' slots for a big one). Ids are not reused by the in-order replay, so a pool that would pass it
  // is rebuilt compacted from the host mirror instead (ordered_upload)
  uint64_t pool_limit = 1ull << XE_H_SLOT_BITS;
  uint64_t vals_bytes = 0, vals_alloc = 0;
  std::vector<uint8_t> vals;
  std::vector<uint64_t> keys;
  std::vector<uint32_t> state;
  uint32_t count = 0;
  uint8_t* d_vals = nullptr;
  uint64_t* d_keys = nullptr;
  uint32_t* d_state = nullptr;
  uint32_t* d_count = nullptr;
  uint8_t* d_snap = nullptr;
  // rollback points of the pipelined batches in flight: one more than the batches in flight, so the
  // newest batch's epilogue (which stages its successor's) never overwrites the oldest batch's (xe_cancel)
  std::array<uint8_t*, kAsyncDepth + 1> d_asnap{};
  uint8_t* d_rep = nullptr;  // nrep replicas of the value region (zero between runs)
  uint32_t nrep = 1;
  bool nrep_fixed = false;  // nrep was chosen by a run (set_replicas)
  uint64_t rep_stride = 0;
  uint32_t lane = 0;    // width of the map adds of the last run (delta lanes): 0 none, 8 when mixed
  uint32_t wclass = 0;  // width classes of the last run's adds (bit 0: 1 B ... bit 3: 8 B)
  uint32_t ewclass = 0; // width classes of the adds since xe_epoch_begin
  uint8_t* d_ebase = nullptr;  // values at xe_epoch_begin (the epoch's delta base)
  uint32_t live = 0;    // HASH: entry count for replica sizing (host count, refreshed after ordered runs)
  bool host_dirty = true, dev_dirty = false;
  // ordered maps (LRU_HASH / QUEUE / STACK / PERF_EVENT_ARRAY): the host mirror in Go order —
  // LRU: the UsageList (most recently used first) with each key's value; QUEUE / STACK: the Values
  // slice; PERF: the Events slice. An empty `val` is a nil backing (length 0).
  struct Rec {
    std::vector<uint8_t> key;
    bool nil_key = false;
    std::vector<uint8_t> val;
  };
  std::vector<Rec> items;
  bool stack = false;
  uint64_t* d_hdr = nullptr;
  uint32_t* d_link = nullptr;
  uint32_t* d_elen = nullptr;
  uint64_t* d_rec = nullptr;
  uint32_t pool_cap = 0, list_cap = 0;  // capacities of the device copy (grown on XE_FLAG_CAPACITY)
  uint64_t data_cap = 0;
  uint64_t n_vals = 0, n_elen = 0, n_link = 0, n_rec = 0;  // allocated elements of the device arrays
  uint64_t* d_tag = nullptr;  // QUEUE / STACK / PERF: order keys of a parallel run's appends (pool_cap)
  uint64_t n_tag = 0;         // LRU: each value's stamp (xe_interp.h lru_stamp: the UsageList as numbers)
  uint64_t* d_trep = nullptr;   // LRU: trep_r replicas of the stamps (lru_touch in parallel / SPEC passes)
  uint64_t n_trep = 0;
  uint32_t trep_r = 0;
  uint64_t* d_tsnap = nullptr;  // LRU: the stamps at a parallel run's start (its touches are rolled back)
  uint64_t n_tsnap = 0;
  bool links_stale = false;     // LRU: a parallel / keyed run left only stamps (lru_relink rebuilds the links)
  uint8_t* d_vsnap = nullptr; // LRU: the value pool at a parallel run's start (its adds are rolled back)
  uint64_t n_vsnap = 0;
  // LRU: the device rollback point of a keyed or in-order run (lru_dev_snapshot): slot records, links,
  // value lengths, values, stamps, header words — instead of downloading the map into the host mirror
  // before every such run (48 MB over PCIe for a 1M-entry flow table)
  uint64_t* d_rsnap = nullptr; uint64_t n_rsnap = 0;
  uint32_t* d_lsnap = nullptr; uint64_t n_lsnap = 0;
  uint32_t* d_esnap = nullptr; uint64_t n_esnap = 0;
  uint8_t* d_vsnap2 = nullptr; uint64_t n_vsnap2 = 0;
  uint64_t* d_tsnap2 = nullptr; uint64_t n_tsnap2 = 0;
  uint64_t hsnap[8] = {0};
  bool dsnap = false;         // the snapshot is the current run's start
  bool snap_links_stale = false;
  bool ordered() const { return dkind == XE_DM_LRU || dkind == XE_DM_LIST || dkind == XE_DM_PERF; }

  uint64_t* key_at(uint32_t slot) { return keys.data() + uint64_t(slot) * kwords; }
  void pack_key(const void* key, uint64_t* kw) const {
    for (uint32_t w = 0; w < kwords; w++) kw[w] = 0;
    memcpy(kw, key, def.key_size);
  }
  int64_t find(const uint64_t* kw) {
    if (def.key_size == 0) return (state[cap] & XE_SLOT_FULL) ? int64_t(cap) : -1;
    uint32_t idx = uint32_t(xe_hash_words(kw, kwords, def.key_size)) & (cap - 1);
    for (uint32_t p = 0; p < cap; p++) {
      if (!(state[idx] & XE_SLOT_FULL)) return -1;
      if (!memcmp(key_at(idx), kw, kwords * 8)) return idx;
      idx = (idx + 1) & (cap - 1);
    }
    return -1;
  }
  int64_t insert(const uint64_t* kw) {
    if (def.key_size == 0) { state[cap] = XE_SLOT_FULL; count++; return cap; }
    uint32_t idx = uint32_t(xe_hash_words(kw, kwords, def.key_size)) & (cap - 1);
    while (state[idx] & XE_SLOT_FULL) idx = (idx + 1) & (cap - 1);
    memcpy(key_at(idx), kw, kwords * 8);
    state[idx] = XE_SLOT_FULL;
    count++;
    return idx;
  }
  // Keyed runs leave tombstones behind (slot records reserved for a key whose chain did not insert
  // it, xe_interp.h hash_reserve): the device probes run through them; the host mirror is rebuilt
  // without them (same hash, fresh slots) and uploaded again before the next run. True if rebuilt.
  bool drop_tombstones() {
    bool any = false;
    for (uint32_t i = 0; i < cap && !any; i++) any = (state[i] & XE_SLOT_TOMB) != 0;
    if (!any) return false;
    std::vector<uint32_t> full;
    for (uint32_t i = 0; i < cap; i++)
      if (state[i] & XE_SLOT_FULL) full.push_back(i);
    std::vector<uint64_t> k2(full.size() * kwords);
    std::vector<uint8_t> v2(full.size() * def.value_size);
    std::vector<uint32_t> s2(full.size());
    for (size_t j = 0; j < full.size(); j++) {
      memcpy(k2.data() + j * kwords, key_at(full[j]), kwords * 8);
      memcpy(v2.data() + j * def.value_size, vals.data() + uint64_t(full[j]) * def.value_size, def.value_size);
      s2[j] = state[full[j]];
    }
    const uint32_t nil = state[cap];
    std::fill(state.begin(), state.begin() + cap, 0u);
    std::fill(keys.begin(), keys.begin() + uint64_t(cap) * kwords, 0ull);
    std::fill(vals.begin(), vals.begin() + uint64_t(cap) * def.value_size, uint8_t(0));
    count = (nil & XE_SLOT_FULL) ? 1u : 0u;
    for (size_t j = 0; j < full.size(); j++) {
      const int64_t at = insert(k2.data() + j * kwords);
      state[at] = s2[j];
      memcpy(vals.data() + uint64_t(at) * def.value_size, v2.data() + j * def.value_size, def.value_size);
    }
    return true;
  }
  // linear-probing delete with backward shift (keeps probe chains intact without tombstones)
  void erase_slot(uint32_t i) {
    const uint32_t mask = cap - 1;
    if (i == cap) { state[cap] = 0; count--; return; }
    state[i] = 0;
    count--;
    uint32_t j = i;
    for (;;) {
      j = (j + 1) & mask;
      if (!(state[j] & XE_SLOT_FULL)) break;
      uint32_t k = uint32_t(xe_hash_words(key_at(j), kwords, def.key_size)) & mask;
      bool move = (j > i) ? (k <= i || k > j) : (k <= i && k > j);
      if (move) {
        memcpy(key_at(i), key_at(j), kwords * 8);
        memcpy(vals.data() + uint64_t(i) * def.value_size, vals.data() + uint64_t(j) * def.value_size, def.value_size);
        state[i] = state[j];
        state[j] = 0;
        i = j;
      }
    }
  }
};

}  // namespace

struct xe_vm {
  xe_settings settings{};
  std::vector<std::vector<XeUop>> programs{std::vector<XeUop>()};  // index 0 invalid
  int32_t entry = 0;
  std::vector<HostMap> maps{HostMap()};                              // index 0 invalid
  std::string last_error;
  xe_stream_t stream = nullptr;
  // device buffers
  // every program, concatenated (tail calls switch programs): uops + per-program offset / length
  XeUop* d_progs = nullptr;
  int32_t* d_prog_off = nullptr;  // [0..P]: offsets, then [P+1..2P+1]: lengths
  size_t d_progs_n = 0;           // programs uploaded
  size_t d_prog_len = 0;          // length of the entry program
  std::vector<int32_t> prog_off;
  // general lane model arenas (XeGen): parallel launches (one slot per thread of the grid) and the
  // ordered replay (one lane, large capacities, x4 per XE_FLAG_CAPACITY)
  uint8_t* d_arena_par = nullptr;
  uint64_t arena_par_bytes = 0;
  uint8_t* d_arena_seq = nullptr;
  uint64_t arena_seq_bytes = 0;
  uint32_t seq_scale = 1;
  uint64_t* d_ksnap = nullptr;  // HASH slot records + counts before an ordered replay (its rollback point)
  size_t d_ksnap_bytes = 0;
  XeDevMap* d_maps = nullptr;
  size_t d_maps_n = 0;
  std::vector<XeDevMap> dm_uploaded;  // host copy of the device map table (upload only on change)
  unsigned long long* d_aux = nullptr;  // [0..15] stats, [16] flags, [32..] footprints
  // grid sizing: CU count and resident blocks per CU of each kernel (-1 = not queried yet)
  int cus = -1, occ_interp = -1, occ_jit = -1;
  void* occ_jit_fn = nullptr;
  uint32_t occ_nmaps = 0;
  uint32_t last_grid = 0;
  // host-run staging
  void* d_umem = nullptr; size_t d_umem_cap = 0;
  void* d_usnap = nullptr; size_t d_usnap_cap = 0;  // packet bytes before a replayable parallel pass
  void* d_ovl = nullptr; size_t d_ovl_cap = 0;      // descriptor overlap check: sort scratch + flag
  void* d_desc = nullptr; size_t d_desc_cap = 0;
  void* d_res = nullptr; size_t d_res_cap = 0;
  void* d_ver = nullptr; size_t d_ver_cap = 0;
  void* d_regs = nullptr; size_t d_regs_cap = 0;
  std::vector<unsigned long long> last_fp;
  uint32_t last_flags = 0;
  uint32_t last_mode = 0;  // XE_MODE_PARALLEL / XE_MODE_SEQUENTIAL of the last run
  // per-program kernel (JIT engine) for the current entry program
  int32_t jit_idx = -1;
  size_t jit_nmaps = 0;
  size_t jit_nprogs = 0;  // programs of the VM when the kernel was built (tail calls compile them all in)
  void* jit_fn = nullptr;
  bool jit_cyclic = false;
  uint64_t jit_maxpath = 0;  // acyclic kernels: the most instructions a packet can execute
  bool jit_general = false;  // the per-program kernel uses the general lane model (loops, > 57 objects)
  std::string jit_error;
  // its keyed variant (keyed ordered execution), built with it when the program may write map entries
  void* kjit_fn = nullptr;
  void* ljit_fn = nullptr;   // the verdict-only variant (no result / register records)
  bool ljit_ready = false;
  void* sjit_fn = nullptr;   // the scalar one-lane replay (xe_jit.cpp XE_JV_SEQ)
  bool sjit_ready = false;
  bool kjit_ready = false;
  Timer t0, t1, t2;
  // room the ordered maps' device copies keep for one run (elements / events, event bytes), grown
  // ×4 when a run reports XE_FLAG_CAPACITY
  uint64_t ord_slack = 4096, ord_slack_bytes = 1 << 20;
  // pipelined batches (xe_run_batch_device_async): a ring of slots, each with its own statistics /
  // footprint buffer (device + pinned host copy), events and map rollback points; `pending` holds the
  // slots in flight in submission order. d_poison: set by a batch epilogue whose batch must be replayed.
  struct Batch {
    void* d_umem = nullptr; uint64_t umem_len = 0; const void* d_desc = nullptr; uint32_t n = 0;
    void* d_results = nullptr; void* d_verdicts = nullptr; void* d_regs = nullptr;
    xe_stream_t s = nullptr; xe_batch_stats* stats = nullptr;
  };
  struct Slot {
    unsigned long long* d_aux = nullptr;    // zero whenever no batch of the slot is running
    unsigned long long* h_aux = nullptr;
    unsigned long long* h_aux_dev = nullptr;  // h_aux as the batch epilogue writes it
    Timer t0, t1, done;
    Batch b;
    size_t aux_used = 0;
    uint32_t nmaps = 0, grid = 0, engine = 0;
    uint32_t snap = 0;  // index of the batch's rollback point (HostMap::d_asnap)
  };
  std::array<Slot, kAsyncDepth> slots;
  std::vector<uint32_t> pending;
  uint32_t next_slot = 0;
  uint32_t next_snap = 0;  // rollback point of the next pipelined batch
  uint32_t* d_poison = nullptr;
  xe_stream_t cancel_stream = nullptr;  // xe_cancel's write of the poison word (non-blocking stream)
  // rollback point (HostMap::d_asnap index) the last pipelined batch's tail staged for its successor
  // (-1: none valid); anything else that writes device map values invalidates it
  int32_t staged_slot = -1;
  bool draining = false;
  bool delta_base = true;  // the map snapshots are the start of the last batch (false after async batches)
  // shard epoch (xe_epoch_begin): every run since then ORs its footprint here, and the map deltas are
  // taken against the values at the epoch's start (HostMap::d_ebase)
  bool epoch_open = false;
  std::vector<unsigned long long> epoch_fp;
  uint32_t epoch_flags = 0;
  bool epoch_seq = false;
  // keyed ordered execution (xe_internal.h XeKeyed): device buffers, grown on demand; keyed_hint: the
  // last batch needed it, so the next one starts with the SPEC pass instead of a plain parallel run
  XeKeyed kd{};
  uint8_t* d_skip = nullptr;
  uint32_t* d_ksmall = nullptr;  // XE_KS_WORDS counters (xe_internal.h layout)
  uint64_t keyed_n = 0;          // packets the per-packet arrays hold
  uint32_t keyed_dcap = 0, keyed_kw = 0;  // keyed_dcap: the D block's allocated capacity (K.dcap: in use)
  uint32_t keyed_dnext = 0;      // D table size for the next keyed batch (from the last one's D size)
  void* d_ksort = nullptr;
  size_t d_ksort_cap = 0;
  bool keyed_hint = false;
  bool keyed_hint_set = false;  // the first batch's hint was derived from the program (lru_update_sites)
  // after the keyed path refused a batch, the next kKeyedBackoff order-dependent batches go straight to
  // the replay (a program whose batches keep refusing does not pay the SPEC pass every time)
  uint32_t keyed_backoff = 0;
  // parallel list operations (XeListRun): the run's record, the count pass's per-packet flags and their
  // prefix sum (pop ranks)
  XeListRun* d_listrun = nullptr;
  uint32_t* d_popflag = nullptr;
  uint32_t* d_popbase = nullptr;   // XE_POP_SLOTS x pop_n ranks
  uint32_t* d_popused = nullptr;   // the per-slot pop counts the ranks were made from
  size_t pop_n = 0;
  uint32_t seg_depth = 0;           // nesting of packet-order segments (xe_run_batch_device)
  // instruction trace (xe_trace_config): the traced packets (sorted), records kept per packet, device
  // copies (records, per-packet counts)
  std::vector<uint32_t> trace_pk;
  uint32_t trace_max = 0;
  uint32_t* d_trace_pk = nullptr;
  xe_trace_rec* d_trace = nullptr;
  uint32_t* d_trace_cnt = nullptr;
  // helper table (xe_set_helper): host functions and nil entries; the request mailbox (pinned host
  // memory, allocated with the first host function) and its device-visible address
  uint64_t host_helpers[3] = {0, 0, 0};
  uint64_t nil_helpers[3] = {0, 0, 0};
  XeHostCall* h_hostcall = nullptr;
  XeHostCall* d_hostcall = nullptr;
  // ordered maps: after a parallel try of a batch had to be replayed in order, the next kKeyedBackoff
  // batches replay straight away; scratch of the append ordering (XeAppendArgs)
  uint32_t ord_backoff = 0;
  void* d_app = nullptr; size_t d_app_cap = 0;
  void* d_app_sort = nullptr; size_t d_app_sort_cap = 0;
  void* d_relink = nullptr; size_t d_relink_cap = 0;  // lru_relink: sort keys / values + scratch
  uint64_t lru_epoch = 0;  // runs so far: LRU stamps carry it in their top bits (header word 5)
  uint32_t sched = 0;  // chunk -> wave schedule permutation of the parallel passes (xe_debug_set_schedule)
};
// ---- keyed ordered execution buffers (XeKeyed), sized for n packets
static void keyed_free(xe_vm* vm) {
  XeKeyed& K = vm->kd;
  dev_free(K.klog); dev_free(K.kcnt); dev_free(K.dkey); dev_free(K.dkid); dev_free(K.dcomp); dev_free(K.ikey);
  dev_free(K.cstart);
  dev_free(K.dfirst); dev_free(K.dvict); dev_free(K.ekey); dev_free(K.ekey2); dev_free(K.eval); dev_free(K.eval2);
  dev_free(K.ckey); dev_free(K.okey); dev_free(K.order); dev_free(K.iota);
  dev_free(vm->d_skip); dev_free(vm->d_ksmall); dev_free(vm->d_ksort);
  K = XeKeyed{};
  vm->d_skip = nullptr; vm->d_ksmall = nullptr; vm->d_ksort = nullptr;
  vm->d_ksort_cap = 0;
  vm->keyed_n = 0;
  vm->keyed_dcap = vm->keyed_kw = 0;
}
// Per-packet arrays for n packets; the D table with dcap slots (its own size: it is probed at random by
// every keyed access, so it is kept near the live D size — cache-resident — rather than 2n).
static int keyed_alloc(xe_vm* vm, uint32_t n, uint32_t dcap) {
  uint32_t kw = 1;  // dkey entry: map word + the longest HASH key
  for (size_t i = 1; i < vm->maps.size(); i++)
    if (vm->maps[i].dkind == XE_DM_HASH || vm->maps[i].dkind == XE_DM_LRU) kw = std::max(kw, 1 + vm->maps[i].kwords);
  XeKeyed& K = vm->kd;
  if (vm->keyed_n < n || !vm->d_ksmall || vm->keyed_kw < kw) {
    dev_free(K.klog); dev_free(K.kcnt); dev_free(K.ckey); dev_free(K.okey); dev_free(K.order); dev_free(K.iota);
    dev_free(K.ikey); dev_free(vm->d_skip); dev_free(vm->d_ksmall);
    K.klog = K.ikey = nullptr; K.kcnt = K.ckey = K.okey = K.order = K.iota = nullptr;
    vm->d_skip = nullptr; vm->d_ksmall = nullptr;
    vm->keyed_n = 0;
    vm->keyed_dcap = 0;  // the D block is sized with the same key width
    const uint64_t np = std::max<uint64_t>(n, 64);
    if (dev_alloc((void**)&K.klog, np * XE_KLOG * 8) || dev_alloc((void**)&K.kcnt, np * 4) ||
        dev_alloc((void**)&K.ikey, np * XE_KINS * kw * 8) ||
        dev_alloc((void**)&K.ckey, np * 4) || dev_alloc((void**)&K.okey, np * 4) || dev_alloc((void**)&K.order, np * 4) ||
        dev_alloc((void**)&K.iota, np * 4) || dev_alloc((void**)&vm->d_skip, np) ||
        dev_alloc((void**)&vm->d_ksmall, XE_KS_WORDS * 4)) {
      keyed_free(vm);
      return -1;
    }
    vm->keyed_n = np;
    K.dcount = vm->d_ksmall + XE_KS_DCOUNT;
    K.dins = vm->d_ksmall + XE_KS_DINS;
    K.err = vm->d_ksmall + XE_KS_ERR;
    K.changed = vm->d_ksmall + XE_KS_CHANGED;
    K.counts = vm->d_ksmall + XE_KS_NO;
    K.cins = vm->d_ksmall + XE_KS_CINS;
  }
  // the D block only grows: a stream that learns fewer keys per batch runs a smaller table inside the
  // allocation it has (reallocating as the table shrank cost a synchronous free + alloc, ~1.8 ms, in
  // the middle of the stream's second keyed batch)
  if (vm->keyed_dcap < dcap || vm->keyed_kw < kw) {
    dev_free(K.dkey); dev_free(K.dkid); dev_free(K.dcomp); dev_free(K.cstart);
    dev_free(K.dfirst); dev_free(K.dvict); dev_free(K.ekey); dev_free(K.ekey2); dev_free(K.eval); dev_free(K.eval2);
    K.dkey = nullptr; K.dkid = nullptr; K.dcomp = K.cstart = nullptr;
    K.dfirst = K.dvict = K.eval = K.eval2 = nullptr; K.ekey = K.ekey2 = nullptr;
    vm->keyed_dcap = 0;
    if (dev_alloc((void**)&K.dkey, uint64_t(dcap) * kw * 8) || dev_alloc((void**)&K.dkid, uint64_t(dcap) * 8) ||
        dev_alloc((void**)&K.dcomp, uint64_t(dcap) * 4) || dev_alloc((void**)&K.cstart, uint64_t(dcap) * 4) ||
        dev_alloc((void**)&K.dfirst, uint64_t(dcap) * 4) || dev_alloc((void**)&K.dvict, uint64_t(dcap) * 4) ||
        dev_alloc((void**)&K.ekey, uint64_t(dcap) * 8) || dev_alloc((void**)&K.ekey2, uint64_t(dcap) * 8) ||
        dev_alloc((void**)&K.eval, uint64_t(dcap) * 4) || dev_alloc((void**)&K.eval2, uint64_t(dcap) * 4)) {
      keyed_free(vm);
      return -1;
    }
    vm->keyed_dcap = dcap;
    vm->keyed_kw = kw;
  }
  K.kw = vm->keyed_kw;
  K.dcap = dcap;
  return 0;
}

namespace {

constexpr uint32_t kRep = 64;                  // statistics / footprint replicas
constexpr uint32_t kRepWords = 16 + 2 * 64;      // per replica: stats + (read, atomic) per map
constexpr size_t kAuxWords = 16 + size_t(kRep) * kRepWords;
constexpr uint64_t kTailMapBytes = 8 * XE_TAIL_MAP_WORDS;  // value regions the batch epilogue folds / snapshots

int fail(xe_vm* vm, int rc, const std::string& msg) {
  if (vm) vm->last_error = msg;
  return rc;
}

int ensure_buf(void** p, size_t* cap, size_t need) {
  if (*cap >= need && *p) return 0;
  dev_free(*p);
  *p = nullptr;
  size_t c = std::max<size_t>(need, 256);
  if (dev_alloc(p, c)) { *cap = 0; return -1; }
  *cap = c;
  return 0;
}

// Replicas of the value region for deferred 8-byte adds (XeDevMap::rep): enough to spread a hot
// counter's atomics, bounded in memory (HBM is plentiful, but every run folds all replicas).
// Replicas of a value region spread contended map adds over nrep copies (wave % nrep), folded into
// the region after the run. Chosen per run from the live bytes (ARRAY: the region; HASH: entries x
// value size), bounded so the fold reads at most ~160 MB. Measured: C3 (64K Zipf-hot flows in a
// 1M-entry table, a 32 MB + 16 B value region) needs >= 4 (1 replica: 8.2 ms, 2: 1.1-4.0 ms from run
// to run, 4: 1.08 ms, 16: 1.05-1.09 ms over 6 VM placements); C5 (1M uniform flows) is fastest with
// none (3.45 ms; each doubling costs ~5 %). The bound once sat at exactly 128 MB, which the region's
// extra empty-key slot pushed C3 past (2 replicas, the bimodal case).
// HASH maps fold only their used slots (fold_map), so their bound is on the live bytes: C3's 64K hot
// flows get 16 replicas (4 had a slow mode in 3 of 10 fresh processes: 2.13 ms against 1.0 ms,
// profiles/r3/c3_modes.json); an ARRAY folds its whole region.
// the fold reads the live bytes of every replica; the replicas themselves span the whole region (a
// sparse HASH table's too), so their memory is bounded separately (C3: 16 x 32 MB)
bool nrep_bounded(uint32_t want, uint64_t live, uint64_t vals_alloc, bool hash) {
  return uint64_t(want) * (hash ? live : vals_alloc) <= (160ull << 20) && uint64_t(want) * vals_alloc <= (1ull << 30);
}

uint32_t choose_nrep(uint64_t live, uint64_t vals_alloc, bool hash) {
  if (const char* e = xe_tuning_env("XE_NREP")) return uint32_t(std::min(16, std::max(1, atoi(e))));
  uint32_t want = live <= (2ull << 20) ? 16u : live <= (8ull << 20) ? 4u : 1u;
  while (want > 1 && !nrep_bounded(want, live, vals_alloc, hash)) want >>= 1;
  return want;
}

// vals += the replicas (replicas := 0); a HASH map only over the slots that hold or held an entry
int fold_map(HostMap& m, xe_stream_t s) {
  const bool hash = m.dkind == XE_DM_HASH && m.def.value_size > 0;
  const bool lru = m.dkind == XE_DM_LRU;
  const uint64_t words = lru ? (uint64_t(m.pool_cap) * m.def.value_size + 7) / 8 : m.vals_alloc / 8;
  // an LRU pool is folded only over the value ids handed out so far (its header word 3, on the device)
  return launch_rep_fold(m.d_vals, m.d_rep, m.rep_stride / 8, m.nrep, words, hash ? m.d_keys : nullptr,
                         hash ? xe_hash_rwords(m.kwords) : 0, hash || lru ? m.def.value_size : 8, m.cap,
                         lru ? (const void*)m.d_hdr : nullptr, s);
}

int map_alloc_device(HostMap& m) {
  if (m.ordered()) return 0;  // sized at upload (ordered_upload)
  if (dev_alloc((void**)&m.d_vals, m.vals_alloc)) return -1;
  if (dev_alloc((void**)&m.d_snap, m.vals_alloc)) return -1;
  m.nrep = 1;  // replicas are sized per run (set_replicas)
  m.nrep_fixed = false;
  m.rep_stride = (m.vals_alloc + 255) & ~uint64_t(255);
  if (const char* e = xe_tuning_env("XE_REP_SKEW")) m.rep_stride = ((m.vals_alloc + 4095) & ~uint64_t(4095)) + uint64_t(atoll(e));
  if (m.dkind == XE_DM_HASH) {
    if (dev_alloc((void**)&m.d_keys, size_t(m.cap + 1) * xe_hash_rwords(m.kwords) * 8)) return -1;
    if (dev_alloc((void**)&m.d_count, 8)) return -1;
  }
  return 0;
}

void map_free_device(HostMap& m) {
  for (auto& p : m.d_asnap) { dev_free(p); p = nullptr; }
  dev_free(m.d_ebase);
  m.d_ebase = nullptr;
  dev_free(m.d_vals); dev_free(m.d_snap); dev_free(m.d_keys); dev_free(m.d_state); dev_free(m.d_count); dev_free(m.d_rep);
  m.d_vals = m.d_snap = nullptr; m.d_keys = nullptr; m.d_state = m.d_count = nullptr; m.d_rep = nullptr;
  dev_free(m.d_hdr); dev_free(m.d_link); dev_free(m.d_elen); dev_free(m.d_rec);
  m.d_hdr = nullptr; m.d_link = nullptr; m.d_elen = nullptr; m.d_rec = nullptr;
  m.pool_cap = m.list_cap = 0;
  m.data_cap = 0;
  m.n_vals = m.n_elen = m.n_link = m.n_rec = 0;
  dev_free(m.d_tag);
  m.d_tag = nullptr;
  m.n_tag = 0;
  dev_free(m.d_trep);
  m.d_trep = nullptr;
  m.n_trep = 0;
  m.trep_r = 0;
  dev_free(m.d_vsnap);
  m.d_vsnap = nullptr;
  m.n_vsnap = 0;
  dev_free(m.d_tsnap);
  m.d_tsnap = nullptr;
  m.n_tsnap = 0;
  dev_free(m.d_rsnap); dev_free(m.d_lsnap); dev_free(m.d_esnap); dev_free(m.d_vsnap2); dev_free(m.d_tsnap2);
  m.d_rsnap = nullptr; m.d_lsnap = nullptr; m.d_esnap = nullptr; m.d_vsnap2 = nullptr; m.d_tsnap2 = nullptr;
  m.n_rsnap = m.n_lsnap = m.n_esnap = m.n_vsnap2 = m.n_tsnap2 = 0;
  m.dsnap = false;
  m.links_stale = false;
}

// Ordered maps on the device (xe_interp.h, general model; XeDevMap comment): rebuilt from the host
// mirror with room for `slack` more elements / events (and slack_bytes more event bytes).
int ordered_upload(xe_vm* vm, HostMap& m, uint64_t slack, uint64_t slack_bytes);
int ordered_download(xe_vm* vm, HostMap& m);

// The device map table (XeDevMap per map) from the host maps; uploaded when it changed.
int upload_map_table(xe_vm* vm, xe_stream_t s) {
  std::vector<XeDevMap> dm(vm->maps.size());
  memset(dm.data(), 0, dm.size() * sizeof(XeDevMap));
  for (size_t i = 1; i < vm->maps.size(); i++) {
    HostMap& m = vm->maps[i];
    XeDevMap& d = dm[i];
    d.kind = m.dkind;
    d.btype = m.def.type;
    d.key_size = m.def.key_size;
    d.value_size = m.def.value_size;
    d.max_entries = m.def.max_entries;
    d.big = m.big;
    d.vals_bytes = m.vals_bytes;
    d.vals = m.d_vals;
    d.keys = m.d_keys;
    d.state = m.d_state;
    d.count = m.d_count;
    d.cap = m.cap;
    d.kwords = m.kwords;
    d.rwords = (m.dkind == XE_DM_HASH || m.dkind == XE_DM_LRU) ? xe_hash_rwords(m.kwords) : 0;
    d.rep = m.d_rep;
    d.rep_stride = m.rep_stride;
    d.nrep = m.nrep;
    d.hdr = m.d_hdr;
    d.link = m.d_link;
    d.elen = m.d_elen;
    d.rec = m.d_rec;  // PERF: event records; LRU: the one-lane replay's order log (lru_log_build)
    d.pool_cap = m.pool_cap;
    d.list_cap = m.list_cap;
    if (m.dkind == XE_DM_LRU) {  // the stamp replicas (xe_interp.h lru_touch)
      d.state = (uint32_t*)m.d_trep;
      d.list_cap = m.trep_r;
    }
    d.data_cap = m.data_cap;
    d.tag = m.d_tag;
  }
  if (vm->d_maps_n < dm.size()) {
    dev_free(vm->d_maps);
    vm->d_maps = nullptr;
    if (dev_alloc((void**)&vm->d_maps, dm.size() * sizeof(XeDevMap))) return fail(vm, XE_ERR_DEVICE, "device alloc (maps)");
    vm->d_maps_n = dm.size();
  }
  if (vm->dm_uploaded.size() != dm.size() || memcmp(vm->dm_uploaded.data(), dm.data(), dm.size() * sizeof(XeDevMap))) {
    if (h2d(vm->d_maps, dm.data(), dm.size() * sizeof(XeDevMap), s) || dsync(s))
      return fail(vm, XE_ERR_DEVICE, "map table upload");
    vm->dm_uploaded = dm;
  }
  return XE_OK;
}

int map_upload(xe_vm* vm, HostMap& m) {
  if (m.ordered()) return ordered_upload(vm, m, vm->ord_slack, vm->ord_slack_bytes);
  if (h2d(m.d_vals, m.vals.data(), m.vals_alloc, vm->stream)) return -1;
  // the delta base is the uploaded state until a run takes its own snapshot
  if (h2d(m.d_snap, m.vals.data(), m.vals_alloc, vm->stream)) return -1;
  if (m.dkind == XE_DM_HASH) {
    // interleave state and key words into the device slot records
    const uint32_t rw = xe_hash_rwords(m.kwords);
    std::vector<uint64_t> rec(size_t(m.cap + 1) * rw, 0);
    for (size_t i = 0; i <= m.cap; i++) {
      rec[i * rw] = m.state[i];
      for (uint32_t w = 0; w < m.kwords; w++) rec[i * rw + 1 + w] = m.keys[i * m.kwords + w];
    }
    if (h2d(m.d_keys, rec.data(), rec.size() * 8, vm->stream)) return -1;
    if (dsync(vm->stream)) return -1;  // rec is a host temporary
    if (h2d(m.d_count, &m.count, 4, vm->stream)) return -1;
  }
  if (dsync(vm->stream)) return -1;
  m.host_dirty = false;
  m.live = m.count;
  return 0;
}

int lru_relink(xe_vm* vm, HostMap& m, xe_stream_t s, bool renumber = false) {
  if ((!m.links_stale && !renumber) || m.dkind != XE_DM_LRU) return 0;
  uint64_t hdr[8];
  if (d2h(hdr, m.d_hdr, 64, s) || dsync(s)) return -1;
  size_t bytes = 0;
  if (launch_lru_relink(m.d_tag, m.pool_cap, uint32_t(hdr[2]), m.d_link, m.d_hdr, nullptr, &bytes, 0, s) ||
      ensure_buf(&vm->d_relink, &vm->d_relink_cap, bytes) ||
      launch_lru_relink(m.d_tag, m.pool_cap, uint32_t(hdr[2]), m.d_link, m.d_hdr, vm->d_relink, &bytes, renumber ? 1 : 0, s) ||
      dsync(s))
    return -1;
  m.links_stale = false;
  return 0;
}

template <class T>
int ensure_dev(T** p, uint64_t& have, uint64_t need_elems);

// The one-lane replay's order log of an LRU map (xe_interp.h lru_log_push, in d_rec): room for twice the
// pool, seeded with the live values by stamp, oldest first (the stamps sorted on the device, as lru_relink
// does). 1: the log was (re)allocated and the map table must be uploaded again; 0; -1 on error.
const uint32_t* lru_sorted_ids(const void* scratch, uint32_t pool);
int lru_log_build(xe_vm* vm, HostMap& m, xe_stream_t s) {
  uint64_t cap = 1024;
  while (cap < 2ull * m.pool_cap) cap <<= 1;
  int grown = 0;
  if (m.data_cap < cap) {
    if (ensure_dev(&m.d_rec, m.n_rec, 8 + 2 * cap)) return -1;
    m.data_cap = cap;
    grown = 1;
  }
  size_t bytes = 0;
  if (launch_lru_relink(m.d_tag, m.pool_cap, m.pool_cap, m.d_link, m.d_hdr, nullptr, &bytes, 2, s) ||
      ensure_buf(&vm->d_relink, &vm->d_relink_cap, bytes) ||
      launch_lru_relink(m.d_tag, m.pool_cap, m.pool_cap, m.d_link, m.d_hdr, vm->d_relink, &bytes, 2, s) ||
      launch_lru_log(m.d_tag, m.pool_cap, lru_sorted_ids(vm->d_relink, m.pool_cap), m.d_hdr, m.d_rec, s))
    return -1;
  return grown;
}

// An LRU map's device rollback point (see HostMap::d_rsnap): device-to-device copies of every array the
// map lives in, taken at the start of a keyed or in-order run, so a rollback needs no host mirror
int lru_dev_snapshot(HostMap& m, xe_stream_t s) {
  const uint64_t rw = xe_hash_rwords(m.kwords), rec = uint64_t(m.cap + 1) * rw, pool = m.pool_cap;
  const uint64_t vb = pool * m.def.value_size;
  if (ensure_dev(&m.d_rsnap, m.n_rsnap, rec) || ensure_dev(&m.d_lsnap, m.n_lsnap, 4 * pool) ||
      ensure_dev(&m.d_esnap, m.n_esnap, pool) || ensure_dev(&m.d_vsnap2, m.n_vsnap2, vb) ||
      ensure_dev(&m.d_tsnap2, m.n_tsnap2, pool))
    return -1;
  if (d2d(m.d_rsnap, m.d_keys, rec * 8, s) || (pool && d2d(m.d_lsnap, m.d_link, 16 * pool, s)) ||
      (pool && d2d(m.d_esnap, m.d_elen, 4 * pool, s)) || (vb && d2d(m.d_vsnap2, m.d_vals, vb, s)) ||
      (pool && d2d(m.d_tsnap2, m.d_tag, 8 * pool, s)) || d2h(m.hsnap, m.d_hdr, 64, s) || dsync(s))
    return -1;
  m.dsnap = true;
  m.snap_links_stale = m.links_stale;
  return 0;
}
int lru_dev_restore(HostMap& m, xe_stream_t s) {
  const uint64_t rw = xe_hash_rwords(m.kwords), rec = uint64_t(m.cap + 1) * rw, pool = m.pool_cap;
  const uint64_t vb = pool * m.def.value_size;
  if (d2d(m.d_keys, m.d_rsnap, rec * 8, s) || (pool && d2d(m.d_link, m.d_lsnap, 16 * pool, s)) ||
      (pool && d2d(m.d_elen, m.d_esnap, 4 * pool, s)) || (vb && d2d(m.d_vals, m.d_vsnap2, vb, s)) ||
      (pool && d2d(m.d_tag, m.d_tsnap2, 8 * pool, s)) || h2d(m.d_hdr, m.hsnap, 64, s) || dsync(s))
    return -1;
  m.links_stale = m.snap_links_stale;
  return 0;
}

// where launch_lru_relink leaves the pool's value ids sorted by stamp, most recent first (its scratch:
// sorted stamps, ids in, ids out)
const uint32_t* lru_sorted_ids(const void* scratch, uint32_t pool) {
  return (const uint32_t*)((const uint8_t*)scratch + size_t(pool) * 8) + pool;
}

// The 16-bit run epoch of the LRU stamps (xe_interp.h lru_stamp: epoch << 48) is about to wrap: rewrite
// every map's stamps as their ranks in its UsageList (relinking first where only stamps are current), so
// the next run can start again at epoch 1 and still sort after everything that came before.
constexpr uint64_t kLruEpochMax = 0xffff;
int lru_renumber(xe_vm* vm, xe_stream_t s) {
  for (size_t i = 1; i < vm->maps.size(); i++)
    if (vm->maps[i].dkind == XE_DM_LRU && vm->maps[i].d_tag && lru_relink(vm, vm->maps[i], s, true)) return -1;
  vm->lru_epoch = 0;
  return 0;
}

int map_download(xe_vm* vm, HostMap& m) {
  if (!m.dev_dirty) return 0;
  if (m.ordered()) {
    if (m.dkind == XE_DM_LRU && lru_relink(vm, m, vm->stream)) return -1;
    if (ordered_download(vm, m)) return -1;
    m.dev_dirty = false;
    return 0;
  }
  if (d2h(m.vals.data(), m.d_vals, m.vals_alloc, vm->stream)) return -1;
  if (m.dkind == XE_DM_HASH) {
    const uint32_t rw = xe_hash_rwords(m.kwords);
    std::vector<uint64_t> rec(size_t(m.cap + 1) * rw, 0);
    if (d2h(rec.data(), m.d_keys, rec.size() * 8, vm->stream) || dsync(vm->stream)) return -1;
    for (size_t i = 0; i <= m.cap; i++) {
      m.state[i] = uint32_t(rec[i * rw]);
      for (uint32_t w = 0; w < m.kwords; w++) m.keys[i * m.kwords + w] = rec[i * rw + 1 + w];
    }
    if (d2h(&m.count, m.d_count, 4, vm->stream)) return -1;
  }
  if (dsync(vm->stream)) return -1;
  m.dev_dirty = false;
  m.live = m.count;
  if (m.dkind == XE_DM_HASH && m.drop_tombstones()) m.host_dirty = true;  // the device gets the clean layout
  return 0;
}

// host-side slot of `key` in an open-addressing table of `cap` slots laid out like the device's
// (xe_hash_words, linear probing; the nil key takes slot cap)
uint32_t host_probe(const std::vector<uint64_t>& rec, uint32_t rw, uint32_t cap, const uint64_t* kw, uint32_t kwords,
                    uint32_t key_size) {
  uint32_t idx = uint32_t(xe_hash_words(kw, kwords, key_size)) & (cap - 1);
  while (rec[size_t(idx) * rw] & XE_SLOT_FULL) idx = (idx + 1) & (cap - 1);
  return idx;
}

template <class T>
int ensure_dev(T** p, uint64_t& have, uint64_t need_elems) {  // grow-only device array
  if (*p && have >= need_elems) return 0;
  dev_free(*p);
  *p = nullptr;
  if (dev_alloc((void**)p, size_t(std::max<uint64_t>(need_elems, 1)) * sizeof(T))) { have = 0; return -1; }
  have = need_elems;
  return 0;
}

int ordered_upload(xe_vm* vm, HostMap& m, uint64_t slack, uint64_t slack_bytes) {
  const uint64_t n = m.items.size();
  const uint32_t vs = m.def.value_size;
  xe_stream_t st = vm->stream;
  std::vector<uint64_t> hdr(8, 0);
  if (m.dkind == XE_DM_PERF) {
    std::vector<uint64_t> rec(2 * (n + slack), 0);
    uint64_t used = 0;
    for (uint64_t i = 0; i < n; i++) { rec[2 * i] = used; rec[2 * i + 1] = m.items[i].val.size(); used += (m.items[i].val.size() + 7) & ~7ull; }
    std::vector<uint8_t> data(std::max<uint64_t>(used, 8), 0);
    for (uint64_t i = 0; i < n; i++) if (!m.items[i].val.empty()) memcpy(&data[rec[2 * i]], m.items[i].val.data(), m.items[i].val.size());
    if (ensure_dev(&m.d_rec, m.n_rec, 2 * (n + slack))) return -1;
    if (ensure_dev(&m.d_vals, m.n_vals, used + slack_bytes + 8)) return -1;
    m.pool_cap = uint32_t(n + slack);
    m.data_cap = used + slack_bytes;
    hdr[0] = n; hdr[1] = used;
    if (h2d(m.d_rec, rec.data(), rec.size() * 8, st) || h2d(m.d_vals, data.data(), data.size(), st)) return -1;
  } else {
    // An LRU_HASH's value pool starts with room for MaxEntries values (up to 256 MB of them): a batch that
    // learns many flows then finds its value ids instead of growing the pool and starting over (a full
    // download / upload of the map and a second SPEC pass: ~50 ms of a 4M-packet C3-LRU batch).
    uint64_t room = 0;
    if (m.dkind == XE_DM_LRU) room = std::min<uint64_t>(m.def.max_entries, (256ull << 20) / std::max<uint32_t>(vs, 1));
    uint64_t pool = std::max(n, room) + slack;
    // an LRU pool never passes the value ids its handles can name (HostMap::pool_limit): this upload is
    // compacted (the mirror's values get ids 0..n-1), and a batch that still runs out fails as one
    // that outgrows the device (xe_interp.h lru_insert XE_EV_CAP) instead of aliasing another map's values
    if (m.dkind == XE_DM_LRU) {
      if (n + 1 > m.pool_limit) return -1;
      pool = std::min(pool, m.pool_limit);
    }
    std::vector<uint8_t> vals(std::max<uint64_t>(pool * vs, 8), 0);
    std::vector<uint32_t> elen(pool, 0);
    for (uint64_t i = 0; i < n; i++) {
      elen[i] = uint32_t(m.items[i].val.size());
      if (elen[i]) memcpy(&vals[i * vs], m.items[i].val.data(), std::min<size_t>(vs, m.items[i].val.size()));
    }
    std::vector<uint32_t> link;
    if (m.dkind == XE_DM_LRU) {
      const uint32_t rw = xe_hash_rwords(m.kwords);
      std::vector<uint64_t> rec(size_t(m.cap + 1) * rw, 0);
      link.assign(4 * pool, XE_NONE);
      for (uint64_t i = 0; i < n; i++) {
        uint32_t slot = m.cap;
        if (!m.items[i].nil_key) {
          uint64_t kw[XE_MAX_KEY / 8] = {0};
          memcpy(kw, m.items[i].key.data(), m.def.key_size);
          slot = host_probe(rec, rw, m.cap, kw, m.kwords, m.def.key_size);
          for (uint32_t w = 0; w < m.kwords; w++) rec[size_t(slot) * rw + 1 + w] = kw[w];
        }
        rec[size_t(slot) * rw] = XE_SLOT_FULL | (i << 32);
        link[4 * i] = i ? uint32_t(i - 1) : XE_NONE;
        link[4 * i + 1] = i + 1 < n ? uint32_t(i + 1) : XE_NONE;
        link[4 * i + 2] = slot;
      }
      if (!m.d_keys && dev_alloc((void**)&m.d_keys, rec.size() * 8)) return -1;
      if (h2d(m.d_keys, rec.data(), rec.size() * 8, st)) return -1;
      hdr[0] = n ? 0 : XE_NONE; hdr[1] = n ? n - 1 : XE_NONE; hdr[2] = n; hdr[3] = n;
      for (uint64_t i = 0; i < n && !hdr[4]; i++)  // a value not value_size long (xe_interp.h bmem_resolve)
        hdr[4] = elen[i] != vs ? 1 : 0;
      hdr[5] = vm->lru_epoch << 48;  // the stamp base of the run in progress (xe_interp.h lru_stamp)
      hdr[6] = 0;
    } else {  // QUEUE / STACK: element i is Values[i]; the list starts at 0
      link.resize(pool);
      for (uint64_t i = 0; i < pool; i++) link[i] = uint32_t(i);
      hdr[0] = 0; hdr[1] = n; hdr[2] = n; hdr[4] = m.stack ? 1 : 0;
      m.list_cap = uint32_t(pool);
    }
    if (ensure_dev(&m.d_vals, m.n_vals, pool * vs + 8) || ensure_dev(&m.d_elen, m.n_elen, pool) ||
        ensure_dev(&m.d_link, m.n_link, link.size()))
      return -1;
    m.pool_cap = uint32_t(pool);
    if (h2d(m.d_vals, vals.data(), vals.size(), st) || h2d(m.d_elen, elen.data(), elen.size() * 4, st) ||
        h2d(m.d_link, link.data(), link.size() * 4, st))
      return -1;
  }
  if (ensure_dev(&m.d_tag, m.n_tag, m.pool_cap)) return -1;
  if (m.dkind == XE_DM_LRU) {
    // replicas of the stamps for the touches of parallel passes (zero between runs): 16, or as many as
    // 256 MB hold; without them a C3-LRU pass took 7.3 ms of same-word atomics on the hot flows' stamps
    // (0.2-0.5 ms for the same pass over a HASH table, profiles/r5/c3lru_keyed_kernel_trace.csv)
    uint32_t r = 16;
    while (r > 1 && uint64_t(r) * m.pool_cap * 8 > (256ull << 20)) r >>= 1;
    if (r > 1 && (ensure_dev(&m.d_trep, m.n_trep, uint64_t(r) * m.pool_cap) ||
                  dmemset(m.d_trep, 0, uint64_t(r) * m.pool_cap * 8, st)))
      return -1;
    m.trep_r = r > 1 ? r : 0;
  }
  if (m.dkind == XE_DM_LRU) {  // stamps in UsageList order (epoch 0: every run's touches are newer)
    std::vector<uint64_t> tag(m.pool_cap, 0);
    for (uint64_t i = 0; i < n; i++) tag[i] = n - i;
    if (h2d(m.d_tag, tag.data(), tag.size() * 8, st) || dsync(st)) return -1;
    m.links_stale = false;
  }
  if (!m.d_hdr && dev_alloc((void**)&m.d_hdr, 8 * 8)) return -1;
  if (h2d(m.d_hdr, hdr.data(), 64, st) || dsync(st)) return -1;
  m.host_dirty = false;
  return 0;
}

int ordered_download(xe_vm* vm, HostMap& m) {
  xe_stream_t st = vm->stream;
  std::vector<uint64_t> hdr(8, 0);
  if (d2h(hdr.data(), m.d_hdr, 64, st) || dsync(st)) return -1;
  const uint32_t vs = m.def.value_size;
  m.items.clear();
  if (m.dkind == XE_DM_PERF) {
    const uint64_t n = hdr[0], used = hdr[1];
    std::vector<uint64_t> rec(2 * n + 2);
    std::vector<uint8_t> data(used + 8);
    if (d2h(rec.data(), m.d_rec, 2 * n * 8, st) || d2h(data.data(), m.d_vals, used, st) || dsync(st)) return -1;
    for (uint64_t i = 0; i < n; i++) {
      HostMap::Rec r;
      r.val.assign(data.begin() + long(rec[2 * i]), data.begin() + long(rec[2 * i] + rec[2 * i + 1]));
      m.items.push_back(std::move(r));
    }
    return 0;
  }
  const uint64_t pool = m.dkind == XE_DM_LRU ? hdr[3] : hdr[2];
  std::vector<uint8_t> vals(pool * vs + 8);
  std::vector<uint32_t> elen(pool + 1);
  if (d2h(vals.data(), m.d_vals, pool * vs, st) || d2h(elen.data(), m.d_elen, pool * 4, st)) return -1;
  if (m.dkind == XE_DM_LRU) {
    const uint32_t rw = xe_hash_rwords(m.kwords);
    std::vector<uint64_t> rec(size_t(m.cap + 1) * rw);
    std::vector<uint32_t> link(4 * pool + 4);
    if (d2h(rec.data(), m.d_keys, rec.size() * 8, st) || d2h(link.data(), m.d_link, 4 * pool * 4, st) || dsync(st)) return -1;
    for (uint32_t v = uint32_t(hdr[0]); v != XE_NONE; v = link[4 * size_t(v) + 1]) {
      HostMap::Rec r;
      const uint32_t slot = link[4 * size_t(v) + 2];
      r.nil_key = slot == m.cap;
      if (!r.nil_key) {
        r.key.resize(m.def.key_size);
        memcpy(r.key.data(), &rec[size_t(slot) * rw + 1], m.def.key_size);
      }
      r.val.assign(vals.begin() + long(size_t(v) * vs), vals.begin() + long(size_t(v) * vs + elen[v]));
      m.items.push_back(std::move(r));
    }
    return 0;
  }
  std::vector<uint32_t> link(m.list_cap + 1);
  if (d2h(link.data(), m.d_link, size_t(m.list_cap) * 4, st) || dsync(st)) return -1;
  const uint64_t head = hdr[0], cnt = hdr[1];
  for (uint64_t i = 0; i < cnt; i++) {
    const uint32_t id = link[m.stack ? i : (head + i) % m.list_cap];
    HostMap::Rec r;
    r.val.assign(vals.begin() + long(size_t(id) * vs), vals.begin() + long(size_t(id) * vs + elen[id]));
    m.items.push_back(std::move(r));
  }
  return 0;
}

// Go semantics of the ordered maps on the host mirror (userspace Map calls): LRU promote / delete
// (maps_hash_lru.go:51-68,163-183)
size_t lru_index(const HostMap& m, const std::vector<uint8_t>& key) {
  for (size_t i = 0; i < m.items.size(); i++)
    if (!m.items[i].nil_key && m.items[i].key == key) return i;
  return m.items.size();
}
void lru_promote_host(HostMap& m, size_t i) {
  if (i == 0 || i >= m.items.size()) return;
  HostMap::Rec r = std::move(m.items[i]);
  m.items.erase(m.items.begin() + long(i));
  m.items.insert(m.items.begin(), std::move(r));
}

HostMap* get_map(xe_vm* vm, int32_t idx) {
  if (!vm || idx < 1 || idx >= int32_t(vm->maps.size())) return nullptr;
  if (!vm->pending.empty() && xe_sync(vm)) return nullptr;  // map state after every pipelined batch
  return &vm->maps[idx];
}

int prepare_run(xe_vm* vm, xe_stream_t s) {
  if (vm->entry < 1 || vm->entry >= int32_t(vm->programs.size()))
    return fail(vm, XE_ERR_INVAL, "no program loaded at PI");
  if (set_device(vm->settings.device)) return fail(vm, XE_ERR_DEVICE, "hipSetDevice failed");
  if (vm->d_progs_n != vm->programs.size() - 1) {  // program table: every program of the VM
    const size_t np = vm->programs.size() - 1;
    std::vector<XeUop> all;
    std::vector<int32_t> tab(2 * (np + 1), 0);
    for (size_t p = 1; p <= np; p++) {
      tab[p] = int32_t(all.size());
      tab[np + 1 + p] = int32_t(vm->programs[p].size());
      all.insert(all.end(), vm->programs[p].begin(), vm->programs[p].end());
    }
    dev_free(vm->d_progs);
    dev_free(vm->d_prog_off);
    vm->d_progs = nullptr;
    vm->d_prog_off = nullptr;
    if (dev_alloc((void**)&vm->d_progs, std::max<size_t>(all.size(), 1) * sizeof(XeUop)) ||
        dev_alloc((void**)&vm->d_prog_off, tab.size() * 4))
      return fail(vm, XE_ERR_DEVICE, "device alloc (programs)");
    if ((!all.empty() && h2d(vm->d_progs, all.data(), all.size() * sizeof(XeUop), vm->stream)) ||
        h2d(vm->d_prog_off, tab.data(), tab.size() * 4, vm->stream) || dsync(vm->stream))
      return fail(vm, XE_ERR_DEVICE, "program upload");
    vm->prog_off = tab;
    vm->d_progs_n = np;
  }
  vm->d_prog_len = vm->programs[vm->entry].size();
  for (size_t i = 1; i < vm->maps.size(); i++) {
    HostMap& m = vm->maps[i];
    if (m.host_dirty) {
      vm->staged_slot = -1;  // the device values change under the staged snapshots
      if (map_upload(vm, m)) return fail(vm, XE_ERR_DEVICE, "map upload");
    }
    // LRU_HASH value pools take replicas like an ARRAY region: a hot flow's adds otherwise meet on one
    // word from every wave (C3-LRU keyed: 5.3 of a 7.5 ms batch were its map adds, profiles/r5/lru_ab.txt)
    const bool lru = m.dkind == XE_DM_LRU;
    const uint64_t region = lru ? ((uint64_t(m.pool_cap) * m.def.value_size + 7) & ~uint64_t(7)) : m.vals_alloc;
    if (lru && ((region + 255) & ~uint64_t(255)) != m.rep_stride) {  // first run, or the pool grew
      dev_free(m.d_rep);
      m.d_rep = nullptr;
      m.nrep = 1;
      m.nrep_fixed = false;
      m.rep_stride = (region + 255) & ~uint64_t(255);  // (read from the descriptor table: no recompile)
    }
    // (an LRU map's live bytes are not tracked on the host: the tier for a small one, bounded by the pool)
    const uint64_t live = m.dkind == XE_DM_HASH ? uint64_t(m.live) * m.def.value_size : lru ? 0 : m.vals_bytes;
    uint32_t want = (m.dkind == XE_DM_ARRAY || m.dkind == XE_DM_HASH || (lru && region))
                        ? choose_nrep(live, region, m.dkind == XE_DM_HASH) : 1u;
    // the replica count is compiled into the per-program kernel: once chosen it stays while its fold stays
    // bounded, so a table that grows over a stream of batches (C3-learn: 1 -> 5 MB live, 16 -> 4 replicas
    // by the tiers) does not recompile mid-stream (a 9 s hiprtc compile in the measured stream)
    if (m.nrep_fixed && want != m.nrep && !xe_tuning_env("XE_NREP") &&
        (m.nrep == 1 || nrep_bounded(m.nrep, live, region, m.dkind == XE_DM_HASH)))
      want = m.nrep;
    m.nrep_fixed = true;
    if (want != m.nrep) {  // replicas are all zero between runs (the fold clears them)
      dev_free(m.d_rep);
      m.d_rep = nullptr;
      const uint32_t had = m.nrep;
      m.nrep = 1;
      // replicas only spread contended adds: when the device cannot hold them, run without
      while (want > 1 && dev_alloc((void**)&m.d_rep, m.rep_stride * want)) {
        m.d_rep = nullptr;
        want >>= 1;
      }
      if (want > 1 && (dmemset(m.d_rep, 0, m.rep_stride * want, vm->stream) || dsync(vm->stream)))
        return fail(vm, XE_ERR_DEVICE, "device memset (map replicas)");
      if (want <= 1) {
        dev_free(m.d_rep);
        m.d_rep = nullptr;
        want = 1;
      }
      m.nrep = want;
      if (m.nrep != had) vm->jit_idx = -1;  // the replica count is compiled into the per-program kernel
    }
    if (xe_tuning_env("XE_PRINT_ALLOC"))  // placement experiments (tuning build only)
      fprintf(stderr, "{\"map\": %zu, \"vals\": \"%p\", \"keys\": \"%p\", \"rep\": \"%p\", \"nrep\": %u, \"rep_stride\": %llu}\n",
              i, (void*)m.d_vals, (void*)m.d_keys, (void*)m.d_rep, m.nrep, (unsigned long long)m.rep_stride);
  }
  if (int rc = upload_map_table(vm, s)) return rc;
  if (!vm->d_aux && dev_alloc((void**)&vm->d_aux, kAuxWords * 8)) return fail(vm, XE_ERR_DEVICE, "device alloc (aux)");
  return XE_OK;
}

// ---- general lane model arena (XeGen, xe_internal.h): interleaved per-lane fields, 256-B aligned
XeGen gen_layout(uint32_t nl, uint32_t nobj, uint32_t nframes, uint32_t nvc, uint32_t nbm, uint64_t nbytes, uint64_t* total) {
  XeGen g{};
  g.nl = nl; g.nobj = nobj; g.nframes = nframes; g.nvc = nvc; g.nbm = nbm; g.nbytes = nbytes;
  g.mark_words = (((nobj + 31) & ~31u) + ((nvc + 31) & ~31u) + ((nbm + 31) & ~31u)) / 32;
  uint64_t at = 0;
  auto field = [&](uint64_t& off, uint64_t bytes_per_lane) {
    off = at;
    at = (at + bytes_per_lane * nl + 255) & ~uint64_t(255);
  };
  field(g.o_ov, 8ull * nobj);
  field(g.o_oh, 4ull * nobj);
  field(g.o_ot, 4ull * nobj);
  field(g.o_ofree, 4ull * nobj);
  field(g.o_mark, 4ull * g.mark_words);
  field(g.o_frm, 2ull * XE_FRAME_SIZE * nframes);
  field(g.o_ctx, 2ull * 24);
  field(g.o_vc, 2ull * XE_FRAME_SIZE * nvc);
  field(g.o_vcinfo, 4ull * nvc);
  field(g.o_vfree, 4ull * nvc);
  field(g.o_bm, 16ull * nbm);
  field(g.o_bfree, 4ull * nbm);
  field(g.o_pres, 4ull * 17 * 8);
  g.o_key = at;
  field(g.o_bytes, nbytes);
  *total = at;
  return g;
}

// Parallel-mode grid: exactly the blocks that are resident at once (persistent waves walking the
// chunks, see parallel_packets), never more than one 64-packet chunk per wave. A second generation of
// blocks would run its full share after the first finishes, and every extra wave adds its per-wave
// flush (map atomics, statistics) to the same few addresses.
// At most 4 blocks (16 waves) per CU even when more would be resident: C2 0.300 -> 0.279 ms at 16 waves
// against 24 (6 blocks), the same floor the bare access pattern shows (tools/sol_c2.hip: 16 waves
// per CU fastest); C3-C5 were already at 16 and lose below it (profiles/r4/grid_ab.json).
constexpr int kMaxBlocksPerCu = 4;
uint32_t grid_blocks(uint32_t n, int per_cu, int cus) {
  uint64_t chunks = (uint64_t(n) + 63) / 64;
  uint64_t blocks = (chunks + 3) / 4;  // 4 waves per 256-thread block
  if (per_cu > kMaxBlocksPerCu) per_cu = kMaxBlocksPerCu;
  uint64_t maxb = (per_cu > 0 && cus > 0) ? uint64_t(per_cu) * uint64_t(cus) : 256ull * 4;
  if (const char* e = xe_tuning_env("XE_MAX_BLOCKS")) maxb = std::max(1ll, atoll(e));
  return uint32_t(std::max<uint64_t>(1, std::min(blocks, maxb)));
}

}  // namespace

extern "C" {

int xe_default_settings(xe_settings* s) {
  if (!s) return XE_ERR_INVAL;
  memset(s, 0, sizeof *s);
  s->stack_frame_size = 256;
  s->max_stack_frames = 8;
  s->max_steps = 1u << 20;
  s->ingress_ifindex = 1;
  s->rx_queue_index = 0;
  s->device = 0;
  s->mode = XE_MODE_AUTO;
  return XE_OK;
}

int xe_create(const xe_settings* s, xe_vm** out) {
  if (!out) return XE_ERR_INVAL;
  xe_vm* vm = new xe_vm();
  if (s) vm->settings = *s;
  else xe_default_settings(&vm->settings);
  if (vm->settings.stack_frame_size == 0) vm->settings.stack_frame_size = 256;
  if (vm->settings.max_stack_frames == 0) vm->settings.max_stack_frames = 8;
  if (vm->settings.max_steps == 0) vm->settings.max_steps = 1u << 20;
  if (vm->settings.stack_frame_size != 256 || vm->settings.max_stack_frames != 8) {
    delete vm;
    return XE_ERR_UNSUPPORTED;  // the device frame layout is fixed to DefaultVMSettings
  }
  if (set_device(vm->settings.device)) { delete vm; return XE_ERR_DEVICE; }
#ifndef XE_HOSTSIM
  if (hipStreamCreateWithFlags(&vm->stream, hipStreamNonBlocking) != hipSuccess) { delete vm; return XE_ERR_DEVICE; }
#endif
  *out = vm;
  return XE_OK;
}

void xe_destroy(xe_vm* vm) {
  if (!vm) return;
  set_device(vm->settings.device);
  for (uint32_t si : vm->pending) (void)vm->slots[si].done.wait();  // no launch may outlive its buffers
  vm->pending.clear();
  for (auto& sl : vm->slots) {
    dev_free(sl.d_aux); host_free(sl.h_aux);
    sl.t0.fini(); sl.t1.fini(); sl.done.fini();
  }
  dev_free(vm->d_poison);
  stream_destroy(vm->cancel_stream);
  dev_free(vm->d_trace_pk); dev_free(vm->d_trace); dev_free(vm->d_trace_cnt);
  dev_free(vm->d_listrun); dev_free(vm->d_popflag); dev_free(vm->d_popbase); dev_free(vm->d_popused);
  host_free(vm->h_hostcall);
  for (auto& m : vm->maps) map_free_device(m);
  dev_free(vm->d_progs); dev_free(vm->d_prog_off); dev_free(vm->d_maps); dev_free(vm->d_aux);
  dev_free(vm->d_arena_par); dev_free(vm->d_arena_seq); dev_free(vm->d_ksnap);
  dev_free(vm->d_umem); dev_free(vm->d_desc); dev_free(vm->d_res); dev_free(vm->d_ver); dev_free(vm->d_regs);
  dev_free(vm->d_usnap); dev_free(vm->d_ovl); dev_free(vm->d_app); dev_free(vm->d_app_sort); dev_free(vm->d_relink);
  keyed_free(vm);
  vm->t0.fini(); vm->t1.fini(); vm->t2.fini();
#ifndef XE_HOSTSIM
  if (vm->stream) (void)hipStreamDestroy(vm->stream);
#endif
  delete vm;
}

const char* xe_last_error(const xe_vm* vm) { return vm ? vm->last_error.c_str() : "null vm"; }

int xe_add_raw_program(xe_vm* vm, const uint64_t* insns, uint32_t n, int32_t* idx) {
  if (!vm || (!insns && n)) return XE_ERR_INVAL;
  if (int rc = xe_sync(vm)) return rc;  // a replay of a pipelined batch must see the VM it was queued on
  std::vector<XeUop> prog;
  std::string err;
  int rc = translate(insns, n, prog, err);
  if (rc) return fail(vm, rc, err);
  lift_rmw(prog);
  vm->programs.push_back(std::move(prog));
  if (idx) *idx = int32_t(vm->programs.size() - 1);
  return XE_OK;
}

int xe_set_entrypoint(xe_vm* vm, int32_t idx) {  // emulator/vm.go:100-108
  if (!vm) return XE_ERR_INVAL;
  if (int rc = xe_sync(vm)) return rc;
  if (idx < 1 || int32_t(vm->programs.size()) <= idx) return fail(vm, XE_ERR_INVAL, "program index out of bounds");
  vm->entry = idx;
  return XE_OK;
}

int xe_add_map(xe_vm* vm, const xe_map_def* def, const void* init, size_t init_len, int32_t* idx) {
  if (!vm || !def) return XE_ERR_INVAL;
  vm->staged_slot = -1;
  if (int rc = xe_sync(vm)) return rc;
  if (vm->maps.size() > XE_H_MAX_MAPS) return fail(vm, XE_ERR_UNSUPPORTED, "at most 63 maps");
  HostMap m;
  m.def = *def;
  switch (def->type) {  // AbstractMapToVM, emulator/maps.go:92-155
    case XE_MAP_ARRAY: case XE_MAP_PERCPU_ARRAY: case XE_MAP_PROG_ARRAY: case XE_MAP_ARRAY_OF_MAPS:
      m.dkind = XE_DM_ARRAY;
      m.vals_bytes = uint64_t(def->value_size) * def->max_entries;
      break;
    case XE_MAP_HASH: case XE_MAP_PERCPU_HASH: case XE_MAP_HASH_OF_MAPS:
      if (def->key_size > XE_MAX_KEY) return fail(vm, XE_ERR_UNSUPPORTED, "device hash maps support keys up to 64 bytes");
      m.dkind = XE_DM_HASH;
      if (def->max_entries > kHashCapMax) return fail(vm, XE_ERR_UNSUPPORTED, "hash map max_entries too large (<= 2^27)");
      m.cap = uint32_t(hash_cap(def->max_entries));
      m.kwords = (def->key_size + 7) / 8;
      m.vals_bytes = uint64_t(m.cap + 1) * def->value_size;
      m.keys.assign(size_t(m.cap + 1) * m.kwords, 0);
      m.state.assign(size_t(m.cap) + 1, 0);
      break;
    case XE_MAP_LRU_HASH: case XE_MAP_LRU_PERCPU_HASH:
      if (def->key_size > XE_MAX_KEY) return fail(vm, XE_ERR_UNSUPPORTED, "device hash maps support keys up to 64 bytes");
      m.dkind = XE_DM_LRU;
      if (def->max_entries > (kHashCapMax >> 1)) return fail(vm, XE_ERR_UNSUPPORTED, "LRU hash map max_entries too large (<= 2^26)");
      m.cap = uint32_t(hash_cap(def->max_entries));
      // value ids: room for MaxEntries live values and as many inserts again before the pool is compacted
      if (def->max_entries >= (1u << (XE_H_SLOT_BITS - 2)))
        m.pool_limit = std::min<uint64_t>(kHashCapMax, uint64_t(big_fields(2ull * def->max_entries + (1u << 20))) << XE_H_SLOT_BITS);
      m.kwords = (def->key_size + 7) / 8;
      break;
    case XE_MAP_QUEUE: case XE_MAP_STACK:
      m.dkind = XE_DM_LIST;
      m.stack = def->type == XE_MAP_STACK;
      break;
    case XE_MAP_PERF_EVENT_ARRAY:
      m.dkind = XE_DM_PERF;
      break;
    default:  // AbstractMapToVM, emulator/maps.go:155
      return fail(vm, XE_ERR_MAPTYPE, "map type not yet implemented");
  }
  {
    // value handles of slots / value ids past 23 bits (an LRU map's pool grows past MaxEntries) take the
    // big-map encoding, which needs map indices below XE_H_BIG (xe_internal.h)
    uint32_t nbig = 0, used = 0;
    for (size_t i = 1; i < vm->maps.size(); i++) {
      nbig += vm->maps[i].big ? 1 : 0;
      used += vm->maps[i].big_nf;
    }
    const uint32_t nf = m.dkind == XE_DM_HASH ? big_fields(uint64_t(m.cap) + 1)
                        : m.dkind == XE_DM_LRU ? big_fields(m.pool_limit) : 0;
    if (nf > 1) {
      if (used + nf > XE_H_BIG_FIELDS)
        return fail(vm, XE_ERR_UNSUPPORTED, "the VM's hash maps above 4M entries need more than 2^28 value handles together");
      if (vm->maps.size() > XE_H_BIG - 1) return fail(vm, XE_ERR_UNSUPPORTED, "a hash map above 4M entries must be among the first 31 maps");
      m.big = used + 1;
      m.big_nf = nf;
    } else if (nbig && vm->maps.size() > XE_H_BIG - 1) {
      return fail(vm, XE_ERR_UNSUPPORTED, "at most 31 maps in a VM with a hash map above 4M entries");
    }
  }
  m.vals_alloc = std::max<uint64_t>(8, (m.vals_bytes + 7) & ~uint64_t(7));
  m.vals.assign(m.vals_alloc, 0);
  if (init && (def->type == XE_MAP_ARRAY || def->type == XE_MAP_PERCPU_ARRAY))
    memcpy(m.vals.data(), init, std::min<uint64_t>(init_len, m.vals_bytes));
  if (set_device(vm->settings.device) || map_alloc_device(m)) {
    map_free_device(m);
    return fail(vm, XE_ERR_DEVICE, "device alloc (map)");
  }
  m.host_dirty = true;
  vm->maps.push_back(std::move(m));
  vm->jit_idx = -1;  // map geometry is compiled into the per-program kernel
  if (idx) *idx = int32_t(vm->maps.size() - 1);
  return XE_OK;
}

int xe_map_lookup(xe_vm* vm, int32_t mi, const void* key, void* value) {
  HostMap* m = get_map(vm, mi);
  if (!m || !key) return XE_ERR_INVAL;
  set_device(vm->settings.device);
  if (map_download(vm, *m)) return fail(vm, XE_ERR_DEVICE, "map download");
  if (m->ordered()) {
    const HostMap::Rec* r = nullptr;
    if (m->dkind == XE_DM_LRU) {  // userspace Lookup promotes too (maps_hash_lru.go:70-91)
      const size_t i = lru_index(*m, std::vector<uint8_t>((const uint8_t*)key, (const uint8_t*)key + m->def.key_size));
      if (i == m->items.size()) return 0;
      lru_promote_host(*m, i);
      m->host_dirty = true;
      r = &m->items[0];
    } else {  // QUEUE / STACK / PERF by index (maps_queue.go:39-58, maps_stack.go:38-58, maps_perf_event_array.go:45-65)
      uint32_t kv;
      memcpy(&kv, key, 4);
      if (kv >= m->items.size()) return 0;
      r = &m->items[m->dkind == XE_DM_LIST && m->stack ? m->items.size() - 1 - kv : kv];
    }
    if (value) {
      const size_t n = m->dkind == XE_DM_PERF ? r->val.size() : m->def.value_size;
      memset(value, 0, n);
      memcpy(value, r->val.data(), std::min(n, r->val.size()));
    }
    return 1;
  }
  if (m->dkind == XE_DM_ARRAY) {
    uint32_t kv; memcpy(&kv, key, 4);
    if (kv >= m->def.max_entries) return 0;
    if (value) memcpy(value, m->vals.data() + uint64_t(kv) * m->def.value_size, m->def.value_size);
    return 1;
  }
  uint64_t kw[XE_MAX_KEY / 8];
  m->pack_key(key, kw);
  int64_t s = m->find(kw);
  if (s < 0) return 0;
  if (value) {
    memset(value, 0, m->def.value_size);
    if (!(m->state[s] & XE_SLOT_VLEN0)) memcpy(value, m->vals.data() + uint64_t(s) * m->def.value_size, m->def.value_size);
  }
  return 1;
}

int xe_map_update(xe_vm* vm, int32_t mi, const void* key, const void* value) {
  HostMap* m = get_map(vm, mi);
  if (!m || !key || !value) return XE_ERR_INVAL;
  set_device(vm->settings.device);
  if (map_download(vm, *m)) return fail(vm, XE_ERR_DEVICE, "map download");
  if (m->dkind == XE_DM_LRU) {  // HashMapLRU.Update, maps_hash_lru.go:93-161
    std::vector<uint8_t> k((const uint8_t*)key, (const uint8_t*)key + m->def.key_size);
    size_t i = lru_index(*m, k);
    if (i == m->items.size()) {
      if (m->items.size() + 1 > m->def.max_entries) {
        if (m->items.empty()) return fail(vm, XE_ERR_NOMEM, "map is full");
        m->items.pop_back();  // evict the least recently used
      }
      HostMap::Rec r;
      r.key = k;
      m->items.push_back(std::move(r));
      i = m->items.size() - 1;
    }
    m->items[i].val.assign((const uint8_t*)value, (const uint8_t*)value + m->def.value_size);
    lru_promote_host(*m, i);
    m->host_dirty = true;
    return XE_OK;
  }
  if (m->ordered()) return fail(vm, XE_ERR_INVAL, "update not available on this map type");
  if (m->dkind == XE_DM_ARRAY) {
    uint32_t kv; memcpy(&kv, key, 4);
    if (kv >= m->def.max_entries) return fail(vm, XE_ERR_INVAL, "key out of range");
    memcpy(m->vals.data() + uint64_t(kv) * m->def.value_size, value, m->def.value_size);
  } else {
    uint64_t kw[XE_MAX_KEY / 8];
    m->pack_key(key, kw);
    int64_t s = m->find(kw);
    if (s < 0) {
      if (uint64_t(m->count) + 1 > m->def.max_entries) return fail(vm, XE_ERR_NOMEM, "map is full");
      s = m->insert(kw);
    }
    m->state[s] &= ~XE_SLOT_VLEN0;
    memcpy(m->vals.data() + uint64_t(s) * m->def.value_size, value, m->def.value_size);
  }
  m->host_dirty = true;
  return XE_OK;
}

int xe_map_update_batch(xe_vm* vm, int32_t mi, const void* keys, const void* values, uint64_t count) {
  HostMap* m = get_map(vm, mi);
  if (!m || (count && (!keys || !values))) return XE_ERR_INVAL;
  const size_t ks = m->dkind == XE_DM_ARRAY ? 4 : m->def.key_size, vs = m->def.value_size;
  if (m->dkind == XE_DM_LRU && count > 1) {
    // The updates one by one leave every updated key ahead of the others, the last updated first, each
    // holding its last value (maps_hash_lru.go:93-161: every Update promotes): built directly when nothing
    // is evicted on the way (the keys already present plus the new ones fit MaxEntries).
    set_device(vm->settings.device);
    if (map_download(vm, *m)) return fail(vm, XE_ERR_DEVICE, "map download");
    std::map<std::vector<uint8_t>, size_t> pos;
    for (size_t i = 0; i < m->items.size(); i++)
      if (!m->items[i].nil_key) pos[m->items[i].key] = i;
    std::map<std::vector<uint8_t>, uint64_t> last;
    for (uint64_t i = 0; i < count; i++) {
      const uint8_t* k = (const uint8_t*)keys + i * ks;
      last[std::vector<uint8_t>(k, k + ks)] = i;
    }
    uint64_t fresh = 0;
    for (const auto& kv : last) fresh += pos.count(kv.first) ? 0 : 1;
    if (m->items.size() + fresh <= m->def.max_entries) {
      std::vector<std::pair<uint64_t, const std::vector<uint8_t>*>> order;
      for (const auto& kv : last) order.push_back({kv.second, &kv.first});
      std::sort(order.begin(), order.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
      std::vector<HostMap::Rec> items;
      items.reserve(m->items.size() + fresh);
      for (const auto& o : order) {
        HostMap::Rec r;
        r.key = *o.second;
        const uint8_t* v = (const uint8_t*)values + o.first * vs;
        r.val.assign(v, v + vs);
        items.push_back(std::move(r));
      }
      for (auto& r : m->items)
        if (r.nil_key || !last.count(r.key)) items.push_back(std::move(r));
      m->items = std::move(items);
      m->host_dirty = true;
      return XE_OK;
    }
  }
  for (uint64_t i = 0; i < count; i++)
    if (int rc = xe_map_update(vm, mi, (const uint8_t*)keys + i * ks, (const uint8_t*)values + i * vs)) return rc;
  return XE_OK;
}

int xe_map_delete(xe_vm* vm, int32_t mi, const void* key) {
  HostMap* m = get_map(vm, mi);
  if (!m || !key || (m->dkind != XE_DM_HASH && m->dkind != XE_DM_LRU)) return XE_ERR_INVAL;
  set_device(vm->settings.device);
  if (map_download(vm, *m)) return fail(vm, XE_ERR_DEVICE, "map download");
  if (m->dkind == XE_DM_LRU) {  // delete, maps_hash_lru.go:163-183
    const size_t i = lru_index(*m, std::vector<uint8_t>((const uint8_t*)key, (const uint8_t*)key + m->def.key_size));
    if (i < m->items.size()) {
      m->items.erase(m->items.begin() + long(i));
      m->host_dirty = true;
    }
    return XE_OK;
  }
  uint64_t kw[XE_MAX_KEY / 8];
  m->pack_key(key, kw);
  int64_t s = m->find(kw);
  if (s >= 0) {
    memset(m->vals.data() + uint64_t(s) * m->def.value_size, 0, m->def.value_size);
    m->erase_slot(uint32_t(s));
    m->host_dirty = true;
  }
  return XE_OK;
}

int xe_map_count(xe_vm* vm, int32_t mi, uint64_t* count) {
  HostMap* m = get_map(vm, mi);
  if (!m || !count) return XE_ERR_INVAL;
  set_device(vm->settings.device);
  if (map_download(vm, *m)) return fail(vm, XE_ERR_DEVICE, "map download");
  *count = m->dkind == XE_DM_ARRAY ? m->def.max_entries : m->ordered() ? m->items.size() : m->count;
  return XE_OK;
}

int xe_map_dump(xe_vm* vm, int32_t mi, void* keys_or_raw, void* values, uint64_t cap, uint64_t* count) {
  HostMap* m = get_map(vm, mi);
  if (!m) return XE_ERR_INVAL;
  set_device(vm->settings.device);
  if (map_download(vm, *m)) return fail(vm, XE_ERR_DEVICE, "map download");
  if (m->dkind == XE_DM_LRU) {  // MA6: (key, value) sorted by key bytes, the nil key first
    if (count) *count = m->items.size();
    if (!keys_or_raw && !values) return XE_OK;
    if (cap < m->items.size()) return fail(vm, XE_ERR_INVAL, "dump buffer too small");
    std::vector<size_t> order(m->items.size());
    for (size_t i = 0; i < order.size(); i++) order[i] = i;
    std::sort(order.begin(), order.end(), [&](size_t a, size_t b) {
      const auto& x = m->items[a];
      const auto& y = m->items[b];
      if (x.nil_key || y.nil_key) return x.nil_key && !y.nil_key;
      return x.key < y.key;
    });
    for (size_t j = 0; j < order.size(); j++) {
      const auto& r = m->items[order[j]];
      if (keys_or_raw) {
        uint8_t* kd = (uint8_t*)keys_or_raw + j * m->def.key_size;
        memset(kd, 0, m->def.key_size);
        if (!r.nil_key) memcpy(kd, r.key.data(), m->def.key_size);
      }
      if (values) {
        uint8_t* vd = (uint8_t*)values + j * m->def.value_size;
        memset(vd, 0, m->def.value_size);
        memcpy(vd, r.val.data(), std::min<size_t>(r.val.size(), m->def.value_size));
      }
    }
    return XE_OK;
  }
  if (m->ordered()) {  // QUEUE / STACK / PERF: xe_map_dump_list
    if (count) *count = m->items.size();
    return XE_OK;
  }
  if (m->dkind == XE_DM_ARRAY) {
    if (count) *count = m->def.max_entries;
    if (keys_or_raw && cap >= m->def.max_entries) memcpy(keys_or_raw, m->vals.data(), m->vals_bytes);
    return XE_OK;
  }
  if (count) *count = m->count;
  if (!keys_or_raw && !values) return XE_OK;
  if (cap < m->count) return fail(vm, XE_ERR_INVAL, "dump buffer too small");
  const uint32_t ks = m->def.key_size, vs = m->def.value_size;
  std::vector<uint32_t> slots;
  slots.reserve(m->count);
  for (uint32_t s = 0; s <= m->cap; s++)
    if (m->state[s] & XE_SLOT_FULL) slots.push_back(s);
  auto keyp = [&](uint32_t s) -> const uint8_t* { return reinterpret_cast<const uint8_t*>(m->key_at(s)); };
  // MA6: sorted by key bytes; the nil/empty key (slot cap) sorts first
  std::sort(slots.begin(), slots.end(), [&](uint32_t a, uint32_t b) {
    if (a == m->cap || b == m->cap) return a == m->cap && b != m->cap;
    return memcmp(keyp(a), keyp(b), ks) < 0;
  });
  for (size_t i = 0; i < slots.size(); i++) {
    uint32_t s = slots[i];
    if (keys_or_raw) {
      uint8_t* kd = (uint8_t*)keys_or_raw + i * ks;
      if (s == m->cap) memset(kd, 0, ks); else memcpy(kd, keyp(s), ks);
    }
    if (values) {
      uint8_t* vd = (uint8_t*)values + i * vs;
      if (m->state[s] & XE_SLOT_VLEN0) memset(vd, 0, vs);
      else memcpy(vd, m->vals.data() + uint64_t(s) * vs, vs);
    }
  }
  return XE_OK;
}

// Can the program write packet memory? A conservative may-point-to analysis over the micro-op CFG:
// per register the bits PKT (may hold a packet pointer), CTX and FRM (ValueMemory-backed pointers),
// plus one flow-insensitive set of what may have been spilled into ValueMemory (stack/ctx hold
// pointer objects, emulator/memory.go:23-30). Packet pointers originate in ctx loads
// (the xdp_md data/data_end fields); map values are ByteMemory and only ever yield scalars.
static bool may_write_packet(const std::vector<XeUop>& prog) {
  enum : uint8_t { T_PKT = 1, T_CTX = 2, T_FRM = 4 };
  const size_t n = prog.size();
  if (!n) return false;
  std::vector<std::array<uint8_t, 11>> in(n);
  std::vector<bool> reach(n, false);
  std::array<uint8_t, 11> entry{};
  entry[1] = T_CTX;
  entry[10] = T_FRM;
  uint8_t spilled = 0;
  for (int round = 0; round < 64; round++) {
    for (auto& r : in) r.fill(0);
    std::fill(reach.begin(), reach.end(), false);
    in[0] = entry;
    reach[0] = true;
    const uint8_t spilled0 = spilled;
    bool changed = true;
    while (changed) {
      changed = false;
      for (size_t pc = 0; pc < n; pc++) {
        if (!reach[pc]) continue;
        const XeUop& u = prog[pc];
        std::array<uint8_t, 11> r = in[pc];
        auto reg = [&](int x) -> uint8_t { return x <= 10 ? r[x] : 0; };
        auto set = [&](int x, uint8_t v) { if (x <= 10) r[x] = v; };
        int succ[2] = {int(pc) + 1, -1};
        std::array<uint8_t, 11> after = {};  // a call's fall-through: the state the callee returns with
        bool call = false;
        switch (u.cls) {
          case U_FAIL: case U_EXIT: succ[0] = -1; break;
          case U_CALLX: return true;  // not analysed: be conservative
          case U_CALLBPF:
            // the callee starts from the caller's registers in a new frame; back after the call, R6..R9
            // are the caller's (inst_exit.go:22-48) and R0..R5 whatever the callee left: anything
            call = true;
            after = r;
            for (int x = 0; x <= 5; x++) after[x] = T_PKT | T_CTX | T_FRM;
            r[10] = T_FRM;
            succ[0] = int(pc) + u.imm + 1;
            succ[1] = int(pc) + 1;
            break;
          case U_JA: succ[0] = u.tgt + 1; break;
          case U_JMP: succ[1] = u.tgt + 1; break;
          case U_MOVI: set(u.dst, 0); break;
          case U_MOVR: set(u.dst, reg(u.src)); break;
          case U_ALU: set(u.dst, uint8_t(reg(u.dst) | ((u.fl & UF_REG) ? reg(u.src) : 0))); break;
          case U_LDX: {
            const uint8_t s = reg(u.src);
            set(u.dst, uint8_t(((s & T_CTX) ? T_PKT : 0) | ((s & (T_CTX | T_FRM)) ? spilled : 0)));
            break;
          }
          case U_ST: case U_STX: case U_ATOMIC:
            if (reg(u.dst) & T_PKT) return true;
            if (u.cls == U_STX && (reg(u.dst) & (T_CTX | T_FRM))) spilled |= reg(u.src);
            break;
          case U_HELPER:
            if (u.imm == 12) return true;                      // tail call: another program runs on
            if (u.imm == 88 && (reg(2) & T_PKT)) return true;  // pop writes the element through R2
            set(0, 0);                                         // R0 := map value pointer or scalar
            break;
          default: break;                   // NOP, NEG, END, LDIMM64 (in place: taint kept)
        }
        for (int k = 0; k < 2; k++) {
          const int t = succ[k];
          if (t < 0 || t >= int(n)) continue;
          std::array<uint8_t, 11> m = in[t];
          const std::array<uint8_t, 11>& src = (call && k == 1) ? after : r;
          for (int x = 0; x <= 10; x++) m[x] |= src[x];
          if (!reach[t] || m != in[t]) { in[t] = m; reach[t] = true; changed = true; }
        }
      }
    }
    if (spilled == spilled0) return false;  // fixed point including the spill set
  }
  return true;
}

// Can the program run as a per-program kernel? Every program can: bpf-to-bpf calls, tail calls (every
// program of the VM compiled in), indirect helper calls and the ordered maps take the kernel's dynamic
// form over the general lane model (xe_jit.cpp generate_dynamic).
static bool jit_possible(const xe_vm* vm) { return vm->entry >= 1 && vm->entry < int32_t(vm->programs.size()); }

// the VM's programs as pointer / length tables (index 0 unused) for the kernel generator
struct ProgTab {
  std::vector<const XeUop*> p;
  std::vector<uint32_t> n;
};
static ProgTab prog_tab(const xe_vm* vm) {
  ProgTab t;
  t.p.assign(vm->programs.size(), nullptr);
  t.n.assign(vm->programs.size(), 0);
  for (size_t q = 1; q < vm->programs.size(); q++) {
    t.p[q] = vm->programs[q].data();
    t.n[q] = uint32_t(vm->programs[q].size());
  }
  return t;
}
static bool has_callbpf(const xe_vm* vm) {
  for (size_t p = 1; p < vm->programs.size(); p++)
    for (const XeUop& u : vm->programs[p])
      if (u.cls == U_CALLBPF) return true;
  return false;
}
// The ordered maps a parallel run can serve: QUEUE / STACK pushes and PERF outputs (appends, put in
// packet order after the run), LRU_HASH lookups (promotions, applied by last touch after the run),
// LRU_HASH updates (keyed chains), and QUEUE / STACK pops, peeks and lookups (list_ops: a count pass
// ranks the pops in packet order). What remains raises XE_FLAG_ORDERED and the batch replays in packet
// order: PERF event lookups, LRU deletes and evictions, a second pop in one packet, a list position that
// depends on a push made earlier in the batch.
static bool ordered_parallel_ok(const xe_vm* vm) {
  // a static screen: indirect helper calls are not analysed (a pop behind one would find no count pass)
  for (size_t p = 1; p < vm->programs.size(); p++)
    for (const XeUop& u : vm->programs[p])
      if (u.cls == U_CALLX) return false;
  return true;
}
// the VM's programs may pop a QUEUE / STACK (the parallel run then starts with the count pass)
static bool may_pop(const xe_vm* vm) {
  for (size_t p = 1; p < vm->programs.size(); p++)
    for (const XeUop& u : vm->programs[p])
      if (u.cls == U_HELPER && u.imm == 88) return true;
  return false;
}
static bool has_list_maps(const xe_vm* vm) {
  for (size_t i = 1; i < vm->maps.size(); i++)
    if (vm->maps[i].dkind == XE_DM_LIST) return true;
  return false;
}
// the ordered maps' header words (counts, next ids, event bytes) at the start of a parallel run, and
// the LRU maps' value pools (a parallel run adds into looked-up values in place)
static int ordered_hdr_read(xe_vm* vm, std::vector<uint64_t>& out, xe_stream_t s, bool snap_pools = true) {
  out.assign(vm->maps.size() * 8, 0);
  for (size_t i = 1; i < vm->maps.size(); i++) {
    HostMap& m = vm->maps[i];
    if (m.ordered() && d2h(&out[i * 8], m.d_hdr, 64, s)) return -1;
    if (snap_pools && m.dkind == XE_DM_LRU) {
      const uint64_t vb = uint64_t(m.pool_cap) * m.def.value_size;
      if (ensure_dev(&m.d_vsnap, m.n_vsnap, vb) || (vb && d2d(m.d_vsnap, m.d_vals, vb, s))) return -1;
      if (ensure_dev(&m.d_tsnap, m.n_tsnap, m.pool_cap) ||
          (m.pool_cap && d2d(m.d_tsnap, m.d_tag, uint64_t(m.pool_cap) * 8, s)))
        return -1;
    }
  }
  return dsync(s);
}
// back to the headers of a parallel run's start; the LRU maps' touches of the run are dropped
static int ordered_hdr_restore(xe_vm* vm, const std::vector<uint64_t>& h, xe_stream_t s) {
  for (size_t i = 1; i < vm->maps.size(); i++) {
    HostMap& m = vm->maps[i];
    if (m.ordered() && h2d(m.d_hdr, &h[i * 8], 64, s)) return -1;
    if (m.dkind == XE_DM_LRU && m.d_tag && m.d_tsnap && m.pool_cap &&
        d2d(m.d_tag, m.d_tsnap, uint64_t(m.pool_cap) * 8, s))
      return -1;
    const uint64_t vb = uint64_t(m.pool_cap) * m.def.value_size;
    if (m.dkind == XE_DM_LRU && vb && d2d(m.d_vals, m.d_vsnap, vb, s)) return -1;
  }
  return dsync(s);
}
// The promotions of a parallel / keyed run's LRU touches: every touch left its stamp (epoch | packet |
// touch count) with an atomic max, so the UsageList is now "the live values by stamp, descending" — in
// packet order every touched key ended up ahead of the untouched ones, the most recently touched first
// (maps_hash_lru.go:51-91 per touch). Nothing to do until something needs the links (lru_relink).
static int lru_finalize(xe_vm*, HostMap& m, xe_stream_t) {
  m.links_stale = true;
  return 0;
}

// Rebuild an LRU map's UsageList links from the stamps on the device: the pool sorted by stamp,
// descending (radix sort), its first `count` values linked in that order (head = most recent). Before
// a one-lane replay (it promotes and evicts through the links) and before the host reads the map.

// put the appends of a parallel run (header words `h0` before it) into packet order
static int ordered_finalize(xe_vm* vm, const std::vector<uint64_t>& h0, uint32_t n, xe_stream_t s) {
  std::vector<uint64_t> h1;
  if (ordered_hdr_read(vm, h1, s, false)) return -1;  // the header words only (no pool snapshot)
  for (size_t i = 1; i < vm->maps.size(); i++) {
    HostMap& m = vm->maps[i];
    if (m.dkind == XE_DM_LRU) {
      if (lru_finalize(vm, m, s)) return -1;
      continue;
    }
    if (!m.ordered()) continue;
    const bool perf = m.dkind == XE_DM_PERF;
    const uint64_t base = perf ? h0[i * 8] : h0[i * 8 + 2];
    const uint64_t k = (perf ? h1[i * 8] : h1[i * 8 + 2]) - base;
    if (!k) continue;
    XeAppendArgs A{};
    const size_t need = size_t(k) * (8 + 8 + 4 + 4 + (perf ? 16 : 0)) + 256;
    if (ensure_buf(&vm->d_app, &vm->d_app_cap, need)) return -1;
    uint8_t* b = (uint8_t*)vm->d_app;
    A.keys_in = (uint64_t*)b; A.keys_out = A.keys_in + k;
    A.rec_tmp = perf ? A.keys_out + k : nullptr;
    A.ids_in = (uint32_t*)(A.keys_out + k + (perf ? 2 * k : 0)); A.ids_out = A.ids_in + k;
    A.tag = m.d_tag; A.rec = m.d_rec; A.link = m.d_link;
    A.base = base; A.k = uint32_t(k); A.perf = perf ? 1 : 0; A.stack = m.stack ? 1 : 0;
    A.head = h0[i * 8]; A.cnt0 = h0[i * 8 + 1]; A.list_cap = m.list_cap;
    // tags: packet index << 16 | append number
    uint32_t end_bit = 17;
    while (end_bit < 64 && (uint64_t(1) << (end_bit - 16)) < uint64_t(n) + 1) end_bit++;
    size_t sb = 0;
    if (launch_append(&A, end_bit, nullptr, &sb, s) || ensure_buf(&vm->d_app_sort, &vm->d_app_sort_cap, sb) ||
        launch_append(&A, end_bit, vm->d_app_sort, &sb, s))
      return -1;
  }
  return dsync(s);
}

// After a parallel pass that ran out of an ordered map's device room (header words h0 before it):
// restore the headers, bring the host mirror to the batch's start and rebuild the device copies with
// room for twice what the pass tried to append. 1: grown, 0: no ordered map was short, < 0: error.
static int ordered_grow(xe_vm* vm, const std::vector<uint64_t>& h0, xe_stream_t s) {
  std::vector<uint64_t> h1;
  // the header words only: the LRU pools' snapshot is the pass's start, which the restore below needs
  if (ordered_hdr_read(vm, h1, s, false)) return -1;
  bool short_room = false;
  uint64_t slack = vm->ord_slack, bytes = vm->ord_slack_bytes;
  for (size_t i = 1; i < vm->maps.size(); i++) {
    const HostMap& m = vm->maps[i];
    if (m.dkind == XE_DM_PERF) {
      const uint64_t ev = h1[i * 8] - h0[i * 8], by = h1[i * 8 + 1] - h0[i * 8 + 1];
      short_room = short_room || h1[i * 8] > m.pool_cap || h1[i * 8 + 1] > m.data_cap;
      slack = std::max<uint64_t>(slack, 2 * ev + 4096);
      bytes = std::max<uint64_t>(bytes, 2 * by + (1 << 20));
    } else if (m.dkind == XE_DM_LIST) {
      const uint64_t k = h1[i * 8 + 2] - h0[i * 8 + 2];
      short_room = short_room || h1[i * 8 + 2] > m.pool_cap || h1[i * 8 + 1] > m.list_cap;
      slack = std::max<uint64_t>(slack, 2 * k + 4096);
    }
  }
  if (!short_room) return 0;
  if (ordered_hdr_restore(vm, h0, s)) return -1;
  vm->ord_slack = slack;
  vm->ord_slack_bytes = bytes;
  for (size_t i = 1; i < vm->maps.size(); i++) {
    HostMap& m = vm->maps[i];
    if (!m.ordered()) continue;
    m.dev_dirty = true;  // the device copy (at the batch's start again) is the current state
    if (map_download(vm, m) || ordered_upload(vm, m, vm->ord_slack, vm->ord_slack_bytes)) return -1;
  }
  return 1;
}

// the entry program calls bpf_map_update_elem and the VM has an LRU_HASH: such an update never runs in
// the plain parallel pass (LRU inserts and updates take the keyed path), and rolling a failed pass back
// rebuilds the ordered maps from the host mirror, so the VM's first batch starts with the keyed path
static bool lru_update_sites(const xe_vm* vm) {
  bool lru = false;
  for (size_t i = 1; i < vm->maps.size(); i++) lru = lru || vm->maps[i].dkind == XE_DM_LRU;
  if (!lru || vm->entry < 1 || size_t(vm->entry) >= vm->programs.size()) return false;
  for (const XeUop& u : vm->programs[size_t(vm->entry)])
    if (u.cls == U_HELPER && u.imm == 2) return true;
  return false;
}

static bool has_ordered_maps(const xe_vm* vm) {
  for (size_t i = 1; i < vm->maps.size(); i++)
    if (vm->maps[i].ordered()) return true;
  return false;
}

// arena for `nl` lanes: parallel capacities are modest (a lane that runs out raises XE_FLAG_CAPACITY
// and the batch is replayed in order), the ordered replay's single lane gets x seq_scale more
static int ensure_arena(xe_vm* vm, bool seq, uint32_t nl, XeGen& g) {
  const bool calls = has_callbpf(vm);
  const uint32_t k = seq ? vm->seq_scale : 1u;
  const uint32_t nobj = seq ? 65536u * k : 256u;
  const uint32_t nframes = calls ? 8u : 1u;
  const uint32_t nvc = calls ? (seq ? 4096u * k : 16u) : 0u;
  const uint32_t nbm = calls ? (seq ? 4096u * k : 16u) : 0u;
  const uint64_t nbytes = calls ? (seq ? (uint64_t(64) << 20) * k : 4096u) : 0u;
  uint64_t total = 0;
  g = gen_layout(nl, nobj, nframes, nvc, nbm, nbytes, &total);
  uint8_t*& buf = seq ? vm->d_arena_seq : vm->d_arena_par;
  uint64_t& have = seq ? vm->arena_seq_bytes : vm->arena_par_bytes;
  if (!buf || have < total) {
    dev_free(buf);
    buf = nullptr;
    have = 0;
    if (dev_alloc((void**)&buf, size_t(total))) return -1;
    have = total;
  }
  g.base = buf;
  return 0;
}

namespace {

// The helper table differs from LinuxHelperFunctions (xe_set_helper) or a trace is configured: both live in
// the interpreter kernel only (xe_interp.h XE_HELPER_TABLE / XE_TRACE).
bool interp_only(const xe_vm* vm) {
  return (vm->host_helpers[0] | vm->host_helpers[1] | vm->host_helpers[2] | vm->nil_helpers[0] | vm->nil_helpers[1] |
          vm->nil_helpers[2]) != 0 ||
         !vm->trace_pk.empty();
}

// Some program of the VM may call a host function (directly, or through CallHelperIndirect): its batches
// run in packet order on one lane, the only place a host function is called.
bool calls_host_helper(const xe_vm* vm) {
  if (!(vm->host_helpers[0] | vm->host_helpers[1] | vm->host_helpers[2])) return false;
  for (size_t q = 1; q < vm->programs.size(); q++)
    for (const XeUop& u : vm->programs[q]) {
      if (u.cls == U_CALLX) return true;
      if (u.cls == U_HELPER && u.imm >= 0 && u.imm < 192 && ((vm->host_helpers[u.imm >> 6] >> (u.imm & 63)) & 1)) return true;
    }
  return false;
}

// launch parameters of a batch (flags / replica records at aux)
XeParams batch_params(xe_vm* vm, void* d_umem, uint64_t umem_len, const void* d_desc, uint32_t n, void* d_results,
                      void* d_verdicts, void* d_regs, unsigned long long* aux) {
  XeParams P{};
  P.progs = vm->d_progs;
  P.prog_off = vm->d_prog_off;
  P.prog_lens = vm->d_prog_off + vm->d_progs_n + 1;
  P.nprogs = uint32_t(vm->d_progs_n);
  P.entry = vm->entry;
  P.prog = vm->d_progs + vm->prog_off[size_t(vm->entry)];
  P.prog_len = int32_t(vm->d_prog_len);
  P.umem = (uint8_t*)d_umem;
  P.umem_len = umem_len;
  P.desc = (const xe_desc*)d_desc;
  P.n = n;
  P.nmaps = uint32_t(vm->maps.size() - 1);
  for (size_t i = 1; i < vm->maps.size(); i++)
    for (uint32_t f = 0; vm->maps[i].big && f < vm->maps[i].big_nf; f++) {
      P.bigmap[vm->maps[i].big - 1 + f] = uint8_t(i);
      P.bigoff[vm->maps[i].big - 1 + f] = uint8_t(f);
    }
  P.results = (xe_result*)d_results;
  P.verdicts = (uint32_t*)d_verdicts;
  P.regs = (xe_regs*)d_regs;
  P.maps = vm->d_maps;
  P.max_steps = vm->settings.max_steps;
  P.ingress = vm->settings.ingress_ifindex;
  P.rxq = vm->settings.rx_queue_index;
  P.flags = reinterpret_cast<uint32_t*>(aux);
  P.rep = aux + 16;
  P.nrep = kRep;
  P.rep_words = 16 + 2 * (P.nmaps + 1);
  P.sched = vm->sched;
  if (!vm->trace_pk.empty()) {
    P.trace_pk = vm->d_trace_pk;
    P.trace = vm->d_trace;
    P.trace_cnt = vm->d_trace_cnt;
    P.trace_npk = uint32_t(vm->trace_pk.size());
    P.trace_max = vm->trace_max;
  }
  for (int w = 0; w < 3; w++) {
    P.host_helpers[w] = vm->host_helpers[w];
    P.nil_helpers[w] = vm->nil_helpers[w];
  }
  P.hostcall = vm->d_hostcall;
  return P;
}

// The kernel a batch runs: the per-program kernel (compiled on first use for this program and map
// geometry) unless the settings or the program need the interpreter.
int select_engine(xe_vm* vm, void*& jit, bool& jit_general) {
  jit = nullptr;
  jit_general = false;
  const uint32_t engine = vm->settings.engine;
  if (engine == XE_ENGINE_JIT && interp_only(vm))
    return fail(vm, XE_ERR_UNSUPPORTED, "a changed helper table or an instruction trace needs the interpreter engine");
#ifndef XE_HOSTSIM
  if (engine != XE_ENGINE_INTERP && jit_possible(vm) && !interp_only(vm)) {
    if (vm->jit_idx != vm->entry || vm->jit_nmaps != vm->maps.size() || vm->jit_nprogs != vm->programs.size()) {
      // the kernel is specialised on the program and the map geometry (xe_jit.cpp)
      const ProgTab t = prog_tab(vm);
      const char* jerr = "";
      vm->jit_fn = xe_jit_get(t.p.data(), t.n.data(), uint32_t(vm->programs.size() - 1), vm->entry, vm->settings.device,
                              vm->dm_uploaded.data(), uint32_t(vm->dm_uploaded.size() - 1), &vm->jit_cyclic,
                              &vm->jit_general, &jerr, 0, &vm->jit_maxpath);
      vm->jit_error = jerr ? jerr : "";
      vm->jit_idx = vm->entry;
      vm->jit_nmaps = vm->maps.size();
      vm->jit_nprogs = vm->programs.size();
      vm->kjit_ready = false;
      vm->kjit_fn = nullptr;
      vm->ljit_ready = false;
      vm->ljit_fn = nullptr;
      vm->sjit_ready = false;
      vm->sjit_fn = nullptr;
    }
    jit = vm->jit_fn;
    jit_general = vm->jit_general;
    // acyclic kernels carry no budget checks: exact only while the budget cannot be reached
    if (jit && !vm->jit_cyclic && vm->settings.max_steps < std::max<uint64_t>(vm->d_prog_len, vm->jit_maxpath)) jit = nullptr;
  }
  if (!jit && engine == XE_ENGINE_JIT) return fail(vm, XE_ERR_DEVICE, "JIT engine unavailable: " + vm->jit_error);
#endif
  return XE_OK;
}

// The keyed variant of the selected per-program kernel (null: the interpreter runs the keyed passes,
// or the variant cannot be built). Built once per kernel, ahead of the batch that first needs it
// (xe_prepare, or the start of a run whose program may write map entries), so no batch's device time
// includes a compile.
void* keyed_kernel(xe_vm* vm, void* jit) {
#ifndef XE_HOSTSIM
  if (!jit) return nullptr;
  if (!vm->kjit_ready) {
    const ProgTab t = prog_tab(vm);
    bool cy = false, ge = false;
    const char* jerr = "";
    vm->kjit_fn = xe_jit_get(t.p.data(), t.n.data(), uint32_t(vm->programs.size() - 1), vm->entry, vm->settings.device,
                             vm->dm_uploaded.data(), uint32_t(vm->dm_uploaded.size() - 1), &cy, &ge, &jerr, 1, nullptr);
    vm->kjit_ready = true;
  }
  return vm->kjit_fn;
#else
  (void)vm; (void)jit;
  return nullptr;
#endif
}

// The scalar replay variant of the selected per-program kernel (xe_jit.cpp XE_JV_SEQ, xe_interp.h
// XE_UNIFORM) for in-order replays of at least kSeqScalarMin packets (a shorter replay costs less than
// the variant's compile); null when the program has none (the general lane model).
constexpr uint32_t kSeqScalarMin = 16384;
void* seq_kernel(xe_vm* vm, void* jit) {
#ifndef XE_HOSTSIM
  if (!jit) return nullptr;
  if (!vm->sjit_ready) {
    const ProgTab t = prog_tab(vm);
    bool cy = false, ge = false;
    const char* jerr = "";
    vm->sjit_fn = xe_jit_get(t.p.data(), t.n.data(), uint32_t(vm->programs.size() - 1), vm->entry, vm->settings.device,
                             vm->dm_uploaded.data(), uint32_t(vm->dm_uploaded.size() - 1), &cy, &ge, &jerr, 3, nullptr);
    vm->sjit_ready = true;
  }
  return vm->sjit_fn;
#else
  (void)vm;
  (void)jit;
  return nullptr;
#endif
}

// The verdict-only variant of the selected per-program kernel (xe_jit.cpp XE_JV_LEAN) for parallel runs
// that ask for no result / register records; the plain kernel when it cannot be built.
void* lean_kernel(xe_vm* vm, void* jit) {
#ifndef XE_HOSTSIM
  if (!jit) return nullptr;
  if (!vm->ljit_ready) {
    const ProgTab t = prog_tab(vm);
    bool cy = false, ge = false;
    const char* jerr = "";
    vm->ljit_fn = xe_jit_get(t.p.data(), t.n.data(), uint32_t(vm->programs.size() - 1), vm->entry, vm->settings.device,
                             vm->dm_uploaded.data(), uint32_t(vm->dm_uploaded.size() - 1), &cy, &ge, &jerr, 2, nullptr);
    vm->ljit_ready = true;
  }
  return vm->ljit_fn ? vm->ljit_fn : jit;
#else
  (void)vm;
  return jit;
#endif
}

bool keyed_candidate(const xe_vm* vm) {
  const auto& prog = vm->programs[vm->entry];
  return vm->settings.mode == XE_MODE_AUTO && xe_jit_may_write_entries(prog.data(), prog.size()) != 0;
}

// parallel-mode grid for the selected kernel (resident blocks; the general model's arena bounds it)
uint32_t parallel_grid(xe_vm* vm, void* jit, bool general, uint32_t n, uint32_t nmaps) {
  if (vm->cus < 0) vm->cus = cu_count(vm->settings.device);
  int& occ = jit ? vm->occ_jit : vm->occ_interp;
  if ((jit && jit != vm->occ_jit_fn) || nmaps != vm->occ_nmaps) {
    vm->occ_jit_fn = jit ? jit : vm->occ_jit_fn;
    vm->occ_nmaps = nmaps;
    vm->occ_jit = vm->occ_interp = -1;
  }
  if (occ < 0) occ = blocks_per_cu(jit, nmaps);
  uint32_t g = grid_blocks(n, occ, vm->cus);
  if (general) g = std::min<uint32_t>(g, 512);  // bounds the per-lane arena
  return g;
}

// sum / OR the per-wave replica records: red[0] flags, [1] steps, [2..9] status histogram,
// [XE_REC_WIDTH0 + 2 + k] width classes, [16 + 2m] / [17 + 2m] read / atomic masks of map m
void reduce_aux(const unsigned long long* aux, uint32_t nmaps, uint32_t rep_words, std::vector<unsigned long long>& red) {
  red.assign(16 + 2 * size_t(nmaps + 1), 0);
  red[0] = aux[0];
  for (uint32_t r = 0; r < kRep; r++) {
    const unsigned long long* rec = aux + 16 + size_t(r) * rep_words;
    red[1] += rec[0];
    for (int k = 0; k < 8; k++) red[2 + k] += rec[1 + k];
    for (int k = 0; k < 4; k++) red[XE_REC_WIDTH0 + 2 + k] |= rec[XE_REC_WIDTH0 + k];
    for (uint32_t w = 0; w < 2 * (nmaps + 1); w++) red[16 + w] |= rec[16 + w];
  }
}

// order-dependent map effects in a parallel run: an ordered write or a lane out of arena, a read of
// a field other lanes add to, or adds of more than one width on a map (a narrow add's carry stops
// at its own top byte)
bool run_conflict(const std::vector<unsigned long long>& red, uint32_t nmaps) {
  bool conflict = (uint32_t(red[0]) & (XE_FLAG_ORDERED | XE_FLAG_CAPACITY)) != 0;
  for (uint32_t m = 1; m <= nmaps && m < 64; m++) {
    if (red[16 + 2 * m] & red[16 + 2 * m + 1]) conflict = true;
    const unsigned wc = unsigned(red[XE_REC_WIDTH0 + 2 + m / 16] >> (4 * (m % 16))) & 15u;
    if (wc & (wc - 1)) conflict = true;
  }
  return conflict;
}

// per-map add widths of the last run (the lanes of the cross-shard deltas)
uint32_t lane_of(unsigned wc) { return wc == 0u ? 0u : wc == 1u ? 1u : wc == 2u ? 2u : wc == 4u ? 4u : 8u; }

void record_widths(xe_vm* vm, const std::vector<unsigned long long>& red, uint32_t nmaps) {
  for (uint32_t m = 1; m <= nmaps && m < 64; m++) {
    const unsigned wc = unsigned(red[XE_REC_WIDTH0 + 2 + m / 16] >> (4 * (m % 16))) & 15u;
    vm->maps[m].wclass = wc;
    vm->maps[m].lane = lane_of(wc);
    vm->maps[m].ewclass |= wc;
  }
}

// the last run's flags, mode and footprint (xe_footprint), ORed into the open shard epoch
void note_run(xe_vm* vm, const std::vector<unsigned long long>& red, uint32_t mode) {
  vm->last_flags = uint32_t(red[0]);
  vm->last_mode = mode;
  vm->last_fp.assign(red.begin() + 16, red.end());
  if (!vm->epoch_open) return;
  vm->epoch_flags |= vm->last_flags;
  vm->epoch_seq = vm->epoch_seq || mode == XE_MODE_SEQUENTIAL || mode == XE_MODE_KEYED;
  if (vm->epoch_fp.size() < vm->last_fp.size()) vm->epoch_fp.resize(vm->last_fp.size(), 0);
  for (size_t i = 0; i < vm->last_fp.size(); i++) vm->epoch_fp[i] |= vm->last_fp[i];
}

}  // namespace

// Packet-order segments (XE_MODE_SEGMENTS): the batch's packets [0, cut), then windows of the rest, as
// batches one after the other (any of them cut again), each through the whole path; statistics summed.
// The failed pass is rolled back first exactly as for the in-order fallback (map values, packets, the
// ordered maps' headers, LRU stamps and values from their snapshots), and each segment takes a new LRU
// epoch, so its stamps order after the segment before it as packet order does. Not with a packet trace
// (it names packets by batch index), and at most kSegDepth cuts (the rest then takes the usual fallback).
constexpr uint32_t kSegMin = 64, kSegDepth = 64;
static bool segments_ok(const xe_vm* vm, const XeParams& P) { return !P.trace && vm->seg_depth < kSegDepth; }
static int run_segments(xe_vm* vm, void* d_umem, uint64_t umem_len, const void* d_desc, uint32_t n, uint32_t cut,
                        void* d_results, void* d_verdicts, void* d_regs, void* stream, xe_batch_stats* stats) {
  // [0, cut) ran exactly in the failed pass; after it, windows that double ([cut, 3 cut), ...), each a
  // batch of its own (cut again inside when it must): the failed pass of a window covers that window,
  // not all that follows, so a batch cut many times costs about one pass over it, not one per cut
  auto at = [](void* p, size_t k) -> void* { return p ? (void*)((uint8_t*)p + k) : nullptr; };
  auto rank = [](uint32_t m) { return m == XE_MODE_SEQUENTIAL ? 3 : m == XE_MODE_KEYED ? 2 : 1; };
  xe_batch_stats acc{};
  acc.mode_used = XE_MODE_PARALLEL;
  vm->seg_depth++;
  int rc = XE_OK;
  uint64_t pos = 0, len = cut;
  while (rc == XE_OK && pos < n) {
    xe_batch_stats b{};
    rc = xe_run_batch_device(vm, d_umem, umem_len, (const uint8_t*)d_desc + size_t(pos) * sizeof(xe_desc), uint32_t(len),
                             at(d_results, size_t(pos) * sizeof(xe_result)), at(d_verdicts, size_t(pos) * 4),
                             at(d_regs, size_t(pos) * sizeof(xe_regs)), stream, &b);
    acc.steps += b.steps;
    for (int k = 0; k < 8; k++) acc.status_count[k] += b.status_count[k];
    if (rank(b.mode_used) > rank(acc.mode_used)) acc.mode_used = b.mode_used;
    acc.kernel_ms += b.kernel_ms;
    acc.total_ms += b.total_ms;
    acc.engine_used = b.engine_used;
    acc.grid_blocks = std::max(acc.grid_blocks, b.grid_blocks);
    pos += len;
    len = std::min<uint64_t>(n - pos, 2 * len);
  }
  vm->seg_depth--;
  if (rc != XE_OK) return rc;
  if (stats) {
    *stats = acc;
    stats->packets = n;
    // the slowest path any segment took; segments that all ran in parallel report XE_MODE_SEGMENTS
    if (stats->mode_used == XE_MODE_PARALLEL) stats->mode_used = XE_MODE_SEGMENTS;
    stats->conflict = 1;
  }
  return XE_OK;
}

int xe_run_batch_device(xe_vm* vm, void* d_umem, uint64_t umem_len, const void* d_desc, uint32_t n,
                        void* d_results, void* d_verdicts, void* d_regs, void* stream, xe_batch_stats* stats) {
  if (!vm) return XE_ERR_INVAL;
  // (tuning build: XE_HOST_TIMING=1 prints host-side marks of the batch, milliseconds since its start)
  const auto tm0 = std::chrono::steady_clock::now();
  auto tmark = [&](const char* what) {
    if (xe_tuning_env("XE_HOST_TIMING"))
      fprintf(stderr, "host %-14s %8.3f ms (n=%u)\n", what,
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tm0).count(), n);
  };
  vm->staged_slot = -1;  // this run writes the maps outside the pipeline
  for (size_t i = 1; i < vm->maps.size(); i++) vm->maps[i].dsnap = false;  // rollback points are per run
  if (stats) memset(stats, 0, sizeof *stats);
  if (int rc = xe_sync(vm)) return rc;  // pipelined batches first: they precede this one
  xe_stream_t s = stream ? (xe_stream_t)stream : vm->stream;
  if (int rc = prepare_run(vm, s)) return rc;
  tmark("prepare_run");
  if (n && (!d_umem || !d_desc)) return fail(vm, XE_ERR_INVAL, "null umem/desc");
  vm->delta_base = true;

  XeParams P = batch_params(vm, d_umem, umem_len, d_desc, n, d_results, d_verdicts, d_regs, vm->d_aux);
  const size_t aux_used = 16 + size_t(kRep) * P.rep_words;
  // LRU stamps of this run sort after every earlier run's (xe_interp.h lru_stamp; header word 5)
  {
    bool lru = false;
    for (size_t i = 1; i < vm->maps.size(); i++) lru = lru || vm->maps[i].dkind == XE_DM_LRU;
    if (lru && vm->lru_epoch >= kLruEpochMax && lru_renumber(vm, s)) return fail(vm, XE_ERR_DEVICE, "LRU renumber");
    const uint64_t e[2] = {lru ? (++vm->lru_epoch) << 48 : 0, 0};  // stamp base, one-lane touch counter
    for (size_t i = 1; i < vm->maps.size(); i++)
      if (vm->maps[i].dkind == XE_DM_LRU && (h2d(vm->maps[i].d_hdr + 5, e, 16, s) || dsync(s)))
        return fail(vm, XE_ERR_DEVICE, "LRU epoch");
  }
  if (P.trace && dmemset(vm->d_trace_cnt, 0, vm->trace_pk.size() * 4, s)) return fail(vm, XE_ERR_DEVICE, "trace reset");
  // host functions are called in packet order only
  const bool hostcalls = calls_host_helper(vm);

  const uint32_t mode = vm->settings.mode;
  void* jit = nullptr;
  bool jit_general = false;
  if (int rc = select_engine(vm, jit, jit_general)) return rc;
  const bool general = !jit || jit_general;  // lanes keep their state in the XeGen arena
  auto launch = [&](const XeParams* p, uint32_t b, uint32_t t) {
    return jit ? launch_jit(jit, p, b, t, s) : launch_interp(p, b, t, s);
  };
  // one prologue launch: snapshot the map values (rollback point for the ordered fallback and base of
  // the shard deltas) and zero the statistics words
  {
    std::vector<const void*> src;
    std::vector<void*> dst;
    std::vector<uint64_t> words;
    for (size_t i = 1; i < vm->maps.size(); i++) {
      HostMap& m = vm->maps[i];
      if (m.ordered()) continue;
      src.push_back(m.d_vals);
      dst.push_back(m.d_snap);
      words.push_back(m.vals_alloc / 8);
    }
    if (launch_prologue(src.data(), dst.data(), words.data(), uint32_t(src.size()), vm->d_aux, aux_used, s))
      return fail(vm, XE_ERR_DEVICE, "prologue");
  }
  // the ordered replay must also start from the original packet bytes
  const bool keep_pkts = mode == XE_MODE_AUTO && umem_len && may_write_packet(vm->programs[vm->entry]);
  if (keep_pkts && (ensure_buf(&vm->d_usnap, &vm->d_usnap_cap, umem_len) || d2d(vm->d_usnap, d_umem, umem_len, s)))
    return fail(vm, XE_ERR_DEVICE, "packet snapshot");
  // A packet-writing program over descriptors whose bytes overlap: in the reference's order a later
  // packet reads what an earlier one wrote, which parallel lanes cannot reproduce; in order straight away.
  bool overlap = false;
  if (keep_pkts && n > 1) {
    size_t need = 0;
    uint32_t flag = 0;
    if (launch_desc_overlap(d_desc, n, umem_len, nullptr, &need, nullptr, s) ||
        ensure_buf(&vm->d_ovl, &vm->d_ovl_cap, need + 256))
      return fail(vm, XE_ERR_DEVICE, "device alloc (descriptor overlap check)");
    uint32_t* d_flag = (uint32_t*)((uint8_t*)vm->d_ovl + ((need + 255) & ~size_t(255)));
    if (launch_desc_overlap(d_desc, n, umem_len, vm->d_ovl, &need, d_flag, s) || d2h(&flag, d_flag, 4, s) || dsync(s))
      return fail(vm, XE_ERR_DEVICE, "descriptor overlap check");
    overlap = flag != 0;
  }
  std::vector<unsigned long long> aux(aux_used);
  std::vector<unsigned long long> red;
  // sum / OR the per-wave replicas: [0] flags, replica r at 16 + r * rep_words
  auto reduce = [&]() { reduce_aux(aux.data(), P.nmaps, P.rep_words, red); };
  auto read_aux = [&]() -> int {
    if (d2h(aux.data(), vm->d_aux, aux_used * 8, s) || dsync(s)) return -1;
    reduce();
    return 0;
  };
  // roll maps and packets back to the run's start
  auto rollback = [&](bool hash_records) -> int {
    for (size_t i = 1; i < vm->maps.size(); i++) {
      HostMap& m = vm->maps[i];
      if (!m.ordered() && d2d(m.d_vals, m.d_snap, m.vals_alloc, s)) return -1;
    }
    if (hash_records) {
      uint64_t off = 0;
      for (size_t i = 1; i < vm->maps.size(); i++) {
        HostMap& m = vm->maps[i];
        if (m.dkind != XE_DM_HASH) continue;
        const uint64_t rb = uint64_t(m.cap + 1) * xe_hash_rwords(m.kwords) * 8;
        if (d2d(m.d_keys, (uint8_t*)vm->d_ksnap + off, rb, s) || d2d(m.d_count, (uint8_t*)vm->d_ksnap + off + rb, 4, s)) return -1;
        off += rb + 8;
      }
      for (size_t i = 1; i < vm->maps.size(); i++) {  // the ordered maps come back from their rollback point:
        HostMap& m = vm->maps[i];                       // an LRU map's device snapshot, the others' host mirror
        if (m.dkind == XE_DM_LRU && m.dsnap) {
          if (lru_dev_restore(m, s)) return -1;
        } else if (m.ordered() && ordered_upload(vm, m, vm->ord_slack, vm->ord_slack_bytes)) {
          return -1;
        }
      }
    }
    if (keep_pkts && d2d(d_umem, vm->d_usnap, umem_len, s)) return -1;
    return dmemset(vm->d_aux, 0, aux_used * 8, s);
  };
  // The exact ordered replay: one lane walks the packets in order. Its arena (and the ordered maps'
  // room) grows x4 and the replay restarts from the rollback point whenever it runs out.
  // rollback point of what the parallel pass never writes: hash slot records (+ counts)
  auto snap_records = [&]() -> int {
    uint64_t kb = 0;
    for (size_t i = 1; i < vm->maps.size(); i++)
      if (vm->maps[i].dkind == XE_DM_HASH) kb += uint64_t(vm->maps[i].cap + 1) * xe_hash_rwords(vm->maps[i].kwords) * 8 + 8;
    if (kb && ensure_buf((void**)&vm->d_ksnap, &vm->d_ksnap_bytes, kb)) return fail(vm, XE_ERR_DEVICE, "device alloc (snapshot)");
    uint64_t off = 0;
    for (size_t i = 1; i < vm->maps.size(); i++) {
      HostMap& m = vm->maps[i];
      if (m.dkind != XE_DM_HASH) continue;
      const uint64_t rb = uint64_t(m.cap + 1) * xe_hash_rwords(m.kwords) * 8;
      if (d2d((uint8_t*)vm->d_ksnap + off, m.d_keys, rb, s) || d2d((uint8_t*)vm->d_ksnap + off + rb, m.d_count, 4, s))
        return fail(vm, XE_ERR_DEVICE, "snapshot");
      off += rb + 8;
    }
    return XE_OK;
  };
  auto sequential = [&](float& ms) -> int {
    // rollback point of what the parallel pass never writes: hash slot records, the ordered maps
    if (int rc = snap_records()) return rc;
    for (size_t i = 1; i < vm->maps.size(); i++) {
      HostMap& m = vm->maps[i];
      if (m.dkind == XE_DM_LRU) {  // rollback point on the device (the replay keeps its own order log)
        if (lru_dev_snapshot(m, s)) return fail(vm, XE_ERR_DEVICE, "LRU snapshot");
      } else if (m.ordered() && map_download(vm, m)) {
        return fail(vm, XE_ERR_DEVICE, "map download");
      }
    }
    // the replay lane's packets are staged 64 at a time by the whole wave unless a packet may write
    // packet bytes a later packet reads (its window must then be fetched after the earlier writes)
    P.seq_prefetch = may_write_packet(vm->programs[vm->entry]) ? 0u : 1u;
    // and run ahead of the lane (per-program kernels; XE_SEQ_PEEK=0 in the tuning build: A/B)
    if (P.seq_prefetch) {
      const char* pk = xe_tuning_env("XE_SEQ_PEEK");
      if (!pk || atoi(pk)) P.seq_prefetch |= 2u;
    }
    for (int attempt = 0;; attempt++) {
      P.mode = XE_MODE_SEQUENTIAL;
      if (general && ensure_arena(vm, true, 1, P.gen)) return fail(vm, XE_ERR_NOMEM, "device alloc (replay arena)");
      bool table = false;  // the LRU maps' order logs from their stamps (the run's start state)
      for (size_t i = 1; i < vm->maps.size(); i++) {
        if (vm->maps[i].dkind != XE_DM_LRU) continue;
        const int r = lru_log_build(vm, vm->maps[i], s);
        if (r < 0) return fail(vm, XE_ERR_DEVICE, "LRU order log");
        table = table || r > 0;
      }
      if (table) {
        if (int rc = upload_map_table(vm, s)) return rc;
        P.maps = vm->d_maps;
      }
      vm->t1.rec(s);
      // a long replay on the scalar variant of the per-program kernel (every lane runs the packet)
      void* sj = (jit && !jit_general && n >= kSeqScalarMin) ? seq_kernel(vm, jit) : nullptr;
      if (sj ? launch_jit(sj, &P, 1, 64, s) : launch(&P, 1, 64)) return fail(vm, XE_ERR_DEVICE, "kernel launch");
      vm->t2.rec(s);
      if (hostcalls && serve_hostcalls(vm->h_hostcall, s)) return fail(vm, XE_ERR_DEVICE, "kernel failed (host helpers)");
      if (read_aux()) return fail(vm, XE_ERR_DEVICE, "kernel failed");
      ms += Timer::ms(vm->t1, vm->t2);
      if (!(red[0] & XE_FLAG_CAPACITY)) {
        for (size_t i = 1; i < vm->maps.size(); i++)  // the replay kept stamps and its log, not the links
          if (vm->maps[i].dkind == XE_DM_LRU) vm->maps[i].links_stale = true;
        return XE_OK;
      }
      if (attempt >= 6) return fail(vm, XE_ERR_NOMEM, "the ordered replay outgrew its device arena");
      vm->seq_scale *= 4;
      vm->ord_slack *= 4;
      vm->ord_slack_bytes *= 4;
      if (rollback(true)) return fail(vm, XE_ERR_DEVICE, "rollback");
      // the ordered maps' room grows with the slack: an LRU map, back at its start state on the device,
      // goes through the host mirror into a larger pool, and that becomes the next attempt's rollback point
      for (size_t i = 1; i < vm->maps.size(); i++) {
        HostMap& m = vm->maps[i];
        if (m.dkind != XE_DM_LRU) continue;
        m.dev_dirty = true;
        if (map_download(vm, m)) return fail(vm, XE_ERR_DEVICE, "map download");
        m.host_dirty = true;
      }
      if (prepare_run(vm, s)) return fail(vm, XE_ERR_DEVICE, "rollback");
      for (size_t i = 1; i < vm->maps.size(); i++)
        if (vm->maps[i].dkind == XE_DM_LRU && lru_dev_snapshot(vm->maps[i], s)) return fail(vm, XE_ERR_DEVICE, "LRU snapshot");
      P.maps = vm->d_maps;
    }
  };

  // fold the 8-byte-add replicas into the value regions (and zero them for the next run)
  auto fold = [&]() -> int {
    for (size_t i = 1; i < vm->maps.size(); i++) {
      HostMap& m = vm->maps[i];
      if (m.nrep > 1 && fold_map(m, s)) return -1;
      if (m.dkind == XE_DM_LRU && m.trep_r > 1 && launch_lru_tag_fold(m.d_tag, m.d_trep, m.pool_cap, m.trep_r, m.d_hdr, s)) return -1;
    }
    return 0;
  };
  const bool ordmaps = has_ordered_maps(vm);
  // Keyed ordered execution (xe_internal.h): the SPEC pass, the build, the parallel pass of the packets
  // on no chain, the chains. Returns 1 when the batch has to take the one-lane replay instead (maps,
  // packets and records rolled back), 0 when done (used: XE_MODE_PARALLEL when no packet wrote a map
  // entry, so the SPEC pass was an ordinary parallel run; else XE_MODE_KEYED), < 0 on error.
  // (tuning build: XE_KEYED_TRACE=1 names why a keyed attempt gave up or started over)
  auto keyed_trace = [&](const char* why) {
    if (xe_tuning_env("XE_KEYED_TRACE")) fprintf(stderr, "keyed: %s (n=%u)\n", why, n);
  };
  auto keyed = [&](uint32_t& used_out) -> int {
    void* kjit = keyed_kernel(vm, jit);  // the per-program kernel's keyed variant
    if (jit && !kjit) return 1;
    auto klaunch = [&](const XeParams* p, uint32_t b) { return kjit ? launch_jit(kjit, p, b, 256, s) : launch_interp(p, b, 256, s); };
    // D table: 4x the last keyed batch's D keys (first time: n / 4), at most 2n (D holds <= n keys)
    uint32_t dmax = 4096, dcap = 4096;
    while (dmax < 2ull * n && dmax < (1u << 30)) dmax <<= 1;
    const uint64_t dwant = vm->keyed_dnext ? vm->keyed_dnext : std::max<uint64_t>(4096, n / 4);
    while (dcap < dwant && dcap < dmax) dcap <<= 1;
    tmark("keyed start");
    if (keyed_alloc(vm, n, dcap)) return fail(vm, XE_ERR_NOMEM, "device alloc (keyed execution)");
    tmark("keyed alloc");
    // ordered maps (LRU_HASH keys, appends): the host mirror holds the batch's start (rollback(true)
    // rebuilds the device copies from it), kh0 their header words / LRU value pools for the cheaper
    // rollbacks before any record was claimed
    std::vector<uint64_t> kh0;
    if (ordmaps) {
      for (size_t i = 1; i < vm->maps.size(); i++) {
        HostMap& m = vm->maps[i];
        if (m.dkind == XE_DM_LRU) {
          if (lru_dev_snapshot(m, s)) return fail(vm, XE_ERR_DEVICE, "LRU snapshot");
        } else if (m.ordered() && map_download(vm, m)) {
          return fail(vm, XE_ERR_DEVICE, "map download");
        }
      }
      tmark("map snapshot");
      if (ordered_hdr_read(vm, kh0, s)) return fail(vm, XE_ERR_DEVICE, "ordered map header");
      tmark("hdr read");
    }
    auto krollback = [&]() -> int {
      if (rollback(false)) return -1;
      return ordmaps ? ordered_hdr_restore(vm, kh0, s) : 0;
    };
    XeKeyed K = vm->kd;
    K.n = n;
    if (dmemset(K.dkid, 0, uint64_t(K.dcap) * 8, s) || dmemset(vm->d_ksmall, 0, XE_KS_WORDS * 4, s) ||
        dmemset(K.dfirst, 0xff, uint64_t(K.dcap) * 4, s) || dmemset(K.dvict, 0xff, uint64_t(K.dcap) * 4, s))
      return fail(vm, XE_ERR_DEVICE, "keyed reset");
    const uint32_t grid = parallel_grid(vm, kjit, general, n, P.nmaps);
    XeParams X = P;
    if (general && ensure_arena(vm, false, grid * 256, X.gen)) return fail(vm, XE_ERR_NOMEM, "device alloc (arena)");
    tmark("arena");
    // 1. SPEC: every packet against the start state, writes held back, keys logged
    X.mode = XE_MODE_SPEC;
    X.K = K;
    if (klaunch(&X, grid) || fold()) return fail(vm, XE_ERR_DEVICE, "kernel launch (keyed spec)");
    if (read_aux()) return fail(vm, XE_ERR_DEVICE, "kernel failed (keyed spec)");
    uint32_t flags = uint32_t(red[0]);
    if (ordmaps && (flags & XE_FLAG_CAPACITY) && !(flags & XE_FLAG_ORDERED)) {
      // appends past an ordered map's device room (the parallel branch's ordered_grow): the room
      // grows to what the pass tried to append and the keyed path starts over
      const int g = ordered_grow(vm, kh0, s);
      if (g < 0) return fail(vm, XE_ERR_DEVICE, "ordered map room");
      if (g == 1) {
        if (rollback(false) || prepare_run(vm, s)) return fail(vm, XE_ERR_DEVICE, "rollback");
        P.maps = vm->d_maps;
        keyed_trace("spec capacity: grown");
        return 2;
      }
    }
    if (flags & (XE_FLAG_ORDERED | XE_FLAG_CAPACITY)) { keyed_trace("spec ordered/capacity"); return krollback() ? -1 : 1; }
    if (!(flags & XE_FLAG_KEYED)) {  // no packet wrote a map entry: an ordinary parallel run
      if (run_conflict(red, P.nmaps)) { keyed_trace("spec conflict"); return krollback() ? -1 : 1; }
      if (ordmaps && ordered_finalize(vm, kh0, n, s)) return fail(vm, XE_ERR_DEVICE, "ordered map appends");
      used_out = XE_MODE_PARALLEL;
      return 0;
    }
    // 2. build: D, chains (union-find rounds), each packet's chain, the sorted order
    auto step = [&](uint32_t st, uint32_t items) { return launch_keyed(&K, vm->d_maps, vm->d_skip, st, items, s); };
    std::vector<uint32_t> small(XE_KS_WORDS);
    auto read_small = [&]() { return d2h(small.data(), vm->d_ksmall, XE_KS_WORDS * 4, s) || dsync(s); };
    if (step(XE_KS_DSET, n)) return fail(vm, XE_ERR_DEVICE, "keyed build");
    for (int round = 0;; round++) {
      if (round >= 64) { keyed_trace("union rounds"); return krollback() ? -1 : 1; }
      if (dmemset(K.changed, 0, 4, s) || step(XE_KS_UNION, n) || read_small()) return fail(vm, XE_ERR_DEVICE, "keyed build");
      if (!small[XE_KS_CHANGED]) break;
    }
    if (step(XE_KS_COMPRESS, K.dcap) || step(XE_KS_ASSIGN, n) || step(XE_KS_COUNT, K.dcap) || read_small())
      return fail(vm, XE_ERR_DEVICE, "keyed build");
    if (small[XE_KS_ERR] & 8u) {  // D outgrew its table: once more with room for every packet's key
      vm->keyed_dnext = dmax;
      if (dcap < dmax) { keyed_trace("D full"); return krollback() ? -1 : 2; }
    }
    // key log overflow (1), a root walk that did not end (16): the in-order replay
    if (small[XE_KS_ERR]) { keyed_trace(small[XE_KS_ERR] & 16u ? "root walk" : "key log overflow"); return krollback() ? -1 : 1; }
    {
      uint64_t nd = 0;
      for (uint32_t i = 0; i < 64; i++) nd += small[XE_KS_DCOUNT + i];
      uint64_t next = 4096;
      while (next < 4 * nd && next < dmax) next <<= 1;
      vm->keyed_dnext = uint32_t(next);
    }
    std::map<size_t, uint64_t> evict;  // LRU map -> the evictions its inserts make
    // a HASH insert can fail for capacity only in an order-dependent way (and an LRU insert would evict
    // by the batch's order of touches): every key some packet inserts fits. Only an absent key's insert
    // meets the capacity rule (maps_hash.go:84-89, maps_hash_lru.go:114-119) and nothing deletes in a
    // keyed batch, so the bound is the live count + the D keys a packet inserts (XE_KS_DINS); keys
    // that are only looked up, promoted or updated in place do not count
    for (size_t i = 1; i < vm->maps.size() && i < 64; i++) {
      HostMap& m = vm->maps[i];
      const uint64_t nd = small[XE_KS_DINS + i];
      if ((m.dkind != XE_DM_HASH && m.dkind != XE_DM_LRU) || !nd) continue;
      uint64_t cnt = 0;
      if (m.dkind == XE_DM_HASH) {
        uint32_t c32 = 0;
        if (d2h(&c32, m.d_count, 4, s) || dsync(s)) return fail(vm, XE_ERR_DEVICE, "count");
        cnt = c32;
      } else {
        cnt = kh0[i * 8 + 2];
        // value ids for every new key that does not take over its victim's (keyed_lruid_item): grow the
        // pool and run again
        const uint64_t ev = cnt + nd > m.def.max_entries ? cnt + nd - m.def.max_entries : 0;
        if (kh0[i * 8 + 3] + (nd - ev) > m.pool_cap) {
          if (krollback() || map_download(vm, m)) return -1;  // the mirror: the batch's start
          vm->ord_slack = std::max<uint64_t>(vm->ord_slack, 2 * nd + 4096);
          m.host_dirty = true;  // rebuilt from the mirror with the larger pool
          if (prepare_run(vm, s)) return fail(vm, XE_ERR_DEVICE, "ordered map room");
          P.maps = vm->d_maps;
          keyed_trace("LRU pool grown");
          return 2;
        }
      }
      if (cnt + nd > m.def.max_entries) {
        if (m.dkind != XE_DM_LRU) { keyed_trace("capacity"); return krollback() ? -1 : 1; }
        evict[i] = cnt + nd - m.def.max_entries;  // the batch's inserts evict: planned below
      }
    }
    // LRU evictions (xe_interp.h keyed_evict_item): rank every LRU map's new keys by their first
    // inserting packet, give the inserts past the map's room the oldest values of the batch's start as
    // victims, and replay in order if any packet of the batch touches one of them
    if (!evict.empty()) {
      size_t eb = 0;
      if (step(XE_KS_FIRST, n) || step(XE_KS_EKEY, K.dcap) || launch_keyed_esort(&K, nullptr, &eb, s) ||
          ensure_buf(&vm->d_ksort, &vm->d_ksort_cap, eb) || launch_keyed_esort(&K, vm->d_ksort, &eb, s))
        return fail(vm, XE_ERR_DEVICE, "keyed evictions");
      uint64_t off = 0;
      for (size_t i = 1; i < vm->maps.size() && i < 64; i++) {
        HostMap& m = vm->maps[i];
        if (m.dkind != XE_DM_LRU) continue;
        const uint32_t nd = small[XE_KS_DINS + i];
        if (evict.count(i)) {
          const uint64_t cnt = kh0[i * 8 + 2];
          // the start's UsageList by stamp (the stamps at the batch's start: the snapshot of ordered_hdr_read)
          size_t rb = 0;
          if (launch_lru_relink(m.d_tsnap, m.pool_cap, uint32_t(cnt), m.d_link, m.d_hdr, nullptr, &rb, 2, s) ||
              ensure_buf(&vm->d_relink, &vm->d_relink_cap, rb) ||
              launch_lru_relink(m.d_tsnap, m.pool_cap, uint32_t(cnt), m.d_link, m.d_hdr, vm->d_relink, &rb, 2, s))
            return fail(vm, XE_ERR_DEVICE, "keyed evictions (order)");
          K.em = uint32_t(i);
          K.eoff = uint32_t(off);
          K.efree = uint32_t(m.def.max_entries - cnt);
          K.ecnt0 = uint32_t(cnt);
          K.etsnap = m.d_tsnap;
          K.vorder = lru_sorted_ids(vm->d_relink, m.pool_cap);
          if (step(XE_KS_EVICT, nd) || step(XE_KS_EMARK, nd)) return fail(vm, XE_ERR_DEVICE, "keyed evictions");
        }
        off += nd;
      }
      if (read_small()) return fail(vm, XE_ERR_DEVICE, "keyed evictions");
      if (small[XE_KS_ERR] & 8u) {  // the victims' keys did not fit the D table
        vm->keyed_dnext = dmax;
        if (dcap < dmax) { keyed_trace("D full (victims)"); return krollback() ? -1 : 2; }
      }
      if (small[XE_KS_ERR]) { keyed_trace("eviction seen by the batch"); return krollback() ? -1 : 1; }
      K.em = 0;
    }
    uint32_t end_bit = 1;
    while ((1ull << end_bit) <= K.dcap) end_bit++;
    size_t sb = 0;
    if (step(XE_KS_IOTA, n) || launch_keyed_sort(&K, n, end_bit, nullptr, &sb, s) ||
        ensure_buf(&vm->d_ksort, &vm->d_ksort_cap, sb) || launch_keyed_sort(&K, n, end_bit, vm->d_ksort, &sb, s))
      return fail(vm, XE_ERR_DEVICE, "keyed sort");
    if (step(XE_KS_NCHAIN, n) || read_small()) return fail(vm, XE_ERR_DEVICE, "keyed build");
    K.nO = small[XE_KS_NO];
    // one chain with more than half the packets (a hot key written by most of them): its lane would
    // take longer than the staged one-lane replay of the whole batch
    if (step(XE_KS_CSTART, K.nO) || step(XE_KS_CLONG, K.nO) || read_small()) return fail(vm, XE_ERR_DEVICE, "keyed build");
    if (small[XE_KS_LONG]) { keyed_trace("long chain"); return krollback() ? -1 : 1; }
    // 3. back to the start state; reserve a slot record for every new HASH key of D
    if (krollback() || snap_records()) return fail(vm, XE_ERR_DEVICE, "rollback");
    if (ordmaps && step(XE_KS_LRUID, K.dcap)) return fail(vm, XE_ERR_DEVICE, "keyed value ids");
    if (step(XE_KS_RESERVE, K.dcap) || read_small()) return fail(vm, XE_ERR_DEVICE, "keyed reserve");
    if (small[XE_KS_ERR]) { keyed_trace("reserve"); return rollback(true) ? -1 : 1; }
    // 4. the packets on no chain, in parallel (the fast kernel: the skip mask is its only keyed input)
    X.mode = XE_MODE_PARALLEL;
    X.K = K;
    X.K.skip = vm->d_skip;
    if (K.nO < n) {
      XeParams Y = X;
      const uint32_t pgrid = parallel_grid(vm, jit, general, n, P.nmaps);
      if (general && ensure_arena(vm, false, pgrid * 256, Y.gen)) return fail(vm, XE_ERR_NOMEM, "device alloc (arena)");
      if (launch(&Y, pgrid, 256) || fold()) return fail(vm, XE_ERR_DEVICE, "kernel launch (keyed parallel)");
    }
    // 5. the chains in packet order: the compacted chain list is a work queue the waves claim from
    {
      size_t sb2 = 0;
      if (step(XE_KS_CFLAG, K.nO) || launch_keyed_scan(&K, K.nO, nullptr, &sb2, s) ||
          ensure_buf(&vm->d_ksort, &vm->d_ksort_cap, sb2) || launch_keyed_scan(&K, K.nO, vm->d_ksort, &sb2, s) ||
          step(XE_KS_CLIST, K.nO) || dmemset(vm->d_ksmall + XE_KS_CNEXT, 0, 4, s))
        return fail(vm, XE_ERR_DEVICE, "keyed chain list");
    }
    X.mode = XE_MODE_CHAIN;
    X.K.skip = nullptr;
    const uint32_t cgrid = std::max<uint32_t>(1, std::min<uint32_t>(grid, (K.nO + 255) / 256));
    if (general && ensure_arena(vm, false, cgrid * 256, X.gen)) return fail(vm, XE_ERR_NOMEM, "device alloc (arena)");
    if (klaunch(&X, cgrid) || step(XE_KS_UNNEW, K.dcap)) return fail(vm, XE_ERR_DEVICE, "kernel launch (keyed chains)");
    if (read_aux() || read_small()) return fail(vm, XE_ERR_DEVICE, "kernel failed (keyed chains)");
    if (run_conflict(red, P.nmaps)) { keyed_trace("chain conflict"); return rollback(true) ? -1 : 1; }  // a packet left its chain / an order-dependent add
    // the chains' inserts into the map counts (LRU_HASH: header word 2, less its evictions). An LRU map
    // with evictions must have seen every ranked insert: one that did not happen shifts the victims of
    // the inserts after it
    for (const auto& [i, ev] : evict) {
      uint32_t add = 0;
      for (uint32_t k = 0; k < XE_KSTRIPES; k++) add += small[XE_KS_CINS + i * XE_KSTRIPES + k];
      if (add != small[XE_KS_DINS + i]) { keyed_trace("eviction ranks"); return rollback(true) ? -1 : 1; }
    }
    for (size_t i = 1; i < vm->maps.size() && i < 64; i++) {
      HostMap& m = vm->maps[i];
      uint32_t add = 0;
      for (uint32_t k = 0; k < XE_KSTRIPES; k++) add += small[XE_KS_CINS + i * XE_KSTRIPES + k];
      if (!add) continue;
      if (m.dkind == XE_DM_HASH) {
        uint32_t cnt = 0;
        if (d2h(&cnt, m.d_count, 4, s) || dsync(s)) return fail(vm, XE_ERR_DEVICE, "count");
        cnt += add;
        if (h2d(m.d_count, &cnt, 4, s) || dsync(s)) return fail(vm, XE_ERR_DEVICE, "count");
      } else if (m.dkind == XE_DM_LRU) {
        uint64_t cnt = 0;
        if (d2h(&cnt, m.d_hdr + 2, 8, s) || dsync(s)) return fail(vm, XE_ERR_DEVICE, "count");
        cnt += add;
        if (evict.count(i)) cnt -= evict[i];
        if (h2d(m.d_hdr + 2, &cnt, 8, s) || dsync(s)) return fail(vm, XE_ERR_DEVICE, "count");
      }
    }
    // the appends and LRU touches of both passes into packet order
    if (ordmaps && ordered_finalize(vm, kh0, n, s)) return fail(vm, XE_ERR_DEVICE, "ordered map appends");
    vm->last_grid = grid;
    used_out = XE_MODE_KEYED;
    return 0;
  };

  if (jit && keyed_candidate(vm)) keyed_kernel(vm, jit);  // built before the timed region
  vm->t0.rec(s);
  bool conflict = false;
  uint32_t used = XE_MODE_PARALLEL;
  float kms = 0;
  // ordered maps: appends and LRU lookups run in parallel (put in packet order afterwards), LRU updates
  // through the keyed path; a batch with any other operation on them (pops, peeks, list lookups, an LRU
  // eviction) replays in order, and so do the next few after such a batch
  tmark("setup");
  if (!vm->keyed_hint_set && n > 0) {
    vm->keyed_hint_set = true;
    if (lru_update_sites(vm)) vm->keyed_hint = true;
  }
  const bool ord_par = !ordmaps || ordered_parallel_ok(vm);
  const bool keyed_ok = mode == XE_MODE_AUTO && n > 0 && !overlap && ord_par;
  bool ord_seq = mode == XE_MODE_AUTO && ordmaps && (!ord_par || vm->ord_backoff);
  if (ord_seq && vm->ord_backoff) vm->ord_backoff--;
  std::vector<uint64_t> ord_h0;
  if (mode == XE_MODE_SEQUENTIAL || ord_seq || overlap || hostcalls) {
    used = XE_MODE_SEQUENTIAL;
    if (int rc = sequential(kms)) return rc;
  } else if (keyed_ok && vm->keyed_hint) {
    // the last batch wrote map entries: straight to the keyed path
    int r = keyed(used);
    for (int t = 0; r == 2 && t < 3; t++) r = keyed(used);  // its D table / an LRU pool was too small
    if (r == 2) r = 1;
    if (r < 0) return r;
    if (r == 1) {
      vm->keyed_backoff = kKeyedBackoff;
      if (ordmaps) vm->ord_backoff = kKeyedBackoff;
      used = XE_MODE_SEQUENTIAL;
      if (int rc = sequential(kms)) return rc;
    }
    conflict = used != XE_MODE_PARALLEL;
    vm->t1.rec(s);
    if (dsync(s)) return fail(vm, XE_ERR_DEVICE, "sync");
    kms += Timer::ms(vm->t0, vm->t1);
  } else {
    P.mode = XE_MODE_PARALLEL;
    void* pj = (jit && !P.results && !P.regs) ? lean_kernel(vm, jit) : jit;  // verdicts only: the lean variant
    vm->last_grid = parallel_grid(vm, pj, general, n, P.nmaps);
    if (general && ensure_arena(vm, false, vm->last_grid * 256, P.gen)) return fail(vm, XE_ERR_NOMEM, "device alloc (arena)");
    uint32_t flags = 0;
    uint32_t seg_cut = 0;  // > 0: the batch may run as packet-order segments cut there
    // QUEUE / STACK pops, peeks and lookups in parallel (xe_interp.h list_pos): the run's list record,
    // and for a program that may pop, a count pass first (which packets pop: their prefix sum is each
    // pop's rank in packet order), then the pass proper from the batch's start again
    const bool lists = ordmaps && n > 0 && has_list_maps(vm);
    const bool pops = lists && may_pop(vm);
    bool list_conflict = false;
    uint64_t popped = 0;  // the lists the batch's pops were ranked on (bit m)
    if (lists) {
      if (!vm->d_listrun && dev_alloc((void**)&vm->d_listrun, sizeof(XeListRun))) return fail(vm, XE_ERR_NOMEM, "device alloc (lists)");
      P.list = vm->d_listrun;
      if (pops && vm->pop_n < n) {
        dev_free(vm->d_popflag); dev_free(vm->d_popbase); dev_free(vm->d_popused);
        vm->d_popflag = vm->d_popbase = vm->d_popused = nullptr;
        vm->pop_n = 0;
        if (dev_alloc((void**)&vm->d_popflag, size_t(n) * 4) || dev_alloc((void**)&vm->d_popbase, size_t(n) * 4 * XE_POP_SLOTS) ||
            dev_alloc((void**)&vm->d_popused, size_t(n) * 4))
          return fail(vm, XE_ERR_NOMEM, "device alloc (pop ranks)");
        vm->pop_n = n;
      }
    }
    XeListRun lr{};
    auto list_init = [&]() -> int {  // start counts from the headers, no sensitive op, no push yet
      memset(&lr, 0, sizeof lr);
      for (size_t i = 1; i < vm->maps.size() && i < 64; i++)
        if (vm->maps[i].dkind == XE_DM_LIST) lr.cnt0[i] = uint32_t(ord_h0[i * 8 + 1]);
      for (int i = 0; i < 64; i++) lr.push[i] = lr.senslo[i] = 0xffffffffu;
      return h2d(vm->d_listrun, &lr, sizeof lr, s);
    };
    auto list_read = [&]() -> int { return d2h(&lr, vm->d_listrun, sizeof lr, s) || dsync(s); };
    auto pass = [&]() -> int {
      if (pj ? launch_jit(pj, &P, vm->last_grid, 256, s) : launch_interp(&P, vm->last_grid, 256, s))
        return fail(vm, XE_ERR_DEVICE, "kernel launch");
      vm->t1.rec(s);  // kernel_ms: the emulator kernel alone
      if (fold()) return fail(vm, XE_ERR_DEVICE, "replica fold");
      if (read_aux()) return fail(vm, XE_ERR_DEVICE, "kernel failed");
      kms = Timer::ms(vm->t0, vm->t1);
      flags = uint32_t(red[0]);
      conflict = run_conflict(red, P.nmaps);
      return XE_OK;
    };
    for (int attempt = 0;; attempt++) {
      if (ordmaps && ordered_hdr_read(vm, ord_h0, s)) return fail(vm, XE_ERR_DEVICE, "ordered map header");
      if (lists && list_init()) return fail(vm, XE_ERR_DEVICE, "list run");
      tmark("ordered hdr");
      if (pops) {
        P.pop_mode = 1;
        P.popflag = vm->d_popflag;
        P.popbase = nullptr;
        if (dmemset(vm->d_popflag, 0, size_t(n) * 4, s)) return fail(vm, XE_ERR_DEVICE, "pop flags");
        if (int rc = pass()) return rc;
        tmark("count pass");
        if (!conflict) {
          if (list_read()) return fail(vm, XE_ERR_DEVICE, "list run");
          // Ranked passes: each popped list gets a slot; a packet's pops of it are counted in 8 bits of its
          // word (the count pass's first pops, then what the last ranked pass observed), the counts of each
          // slot are scanned into ranks, and the pass runs again from the batch's start until every packet
          // made exactly the pops it was ranked by (a pop after a peek, a second pop, or pops from another
          // list change what the count pass saw). Up to 4 passes; then, or with more than XE_POP_SLOTS
          // popped lists, the batch replays in order.
          uint64_t mask = lr.popmask;
          bool ranked = false;
          for (int it = 0; it < 4 && !conflict; it++) {
            if (__builtin_popcountll(mask) > int(XE_POP_SLOTS)) break;
            XePopSlots sl;
            memset(sl.slot, 0xff, sizeof sl.slot);
            uint32_t ns = 0;
            for (uint32_t m = 0; m < 64; m++)
              if ((mask >> m) & 1) sl.slot[m] = uint8_t(ns++);
            memcpy(P.pop_slot, sl.slot, sizeof sl.slot);
            P.pop_stride = n;
            // the counts to rank by: packed count-pass flags first, then the last pass's observed counts
            if (it == 0 ? launch_pop(vm->d_popflag, vm->d_popused, n, 0, 0, sl, nullptr, s)
                        : d2d(vm->d_popused, vm->d_popflag, size_t(n) * 4, s))
              return fail(vm, XE_ERR_DEVICE, "pop ranks");
            for (uint32_t j = 0; j < ns; j++) {
              XeKeyed S{};
              S.iota = vm->d_popflag;  // (free until the pass writes its observed counts)
              S.ckey = vm->d_popbase + size_t(j) * n;
              size_t sb = 0;
              if (launch_pop(vm->d_popused, vm->d_popflag, n, 1, j, sl, nullptr, s) ||
                  launch_keyed_scan(&S, n, nullptr, &sb, s) || ensure_buf(&vm->d_ksort, &vm->d_ksort_cap, sb) ||
                  launch_keyed_scan(&S, n, vm->d_ksort, &sb, s))
                return fail(vm, XE_ERR_DEVICE, "pop ranks");
            }
            if (rollback(false) || ordered_hdr_restore(vm, ord_h0, s) || list_init()) return fail(vm, XE_ERR_DEVICE, "pop ranks");
            tmark("ranks");
            P.pop_mode = 2;
            P.popbase = vm->d_popbase;
            if (int rc = pass()) return rc;
            tmark("ranked pass");
            if (conflict) break;
            if (list_read()) return fail(vm, XE_ERR_DEVICE, "list run");
            if (lr.newlist) {  // a pop of a list with no slot: rank it too
              mask |= lr.popmask;
              continue;
            }
            if (ensure_buf(&vm->d_ksort, &vm->d_ksort_cap, 256)) return fail(vm, XE_ERR_NOMEM, "pop ranks");
            uint32_t* d_flag = (uint32_t*)vm->d_ksort;  // (the scans' scratch, free now)
            uint32_t mismatch = 0;
            if (dmemset(d_flag, 0, 4, s) || launch_pop(vm->d_popflag, vm->d_popused, n, 2, 0, sl, d_flag, s) ||
                d2h(&mismatch, d_flag, 4, s) || dsync(s))
              return fail(vm, XE_ERR_DEVICE, "pop ranks");
            if (!mismatch) {
              ranked = true;
              popped = mask;
              break;
            }
          }
          if (!ranked && !conflict) {
            list_conflict = conflict = true;
            flags |= XE_FLAG_ORDERED;
          }
        }
      } else if (int rc = pass()) {
        return rc;
      }
      if (!conflict && lists) {  // exact only if no list position depended on an earlier push
        if (list_read()) return fail(vm, XE_ERR_DEVICE, "list run");
        for (int i = 0; i < 64; i++)
          if (lr.sens[i] > lr.push[i]) list_conflict = true;
        if (list_conflict) {
          conflict = true;
          // Segments: the packets before the first position that may have depended on an earlier push
          // ran exactly; from there on the batch is a batch of its own whose start contents hold those
          // pushes. The cut: per list, its first such packet (its first packet with a position, when that
          // comes at or after its first push; else its first push, before which nothing was pushed).
          // (Any cut keeps the packet loop's order — two batches are the same loop — so a pass that also
          // ran out of an ordered map's room still cuts: each segment grows the room itself. A lane that
          // needed an ordered map write elsewhere would need the fallback in every segment: no cut.)
          if (!(flags & XE_FLAG_ORDERED)) {
            seg_cut = n;
            for (int i = 0; i < 64; i++)
              if (lr.sens[i] > lr.push[i]) seg_cut = std::min(seg_cut, lr.senslo[i] >= lr.push[i] ? lr.senslo[i] : lr.push[i]);
          }
          flags |= XE_FLAG_ORDERED;
        }
      }
      // appends past an ordered map's device room: the atomics counted every attempted append, so the
      // room grows to what the batch needs and the parallel pass runs once more (up to three times: a
      // count pass stops its packets at their first pop, so its appends undercount the ranked pass's)
      if (ordmaps && attempt < 3 && (flags & XE_FLAG_CAPACITY) && !(flags & XE_FLAG_ORDERED)) {
        const int g = ordered_grow(vm, ord_h0, s);
        if (g < 0) return fail(vm, XE_ERR_DEVICE, "ordered map room");
        if (g == 1) {
          if (rollback(false) || prepare_run(vm, s)) return fail(vm, XE_ERR_DEVICE, "rollback");
          P.maps = vm->d_maps;
          continue;
        }
      }
      break;
    }
    // (a segment costs a pass over what follows it: at least kSegMin packets, else the usual fallback)
    tmark("passes done");
    if (conflict && mode == XE_MODE_AUTO && seg_cut >= kSegMin && seg_cut < n && segments_ok(vm, P)) {
      if (rollback(false) || (ordmaps && ordered_hdr_restore(vm, ord_h0, s))) return fail(vm, XE_ERR_DEVICE, "rollback");
      return run_segments(vm, d_umem, umem_len, d_desc, n, seg_cut, d_results, d_verdicts, d_regs, stream, stats);
    }
    if (conflict && (mode == XE_MODE_AUTO || (flags & XE_FLAG_CAPACITY))) {
      // order-dependent batch (or a lane out of arena): roll the maps back; map-entry writes take the
      // keyed path, everything else (and what the keyed path refuses) the replay in packet order.
      // A pass that also ran out of an ordered map's room (appends beside an ordered write) grows it
      // first, so the keyed path does not inherit the shortage.
      bool grown = false;
      if (ordmaps && (flags & XE_FLAG_CAPACITY) && (flags & XE_FLAG_ORDERED)) {
        const int g = ordered_grow(vm, ord_h0, s);  // (restores the ordered maps itself)
        if (g < 0) return fail(vm, XE_ERR_DEVICE, "ordered map room");
        grown = g == 1;
      }
      if (rollback(false)) return fail(vm, XE_ERR_DEVICE, "rollback");
      if (grown) {
        if (prepare_run(vm, s)) return fail(vm, XE_ERR_DEVICE, "rollback");
        P.maps = vm->d_maps;
      } else if (ordmaps) {  // the appends of the run are past the restored counts: unreferenced
        if (ordered_hdr_restore(vm, ord_h0, s)) return fail(vm, XE_ERR_DEVICE, "rollback (ordered maps)");
      }
      int r = 1;
      const bool try_keyed = keyed_ok && (flags & XE_FLAG_ORDERED) && (!(flags & XE_FLAG_CAPACITY) || grown) && !list_conflict;
      if (try_keyed && vm->keyed_backoff) vm->keyed_backoff--;
      else if (try_keyed) {
        vm->t2.rec(s);
        r = keyed(used);
        for (int t = 0; r == 2 && t < 3; t++) r = keyed(used);  // its D table / an LRU pool was too small
        if (r == 2) r = 1;
        if (r < 0) return r;
        if (r == 1) vm->keyed_backoff = kKeyedBackoff;
        if (r == 0) {
          vm->t1.rec(s);
          if (dsync(s)) return fail(vm, XE_ERR_DEVICE, "sync");
          kms += Timer::ms(vm->t2, vm->t1);
        }
      }
      if (r == 1) {
        if (ordmaps) vm->ord_backoff = kKeyedBackoff;
        used = XE_MODE_SEQUENTIAL;
        if (int rc = sequential(kms)) return rc;
      }
    } else if (!conflict) {
      vm->keyed_backoff = 0;
      // the run's results stand: its appends into packet order, then its pops off the popped list (a
      // stack's pushes all came after its pops, so they land on the lowered top)
      if (ordmaps) {
        std::vector<uint64_t> h0 = ord_h0;
        std::vector<std::pair<uint32_t, uint64_t>> took;  // (list, its elements the batch popped)
        if (popped) {
          uint32_t last_used = 0;
          if (d2h(&last_used, vm->d_popused + (n - 1), 4, s) || dsync(s)) return fail(vm, XE_ERR_DEVICE, "pop count");
          uint32_t j = 0;
          for (uint32_t mi = 0; mi < 64; mi++) {
            if (!((popped >> mi) & 1)) continue;
            uint32_t base = 0;
            if (d2h(&base, vm->d_popbase + size_t(j) * n + (n - 1), 4, s) || dsync(s)) return fail(vm, XE_ERR_DEVICE, "pop count");
            const uint64_t k = std::min<uint64_t>(uint64_t(base) + ((last_used >> (8 * j)) & 0xffu), ord_h0[mi * 8 + 1]);
            if (vm->maps[mi].stack) h0[mi * 8 + 1] -= k;
            if (k) took.push_back({mi, k});
            j++;
          }
        }
        tmark("before finalize");
        if (ordered_finalize(vm, h0, n, s)) return fail(vm, XE_ERR_DEVICE, "ordered map appends");
        tmark("finalize");
        for (const auto& t : took) {
          HostMap& m = vm->maps[t.first];
          const uint64_t k = t.second;
          uint64_t hdr[8];
          if (d2h(hdr, m.d_hdr, 64, s) || dsync(s)) return fail(vm, XE_ERR_DEVICE, "pops");
          if (!m.stack) hdr[0] = (hdr[0] + k) % m.list_cap;
          hdr[1] -= k;
          if (h2d(m.d_hdr, hdr, 64, s) || dsync(s)) return fail(vm, XE_ERR_DEVICE, "pops");
        }
      }
    }
  }
  if (n > 0) vm->keyed_hint = used == XE_MODE_KEYED;  // (an empty batch, e.g. a map upload, says nothing)
  if (used == XE_MODE_KEYED) red[0] |= XE_FLAG_ORDERED;  // order-dependent effects (shard checks replay it)
  record_widths(vm, red, P.nmaps);
  if (used == XE_MODE_SEQUENTIAL || used == XE_MODE_KEYED) {
    // in-program inserts change the entry count: refresh the replica-sizing hint
    std::vector<uint32_t> counts(vm->maps.size(), 0);
    for (size_t i = 1; i < vm->maps.size(); i++)
      if (vm->maps[i].dkind == XE_DM_HASH && d2h(&counts[i], vm->maps[i].d_count, 4, s)) return fail(vm, XE_ERR_DEVICE, "count");
    if (dsync(s)) return fail(vm, XE_ERR_DEVICE, "sync");
    for (size_t i = 1; i < vm->maps.size(); i++)
      if (vm->maps[i].dkind == XE_DM_HASH) vm->maps[i].live = counts[i];
  }
  note_run(vm, red, used);
  tmark("done");
  if (n > 0)  // an empty batch (a map upload) changes no map: the host mirrors stay current
    for (size_t i = 1; i < vm->maps.size(); i++) vm->maps[i].dev_dirty = true;
  if (stats) {
    stats->packets = n;
    stats->steps = red[1];
    for (int k = 0; k < 8; k++) stats->status_count[k] = red[2 + k];
    stats->mode_used = used;
    stats->conflict = conflict ? 1 : 0;
    stats->kernel_ms = kms;
    stats->total_ms = kms;
    stats->engine_used = jit ? XE_ENGINE_JIT : XE_ENGINE_INTERP;
    stats->grid_blocks = used == XE_MODE_SEQUENTIAL ? 1 : vm->last_grid;
  }
  return XE_OK;
}

namespace {

// Complete the oldest pipelined batch: wait for its read-back, then publish its statistics, or — when
// its epilogue decided on an in-order replay — roll the maps back to its start and re-run it and every
// later batch (they did nothing on the device) through the synchronous path, in submission order.
int complete_oldest(xe_vm* vm) {
  const uint32_t si = vm->pending.front();
  xe_vm::Slot& sl = vm->slots[si];
  if (sl.done.wait()) {
    vm->pending.clear();
    return fail(vm, XE_ERR_DEVICE, "kernel failed (pipelined batch)");
  }
  const unsigned long long* aux = sl.h_aux;
  if (aux[XE_AUX_DECISION]) {
    vm->staged_slot = -1;
    const xe_stream_t s = sl.b.s;
    for (size_t i = 1; i < vm->maps.size(); i++) {
      HostMap& m = vm->maps[i];
      if (!m.ordered() && d2d(m.d_vals, m.d_asnap[sl.snap], m.vals_alloc, s)) return fail(vm, XE_ERR_DEVICE, "rollback");
    }
    if (dmemset(vm->d_poison, 0, 4, s)) return fail(vm, XE_ERR_DEVICE, "rollback");
    std::vector<xe_vm::Batch> redo;
    for (uint32_t k : vm->pending) redo.push_back(vm->slots[k].b);
    vm->pending.clear();
    for (const xe_vm::Batch& b : redo)
      if (int rc = xe_run_batch_device(vm, b.d_umem, b.umem_len, b.d_desc, b.n, b.d_results, b.d_verdicts, b.d_regs, b.s,
                                       b.stats))
        return rc;
    return XE_OK;
  }
  std::vector<unsigned long long> red;
  reduce_aux(aux, sl.nmaps, 16 + 2 * (sl.nmaps + 1), red);
  record_widths(vm, red, sl.nmaps);
  note_run(vm, red, XE_MODE_PARALLEL);
  if (xe_batch_stats* st = sl.b.stats) {
    st->packets = sl.b.n;
    st->steps = red[1];
    for (int k = 0; k < 8; k++) st->status_count[k] = red[2 + k];
    st->mode_used = XE_MODE_PARALLEL;
    st->conflict = run_conflict(red, sl.nmaps) ? 1 : 0;  // reported, not replayed (XE_MODE_PARALLEL)
    st->kernel_ms = Timer::ms(sl.t0, sl.t1);
    st->total_ms = st->kernel_ms;
    st->engine_used = sl.engine;
    st->grid_blocks = sl.grid;
  }
  vm->pending.erase(vm->pending.begin());
  return XE_OK;
}

}  // namespace

// Build what the next batch runs, ahead of it: upload the maps, pick the engine and compile the
// per-program kernel for the current program and map geometry (and its keyed variant when the program
// may write map entries). Optional: the first batch does the same when this was not called.
int xe_prepare(xe_vm* vm) {
  if (!vm) return XE_ERR_INVAL;
  if (int rc = xe_sync(vm)) return rc;
  if (int rc = prepare_run(vm, vm->stream)) return rc;
  void* jit = nullptr;
  bool jit_general = false;
  if (int rc = select_engine(vm, jit, jit_general)) return rc;
  if (jit && keyed_candidate(vm)) keyed_kernel(vm, jit);
  if (jit) lean_kernel(vm, jit);
  return dsync(vm->stream) ? fail(vm, XE_ERR_DEVICE, "sync") : XE_OK;
}

// The generated source of a kernel xe_prepare would build (variant 0: the per-program kernel, 1: its
// keyed variant, 2: its verdict-only variant), for a process that fills the kernel cache
// (xe_compile_kernel_source).
int xe_kernel_source(xe_vm* vm, int variant, char* buf, size_t cap, size_t* len) {
  if (!vm || variant < 0 || variant > 3) return XE_ERR_INVAL;
  // the host simulation generates the same sources (ahead-of-time kernel builds on a machine without a
  // GPU: gobpfld_amd/aot.py) but runs none of them
  if (int rc = xe_sync(vm)) return rc;
  if (int rc = prepare_run(vm, vm->stream)) return rc;
  if (vm->settings.engine == XE_ENGINE_INTERP || !jit_possible(vm))
    return fail(vm, XE_ERR_UNSUPPORTED, "the program runs on the interpreter");
  if (variant == 1 && !keyed_candidate(vm)) return fail(vm, XE_ERR_UNSUPPORTED, "no keyed variant for this program");
  const ProgTab t = prog_tab(vm);
  const size_t n = xe_jit_source_for(t.p.data(), t.n.data(), uint32_t(vm->programs.size() - 1), vm->entry,
                                     vm->dm_uploaded.data(), uint32_t(vm->dm_uploaded.size() - 1), variant, buf, cap);
  if (len) *len = n;
  if (n == 0) return fail(vm, XE_ERR_UNSUPPORTED, "no such kernel variant for this program");
  return XE_OK;
}

#ifdef XE_HOSTSIM
// the host simulation compiles no per-program kernels (it links only the generator of xe_jit.cpp)
int xe_set_kernel_cache(const char*) { return XE_OK; }
int xe_compile_kernel_source(const char*, const char*, const char*, char* err, size_t errlen) {
  if (err && errlen) err[0] = 0;
  return XE_ERR_UNSUPPORTED;
}
int xe_kernel_object_name(const char*, const char*, char*, size_t) { return XE_ERR_UNSUPPORTED; }
int xe_kernel_cache_stats(uint64_t* hits, uint64_t* compiles, double* compile_s) {
  if (hits) *hits = 0;
  if (compiles) *compiles = 0;
  if (compile_s) *compile_s = 0;
  return XE_OK;
}
#endif

int xe_sync(xe_vm* vm) {
  if (!vm) return XE_ERR_INVAL;
  while (!vm->pending.empty())
    if (int rc = complete_oldest(vm)) {
      vm->pending.clear();
      return rc;
    }
  return XE_OK;
}

// RunContext's ctx.Err() (emulator/vm.go:117-134) for the pipelined batches: drop every batch not
// completed yet. The poison word makes the queued launches return at their first wave; the maps go back
// to the oldest dropped batch's rollback point (the snapshot its prologue or its predecessor's epilogue
// took before it ran), with the value replicas cleared.
int xe_cancel(xe_vm* vm, uint32_t* cancelled) {
  if (!vm) return XE_ERR_INVAL;
  if (cancelled) *cancelled = 0;
  if (vm->pending.empty()) return XE_OK;
  set_device(vm->settings.device);
  const uint32_t si = vm->pending.front();
  const xe_stream_t s = vm->slots[si].b.s;
  if (poison_async(vm->d_poison, &vm->cancel_stream) || dsync(s)) {
    vm->pending.clear();
    return fail(vm, XE_ERR_DEVICE, "cancel");
  }
  for (size_t i = 1; i < vm->maps.size(); i++) {
    HostMap& m = vm->maps[i];
    if (m.ordered()) continue;  // (maps of this kind never pipeline)
    if (d2d(m.d_vals, m.d_asnap[vm->slots[si].snap], m.vals_alloc, s)) return fail(vm, XE_ERR_DEVICE, "cancel (rollback)");
    if (m.nrep > 1 && m.d_rep && dmemset(m.d_rep, 0, m.rep_stride * m.nrep, s)) return fail(vm, XE_ERR_DEVICE, "cancel");
  }
  for (uint32_t k : vm->pending) {
    xe_vm::Slot& sl = vm->slots[k];
    if (dmemset(sl.d_aux, 0, kAuxWords * 8, s)) return fail(vm, XE_ERR_DEVICE, "cancel");
    if (xe_batch_stats* st = sl.b.stats) {
      memset(st, 0, sizeof *st);
      st->packets = sl.b.n;
      st->mode_used = XE_MODE_CANCELLED;
      st->engine_used = sl.engine;
      st->grid_blocks = sl.grid;
    }
  }
  if (cancelled) *cancelled = uint32_t(vm->pending.size());
  vm->pending.clear();
  vm->staged_slot = -1;
  if (dmemset(vm->d_poison, 0, 4, s) || dsync(s)) return fail(vm, XE_ERR_DEVICE, "cancel");
  return XE_OK;
}

int xe_trace_config(xe_vm* vm, const uint32_t* packets, uint32_t npk, uint32_t max_steps) {
  if (!vm || (npk && !packets) || npk > XE_TRACE_MAX_PACKETS || max_steps > XE_TRACE_MAX_STEPS) return XE_ERR_INVAL;
  if (npk && !max_steps) return XE_ERR_INVAL;
  if (int rc = xe_sync(vm)) return rc;
  set_device(vm->settings.device);
  dev_free(vm->d_trace_pk); dev_free(vm->d_trace); dev_free(vm->d_trace_cnt);
  vm->d_trace_pk = nullptr; vm->d_trace = nullptr; vm->d_trace_cnt = nullptr;
  vm->trace_pk.assign(packets, packets + npk);
  std::sort(vm->trace_pk.begin(), vm->trace_pk.end());
  vm->trace_pk.erase(std::unique(vm->trace_pk.begin(), vm->trace_pk.end()), vm->trace_pk.end());
  vm->trace_max = npk ? max_steps : 0;
  if (vm->trace_pk.empty()) return XE_OK;
  const size_t k = vm->trace_pk.size();
  if (dev_alloc((void**)&vm->d_trace_pk, k * 4) || dev_alloc((void**)&vm->d_trace, k * max_steps * sizeof(xe_trace_rec)) ||
      dev_alloc((void**)&vm->d_trace_cnt, k * 4) || h2d(vm->d_trace_pk, vm->trace_pk.data(), k * 4, vm->stream) ||
      dmemset(vm->d_trace_cnt, 0, k * 4, vm->stream) || dsync(vm->stream)) {
    vm->trace_pk.clear();
    return fail(vm, XE_ERR_NOMEM, "device alloc (trace)");
  }
  return XE_OK;
}

int xe_trace_read(xe_vm* vm, uint32_t packet, xe_trace_rec* out, uint32_t cap, uint32_t* nsteps) {
  if (!vm || !nsteps) return XE_ERR_INVAL;
  if (int rc = xe_sync(vm)) return rc;
  auto it = std::lower_bound(vm->trace_pk.begin(), vm->trace_pk.end(), packet);
  if (it == vm->trace_pk.end() || *it != packet) return fail(vm, XE_ERR_INVAL, "packet is not traced");
  const size_t slot = size_t(it - vm->trace_pk.begin());
  set_device(vm->settings.device);
  uint32_t cnt = 0;
  if (d2h(&cnt, vm->d_trace_cnt + slot, 4, vm->stream) || dsync(vm->stream)) return fail(vm, XE_ERR_DEVICE, "trace read");
  *nsteps = cnt;
  if (!out || !cap) return XE_OK;
  const uint32_t c = std::min(cap, cnt);
  if (c && (d2h(out, vm->d_trace + slot * vm->trace_max, size_t(c) * sizeof(xe_trace_rec), vm->stream) || dsync(vm->stream)))
    return fail(vm, XE_ERR_DEVICE, "trace read");
  return XE_OK;
}

int xe_set_helper(xe_vm* vm, uint32_t id, xe_helper_fn fn, void* user) {
  if (!vm || id >= 192) return XE_ERR_INVAL;
  if (int rc = xe_sync(vm)) return rc;
  const uint64_t b = 1ull << (id & 63);
  if (fn) {
    if (!vm->h_hostcall) {
      set_device(vm->settings.device);
      void* h = nullptr;
      void* d = nullptr;
      if (host_alloc_coherent(&h, sizeof(XeHostCall)) || host_device_ptr(&d, h)) return fail(vm, XE_ERR_NOMEM, "host helper mailbox");
      vm->h_hostcall = (XeHostCall*)h;
      vm->d_hostcall = (XeHostCall*)d;
    }
    vm->h_hostcall->fn[id] = fn;
    vm->h_hostcall->user[id] = user;
    vm->host_helpers[id >> 6] |= b;
    vm->nil_helpers[id >> 6] &= ~b;
  } else {
    vm->host_helpers[id >> 6] &= ~b;
    vm->nil_helpers[id >> 6] |= b;
  }
  return XE_OK;
}

int xe_reset_helper(xe_vm* vm, uint32_t id) {
  if (!vm || id >= 192) return XE_ERR_INVAL;
  if (int rc = xe_sync(vm)) return rc;
  const uint64_t b = 1ull << (id & 63);
  vm->host_helpers[id >> 6] &= ~b;
  vm->nil_helpers[id >> 6] &= ~b;
  return XE_OK;
}

int xe_run_batch_device_async(xe_vm* vm, void* d_umem, uint64_t umem_len, const void* d_desc, uint32_t n,
                              void* d_results, void* d_verdicts, void* d_regs, void* stream, xe_batch_stats* stats) {
  if (!vm) return XE_ERR_INVAL;
  if (stats) memset(stats, 0, sizeof *stats);
  xe_stream_t s = stream ? (xe_stream_t)stream : vm->stream;
  const bool entry_ok = vm->entry >= 1 && vm->entry < int32_t(vm->programs.size());
  // batches that cannot pipeline run synchronously, after everything in flight
  // (keyed_hint: the last batch wrote map entries, this one starts with the keyed path's SPEC pass)
  if (!entry_ok || vm->settings.mode == XE_MODE_SEQUENTIAL || has_ordered_maps(vm) || vm->keyed_hint ||
      (umem_len && may_write_packet(vm->programs[vm->entry])) || !vm->trace_pk.empty() || calls_host_helper(vm))
    return xe_run_batch_device(vm, d_umem, umem_len, d_desc, n, d_results, d_verdicts, d_regs, stream, stats);
  if (n && (!d_umem || !d_desc)) return fail(vm, XE_ERR_INVAL, "null umem/desc");
  // the pipeline is stream order: a batch on another stream waits for the ones in flight
  if (!vm->pending.empty() && vm->slots[vm->pending.back()].b.s != s)
    if (int rc = xe_sync(vm)) return rc;
  while (vm->pending.size() >= kAsyncDepth)
    if (int rc = complete_oldest(vm)) {
      vm->pending.clear();
      return rc;
    }
  if (int rc = prepare_run(vm, s)) return rc;
  void* jit = nullptr;
  bool jit_general = false;
  if (int rc = select_engine(vm, jit, jit_general)) return rc;
  const bool general = !jit || jit_general;

  const uint32_t si = vm->next_slot;
  const uint32_t ai = vm->next_snap, nai = (ai + 1) % (kAsyncDepth + 1);  // its rollback point, the next one's
  xe_vm::Slot& sl = vm->slots[si];
  if (!sl.d_aux) {  // the slot's records start zeroed; every batch epilogue zeroes them again
    if (dev_alloc((void**)&sl.d_aux, kAuxWords * 8) || dmemset(sl.d_aux, 0, kAuxWords * 8, s))
      return fail(vm, XE_ERR_DEVICE, "alloc (pipelined batch records)");
  }
  if (!sl.h_aux) {
    if (host_alloc((void**)&sl.h_aux, kAuxWords * 8) || host_device_ptr((void**)&sl.h_aux_dev, sl.h_aux))
      return fail(vm, XE_ERR_DEVICE, "alloc (pipelined batch records)");
  }
  if (!vm->d_poison) {
    if (dev_alloc((void**)&vm->d_poison, 8) || dmemset(vm->d_poison, 0, 8, s)) return fail(vm, XE_ERR_DEVICE, "alloc (poison)");
  }
  XeParams P = batch_params(vm, d_umem, umem_len, d_desc, n, d_results, d_verdicts, d_regs, sl.d_aux);
  P.mode = XE_MODE_PARALLEL;
  P.poison = vm->d_poison;
  const size_t aux_used = 16 + size_t(kRep) * P.rep_words;
  // One epilogue launch publishes the records to the pinned host copy and decides on the replay;
  // small maps are folded and snapshotted for the next batch there too, the others keep the
  // prologue snapshot and their own fold launch. This batch's rollback point: the snapshot the
  // previous batch's epilogue staged, when nothing has written the maps since.
  const bool staged = vm->staged_slot == int32_t(ai) && !vm->pending.empty() && vm->slots[vm->pending.back()].b.s == s;
  XeTailArgs A{};
  A.aux = sl.d_aux;
  A.host_aux = sl.h_aux_dev;
  A.poison = vm->d_poison;
  A.aux_words = uint32_t(aux_used);
  A.nrep = kRep;
  A.rep_words = P.rep_words;
  A.nmaps = P.nmaps;
  A.mode = vm->settings.mode;
  std::vector<const void*> src;
  std::vector<void*> dst;
  std::vector<uint64_t> words;
  std::vector<size_t> big;  // maps folded by their own launch
  for (size_t i = 1; i < vm->maps.size(); i++) {
    HostMap& m = vm->maps[i];
    for (uint32_t k : {ai, nai})
      if (!m.d_asnap[k] && dev_alloc((void**)&m.d_asnap[k], m.vals_alloc))
        return fail(vm, XE_ERR_DEVICE, "device alloc (batch snapshot)");
    const bool small = m.vals_alloc <= kTailMapBytes && A.ntail < XE_TAIL_MAPS;
    if (small) {
      XeTailMap& T = A.tail[A.ntail++];
      T.vals = (unsigned long long*)m.d_vals;
      T.rep = (unsigned long long*)m.d_rep;
      T.snap = (unsigned long long*)m.d_asnap[nai];
      T.words = m.vals_alloc / 8;
      T.stride_words = m.rep_stride / 8;
      T.nrep = m.nrep > 1 ? m.nrep : 0;
    } else {
      big.push_back(i);
    }
    if (!small || !staged) {
      src.push_back(m.d_vals);
      dst.push_back(m.d_asnap[ai]);
      words.push_back(m.vals_alloc / 8);
    }
  }
  if (jit && !P.results && !P.regs) jit = lean_kernel(vm, jit);  // verdicts only: the lean variant
  const uint32_t grid = parallel_grid(vm, jit, general, n, P.nmaps);
  if (general && ensure_arena(vm, false, grid * 256, P.gen)) return fail(vm, XE_ERR_NOMEM, "device alloc (arena)");
  if (!src.empty() && launch_prologue(src.data(), dst.data(), words.data(), uint32_t(src.size()), nullptr, 0, s))
    return fail(vm, XE_ERR_DEVICE, "prologue");
  sl.t0.rec(s);
  if ((jit ? launch_jit(jit, &P, grid, 256, s) : launch_interp(&P, grid, 256, s))) return fail(vm, XE_ERR_DEVICE, "kernel launch");
  sl.t1.rec(s);
  for (size_t i : big) {
    HostMap& m = vm->maps[i];
    if (m.nrep > 1 && fold_map(m, s))
      return fail(vm, XE_ERR_DEVICE, "replica fold");
  }
  if (launch_tail(&A, s)) return fail(vm, XE_ERR_DEVICE, "epilogue");
  sl.done.rec(s);
  vm->staged_slot = int32_t(nai);
  sl.snap = ai;
  vm->next_snap = nai;
  sl.b = xe_vm::Batch{d_umem, umem_len, d_desc, n, d_results, d_verdicts, d_regs, s, stats};
  sl.aux_used = aux_used;
  sl.nmaps = P.nmaps;
  sl.grid = grid;
  sl.engine = jit ? XE_ENGINE_JIT : XE_ENGINE_INTERP;
  vm->last_grid = grid;
  vm->pending.push_back(si);
  vm->next_slot = (si + 1) % kAsyncDepth;
  vm->delta_base = false;
  for (size_t i = 1; i < vm->maps.size(); i++) vm->maps[i].dev_dirty = true;
  return XE_OK;
}

int xe_run_batch_host(xe_vm* vm, uint8_t* umem, uint64_t umem_len, const xe_desc* desc, uint32_t n,
                      xe_result* results, uint32_t* verdicts, xe_regs* regs, xe_batch_stats* stats) {
  if (!vm) return XE_ERR_INVAL;
  if (set_device(vm->settings.device)) return fail(vm, XE_ERR_DEVICE, "hipSetDevice failed");
  xe_stream_t s = vm->stream;
  if (ensure_buf(&vm->d_umem, &vm->d_umem_cap, umem_len) || ensure_buf(&vm->d_desc, &vm->d_desc_cap, size_t(n) * 16) ||
      ensure_buf(&vm->d_res, &vm->d_res_cap, size_t(n) * sizeof(xe_result)) ||
      ensure_buf(&vm->d_ver, &vm->d_ver_cap, size_t(n) * 4) ||
      (regs && ensure_buf(&vm->d_regs, &vm->d_regs_cap, size_t(n) * sizeof(xe_regs))))
    return fail(vm, XE_ERR_DEVICE, "device alloc (batch)");
  Timer a, b;
  a.rec(s);
  if ((umem_len && h2d(vm->d_umem, umem, umem_len, s)) || (n && h2d(vm->d_desc, desc, size_t(n) * 16, s)))
    return fail(vm, XE_ERR_DEVICE, "H2D");
  int rc = xe_run_batch_device(vm, vm->d_umem, umem_len, vm->d_desc, n, results ? vm->d_res : nullptr,
                               verdicts ? vm->d_ver : nullptr, regs ? vm->d_regs : nullptr, s, stats);
  if (rc) return rc;
  if ((results && d2h(results, vm->d_res, size_t(n) * sizeof(xe_result), s)) ||
      (verdicts && d2h(verdicts, vm->d_ver, size_t(n) * 4, s)) ||
      (regs && d2h(regs, vm->d_regs, size_t(n) * sizeof(xe_regs), s)) ||
      (umem_len && may_write_packet(vm->programs[vm->entry]) && d2h(umem, vm->d_umem, umem_len, s)))
    return fail(vm, XE_ERR_DEVICE, "D2H");
  b.rec(s);
  if (dsync(s)) return fail(vm, XE_ERR_DEVICE, "sync");
  if (stats) stats->total_ms = Timer::ms(a, b);
  a.fini(); b.fini();
  return XE_OK;
}

int xe_map_dump_list(xe_vm* vm, int32_t mi, void* data, uint64_t data_cap, uint32_t* lens, uint64_t cap, uint64_t* count,
                     uint64_t* bytes) {
  HostMap* m = get_map(vm, mi);
  if (!m || (m->dkind != XE_DM_LIST && m->dkind != XE_DM_PERF)) return XE_ERR_INVAL;
  set_device(vm->settings.device);
  if (map_download(vm, *m)) return fail(vm, XE_ERR_DEVICE, "map download");
  uint64_t total = 0;
  for (auto& r : m->items) total += r.val.size();
  if (count) *count = m->items.size();
  if (bytes) *bytes = total;
  if (!data && !lens) return XE_OK;
  if (cap < m->items.size() || (data && data_cap < total)) return fail(vm, XE_ERR_INVAL, "dump buffer too small");
  uint64_t off = 0;
  for (size_t i = 0; i < m->items.size(); i++) {
    if (lens) lens[i] = uint32_t(m->items[i].val.size());
    if (data && !m->items[i].val.empty()) memcpy((uint8_t*)data + off, m->items[i].val.data(), m->items[i].val.size());
    off += m->items[i].val.size();
  }
  return XE_OK;
}

int xe_map_lru_order(xe_vm* vm, int32_t mi, void* keys, uint64_t cap, uint64_t* count) {
  HostMap* m = get_map(vm, mi);
  if (!m || m->dkind != XE_DM_LRU) return XE_ERR_INVAL;
  set_device(vm->settings.device);
  if (map_download(vm, *m)) return fail(vm, XE_ERR_DEVICE, "map download");
  if (count) *count = m->items.size();
  if (!keys) return XE_OK;
  if (cap < m->items.size()) return fail(vm, XE_ERR_INVAL, "buffer too small");
  for (size_t i = 0; i < m->items.size(); i++) {
    uint8_t* kd = (uint8_t*)keys + i * m->def.key_size;
    memset(kd, 0, m->def.key_size);
    if (!m->items[i].nil_key) memcpy(kd, m->items[i].key.data(), m->def.key_size);
  }
  return XE_OK;
}

int xe_map_push(xe_vm* vm, int32_t mi, const void* value) {
  HostMap* m = get_map(vm, mi);
  if (!m || !value || m->dkind != XE_DM_LIST) return XE_ERR_INVAL;
  set_device(vm->settings.device);
  if (map_download(vm, *m)) return fail(vm, XE_ERR_DEVICE, "map download");
  HostMap::Rec r;
  r.val.assign((const uint8_t*)value, (const uint8_t*)value + m->def.value_size);
  m->items.push_back(std::move(r));
  m->host_dirty = true;
  return XE_OK;
}

int xe_map_values_bytes(xe_vm* vm, int32_t mi, uint64_t* bytes) {
  HostMap* m = get_map(vm, mi);
  if (!m || !bytes) return XE_ERR_INVAL;
  *bytes = m->vals_alloc;
  return XE_OK;
}

int xe_map_delta(xe_vm* vm, int32_t mi, uint32_t lane, void* d_out, void* stream) {
  HostMap* m = get_map(vm, mi);
  if (!m || !d_out) return XE_ERR_INVAL;
  if (!vm->epoch_open && !vm->delta_base)
    return fail(vm, XE_ERR_INVAL, "map deltas are taken against a synchronous batch's start or a shard epoch");
  if (vm->epoch_open)
    if (int rc = xe_sync(vm)) return rc;
  set_device(vm->settings.device);
  xe_stream_t s = stream ? (xe_stream_t)stream : vm->stream;
  if (lane != 0 && lane != 1 && lane != 2 && lane != 4 && lane != 8) return XE_ERR_INVAL;
  const uint32_t dl = vm->epoch_open ? lane_of(m->ewclass) : m->lane;
  if (launch_delta(m->d_vals, vm->epoch_open ? m->d_ebase : m->d_snap, d_out, m->vals_alloc, lane ? lane : dl ? dl : 8, s) ||
      dsync(s))
    return fail(vm, XE_ERR_DEVICE, "delta");
  return XE_OK;
}

int xe_map_apply_delta(xe_vm* vm, int32_t mi, uint32_t lane, const void* d_in, void* stream) {
  if (vm) vm->staged_slot = -1;
  HostMap* m = get_map(vm, mi);
  if (!m || !d_in) return XE_ERR_INVAL;
  if (!vm->epoch_open && !vm->delta_base)
    return fail(vm, XE_ERR_INVAL, "map deltas are taken against a synchronous batch's start or a shard epoch");
  if (vm->epoch_open)
    if (int rc = xe_sync(vm)) return rc;
  set_device(vm->settings.device);
  xe_stream_t s = stream ? (xe_stream_t)stream : vm->stream;
  if (lane != 0 && lane != 1 && lane != 2 && lane != 4 && lane != 8) return XE_ERR_INVAL;
  const uint32_t dl = vm->epoch_open ? lane_of(m->ewclass) : m->lane;
  if (launch_apply_delta(m->d_vals, vm->epoch_open ? m->d_ebase : m->d_snap, d_in, m->vals_alloc, lane ? lane : dl ? dl : 8, s) ||
      dsync(s))
    return fail(vm, XE_ERR_DEVICE, "apply delta");
  m->dev_dirty = true;
  return XE_OK;
}

// Shard epochs: deltas over several batches (synchronous or pipelined) against the values at the
// epoch's start, with the footprints of every batch in between ORed together.
int xe_epoch_begin(xe_vm* vm, void* stream) {
  if (!vm) return XE_ERR_INVAL;
  if (int rc = xe_sync(vm)) return rc;
  if (set_device(vm->settings.device)) return fail(vm, XE_ERR_DEVICE, "hipSetDevice failed");
  xe_stream_t s = stream ? (xe_stream_t)stream : vm->stream;
  if (int rc = prepare_run(vm, s)) return rc;  // host-side map changes reach the device first
  std::vector<const void*> src;
  std::vector<void*> dst;
  std::vector<uint64_t> words;
  for (size_t i = 1; i < vm->maps.size(); i++) {
    HostMap& m = vm->maps[i];
    m.ewclass = 0;
    if (m.ordered()) continue;
    if (!m.d_ebase && dev_alloc((void**)&m.d_ebase, m.vals_alloc)) return fail(vm, XE_ERR_NOMEM, "device alloc (epoch base)");
    src.push_back(m.d_vals);
    dst.push_back(m.d_ebase);
    words.push_back(m.vals_alloc / 8);
  }
  if (!src.empty() && (launch_prologue(src.data(), dst.data(), words.data(), uint32_t(src.size()), nullptr, 0, s) || dsync(s)))
    return fail(vm, XE_ERR_DEVICE, "epoch snapshot");
  vm->epoch_open = true;
  vm->epoch_fp.assign(16 + 2 * (vm->maps.size() + 1), 0);
  vm->epoch_flags = 0;
  vm->epoch_seq = false;
  return XE_OK;
}

int xe_epoch_end(xe_vm* vm) {
  if (!vm) return XE_ERR_INVAL;
  if (int rc = xe_sync(vm)) return rc;
  vm->epoch_open = false;
  return XE_OK;
}

int xe_map_delta_lane(xe_vm* vm, int32_t mi, uint32_t* lane_bytes) {
  HostMap* m = get_map(vm, mi);
  if (!m || !lane_bytes) return XE_ERR_INVAL;
  *lane_bytes = vm->epoch_open ? lane_of(m->ewclass) : m->lane;
  return XE_OK;
}

int xe_footprint(xe_vm* vm, uint64_t* out, uint32_t cap_words, uint32_t* nwords) {
  if (!vm) return XE_ERR_INVAL;
  if (int rc = xe_sync(vm)) return rc;
  const uint32_t nm = uint32_t(vm->maps.size() - 1);
  const uint32_t need = 1 + 3 * nm;
  if (nwords) *nwords = need;
  if (!out) return XE_OK;
  if (cap_words < need) return XE_ERR_INVAL;
  const bool ep = vm->epoch_open;
  const uint32_t flags = ep ? vm->epoch_flags : vm->last_flags;
  const std::vector<unsigned long long>& fp = ep ? vm->epoch_fp : vm->last_fp;
  uint64_t f = ep ? XE_FPF_EPOCH : 0;
  if (flags & XE_FLAG_ORDERED) f |= XE_FPF_ORDERED;
  if (ep ? vm->epoch_seq : (vm->last_mode == XE_MODE_SEQUENTIAL || vm->last_mode == XE_MODE_KEYED)) f |= XE_FPF_SEQUENTIAL;
  // ordered maps (appends included) are never summed across shards: their lists follow packet order
  if (has_ordered_maps(vm)) f |= XE_FPF_SEQUENTIAL;
  if (flags & XE_FLAG_UNALIGNED) f |= XE_FPF_UNALIGNED;
  out[0] = f;
  for (uint32_t m = 1; m <= nm; m++) {
    const size_t r = 2 * size_t(m);
    out[1 + 3 * (m - 1)] = r < fp.size() ? fp[r] : 0;
    out[2 + 3 * (m - 1)] = r + 1 < fp.size() ? fp[r + 1] : 0;
    out[3 + 3 * (m - 1)] = ep ? vm->maps[m].ewclass : vm->maps[m].wclass;
  }
  return XE_OK;
}

int xe_shard_check(const uint64_t* fps, uint32_t ngpus, uint32_t nwords, uint32_t* lanes) {
  if (!fps || !ngpus || nwords < 1 || (nwords - 1) % 3) return XE_ERR_INVAL;
  const uint32_t nm = (nwords - 1) / 3;
  bool ok = true, epoch = false;
  for (uint32_t k = 0; k < ngpus; k++) epoch = epoch || (fps[size_t(k) * nwords] & XE_FPF_EPOCH);
  for (uint32_t m = 0; m < nm; m++) {
    uint64_t added = 0;  // fields earlier shards added to
    uint32_t wc = 0;
    for (uint32_t k = 0; k < ngpus; k++) {
      const uint64_t* f = fps + size_t(k) * nwords;
      if (f[1 + 3 * m] & added) ok = false;  // shard k read a field an earlier shard changed
      added |= f[2 + 3 * m];
      wc |= uint32_t(f[3 + 3 * m]);
    }
    // An epoch spans several batches: a shard's reads in a later batch follow every shard's adds of
    // the earlier ones in the reference's order (batch after batch, shards in order), so a read may
    // meet no other shard's adds at all.
    for (uint32_t k = 0; epoch && k < ngpus; k++) {
      uint64_t others = 0;
      for (uint32_t j = 0; j < ngpus; j++)
        if (j != k) others |= fps[size_t(j) * nwords + 2 + 3 * m];
      if (fps[size_t(k) * nwords + 1 + 3 * m] & others) ok = false;
    }
    if (wc & (wc - 1)) ok = false;  // two widths: a narrow add's carry stops at its own field
    if (lanes) lanes[m] = wc == 0u ? 0u : wc == 1u ? 1u : wc == 2u ? 2u : wc == 4u ? 4u : 8u;
  }
  for (uint32_t k = 0; k < ngpus; k++)
    if (fps[size_t(k) * nwords] & (XE_FPF_ORDERED | XE_FPF_SEQUENTIAL | XE_FPF_UNALIGNED)) ok = false;
  return ok ? 1 : 0;
}

// Ordered maps (LRU_HASH, QUEUE, STACK, PERF_EVENT_ARRAY) keep their state in element pools and list
// links, so their image is a serialisation of the host mirror in Go order (UsageList / Values /
// Events), whose length follows the contents: [u64 magic][u64 records][u64 image bytes], then per
// record {u32 nil_key, u32 key bytes, u32 value bytes, u32 0} and the key and value bytes, each padded
// to 8. xe_map_state_bytes reports the current state's image size (the exporter's size is the one
// the importer reads).
}  // extern "C"
namespace {
constexpr uint64_t kOrdImageMagic = 0x78656f7264696d67ull;  // "xeordimg"
uint64_t pad8(uint64_t v) { return (v + 7) & ~uint64_t(7); }
uint64_t ordered_image_bytes(const HostMap& m) {
  uint64_t b = 24;
  for (const HostMap::Rec& r : m.items) b += 16 + pad8(r.key.size()) + pad8(r.val.size());
  return b;
}
std::vector<uint8_t> ordered_image(const HostMap& m) {
  std::vector<uint8_t> img(ordered_image_bytes(m), 0);
  uint64_t hdr[3] = {kOrdImageMagic, m.items.size(), img.size()};
  memcpy(img.data(), hdr, 24);
  uint64_t at = 24;
  for (const HostMap::Rec& r : m.items) {
    const uint32_t rh[4] = {r.nil_key ? 1u : 0u, uint32_t(r.key.size()), uint32_t(r.val.size()), 0u};
    memcpy(&img[at], rh, 16);
    at += 16;
    if (!r.key.empty()) memcpy(&img[at], r.key.data(), r.key.size());
    at += pad8(r.key.size());
    if (!r.val.empty()) memcpy(&img[at], r.val.data(), r.val.size());
    at += pad8(r.val.size());
  }
  return img;
}
// the image of a map of the same geometry back into the host mirror; false when malformed
bool ordered_from_image(HostMap& m, const std::vector<uint8_t>& img) {
  if (img.size() < 24) return false;
  uint64_t hdr[3];
  memcpy(hdr, img.data(), 24);
  if (hdr[0] != kOrdImageMagic || hdr[2] != img.size()) return false;
  std::vector<HostMap::Rec> items;
  uint64_t at = 24;
  for (uint64_t i = 0; i < hdr[1]; i++) {
    if (at + 16 > img.size()) return false;
    uint32_t rh[4];
    memcpy(rh, &img[at], 16);
    at += 16;
    if (at + pad8(rh[1]) + pad8(rh[2]) > img.size()) return false;
    if ((m.dkind == XE_DM_LRU && !rh[0] && rh[1] != m.def.key_size) || (m.dkind != XE_DM_LRU && rh[1] != 0)) return false;
    HostMap::Rec r;
    r.nil_key = rh[0] != 0;
    r.key.assign(img.begin() + long(at), img.begin() + long(at + rh[1]));
    at += pad8(rh[1]);
    r.val.assign(img.begin() + long(at), img.begin() + long(at + rh[2]));
    at += pad8(rh[2]);
    items.push_back(std::move(r));
  }
  if (at != img.size()) return false;
  m.items = std::move(items);
  return true;
}
}  // namespace
extern "C" {

int xe_map_state_bytes(xe_vm* vm, int32_t mi, uint64_t* bytes) {
  HostMap* m = get_map(vm, mi);
  if (!m || !bytes) return XE_ERR_INVAL;
  if (m->ordered()) {
    if (set_device(vm->settings.device) || map_download(vm, *m)) return fail(vm, XE_ERR_DEVICE, "map download");
    *bytes = ordered_image_bytes(*m);
    return XE_OK;
  }
  *bytes = m->vals_alloc + (m->dkind == XE_DM_HASH ? uint64_t(m->cap + 1) * xe_hash_rwords(m->kwords) * 8 + 8 : 0);
  return XE_OK;
}

// [values][slot records][count u32, pad]: device-to-device copies on the VM's device (ordered maps:
// the serialised image above). Pipelined batches complete first (their replays rewrite the maps).
int xe_map_state_export(xe_vm* vm, int32_t mi, void* d_out, void* stream) {
  if (!vm) return XE_ERR_INVAL;
  if (int rc = xe_sync(vm)) return rc;
  HostMap* m = get_map(vm, mi);
  if (!m || !d_out) return XE_ERR_INVAL;
  set_device(vm->settings.device);
  xe_stream_t s = stream ? (xe_stream_t)stream : vm->stream;
  if (m->ordered()) {
    if (map_download(vm, *m)) return fail(vm, XE_ERR_DEVICE, "map download");
    const std::vector<uint8_t> img = ordered_image(*m);
    if (h2d(d_out, img.data(), img.size(), s) || dsync(s)) return fail(vm, XE_ERR_DEVICE, "state export");
    return XE_OK;
  }
  if (m->host_dirty && map_upload(vm, *m)) return fail(vm, XE_ERR_DEVICE, "map upload");
  uint8_t* o = (uint8_t*)d_out;
  if (d2d(o, m->d_vals, m->vals_alloc, s)) return fail(vm, XE_ERR_DEVICE, "state export");
  if (m->dkind == XE_DM_HASH) {
    const uint64_t rb = uint64_t(m->cap + 1) * xe_hash_rwords(m->kwords) * 8;
    if (d2d(o + m->vals_alloc, m->d_keys, rb, s) || d2d(o + m->vals_alloc + rb, m->d_count, 4, s))
      return fail(vm, XE_ERR_DEVICE, "state export");
  }
  if (dsync(s)) return fail(vm, XE_ERR_DEVICE, "state export");
  return XE_OK;
}

int xe_map_state_import(xe_vm* vm, int32_t mi, const void* d_in, void* stream) {
  if (!vm) return XE_ERR_INVAL;
  if (int rc = xe_sync(vm)) return rc;
  vm->staged_slot = -1;
  HostMap* m = get_map(vm, mi);
  if (!m || !d_in) return XE_ERR_INVAL;
  set_device(vm->settings.device);
  xe_stream_t s = stream ? (xe_stream_t)stream : vm->stream;
  if (m->ordered()) {
    uint64_t hdr[3] = {0, 0, 0};
    if (d2h(hdr, d_in, 24, s) || dsync(s)) return fail(vm, XE_ERR_DEVICE, "state import");
    if (hdr[0] != kOrdImageMagic || hdr[2] < 24 || hdr[2] > (uint64_t(1) << 40))
      return fail(vm, XE_ERR_INVAL, "state import: not an ordered-map image");
    std::vector<uint8_t> img(hdr[2]);
    if (d2h(img.data(), d_in, img.size(), s) || dsync(s)) return fail(vm, XE_ERR_DEVICE, "state import");
    if (!ordered_from_image(*m, img)) return fail(vm, XE_ERR_INVAL, "state import: malformed ordered-map image");
    m->host_dirty = true;  // the device copy is rebuilt from the mirror before the next run
    m->dev_dirty = false;
    return XE_OK;
  }
  if (m->host_dirty && map_upload(vm, *m)) return fail(vm, XE_ERR_DEVICE, "map upload");
  const uint8_t* in = (const uint8_t*)d_in;
  if (d2d(m->d_vals, in, m->vals_alloc, s) || d2d(m->d_snap, in, m->vals_alloc, s)) return fail(vm, XE_ERR_DEVICE, "state import");
  if (m->dkind == XE_DM_HASH) {
    const uint64_t rb = uint64_t(m->cap + 1) * xe_hash_rwords(m->kwords) * 8;
    if (d2d(m->d_keys, in + m->vals_alloc, rb, s) || d2d(m->d_count, in + m->vals_alloc + rb, 4, s))
      return fail(vm, XE_ERR_DEVICE, "state import");
    uint32_t c = 0;
    if (d2h(&c, m->d_count, 4, s)) return fail(vm, XE_ERR_DEVICE, "state import");
    if (dsync(s)) return fail(vm, XE_ERR_DEVICE, "state import");
    m->live = c;
  }
  if (dsync(s)) return fail(vm, XE_ERR_DEVICE, "state import");
  m->dev_dirty = true;
  return XE_OK;
}

int xe_debug_set_schedule(xe_vm* vm, uint32_t sched) {
  if (!vm) return XE_ERR_INVAL;
  if (int rc = xe_sync(vm)) return rc;
  vm->sched = sched;
  return XE_OK;
}

int xe_debug_set_lru_epoch(xe_vm* vm, uint64_t epoch) {
  if (!vm || epoch > kLruEpochMax) return XE_ERR_INVAL;
  if (int rc = xe_sync(vm)) return rc;
  vm->lru_epoch = epoch;
  return XE_OK;
}

int xe_debug_map_pool(xe_vm* vm, int32_t mi, uint64_t* room, uint64_t* next_id) {
  HostMap* m = get_map(vm, mi);
  if (!m || !m->ordered()) return XE_ERR_INVAL;
  if (int rc = xe_sync(vm)) return rc;
  set_device(vm->settings.device);
  if (int rc = prepare_run(vm, vm->stream)) return rc;  // the device copy exists (it is built lazily)
  uint64_t hdr[8];
  if (d2h(hdr, m->d_hdr, 64, vm->stream) || dsync(vm->stream)) return fail(vm, XE_ERR_DEVICE, "map header");
  if (room) *room = m->pool_cap;
  if (next_id) *next_id = m->dkind == XE_DM_PERF ? hdr[0] : hdr[m->dkind == XE_DM_LRU ? 3 : 2];
  return XE_OK;
}

// debug/inspection: translate raw eBPF into micro-ops (returns count, or a negative XE_ERR_*)
int xe_translate_uops(const uint64_t* insns, uint32_t n, void* out, uint32_t cap) {
  std::vector<XeUop> prog;
  std::string err;
  int rc = translate(insns, n, prog, err);
  if (rc) return rc;
  lift_rmw(prog);
  if (out && cap >= prog.size()) memcpy(out, prog.data(), prog.size() * sizeof(XeUop));
  return int(prog.size());
}

// debug: 1 if the translated program may write packet memory (drives the replay's packet snapshot)
int xe_debug_may_write_packet(const uint64_t* insns, uint32_t n) {
  std::vector<XeUop> prog;
  std::string err;
  int rc = translate(insns, n, prog, err);
  if (rc) return rc;
  return may_write_packet(prog) ? 1 : 0;
}

// ---- internal hooks for xe_multi.cpp (not part of include/xdpemu.h)
int xe_internal_vm_device(const xe_vm* vm) { return vm ? vm->settings.device : -1; }
void* xe_internal_vm_stream(xe_vm* vm) { return vm ? (void*)vm->stream : nullptr; }
int xe_internal_nmaps(const xe_vm* vm) { return vm ? int(vm->maps.size()) - 1 : -1; }
int xe_internal_may_write_packet(const xe_vm* vm) {
  if (!vm || vm->entry < 1 || vm->entry >= int32_t(vm->programs.size())) return 1;
  return may_write_packet(vm->programs[vm->entry]) ? 1 : 0;
}
int xe_internal_delta_sum(xe_vm* vm, void* acc, const void* in, uint64_t bytes, uint32_t lane) {
  set_device(vm->settings.device);
  return launch_delta_sum(acc, in, bytes, lane, vm->stream) || dsync(vm->stream) ? XE_ERR_DEVICE : XE_OK;
}
int xe_internal_alloc(xe_vm* vm, void** p, uint64_t bytes) {
  set_device(vm->settings.device);
  return dev_alloc(p, size_t(bytes)) ? XE_ERR_NOMEM : XE_OK;
}
void xe_internal_free(xe_vm* vm, void* p) {
  set_device(vm->settings.device);
  dev_free(p);
}
int xe_internal_copy(xe_vm* vm, void* dst, const void* src, uint64_t bytes) {
  set_device(vm->settings.device);
  return d2d(dst, src, size_t(bytes), vm->stream) || dsync(vm->stream) ? XE_ERR_DEVICE : XE_OK;
}

const char* xe_version(void) {
#ifdef XE_HOSTSIM
  return "xdpemu-hostsim 0.1 (CPU test build of the device logic; not the product)";
#else
  return "xdpemu 0.1 gfx950";
#endif
}

int xe_device_count(int* n) {
  if (!n) return XE_ERR_INVAL;
#ifdef XE_HOSTSIM
  *n = 0;
  return XE_OK;
#else
  return hipGetDeviceCount(n) == hipSuccess ? XE_OK : XE_ERR_DEVICE;
#endif
}

}  // extern "C"
