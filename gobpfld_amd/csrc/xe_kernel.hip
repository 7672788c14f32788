// xe_kernel.hip — gfx950 kernels of the batched eBPF/XDP emulator.
//
// xe_interp_kernel: the shared micro-op interpreter over the general lane model (every program: loops,
// bpf-to-bpf calls, tail calls, the ordered maps). One lane per packet (wave64), grid-stride over
// 64-packet chunks in parallel mode (software-pipelined, parallel_packets); a single lane walking the
// packets in order in sequential mode (exact fallback for order-dependent map effects). xe_delta_kernel / xe_apply_delta_kernel: u64 counter deltas for
// the multi-GPU all-reduce.
#include "xe_interp.h"

#include <hipcub/device/device_radix_sort.hpp>
#include <hipcub/device/device_scan.hpp>

extern "C" __global__ void __launch_bounds__(256) xe_interp_kernel(XeParams P) {
  __shared__ __attribute__((aligned(16))) uint8_t hdr_lds[XE_HDR_LDS_BYTES];
  __shared__ XePend pend_lds[4];
  extern __shared__ __attribute__((aligned(16))) uint8_t xe_dyn_lds[];  // (nmaps + 1) map descriptors
  XeLane L;  // general lane model: objects, frames and clones in the P.gen arena
  L.hdrbuf = (XE_LP(uint8_t))(hdr_lds + (threadIdx.x >> 6) * XE_HDR_WAVE_BYTES);
  const int lane = xe_lane();
  stage_maps(L, P, (XE_LP(XeDevMap))xe_dyn_lds);
  wave_state_init(L, P, (blockIdx.x * blockDim.x + threadIdx.x) >> 6, &pend_lds[threadIdx.x >> 6]);
  if (P.mode == XE_MODE_SEQUENTIAL) {
    if (blockIdx.x != 0 || threadIdx.x >= 64) return;
    seq_packets(L, P, [&](uint32_t i, bool valid) { run_staged(L, P, i, valid); }, [](bool) {});
  } else if (P.mode == XE_MODE_CHAIN) {
    chain_packets(L, P, blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x,
                  [&](uint32_t i, bool valid) { run_staged(L, P, i, valid); });
  } else {
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    parallel_packets(L, P, wave, nwaves, [&](uint32_t i, bool valid) { run_staged(L, P, i, valid); });
  }
  flush_wave_state(L, P);
}

// Map-value deltas for the multi-GPU reduction, lane-wise at the width of the map's adds (T): a
// narrow counter wraps at its own width, so a u64 word difference would borrow across fields.
// C is the reduction container: T itself, except u16 lanes which travel as u32 (RCCL has no 16-bit
// integer sum); the container sum is truncated back to T on apply, so it wraps exactly like T.
template <class T, class C>
__global__ void xe_delta_kernel(const T* cur, const T* snap, C* out, uint64_t n) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x)
    out[i] = C(T(cur[i] - snap[i]));
}
template <class T, class C>
__global__ void xe_apply_delta_kernel(T* cur, const T* snap, const C* delta, uint64_t n) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x)
    cur[i] = T(snap[i] + T(delta[i]));
}
// acc[i] += in[i] over containers (VMs sharing one device exchange through this instead of RCCL)
template <class C>
__global__ void xe_sum_kernel(C* acc, const C* in, uint64_t n) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x)
    acc[i] = C(acc[i] + in[i]);
}

// vals += sum of the replicas; replicas := 0 (only words that received adds are written). All nrep
// loads are issued before any store so they overlap (no store may alias a later load). HASH maps (recs != nullptr): only the words of slots that
// hold or held an entry (slot state != 0) — a replica of a never-used slot is zero, since a map add
// needs a value pointer and a lookup only returns one for a full slot — so a large, sparsely filled
// table folds its replicas at the cost of one slot-state read per value word.
extern "C" __global__ void xe_rep_fold_kernel(unsigned long long* __restrict__ vals, unsigned long long* __restrict__ rep,
                                              uint64_t stride_words, uint32_t nrep, uint64_t nwords,
                                              const unsigned long long* __restrict__ recs, uint32_t rwords, uint32_t vsize,
                                              uint32_t cap, const unsigned long long* __restrict__ lim) {
  // an LRU value pool: only the value ids handed out so far (header word 3) can hold replica adds
  if (lim) nwords = nwords < (lim[3] * vsize + 7) / 8 ? nwords : (lim[3] * vsize + 7) / 8;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < nwords; i += uint64_t(gridDim.x) * blockDim.x) {
    if (recs) {
      const uint64_t s0 = 8 * i / vsize, s1 = (8 * i + 7) / vsize;
      const bool live = (s0 <= cap && recs[s0 * rwords] != 0) || (s1 != s0 && s1 <= cap && recs[s1 * rwords] != 0);
      if (!live) continue;
    }
    unsigned long long v[16];
#pragma unroll
    for (uint32_t k = 0; k < 16; k++) v[k] = k < nrep ? rep[k * stride_words + i] : 0ull;
    unsigned long long s = 0;
#pragma unroll
    for (uint32_t k = 0; k < 16; k++) {
      s += v[k];
      if (v[k]) rep[k * stride_words + i] = 0;
    }
    if (s) vals[i] += s;
  }
}

// Run prologue in one launch: snapshot up to XE_PRO_SEGS map value regions (u64 words) and zero the
// statistics / flag words (replaces a copy per map plus a fill: each costs a launch).
#define XE_PRO_SEGS 8
struct XeProlog {
  const unsigned long long* src[XE_PRO_SEGS];
  unsigned long long* dst[XE_PRO_SEGS];
  uint64_t words[XE_PRO_SEGS];
  uint32_t nseg;
  unsigned long long* zero;
  uint64_t zero_words;
};
extern "C" __global__ void xe_prologue_kernel(XeProlog A) {
  const uint64_t tid = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x, nth = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t i = tid; i < A.zero_words; i += nth) A.zero[i] = 0;
  for (uint32_t g = 0; g < A.nseg; g++)
    for (uint64_t i = tid; i < A.words[g]; i += nth) A.dst[g][i] = A.src[g][i];
}

// Pipelined-batch epilogue (XeTailArgs, xe_internal.h): one block after the batch's kernel. A launch
// boundary orders it after every wave of the batch, so plain loads see all their adds and records.
// Thread w ORs record word w over the replicas (LDS), thread 0 decides the replay exactly as the
// synchronous run does; then the small maps are folded and snapshotted for the next batch unless an
// earlier batch is being replayed (poison set): that replay restarts from its own snapshot, which
// this slot's successor may hold (the ring wraps), and every later batch re-runs synchronously.
extern "C" __global__ void __launch_bounds__(1024) xe_tail_kernel(XeTailArgs A) {
  __shared__ unsigned long long orw[257];
  const uint32_t t = threadIdx.x, nt = blockDim.x;
  for (uint32_t w = t; w <= 256; w += nt) orw[w] = 0;
  const bool poisoned = *(volatile uint32_t*)A.poison != 0;
  __syncthreads();
  for (uint32_t i = t; i < A.aux_words; i += nt) {
    const unsigned long long v = A.aux[i];
    if (v) A.aux[i] = 0;
    A.host_aux[i] = v;
    if (i == 0) orw[256] = v;
    else if (i >= 16 && v) atomicOr(&orw[(i - 16) % A.rep_words], v);
  }
  __syncthreads();
  if (t == 0) {
    const bool replay = !poisoned && xe_replay_decision(uint32_t(orw[256]), orw, A.rep_words, A.nmaps, A.mode);
    A.host_aux[XE_AUX_DECISION] = replay ? 1ull : 0ull;
    if (replay) *A.poison = 1u;
  }
  if (poisoned) return;
  for (uint32_t f = 0; f < A.ntail; f++) {
    const XeTailMap& T = A.tail[f];
    for (uint64_t i = t; i < T.words; i += nt) {
      unsigned long long r[16];
#pragma unroll
      for (uint32_t k = 0; k < 16; k++) r[k] = k < T.nrep ? T.rep[k * T.stride_words + i] : 0ull;
      unsigned long long s = 0;
#pragma unroll
      for (uint32_t k = 0; k < 16; k++) {
        s += r[k];
        if (r[k]) T.rep[k * T.stride_words + i] = 0;
      }
      const unsigned long long v = T.vals[i] + s;
      if (s) T.vals[i] = v;
      T.snap[i] = v;
    }
  }
}
extern "C" int xe_launch_tail(const XeTailArgs* A, hipStream_t s) {
  if (A->rep_words > 256) return -1;
  hipLaunchKernelGGL(xe_tail_kernel, dim3(1), dim3(1024), 0, s, *A);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Descriptor overlap check (packet-writing programs): the reference walks the packets in order, so a
// packet whose bytes another packet of the batch also covers sees that packet's writes when it comes
// later. Parallel lanes cannot reproduce that; such a batch runs the in-order path. Exact: the
// descriptors' byte ranges [addr, addr + len) (empty or outside the UMEM: none) sorted by start
// overlap iff two neighbours do.
__global__ void xe_desc_split_kernel(const xe_desc* d, uint32_t n, uint64_t umem_len, unsigned long long* key,
                                     uint32_t* len) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t a = d[i].addr;
    uint32_t l = d[i].len;
    if (a > umem_len || uint64_t(l) > umem_len - a) l = 0;  // desc_fix: such a frame has no bytes
    key[i] = l ? a : ~0ull;
    len[i] = l;
  }
}
__global__ void xe_desc_overlap_kernel(const unsigned long long* key, const uint32_t* len, uint32_t n, uint32_t* flag) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i + 1 < n; i += uint64_t(gridDim.x) * blockDim.x)
    if (len[i] && len[i + 1] && key[i] + len[i] > key[i + 1]) *flag = 1u;
}
// scratch == nullptr: *scratch_bytes receives the size needed; otherwise *flag (device) := overlap
extern "C" int xe_launch_desc_overlap(const void* desc, uint32_t n, uint64_t umem_len, void* scratch, size_t* scratch_bytes,
                                      uint32_t* flag, hipStream_t s) {
  const size_t arr = ((size_t(n) * 8 + 255) & ~size_t(255)) * 2 + ((size_t(n) * 4 + 255) & ~size_t(255)) * 2;
  size_t tmp = 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                         (uint32_t*)nullptr, (uint32_t*)nullptr, int(n), 0, 64, s) != hipSuccess)
    return -1;
  if (!scratch) {
    *scratch_bytes = arr + tmp;
    return 0;
  }
  if (*scratch_bytes < arr + tmp) return -1;
  uint8_t* p = (uint8_t*)scratch;
  auto take = [&](size_t bytes) { uint8_t* q = p; p += (bytes + 255) & ~size_t(255); return q; };
  unsigned long long* k0 = (unsigned long long*)take(size_t(n) * 8);
  unsigned long long* k1 = (unsigned long long*)take(size_t(n) * 8);
  uint32_t* l0 = (uint32_t*)take(size_t(n) * 4);
  uint32_t* l1 = (uint32_t*)take(size_t(n) * 4);
  const uint32_t blocks = n / 256 + 1 < 4096 ? n / 256 + 1 : 4096;
  if (hipMemsetAsync(flag, 0, 4, s) != hipSuccess) return -1;
  hipLaunchKernelGGL(xe_desc_split_kernel, dim3(blocks), dim3(256), 0, s, (const xe_desc*)desc, n, umem_len, k0, l0);
  if (hipcub::DeviceRadixSort::SortPairs(p, tmp, k0, k1, l0, l1, int(n), 0, 64, s) != hipSuccess) return -1;
  hipLaunchKernelGGL(xe_desc_overlap_kernel, dim3(blocks), dim3(256), 0, s, k1, l1, n, flag);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Keyed ordered execution: the build steps between the XE_MODE_SPEC pass and the chains (xe_interp.h
// keyed_step), one grid-stride launch per step, and the sort of the packets by chain.
extern "C" __global__ void xe_keyed_kernel(XeKeyed K, const XeDevMap* maps, uint8_t* skip, uint32_t step, uint32_t items) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < items; i += uint64_t(gridDim.x) * blockDim.x)
    keyed_step(K, maps, skip, step, uint32_t(i));
}
// D keys per map (XE_KS_COUNT), and those of them a packet inserts (their first writer logged an
// insert: the key words went with the D slot, XE_KEY_VALID): block histograms in LDS, one atomic per map
// per block
extern "C" __global__ void xe_keyed_count_kernel(XeKeyed K) {
  __shared__ unsigned int hist[64], ins[64];
  if (threadIdx.x < 64) hist[threadIdx.x] = ins[threadIdx.x] = 0;
  __syncthreads();
  for (uint64_t x = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; x < K.dcap; x += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t kid = K.dkid[x];
    if (kid) {
      atomicAdd(&hist[kid >> 58], 1u);
      if (K.dkey[x * K.kw] & XE_KEY_VALID) atomicAdd(&ins[kid >> 58], 1u);
    }
  }
  __syncthreads();
  if (threadIdx.x < 64 && hist[threadIdx.x]) atomicAdd(K.dcount + threadIdx.x, hist[threadIdx.x]);
  if (threadIdx.x < 64 && ins[threadIdx.x]) atomicAdd(K.dins + threadIdx.x, ins[threadIdx.x]);
}
extern "C" int xe_launch_keyed(const XeKeyed* K, const XeDevMap* maps, uint8_t* skip, uint32_t step, uint32_t items,
                               hipStream_t s) {
  if (!items) return 0;
  if (step == XE_KS_COUNT) {
    hipLaunchKernelGGL(xe_keyed_count_kernel, dim3(1024), dim3(256), 0, s, *K);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  const uint32_t blocks = items / 256 + 1 < 8192 ? items / 256 + 1 : 8192;
  hipLaunchKernelGGL(xe_keyed_kernel, dim3(blocks), dim3(256), 0, s, *K, maps, skip, step, items);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
// (ckey, iota = 0..n-1) -> (okey, order), by chain key bits [0, end_bit); LSD radix sort is stable, so a
// chain's packets stay in packet order. scratch == nullptr: *bytes receives the scratch size.
extern "C" int xe_launch_keyed_sort(const XeKeyed* K, uint32_t n, uint32_t end_bit, void* scratch, size_t* bytes, hipStream_t s) {
  size_t tmp = 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, (const uint32_t*)nullptr, (uint32_t*)nullptr, (const uint32_t*)nullptr,
                                         (uint32_t*)nullptr, int(n), 0, int(end_bit), s) != hipSuccess)
    return -1;
  if (!scratch) {
    *bytes = tmp;
    return 0;
  }
  if (*bytes < tmp) return -1;
  return hipcub::DeviceRadixSort::SortPairs(scratch, tmp, K->ckey, K->okey, K->iota, K->order, int(n), 0, int(end_bit), s) ==
                 hipSuccess
             ? 0
             : -1;
}

// One ordered map's parallel appends put in packet order (XeAppendArgs): step 0 gathers the run's tags
// with the element ids (PERF: and sets the run's event records aside), a radix sort orders them by tag,
// step 1 writes the sorted ids into the list positions (QUEUE / STACK) or permutes the event records.
__global__ void xe_append_kernel(XeAppendArgs A, int step) {
  const uint64_t j = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j >= A.k) return;
  if (step == 0) {
    A.keys_in[j] = A.tag[A.base + j];
    A.ids_in[j] = uint32_t(A.base + j);
    if (A.perf) {
      A.rec_tmp[2 * j] = A.rec[2 * (A.base + j)];
      A.rec_tmp[2 * j + 1] = A.rec[2 * (A.base + j) + 1];
    }
    return;
  }
  const uint32_t id = A.ids_out[j];
  if (A.perf) {
    const uint64_t o = uint64_t(id) - A.base;
    A.rec[2 * (A.base + j)] = A.rec_tmp[2 * o];
    A.rec[2 * (A.base + j) + 1] = A.rec_tmp[2 * o + 1];
  } else {
    A.link[A.stack ? A.cnt0 + j : (A.head + A.cnt0 + j) % A.list_cap] = id;
  }
}

extern "C" int xe_launch_append(const XeAppendArgs* A, uint32_t end_bit, void* scratch, size_t* bytes, hipStream_t s) {
  size_t tmp = 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, (const uint64_t*)nullptr, (uint64_t*)nullptr, (const uint32_t*)nullptr,
                                         (uint32_t*)nullptr, int(A->k), 0, int(end_bit), s) != hipSuccess)
    return -1;
  if (!scratch) {
    *bytes = tmp;
    return 0;
  }
  if (*bytes < tmp) return -1;
  const uint32_t blocks = (A->k + 255) / 256;
  hipLaunchKernelGGL(xe_append_kernel, dim3(blocks), dim3(256), 0, s, *A, 0);
  if (hipGetLastError() != hipSuccess) return -1;
  if (hipcub::DeviceRadixSort::SortPairs(scratch, tmp, A->keys_in, A->keys_out, A->ids_in, A->ids_out, int(A->k), 0,
                                         int(end_bit), s) != hipSuccess)
    return -1;
  hipLaunchKernelGGL(xe_append_kernel, dim3(blocks), dim3(256), 0, s, *A, 1);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// exclusive scan of the chain-start flags (iota) into ckey: each chain's index in the compacted list
extern "C" int xe_launch_keyed_scan(const XeKeyed* K, uint32_t n, void* scratch, size_t* bytes, hipStream_t s) {
  size_t tmp = 0;
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, (const uint32_t*)nullptr, (uint32_t*)nullptr, int(n), s) != hipSuccess)
    return -1;
  if (!scratch) {
    *bytes = tmp;
    return 0;
  }
  if (*bytes < tmp) return -1;
  return hipcub::DeviceScan::ExclusiveSum(scratch, tmp, K->iota, K->ckey, int(n), s) == hipSuccess ? 0 : -1;
}

// Pops ranked in parallel (xe_runtime.cpp, list operations): mode 0 packs the count pass's flags (1 + the
// map a packet pops first) into per-slot counts, mode 1 extracts slot `arg`'s 8-bit counts for its scan,
// mode 2 sets *flag when a ranked pass's observed counts (src) differ from the ones ranked by (dst)
__global__ void xe_pop_kernel(const uint32_t* src, uint32_t* dst, uint32_t n, uint32_t mode, uint32_t arg, XePopSlots sl,
                              uint32_t* flag) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t v = src[i];
    if (mode == 0) dst[i] = v ? 1u << (8u * (sl.slot[(v - 1u) & 63u] & 3u)) : 0u;
    else if (mode == 1) dst[i] = (v >> (8u * arg)) & 0xffu;
    else if (v != dst[i]) *flag = 1u;
  }
}
extern "C" int xe_launch_pop(const uint32_t* src, uint32_t* dst, uint32_t n, uint32_t mode, uint32_t arg, XePopSlots sl,
                             uint32_t* flag, hipStream_t s) {
  const uint32_t blocks = n / 256 + 1 < 8192 ? n / 256 + 1 : 8192;
  hipLaunchKernelGGL(xe_pop_kernel, dim3(blocks), dim3(256), 0, s, src, dst, n, mode, arg, sl, flag);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// An LRU map's UsageList from its stamps (xe_runtime.cpp lru_relink): the pool's value ids sorted by
// stamp, descending, then the first cnt of them linked in that order; `renumber` also rewrites the
// stamps as their ranks from the tail (cnt .. 1: epoch 0, below every later run's stamps).
__global__ void xe_iota_kernel(uint32_t* v, uint32_t n) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) v[i] = uint32_t(i);
}
__global__ void xe_lru_link_kernel(const uint32_t* order, uint32_t cnt, uint32_t* link, uint64_t* hdr, uint64_t* tag,
                                   int renumber) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < cnt; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t v = order[i];
    if (renumber) tag[v] = cnt - i;
    link[4 * uint64_t(v)] = i ? order[i - 1] : XE_NONE;
    link[4 * uint64_t(v) + 1] = i + 1 < cnt ? order[i + 1] : XE_NONE;
    if (i == 0) hdr[0] = v;
    if (i + 1 == cnt) hdr[1] = v;
  }
}
__global__ void xe_lru_empty_kernel(uint64_t* hdr) { hdr[0] = XE_NONE; hdr[1] = XE_NONE; }
extern "C" int xe_launch_lru_relink(uint64_t* tag, uint32_t pool, uint32_t cnt, uint32_t* link, uint64_t* hdr, void* scratch,
                                    size_t* bytes, int renumber, hipStream_t s) {
  // scratch: sorted stamps (pool u64), value ids in / out (pool u32 each), then the sort's own storage
  const size_t fixed = (size_t(pool) * 16 + 255) & ~size_t(255);
  size_t tmp = 0;
  if (hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tmp, (const unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                                   (const uint32_t*)nullptr, (uint32_t*)nullptr, int(pool), 0, 64, s) != hipSuccess)
    return -1;
  if (!scratch) {
    *bytes = fixed + tmp;
    return 0;
  }
  if (*bytes < fixed + tmp || cnt > pool) return -1;
  if (!cnt || !pool) {
    if (renumber == 2) return 0;  // nothing live: no order to give
    hipLaunchKernelGGL(xe_lru_empty_kernel, dim3(1), dim3(1), 0, s, hdr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  uint8_t* b = (uint8_t*)scratch;
  unsigned long long* keys_out = (unsigned long long*)b;
  uint32_t* vin = (uint32_t*)(b + size_t(pool) * 8);
  uint32_t* vout = vin + pool;
  const uint32_t blocks = pool / 256 + 1 < 8192 ? pool / 256 + 1 : 8192;
  hipLaunchKernelGGL(xe_iota_kernel, dim3(blocks), dim3(256), 0, s, vin, pool);
  if (hipGetLastError() != hipSuccess) return -1;
  if (hipcub::DeviceRadixSort::SortPairsDescending(b + fixed, tmp, (const unsigned long long*)tag, keys_out, vin, vout, int(pool),
                                                   0, 64, s) != hipSuccess)
    return -1;
  if (renumber == 2) return hipGetLastError() == hipSuccess ? 0 : -1;  // the order only (vout)
  hipLaunchKernelGGL(xe_lru_link_kernel, dim3(blocks), dim3(256), 0, s, vout, cnt, link, hdr, tag, renumber);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// An LRU map's stamp replicas (xe_interp.h lru_touch) into its stamps, and zeroed: one u64 per value
// and replica read, the touched ones written
__global__ void xe_lru_tag_fold_kernel(uint64_t* tag, uint64_t* rep, uint32_t pool, uint32_t r, const uint64_t* hdr) {
  const uint64_t n = hdr[3] < pool ? hdr[3] : pool;  // the value ids handed out so far
  for (uint64_t v = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; v < n; v += uint64_t(gridDim.x) * blockDim.x) {
    uint64_t mx = 0;
    for (uint32_t k = 0; k < r; k++) {
      const uint64_t x = rep[k * uint64_t(pool) + v];
      if (x) {
        mx = x > mx ? x : mx;
        rep[k * uint64_t(pool) + v] = 0;
      }
    }
    if (mx > tag[v]) tag[v] = mx;
  }
}
extern "C" int xe_launch_lru_tag_fold(uint64_t* tag, uint64_t* rep, uint32_t pool, uint32_t r, const uint64_t* hdr,
                                      hipStream_t s) {
  if (!pool) return 0;
  const uint32_t blocks = pool / 256 + 1 < 8192 ? pool / 256 + 1 : 8192;
  hipLaunchKernelGGL(xe_lru_tag_fold_kernel, dim3(blocks), dim3(256), 0, s, tag, rep, pool, r, hdr);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// The one-lane replay's order log of an LRU map (xe_interp.h lru_log_push): the live values (the first
// hdr[2] of `order`, the pool sorted by stamp, descending) oldest first as {stamp, value id}, from word 8
__global__ void xe_lru_log_kernel(const uint64_t* tag, const uint32_t* order, const uint64_t* hdr, uint64_t* log) {
  const uint64_t cnt = hdr[2];
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < cnt; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t v = order[cnt - 1 - i];
    log[8 + 2 * i] = tag[v];
    log[9 + 2 * i] = v;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    log[0] = 0;
    log[1] = cnt;
    log[2] = log[3] = 0xffffffffull;  // no freed value ids (xe_interp.h lru_free_push)
  }
}
extern "C" int xe_launch_lru_log(const uint64_t* tag, uint32_t pool, const uint32_t* order, const uint64_t* hdr, uint64_t* log,
                                 hipStream_t s) {
  const uint32_t blocks = pool / 256 + 1 < 8192 ? pool / 256 + 1 : 8192;
  hipLaunchKernelGGL(xe_lru_log_kernel, dim3(blocks), dim3(256), 0, s, tag, order, hdr, log);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// keyed LRU evictions: the D table's LRU inserts sorted by (map, first inserting packet)
extern "C" int xe_launch_keyed_esort(const XeKeyed* K, void* scratch, size_t* bytes, hipStream_t s) {
  size_t tmp = 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, (const unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                         (const uint32_t*)nullptr, (uint32_t*)nullptr, int(K->dcap), 0, 64, s) != hipSuccess)
    return -1;
  if (!scratch) {
    *bytes = tmp;
    return 0;
  }
  if (*bytes < tmp) return -1;
  return hipcub::DeviceRadixSort::SortPairs(scratch, tmp, (const unsigned long long*)K->ekey, (unsigned long long*)K->ekey2,
                                            K->eval, K->eval2, int(K->dcap), 0, 64, s) == hipSuccess ? 0 : -1;
}

// host-side launchers (called from xe_runtime.cpp)
extern "C" int xe_launch_interp(const XeParams* P, uint32_t blocks, uint32_t threads, hipStream_t s) {
  hipLaunchKernelGGL(xe_interp_kernel, dim3(blocks), dim3(threads), (P->nmaps + 1) * sizeof(XeDevMap), s, *P);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
// resident 256-thread blocks per CU for the interpreter kernel (grid sizing)
extern "C" int xe_interp_occupancy(uint32_t nmaps) {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, xe_interp_kernel, 256, (nmaps + 1) * sizeof(XeDevMap)) != hipSuccess) return 0;
  return nb;
}
template <class T, class C = T>
static int launch_delta_t(const void* cur, const void* snap, void* out, uint64_t n, hipStream_t s) {
  uint32_t blocks = uint32_t(n / 256 + 1);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL((xe_delta_kernel<T, C>), dim3(blocks), dim3(256), 0, s, (const T*)cur, (const T*)snap, (C*)out, n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
template <class T, class C = T>
static int launch_apply_t(void* cur, const void* snap, const void* delta, uint64_t n, hipStream_t s) {
  uint32_t blocks = uint32_t(n / 256 + 1);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL((xe_apply_delta_kernel<T, C>), dim3(blocks), dim3(256), 0, s, (T*)cur, (const T*)snap, (const C*)delta, n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
template <class C>
static int launch_sum_t(void* acc, const void* in, uint64_t n, hipStream_t s) {
  uint32_t blocks = uint32_t(n / 256 + 1);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL((xe_sum_kernel<C>), dim3(blocks), dim3(256), 0, s, (C*)acc, (const C*)in, n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
// acc += in over the delta containers of `lane` for a value region of `bytes`
extern "C" int xe_launch_delta_sum(void* acc, const void* in, uint64_t bytes, uint32_t lane, hipStream_t s) {
  switch (lane) {
    case 1: return launch_sum_t<uint8_t>(acc, in, bytes, s);
    case 2: case 4: return launch_sum_t<uint32_t>(acc, in, bytes / lane, s);
    default: return launch_sum_t<unsigned long long>(acc, in, bytes / 8, s);
  }
}
// bytes: length of the value region (multiple of 8); lane: 1, 2, 4 or 8
extern "C" int xe_launch_delta(const void* cur, const void* snap, void* out, uint64_t bytes, uint32_t lane, hipStream_t s) {
  switch (lane) {
    case 1: return launch_delta_t<uint8_t>(cur, snap, out, bytes, s);
    case 2: return launch_delta_t<uint16_t, uint32_t>(cur, snap, out, bytes / 2, s);
    case 4: return launch_delta_t<uint32_t>(cur, snap, out, bytes / 4, s);
    default: return launch_delta_t<unsigned long long>(cur, snap, out, bytes / 8, s);
  }
}
extern "C" int xe_launch_apply_delta(void* cur, const void* snap, const void* delta, uint64_t bytes, uint32_t lane,
                                     hipStream_t s) {
  switch (lane) {
    case 1: return launch_apply_t<uint8_t>(cur, snap, delta, bytes, s);
    case 2: return launch_apply_t<uint16_t, uint32_t>(cur, snap, delta, bytes / 2, s);
    case 4: return launch_apply_t<uint32_t>(cur, snap, delta, bytes / 4, s);
    default: return launch_apply_t<unsigned long long>(cur, snap, delta, bytes / 8, s);
  }
}
extern "C" int xe_launch_prologue(const void* const* src, void* const* dst, const uint64_t* words, uint32_t nseg,
                                  void* zero, uint64_t zero_words, hipStream_t s) {
  for (uint32_t base = 0; base < nseg || base == 0; base += XE_PRO_SEGS) {
    XeProlog A{};
    A.nseg = nseg - base < XE_PRO_SEGS ? nseg - base : XE_PRO_SEGS;
    uint64_t mx = base == 0 ? zero_words : 0;
    for (uint32_t g = 0; g < A.nseg; g++) {
      A.src[g] = (const unsigned long long*)src[base + g];
      A.dst[g] = (unsigned long long*)dst[base + g];
      A.words[g] = words[base + g];
      if (A.words[g] > mx) mx = A.words[g];
    }
    A.zero = (unsigned long long*)zero;
    A.zero_words = base == 0 ? zero_words : 0;
    uint64_t blocks = (mx + 255) / 256;
    blocks = blocks < 1 ? 1 : blocks > 4096 ? 4096 : blocks;
    hipLaunchKernelGGL(xe_prologue_kernel, dim3(uint32_t(blocks)), dim3(256), 0, s, A);
    if (hipGetLastError() != hipSuccess) return -1;
    if (nseg == 0) break;
  }
  return 0;
}
extern "C" int xe_launch_rep_fold(void* vals, void* rep, uint64_t stride_words, uint32_t nrep, uint64_t nwords,
                                  const void* recs, uint32_t rwords, uint32_t vsize, uint32_t cap, const void* lim,
                                  hipStream_t s) {
  uint32_t blocks = uint32_t(nwords / 256 + 1);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(xe_rep_fold_kernel, dim3(blocks), dim3(256), 0, s, (unsigned long long*)vals, (unsigned long long*)rep,
                     stride_words, nrep, nwords, (const unsigned long long*)recs, rwords, vsize, cap,
                     (const unsigned long long*)lim);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
