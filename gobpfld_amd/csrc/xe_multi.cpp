// xe_multi.cpp — one process, N devices: xe_run_batch_multi (include/xdpemu.h).
//
// The batch is split into contiguous packet shards, shard k on vms[k] (its own device and stream).
// The reference runs the packets of all shards in one loop, in order (emulator/vm.go:110-173 per
// packet); the shards run concurrently here, so the result is made exact afterwards:
//   * xe_shard_check proves that the shards' map effects commute (only aligned single-width adds, no
//     shard reading a field an earlier shard added to, no ordered path): then every VM ends at
//     init + sum of the per-map deltas — one all-reduce per map over RCCL (xGMI) between devices;
//   * otherwise the shards are replayed in order: shard k imports the whole map state shard k-1 ended
//     with (RCCL send/recv) and runs again; the last state then goes to every VM (RCCL broadcast).
// VMs that share a device (a one-GPU test of this path) exchange through device kernels instead of
// RCCL, which refuses duplicate devices in one communicator.
#include "xe_internal.h"

#include <cstring>
#include <string>
#include <thread>
#include <vector>

#ifndef XE_HOSTSIM
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#endif

// internal hooks of xe_runtime.cpp
extern "C" int xe_internal_vm_device(const xe_vm* vm);
extern "C" void* xe_internal_vm_stream(xe_vm* vm);
extern "C" int xe_internal_nmaps(const xe_vm* vm);
extern "C" int xe_internal_may_write_packet(const xe_vm* vm);
extern "C" int xe_internal_delta_sum(xe_vm* vm, void* acc, const void* in, uint64_t bytes, uint32_t lane);
extern "C" int xe_internal_alloc(xe_vm* vm, void** p, uint64_t bytes);
extern "C" void xe_internal_free(xe_vm* vm, void* p);
extern "C" int xe_internal_copy(xe_vm* vm, void* dst, const void* src, uint64_t bytes);

struct xe_multi {
  std::vector<xe_vm*> vms;
  bool rccl = false;
#ifndef XE_HOSTSIM
  std::vector<ncclComm_t> comms;
#endif
  // per VM: one device buffer per map, sized for the larger of its delta containers and its state image
  std::vector<std::vector<void*>> buf;
  std::vector<std::vector<uint64_t>> buf_bytes;
  std::vector<void*> usnap;  // per VM: packet bytes before the first pass (in-order replay of packet writers)
  std::vector<uint64_t> usnap_bytes;
  std::string err;
};

namespace {

int mfail(xe_multi* m, int rc, const std::string& msg) {
  m->err = msg;
  return rc;
}

int ensure(xe_multi* m, size_t k, void*& p, uint64_t& have, uint64_t need) {
  if (p && have >= need) return 0;
  if (p) xe_internal_free(m->vms[k], p);
  p = nullptr;
  have = 0;
  if (xe_internal_alloc(m->vms[k], &p, need ? need : 8)) return -1;
  have = need;
  return 0;
}

#ifndef XE_HOSTSIM
ncclDataType_t container_type(uint32_t lane) {
  return lane == 1 ? ncclUint8 : lane == 8 ? ncclUint64 : ncclUint32;
}
#endif

// delta containers of a map whose value region is `bytes` long, in lanes of `lane`
uint64_t delta_bytes(uint64_t bytes, uint32_t lane) { return lane == 2 ? 2 * bytes : bytes; }

// buf[k][mi - 1] := the sum over k of the VMs' deltas of map mi (vb value bytes, db container bytes)
int reduce_sum(xe_multi* m, int mi, uint32_t lane, uint64_t vb, uint64_t db) {
  const size_t G = m->vms.size(), j = size_t(mi - 1);
  if (m->rccl) {
#ifndef XE_HOSTSIM
    const size_t cnt = size_t(db / (lane == 8 ? 8 : lane == 1 ? 1 : 4));
    if (ncclGroupStart() != ncclSuccess) return -1;
    for (size_t k = 0; k < G; k++)
      if (ncclAllReduce(m->buf[k][j], m->buf[k][j], cnt, container_type(lane), ncclSum, m->comms[k],
                        (hipStream_t)xe_internal_vm_stream(m->vms[k])) != ncclSuccess)
        return -1;
    return ncclGroupEnd() == ncclSuccess ? 0 : -1;
#else
    return -1;
#endif
  }
  for (size_t k = 1; k < G; k++)  // same device: accumulate into VM 0's buffer, then hand it to the rest
    if (xe_internal_delta_sum(m->vms[0], m->buf[0][j], m->buf[k][j], vb, lane)) return -1;
  for (size_t k = 1; k < G; k++)
    if (xe_internal_copy(m->vms[k], m->buf[k][j], m->buf[0][j], db)) return -1;
  return 0;
}

}  // namespace

extern "C" {

int xe_multi_create(xe_vm* const* vms, uint32_t ngpus, xe_multi** out) {
  if (!vms || !ngpus || !out) return XE_ERR_INVAL;
  xe_multi* m = new xe_multi();
  m->vms.assign(vms, vms + ngpus);
  std::vector<int> devs;
  for (auto* v : m->vms) {
    if (!v) { delete m; return XE_ERR_INVAL; }
    devs.push_back(xe_internal_vm_device(v));
  }
  bool distinct = ngpus > 1;
  for (size_t i = 0; i < devs.size(); i++)
    for (size_t j = i + 1; j < devs.size(); j++) distinct = distinct && devs[i] != devs[j];
#ifndef XE_HOSTSIM
  if (distinct) {
    m->comms.resize(ngpus);
    if (ncclCommInitAll(m->comms.data(), int(ngpus), devs.data()) != ncclSuccess) {
      delete m;
      return XE_ERR_DEVICE;
    }
    m->rccl = true;
  }
#else
  (void)distinct;
#endif
  m->buf.assign(ngpus, {});
  m->buf_bytes.assign(ngpus, {});
  m->usnap.assign(ngpus, nullptr);
  m->usnap_bytes.assign(ngpus, 0);
  *out = m;
  return XE_OK;
}

void xe_multi_destroy(xe_multi* m) {
  if (!m) return;
  for (size_t k = 0; k < m->vms.size(); k++) {
    for (void* p : m->buf[k]) xe_internal_free(m->vms[k], p);
    if (m->usnap[k]) xe_internal_free(m->vms[k], m->usnap[k]);
  }
#ifndef XE_HOSTSIM
  for (auto c : m->comms) ncclCommDestroy(c);
#endif
  delete m;
}

const char* xe_multi_last_error(const xe_multi* m) { return m ? m->err.c_str() : "null multi"; }

int xe_run_batch_multi(xe_multi* m, void* const* d_umem, const uint64_t* umem_len, const void* const* d_desc,
                       const uint32_t* n, void* const* d_results, void* const* d_verdicts, xe_batch_stats* stats,
                       uint32_t* replayed) {
  if (!m || !d_umem || !umem_len || !d_desc || !n) return XE_ERR_INVAL;
  const size_t G = m->vms.size();
  const int nmaps = xe_internal_nmaps(m->vms[0]);
  for (size_t k = 0; k < G; k++)
    if (xe_internal_nmaps(m->vms[k]) != nmaps) return mfail(m, XE_ERR_INVAL, "VMs differ in their map tables");
  if (replayed) *replayed = 0;
  std::vector<xe_batch_stats> st(G);
  std::vector<int> rc(G, 0);
  auto run = [&](size_t k) {
    rc[k] = xe_run_batch_device(m->vms[k], d_umem[k], umem_len[k], d_desc[k], n[k], d_results ? d_results[k] : nullptr,
                                d_verdicts ? d_verdicts[k] : nullptr, nullptr, nullptr, &st[k]);
  };
  // packet writers: keep each shard's packet bytes for a possible in-order replay
  const bool writes = xe_internal_may_write_packet(m->vms[0]) != 0;
  if (writes)
    for (size_t k = 1; k < G; k++) {
      if (ensure(m, k, m->usnap[k], m->usnap_bytes[k], umem_len[k]) ||
          xe_internal_copy(m->vms[k], m->usnap[k], d_umem[k], umem_len[k]))
        return mfail(m, XE_ERR_DEVICE, "packet snapshot");
    }
  {
    std::vector<std::thread> th;
    for (size_t k = 0; k < G; k++) th.emplace_back(run, k);
    for (auto& t : th) t.join();
  }
  for (size_t k = 0; k < G; k++)
    if (rc[k]) return mfail(m, rc[k], std::string("shard ") + std::to_string(k) + ": " + xe_last_error(m->vms[k]));

  uint32_t nw = 0;
  xe_footprint(m->vms[0], nullptr, 0, &nw);
  std::vector<uint64_t> fps(size_t(nw) * G, 0);
  for (size_t k = 0; k < G; k++) xe_footprint(m->vms[k], fps.data() + k * nw, nw, &nw);
  std::vector<uint32_t> lanes(size_t(nmaps) + 1, 0);
  const int ok = xe_shard_check(fps.data(), uint32_t(G), nw, lanes.data());
  for (size_t k = 0; k < G; k++) {
    m->buf[k].resize(size_t(nmaps), nullptr);
    m->buf_bytes[k].resize(size_t(nmaps), 0);
  }
  auto map_buf = [&](size_t k, int mi, uint64_t need) -> void* {
    if (ensure(m, k, m->buf[k][size_t(mi - 1)], m->buf_bytes[k][size_t(mi - 1)], need)) return nullptr;
    return m->buf[k][size_t(mi - 1)];
  };

  if (ok == 1) {
    // ---- commuting shards: init + sum of the deltas on every VM
    for (int mi = 1; mi <= nmaps; mi++) {
      const uint32_t lane = lanes[size_t(mi - 1)];
      if (!lane) continue;
      uint64_t vb = 0;
      xe_map_values_bytes(m->vms[0], mi, &vb);
      const uint64_t db = delta_bytes(vb, lane);
      for (size_t k = 0; k < G; k++) {
        void* b = map_buf(k, mi, db);
        if (!b || xe_map_delta(m->vms[k], mi, lane, b, nullptr)) return mfail(m, XE_ERR_DEVICE, "map delta");
      }
      // sum the deltas into every VM's buffer: one RCCL all-reduce across distinct devices, device
      // kernels when the VMs share one — the only line that differs between the two
      if (reduce_sum(m, mi, lane, vb, db)) return mfail(m, XE_ERR_DEVICE, "delta all-reduce");
      for (size_t k = 0; k < G; k++)
        if (xe_map_apply_delta(m->vms[k], mi, lane, m->buf[k][size_t(mi - 1)], nullptr))
          return mfail(m, XE_ERR_DEVICE, "apply delta");
    }
  } else {
    // ---- in-order replay: shard k starts from the state shard k-1 ended with
    if (replayed) *replayed = 1;
    std::vector<uint64_t> sb(size_t(nmaps) + 1, 0);
    auto transfer = [&](size_t from, size_t to) -> int {  // whole map state, VM `from` -> VM `to`
      for (int mi = 1; mi <= nmaps; mi++) {
        // the exporter's image size (an ordered map's image follows its contents)
        if (xe_map_state_bytes(m->vms[from], mi, &sb[size_t(mi)])) return -1;
        void* src = map_buf(from, mi, sb[size_t(mi)]);
        void* dst = map_buf(to, mi, sb[size_t(mi)]);
        if (!src || !dst || xe_map_state_export(m->vms[from], mi, src, nullptr)) return -1;
        if (m->rccl) {
#ifndef XE_HOSTSIM
          if (ncclGroupStart() != ncclSuccess) return -1;
          if (ncclSend(src, size_t(sb[size_t(mi)]), ncclUint8, int(to), m->comms[from],
                       (hipStream_t)xe_internal_vm_stream(m->vms[from])) != ncclSuccess ||
              ncclRecv(dst, size_t(sb[size_t(mi)]), ncclUint8, int(from), m->comms[to],
                       (hipStream_t)xe_internal_vm_stream(m->vms[to])) != ncclSuccess)
            return -1;
          if (ncclGroupEnd() != ncclSuccess) return -1;
#endif
        } else {
          dst = src;  // same device: import straight from the exporter's buffer
        }
        if (xe_map_state_import(m->vms[to], mi, dst, nullptr)) return -1;
      }
      return 0;
    };
    for (size_t k = 1; k < G; k++) {
      if (transfer(k - 1, k)) return mfail(m, XE_ERR_DEVICE, "state transfer");
      if (writes && xe_internal_copy(m->vms[k], d_umem[k], m->usnap[k], umem_len[k]))
        return mfail(m, XE_ERR_DEVICE, "packet restore");
      run(k);
      if (rc[k]) return mfail(m, rc[k], std::string("replay shard ") + std::to_string(k) + ": " + xe_last_error(m->vms[k]));
    }
    for (size_t k = 0; k + 1 < G; k++)
      if (transfer(G - 1, k)) return mfail(m, XE_ERR_DEVICE, "final state broadcast");
  }
  if (stats)
    for (size_t k = 0; k < G; k++) stats[k] = st[k];
  return XE_OK;
}

}  // extern "C"
