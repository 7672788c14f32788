// xe_kernel.hip — gfx950 kernels of the batched eBPF/XDP emulator.
//
// xe_interp_kernel: one lane per packet (wave64), grid-stride over 64-packet chunks in parallel
// mode (software-pipelined, parallel_packets); a single lane walking the packets in order in sequential mode (exact fallback for
// order-dependent map effects). xe_delta_kernel / xe_apply_delta_kernel: u64 counter deltas for
// the multi-GPU all-reduce.
#include "xe_interp.h"

extern "C" __global__ void __launch_bounds__(256) xe_interp_kernel(XeParams P) {
  __shared__ __attribute__((aligned(16))) uint8_t hdr_lds[4 * XE_HDR_WAVE_BYTES];
  __shared__ XePend pend_lds[4];
  extern __shared__ __attribute__((aligned(16))) uint8_t xe_dyn_lds[];  // (nmaps + 1) map descriptors
  XeMem M;
  XeLane L;
  L.mem = &M;
  L.hdrbuf = (XE_LP(uint8_t))(hdr_lds + (threadIdx.x >> 6) * XE_HDR_WAVE_BYTES);
  const int lane = xe_lane();
  stage_maps(L, P, (XE_LP(XeDevMap))xe_dyn_lds);
  wave_state_init(L, P, (blockIdx.x * blockDim.x + threadIdx.x) >> 6, &pend_lds[threadIdx.x >> 6]);
  if (P.mode == XE_MODE_SEQUENTIAL) {
    if (blockIdx.x != 0 || threadIdx.x >= 64) return;
    for (uint32_t i = 0; i < P.n; i++) run_packet(L, P, i, lane == 0);
  } else {
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    parallel_packets(L, P, wave, nwaves, [&](uint32_t i, bool valid) { run_staged(L, P, i, valid); });
  }
  flush_wave_state(L, P);
}

extern "C" __global__ void xe_delta_kernel(const unsigned long long* cur, const unsigned long long* snap,
                                           unsigned long long* out, uint64_t nwords) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < nwords; i += uint64_t(gridDim.x) * blockDim.x)
    out[i] = cur[i] - snap[i];
}

extern "C" __global__ void xe_apply_delta_kernel(unsigned long long* cur, const unsigned long long* snap,
                                                 const unsigned long long* delta, uint64_t nwords) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < nwords; i += uint64_t(gridDim.x) * blockDim.x)
    cur[i] = snap[i] + delta[i];
}

// vals += sum of the replicas; replicas := 0 (only words that received adds are written)
extern "C" __global__ void xe_rep_fold_kernel(unsigned long long* vals, unsigned long long* rep, uint64_t stride_words,
                                              uint32_t nrep, uint64_t nwords) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < nwords; i += uint64_t(gridDim.x) * blockDim.x) {
    unsigned long long s = 0;
    for (uint32_t k = 0; k < nrep; k++) {
      const unsigned long long v = rep[k * stride_words + i];
      if (v) { s += v; rep[k * stride_words + i] = 0; }
    }
    if (s) vals[i] += s;
  }
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
extern "C" int xe_launch_delta(const void* cur, const void* snap, void* out, uint64_t nwords, hipStream_t s) {
  uint32_t blocks = uint32_t(nwords / 256 + 1);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(xe_delta_kernel, dim3(blocks), dim3(256), 0, s, (const unsigned long long*)cur,
                     (const unsigned long long*)snap, (unsigned long long*)out, nwords);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
extern "C" int xe_launch_rep_fold(void* vals, void* rep, uint64_t stride_words, uint32_t nrep, uint64_t nwords, hipStream_t s) {
  uint32_t blocks = uint32_t(nwords / 256 + 1);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(xe_rep_fold_kernel, dim3(blocks), dim3(256), 0, s, (unsigned long long*)vals, (unsigned long long*)rep,
                     stride_words, nrep, nwords);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
extern "C" int xe_launch_apply_delta(void* cur, const void* snap, const void* delta, uint64_t nwords, hipStream_t s) {
  uint32_t blocks = uint32_t(nwords / 256 + 1);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(xe_apply_delta_kernel, dim3(blocks), dim3(256), 0, s, (unsigned long long*)cur,
                     (const unsigned long long*)snap, (const unsigned long long*)delta, nwords);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
