// calib_hash.hip — the memory shapes of the C5 per-flow hash workload in isolation (no emulator).
//
// 33,554,432 "packets", each mapped by a mix hash to one of 2M slots (records 32 B = {state, key
// 16 B, pad}, values 16 B = {pkts, bytes}), as xe_jit_kernel lays out a 16-B-key / 16-B-value HASH
// map with cap 2M. Kernels, one timing each (HIP events, best of 5):
//   atom_sep   two no-return 8-B atomics per packet from one lane (pkts += 1, bytes += len): the
//              emulator's shape today, 2 wave-instructions with 64 random lines each
//   atom_pair  the same 2 adds per packet, but lanes 2j / 2j+1 carry packet j's two fields, so one
//              wave-instruction holds 32 packets x 2 adjacent 8-B fields (16 B of one line)
//   atom_one   one 8-B atomic per packet (the floor of one request per packet)
//   probe_lane one lane loads its packet's whole 64-B record group (4 x dwordx4, one wait)
//   probe_rec  one lane loads only its 32-B record (2 x dwordx4)
//   probe_coop four lanes load one packet's 64-B group (1 x dwordx4 each): 16 packets per instruction
// Prints one JSON line; packets/s and memory-side requests are what the C5 statement cites.
//   hipcc --offload-arch=gfx950 -O3 tools/calib_hash.hip -o tools/calib_hash
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

constexpr uint32_t kSlots = 1u << 21;

__device__ __forceinline__ uint32_t slot_of(uint64_t i) {
  uint64_t z = i + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return uint32_t(z ^ (z >> 31)) & (kSlots - 1);
}

__global__ void __launch_bounds__(256) atom_sep(unsigned long long* vals, uint64_t n) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t s = slot_of(i);
    __hip_atomic_fetch_add(vals + 2 * uint64_t(s), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(vals + 2 * uint64_t(s) + 1, 64ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void __launch_bounds__(256) atom_pair(unsigned long long* vals, uint64_t n) {
  // thread t handles field (t & 1) of packet t / 2
  for (uint64_t t = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; t < 2 * n; t += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t s = slot_of(t >> 1);
    __hip_atomic_fetch_add(vals + 2 * uint64_t(s) + (t & 1), (t & 1) ? 64ull : 1ull, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void __launch_bounds__(256) atom_one(unsigned long long* vals, uint64_t n) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x)
    __hip_atomic_fetch_add(vals + 2 * uint64_t(slot_of(i)), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void __launch_bounds__(256) probe_lane(const u4* rec, uint64_t n, unsigned* out) {
  unsigned acc = 0;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    const u4* g = rec + uint64_t(slot_of(i) & ~1u) * 2;  // 64-B group = 2 records of 32 B
    u4 a, b, c, d;
    asm volatile(
        "global_load_dwordx4 %0, %4, off\n\tglobal_load_dwordx4 %1, %4, off offset:16\n\t"
        "global_load_dwordx4 %2, %4, off offset:32\n\tglobal_load_dwordx4 %3, %4, off offset:48\n\t"
        "s_waitcnt vmcnt(0)"
        : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d) : "v"(g));
    acc += a.x ^ b.y ^ c.z ^ d.w;
  }
  if (acc == 0x9e3779b9u) out[0] = acc;
}

__global__ void __launch_bounds__(256) probe_rec(const u4* rec, uint64_t n, unsigned* out) {
  unsigned acc = 0;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    const u4* g = rec + uint64_t(slot_of(i)) * 2;
    u4 a, b;
    asm volatile("global_load_dwordx4 %0, %2, off\n\tglobal_load_dwordx4 %1, %2, off offset:16\n\ts_waitcnt vmcnt(0)"
                 : "=&v"(a), "=&v"(b) : "v"(g));
    acc += a.x ^ b.y;
  }
  if (acc == 0x9e3779b9u) out[0] = acc;
}

__global__ void __launch_bounds__(256) probe_coop(const u4* rec, uint64_t n, unsigned* out) {
  unsigned acc = 0;
  // thread t loads quarter (t & 3) of packet t / 4's group
  for (uint64_t t = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; t < 4 * n; t += uint64_t(gridDim.x) * blockDim.x) {
    const u4* g = rec + uint64_t(slot_of(t >> 2) & ~1u) * 2 + (t & 3);
    u4 a;
    asm volatile("global_load_dwordx4 %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=&v"(a) : "v"(g));
    acc += a.x ^ a.w;
  }
  if (acc == 0x9e3779b9u) out[0] = acc;
}

int main() {
  const uint64_t n = 1ull << 25;
  unsigned long long* vals = nullptr;
  u4* rec = nullptr;
  unsigned* o = nullptr;
  if (hipMalloc(&vals, size_t(kSlots) * 16) != hipSuccess || hipMalloc(&rec, size_t(kSlots) * 32) != hipSuccess ||
      hipMalloc(&o, 64) != hipSuccess)
    return 1;
  (void)hipMemset(vals, 0, size_t(kSlots) * 16);
  (void)hipMemset(rec, 0x11, size_t(kSlots) * 32);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const dim3 grid(1024), blk(256);
  auto timeit = [&](auto launch) {
    float best = 1e30f;
    for (int r = 0; r < 6; r++) {
      (void)hipEventRecord(e0, 0);
      launch();
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (r > 0 && ms < best) best = ms;
    }
    return best;
  };
  const float t_sep = timeit([&] { hipLaunchKernelGGL(atom_sep, grid, blk, 0, 0, vals, n); });
  const float t_pair = timeit([&] { hipLaunchKernelGGL(atom_pair, grid, blk, 0, 0, vals, n); });
  const float t_one = timeit([&] { hipLaunchKernelGGL(atom_one, grid, blk, 0, 0, vals, n); });
  const float t_lane = timeit([&] { hipLaunchKernelGGL(probe_lane, grid, blk, 0, 0, rec, n, o); });
  const float t_rec = timeit([&] { hipLaunchKernelGGL(probe_rec, grid, blk, 0, 0, rec, n, o); });
  const float t_coop = timeit([&] { hipLaunchKernelGGL(probe_coop, grid, blk, 0, 0, rec, n, o); });
  // 2x the adds of every timed launch landed: check one slot-independent invariant (sum of pkts)
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("{\"packets\": %llu, \"slots\": %u, \"grid\": [1024, 256], \"best_ms\": {\"atom_sep\": %.4f, \"atom_pair\": %.4f, "
         "\"atom_one\": %.4f, \"probe_lane\": %.4f, \"probe_rec\": %.4f, \"probe_coop\": %.4f}, "
         "\"g_atomics_per_s\": {\"atom_sep\": %.2f, \"atom_pair\": %.2f, \"atom_one\": %.2f}}\n",
         (unsigned long long)n, kSlots, t_sep, t_pair, t_one, t_lane, t_rec, t_coop, 2.0 * n / t_sep / 1e6,
         2.0 * n / t_pair / 1e6, 1.0 * n / t_one / 1e6);
  (void)hipFree(vals);
  (void)hipFree(rec);
  (void)hipFree(o);
  return 0;
}
