// sol_c5.hip — C5's memory shape on gfx950 with no emulation, and where its map adds could go.
//
// C5 (BASELINE configs[4], per GPU): 33,554,432 back-to-back 64-B packets; per packet its 16-B
// descriptor, the header rows holding bytes [12, 42) (three 16-B rows), a 16-B flow key taken from
// them, one probe of a 2M-slot open-addressing table of 32-B records {state, key, pad} in 64-B groups
// (linear probing, 1M flows: load 0.5; 6 % of packets miss), then {pkts += 1, bytes += len} on the
// flow's 16-B value, and a 4-B verdict. Persistent waves walk 64-packet chunks (16 waves per CU); the
// next chunk's descriptors and rows are loaded while the current one runs. Variants (one process):
//   atomic    the adds as the emulator makes them: one agent-scope 8-B atomic per field, lanes 2j / 2j+1
//             carrying packet j's two fields (one memory-side request per packet)
//   none      no adds (the rest of the shape alone)
//   wgatomic  the same atomics at workgroup scope: executed in the issuing XCD's L2 — NOT correct across
//             XCDs, timed only to price an L2 atomic against a memory-side one
//   log       no atomics in the pass: each packet appends {slot, len} (8 B) to its wave's region for the
//             value's partition (slot >> 6) & 7; a second kernel applies the regions, every partition
//             by the waves of ONE XCD (an owner word per partition, claimed with the XCD id from
//             HW_REG_XCC_ID), with workgroup-scope atomics that execute in that XCD's L2
// Every variant but wgatomic is checked against the host's per-slot counts; timings are HIP events,
// best of 5 after one warm-up. One JSON line.
//   hipcc --offload-arch=gfx950 -O3 tools/sol_c5.hip -o tools/sol_c5 && tools/sol_c5
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));
#define GP(T) __attribute__((address_space(1))) T*

constexpr uint32_t kSlots = 1u << 21;   // C5: 1M flows at half load
constexpr uint32_t kFlows = 1u << 20;
constexpr uint32_t kParts = 8;          // value partitions (one per XCD)
constexpr uint32_t kBlocks = 1024;      // 256 CUs x 4 blocks of 256 threads = 16 waves per CU
constexpr uint32_t kWaves = kBlocks * 4;

struct Desc {
  uint64_t addr;
  uint32_t len;
  uint32_t opt;
};

__host__ __device__ inline uint64_t mix(uint64_t a, uint64_t b) {
  uint64_t z = a * 0x9E3779B97F4A7C15ull ^ (b + 0x632BE59BD9B4E019ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__host__ __device__ inline uint32_t part_of(uint32_t slot) { return (slot >> 6) & (kParts - 1); }

__device__ __forceinline__ u4 ld16(const void* p) { return *(GP(const u4))p; }

// the probe: the 64-B group holding the home slot, then the next groups until a match or an empty slot
__device__ __forceinline__ int64_t probe(const uint64_t* rec, uint64_t k0, uint64_t k1) {
  uint32_t idx = uint32_t(mix(k0, k1)) & (kSlots - 1);
  for (uint32_t n = 0; n < kSlots; n += 2) {
    const uint32_t g = idx & ~1u, first = idx & 1u;
    GP(const u4) r = (GP(const u4))(rec + uint64_t(g) * 4);
    u4 a, b, c, d;
    asm volatile(
        "global_load_dwordx4 %0, %4, off\n\tglobal_load_dwordx4 %1, %4, off offset:16\n\t"
        "global_load_dwordx4 %2, %4, off offset:32\n\tglobal_load_dwordx4 %3, %4, off offset:48\n\t"
        "s_waitcnt vmcnt(0)"
        : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d) : "v"(r));
    const uint64_t s0 = a.x | (uint64_t(a.y) << 32), x0 = a.z | (uint64_t(a.w) << 32), y0 = b.x | (uint64_t(b.y) << 32);
    const uint64_t s1 = c.x | (uint64_t(c.y) << 32), x1 = c.z | (uint64_t(c.w) << 32), y1 = d.x | (uint64_t(d.y) << 32);
    const bool h0 = first == 0 && (s0 & 1) && x0 == k0 && y0 == k1, e0 = first == 0 && !(s0 & 1);
    const bool h1 = (s1 & 1) && x1 == k0 && y1 == k1, e1 = !(s1 & 1);
    if (h0) return g;
    if (e0) return -1;
    if (h1) return g + 1;
    if (e1) return -1;
    idx = (g + 2) & (kSlots - 1);
  }
  return -1;
}

template <int V>  // 0 atomic, 1 none, 2 wgatomic, 3 log
__global__ void __launch_bounds__(256) pass(const uint8_t* __restrict__ umem, const Desc* __restrict__ desc, uint32_t n,
                                            const uint64_t* __restrict__ rec, unsigned long long* vals,
                                            uint32_t* __restrict__ ver, uint64_t* __restrict__ lg, uint32_t capw,
                                            uint32_t* __restrict__ lcnt) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nwaves = (gridDim.x * blockDim.x) >> 6;
  const uint32_t nchunks = (n + 63) / 64;
  uint32_t cnt[kParts] = {0};
  // prefetch: descriptor and rows of the wave's first chunk
  uint32_t c = wave;
  uint64_t a = 0;
  uint32_t len = 0;
  u4 r0 = {}, r1 = {}, r2 = {};
  auto fetch = [&](uint32_t cc, uint64_t& aa, uint32_t& ll, u4& x0, u4& x1, u4& x2) {
    const uint32_t i = cc * 64 + lane;
    if (cc < nchunks && i < n) {
      const u4 dd = ld16(desc + i);
      aa = dd.x | (uint64_t(dd.y) << 32);
      ll = dd.z;
      x0 = ld16(umem + aa);
      x1 = ld16(umem + aa + 16);
      x2 = ld16(umem + aa + 32);
    }
  };
  fetch(c, a, len, r0, r1, r2);
  for (; c < nchunks; c += nwaves) {
    const uint32_t i = c * 64 + lane;
    const bool valid = i < n;
    const u4 w0 = r0, w1 = r1, w2 = r2;
    const uint32_t l = len;
    fetch(c + nwaves, a, len, r0, r1, r2);  // the next chunk's loads in flight during this one
    // the flow key: bytes 26..41 (saddr, daddr, ports, proto) of the window
    const uint64_t k0 = (uint64_t(w1.z) >> 16) | (uint64_t(w1.w) << 16) | (uint64_t(w2.x & 0xffff) << 48);
    const uint64_t k1 = (uint64_t(w2.x) >> 16) | (uint64_t(w2.y) << 16) | (uint64_t(w2.z & 0xff) << 48);
    const bool ipv4 = (w0.w & 0xffff) == 0x0008;
    const int64_t slot = valid && ipv4 ? probe(rec, k0, k1) : -1;
    if (valid) ver[i] = ipv4 ? 2u : 1u;
    if (V == 0 || V == 2) {
      // lanes 2j / 2j+1 add packet j's two fields (two rounds for 64 packets)
#pragma unroll
      for (int half = 0; half < 2; half++) {
        const int src = half * 32 + int(lane >> 1);
        const int64_t s = __shfl(slot, src);
        const uint32_t ln = __shfl(l, src);
        if (s >= 0) {
          unsigned long long* p = vals + 2 * uint64_t(s) + (lane & 1);
          const unsigned long long v = (lane & 1) ? ln : 1ull;
          if (V == 0) __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          else __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
    } else if (V == 3) {
      const uint32_t pt = slot >= 0 ? part_of(uint32_t(slot)) : kParts;
#pragma unroll
      for (uint32_t p = 0; p < kParts; p++) {
        const uint64_t m = __ballot(pt == p);
        if (!m) continue;
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
        if (pt == p)
          __builtin_nontemporal_store(uint64_t(uint32_t(slot)) | (uint64_t(l) << 32),
                                      lg + (uint64_t(p) * nwaves + wave) * capw + cnt[p] + rank);
        cnt[p] += uint32_t(__builtin_popcountll(m));
      }
    } else {
      if (slot == 0x7fffffff) vals[0] = 0;  // keeps the probe live
    }
  }
  if (V == 3 && lane < kParts) {
    uint32_t v = 0;
#pragma unroll
    for (uint32_t p = 0; p < kParts; p++) v = lane == p ? cnt[p] : v;
    lcnt[lane * nwaves + wave] = v;
  }
}

__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 3)" : "=s"(x));
  return x;
}

// Apply the log: partition p belongs to the first XCD that claims it (owner[p]); its regions are then
// taken one per wave (next[p]) by that XCD's waves only, and their adds execute in that XCD's L2.
__global__ void __launch_bounds__(256) apply(const uint64_t* __restrict__ lg, const uint32_t* __restrict__ lcnt, uint32_t nw,
                                             uint32_t capw, unsigned long long* vals, uint32_t* owner, uint32_t* next) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t x = xcc_id();
  for (uint32_t k = 0; k < kParts; k++) {
    const uint32_t p = (x + k) % kParts;  // own partition first, then any nobody owns yet
    uint32_t o = __hip_atomic_load(owner + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (o == 0xffffffffu) {
      uint32_t want = 0xffffffffu;
      uint32_t got = 0;
      if (lane == 0) {
        __hip_atomic_compare_exchange_strong(owner + p, &want, x, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        got = want;  // the previous value: 0xffffffff = this wave claimed it
      }
      got = __shfl(got, 0);
      o = got == 0xffffffffu ? x : got;
    }
    if (o != x) continue;
    for (;;) {
      uint32_t r = 0;
      if (lane == 0) r = __hip_atomic_fetch_add(next + p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      r = __shfl(r, 0);
      if (r >= nw) break;
      const uint32_t c = lcnt[p * nw + r];
      const uint64_t* e = lg + (uint64_t(p) * nw + r) * capw;
      for (uint32_t j = lane; j < c; j += 64) {
        const uint64_t v = __builtin_nontemporal_load(e + j);
        unsigned long long* q = vals + 2 * (v & 0xffffffffull);
        __hip_atomic_fetch_add(q, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(q + 1, v >> 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
  }
}

int main() {
  const uint32_t n = 1u << 25;
  // ---- host: table of 1M random flows (linear probing), packets (94 % hits)
  std::vector<uint64_t> rec(size_t(kSlots) * 4, 0);
  std::vector<uint64_t> keys(2 * size_t(kFlows));
  uint64_t st = 12345;
  auto rnd = [&]() { st = st * 6364136223846793005ull + 1442695040888963407ull; return mix(st, st >> 17); };
  for (uint32_t f = 0; f < kFlows; f++) {
    uint64_t k0 = rnd() & 0x0000ffffffffffffull, k1 = rnd() & 0x00ffffffffffffffull;
    keys[2 * f] = k0;
    keys[2 * f + 1] = k1;
    uint32_t idx = uint32_t(mix(k0, k1)) & (kSlots - 1);
    while (rec[size_t(idx) * 4] & 1) idx = (idx + 1) & (kSlots - 1);
    rec[size_t(idx) * 4] = 1;
    rec[size_t(idx) * 4 + 1] = k0;
    rec[size_t(idx) * 4 + 2] = k1;
  }
  std::vector<uint8_t> umem(size_t(n) * 64, 0);
  std::vector<Desc> desc(n);
  std::vector<int64_t> slot_of(n);
  for (uint32_t i = 0; i < n; i++) {
    uint8_t* p = &umem[size_t(i) * 64];
    p[12] = 0x08;
    p[13] = 0x00;
    uint64_t k0, k1;
    const uint64_t r = rnd();
    if (r % 100 < 94) {
      const uint32_t f = uint32_t((r >> 8) % kFlows);
      k0 = keys[2 * f];
      k1 = keys[2 * f + 1];
    } else {
      k0 = rnd() & 0x0000ffffffffffffull;
      k1 = rnd() & 0x00ffffffffffffffull;
    }
    // bytes 26..41 hold the key (k0: 6 bytes + 2 of k1's word split as in the device extraction)
    const uint64_t w0 = k0 & 0xffffffffffffull, w1 = k1;
    for (int b = 0; b < 6; b++) p[26 + b] = uint8_t(w0 >> (8 * b));
    for (int b = 0; b < 2; b++) p[32 + b] = uint8_t((k0 >> 48) >> (8 * b));
    for (int b = 0; b < 7; b++) p[34 + b] = uint8_t(w1 >> (8 * b));
    desc[i] = Desc{uint64_t(i) * 64, 64, 0};
  }
  // the device's key extraction, restated: compute the probe result on the host for the check
  std::vector<unsigned long long> want(size_t(kSlots) * 2, 0);
  for (uint32_t i = 0; i < n; i++) {
    const uint8_t* p = &umem[size_t(i) * 64];
    uint64_t k0 = 0, k1 = 0;
    for (int b = 0; b < 8; b++) k0 |= uint64_t(p[26 + b]) << (8 * b);
    for (int b = 0; b < 7; b++) k1 |= uint64_t(p[34 + b]) << (8 * b);
    uint32_t idx = uint32_t(mix(k0, k1)) & (kSlots - 1);
    int64_t s = -1;
    while (rec[size_t(idx) * 4] & 1) {
      if (rec[size_t(idx) * 4 + 1] == k0 && rec[size_t(idx) * 4 + 2] == k1) { s = idx; break; }
      idx = (idx + 1) & (kSlots - 1);
    }
    if (s >= 0) { want[2 * s] += 1; want[2 * s + 1] += 64; }
  }
  // ---- device
  uint8_t* d_umem; Desc* d_desc; uint64_t* d_rec; unsigned long long* d_vals; uint32_t* d_ver;
  uint64_t* d_log; uint32_t* d_lcnt; uint32_t* d_own;
  const uint32_t capw = ((n + 63) / 64 / kWaves + 1) * 64;
  if (hipMalloc(&d_umem, umem.size()) || hipMalloc(&d_desc, desc.size() * sizeof(Desc)) ||
      hipMalloc(&d_rec, rec.size() * 8) || hipMalloc(&d_vals, size_t(kSlots) * 16) || hipMalloc(&d_ver, size_t(n) * 4) ||
      hipMalloc(&d_log, size_t(kParts) * kWaves * capw * 8) || hipMalloc(&d_lcnt, size_t(kParts) * kWaves * 4) ||
      hipMalloc(&d_own, 2 * kParts * 4))
    return 1;
  (void)hipMemcpy(d_umem, umem.data(), umem.size(), hipMemcpyHostToDevice);
  (void)hipMemcpy(d_desc, desc.data(), desc.size() * sizeof(Desc), hipMemcpyHostToDevice);
  (void)hipMemcpy(d_rec, rec.data(), rec.size() * 8, hipMemcpyHostToDevice);
  hipEvent_t e0, e1, e2;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1); (void)hipEventCreate(&e2);
  const dim3 grid(kBlocks), blk(256);
  auto run = [&](int v, float& t1, float& t2) {
    (void)hipMemset(d_vals, 0, size_t(kSlots) * 16);
    (void)hipMemset(d_own, 0xff, kParts * 4);
    (void)hipMemset(d_own + kParts, 0, kParts * 4);
    (void)hipEventRecord(e0, 0);
    if (v == 0) hipLaunchKernelGGL(pass<0>, grid, blk, 0, 0, d_umem, d_desc, n, d_rec, d_vals, d_ver, d_log, capw, d_lcnt);
    if (v == 1) hipLaunchKernelGGL(pass<1>, grid, blk, 0, 0, d_umem, d_desc, n, d_rec, d_vals, d_ver, d_log, capw, d_lcnt);
    if (v == 2) hipLaunchKernelGGL(pass<2>, grid, blk, 0, 0, d_umem, d_desc, n, d_rec, d_vals, d_ver, d_log, capw, d_lcnt);
    if (v == 3) hipLaunchKernelGGL(pass<3>, grid, blk, 0, 0, d_umem, d_desc, n, d_rec, d_vals, d_ver, d_log, capw, d_lcnt);
    (void)hipEventRecord(e1, 0);
    if (v == 3) hipLaunchKernelGGL(apply, dim3(2048), blk, 0, 0, d_log, d_lcnt, kWaves, capw, d_vals, d_own, d_own + kParts);
    (void)hipEventRecord(e2, 0);
    (void)hipEventSynchronize(e2);
    (void)hipEventElapsedTime(&t1, e0, e1);
    (void)hipEventElapsedTime(&t2, e1, e2);
  };
  const char* names[4] = {"atomic", "none", "wgatomic", "log"};
  float best1[4], best2[4];
  int ok[4];
  std::vector<unsigned long long> got(size_t(kSlots) * 2);
  for (int v = 0; v < 4; v++) {
    best1[v] = best2[v] = 1e30f;
    ok[v] = -1;
    for (int r = 0; r < 6; r++) {
      float t1, t2;
      run(v, t1, t2);
      if (r > 0 && t1 + t2 < best1[v] + best2[v]) { best1[v] = t1; best2[v] = t2; }
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    if (v == 0 || v == 3) {
      (void)hipMemcpy(got.data(), d_vals, got.size() * 8, hipMemcpyDeviceToHost);
      ok[v] = memcmp(got.data(), want.data(), got.size() * 8) == 0;
    }
  }
  uint32_t own[kParts];
  (void)hipMemcpy(own, d_own, sizeof own, hipMemcpyDeviceToHost);
  printf("{\"packets\": %u, \"slots\": %u, \"flows\": %u, \"grid\": [%u, 256], \"variants\": {", n, kSlots, kFlows, kBlocks);
  for (int v = 0; v < 4; v++)
    printf("%s\"%s\": {\"pass_ms\": %.4f, \"apply_ms\": %.4f, \"total_ms\": %.4f, \"exact\": %s}", v ? ", " : "", names[v],
           best1[v], best2[v], best1[v] + best2[v], ok[v] < 0 ? "null" : ok[v] ? "true" : "false");
  printf("}, \"partition_owner_xcc\": [");
  for (uint32_t p = 0; p < kParts; p++) printf("%s%u", p ? ", " : "", own[p]);
  printf("]}\n");
  return 0;
}
