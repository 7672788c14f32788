// sol_c2.hip — speed of light of C2's memory shape on gfx950, with no emulation at all.
//
// Per packet exactly the algorithmic bytes of SURVEY §8(d): its 16-B descriptor (xe_desc), the rows of
// its header window that hold bytes [12, 28) (two 16-B rows, LDS-DMA like the emulator kernel), and a
// 4-B verdict store (a trivial function of the window: ethertype == IPv4). 16,777,216 back-to-back 64-B
// packets, persistent waves walking 64-packet chunks as the emulator does. Variants:
//   0 sync      descriptor -> DMA -> wait -> verdict, nothing in flight across chunks
//   1 pipe1     the emulator's pipeline: window one chunk ahead, descriptor two ahead
//   2 pipe2     window two chunks ahead (three LDS buffers), descriptor three ahead
//   3 plain1    pipe1 with plain 16-B global loads of the rows instead of LDS-DMA
// The best variant's time is the floor for the emulator kernel on this workload: what the access
// pattern itself costs, the emulation removed.
//   hipcc --offload-arch=gfx950 -O3 tools/sol_c2.hip -o tools/sol_c2 && tools/sol_c2
// C4's shape (round 6): `tools/sol_c2 1500 3` — 1,500-B packets back to back, the three rows that hold
// header bytes [12, 42) from the 16-B aligned address at or below byte 12 (the emulator's C4 window).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));
#define GP(T) __attribute__((address_space(1))) T*
#define LP(T) __attribute__((address_space(3))) T*

struct Desc {
  uint64_t addr;
  uint32_t len;
  uint32_t opt;
};

__device__ __forceinline__ void glds16(GP(const uint8_t) src, uint32_t d) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(d) : "memory");
}
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void wait_vm1() { asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); }

constexpr int ROWB = 64 * 16;  // one row for the wave

template <int V, int ROWS>
__global__ void __launch_bounds__(256) sol(const uint8_t* __restrict__ umem, const Desc* __restrict__ desc, uint32_t n,
                                           uint32_t* __restrict__ ver) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4][V == 2 ? 3 : 2][ROWS * ROWB];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nwaves = (gridDim.x * blockDim.x) >> 6;
  const uint32_t nchunks = (n + 63) / 64;
  auto dload = [&](uint32_t c, uint64_t& a) {
    const uint32_t i = c * 64 + lane;
    a = (c < nchunks && i < n) ? ((GP(const uint64_t))(desc + i))[0] : 0;
  };
  auto issue = [&](uint64_t a, int buf) {
    GP(const uint8_t) src = (GP(const uint8_t))(umem + ((a + 12) & ~uint64_t(15)));
    const uint32_t d = uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(uintptr_t(&lds[w][buf][0])))));
    for (int k = 0; k < ROWS; k++) glds16(src + 16 * k, d + k * ROWB);
  };
  auto finish = [&](uint32_t c, int buf) {
    const uint32_t i = c * 64 + lane;
    const uint8_t* row = &lds[w][buf][lane * 16];
    const uint32_t et = (uint32_t(row[12]) << 8) | row[13];
    if (i < n) ver[i] = et == 0x0800 ? 2u : 1u;
  };
  if (V == 0) {
    for (uint32_t c = wave; c < nchunks; c += nwaves) {
      uint64_t a;
      dload(c, a);
      issue(a, 0);
      wait_vm();
      finish(c, 0);
    }
  } else if (V == 1 || V == 3) {
    uint32_t c = wave;
    if (c >= nchunks) return;
    uint64_t a0, a1;
    dload(c, a0);
    dload(c + nwaves, a1);
    u4 r0[ROWS], r1[ROWS];
    int cur = 0;
    if (V == 1) issue(a0, 0);
    else for (int k = 0; k < ROWS; k++) r0[k] = *(GP(const u4))(umem + ((a0 + 12) & ~uint64_t(15)) + 16 * k);
    for (;;) {
      wait_vm();
      if (V == 3) {
        for (int k = 0; k < ROWS; k++) *(u4*)&lds[w][cur][k * ROWB + lane * 16] = r0[k];
      }
      const uint32_t c1 = c + nwaves, c2 = c1 + nwaves;
      if (c1 < nchunks) {
        if (V == 1) issue(a1, cur ^ 1);
        else for (int k = 0; k < ROWS; k++) r1[k] = *(GP(const u4))(umem + ((a1 + 12) & ~uint64_t(15)) + 16 * k);
      }
      uint64_t a2;
      dload(c2, a2);
      finish(c, cur);
      if (c1 >= nchunks) break;
      c = c1; a1 = a2; cur ^= 1;
      if (V == 3) for (int k = 0; k < ROWS; k++) r0[k] = r1[k];
    }
    wait_vm();
  } else {  // V == 2: two chunks of windows in flight
    uint32_t c = wave;
    if (c >= nchunks) return;
    uint64_t a0, a1, a2;
    dload(c, a0);
    dload(c + nwaves, a1);
    dload(c + 2 * nwaves, a2);
    wait_vm();
    issue(a0, 0);
    if (c + nwaves < nchunks) issue(a1, 1);
    int cur = 0;
    for (;;) {
      wait_vm();  // (simple form: everything issued before this point)
      const uint32_t c2 = c + 2 * nwaves, c3 = c2 + nwaves;
      if (c2 < nchunks) issue(a2, (cur + 2) % 3);
      uint64_t a3;
      dload(c3, a3);
      finish(c, cur);
      if (c + nwaves >= nchunks) break;
      c += nwaves; a2 = a3; cur = (cur + 1) % 3;
    }
    wait_vm();
  }
}

int main(int argc, char** argv) {
  const uint32_t n = 16u << 20;
  const uint32_t pkt = argc > 1 ? uint32_t(atoi(argv[1])) : 64u;
  const int rows = argc > 2 ? atoi(argv[2]) : 2;
  if (rows != 2 && rows != 3) return 2;
  const uint64_t bytes = uint64_t(n) * pkt + 64;
  std::vector<Desc> hd(n);
  for (uint32_t i = 0; i < n; i++) hd[i] = Desc{uint64_t(i) * pkt, pkt, 0};
  uint8_t* um;
  Desc* dd;
  uint32_t* ver;
  if (hipMalloc(&um, bytes) || hipMalloc(&dd, uint64_t(n) * 16) || hipMalloc(&ver, uint64_t(n) * 4)) return 1;
  (void)hipMemset(um, 0x08, bytes);
  (void)hipMemcpy(dd, hd.data(), uint64_t(n) * 16, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const double alg = double(n) * 84.0;
  for (int V = 0; V < 4; V++) {
    for (int bpc : {4, 6, 8}) {
      const uint32_t blocks = 256 * bpc;
      auto launch = [&]() {
        if (rows == 2) {
          if (V == 0) hipLaunchKernelGGL((sol<0, 2>), dim3(blocks), dim3(256), 0, 0, um, dd, n, ver);
          if (V == 1) hipLaunchKernelGGL((sol<1, 2>), dim3(blocks), dim3(256), 0, 0, um, dd, n, ver);
          if (V == 2) hipLaunchKernelGGL((sol<2, 2>), dim3(blocks), dim3(256), 0, 0, um, dd, n, ver);
          if (V == 3) hipLaunchKernelGGL((sol<3, 2>), dim3(blocks), dim3(256), 0, 0, um, dd, n, ver);
        } else {
          if (V == 0) hipLaunchKernelGGL((sol<0, 3>), dim3(blocks), dim3(256), 0, 0, um, dd, n, ver);
          if (V == 1) hipLaunchKernelGGL((sol<1, 3>), dim3(blocks), dim3(256), 0, 0, um, dd, n, ver);
          if (V == 2) hipLaunchKernelGGL((sol<2, 3>), dim3(blocks), dim3(256), 0, 0, um, dd, n, ver);
          if (V == 3) hipLaunchKernelGGL((sol<3, 3>), dim3(blocks), dim3(256), 0, 0, um, dd, n, ver);
        }
      };
      float best = 1e9;
      for (int rep = 0; rep < 12; rep++) {  // one launch at a time (idle between launches)
        (void)hipEventRecord(e0);
        launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (rep >= 2 && ms < best) best = ms;
      }
      float b2b;  // 20 launches back to back, as the bench's pipelined steps run
      (void)hipEventRecord(e0);
      for (int rep = 0; rep < 20; rep++) launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      (void)hipEventElapsedTime(&b2b, e0, e1);
      b2b /= 20;
      printf("{\"pkt\": %u, \"rows\": %d, \"variant\": %d, \"blocks_per_cu\": %d, \"best_ms\": %.4f, \"b2b_ms\": %.4f, \"alg_TBps_best\": %.3f, "
             "\"alg_TBps_b2b\": %.3f}\n", pkt, rows, V, bpc, best, b2b, alg / (best * 1e-3) / 1e12, alg / (b2b * 1e-3) / 1e12);
      fflush(stdout);
    }
  }
  return 0;
}
