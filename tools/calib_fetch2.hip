// calib_fetch2.hip — FETCH_SIZE accounting for the emulator's NON-streaming read shapes.
//
// calib_fetch.hip pins the x2 correction for wide streaming reads (16 B per lane, consecutive lanes
// on consecutive bytes). The header windows of C3/C4 (packets back to back at IMIX / 1500-B strides)
// and the hash probes of C3/C5 are sparse: each lane reads 64 B somewhere of its own. Kernels here
// request a known number of bytes in those shapes, each launched alone so one `rocprofv3 --pmc
// FETCH_SIZE` (or TCC_EA0_RDREQ_sum) pass gives the reported value per shape:
//   win1500   4M "packets" at a 1500-B stride: the 64-B window from the 16-B aligned address below
//             the packet, as 4 LDS-DMA rows (global_load_lds_dwordx4, the kernel's hdr_issue)
//   win2048   the same at a 2048-B stride (every window one aligned 64-B block)
//   rand1g    16M random 64-B blocks (4 x dwordx4 per lane, one wait; the kernel's probe group) in a
//             1 GiB table (4x the Infinity Cache)
//   rand64m   the same in a 64 MB table (C5's slot records: Infinity-Cache resident)
// Prints the requested bytes and the distinct 64-B blocks touched per kernel.
//   hipcc --offload-arch=gfx950 -O3 tools/calib_fetch2.hip -o tools/calib_fetch2
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void glds16(const unsigned char* src, unsigned d) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(d) : "memory");
}

__global__ void __launch_bounds__(256) window(const unsigned char* __restrict__ umem, uint64_t n, uint64_t stride,
                                              unsigned* out) {
  __shared__ __attribute__((aligned(16))) unsigned char buf[4 * 4 * 1024];
  const unsigned wbase = unsigned(uintptr_t(buf)) + (threadIdx.x >> 6) * 4096;
  unsigned acc = 0;
  for (uint64_t p0 = blockIdx.x * uint64_t(blockDim.x); p0 < n; p0 += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t p = p0 + threadIdx.x < n ? p0 + threadIdx.x : 0;
    const unsigned char* src = umem + ((p * stride) & ~uint64_t(15));
    const unsigned d = __builtin_amdgcn_readfirstlane(wbase);
    glds16(src, d);
    glds16(src + 16, d + 1024);
    glds16(src + 32, d + 2048);
    glds16(src + 48, d + 3072);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    acc ^= *(volatile unsigned*)(buf + (threadIdx.x >> 6) * 4096 + (threadIdx.x & 63) * 16);
  }
  if (acc == 0x9e3779b9u) out[0] = acc;
}

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void __launch_bounds__(256) random_blocks(const u4* __restrict__ tab, uint64_t nblocks, uint64_t n,
                                                     unsigned* out) {
  unsigned acc = 0;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    const u4* g = tab + (mix(i + 0x9E3779B97F4A7C15ull) % nblocks) * 4;
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

int main() {
  const uint64_t npk = 4ull << 20, nrand = 16ull << 20;
  const size_t big = size_t(1) << 30, small = size_t(64) << 20, span = npk * 2048 + 4096;
  unsigned char *umem = nullptr, *t1 = nullptr, *t2 = nullptr;
  unsigned* o = nullptr;
  if (hipMalloc(&umem, span) != hipSuccess || hipMalloc(&t1, big) != hipSuccess || hipMalloc(&t2, small) != hipSuccess ||
      hipMalloc(&o, 64) != hipSuccess)
    return 1;
  (void)hipMemset(umem, 0x5a, span);
  (void)hipMemset(t1, 0x11, big);
  (void)hipMemset(t2, 0x22, small);
  (void)hipDeviceSynchronize();
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(window, dim3(1024), dim3(256), 0, 0, umem, npk, uint64_t(1500), o);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(window, dim3(1024), dim3(256), 0, 0, umem, npk, uint64_t(2048), o);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(random_blocks, dim3(1024), dim3(256), 0, 0, (const u4*)t1, uint64_t(big / 64), nrand, o);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(random_blocks, dim3(1024), dim3(256), 0, 0, (const u4*)t2, uint64_t(small / 64), nrand, o);
    (void)hipDeviceSynchronize();
  }
  // distinct 64-B blocks of the 1500-B windows: [a & ~15, (a & ~15) + 64) touches 1 or 2 blocks
  uint64_t blocks1500 = 0;
  for (uint64_t p = 0; p < npk; p++) {
    const uint64_t lo = (p * 1500) & ~uint64_t(15), hi = lo + 63;
    blocks1500 += (hi >> 6) - (lo >> 6) + 1;
  }
  printf("{\"launch_order\": [\"win1500\", \"win2048\", \"rand1g\", \"rand64m\"], \"requested_bytes\": {\"win1500\": %llu, "
         "\"win2048\": %llu, \"rand1g\": %llu, \"rand64m\": %llu}, \"blocks64_touched\": {\"win1500\": %llu, \"win2048\": %llu}}\n",
         (unsigned long long)(npk * 64), (unsigned long long)(npk * 64), (unsigned long long)(nrand * 64),
         (unsigned long long)(nrand * 64), (unsigned long long)blocks1500, (unsigned long long)npk);
  (void)hipFree(umem);
  (void)hipFree(t1);
  (void)hipFree(t2);
  (void)hipFree(o);
  return 0;
}
