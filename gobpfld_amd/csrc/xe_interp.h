// xe_interp.h — the batched eBPF/XDP interpreter core.
//
// One lane interprets one packet. The 64 lanes of a wave share one micro-op stream: each step the
// wave picks the minimum PC among its running lanes (ballot + readlane; uniform fast path), fetches
// that micro-op with a scalar load and executes it on the lanes sitting at that PC. Forward branches
// dominate XDP programs, so diverged lanes re-converge at join points.
//
// Register/memory model — an exact encoding of gobpfld's object model (emulator/registers.go,
// emulator/memory.go):
//   * R0..R10 are {value (i64), memory handle (u32), tag (kind | readonly | alias id)}.
//   * Objects stored in a ValueMemory (the 24-byte xdp_md ctx, 256-byte stack frames, clones of
//     either) live in a per-lane object table; ValueMemory bytes hold object ids (0 = nil).
//   * LDX from a ValueMemory makes the register alias the stored object (emulator/memory.go:37-52,
//     emulator/inst_load.go:112); in-place ALU ops on an aliased register update the object and
//     every other register aliasing it, exactly like mutating the shared Go object.
//
// Two lane models share every handler below:
//   * fields model (XE_MEM_FIELDS, per-program kernels of programs that provably fit): the object
//     table, frame 0 and the ctx are named fields that fold into VGPRs — the fast path;
//   * general model (XE_GEN, everything else: loops, > 57 live objects, bpf-to-bpf calls with the
//     frames 1..7 and the Registers.Clone deep copies they make, tail calls, nil registers, the
//     LRU / queue / stack / perf maps): the same objects in a per-lane device arena (XeGen) with
//     mark-sweep collection; running out of arena is never a packet status — the host replays the
//     batch in order with a larger arena.
//
// Maps: ARRAY memory and HASH slot values are device-global. In parallel mode only commutative map
// effects are executed (atomic adds); a lane that would perform a non-atomic map write aborts the
// batch (XE_FLAG_ORDERED) and the host re-runs it in exact packet order (sequential mode). Lanes
// record read / atomic footprints per map so the host can verify order-independence.
//
// The same source builds the gfx950 kernels (xe_kernel.hip, per-program kernels via xe_jit.cpp) and,
// with XE_HOSTSIM, a wave-size-1 host simulation used only by CPU tests to exercise this logic.
#pragma once
#include "xe_internal.h"

// XE_UNIFORM: the scalar form of the one-lane replay (a per-program kernel variant, xe_jit.cpp
// XE_JV_SEQ). Every lane of the one wave runs the same packet with the same state, so the lane state is
// wave-uniform: loads are read back with readfirstlane and the arithmetic and branches that follow run
// on the scalar unit (one SALU instruction per cycle and SCC branches instead of wave64 VALU at four
// cycles and EXEC-masked regions); an atomic is issued by lane 0 alone and its result broadcast.
#ifndef XE_UNIFORM
#define XE_UNIFORM 0
#endif

#if defined(__HIPCC__)
#define XE_DEV __device__ __forceinline__
#define XE_WAVE 64
typedef unsigned int xe_u4 __attribute__((ext_vector_type(4)));
XE_DEV unsigned long long xe_ballot(bool p) { return __ballot(p); }
XE_DEV int xe_readfirst(int v) { return __builtin_amdgcn_readfirstlane(v); }
XE_DEV int xe_readlane(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
XE_DEV uint64_t xe_readlane64(uint64_t v, int l) {
  return uint64_t(uint32_t(__builtin_amdgcn_readlane(int(uint32_t(v)), l))) |
         (uint64_t(uint32_t(__builtin_amdgcn_readlane(int(uint32_t(v >> 32)), l))) << 32);
}
XE_DEV int xe_lane() { return __lane_id(); }
// force a loaded value to be materialised at this point (its s_waitcnt lands here)
XE_DEV void xe_pin(uint64_t& x) { asm volatile("" : "+v"(x)); }
// Global-memory pointers (packets, maps, replicas, flags) reach the kernel through memory, so the
// compiler sees generic pointers and would emit flat instructions; XE_GP casts them to the global
// address space (global_load / global_atomic, vmcnt-only waits).
#define XE_GP(T) __attribute__((address_space(1))) T*
#define XE_LP(T) __attribute__((address_space(3))) T*
// wave-uniform copies of a value every lane holds (XE_UNIFORM); identity otherwise
XE_DEV uint32_t xe_uni32(uint32_t v) { return XE_UNIFORM ? uint32_t(__builtin_amdgcn_readfirstlane(int(v))) : v; }
XE_DEV uint64_t xe_uni64(uint64_t v) {
  if (!XE_UNIFORM) return v;
  return uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(v))))) |
         (uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(v >> 32))))) << 32);
}
// an atomic issued once per wave in XE_UNIFORM (by lane 0, its result broadcast), by every lane otherwise
#define XE_ONCE(T, expr)                                  \
  do {                                                    \
    if (!XE_UNIFORM) return expr;                         \
    T r_ = 0;                                             \
    if (__lane_id() == 0) r_ = expr;                      \
    return (T)(xe_uni64(uint64_t(r_)));                   \
  } while (0)
#define XE_ONCE_VOID(stmt)                                \
  do {                                                    \
    if (!XE_UNIFORM || __lane_id() == 0) stmt;            \
  } while (0)
XE_DEV unsigned long long xe_atomic_add64(unsigned long long* p, unsigned long long v) {
  XE_ONCE(unsigned long long, __hip_atomic_fetch_add((XE_GP(unsigned long long))p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
XE_DEV unsigned int xe_atomic_cas32_(unsigned int* p, unsigned int c, unsigned int v) {
  __hip_atomic_compare_exchange_strong((XE_GP(unsigned int))p, &c, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
  return c;
}
XE_DEV unsigned int xe_atomic_cas32(unsigned int* p, unsigned int c, unsigned int v) {
  XE_ONCE(unsigned int, xe_atomic_cas32_(p, c, v));
}
XE_DEV void xe_atomic_or32(unsigned int* p, unsigned int v) {
  XE_ONCE_VOID(__hip_atomic_fetch_or((XE_GP(unsigned int))p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
XE_DEV void xe_atomic_or64(unsigned long long* p, unsigned long long v) {
  XE_ONCE_VOID(__hip_atomic_fetch_or((XE_GP(unsigned long long))p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
XE_DEV void xe_atomic_max64(unsigned long long* p, unsigned long long v) {
  XE_ONCE_VOID(__hip_atomic_fetch_max((XE_GP(unsigned long long))p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
XE_DEV unsigned int xe_atomic_add32(unsigned int* p, unsigned int v) {
  XE_ONCE(unsigned int, __hip_atomic_fetch_add((XE_GP(unsigned int))p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
XE_DEV unsigned int xe_load_relaxed32(unsigned int* p) {
  return xe_uni32(__hip_atomic_load((XE_GP(unsigned int))p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
XE_DEV unsigned long long xe_atomic_cas64_(unsigned long long* p, unsigned long long c, unsigned long long v) {
  __hip_atomic_compare_exchange_strong((XE_GP(unsigned long long))p, &c, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
  return c;
}
XE_DEV unsigned long long xe_atomic_cas64(unsigned long long* p, unsigned long long c, unsigned long long v) {
  XE_ONCE(unsigned long long, xe_atomic_cas64_(p, c, v));
}
XE_DEV unsigned int xe_atomic_min32(unsigned int* p, unsigned int v) {
  XE_ONCE(unsigned int, __hip_atomic_fetch_min((XE_GP(unsigned int))p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
XE_DEV unsigned long long xe_load_relaxed64(unsigned long long* p) {
  return xe_uni64(__hip_atomic_load((XE_GP(unsigned long long))p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
XE_DEV void xe_atomic_max32(unsigned int* p, unsigned int v) {
  XE_ONCE_VOID(__hip_atomic_fetch_max((XE_GP(unsigned int))p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
XE_DEV uint64_t xe_lanemask_lt() { return (1ull << __lane_id()) - 1ull; }
XE_DEV uint32_t xe_shfl32(uint32_t v, int l) { return uint32_t(__shfl(int(v), l)); }
#else
#define XE_DEV static inline
#define XE_WAVE 1
struct xe_u4 {
  unsigned int v[4];
  unsigned int operator[](int k) const { return v[k]; }
};
#define XE_GP(T) T*
#define XE_LP(T) T*
XE_DEV unsigned long long xe_ballot(bool p) { return p ? 1ull : 0ull; }
XE_DEV int xe_readfirst(int v) { return v; }
XE_DEV int xe_readlane(int v, int) { return v; }
XE_DEV uint64_t xe_readlane64(uint64_t v, int) { return v; }
XE_DEV int xe_lane() { return 0; }
XE_DEV void xe_pin(uint64_t&) {}
XE_DEV uint32_t xe_uni32(uint32_t v) { return v; }
XE_DEV uint64_t xe_uni64(uint64_t v) { return v; }
XE_DEV unsigned long long xe_atomic_add64(unsigned long long* p, unsigned long long v) { return __atomic_fetch_add(p, v, __ATOMIC_RELAXED); }
XE_DEV unsigned int xe_atomic_cas32(unsigned int* p, unsigned int c, unsigned int v) { __atomic_compare_exchange_n(p, &c, v, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED); return c; }
XE_DEV void xe_atomic_or32(unsigned int* p, unsigned int v) { __atomic_fetch_or(p, v, __ATOMIC_RELAXED); }
XE_DEV void xe_atomic_or64(unsigned long long* p, unsigned long long v) { __atomic_fetch_or(p, v, __ATOMIC_RELAXED); }
XE_DEV void xe_atomic_max64(unsigned long long* p, unsigned long long v) {
  unsigned long long c = __atomic_load_n(p, __ATOMIC_RELAXED);
  while (c < v && !__atomic_compare_exchange_n(p, &c, v, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {}
}
XE_DEV unsigned int xe_atomic_add32(unsigned int* p, unsigned int v) { return __atomic_fetch_add(p, v, __ATOMIC_RELAXED); }
XE_DEV unsigned int xe_load_relaxed32(unsigned int* p) { return __atomic_load_n(p, __ATOMIC_RELAXED); }
XE_DEV unsigned long long xe_atomic_cas64(unsigned long long* p, unsigned long long c, unsigned long long v) {
  __atomic_compare_exchange_n(p, &c, v, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED);
  return c;
}
XE_DEV unsigned int xe_atomic_min32(unsigned int* p, unsigned int v) {
  unsigned int o = __atomic_load_n(p, __ATOMIC_RELAXED);
  while (v < o && !__atomic_compare_exchange_n(p, &o, v, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {}
  return o;
}
XE_DEV unsigned long long xe_load_relaxed64(unsigned long long* p) { return __atomic_load_n(p, __ATOMIC_RELAXED); }
XE_DEV void xe_atomic_max32(unsigned int* p, unsigned int v) {
  unsigned int o = __atomic_load_n(p, __ATOMIC_RELAXED);
  while (o < v && !__atomic_compare_exchange_n(p, &o, v, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {}
}
XE_DEV uint64_t xe_lanemask_lt() { return 0; }
XE_DEV uint32_t xe_shfl32(uint32_t v, int) { return v; }
#endif

// Wave-aggregated counters: same-address atomics serialise at the memory side, so the lanes of a wave
// that bump one counter do it with one atomic. Call with every active lane (want: this lane counts).
// Returns this lane's index among the wave's counting lanes (offset from the old counter value).
XE_DEV uint32_t xe_wave_alloc(unsigned int* counter, bool want) {
  const uint64_t m = xe_ballot(want);
  if (!m) return 0;
  const int leader = __builtin_ctzll(m);
  uint32_t base = 0;
  if (xe_lane() == leader) base = xe_atomic_add32(counter, uint32_t(__builtin_popcountll(m)));
  base = xe_shfl32(base, leader);
  return base + uint32_t(__builtin_popcountll(m & xe_lanemask_lt()));
}
// the same with a counter per lane: lanes grouped by counter address, one atomic per address per wave
XE_DEV uint32_t xe_wave_alloc_at(unsigned int* p, bool want) {
  uint64_t m = xe_ballot(want);
  const uint64_t a = uint64_t(uintptr_t(p));
  uint32_t mine = 0;
  while (m) {
    const int leader = __builtin_ctzll(m);
    const uint64_t la = uint64_t(xe_shfl32(uint32_t(a), leader)) | (uint64_t(xe_shfl32(uint32_t(a >> 32), leader)) << 32);
    const uint64_t same = m & xe_ballot(a == la);
    uint32_t base = 0;
    if (xe_lane() == leader) base = xe_atomic_add32(p, uint32_t(__builtin_popcountll(same)));
    base = xe_shfl32(base, leader);
    if ((same >> xe_lane()) & 1ull) mine = base + uint32_t(__builtin_popcountll(same & xe_lanemask_lt()));
    m &= ~same;
  }
  return mine;
}
// *p += 1 for every lane with want, lanes grouped by counter address (one atomic per address per wave)
XE_DEV void xe_wave_count(unsigned int* p, bool want) {
  uint64_t m = xe_ballot(want);
  const uint64_t a = uint64_t(uintptr_t(p));
  while (m) {
    const int leader = __builtin_ctzll(m);
    const uint64_t la = uint64_t(xe_shfl32(uint32_t(a), leader)) | (uint64_t(xe_shfl32(uint32_t(a >> 32), leader)) << 32);
    const uint64_t same = m & xe_ballot(a == la);
    if (xe_lane() == leader) xe_atomic_add32(p, uint32_t(__builtin_popcountll(same)));
    m &= ~same;
  }
}

// per-packet result / register records (xe_result, xe_regs); 0: a verdict-only kernel variant
#ifndef XE_RECORDS
#define XE_RECORDS 1
#endif

#if defined(XE_MEM_FIELDS)
#define XE_GEN 0
#else
#define XE_GEN 1
#endif
// Rare, large paths of the general model stay out of line (collection, clones, calls, ordered maps),
// so the interpreter's dispatch loop keeps its registers.
#if defined(__HIPCC__)
#define XE_COLD __device__ __attribute__((noinline))
#else
#define XE_COLD static
#endif

// map kinds present in the VM (the per-program kernel sets these from the VM's maps, so helper paths
// for absent kinds are compiled out; the interpreter keeps all)
#ifndef XE_HAS_ARRAY
#define XE_HAS_ARRAY 1
#endif
#ifndef XE_HAS_HASH
#define XE_HAS_HASH 1
#endif
#if !XE_GEN
#undef XE_HAS_ORDERED
#if defined(XE_FIELDS_LRU) && XE_FIELDS_LRU
#define XE_HAS_ORDERED 1  // the fields model over LRU_HASH maps (xe_jit.cpp lru_static: no queue / stack / perf)
#else
#define XE_HAS_ORDERED 0  // LRU / queue / stack / perf maps and their helpers: otherwise general model only
#endif
#elif !defined(XE_HAS_ORDERED)
#define XE_HAS_ORDERED 1
#endif
// The VM's helper table (host / nil entries, xe_set_helper) and the instruction trace (xe_trace_config)
// exist in the interpreter kernel (and the host simulation) only: the runtime does not pick a
// per-program kernel while either is in use.
#if XE_GEN && !defined(__HIPCC_RTC__)
#define XE_HELPER_TABLE 1
#define XE_TRACE 1
#else
#define XE_HELPER_TABLE 0
#define XE_TRACE 0
#endif

// Deferred commit (lane_commit, parallel_packets): a chunk's verdict stores and paired-add flush are
// issued after the next chunk's prefetch instead of at the end of the chunk. The prefetch wait at the
// top of every chunk is a vmcnt(0) (it must cover the LDS-DMA the compiler does not track): issued at
// the end of the chunk, those stores and atomics put their completion latency on that wait.
#ifndef XE_DEFER_COMMIT
#define XE_DEFER_COMMIT 1
#endif

// Paired deferral of 8-byte map adds (pend_add / pend_flush): the per-program kernel enables it when
// a packet can make more than one such add; the interpreter keeps it on.
// Committer wave (XE_COMMITTER, parallel mode, programs with paired adds): wave 3 of each block issues
// the map-add atomics of waves 0..2, which hand their paired blocks over through an LDS ring. vmcnt counts
// loads, stores and atomics together in issue order, so a wave that issues its own atomics waits for them
// at its next header / probe wait (C5: the adds cost 0.63 of 2.04 ms, profiles/r5/c5_ab.json); the
// committer never loads, so nothing waits on them but the committer itself.
#if !defined(XE_COMMITTER) || !defined(__HIPCC__)
#undef XE_COMMITTER
#define XE_COMMITTER 0
#endif
#ifndef XE_PAIR_ADDS
#define XE_PAIR_ADDS 1
#endif
#if XE_COMMITTER && !XE_PAIR_ADDS
#undef XE_COMMITTER
#define XE_COMMITTER 0
#endif

// Keyed ordered execution (XE_MODE_SPEC / XE_MODE_CHAIN, xe_internal.h): compiled into the interpreter
// and the host simulation; a per-program kernel builds it only into its keyed variant, so the kernel
// of the parallel fast path carries none of its registers.
#ifndef XE_KEYED
#define XE_KEYED 1
#endif

// status histogram with one ballot for an all-OK chunk; the skip mask in parallel passes (A/B knobs)
#ifndef XE_HIST_FAST
#define XE_HIST_FAST 1
#endif
#ifndef XE_SKIP_MASK
#define XE_SKIP_MASK 1
#endif

// maps whose read / atomic footprints a lane keeps in registers (the rest OR straight into the wave's
// record); a per-program kernel sets it to the VM's map count
#ifndef XE_FP_MAPS
#define XE_FP_MAPS 4
#endif

// Register class masks: what a register may hold at an instruction, computed by the per-program
// kernel generator (xe_jit.cpp, a forward union dataflow over the program). Handlers take the mask
// of the registers they dereference and skip the branches of impossible classes; the interpreter
// passes XE_CM_ALL. XE_CM_ALIAS: the register may alias an object stored in a ValueMemory.
#define XE_CM_IMM 1u
#define XE_CM_PKT 2u
#define XE_CM_CTX 4u
#define XE_CM_STACK 8u
#define XE_CM_ARRAY 16u
#define XE_CM_HASH 32u
#define XE_CM_ALIAS 64u
#define XE_CM_VM (XE_CM_CTX | XE_CM_STACK)
#define XE_CM_MAPS (XE_CM_ARRAY | XE_CM_HASH)
#define XE_CM_ALL 127u

// Packet header window staged in LDS per lane (the first 64 bytes are the hot bytes).
// The window covers the packet bytes [XE_HDR_LO, XE_HDR_HI) a program can read: the per-program
// generator derives them from a packet-offset interval analysis (xe_jit.cpp packet_read_range), the
// shared interpreter keeps [0, 64). It is fetched by LDS-DMA (global_load_lds_dwordx4: no VGPR
// destination) from the 16-byte aligned address at or below packet byte XE_HDR_LO, as up to
// XE_HDR_ROWS rows of 16 bytes per lane — only the rows that hold bytes of [XE_HDR_LO, min(len,
// XE_HDR_HI)), so a program that reads 30 header bytes moves one or two 64-B blocks, not always two;
// one DMA instruction writes one row for the whole wave, lane-linear (row k of lane l at
// k * XE_HDR_ROW + l * 16). A lane's logical byte b lives at physical byte b + hsh of its rows
// (hsh = ((addr + XE_HDR_LO) & 15) - XE_HDR_LO). Reads outside the window go to HBM, so the window
// bounds only decide speed, never results.
// Two such buffers per wave: the next chunk's window is in flight while the current one executes.
#ifndef XE_HDR_LO
#define XE_HDR_LO 0
#endif
#ifndef XE_HDR_HI
#define XE_HDR_HI 64
#endif
#define XE_HDR_SPAN_ROWS ((XE_HDR_HI - XE_HDR_LO + 30) / 16)  // rows for the span at any 16-B phase
#define XE_HDR_ROWS (XE_HDR_HI <= XE_HDR_LO ? 0 : XE_HDR_SPAN_ROWS < 4 ? XE_HDR_SPAN_ROWS : 4)
#define XE_HDR_ROW (XE_WAVE * 16)                  // bytes of one row for the whole wave
#define XE_HDR_BUF (XE_HDR_ROWS * XE_HDR_ROW)      // one buffer
#define XE_HDR_WAVE_BYTES (2 * XE_HDR_BUF)         // double buffer per wave
#define XE_HDR_LDS_BYTES (4 * XE_HDR_WAVE_BYTES > 16 ? 4 * XE_HDR_WAVE_BYTES : 16)  // per 256-thread block

// kernel-internal error encoding
#define XE_EV_PANIC 0x1000
#define XE_EV_UNSUP 0x2000
#define XE_EV_CAP 0x3000
#define XE_EV_ORD 0x4000
#define XE_EV_EXIT 0x8000
#define XE_EV_STOP 0x6000  // the count pass of parallel list operations: the lane's packet stops here
#ifndef XE_SEQ_PEEK
#define XE_SEQ_PEEK 0  // the one-lane replay's runahead (seq_packets), per-program kernels only
#endif
#define XE_EV_CLASS(e) ((e) & 0xf000)
#define XE_IS_PANIC(e) (XE_EV_CLASS(e) == XE_EV_PANIC)

#define XE_NOBJ 64
// Fields model: stack frames 0..XE_NFRAMES-1 (frame f at byte-map words 32 f .. 32 f + 31; more than one
// when the per-program kernel inlines bpf-to-bpf calls, xe_jit.cpp flatten_calls), then the ctx
#ifndef XE_NFRAMES
#define XE_NFRAMES 1
#endif
#define XE_STACK_WORDS 32                   // one 256-byte frame
#define XE_CTX_WORD0 (32 * XE_NFRAMES)      // ctx bytes 0..23 = the three words after the frames
#define XE_NWORDS (XE_CTX_WORD0 + 3)
#define XE_DIRTY_WORDS ((XE_NWORDS + 63) / 64)
static_assert(XE_DIRTY_WORDS <= 4, "fields model: at most 256 byte-map words");
#define XE_CTX_LEN 24
#define XE_FRAME 256        // DefaultVMSettings().StackFrameSize (emulator/vm.go:291-296)
#define XE_MAX_FRAMES 8     // DefaultVMSettings().MaxStackFrames

// tag layout: kind (2 bits) | readonly (bit 2) | alias object id << 8
#define XE_T_KIND(t) ((t) & 3u)
#define XE_T_RO 4u
#define XE_T_ALIAS(t) ((t) >> 8)
#define XE_ISPTR(t) (XE_T_KIND(t) == XE_KIND_MEMPTR || XE_T_KIND(t) == XE_KIND_FRAMEPTR)
// a method call on a nil RegisterValue panics (only the general model has nil registers)
#define XE_NILCHK(R) do { if (XE_GEN && XE_T_KIND((R).t) == XE_KIND_NIL) return XE_EV_PANIC | XE_P_NIL_DEREF; } while (0)

XE_DEV int64_t xe_wadd(int64_t a, int64_t b) { return int64_t(uint64_t(a) + uint64_t(b)); }
XE_DEV int64_t xe_wmul(int64_t a, int64_t b) { return int64_t(uint64_t(a) * uint64_t(b)); }
XE_DEV int32_t xe_i32(int64_t v) { return int32_t(uint32_t(uint64_t(v))); }

// default ctx words: bytes 0-3 object 1 (data), 4-7 object 2 (data_end), ... 20-23 object 6
XE_DEV uint64_t xe_ctx_default_word(int w) {
  return w == XE_CTX_WORD0 ? 0x0202020201010101ull
       : w == XE_CTX_WORD0 + 1 ? 0x0404040403030303ull
       : 0x0606060605050505ull;
}

// Fields model: the per-program kernel (xe_jit.cpp emit_mem_fields) supplies XeMem as named fields
// with the xm_* accessors: object ids 1..XE_OBJ_LIMIT-1 (its static bound), XE_NWORDS byte-map words
// (frame 0 + ctx, 8 object ids per word).
#if !XE_GEN
#define XE_UNROLL_VM _Pragma("unroll")
#else
#define XE_UNROLL_VM _Pragma("unroll 1")
#endif

// Per-wave accumulator table of deferred map adds (parallel mode only), in LDS: XE_ACC direct-mapped
// entries {tag = field address | size << 56, sum, score}. A field that owns its entry is added with
// an LDS atomic; every other add goes straight to HBM as one vector atomic. An entry is claimed when
// free, and taken over (its sum flushed to HBM) when misses have worn its score down, so the hot
// counters of a skewed stream end up owning entries and reach HBM once per wave instead of once per
// packet (C3's Zipf flows, C2's per-proto array). Flushed when the wave retires (flush_wave_state).
#ifndef XE_ACC
#define XE_ACC 64
#endif
// log2(XE_ACC): acc_slot takes that many top bits of its hash (64..1024 entries)
#define XE_ACC_BITS (XE_ACC >= 1024 ? 10 : XE_ACC >= 512 ? 9 : XE_ACC >= 256 ? 8 : XE_ACC >= 128 ? 7 : 6)
struct XeAcc {
  unsigned long long tag[XE_ACC];
  unsigned long long sum[XE_ACC];
  int score[XE_ACC];
};
typedef XeAcc XePend;

struct XeReg {
  int64_t v;   // RegisterValue.Value()
  uint32_t h;  // memory handle (pointers)
  uint32_t t;  // kind | readonly | alias id
};

#if defined(XE_REGS_FIELDS)
// per-program kernels (JIT): every register index is a compile-time constant, so named fields fold
// to plain VGPRs
#define XE_REG_DECL XeReg r0, r1, r2, r3, r4, r5, r6, r7, r8, r9, r10;
#elif defined(__HIPCC__)
// interpreter kernel: vector values; element access with a wave-uniform index lowers to VGPR
// indexing (s_set_gpr_idx) instead of a scratch-memory array
typedef long long xe_v16l __attribute__((ext_vector_type(16)));
typedef unsigned int xe_v16u __attribute__((ext_vector_type(16)));
#define XE_REG_DECL xe_v16l rv; xe_v16u rh; xe_v16u rt;
#else  // host simulation: plain arrays
#define XE_REG_DECL long long rv[16]; unsigned int rh[16]; unsigned int rt[16];
#endif

struct XeLane {
  // registers R0..R10 (see reg_get/reg_put)
  XE_REG_DECL
#if !XE_GEN
  // fields model: object table + frame 0 / ctx byte maps (a separate struct so that the register
  // fields above stay splittable into VGPRs)
  struct XeMem* mem;
  uint64_t oused;     // allocated object ids
  // ValueMemory words written since Reset (bit w of the 256-bit mask: word w). Separate scalars, not an
  // array: a dynamically indexed member array would push the whole lane state to scratch memory.
  uint64_t dirty0, dirty1, dirty2, dirty3;
#else
  const XeGen* G;     // arena layout (P.gen, in the kernel-argument segment: scalar loads)
  uint32_t gl;        // this lane's slot in the arena
  uint32_t onext, ofree;  // object ids: bump pointer, free-list length
  uint32_t vnext, vfree;  // ValueMemory clones
  uint32_t bnext, bfree;  // private ByteMemories
  uint64_t bused;         // private byte arena in use
  uint64_t fdirty[2];     // frame f, group g (16 slots): bit f * 16 + g = written since the frame was wiped
  uint32_t ctxdirty;      // ctx slot s written (otherwise it holds the default object 1 + s / 4)
  uint32_t npres;         // PreservedRegisters depth = R10's frame index
  int32_t pi;             // program index (Registers.PI)
  uint32_t npristine;     // private ByteMemories still reading through to their source
#endif
#if XE_GEN || XE_HAS_ORDERED
  uint32_t pidx;          // the packet's index in the batch (order key of its parallel appends)
  uint32_t oseq;          // appends the packet made so far
  uint32_t npops;         // list pops the packet made so far (parallel list operations, P.list)
#endif
  uint64_t odef;      // ids 1..6 still holding their ctx default
#if XE_SEQ_PEEK
  int peek;           // the runahead of the one-lane replay is running (seq_packets; wave-uniform)
#endif
  // packet
  uint8_t* pkt;
  int64_t plen;
  XE_LP(uint8_t) hdr;      // this lane's column of the current LDS header buffer (+ lane * 16)
  XE_LP(uint8_t) hdrbuf;   // the wave's two header buffers (wave-uniform)
  XE_LP(const XeDevMap) maps;  // map descriptor table (LDS copy of P.maps, stage_maps)
  int32_t hdr_len;         // logical bytes [XE_HDR_LO, hdr_len) are served from the window
  int32_t hsh;             // physical offset of logical byte 0 in the lane's rows (may be negative)
  // per-lane map footprints for maps 1..4 (others go straight to global)
  uint64_t fpr[XE_FP_MAPS];
  uint64_t fpa[XE_FP_MAPS];
  // xdp_md ingress_ifindex / rx_queue_index values of the lazily materialised ctx objects 4, 5
  uint32_t ingress, rxq;
  // wave-uniform batch statistics, flushed once per wave (flush_wave_state)
  uint64_t acc_steps;
  uint32_t acc_status[8];
  unsigned long long* rep;  // this wave's statistics / footprint replica record
  uint32_t wave;            // global wave index (map value replica = wave % nrep)
  uint32_t awidth;          // atomic width classes used on maps 1..4 (4 bits per map)
  XePend* pend;             // this wave's deferred-atomic cache (LDS); null = apply immediately
#if XE_COMMITTER
  XE_LP(struct XeRing) ring;  // the committer's ring this wave's paired blocks go to (null: flush them itself)
#endif
#if XE_PAIR_ADDS
  // this packet's deferred 8-byte adds into one 16-byte block of a map value (pend_add): tag = block
  // address | map << 48 | word mask << 56, sums of word 0 / word 1; flushed by lane_finish, or by
  // lane_commit one chunk later (deferred commit)
  uint64_t pb_tag, pb_s0, pb_s1;
#endif
  // deferred commit (parallel mode, XE_DEFER_COMMIT): the last chunk's verdict, stored by lane_commit
  // after the next chunk's prefetch is issued
  bool defer;
  int32_t dv_i;   // packet index, -1: nothing pending
  uint32_t dv;
#if XE_KEYED
  // keyed ordered execution: the keys the current packet touched (XE_MODE_SPEC, written out by
  // lane_finish; bit 0 = written), how many, whether a write was held back, and the lane's chain
  // (XE_MODE_CHAIN)
  uint64_t klog[XE_KLOG];
  uint32_t kn;
  uint32_t kpkt;  // the packet's index (its ikey slots)
  uint32_t kins;  // held-back inserts of the packet so far
  bool kwr;
  bool kany;  // some packet of this wave held a write back (XE_FLAG_KEYED at the wave's flush)
  uint32_t kchain;
  uint32_t kh;  // the last HASH value handle a lookup returned and its key id (value accesses through
  uint64_t kk;  // it need not re-read the slot's key words)
#endif
};

// ------------------------------------------------------------------ registers
// By-value element access on the vector members: the index is wave-uniform (micro-op fields), so
// the backend emits VGPR-indexed moves; with a constant index (helpers, JIT) it is a plain VGPR.
#if defined(XE_REGS_FIELDS)
XE_DEV XeReg reg_get(const XeLane& L, int i) {
  switch (i) {
    case 0: return L.r0; case 1: return L.r1; case 2: return L.r2; case 3: return L.r3;
    case 4: return L.r4; case 5: return L.r5; case 6: return L.r6; case 7: return L.r7;
    case 8: return L.r8; case 9: return L.r9; default: return L.r10;
  }
}
XE_DEV void reg_put(XeLane& L, int i, const XeReg& r) {
  switch (i) {
    case 0: L.r0 = r; break; case 1: L.r1 = r; break; case 2: L.r2 = r; break; case 3: L.r3 = r; break;
    case 4: L.r4 = r; break; case 5: L.r5 = r; break; case 6: L.r6 = r; break; case 7: L.r7 = r; break;
    case 8: L.r8 = r; break; case 9: L.r9 = r; break; default: L.r10 = r; break;
  }
}
#else
XE_DEV XeReg reg_get(const XeLane& L, int i) {
  return XeReg{int64_t(L.rv[i]), L.rh[i], L.rt[i]};
}
XE_DEV void reg_put(XeLane& L, int i, const XeReg& r) {
  L.rv[i] = (long long)r.v;
  L.rh[i] = r.h;
  L.rt[i] = r.t;
}
#endif

// ------------------------------------------------------------------ object table + ValueMemory
// A ValueMemory region: fields model r = first byte-map word (frame 0 = 0, ctx = 32); general model
// r = 0..7 frame, 8 ctx, 16 + k ValueMemory clone k.
struct XeVR {
  int r;
  int64_t len;
};

#if !XE_GEN
XE_DEV void obj_get(const XeLane& L, int id, int64_t& v, uint32_t& h, uint32_t& t) {
  if ((L.odef >> id) & 1ull) {
    // xdp_md objects: data, data_end, data_meta = MemoryPtr{pkt}, then 3 IMMs
    h = id <= 3 ? xe_h_make(XE_H_PKT, 0, 0) : 0u;
    t = id <= 3 ? uint32_t(XE_KIND_MEMPTR) : uint32_t(XE_KIND_IMM);
    v = id == 2 ? L.plen : id == 4 ? int64_t(L.ingress) : id == 5 ? int64_t(L.rxq) : 0;
    return;
  }
  v = xm_ov(*L.mem, id);
  h = xm_oh(*L.mem, id);
  t = xm_ot(*L.mem, id);
}
XE_DEV void obj_set(XeLane& L, int id, int64_t v, uint32_t h, uint32_t t) {
  xm_set_obj(*L.mem, id, v, h, t);
  L.odef &= ~(1ull << id);
}
XE_DEV void obj_set_val(XeLane& L, int id, int64_t v) {
  if ((L.odef >> id) & 1ull) {
    int64_t ov; uint32_t oh, ot;
    obj_get(L, id, ov, oh, ot);
    obj_set(L, id, v, oh, ot);
  } else {
    xm_set_ov(*L.mem, id, v);
  }
}
// A word index the optimiser cannot fold selects among the values, laundered (as the xm_* accessors do):
// left as plain selects they become one load through a selected address into the lane state, which
// keeps the whole XeLane out of registers (scratch memory).
XE_DEV uint64_t dirty_word(const XeLane& L, int w) {  // the dirty-mask word holding bit w
  if (XE_DIRTY_WORDS == 1) return L.dirty0;
  if (__builtin_constant_p(w)) return w < 64 ? L.dirty0 : w < 128 ? L.dirty1 : w < 192 ? L.dirty2 : L.dirty3;
  uint64_t a = L.dirty0, b = L.dirty1, c = L.dirty2, d = L.dirty3;
#if defined(__HIPCC__)
  asm("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
#endif
  return w < 64 ? a : w < 128 ? b : w < 192 ? c : d;
}
XE_DEV void dirty_or(XeLane& L, int w, uint64_t bits) {
  if (XE_DIRTY_WORDS == 1) { L.dirty0 |= bits; return; }
  L.dirty0 |= w < 64 ? bits : 0ull;
  L.dirty1 |= w >= 64 && w < 128 ? bits : 0ull;
  L.dirty2 |= w >= 128 && w < 192 ? bits : 0ull;
  L.dirty3 |= w >= 192 ? bits : 0ull;
}
XE_DEV void dirty_clear(XeLane& L, int w, uint64_t bits) {
  if (XE_DIRTY_WORDS == 1) { L.dirty0 &= ~bits; return; }
  L.dirty0 &= w < 64 ? ~bits : ~0ull;
  L.dirty1 &= w >= 64 && w < 128 ? ~bits : ~0ull;
  L.dirty2 &= w >= 128 && w < 192 ? ~bits : ~0ull;
  L.dirty3 &= w >= 192 ? ~bits : ~0ull;
}
XE_DEV uint64_t bm_word(const XeLane& L, int w) {
  if ((dirty_word(L, w) >> (w & 63)) & 1ull) return xm_bm(*L.mem, w);
  return w >= XE_CTX_WORD0 ? xe_ctx_default_word(w) : 0ull;
}
XE_DEV void bm_set_word(XeLane& L, int w, uint64_t v) {
  xm_set_bm(*L.mem, w, v);
  dirty_or(L, w, 1ull << (w & 63));
}
// the per-program kernel only uses this model when no path can exhaust the ids (xe_jit.cpp)
XE_DEV int obj_alloc(XeLane& L) {
  if (L.oused == ~0ull) return -1;
  int id = __builtin_ctzll(~L.oused);
  L.oused |= 1ull << id;
  return id;
}
XE_DEV XeVR vmem_region(const XeLane&, uint32_t h) {
  return xe_h_cls(h) == XE_H_CTX ? XeVR{XE_CTX_WORD0, XE_CTX_LEN}
                                  : XeVR{XE_NFRAMES > 1 ? XE_STACK_WORDS * int(xe_h_map(h)) : 0, XE_FRAME};
}
XE_DEV int vmem_id(const XeLane& L, XeVR R, int64_t off) {
  uint64_t word = bm_word(L, R.r + int(off >> 3));
  return int((word >> (8 * (off & 7))) & 0xffu);
}
XE_DEV int vmem_fill(XeLane& L, XeVR R, int64_t off, int size, int id) {
  int64_t end = off + size;
  int w0 = int(off >> 3), w1 = int((end - 1) >> 3);
  XE_UNROLL_VM
  for (int w = w0; w <= w1; w++) {
    int64_t lo = off > int64_t(w) * 8 ? off - int64_t(w) * 8 : 0;
    int64_t hi = end < int64_t(w + 1) * 8 ? end - int64_t(w) * 8 : 8;
    uint64_t mask = (hi - lo == 8) ? ~0ull : (((1ull << (8 * (hi - lo))) - 1ull) << (8 * lo));
    uint64_t word = bm_word(L, R.r + w);
    word = (word & ~mask) | ((uint64_t(id) * 0x0101010101010101ull) & mask);
    bm_set_word(L, R.r + w, word);
  }
  return 0;
}
#else  // ---- general model: the arena
template <class T>
XE_DEV XE_GP(T) gat(const XeLane& L, uint64_t field, uint64_t elem) {
  return (XE_GP(T))(L.G->base + field + (elem * L.G->nl + L.gl) * sizeof(T));
}
XE_DEV XE_GP(uint8_t) lane_bytes(const XeLane& L) { return (XE_GP(uint8_t))(L.G->base + L.G->o_bytes + uint64_t(L.gl) * L.G->nbytes); }

XE_DEV void obj_get(const XeLane& L, int id, int64_t& v, uint32_t& h, uint32_t& t) {
  if (id < 64 && ((L.odef >> id) & 1ull)) {
    h = id <= 3 ? xe_h_make(XE_H_PKT, 0, 0) : 0u;
    t = id <= 3 ? uint32_t(XE_KIND_MEMPTR) : uint32_t(XE_KIND_IMM);
    v = id == 2 ? L.plen : id == 4 ? int64_t(L.ingress) : id == 5 ? int64_t(L.rxq) : 0;
    return;
  }
  v = *gat<int64_t>(L, L.G->o_ov, uint32_t(id));
  h = *gat<uint32_t>(L, L.G->o_oh, uint32_t(id));
  t = *gat<uint32_t>(L, L.G->o_ot, uint32_t(id));
}
XE_DEV void obj_set(XeLane& L, int id, int64_t v, uint32_t h, uint32_t t) {
  *gat<int64_t>(L, L.G->o_ov, uint32_t(id)) = v;
  *gat<uint32_t>(L, L.G->o_oh, uint32_t(id)) = h;
  *gat<uint32_t>(L, L.G->o_ot, uint32_t(id)) = t;
  if (id < 64) L.odef &= ~(1ull << id);
}
XE_DEV void obj_set_val(XeLane& L, int id, int64_t v) {
  if (id < 64 && ((L.odef >> id) & 1ull)) {
    int64_t ov; uint32_t oh, ot;
    obj_get(L, id, ov, oh, ot);
    obj_set(L, id, v, oh, ot);
  } else {
    *gat<int64_t>(L, L.G->o_ov, uint32_t(id)) = v;
  }
}

// -- ValueMemory regions
XE_DEV uint32_t vc_len(const XeLane& L, uint32_t k) { return *gat<uint32_t>(L, L.G->o_vcinfo, k) & 0xffffu; }
XE_DEV uint32_t vc_src(const XeLane& L, uint32_t k) { return *gat<uint32_t>(L, L.G->o_vcinfo, k) >> 16; }  // XE_H_CTX / XE_H_STACK
XE_DEV XeVR vmem_region(const XeLane& L, uint32_t h) {
  const uint32_t c = xe_h_cls(h);
  if (c == XE_H_CTX) return XeVR{8, XE_CTX_LEN};
  if (c == XE_H_VCLONE) return XeVR{16 + int(xe_h_slot(h)), int64_t(vc_len(L, xe_h_slot(h)))};
  return XeVR{int(xe_h_map(h)), XE_FRAME};
}
XE_DEV bool frame_group_dirty(const XeLane& L, int f, int g) {
  const int bit = f * 16 + g;
  return (L.fdirty[bit >> 6] >> (bit & 63)) & 1ull;
}
XE_DEV int vmem_id(const XeLane& L, XeVR R, int64_t off) {
  if (R.r < 8) {
    if (!frame_group_dirty(L, R.r, int(off >> 4))) return 0;
    return *gat<uint16_t>(L, L.G->o_frm, uint64_t(R.r) * XE_FRAME + uint64_t(off));
  }
  if (R.r == 8) {
    if (!((L.ctxdirty >> off) & 1u)) return 1 + int(off >> 2);
    return *gat<uint16_t>(L, L.G->o_ctx, uint64_t(off));
  }
  return *gat<uint16_t>(L, L.G->o_vc, uint64_t(R.r - 16) * XE_FRAME + uint64_t(off));
}
XE_DEV void vmem_set(XeLane& L, XeVR R, int64_t off, int id) {
  if (R.r < 8) {
    const int g = int(off >> 4);
    if (!frame_group_dirty(L, R.r, g)) {  // the group held nil since the frame was wiped
#pragma unroll 1
      for (int s = 0; s < 16; s++) *gat<uint16_t>(L, L.G->o_frm, uint64_t(R.r) * XE_FRAME + uint64_t(g * 16 + s)) = 0;
      const int bit = R.r * 16 + g;
      L.fdirty[bit >> 6] |= 1ull << (bit & 63);
    }
    *gat<uint16_t>(L, L.G->o_frm, uint64_t(R.r) * XE_FRAME + uint64_t(off)) = uint16_t(id);
  } else if (R.r == 8) {
    *gat<uint16_t>(L, L.G->o_ctx, uint64_t(off)) = uint16_t(id);
    L.ctxdirty |= 1u << off;
  } else {
    *gat<uint16_t>(L, L.G->o_vc, uint64_t(R.r - 16) * XE_FRAME + uint64_t(off)) = uint16_t(id);
  }
}
XE_DEV int vmem_fill(XeLane& L, XeVR R, int64_t off, int size, int id) {
#pragma unroll 1
  for (int i = 0; i < size; i++) vmem_set(L, R, off + i, id);
  return 0;
}

// -- private ByteMemories: {source handle, materialised offset (XE_NONE while it reads through), length,
//    region | map << 8 for the parity record}
#define XE_BM_SRC 0
#define XE_BM_MAT 1
#define XE_BM_LEN 2
#define XE_BM_INFO 3
XE_DEV XE_GP(uint32_t) bm_field(const XeLane& L, uint32_t k, int f) { return gat<uint32_t>(L, L.G->o_bm, uint64_t(k) * 4 + uint64_t(f)); }

// -- preserved registers (bpf-to-bpf calls): entry e = {pc, then R6..R9 as (v lo, v hi, h, t)}
XE_DEV XE_GP(uint32_t) pres_word(const XeLane& L, uint32_t e, int w) { return gat<uint32_t>(L, L.G->o_pres, uint64_t(e) * 17 + uint64_t(w)); }
XE_DEV XeReg pres_get(const XeLane& L, uint32_t e, int r) {
  const int w = 1 + 4 * r;
  return XeReg{int64_t(uint64_t(*pres_word(L, e, w)) | (uint64_t(*pres_word(L, e, w + 1)) << 32)), *pres_word(L, e, w + 2),
               *pres_word(L, e, w + 3)};
}
XE_DEV void pres_put(XeLane& L, uint32_t e, int r, const XeReg& R) {
  const int w = 1 + 4 * r;
  *pres_word(L, e, w) = uint32_t(uint64_t(R.v));
  *pres_word(L, e, w + 1) = uint32_t(uint64_t(R.v) >> 32);
  *pres_word(L, e, w + 2) = R.h;
  *pres_word(L, e, w + 3) = R.t;
}

// -- mark-sweep collection of object ids, ValueMemory clones and private ByteMemories. Roots: R0-R9,
//    the preserved registers, frames 0..depth, the ctx; then to a fixed point: the slots of live
//    clones, the memories of live pointer objects, the sources of live ByteMemory clones.
XE_DEV XE_GP(uint32_t) mark_word(const XeLane& L, uint32_t w) { return gat<uint32_t>(L, L.G->o_mark, w); }
XE_DEV bool mark_set(XeLane& L, uint32_t bit) {  // returns true when newly marked
  XE_GP(uint32_t) p = mark_word(L, bit >> 5);
  const uint32_t m = 1u << (bit & 31);
  if (*p & m) return false;
  *p |= m;
  return true;
}
XE_DEV bool mark_get(const XeLane& L, uint32_t bit) { return (*mark_word(L, bit >> 5) >> (bit & 31)) & 1u; }
XE_DEV uint32_t vc_bit(const XeLane& L, uint32_t k) { return ((L.G->nobj + 31) & ~31u) + k; }
XE_DEV uint32_t bm_bit(const XeLane& L, uint32_t k) { return ((L.G->nobj + 31) & ~31u) + ((L.G->nvc + 31) & ~31u) + k; }
XE_DEV bool mark_handle(XeLane& L, uint32_t h) {
  const uint32_t c = xe_h_cls(h);
  if (c == XE_H_VCLONE) return mark_set(L, vc_bit(L, xe_h_slot(h)));
  if (c == XE_H_BMEM) return mark_set(L, bm_bit(L, xe_h_slot(h)));
  return false;
}
XE_DEV bool mark_obj(XeLane& L, int id) { return id > 0 && mark_set(L, uint32_t(id)); }

XE_COLD void gen_gc(XeLane& L) {
#pragma unroll 1
  for (uint32_t w = 0; w < L.G->mark_words; w++) *mark_word(L, w) = 0;
#pragma unroll 1
  for (int r = 0; r < 10; r++) {
    const XeReg R = reg_get(L, r);
    mark_obj(L, int(XE_T_ALIAS(R.t)));
    if (XE_ISPTR(R.t)) mark_handle(L, R.h);
  }
#pragma unroll 1
  for (uint32_t e = 0; e < L.npres; e++)
#pragma unroll 1
    for (int r = 0; r < 4; r++) {
      const XeReg R = pres_get(L, e, r);
      if (XE_ISPTR(R.t)) mark_handle(L, R.h);
    }
#pragma unroll 1
  for (uint32_t f = 0; f <= L.npres && f < L.G->nframes; f++)
#pragma unroll 1
    for (int s = 0; s < XE_FRAME; s++) mark_obj(L, vmem_id(L, XeVR{int(f), XE_FRAME}, s));
#pragma unroll 1
  for (int s = 0; s < XE_CTX_LEN; s++) mark_obj(L, vmem_id(L, XeVR{8, XE_CTX_LEN}, s));
  for (bool grew = true; grew;) {
    grew = false;
#pragma unroll 1
    for (uint32_t k = 0; k < L.vnext; k++)
      if (mark_get(L, vc_bit(L, k)))
#pragma unroll 1
        for (uint32_t s = 0; s < vc_len(L, k); s++) grew |= mark_obj(L, vmem_id(L, XeVR{16 + int(k), XE_FRAME}, s));
#pragma unroll 1
    for (uint32_t id = 1; id < L.onext; id++)
      if (mark_get(L, id)) {
        int64_t v; uint32_t h, t;
        obj_get(L, int(id), v, h, t);
        if (XE_ISPTR(t)) grew |= mark_handle(L, h);
      }
#pragma unroll 1
    for (uint32_t k = 0; k < L.bnext; k++)
      if (mark_get(L, bm_bit(L, k)) && *bm_field(L, k, XE_BM_MAT) == XE_NONE) grew |= mark_handle(L, *bm_field(L, k, XE_BM_SRC));
  }
  L.ofree = 0;
#pragma unroll 1
  for (uint32_t id = 1; id < L.onext; id++)
    if (!mark_get(L, id)) *gat<uint32_t>(L, L.G->o_ofree, L.ofree++) = id;
  L.vfree = 0;
#pragma unroll 1
  for (uint32_t k = 0; k < L.vnext; k++)
    if (!mark_get(L, vc_bit(L, k))) *gat<uint32_t>(L, L.G->o_vfree, L.vfree++) = k;
  L.bfree = 0;
  bool any_bytes = false;
#pragma unroll 1
  for (uint32_t k = 0; k < L.bnext; k++) {
    if (!mark_get(L, bm_bit(L, k))) {
      if (*bm_field(L, k, XE_BM_MAT) == XE_NONE && *bm_field(L, k, XE_BM_SRC) != XE_NONE) L.npristine--;
      *bm_field(L, k, XE_BM_SRC) = XE_NONE;  // a free record never matches a source
      *bm_field(L, k, XE_BM_MAT) = 0;
      *gat<uint32_t>(L, L.G->o_bfree, L.bfree++) = k;
    } else if (*bm_field(L, k, XE_BM_MAT) != XE_NONE) {
      any_bytes = true;
    }
  }
  if (!any_bytes) L.bused = 0;
}

XE_DEV int obj_alloc(XeLane& L) {
  if (L.ofree) return int(*gat<uint32_t>(L, L.G->o_ofree, --L.ofree));
  if (L.onext < L.G->nobj) return int(L.onext++);
  gen_gc(L);
  if (L.ofree) return int(*gat<uint32_t>(L, L.G->o_ofree, --L.ofree));
  return -1;
}
XE_DEV int vc_alloc(XeLane& L) {
  if (L.vfree) return int(*gat<uint32_t>(L, L.G->o_vfree, --L.vfree));
  if (L.vnext < L.G->nvc) return int(L.vnext++);
  gen_gc(L);
  if (L.vfree) return int(*gat<uint32_t>(L, L.G->o_vfree, --L.vfree));
  return -1;
}
XE_DEV int bm_alloc(XeLane& L) {
  if (L.bfree) return int(*gat<uint32_t>(L, L.G->o_bfree, --L.bfree));
  if (L.bnext < L.G->nbm) return int(L.bnext++);
  gen_gc(L);
  if (L.bfree) return int(*gat<uint32_t>(L, L.G->o_bfree, --L.bfree));
  return -1;
}
XE_DEV int64_t bytes_alloc(XeLane& L, uint64_t n) {
  const uint64_t need = (n + 7) & ~uint64_t(7);
  if (L.bused + need > L.G->nbytes) {
    gen_gc(L);
    if (L.bused + need > L.G->nbytes) return -1;
  }
  const uint64_t at = L.bused;
  L.bused += need;
  return int64_t(at);
}
#endif

// ------------------------------------------------------------------ register writes
XE_DEV void reg_replace(XeLane& L, int d, uint32_t kind, uint32_t h, int64_t v, uint32_t alias_and_ro) {
  reg_put(L, d, XeReg{v, h, kind | alias_and_ro});
}

// every register aliasing object `a` sees its new value
XE_DEV void alias_refresh(XeLane& L, uint32_t a, int64_t v) {
#pragma unroll
  for (int j = 0; j < 10; j++) {
    XeReg q = reg_get(L, j);
    if (XE_T_ALIAS(q.t) == a) { q.v = v; reg_put(L, j, q); }
  }
}

// RegisterValue.Assign on register d's object (in place; registers.go:194-197,243-247,305-313)
XE_DEV int reg_inplace(XeLane& L, int d, int64_t v, uint32_t cm = XE_CM_ALL) {
  XeReg r = reg_get(L, d);
  XE_NILCHK(r);
  if (XE_T_KIND(r.t) == XE_KIND_FRAMEPTR && (r.t & XE_T_RO)) return XE_E_READONLY;
  r.v = v;
  reg_put(L, d, r);
  uint32_t a = XE_T_ALIAS(r.t);
  if ((cm & XE_CM_ALIAS) && a) {
    obj_set_val(L, int(a), v);
    alias_refresh(L, a, v);
  }
  return 0;
}

// ------------------------------------------------------------------ footprints
// descriptor of map m from the LDS table (only the fields a caller uses survive optimisation)
XE_DEV XeDevMap map_desc(const XeLane& L, uint32_t m) {
  XeDevMap M;
  uint32_t* d = reinterpret_cast<uint32_t*>(&M);
  XE_LP(const uint32_t) src = (XE_LP(const uint32_t))(L.maps + m);
#pragma unroll
  for (uint32_t k = 0; k < sizeof(XeDevMap) / 4; k++) d[k] = src[k];
#if defined(XE_JIT_GEOM)
  xe_jit_geom(m, M);  // per-program kernel: map geometry as compile-time constants
#endif
  return M;
}

// HASH / LRU_HASH value handles (xe_internal.h XE_H_BIG): slot (or value id) s of map m, and back
XE_DEV uint32_t hv_make(const XeDevMap& M, uint32_t m, uint32_t s) {
  if (s < (1u << XE_H_SLOT_BITS) || !M.big) return xe_h_make(XE_H_HASH, m, s);
  return xe_h_make(XE_H_HASH, XE_H_BIG + (M.big - 1u) + (s >> XE_H_SLOT_BITS), s & ((1u << XE_H_SLOT_BITS) - 1u));
}
XE_DEV uint32_t hv_map(const XeParams& P, uint32_t h) {
  const uint32_t m = xe_h_map(h);
  return m >= XE_H_BIG ? uint32_t(P.bigmap[m - XE_H_BIG]) : m;
}
XE_DEV uint32_t hv_slot(const XeParams& P, uint32_t h) {
  const uint32_t m = xe_h_map(h);
  return (m >= XE_H_BIG ? uint32_t(P.bigoff[m - XE_H_BIG]) << XE_H_SLOT_BITS : 0u) | xe_h_slot(h);
}

XE_DEV uint64_t fp_bits(const XeDevMap& M, bool array, int64_t off, int size) {
  uint64_t vs = M.value_size;
  if (vs == 0) return ~0ull;
  uint64_t o = !array ? uint64_t(off)
             : (uint64_t(off) >> 32) == 0 ? uint64_t(uint32_t(off) % uint32_t(vs)) : uint64_t(off) % vs;
  uint64_t e = o + uint64_t(size);  // exclusive
  if (e > vs) return ~0ull;         // straddles two values
  uint64_t lo, hi;
  if (vs <= 64) { lo = o; hi = e - 1; }
  else { lo = o * 64 / vs; hi = (e - 1) * 64 / vs; }
  uint64_t top = hi >= 63 ? ~0ull : ((1ull << (hi + 1)) - 1ull);
  return top & ~((1ull << lo) - 1ull);
}

// atomic adds of different widths on one map do not commute in general (a narrow add stops its
// carry at its own top byte): the host treats a map with more than one width class as a conflict
XE_DEV void width_record(XeLane& L, const XeParams& P, uint32_t m, int size, uint64_t addr) {
  const uint32_t cls = size == 8 ? 3u : size == 4 ? 2u : size == 2 ? 1u : 0u;
  if (addr & uint64_t(size - 1)) xe_atomic_or32(P.flags, XE_FLAG_UNALIGNED);
  if (m >= 1 && m <= 4) L.awidth |= 1u << (4 * m + cls);
  else xe_atomic_or64(&L.rep[XE_REC_WIDTH0 + m / 16], 1ull << (4 * (m % 16) + cls));
}

XE_DEV void fp_record(XeLane& L, const XeParams& P, uint32_t m, bool atomic, uint64_t bits) {
  if (m >= 1 && m <= XE_FP_MAPS) {
#pragma unroll
    for (int k = 0; k < XE_FP_MAPS; k++) {
      if (uint32_t(k + 1) == m) {
        if (atomic) L.fpa[k] |= bits; else L.fpr[k] |= bits;
      }
    }
  } else {
    xe_atomic_or64(&L.rep[16 + m * 2 + (atomic ? 1 : 0)], bits);
  }
}

// ------------------------------------------------------------------ keyed ordered execution
// (xe_internal.h XE_MODE_SPEC / XE_MODE_CHAIN)
XE_DEV bool xe_concurrent(const XeParams& P) { return P.mode != XE_MODE_SEQUENTIAL; }

#if XE_KEYED
// key ids: HASH keys by their zero-padded words (the nil key has its own), ARRAY keys by element index
XE_DEV uint64_t kid_hash(uint32_t m, const XeDevMap& M, const uint64_t* kw, bool empty) {
  return xe_kid(m, empty ? XE_KID_NIL_KEY : xe_hash_words(kw, M.kwords, M.key_size));
}
XE_DEV uint64_t kid_array(uint32_t m, uint64_t elem) { return xe_kid(m, XE_KID_ARRAY_TAG ^ elem); }
// the key of HASH slot `slot` (its record's key words; slot cap is the nil key's)
XE_DEV uint64_t kid_slot(uint32_t m, const XeDevMap& M, uint32_t slot) {
  if (slot == M.cap) return xe_kid(m, XE_KID_NIL_KEY);
  uint64_t kw[XE_MAX_KEY / 8];
  XE_GP(const uint64_t) r = (XE_GP(const uint64_t))M.keys + uint64_t(slot) * M.rwords + 1;
#pragma unroll
  for (uint32_t w = 0; w < XE_MAX_KEY / 8; w++) kw[w] = w < M.kwords ? r[w] : 0;
  return xe_kid(m, xe_hash_words(kw, M.kwords, M.key_size));
}

// D table (the keys some packet writes): open addressing over key ids, 0 = free
XE_DEV int64_t dset_find(const XeKeyed& K, uint64_t kid) {
  if (!kid) return -1;  // (key ids are never 0; 0 marks a free D slot)
  uint32_t idx = uint32_t(kid >> 4) & (K.dcap - 1);
#pragma unroll 1
  for (uint32_t p = 0; p < K.dcap; p++) {
    const uint64_t k = ((XE_GP(const uint64_t))K.dkid)[idx];
    if (k == kid) return int64_t(idx);
    if (k == 0) return -1;
    idx = (idx + 1) & (K.dcap - 1);
  }
  return -1;
}

XE_DEV int64_t keyed_dset_insert(const XeKeyed& K, uint64_t kid);

// A map key the lane's packet touches (read / add: write = false; an ARRAY / HASH write: true).
// SPEC: log it (repeats fold into one entry). CHAIN: a key of D must belong to the lane's chain, a
// key outside D must not be written; otherwise the packet has left what the schedule proved
// independent and the batch takes the one-lane replay (XE_EV_ORD). *dkey: the key is the chain's own
// (its accesses are ordered by the chain: no footprints, adds applied in place).
XE_DEV int key_touch(XeLane& L, const XeParams& P, uint64_t kid, bool write, bool* dkey = nullptr) {
  if (dkey) *dkey = false;
  if (P.mode == XE_MODE_SPEC) {
    bool found = false;
#pragma unroll
    for (uint32_t j = 0; j < XE_KLOG; j++) {
      if (j < L.kn && (L.klog[j] & ~XE_KLOG_FLAGS) == kid) {
        found = true;
        if (write) L.klog[j] |= XE_KLOG_W;
      }
    }
    if (!found) {
#pragma unroll
      for (uint32_t j = 0; j < XE_KLOG; j++)
        if (j == L.kn) L.klog[j] = kid | (write ? 1ull : 0ull);
      L.kn++;
    }
    if (write) L.kwr = true;
    return 0;
  }
  if (P.mode == XE_MODE_CHAIN) {
    const int64_t d = dset_find(P.K, kid);
    if (d < 0) return write ? XE_EV_ORD : 0;
    if (((XE_GP(const uint32_t))P.K.dcomp)[d] != L.kchain) return XE_EV_ORD;
    if (dkey) *dkey = true;
  }
  return 0;
}
// the ARRAY elements [off, off + size) of map m spans (a value pointer covers the whole array)
XE_DEV int key_touch_array(XeLane& L, const XeParams& P, uint32_t m, const XeDevMap& M, int64_t off, int64_t size, bool write,
                           bool* dkey = nullptr) {
  if (M.value_size == 0 || size <= 0) return 0;
  const uint64_t lo = uint64_t(off) / M.value_size, hi = uint64_t(off + size - 1) / M.value_size;
  bool all = true;
#pragma unroll 1
  for (uint64_t e = lo; e <= hi; e++) {
    bool d = false;
    if (int r = key_touch(L, P, kid_array(m, e), write, &d)) return r;
    all = all && d;
  }
  if (dkey) *dkey = all;
  return 0;
}
#endif

// ------------------------------------------------------------------ ByteMemory access
struct XeBMem {
  uint8_t* base;
  int64_t len;
  uint32_t map;     // map whose memory this is (footprints); 0 = the packet or a lane-private copy
  bool array;
};

// Map memories — and, in the general model, list / perf elements and lane-private ByteMemories (a
// clone still reading through resolves to its source). The packet itself takes the header-window path.
// the lane runs the one-lane replay's runahead (seq_packets): shared writes stop its packet there
XE_DEV bool xe_peeking(const XeLane& L) {
#if XE_SEQ_PEEK
  return xe_readfirst(L.peek) != 0;
#else
  (void)L;
  return false;
#endif
}

XE_DEV bool bmem_resolve(const XeLane& L, const XeParams& P, uint32_t h, XeBMem& B) {
#if XE_GEN
  while (xe_h_cls(h) == XE_H_BMEM) {
    const uint32_t k = xe_h_slot(h);
    const uint32_t mat = *bm_field(L, k, XE_BM_MAT);
    if (mat != XE_NONE) {
      B.base = (uint8_t*)(lane_bytes(L) + mat);
      B.len = int64_t(*bm_field(L, k, XE_BM_LEN));
      B.map = 0;
      B.array = false;
      return true;
    }
    h = *bm_field(L, k, XE_BM_SRC);
  }
  if (xe_h_cls(h) == XE_H_PKT) {
    B.base = L.pkt; B.len = L.plen; B.map = 0; B.array = false;
    return true;
  }
#endif
  uint32_t c = xe_h_cls(h);
  uint32_t m = c == XE_H_HASH ? hv_map(P, h) : xe_h_map(h);
  const XeDevMap M = map_desc(L, m);
  B.map = m;
  if (!XE_HAS_HASH || (XE_HAS_ARRAY && c == XE_H_ARRAY)) {
    B.base = M.vals; B.len = int64_t(M.vals_bytes); B.array = true; return true;
  }
  B.array = false;
#if XE_HAS_ORDERED
  if (c == XE_H_QVAL) {
    const uint64_t id = xe_h_slot(h);
    if (M.kind == XE_DM_PERF) {
      B.base = M.vals + ((XE_GP(const uint64_t))M.rec)[2 * id];
      B.len = int64_t(((XE_GP(const uint64_t))M.rec)[2 * id + 1]);
    } else {
      B.base = M.vals + id * M.value_size;
      B.len = int64_t(((XE_GP(const uint32_t))M.elen)[id]);
    }
    return true;
  }
  if (M.kind == XE_DM_LRU) {
    const uint64_t vid = hv_slot(P, h);
    B.base = M.vals + vid * M.value_size;
    // header word 4: some value may have a nil backing (an update whose value pointer was unreadable);
    // until then every value is value_size long and its length word is not read (one dependent load
    // less per value access)
    B.len = ((XE_GP(const uint64_t))M.hdr)[4] ? int64_t(((XE_GP(const uint32_t))M.elen)[vid]) : int64_t(M.value_size);
    return true;
  }
#endif
  uint32_t slot = hv_slot(P, h);
  B.base = M.vals + uint64_t(slot) * M.value_size;
  B.len = (uint32_t(((XE_GP(const uint64_t))M.keys)[uint64_t(slot) * M.rwords]) & XE_SLOT_VLEN0) ? 0 : int64_t(M.value_size);
  return true;
}

#if XE_KEYED
// the keys of an access to map memory B (handle h) at [off, off + size) (keyed modes only)
XE_DEV int key_touch_mem(XeLane& L, const XeParams& P, uint32_t h, const XeBMem& B, int64_t off, int64_t size, bool write,
                         bool* dkey = nullptr) {
  if (dkey) *dkey = false;
  if (!B.map || (P.mode != XE_MODE_SPEC && P.mode != XE_MODE_CHAIN)) return 0;
  const XeDevMap M = map_desc(L, B.map);
  if (B.array) return key_touch_array(L, P, B.map, M, off, size, write, dkey);
  if (M.kind == XE_DM_LRU && xe_h_cls(h) == XE_H_HASH) {  // an LRU value: the key of its slot record
    if (h == L.kh) return key_touch(L, P, L.kk, write, dkey);
    const uint32_t slot = ((XE_GP(const uint32_t))M.link)[4 * uint64_t(hv_slot(P, h)) + 2];
    return key_touch(L, P, kid_slot(B.map, M, slot), write, dkey);
  }
  // queue / stack elements and perf events follow packet order: a write to one is never keyed
  if (M.kind != XE_DM_HASH) return write ? XE_EV_ORD : 0;
  return key_touch(L, P, h == L.kh ? L.kk : kid_slot(B.map, M, hv_slot(P, h)), write, dkey);
}
#endif

#if XE_GEN
// Give private ByteMemory k its own copy of the bytes it has been reading through to (its source as
// it is now, which is what Registers.Clone copied at call time, registers.go:233-240: every write to
// the source since then made this copy first). Taking a map's bytes while other lanes add to them is
// order-dependent: parallel mode aborts to the ordered replay instead.
XE_COLD int bm_materialize(XeLane& L, const XeParams& P, uint32_t k) {
  const uint32_t n = *bm_field(L, k, XE_BM_LEN);
  const int64_t at = bytes_alloc(L, n);
  if (at < 0) return XE_EV_CAP;
  if (*bm_field(L, k, XE_BM_SRC) == XE_NONE || *bm_field(L, k, XE_BM_MAT) != XE_NONE) return 0;  // collected meanwhile
  XeBMem S;
  bmem_resolve(L, P, *bm_field(L, k, XE_BM_SRC), S);
  if (xe_concurrent(P) && S.map) return XE_EV_ORD;
  XE_GP(uint8_t) d = lane_bytes(L) + at;
#pragma unroll 1
  for (uint32_t i = 0; i < n; i++) d[i] = ((XE_GP(const uint8_t))S.base)[i];
  *bm_field(L, k, XE_BM_MAT) = uint32_t(at);
  L.npristine--;
  return 0;
}
// Before this lane writes the ByteMemory identified by `ident`, every private copy still reading
// through to it takes its bytes.
XE_DEV int bm_before_write(XeLane& L, const XeParams& P, uint32_t ident) {
  if (!L.npristine) return 0;
#pragma unroll 1
  for (uint32_t k = 0; k < L.bnext; k++) {
    if (*bm_field(L, k, XE_BM_MAT) != XE_NONE || *bm_field(L, k, XE_BM_SRC) != ident) continue;
    if (int e = bm_materialize(L, P, k)) return e;
  }
  return 0;
}
XE_DEV uint32_t bm_ident(uint32_t h) { return xe_h_cls(h) == XE_H_ARRAY ? xe_h_make(XE_H_ARRAY, xe_h_map(h), 0) : h; }
// a write through handle h: its readers-through copy first; a private ByteMemory still reading
// through to its source gets its own bytes
XE_DEV int bm_prepare_write(XeLane& L, const XeParams& P, uint32_t h) {
  if (int e = bm_before_write(L, P, bm_ident(h))) return e;
  if (xe_h_cls(h) == XE_H_BMEM && *bm_field(L, xe_h_slot(h), XE_BM_MAT) == XE_NONE) return bm_materialize(L, P, xe_h_slot(h));
  return 0;
}
#endif

#if !XE_GEN
// the fields model has no private ByteMemories (clones exist only in the general model)
XE_DEV int bm_before_write(XeLane&, const XeParams&, uint32_t) { return 0; }
#endif

// Go bounds check with wrapping add; passing the check with off >= len (overflow) panics at the index
XE_DEV int bounds(int64_t off, int64_t size, int64_t len) {
  if (off < 0 || xe_wadd(off, size) > len) return XE_E_OOB;
  if (off >= len && size > 0) return XE_EV_PANIC | XE_P_INDEX;
  return 0;
}

XE_DEV uint64_t load_le(const uint8_t* p0, int size) {
  XE_GP(const uint8_t) p = (XE_GP(const uint8_t))p0;
  uintptr_t a = uintptr_t(p0);
  if ((a & uintptr_t(size - 1)) == 0) {
    switch (size) {
      case 1: return xe_uni32(*p);
      case 2: return xe_uni32(*(XE_GP(const uint16_t))p);
      case 4: return xe_uni32(*(XE_GP(const uint32_t))p);
      default: return xe_uni64(*(XE_GP(const uint64_t))p);
    }
  }
  uint64_t x = 0;
#pragma unroll 1
  for (int b = 0; b < size; b++) x |= uint64_t(p[b]) << (8 * b);
  return xe_uni64(x);
}

XE_DEV void store_le(uint8_t* p0, int size, uint64_t x) {
  XE_GP(uint8_t) p = (XE_GP(uint8_t))p0;
  uintptr_t a = uintptr_t(p0);
  if ((a & uintptr_t(size - 1)) == 0) {
    switch (size) {
      case 1: *p = uint8_t(x); return;
      case 2: *(XE_GP(uint16_t))p = uint16_t(x); return;
      case 4: *(XE_GP(uint32_t))p = uint32_t(x); return;
      default: *(XE_GP(uint64_t))p = x; return;
    }
  }
#pragma unroll 1
  for (int b = 0; b < size; b++) p[b] = uint8_t(x >> (8 * b));
}

// ---- header window (LDS): physical byte pb of this lane
XE_DEV XE_LP(uint8_t) hdr_at(const XeLane& L, int pb) { return L.hdr + (pb >> 4) * XE_HDR_ROW + (pb & 15); }
XE_DEV uint32_t hdr_dword(const XeLane& L, int pd) { return *(XE_LP(const uint32_t))hdr_at(L, pd); }

// little-endian read of `size` bytes at logical offset off (off + size <= hdr_len): the aligned
// dwords covering the bytes and a funnel shift, no per-byte loop and no alignment branch
XE_DEV uint64_t hdr_read_(const XeLane& L, int off, int size);
XE_DEV uint64_t hdr_read(const XeLane& L, int off, int size) { return xe_uni64(hdr_read_(L, off, size)); }
XE_DEV uint64_t hdr_read_(const XeLane& L, int off, int size) {
  const int pb = off + L.hsh;
  if (size == 1) return *hdr_at(L, pb);
  const int p0 = pb & ~3;
  const int sh = (pb & 3) * 8;
  const int last = pb + size - 1;
  const uint64_t d0 = hdr_dword(L, p0);
  const uint64_t d1 = hdr_dword(L, last >= p0 + 4 ? p0 + 4 : p0);
  const uint64_t lo = (d0 | (d1 << 32)) >> sh;
  if (size == 2) return lo & 0xffffull;
  if (size == 4) return lo & 0xffffffffull;
  const uint64_t d2 = hdr_dword(L, last >= p0 + 8 ? p0 + 8 : p0);
  return sh ? (lo | (d2 << (64 - sh))) : lo;
}
XE_DEV void hdr_write(XeLane& L, int off, int size, uint64_t x) {
#pragma unroll 1
  for (int b = 0; b < size; b++) *hdr_at(L, off + L.hsh + b) = uint8_t(x >> (8 * b));
}

// packet ByteMemory access through the header window when possible. A per-program kernel's
// XE_HDR_LO is the least offset its packet-read analysis proved for any read (XE_HDR_LO_PROVEN), so a
// load needs no lower-bound test there; stores are not part of the analysis and keep it.
XE_DEV bool in_window(const XeLane& L, int64_t off, int size) {
#if XE_HDR_LO > 0
  if (off < XE_HDR_LO) return false;
#endif
  return off + size <= L.hdr_len;
}
XE_DEV bool in_window_read(const XeLane& L, int64_t off, int size) {
#if XE_HDR_LO > 0 && !defined(XE_HDR_LO_PROVEN)
  if (off < XE_HDR_LO) return false;
#endif
  return off + size <= L.hdr_len;
}
XE_DEV uint64_t pkt_load(const XeLane& L, int64_t off, int size) {
  if (in_window_read(L, off, size)) return hdr_read(L, int(off), size);
  uint64_t x = load_le(L.pkt + off, size);
  xe_pin(x);  // wait here, on the rare path, not at the join (where it would drain the prefetch)
  return x;
}
XE_DEV void pkt_store(XeLane& L, int64_t off, int size, uint64_t x) {
  store_le(L.pkt + off, size, x);
  if (in_window(L, off, size)) hdr_write(L, int(off), size, x);
}

// Atomic little-endian add of `add` into the `size`-byte field at p (any alignment), truncating
// at the field's top byte exactly like a read/add/write of that width (inst_atomic.go:44-59). Each
// 32-bit word is updated with a CAS on its masked bytes; the carry out of a word's slice feeds the
// next word's add, so the sum over all lanes is exact whatever the interleaving.
XE_DEV void atomic_add_field(uint8_t* p, int size, uint64_t add) {
  uintptr_t a = uintptr_t(p);
  if (size == 8 && (a & 7) == 0) { xe_atomic_add64(reinterpret_cast<unsigned long long*>(p), add); return; }
  if (size == 4 && (a & 3) == 0) { xe_atomic_add32(reinterpret_cast<unsigned int*>(p), uint32_t(add)); return; }
  uintptr_t start = a, end = a + uintptr_t(size);
  uint64_t carry = 0;
  uintptr_t w = start & ~uintptr_t(3);
  int consumed = 0;  // field bytes consumed so far
#pragma unroll 1
  while (w < end) {
    int lo = start > w ? int(start - w) : 0;
    int hi = end < w + 4 ? int(end - w) : 4;  // exclusive
    int nb = hi - lo;
    uint32_t mask = (nb == 4 ? 0xffffffffu : ((1u << (8 * nb)) - 1u)) << (8 * lo);
    uint64_t part = (consumed < 8 ? (add >> (8 * consumed)) : 0) & (nb == 4 ? 0xffffffffull : ((1ull << (8 * nb)) - 1ull));
    uint64_t addend = part + carry;  // may exceed the slice width by one carry bit
    unsigned int* wp = reinterpret_cast<unsigned int*>(w);
    unsigned int old = *(XE_GP(unsigned int))wp, assumed;
    uint64_t sum;
    do {
      assumed = old;
      uint64_t cur = (uint64_t(assumed) & mask) >> (8 * lo);
      sum = cur + addend;
      uint32_t nw = (assumed & ~mask) | (uint32_t(sum << (8 * lo)) & mask);
      old = xe_atomic_cas32(wp, assumed, nw);
    } while (old != assumed);
    carry = sum >> (8 * nb);
    consumed += nb;
    w += 4;
  }
}

#if defined(__HIPCC__)
XE_DEV unsigned long long xe_lds_cas64(XE_LP(unsigned long long) p, unsigned long long c, unsigned long long v) {
  __hip_atomic_compare_exchange_strong(p, &c, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  return c;
}
XE_DEV void xe_lds_add64(XE_LP(unsigned long long) p, unsigned long long v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
XE_DEV unsigned long long xe_lds_xchg64(XE_LP(unsigned long long) p, unsigned long long v) {
  return __hip_atomic_exchange(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
XE_DEV int xe_lds_add32(XE_LP(int) p, int v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
#else
XE_DEV unsigned long long xe_lds_cas64(unsigned long long* p, unsigned long long c, unsigned long long v) {
  unsigned long long o = *p;
  if (o == c) *p = v;
  return o;
}
XE_DEV void xe_lds_add64(unsigned long long* p, unsigned long long v) { *p += v; }
XE_DEV unsigned long long xe_lds_xchg64(unsigned long long* p, unsigned long long v) { unsigned long long o = *p; *p = v; return o; }
XE_DEV int xe_lds_add32(int* p, int v) { int o = *p; *p += v; return o; }
#endif

XE_DEV uint32_t acc_slot(uint64_t addr) {
  return uint32_t(((addr >> 2) * 0x9E3779B97F4A7C15ull) >> (64 - XE_ACC_BITS)) & (XE_ACC - 1);
}

// One HBM add of a (deferred) sum into an aligned 4/8-byte field of map m. 8-byte adds go to this
// wave's replica of the value region when the map has replicas, which spreads a hot counter over
// nrep addresses (same-address atomics serialise at the memory side).
XE_DEV void field_add(const XeLane& L, uint32_t m, uint64_t addr, int size, uint64_t v) {
  if (size == 8) {
    const XeDevMap M = map_desc(L, m);
    if (M.nrep > 1) addr = uint64_t(uintptr_t(M.rep)) + uint64_t(L.wave % M.nrep) * M.rep_stride + (addr - uint64_t(uintptr_t(M.vals)));
    xe_atomic_add64(reinterpret_cast<unsigned long long*>(uintptr_t(addr)), v);
  } else {
    xe_atomic_add32(reinterpret_cast<unsigned int*>(uintptr_t(addr)), uint32_t(v));
  }
}
// accumulator tag = field address (48 bits) | map << 48 | size << 56
XE_DEV void acc_apply(const XeLane& L, unsigned long long tag, unsigned long long v) {
  field_add(L, uint32_t((tag >> 48) & 0xffu), tag & 0xffffffffffffull, int(tag >> 56), v);
}

#if XE_PAIR_ADDS
// Paired deferral. Memory-side atomics cost one request per 64-byte line per wave-instruction, not
// per lane: two 8-byte adds of one packet into adjacent fields (C5's {pkts, bytes}) cost two requests
// when the lane issues them itself, one when two neighbouring lanes issue them in the same
// instruction (tools/calib_hash.hip: 23.5 vs 47 G adds/s). A packet's 8-byte adds that miss the
// accumulator table therefore collect in one 16-byte block per lane, and lane_finish flushes the
// blocks of the whole wave with word w of lane j's block on lane 2j + w. Exact: the adds commute
// modulo 2^64 and no lane reads a field that receives adds in a parallel run (run_conflict).
XE_DEV bool pend_add(XeLane& L, uint32_t m, uint64_t addr, uint64_t add) {
  const uint64_t blk = (addr & ~uint64_t(15)) | (uint64_t(m) << 48);
  const uint64_t w = (addr >> 3) & 1;
  if (L.pb_tag && (L.pb_tag & ((1ull << 56) - 1)) != blk) return false;
  L.pb_tag |= blk | (1ull << (56 + w));
  if (w) L.pb_s1 += add; else L.pb_s0 += add;
  return true;
}
XE_DEV void pend_word(const XeLane& L, uint64_t tag, uint64_t s, uint32_t w) {
  if (s && ((tag >> (56 + w)) & 1)) field_add(L, uint32_t((tag >> 48) & 0xffu), (tag & 0xffffffffffffull) + 8 * w, 8, s);
}
// all lanes: apply every lane's block (two vector atomics for the wave) and clear it
XE_DEV void pend_flush(XeLane& L) {
#if defined(__HIPCC__)
  const uint32_t lane = uint32_t(xe_lane()), w = lane & 1u;
#pragma unroll
  for (uint32_t h = 0; h < 2; h++) {
    const int src = int(32 * h + (lane >> 1));
    const uint64_t tag = __shfl(L.pb_tag, src), s0 = __shfl(L.pb_s0, src), s1 = __shfl(L.pb_s1, src);
    pend_word(L, tag, w ? s1 : s0, w);
  }
#else
  pend_word(L, L.pb_tag, L.pb_s0, 0);
  pend_word(L, L.pb_tag, L.pb_s1, 1);
#endif
  L.pb_tag = L.pb_s0 = L.pb_s1 = 0;
}
#endif

#if XE_COMMITTER
// The committer's rings (LDS, one per producer wave): XE_RING_D chunks of paired blocks. A producer
// writes a chunk's blocks and then its head; the committer applies a chunk (pend_flush's two wave atomics)
// and then advances the tail. LDS operations of a wave complete in order and are visible to the block's
// other waves once complete, so an lgkmcnt(0) wait between the data and the index write is the release.
#define XE_RING_D 2
struct XeRing {
  unsigned int head, tail, done, pad;
  unsigned long long tag[XE_RING_D][XE_WAVE], s0[XE_RING_D][XE_WAVE], s1[XE_RING_D][XE_WAVE];
};
XE_DEV void lds_release() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// (LDS address space throughout: a generic pointer would make these flat accesses, which count in vmcnt too)
#define XE_RW(x) (*(XE_LP(volatile unsigned int))&(x))
XE_DEV unsigned int ring_word(XE_LP(volatile unsigned int) w) {
  const unsigned int v = *w;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  return uint32_t(xe_readfirst(int(v)));
}
// producer (all lanes): this chunk's paired blocks to the committer instead of its own atomics
XE_DEV void ring_put(XeLane& L, XE_LP(XeRing) R) {
  const unsigned int h = ring_word(&XE_RW(R->head));  // only this wave writes head
  uint32_t spins = 0;
  while (h - ring_word(&XE_RW(R->tail)) >= XE_RING_D) {  // the committer has not taken chunk h - D yet
    __builtin_amdgcn_s_sleep(1);
    if (++spins >= (1u << 26)) { pend_flush(L); return; }  // (unreachable: the committer runs until every producer is done)
  }
  const uint32_t s = h % XE_RING_D, lane = uint32_t(xe_lane());
  R->tag[s][lane] = L.pb_tag;
  R->s0[s][lane] = L.pb_s0;
  R->s1[s][lane] = L.pb_s1;
  lds_release();
  if (lane == 0) XE_RW(R->head) = h + 1;
  lds_release();
  L.pb_tag = L.pb_s0 = L.pb_s1 = 0;
}
XE_DEV void ring_done(XE_LP(XeRing) R) {
  lds_release();
  if (xe_lane() == 0) XE_RW(R->done) = 1;
  lds_release();
}
// the committer wave: apply every producer's chunks until all of them are done and drained. The bound
// only guards against a protocol error (it sets XE_FLAG_CAPACITY: the batch replays, nothing is lost
// silently); a producer finishes its walk in far fewer iterations.
XE_DEV void committer_loop(XeLane& L, const XeParams& P, XE_LP(XeRing) rings, uint32_t nprod) {
  const uint32_t lane = uint32_t(xe_lane()), w = lane & 1u;
  unsigned int tail[4] = {0, 0, 0, 0};
#pragma unroll 1
  for (uint32_t it = 0; it < (1u << 28); it++) {
    bool progress = false, all = true;
#pragma unroll
    for (uint32_t p = 0; p < 3; p++) {
      if (p >= nprod) break;
      XE_LP(XeRing) R = rings + p;
      const unsigned int done = ring_word(&XE_RW(R->done));  // done before head: a done producer's head is final
      const unsigned int h = ring_word(&XE_RW(R->head));
#pragma unroll 1
      while (tail[p] != h) {
        const uint32_t s = tail[p] % XE_RING_D;
#pragma unroll
        for (uint32_t hh = 0; hh < 2; hh++) {  // pend_flush: word w of lane j's block on lane 2j + w
          const uint32_t src = 32u * hh + (lane >> 1);
          pend_word(L, R->tag[s][src], w ? R->s1[s][src] : R->s0[s][src], w);
        }
        lds_release();  // the blocks are read before the slot is handed back
        tail[p]++;
        if (lane == 0) XE_RW(R->tail) = tail[p];
        progress = true;
      }
      all = all && done && tail[p] == h;
    }
    if (all) return;
    if (!progress) __builtin_amdgcn_s_sleep(1);
  }
  if (lane == 0) xe_atomic_or32(P.flags, XE_FLAG_CAPACITY);
}
#endif

// Add `add` to the `size`-byte field at p of map m. Deferred (parallel mode): naturally aligned 4/8-
// byte fields go through the wave's accumulator table, 8-byte adds that miss it collect in the lane's
// paired block (pend_add) where enabled, and 8-byte adds that reach HBM go to the wave's replica.
// Exact in every case: the field add is modulo 2^(8*size), so adding a sum later equals adding its
// parts now; an entry changes owner only after its sum has been taken (exchange) and before any lane
// of this instruction adds to it (the adds re-read the tag after the claim / take-over step), so no
// part is lost or credited to another field.
XE_DEV void wave_atomic_add_field(XeLane& L, uint32_t m, bool defer, uint8_t* p, int size, uint64_t add) {
#if defined(XE_DEBUG_NO_ATOMIC)  // cost experiments only: map adds are dropped (results are wrong)
  return;
#endif
  XePend* acc = L.pend;
  const uint64_t addr = uint64_t(uintptr_t(p));
  if (defer && (size == 8 || size == 4) && (addr & uint64_t(size - 1)) == 0) {
    const uint64_t tag = addr | (uint64_t(m) << 48) | (uint64_t(size) << 56);
    const uint32_t k = acc_slot(addr);
    XE_LP(unsigned long long) tp = (XE_LP(unsigned long long))&acc->tag[k];
    XE_LP(int) sp = (XE_LP(int))&acc->score[k];
    const unsigned long long t = *tp;
    bool pended = false;
    if (t == 0) {
      if (xe_lds_cas64(tp, 0ull, tag) == 0) *sp = 1;
#if XE_PAIR_ADDS
    } else if (t != tag && size == 8 && pend_add(L, m, addr, add)) {
      pended = true;  // a miss: into this packet's paired block (the owner keeps its entry)
#endif
    } else if (t != tag) {
      // a miss wears the owner's score down; the lane that exhausts it takes the entry over
      if (xe_lds_add32(sp, -1) <= 1 && xe_lds_cas64(tp, t, tag) == t) {
        const unsigned long long old = xe_lds_xchg64((XE_LP(unsigned long long))&acc->sum[k], 0ull);
        *sp = 2;
        if (old) acc_apply(L, t, old);
      }
    }
    if (pended) return;
    if (*tp == tag) {
      xe_lds_add64((XE_LP(unsigned long long))&acc->sum[k], add);
      if (t == tag) xe_lds_add32(sp, 1);
      return;
    }
    field_add(L, m, addr, size, add);
    return;
  }
  atomic_add_field(p, size, add);
}

// all lanes: lane k applies entry k (one vector atomic for the whole table) and clears it
XE_DEV void acc_flush(const XeLane& L) {
  XePend* acc = L.pend;
#pragma unroll 1
  for (uint32_t k0 = 0; k0 < XE_ACC; k0 += XE_WAVE) {
    const uint32_t k = k0 + uint32_t(xe_lane());
    const unsigned long long t = acc->tag[k];
    if (t) {
      if (acc->sum[k]) acc_apply(L, t, acc->sum[k]);
      acc->tag[k] = 0;
      acc->sum[k] = 0;
    }
  }
}

// ------------------------------------------------------------------ ValueMemory access
XE_DEV bool is_vm_cls(uint32_t c) { return c == XE_H_CTX || c == XE_H_STACK || (XE_GEN && c == XE_H_VCLONE); }

// ValueMemory.Read, memory.go:32-53 -> object id
XE_DEV int vmem_read(const XeLane& L, uint32_t h, int64_t off, int size, int& id) {
  const XeVR R = vmem_region(L, h);
  if (int e = bounds(off, size, R.len)) return e;
  int first = vmem_id(L, R, off);
  XE_UNROLL_VM
  for (int i = 1; i < size; i++)
    if (vmem_id(L, R, off + i) != first) return XE_E_NONCONTIG;
  if (!first) return XE_E_UNINIT;
  id = first;
  return 0;
}

// ------------------------------------------------------------------ generic memory ops
// Memory.Read for either kind. Outputs the RegisterValue to put in a register.
XE_DEV int mem_read(XeLane& L, const XeParams& P, uint32_t h, int64_t off, int size, bool track,
                    uint32_t& kind, uint32_t& oh, int64_t& val, uint32_t& alias, uint32_t cm = XE_CM_ALL) {
  uint32_t c = xe_h_cls(h);
  if ((cm & XE_CM_VM) && is_vm_cls(c)) {
    int id = 0;
    if (int e = vmem_read(L, h, off, size, id)) return e;
    uint32_t t;
    obj_get(L, id, val, oh, t);
    kind = XE_T_KIND(t);
    alias = (uint32_t(id) << 8) | (t & XE_T_RO);
    return 0;
  }
  if ((cm & XE_CM_PKT) && c == XE_H_PKT) {
    if (int e = bounds(off, size, L.plen)) return e;
    val = int64_t(pkt_load(L, off, size));
    kind = XE_KIND_IMM;
    oh = 0;
    alias = 0;
    return 0;
  }
  if (!(cm & XE_CM_MAPS)) return XE_EV_UNSUP;  // excluded by the class analysis (never reached)
  XeBMem B;
  bmem_resolve(L, P, h, B);
  if (int e = bounds(off, size, B.len)) return e;
  bool own = false;
#if XE_KEYED
  if (int e = key_touch_mem(L, P, h, B, off, size, false, &own)) return e;
#endif
  if (track && B.map && !own) fp_record(L, P, B.map, false, fp_bits(map_desc(L, B.map), B.array, off, size));
  val = int64_t(load_le(B.base + off, size));
  kind = XE_KIND_IMM;
  oh = 0;
  alias = 0;
  return 0;
}

// Memory.Write of a new object {kind, oh, val} (ST: new IMM; STX: Copy of src)
XE_DEV int mem_write(XeLane& L, const XeParams& P, uint32_t h, int64_t off, int size,
                     uint32_t kind, uint32_t oh, int64_t val, uint32_t cm = XE_CM_ALL) {
  uint32_t c = xe_h_cls(h);
  if ((cm & XE_CM_VM) && is_vm_cls(c)) {
    const XeVR R = vmem_region(L, h);
    if (int e = bounds(off, size, R.len)) return e;
    int id = obj_alloc(L);
    if (id < 0) return XE_EV_CAP;
    obj_set(L, id, val, oh, kind);
    vmem_fill(L, R, off, size, id);
    return 0;
  }
  if ((cm & XE_CM_PKT) && c == XE_H_PKT) {
    if (int e = bounds(off, size, L.plen)) return e;
#if XE_GEN
    if (int e = bm_before_write(L, P, h)) return e;
#endif
    pkt_store(L, off, size, uint64_t(val));
    return 0;
  }
  if (!(cm & XE_CM_MAPS)) return XE_EV_UNSUP;  // excluded by the class analysis (never reached)
  XeBMem B;
  bmem_resolve(L, P, h, B);
  if (int e = bounds(off, size, B.len)) return e;
  if (P.mode == XE_MODE_PARALLEL && B.map) return XE_EV_ORD;  // non-commutative shared write
#if XE_KEYED
  if (int e = key_touch_mem(L, P, h, B, off, size, true)) return e;
  if (P.mode == XE_MODE_SPEC && B.map) return 0;  // held back: its key is logged as written
#endif
#if XE_GEN
  if (int e = bm_prepare_write(L, P, h)) return e;
  bmem_resolve(L, P, h, B);
#endif
  store_le(B.base + off, size, uint64_t(val));
  return 0;
}

// PointerValue.ReadRange (registers.go:218-220,273-281; memory.go:55-95,176-185).
// emit(i, byte) receives the output bytes. Returns 0 / XE_E_OOB / panic.
template <class Emit>
XE_DEV int ptr_read_range(XeLane& L, const XeParams& P, const XeReg& R, int64_t count, Emit emit, uint32_t cm = XE_CM_ALL) {
  uint32_t kind = XE_T_KIND(R.t);
  uint32_t h = R.h;
  int64_t off = kind == XE_KIND_FRAMEPTR ? xe_wadd(XE_FRAME, R.v) : R.v;
  uint32_t c = xe_h_cls(h);
  if ((cm & XE_CM_VM) && is_vm_cls(c)) {
    const XeVR Rg = vmem_region(L, h);
    if (off < 0 || xe_wadd(off, count) > Rg.len) return XE_E_OOB;
    if (count < 0) return XE_EV_PANIC | XE_P_MAKESLICE;
    if (off >= Rg.len && count > 0) return XE_EV_PANIC | XE_P_INDEX;
    // Byte groups of equal object references, each written 1/2/4/8 bytes wide (memory.go:61-91).
    // Written as fixed-trip loops (skip counts the bytes a wide write already produced) so that a
    // per-program kernel with a constant count unrolls it fully and folds the object ids.
    int skip = 0;
    XE_UNROLL_VM
    for (int64_t i = 0; i < count; i++) {
      if (skip > 0) { skip--; continue; }
      const int v = vmem_id(L, Rg, off + i);
      if (!v) { emit(i, 0); continue; }
      int size = 1;
      bool run = true;
      XE_UNROLL_VM
      for (int j = 1; j < 8; j++) {
        run = run && i + j < count && vmem_id(L, Rg, off + i + j) == v;
        size += run ? 1 : 0;
      }
      const int w = size > 4 ? 8 : size > 2 ? 4 : size > 1 ? 2 : 1;
      if (i + w > count) return XE_EV_PANIC | XE_P_INDEX;
      int64_t ov; uint32_t oh, ot;
      obj_get(L, v, ov, oh, ot);
      XE_UNROLL_VM
      for (int b = 0; b < 8; b++)
        if (b < w) emit(i + b, uint8_t(uint64_t(ov) >> (8 * b)));
      skip = w - 1;
    }
    return 0;
  }
  if ((cm & XE_CM_PKT) && c == XE_H_PKT) {
    if (off < 0 || xe_wadd(off, count) > L.plen) return XE_E_OOB;
    if (count < 0) return XE_EV_PANIC | XE_P_MAKESLICE;
#pragma unroll 1
    for (int64_t i = 0; i < count; i++) emit(i, uint8_t(pkt_load(L, off + i, 1)));
    return 0;
  }
  if (!(cm & XE_CM_MAPS)) return XE_EV_UNSUP;  // excluded by the class analysis (never reached)
  XeBMem B;
  bmem_resolve(L, P, h, B);
  if (off < 0 || xe_wadd(off, count) > B.len) return XE_E_OOB;
  if (count < 0) return XE_EV_PANIC | XE_P_MAKESLICE;
  bool own = false;
#if XE_KEYED
  if (count > 0)
    if (int e = key_touch_mem(L, P, h, B, off, count, false, &own)) return e;
#endif
  if (count > 0 && B.map && !own) fp_record(L, P, B.map, false, fp_bits(map_desc(L, B.map), B.array, off, int(count)));
#pragma unroll 1
  for (int64_t i = 0; i < count; i++) emit(i, ((XE_GP(const uint8_t))B.base)[off + i]);
  return 0;
}

// ------------------------------------------------------------------ hash map
XE_DEV uint64_t hash_word0(const XeDevMap& M, uint64_t slot) { return xe_uni64(((XE_GP(const uint64_t))M.keys)[slot * M.rwords]); }
XE_DEV uint32_t hash_state(const XeDevMap& M, uint64_t slot) { return uint32_t(hash_word0(M, slot)); }
XE_DEV void hash_set_state(const XeDevMap& M, uint64_t slot, uint32_t st) {
  ((XE_GP(uint64_t))M.keys)[slot * M.rwords] = (hash_word0(M, slot) & ~0xffffffffull) | st;
}

// Linear probing over slot records: the state word and the key words of a record are loaded
// together (independent loads of one line), then compared. LRU maps leave tombstones behind evictions.
//
// When the record geometry is a compile-time constant (per-program kernels), one probe step loads
// every record from the probe position to the end of its XE_PROBE_GROUP-byte group at once and then
// scans them in slot order: the same first-match / stop-at-empty walk as one record at a time, but a
// chain that stays inside a cache line costs one memory round trip instead of one per record.
#ifndef XE_PROBE_GROUP
#define XE_PROBE_GROUP 64
#endif
#if defined(__HIPCC__) && XE_PROBE_GROUP
XE_DEV void xe_group_load(XE_GP(const uint64_t) p, uint64_t* w) {
  static_assert(XE_PROBE_GROUP == 64 || XE_PROBE_GROUP == 128, "probe group: 64 or 128 bytes");
  xe_u4 a[XE_PROBE_GROUP / 16];
#if XE_PROBE_GROUP == 64
  asm volatile(
      "global_load_dwordx4 %0, %4, off\n\tglobal_load_dwordx4 %1, %4, off offset:16\n\t"
      "global_load_dwordx4 %2, %4, off offset:32\n\tglobal_load_dwordx4 %3, %4, off offset:48\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(a[0]), "=&v"(a[1]), "=&v"(a[2]), "=&v"(a[3])
      : "v"(p));
#else
  asm volatile(
      "global_load_dwordx4 %0, %8, off\n\tglobal_load_dwordx4 %1, %8, off offset:16\n\t"
      "global_load_dwordx4 %2, %8, off offset:32\n\tglobal_load_dwordx4 %3, %8, off offset:48\n\t"
      "global_load_dwordx4 %4, %8, off offset:64\n\tglobal_load_dwordx4 %5, %8, off offset:80\n\t"
      "global_load_dwordx4 %6, %8, off offset:96\n\tglobal_load_dwordx4 %7, %8, off offset:112\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(a[0]), "=&v"(a[1]), "=&v"(a[2]), "=&v"(a[3]), "=&v"(a[4]), "=&v"(a[5]), "=&v"(a[6]), "=&v"(a[7])
      : "v"(p));
#endif
#pragma unroll
  for (int j = 0; j < XE_PROBE_GROUP / 8; j++)
    w[j] = xe_uni64(uint64_t(a[j >> 1][2 * (j & 1)]) | (uint64_t(a[j >> 1][2 * (j & 1) + 1]) << 32));
}
#endif
XE_DEV int64_t hash_find(const XeDevMap& M, const uint64_t* kw, bool empty) {
  if (empty) return (hash_state(M, M.cap) & XE_SLOT_FULL) ? int64_t(M.cap) : -1;
  uint64_t hv = xe_hash_words(kw, M.kwords, M.key_size);
  uint32_t mask = M.cap - 1;
  uint32_t idx = uint32_t(hv) & mask;
#if defined(XE_DEBUG_NO_PROBE)  // cost experiments only: every key "hits" its home slot (results are wrong)
  return int64_t(idx);
#endif
#if defined(__HIPCC__) && XE_PROBE_GROUP
  if (__builtin_constant_p(M.rwords) && __builtin_constant_p(M.kwords) && __builtin_constant_p(M.cap) &&
      M.rwords * 8 < XE_PROBE_GROUP && M.cap >= XE_PROBE_GROUP / (M.rwords * 8)) {
    constexpr uint32_t kMaxG = XE_PROBE_GROUP / 8;  // records per group for 1-word records
    static_assert(kMaxG <= 32, "hit / stop masks");
    const uint32_t G = XE_PROBE_GROUP / (M.rwords * 8);
#pragma unroll 1
    for (uint32_t probe = 0; probe < M.cap;) {
      const uint32_t first = idx & (G - 1);
      XE_GP(const uint64_t) r = (XE_GP(const uint64_t))M.keys + uint64_t(idx - first) * M.rwords;
      // the whole group (it lies inside the record array: cap is a multiple of G) in one burst of
      // 16-byte loads with a single wait: the compiler would otherwise interleave each record's load
      // with its compare under register pressure, one round trip per record again
      uint64_t w[XE_PROBE_GROUP / 8];
      xe_group_load(r, w);
      // branch-free scan (a compare under a branch would let the compiler sink its load behind the
      // other records' wait): bit g of hit / stop = record g matches / ends the chain
      uint32_t hit = 0, stop = 0;
#pragma unroll
      for (uint32_t g = 0; g < kMaxG; g++) {
        if (g >= G) continue;
        const uint32_t st = uint32_t(w[g * M.rwords]);
        const bool full = (st & XE_SLOT_FULL) != 0;
        bool eq = true;
#pragma unroll
        for (uint32_t k = 0; k < XE_MAX_KEY / 8; k++)
          if (k < M.kwords) eq = eq && (w[g * M.rwords + k + 1] == kw[k]);
        hit |= uint32_t(full && eq) << g;
        stop |= uint32_t(!full && !(st & XE_SLOT_TOMB)) << g;
      }
      const uint32_t act = (hit | stop) & (~0u << first);
      if (act) {
        const uint32_t g0 = uint32_t(__builtin_ctz(act));
        return ((hit >> g0) & 1u) ? int64_t(idx - first + g0) : -1;
      }
      probe += G - first;
      idx = (idx - first + G) & mask;
    }
    return -1;
  }
#endif
#pragma unroll 1
  for (uint32_t probe = 0; probe < M.cap; probe++) {
    XE_GP(const uint64_t) r = (XE_GP(const uint64_t))M.keys + uint64_t(idx) * M.rwords;
    uint64_t w[XE_MAX_KEY / 8 + 1];
#pragma unroll
    for (uint32_t k = 0; k <= XE_MAX_KEY / 8; k++)
      if (k <= M.kwords) w[k] = r[k];
    const uint32_t st = uint32_t(w[0]);
    if (!(st & XE_SLOT_FULL)) {
      if (!(st & XE_SLOT_TOMB)) return -1;  // tombstones: LRU evictions, keyed reservations
      idx = (idx + 1) & mask;
      continue;
    }
    bool eq = true;
#pragma unroll
    for (uint32_t k = 0; k < XE_MAX_KEY / 8; k++)
      if (k < M.kwords) eq = eq && (w[k + 1] == kw[k]);
    if (eq) return int64_t(idx);
    idx = (idx + 1) & mask;
  }
  return -1;
}

// insert a new key (sequential mode only); returns slot (LRU: the first free or tombstone slot)
XE_DEV int64_t hash_insert_new(const XeDevMap& M, const uint64_t* kw, bool empty) {
  if (empty) {
    hash_set_state(M, M.cap, XE_SLOT_FULL);
    if (M.kind == XE_DM_HASH) *M.count += 1;
    return int64_t(M.cap);
  }
  uint64_t hv = xe_hash_words(kw, M.kwords, M.key_size);
  uint32_t mask = M.cap - 1;
  uint32_t idx = uint32_t(hv) & mask;
  while (hash_state(M, idx) & XE_SLOT_FULL) idx = (idx + 1) & mask;
  uint64_t* k = M.keys + uint64_t(idx) * M.rwords + 1;
  for (uint32_t w = 0; w < M.kwords; w++) k[w] = kw[w];
  hash_set_state(M, idx, XE_SLOT_FULL);
  if (M.kind == XE_DM_HASH) *M.count += 1;
  return int64_t(idx);
}

#if XE_KEYED
// XE_MODE_CHAIN insert of an absent key: it takes the record reserved for it before the chains ran
// (xe_keyed_reserve: a tombstone holding the key words), so no two lanes ever claim slots. -1: the
// key has no reservation (its chain left the schedule). The entry count goes to the striped counter
// cnt (folded into the map's count after the chains; no insert of a chain can hit the capacity).
XE_DEV int64_t hash_claim(const XeDevMap& M, const uint64_t* kw, bool empty, unsigned int* cnt) {
  if (empty) {
    hash_set_state(M, M.cap, XE_SLOT_FULL);
    xe_wave_count(cnt, true);
    return int64_t(M.cap);
  }
  const uint32_t mask = M.cap - 1;
  uint32_t idx = uint32_t(xe_hash_words(kw, M.kwords, M.key_size)) & mask;
#pragma unroll 1
  for (uint32_t probe = 0; probe < M.cap; probe++) {
    XE_GP(uint64_t) r = (XE_GP(uint64_t))M.keys + uint64_t(idx) * M.rwords;
    const uint32_t st = uint32_t(r[0]);
    if (!(st & (XE_SLOT_FULL | XE_SLOT_TOMB | XE_SLOT_BUSY))) return -1;
    if (st & XE_SLOT_TOMB) {
      bool eq = true;
      for (uint32_t k = 0; k < M.kwords; k++) eq = eq && r[1 + k] == kw[k];
      if (eq) {
        r[0] = (r[0] & ~0xffffffffull) | XE_SLOT_FULL;  // an LRU record keeps its reserved value id
        xe_wave_count(cnt, true);
        return int64_t(idx);
      }
    }
    idx = (idx + 1) & mask;
  }
  return -1;
}

// Reserve a record for HASH key kw of map M (one lane per distinct key; the keyed build): the key's
// present or earlier reserved record, else the first free slot of its chain, claimed BUSY by CAS,
// then the key words, then the tombstone state marked NEW. Records claimed in this launch (BUSY, NEW)
// hold other keys (each key has one reserving lane) and are passed without reading their key words,
// so no load needs acquire ordering. Returns false when the table has no free slot.
// hi: the record's high word for an LRU map (its reserved value id << 32), 0 for HASH; a tombstone already
// holding the key (an earlier unused reservation, an LRU eviction) takes it too.
XE_DEV bool hash_reserve(const XeDevMap& M, const uint64_t* kw, uint64_t hi = 0) {
  const uint32_t mask = M.cap - 1;
  uint32_t idx = uint32_t(xe_hash_words(kw, M.kwords, M.key_size)) & mask;
#pragma unroll 1
  for (uint32_t probe = 0; probe < M.cap;) {
    unsigned long long* r = reinterpret_cast<unsigned long long*>(M.keys + uint64_t(idx) * M.rwords);
    const unsigned long long w0 = xe_load_relaxed64(r);
    const uint32_t st = uint32_t(w0);
    if ((st & (XE_SLOT_FULL | XE_SLOT_TOMB)) && !(st & XE_SLOT_NEW)) {
      bool eq = true;
      for (uint32_t k = 0; k < M.kwords; k++) eq = eq && ((XE_GP(const uint64_t))r)[1 + k] == kw[k];
      if (eq) {
        if (hi && !(st & XE_SLOT_FULL)) ((XE_GP(uint64_t))r)[0] = XE_SLOT_TOMB | hi;
        return true;
      }
    } else if (!(st & (XE_SLOT_BUSY | XE_SLOT_NEW | XE_SLOT_FULL | XE_SLOT_TOMB))) {
      if (xe_atomic_cas64(r, w0, XE_SLOT_BUSY) != w0) continue;  // lost the slot: look at it again
      for (uint32_t k = 0; k < M.kwords; k++) ((XE_GP(uint64_t))r)[1 + k] = kw[k];
      ((XE_GP(uint64_t))r)[0] = XE_SLOT_TOMB | XE_SLOT_NEW | hi;
      return true;
    }
    idx = (idx + 1) & mask;
    probe++;
  }
  return false;
}
#endif

// read a key through a pointer register into zero-padded words; ReadRange errors give the nil key
// (maps_hash.go:50-53). Returns a panic code or 0. `kp`: the key words a per-program kernel proved
// equal to what the ReadRange returns (xe_jit.cpp key_shadows) — taken as they are.
XE_DEV int read_key(XeLane& L, const XeParams& P, const XeReg& R, const XeDevMap& M, uint64_t* kw, bool& empty,
                    uint32_t cm = XE_CM_ALL, const uint64_t* kp = nullptr) {
  if (kp) {
    for (int w = 0; w < XE_MAX_KEY / 8; w++) kw[w] = kp[w];
    empty = false;
    return 0;
  }
  for (int w = 0; w < XE_MAX_KEY / 8; w++) kw[w] = 0;
  int e = ptr_read_range(L, P, R, int64_t(M.key_size), [&](int64_t i, uint8_t b) {
    kw[i >> 3] |= uint64_t(b) << (8 * (i & 7));
  }, cm);
  if (XE_IS_PANIC(e)) return e;
  empty = e != 0 || M.key_size == 0;
  if (empty)
    for (int w = 0; w < XE_MAX_KEY / 8; w++) kw[w] = 0;
  return 0;
}

// The key bytes bpf_map_peek_elem hands to Lookup: ReadRange of a 4-slot ValueMemory holding one IMM 0
// (helper_functions.go:345-355): > 4 bytes is out of range (nil key), 3 bytes widen to 4 and panic.
XE_DEV int peek_key(const XeDevMap& M, uint64_t* kw, bool& empty) {
  for (int w = 0; w < XE_MAX_KEY / 8; w++) kw[w] = 0;
  empty = M.key_size > 4 || M.key_size == 0;
  if (M.key_size == 3) return XE_EV_PANIC | XE_P_INDEX;
  return 0;
}

#if XE_HAS_ORDERED
// ---- LRU_HASH (emulator/maps_hash_lru.go): value ids index the value pool; the UsageList is a doubly
// linked list over them (head = most recently used). link[4 v] = prev, [4 v + 1] = next, [4 v + 2] = slot.
XE_DEV XE_GP(uint32_t) lru_link(const XeDevMap& M, uint32_t v, int f) { return (XE_GP(uint32_t))M.link + 4 * uint64_t(v) + f; }
XE_DEV XE_GP(uint64_t) map_hdr(const XeDevMap& M, int w) { return (XE_GP(uint64_t))M.hdr + w; }
// A value's stamp (M.tag[v]): its place in the UsageList as a number, larger = more recently used, 0 =
// not in the list. Every touch writes the run's epoch (header word 5 = epoch << 48, set by the host per
// run) plus a number that grows in packet order within the run, so the list is also "the live values by
// stamp, descending": the parallel and keyed runs keep only stamps (lru_touch), and the host rebuilds the
// links from them on the device when a one-lane replay or a host read needs them (xe_runtime.cpp
// lru_relink). The fields never overlap: a concurrent touch adds packet << 16 | touch (packet < 2^32,
// touch < 2^16, lru_touch sends a packet's 65,536th touch to the replay); the one lane walking the batch
// in order counts its touches in header word 6 instead (< 2^48, no per-packet limit). The host renumbers
// every stamp before the 16-bit epoch would wrap (xe_runtime.cpp lru_renumber).
XE_DEV uint64_t lru_stamp(XeLane& L, const XeDevMap& M) {
  return *map_hdr(M, 5) | (uint64_t(L.pidx) << 16) | (L.oseq++ & 0xffffu);
}
XE_DEV uint64_t lru_stamp_seq(const XeDevMap& M) {  // one lane, packet order: the run's touch counter
  const uint64_t c = *map_hdr(M, 6) + 1;
  *map_hdr(M, 6) = c;
  return *map_hdr(M, 5) | (c & ((1ull << 48) - 1));
}
// The one-lane replay keeps no links either: its UsageList is an order log of touches in M.rec — word 0
// the first entry that may be live, word 1 the end, then a ring of M.data_cap (a power of two) entries
// {stamp, value id} from word 8. Every touch (promote, insert) appends; an entry is live while its stamp
// is still its value's, so the first live entry is the least recently used value, the one an insert into
// a full map evicts (maps_hash_lru.go:118-124, UsageList[len-1]). A touch is two stores instead of the
// list's chain of dependent loads (unlink, push to the head). The runtime seeds the log with the live
// values by stamp, oldest first, before each replay (xe_runtime.cpp lru_log_build), keeps data_cap at
// least twice the pool (so a compaction always frees half of it) and after the replay rebuilds the links
// from the stamps when something needs them, as after a parallel run (lru_relink).
XE_DEV XE_GP(uint64_t) lru_log_at(const XeDevMap& M, uint64_t j) {
  return (XE_GP(uint64_t))M.rec + 8 + 2 * (j & (M.data_cap - 1));
}
XE_DEV bool lru_log_live(const XeDevMap& M, uint64_t st, uint64_t v) { return ((XE_GP(const uint64_t))M.tag)[uint32_t(v)] == st; }
XE_DEV void lru_log_compact(const XeDevMap& M) {  // the live entries moved up behind the first, in order
  XE_GP(uint64_t) lg = (XE_GP(uint64_t))M.rec;
  const uint64_t h = lg[0], t = lg[1];
  uint64_t w = h;
#pragma unroll 1
  for (uint64_t r = h; r < t; r++) {
    XE_GP(const uint64_t) e = lru_log_at(M, r);
    const uint64_t st = e[0], v = e[1];
    if (!lru_log_live(M, st, v)) continue;
    XE_GP(uint64_t) o = lru_log_at(M, w++);
    o[0] = st;
    o[1] = v;
  }
  lg[1] = w;
}
XE_DEV void lru_log_push(const XeDevMap& M, uint32_t v, uint64_t st) {
  XE_GP(uint64_t) lg = (XE_GP(uint64_t))M.rec;
  if (lg[1] - lg[0] >= M.data_cap) lru_log_compact(M);
  const uint64_t t = lg[1];
  XE_GP(uint64_t) e = lru_log_at(M, t);
  e[0] = st;
  e[1] = v;
  lg[1] = t + 1;
}
XE_DEV uint32_t lru_log_oldest(const XeDevMap& M) {  // the least recently used live value (XE_NONE: none)
  XE_GP(uint64_t) lg = (XE_GP(uint64_t))M.rec;
  uint64_t h = lg[0];
  const uint64_t t = lg[1];
  uint32_t v = XE_NONE;
#pragma unroll 1
  for (; h < t; h++) {
    XE_GP(const uint64_t) e = lru_log_at(M, h);
    if (lru_log_live(M, e[0], e[1])) { v = uint32_t(e[1]); break; }
  }
  lg[0] = h;
  return v;
}
XE_DEV void lru_promote(XeLane& L, const XeDevMap& M, uint32_t v) {  // promote, :51-68
  const uint64_t st = lru_stamp_seq(M);
  ((XE_GP(uint64_t))M.tag)[v] = st;
  lru_log_push(M, v, st);
}
XE_DEV uint32_t lru_vid(const XeDevMap& M, int64_t slot) { return uint32_t(hash_word0(M, uint64_t(slot)) >> 32); }
// Concurrent modes: a touch (lookup hit, update) of value v by this packet — its last touch in packet order
// is what the UsageList keeps (the runtime relinks by it, lru_finalize)
// A hot flow's value takes an atomic max from most waves of a pass, all on one word: the parallel and
// SPEC passes skip the touches that cannot raise the word and spread the rest over M.list_cap replicas
// of the stamps (in M.state, pool_cap words apart; wave w uses replica w % list_cap), which the runtime
// folds into M.tag after the launch (xe_runtime.cpp lru_tag_fold). A chain's touches (one lane per key)
// go to M.tag itself.
XE_DEV int lru_touch(XeLane& L, const XeParams& P, const XeDevMap& M, uint32_t v) {
#if defined(XE_DEBUG_NO_LRU_TOUCH)  // cost experiments only: touches dropped (the UsageList is wrong)
  return 0;
#endif
  if (L.oseq >= 0xffffu) return XE_EV_ORD;
  unsigned long long* t = (unsigned long long*)M.tag + v;
  if (P.mode == XE_MODE_CHAIN) {
    xe_atomic_max64(t, lru_stamp(L, M));
    return 0;
  }
  if (M.list_cap > 1) t = (unsigned long long*)M.state + uint64_t(L.wave % M.list_cap) * M.pool_cap + v;
  // a hot flow's word almost always holds a newer stamp already (the waves walk the batch in step, so a
  // touch is rarely the newest so far): read it first. A stale read from this CU's cache is never too
  // new (stamps only grow), so a skipped atomic could never have raised the word.
  const unsigned long long st = lru_stamp(L, M);
  if (*(XE_GP(const unsigned long long))t < st) xe_atomic_max64(t, st);
  return 0;
}
// LRU lookup of a key (no promotion); value id or XE_NONE
XE_DEV uint32_t lru_find(const XeDevMap& M, const uint64_t* kw, bool empty) {
  const int64_t s = hash_find(M, kw, empty);
  return s < 0 ? XE_NONE : lru_vid(M, s);
}
// delete, :163-183 (evicted values keep their pool entry: pointers to them stay valid)
XE_DEV void lru_erase(const XeDevMap& M, uint32_t v) {
  ((XE_GP(uint64_t))M.tag)[v] = 0;  // out of the list (its log entries are no longer live)
  const uint32_t slot = *lru_link(M, v, 2);
  ((XE_GP(uint64_t))M.keys)[uint64_t(slot) * M.rwords] = XE_SLOT_TOMB;
  *map_hdr(M, 2) -= 1;
}
// The one-lane replay reuses evicted value ids. A packet may still hold a pointer to the value it evicted
// (Go keeps that ByteMemory alive), so an id freed by packet p is handed out again only to a later packet:
// a FIFO of freed ids in order-log words 2 (first) / 3 (last), linked through the freed entries' link
// words 0 (next) and 1 (the freeing packet), which only lru_relink's host-side list uses (rebuilt from the
// stamps after the run); the runtime empties it with every seed of the log (xe_lru_log_kernel). Without
// it the pool only grew: a stream of evicting replays climbed to the value ids the handles can name.
XE_DEV void lru_free_push(const XeLane& L, const XeDevMap& M, uint32_t v) {
  XE_GP(uint64_t) lg = (XE_GP(uint64_t))M.rec;
  *lru_link(M, v, 0) = XE_NONE;
  *lru_link(M, v, 1) = L.pidx;
  if (lg[3] == XE_NONE) lg[2] = v;
  else *lru_link(M, uint32_t(lg[3]), 0) = v;
  lg[3] = v;
}
XE_DEV uint32_t lru_free_pop(const XeLane& L, const XeDevMap& M) {
  XE_GP(uint64_t) lg = (XE_GP(uint64_t))M.rec;
  const uint64_t h = lg[2];
  if (h == XE_NONE || *lru_link(M, uint32_t(h), 1) >= L.pidx) return XE_NONE;
  lg[2] = *lru_link(M, uint32_t(h), 0);
  if (lg[2] == XE_NONE) lg[3] = XE_NONE;
  return uint32_t(h);
}
XE_DEV int lru_insert(XeLane& L, const XeDevMap& M, const uint64_t* kw, bool empty, uint32_t& v) {
  v = lru_free_pop(L, M);
  if (v == XE_NONE) {
    const uint64_t nv = *map_hdr(M, 3);
    if (nv >= M.pool_cap) return XE_EV_CAP;
    v = uint32_t(nv);
    *map_hdr(M, 3) = nv + 1;
  }
  const int64_t slot = hash_insert_new(M, kw, empty);
  ((XE_GP(uint64_t))M.keys)[uint64_t(slot) * M.rwords] = XE_SLOT_FULL | (uint64_t(v) << 32);
  *lru_link(M, v, 2) = uint32_t(slot);
  ((XE_GP(uint32_t))M.elen)[v] = M.value_size;
  *map_hdr(M, 2) += 1;
  const uint64_t st = lru_stamp_seq(M);  // appended to the UsageList, then promoted to its top (:144-150)
  ((XE_GP(uint64_t))M.tag)[v] = st;
  lru_log_push(M, v, st);
  return 0;
}

// ---- QUEUE / STACK (emulator/maps_queue.go, maps_stack.go): element ids index the element pool;
// link holds the list (a ring of list_cap ids for a queue). hdr = {head, count, next id, -, is_stack}
XE_DEV uint32_t list_at(const XeDevMap& M, uint64_t i) {  // Values[i] in Go slice order
  const uint64_t head = *map_hdr(M, 0);
  return ((XE_GP(const uint32_t))M.link)[*map_hdr(M, 4) ? i : (head + i) % M.list_cap];
}

// ---- QUEUE / STACK operations in a parallel run (P.list; xe_runtime.cpp runs the passes).
// In packet order, packet i's list operations see the batch's start contents minus the pops of the
// packets before it (popbase[i], the count pass's prefix sum) and of its own earlier pops, plus the
// pushes of the packets before it. Pushes only append (after the last element), so a queue position
// inside the start contents does not depend on them; anything else (a queue position past them, any
// stack position: pushes land on top) assumes no push came before and records the packet in sens, and
// the host replays the batch in order when a push did (push[m] < sens[m]).
XE_DEV bool list_par(const XeParams& P) { return P.list && P.mode == XE_MODE_PARALLEL; }
// (only a popped list loses elements: a peek or lookup of another list sees its start contents)
XE_DEV uint64_t list_pops_before(const XeLane& L, const XeParams& P, uint32_t m) {
  const uint32_t j = P.pop_mode == 2 ? uint32_t(P.pop_slot[m]) : 0xffu;
  if (j >= XE_POP_SLOTS) return 0;
  return uint64_t(P.popbase[uint64_t(j) * P.pop_stride + L.pidx]) + ((L.npops >> (8 * j)) & 0xffu);
}
XE_DEV void list_mark_sens(const XeLane& L, const XeParams& P, uint32_t m) {
  xe_atomic_max32(&P.list->sens[m], L.pidx + 1u);
  xe_atomic_min32(&P.list->senslo[m], L.pidx);
}
// position (Go slice index) of Values[kv] for the lane's packet; false: out of range
XE_DEV bool list_pos(const XeLane& L, const XeParams& P, uint32_t m, const XeDevMap& M, int64_t kv, int64_t& pos) {
  const int64_t q = int64_t(list_pops_before(L, P, m)), cnt0 = int64_t(P.list->cnt0[m]);
  if (!*map_hdr(M, 4)) {  // queue: front = start position q
    if (kv < 0) return false;
    if (q + kv >= cnt0) { list_mark_sens(L, P, m); return false; }
    pos = q + kv;
    return true;
  }
  list_mark_sens(L, P, m);  // stack: Lookup(kv) counts from the top
  const int64_t c = cnt0 - q;
  if (kv < 0 || kv >= c) return false;
  pos = c - 1 - kv;
  return true;
}
#endif

// ------------------------------------------------------------------ helpers
// regToMap, helper_functions.go:109-130. m = 0 means "R0 := 0, helper returns nil".
XE_DEV int reg_to_map(XeLane& L, const XeParams& P, uint32_t& m, uint32_t cm1 = XE_CM_ALL) {
  const XeReg R1 = reg_get(L, 1);
  XE_NILCHK(R1);
  int64_t idx = R1.v;
  if ((cm1 & ~(XE_CM_IMM | XE_CM_ALIAS)) && XE_T_KIND(R1.t) == XE_KIND_MEMPTR) {
    uint32_t k, oh, al; int64_t v;
    if (int e = mem_read(L, P, R1.h, R1.v, 4, true, k, oh, v, al, cm1)) return e;
    idx = v;
  }
  if (idx < 1 || idx > int64_t(P.nmaps)) {
    reg_replace(L, 0, XE_KIND_IMM, 0, 0, 0);
    m = 0;
    return 0;
  }
  m = uint32_t(idx);
  return 0;
}

XE_DEV int helper_errno_result(XeLane& L, int64_t v) {
  reg_replace(L, 0, XE_KIND_IMM, 0, v, 0);
  return 0;
}
XE_DEV int in_helper(int e) { return (e & 0xf000) ? e : (e | XE_E_IN_HELPER); }

// Map.Lookup of map m for `key` (a register value: pointer or not). Sets out (the RegisterValue
// Lookup returns) or returns errno via *errno_out (sentinel errors), a VM error or a panic.
// ArrayMap.Lookup maps_array.go:65-87, HashMap.Lookup maps_hash.go:44-63, HashMapLRU.Lookup
// maps_hash_lru.go:70-91, QueueMap/StackMap.Lookup maps_queue.go:39-58 / maps_stack.go:38-58,
// PerfEventArray.Lookup maps_perf_event_array.go:45-65. `peek`: the key is bpf_map_peek_elem's IMM 0.
XE_DEV int map_lookup(XeLane& L, const XeParams& P, uint32_t m, const XeReg& K, bool peek, XeReg& out, int64_t& err,
                      uint32_t cm2 = XE_CM_ALL, const uint64_t* kp = nullptr) {
  const XeDevMap M = map_desc(L, m);
  err = 0;
  out = XeReg{0, 0, XE_KIND_IMM};
  if (!peek && !XE_ISPTR(K.t)) { err = -14; return 0; }  // errMapKeyNoPtr
  if (XE_HAS_ARRAY && M.kind == XE_DM_ARRAY) {
    int64_t kv = 0;
    if (!peek) {
      uint32_t kind = XE_T_KIND(K.t);
      int64_t off = kind == XE_KIND_FRAMEPTR ? xe_wadd(XE_FRAME, K.v) : K.v;
      uint32_t k, oh, al;
      int e = mem_read(L, P, K.h, off, 4, true, k, oh, kv, al, cm2);
      if (XE_IS_PANIC(e)) return e;
      if (e) return XE_EV_PANIC | XE_P_NIL_DEREF;  // error ignored, nil keyValReg.Value()
    }
    int64_t voff = xe_wmul(kv, int64_t(M.value_size));
    if (voff < int64_t(M.vals_bytes)) out = XeReg{voff, xe_h_make(XE_H_ARRAY, m, 0), XE_KIND_MEMPTR};
    return 0;
  }
  if ((XE_HAS_HASH && M.kind == XE_DM_HASH) || (XE_HAS_ORDERED && M.kind == XE_DM_LRU)) {
    uint64_t kw[XE_MAX_KEY / 8];
    bool empty = false;
    if (int e = peek ? peek_key(M, kw, empty) : read_key(L, P, K, M, kw, empty, cm2, kp)) return e;
#if XE_KEYED
    uint64_t kid = 0;
    if ((M.kind == XE_DM_HASH || M.kind == XE_DM_LRU) && (P.mode == XE_MODE_SPEC || P.mode == XE_MODE_CHAIN)) {
      kid = kid_hash(m, M, kw, empty);  // the key's presence is read
      if (int e = key_touch(L, P, kid, false)) return e;
    }
#endif
#if XE_HAS_ORDERED
    if (M.kind == XE_DM_LRU) {
      const uint32_t v = lru_find(M, kw, empty);
      if (v == XE_NONE) return 0;
      if (xe_concurrent(P)) {
        // a lookup promotes (maps_hash_lru.go:70-91): in packet order the key ends up at the head as
        // often as it was touched last; the run keeps each value's last touch (packet << 16 | call) + 1
        // and the runtime moves the touched keys to the UsageList's head by it (ordered_finalize)
        if (int e = lru_touch(L, P, M, v)) return e;
        out = XeReg{0, hv_make(M, m, v), XE_KIND_MEMPTR};
#if XE_KEYED
        if (kid) { L.kh = out.h; L.kk = kid; }
#endif
        return 0;
      }
      if (!xe_peeking(L)) lru_promote(L, M, v);
      out = XeReg{0, hv_make(M, m, v), XE_KIND_MEMPTR};
      return 0;
    }
#endif
    int64_t slot = hash_find(M, kw, empty);
    if (slot >= 0) out = XeReg{0, hv_make(M, m, uint32_t(slot)), XE_KIND_MEMPTR};
#if XE_KEYED
    if (slot >= 0 && kid) { L.kh = out.h; L.kk = kid; }
#endif
    return 0;
  }
#if XE_HAS_ORDERED
  if (M.kind == XE_DM_LIST || M.kind == XE_DM_PERF) {
    if (xe_peeking(L)) return XE_EV_STOP;
    // the list changes in packet order: in parallel only through the list-run rules (list_par)
    if (xe_concurrent(P) && !(M.kind == XE_DM_LIST && list_par(P))) return XE_EV_ORD;
    // count pass: the packet's rank needs only its pops before here (none): it stops (a later pop of it
    // finds no rank in the next pass and replays the batch in order)
    if (xe_concurrent(P) && P.pop_mode == 1) return XE_EV_STOP;
    int64_t kv = 0;
    if (!peek) {
      int64_t off = XE_T_KIND(K.t) == XE_KIND_FRAMEPTR ? xe_wadd(XE_FRAME, K.v) : K.v;
      uint32_t k, oh, al;
      int e = mem_read(L, P, K.h, off, 4, true, k, oh, kv, al, cm2);
      if (XE_IS_PANIC(e)) return e;
      if (e) return XE_EV_PANIC | XE_P_NIL_DEREF;
    }
    if (M.kind == XE_DM_PERF) {
      const int64_t cnt = int64_t(*map_hdr(M, 0));
      if (kv >= cnt) return 0;
      if (kv < 0) return XE_EV_PANIC | XE_P_INDEX;
      out = XeReg{0, xe_h_make(XE_H_QVAL, m, uint32_t(kv)), XE_KIND_MEMPTR};
      return 0;
    }
    if (xe_concurrent(P)) {  // Values[kv] in packet order: list_pos
      int64_t pos;
      if (!list_pos(L, P, m, M, kv, pos)) { err = -7; return 0; }  // errMapOutOfMemory
      out = XeReg{0, xe_h_make(XE_H_QVAL, m, list_at(M, uint64_t(pos))), XE_KIND_MEMPTR};
      return 0;
    }
    const int64_t cnt = int64_t(*map_hdr(M, 1));
    if (kv < 0 || kv >= cnt) { err = -7; return 0; }  // errMapOutOfMemory
    const uint32_t id = list_at(M, uint64_t(*map_hdr(M, 4) ? cnt - 1 - kv : kv));
    out = XeReg{0, xe_h_make(XE_H_QVAL, m, id), XE_KIND_MEMPTR};
    return 0;
  }
#endif
  return XE_EV_UNSUP;
}

// MapLookupElement, helper_functions.go:46-73
XE_DEV int helper_lookup(XeLane& L, const XeParams& P, uint32_t cm1 = XE_CM_ALL, uint32_t cm2 = XE_CM_ALL,
                         const uint64_t* kp = nullptr) {
  uint32_t m;
  if (int e = reg_to_map(L, P, m, cm1)) return in_helper(e);
  if (!m) return 0;
  XeReg out;
  int64_t err;
  if (int e = map_lookup(L, P, m, reg_get(L, 2), false, out, err, cm2, kp)) return in_helper(e);
  if (err) return helper_errno_result(L, err);
  reg_put(L, 0, out);
  return 0;
}

// ReadRange(0, n) of register R into the bytes at dst (a map value / pool element). Returns 0, a
// panic, or 1 when the range could not be read (the Go code ignores that error and stores a nil backing).
XE_DEV int read_value_into(XeLane& L, const XeParams& P, const XeReg& R, int64_t n, uint8_t* dst, uint32_t cm = XE_CM_ALL) {
  int ve = ptr_read_range(L, P, R, n, [&](int64_t, uint8_t) {}, cm);  // validate first: a panic leaves dst untouched
  if (XE_IS_PANIC(ve)) return ve;
  if (ve) return 1;
  ptr_read_range(L, P, R, n, [&](int64_t i, uint8_t b) { ((XE_GP(uint8_t))dst)[i] = b; }, cm);
  return 0;
}

// MapUpdateElement, helper_functions.go:76-101
XE_DEV int helper_update(XeLane& L, const XeParams& P, uint32_t cm1 = XE_CM_ALL, uint32_t cm2 = XE_CM_ALL,
                         uint32_t cm3 = XE_CM_ALL, const uint64_t* kp = nullptr) {
  uint32_t m;
  if (int e = reg_to_map(L, P, m, cm1)) return in_helper(e);
  if (!m) return 0;
  XE_NILCHK(reg_get(L, 4));  // BPFAttrMapElemFlags(R4.Value())
  const XeDevMap M = map_desc(L, m);
  const XeReg R2 = reg_get(L, 2), R3 = reg_get(L, 3);
  if (XE_HAS_ARRAY && M.kind == XE_DM_ARRAY) {  // ArrayMap.Update, maps_array.go:89-131
    if (XE_T_KIND(R3.t) != XE_KIND_MEMPTR) return helper_errno_result(L, -14);
    if (XE_T_KIND(R2.t) != XE_KIND_MEMPTR) return helper_errno_result(L, -14);
    uint32_t k, oh, al; int64_t kv;
    if (int e = mem_read(L, P, R2.h, R2.v, 4, true, k, oh, kv, al, cm2)) return in_helper(e);
    if (kv >= int64_t(M.vals_bytes)) return helper_errno_result(L, -7);
#if XE_KEYED
    if (int e = key_touch(L, P, kid_array(m, uint64_t(kv)), true)) return e;  // element kv is written
#endif
#pragma unroll 1
    for (int64_t i = 0; i < int64_t(M.value_size); i++) {
      int64_t v;
      if (int e = mem_read(L, P, R3.h, i, 1, true, k, oh, v, al, cm3)) return in_helper(e);  // ignores the value ptr offset
      int64_t dst = xe_wadd(xe_wmul(kv, int64_t(M.value_size)), i);
      if (int e = bounds(dst, 1, int64_t(M.vals_bytes))) return in_helper(e);
      if (P.mode == XE_MODE_PARALLEL) return XE_EV_ORD;
      if (P.mode == XE_MODE_SPEC) continue;  // held back
#if XE_GEN
      if (int e = bm_before_write(L, P, xe_h_make(XE_H_ARRAY, m, 0))) return e;
#endif
      M.vals[dst] = uint8_t(v);
    }
    return helper_errno_result(L, 0);
  }
  if (XE_HAS_HASH && M.kind == XE_DM_HASH) {  // HashMap.Update, maps_hash.go:65-123
    if (!XE_ISPTR(R2.t)) return helper_errno_result(L, -14);
    uint64_t kw[XE_MAX_KEY / 8];
    bool empty = false;
    if (int e = read_key(L, P, R2, M, kw, empty, cm2, kp)) return e;
#if XE_KEYED
    const uint64_t kid = kid_hash(m, M, kw, empty);
    if (int e = key_touch(L, P, kid, false)) return e;  // presence (and the count) are read
#endif
    int64_t slot = hash_find(M, kw, empty);
    if (slot < 0 && uint64_t(*M.count) + 1 > M.max_entries) return helper_errno_result(L, -7);
    if (!XE_ISPTR(R3.t)) return helper_errno_result(L, -14);
    // value ReadRange: validate first (a panic must leave the map untouched)
    int ve = ptr_read_range(L, P, R3, int64_t(M.value_size), [&](int64_t, uint8_t) {}, cm3);
    if (XE_IS_PANIC(ve)) return ve;
    if (P.mode == XE_MODE_PARALLEL) return XE_EV_ORD;
#if XE_KEYED
    if (int e = key_touch(L, P, kid, true)) return e;
    if (P.mode == XE_MODE_SPEC) {  // held back; a new key goes to the insert log (its slot is reserved)
      // a new key: its words go to the packet's next ikey slot (the build reserves its slot record)
      if (slot < 0) {
        if (L.kins >= XE_KINS) {
          L.kn = XE_KLOG + 1;  // more inserts than slots: reported as a key-log overflow
        } else {
          XE_GP(uint64_t) en = (XE_GP(uint64_t))P.K.ikey + (uint64_t(L.kpkt) * XE_KINS + L.kins) * P.K.kw;
#pragma unroll
          for (uint32_t w = 0; w < XE_MAX_KEY / 8; w++)  // constant trip count: kw stays in registers
            if (w + 1 < P.K.kw) en[1 + w] = kw[w];
          en[0] = uint64_t(m) | (empty ? 0x100ull : 0ull) | XE_KEY_VALID;
#pragma unroll
          for (uint32_t j = 0; j < XE_KLOG; j++)
            if (j < L.kn && (L.klog[j] & ~XE_KLOG_FLAGS) == kid) L.klog[j] |= XE_KLOG_INS | (uint64_t(L.kins) << 3);
          L.kins++;
        }
      }
      return helper_errno_result(L, 0);
    }
    if (slot < 0 && P.mode == XE_MODE_CHAIN) {
      slot = hash_claim(M, kw, empty, P.K.cins + m * XE_KSTRIPES + (L.wave % XE_KSTRIPES));
      if (slot < 0) return XE_EV_ORD;
    }
#endif
    if (slot < 0) slot = hash_insert_new(M, kw, empty);
#if XE_GEN
    if (int e = bm_before_write(L, P, hv_make(M, m, uint32_t(slot)))) return e;
#endif
    uint8_t* dst = M.vals + uint64_t(slot) * M.value_size;
    if (ve) {
      hash_set_state(M, uint64_t(slot), hash_state(M, uint64_t(slot)) | XE_SLOT_VLEN0);  // nil backing
    } else {
      hash_set_state(M, uint64_t(slot), hash_state(M, uint64_t(slot)) & ~XE_SLOT_VLEN0);
      ptr_read_range(L, P, R3, int64_t(M.value_size), [&](int64_t i, uint8_t b) { dst[i] = b; }, cm3);
    }
    return helper_errno_result(L, 0);
  }
#if XE_HAS_ORDERED
  if (M.kind == XE_DM_LRU) {  // HashMapLRU.Update, maps_hash_lru.go:93-161
    if (!XE_ISPTR(R2.t)) return helper_errno_result(L, -14);
    if (P.mode == XE_MODE_PARALLEL) return XE_EV_ORD;
    uint64_t kw[XE_MAX_KEY / 8];
    bool empty = false;
    if (int e = read_key(L, P, R2, M, kw, empty, cm2, kp)) return e;
#if XE_KEYED
    const uint64_t kid = kid_hash(m, M, kw, empty);
    if (P.mode == XE_MODE_SPEC || P.mode == XE_MODE_CHAIN)
      if (int e = key_touch(L, P, kid, false)) return e;  // presence (and the count) are read
#endif
    uint32_t v = lru_find(M, kw, empty);
    // keyed batches (XE_MODE_SPEC / XE_MODE_CHAIN) decide evictions in the build instead: SPEC logs the
    // insert, a chain's insert deletes the victim the build gave it (keyed_evict_item)
    if (v == XE_NONE && *map_hdr(M, 2) + 1 > M.max_entries && P.mode != XE_MODE_SPEC && P.mode != XE_MODE_CHAIN) {
      if (xe_concurrent(P)) return XE_EV_ORD;
      const uint32_t tail = lru_log_oldest(M);
      if (tail == XE_NONE) return XE_EV_PANIC | XE_P_INDEX;  // UsageList[len-1] of an empty list
      if (int e = bm_before_write(L, P, hv_make(M, m, tail))) return e;
      lru_erase(M, tail);  // evicted before the value is checked
      lru_free_push(L, M, tail);
    }
#if XE_KEYED
    // a new key whose value check fails: in the reference the eviction of a full map has already happened
    // (:113-119 before :134-137) and stays. Keyed batches decide evictions in the build from the logged
    // inserts, and this packet logs none, so whether the map is full here depends on the other packets'
    // inserts: the batch replays in order
    if (v == XE_NONE && (P.mode == XE_MODE_SPEC || P.mode == XE_MODE_CHAIN) && !XE_ISPTR(R3.t)) return XE_EV_ORD;
#endif
    if (!XE_ISPTR(R3.t)) return helper_errno_result(L, -14);
    int ve = ptr_read_range(L, P, R3, int64_t(M.value_size), [&](int64_t, uint8_t) {}, cm3);
#if XE_KEYED
    if (XE_IS_PANIC(ve) && v == XE_NONE && (P.mode == XE_MODE_SPEC || P.mode == XE_MODE_CHAIN)) return XE_EV_ORD;
#endif
    if (XE_IS_PANIC(ve)) return ve;
#if XE_KEYED
    if (P.mode == XE_MODE_SPEC || P.mode == XE_MODE_CHAIN)
      if (int e = key_touch(L, P, kid, true)) return e;
    if (P.mode == XE_MODE_SPEC) {  // held back; a new key goes to the insert log (its record is reserved)
      if (v == XE_NONE) {
        if (L.kins >= XE_KINS) {
          L.kn = XE_KLOG + 1;  // more inserts than slots: reported as a key-log overflow
        } else {
          XE_GP(uint64_t) en = (XE_GP(uint64_t))P.K.ikey + (uint64_t(L.kpkt) * XE_KINS + L.kins) * P.K.kw;
#pragma unroll
          for (uint32_t w = 0; w < XE_MAX_KEY / 8; w++)
            if (w + 1 < P.K.kw) en[1 + w] = kw[w];
          en[0] = uint64_t(m) | (empty ? 0x100ull : 0ull) | XE_KEY_VALID;
#pragma unroll
          for (uint32_t j = 0; j < XE_KLOG; j++)
            if (j < L.kn && (L.klog[j] & ~XE_KLOG_FLAGS) == kid) L.klog[j] |= XE_KLOG_INS | (uint64_t(L.kins) << 3);
          L.kins++;
        }
      }
      return helper_errno_result(L, 0);
    }
    if (P.mode == XE_MODE_CHAIN && v == XE_NONE) {
      // the first insert of the key must be the one the build ranked (XE_KS_FIRST: its victim, if any,
      // was chosen by that rank)
      const int64_t d = dset_find(P.K, kid);
      if (d < 0) return XE_EV_ORD;
      const uint32_t first = P.K.dfirst[d];
      if (first != XE_NONE && first != L.pidx) return XE_EV_ORD;
      // the record reserved for this key holds its value id (xe_runtime.cpp keyed: XE_KS_LRUID, RESERVE)
      const int64_t slot = empty ? -1 : hash_claim(M, kw, false, P.K.cins + m * XE_KSTRIPES + (L.wave % XE_KSTRIPES));
      if (slot < 0) return XE_EV_ORD;  // the nil key (no reservation) or a key that left its chain
      v = lru_vid(M, slot);
      const uint32_t victim = P.K.dvict[d];
      if (victim != XE_NONE) {
        // delete, :163-183: out of the UsageList (stamp 0), its record a tombstone; the new key's value id
        // is the victim's (keyed_lruid_item), whose pool entry it overwrites below
        ((XE_GP(uint64_t))M.tag)[victim] = 0;
        ((XE_GP(uint64_t))M.keys)[uint64_t(*lru_link(M, victim, 2)) * M.rwords] = XE_SLOT_TOMB;
      }
      *lru_link(M, v, 2) = uint32_t(slot);
    }
#endif
    if (v == XE_NONE) {
      if (int e = lru_insert(L, M, kw, empty, v)) return e;
    } else if (xe_concurrent(P)) {
      if (int e = lru_touch(L, P, M, v)) return e;  // appended + promoted, or promoted (:144-150)
      if (int e = bm_before_write(L, P, hv_make(M, m, v))) return e;
    } else {
      lru_promote(L, M, v);
      if (int e = bm_before_write(L, P, hv_make(M, m, v))) return e;
    }
    uint8_t* dst = M.vals + uint64_t(v) * M.value_size;
    ((XE_GP(uint32_t))M.elen)[v] = ve ? 0u : M.value_size;
    if (ve) *map_hdr(M, 4) = 1;  // a nil-backed value exists (bmem_resolve reads lengths from now on)
    if (!ve) ptr_read_range(L, P, R3, int64_t(M.value_size), [&](int64_t i, uint8_t b) { ((XE_GP(uint8_t))dst)[i] = b; }, cm3);
    return helper_errno_result(L, 0);
  }
  if (M.kind == XE_DM_PERF) return helper_errno_result(L, -1);  // errMapNotImplemented -> eperm
  if (M.kind == XE_DM_LIST) return XE_E_MAP_OP | XE_E_IN_HELPER;  // "update not available on this map type"
#endif
  return XE_EV_UNSUP;
}

#if XE_HAS_ORDERED
// QueueMap/StackMap.Push (maps_queue.go:60-77) and PerfEventArray.Push (maps_perf_event_array.go:101-115):
// append ReadRange(0, size) of register R (nil backing when the range cannot be read)
XE_COLD int list_push(XeLane& L, const XeParams& P, uint32_t m, const XeDevMap& M, const XeReg& R, int64_t size, int64_t& err) {
  err = 0;
  if (!XE_ISPTR(R.t)) { err = -14; return 0; }  // errMapValNoPtr / errMapKeyNoPtr
  if (M.kind == XE_DM_PERF) {
    const uint64_t c = *map_hdr(M, 0), used = *map_hdr(M, 1);
    int ve = ptr_read_range(L, P, R, size, [&](int64_t, uint8_t) {});
    if (XE_IS_PANIC(ve)) return ve;
    const uint64_t n = ve ? 0 : uint64_t(size);
    if (c >= M.pool_cap || used + n > M.data_cap) return XE_EV_CAP;
    if (n) ptr_read_range(L, P, R, size, [&](int64_t i, uint8_t b) { ((XE_GP(uint8_t))M.vals)[used + uint64_t(i)] = b; });
    ((XE_GP(uint64_t))M.rec)[2 * c] = used;
    ((XE_GP(uint64_t))M.rec)[2 * c + 1] = n;
    *map_hdr(M, 0) = c + 1;
    *map_hdr(M, 1) = used + ((n + 7) & ~uint64_t(7));
    return 0;
  }
  const uint64_t id = *map_hdr(M, 2), cnt = *map_hdr(M, 1);
  if (id >= M.pool_cap || cnt >= M.list_cap) return XE_EV_CAP;
  uint8_t* dst = M.vals + id * M.value_size;
  int e = read_value_into(L, P, R, size, dst);
  if (XE_IS_PANIC(e)) return e;
  ((XE_GP(uint32_t))M.elen)[id] = e ? 0u : uint32_t(size);
  *map_hdr(M, 2) = id + 1;
  const uint64_t at = *map_hdr(M, 4) ? cnt : (*map_hdr(M, 0) + cnt) % M.list_cap;
  ((XE_GP(uint32_t))M.link)[at] = uint32_t(id);
  *map_hdr(M, 1) = cnt + 1;
  return 0;
}

// The same append in parallel mode: element ids / event slots and event bytes are claimed with atomics
// (in whatever order lanes get there) and each element is tagged with its packet index and the packet's
// append number; after the run the runtime sorts the run's elements by tag into their list positions /
// event records (XeAppendArgs), which is the order the packet-by-packet loop appends them in. Push never
// fails in the reference (an unbounded Go append), so appends commute up to that order.
XE_COLD int list_push_par(XeLane& L, const XeParams& P, uint32_t m, const XeDevMap& M, const XeReg& R, int64_t size,
                          int64_t& err) {
  err = 0;
  if (!XE_ISPTR(R.t)) { err = -14; return 0; }
  if (L.oseq >= 0xffffu) return XE_EV_ORD;  // the tag's append number is 16 bits
  if (P.list && M.kind == XE_DM_LIST) xe_atomic_min32(&P.list->push[m], L.pidx);  // (list_pos)
  const uint64_t tag = (uint64_t(L.pidx) << 16) | L.oseq++;
  if (M.kind == XE_DM_PERF) {
    int ve = ptr_read_range(L, P, R, size, [&](int64_t, uint8_t) {});
    if (XE_IS_PANIC(ve)) return ve;
    const uint64_t n = ve ? 0 : uint64_t(size);
    const uint64_t c = xe_atomic_add64((unsigned long long*)map_hdr(M, 0), 1ull);
    const uint64_t used = xe_atomic_add64((unsigned long long*)map_hdr(M, 1), (n + 7) & ~uint64_t(7));
    if (c >= M.pool_cap || used + n > M.data_cap) return XE_EV_CAP;
    if (n) ptr_read_range(L, P, R, size, [&](int64_t i, uint8_t b) { ((XE_GP(uint8_t))M.vals)[used + uint64_t(i)] = b; });
    ((XE_GP(uint64_t))M.rec)[2 * c] = used;
    ((XE_GP(uint64_t))M.rec)[2 * c + 1] = n;
    ((XE_GP(uint64_t))M.tag)[c] = tag;
    return 0;
  }
  const uint64_t id = xe_atomic_add64((unsigned long long*)map_hdr(M, 2), 1ull);
  const uint64_t cnt = xe_atomic_add64((unsigned long long*)map_hdr(M, 1), 1ull);
  if (id >= M.pool_cap || cnt >= M.list_cap) return XE_EV_CAP;
  uint8_t* dst = M.vals + id * M.value_size;
  int e = read_value_into(L, P, R, size, dst);
  if (XE_IS_PANIC(e)) return e;
  ((XE_GP(uint32_t))M.elen)[id] = e ? 0u : uint32_t(size);
  ((XE_GP(uint64_t))M.tag)[id] = tag;
  return 0;
}

// TailCall, helper_functions.go:133-210. Returns XE_EV_JUMP on success (PI switched, PC := -1).
#define XE_EV_JUMP 0x5000
XE_COLD int helper_tail_call(XeLane& L, const XeParams& P) {
#if XE_GEN
  const XeReg R2 = reg_get(L, 2);
  XE_NILCHK(R2);
  if (R2.v < 1 || R2.v > int64_t(P.nmaps)) return helper_errno_result(L, -14);
  const uint32_t m = uint32_t(R2.v);
  const XeDevMap M = map_desc(L, m);
  if (M.btype != XE_MAP_PROG_ARRAY) return helper_errno_result(L, -14);
  // key: a ValueMemory of 4 slots all holding the R3 object itself: Deref(0, W) returns it
  const XeReg R3 = reg_get(L, 3);
  XE_NILCHK(R3);
  const int64_t off = xe_wmul(R3.v, int64_t(M.value_size));
  if (off >= int64_t(M.vals_bytes)) return XE_E_MAP_OP | XE_E_IN_HELPER;  // "lookup didn't return a pointer"
  uint32_t k, oh, al; int64_t prog;
  if (int e = mem_read(L, P, xe_h_make(XE_H_ARRAY, m, 0), off, 4, true, k, oh, prog, al)) return in_helper(e);
  if (int64_t(P.nprogs) + 1 < prog) return helper_errno_result(L, -14);  // len(vm.Programs) < progIdx
  if (prog == 0) return XE_E_NO_PROGRAM | XE_E_IN_HELPER;
  L.pi = int32_t(prog);
  reg_replace(L, 0, XE_KIND_IMM, 0, 0, 0);
  return XE_EV_JUMP;
#else
  return XE_EV_UNSUP;
#endif
}
#endif

#if XE_HELPER_TABLE
// A host helper (xe_set_helper, VM.HelperFunctions): R1..R5 go to the host thread that runs the batch
// through the mailbox, R0 comes back as an IMM. Packet order only (the one-lane path): a parallel pass
// defers the packet to it.
XE_COLD int host_helper(XeLane& L, const XeParams& P, uint32_t id) {
  if (xe_concurrent(P) || !P.hostcall) return XE_EV_ORD;
  int64_t a[5];
  uint8_t k[5];
#pragma unroll
  for (int r = 0; r < 5; r++) {
    const XeReg R = reg_get(L, r + 1);
    a[r] = R.v;
    k[r] = uint8_t(XE_T_KIND(R.t));
  }
  XeHostCall* H = P.hostcall;
  int32_t err = 0;
  int64_t r0 = 0;
#if defined(__HIPCC__)
  const uint32_t seq = __hip_atomic_load(&H->req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + 1u;
  __hip_atomic_store(&H->id, id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&H->packet, L.pidx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#pragma unroll
  for (int r = 0; r < 5; r++) {
    __hip_atomic_store(&H->args[r], a[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    H->kinds[r] = k[r];
  }
  __hip_atomic_store(&H->req, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint64_t t0 = wall_clock64();
  while (__hip_atomic_load(&H->ack, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != seq) {
    if (wall_clock64() - t0 > XE_HOSTCALL_TIMEOUT_TICKS) return XE_E_HOST_HELPER | XE_E_IN_HELPER;  // nobody served it
    __builtin_amdgcn_s_sleep(32);
  }
  err = __hip_atomic_load(&H->err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  r0 = __hip_atomic_load(&H->r0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#else  // host simulation: the kernel runs on the calling thread, which calls the function in place
  err = H->fn[id] ? H->fn[id](H->user[id], L.pidx, a, k, &r0) : 1;
#endif
  if (err) return XE_E_HOST_HELPER | XE_E_IN_HELPER;
  reg_replace(L, 0, XE_KIND_IMM, 0, r0, 0);
  return 0;
}
#endif

XE_DEV int call_helper(XeLane& L, const XeParams& P, int64_t fn, uint32_t cm1 = XE_CM_ALL, uint32_t cm2 = XE_CM_ALL,
                       uint32_t cm3 = XE_CM_ALL) {
  if (xe_peeking(L) && fn != 1) return XE_EV_STOP;
  if (fn >= 192) return XE_E_NO_HELPER;
  if (fn < 0) return XE_EV_PANIC | XE_P_INDEX;
#if XE_HELPER_TABLE
  {
    const uint32_t w = uint32_t(fn) >> 6;
    const uint64_t b = 1ull << (uint32_t(fn) & 63u);
    if (P.nil_helpers[w] & b) return XE_E_NO_HELPER;  // inst_call_helper.go:26-28
    if (P.host_helpers[w] & b) return host_helper(L, P, uint32_t(fn));
  }
#endif
  switch (fn) {
    case 1: return helper_lookup(L, P, cm1, cm2);
    case 2: return helper_update(L, P, cm1, cm2, cm3);
    case 3: return XE_E_NOT_IMPL | XE_E_IN_HELPER;
    case 14: reg_replace(L, 0, XE_KIND_IMM, 0, (int64_t(1234) << 32) + 5678, 0); return 0;
#if XE_HAS_ORDERED
    case 12: return helper_tail_call(L, P);
    case 25: {  // PerfEventOutput :219-252: R2 = map index (no deref), R4 = data, R5 = size
      const XeReg R2 = reg_get(L, 2);
      XE_NILCHK(R2);
      if (R2.v < 1 || R2.v > int64_t(P.nmaps)) return helper_errno_result(L, -14);
      const uint32_t m = uint32_t(R2.v);
      const XeDevMap M = map_desc(L, m);
      if (M.kind != XE_DM_PERF) return helper_errno_result(L, -14);
      const XeReg R5 = reg_get(L, 5);
      XE_NILCHK(R5);
      int64_t err;
      if (xe_concurrent(P)) {  // appended in packet order after the run (list_push_par)
        if (int e = list_push_par(L, P, m, M, reg_get(L, 4), R5.v, err)) return in_helper(e);
        return helper_errno_result(L, err);
      }
      if (int e = list_push(L, P, m, M, reg_get(L, 4), R5.v, err)) return in_helper(e);
      return helper_errno_result(L, err);
    }
    case 87: {  // MapPushElement :255-281
      uint32_t m;
      if (int e = reg_to_map(L, P, m, cm1)) return in_helper(e);
      if (!m) return 0;
      const XeDevMap M = map_desc(L, m);
      if (M.kind != XE_DM_LIST && M.kind != XE_DM_PERF) return XE_E_MAP_OP | XE_E_IN_HELPER;  // "push not available"
      int64_t err;
      if (xe_concurrent(P)) {
        if (int e = list_push_par(L, P, m, M, reg_get(L, 2), int64_t(M.value_size), err)) return in_helper(e);
        return helper_errno_result(L, err);
      }
      if (int e = list_push(L, P, m, M, reg_get(L, 2), int64_t(M.value_size), err)) return in_helper(e);
      return helper_errno_result(L, err);
    }
    case 88: {  // MapPopElement :284-332
      uint32_t m;
      if (int e = reg_to_map(L, P, m, cm1)) return in_helper(e);
      if (!m) return 0;
      reg_replace(L, 0, XE_KIND_IMM, 0, 0, 0);
      const XeDevMap M = map_desc(L, m);
      if (M.kind != XE_DM_LIST) return XE_E_MAP_OP | XE_E_IN_HELPER;  // "pop not available"
      XeReg val{0, 0, XE_KIND_IMM};
      if (xe_concurrent(P)) {
        // the count pass flags the packet's first pop and stops it; a ranked pass pops the element at
        // the packet's rank among the batch's pops of the list, and counts the pop (the runtime checks
        // the counts against the ones it ranked by, and runs the pass again until they agree)
        if (!list_par(P) || P.pop_mode == 0) return XE_EV_ORD;
        if (P.pop_mode == 1) {
          P.popflag[L.pidx] = 1u + m;
          xe_atomic_or64(&P.list->popmask, 1ull << m);
          return XE_EV_STOP;
        }
        const uint32_t j = P.pop_slot[m];
        if (j >= XE_POP_SLOTS) {  // a list nobody was ranked on: give it a slot and run the pass again
          xe_atomic_or64(&P.list->popmask, 1ull << m);
          xe_atomic_or64(&P.list->newlist, 1ull);
          return XE_EV_STOP;
        }
        if (((L.npops >> (8 * j)) & 0xffu) == 0xffu) return XE_EV_ORD;  // (255 pops of one list in a packet)
        int64_t pos;
        if (list_pos(L, P, m, M, 0, pos)) val = XeReg{0, xe_h_make(XE_H_QVAL, m, list_at(M, uint64_t(pos))), XE_KIND_MEMPTR};
        L.npops += 1u << (8 * j);
      } else if (const uint64_t cnt = *map_hdr(M, 1)) {
        uint32_t id;
        if (*map_hdr(M, 4)) {
          id = list_at(M, cnt - 1);
        } else {
          id = list_at(M, 0);
          *map_hdr(M, 0) = (*map_hdr(M, 0) + 1) % M.list_cap;
        }
        *map_hdr(M, 1) = cnt - 1;
        val = XeReg{0, xe_h_make(XE_H_QVAL, m, id), XE_KIND_MEMPTR};
      }
      const XeReg R2 = reg_get(L, 2);
      if (XE_T_KIND(R2.t) == XE_KIND_MEMPTR || XE_T_KIND(R2.t) == XE_KIND_FRAMEPTR) {
        const int64_t off = XE_T_KIND(R2.t) == XE_KIND_FRAMEPTR ? xe_wadd(XE_FRAME, R2.v) : R2.v;
        if (int e = mem_write(L, P, R2.h, off, 8, XE_T_KIND(val.t), val.h, val.v)) return in_helper(e);  // "write memory"
        return 0;
      }
      return helper_errno_result(L, -14);
    }
    case 89: {  // MapPeekElement :335-374: R2 := Lookup(IMM 0 key) — nil when the lookup failed
      uint32_t m;
      if (int e = reg_to_map(L, P, m, cm1)) return in_helper(e);
      if (!m) return 0;
      XeReg out;
      int64_t err;
      if (int e = map_lookup(L, P, m, XeReg{0, 0, XE_KIND_IMM}, true, out, err)) return in_helper(e);
      reg_replace(L, 0, XE_KIND_IMM, 0, err, 0);
      if (err) reg_replace(L, 2, XE_KIND_NIL, 0, 0, 0);
      else reg_put(L, 2, out);
      return 0;
    }
#else
    case 12: case 25: case 87: case 88: case 89: return XE_EV_UNSUP;
#endif
  }
  return XE_E_NO_HELPER;
}

#if !XE_GEN
// ---- bpf-to-bpf calls inlined into the per-program kernel (fields model; xe_jit.cpp flatten_calls).
// The generator inlines a call only where R6..R9 can hold just scalars or pointers into a packet the
// program never writes, so the Registers.Clone the call preserves (registers.go:233-240,294-303) is the
// value itself with its alias to a stored object dropped; only R6..R9 (and PC) come back at Exit.
XE_DEV XeReg inl_clone(const XeReg& R) { return XeReg{R.v, R.h, XE_T_KIND(R.t)}; }
// CallBPF (inst_call_bpf.go:18-44): preserve R6..R9, R10 := the next frame (index f), wiped
XE_DEV void inl_call(XeLane& L, int f, XeReg& s6, XeReg& s7, XeReg& s8, XeReg& s9) {
  s6 = inl_clone(reg_get(L, 6));
  s7 = inl_clone(reg_get(L, 7));
  s8 = inl_clone(reg_get(L, 8));
  s9 = inl_clone(reg_get(L, 9));
  // frame f's 32 words are bits 32 f .. 32 f + 31 of the mask: half of one mask word
  dirty_clear(L, XE_STACK_WORDS * f, 0xffffffffull << ((XE_STACK_WORDS * f) & 63));
  reg_replace(L, 10, XE_KIND_FRAMEPTR, xe_h_make(XE_H_STACK, uint32_t(f), 0), 0, XE_T_RO);
}
// Exit inside a call (inst_exit.go:22-48): R6..R9 from the preserved clones, R10 := the caller's frame f
XE_DEV void inl_ret(XeLane& L, int f, const XeReg& s6, const XeReg& s7, const XeReg& s8, const XeReg& s9) {
  reg_put(L, 6, s6);
  reg_put(L, 7, s7);
  reg_put(L, 8, s8);
  reg_put(L, 9, s9);
  reg_replace(L, 10, XE_KIND_FRAMEPTR, xe_h_make(XE_H_STACK, uint32_t(f), 0), 0, XE_T_RO);
}
#endif

// ------------------------------------------------------------------ ALU
XE_DEV int shift_check(int64_t s) { return s < 0 ? (XE_EV_PANIC | XE_P_NEG_SHIFT) : 0; }

XE_DEV int alu_compute(uint32_t op, bool wide, int64_t d, int64_t s, int64_t& out) {
  if (!wide) {
    int32_t a = xe_i32(d), b = xe_i32(s);
    switch (op) {
      case 0x00: out = int64_t(int32_t(uint32_t(a) + uint32_t(b))); return 0;
      case 0x10: out = int64_t(int32_t(uint32_t(a) - uint32_t(b))); return 0;
      case 0x20: out = int64_t(int32_t(uint32_t(a) * uint32_t(b))); return 0;
      case 0x50: out = int64_t(a & b); return 0;
      case 0x40: out = int64_t(a | b); return 0;
      case 0xa0: out = int64_t(a ^ b); return 0;
      case 0x30:
        if (b == 0) return XE_EV_PANIC | XE_P_DIV0;
        out = b == -1 ? int64_t(int32_t(0u - uint32_t(a))) : int64_t(a / b);
        return 0;
      case 0x90:
        if (b == 0) return XE_EV_PANIC | XE_P_DIV0;
        out = b == -1 ? 0 : int64_t(a % b);
        return 0;
      case 0x60: if (int e = shift_check(b)) return e; out = b >= 32 ? 0 : int64_t(uint32_t(uint32_t(d) << b)); return 0;
      case 0x70: if (int e = shift_check(b)) return e; out = b >= 32 ? 0 : int64_t(uint32_t(d) >> b); return 0;
      case 0xc0: if (int e = shift_check(b)) return e; out = int64_t(b >= 32 ? (a < 0 ? -1 : 0) : (a >> b)); return 0;
    }
  } else {
    switch (op) {
      case 0x00: out = xe_wadd(d, s); return 0;
      case 0x10: out = int64_t(uint64_t(d) - uint64_t(s)); return 0;
      case 0x20: out = xe_wmul(d, s); return 0;
      case 0x50: out = d & s; return 0;
      case 0x40: out = d | s; return 0;
      case 0xa0: out = d ^ s; return 0;
      case 0x30:
        if (s == 0) return XE_EV_PANIC | XE_P_DIV0;
        out = s == -1 ? int64_t(0ull - uint64_t(d)) : d / s;
        return 0;
      case 0x90:
        if (s == 0) return XE_EV_PANIC | XE_P_DIV0;
        out = s == -1 ? 0 : d % s;
        return 0;
      case 0x60: if (int e = shift_check(s)) return e; out = s >= 64 ? 0 : int64_t(uint64_t(d) << s); return 0;
      case 0x70: if (int e = shift_check(s)) return e; out = s >= 64 ? 0 : int64_t(uint64_t(d) >> s); return 0;
      case 0xc0: if (int e = shift_check(s)) return e; out = s >= 64 ? (d < 0 ? -1 : 0) : (d >> s); return 0;
    }
  }
  out = 0;
  return 0;
}

XE_DEV bool jmp_cond(uint32_t op, bool wide, int64_t d, int64_t s) {
  if (!wide) {
    int32_t a = xe_i32(d), b = xe_i32(s);
    uint32_t ua = uint32_t(a), ub = uint32_t(b);
    switch (op) {
      case 0x10: return a == b;
      case 0x50: return a != b;
      case 0x20: return ua > ub;
      case 0x30: return ua >= ub;
      case 0x60: return a > b;
      case 0x70: return a >= b;
      case 0xc0: return a <= b;  // JSLT as written (inst_jslt.go:24,77)
      case 0xd0: return a <= b;
    }
  } else {
    switch (op) {
      case 0x10: return d == s;
      case 0x50: return d != s;
      case 0x20: return uint64_t(d) > uint64_t(s);
      case 0x30: return uint64_t(d) >= uint64_t(s);
      case 0x60: return d > s;
      case 0x70: return d >= s;
      case 0xc0: return d <= s;  // inst_jslt.go:48,106
      case 0xd0: return d <= s;
    }
  }
  return false;
}

// effective offset of a pointer register + insn offset (inst_load.go:91-101)
XE_DEV int64_t ptr_eff(const XeReg& R, int32_t ioff) {
  return XE_T_KIND(R.t) == XE_KIND_FRAMEPTR ? xe_wadd(xe_wadd(XE_FRAME, R.v), ioff) : xe_wadd(R.v, ioff);
}

// lifted read-modify-writes run as adds only where lanes run concurrently and no register record
// could show the loaded value
XE_DEV bool lift_active(const XeParams& P) { return xe_concurrent(P) && !P.regs; }

// ---- per-class handlers (exec_uop dispatches; the JIT calls them directly with constant uops)
XE_DEV int uop_alu(XeLane& L, const XeParams& P, const XeUop& u, uint32_t cmd = XE_CM_ALL) {
  const int d = u.dst, s = u.src;
  const bool wide = u.fl & UF_WIDE, reg = u.fl & UF_REG;
  const XeReg D = reg_get(L, d);
  XE_NILCHK(D);
  const XeReg S = reg ? reg_get(L, s) : XeReg{int64_t(u.imm), 0, 0};
  if (reg) XE_NILCHK(S);
  if (reg && u.x == 0x00 && XE_T_KIND(S.t) != XE_KIND_IMM) {
    // inst_add.go:82-98,131-147: dst becomes a Copy of the pointer src with the sum as offset
    int64_t v = wide ? xe_wadd(D.v, S.v) : int64_t(int32_t(uint32_t(xe_i32(D.v)) + uint32_t(xe_i32(S.v))));
    reg_replace(L, d, XE_T_KIND(S.t), S.h, v, 0);
    return 0;
  }
  if ((u.x == 0x30 || u.x == 0x90) && S.v == 0) return XE_E_DIV0;
  int64_t v;
  if (int e = alu_compute(u.x, wide, D.v, S.v, v)) return e;
  return reg_inplace(L, d, v, cmd);
}

XE_DEV int uop_movi(XeLane& L, const XeUop& u) {
  reg_replace(L, u.dst, XE_KIND_IMM, 0, int64_t(u.imm), 0);
  return 0;
}

XE_DEV int uop_movr(XeLane& L, const XeUop& u) {
  const XeReg S = reg_get(L, u.src);
  XE_NILCHK(S);
  reg_replace(L, u.dst, XE_T_KIND(S.t), S.h, S.v, 0);
  return 0;
}

XE_DEV int uop_neg(XeLane& L, const XeUop& u, uint32_t cmd = XE_CM_ALL) {
  const XeReg D = reg_get(L, u.dst);
  XE_NILCHK(D);
  int64_t v = (u.fl & UF_WIDE) ? int64_t(0ull - uint64_t(D.v)) : int64_t(int32_t(0u - uint32_t(xe_i32(D.v))));
  return reg_inplace(L, u.dst, v, cmd);
}

XE_DEV int uop_end(XeLane& L, const XeUop& u, uint32_t cmd = XE_CM_ALL) {
  const XeReg D = reg_get(L, u.dst);
  XE_NILCHK(D);
  uint64_t rv = uint64_t(D.v), v;
  if (u.x == 0) {
    v = u.imm == 16 ? uint64_t(__builtin_bswap16(uint16_t(rv)))
      : u.imm == 32 ? uint64_t(__builtin_bswap32(uint32_t(rv))) : __builtin_bswap64(rv);
  } else {
    v = u.imm == 16 ? uint64_t(uint16_t(rv)) : u.imm == 32 ? uint64_t(uint32_t(rv)) : rv;
  }
  return reg_inplace(L, u.dst, int64_t(v), cmd);
}

// returns whether the branch is taken (nil operands are checked by the caller: jmp_nil)
XE_DEV bool uop_jmp(const XeLane& L, const XeUop& u) {
  const bool wide = u.fl & UF_WIDE;
  const XeReg D = reg_get(L, u.dst);
  if (u.fl & UF_REG) {
    const XeReg S = reg_get(L, u.src);
    bool same = XE_T_KIND(D.t) == XE_T_KIND(S.t);
    bool c = jmp_cond(u.x, wide, D.v, S.v);
    return u.x == 0x50 ? (!same || c) : (same && c);
  }
  bool imm = XE_T_KIND(D.t) == XE_KIND_IMM;
  bool c = jmp_cond(u.x, wide, D.v, int64_t(u.imm));
  return u.x == 0x50 ? (!imm || c) : (imm && c);
}
XE_DEV int jmp_nil(const XeLane& L, const XeUop& u) {
  XE_NILCHK(reg_get(L, u.dst));
  if (u.fl & UF_REG) XE_NILCHK(reg_get(L, u.src));
  return 0;
}

XE_DEV int uop_ldimm64(XeLane& L, const XeParams& P, const XeUop& u, uint32_t cmd = XE_CM_ALL) {
  const int d = u.dst, s = u.src;
  if (s == 1) { reg_replace(L, d, XE_KIND_IMM, 0, int64_t(uint32_t(u.imm)), 0); return 0; }
  if (s == 2) {  // BPF_PSEUDO_MAP_FD_VALUE, inst_load.go:36-63
    uint32_t m = uint32_t(u.imm);
    if (uint64_t(m) >= uint64_t(P.nmaps) + 1) return XE_E_NO_MAP;
    if (m == 0) return XE_EV_PANIC | XE_P_NIL_MAP;
    const XeDevMap M = map_desc(L, m);
    if (XE_HAS_ARRAY && M.kind == XE_DM_ARRAY) {
      if (M.vals_bytes == 0) return XE_E_MAP_NOT_PTR;
      reg_replace(L, d, XE_KIND_MEMPTR, xe_h_make(XE_H_ARRAY, m, 0), int64_t(u.x), 0);
      return 0;
    }
    if (XE_HAS_HASH && M.kind == XE_DM_HASH) {
      uint64_t kw[XE_MAX_KEY / 8] = {0, 0, 0, 0, 0, 0, 0, 0};
      bool empty = M.key_size > 4 || M.key_size == 0;  // ReadRange of a 4-byte tmp memory
#if XE_KEYED
      if (int e = key_touch(L, P, kid_hash(m, M, kw, empty), false)) return e;
#endif
      int64_t slot = hash_find(M, kw, empty);
      if (slot < 0) return XE_E_MAP_NOT_PTR;
      reg_replace(L, d, XE_KIND_MEMPTR, hv_make(M, m, uint32_t(slot)), int64_t(u.x), 0);
      return 0;
    }
    return XE_EV_UNSUP;
  }
  return reg_inplace(L, d, int64_t((uint64_t(u.x) << 32) + uint64_t(uint32_t(u.imm))), cmd);
}

XE_DEV int uop_ldx(XeLane& L, const XeParams& P, const XeUop& u, uint32_t cms = XE_CM_ALL) {
  const XeReg S = reg_get(L, u.src);
  XE_NILCHK(S);
  if ((cms & XE_CM_IMM) && XE_T_KIND(S.t) == XE_KIND_IMM) return XE_E_NONPTR_LOAD;
  uint32_t kind, oh, al; int64_t v;
  // a lifted load's value only reaches memory through the paired store's add: no read footprint
  const bool track = !((u.fl & UF_LIFT) && lift_active(P));
  if (int e = mem_read(L, P, S.h, ptr_eff(S, u.tgt), uop_size(u), track, kind, oh, v, al, cms)) return e;
  if (u.fl & UF_BADDST) return XE_E_ASSIGN_REG;
  reg_replace(L, u.dst, kind, oh, v, al);
  return 0;
}

// ST (u.cls == U_ST, value = imm) and STX
XE_DEV int uop_store(XeLane& L, const XeParams& P, const XeUop& u, uint32_t cmd = XE_CM_ALL) {
  const bool st = u.cls == U_ST;
  const XeReg S = st ? XeReg{int64_t(u.imm), 0, uint32_t(XE_KIND_IMM)} : reg_get(L, u.src);
  XE_NILCHK(S);  // STX: src.Copy() before the destination (inst_store.go:64-70)
  const XeReg D = reg_get(L, u.dst);
  XE_NILCHK(D);
  if ((cmd & XE_CM_IMM) && XE_T_KIND(D.t) == XE_KIND_IMM) return XE_E_NONPTR_STORE;
  if (xe_peeking(L) && !is_vm_cls(xe_h_cls(D.h))) return XE_EV_STOP;
  const int64_t off = ptr_eff(D, u.tgt);
  const int size = uop_size(u);
  if ((cmd & XE_CM_MAPS) && (u.fl & UF_LIFT) && lift_active(P)) {
    const uint32_t c = xe_h_cls(D.h);
    if (c == XE_H_ARRAY || c == XE_H_HASH) {
      XeBMem B;
      bmem_resolve(L, P, D.h, B);
      bool own = false;  // a key of this lane's chain (XE_MODE_CHAIN): the plain store below
#if XE_KEYED
      if (B.map && P.mode == XE_MODE_CHAIN) {
        if (int e = bounds(off, size, B.len)) return e;
        if (int e = key_touch_mem(L, P, D.h, B, off, size, false, &own)) return e;
      }
#endif
      if (B.map && !own) {  // the lifted read-modify-write of a map value: add the addend (lift_rmw)
        if (int e = bounds(off, size, B.len)) return e;
#if XE_KEYED
        if (P.mode == XE_MODE_SPEC)
          if (int e = key_touch_mem(L, P, D.h, B, off, size, false)) return e;
#endif
        int64_t k = int64_t(u.imm);
        if (u.x & 0xff) k = reg_get(L, int(u.x & 0xff) - 1).v;
        if (u.x & 0x100) k = int64_t(0ull - uint64_t(k));
        fp_record(L, P, B.map, true, fp_bits(map_desc(L, B.map), B.array, off, size));
        width_record(L, P, B.map, size, uint64_t(uintptr_t(B.base + off)));
        wave_atomic_add_field(L, B.map, P.mode != XE_MODE_CHAIN, B.base + off, size, uint64_t(k));
        return 0;
      }
    }
  }
  return mem_write(L, P, D.h, off, size, XE_T_KIND(S.t), S.h, S.v, cmd);
}

XE_DEV int uop_atomic(XeLane& L, const XeParams& P, const XeUop& u, uint32_t cmd = XE_CM_ALL) {
  const XeReg D = reg_get(L, u.dst);
  XE_NILCHK(D);
  if ((cmd & XE_CM_IMM) && XE_T_KIND(D.t) == XE_KIND_IMM) return XE_E_NONPTR_STORE;
  if (xe_peeking(L) && !is_vm_cls(xe_h_cls(D.h))) return XE_EV_STOP;
  const uint32_t h = D.h;
  const int64_t off = ptr_eff(D, u.tgt);
  const int size = uop_size(u);
  const uint32_t c = xe_h_cls(h);
  if ((cmd & XE_CM_VM) && is_vm_cls(c)) {
    int id = 0;
    if (int e = vmem_read(L, h, off, size, id)) return e;
    if (u.fl & UF_BADSRC) return XE_E_BAD_REG;
    const XeReg S = reg_get(L, u.src);
    XE_NILCHK(S);
    int64_t ov; uint32_t oh, ot;
    obj_get(L, id, ov, oh, ot);
    if (XE_T_KIND(ot) == XE_KIND_FRAMEPTR && (ot & XE_T_RO)) return XE_E_READONLY;
    int64_t nv = xe_wadd(ov, S.v);
    obj_set_val(L, id, nv);
    alias_refresh(L, uint32_t(id), nv);
    return 0;
  }
  if ((cmd & XE_CM_PKT) && c == XE_H_PKT) {
    if (int e = bounds(off, size, L.plen)) return e;
    if (u.fl & UF_BADSRC) return XE_E_BAD_REG;
    const XeReg S = reg_get(L, u.src);
    XE_NILCHK(S);
#if XE_GEN
    if (int e = bm_before_write(L, P, h)) return e;
#endif
    pkt_store(L, off, size, pkt_load(L, off, size) + uint64_t(S.v));
    return 0;
  }
  if (!(cmd & XE_CM_MAPS)) return XE_EV_UNSUP;  // excluded by the class analysis (never reached)
  XeBMem B;
  bmem_resolve(L, P, h, B);
  if (int e = bounds(off, size, B.len)) return e;
  if (u.fl & UF_BADSRC) return XE_E_BAD_REG;
  const XeReg S = reg_get(L, u.src);
  XE_NILCHK(S);
#if XE_GEN
  if (int e = bm_prepare_write(L, P, h)) return e;
  if (!B.map) {  // a lane-private ByteMemory: a plain read, add, write
    bmem_resolve(L, P, h, B);
    store_le(B.base + off, size, load_le(B.base + off, size) + uint64_t(S.v));
    return 0;
  }
#endif
  bool own = false;  // a key of this lane's chain: ordered by the chain, no footprint
#if XE_KEYED
  if (int e = key_touch_mem(L, P, h, B, off, size, false, &own)) return e;
#endif
  if (!own) {
    fp_record(L, P, B.map, true, fp_bits(map_desc(L, B.map), B.array, off, size));
    width_record(L, P, B.map, size, uint64_t(uintptr_t(B.base + off)));
  }
  wave_atomic_add_field(L, B.map, P.mode == XE_MODE_PARALLEL || P.mode == XE_MODE_SPEC, B.base + off, size, uint64_t(S.v));
  return 0;
}

XE_DEV int uop_helper(XeLane& L, const XeParams& P, const XeUop& u, uint32_t cm1 = XE_CM_ALL, uint32_t cm2 = XE_CM_ALL,
                      uint32_t cm3 = XE_CM_ALL) {
  int64_t fn = int64_t(u.imm);
  if (u.cls == U_CALLX) {
    const XeReg F = reg_get(L, u.dst);
    XE_NILCHK(F);
    fn = F.v;
  }
  return call_helper(L, P, fn, cm1, cm2, cm3);
}

// bpf_map_lookup_elem / bpf_map_update_elem of a HASH / LRU_HASH map whose key words the per-program kernel
// built from the registers it stored into the frame (xe_jit.cpp key_shadows proves them equal to the
// ReadRange of R2); everything else about the call is call_helper's (ids 1 and 2 are never replaced
// in a per-program kernel: a VM with a host or nil helper runs on the interpreter).
XE_DEV int uop_helper_key(XeLane& L, const XeParams& P, const XeUop& u, uint32_t cm1, uint32_t cm2, uint32_t cm3,
                          const uint64_t* kp) {
  if (xe_peeking(L) && u.imm != 1) return XE_EV_STOP;
  return u.imm == 1 ? helper_lookup(L, P, cm1, cm2, kp) : helper_update(L, P, cm1, cm2, cm3, kp);
}

#if XE_GEN
// ---- bpf-to-bpf calls (general model)
// RegisterValue.Clone of a pointer's memory (registers.go:233-240,294-303): a ValueMemory is copied
// slot by slot (the objects stay shared, memory.go:109-116); a ByteMemory becomes a lane-private
// ByteMemory that reads through to its source until either is written (memory.go:212-219).
XE_COLD int clone_mem(XeLane& L, const XeParams& P, uint32_t h, uint32_t& out) {
  const uint32_t c = xe_h_cls(h);
  if (is_vm_cls(c)) {
    const XeVR R = vmem_region(L, h);
    const int k = vc_alloc(L);
    if (k < 0) return XE_EV_CAP;
#pragma unroll 1
    for (int64_t s = 0; s < R.len; s++)
      *gat<uint16_t>(L, L.G->o_vc, uint64_t(k) * XE_FRAME + uint64_t(s)) = uint16_t(vmem_id(L, R, s));
    const uint32_t src = c == XE_H_VCLONE ? vc_src(L, xe_h_slot(h)) : c;
    *gat<uint32_t>(L, L.G->o_vcinfo, uint32_t(k)) = uint32_t(R.len) | (src << 16);
    out = xe_h_make(XE_H_VCLONE, 0, uint32_t(k));
    return 0;
  }
  const int k = bm_alloc(L);
  if (k < 0) return XE_EV_CAP;
  XeBMem B;
  bmem_resolve(L, P, h, B);
  uint32_t info;
  if (c == XE_H_BMEM) info = *bm_field(L, xe_h_slot(h), XE_BM_INFO);
  else if (c == XE_H_PKT) info = XE_REGION_PACKET;
  else if (c == XE_H_ARRAY) info = XE_REGION_ARRAY | (xe_h_map(h) << 8);
  else if (c == XE_H_HASH) info = XE_REGION_HASHVAL | (hv_map(P, h) << 8);
  else info = (map_desc(L, xe_h_map(h)).kind == XE_DM_PERF ? XE_REGION_PERF : XE_REGION_QUEUEVAL) | (xe_h_map(h) << 8);
  *bm_field(L, uint32_t(k), XE_BM_SRC) = bm_ident(h);
  *bm_field(L, uint32_t(k), XE_BM_MAT) = XE_NONE;
  *bm_field(L, uint32_t(k), XE_BM_LEN) = uint32_t(B.len);
  *bm_field(L, uint32_t(k), XE_BM_INFO) = info;
  L.npristine++;
  out = xe_h_make(XE_H_BMEM, 0, uint32_t(k));
  return 0;
}

// CallBPF, emulator/inst_call_bpf.go:18-44: push Registers.Clone() (only its PC and R6..R9 are ever
// restored), move R10 to the next, wiped, stack frame, jump. The clone happens first, so a nil register
// panics even when the frame index then overflows.
XE_COLD int uop_callbpf(XeLane& L, const XeParams& P, const XeUop& u, int32_t pc, int32_t& tgt) {
#pragma unroll 1
  for (int r = 0; r < 10; r++) XE_NILCHK(reg_get(L, r));
  if (L.npres + 1 >= XE_MAX_FRAMES || L.npres + 1 >= L.G->nframes) return XE_EV_PANIC | XE_P_INDEX;  // &StackFrames[Index+1]
  const uint32_t e = L.npres;
#pragma unroll 1
  for (int r = 6; r < 10; r++) {
    const XeReg R = reg_get(L, r);
    XeReg C{R.v, 0, XE_T_KIND(R.t) | (XE_T_KIND(R.t) == XE_KIND_FRAMEPTR ? (R.t & XE_T_RO) : 0u)};
    if (XE_ISPTR(R.t))
      if (int err = clone_mem(L, P, R.h, C.h)) return err;
    pres_put(L, e, r - 6, C);
  }
  *pres_word(L, e, 0) = uint32_t(pc);
  L.npres = e + 1;
  const int bit = int(L.npres) * 16;  // wipe frame npres: all its groups read as nil again
  L.fdirty[bit >> 6] &= ~(0xffffull << (bit & 63));
  reg_replace(L, 10, XE_KIND_FRAMEPTR, xe_h_make(XE_H_STACK, L.npres, 0), 0, XE_T_RO);
  tgt = pc + u.imm;
  return 0;
}

// Exit, emulator/inst_exit.go:22-48: inside a call, restore PC, R6..R9 (the clones) and R10.
XE_DEV int uop_exit(XeLane& L, int32_t& tgt) {
  if (L.npres == 0) return XE_EV_EXIT;
  const uint32_t e = --L.npres;
#pragma unroll 1
  for (int r = 6; r < 10; r++) reg_put(L, r, pres_get(L, e, r - 6));
  reg_replace(L, 10, XE_KIND_FRAMEPTR, xe_h_make(XE_H_STACK, L.npres, 0), 0, XE_T_RO);
  tgt = int32_t(*pres_word(L, e, 0));
  return 0;
}
#endif

// ------------------------------------------------------------------ one instruction
// Executes uop u (at pc) on this lane. Returns 0 (continue; `tgt` = PC after the instruction,
// before Step's increment), XE_EV_EXIT, or an error code.
XE_DEV int exec_uop(XeLane& L, const XeParams& P, const XeUop& u, int32_t pc, int32_t& tgt) {
  tgt = pc;
  switch (u.cls) {
    case U_FAIL: return u.imm;
    case U_NOP: return 0;
#if XE_GEN
    case U_EXIT: return uop_exit(L, tgt);
#else
    case U_EXIT: return XE_EV_EXIT;
#endif
    case U_JA: tgt = u.tgt; return 0;
    case U_ALU: return uop_alu(L, P, u);
    case U_MOVI: return uop_movi(L, u);
    case U_MOVR: return uop_movr(L, u);
    case U_NEG: return uop_neg(L, u);
    case U_END: return uop_end(L, u);
    case U_JMP:
      if (int e = jmp_nil(L, u)) return e;
      if (uop_jmp(L, u)) tgt = u.tgt;
      return 0;
    case U_LDIMM64: return uop_ldimm64(L, P, u);
    case U_LDX: return uop_ldx(L, P, u);
    case U_ST:
    case U_STX: return uop_store(L, P, u);
    case U_ATOMIC: return uop_atomic(L, P, u);
    case U_HELPER:
    case U_CALLX: {
      int e = uop_helper(L, P, u);
#if XE_HAS_ORDERED
      if (e == XE_EV_JUMP) { tgt = -1; return 0; }  // tail call: PC := -1 in the new program
#endif
      return e;
    }
#if XE_GEN
    case U_CALLBPF: return uop_callbpf(L, P, u, pc, tgt);
#else
    case U_CALLBPF: return XE_EV_UNSUP;
#endif
  }
  return XE_EV_UNSUP;
}

// ------------------------------------------------------------------ wave driver
// minimum of v over the wave (all lanes active)
XE_DEV int wave_min(int v) {
  int cur = xe_readfirst(v);
  unsigned long long lt = xe_ballot(v < cur);
  while (lt) {
    int l = __builtin_ctzll(lt);
    cur = xe_readlane(v, l);
    lt = xe_ballot(v < cur);
  }
  return cur;
}

// Descriptor of packet i (xsk.go:695-701 layout) as two raw words {addr}, {len | options << 32}
// (no use of the loaded values here, so the load stays in flight until desc_fix).
XE_DEV void desc_load(const XeParams& P, uint32_t i, bool valid, uint64_t& lo, uint64_t& hi) {
  lo = 0;
  hi = 0;
  if (valid) {
    XE_GP(const uint64_t) d = (XE_GP(const uint64_t))(P.desc + i);
    lo = d[0];
    hi = d[1];
  }
}
// A frame outside the UMEM gets length 0, so every access to it fails the ByteMemory bounds check.
XE_DEV void desc_fix(const XeParams& P, uint64_t lo, uint64_t hi, uint64_t& a, uint32_t& l) {
  a = lo;
  l = uint32_t(hi);
  if (a > P.umem_len || uint64_t(l) > P.umem_len - a) l = 0;
}
XE_DEV void desc_fetch(const XeParams& P, uint32_t i, bool valid, uint64_t& a, uint32_t& l) {
  uint64_t lo, hi;
  desc_load(P, i, valid, lo, hi);
  desc_fix(P, lo, hi, a, l);
}

#if defined(__HIPCC__)
// One LDS-DMA row: 16 bytes per lane from src into LDS at d + lane * 16 (d wave-uniform). Inline asm
// on purpose: the compiler would otherwise make every later LDS read of the kernel wait for the DMA
// (vmcnt(0)), which serialises the prefetch with the work it is meant to overlap. The matching wait
// is explicit (hdr_wait).
XE_DEV void glds16(XE_GP(const uint8_t) src, uint32_t d) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(d) : "memory");
}
#endif

// Rows of a packet's header window: those holding bytes of [XE_HDR_LO, min(len, XE_HDR_HI)) counted
// from the 16-byte aligned address at or below byte XE_HDR_LO (0 when the packet ends before it).
XE_DEV int hdr_rows(uint64_t a, uint32_t l) {
#if XE_HDR_ROWS == 0
  (void)a; (void)l;
  return 0;
#else
  const int end = l < uint32_t(XE_HDR_HI) ? int(l) : XE_HDR_HI;
  if (end <= XE_HDR_LO) return 0;
  const int r = (end - XE_HDR_LO + int((a + XE_HDR_LO) & 15) + 15) >> 4;
  return r < XE_HDR_ROWS ? r : XE_HDR_ROWS;
#endif
}

// Issue the LDS-DMA of a packet's header window into buffer `buf` (wave-uniform): row k on the lanes
// whose window has more than k rows. Returns false (nothing issued for this lane) when the rows would
// run past the UMEM; lane_stage then copies the bytes one by one.
XE_DEV bool hdr_issue(const XeParams& P, XE_LP(uint8_t) buf, uint64_t a, uint32_t l, bool valid) {
#if XE_HDR_ROWS == 0
  (void)P; (void)buf; (void)a; (void)l; (void)valid;
  return false;
#else
  const uint64_t al = (a + XE_HDR_LO) & ~uint64_t(15);
  const int nr = valid ? hdr_rows(a, l) : 0;
  const bool fast = valid && al + 16 * uint64_t(nr) <= P.umem_len;
  if (fast) {
#if defined(__HIPCC__)
    XE_GP(const uint8_t) src = (XE_GP(const uint8_t))(P.umem + al);
    const uint32_t d = uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(uintptr_t(buf)))));
#pragma unroll
    for (int k = 0; k < XE_HDR_ROWS; k++)
      if (k < nr) glds16(src + 16 * k, d + k * XE_HDR_ROW);
#else
    for (int k = 0; k < nr; k++)
      for (int b = 0; b < 16; b++) buf[k * XE_HDR_ROW + b] = P.umem[al + 16 * k + b];
#endif
  }
  return fast;
#endif
}

// the LDS-DMA writes of this wave have landed (the compiler does not track them for LDS reads)
XE_DEV void hdr_wait() {
#if defined(__HIPCC__)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
}

// Reset (emulator/vm.go:211-246) + the per-packet harness ctx for the packet
// whose descriptor (a, l) was fetched by desc_fetch and whose window was issued into buffer `buf`
// (hdr_issue returned `fast`; hdr_wait done).
XE_DEV void lane_stage(XeLane& L, const XeParams& P, bool valid, uint64_t a, uint32_t l, bool fast,
                       XE_LP(uint8_t) buf, int col = -1) {
#pragma unroll
  for (int r = 0; r < 10; r++) reg_replace(L, r, XE_KIND_IMM, 0, 0, 0);
  reg_replace(L, 10, XE_KIND_FRAMEPTR, xe_h_make(XE_H_STACK, 0, 0), 0, XE_T_RO);
  reg_replace(L, 1, XE_KIND_MEMPTR, xe_h_make(XE_H_CTX, 0, 0), 0, 0);
#if !XE_GEN
  L.dirty0 = L.dirty1 = L.dirty2 = L.dirty3 = 0;
  L.oused = 0x7full | (XE_OBJ_LIMIT >= 64 ? 0ull : (~0ull << (XE_OBJ_LIMIT & 63)));
#else
  L.onext = 7;  // ids 1..6: the xdp_md objects
  L.ofree = L.vnext = L.vfree = L.bnext = L.bfree = 0;
  L.bused = 0;
  L.fdirty[0] = L.fdirty[1] = 0;
  L.ctxdirty = 0;
  L.npres = 0;  // the harness sets PreservedRegisters = nil
  L.pi = P.entry;
  L.npops = 0;
  L.npristine = 0;
#endif
#if !XE_GEN && XE_HAS_ORDERED
  L.npops = 0;
#endif
  L.odef = 0x7eull;
  L.pkt = P.umem;
  L.plen = 0;
  L.hdr_len = 0;
  L.hdr = buf + (col < 0 ? xe_lane() : col) * 16;  // col: the staged packet's column (sequential mode)
  const int sh = fast ? int((a + XE_HDR_LO) & 15) : 0;
  L.hsh = sh - XE_HDR_LO;
  if (valid) {
    L.pkt = P.umem + a;
    L.plen = int64_t(l);
    const int nr = hdr_rows(a, l);
    const int win = XE_HDR_LO + 16 * nr - sh;  // end of the window's logical bytes
    const int hl = nr == 0 ? 0 : l < uint32_t(win) ? int(l) : win;
    L.hdr_len = hl;
    if (!fast) {
#pragma unroll 1
      for (int b = XE_HDR_LO; b < hl; b++) *hdr_at(L, b + L.hsh) = ((XE_GP(const uint8_t))L.pkt)[b];
    }
  }
  L.ingress = P.ingress;
  L.rxq = P.rxq;
}

// synchronous form (ordered mode): descriptor, window, wait, stage into buffer 0
XE_DEV void lane_reset(XeLane& L, const XeParams& P, uint32_t i, bool valid) {
  uint64_t a;
  uint32_t l;
  desc_fetch(P, i, valid, a, l);
  const bool fast = hdr_issue(P, L.hdrbuf, a, l, valid);
  hdr_wait();
  lane_stage(L, P, valid, a, l, fast, L.hdrbuf);
}

XE_DEV void lane_commit(XeLane& L, const XeParams& P);

// Sequential-mode driver (the exact in-order replay): lane 0 runs the packets one after another.
// With P.seq_prefetch the whole wave first stages the next XE_WAVE packets (lane k: descriptor and
// header window of packet c0 + k, the window in lane k's column), so the replay lane's per-packet
// chain is the program's own work instead of descriptor -> window -> program round trips; without it
// (a program may write packet bytes a later packet reads) each packet is fetched just before it runs.
// body(i, valid) runs the staged packet on the lanes where valid and calls lane_finish (all lanes).
//
// Runahead (P.seq_prefetch & 2, per-program kernels with XE_SEQ_PEEK): before the replay lane runs the
// 64 staged packets, every lane runs its own one with all shared writes stopped (xe_peeking: a store or
// atomic outside the lane's stack, any helper but bpf_map_lookup_elem, an LRU lookup's promotion), and
// its results dropped. What it leaves behind is the map lines its lookups read — hash probes, values —
// in this CU's caches, so the replay lane's dependent loads hit there instead of going to HBM one at a time.
template <class Body, class Peek>
XE_DEV void seq_packets(XeLane& L, const XeParams& P, Body body, Peek peek) {
  const uint32_t lane = uint32_t(xe_lane());
  for (uint32_t c0 = 0; c0 < P.n; c0 += XE_WAVE) {
    const uint32_t m = P.n - c0 < XE_WAVE ? P.n - c0 : XE_WAVE;
    uint64_t a = 0;
    uint32_t l = 0;
    bool f = false;
    if (P.seq_prefetch) {
      const bool v = lane < m;
      desc_fetch(P, c0 + lane, v, a, l);
      f = hdr_issue(P, L.hdrbuf, a, l, v);
      hdr_wait();
#if XE_SEQ_PEEK && !XE_UNIFORM
      if (P.seq_prefetch & 2u) {
        lane_stage(L, P, v, a, l, f, L.hdrbuf, int(lane));
        L.peek = 1;
        peek(v);
        L.peek = 0;
      }
#endif
    }
#pragma unroll 1
    for (uint32_t k = 0; k < m; k++) {
      // XE_UNIFORM: every lane runs packet k (the same state everywhere: the scalar replay)
      const bool valid = XE_UNIFORM || lane == 0;
      // every lane stages packet k (only lane 0 runs it): the lane state is then wave-uniform, which
      // lets the compiler keep much of the replay's arithmetic on the scalar unit
      if (P.seq_prefetch)
        lane_stage(L, P, true, xe_readlane64(a, int(k)), uint32_t(xe_readlane(int(l), int(k))),
                   xe_readlane(int(f), int(k)) != 0, L.hdrbuf, int(k));
      else
        lane_reset(L, P, c0 + k, valid);
#if XE_HAS_ORDERED
      L.pidx = c0 + k;  // order keys of the packet's LRU stamps (lru_stamp)
      L.oseq = 0;
#endif
      body(c0 + k, valid);
    }
  }
}

// Parallel-mode driver: wave `wave` of `nwaves` walks chunks wave, wave + nwaves, ... of XE_WAVE
// packets (one per lane). Software-pipelined: while chunk c executes, the header window of the next
// chunk and the descriptor of the one after are already in flight, so HBM latency overlaps the
// interpretation instead of stalling every chunk twice (descriptor -> header). The abort flag (an
// ordered write somewhere in the batch) is polled the same way, one chunk behind.
// body(i, valid) runs the staged packet and calls lane_finish; all lanes call it together.
// packet i runs in this parallel pass (the keyed path's pass leaves out the packets on chains)
XE_DEV bool pkt_in_pass(const XeParams& P, uint32_t i) {
#if XE_SKIP_MASK
  if (P.K.skip && i < P.n && ((XE_GP(const uint8_t))P.K.skip)[i]) return false;
#endif
  return i < P.n;
}
// the key log of the lane's next packet starts empty
XE_DEV void key_begin(XeLane& L, uint32_t i) {
#if XE_KEYED
  L.kn = 0;
  L.kpkt = i;
  L.kins = 0;
  L.kwr = false;
  L.kh = XE_NONE;
#else
  (void)L;
  (void)i;
#endif
}

// first packet of the c-th chunk of the walk (P.sched: a permuted chunk order, for determinism tests)
XE_DEV uint32_t chunk_base(const XeParams& P, uint32_t c, uint32_t nchunks) {
  if (P.sched && c < nchunks) c = uint32_t((uint64_t(nchunks) - 1 - c + P.sched) % nchunks);
  return c * XE_WAVE;
}

template <class Body>
XE_DEV void parallel_packets(XeLane& L, const XeParams& P, uint32_t wave, uint32_t nwaves, Body body) {
  const uint32_t lane = uint32_t(xe_lane());
  const uint32_t nchunks = (P.n + (XE_WAVE - 1)) / XE_WAVE;
  uint32_t c = wave;
  if (c >= nchunks) return;
  // an earlier pipelined batch is being replayed in order: this one re-runs afterwards
  if (P.poison && xe_readfirst(int(xe_load_relaxed32(const_cast<unsigned int*>(P.poison))))) return;
  uint32_t i0 = chunk_base(P, c, nchunks) + lane;
  bool v0 = pkt_in_pass(P, i0);
  uint64_t a0;
  uint32_t l0;
  desc_fetch(P, i0, v0, a0, l0);
  uint32_t c1 = c + nwaves;
  uint32_t i1 = chunk_base(P, c1, nchunks) + lane;
  bool v1 = c1 < nchunks && pkt_in_pass(P, i1);
  uint64_t r1lo, r1hi;  // raw descriptor of chunk c1, in flight
  desc_load(P, i1, v1, r1lo, r1hi);
  uint32_t cur = 0;  // buffer of chunk c (wave-uniform)
  bool f0 = hdr_issue(P, L.hdrbuf, a0, l0, v0);
  L.defer = XE_DEFER_COMMIT != 0;
  L.dv_i = -1;
  for (;;) {
    hdr_wait();  // window of chunk c and descriptor of chunk c1 (issued a whole chunk ago)
    lane_stage(L, P, v0, a0, l0, f0, L.hdrbuf + cur * XE_HDR_BUF);
    // in flight during body(c): the window of chunk c1, the descriptor of chunk c2, the abort flag
    uint64_t a1;
    uint32_t l1;
    desc_fix(P, r1lo, r1hi, a1, l1);
    const bool f1 = hdr_issue(P, L.hdrbuf + (cur ^ 1u) * XE_HDR_BUF, a1, l1, v1);
    const uint32_t c2 = c1 + nwaves;
    const uint32_t i2 = chunk_base(P, c2, nchunks) + lane;
    const bool v2 = c2 < nchunks && pkt_in_pass(P, i2);
    desc_load(P, i2, v2, r1lo, r1hi);
    const uint32_t abort_flags = xe_load_relaxed32(P.flags);
    lane_commit(L, P);  // the previous chunk's verdicts and adds, behind this chunk's prefetch
    key_begin(L, i0);
#if XE_HAS_ORDERED
    L.pidx = i0;
    L.oseq = 0;
#endif
    body(i0, v0);
    if (c1 >= nchunks) break;
    // a lane elsewhere needed an ordered write: this run will be discarded, stop early
    if (xe_readfirst(int(abort_flags)) & XE_FLAG_ORDERED) break;
    i0 = i1; v0 = v1; a0 = a1; l0 = l1; f0 = f1;
    c1 = c2; i1 = i2; v1 = v2;
    cur ^= 1u;
  }
  lane_commit(L, P);
  L.defer = false;
  hdr_wait();  // no LDS-DMA may be outstanding when the wave retires
}

#if XE_KEYED
// ---- keyed build steps, one call per item (xe_kernel.hip runs them as grids, the host simulation as
// loops). After XE_MODE_SPEC: the D table of written keys, union-find over the D keys each packet
// touches (rounds until nothing changes), the roots, each packet's chain (dcap: none), the chain
// starts in the sorted order, and one slot reservation per new HASH key.
// put key id `kid` into D; true when this call added it
// put key id `kid` into D; returns its slot when this call added it, else -1
XE_DEV int64_t keyed_dset_insert(const XeKeyed& K, uint64_t kid) {
  const uint32_t mask = K.dcap - 1;
  uint32_t idx = uint32_t(kid >> 4) & mask;
  int64_t added = -1;
  bool done = false;
#pragma unroll 1
  for (uint32_t probe = 0; probe < K.dcap && !done; probe++) {
    const unsigned long long cur = xe_load_relaxed64(reinterpret_cast<unsigned long long*>(K.dkid + idx));
    if (cur == kid) { done = true; break; }
    if (cur == 0) {
      const unsigned long long old = xe_atomic_cas64(reinterpret_cast<unsigned long long*>(K.dkid + idx), 0ull, kid);
      if (old == 0) {
        K.dcomp[idx] = idx;
        K.dkey[uint64_t(idx) * K.kw] = 0;  // no key words (yet): not an insert
        added = int64_t(idx);
        done = true;
        break;
      }
      if (old == kid) { done = true; break; }
    }
    idx = (idx + 1) & mask;
  }
  if (!done) xe_atomic_or32(K.err, 8u);  // D is full
  return added;
}
XE_DEV void keyed_dset_item(const XeKeyed& K, uint32_t i) {
  const uint32_t n = K.kcnt[i];
  if (n > XE_KLOG) { xe_atomic_or32(K.err, 1u); return; }
#pragma unroll 1
  for (uint32_t j = 0; j < n; j++) {
    const uint64_t e = K.klog[uint64_t(i) * XE_KLOG + j];
    if (!(e & XE_KLOG_W)) continue;
    const int64_t d = keyed_dset_insert(K, e & ~XE_KLOG_FLAGS);
    if (d >= 0 && (e & XE_KLOG_INS)) {  // the key's first writer: an insert, its words go with the D slot
      const uint64_t* src = K.ikey + (uint64_t(i) * XE_KINS + ((e >> 3) & 1ull)) * K.kw;
      uint64_t* dst = K.dkey + uint64_t(d) * K.kw;
      for (uint32_t w = 0; w < K.kw; w++) dst[w] = src[w];
    }
  }
}
XE_DEV uint32_t keyed_root(const XeKeyed& K, uint32_t x) {
  // parents only decrease (keyed_union_item hooks under the smaller root), so the walk ends within dcap
  // hops at a node that is its own parent. A parent outside D or a walk that does not end means the D
  // table is not what the build wrote: the batch goes to the in-order replay (err bit 16, any err bit
  // rolls the keyed path back) instead of forming chains from a partial root.
#pragma unroll 1
  for (uint32_t hop = 0; hop < K.dcap; hop++) {
    const uint32_t p = xe_load_relaxed32(K.dcomp + x);
    if (p == x) return x;
    if (p >= K.dcap) break;
    x = p;
  }
  xe_atomic_or32(K.err, 16u);
  return x;
}
// hook every root of packet i's D keys under the smallest (parents only decrease: rounds converge)
XE_DEV void keyed_union_item(const XeKeyed& K, uint32_t i) {
  // an overflowed log (kcnt > XE_KLOG: the batch takes the replay) may hold entries never written
  const uint32_t n = K.kcnt[i];
  if (n < 2 || n > XE_KLOG) return;
  uint32_t r = XE_NONE;
#pragma unroll 1
  for (uint32_t j = 0; j < n; j++) {
    const int64_t d = dset_find(K, K.klog[uint64_t(i) * XE_KLOG + j] & ~XE_KLOG_FLAGS);
    if (d >= 0) { const uint32_t q = keyed_root(K, uint32_t(d)); r = q < r ? q : r; }
  }
  if (r == XE_NONE) return;
#pragma unroll 1
  for (uint32_t j = 0; j < n; j++) {
    const int64_t d = dset_find(K, K.klog[uint64_t(i) * XE_KLOG + j] & ~XE_KLOG_FLAGS);
    if (d < 0) continue;
    const uint32_t q = keyed_root(K, uint32_t(d));
    if (q != r && xe_atomic_min32(K.dcomp + q, r) > r) xe_atomic_or32(K.changed, 1u);
  }
}
XE_DEV void keyed_compress_item(const XeKeyed& K, uint32_t x) {
  if (((XE_GP(const unsigned long long))K.dkid)[x]) K.dcomp[x] = keyed_root(K, x);
}
XE_DEV void keyed_assign_item(const XeKeyed& K, uint32_t i, uint8_t* skip) {
  const uint32_t n = K.kcnt[i] <= XE_KLOG ? K.kcnt[i] : 0u;  // (overflow: see keyed_union_item)
  uint32_t c = K.dcap;
  int64_t d[XE_KLOG];
#pragma unroll
  for (uint32_t j = 0; j < XE_KLOG; j++) d[j] = j < n ? dset_find(K, K.klog[uint64_t(i) * XE_KLOG + j] & ~XE_KLOG_FLAGS) : -1;
#pragma unroll
  for (uint32_t j = 0; j < XE_KLOG; j++)
    if (c == K.dcap && d[j] >= 0) c = K.dcomp[d[j]];
  K.ckey[i] = c;
  skip[i] = c != K.dcap ? 1 : 0;
}
// after the sort: nO = the number of packets on chains (sorted keys before the first "none")
XE_DEV void keyed_nchain_item(const XeKeyed& K, uint32_t p) {
  const bool on = K.okey[p] != K.dcap;
  const bool next = p + 1 < K.n && K.okey[p + 1] != K.dcap;
  if (on && !next) K.counts[0] = p + 1;
}
// D slot x: a new HASH key held back by SPEC gets its slot record reserved
XE_DEV void keyed_reserve_item(const XeKeyed& K, const XeDevMap* maps, uint32_t x) {
  if (!((XE_GP(const unsigned long long))K.dkid)[x]) return;
  const uint64_t* en = K.dkey + uint64_t(x) * K.kw;
  if (!(en[0] & XE_KEY_VALID) || (en[0] & 0x100ull)) return;  // not an insert / the nil key's own slot
  const uint32_t m = uint32_t(en[0] & 0xffu);
  uint64_t kw[XE_MAX_KEY / 8];
#pragma unroll
  for (uint32_t w = 0; w < XE_MAX_KEY / 8; w++) kw[w] = w + 1 < K.kw ? en[1 + w] : 0;
  // an LRU key's record carries the value id XE_KS_LRUID gave it
  const uint64_t hi = maps[m].kind == XE_DM_LRU ? (en[0] & ~0xffffffffull) : 0ull;
  if (!hash_reserve(maps[m], kw, hi)) xe_atomic_or32(K.err, 2u);
}
// D slot x: a new LRU key gets a value id from its map's pool (next id, hdr[3]); lanes taking ids from
// the same map share one atomic per wave. Every lane of the launch calls this (no early exit).
// An insert that evicts (keyed_evict_item) takes over its victim's value id instead: no packet of the
// batch holds a pointer to the victim's value (none touches it), so the pool does not grow by evictions.
XE_DEV void keyed_lruid_item(const XeKeyed& K, const XeDevMap* maps, uint32_t x) {
  bool want = false;
  uint32_t m = 0, victim = XE_NONE;
  XE_GP(uint64_t) en = (XE_GP(uint64_t))K.dkey + uint64_t(x) * K.kw;
  if (((XE_GP(const unsigned long long))K.dkid)[x] && (en[0] & XE_KEY_VALID) && !(en[0] & 0x100ull)) {
    m = uint32_t(en[0] & 0xffu);
    want = maps[m].kind == XE_DM_LRU;
    victim = want ? K.dvict[x] : XE_NONE;
  }
  const bool alloc = want && victim == XE_NONE;
  unsigned int* next = alloc ? (unsigned int*)maps[m].hdr + 6 : (unsigned int*)K.err;  // hdr[3], low word
  const uint32_t id = xe_wave_alloc_at(next, alloc);
  if (want) en[0] = (en[0] & 0xffffffffull) | (uint64_t(alloc ? id : victim) << 32);
}
// ---- LRU evictions in a keyed batch (maps_hash_lru.go:114-119: an insert into a full map first deletes
// UsageList[len-1]). In packet order the UsageList's tail is the least recently used value that no packet
// of the batch has touched yet, because every touch and insert moves a key to the head. When none of the
// E oldest values of the batch's start is touched by any packet, the j-th evicting insert in packet order
// (an insert of a new key is evicting once the live count has reached MaxEntries) deletes exactly the
// j-th oldest of them: the build ranks the inserts of new keys by the packet that first inserts them,
// the chains delete the victims at those inserts, and any packet that would see a victim — in SPEC
// (its stamp moved, or its key is written) or in the chains (its key is now a D entry of no chain) —
// sends the batch to the in-order replay.
//   XE_KS_FIRST (packets): the first inserting packet of every D key
XE_DEV void keyed_first_item(const XeKeyed& K, uint32_t i) {
  const uint32_t n = K.kcnt[i];
  if (n > XE_KLOG) return;
#pragma unroll 1
  for (uint32_t j = 0; j < n; j++) {
    const uint64_t e = K.klog[uint64_t(i) * XE_KLOG + j];
    if (!(e & XE_KLOG_INS)) continue;
    const int64_t d = dset_find(K, e & ~XE_KLOG_FLAGS);
    if (d >= 0) xe_atomic_min32(K.dfirst + d, i);
  }
}
//   XE_KS_EKEY (D slots): sort keys map << 32 | first insert of the LRU inserts (everything else last)
XE_DEV void keyed_ekey_item(const XeKeyed& K, const XeDevMap* maps, uint32_t x) {
  uint64_t key = ~0ull;
  if (((XE_GP(const unsigned long long))K.dkid)[x]) {
    const uint64_t en = K.dkey[uint64_t(x) * K.kw];
    const uint32_t m = uint32_t(en & 0xffu);
    if ((en & XE_KEY_VALID) && maps[m].kind == XE_DM_LRU) key = (uint64_t(m) << 32) | K.dfirst[x];
  }
  K.ekey[x] = key;
  K.eval[x] = x;
  K.dvict[x] = XE_NONE;
}
//   XE_KS_EVICT (the inserts of map em, i-th in packet order): the victim of the i-th insert
XE_DEV void keyed_evict_item(const XeKeyed& K, const XeDevMap* maps, uint32_t i) {
  const uint32_t d = K.eval2[K.eoff + i];
  if (i < K.efree) return;  // the map still had room: no eviction
  const uint32_t q = i - K.efree;
  if (q >= K.ecnt0) { xe_atomic_or32(K.err, 32u); return; }  // it would evict a key this batch inserted
  const uint32_t v = K.vorder[K.ecnt0 - 1 - q];
  const XeDevMap& M = maps[K.em];
  // touched by some packet: a SPEC lookup moved its stamp, or some packet writes its key
  const bool moved = ((XE_GP(const uint64_t))M.tag)[v] != K.etsnap[v];
  const uint32_t slot = ((XE_GP(const uint32_t))M.link)[4 * uint64_t(v) + 2];
  if (moved || dset_find(K, kid_slot(K.em, M, slot)) >= 0) { xe_atomic_or32(K.err, 32u); return; }
  K.dvict[d] = v;
}
//   XE_KS_EMARK (the same items): each victim's key becomes a D entry of no chain, so a chain packet that
//   would still look it up leaves its chain (key_touch) instead of seeing it present or deleted
XE_DEV void keyed_emark_item(const XeKeyed& K, const XeDevMap* maps, uint32_t i) {
  const uint32_t d = K.eval2[K.eoff + i];
  const uint32_t v = K.dvict[d];
  if (v == XE_NONE) return;
  const XeDevMap& M = maps[K.em];
  const uint32_t slot = ((XE_GP(const uint32_t))M.link)[4 * uint64_t(v) + 2];
  keyed_dset_insert(K, kid_slot(K.em, M, slot));
}

// D slot x, after the chains: the reservation of a new HASH key loses its "claimed in this launch" mark
// (a chain's insert already turned it FULL; an unused one stays a plain tombstone holding its key), so a
// later keyed batch's hash_reserve finds it by its key words instead of reserving another record
XE_DEV void keyed_unnew_item(const XeKeyed& K, const XeDevMap* maps, uint32_t x) {
  if (!((XE_GP(const unsigned long long))K.dkid)[x]) return;
  const uint64_t* en = K.dkey + uint64_t(x) * K.kw;
  if (!(en[0] & XE_KEY_VALID) || (en[0] & 0x100ull)) return;
  const XeDevMap& M = maps[uint32_t(en[0] & 0xffu)];
  uint64_t kw[XE_MAX_KEY / 8];
#pragma unroll
  for (uint32_t w = 0; w < XE_MAX_KEY / 8; w++) kw[w] = w + 1 < K.kw ? en[1 + w] : 0;
  const uint32_t mask = M.cap - 1;
  uint32_t idx = uint32_t(xe_hash_words(kw, M.kwords, M.key_size)) & mask;
#pragma unroll 1
  for (uint32_t probe = 0; probe < M.cap; probe++) {
    uint64_t* r = M.keys + uint64_t(idx) * M.rwords;
    const uint32_t st = uint32_t(r[0]);
    if (!(st & (XE_SLOT_FULL | XE_SLOT_TOMB))) return;  // the chain ends: nothing reserved for it
    bool eq = true;
    for (uint32_t k = 0; k < M.kwords; k++) eq = eq && r[1 + k] == kw[k];
    if (eq) {
      if (st & XE_SLOT_NEW) r[0] = (r[0] & ~uint64_t(XE_SLOT_NEW));
      return;
    }
    idx = (idx + 1) & mask;
  }
}
// chain lengths: a chain holding more than half the batch runs faster as the staged one-lane replay
XE_DEV void keyed_cstart_item(const XeKeyed& K, uint32_t p) {
  if (p == 0 || K.okey[p] != K.okey[p - 1]) K.cstart[K.okey[p]] = p;
}
XE_DEV void keyed_clong_item(const XeKeyed& K, uint32_t p) {
  if (p + 1 < K.nO && K.okey[p + 1] == K.okey[p]) return;  // not a chain's last packet
  if (uint64_t(p + 1 - K.cstart[K.okey[p]]) * 2 > K.n) K.counts[1] = 1;
}
// the compacted chain list: iota[p] = 1 where a chain starts, an exclusive scan of it into ckey, then
// cstart[ckey[p]] = p (cstart is free again once the long-chain check has run) and the chain count
XE_DEV void keyed_cflag_item(const XeKeyed& K, uint32_t p) {
  K.iota[p] = (p == 0 || K.okey[p] != K.okey[p - 1]) ? 1u : 0u;
}
XE_DEV void keyed_clist_item(const XeKeyed& K, uint32_t p) {
  if (K.iota[p]) K.cstart[K.ckey[p]] = p;
  if (p + 1 == K.nO) K.counts[2] = K.ckey[p] + K.iota[p];
}
XE_DEV void keyed_step(const XeKeyed& K, const XeDevMap* maps, uint8_t* skip, uint32_t step, uint32_t i) {
  switch (step) {
    case XE_KS_DSET: keyed_dset_item(K, i); break;
    case XE_KS_UNION: keyed_union_item(K, i); break;
    case XE_KS_COMPRESS: keyed_compress_item(K, i); break;
    case XE_KS_ASSIGN: keyed_assign_item(K, i, skip); break;
    case XE_KS_IOTA: K.iota[i] = i; break;
    case XE_KS_NCHAIN: keyed_nchain_item(K, i); break;
    case XE_KS_RESERVE: keyed_reserve_item(K, maps, i); break;
    case XE_KS_CSTART: keyed_cstart_item(K, i); break;
    case XE_KS_CLONG: keyed_clong_item(K, i); break;
    case XE_KS_UNNEW: keyed_unnew_item(K, maps, i); break;
    case XE_KS_CFLAG: keyed_cflag_item(K, i); break;
    case XE_KS_CLIST: keyed_clist_item(K, i); break;
    case XE_KS_LRUID: keyed_lruid_item(K, maps, i); break;
    case XE_KS_FIRST: keyed_first_item(K, i); break;
    case XE_KS_EKEY: keyed_ekey_item(K, maps, i); break;
    case XE_KS_EVICT: keyed_evict_item(K, maps, i); break;
    case XE_KS_EMARK: keyed_emark_item(K, maps, i); break;
    default: break;
  }
}

// Chain-mode driver (XE_MODE_CHAIN, keyed ordered execution): the chains (cstart[0..nch): first
// positions in the sorted order; a chain's packets are order[p..] while the sorted key stays the same)
// are a work queue. A wave claims XE_WAVE chain indices at a time (one atomic on counts[3]); every lane
// that has finished its chain takes the next unassigned index of the wave's claim, so a lane with a
// short chain goes on to another instead of idling until the wave's longest chain ends. All lanes of a
// wave call body together until the queue is empty and every lane is done.
template <class Body>
XE_DEV void chain_packets(XeLane& L, const XeParams& P, uint32_t g, uint32_t nthreads, Body body) {
  (void)g;
  (void)nthreads;
  const uint32_t nch = xe_load_relaxed32(P.K.counts + 2);
  uint32_t qn = 0, qe = 0;  // wave-uniform: the wave's claimed chain indices not yet handed out
  bool drained = false;     // wave-uniform: the queue has no chains left
  uint32_t p = 0, pend = 0, key = 0;
  bool have = false;
#pragma unroll 1
  for (;;) {
    const uint64_t idle = xe_ballot(!have);
    if (idle && qn >= qe && !drained) {
      uint32_t base = 0;
      if (xe_lane() == __builtin_ctzll(idle)) base = xe_atomic_add32(P.K.counts + 3, uint32_t(XE_WAVE));
      base = uint32_t(xe_readlane(int(base), int(__builtin_ctzll(idle))));
      if (base >= nch) drained = true;
      else { qn = base; qe = base + XE_WAVE < nch ? base + XE_WAVE : nch; }
    }
    if (idle && qn < qe) {
      const uint32_t rank = uint32_t(__builtin_popcountll(idle & xe_lanemask_lt()));
      if (!have && qn + rank < qe) {
        const uint32_t c = qn + rank;
        p = P.K.cstart[c];
        pend = c + 1 < nch ? P.K.cstart[c + 1] : P.K.nO;
        key = P.K.okey[p];
        have = true;
      }
      const uint32_t given = uint32_t(__builtin_popcountll(idle));
      qn = qn + given < qe ? qn + given : qe;
    }
    if (!xe_ballot(have)) {
      if (drained) break;
      continue;
    }
    const uint32_t i = have ? P.K.order[p] : 0u;
    L.kchain = key;
    lane_reset(L, P, i, have);
    key_begin(L, i);
#if XE_HAS_ORDERED
    L.pidx = i;  // order keys of the packet's appends and LRU touches
    L.oseq = 0;
#endif
    body(i, have);
    if (have && ++p >= pend) have = false;
  }
}
#endif

// map an exec_uop error to the lane's final status/code
XE_DEV void status_from_error(int e, int& status, int& code) {
  if (e == XE_EV_EXIT) { status = XE_ST_OK; }
  else if (XE_EV_CLASS(e) == XE_EV_ORD) { status = XE_ST_INTERNAL_ORDERED; }
  else if (e == XE_EV_STOP) { status = XE_ST_OK; }  // (the count pass's records are discarded)
  else if (XE_EV_CLASS(e) == XE_EV_CAP) { status = XE_ST_INTERNAL_CAPACITY; }
  else if (XE_EV_CLASS(e) == XE_EV_UNSUP) { status = XE_ST_UNSUPPORTED; }
  else if (XE_IS_PANIC(e)) { status = XE_ST_PANIC; code = e & 0xff; }
  else { status = XE_ST_VMERR; code = e & 0xffff; }
}

// results, parity record, flags and batch statistics for the lane's packet (all lanes call this)
XE_DEV void lane_finish(XeLane& L, const XeParams& P, uint32_t i, bool valid, int status, int code,
                        int32_t res_pc, uint64_t steps) {
#if XE_PAIR_ADDS
  if (!L.defer) pend_flush(L);
#endif
  if (status == XE_ST_INTERNAL_ORDERED) xe_atomic_or32(P.flags, XE_FLAG_ORDERED);
  if (status == XE_ST_INTERNAL_CAPACITY) xe_atomic_or32(P.flags, XE_FLAG_CAPACITY);
#if XE_HAS_ORDERED
  if (P.pop_mode == 2 && valid) P.popflag[i] = L.npops;  // the pops the packet made, for the runtime's check
#endif
#if XE_KEYED
  if (P.mode == XE_MODE_SPEC) {  // the packet's key log
    if (valid) {
      P.K.kcnt[i] = L.kn;
#pragma unroll
      for (uint32_t j = 0; j < XE_KLOG; j++)
        if (j < L.kn) P.K.klog[uint64_t(i) * XE_KLOG + j] = L.klog[j];
    }
    L.kany = L.kany || xe_ballot(valid && L.kwr) != 0;  // flagged once per wave (flush_wave_state)
  }
#endif
  if (valid) {
    const XeReg R0 = reg_get(L, 0);
    if (XE_RECORDS && P.results) {
      xe_result r;
      r.status = uint8_t(status);
      r.r0_kind = uint8_t(XE_T_KIND(R0.t));
      r.code = uint16_t(code);
      r.pc = uint32_t(res_pc);
      r.r0 = R0.v;
      P.results[i] = r;
    }
    if (P.verdicts) {
      if (L.defer) { L.dv_i = int32_t(i); L.dv = uint32_t(uint64_t(R0.v)); }
      else P.verdicts[i] = uint32_t(uint64_t(R0.v));
    }
    if (XE_RECORDS && P.regs) {
      xe_regs g;
#pragma unroll
      for (int r = 0; r < 10; r++) {
        const XeReg R = reg_get(L, r);
        g.val[r] = R.v;
        uint32_t k = XE_T_KIND(R.t);
        g.kind[r] = uint8_t(k);
        if (k == XE_KIND_IMM || k == XE_KIND_NIL) { g.region[r] = 0xff; g.map[r] = 0; }
        else {
          uint32_t c = xe_h_cls(R.h), rg = c, mp = c == XE_H_ARRAY ? xe_h_map(R.h) : c == XE_H_HASH ? hv_map(P, R.h) : 0;
#if XE_GEN
          // clones report the region of the memory they copied (Clone keeps it, memory.go:109-116,212-219)
          if (c == XE_H_VCLONE) { rg = vc_src(L, xe_h_slot(R.h)); mp = 0; }
          else if (c == XE_H_BMEM) { const uint32_t inf = *bm_field(L, xe_h_slot(R.h), XE_BM_INFO); rg = inf & 0xff; mp = inf >> 8; }
          else if (c == XE_H_QVAL) { rg = map_desc(L, xe_h_map(R.h)).kind == XE_DM_PERF ? XE_REGION_PERF : XE_REGION_QUEUEVAL; mp = xe_h_map(R.h); }
#endif
          g.region[r] = uint8_t(rg);
          g.map[r] = uint8_t(mp);
        }
      }
      g.pad[0] = g.pad[1] = 0;
      g.steps = uint32_t(steps);
      P.regs[i] = g;
    }
  }
  // batch statistics: per-lane step sums and wave-uniform status counts, flushed once per wave (the
  // scalar replay counts its packet once, on lane 0)
  if (XE_UNIFORM) valid = valid && xe_lane() == 0;
  L.acc_steps += valid ? steps : 0;
#if XE_HIST_FAST
  // status histogram: one ballot when every packet of the chunk ended OK (the common case)
  const unsigned long long vb = xe_ballot(valid), bad = xe_ballot(valid && status != XE_ST_OK);
  L.acc_status[0] += uint32_t(__builtin_popcountll(vb & ~bad));
  if (bad) {
#pragma unroll
    for (int st = 1; st < 8; st++) L.acc_status[st] += uint32_t(__builtin_popcountll(xe_ballot(valid && status == st)));
  }
#else
#pragma unroll
  for (int st = 0; st < 8; st++) L.acc_status[st] += uint32_t(__builtin_popcountll(xe_ballot(valid && status == st)));
#endif
}

// the stores lane_finish deferred (all lanes of the wave together)
XE_DEV void lane_commit(XeLane& L, const XeParams& P) {
#if XE_COMMITTER
  if (L.ring) ring_put(L, L.ring);
  else pend_flush(L);
#elif XE_PAIR_ADDS
  pend_flush(L);
#endif
  if (L.dv_i >= 0) P.verdicts[L.dv_i] = L.dv;
  L.dv_i = -1;
}

// Copy the map descriptor table into LDS (all threads of the block; barrier inside): helpers read
// map fields with LDS loads (lgkmcnt only) instead of vector global loads whose vmcnt wait would
// also drain the header prefetch.
XE_DEV void stage_maps(XeLane& L, const XeParams& P, XE_LP(XeDevMap) lds) {
#if defined(__HIPCC__)
  const uint32_t words = (P.nmaps + 1) * uint32_t(sizeof(XeDevMap) / 4);
  for (uint32_t t = threadIdx.x; t < words; t += blockDim.x)
    ((XE_LP(uint32_t))lds)[t] = ((XE_GP(const uint32_t))P.maps)[t];
  __syncthreads();
  L.maps = lds;
#else
  (void)lds;
  L.maps = P.maps;
#endif
}

XE_DEV void wave_state_init(XeLane& L, const XeParams& P, uint32_t wave, XePend* pend) {
#if XE_SEQ_PEEK
  L.peek = 0;
#endif
#if XE_GEN
  L.G = &P.gen;
  L.gl = P.mode == XE_MODE_SEQUENTIAL ? 0u : wave * XE_WAVE + uint32_t(xe_lane());
#endif
  L.rep = P.rep + uint64_t(wave % P.nrep) * P.rep_words;
  L.wave = wave;
  L.awidth = 0;
  L.pend = pend;
#if XE_COMMITTER
  L.ring = nullptr;
#endif
  L.defer = false;
  L.dv_i = -1;
  L.dv = 0;
#if XE_PAIR_ADDS
  L.pb_tag = L.pb_s0 = L.pb_s1 = 0;
#endif
#pragma unroll 1
  for (uint32_t k = uint32_t(xe_lane()); k < XE_ACC; k += XE_WAVE) { pend->tag[k] = 0; pend->sum[k] = 0; pend->score[k] = 0; }
#pragma unroll
  for (int k = 0; k < XE_FP_MAPS; k++) { L.fpr[k] = 0; L.fpa[k] = 0; }
  L.acc_steps = 0;
#pragma unroll
  for (int st = 0; st < 8; st++) L.acc_status[st] = 0;
#if XE_KEYED
  L.kany = false;
#endif
}

#if XE_GEN
#define XE_LANE_PI(L) ((L).pi)
#else
#define XE_LANE_PI(L) (P.entry)
#endif
// Interpreter engine (general model): runs the harness for the staged packet `i` on this lane
// (valid=false: the lane idles). All lanes of the wave must call this together. A lane's position is
// (program index, PC): the wave runs the lanes at the smallest index into the concatenated program
// table, so lanes that tail-called into another program keep their own stream.
#if XE_TRACE
// the slot of packet i among the traced packets (sorted), -1 if it is not traced
XE_DEV int32_t trace_slot(const XeParams& P, uint32_t i) {
  uint32_t lo = 0, hi = P.trace_npk;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (P.trace_pk[mid] < i) lo = mid + 1;
    else hi = mid;
  }
  return lo < P.trace_npk && P.trace_pk[lo] == i ? int32_t(lo) : -1;
}
// one Step's record: what VM.String prints after it (emulator/vm.go:248-270)
XE_COLD void trace_put(XeLane& L, const XeParams& P, int32_t slot, uint32_t i, uint64_t step, int32_t pc) {
  xe_trace_rec r;
  r.packet = i;
  r.step = uint32_t(step);
  r.pc = pc;
  r.pi = L.pi;
  r.sf = L.npres;
  r.pad = 0;
#pragma unroll 1
  for (int k = 0; k <= 10; k++) {
    const XeReg R = reg_get(L, k);
    r.val[k] = R.v;
    r.kind[k] = uint8_t(XE_T_KIND(R.t));
  }
  P.trace[uint64_t(slot) * P.trace_max + step] = r;
}
#endif

// finish = false: the runahead of the one-lane replay (seq_packets), no records, no trace
XE_DEV void run_staged(XeLane& L, const XeParams& P, uint32_t i, bool valid, bool finish = true) {
  int status = valid ? -1 : XE_ST_OK;  // -1 = running
  int code = 0;
  int32_t pc = 0, res_pc = 0;
  uint64_t steps = 0;
#if XE_GEN
  L.pidx = i;
  L.oseq = 0;
#endif
#if XE_TRACE
  const int32_t tslot = finish && valid && P.trace ? trace_slot(P, i) : -1;
  uint64_t tdone = 0;  // steps that completed
#endif

  for (;;) {
    int key = 0x7fffffff;
    if (status == -1) {
      if (steps >= P.max_steps) {
        status = XE_ST_BUDGET; res_pc = pc;  // the Go VM has no budget: it would run on
      } else if (XE_LANE_PI(L) < 1 || XE_LANE_PI(L) > int32_t(P.nprogs)) {
        status = XE_ST_VMERR; code = XE_E_NO_PROGRAM; res_pc = pc;  // vm.go:138-140
      } else if (pc < 0 || pc >= P.prog_lens[XE_LANE_PI(L)]) {
        status = XE_ST_PANIC; code = XE_P_INDEX; res_pc = pc;  // program[PC] (vm.go:143)
      } else {
        key = P.prog_off[XE_LANE_PI(L)] + pc;
      }
    }
    const int sel = wave_min(key);
    if (sel == 0x7fffffff) break;
    if (key == sel) {
      const XeUop u = P.progs[sel];  // wave-uniform: scalar load
      const int32_t plen = P.prog_lens[XE_LANE_PI(L)];  // Step's `program` (vm.go:141)
      steps++;
      int32_t tgt;
      int e = exec_uop(L, P, u, pc, tgt);
      res_pc = pc;
#if XE_TRACE
      if (tslot >= 0 && (e == 0 || e == XE_EV_EXIT)) {  // Step returned without an error
        if (tdone < P.trace_max) trace_put(L, P, tslot, i, tdone, pc);
        tdone++;
      }
#endif
      if (e == 0) {
        if (int64_t(plen) <= int64_t(tgt) + 1) {  // vm.go:162-167
          status = XE_ST_VMERR; code = XE_E_BAD_PC;
        } else {
          pc = tgt + 1;
        }
      } else {
        status_from_error(e, status, code);
      }
    }
  }
#if XE_TRACE
  if (tslot >= 0) P.trace_cnt[tslot] = uint32_t(tdone < P.trace_max ? tdone : P.trace_max);
#endif
  if (finish) lane_finish(L, P, i, valid, status, code, res_pc, steps);
}

XE_DEV void run_packet(XeLane& L, const XeParams& P, uint32_t i, bool valid) {
  lane_reset(L, P, i, valid);
  run_staged(L, P, i, valid);
}

// flush per-lane footprints of maps 1..4 (wave OR-reduction) and the batch statistics: one atomic
// per word per wave
XE_DEV void flush_wave_state(XeLane& L, const XeParams& P) {
  acc_flush(L);
  unsigned long long steps = L.acc_steps;
  unsigned int aw = L.awidth;
#if defined(__HIPCC__)
  for (int o = 32; o > 0; o >>= 1) aw |= __shfl_xor(aw, o);
#endif
  if (xe_lane() == 0 && aw) xe_atomic_or64(&L.rep[XE_REC_WIDTH0], aw);
#if XE_KEYED
  if (xe_lane() == 0 && L.kany) xe_atomic_or32(P.flags, XE_FLAG_KEYED);
#endif
#if defined(__HIPCC__)
  for (int o = 32; o > 0; o >>= 1) steps += __shfl_xor(steps, o);
#endif
  if (xe_lane() == 0) {
    if (steps) xe_atomic_add64(&L.rep[0], steps);
#pragma unroll
    for (int st = 0; st < 8; st++)
      if (L.acc_status[st]) xe_atomic_add64(&L.rep[1 + st], L.acc_status[st]);
  }
#pragma unroll
  for (int k = 0; k < XE_FP_MAPS; k++) {
    unsigned long long r = L.fpr[k], a = L.fpa[k];
#if defined(__HIPCC__)
    for (int o = 32; o > 0; o >>= 1) { r |= __shfl_xor(r, o); a |= __shfl_xor(a, o); }
#endif
    if (xe_lane() == 0) {
      if (r) xe_atomic_or64(&L.rep[16 + (k + 1) * 2], r);
      if (a) xe_atomic_or64(&L.rep[16 + (k + 1) * 2 + 1], a);
    }
  }
}

