// xe_internal.h — shared host/device definitions of the batched eBPF/XDP emulator.
//
// Micro-op table (host translator -> device interpreter), per-lane memory handles, the device
// map descriptors and the hash-table layout. Portable between hipcc (device + host) and g++ (the
// test-only host simulation build, XE_HOSTSIM).
#pragma once
#if !defined(__HIPCC_RTC__)
#include <stdint.h>
#endif
#include "../../include/xdpemu.h"

#if defined(__HIPCC_RTC__)
#define XE_HD __host__ __device__ __forceinline__
#elif defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define XE_HD __host__ __device__ __forceinline__
#else
#define XE_HD static inline
#endif

// Tuning knobs (A/B experiments through the environment) exist only in the debug build
// (-DXE_TUNING: gobpfld_amd/libxdpemu_tuning.so, gobpfld_amd/build.py build_tuning); the product library
// never reads the environment.
#if !defined(__HIPCC_RTC__)
#if defined(XE_TUNING)
#include <stdlib.h>
static inline const char* xe_tuning_env(const char* name) { return getenv(name); }
#else
static inline const char* xe_tuning_env(const char*) { return nullptr; }
#endif
#endif

// ---------------------------------------------------------------- micro-ops
// One 16-byte record per eBPF instruction slot (the LD_IMM64 filler keeps its own slot, exactly
// as ebpf.Decode emits a Nop, ebpf/decode.go:34), so PCs stay identical to the reference's.
enum XeUopClass : uint8_t {
  U_FAIL = 0,   // statically determined error: imm = (status << 16) | code
  U_NOP,        // emulator/inst_nop.go
  U_EXIT,       // emulator/inst_exit.go
  U_JA,         // emulator/inst_ja.go
  U_ALU,        // x = BPF op nibble; fl: WIDE, REG
  U_MOVI,       // emulator/inst_mov.go:20-46
  U_MOVR,       // emulator/inst_mov.go:60-99
  U_NEG,        // emulator/inst_neg.go
  U_END,        // emulator/inst_end.go; x = 0 (to_le) / 8 (to_be); imm = 16/32/64
  U_JMP,        // x = BPF jmp op nibble; fl: WIDE (64-bit compare), REG
  U_LDIMM64,    // emulator/inst_load.go:21-71; src = pseudo src; imm = Val1; x = Val2
  U_LDX,        // emulator/inst_load.go:84-118
  U_ST,         // emulator/inst_store.go:20-51
  U_STX,        // emulator/inst_store.go:64-99
  U_ATOMIC,     // emulator/inst_atomic.go:20-65
  U_HELPER,     // CallHelper with a known helper id (imm)
  U_CALLX,      // CallHelperIndirect; dst = register holding the helper id
  U_CALLBPF,    // bpf-to-bpf call, emulator/inst_call_bpf.go (general lane model)
  U_CALLI,      // per-program kernels only: a bpf-to-bpf call inlined (xe_jit.cpp flatten_calls)
  U_RETI,       // per-program kernels only: the Exit that returns from an inlined call
  U_NCLASSES
};

enum : uint8_t {
  UF_WIDE = 1,       // 64-bit ALU / JMP
  UF_REG = 2,        // BPF_X form
  UF_BADDST = 4,     // LDX: Assign(dst) will fail after the read (dst > 9)
  UF_BADSRC = 8,     // ATOMIC: Get(src) will fail after the read (src > 9)
  UF_LIFT = 0x40,    // LDX / STX of a lifted read-modify-write (lift_rmw, xe_runtime.cpp)
};

struct XeUop {
  uint8_t cls;
  uint8_t dst;
  uint8_t src;
  uint8_t fl;    // UF_* | (size_log2 << 4) for memory ops
  int32_t imm;
  int32_t tgt;   // jumps: PC after the jump is taken (pc + off), i.e. before the +1 of Step
  uint32_t x;
};
static_assert(sizeof(XeUop) == 16, "uop must be 16 bytes (one s_load_dwordx4)");

XE_HD int uop_size(const XeUop& u) { return 1 << ((u.fl >> 4) & 3); }

// ---------------------------------------------------------------- memory handles
// A pointer register's Memory is encoded in 32 bits: class (3) | map index (6) | slot (23).
#define XE_H_CLS_SHIFT 29
#define XE_H_PKT 0u     // the packet ByteMemory
#define XE_H_CTX 1u     // the xdp_md ctx ValueMemory
#define XE_H_STACK 2u   // stack frame ValueMemory; map field = frame index (StackFrames[i])
#define XE_H_ARRAY 3u   // ArrayMap memory of map m
#define XE_H_HASH 4u    // HASH value (slot) / LRU_HASH value (value id) of map m
#define XE_H_VCLONE 5u  // general model: a lane-private ValueMemory clone (Registers.Clone at a call)
#define XE_H_BMEM 6u    // general model: a lane-private ByteMemory (a clone, or a popped element copy)
#define XE_H_QVAL 7u    // QUEUE / STACK element (slot = element id) or PERF event (slot = event index)
#define XE_H_MAX_MAPS 63
#define XE_H_SLOT_BITS 23
// A HASH / LRU_HASH map whose slots (value ids) do not fit 23 bits is a "big map" (and then the VM holds
// at most 31 maps): the 32 map-field values XE_H_BIG..63 are shared out among the big maps, each taking
// a run of fields [base, base + f) with f * 2^23 >= its slots (its value-id pool for an LRU map), and a
// value handle of slot s carries map field XE_H_BIG + base + (s >> 23), so up to 2^28 slots over all big
// maps stay one 32-bit handle — one map of up to 2^27 slots (MaxEntries up to 2^27) and others beside it
// (xe_interp.h hv_make / hv_map / hv_slot; xe_runtime.cpp xe_add_map hands the fields out)
#define XE_H_BIG 32u
#define XE_H_BIG_FIELDS 32u
XE_HD uint32_t xe_h_make(uint32_t cls, uint32_t map, uint32_t slot) {
  return (cls << XE_H_CLS_SHIFT) | (map << XE_H_SLOT_BITS) | slot;
}
XE_HD uint32_t xe_h_cls(uint32_t h) { return h >> XE_H_CLS_SHIFT; }
XE_HD uint32_t xe_h_map(uint32_t h) { return (h >> XE_H_SLOT_BITS) & 63u; }
XE_HD uint32_t xe_h_slot(uint32_t h) { return h & ((1u << XE_H_SLOT_BITS) - 1u); }

// ---------------------------------------------------------------- device maps
enum : uint32_t { XE_DM_NONE = 0, XE_DM_ARRAY = 1, XE_DM_HASH = 2, XE_DM_LRU = 3, XE_DM_LIST = 4, XE_DM_PERF = 5 };
#define XE_SLOT_FULL 1u
#define XE_SLOT_VLEN0 2u   // HashMap value whose backing became nil (maps_hash.go:108-115)
#define XE_SLOT_TOMB 4u    // LRU_HASH: evicted / deleted slot (probe chains run through it)
#define XE_NONE 0xffffffffu
#define XE_MAX_KEY 64      // device hash keys up to 64 bytes (8 words)

struct XeDevMap {
  uint32_t kind;        // XE_DM_*
  uint32_t btype;       // bpftypes.BPFMapType (XE_MAP_*): TailCall wants a PROG_ARRAY
  uint32_t key_size;
  uint32_t value_size;
  uint32_t max_entries;
  uint32_t big;         // HASH / LRU_HASH with slots past the handle's 23-bit slot field: 1 + the first of
                        // its big-map fields (value handles, xe_interp.h hv_make), 0 otherwise
  uint64_t vals_bytes;  // ARRAY: value_size*max_entries; HASH: (cap+1)*value_size
  uint8_t* vals;        // ARRAY memory / HASH slot values (slot cap = the nil-key slot)
  uint64_t* keys;       // HASH: (cap+1) slot records of rwords u64 words: [0] = slot state, then the
                        // zero-padded key words (one probe touches one record, one cache line)
  uint32_t* state;      // LRU: list_cap replicas of the stamps (pool_cap u64 words each) for the
                        // touches of a parallel / SPEC pass (xe_interp.h lru_touch); otherwise unused
  uint32_t* count;      // HASH: number of entries (device word)
  uint32_t cap;         // HASH: power-of-two slot count
  uint32_t kwords;      // HASH: (key_size+7)/8
  // replicas of the value region for deferred 8-byte adds in parallel mode (wave w adds into replica
  // w % nrep; the runtime folds them into vals after the launch and leaves them zeroed)
  uint8_t* rep;
  uint64_t rep_stride;  // bytes between replicas
  uint32_t nrep;        // 1 = adds go to vals directly
  uint32_t rwords;      // HASH: u64 words per slot record (power of two >= 1 + kwords)
  // LRU_HASH / QUEUE / STACK / PERF_EVENT_ARRAY (ordered maps; the general lane model only)
  //   LRU:  keys = slot records ([0] = state | value id << 32), vals = value pool (pool_cap values),
  //         link = prev/next value ids (UsageList as a linked list), elen = value length (0: nil backing),
  //         hdr = {head (MRU), tail (LRU), count, next value id, any nil-backed value, stamp base, touch counter}, tag = stamps; the one-lane replay's
  //         order log in rec, data_cap entries (xe_interp.h lru_log_push)
  //   LIST: vals = element pool, elen = element length, link = the list (ring of list_cap ids for a
  //         queue), hdr = {head, count, next element id, 0, is_stack}
  //   PERF: vals = event bytes (data_cap), rec = {offset, length} per event, hdr = {count, data used}
  uint64_t* hdr;
  uint32_t* link;
  uint32_t* elen;
  uint64_t* rec;
  uint32_t pool_cap;
  uint32_t list_cap;
  uint64_t data_cap;
  // parallel appends (QUEUE / STACK push, PERF output in parallel mode): per pool element / event, the
  // order key (packet index << 16 | the packet's append number) of the element appended in this run
  uint64_t* tag;
};

// One ordered map's appends of a parallel run put in packet order (xe_append_kernel): the new
// elements / events [base, base + k) sorted by their tags; QUEUE / STACK get the sorted ids in their
// list positions cnt0 .. cnt0 + k - 1, PERF gets its event records permuted.
struct XeAppendArgs {
  uint64_t* tag;             // XeDevMap::tag
  uint64_t* keys_in;         // [k] scratch
  uint64_t* keys_out;
  uint32_t* ids_in;
  uint32_t* ids_out;
  uint64_t* rec;             // PERF: XeDevMap::rec
  uint64_t* rec_tmp;         // PERF: [2k] scratch
  uint32_t* link;            // LIST: XeDevMap::link
  uint64_t base;             // first new element id / event index
  uint64_t head, cnt0, list_cap;
  uint32_t k;
  uint32_t perf;
  uint32_t stack;
};

XE_HD uint32_t xe_hash_rwords(uint32_t kwords) {
  uint32_t r = 1;
  while (r < 1 + kwords) r <<= 1;
  return r;
}

// Word-wise multiplicative hash over the zero-padded key words. The reference hashes with sha256
// (maps_hash.go:55); the function is unobservable (only key equality matters), so a cheap one is
// used. Host and device compute the identical slot layout.
XE_HD uint64_t xe_hash_words(const uint64_t* w, uint32_t nwords, uint32_t key_size) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t(key_size) * 0xC2B2AE3D27D4EB4Full);
  for (uint32_t i = 0; i < nwords; i++) {
    h ^= w[i];
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 32;
  }
  h ^= h >> 29;
  h *= 0xc4ceb9fe1a85ec53ull;
  h ^= h >> 32;
  return h;
}

// kernel-side status of a lane beyond the public XE_ST_*
#define XE_ST_INTERNAL_ORDERED 6
#define XE_ST_INTERNAL_CAPACITY 7  // general model: the lane's arena ran out (the host replays with more)

// replica record words: [0] steps, [1..8] status histogram, [9..12] atomic width classes (4 bits per
// map: 1, 2, 4, 8 bytes), [16 + 2m] read mask and [17 + 2m] atomic mask of map m
#define XE_REC_WIDTH0 9

// flags word bits (device -> host)
#define XE_FLAG_ORDERED 1u   // a lane needed a non-commutative map write in parallel mode
#define XE_FLAG_CAPACITY 2u   // a lane ran out of its arena (general model): the host replays with more
#define XE_FLAG_UNALIGNED 4u  // a map add not aligned to its own width (cross-shard delta lanes inexact)
#define XE_FLAG_KEYED 8u      // XE_MODE_SPEC: a packet's ARRAY / HASH write was held back (its key logged)

// ---------------------------------------------------------------- keyed ordered execution
// Kernel-internal modes of the keyed path (xe_runtime.cpp keyed_run, xe_interp.h key_touch). A batch
// whose packets write map entries runs, instead of on one lane in packet order:
//   XE_MODE_SPEC   every packet in parallel against the batch's start state, its ARRAY / HASH writes
//                  held back; each packet logs the map keys it touches (read / add / write);
//   (build)        the keys some packet writes form the set D; packets touching a D key are joined
//                  into chains (connected components over their D keys), each chain sorted in packet
//                  order; absent HASH keys of D get a reserved slot record (tombstone + key words);
//   XE_MODE_PARALLEL + skip: the packets on no chain, in parallel (they only read / add keys nobody
//                  writes: commutative, checked by the usual footprints);
//   XE_MODE_CHAIN  one lane per chain, in packet order, writes applied. Every key a chain packet
//                  touches must be a key of its own chain, and every key it writes must be in D;
//                  anything else aborts (XE_FLAG_ORDERED) and the batch is replayed on one lane.
// Keys of different chains never meet, so the result is the reference's packet order.
#define XE_MODE_SPEC 16u
#define XE_MODE_CHAIN 17u
#define XE_KLOG 4u            // keys a packet may touch (more: the batch takes the one-lane replay)
#define XE_SLOT_BUSY 8u       // a slot record being reserved (key words not yet written)
#define XE_SLOT_NEW 16u       // a tombstone reserved by the current reservation launch

// key id of map m's key: 6 bits of map index, 54 bits of a mixed key hash, low nibble 0b0010 (never 0;
// the key log uses bit 0 as the "written" mark, bit 2 "an insert whose key words are in ikey slot
// bit 3")
XE_HD uint64_t xe_kid_mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}
XE_HD uint64_t xe_kid(uint32_t m, uint64_t h) {
  return (uint64_t(m & 63u) << 58) | (xe_kid_mix(h) & ((1ull << 58) - 16ull)) | 2ull;
}
#define XE_KLOG_W 1ull        // key log entry: the key is written
#define XE_KLOG_INS 4ull      // ... by an insert whose key words are in the packet's ikey slot (bit 3)
#define XE_KLOG_FLAGS 0xDull
#define XE_KINS 2u            // ikey slots per packet (more held-back inserts: the one-lane replay)
// build steps (xe_interp.h keyed_step; items: packets, D slots, or insert-log entries)
enum : uint32_t { XE_KS_DSET = 0, XE_KS_UNION, XE_KS_COMPRESS, XE_KS_ASSIGN, XE_KS_IOTA, XE_KS_NCHAIN, XE_KS_RESERVE,
                  XE_KS_COUNT, XE_KS_CSTART, XE_KS_CLONG, XE_KS_UNNEW, XE_KS_CFLAG, XE_KS_CLIST,
                  XE_KS_LRUID, XE_KS_FIRST, XE_KS_EKEY, XE_KS_EVICT, XE_KS_EMARK };
// Same-address atomics serialise at the memory side, so nothing that many lanes do bumps one counter:
// a new HASH key's words go to its D slot (whose CAS winner is unique), D keys per map are counted by
// a per-block histogram over the D table, and the chains' inserts go to striped counters (by wave).
// Small-buffer layout (u32 words):
#define XE_KSTRIPES 32
#define XE_KS_DCOUNT 0                      // [64 maps] D keys per map
#define XE_KS_ERR 64                        // build errors
#define XE_KS_CHANGED 65                    // union-find round changed something
#define XE_KS_NO 66                         // packets on chains
#define XE_KS_LONG 67                       // some chain holds more than half the batch
#define XE_KS_NCH 68                        // chains (the compacted chain list's length)
#define XE_KS_CNEXT 69                      // the chain pass's work queue: next unclaimed chain
#define XE_KS_DINS 128                      // [64 maps] D keys some packet inserts (absent at the start)
#define XE_KS_CINS 192                      // [64 maps][XE_KSTRIPES] inserts the chains made
#define XE_KS_WORDS (192 + 64 * XE_KSTRIPES)
#define XE_KEY_VALID 0x200ull               // dkey entry word 0: map index | nil-key 0x100 | valid | LRU value id << 32
#define XE_KID_ARRAY_TAG 0xA7A7A7A700000000ull
#define XE_KID_NIL_KEY 0x6e696c6b65790001ull  // the nil (empty) hash key

struct XeKeyed {
  uint64_t* klog;      // [n * XE_KLOG] key ids a packet touched (| 1: written)
  uint32_t* kcnt;      // [n] keys the packet touched (> XE_KLOG: overflow)
  uint32_t dcap;       // D table slots (power of two)
  uint32_t kw;         // words of a dkey entry: 1 + the longest HASH key's words
  uint64_t* dkid;      // D table: key ids (0 = free)
  uint32_t* dcomp;     // D table: chain (union-find parent, then the root)
  uint32_t* cstart;    // [dcap] position of chain (root) c's first packet in order[]
  uint64_t* dkey;      // D table: [dcap * kw] a held-back insert's key (word 0: map | 0x100 nil | VALID)
  uint64_t* ikey;      // [n * XE_KINS * kw] the key words of a packet's held-back inserts (SPEC)
  uint32_t* dcount;    // [64] D keys per map (sizes the next batch's D table)
  uint32_t* dins;      // [64] D keys per map that a packet inserts (the capacity bound: count + dins)
  uint32_t* cins;      // [64][XE_KSTRIPES] inserts made by the chains (added to the map counts after)
  uint32_t* err;       // build errors: 1 key log overflow, 2 no slot for a reservation, 8 D full, 16 root walk,
                       // 32 an eviction the batch's own packets could see
  uint32_t* changed;   // union-find round changed something
  uint32_t* ckey;      // [n] chain of packet i (dcap: none)
  uint32_t* okey;      // [n] sorted chain keys
  uint32_t* order;     // [n] packet indices sorted by chain, in packet order within a chain
  uint32_t* iota;      // [n] 0..n-1 (sort input)
  uint32_t* counts;    // [0] packets on chains (nO), [1] a long chain, [2] chains, [3] the chain pass's queue
  const uint8_t* skip; // [n] 1 = the packet runs on a chain (the parallel pass leaves it out)
  uint32_t n;          // packets of the batch
  uint32_t nO;         // packets on chains: order[0..nO) (a chain starts where the sorted key changes)
  // LRU evictions in a keyed batch (xe_interp.h keyed_evict_item): the inserts of new keys, in packet
  // order of their first insert, take the oldest live values of the batch's start as victims
  uint32_t* dfirst;    // [dcap] first packet that inserts D key x (XE_NONE: none)
  uint32_t* dvict;     // [dcap] the value id the insert of D key x evicts (XE_NONE: none)
  uint64_t* ekey;      // [dcap] sort keys: map << 32 | dfirst of the LRU inserts, ~0 for anything else
  uint64_t* ekey2;     // [dcap] sorted
  uint32_t* eval;      // [dcap] D indices (sort values)
  uint32_t* eval2;     // [dcap] D indices in (map, first insert) order
  const uint64_t* etsnap;  // the evicting map's value stamps at the batch's start
  const uint32_t* vorder;  // its value ids by start stamp, most recent first (the UsageList of the start)
  uint32_t em, eoff, efree, ecnt0;  // map; its first sorted position; inserts before the first eviction; live count
};

// General lane model (xe_interp.h, XE_GEN): the Go object model without fixed limits, per lane in a
// device arena. Lanes are interleaved (element e of lane l at [e * nl + l]) so the lanes of a wave
// touching the same element touch one contiguous line. Capacities are per lane; running out raises
// XE_FLAG_CAPACITY and the host replays the batch in order with a larger arena (never a packet status).
struct XeGen {
  uint8_t* base;
  uint32_t nl;       // lanes sharing the arena
  uint32_t nobj;     // object ids < nobj (0 = nil, 1..6 = the xdp_md objects)
  uint32_t nframes;  // stack frames kept per lane (1, or 8 = MaxStackFrames with bpf-to-bpf calls)
  uint32_t nvc;      // ValueMemory clones
  uint32_t nbm;      // private ByteMemories
  uint32_t nkey;     // key scratch bytes (hash keys longer than XE_MAX_KEY)
  uint64_t nbytes;   // private byte arena per lane
  uint64_t o_ov, o_oh, o_ot, o_ofree, o_mark, o_frm, o_ctx, o_vc, o_vcinfo, o_vfree, o_bm, o_bfree, o_pres, o_key;
  uint64_t o_bytes;  // per-lane contiguous: lane l's bytes at o_bytes + l * nbytes
  uint32_t mark_words;  // u32 mark words per lane: objects, then VCs, then BMs
  uint32_t pad;
};

// Pipelined-batch epilogue (xe_tail_kernel, one launch after the batch's kernel): publishes the
// batch records to host_aux (a device-visible pointer into the slot's pinned host record) and
// zeroes them for the slot's next batch, decides on the in-order replay, and folds + snapshots the
// ntail small maps (the next batch's rollback point, so that batch needs no prologue launch).
#define XE_TAIL_MAPS 4
#define XE_TAIL_MAP_WORDS 2048  // largest such value region (u64 words, 16 KB)
struct XeTailMap {
  unsigned long long* vals;
  unsigned long long* rep;   // nrep replicas (nrep 0: none)
  unsigned long long* snap;
  uint64_t words;
  uint64_t stride_words;
  uint32_t nrep;
  uint32_t pad;
};
struct XeTailArgs {
  unsigned long long* aux;       // [0] flags, [16 + r * rep_words + w] wave record replica r
  unsigned long long* host_aux;
  uint32_t* poison;
  uint32_t aux_words, nrep, rep_words, nmaps, mode, ntail;
  XeTailMap tail[XE_TAIL_MAPS];
};

// List maps in a parallel run (XeParams::list): each QUEUE / STACK map's element count at the batch's
// start, and per map the facts that decide afterwards whether the run equals packet order: sens = 1 + the
// last packet whose list operation assumed no push happened before it in the batch, push = the first
// packet that pushed (0xffffffff: none). Exact iff sens <= push for every map. popmask: maps popped;
// newlist: a ranked pass met a pop of a list that has no rank slot yet (the pass is run again).
struct XeListRun {
  uint32_t cnt0[64];
  uint32_t sens[64];    // 1 + the last packet with a position that assumed no earlier push (list_pos)
  uint32_t push[64];    // the first packet that pushed
  uint32_t senslo[64];  // the first packet with such a position (the runtime's segment cut)
  unsigned long long popmask;
  unsigned long long newlist;
};
// Pops ranked in parallel: at most XE_POP_SLOTS popped lists per batch, a packet's pops of each counted in
// 8 bits of one word (XeLane::npops, XeParams::popflag)
#define XE_POP_SLOTS 4u
struct XePopSlots {
  uint8_t slot[64];
};

// per-launch parameters
struct XeParams {
  const XeUop* prog;
  int32_t prog_len;
  uint32_t mode;          // XE_MODE_PARALLEL or XE_MODE_SEQUENTIAL
  uint8_t* umem;
  uint64_t umem_len;
  const xe_desc* desc;
  uint32_t n;
  uint32_t nmaps;         // len(vm.Maps) - 1
  uint8_t bigmap[XE_H_BIG_FIELDS];  // map field XE_H_BIG + f: the big map's index, and the field's place
  uint8_t bigoff[XE_H_BIG_FIELDS];  // in that map's run (slot bits 23 and up of the handle)
  xe_result* results;
  uint32_t* verdicts;
  xe_regs* regs;
  const XeDevMap* maps;   // [0..nmaps], index 0 unused
  uint64_t max_steps;
  uint32_t ingress;
  uint32_t rxq;
  uint32_t* flags;             // XE_FLAG_*
  // per-wave flushes go to replica (wave % nrep) to avoid same-address atomic chains; the host
  // reduces the replicas: record = [0] steps, [1..8] status histogram, [16 + 2m] read mask and
  // [17 + 2m] atomic mask of map m
  unsigned long long* rep;
  uint32_t nrep;
  uint32_t rep_words;
  // every program of the VM, concatenated (tail calls switch programs, emulator/helper_functions.go:133-210)
  const XeUop* progs;
  const int32_t* prog_off;  // [0..nprogs]: program p at progs + prog_off[p], prog_off[0] unused
  const int32_t* prog_lens;
  uint32_t nprogs;          // len(vm.Programs) - 1
  int32_t entry;            // PI at Reset (SetEntrypoint)
  XeGen gen;
  // pipelined batches (xe_run_batch_device_async): set on the device by an earlier batch's epilogue
  // when that batch must be replayed in order; the launch then does nothing (null: synchronous run)
  const uint32_t* poison;
  // sequential mode: stage the next 64 packets' descriptors and header windows with the whole wave
  // (no program of the VM writes packet bytes), then run them one after another on lane 0
  uint32_t seq_prefetch;  // sequential mode: 1 = the wave stages 64 packets at a time, 2 = and runs ahead (XE_SEQ_PEEK)
  // keyed ordered execution (XE_MODE_SPEC / XE_MODE_CHAIN, and the skip mask of its parallel pass)
  XeKeyed K;
  // chunk -> wave schedule of the parallel pass (xe_debug_set_schedule): 0 = wave w walks chunks
  // w, w + nwaves, ...; s > 0 = the walk visits chunk (nchunks - 1 - c + s) mod nchunks instead (a
  // permutation; the results may not depend on it)
  uint32_t sched;
  // instruction trace (xe_trace_config; interpreter engine): the traced packets' batch indices, sorted;
  // trace_max records per traced packet and the count each run wrote (null trace: off)
  const uint32_t* trace_pk;
  xe_trace_rec* trace;
  uint32_t* trace_cnt;
  uint32_t trace_npk, trace_max;
  // QUEUE / STACK pops, peeks and lookups in a parallel run (xe_runtime.cpp, "list operations"): null
  // list: off (such an operation raises XE_FLAG_ORDERED). pop_mode 1 = the count pass (a lane stops at
  // its packet's first list operation, flagging popflag[i] = 1 + the map it pops), 2 = a ranked pass: the
  // k-th pop of list m by packet i takes the element at rank popbase[slot * pop_stride + i] + k among the
  // batch's pops of m in packet order (slot = pop_slot[m]), and every packet writes the pops it made
  // (8 bits per slot) to popflag[i]; the runtime reruns the pass until they are the counts it ranked by.
  XeListRun* list;
  uint32_t pop_mode;
  uint32_t pop_stride;
  uint8_t pop_slot[64];   // rank slot of each popped list (0xff: none)
  uint32_t* popflag;
  const uint32_t* popbase;
  // helper table (xe_set_helper): bit id of host[] = a host function, of nil[] = a nil entry
  uint64_t host_helpers[3];
  uint64_t nil_helpers[3];
  struct XeHostCall* hostcall;  // the request mailbox (pinned host memory), sequential mode
};

// Host helper request mailbox (xe_set_helper): the one-lane replay writes the arguments and bumps req
// (system-scope release); the host thread that runs the batch polls it while the kernel runs, calls the
// function, writes r0 / err and sets ack = req (release); the lane spins on ack with a time limit.
#define XE_HOSTCALL_TIMEOUT_TICKS (100ull * 1000 * 1000 * 30)  // 30 s of the 100 MHz constant clock
struct XeHostCall {
  uint32_t req;
  uint32_t ack;
  uint32_t id;
  uint32_t packet;
  int64_t args[5];
  uint8_t kinds[5];
  uint8_t pad[3];
  int32_t err;
  int64_t r0;
  // host side only (the host simulation calls the function in place)
  xe_helper_fn fn[192];
  void* user[192];
};

// Decision of the pipelined-batch epilogue (aux word XE_AUX_DECISION): the batch must be replayed in
// packet order (same rule as the synchronous run's conflict check)
#define XE_AUX_DECISION 1

// The replay rule on the wave records OR-reduced over the replicas (orw[w] = OR of word w): an
// ordered write or a lane out of arena, a read of a field other lanes add to, or adds of more than
// one width on a map (xe_runtime.cpp run_conflict states it on the reduced host copy).
template <class Words>
XE_HD bool xe_replay_decision(uint32_t flags, Words orw, uint32_t rep_words, uint32_t nmaps, uint32_t mode) {
  bool conflict = (flags & (XE_FLAG_ORDERED | XE_FLAG_CAPACITY)) != 0;
  for (uint32_t m = 1; m <= nmaps && m < 64 && 17 + 2 * m < rep_words; m++) {
    if (orw[16 + 2 * m] & orw[16 + 2 * m + 1]) conflict = true;
    const unsigned wc = unsigned(orw[XE_REC_WIDTH0 + m / 16] >> (4 * (m % 16))) & 15u;
    if (wc & (wc - 1)) conflict = true;
  }
  return conflict && (mode == XE_MODE_AUTO || (flags & XE_FLAG_CAPACITY));
}
