/*
 * xdpemu.h — C ABI of the MI355X-native batched eBPF/XDP emulator.
 *
 * Drop-in boundary for the userspace VM of dylandreimerink/gobpfld (`emulator/`).
 * Every entry point names the reference interface it replaces (paths relative to the
 * reference module root). The Go-side cgo binding a maintainer would add is shown in
 * INTEGRATION.md.
 *
 * Conventions:
 *   - integer return codes: 0 = ok, negative = errno-like (XE_ERR_*); xe_last_error() has text;
 *   - per-packet failures are reported in xe_result.status, never as a call failure;
 *   - the library copies programs and map definitions;
 *   - one xe_vm per host thread (the reference VM is not goroutine-safe either, emulator/vm.go:14-28).
 *
 * Plain pointers and sizes only: no torch or HIP types in the signatures. Device pointers are
 * passed as `void*`/`const void*` and a HIP stream as `void*` (0 = the VM's own stream).
 */
#ifndef XDPEMU_H
#define XDPEMU_H

#if !defined(__HIPCC_RTC__)
#include <stddef.h>
#include <stdint.h>
#else /* hiprtc (per-program kernels): no C library headers */
typedef unsigned char uint8_t;
typedef unsigned short uint16_t;
typedef unsigned int uint32_t;
typedef unsigned long long uint64_t;
typedef signed char int8_t;
typedef short int16_t;
typedef int int32_t;
typedef long long int64_t;
typedef unsigned long uintptr_t;
typedef __SIZE_TYPE__ size_t;
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* ---- call return codes ---------------------------------------------------------------- */
#define XE_OK 0
#define XE_ERR_INVAL (-22)     /* bad argument / bad index (e.g. SetEntrypoint out of bounds) */
#define XE_ERR_DECODE (-100)   /* ebpf.Decode rejected the program   (ebpf/decode.go:905-913) */
#define XE_ERR_TRANSLATE (-101) /* emulator.Translate rejected it      (emulator/inst.go:230-231) */
#define XE_ERR_MAPTYPE (-102)  /* AbstractMapToVM: type not implemented (emulator/maps.go:155) */
#define XE_ERR_NOMEM (-12)
#define XE_ERR_DEVICE (-200)   /* HIP runtime failure */
#define XE_ERR_UNSUPPORTED (-95)

/* ---- per-packet status (parity taxonomy) -------------------- */
#define XE_ST_OK 0          /* top-level exit; verdict = R0 (emulator/inst_exit.go:24-26)          */
#define XE_ST_VMERR 1       /* Run() returned a *VMError (emulator/vm.go:175-180)                  */
#define XE_ST_PANIC 2       /* the Go VM would panic (runtime error not recovered anywhere)        */
#define XE_ST_BUDGET 3      /* step budget exhausted (the Go VM has none and would hang)           */
#define XE_ST_UNSUPPORTED 4 /* reserved: no instruction or helper of the reference reports it      */

/* VMERR codes (xe_result.code when status == XE_ST_VMERR). Errors raised inside a helper
 * (emulator/inst_call_helper.go:30-33) carry XE_E_IN_HELPER in addition. */
#define XE_E_NO_PROGRAM 1   /* emulator/vm.go:138-140 */
#define XE_E_BAD_REG 2      /* Registers.Get/Copy unknown register, emulator/registers.go:88,115 */
#define XE_E_ASSIGN_REG 3   /* Registers.Assign can't assign, emulator/registers.go:145 */
#define XE_E_READONLY 4     /* FramePointer.Assign on a readonly pointer, emulator/registers.go:306-308 */
#define XE_E_DIV0 5         /* emulator/inst_div.go:10, emulator/inst_mod.go:10 */
#define XE_E_NONPTR_LOAD 6  /* emulator/inst_load.go:103-105 */
#define XE_E_NONPTR_STORE 7 /* emulator/inst_store.go:41-43,89-91; emulator/inst_atomic.go:40-42 */
#define XE_E_OOB 8          /* emulator/memory.go:33-35,56-58,98-100,136-138,177-179,188-190 */
#define XE_E_NONCONTIG 9    /* emulator/memory.go:43-45 */
#define XE_E_UNINIT 10      /* emulator/memory.go:48-50 */
#define XE_E_BAD_PC 11      /* emulator/vm.go:114-115,162-167 */
#define XE_E_NOT_IMPL 12    /* emulator/inst_load.go:131-148, helper 3 (helper_functions.go:104-106) */
#define XE_E_NO_HELPER 13   /* emulator/inst_call_helper.go:21-28,55-63 */
#define XE_E_NO_MAP 14      /* emulator/inst_load.go:39-41 */
#define XE_E_MAP_NOT_PTR 15 /* emulator/inst_load.go:49-52 */
#define XE_E_MAP_OP 16      /* map Lookup/Update/Push/Pop returned an error the helper does not map to
                             * errno, e.g. "update not available on this map type" (maps.go:61-82),
                             * "lookup didn't return a pointer" (helper_functions.go:178-181) */
#define XE_E_HOST_HELPER 17 /* a host helper (xe_set_helper) returned an error: "helper function paniced"
                             * (emulator/inst_call_helper.go:30-33); always with XE_E_IN_HELPER */
#define XE_E_IN_HELPER 0x80

/* PANIC codes (xe_result.code when status == XE_ST_PANIC) */
#define XE_P_NIL_DEREF 1 /* nil interface method call, e.g. emulator/maps_array.go:72-75 */
#define XE_P_NEG_SHIFT 2 /* Go shift by a negative count, emulator/inst_lsh.go:26 etc. */
#define XE_P_DIV0 3      /* int32 divide by zero after a non-zero 64-bit check, emulator/inst_div.go:96 */
#define XE_P_INDEX 4     /* index/slice out of range (negative PC, negative helper id, ReadRange) */
#define XE_P_NIL_MAP 5   /* vm.Maps[0] == nil used as a map, emulator/inst_load.go:43-44 */
#define XE_P_MAKESLICE 6 /* make([]byte, negative) in ReadRange, e.g. bpf_perf_event_output size < 0 */

/* register kinds (emulator/registers.go:176-324) */
#define XE_KIND_IMM 0
#define XE_KIND_MEMPTR 1
#define XE_KIND_FRAMEPTR 2
#define XE_KIND_NIL 3 /* nil RegisterValue: R2 after bpf_map_peek_elem on an empty map (helper_functions.go:356-371) */

/* memory regions a pointer can refer to (parity records) */
#define XE_REGION_PACKET 0
#define XE_REGION_CTX 1
#define XE_REGION_STACK 2
#define XE_REGION_ARRAY 3
#define XE_REGION_HASHVAL 4  /* HASH and LRU_HASH values */
#define XE_REGION_QUEUEVAL 5 /* QUEUE / STACK elements */
#define XE_REGION_PERF 6     /* PERF_EVENT_ARRAY events (Lookup shares the event bytes) */

/* map types: numeric values of bpftypes.BPFMapType (bpftypes/bpf_types.go:155-277) */
#define XE_MAP_HASH 1
#define XE_MAP_ARRAY 2
#define XE_MAP_PROG_ARRAY 3
#define XE_MAP_PERF_EVENT_ARRAY 4
#define XE_MAP_PERCPU_HASH 5
#define XE_MAP_PERCPU_ARRAY 6
#define XE_MAP_LRU_HASH 9
#define XE_MAP_LRU_PERCPU_HASH 10
#define XE_MAP_ARRAY_OF_MAPS 12
#define XE_MAP_HASH_OF_MAPS 13
#define XE_MAP_QUEUE 22
#define XE_MAP_STACK 23

/* engines */
#define XE_ENGINE_AUTO 0   /* per-program gfx950 kernel (hiprtc), interpreter if it cannot be built */
#define XE_ENGINE_INTERP 1 /* shared micro-op interpreter kernel */
#define XE_ENGINE_JIT 2    /* per-program kernel only (error if it cannot be built) */

/* run modes */
#define XE_MODE_AUTO 0       /* parallel, verified; on conflict: map-entry writes as per-key chains  */
                             /* (XE_MODE_KEYED), anything else ordered device execution            */
#define XE_MODE_PARALLEL 1   /* parallel only; conflicts reported in stats, results kept            */
#define XE_MODE_SEQUENTIAL 2 /* exact packet order on one device lane                             */
#define XE_MODE_KEYED 3      /* (xe_batch_stats.mode_used only) map-entry writes: per-key chains  */
#define XE_MODE_CANCELLED 4  /* (xe_batch_stats.mode_used only) a pipelined batch xe_cancel dropped */
#define XE_MODE_SEGMENTS 5   /* (xe_batch_stats.mode_used only) XE_MODE_AUTO ran the batch as packet-order */
                             /* segments, each in parallel: a QUEUE / STACK position depended on a push of */
                             /* an earlier packet, so the packets from there on ran after those before it */

/* AF_XDP descriptor, exactly the layout of gobpfld's xsk.go:695-701 */
typedef struct xe_desc {
    uint64_t addr;
    uint32_t len;
    uint32_t options;
} xe_desc;

/* per-packet result */
typedef struct xe_result {
    uint8_t status;  /* XE_ST_* */
    uint8_t r0_kind; /* XE_KIND_* of R0 */
    uint16_t code;   /* XE_E_* / XE_P_* */
    uint32_t pc;     /* PC of the exiting / faulting instruction */
    int64_t r0;      /* R0.Value() (emulator/registers.go:91-116) */
} xe_result;

/* optional parity record: R0..R9 after the run (VMError snapshot registers on error) */
typedef struct xe_regs {
    int64_t val[10];
    uint8_t kind[10];
    uint8_t region[10];  /* XE_REGION_* for pointers, 0xff for IMM */
    uint8_t map[10];     /* map index for ARRAY/HASHVAL regions, else 0 */
    uint8_t pad[2];
    uint32_t steps;      /* instructions executed */
} xe_regs;

/* gobpfld.BPFMapDef (map_definition.go:15-27) */
typedef struct xe_map_def {
    uint32_t type;
    uint32_t key_size;
    uint32_t value_size;
    uint32_t max_entries;
    uint32_t flags;
} xe_map_def;

/* emulator.VMSettings (emulator/vm.go:282-296) plus the harness/device knobs */
typedef struct xe_settings {
    int32_t stack_frame_size; /* must be 256 (DefaultVMSettings) */
    int32_t max_stack_frames; /* 8 */
    uint64_t max_steps;       /* per-packet step budget; 0 = default (1<<20) */
    uint32_t ingress_ifindex; /* xdp_md.ingress_ifindex seen by every packet (default 1) */
    uint32_t rx_queue_index;  /* xdp_md.rx_queue_index (default 0) */
    int32_t device;           /* HIP device ordinal */
    uint32_t mode;            /* XE_MODE_* */
    uint32_t engine;          /* XE_ENGINE_* */
} xe_settings;

typedef struct xe_batch_stats {
    uint64_t packets;
    uint64_t steps;            /* instructions retired over the batch */
    uint64_t status_count[8];  /* histogram of xe_result.status */
    uint32_t mode_used;        /* XE_MODE_PARALLEL, _KEYED, _SEQUENTIAL, _SEGMENTS (_CANCELLED) */
    uint32_t conflict;         /* 1 if the parallel run was order-dependent */
    float kernel_ms;           /* device time of the interpreter launch(es) */
    float total_ms;            /* device time of the whole call */
    uint32_t engine_used;      /* XE_ENGINE_INTERP or XE_ENGINE_JIT */
    uint32_t grid_blocks;      /* blocks of the parallel launch (1 for the ordered path) */
} xe_batch_stats;

typedef struct xe_vm xe_vm;

/* --- VM lifetime --- */
/* NewVM, emulator/vm.go:30-48 */
int xe_default_settings(xe_settings* s);
int xe_create(const xe_settings* s, xe_vm** out);
void xe_destroy(xe_vm* vm);
/* text of the last failed call on this vm */
const char* xe_last_error(const xe_vm* vm);

/* --- programs: AddRawProgram emulator/vm.go:61-73 (Decode + Translate) --- */
/* insns: n raw 8-byte eBPF instructions (ebpf.RawInstruction, ebpf/ebpf.go:46-56).
 * *prog_idx receives the 1-based program index (emulator/vm.go:36-38,56). */
int xe_add_raw_program(xe_vm* vm, const uint64_t* insns, uint32_t n, int32_t* prog_idx);
/* SetEntrypoint, emulator/vm.go:100-108 */
int xe_set_entrypoint(xe_vm* vm, int32_t prog_idx);

/* --- maps: AddMap / AddAbstractMap emulator/vm.go:75-98, AbstractMapToVM emulator/maps.go:85-156 --- */
/* init/init_len: optional initial bytes of an ARRAY/PERCPU_ARRAY (ArrayMap.Init InitialData,
 * emulator/maps_array.go:19-44). *map_idx receives the 1-based map index. */
int xe_add_map(xe_vm* vm, const xe_map_def* def, const void* init, size_t init_len, int32_t* map_idx);
/* host-side key/value access (Map.Lookup / Map.Update from Go userspace code):
 * lookup returns 1 if found (value copied), 0 if absent. */
int xe_map_lookup(xe_vm* vm, int32_t map_idx, const void* key, void* value_out);
int xe_map_update(xe_vm* vm, int32_t map_idx, const void* key, const void* value);
int xe_map_delete(xe_vm* vm, int32_t map_idx, const void* key);
/* bulk form of xe_map_update (count consecutive keys / values); stops at the first failure and
 * returns its code (the kernel-map counterpart is gobpfld's BPFMap.UpdateBatch, map.go) */
int xe_map_update_batch(xe_vm* vm, int32_t map_idx, const void* keys, const void* values, uint64_t count);
/* Final-state dump. ARRAY: raw ValueSize*MaxEntries bytes into `keys_or_raw`.
 * HASH: entries sorted by key bytes; keys into keys_or_raw (count*key_size), values into values
 * (count*value_size). Pass NULL buffers to query the count/byte size in *count / *bytes. */
int xe_map_count(xe_vm* vm, int32_t map_idx, uint64_t* count);
int xe_map_dump(xe_vm* vm, int32_t map_idx, void* keys_or_raw, void* values, uint64_t cap_entries,
                uint64_t* count);

/* Ordered maps (LRU_HASH, QUEUE, STACK, PERF_EVENT_ARRAY; emulator/maps_hash_lru.go, maps_queue.go,
 * maps_stack.go, maps_perf_event_array.go). xe_map_lookup on an LRU_HASH promotes the key as the Go
 * Lookup does; on a QUEUE / STACK / PERF_EVENT_ARRAY the key is a u32 index into the list.
 * QUEUE / STACK / PERF_EVENT_ARRAY contents in Go slice order (queue front first, stack bottom first,
 * events oldest first): `data` receives the records back to back, `lens` their lengths (0 for a nil
 * backing). NULL buffers query *count and *bytes. */
int xe_map_dump_list(xe_vm* vm, int32_t map_idx, void* data, uint64_t data_cap, uint32_t* lens, uint64_t cap,
                     uint64_t* count, uint64_t* bytes);
/* LRU_HASH UsageList (maps_hash_lru.go:21-24): keys, most recently used first, key_size bytes each */
int xe_map_lru_order(xe_vm* vm, int32_t map_idx, void* keys, uint64_t cap, uint64_t* count);
/* QueueMap/StackMap.Push from userspace (maps_queue.go:60-77): one value_size element */
int xe_map_push(xe_vm* vm, int32_t map_idx, const void* value);

/* --- running: the per-packet harness of SURVEY Appendix B over a batch ---
 * Each packet i runs Reset; R1 = &MemoryPtr{ctx}; Run (emulator/vm.go:110-173, 211-246).
 * Device-resident form: umem, desc, out (and regs if non-NULL) are device pointers.
 * verdicts (device, optional) receives uint32(R0) per packet. */
int xe_run_batch_device(xe_vm* vm, void* d_umem, uint64_t umem_len, const void* d_desc, uint32_t n,
                        void* d_results, void* d_verdicts, void* d_regs, void* stream,
                        xe_batch_stats* stats);
/* Pipelined form of xe_run_batch_device for a stream of batches (a serving loop): enqueues the batch
 * behind those still in flight on the same stream and returns without waiting. The observable result
 * is exactly that of calling xe_run_batch_device for each batch in submission order: each batch's
 * conflict check runs on the device at its end (a one-block epilogue launch that also writes the
 * batch's records straight into pinned host memory and, for value regions up to 16 KB, folds the
 * replicas and snapshots the next batch's rollback point); a batch that must be replayed in
 * packet order stops the batches queued behind it from running, and xe_sync (or the next call that
 * needs the VM's state) rolls the maps back to that batch's start and re-runs it and its successors
 * through the synchronous path. *stats is filled when the batch completes: keep it (and the batch
 * buffers) valid until xe_sync returns. Batches that cannot pipeline (sequential mode, ordered maps,
 * programs that may write packet bytes) run synchronously after everything in flight. Every other
 * entry point that reads or changes VM state completes the pipelined batches first. After pipelined
 * batches, xe_map_delta / xe_map_apply_delta need a synchronous batch first (their base snapshot)
 * unless a shard epoch is open (xe_epoch_begin). Up to 3 batches are in flight per VM.
 * Not a reference entry point: the Go harness runs one packet at a time. */
int xe_run_batch_device_async(xe_vm* vm, void* d_umem, uint64_t umem_len, const void* d_desc, uint32_t n,
                              void* d_results, void* d_verdicts, void* d_regs, void* stream,
                              xe_batch_stats* stats);
/* Complete every pipelined batch (replays included); returns the first error. */
int xe_sync(xe_vm* vm);
/* RunContext's cancellation (emulator/vm.go:117-134: ctx.Err() checked between steps) for the pipelined
 * batches: every batch submitted with xe_run_batch_device_async whose stats are not filled yet is dropped.
 * Batches still queued on the device exit at their first wave, the maps are put back to the state before
 * the oldest dropped batch, and each dropped batch's stats get mode_used = XE_MODE_CANCELLED (its records
 * and verdicts are undefined). The VM then holds exactly the effects of the batches that completed, in
 * submission order. *cancelled (may be NULL) receives how many were dropped. */
int xe_cancel(xe_vm* vm, uint32_t* cancelled);
/* Build ahead of the next batch what it will run: map upload, engine choice and the per-program gfx950
 * kernel for the current program and map geometry (plus its keyed-execution variant when the program
 * may write map entries), so no batch pays a compile. Optional (the first batch does it otherwise); safe
 * to call from several host threads on different VMs (their kernels compile concurrently).
 * Not a reference entry point: the Go VM interprets (emulator/vm.go:110-173) and compiles nothing. */
int xe_prepare(xe_vm* vm);
/* Host-memory form (end-to-end: pinned staging + hipMemcpyAsync H2D/D2H). Packet writes made by the
 * program are copied back into umem (only when the program can write packet memory at all: a
 * may-point-to analysis of the program at load). results/regs may be NULL.
 * For a program that may write packet bytes, a batch whose descriptors cover overlapping bytes runs
 * in packet order (XE_MODE_AUTO; an exact check over the sorted byte ranges): in the reference's
 * loop a later packet reads what an earlier one wrote. */
int xe_run_batch_host(xe_vm* vm, uint8_t* umem, uint64_t umem_len, const xe_desc* desc, uint32_t n,
                      xe_result* results, uint32_t* verdicts, xe_regs* regs, xe_batch_stats* stats);

/* --- multi-GPU shard support: counter deltas for an RCCL all-reduce ---
 * Shards are contiguous packet ranges run in index order: shard k holds the packets after those of
 * shards < k, exactly the order of the reference's per-packet loop. Every shard's VM starts from the
 * same map contents (and hash slot layout). After the runs, either the per-map deltas are summed
 * (when xe_shard_check proves the effects commute across shards) or the shards are replayed in order,
 * each starting from the map state the previous one ended with (xe_map_state_export / _import).
 *
 * Values region of a map as a flat little-endian byte image (ARRAY: ValueSize*MaxEntries; HASH: the
 * device slot table's values, identical layout on every replica built the same way). */
int xe_map_values_bytes(xe_vm* vm, int32_t map_idx, uint64_t* bytes);
/* d_out (device) := current values - snapshot taken at the start of the last run, in lanes of `lane`
 * bytes (1, 2, 4, 8; 0 = the width of the map's adds in the last run): a narrow counter wraps at its
 * own width. Lane 2 deltas are written widened to u32 containers (2 * bytes long: RCCL has no 16-bit
 * integer sum); every other lane is written at its own width (bytes long). */
int xe_map_delta(xe_vm* vm, int32_t map_idx, uint32_t lane, void* d_out, void* stream);
/* values := snapshot + d_in (same lanes and containers as xe_map_delta), wrapping per lane */
int xe_map_apply_delta(xe_vm* vm, int32_t map_idx, uint32_t lane, const void* d_in, void* stream);
/* width in bytes of the last run's adds into this map (1, 2, 4 or 8), 0 when there were none, 8 when
 * more than one width was used (such a run is order-dependent and was replayed in order) */
int xe_map_delta_lane(xe_vm* vm, int32_t map_idx, uint32_t* lane_bytes);
/* Footprint record of the last run, for cross-shard checks: out[0] = XE_FPF_* flags, then for each
 * map m = 1..nmaps three words: read mask, atomic-add mask (64 field positions of a value) and the
 * width classes of its adds (bit 0: 1 B, 1: 2 B, 2: 4 B, 3: 8 B). nwords = 1 + 3 * nmaps. */
#define XE_FPF_ORDERED 1    /* a lane needed a non-commutative map write */
#define XE_FPF_SEQUENTIAL 2 /* the results come from the exact ordered replay or the keyed chains   */
                            /* (map writes in order)                                               */
#define XE_FPF_UNALIGNED 4  /* a map add was not aligned to its own width */
#define XE_FPF_EPOCH 8      /* the record covers a shard epoch (xe_epoch_begin): several batches */
int xe_footprint(xe_vm* vm, uint64_t* out, uint32_t cap_words, uint32_t* nwords);
/* Cross-shard exactness check over the footprints (xe_footprint records, nwords each) of ngpus
 * shards given in shard order. Returns 1 when init + the sum of the per-map deltas equals the state
 * one VM reaches over all shards in order and every shard saw the map values that VM would have
 * shown it: no shard used the ordered path, no shard read a field an earlier shard added to, one add
 * width per map everywhere, aligned adds. lanes[m - 1] receives the lane of map m (0 = no adds).
 * Returns 0 when the shards must be replayed in order instead. */
int xe_shard_check(const uint64_t* fps, uint32_t ngpus, uint32_t nwords, uint32_t* lanes);
/* Shard epoch: from xe_epoch_begin (after the batches before it are complete) until xe_epoch_end,
 * xe_footprint ORs the footprints of every batch run in between (synchronous and pipelined, flag
 * XE_FPF_EPOCH) and xe_map_delta / xe_map_apply_delta / xe_map_delta_lane work against the map values
 * at the epoch's start, so shards can run many batches and exchange once. With XE_FPF_EPOCH
 * xe_shard_check also refuses a read of a field ANY other shard added to (a later batch of one shard
 * follows every shard's earlier batches in the reference's order). Replaces the per-batch exchange
 * of SURVEY §8e for streams of batches; the reference is one VM walking every packet in order
 * (emulator/vm.go:110-173 per packet). */
int xe_epoch_begin(xe_vm* vm, void* stream);
int xe_epoch_end(xe_vm* vm);
/* Whole map state (values, hash slot records and entry count) as a device byte image, for the in-order
 * shard replay: export on the shard that finished, import on the next (same map geometry). */
int xe_map_state_bytes(xe_vm* vm, int32_t map_idx, uint64_t* bytes);
int xe_map_state_export(xe_vm* vm, int32_t map_idx, void* d_out, void* stream);
int xe_map_state_import(xe_vm* vm, int32_t map_idx, const void* d_in, void* stream);

/* --- one process, N devices (SURVEY §8b xe_run_batch_multi): the Go host shards a batch over the
 * GPUs of a node through the FFI alone. vms[k] runs on its own device with identical programs, maps
 * and map contents (the caller sets each up the same way). Exchange over RCCL (xGMI) when the devices
 * are distinct; VMs sharing a device (tests on one GPU) exchange through device kernels instead. */
typedef struct xe_multi xe_multi;
int xe_multi_create(xe_vm* const* vms, uint32_t ngpus, xe_multi** out);
void xe_multi_destroy(xe_multi* m);
/* Shard k: d_umem[k] (umem_len[k] bytes), d_desc[k] (n[k] descriptors), results/verdicts (may be
 * NULL) — all on vms[k]'s device. Runs the shards concurrently, then makes every VM's maps equal to
 * the single-VM result: delta all-reduce when xe_shard_check passes, otherwise the in-order replay
 * (results of the replayed shards are rewritten). stats (may be NULL) receives ngpus records;
 * *replayed (may be NULL) is 1 when the in-order replay ran. */
int xe_run_batch_multi(xe_multi* m, void* const* d_umem, const uint64_t* umem_len, const void* const* d_desc,
                       const uint32_t* n, void* const* d_results, void* const* d_verdicts, xe_batch_stats* stats,
                       uint32_t* replayed);
const char* xe_multi_last_error(const xe_multi* m);

/* --- per-program kernel cache (no reference counterpart: the Go VM compiles nothing) ---
 * A process-wide directory of compiled per-program kernels (code objects named by a hash of the
 * generated source, the interpreter headers, the options and the gfx target); NULL/"" disables it.
 * hiprtc compiles one kernel at a time per process, so a caller with many programs can have other
 * processes fill the cache: xe_kernel_source gives the source xe_prepare would compile (variant 0: the
 * per-program kernel, 1: its keyed-execution variant, 2: its verdict-only variant — the one parallel
 * runs without result / register records use; XE_ERR_UNSUPPORTED when the VM runs none) and
 * xe_compile_kernel_source compiles one into the directory without a device. NULL buf queries *len. */
int xe_set_kernel_cache(const char* dir);
int xe_kernel_source(xe_vm* vm, int variant, char* buf, size_t cap, size_t* len);
int xe_compile_kernel_source(const char* src, const char* arch, const char* dir, char* err, size_t errlen);
/* the file name (in the cache directory) of the code object a source compiles to for `arch` */
int xe_kernel_object_name(const char* src, const char* arch, char* buf, size_t cap);
/* Kernel build statistics of this process: code objects loaded from the cache directory, per-program
 * kernels compiled in-process by hiprtc (cache misses) and their total wall seconds. Diagnostics only
 * (the -m gpu suite reports tests that compiled). */
int xe_kernel_cache_stats(uint64_t* hits, uint64_t* compiles, double* compile_s);

/* --- Step / VM.String (emulator/vm.go:137-173, 248-270): per-packet instruction trace ---
 * xe_trace_config selects packets by their index in each batch (at most XE_TRACE_MAX_PACKETS; duplicates
 * collapse) and keeps the first max_steps steps of each (at most XE_TRACE_MAX_STEPS): after every
 * instruction that completes (Step returns without an error; the exiting instruction included) one record
 * of what VM.String prints — PC, PI, SF and R0..R10. While a trace is configured batches run on the
 * interpreter engine and synchronously (pipelined batches too); a batch that is replayed in order or
 * through the keyed path re-records what it re-runs, so the records are those of the execution whose
 * results the batch reports. npk = 0 turns tracing off. */
#define XE_TRACE_MAX_PACKETS 4096
#define XE_TRACE_MAX_STEPS 65536
typedef struct xe_trace_rec {
    uint32_t packet;  /* index in the batch */
    uint32_t step;    /* 0-based: the packet's step-th instruction */
    int32_t pc;       /* PC of that instruction (Registers.PC before Step's increment) */
    int32_t pi;       /* Registers.PI after it (a tail call changes it) */
    uint32_t sf;      /* Registers.SF after it: bpf-to-bpf call depth */
    uint8_t kind[11]; /* R0..R10: XE_KIND_* */
    uint8_t pad;
    int64_t val[11];  /* R0..R10: RegisterValue.Value() (a pointer's offset) */
} xe_trace_rec;
int xe_trace_config(xe_vm* vm, const uint32_t* packets, uint32_t npk, uint32_t max_steps);
/* Records of packet `packet` of the last batch run (it must be one xe_trace_config named): out[0..*nsteps),
 * *nsteps = min(steps the packet completed, max_steps); cap = room in out (NULL/0: query *nsteps). */
int xe_trace_read(xe_vm* vm, uint32_t packet, xe_trace_rec* out, uint32_t cap, uint32_t* nsteps);

/* --- the VM's helper table (VM.HelperFunctions, emulator/vm.go:23,35; HelperFunc,
 * emulator/helper_functions.go:17) ---
 * A host helper is called with R1..R5 (RegisterValue.Value() and XE_KIND_* of each: pointers pass their
 * offset; the emulator's memory stays on the device) and the packet's index in the batch; it returns 0 and
 * sets *r0, which becomes R0 (an IMM), or non-zero: the packet stops with XE_ST_VMERR, code
 * XE_E_HOST_HELPER | XE_E_IN_HELPER ("helper function paniced", inst_call_helper.go:30-33). R1..R5 are
 * left as they were (a HelperFunc "should never touch R6-R9" and the built-ins leave R1-R5 alone).
 * Host helpers run in packet order on the exact one-lane path (the parallel pass defers a packet that
 * calls one to it), on the host thread that called the batch, which serves the device's requests while
 * the batch runs. */
typedef int (*xe_helper_fn)(void* user, uint32_t packet, const int64_t args[5], const uint8_t kinds[5], int64_t* r0);
/* id < 192 (LinuxHelperFunctions' table size). fn != NULL: the host function replaces table entry id
 * (a built-in included); fn == NULL: the entry becomes nil (a call fails with XE_E_NO_HELPER,
 * inst_call_helper.go:26-28). */
int xe_set_helper(xe_vm* vm, uint32_t id, xe_helper_fn fn, void* user);
/* entry id back to LinuxHelperFunctions' (emulator/helper_functions.go:20-44): the built-in or nil */
int xe_reset_helper(xe_vm* vm, uint32_t id);

/* --- debug hooks (no reference counterpart) ---
 * Permute the chunk -> wave schedule of the parallel passes (0 = the default walk; s > 0 = a fixed
 * permutation of the 64-packet chunks). Results, register records and map contents may not depend on
 * it: the determinism tests run one batch under several schedules and compare. */
int xe_debug_set_schedule(xe_vm* vm, uint32_t sched);
/* Set the run counter the LRU stamps carry in their top 16 bits (xe_interp.h lru_stamp), so a test can
 * reach the renumbering the runtime does before it wraps (0 <= epoch <= 0xffff) without 65,535 runs. */
int xe_debug_set_lru_epoch(xe_vm* vm, uint64_t epoch);
/* An ordered map's device value pool: its room (value ids) and the next fresh id (LRU_HASH / QUEUE /
 * STACK; PERF: event records). Tests check that a stream of evicting batches keeps the pool's size. */
int xe_debug_map_pool(xe_vm* vm, int32_t map, uint64_t* room, uint64_t* next_id);

/* build / device info */
const char* xe_version(void);
int xe_device_count(int* n);

#ifdef __cplusplus
}
#endif
#endif /* XDPEMU_H */
