/*
 * oracle.h — TEST INFRASTRUCTURE ONLY. CPU restatement of gobpfld's `emulator/` package.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and
 * only as the checker. The product path (gobpfld_amd / libxdpemu) never links or calls it.
 *
 * The API mirrors include/xdpemu.h (same structs, `orc_` prefix) so tests can run the same batch
 * through both and compare results bit for bit.
 */
#ifndef XDPEMU_ORACLE_H
#define XDPEMU_ORACLE_H
#include "../include/xdpemu.h"
#ifdef __cplusplus
extern "C" {
#endif
typedef struct orc_vm orc_vm;
int orc_create(const xe_settings* s, orc_vm** out);
void orc_destroy(orc_vm* vm);
const char* orc_last_error(const orc_vm* vm);
int orc_add_raw_program(orc_vm* vm, const uint64_t* insns, uint32_t n, int32_t* prog_idx);
int orc_set_entrypoint(orc_vm* vm, int32_t idx);
int orc_add_map(orc_vm* vm, const xe_map_def* def, const void* init, size_t init_len, int32_t* map_idx);
int orc_map_lookup(orc_vm* vm, int32_t map_idx, const void* key, void* value_out);
int orc_map_update(orc_vm* vm, int32_t map_idx, const void* key, const void* value);
int orc_map_delete(orc_vm* vm, int32_t map_idx, const void* key);
int orc_map_update_batch(orc_vm* vm, int32_t map_idx, const void* keys, const void* values, uint64_t count);
int orc_map_count(orc_vm* vm, int32_t map_idx, uint64_t* count);
int orc_map_dump(orc_vm* vm, int32_t map_idx, void* keys_or_raw, void* values, uint64_t cap, uint64_t* count);
int orc_map_dump_list(orc_vm* vm, int32_t map_idx, void* data, uint64_t data_cap, uint32_t* lens, uint64_t cap,
                      uint64_t* count, uint64_t* bytes);
int orc_map_lru_order(orc_vm* vm, int32_t map_idx, void* keys, uint64_t cap, uint64_t* count);
int orc_map_push(orc_vm* vm, int32_t map_idx, const void* value);
/* Sequential per-packet harness over host memory; packet writes land in umem. */
int orc_run_batch(orc_vm* vm, uint8_t* umem, uint64_t umem_len, const xe_desc* desc, uint32_t n,
                  xe_result* results, uint32_t* verdicts, xe_regs* regs, xe_batch_stats* stats);
/* decode-only entry for decoder KATs: writes one type-name line per decoded instruction into buf
 * (ebpf.Instruction %T names, e.g. "Add64Register"); returns XE_OK / XE_ERR_DECODE / XE_ERR_TRANSLATE */
/* decode + Go String() rendering of every instruction (one per line) */
int orc_decode_text(const uint64_t* insns, uint32_t n, char* buf, size_t buflen);
int orc_decode_names(const uint64_t* insns, uint32_t n, char* buf, size_t buflen);
/* Step-by-step records (xe_trace_config / xe_trace_read semantics): after every Step that returns without
 * an error, the registers as VM.String prints them (emulator/vm.go:137-173, 248-270) */
int orc_trace_config(orc_vm* vm, const uint32_t* packets, uint32_t npk, uint32_t max_steps);
int orc_trace_read(orc_vm* vm, uint32_t packet, xe_trace_rec* out, uint32_t cap, uint32_t* nsteps);
/* VM.HelperFunctions entries (xe_set_helper / xe_reset_helper semantics) */
int orc_set_helper(orc_vm* vm, uint32_t id, xe_helper_fn fn, void* user);
int orc_reset_helper(orc_vm* vm, uint32_t id);
#ifdef __cplusplus
}
#endif
#endif
