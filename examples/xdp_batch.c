/*
 * xdp_batch.c — the C ABI (include/xdpemu.h) driven from plain C, the way a cgo binding would
 * (INTEGRATION.md): NewVM, AddMap, AddRawProgram, SetEntrypoint, then one batch of packets that
 * start and end in host memory (xe_run_batch_host), and the final map state.
 *
 * The program counts packets per EtherType low byte in an ARRAY map and returns XDP_PASS:
 *   r2 = *(u8 *)(ctx->data + 13); key = r2; v = lookup(map 1, &key); if v: *v += 1 (lock xadd)
 * The map starts from initial data given the way gobpfld's AbstractMap.InitialData holds it
 * ({int key: []byte value}, map_abstract.go:33), flattened as ArrayMap.Init does
 * (emulator/maps_array.go:19-44) — the same translation as INTEGRATION.md's initialImage.
 *
 *   gcc -O2 -Iinclude examples/xdp_batch.c -Lgobpfld_amd -lxdpemu -Wl,-rpath,$PWD/gobpfld_amd
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "xdpemu.h"

/* eBPF instruction: op, dst | src << 4, off, imm (little endian, ebpf/ebpf.go:46-76) */
static uint64_t insn(uint8_t op, uint8_t dst, uint8_t src, int16_t off, int32_t imm) {
  return (uint64_t)op | (uint64_t)(dst | (src << 4)) << 8 | (uint64_t)(uint16_t)off << 16 | (uint64_t)(uint32_t)imm << 32;
}

/* one InitialData entry: key -> value bytes */
typedef struct { int key; const uint8_t* val; size_t len; } initial_entry;

/* ArrayMap.Init: copy each value at key*ValueSize (running on into later entries when longer) in
 * ascending key order (Go ranges over the map in random order; order only matters when copies
 * overlap); a key past the memory is an error (Go panics on the slice bound). */
static int initial_image(const xe_map_def* d, const initial_entry* e, size_t n, uint8_t* img) {
  const size_t size = (size_t)d->value_size * d->max_entries;
  memset(img, 0, size);
  int last = -1;
  for (size_t done = 0; done < n; done++) {
    const initial_entry* next = NULL;  /* smallest key above the last one applied */
    for (size_t j = 0; j < n; j++)
      if (e[j].key > last && (!next || e[j].key < next->key)) next = &e[j];
    if (!next) break;
    if (next->key < 0 || (size_t)next->key * d->value_size > size) return -1;
    const size_t off = (size_t)next->key * d->value_size;
    memcpy(img + off, next->val, next->len < size - off ? next->len : size - off);
    last = next->key;
  }
  return 0;
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 4096;
  const uint64_t prog[] = {
      insn(0x61, 6, 1, 0, 0),      /* r6 = *(u32 *)(r1 + 0)   ctx->data            */
      insn(0x71, 2, 6, 13, 0),     /* r2 = *(u8 *)(r6 + 13)   EtherType low byte   */
      insn(0x63, 10, 2, -4, 0),    /* *(u32 *)(r10 - 4) = r2                       */
      insn(0x18, 1, 1, 0, 1),      /* r1 = map 1 (BPF_PSEUDO_MAP_FD, VM index)     */
      insn(0x00, 0, 0, 0, 0),
      insn(0xbf, 2, 10, 0, 0),     /* r2 = r10                                     */
      insn(0x07, 2, 0, 0, -4),     /* r2 += -4                                     */
      insn(0x85, 0, 0, 0, 1),      /* call bpf_map_lookup_elem                     */
      insn(0x15, 0, 0, 2, 0),      /* if r0 == 0 goto +2                           */
      insn(0xb7, 1, 0, 0, 1),      /* r1 = 1                                       */
      insn(0xdb, 0, 1, 0, 0),      /* lock *(u64 *)(r0 + 0) += r1                  */
      insn(0xb7, 0, 0, 0, 2),      /* r0 = XDP_PASS                                */
      insn(0x95, 0, 0, 0, 0),      /* exit                                         */
  };
  xe_settings s;
  xe_vm* vm = NULL;
  int32_t map = 0, p = 0;
  xe_map_def def = {XE_MAP_ARRAY, 4, 8, 256, 0};
  /* InitialData {2: u64 7, 0: u64 1000} */
  static const uint8_t v0[8] = {0xe8, 0x03}, v2[8] = {7};
  const initial_entry init[] = {{2, v2, 8}, {0, v0, 8}};
  uint8_t img[256 * 8];
  xe_default_settings(&s);
  int rc = xe_create(&s, &vm);
  if (rc) { printf("xe_create: %d\n", rc); return 2; }
  if (initial_image(&def, init, 2, img)) { printf("initial data outside the map\n"); return 1; }
  if ((rc = xe_add_map(vm, &def, img, sizeof img, &map)) || (rc = xe_add_raw_program(vm, prog, sizeof prog / 8, &p)) ||
      (rc = xe_set_entrypoint(vm, p))) {
    printf("setup: %d %s\n", rc, xe_last_error(vm));
    return 1;
  }
  uint8_t* umem = calloc(n, 64);
  xe_desc* desc = calloc(n, sizeof *desc);
  uint32_t* verdicts = calloc(n, 4);
  for (uint32_t i = 0; i < n; i++) {
    desc[i].addr = (uint64_t)i * 64;
    desc[i].len = 64;
    umem[i * 64 + 13] = (uint8_t)(i % 3);  /* EtherType low bytes 0, 1, 2 */
  }
  xe_batch_stats st;
  rc = xe_run_batch_host(vm, umem, (uint64_t)n * 64, desc, n, NULL, verdicts, NULL, &st);
  if (rc) { printf("run: %d %s\n", rc, xe_last_error(vm)); return 1; }
  uint64_t counts[256];
  uint64_t got = 0;
  xe_map_dump(vm, map, counts, NULL, 256, &got);
  uint32_t pass = 0;
  for (uint32_t i = 0; i < n; i++) pass += verdicts[i] == 2;
  printf("%s packets=%u pass=%u counts=%llu,%llu,%llu steps=%llu engine=%u\n", xe_version(), n, pass,
         (unsigned long long)counts[0], (unsigned long long)counts[1], (unsigned long long)counts[2],
         (unsigned long long)st.steps, st.engine_used);
  xe_destroy(vm);
  free(umem);
  free(desc);
  free(verdicts);
  return pass == n && counts[0] + counts[1] + counts[2] == (uint64_t)n + 1007 && counts[0] >= 1000 && counts[2] >= 7 ? 0 : 1;
}
