// oracle.cpp — TEST INFRASTRUCTURE ONLY (see oracle.h). Parity oracle for the device emulator.
//
// A CPU restatement of dylandreimerink/gobpfld `emulator/` + `ebpf/decode.go`, written to follow
// the Go source structure: registers hold *objects* with identity (IMMValue / MemoryPtr /
// FramePointer), ValueMemory stores object references per byte, ByteMemory stores bytes, maps are
// ArrayMap / HashMap. Go runtime panics become C++ exceptions (GoPanic); Go `error` returns become
// integer codes. Every function cites the reference file:line it restates. Paths are relative to
// the reference module root.
//
// Pinning: decoder accept/reject + type mapping is checked against the reference's own fixture
// ebpf/asm_test.bpfasm (tests/golden/asm_test.bpfasm); VM execution semantics have no reference
// fixture (the reference has no VM test and no Go toolchain is available) — see DESIGN.md §Oracle.
#include "oracle.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <list>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace orc {

struct GoPanic { int code; };
struct Unsupported {};

// ---------------------------------------------------------------- instructions (ebpf/*.go)
enum Kind : uint8_t {
  K_LDIMM64, K_NOP, K_LDABS, K_LDIND, K_LDX, K_ST, K_STX, K_ATOMIC, K_ALU, K_NEG, K_END,
  K_JA, K_JMP, K_CALL, K_CALLBPF, K_CALLX, K_EXIT
};
// ALU op codes are the BPF_* op nibble (ebpf/ebpf.go:267-296); jumps likewise (:298-327).
enum { OP_ADD = 0x00, OP_SUB = 0x10, OP_MUL = 0x20, OP_DIV = 0x30, OP_OR = 0x40, OP_AND = 0x50,
       OP_LSH = 0x60, OP_RSH = 0x70, OP_NEG = 0x80, OP_MOD = 0x90, OP_XOR = 0xa0, OP_MOV = 0xb0,
       OP_ARSH = 0xc0, OP_END = 0xd0 };
enum { J_JA = 0x00, J_JEQ = 0x10, J_JGT = 0x20, J_JGE = 0x30, J_JSET = 0x40, J_JNE = 0x50,
       J_JSGT = 0x60, J_JSGE = 0x70, J_CALL = 0x80, J_CALLX = 0x88, J_EXIT = 0x90, J_JLT = 0xa0,
       J_JLE = 0xb0, J_JSLT = 0xc0, J_JSLE = 0xd0 };

struct Inst {
  Kind k;
  uint8_t op = 0;       // ALU/JMP op nibble, atomic imm, END: 0 = to_le / 8 = to_be
  bool wide = false;    // ALU64 / JMP (64-bit) vs ALU32 / JMP32
  bool reg = false;     // BPF_X form
  uint8_t dst = 0, src = 0;
  int16_t off = 0;
  int32_t imm = 0;
  uint32_t val1 = 0, val2 = 0;  // LoadConstant64bit (ebpf/decode.go:28-33)
  uint8_t size = 0;             // ebpf.Size code
};

static int sizeBytes(uint8_t s) {  // ebpf.Size.Bytes, ebpf/ebpf.go:132-145
  switch (s) { case 0x00: return 4; case 0x08: return 2; case 0x10: return 1; case 0x18: return 8; }
  return 0;
}

static const char* aluName(uint8_t op) {
  switch (op) {
    case OP_ADD: return "Add"; case OP_SUB: return "Sub"; case OP_MUL: return "Mul";
    case OP_DIV: return "Div"; case OP_OR: return "Or"; case OP_AND: return "And";
    case OP_LSH: return "Lsh"; case OP_RSH: return "Rsh"; case OP_MOD: return "Mod";
    case OP_XOR: return "Xor"; case OP_MOV: return "Mov"; case OP_ARSH: return "ARSH";
  }
  return "?";
}
static const char* jmpName(uint8_t op) {
  switch (op) {
    case J_JEQ: return "JumpEqual"; case J_JGT: return "JumpGreaterThan";
    case J_JGE: return "JumpGreaterThanEqual"; case J_JSET: return "JumpAnd";
    case J_JNE: return "JumpNotEqual"; case J_JSGT: return "JumpSignedGreaterThan";
    case J_JSGE: return "JumpSignedGreaterThanOrEqual"; case J_JLT: return "JumpSmallerThan";
    case J_JLE: return "JumpSmallerThanEqual"; case J_JSLT: return "JumpSignedSmallerThan";
    case J_JSLE: return "JumpSignedSmallerThanOrEqual";
  }
  return "?";
}

// Go type name of the decoded instruction (for decoder KATs against ebpf/asm_test.bpfasm).
static std::string typeName(const Inst& i) {
  switch (i.k) {
    case K_LDIMM64: return "LoadConstant64bit";
    case K_NOP: return "Nop";
    case K_LDABS: return "LoadSocketBufConstant";
    case K_LDIND: return "LoadSocketBuf";
    case K_LDX: return "LoadMemory";
    case K_ST: return "StoreMemoryConstant";
    case K_STX: return "StoreMemoryRegister";
    case K_ATOMIC:
      switch (i.op & 0xfe) {
        case 0x00: return "AtomicAdd"; case 0x10: return "AtomicSub"; case 0x50: return "AtomicAnd";
        case 0x40: return "AtomicOr"; case 0xa0: return "AtomicXor";
        case 0xe0: return "AtomicExchange"; case 0xf0: return "AtomicCompareAndExchange";
      }
      return "?";
    case K_ALU: return std::string(aluName(i.op)) + (i.wide ? "64" : "32") + (i.reg ? "Register" : "");
    case K_NEG: return i.wide ? "Neg64" : "Neg32";
    case K_END: return std::string("End") + std::to_string(i.imm) + (i.op ? "ToBE" : "ToLE");
    case K_JA: return "Jump";
    case K_JMP: return std::string(jmpName(i.op)) + (i.reg ? "Register" : "") + (i.wide ? "" : "32");
    case K_CALL: return "CallHelper";
    case K_CALLBPF: return "CallBPF";
    case K_CALLX: return "CallHelperIndirect";
    case K_EXIT: return "Exit";
  }
  return "?";
}

// ebpf.Decode, ebpf/decode.go:8-917. Returns false on a decode error.
static bool decode(const uint64_t* raw, uint32_t n, std::vector<Inst>& out, std::string& err) {
  out.clear();
  for (uint32_t i = 0; i < n; i++) {
    uint64_t r = raw[i];
    uint8_t op = uint8_t(r & 0xff);
    uint8_t regs = uint8_t((r >> 8) & 0xff);
    Inst in{};
    in.dst = regs & 0x0f;          // GetDestReg, ebpf/ebpf.go:63-65
    in.src = (regs >> 4) & 0x0f;   // GetSourceReg, ebpf/ebpf.go:71-73
    in.off = int16_t((r >> 16) & 0xffff);
    in.imm = int32_t(uint32_t(r >> 32));
    uint8_t cls = op & 0x07;
    bool ok = true;
    if (op == 0x18) {  // BPF_LD|BPF_DW|BPF_IMM, decode.go:21-36
      if (i + 1 >= n) { err = "load double word imm op code found but not enough instructions"; return false; }
      in.k = K_LDIMM64;
      in.val1 = uint32_t(in.imm);
      in.val2 = uint32_t(raw[i + 1] >> 32);
      out.push_back(in);
      Inst nop{}; nop.k = K_NOP;
      out.push_back(nop);
      i++;
      continue;
    }
    switch (op) {
      case 0x20: case 0x28: case 0x30: case 0x38:  // LD ABS, decode.go:38-60
        in.k = K_LDABS; in.size = op & 0x18; break;
      case 0x40: case 0x48: case 0x50: case 0x58:  // LD IND, decode.go:62-88
        in.k = K_LDIND; in.size = op & 0x18; break;
      case 0x61: case 0x69: case 0x71: case 0x79:  // LDX MEM, decode.go:90-100
        in.k = K_LDX; in.size = op ^ 0x61; break;
      case 0x62: case 0x6a: case 0x72: case 0x7a:  // ST MEM, decode.go:102-111
        in.k = K_ST; in.size = op ^ 0x62; break;
      case 0x63: case 0x6b: case 0x73: case 0x7b:  // STX MEM, decode.go:113-122
        in.k = K_STX; in.size = op ^ 0x63; break;
      case 0xc3: case 0xcb: case 0xd3: case 0xdb: {  // STX ATOMIC, decode.go:124-184
        in.k = K_ATOMIC; in.size = op ^ 0xc3;
        int32_t a = in.imm;
        if (a == 0x00 || a == 0x01 || a == 0x10 || a == 0x11 || a == 0x50 || a == 0x51 ||
            a == 0x40 || a == 0x41 || a == 0xa0 || a == 0xa1 || a == 0xe1 || a == 0xf1)
          in.op = uint8_t(a);
        else ok = false;
        break;
      }
      default:
        if (cls == 0x04 || cls == 0x07) {  // ALU / ALU64, decode.go:186-540
          uint8_t aop = op & 0xf0;
          bool x = (op & 0x08) != 0;
          in.wide = cls == 0x07;
          if (aop == OP_NEG) {  // decode.go:394-402 (BPF_K only)
            if (x) { ok = false; break; }
            in.k = K_NEG;
          } else if (aop == OP_END) {  // decode.go:510-540 (ALU class only, imm 16/32/64)
            if (cls != 0x04 || !(in.imm == 16 || in.imm == 32 || in.imm == 64)) { ok = false; break; }
            in.k = K_END; in.op = x ? 8 : 0;
          } else if (aop == 0xe0 || aop == 0xf0) {
            ok = false;
          } else {
            in.k = K_ALU; in.op = aop; in.reg = x;
          }
        } else if (cls == 0x05 || cls == 0x06) {  // JMP / JMP32, decode.go:544-902
          uint8_t jop = op & 0xf0;
          bool x = (op & 0x08) != 0;
          in.wide = cls == 0x05;
          if (cls == 0x05 && op == 0x05) { in.k = K_JA; break; }            // decode.go:544-547
          if (cls == 0x05 && op == 0x85) { in.k = in.src == 1 ? K_CALLBPF : K_CALL; break; }  // :761-771
          if (cls == 0x05 && op == 0x8d) { in.k = K_CALLX; break; }         // :773-777
          if (cls == 0x05 && op == 0x95) { in.k = K_EXIT; break; }          // :781-782
          switch (jop) {
            case J_JEQ: case J_JGT: case J_JGE: case J_JSET: case J_JNE: case J_JSGT: case J_JSGE:
            case J_JLT: case J_JLE: case J_JSLT: case J_JSLE:
              in.k = K_JMP; in.op = jop; in.reg = x; break;
            default: ok = false;
          }
        } else {
          ok = false;
        }
    }
    if (!ok) {
      char b[160];
      snprintf(b, sizeof b, "unable to decode raw instruction, inst: %u, op: %2x", i, op);
      err = b;
      return false;
    }
    out.push_back(in);
  }
  return true;
}

// emulator.Translate, emulator/inst.go:21-238: JLT/JLE/JSET and every atomic except ADD are rejected.
static bool translate(const std::vector<Inst>& prog, std::string& err) {
  for (size_t i = 0; i < prog.size(); i++) {
    const Inst& in = prog[i];
    bool bad = (in.k == K_JMP && (in.op == J_JLT || in.op == J_JLE || in.op == J_JSET)) ||
               (in.k == K_ATOMIC && (in.op & 0xfe) != 0x00);
    if (bad) {
      err = "can't translate instruction at " + std::to_string(i) + " of type *ebpf." + typeName(in);
      return false;
    }
  }
  return true;
}


// Go String() of each decoded instruction (ebpf/*.go String methods), used to pin the decoder
// against the reference fixture ebpf/asm_test.bpfasm (TestDecodeEncodeSymmetry, ebpf/asm_test.go).
static const char* kHelperNames[] = {
    "", "bpf_map_lookup_elem", "bpf_map_update_elem", "bpf_map_delete_elem", "bpf_probe_read",
    "bpf_ktime_get_ns", "bpf_trace_printk", "bpf_get_prandom_u32", "bpf_get_smp_processor_id",
    "bpf_skb_store_bytes", "bpf_l3_csum_replace", "bpf_l4_csum_replace", "bpf_tail_call",
    "bpf_clone_redirect", "bpf_get_current_pid_tgid", "bpf_get_current_uid_gid",
    "bpf_get_current_comm", "bpf_get_cgroup_classid", "bpf_skb_vlan_push", "bpf_skb_vlan_pop",
    "bpf_skb_get_tunnel_key", "bpf_skb_set_tunnel_key", "bpf_perf_event_read", "bpf_redirect",
    "bpf_get_route_realm", "bpf_perf_event_output", "bpf_skb_load_bytes", "bpf_get_stackid",
    "bpf_csum_diff", "bpf_skb_get_tunnel_opt", "bpf_skb_set_tunnel_opt", "bpf_skb_change_proto",
    "bpf_skb_change_type", "bpf_skb_under_cgroup", "bpf_get_hash_recalc", "bpf_get_current_task",
    "bpf_probe_write_user"};

static std::string regName(int r) { return r < 11 ? std::to_string(r) : std::string("invalid"); }
static const char* sizeName(uint8_t s) {
  switch (s) { case 0x00: return "u32"; case 0x08: return "u16"; case 0x10: return "u8"; case 0x18: return "u64"; }
  return "invalid";
}
static std::string signedOff(int64_t off) {  // "+ 456" / "- 456"
  return off < 0 ? "- " + std::to_string(-off) : "+ " + std::to_string(off);
}
static std::string plusd(int64_t v) { return (v >= 0 ? "+" : "") + std::to_string(v); }  // Go %+d

static std::string goString(const Inst& i) {
  std::string d = regName(i.dst), s = regName(i.src);
  const char* p = i.wide ? "r" : "w";
  switch (i.k) {
    case K_LDIMM64:
      if (i.src == 1) return "r" + d + " = map fd#" + std::to_string(i.val1);
      if (i.src == 2) return "r" + d + " = map value#" + std::to_string(i.val1) + "[" + std::to_string(i.val2) + "]";
      return "r" + d + " = " + std::to_string((uint64_t(i.val2) << 32) + uint64_t(i.val1)) + " ll";
    case K_NOP: return "nop";
    case K_LDABS: return std::string("r0 = ntohl((") + sizeName(i.size) + ") (((struct sk_buff *) r6)->data[" + std::to_string(i.imm) + "]))";
    case K_LDIND: return std::string("r0 = ntohl((") + sizeName(i.size) + ") (((struct sk_buff *) r6)->data[r" + s + " " + signedOff(i.imm) + "]))";
    case K_LDX: return "r" + d + " = *(" + sizeName(i.size) + " *)(r" + s + " " + signedOff(i.off) + ")";
    case K_ST: return std::string("*(") + sizeName(i.size) + " *)(r" + d + " " + signedOff(i.off) + ") = " + std::to_string(i.imm);
    case K_STX: return std::string("*(") + sizeName(i.size) + " *)(r" + d + " " + signedOff(i.off) + ") = r" + s;
    case K_ATOMIC: {
      std::string reg = i.size == 0x00 ? "w" : "r";
      std::string mem = std::string("*(") + sizeName(i.size) + " *)(r" + d + " " + signedOff(i.off) + ")";
      switch (i.op & 0xfe) {
        case 0x00: return "lock " + mem + " += " + reg + s;
        case 0x10: return "lock " + mem + " -= " + reg + s;
        case 0x50: return "lock " + mem + " &= " + reg + s;
        case 0x40: return "lock " + mem + " |= " + reg + s;
        case 0xa0: return "lock " + mem + " ^= " + reg + s;
        case 0xe0: return reg + s + " = xchg(r" + d + " " + signedOff(i.off) + ", " + reg + s + ")";
        case 0xf0: return reg + "0 = cmpxchg(r" + d + " " + signedOff(i.off) + ", " + reg + "0, " + reg + s + ")";
      }
      return "?";
    }
    case K_ALU: {
      const char* op = "?";
      switch (i.op) {
        case OP_ADD: op = "+="; break; case OP_SUB: op = "-="; break; case OP_MUL: op = "*="; break;
        case OP_DIV: op = "/="; break; case OP_OR: op = "|="; break; case OP_AND: op = "&="; break;
        case OP_LSH: op = "<<="; break; case OP_RSH: op = ">>="; break; case OP_MOD: op = "%="; break;
        case OP_XOR: op = "^="; break; case OP_MOV: op = "="; break; case OP_ARSH: op = "s>>="; break;
      }
      std::string rhs = i.reg ? std::string(p) + s : std::to_string(i.imm);
      return std::string(p) + d + " " + op + " " + rhs;
    }
    case K_NEG: return std::string(p) + d + " = -" + p + d;
    case K_END: return "r" + d + " = " + (i.op ? "be" : "le") + std::to_string(i.imm) + " r" + d;
    case K_JA: return "goto " + plusd(i.off);
    case K_JMP: {
      const char* op = "?";
      switch (i.op) {
        case J_JEQ: op = "=="; break; case J_JGT: op = ">"; break; case J_JGE: op = ">="; break;
        case J_JSET: op = "&"; break; case J_JNE: op = "!="; break; case J_JSGT: op = "s>"; break;
        case J_JSGE: op = "s>="; break; case J_JLT: op = "<"; break; case J_JLE: op = "<="; break;
        case J_JSLT: op = "s<"; break; case J_JSLE: op = "s<="; break;
      }
      std::string rhs = i.reg ? std::string(p) + s : std::to_string(i.imm);
      return std::string("if ") + p + d + " " + op + " " + rhs + " goto " + plusd(i.off);
    }
    case K_CALL: return "call " + std::to_string(i.imm) + "#" + ((i.imm >= 0 && i.imm <= 36) ? kHelperNames[i.imm] : "");
    case K_CALLBPF: return "call " + plusd(i.imm);
    case K_CALLX: return "callx r" + regName(uint8_t(i.imm));
    case K_EXIT: return "exit";
  }
  return "?";
}

// ---------------------------------------------------------------- values & memory
struct Memory;
struct RV {  // RegisterValue, emulator/registers.go:151-166
  virtual ~RV() {}
  virtual int kind() const = 0;
  virtual int64_t Value() const = 0;
};
struct IMM : RV {  // IMMValue, registers.go:176-206
  int64_t v;
  explicit IMM(int64_t x) : v(x) {}
  int kind() const override { return XE_KIND_IMM; }
  int64_t Value() const override { return v; }
};
struct MemPtr : RV {  // MemoryPtr, registers.go:209-250
  Memory* mem; int64_t off;
  MemPtr(Memory* m, int64_t o) : mem(m), off(o) {}
  int kind() const override { return XE_KIND_MEMPTR; }
  int64_t Value() const override { return off; }
};
struct FramePtr : RV {  // FramePointer, registers.go:258-324
  Memory* mem; int index; int64_t off; bool ro;
  FramePtr(Memory* m, int idx, int64_t o, bool r) : mem(m), index(idx), off(o), ro(r) {}
  int kind() const override { return XE_KIND_FRAMEPTR; }
  int64_t Value() const override { return off; }
};

struct VM;
struct Memory {  // emulator/memory.go:11-18
  int region = 0, mapidx = 0;
  virtual ~Memory() {}
  virtual int Read(int64_t off, int size, RV** out, VM* vm) = 0;
  virtual int ReadRange(int64_t off, int64_t count, std::vector<uint8_t>* out) = 0;
  virtual int Write(int64_t off, RV* v, int size) = 0;
  virtual int64_t Size() const = 0;
  virtual Memory* Clone(VM* vm) = 0;
  virtual bool isValueMemory() const { return false; }
};

static inline int64_t wadd(int64_t a, int64_t b) { return int64_t(uint64_t(a) + uint64_t(b)); }

// A RegisterValue interface may be nil: bpf_map_peek_elem on an empty queue/stack sets R2 = nil
// (helper_functions.go:356-371). Calling a method on it panics; a type assertion on it fails.
static int64_t V(const RV* r) { if (!r) throw GoPanic{XE_P_NIL_DEREF}; return r->Value(); }
static int KindOf(const RV* r) { if (!r) throw GoPanic{XE_P_NIL_DEREF}; return r->kind(); }
static inline int64_t wmul(int64_t a, int64_t b) { return int64_t(uint64_t(a) * uint64_t(b)); }

// Go bounds check `offset < 0 || offset+size > len` with wrapping addition; an index that passes
// the check but is still >= len (only via overflow) panics at the slice index.
static int boundsCheck(int64_t off, int64_t size, int64_t len) {
  if (off < 0 || wadd(off, size) > len) return XE_E_OOB;
  if (off >= len && size > 0) throw GoPanic{XE_P_INDEX};
  return 0;
}

struct ValueMemory : Memory {  // emulator/memory.go:23-120
  std::vector<RV*> mapping;
  bool isValueMemory() const override { return true; }
  int64_t Size() const override { return int64_t(mapping.size()); }
  int Read(int64_t off, int size, RV** out, VM*) override {  // memory.go:32-53
    if (int e = boundsCheck(off, size, Size())) return e;
    RV* val = mapping[off];
    for (int64_t i = off; i < off + size; i++)
      if (mapping[i] != val) return XE_E_NONCONTIG;
    if (!val) return XE_E_UNINIT;
    *out = val;
    return 0;
  }
  int ReadRange(int64_t off, int64_t count, std::vector<uint8_t>* out) override {  // memory.go:55-95
    if (off < 0 || wadd(off, count) > Size()) return XE_E_OOB;
    if (count < 0) throw GoPanic{XE_P_MAKESLICE};  // make([]byte, count)
    std::vector<uint8_t> r(size_t(count), 0);
    for (int64_t i = 0; i < count;) {
      RV* v = mapping[off + i];
      if (!v) { r[i] = 0; i++; continue; }
      int size = 1;
      for (int64_t j = i + 1; j < i + 8 && j < count; j++) {
        if (v != mapping[off + j]) break;
        size++;
      }
      uint64_t x = uint64_t(v->Value());
      int w = size > 4 ? 8 : size > 2 ? 4 : size > 1 ? 2 : 1;
      if (i + w > count) throw GoPanic{XE_P_INDEX};  // r[i:i+w] beyond cap(r) panics
      for (int b = 0; b < w; b++) r[i + b] = uint8_t(x >> (8 * b));
      i += w;
    }
    *out = std::move(r);
    return 0;
  }
  int Write(int64_t off, RV* v, int size) override {  // memory.go:97-107
    if (int e = boundsCheck(off, size, Size())) return e;
    for (int64_t i = off; i < off + size; i++) mapping[i] = v;
    return 0;
  }
  Memory* Clone(VM* vm) override;
};

struct ByteMemory : Memory {  // emulator/memory.go:125-223 (little endian; ByteOrder nil => LE)
  uint8_t* ext = nullptr;            // packet bytes live in the caller's umem
  std::vector<uint8_t> own;          // map memories own their backing
  int64_t len = 0;
  uint8_t* data() { return ext ? ext : own.data(); }
  int64_t Size() const override { return len; }
  int Read(int64_t off, int size, RV** out, VM* vm) override;
  int ReadRange(int64_t off, int64_t count, std::vector<uint8_t>* out) override {  // memory.go:176-185
    if (off < 0 || wadd(off, count) > len) return XE_E_OOB;
    if (count < 0) throw GoPanic{XE_P_MAKESLICE};
    out->assign(data() + off, data() + off + count);
    return 0;
  }
  int Write(int64_t off, RV* v, int size) override {  // memory.go:187-210
    if (int e = boundsCheck(off, size, len)) return e;
    uint64_t x = uint64_t(v->Value());
    for (int b = 0; b < size; b++) data()[off + b] = uint8_t(x >> (8 * b));
    return 0;
  }
  void setBacking(std::vector<uint8_t>&& b) { ext = nullptr; own = std::move(b); len = int64_t(own.size()); }
  Memory* Clone(VM* vm) override;
};

// ---------------------------------------------------------------- maps
enum MapErr { ME_OK = 0, ME_KEY_NO_PTR = 1, ME_VAL_NO_PTR = 2, ME_OOM = 3, ME_NOT_IMPL = 4 };
constexpr int ME_GENERIC = 0x100 | XE_E_MAP_OP;  // a non-sentinel error: the helper aborts the VM
struct Map {
  xe_map_def def{};
  int index = 0;
  virtual ~Map() {}
  // return ME_* or (0x100 | memory error code) for a generic error that aborts the VM
  virtual int Lookup(VM* vm, RV* key, RV** out) = 0;
  // AbstractMap defaults (emulator/maps.go:61-82): "... not available on this map type"
  virtual int Update(VM*, RV*, RV*, RV**) { return ME_GENERIC; }
  virtual int Push(VM*, RV*, int64_t) { return ME_GENERIC; }
  virtual int Pop(VM*, RV**) { return ME_GENERIC; }
  virtual bool isHash() const { return false; }
};

struct VM {
  xe_settings settings{};
  RV* R[10] = {};
  FramePtr* R10 = nullptr;
  int64_t PC = 0;
  int PI = 0;
  int entry = 0;  // SetEntrypoint's index: the harness starts every packet there
  std::vector<ValueMemory> frames;
  struct Preserved { int64_t PC; RV* R[4]; };
  std::vector<Preserved> preserved;
  std::vector<std::vector<Inst>> programs;
  std::vector<Map*> maps;
  std::vector<std::unique_ptr<RV>> arena;
  std::vector<std::unique_ptr<Memory>> memArena;
  std::string lastError;
  uint64_t steps = 0;
  // VM.HelperFunctions (vm.go:23,35): entries changed from LinuxHelperFunctions (helper_functions.go:20-44)
  enum HelperEntry : uint8_t { H_BUILTIN = 0, H_HOST, H_NIL };
  HelperEntry helper[192] = {};
  xe_helper_fn helper_fn[192] = {};
  void* helper_user[192] = {};
  uint32_t packet = 0;  // the harness's packet index (passed to host helpers)
  // Step records of the traced packets (orc_trace_config)
  std::vector<uint32_t> trace_pk;
  uint32_t trace_max = 0;
  std::vector<std::vector<xe_trace_rec>> trace;

  template <class T, class... A> T* mk(A&&... a) {
    T* p = new T(std::forward<A>(a)...);
    arena.emplace_back(p);
    return p;
  }
  IMM* newIMM(int64_t v) { return mk<IMM>(v); }
};

int ByteMemory::Read(int64_t off, int size, RV** out, VM* vm) {  // memory.go:135-174
  if (int e = boundsCheck(off, size, len)) return e;
  uint64_t x = 0;
  for (int b = 0; b < size; b++) x |= uint64_t(data()[off + b]) << (8 * b);
  *out = vm->newIMM(int64_t(x));
  return 0;
}
Memory* ValueMemory::Clone(VM* vm) {  // memory.go:109-116
  auto* c = new ValueMemory(*this);
  vm->memArena.emplace_back(c);
  return c;
}
Memory* ByteMemory::Clone(VM* vm) {  // memory.go:212-219: copies the bytes
  auto* c = new ByteMemory();
  c->region = region; c->mapidx = mapidx;
  c->own.assign(data(), data() + len);
  c->len = len;
  vm->memArena.emplace_back(c);
  return c;
}

// RegisterValue.Copy (registers.go:186-188, 222-227, 283-292): FramePointer copies are writable.
static RV* copyRV(VM* vm, RV* r) {
  switch (KindOf(r)) {
    case XE_KIND_IMM: return vm->newIMM(r->Value());
    case XE_KIND_MEMPTR: { auto* p = static_cast<MemPtr*>(r); return vm->mk<MemPtr>(p->mem, p->off); }
    default: { auto* p = static_cast<FramePtr*>(r); return vm->mk<FramePtr>(p->mem, p->index, p->off, false); }
  }
}
// RegisterValue.Clone (registers.go:190-192, 229-240, 294-303): deep-copies the memory.
static RV* cloneRV(VM* vm, RV* r) {
  switch (KindOf(r)) {
    case XE_KIND_IMM: return vm->newIMM(r->Value());
    case XE_KIND_MEMPTR: { auto* p = static_cast<MemPtr*>(r); return vm->mk<MemPtr>(p->mem->Clone(vm), p->off); }
    default: { auto* p = static_cast<FramePtr*>(r); return vm->mk<FramePtr>(p->mem->Clone(vm), p->index, p->off, p->ro); }
  }
}
// RegisterValue.Assign (registers.go:194-197, 243-247, 305-313)
static int assignRV(RV* r, int64_t v) {
  switch (KindOf(r)) {
    case XE_KIND_IMM: static_cast<IMM*>(r)->v = v; return 0;
    case XE_KIND_MEMPTR: static_cast<MemPtr*>(r)->off = v; return 0;
    default: {
      auto* p = static_cast<FramePtr*>(r);
      if (p->ro) return XE_E_READONLY;
      p->off = v;
      return 0;
    }
  }
}
static bool isPointer(RV* r) { return r && r->kind() != XE_KIND_IMM; }  // PointerValue type assertion (nil: false)
static bool isMemPtr(RV* r) { return r && r->kind() == XE_KIND_MEMPTR; }  // *MemoryPtr type assertion

// PointerValue.Deref / ReadRange (registers.go:218-220, 273-281)
static int derefRV(VM* vm, RV* r, int64_t offset, int size, RV** out) {
  if (r->kind() == XE_KIND_MEMPTR) {
    auto* p = static_cast<MemPtr*>(r);
    return p->mem->Read(wadd(p->off, offset), size, out, vm);
  }
  auto* p = static_cast<FramePtr*>(r);
  return p->mem->Read(wadd(wadd(p->mem->Size(), p->off), offset), size, out, vm);
}
static int readRangeRV(RV* r, int64_t offset, int64_t count, std::vector<uint8_t>* out) {
  if (r->kind() == XE_KIND_MEMPTR) {
    auto* p = static_cast<MemPtr*>(r);
    return p->mem->ReadRange(wadd(p->off, offset), count, out);
  }
  auto* p = static_cast<FramePtr*>(r);
  return p->mem->ReadRange(wadd(wadd(p->mem->Size(), p->off), offset), count, out);
}

struct ArrayMap : Map {  // emulator/maps_array.go
  ByteMemory memory;
  int Lookup(VM* vm, RV* key, RV** out) override {  // maps_array.go:65-87
    if (!isPointer(key)) return ME_KEY_NO_PTR;
    RV* kr = nullptr;
    derefRV(vm, key, 0, 4, &kr);  // error not checked (`if !ok`, :72): nil .Value() panics
    if (!kr) throw GoPanic{XE_P_NIL_DEREF};
    int64_t kv = kr->Value();
    int64_t off = wmul(kv, int64_t(def.value_size));
    if (off >= memory.Size()) { *out = vm->newIMM(0); return 0; }
    *out = vm->mk<MemPtr>(&memory, off);
    return 0;
  }
  int Update(VM* vm, RV* key, RV* value, RV** out) override {  // maps_array.go:89-131
    if (!isMemPtr(value)) return ME_VAL_NO_PTR;
    if (!isMemPtr(key)) return ME_VAL_NO_PTR;
    RV* kvr = nullptr;
    if (int e = derefRV(vm, key, 0, 4, &kvr)) return 0x100 | e;
    int64_t kv = kvr->Value();
    if (kv >= memory.Size()) return ME_OOM;
    auto* vp = static_cast<MemPtr*>(value);
    for (int64_t i = 0; i < int64_t(def.value_size); i++) {
      RV* v = nullptr;
      if (int e = vp->mem->Read(i, 1, &v, vm)) return 0x100 | e;  // ignores vp->off
      if (int e = memory.Write(wadd(wmul(kv, def.value_size), i), v, 1)) return 0x100 | e;
    }
    *out = vm->newIMM(0);
    return 0;
  }
};

struct HashMap : Map {  // emulator/maps_hash.go; sha256(key) is unobservable, so key bytes index
  std::map<std::vector<uint8_t>, std::unique_ptr<ByteMemory>> values;
  bool isHash() const override { return true; }
  std::vector<uint8_t> keyBytes(RV* key) {  // :50-53: ReadRange error ignored -> nil key
    std::vector<uint8_t> k;
    if (readRangeRV(key, 0, def.key_size, &k) != 0) k.clear();
    return k;
  }
  int Lookup(VM* vm, RV* key, RV** out) override {  // maps_hash.go:44-63
    if (!isPointer(key)) return ME_KEY_NO_PTR;
    auto it = values.find(keyBytes(key));
    if (it == values.end()) { *out = vm->newIMM(0); return 0; }
    *out = vm->mk<MemPtr>(it->second.get(), 0);
    return 0;
  }
  int Update(VM* vm, RV* key, RV* value, RV** out) override {  // maps_hash.go:65-123
    if (!isPointer(key)) return ME_KEY_NO_PTR;
    std::vector<uint8_t> kb = keyBytes(key);
    auto it = values.find(kb);
    if (it == values.end() && values.size() + 1 > def.max_entries) return ME_OOM;
    if (!isPointer(value)) return ME_VAL_NO_PTR;
    std::vector<uint8_t> vb;
    if (readRangeRV(value, 0, def.value_size, &vb) != 0) vb.clear();  // nil backing on error
    if (it == values.end()) {
      auto m = std::make_unique<ByteMemory>();
      m->region = XE_REGION_HASHVAL; m->mapidx = index;
      it = values.emplace(kb, std::move(m)).first;
    }
    it->second->setBacking(std::move(vb));  // existing pointers see the new bytes
    *out = vm->newIMM(0);
    return 0;
  }
};

// HashMapLRU, emulator/maps_hash_lru.go. Entries keyed by key bytes (sha256 is unobservable; a
// ReadRange error gives the empty key, as `if !ok` ignores it, :76-79); UsageList holds keys, MRU first.
// The UsageList slice is kept as a linked list plus an index of its elements: the same sequence after every
// operation (keys are unique in it), with promote / delete in O(log n) instead of the slice's O(n) shifts,
// so the oracle can replay bench-sized batches.
struct LRUHashMap : Map {
  std::map<std::vector<uint8_t>, std::unique_ptr<ByteMemory>> values;
  std::list<std::vector<uint8_t>> usage;  // UsageList, index 0 first
  std::map<std::vector<uint8_t>, std::list<std::vector<uint8_t>>::iterator> upos;  // its elements
  std::vector<std::unique_ptr<ByteMemory>> evicted;  // evicted values stay valid for pointers still held
  void append(const std::vector<uint8_t>& key) {  // m.UsageList = append(m.UsageList, keyHash)
    usage.push_back(key);
    upos[key] = std::prev(usage.end());
  }
  bool isHash() const override { return true; }
  std::vector<uint8_t> keyBytes(RV* key) {
    std::vector<uint8_t> k;
    if (readRangeRV(key, 0, def.key_size, &k) != 0) k.clear();
    return k;
  }
  void promote(const std::vector<uint8_t>& key) {  // :51-68: not found or already first: nothing
    auto p = upos.find(key);
    if (p == upos.end() || p->second == usage.begin()) return;
    usage.splice(usage.begin(), usage, p->second);  // the keys above it move one down, it goes first
  }
  void erase(const std::vector<uint8_t>& key) {  // delete, :163-183
    auto p = upos.find(key);
    if (p == upos.end()) return;
    usage.erase(p->second);
    upos.erase(p);
    auto it = values.find(key);
    if (it != values.end()) { evicted.push_back(std::move(it->second)); values.erase(it); }
  }
  int Lookup(VM* vm, RV* key, RV** out) override {  // :70-91
    if (!isPointer(key)) return ME_KEY_NO_PTR;
    std::vector<uint8_t> kb = keyBytes(key);
    auto it = values.find(kb);
    if (it == values.end()) { *out = vm->newIMM(0); return 0; }
    promote(kb);
    *out = vm->mk<MemPtr>(it->second.get(), 0);
    return 0;
  }
  int Update(VM* vm, RV* key, RV* value, RV** out) override {  // :93-161
    if (!isPointer(key)) return ME_KEY_NO_PTR;
    std::vector<uint8_t> kb = keyBytes(key);
    auto it = values.find(kb);
    const bool found = it != values.end();
    if (!found && values.size() + 1 > def.max_entries) {
      if (usage.empty()) throw GoPanic{XE_P_INDEX};  // UsageList[len-1] of an empty list
      erase(std::vector<uint8_t>(usage.back()));      // evicted before the value is even checked
    }
    if (!isPointer(value)) return ME_VAL_NO_PTR;
    std::vector<uint8_t> vb;
    if (readRangeRV(value, 0, def.value_size, &vb) != 0) vb.clear();
    if (!found) {
      auto m = std::make_unique<ByteMemory>();
      m->region = XE_REGION_HASHVAL; m->mapidx = index;
      it = values.emplace(kb, std::move(m)).first;
      append(kb);
    }
    promote(kb);
    it->second->setBacking(std::move(vb));
    *out = vm->newIMM(0);
    return 0;
  }
};

// QueueMap / StackMap, emulator/maps_queue.go, emulator/maps_stack.go: an unbounded list of value
// memories (MaxEntries is not enforced). Elements stay alive after Pop (registers may hold them).
struct ListMap : Map {
  bool stack = false;
  std::vector<ByteMemory*> list;
  std::vector<std::unique_ptr<ByteMemory>> pool;
  ByteMemory* make(std::vector<uint8_t>&& b) {
    auto m = std::make_unique<ByteMemory>();
    m->region = XE_REGION_QUEUEVAL; m->mapidx = index;
    m->setBacking(std::move(b));
    pool.push_back(std::move(m));
    return pool.back().get();
  }
  int Lookup(VM* vm, RV* key, RV** out) override {  // maps_queue.go:39-58, maps_stack.go:38-58
    if (!isPointer(key)) return ME_KEY_NO_PTR;
    RV* kr = nullptr;
    derefRV(vm, key, 0, 4, &kr);  // error ignored (`if !ok`): nil keyVal.Value() panics
    if (!kr) throw GoPanic{XE_P_NIL_DEREF};
    const int64_t i = kr->Value();
    if (i < 0 || i >= int64_t(list.size())) return ME_OOM;
    *out = vm->mk<MemPtr>(stack ? list[list.size() - 1 - size_t(i)] : list[size_t(i)], 0);
    return 0;
  }
  int Push(VM*, RV* value, int64_t size) override {  // :60-77
    if (!isPointer(value)) return ME_VAL_NO_PTR;
    std::vector<uint8_t> vb;
    if (readRangeRV(value, 0, size, &vb) != 0) vb.clear();
    list.push_back(make(std::move(vb)));
    return 0;
  }
  int Pop(VM* vm, RV** out) override {  // maps_queue.go:79-91, maps_stack.go:79-90
    if (list.empty()) { *out = vm->newIMM(0); return 0; }
    ByteMemory* v = stack ? list.back() : list.front();
    if (stack) list.pop_back(); else list.erase(list.begin());
    *out = vm->mk<MemPtr>(v, 0);
    return 0;
  }
};

// PerfEventArray, emulator/maps_perf_event_array.go: an unbounded list of events; Lookup shares the
// event's bytes (:61-64), Update is not implemented (:67-77).
struct PerfMap : Map {
  std::vector<ByteMemory*> events;
  std::vector<std::unique_ptr<ByteMemory>> pool;
  int Lookup(VM* vm, RV* key, RV** out) override {  // :45-65
    if (!isPointer(key)) return ME_KEY_NO_PTR;
    RV* kr = nullptr;
    derefRV(vm, key, 0, 4, &kr);
    if (!kr) throw GoPanic{XE_P_NIL_DEREF};
    const int64_t kv = kr->Value();
    if (int64_t(int(kv)) >= int64_t(events.size())) { *out = vm->newIMM(0); return 0; }
    if (int(kv) < 0) throw GoPanic{XE_P_INDEX};
    *out = vm->mk<MemPtr>(events[size_t(int(kv))], 0);
    return 0;
  }
  int Update(VM*, RV*, RV*, RV**) override { return ME_NOT_IMPL; }
  int Push(VM*, RV* value, int64_t size) override {  // :101-115
    if (!isPointer(value)) return ME_KEY_NO_PTR;
    std::vector<uint8_t> vb;
    if (readRangeRV(value, 0, size, &vb) != 0) vb.clear();
    auto m = std::make_unique<ByteMemory>();
    m->region = XE_REGION_PERF; m->mapidx = index;
    m->setBacking(std::move(vb));
    pool.push_back(std::move(m));
    events.push_back(pool.back().get());
    return 0;
  }
};

// ---------------------------------------------------------------- registers (registers.go:62-149)
static int regGet(VM* vm, int r, RV** out) {
  if (r < 0 || r > 9) return XE_E_BAD_REG;
  *out = vm->R[r];
  return 0;
}
static int regCopy(VM* vm, int r, RV** out) {
  if (r == 10) { *out = copyRV(vm, vm->R10); return 0; }
  if (r < 0 || r > 9) return XE_E_BAD_REG;
  *out = copyRV(vm, vm->R[r]);
  return 0;
}
static int regAssign(VM* vm, int r, RV* v) {
  if (r < 0 || r > 9) return XE_E_ASSIGN_REG;
  vm->R[r] = v;
  return 0;
}

// ---------------------------------------------------------------- helpers (helper_functions.go)
static int helperErrno(int e) {  // helper_functions.go:57-67
  switch (e) { case ME_KEY_NO_PTR: case ME_VAL_NO_PTR: return -14; case ME_OOM: return -7; case ME_NOT_IMPL: return -1; }
  return 0;
}

// regToMap, helper_functions.go:109-130. Returns VM error code or 0; *m may be null (R0 = 0 set).
static int regToMap(VM* vm, RV* reg, Map** m) {
  int64_t idx = V(reg);
  if (reg->kind() == XE_KIND_MEMPTR) {
    RV* v = nullptr;
    if (int e = derefRV(vm, reg, 0, 4, &v)) return e;
    idx = v->Value();
  }
  if (idx < 1 || idx >= int64_t(vm->maps.size())) {
    vm->R[0] = vm->newIMM(0);
    *m = nullptr;
    return 0;
  }
  *m = vm->maps[idx];
  return 0;
}

// errno IMM for a map sentinel error, or the VM error (IN_HELPER-tagged) for any other
static int mapErr(VM* vm, int me, RV** r0) {
  if (me & 0x100) return (me & 0xff) | XE_E_IN_HELPER;
  *r0 = vm->newIMM(helperErrno(me));
  return 0;
}

// TailCall, helper_functions.go:133-210
static int tailCall(VM* vm) {
  const int64_t mapIdx = V(vm->R[2]);
  if (mapIdx < 1 || mapIdx >= int64_t(vm->maps.size())) { vm->R[0] = vm->newIMM(-14); return 0; }
  Map* m = vm->maps[size_t(mapIdx)];
  if (m->def.type != XE_MAP_PROG_ARRAY) { vm->R[0] = vm->newIMM(-14); return 0; }
  ValueMemory kmem;  // key: a ValueMemory of 4 slots all holding the R3 object itself
  kmem.mapping.assign(4, vm->R[3]);
  MemPtr key(&kmem, 0);
  RV* valReg = nullptr;
  if (int me = m->Lookup(vm, &key, &valReg)) {
    RV* r0 = nullptr;
    if (int e = mapErr(vm, me, &r0)) return e;
    vm->R[0] = r0;
    return 0;
  }
  if (!isPointer(valReg)) return XE_E_MAP_OP | XE_E_IN_HELPER;  // "lookup didn't return a pointer"
  RV* pv = nullptr;
  if (int e = derefRV(vm, valReg, 0, 4, &pv)) return e | XE_E_IN_HELPER;  // "deref value pointer"
  const int64_t progIdx = pv->Value();
  if (int64_t(vm->programs.size()) < progIdx) { vm->R[0] = vm->newIMM(-14); return 0; }  // off by one, :189
  if (progIdx == 0) return XE_E_NO_PROGRAM | XE_E_IN_HELPER;
  vm->PI = int(progIdx);
  vm->PC = -1;
  vm->R[0] = vm->newIMM(0);
  return 0;
}

static int callHelper(VM* vm, int64_t id) {  // returns 0 or VM error code (already IN_HELPER-tagged)
  if (id >= 0 && id < 192 && vm->helper[id] != VM::H_BUILTIN) {
    if (vm->helper[id] == VM::H_NIL) return -1;  // f == nil: "VM has no helper function" (inst_call_helper.go:26-28)
    // f(vm): a host function over R1..R5; an error aborts the run (inst_call_helper.go:30-33)
    int64_t a[5];
    uint8_t k[5];
    for (int r = 0; r < 5; r++) {
      a[r] = vm->R[r + 1] ? vm->R[r + 1]->Value() : 0;
      k[r] = uint8_t(vm->R[r + 1] ? vm->R[r + 1]->kind() : XE_KIND_NIL);
    }
    int64_t r0 = 0;
    if (vm->helper_fn[id](vm->helper_user[id], vm->packet, a, k, &r0)) return XE_E_HOST_HELPER | XE_E_IN_HELPER;
    vm->R[0] = vm->newIMM(r0);
    return 0;
  }
  switch (id) {
    case 1: case 2: {  // MapLookupElement :46-73 / MapUpdateElement :76-101
      Map* m = nullptr;
      if (int e = regToMap(vm, vm->R[1], &m)) return e | XE_E_IN_HELPER;
      if (!m) return 0;
      if (id == 2) V(vm->R[4]);  // BPFAttrMapElemFlags(R4.Value()) is evaluated first
      RV* val = nullptr;
      int me = id == 1 ? m->Lookup(vm, vm->R[2], &val) : m->Update(vm, vm->R[2], vm->R[3], &val);
      if (me && (me = mapErr(vm, me, &val))) return me;
      vm->R[0] = val;
      return 0;
    }
    case 3: return XE_E_NOT_IMPL | XE_E_IN_HELPER;  // MapDeleteElement :104-106
    case 12: return tailCall(vm);
    case 14: vm->R[0] = vm->newIMM((int64_t(1234) << 32) + 5678); return 0;  // :213-216
    case 25: {  // PerfEventOutput :219-252: R2 = map index (no deref), R4 = data, R5 = size
      const int64_t mapIdx = V(vm->R[2]);
      if (mapIdx < 1 || mapIdx >= int64_t(vm->maps.size())) { vm->R[0] = vm->newIMM(-14); return 0; }
      auto* pa = dynamic_cast<PerfMap*>(vm->maps[size_t(mapIdx)]);
      if (!pa) { vm->R[0] = vm->newIMM(-14); return 0; }
      RV* val = vm->newIMM(0);
      if (int me = pa->Push(vm, vm->R[4], V(vm->R[5])))
        if ((me = mapErr(vm, me, &val))) return me;
      vm->R[0] = val;
      return 0;
    }
    case 87: {  // MapPushElement :255-281 (size = ValueSize)
      Map* m = nullptr;
      if (int e = regToMap(vm, vm->R[1], &m)) return e | XE_E_IN_HELPER;
      if (!m) return 0;
      RV* val = vm->newIMM(0);
      if (int me = m->Push(vm, vm->R[2], int64_t(m->def.value_size)))
        if ((me = mapErr(vm, me, &val))) return me;
      vm->R[0] = val;
      return 0;
    }
    case 88: {  // MapPopElement :284-332
      Map* m = nullptr;
      if (int e = regToMap(vm, vm->R[1], &m)) return e | XE_E_IN_HELPER;
      if (!m) return 0;
      vm->R[0] = vm->newIMM(0);
      RV* val = nullptr;
      if (int me = m->Pop(vm, &val)) {
        RV* r0 = nullptr;
        if (int e = mapErr(vm, me, &r0)) return e;
        vm->R[0] = r0;
        return 0;
      }
      RV* r2 = vm->R[2];
      if (r2 && r2->kind() == XE_KIND_MEMPTR) {
        auto* p = static_cast<MemPtr*>(r2);
        if (int e = p->mem->Write(p->off, val, 8)) return e | XE_E_IN_HELPER;  // "write memory"
      } else if (r2 && r2->kind() == XE_KIND_FRAMEPTR) {
        auto* p = static_cast<FramePtr*>(r2);
        if (int e = p->mem->Write(wadd(p->mem->Size(), p->off), val, 8)) return e | XE_E_IN_HELPER;
      } else {
        vm->R[0] = vm->newIMM(-14);
      }
      return 0;
    }
    case 89: {  // MapPeekElement :335-374: R2 := Lookup(key 0) — nil when the lookup failed
      Map* m = nullptr;
      if (int e = regToMap(vm, vm->R[1], &m)) return e | XE_E_IN_HELPER;
      if (!m) return 0;
      IMM* k = vm->newIMM(0);
      ValueMemory kmem;
      kmem.mapping.assign(4, k);
      MemPtr key(&kmem, 0);
      RV* val = nullptr;
      RV* ret = vm->newIMM(0);
      if (int me = m->Lookup(vm, &key, &val)) {
        if ((me = mapErr(vm, me, &ret))) return me;
        val = nullptr;
      }
      vm->R[0] = ret;
      vm->R[2] = val;
      return 0;
    }
  }
  return -1;  // nil helper
}

// ---------------------------------------------------------------- execution (inst_*.go)
static inline int32_t i32(int64_t v) { return int32_t(uint32_t(uint64_t(v))); }
static int64_t goShl32(int64_t x, int64_t s) { if (s < 0) throw GoPanic{XE_P_NEG_SHIFT}; return s >= 32 ? 0 : int64_t(uint32_t(uint32_t(x) << s)); }
static int64_t goShl64(int64_t x, int64_t s) { if (s < 0) throw GoPanic{XE_P_NEG_SHIFT}; return s >= 64 ? 0 : int64_t(uint64_t(x) << s); }
static int64_t goShr32(int64_t x, int64_t s) { if (s < 0) throw GoPanic{XE_P_NEG_SHIFT}; return s >= 32 ? 0 : int64_t(uint32_t(x) >> s); }
static int64_t goShr64(int64_t x, int64_t s) { if (s < 0) throw GoPanic{XE_P_NEG_SHIFT}; return s >= 64 ? 0 : int64_t(uint64_t(x) >> s); }
static int64_t goSar32(int64_t x, int64_t s) { if (s < 0) throw GoPanic{XE_P_NEG_SHIFT}; int32_t v = i32(x); return int64_t(s >= 32 ? (v < 0 ? -1 : 0) : (v >> s)); }
static int64_t goSar64(int64_t x, int64_t s) { if (s < 0) throw GoPanic{XE_P_NEG_SHIFT}; return s >= 64 ? (x < 0 ? -1 : 0) : (x >> s); }
static int32_t goDiv32(int32_t a, int32_t b) { if (b == 0) throw GoPanic{XE_P_DIV0}; if (b == -1) return int32_t(0u - uint32_t(a)); return a / b; }
static int32_t goMod32(int32_t a, int32_t b) { if (b == 0) throw GoPanic{XE_P_DIV0}; if (b == -1) return 0; return a % b; }
static int64_t goDiv64(int64_t a, int64_t b) { if (b == 0) throw GoPanic{XE_P_DIV0}; if (b == -1) return int64_t(0ull - uint64_t(a)); return a / b; }
static int64_t goMod64(int64_t a, int64_t b) { if (b == 0) throw GoPanic{XE_P_DIV0}; if (b == -1) return 0; return a % b; }

// one ALU result for 32-bit (`a` = int32(dst) semantics inside) or 64-bit forms; s = imm or src value
static int64_t aluCompute(uint8_t op, bool wide, bool reg, int64_t d, int64_t s) {
  if (!wide) {
    int32_t a = i32(d), b = i32(s);  // imm is int32 already; reg forms use int32(sv)
    switch (op) {  // inst_{add,sub,mul,and,or,xor}.go:26,81 — int32 wrap then sign-extend
      case OP_ADD: return int64_t(int32_t(uint32_t(a) + uint32_t(b)));
      case OP_SUB: return int64_t(int32_t(uint32_t(a) - uint32_t(b)));
      case OP_MUL: return int64_t(int32_t(uint32_t(a) * uint32_t(b)));
      case OP_AND: return int64_t(a & b);
      case OP_OR: return int64_t(a | b);
      case OP_XOR: return int64_t(a ^ b);
      case OP_DIV: return int64_t(goDiv32(a, b));  // inst_div.go:33,96
      case OP_MOD: return int64_t(goMod32(a, b));  // inst_mod.go:33,96
      case OP_LSH: return goShl32(d, reg ? int64_t(b) : s);  // inst_lsh.go:26,81
      case OP_RSH: return goShr32(d, reg ? int64_t(b) : s);  // inst_rsh.go:26,81
      case OP_ARSH: return goSar32(d, reg ? int64_t(b) : s); // inst_arsh.go:26,81
    }
  } else {
    switch (op) {  // 64-bit forms :51,:111
      case OP_ADD: return wadd(d, s);
      case OP_SUB: return int64_t(uint64_t(d) - uint64_t(s));
      case OP_MUL: return wmul(d, s);
      case OP_AND: return d & s;
      case OP_OR: return d | s;
      case OP_XOR: return d ^ s;
      case OP_DIV: return goDiv64(d, s);
      case OP_MOD: return goMod64(d, s);
      case OP_LSH: return goShl64(d, s);
      case OP_RSH: return goShr64(d, s);
      case OP_ARSH: return goSar64(d, s);
    }
  }
  return 0;
}

static bool jmpCond(uint8_t op, bool wide, int64_t d, int64_t s) {  // conditions :24,:48,:77,:106
  if (!wide) {
    int32_t a = i32(d), b = i32(s);
    uint32_t ua = uint32_t(a), ub = uint32_t(b);
    switch (op) {
      case J_JEQ: return a == b; case J_JNE: return a != b;
      case J_JGT: return ua > ub; case J_JGE: return ua >= ub;
      case J_JSGT: return a > b; case J_JSGE: return a >= b;
      case J_JSLT: return a <= b;  // inst_jslt.go:24,77 (`<=`, as written)
      case J_JSLE: return a <= b;
    }
  } else {
    switch (op) {
      case J_JEQ: return d == s; case J_JNE: return d != s;
      case J_JGT: return uint64_t(d) > uint64_t(s); case J_JGE: return uint64_t(d) >= uint64_t(s);
      case J_JSGT: return d > s; case J_JSGE: return d >= s;
      case J_JSLT: return d <= s;  // inst_jslt.go:48,106
      case J_JSLE: return d <= s;
    }
  }
  return false;
}

// resolve a pointer register for LDX/ST/STX/atomic: inst_load.go:89-106, inst_store.go:28-43
static bool ptrTarget(RV* r, int16_t ioff, Memory** mem, int64_t* off) {
  if (KindOf(r) == XE_KIND_MEMPTR) {
    auto* p = static_cast<MemPtr*>(r);
    *off = wadd(p->off, ioff); *mem = p->mem; return true;
  }
  if (r->kind() == XE_KIND_FRAMEPTR) {
    auto* p = static_cast<FramePtr*>(r);
    *off = wadd(wadd(p->mem->Size(), p->off), ioff); *mem = p->mem; return true;
  }
  return false;
}

enum StepRes { SR_CONT, SR_EXIT };

// Instruction.Execute for one instruction; returns 0 / SR_EXIT marker via *exit, or a VM error code.
static int execute(VM* vm, const Inst& in, bool* exit) {
  switch (in.k) {
    case K_NOP: return 0;  // inst_nop.go:18-20
    case K_LDABS: case K_LDIND: return XE_E_NOT_IMPL;  // inst_load.go:131-148
    case K_ALU: {
      if (in.op == OP_MOV) {  // inst_mov.go
        if (!in.reg) return regAssign(vm, in.dst, vm->newIMM(int64_t(in.imm)));  // :22,:42
        RV* c = nullptr;
        if (int e = regCopy(vm, in.src, &c)) return e;  // :62,:88
        return regAssign(vm, in.dst, c);
      }
      RV* dr = nullptr;
      if (int e = regGet(vm, in.dst, &dr)) return e;
      int64_t dv = V(dr);
      int64_t sv = in.imm;
      if (in.reg) {
        RV* sr = nullptr;
        if (int e = regGet(vm, in.src, &sr)) return e;
        sv = V(sr);
        if (in.op == OP_ADD && isPointer(sr)) {  // inst_add.go:82-98,131-147 pointer edge case
          RV* scp = nullptr;
          regCopy(vm, in.src, &scp);
          int64_t v = in.wide ? wadd(dv, sv) : int64_t(int32_t(uint32_t(i32(dv)) + uint32_t(i32(sv))));
          if (int e = assignRV(scp, v)) return e;
          return regAssign(vm, in.dst, scp);
        }
      }
      if (in.op == OP_DIV || in.op == OP_MOD) {  // inst_div.go:29,58,92,126
        if (in.reg ? sv == 0 : in.imm == 0) return XE_E_DIV0;
      }
      int64_t v = aluCompute(in.op, in.wide, in.reg, dv, sv);
      return assignRV(dr, v);
    }
    case K_NEG: {  // inst_neg.go:26,51
      RV* dr = nullptr;
      if (int e = regGet(vm, in.dst, &dr)) return e;
      int64_t dv = V(dr);
      int64_t v = in.wide ? int64_t(0ull - uint64_t(dv)) : int64_t(int32_t(0u - uint32_t(i32(dv))));
      return assignRV(dr, v);
    }
    case K_END: {  // inst_end.go: to_le swaps, to_be truncates (inverted vs Linux)
      RV* dr = nullptr;
      if (int e = regGet(vm, in.dst, &dr)) return e;
      uint64_t rv = uint64_t(V(dr));
      uint64_t v;
      if (in.op == 0) {
        if (in.imm == 16) v = __builtin_bswap16(uint16_t(rv));
        else if (in.imm == 32) v = __builtin_bswap32(uint32_t(rv));
        else v = __builtin_bswap64(rv);
      } else {
        if (in.imm == 16) v = uint16_t(rv);
        else if (in.imm == 32) v = uint32_t(rv);
        else v = rv;
      }
      return assignRV(dr, int64_t(v));
    }
    case K_JA: vm->PC += in.off; return 0;  // inst_ja.go:18-21
    case K_JMP: {
      RV* dr = nullptr;
      if (int e = regGet(vm, in.dst, &dr)) return e;
      int64_t dv = V(dr);
      bool taken;
      if (!in.reg) {
        bool imm = dr->kind() == XE_KIND_IMM;  // isIMM, inst.go:249-252
        bool c = jmpCond(in.op, in.wide, dv, int64_t(in.imm));
        taken = in.op == J_JNE ? (!imm || c) : (imm && c);  // inst_jne.go:24,48
      } else {
        RV* sr = nullptr;
        if (int e = regGet(vm, in.src, &sr)) return e;
        int64_t sv = V(sr);
        bool same = dr->kind() == sr->kind();  // sameRVType, inst.go:254-258
        bool c = jmpCond(in.op, in.wide, dv, sv);
        taken = in.op == J_JNE ? (!same || c) : (same && c);  // inst_jne.go:77,106
      }
      if (taken) vm->PC += in.off;
      return 0;
    }
    case K_LDIMM64: {  // inst_load.go:21-71
      RV* dr = nullptr;
      if (int e = regGet(vm, in.dst, &dr)) return e;
      if (in.src == 1) return regAssign(vm, in.dst, vm->newIMM(int64_t(in.val1)));
      if (in.src == 2) {
        if (int64_t(in.val1) >= int64_t(vm->maps.size())) return XE_E_NO_MAP;
        Map* m = vm->maps[in.val1];
        if (!m) throw GoPanic{XE_P_NIL_MAP};
        ByteMemory tmp; tmp.own.assign(4, 0); tmp.len = 4;
        MemPtr key(&tmp, 0);
        RV* mv = nullptr;
        int me = m->Lookup(vm, &key, &mv);
        if (me) return XE_E_MAP_OP;
        if (mv->kind() != XE_KIND_MEMPTR) return XE_E_MAP_NOT_PTR;
        static_cast<MemPtr*>(mv)->off = int64_t(in.val2);
        return regAssign(vm, in.dst, mv);
      }
      return assignRV(dr, int64_t((uint64_t(in.val2) << 32) + uint64_t(in.val1)));
    }
    case K_LDX: {  // inst_load.go:84-118
      RV* sr = nullptr;
      if (int e = regCopy(vm, in.src, &sr)) return e;
      Memory* mem; int64_t off;
      if (!ptrTarget(sr, in.off, &mem, &off)) return XE_E_NONPTR_LOAD;
      RV* val = nullptr;
      if (int e = mem->Read(off, sizeBytes(in.size), &val, vm)) return e;
      return regAssign(vm, in.dst, val);
    }
    case K_ST: {  // inst_store.go:20-51
      RV* sv = vm->newIMM(int64_t(in.imm));
      RV* dr = nullptr;
      if (int e = regCopy(vm, in.dst, &dr)) return e;
      Memory* mem; int64_t off;
      if (!ptrTarget(dr, in.off, &mem, &off)) return XE_E_NONPTR_STORE;
      return mem->Write(off, sv, sizeBytes(in.size));
    }
    case K_STX: {  // inst_store.go:64-99
      RV* sr = nullptr;
      if (int e = regGet(vm, in.src, &sr)) return e;
      RV* sv = copyRV(vm, sr);
      RV* dr = nullptr;
      if (int e = regCopy(vm, in.dst, &dr)) return e;
      Memory* mem; int64_t off;
      if (!ptrTarget(dr, in.off, &mem, &off)) return XE_E_NONPTR_STORE;
      return mem->Write(off, sv, sizeBytes(in.size));
    }
    case K_ATOMIC: {  // AtomicAdd, inst_atomic.go:20-65 (Fetch ignored)
      RV* dr = nullptr;
      if (int e = regCopy(vm, in.dst, &dr)) return e;
      Memory* mem; int64_t off;
      if (!ptrTarget(dr, in.off, &mem, &off)) return XE_E_NONPTR_STORE;
      int sz = sizeBytes(in.size);
      RV* dv = nullptr;
      if (int e = mem->Read(off, sz, &dv, vm)) return e;
      RV* sr = nullptr;
      if (int e = regGet(vm, in.src, &sr)) return e;
      if (int e = assignRV(dv, wadd(V(dv), V(sr)))) return e;
      return mem->Write(off, dv, sz);
    }
    case K_CALL: {  // inst_call_helper.go:20-36
      int64_t fn = in.imm;
      if (fn >= 192) return XE_E_NO_HELPER;
      if (fn < 0) throw GoPanic{XE_P_INDEX};
      int e = callHelper(vm, fn);
      return e < 0 ? XE_E_NO_HELPER : e;
    }
    case K_CALLX: {  // inst_call_helper.go:49-71; Register(imm) truncates to uint8
      RV* fr = nullptr;
      if (int e = regGet(vm, uint8_t(in.imm), &fr)) return e;
      int64_t fn = V(fr);
      if (fn >= 192) return XE_E_NO_HELPER;
      if (fn < 0) throw GoPanic{XE_P_INDEX};
      int e = callHelper(vm, fn);
      return e < 0 ? XE_E_NO_HELPER : e;
    }
    case K_CALLBPF: {  // inst_call_bpf.go:18-44
      VM::Preserved p;
      p.PC = vm->PC;
      for (int r = 0; r < 4; r++) p.R[r] = cloneRV(vm, vm->R[6 + r]);  // Registers.Clone
      for (int r = 0; r <= 5; r++) cloneRV(vm, vm->R[r]);  // (clones of R0-R5, R10 are discarded)
      int idx = vm->R10->index + 1;
      if (idx >= int(vm->frames.size())) throw GoPanic{XE_P_INDEX};
      vm->preserved.push_back(p);
      vm->R10 = vm->mk<FramePtr>(&vm->frames[idx], idx, 0, true);
      std::fill(vm->frames[idx].mapping.begin(), vm->frames[idx].mapping.end(), nullptr);
      vm->PC += in.imm;
      return 0;
    }
    case K_EXIT: {  // inst_exit.go:22-48
      if (vm->preserved.empty()) { *exit = true; return 0; }
      VM::Preserved p = vm->preserved.back();
      vm->preserved.pop_back();
      vm->PC = p.PC;
      for (int r = 0; r < 4; r++) vm->R[6 + r] = p.R[r];
      int idx = vm->R10->index - 1;
      if (idx < 0) throw GoPanic{XE_P_INDEX};
      vm->R10 = vm->mk<FramePtr>(&vm->frames[idx], idx, 0, true);
      return 0;
    }
  }
  return 0;
}

// Reset, emulator/vm.go:211-246 (+ harness: PreservedRegisters = nil)
static void reset(VM* vm) {
  vm->arena.clear();
  vm->memArena.clear();
  vm->PC = 0;
  for (int r = 0; r < 10; r++) vm->R[r] = vm->newIMM(0);
  for (auto& f : vm->frames) std::fill(f.mapping.begin(), f.mapping.end(), nullptr);
  vm->R10 = vm->mk<FramePtr>(&vm->frames[0], 0, 0, true);
  vm->preserved.clear();
  vm->steps = 0;
}

static void regionOf(RV* r, uint8_t* region, uint8_t* map) {
  if (!r || r->kind() == XE_KIND_IMM) { *region = 0xff; *map = 0; return; }
  Memory* m = r->kind() == XE_KIND_MEMPTR ? static_cast<MemPtr*>(r)->mem : static_cast<FramePtr*>(r)->mem;
  *region = uint8_t(m->region); *map = uint8_t(m->mapidx);
}

}  // namespace orc

using namespace orc;

struct orc_vm { VM vm; };

extern "C" {

int orc_create(const xe_settings* s, orc_vm** out) {
  auto* o = new orc_vm();
  VM& vm = o->vm;
  if (s) vm.settings = *s;
  if (vm.settings.stack_frame_size <= 0) vm.settings.stack_frame_size = 256;
  if (vm.settings.max_stack_frames <= 0) vm.settings.max_stack_frames = 8;
  if (!vm.settings.max_steps) vm.settings.max_steps = 1u << 20;
  vm.frames.resize(vm.settings.max_stack_frames);
  for (auto& f : vm.frames) { f.mapping.assign(vm.settings.stack_frame_size, nullptr); f.region = XE_REGION_STACK; }
  vm.programs.emplace_back();  // index 0 invalid (vm.go:36-38)
  vm.maps.push_back(nullptr);  // index 0 invalid (vm.go:39-41)
  *out = o;
  return XE_OK;
}

void orc_destroy(orc_vm* o) {
  if (!o) return;
  for (Map* m : o->vm.maps) delete m;
  delete o;
}

const char* orc_last_error(const orc_vm* o) { return o ? o->vm.lastError.c_str() : ""; }

int orc_add_raw_program(orc_vm* o, const uint64_t* insns, uint32_t n, int32_t* idx) {
  std::vector<Inst> prog;
  std::string err;
  if (!decode(insns, n, prog, err)) { o->vm.lastError = "decode: " + err; return XE_ERR_DECODE; }
  if (!translate(prog, err)) { o->vm.lastError = "add program: translate: " + err; return XE_ERR_TRANSLATE; }
  o->vm.programs.push_back(std::move(prog));
  if (idx) *idx = int32_t(o->vm.programs.size() - 1);
  return XE_OK;
}

int orc_set_entrypoint(orc_vm* o, int32_t idx) {  // vm.go:100-108
  if (idx < 1 || int(o->vm.programs.size()) <= idx) { o->vm.lastError = "program index out of bounds"; return XE_ERR_INVAL; }
  o->vm.PI = idx;
  o->vm.entry = idx;
  return XE_OK;
}

int orc_add_map(orc_vm* o, const xe_map_def* def, const void* init, size_t init_len, int32_t* idx) {
  Map* m = nullptr;
  int index = int(o->vm.maps.size());
  switch (def->type) {  // AbstractMapToVM, maps.go:92-155
    case XE_MAP_HASH: case XE_MAP_PERCPU_HASH: case XE_MAP_HASH_OF_MAPS:
      m = new HashMap(); break;
    case XE_MAP_ARRAY: case XE_MAP_PERCPU_ARRAY: case XE_MAP_PROG_ARRAY: case XE_MAP_ARRAY_OF_MAPS: {
      auto* a = new ArrayMap();  // ArrayMap.Init, maps_array.go:19-44
      a->memory.own.assign(size_t(def->value_size) * def->max_entries, 0);
      a->memory.len = int64_t(a->memory.own.size());
      a->memory.region = XE_REGION_ARRAY; a->memory.mapidx = index;
      if (init && (def->type == XE_MAP_ARRAY || def->type == XE_MAP_PERCPU_ARRAY))
        memcpy(a->memory.own.data(), init, std::min(init_len, a->memory.own.size()));
      m = a;
      break;
    }
    case XE_MAP_LRU_HASH: case XE_MAP_LRU_PERCPU_HASH:
      m = new LRUHashMap(); break;
    case XE_MAP_QUEUE: case XE_MAP_STACK: {
      auto* l = new ListMap();
      l->stack = def->type == XE_MAP_STACK;
      m = l;
      break;
    }
    case XE_MAP_PERF_EVENT_ARRAY:
      m = new PerfMap(); break;
    default:
      o->vm.lastError = "map type not implemented";
      return XE_ERR_MAPTYPE;
  }
  m->def = *def;
  m->index = index;
  o->vm.maps.push_back(m);
  if (idx) *idx = index;
  return XE_OK;
}

static Map* getMap(orc_vm* o, int32_t i) {
  if (i < 1 || i >= int32_t(o->vm.maps.size())) return nullptr;
  return o->vm.maps[i];
}

static std::vector<uint8_t> keyvec(const Map* m, const void* key) {
  return std::vector<uint8_t>((const uint8_t*)key, (const uint8_t*)key + m->def.key_size);
}
static void copyOut(void* dst, const ByteMemory* b, size_t n) {  // value bytes, zero-filled past the backing
  memset(dst, 0, n);
  memcpy(dst, b->own.data(), std::min<size_t>(size_t(b->len), n));
}

// Userspace Map.Lookup: LRU lookups promote the key (maps_hash_lru.go:70-91)
int orc_map_lookup(orc_vm* o, int32_t mi, const void* key, void* value) {
  Map* m = getMap(o, mi);
  if (!m) return XE_ERR_INVAL;
  if (auto* h = dynamic_cast<HashMap*>(m)) {
    auto it = h->values.find(keyvec(m, key));
    if (it == h->values.end()) return 0;
    copyOut(value, it->second.get(), m->def.value_size);
    return 1;
  }
  if (auto* l = dynamic_cast<LRUHashMap*>(m)) {
    auto k = keyvec(m, key);
    auto it = l->values.find(k);
    if (it == l->values.end()) return 0;
    l->promote(k);
    copyOut(value, it->second.get(), m->def.value_size);
    return 1;
  }
  auto* a = dynamic_cast<ArrayMap*>(m);
  if (!a) return XE_ERR_INVAL;
  uint32_t kv; memcpy(&kv, key, 4);
  if (kv >= m->def.max_entries) return 0;
  memcpy(value, a->memory.own.data() + size_t(kv) * m->def.value_size, m->def.value_size);
  return 1;
}

// Userspace Map.Update with key/value bytes (flags ignored, as every emulator map does)
int orc_map_update(orc_vm* o, int32_t mi, const void* key, const void* value) {
  Map* m = getMap(o, mi);
  if (!m) return XE_ERR_INVAL;
  if (auto* h = dynamic_cast<HashMap*>(m)) {
    auto k = keyvec(m, key);
    auto it = h->values.find(k);
    if (it == h->values.end()) {
      if (h->values.size() + 1 > m->def.max_entries) return XE_ERR_NOMEM;
      auto bm = std::make_unique<ByteMemory>();
      bm->region = XE_REGION_HASHVAL; bm->mapidx = mi;
      it = h->values.emplace(k, std::move(bm)).first;
    }
    it->second->setBacking(std::vector<uint8_t>((const uint8_t*)value, (const uint8_t*)value + m->def.value_size));
    return XE_OK;
  }
  if (auto* l = dynamic_cast<LRUHashMap*>(m)) {  // maps_hash_lru.go:93-161 with byte-backed key/value
    auto k = keyvec(m, key);
    auto it = l->values.find(k);
    if (it == l->values.end()) {
      if (l->values.size() + 1 > m->def.max_entries) {
        if (l->usage.empty()) return XE_ERR_NOMEM;
        l->erase(std::vector<uint8_t>(l->usage.back()));
      }
      auto bm = std::make_unique<ByteMemory>();
      bm->region = XE_REGION_HASHVAL; bm->mapidx = mi;
      it = l->values.emplace(k, std::move(bm)).first;
      l->append(k);
    }
    l->promote(k);
    it->second->setBacking(std::vector<uint8_t>((const uint8_t*)value, (const uint8_t*)value + m->def.value_size));
    return XE_OK;
  }
  auto* a = dynamic_cast<ArrayMap*>(m);
  if (!a) return XE_ERR_INVAL;
  uint32_t kv; memcpy(&kv, key, 4);
  if (kv >= m->def.max_entries) return XE_ERR_INVAL;
  memcpy(a->memory.own.data() + size_t(kv) * m->def.value_size, value, m->def.value_size);
  return XE_OK;
}

int orc_map_update_batch(orc_vm* o, int32_t mi, const void* keys, const void* values, uint64_t count) {
  Map* m = getMap(o, mi);
  if (!m) return XE_ERR_INVAL;
  const size_t ks = dynamic_cast<ArrayMap*>(m) ? 4 : m->def.key_size, vs = m->def.value_size;
  for (uint64_t i = 0; i < count; i++)
    if (int rc = orc_map_update(o, mi, (const uint8_t*)keys + i * ks, (const uint8_t*)values + i * vs)) return rc;
  return XE_OK;
}

int orc_map_delete(orc_vm* o, int32_t mi, const void* key) {
  Map* m = getMap(o, mi);
  if (!m) return XE_ERR_INVAL;
  if (auto* h = dynamic_cast<HashMap*>(m)) { h->values.erase(keyvec(m, key)); return XE_OK; }
  if (auto* l = dynamic_cast<LRUHashMap*>(m)) { l->erase(keyvec(m, key)); return XE_OK; }
  return XE_ERR_INVAL;
}

// QueueMap/StackMap.Push from userspace: one value_size element
int orc_map_push(orc_vm* o, int32_t mi, const void* value) {
  Map* m = getMap(o, mi);
  auto* l = dynamic_cast<ListMap*>(m);
  if (!l) return XE_ERR_INVAL;
  l->list.push_back(l->make(std::vector<uint8_t>((const uint8_t*)value, (const uint8_t*)value + m->def.value_size)));
  return XE_OK;
}

int orc_map_count(orc_vm* o, int32_t mi, uint64_t* count) {
  Map* m = getMap(o, mi);
  if (!m) return XE_ERR_INVAL;
  if (auto* h = dynamic_cast<HashMap*>(m)) *count = h->values.size();
  else if (auto* l = dynamic_cast<LRUHashMap*>(m)) *count = l->values.size();
  else if (auto* q = dynamic_cast<ListMap*>(m)) *count = q->list.size();
  else if (auto* p = dynamic_cast<PerfMap*>(m)) *count = p->events.size();
  else *count = m->def.max_entries;
  return XE_OK;
}

// MA6: ARRAY = raw bytes; HASH / LRU_HASH = (key, value) sorted by key bytes. A nil-backed value
// (Update whose value ReadRange failed, maps_hash.go:108-115) dumps as zeros; its key as stored.
int orc_map_dump(orc_vm* o, int32_t mi, void* keys_or_raw, void* values, uint64_t cap, uint64_t* count) {
  Map* m = getMap(o, mi);
  if (!m) return XE_ERR_INVAL;
  if (auto* a = dynamic_cast<ArrayMap*>(m)) {
    if (count) *count = m->def.max_entries;
    if (keys_or_raw && cap >= m->def.max_entries) memcpy(keys_or_raw, a->memory.own.data(), a->memory.own.size());
    return XE_OK;
  }
  const std::map<std::vector<uint8_t>, std::unique_ptr<ByteMemory>>* vals = nullptr;
  if (auto* h = dynamic_cast<HashMap*>(m)) vals = &h->values;
  else if (auto* l = dynamic_cast<LRUHashMap*>(m)) vals = &l->values;
  if (!vals) {  // list maps: values in list order (use orc_map_dump_list for the lengths)
    uint64_t n = 0;
    orc_map_count(o, mi, &n);
    if (count) *count = n;
    return XE_OK;
  }
  if (count) *count = vals->size();
  if (!keys_or_raw && !values) return XE_OK;
  if (cap < vals->size()) return XE_ERR_INVAL;
  size_t i = 0;
  for (auto& kv : *vals) {  // std::map iterates in lexicographic key order
    if (keys_or_raw) {
      uint8_t* kd = (uint8_t*)keys_or_raw + i * m->def.key_size;
      memset(kd, 0, m->def.key_size);
      memcpy(kd, kv.first.data(), std::min<size_t>(kv.first.size(), m->def.key_size));
    }
    if (values) copyOut((uint8_t*)values + i * m->def.value_size, kv.second.get(), m->def.value_size);
    i++;
  }
  return XE_OK;
}

// QUEUE / STACK / PERF_EVENT_ARRAY: records in list order (Values / Events slice order)
int orc_map_dump_list(orc_vm* o, int32_t mi, void* data, uint64_t data_cap, uint32_t* lens, uint64_t cap,
                      uint64_t* count, uint64_t* bytes) {
  Map* m = getMap(o, mi);
  const std::vector<ByteMemory*>* list = nullptr;
  if (auto* q = dynamic_cast<ListMap*>(m)) list = &q->list;
  else if (auto* p = dynamic_cast<PerfMap*>(m)) list = &p->events;
  if (!list) return XE_ERR_INVAL;
  uint64_t total = 0;
  for (auto* b : *list) total += uint64_t(b->len);
  if (count) *count = list->size();
  if (bytes) *bytes = total;
  if (!data && !lens) return XE_OK;
  if (cap < list->size() || (data && data_cap < total)) return XE_ERR_INVAL;
  uint64_t off = 0;
  for (size_t i = 0; i < list->size(); i++) {
    const ByteMemory* b = (*list)[i];
    if (lens) lens[i] = uint32_t(b->len);
    if (data && b->len) memcpy((uint8_t*)data + off, b->own.data(), size_t(b->len));
    off += uint64_t(b->len);
  }
  return XE_OK;
}

// LRU_HASH UsageList, most recently used first
int orc_map_lru_order(orc_vm* o, int32_t mi, void* keys, uint64_t cap, uint64_t* count) {
  auto* l = dynamic_cast<LRUHashMap*>(getMap(o, mi));
  if (!l) return XE_ERR_INVAL;
  if (count) *count = l->usage.size();
  if (!keys) return XE_OK;
  if (cap < l->usage.size()) return XE_ERR_INVAL;
  size_t i = 0;
  for (const auto& k : l->usage) {
    uint8_t* kd = (uint8_t*)keys + i++ * l->def.key_size;
    memset(kd, 0, l->def.key_size);
    memcpy(kd, k.data(), std::min<size_t>(k.size(), l->def.key_size));
  }
  return XE_OK;
}

// What VM.String prints after a Step (emulator/vm.go:248-270): PC, PI, SF, R0..R10
static xe_trace_rec traceRec(VM& vm, uint32_t packet, uint32_t step, int64_t pc) {
  xe_trace_rec r{};
  r.packet = packet;
  r.step = step;
  r.pc = int32_t(pc);
  r.pi = vm.PI;
  r.sf = uint32_t(vm.preserved.size());
  for (int k = 0; k < 10; k++) {
    r.val[k] = vm.R[k] ? vm.R[k]->Value() : 0;
    r.kind[k] = uint8_t(vm.R[k] ? vm.R[k]->kind() : XE_KIND_NIL);
  }
  r.val[10] = vm.R10 ? vm.R10->Value() : 0;
  r.kind[10] = XE_KIND_FRAMEPTR;
  return r;
}

int orc_trace_config(orc_vm* o, const uint32_t* packets, uint32_t npk, uint32_t max_steps) {
  if (!o || (npk && !packets) || npk > XE_TRACE_MAX_PACKETS || max_steps > XE_TRACE_MAX_STEPS || (npk && !max_steps))
    return XE_ERR_INVAL;
  VM& vm = o->vm;
  vm.trace_pk.assign(packets, packets + npk);
  std::sort(vm.trace_pk.begin(), vm.trace_pk.end());
  vm.trace_pk.erase(std::unique(vm.trace_pk.begin(), vm.trace_pk.end()), vm.trace_pk.end());
  vm.trace_max = npk ? max_steps : 0;
  vm.trace.assign(vm.trace_pk.size(), {});
  return XE_OK;
}

int orc_trace_read(orc_vm* o, uint32_t packet, xe_trace_rec* out, uint32_t cap, uint32_t* nsteps) {
  if (!o || !nsteps) return XE_ERR_INVAL;
  VM& vm = o->vm;
  auto it = std::lower_bound(vm.trace_pk.begin(), vm.trace_pk.end(), packet);
  if (it == vm.trace_pk.end() || *it != packet) return XE_ERR_INVAL;
  const auto& t = vm.trace[size_t(it - vm.trace_pk.begin())];
  *nsteps = uint32_t(t.size());
  if (out) memcpy(out, t.data(), std::min<size_t>(cap, t.size()) * sizeof(xe_trace_rec));
  return XE_OK;
}

int orc_set_helper(orc_vm* o, uint32_t id, xe_helper_fn fn, void* user) {
  if (!o || id >= 192) return XE_ERR_INVAL;
  o->vm.helper[id] = fn ? VM::H_HOST : VM::H_NIL;
  o->vm.helper_fn[id] = fn;
  o->vm.helper_user[id] = user;
  return XE_OK;
}

int orc_reset_helper(orc_vm* o, uint32_t id) {
  if (!o || id >= 192) return XE_ERR_INVAL;
  o->vm.helper[id] = VM::H_BUILTIN;
  return XE_OK;
}

// Per-packet harness: Reset; ctx ValueMemory of 24 slots holding six objects
// (xdp_md: data, data_end, data_meta, ingress_ifindex, rx_queue_index, egress_ifindex);
// R1 = &MemoryPtr{ctx}; Run under recover(); record status/R0.
int orc_run_batch(orc_vm* o, uint8_t* umem, uint64_t umem_len, const xe_desc* desc, uint32_t n,
                  xe_result* results, uint32_t* verdicts, xe_regs* regs, xe_batch_stats* stats) {
  VM& vm = o->vm;
  if (stats) memset(stats, 0, sizeof *stats);
  for (auto& t : vm.trace) t.clear();
  for (uint32_t p = 0; p < n; p++) {
    reset(&vm);
    vm.packet = p;
    std::vector<xe_trace_rec>* tr = nullptr;  // this packet's Step records (orc_trace_config)
    {
      auto it = std::lower_bound(vm.trace_pk.begin(), vm.trace_pk.end(), p);
      if (it != vm.trace_pk.end() && *it == p) tr = &vm.trace[size_t(it - vm.trace_pk.begin())];
    }
    // Reset keeps PI (emulator/vm.go:211-246); a tail call in the previous packet would otherwise
    // start this one in another program: the harness re-applies SetEntrypoint per packet
    vm.PI = vm.entry;
    ByteMemory pkt;
    pkt.region = XE_REGION_PACKET;
    uint64_t a = desc[p].addr, l = desc[p].len;
    if (a > umem_len || l > umem_len - a) l = 0;
    pkt.ext = umem + a;
    pkt.len = int64_t(l);
    ValueMemory ctx;
    ctx.region = XE_REGION_CTX;
    ctx.mapping.assign(24, nullptr);
    RV* objs[6] = {vm.mk<MemPtr>(&pkt, 0), vm.mk<MemPtr>(&pkt, int64_t(l)), vm.mk<MemPtr>(&pkt, 0),
                   vm.newIMM(vm.settings.ingress_ifindex), vm.newIMM(vm.settings.rx_queue_index),
                   vm.newIMM(0)};
    for (int s = 0; s < 24; s++) ctx.mapping[s] = objs[s / 4];
    vm.R[1] = vm.mk<MemPtr>(&ctx, 0);

    xe_result res{};
    res.status = XE_ST_OK;
    try {
      for (;;) {  // RunContext, vm.go:117-134
        if (vm.steps >= vm.settings.max_steps) { res.status = XE_ST_BUDGET; res.pc = uint32_t(vm.PC); break; }
        // Step, vm.go:137-173
        if (vm.PI < 1 || vm.PI >= int(vm.programs.size())) {
          res.status = XE_ST_VMERR; res.code = XE_E_NO_PROGRAM; res.pc = uint32_t(vm.PC);
          break;
        }
        const auto& prog = vm.programs[vm.PI];
        if (vm.PC < 0 || vm.PC >= int64_t(prog.size())) throw GoPanic{XE_P_INDEX};  // program[PC]
        int64_t pc = vm.PC;
        vm.steps++;
        bool exit = false;
        int e = execute(&vm, prog[pc], &exit);
        res.pc = uint32_t(pc);
        if (e) { res.status = XE_ST_VMERR; res.code = uint16_t(e); break; }
        if (tr && tr->size() < vm.trace_max) tr->push_back(traceRec(vm, p, uint32_t(tr->size()), pc));
        if (exit) break;
        if (int64_t(prog.size()) <= vm.PC + 1) {  // vm.go:162-167
          vm.PC = pc;
          res.status = XE_ST_VMERR; res.code = XE_E_BAD_PC;
          break;
        }
        vm.PC++;
      }
    } catch (GoPanic& gp) {
      res.status = XE_ST_PANIC; res.code = uint16_t(gp.code); res.pc = uint32_t(vm.PC);
    } catch (Unsupported&) {
      res.status = XE_ST_UNSUPPORTED; res.pc = uint32_t(vm.PC);
    }
    res.r0_kind = uint8_t(vm.R[0] ? vm.R[0]->kind() : XE_KIND_NIL);
    res.r0 = vm.R[0] ? vm.R[0]->Value() : 0;
    if (results) results[p] = res;
    if (verdicts) verdicts[p] = uint32_t(uint64_t(res.r0));
    if (regs) {
      xe_regs& rg = regs[p];
      memset(&rg, 0, sizeof rg);
      for (int r = 0; r < 10; r++) {
        rg.val[r] = vm.R[r] ? vm.R[r]->Value() : 0;
        rg.kind[r] = uint8_t(vm.R[r] ? vm.R[r]->kind() : XE_KIND_NIL);
        regionOf(vm.R[r], &rg.region[r], &rg.map[r]);
      }
      rg.steps = uint32_t(vm.steps);
    }
    if (stats) { stats->packets++; stats->steps += vm.steps; stats->status_count[res.status & 7]++; }
  }
  // drop references to this batch's packet/ctx memories
  reset(&vm);
  if (stats) stats->mode_used = XE_MODE_SEQUENTIAL;
  return XE_OK;
}

int orc_decode_text(const uint64_t* insns, uint32_t n, char* buf, size_t buflen) {
  std::vector<Inst> prog;
  std::string err, out;
  if (!decode(insns, n, prog, err)) return XE_ERR_DECODE;
  for (auto& i : prog) out += goString(i) + "\n";
  if (buf && buflen) {
    size_t c = std::min(buflen - 1, out.size());
    memcpy(buf, out.data(), c);
    buf[c] = 0;
  }
  return XE_OK;
}

int orc_decode_names(const uint64_t* insns, uint32_t n, char* buf, size_t buflen) {
  std::vector<Inst> prog;
  std::string err, out;
  int rc = XE_OK;
  if (!decode(insns, n, prog, err)) rc = XE_ERR_DECODE;
  else {
    for (auto& i : prog) out += typeName(i) + "\n";
    if (!translate(prog, err)) rc = XE_ERR_TRANSLATE;
  }
  if (buf && buflen) {
    size_t c = std::min(buflen - 1, out.size());
    memcpy(buf, out.data(), c);
    buf[c] = 0;
  }
  return rc;
}

}  // extern "C"
