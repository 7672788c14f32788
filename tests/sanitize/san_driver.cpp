// san_driver.cpp — TEST INFRASTRUCTURE (SURVEY §5 "race detection / sanitizers"): runs a case file
// (tests/sanitize/cases.py) through two emulator libraries with the include/xdpemu.h ABI — the oracle
// (orc_ prefix) and the host simulation of the device logic (xe_ prefix), both built with
// -fsanitize=address,undefined — and compares every observable bit for bit: call return codes,
// per-packet results, R0-R9 records, verdicts, packet bytes written, final map contents (ARRAY image,
// HASH entries, LRU UsageList, QUEUE / STACK / PERF records). A sanitizer report aborts the process.
//
//   san_driver <oracle.so> <hostsim.so> <cases.bin>
#include <dlfcn.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/xdpemu.h"

namespace {

struct Api {
  void* h = nullptr;
  std::string pre;
  int (*create)(const xe_settings*, void**);
  void (*destroy)(void*);
  int (*default_settings)(xe_settings*);
  int (*add_raw_program)(void*, const uint64_t*, uint32_t, int32_t*);
  int (*set_entrypoint)(void*, int32_t);
  int (*add_map)(void*, const xe_map_def*, const void*, size_t, int32_t*);
  int (*map_update)(void*, int32_t, const void*, const void*);
  int (*map_push)(void*, int32_t, const void*);
  int (*map_dump)(void*, int32_t, void*, void*, uint64_t, uint64_t*);
  int (*map_dump_list)(void*, int32_t, void*, uint64_t, uint32_t*, uint64_t, uint64_t*, uint64_t*);
  int (*map_lru_order)(void*, int32_t, void*, uint64_t, uint64_t*);
  int (*run)(void*, uint8_t*, uint64_t, const xe_desc*, uint32_t, xe_result*, uint32_t*, xe_regs*, xe_batch_stats*);

  template <class F>
  void get(F& f, const char* name, bool required = true) {
    f = reinterpret_cast<F>(dlsym(h, (pre + name).c_str()));
    if (!f && required) { fprintf(stderr, "missing symbol %s%s\n", pre.c_str(), name); exit(3); }
  }
  Api(const char* path, const char* prefix) : pre(prefix) {
    h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!h) { fprintf(stderr, "dlopen %s: %s\n", path, dlerror()); exit(3); }
    get(create, "create"); get(destroy, "destroy"); get(add_raw_program, "add_raw_program");
    get(set_entrypoint, "set_entrypoint"); get(add_map, "add_map"); get(map_update, "map_update");
    get(map_push, "map_push"); get(map_dump, "map_dump"); get(map_dump_list, "map_dump_list");
    get(map_lru_order, "map_lru_order");
    get(default_settings, "default_settings", false);
    get(run, "run_batch_host", false);
    if (!run) get(run, "run_batch");
  }
};

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  template <class T>
  T get() {
    T v;
    if (p + sizeof(T) > end) { fprintf(stderr, "truncated case file\n"); exit(3); }
    memcpy(&v, p, sizeof(T));
    p += sizeof(T);
    return v;
  }
  std::vector<uint8_t> bytes(size_t n) {
    if (p + n > end) { fprintf(stderr, "truncated case file\n"); exit(3); }
    std::vector<uint8_t> v(p, p + n);
    p += n;
    return v;
  }
};

struct Entry { bool push; std::vector<uint8_t> key, val; };
struct Map { xe_map_def def; std::vector<uint8_t> init; std::vector<Entry> ents; };
struct Case {
  std::string name;
  uint64_t max_steps;
  uint32_t mode;
  std::vector<std::vector<uint64_t>> progs;
  std::vector<Map> maps;
  std::vector<uint8_t> umem;
  std::vector<xe_desc> descs;
};

// everything a run leaves observable, serialised; setup failures are part of it (their code)
std::vector<std::pair<size_t, std::string>> g_sections;  // (start offset, what) of the last run_case

std::vector<uint8_t> run_case(Api& A, const Case& c) {
  std::vector<uint8_t> out;
  g_sections.clear();
  auto sec = [&](const std::string& what) { g_sections.emplace_back(out.size(), what); };
  auto put = [&](const void* p, size_t n) { out.insert(out.end(), (const uint8_t*)p, (const uint8_t*)p + n); };
  auto put32 = [&](int32_t v) { put(&v, 4); };
  xe_settings s;
  memset(&s, 0, sizeof s);
  if (A.default_settings) A.default_settings(&s);
  s.stack_frame_size = 256;
  s.max_stack_frames = 8;
  s.max_steps = c.max_steps;
  s.ingress_ifindex = 1;
  s.mode = c.mode;
  void* vm = nullptr;
  int rc = A.create(&s, &vm);
  put32(rc);
  if (rc) return out;
  std::vector<int32_t> midx;
  for (const Map& m : c.maps) {
    int32_t mi = 0;
    rc = A.add_map(vm, &m.def, m.init.empty() ? nullptr : m.init.data(), m.init.size(), &mi);
    put32(rc);
    if (rc) { A.destroy(vm); return out; }
    midx.push_back(mi);
    for (const Entry& e : m.ents) put32(e.push ? A.map_push(vm, mi, e.val.data()) : A.map_update(vm, mi, e.key.data(), e.val.data()));
  }
  int32_t first = 0;
  for (size_t q = 0; q < c.progs.size(); q++) {
    int32_t pi = 0;
    rc = A.add_raw_program(vm, c.progs[q].data(), uint32_t(c.progs[q].size()), &pi);
    put32(rc);
    if (rc) { A.destroy(vm); return out; }
    if (q == 0) first = pi;
  }
  put32(A.set_entrypoint(vm, first));
  const uint32_t n = uint32_t(c.descs.size());
  std::vector<uint8_t> umem(c.umem);
  std::vector<xe_result> res(n);
  std::vector<uint32_t> ver(n);
  std::vector<xe_regs> regs(n);
  xe_batch_stats st;
  memset(&st, 0, sizeof st);
  if (n) { memset(res.data(), 0, n * sizeof(xe_result)); memset(regs.data(), 0, n * sizeof(xe_regs)); }
  rc = A.run(vm, umem.empty() ? nullptr : umem.data(), umem.size(), n ? c.descs.data() : nullptr, n,
             n ? res.data() : nullptr, n ? ver.data() : nullptr, n ? regs.data() : nullptr, &st);
  put32(rc);
  if (rc == 0) {
    sec("results");
    put(res.data(), n * sizeof(xe_result));
    sec("verdicts");
    put(ver.data(), n * sizeof(uint32_t));
    sec("regs");
    for (const xe_regs& r : regs) {  // fields only: the struct's padding is not an observable
      put(r.val, sizeof r.val); put(r.kind, sizeof r.kind); put(r.region, sizeof r.region);
      put(r.map, sizeof r.map); put(&r.steps, sizeof r.steps);
    }
    sec("packet bytes");
    put(umem.data(), umem.size());
    sec("steps");
    put(&st.steps, sizeof st.steps);
    for (size_t i = 0; i < c.maps.size(); i++) {
      sec("map " + std::to_string(i + 1));
      const xe_map_def& d = c.maps[i].def;
      const int32_t mi = midx[i];
      if (d.type == XE_MAP_QUEUE || d.type == XE_MAP_STACK || d.type == XE_MAP_PERF_EVENT_ARRAY) {
        uint64_t cnt = 0, nb = 0;
        put32(A.map_dump_list(vm, mi, nullptr, 0, nullptr, 0, &cnt, &nb));
        std::vector<uint8_t> data(nb + 1);
        std::vector<uint32_t> lens(cnt + 1);
        put32(A.map_dump_list(vm, mi, data.data(), nb, lens.data(), cnt, &cnt, &nb));
        put(&cnt, 8);
        put(lens.data(), cnt * 4);
        put(data.data(), nb);
        continue;
      }
      uint64_t cnt = 0;
      put32(A.map_dump(vm, mi, nullptr, nullptr, 0, &cnt));
      const bool array = d.type == XE_MAP_ARRAY || d.type == XE_MAP_PERCPU_ARRAY || d.type == XE_MAP_PROG_ARRAY ||
                         d.type == XE_MAP_ARRAY_OF_MAPS;
      if (array) {
        std::vector<uint8_t> raw(size_t(d.value_size) * d.max_entries + 1);
        put32(A.map_dump(vm, mi, raw.data(), nullptr, cnt, &cnt));
        put(raw.data(), raw.size() - 1);
      } else {
        std::vector<uint8_t> keys(cnt * d.key_size + 1), vals(cnt * d.value_size + 1);
        put32(A.map_dump(vm, mi, cnt ? keys.data() : nullptr, cnt ? vals.data() : nullptr, cnt, &cnt));
        put(&cnt, 8);
        put(keys.data(), cnt * d.key_size);
        put(vals.data(), cnt * d.value_size);
        if (d.type == XE_MAP_LRU_HASH || d.type == XE_MAP_LRU_PERCPU_HASH) {
          uint64_t lc = 0;
          put32(A.map_lru_order(vm, mi, nullptr, 0, &lc));
          std::vector<uint8_t> lk(lc * d.key_size + 1);
          put32(A.map_lru_order(vm, mi, lk.data(), lc, &lc));
          put(lk.data(), lc * d.key_size);
        }
      }
    }
  }
  A.destroy(vm);
  return out;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc != 4) { fprintf(stderr, "usage: %s oracle.so hostsim.so cases.bin\n", argv[0]); return 2; }
  Api oracle(argv[1], "orc_"), sim(argv[2], "xe_");
  FILE* f = fopen(argv[3], "rb");
  if (!f) { perror(argv[3]); return 2; }
  std::vector<uint8_t> buf;
  for (int ch; (ch = fgetc(f)) != EOF;) buf.push_back(uint8_t(ch));
  fclose(f);
  Reader R{buf.data(), buf.data() + buf.size()};
  if (buf.size() < 12 || memcmp(buf.data(), "XECASES1", 8) != 0) { fprintf(stderr, "bad case file\n"); return 2; }
  R.p += 8;
  const uint32_t ncases = R.get<uint32_t>();
  int bad = 0;
  for (uint32_t ci = 0; ci < ncases; ci++) {
    Case c;
    const uint32_t nl = R.get<uint32_t>();
    std::vector<uint8_t> nm = R.bytes(nl);
    c.name.assign(nm.begin(), nm.end());
    c.max_steps = R.get<uint64_t>();
    c.mode = R.get<uint32_t>();
    const uint32_t np = R.get<uint32_t>();
    for (uint32_t q = 0; q < np; q++) {
      const uint32_t n = R.get<uint32_t>();
      std::vector<uint64_t> p(n);
      for (uint32_t k = 0; k < n; k++) p[k] = R.get<uint64_t>();
      c.progs.push_back(p);
    }
    const uint32_t nm2 = R.get<uint32_t>();
    for (uint32_t m = 0; m < nm2; m++) {
      Map mp;
      mp.def.type = R.get<uint32_t>(); mp.def.key_size = R.get<uint32_t>(); mp.def.value_size = R.get<uint32_t>();
      mp.def.max_entries = R.get<uint32_t>(); mp.def.flags = R.get<uint32_t>();
      mp.init = R.bytes(R.get<uint32_t>());
      const uint32_t ne = R.get<uint32_t>();
      for (uint32_t e = 0; e < ne; e++) {
        Entry en;
        en.push = R.get<uint8_t>() != 0;
        if (!en.push) en.key = R.bytes(mp.def.key_size);
        en.val = R.bytes(mp.def.value_size);
        mp.ents.push_back(en);
      }
      c.maps.push_back(mp);
    }
    const uint32_t npk = R.get<uint32_t>();
    c.umem = R.bytes(size_t(R.get<uint64_t>()));
    c.descs.resize(npk);
    for (uint32_t i = 0; i < npk; i++) {
      c.descs[i].addr = R.get<uint64_t>();
      c.descs[i].len = R.get<uint32_t>();
      c.descs[i].options = R.get<uint32_t>();
    }
    const std::vector<uint8_t> a = run_case(oracle, c), b = run_case(sim, c);
    if (a != b) {
      size_t at = 0;
      while (at < a.size() && at < b.size() && a[at] == b[at]) at++;
      std::string what = "setup";
      for (auto& s : g_sections)
        if (s.first <= at) what = s.second + " +" + std::to_string(at - s.first);
      fprintf(stderr, "MISMATCH %s: observables differ in %s (byte %zu; sizes %zu / %zu): oracle %02x hostsim %02x\n",
              c.name.c_str(), what.c_str(), at, a.size(), b.size(), at < a.size() ? a[at] : 0, at < b.size() ? b[at] : 0);
      bad++;
    }
  }
  printf("%u cases, %d mismatches\n", ncases, bad);
  return bad ? 1 : 0;
}
