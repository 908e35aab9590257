// zb_checked.hip — guard bands and per-launch checks of the checked build (zb_checked.hpp). Linked only into
// libzbgpu_checked.so: a test instrument for finding out-of-bounds writes, not part of the product library.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace zbg {
namespace {

constexpr size_t FRONT = 64 << 10;   // guard before the buffer (biased pointers, negative indices)
constexpr size_t BACK = 256 << 10;   // guard after it
constexpr uint8_t PAT = 0xA5;

struct Alloc {
  uint8_t* raw;
  size_t n;
  std::string site;
};

struct State {
  std::mutex mu;
  std::map<uintptr_t, Alloc> live;  // user pointer -> allocation
  std::vector<uint64_t> tab;        // (ptr, bytes, alloc id) triples of the live guard regions
  bool dirty = true;
  uint64_t* d_tab = nullptr;
  size_t d_tab_cap = 0;
  unsigned long long* d_bad = nullptr;
  hipStream_t s = nullptr;
  FILE* trace = nullptr;
  unsigned long long violations = 0, launches = 0;
  std::string last[8];
  int last_i = 0;
};

State& st() {
  static State* s = [] {
    auto* x = new State();
    if (const char* f = std::getenv("ZB_CHECKED_TRACE")) x->trace = std::fopen(f, "a");
    return x;
  }();
  return *s;
}

void log_line(const std::string& m, bool to_stderr) {
  State& S = st();
  if (S.trace) {
    std::fputs(m.c_str(), S.trace);
    std::fputc('\n', S.trace);
    std::fflush(S.trace);
  }
  if (to_stderr) std::fprintf(stderr, "%s\n", m.c_str());
}

// every byte of every listed region must still be the pattern; bad = the smallest (region << 32 | offset) that is not
__global__ void k_guard_scan(const uint64_t* tab, uint32_t n, unsigned long long* bad) {
  for (uint32_t r = blockIdx.x; r < n; r += gridDim.x) {
    const uint8_t* p = (const uint8_t*)tab[3 * r];
    const uint64_t len = tab[3 * r + 1];
    for (uint64_t i = threadIdx.x; i < len; i += blockDim.x)
      if (p[i] != PAT) atomicMin(bad, (unsigned long long)r << 32 | i);
  }
}

void rebuild_table(State& S) {
  S.tab.clear();
  for (auto& kv : S.live) {  // region 2k: the front band, 2k + 1: the back band (from the first byte past the buffer)
    const Alloc& a = kv.second;
    S.tab.push_back((uint64_t)(uintptr_t)a.raw);
    S.tab.push_back(FRONT);
    S.tab.push_back(kv.first);
    S.tab.push_back((uint64_t)(uintptr_t)(a.raw + FRONT + a.n));
    S.tab.push_back(BACK);
    S.tab.push_back(kv.first);
  }
  S.dirty = false;
}

std::string describe(State& S, uint64_t bad) {
  const uint32_t r = (uint32_t)(bad >> 32), off = (uint32_t)bad;
  const uintptr_t user = (uintptr_t)S.tab[3 * r + 2];
  auto it = S.live.find(user);
  char b[512];
  if (it == S.live.end()) return "unknown region";
  const Alloc& a = it->second;
  if (r % 2 == 0)
    std::snprintf(b, sizeof b, "%s (%zu bytes): front band overwritten %zu bytes before the buffer", a.site.c_str(),
                  a.n, (size_t)(FRONT - off));
  else
    std::snprintf(b, sizeof b, "%s (%zu bytes): back band overwritten at buffer offset %zu", a.site.c_str(), a.n,
                  (size_t)(a.n + off));
  return b;
}

// scans every band; reports and re-arms a damaged one. Caller holds the lock.
void scan(State& S, const char* after) {
  if (S.live.empty()) return;
  if (!S.s) {
    if (hipStreamCreateWithFlags(&S.s, hipStreamNonBlocking) != hipSuccess) return;
    if (hipMalloc(&S.d_bad, sizeof(unsigned long long)) != hipSuccess) return;
  }
  if (S.dirty) {
    rebuild_table(S);
    if (S.tab.size() > S.d_tab_cap) {
      if (S.d_tab) (void)hipFree(S.d_tab);
      S.d_tab_cap = S.tab.size() * 2;
      if (hipMalloc(&S.d_tab, S.d_tab_cap * sizeof(uint64_t)) != hipSuccess) return;
    }
    (void)hipMemcpy(S.d_tab, S.tab.data(), S.tab.size() * sizeof(uint64_t), hipMemcpyHostToDevice);
  }
  const uint32_t n = (uint32_t)(S.tab.size() / 3);
  for (int round = 0; round < 64; round++) {
    unsigned long long bad = ~0ull;
    (void)hipMemcpyAsync(S.d_bad, &bad, sizeof bad, hipMemcpyHostToDevice, S.s);
    hipLaunchKernelGGL(k_guard_scan, dim3(n < 4096 ? n : 4096), dim3(256), 0, S.s, S.d_tab, n, S.d_bad);
    (void)hipMemcpyAsync(&bad, S.d_bad, sizeof bad, hipMemcpyDeviceToHost, S.s);
    (void)hipStreamSynchronize(S.s);
    if (bad == ~0ull) return;
    S.violations++;
    std::string m = "ZB_CHECKED guard violation: " + describe(S, bad) + " -- seen after " + after + "; launches before:";
    for (int k = 1; k <= 8; k++) {
      const std::string& l = S.last[(S.last_i - k + 8) % 8];
      if (!l.empty()) m += " | " + l;
    }
    log_line(m, true);
    const uint32_t r = (uint32_t)(bad >> 32);
    (void)hipMemset((void*)(uintptr_t)S.tab[3 * r], PAT, S.tab[3 * r + 1]);  // re-arm, look for more
    (void)hipDeviceSynchronize();
  }
}

}  // namespace

hipError_t checked_malloc(void** p, size_t n, const char* what, const char* file, int line) {
  State& S = st();
  std::lock_guard<std::mutex> g(S.mu);
  uint8_t* raw = nullptr;
  hipError_t e = hipMalloc((void**)&raw, FRONT + n + BACK);
  if (e != hipSuccess) {
    *p = nullptr;
    return e;
  }
  e = hipMemset(raw, PAT, FRONT + n + BACK);  // (the buffer too: reads of never-written bytes see the pattern)
  if (e != hipSuccess) return e;
  // the fill runs on the null stream, which does not order against the engine's non-blocking stream: it must
  // have completed before the caller queues anything that writes the buffer
  e = hipDeviceSynchronize();
  if (e != hipSuccess) return e;
  *p = raw + FRONT;
  const char* base = std::strrchr(file, '/');
  char site[256];
  std::snprintf(site, sizeof site, "%s @ %s:%d", what, base ? base + 1 : file, line);
  S.live[(uintptr_t)*p] = Alloc{raw, n, site};
  S.dirty = true;
  char m[400];
  std::snprintf(m, sizeof m, "alloc %p +%zu %s", *p, n, site);
  log_line(m, false);
  return hipSuccess;
}

hipError_t checked_free(void* p) {
  if (!p) return hipSuccess;
  State& S = st();
  std::lock_guard<std::mutex> g(S.mu);
  auto it = S.live.find((uintptr_t)p);
  if (it == S.live.end()) return hipFree(p);
  (void)hipDeviceSynchronize();
  scan(S, ("free of " + it->second.site).c_str());
  uint8_t* raw = it->second.raw;
  char m[400];
  std::snprintf(m, sizeof m, "free %p %s", p, it->second.site.c_str());
  log_line(m, false);
  S.live.erase(it);
  S.dirty = true;
  return hipFree(raw);
}

void checked_after_launch(const char* kernel, hipStream_t s, const char* file, int line) {
  State& S = st();
  std::lock_guard<std::mutex> g(S.mu);
  const char* base = std::strrchr(file, '/');
  char at[320];
  std::snprintf(at, sizeof at, "%s (%s:%d)", kernel, base ? base + 1 : file, line);
  S.launches++;
  if (S.trace) log_line(std::string("launch ") + at, false);
  const hipError_t le = hipGetLastError();
  const hipError_t se = hipStreamSynchronize(s);
  if (le != hipSuccess || se != hipSuccess) {
    log_line(std::string("ZB_CHECKED launch failure after ") + at + ": " +
                 hipGetErrorString(le != hipSuccess ? le : se), true);
    S.violations++;
  }
  S.last[S.last_i] = at;
  S.last_i = (S.last_i + 1) % 8;
  scan(S, at);
}

}  // namespace zbg

// test hook of the checked library: guard violations / failed launches so far, and launches checked
extern "C" unsigned long long zb_checked_violations(unsigned long long* launches) {
  zbg::State& S = zbg::st();
  std::lock_guard<std::mutex> g(S.mu);
  if (launches) *launches = S.launches;
  return S.violations;
}
