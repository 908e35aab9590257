// Launch / copy / synchronisation costs of the HIP runtime the process bound (measurement tool, not product code):
// python3 tools/probe/launch_probe.py compares the system ROCm runtime with the one torch bundles.
#include <hip/hip_runtime.h>

#include <dlfcn.h>

#include <chrono>
#include <cstdint>

struct Big {
  uint64_t w[96];  // (a 768-byte argument block)
};
struct Huge {
  uint64_t w[256];  // (2 KB)
};
__global__ void k_huge(Huge b) {
  if (b.w[0] == 12345 && threadIdx.x == 1000) b.w[1] = 1;
}
__global__ void k_empty() {}
__global__ void k_big(Big b) {
  if (b.w[0] == 12345 && threadIdx.x == 1000) b.w[1] = 1;
}
__global__ void k_grid(uint32_t* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0xffffff) p[0] = 1;
}

extern "C" double probe(int kind, int n) {
  static hipStream_t s = nullptr;
  static uint32_t* d = nullptr;
  static uint32_t* h = nullptr;
  if (!s) {
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    (void)hipMalloc(&d, 1 << 20);
    (void)hipHostMalloc(&h, 4096);
  }
  Big b{};
  Huge hb{};
  (void)hipStreamSynchronize(s);
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; i++) {
    switch (kind) {
      case 0: hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s); break;
      case 1: hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, s, b); break;
      case 2: (void)hipMemsetAsync(d, 0, 64, s); break;
      case 3: (void)hipMemcpyAsync(h, d, 64, hipMemcpyDeviceToHost, s); break;
      case 4: hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s); (void)hipStreamSynchronize(s); break;
      case 5: hipLaunchKernelGGL(k_grid, dim3(4096), dim3(256), 0, s, d); break;
      case 7: hipLaunchKernelGGL(k_huge, dim3(1), dim3(64), 0, s, hb); break;
      case 6: { hipEvent_t e; (void)hipEventCreate(&e); (void)hipEventRecord(e, s); (void)hipEventDestroy(e); break; }
    }
  }
  (void)hipStreamSynchronize(s);
  const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  return us / n;
}

extern "C" const char* probe_runtime() {
  Dl_info info{};
  return dladdr((void*)&hipStreamSynchronize, &info) && info.dli_fname ? info.dli_fname : "?";
}
