// zb_checked.hpp — the guard-band build of the engine (libzbgpu_checked.so, `make checked`): a test instrument,
// never the product library.
//
// Compiled with -DZB_CHECKED, every device allocation of the engine (hipMalloc) gets a guard band before and after
// the requested bytes, filled with a known pattern, and every kernel launch (hipLaunchKernelGGL) is followed by a
// stream synchronisation and a device-side scan of every live guard band. A kernel (or a copy / memset queued
// before it) that writes outside its buffer is reported with the allocation site, the side of the band and the
// first offset it touched, and the launch after which it was seen -- instead of corrupting a neighbouring buffer
// silently or faulting only when the page layout puts an unmapped page there. A launch whose synchronisation fails
// (a memory fault, an illegal instruction) names the kernel. ZB_CHECKED_TRACE=<file> logs every allocation and
// every launch to a file, flushed as it goes.
#pragma once
#ifdef ZB_CHECKED
#include <hip/hip_runtime.h>

#include <cstddef>

namespace zbg {
hipError_t checked_malloc(void** p, size_t n, const char* what, const char* file, int line);
hipError_t checked_free(void* p);
void checked_after_launch(const char* kernel, hipStream_t s, const char* file, int line);
}  // namespace zbg

#define hipMalloc(p, n) ::zbg::checked_malloc((void**)(p), (size_t)(n), #p, __FILE__, __LINE__)
#define hipFree(p) ::zbg::checked_free((void*)(p))
#undef hipLaunchKernelGGL
#define hipLaunchKernelGGL(kernel, grid, block, lds, stream, ...)                       \
  do {                                                                                \
    hipLaunchKernelGGLInternal((kernel), (grid), (block), (lds), (stream), ##__VA_ARGS__); \
    ::zbg::checked_after_launch(#kernel, (stream), __FILE__, __LINE__);               \
  } while (0)
#endif
