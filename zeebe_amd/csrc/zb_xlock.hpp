// zb_xlock.hpp — the exact payload tree (zb_xmerge.hpp) inside the kernels: a lane whose document pair the fast
// paths refused takes one of XSLAB_COUNT workspace slabs for the duration of one x_merge / x_map.
//
// The lanes of a wave that need it take their turns one at a time (the mask comes from a ballot, so the loop is
// wave-uniform), and the single active lane spins on the slab's lock. No holder ever waits for anything while
// holding a lock, and a spinning lane is alone in its wave, so every holder makes progress: no deadlock.
#pragma once
#include <hip/hip_runtime.h>

#include "zb_xmerge.hpp"

namespace zbg {

struct XSlabs {
  uint8_t* base;    // XSLAB_COUNT x XSLAB_BYTES
  uint32_t* locks;  // XSLAB_COUNT, 0 = free
};

template <class F>
__device__ __forceinline__ void x_exclusive(const XSlabs& X, bool need, F&& f) {
  uint64_t m = (uint64_t)__ballot(need);
  if (!m) return;
  const int lane = threadIdx.x & 63;
  const uint32_t slot = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) % XSLAB_COUNT;
  while (m) {
    const int l = __ffsll((unsigned long long)m) - 1;
    if (lane == l) {
      while (atomicCAS(&X.locks[slot], 0u, 1u) != 0u) __builtin_amdgcn_s_sleep(4);
      __threadfence();
      f(X.base + (uint64_t)slot * XSLAB_BYTES);
      __threadfence();
      atomicExch(&X.locks[slot], 0u);
    }
    m &= m - 1;
  }
}

}  // namespace zbg
