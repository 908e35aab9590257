// zb_xlock.hpp — the exact payload tree (zb_xmerge.hpp) inside the kernels: a lane whose document pair the fast
// paths refused runs it in a small workspace of its own (x_run) or, when the pair's tree does not fit it, takes one of
// XSLAB_COUNT big workspace slabs for the duration of one x_merge / x_map.
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
  uint32_t* locks;  // XSLAB_COUNT slab locks, then XLANE_GROUPS lane-group locks; 0 = free
  uint8_t* lanes;   // XLANE_COUNT x XLANE_BYTES: XLANE_GROUPS groups of 64 lane workspaces
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
      f(XWs{X.base + (uint64_t)slot * XSLAB_BYTES, XSLAB_BYTES, 0u, 1u});
      __threadfence();
      atomicExch(&X.locks[slot], 0u);
    }
    m &= m - 1;
  }
}

// The XCD this wave runs on (HW_REG_XCC_ID, 0..7)
__device__ __forceinline__ uint32_t xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 7u; }

// The exact tree for every lane with `need`: first each in a XLANE_BYTES workspace of its own, all lanes of the wave at
// once; a pair whose tree does not fit it (X_UNSUP, nothing written yet) then takes a big slab in turns (x_exclusive).
// The wave's lanes use the 64 workspaces of one lane group, which the wave holds for the duration (a lock no holder
// waits on anything while holding). The groups are split among the 8 XCDs and a wave takes one of its own XCD's
// (HW_REG_XCC_ID; within it by the block's rank among the blocks dealt to that XCD): a workspace is only ever
// written through one XCD's L2, so a holder needs no agent-scope fence -- its stores reaching that L2 before the lock
// is released (vmcnt) is enough, and x_merge / x_map read only workspace bytes they wrote in the same call. (Across
// XCDs the per-XCD L2s are not coherent: a workspace shared by two XCDs needed __threadfence -- an L2 write-back and
// an L1 invalidate -- around every hold, 3 ms of an 8.9 ms tick that merges 1M documents through the tree.)
// f(workspace, final) -> X_* status; it commits its outcome unless it returns X_UNSUP with final false.
template <class F>
__device__ __forceinline__ void x_run(const XSlabs& X, bool need, F&& f) {
  bool again = need;
  const uint64_t m = (uint64_t)__ballot(need);
  if (m && X.lanes) {
    const int lane = threadIdx.x & 63;
    constexpr uint32_t GPX = XLANE_GROUPS / 8;  // groups per XCD
    static_assert(XLANE_GROUPS % 8 == 0, "lane groups split evenly over the XCDs");
    const uint32_t local = (uint32_t)(((uint64_t)(blockIdx.x / 8) * (blockDim.x >> 6) + (threadIdx.x >> 6)) % GPX);
    const uint32_t g = __builtin_amdgcn_readfirstlane(xcc_id()) * GPX + local;
    uint32_t* lock = X.locks + XSLAB_COUNT + g;
    const int l0 = __ffsll((unsigned long long)m) - 1;
    if (lane == l0)
      while (atomicCAS(lock, 0u, 1u) != 0u) __builtin_amdgcn_s_sleep(4);
    __builtin_amdgcn_wave_barrier();
    // (the group's 64 workspaces interleaved: XWs)
    if (need) again = f(XWs{X.lanes + (uint64_t)g * 64 * XLANE_BYTES, XLANE_BYTES, (uint32_t)lane, 64u}, false) == X_UNSUP;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (every lane's workspace stores are in the XCD's L2)
    __builtin_amdgcn_wave_barrier();
    if (lane == l0) atomicExch(lock, 0u);
  }
  x_exclusive(X, again, [&](const XWs& w) { (void)f(w, true); });
}

}  // namespace zbg
