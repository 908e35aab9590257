// zb_wavelib.hpp — wave-level helpers of the drain write passes (zb_tdrain.hip, zb_serialize.hip): a DPP scan,
// the wave's LDS visibility point and the 16-byte streaming of a wave's LDS image.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace zbg {

// Inclusive sum over the wave's lanes 0..lane, with DPP row shifts and row broadcasts (VALU only: no LDS round
// trip per step, unlike a shuffle)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return x;
}

// LDS writes of other lanes of the wave are visible to this lane's later reads (and the reverse)
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// image bytes [shift, shift + n) -> out[o, o + n) by one wave: 16-byte non-temporal stores aligned to the
// destination, bytes at the two ends (shared with the neighbouring ranges) one at a time
__device__ __forceinline__ void wave_stream(const uint8_t* img, uint8_t* out, uint64_t o, uint32_t shift, uint32_t n,
                                            int lane) {
  uint8_t* dst = out + o - shift;
  const uint32_t lim = shift + n;
  const uint32_t full_lo = (shift + 15) & ~15u, full_hi = lim & ~15u;
  for (uint32_t c = full_lo + 16 * lane; c < full_hi; c += 16 * 64) {
    const uint4 v = *(const uint4*)(img + c);
    __builtin_nontemporal_store(v.x, (uint32_t*)(dst + c));
    __builtin_nontemporal_store(v.y, (uint32_t*)(dst + c) + 1);
    __builtin_nontemporal_store(v.z, (uint32_t*)(dst + c) + 2);
    __builtin_nontemporal_store(v.w, (uint32_t*)(dst + c) + 3);
  }
  const uint32_t head_end = full_lo < lim ? full_lo : lim;
  const uint32_t tail_lo = full_hi > head_end ? full_hi : head_end;
  const uint32_t nh = head_end - shift;  // at most 15 + 15 bytes: one per lane
  if ((uint32_t)lane < nh) dst[shift + lane] = img[shift + lane];
  else if ((uint32_t)lane < nh + (lim - tail_lo)) dst[tail_lo + lane - nh] = img[tail_lo + lane - nh];
}

}  // namespace zbg
