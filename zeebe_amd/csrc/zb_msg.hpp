// zb_msg.hpp — message correlation helpers shared by the wave pipeline (workflow side) and the
// message-side kernels (zb_msg.hip): partition routing, store hashing, outbox records.
#pragma once
#include <hip/hip_runtime.h>

#include "zb_kernels.hpp"

namespace zbg {

constexpr uint32_t NO_ENTRY = 0xffffffffu;
constexpr uint32_t SUB_BLOB = 112;   // [u32 len][i32 wfp][u8 name_len][u8 ck_len][u16 elem][u32 token][name 48][ck 48]
constexpr uint32_t WIS_BLOB = 120;   // [u32 len][payload document <= 112 B] (CORRELATE command payload)

// SubscriptionUtil.getSubscriptionHashCode (SubscriptionUtil.java:30-38: 31-hash over SIGNED bytes,
// int32 wraparound) -> abs(hash % P) (SubscriptionCommandSender.java:105-109, Java remainder)
__device__ __forceinline__ int32_t subscription_partition(const uint8_t* ck, uint32_t n, int32_t P) {
  uint32_t h = 0;
  for (uint32_t i = 0; i < n; i++) h = h * 31u + (uint32_t)(int32_t)(int8_t)ck[i];
  const int32_t r = (int32_t)h % P;
  return r < 0 ? -r : r;
}

// store hash of (message name, correlation key); equality is always re-checked on the bytes
__device__ __forceinline__ uint64_t fnv_bytes(uint64_t h, const uint8_t* p, uint32_t n) {
  for (uint32_t i = 0; i < n; i++) {
    h ^= p[i];
    h *= 0x100000001b3ull;
  }
  return h;
}
__device__ __forceinline__ uint64_t name_ck_hash(const uint8_t* name, uint32_t nn, const uint8_t* ck, uint32_t nc) {
  uint64_t h = fnv_bytes(0xcbf29ce484222325ull, name, nn);
  h ^= 0x1ff;
  h *= 0x100000001b3ull;
  return fnv_bytes(h, ck, nc);
}

// outbox order: (target partition, source log position, emission index) — the order in which the
// reference's processors produce the commands (side effects run in processing order;
// findSubscriptions returns subscriptions in insertion order)
__device__ __forceinline__ uint64_t outbox_key(int32_t target, int64_t pos, uint32_t emission) {
  return ((uint64_t)target << 58) | (((uint64_t)pos & ((1ull << 34) - 1)) << 24) | (emission & 0xffffffu);
}

// slots for `cnt` records per lane from one atomic per wave (lanes that reach this point together;
// inactive lanes take no part): returns this lane's first slot
__device__ __forceinline__ uint32_t wave_alloc(uint32_t* counter, uint32_t cnt) {
  const uint64_t active = __ballot(1);
  const int lane = (int)(threadIdx.x & 63);
  uint32_t excl = 0, total = 0;
  for (int l = 0; l < 64; l++) {  // uniform loop; reads only active lanes
    if (!((active >> l) & 1)) continue;
    const uint32_t v = __shfl(cnt, l, 64);
    total += v;
    if (l < lane) excl += v;
  }
  const int leader = __ffsll((unsigned long long)active) - 1;
  uint32_t base = 0;
  if (lane == leader && total) base = atomicAdd(counter, total);
  base = __shfl(base, leader, 64);
  return base + excl;
}

}  // namespace zbg
