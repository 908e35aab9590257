// zb_msg.hpp — message correlation helpers shared by the wave pipeline (workflow side) and the
// message-side kernels (zb_msg.hip): partition routing, store hashing, arena blob layouts, outbox records.
#pragma once
#include <hip/hip_runtime.h>

#include "zb_kernels.hpp"
#include "zb_wavelib.hpp"

namespace zbg {

constexpr uint32_t NO_ENTRY = 0xffffffffu;

// ---- arena blobs of the message side ([u32 len][len bytes], 8-aligned; len counts the bytes after the word)
// message (MessageRecord.java:26-42 as stored by MessageDataStore.Message): the PUBLISH command's decoded value
//   [u32 len][u32 name_len][i64 ttl][i64 deadline][u32 ck_len][u32 payload_len][u32 id_len][u32 pad]
//   [name][correlation key][payload document][message id]
constexpr uint32_t MSG_HDR = 40;  // bytes before the name (incl. the length word)
struct MsgView {
  int64_t ttl, deadline;
  const uint8_t *name, *ck, *payload, *id;
  uint32_t nn, nc, np, nid;
};
__device__ __forceinline__ MsgView msg_view(const uint8_t* arena, uint32_t ref) {
  const uint8_t* b = arena + (uint64_t)ref * 8;
  MsgView v;
  v.nn = *(const uint32_t*)(b + 4);
  v.ttl = *(const int64_t*)(b + 8);
  v.deadline = *(const int64_t*)(b + 16);
  v.nc = *(const uint32_t*)(b + 24);
  v.np = *(const uint32_t*)(b + 28);
  v.nid = *(const uint32_t*)(b + 32);
  v.name = b + MSG_HDR;
  v.ck = v.name + v.nn;
  v.payload = v.ck + v.nc;
  v.id = v.payload + v.np;
  return v;
}
// subscription (MessageSubscriptionRecord.java:26-41 as OPEN delivered it):
//   [u32 len][i32 wf_partition][u32 token][u16 elem][u16 pad][u32 name_len][u32 ck_len][name][correlation key]
constexpr uint32_t SUB_HDR = 24;
struct SubView {
  int32_t wfp;
  uint32_t token;
  uint16_t elem;
  const uint8_t *name, *ck;
  uint32_t nn, nc;
};
__device__ __forceinline__ SubView sub_view(const uint8_t* arena, uint32_t ref) {
  const uint8_t* b = arena + (uint64_t)ref * 8;
  SubView v;
  v.wfp = *(const int32_t*)(b + 4);
  v.token = *(const uint32_t*)(b + 8);
  v.elem = *(const uint16_t*)(b + 12);
  v.nn = *(const uint32_t*)(b + 16);
  v.nc = *(const uint32_t*)(b + 20);
  v.name = b + SUB_HDR;
  v.ck = v.name + v.nn;
  return v;
}

// SubscriptionUtil.getSubscriptionHashCode (SubscriptionUtil.java:30-38: 31-hash over SIGNED bytes,
// int32 wraparound) -> abs(hash % P) (SubscriptionCommandSender.java:105-109, Java remainder)
__device__ __forceinline__ int32_t subscription_partition(const uint8_t* ck, uint32_t n, int32_t P) {
  uint32_t h = 0;
  for (uint32_t i = 0; i < n; i++) h = h * 31u + (uint32_t)(int32_t)(int8_t)ck[i];
  const int32_t r = (int32_t)h % P;
  return r < 0 ? -r : r;
}

// store hash of (message name, correlation key): FNV-1a over the bytes, read as the aligned words that hold them (a
// byte loop was a memory request per byte); equality is always re-checked on the bytes
__device__ __forceinline__ uint64_t fnv_words(uint64_t h, const uint8_t* s, uint32_t n) {
  if (!n) return h;
  const uint64_t* a = (const uint64_t*)((uintptr_t)s & ~(uintptr_t)7);
  uint32_t off = (uint32_t)((uintptr_t)s & 7);
  while (n) {
    uint64_t w = *a++ >> (8 * off);
    const uint32_t take = 8 - off < n ? 8 - off : n;
    for (uint32_t k = 0; k < take; k++) {
      h ^= (uint8_t)(w >> (8 * k));
      h *= 0x100000001b3ull;
    }
    n -= take;
    off = 0;
  }
  return h;
}
__device__ __forceinline__ uint64_t name_ck_hash(const uint8_t* name, uint32_t nn, const uint8_t* ck, uint32_t nc) {
  uint64_t h = fnv_words(0xcbf29ce484222325ull, name, nn);
  h ^= 0x1ff;
  h *= 0x100000001b3ull;
  return fnv_words(h, ck, nc);
}

// outbox order: (target partition, source log position, emission index) — the order in which the
// reference's processors produce the commands (side effects run in processing order;
// findSubscriptions returns subscriptions in insertion order). Log positions are 64-bit and never rebased
// (LogEntryDescriptor.java:28-121): the key holds the position relative to the outbox's base (Outbox.pos_base), so
// the fields stay exact for any absolute position; OB_REL_BITS / OB_EMIT_BITS bound what one outbox can hold
// between two takes (outbox_write refuses the rest instead of wrapping).
constexpr int OB_REL_BITS = 34, OB_EMIT_BITS = 24;
__device__ __forceinline__ uint64_t outbox_key(int32_t target, uint64_t rel, uint32_t emission) {
  return ((uint64_t)target << (OB_REL_BITS + OB_EMIT_BITS)) | (rel << OB_EMIT_BITS) | emission;
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

// Slots for ca / cb per thread from one atomic per counter per WORKGROUP. wave_alloc makes one per wave, and
// atomics on one address serialize (~12 ns each on MI355X): 32K of them were 0.4 ms of a 1M-command k_subscribe.
// Every thread of the workgroup calls it at the same point, with all lanes active (DPP scans, barriers inside);
// s: __shared__ uint32_t[2 * (WGS / 64) + 2].
template <int WGS>
__device__ __forceinline__ void block_alloc2(uint32_t* ctr_a, uint32_t ca, uint32_t* ctr_b, uint32_t cb, uint32_t* s,
                                             uint32_t& slot_a, uint32_t& slot_b) {
  constexpr int NW = WGS / 64;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t ia = wave_incl_scan(ca), ib = wave_incl_scan(cb);
  if (lane == 63) {
    s[wv] = ia;
    s[NW + wv] = ib;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    uint32_t tot = 0;
    for (int w = 0; w < NW; w++) tot += s[threadIdx.x * NW + w];
    s[2 * NW + threadIdx.x] = tot ? atomicAdd(threadIdx.x ? ctr_b : ctr_a, tot) : 0u;
  }
  __syncthreads();
  uint32_t pa = s[2 * NW], pb = s[2 * NW + 1];
  for (int w = 0; w < NW; w++)
    if (w < wv) {
      pa += s[w];
      pb += s[NW + w];
    }
  slot_a = pa + ia - ca;
  slot_b = pb + ib - cb;
  __syncthreads();  // (s is reused by the next call)
}
// the same for one 64-bit counter (arena bytes); s64: __shared__ uint64_t[WGS / 64 + 1]
template <int WGS>
__device__ __forceinline__ uint64_t block_alloc64(unsigned long long* ctr, uint64_t c, uint64_t* s64) {
  constexpr int NW = WGS / 64;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t x = c;  // (64-bit inclusive scan by shuffles)
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = (uint64_t)__shfl_up((unsigned long long)x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) s64[wv] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t tot = 0;
    for (int w = 0; w < NW; w++) tot += s64[w];
    s64[NW] = tot ? (uint64_t)atomicAdd(ctr, (unsigned long long)tot) : 0ull;
  }
  __syncthreads();
  uint64_t p = s64[NW];
  for (int w = 0; w < NW; w++)
    if (w < wv) p += s64[w];
  __syncthreads();
  return p + x - c;
}

__device__ __forceinline__ uint32_t var_granules(uint32_t nn, uint32_t nc, uint32_t np) {
  return (nn + nc + np + 7) >> 3;
}

// Bytes appended to an 8-aligned destination as whole 8-byte words: a byte loop was one memory request per byte
// (the message kernels were bound by them). Sources are read as the aligned words that hold them (a load never
// reaches past the aligned word of a source's last byte, so never past its allocation's page); the last word is
// zero-padded, and nothing is written past it.
struct WordWriter {
  uint64_t* d;
  uint64_t acc;
  uint32_t fill;  // bytes in acc (< 8)
  __device__ __forceinline__ explicit WordWriter(uint8_t* dst) : d((uint64_t*)dst), acc(0), fill(0) {}
  // the low nb bytes of w (1 <= nb <= 8; the bytes above them zero)
  __device__ __forceinline__ void push(uint64_t w, uint32_t nb) {
    acc |= w << (8 * fill);
    const uint32_t f = fill + nb;
    if (f >= 8) {
      *d++ = acc;
      acc = fill ? (w >> (8 * (8 - fill))) : 0;
      fill = f - 8;
    } else {
      fill = f;
    }
  }
  __device__ __forceinline__ void bytes(const uint8_t* s, uint32_t n) {
    if (!n) return;
    const uint64_t* a = (const uint64_t*)((uintptr_t)s & ~(uintptr_t)7);
    uint32_t off = (uint32_t)((uintptr_t)s & 7);
    while (n) {
      const uint32_t take = 8 - off < n ? 8 - off : n;
      uint64_t w = *a++ >> (8 * off);
      if (take < 8) w &= (1ull << (8 * take)) - 1;
      push(w, take);
      n -= take;
      off = 0;
    }
  }
  __device__ __forceinline__ void finish() {
    if (fill) *d = acc;
  }
};

// false (nothing written): the source position or the emission index does not fit the order key -- the caller fails
// the partition (DE_UNSUPPORTED) rather than ordering the exchange wrongly
__device__ __forceinline__ bool outbox_write(const Outbox& ob, uint32_t slot, uint32_t var_at, int32_t kind, int32_t target,
                                             int32_t wfp, uint32_t token, int64_t wik, int64_t aik, int64_t spos,
                                             uint16_t elem, const uint8_t* name, uint32_t nn, const uint8_t* ck,
                                             uint32_t nc, const uint8_t* payload, uint32_t np, uint32_t emission) {
  const uint64_t rel = (uint64_t)(spos - ob.pos_base);
  if (spos < ob.pos_base || rel >= (1ull << OB_REL_BITS) || emission >= (1u << OB_EMIT_BITS)) return false;
  zb_exchange_rec r;
  r.kind = kind; r.target_partition = target; r.wf_partition = wfp; r.token = token;
  r.workflow_instance_key = wik; r.activity_instance_key = aik; r.source_position = spos;
  r.elem = elem; r.pad = 0;
  r.name_len = nn; r.ck_len = nc; r.payload_len = np;
  r.var_offset = (uint64_t)var_at * 8;
  WordWriter v(ob.var + (uint64_t)var_at * 8);  // (exactly var_granules(nn, nc, np) words, zero-padded)
  v.bytes(name, nn);
  v.bytes(ck, nc);
  v.bytes(payload, np);
  v.finish();
  ob.rec[slot] = r;
  ob.keys[slot] = outbox_key(target, rel, emission);
  return true;
}

}  // namespace zbg
