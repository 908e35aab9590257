// zb_msg.hip — the message side of correlation and the partition
// exchange (zb_exchange_rec, include/zb_engine.h).
//
//   k_msg_open      MESSAGE_SUBSCRIPTION OPEN commands delivered by workflow partitions: append the
//                   command (key = its log position) and its OPENED event, look for a stored message
//                   (MessageDataStore.findMessage: the first one stored), insert the subscription
//                   (MessageSubscriptionDataStore.addSubscription) — OpenMessageSubscriptionProcessor.java:56-92
//   k_msg_publish   MESSAGE PUBLISH commands: PUBLISHED (+ DELETED when ttl <= 0) keyed by the message
//                   KeyGenerator(0, 1) (MessageService.java:91); every matching subscription becomes a
//                   correlate command in the outbox; the message is stored when ttl > 0
//                   — PublishMessageProcessor.java:58-124
//   k_wis_inject    CORRELATE commands delivered by message partitions -> WORKFLOW_INSTANCE_SUBSCRIPTION
//                   CORRELATE commands at the log tail (processed by the wave pipeline, zb_wave.hip)
//   k_outbox_gather / k_outbox_bounds   the outbox sorted by (target, source position, emission)
//
// The stores are hash tables of chains pushed lock-free (atomicExch on the bucket head) over
// insertion-indexed entry arrays. The reference scans insertion-ordered lists; the entries carry
// their log positions, and the outbox is sorted, so the order of any chain walk never shows.
#include <hip/hip_runtime.h>

#include "zb_devlib.hpp"
#include "zb_kernels.hpp"
#include "zb_msg.hpp"

namespace zbg {

__device__ __forceinline__ bool bytes_equal(const uint8_t* a, const uint8_t* b, uint32_t n) {
  for (uint32_t i = 0; i < n; i++)
    if (a[i] != b[i]) return false;
  return true;
}

// message blob: [u32 len][i64 ttl][u16 name_len][u16 ck_len][u32 payload_len][name][ck][payload]
struct MsgView {
  int64_t ttl;
  const uint8_t *name, *ck, *payload;
  uint32_t nn, nc, np;
};
__device__ __forceinline__ MsgView msg_view(const uint8_t* arena, uint32_t ref) {
  const uint8_t* b = arena + (uint64_t)ref * 8 + 4;
  MsgView v;
  v.ttl = *(const int64_t*)b;
  v.nn = *(const uint16_t*)(b + 8);
  v.nc = *(const uint16_t*)(b + 10);
  v.np = *(const uint32_t*)(b + 12);
  v.name = b + 16;
  v.ck = v.name + v.nn;
  v.payload = v.ck + v.nc;
  return v;
}

__device__ __forceinline__ void write_xchg(zb_exchange_rec* dst, int32_t kind, int32_t target, int32_t wfp, uint32_t token,
                                           int64_t wik, int64_t aik, int64_t spos, uint16_t elem, const uint8_t* name,
                                           uint32_t nn, const uint8_t* ck, uint32_t nc, const uint8_t* payload, uint32_t np) {
  zb_exchange_rec r;
  r.kind = kind; r.target_partition = target; r.wf_partition = wfp; r.token = token;
  r.workflow_instance_key = wik; r.activity_instance_key = aik; r.source_position = spos;
  r.elem = elem; r.name_len = (uint8_t)nn; r.ck_len = (uint8_t)nc; r.payload_len = (uint16_t)np; r.pad = 0;
  for (uint32_t i = 0; i < ZB_XCHG_NAME_MAX; i++) r.name[i] = i < nn ? name[i] : 0;
  for (uint32_t i = 0; i < ZB_XCHG_CK_MAX; i++) r.ck[i] = i < nc ? ck[i] : 0;
  for (uint32_t i = 0; i < ZB_XCHG_PAYLOAD_MAX; i++) r.payload[i] = i < np ? payload[i] : 0;
  *dst = r;
}

// ------------------------------------------------------------------------------ OPEN
__global__ void __launch_bounds__(256) k_msg_open(MsgParams P) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = i < P.n;
  zb_exchange_rec r;
  uint32_t ncorr = 0, best_blob = 0;
  uint64_t h = 0;
  int64_t pos = P.base + i;
  if (act) {
    r = P.in[i];
    // subscription blob (the serializer reads wfp / name / ck from it)
    const uint64_t at = P.arena_base + (uint64_t)i * SUB_BLOB;
    uint8_t* b = P.arena + at;
    *(uint32_t*)b = SUB_BLOB - 4;
    *(int32_t*)(b + 4) = r.wf_partition;
    b[8] = r.name_len; b[9] = r.ck_len;
    *(uint16_t*)(b + 10) = r.elem;
    *(uint32_t*)(b + 12) = r.token;
    for (int k = 0; k < ZB_XCHG_NAME_MAX; k++) b[16 + k] = r.name[k];
    for (int k = 0; k < ZB_XCHG_CK_MAX; k++) b[64 + k] = r.ck[k];
    const uint32_t ref = (uint32_t)(at >> 3);
    zb_rec d;
    d.key = pos;  // positionAsKey (SubscriptionApiCommandMessageHandler.java:144-149)
    d.scope_key = r.activity_instance_key;
    d.inst_key = r.workflow_instance_key;
    d.payload = ref;
    d.elem = r.elem;
    d.intent = 0;  // OPEN
    d.kind = make_kind(ZB_VT_MESSAGE_SUBSCRIPTION, ZB_RT_COMMAND, false);
    P.log[pos] = d;
    P.links[pos] = ~0ull;
    P.srcd[pos] = 0;  // delivered from another partition
    P.vlen[pos] = VLEN_UNKNOWN;
    d.intent = 1;  // OPENED: writeFollowUpEvent(record.getKey(), OPENED, subscriptionRecord)
    d.kind = make_kind(ZB_VT_MESSAGE_SUBSCRIPTION, ZB_RT_EVENT, false);
    P.log[pos + P.n] = d;
    P.links[pos + P.n] = ~0ull;
    P.srcd[pos + P.n] = (uint32_t)P.n;
    P.vlen[pos + P.n] = VLEN_UNKNOWN;
    // MessageDataStore.findMessage(name, correlationKey): the first stored message that matches
    h = name_ck_hash(r.name, r.name_len, r.ck, r.ck_len);
    int64_t best = -1;
    if (P.msg_cap) {
      for (uint32_t e = P.msg_head[h & P.msg_mask]; e != NO_ENTRY; e = P.msg_next[e]) {
        const MsgEntry m = P.msgs[e];
        if (m.h != h || m.dead) continue;
        const MsgView v = msg_view(P.arena, m.blob);
        if (v.nn != r.name_len || v.nc != r.ck_len || !bytes_equal(v.name, r.name, v.nn) ||
            !bytes_equal(v.ck, r.ck, v.nc))
          continue;
        if (best < 0 || m.pos < best) { best = m.pos; best_blob = m.blob; }
      }
    }
    ncorr = best >= 0 ? 1 : 0;
  }
  const uint32_t slot = wave_alloc(P.on, ncorr);
  if (act && ncorr) {
    const MsgView v = msg_view(P.arena, best_blob);
    if (slot >= P.ocap) atomicOr(P.err, (uint32_t)DE_LOG_FULL);
    else if (v.np > ZB_XCHG_PAYLOAD_MAX) atomicOr(P.err, (uint32_t)DE_UNSUPPORTED);
    else {
      write_xchg(P.obox + slot, ZB_XCHG_CORRELATE, r.wf_partition, r.wf_partition, r.token, r.workflow_instance_key,
                 r.activity_instance_key, pos, r.elem, r.name, r.name_len, nullptr, 0, v.payload, v.np);
      P.okeys[slot] = outbox_key(r.wf_partition, pos, 0);
    }
  }
  if (act) {
    // MessageSubscriptionDataStore.addSubscription
    const uint32_t idx = (uint32_t)(P.sub_count + i);
    SubEntry s;
    s.h = h; s.wik = r.workflow_instance_key; s.aik = r.activity_instance_key; s.pos = pos;
    s.blob = (uint32_t)((P.arena_base + (uint64_t)i * SUB_BLOB) >> 3);
    s.idx = idx;
    P.subs[idx] = s;
    P.sub_next[idx] = atomicExch(&P.sub_head[h & P.sub_mask], idx);
  }
}

// ------------------------------------------------------------------------------ PUBLISH
// Publish i of the batch: command at base + i; uniform ttl, so its follow-ups are at
// base + n + i * per (per = 1 PUBLISHED, or 2 with DELETED) and its key is key_base + i.
__global__ void __launch_bounds__(256) k_msg_publish(MsgParams P) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = i < P.n;
  const int64_t pos = P.base + i;
  uint32_t ref = 0, nmatch = 0;
  uint64_t h = 0;
  MsgView v{};
  if (act) {
    zb_rec d = P.log[pos];  // injected PUBLISH command (payload = message blob)
    ref = d.payload;
    v = msg_view(P.arena, ref);
    h = name_ck_hash(v.name, v.nn, v.ck, v.nc);
    const int per = P.ttl > 0 ? 1 : 2;
    const int64_t key = P.key_base + i;
    const int64_t fpos = P.base + P.n + i * per;
    d.key = key;
    d.intent = 1;  // PUBLISHED (batchWriter.addNewEvent)
    d.kind = make_kind(ZB_VT_MESSAGE, ZB_RT_EVENT, false);
    P.log[fpos] = d;
    P.links[fpos] = ~0ull;
    P.srcd[fpos] = (uint32_t)(fpos - pos);
    P.vlen[fpos] = VLEN_UNKNOWN;
    if (per == 2) {  // ttl <= 0: addFollowUpEvent(key, DELETED, messageRecord)
      d.intent = 3;
      d.kind = make_kind(ZB_VT_MESSAGE, ZB_RT_EVENT, true);
      P.log[fpos + 1] = d;
      P.links[fpos + 1] = ~0ull;
      P.srcd[fpos + 1] = (uint32_t)(fpos + 1 - pos);
      P.vlen[fpos + 1] = VLEN_UNKNOWN;
    }
    for (uint32_t e = P.sub_head[h & P.sub_mask]; e != NO_ENTRY; e = P.sub_next[e]) {
      const SubEntry s = P.subs[e];
      if (s.h != h) continue;
      const uint8_t* sb = P.arena + (uint64_t)s.blob * 8;
      if (sb[8] != v.nn || sb[9] != v.nc || !bytes_equal(sb + 16, v.name, v.nn) || !bytes_equal(sb + 64, v.ck, v.nc))
        continue;
      nmatch++;
    }
    if (nmatch && v.np > ZB_XCHG_PAYLOAD_MAX) { atomicOr(P.err, (uint32_t)DE_UNSUPPORTED); nmatch = 0; }
  }
  uint32_t slot = wave_alloc(P.on, nmatch);
  if (act && nmatch) {
    for (uint32_t e = P.sub_head[h & P.sub_mask]; e != NO_ENTRY; e = P.sub_next[e]) {
      const SubEntry s = P.subs[e];
      if (s.h != h) continue;
      const uint8_t* sb = P.arena + (uint64_t)s.blob * 8;
      if (sb[8] != v.nn || sb[9] != v.nc || !bytes_equal(sb + 16, v.name, v.nn) || !bytes_equal(sb + 64, v.ck, v.nc))
        continue;
      const int32_t wfp = *(const int32_t*)(sb + 4);
      if (slot >= P.ocap) { atomicOr(P.err, (uint32_t)DE_LOG_FULL); break; }
      write_xchg(P.obox + slot, ZB_XCHG_CORRELATE, wfp, wfp, *(const uint32_t*)(sb + 12), s.wik, s.aik, pos,
                 *(const uint16_t*)(sb + 10), v.name, v.nn, nullptr, 0, v.payload, v.np);
      P.okeys[slot] = outbox_key(wfp, pos, s.idx);  // findSubscriptions: insertion order
      slot++;
    }
  }
  if (act && P.ttl > 0) {  // messageStore.addMessage
    const uint32_t idx = (uint32_t)(P.msg_count + i);
    MsgEntry m;
    m.h = h; m.key = P.key_base + i; m.pos = pos; m.blob = ref; m.dead = 0;
    P.msgs[idx] = m;
    P.msg_next[idx] = atomicExch(&P.msg_head[h & P.msg_mask], idx);
  }
}

// ------------------------------------------------------------------------------ CORRELATE inbox
__global__ void __launch_bounds__(256) k_wis_inject(MsgParams P) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P.n) return;
  const zb_exchange_rec r = P.in[i];
  const int64_t pos = P.base + i;
  const uint64_t at = P.arena_base + (uint64_t)i * WIS_BLOB;
  uint8_t* b = P.arena + at;
  uint32_t np = r.payload_len;
  if (np == 0 || (np == 1 && r.payload[0] == 0xc0)) {  // DocumentValue: nil / empty -> {}
    np = 1;
    b[4] = 0x80;
  } else {
    for (uint32_t k = 0; k < np && k < ZB_XCHG_PAYLOAD_MAX; k++) b[4 + k] = r.payload[k];
  }
  *(uint32_t*)b = np;
  zb_rec d;
  d.key = pos;  // positionAsKey (SubscriptionApiCommandMessageHandler.java:144-149)
  d.scope_key = r.activity_instance_key;
  d.inst_key = r.workflow_instance_key;
  d.payload = (uint32_t)(at >> 3);
  d.elem = r.elem;
  d.intent = 0;  // CORRELATE
  d.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE_SUBSCRIPTION, ZB_RT_COMMAND, false);
  P.log[pos] = d;
  // row_self: found by activity instance key (k_resolve after this kernel; the sender's row token can be stale
  // once the workflow partition compacted its rows)
  P.links[pos] = ~0ull;
  P.srcd[pos] = 0;
  P.vlen[pos] = VLEN_UNKNOWN;
  P.lookup_keys[i] = r.activity_instance_key;
  P.lookup_pos[i] = pos;
}

// ------------------------------------------------------------------------------ outbox
__global__ void k_outbox_gather(const zb_exchange_rec* src, const uint32_t* idx, zb_exchange_rec* dst, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[idx[i]];
}
// first sorted index of every target partition (targets are the key's top 6 bits)
__global__ void k_outbox_bounds(const uint64_t* keys, uint64_t n, uint64_t* first, int parts) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int t = (int)(keys[i] >> 58);
  const int tp = i == 0 ? -1 : (int)(keys[i - 1] >> 58);
  for (int q = tp + 1; q <= t && q < parts; q++) first[q] = i;
  if (i == n - 1)
    for (int q = t + 1; q < parts; q++) first[q] = n;
}
__global__ void k_iota(uint32_t* p, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = (uint32_t)i;
}

static unsigned blocks(int64_t n) { return (unsigned)((n + 255) / 256); }

void launch_msg_open(const MsgParams& p, hipStream_t s) {
  if (p.n > 0) hipLaunchKernelGGL(k_msg_open, dim3(blocks(p.n)), dim3(256), 0, s, p);
}
void launch_msg_publish(const MsgParams& p, hipStream_t s) {
  if (p.n > 0) hipLaunchKernelGGL(k_msg_publish, dim3(blocks(p.n)), dim3(256), 0, s, p);
}
void launch_wis_inject(const MsgParams& p, hipStream_t s) {
  if (p.n > 0) hipLaunchKernelGGL(k_wis_inject, dim3(blocks(p.n)), dim3(256), 0, s, p);
}
void launch_outbox_gather(const zb_exchange_rec* src, const uint32_t* idx, zb_exchange_rec* dst, uint64_t n,
                          hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_outbox_gather, dim3(blocks((int64_t)n)), dim3(256), 0, s, src, idx, dst, n);
}
void launch_outbox_bounds(const uint64_t* keys, uint64_t n, uint64_t* first, int parts, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_outbox_bounds, dim3(blocks((int64_t)n)), dim3(256), 0, s, keys, n, first, parts);
}
void launch_iota(uint32_t* p, uint64_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_iota, dim3(blocks((int64_t)n)), dim3(256), 0, s, p, n);
}

}  // namespace zbg
