// zb_msg.hip — the message stream processor (MessageService.java:90-129) and
// the partition exchange (zb_exchange_rec batches, include/zb_engine.h).
//
//   k_msg_open      MESSAGE_SUBSCRIPTION OPEN commands delivered by workflow partitions: append the command
//                   (key = its log position) and its OPENED event, look for a stored message
//                   (MessageDataStore.findMessage: the first stored one), insert the subscription
//                   (MessageSubscriptionDataStore.addSubscription) — OpenMessageSubscriptionProcessor.java:56-92
//   k_pub_count     a run of PUBLISH commands, per command: rejected (a message with its id, name and correlation
//                   key is stored: MessageDataStore.hasMessage) or accepted; records written; stored
//   k_pub_emit      PublishMessageProcessor.java:58-124 at the scanned offsets: the rejection (BAD_VALUE), or
//                   PUBLISHED (+ DELETED when ttl <= 0) keyed by the message KeyGenerator(0, 1), a correlate command
//                   per matching subscription (findSubscriptions, insertion order), the message stored when ttl > 0
//   k_msg_delete    a run of DELETE commands: DELETED, the message removed (DeleteMessageProcessor.java:36-45)
//   k_ttl_flags / k_ttl_write   MessageTimeToLiveChecker.run (:44-68): a DELETE command per stored message whose
//                   deadline has passed, in store order
//   k_wis_inject    CORRELATE commands delivered by message partitions -> WORKFLOW_INSTANCE_SUBSCRIPTION
//                   CORRELATE commands at the log tail (processed by the wave pipeline, zb_wave.hip)
//   k_outbox_*      the outbox sorted by (target, source position, emission) into one exchange batch per target
//
// The stores are hash tables of chains pushed lock-free (atomicExch on the bucket head) over insertion-indexed
// entry arrays. The reference scans insertion-ordered lists; entries carry their log positions / insertion
// indices and the outbox is sorted, so the order of a chain walk never shows. Stored messages are in key order
// (keys are handed out in command order), so DELETE finds its message by binary search.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "zb_devlib.hpp"
#include "zb_kernels.hpp"
#include "zb_msg.hpp"

namespace zbg {

__device__ __forceinline__ bool bytes_equal(const uint8_t* a, const uint8_t* b, uint32_t n) {
  for (uint32_t i = 0; i < n; i++)
    if (a[i] != b[i]) return false;
  return true;
}
// n bytes at two 8-aligned addresses inside 8-aligned arena blobs, compared a word at a time (the last word's bytes
// past n -- still inside both blobs -- are masked off)
__device__ __forceinline__ bool words_equal(const uint8_t* a, const uint8_t* b, uint32_t n) {
  const uint64_t* wa = (const uint64_t*)a;
  const uint64_t* wb = (const uint64_t*)b;
  uint64_t diff = 0;
  uint32_t k = 0;
  for (; k + 8 <= n; k += 8) diff |= wa[k / 8] ^ wb[k / 8];
  if (k < n) diff |= (wa[k / 8] ^ wb[k / 8]) & ((1ull << (8 * (n - k))) - 1);
  return diff == 0;
}

__device__ __forceinline__ void put_record(const MsgParams& P, int64_t pos, const zb_rec& d, uint32_t srcd) {
  P.log[pos] = d;
  P.links[pos] = ~0ull;
  P.srcd[pos] = srcd;
  P.vlen[pos] = VLEN_UNKNOWN;
}

// command i of the delivered batches: its header and its variable bytes
__device__ __forceinline__ zb_exchange_rec delivered(const MsgParams& P, int64_t i, const uint8_t*& var) {
  int lo = 0, hi = P.nslices - 1;
  while (lo < hi) {  // last batch whose first command is <= i
    const int mid = (lo + hi + 1) >> 1;
    if ((int64_t)P.slice_first[mid] <= i) lo = mid;
    else hi = mid - 1;
  }
  const uint8_t* bat = P.in + P.slice_off[lo];
  const uint64_t cnt = *(const uint64_t*)bat;
  const zb_exchange_rec r = ((const zb_exchange_rec*)(bat + ZB_XCHG_BATCH_HEADER))[i - (int64_t)P.slice_first[lo]];
  var = bat + ZB_XCHG_BATCH_HEADER + cnt * sizeof(zb_exchange_rec) + r.var_offset;
  return r;
}

__device__ __forceinline__ void flag_error(const MsgParams& P, uint32_t err) {
  if (err) atomicOr(P.err, err);
}

// ------------------------------------------------------------------------------ OPEN
__global__ void __launch_bounds__(256) k_msg_open(MsgParams P) {
  __shared__ uint32_t s_alloc[2 * (256 / 64) + 2];
  __shared__ uint64_t s_alloc64[256 / 64 + 1];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = i < P.n;
  uint32_t err = 0, ncorr = 0, best_blob = 0, gran = 0;
  uint64_t h = 0;
  const int64_t pos = P.base + i;
  zb_exchange_rec r{};
  const uint8_t* var = nullptr;
  uint32_t sref = 0;
  if (act) r = delivered(P, i, var);
  // the subscription blob (the serializer and the store read wf partition / name / correlation key from it)
  const uint32_t blen = SUB_HDR - 4 + r.name_len + r.ck_len;
  const uint64_t bbytes = act ? ((4 + (uint64_t)blen + 7) & ~7ull) : 0;
  const uint64_t bat = block_alloc64<256>((unsigned long long*)&P.hdr->arena_next, bbytes, s_alloc64);
  if (act) {
    const uint8_t* name = var;
    const uint8_t* ck = var + r.name_len;
    uint8_t* b = nullptr;
    if (bat + bbytes > P.arena_cap) err |= DE_ARENA_FULL;
    else {
      b = P.arena + bat;
      sref = (uint32_t)(bat >> 3);
      WordWriter w(b);  // (the SUB_HDR words, then name + key: contiguous in the batch's variable bytes)
      w.push((uint64_t)blen | (uint64_t)(uint32_t)r.wf_partition << 32, 8);
      w.push((uint64_t)r.token | (uint64_t)r.elem << 32, 8);
      w.push((uint64_t)r.name_len | (uint64_t)r.ck_len << 32, 8);
      w.bytes(name, r.name_len + r.ck_len);
      w.finish();
    }
    zb_rec d;
    d.key = pos;  // positionAsKey (SubscriptionApiCommandMessageHandler.java:144-149)
    d.scope_key = r.activity_instance_key;
    d.inst_key = r.workflow_instance_key;
    d.payload = sref;
    d.elem = r.elem;
    d.intent = 0;  // OPEN
    d.kind = make_kind(ZB_VT_MESSAGE_SUBSCRIPTION, ZB_RT_COMMAND, false);
    put_record(P, pos, d, 0);  // delivered from another partition
    d.intent = 1;  // OPENED: writeFollowUpEvent(record.getKey(), OPENED, subscriptionRecord)
    d.kind = make_kind(ZB_VT_MESSAGE_SUBSCRIPTION, ZB_RT_EVENT, false);
    put_record(P, pos + P.n, d, (uint32_t)P.n);
    // MessageDataStore.findMessage(name, correlationKey): the first stored message that matches
    h = name_ck_hash(name, r.name_len, ck, r.ck_len);
    int64_t best = -1;
    if (P.msg_cap) {
      for (uint32_t e = P.msg_head[h & P.msg_mask]; e != NO_ENTRY; e = P.msg_next[e]) {
        const MsgEntry m = P.msgs[e];
        if (m.h != h || m.dead) continue;
        const MsgView v = msg_view(P.arena, m.blob);
        if (v.nn != r.name_len || v.nc != r.ck_len) continue;
        if (b ? !words_equal(v.name, b + SUB_HDR, v.nn + v.nc)  // (name + key contiguous in both blobs, 8-aligned)
              : (!bytes_equal(v.name, name, v.nn) || !bytes_equal(v.ck, ck, v.nc)))
          continue;
        if (best < 0 || m.pos < best) { best = m.pos; best_blob = m.blob; }
      }
    }
    if (best >= 0) {
      ncorr = 1;
      gran = var_granules(r.name_len, 0, msg_view(P.arena, best_blob).np);
    }
  }
  uint32_t slot, vat;
  block_alloc2<256>(P.ob.n, ncorr, P.ob.var_n, gran, s_alloc, slot, vat);
  if (act && ncorr) {
    const MsgView v = msg_view(P.arena, best_blob);
    if (slot >= P.ob.cap || (uint64_t)vat + gran > P.ob.var_cap) err |= DE_LOG_FULL;
    else if (!outbox_write(P.ob, slot, vat, ZB_XCHG_CORRELATE, r.wf_partition, r.wf_partition, r.token,
                           r.workflow_instance_key, r.activity_instance_key, pos, r.elem, var, r.name_len, nullptr, 0,
                           v.payload, v.np, 0))
      err |= DE_UNSUPPORTED;
  }
  if (act) {  // MessageSubscriptionDataStore.addSubscription
    const uint32_t idx = (uint32_t)(P.sub_count + i);
    SubEntry s;
    s.h = h; s.wik = r.workflow_instance_key; s.aik = r.activity_instance_key; s.pos = pos; s.blob = sref; s.idx = idx;
    P.subs[idx] = s;
    P.sub_next[idx] = atomicExch(&P.sub_head[h & P.sub_mask], idx);
  }
  flag_error(P, err);
}

// ------------------------------------------------------------------------------ PUBLISH
// per command: [20:0] records written, [41:21] accepted (a message key), [62:42] stored (ttl > 0)
constexpr int PC_ACC = 21, PC_STORED = 42;
constexpr uint64_t PC_MASK = (1ull << 21) - 1;

__global__ void __launch_bounds__(256) k_pub_count(MsgParams P) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P.n) return;
  const zb_rec d = P.log[P.base + i];
  const MsgView v = msg_view(P.arena, d.payload);
  bool rejected = false;
  if (v.nid) {  // messageRecord.hasMessageId() && messageStore.hasMessage(message) (PublishMessageProcessor :77-84)
    rejected = P.prior[i] != 0;
    if (!rejected && P.msg_cap) {
      const uint64_t h = name_ck_hash(v.name, v.nn, v.ck, v.nc);
      for (uint32_t e = P.msg_head[h & P.msg_mask]; e != NO_ENTRY && !rejected; e = P.msg_next[e]) {
        const MsgEntry m = P.msgs[e];
        if (m.h != h || m.dead) continue;
        const MsgView s = msg_view(P.arena, m.blob);
        rejected = s.nid == v.nid && s.nn == v.nn && s.nc == v.nc && bytes_equal(s.id, v.id, v.nid) &&
                   bytes_equal(s.name, v.name, v.nn) && bytes_equal(s.ck, v.ck, v.nc);
      }
    }
  }
  const uint64_t out = rejected ? 1 : (v.ttl > 0 ? 1 : 2);
  const uint64_t acc = rejected ? 0 : 1, stored = (!rejected && v.ttl > 0) ? 1 : 0;
  P.cnt[i] = out | (acc << PC_ACC) | (stored << PC_STORED);
}

__device__ __forceinline__ bool sub_matches(const SubView& sb, const MsgView& v) {
  // (name + correlation key are contiguous and 8-aligned in both blobs: SUB_HDR, MSG_HDR)
  return sb.nn == v.nn && sb.nc == v.nc && words_equal(sb.name, v.name, v.nn + v.nc);
}

__global__ void __launch_bounds__(256) k_pub_emit(MsgParams P) {
  __shared__ uint32_t s_alloc[2 * (256 / 64) + 2];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = i < P.n;
  const int64_t pos = P.base + i;
  uint32_t err = 0, nmatch = 0, gran = 0;
  uint64_t h = 0;
  zb_rec d{};
  MsgView v{};
  bool acc = false;
  uint64_t off = 0;
  uint32_t e1 = NO_ENTRY;  // the first matching subscription of the chain
  uint32_t idx0 = 0xffffffffu;  // the smallest store index among the matches
  if (act) {
    d = P.log[pos];
    v = msg_view(P.arena, d.payload);
    if (P.uni_out) {  // (the closed form of k_pub_count + scan for a batch without message ids)
      acc = true;
      off = (uint64_t)i * (uint64_t)P.uni_out | (uint64_t)i << PC_ACC | (P.uni_out == 1 ? (uint64_t)i << PC_STORED : 0);
    } else {
      acc = (P.cnt[i] >> PC_ACC) & 1;
      off = P.cnt_off[i];
    }
    const int64_t fpos = P.out_base + (int64_t)(off & PC_MASK);
    zb_rec f = d;  // follow-ups re-encode record.getValue(): the message blob, not the verbatim command value
    if (!acc) {  // writeRejection(record, BAD_VALUE, "message with id '%s' is already published")
      f.kind = make_kind(ZB_VT_MESSAGE, ZB_RT_COMMAND_REJECTION, false);
      put_record(P, fpos, f, (uint32_t)(fpos - pos));
    } else {
      f.key = P.key_base + (int64_t)((off >> PC_ACC) & PC_MASK);
      f.intent = 1;  // PUBLISHED (batchWriter.addNewEvent)
      f.kind = make_kind(ZB_VT_MESSAGE, ZB_RT_EVENT, false);
      put_record(P, fpos, f, (uint32_t)(fpos - pos));
      if (v.ttl <= 0) {  // addFollowUpEvent(key, DELETED, messageRecord): never stored
        f.intent = 3;
        f.kind = make_kind(ZB_VT_MESSAGE, ZB_RT_EVENT, true);
        put_record(P, fpos + 1, f, (uint32_t)(fpos + 1 - pos));
      }
      h = name_ck_hash(v.name, v.nn, v.ck, v.nc);
      for (uint32_t e = P.sub_head[h & P.sub_mask]; e != NO_ENTRY; e = P.sub_next[e]) {
        const SubEntry s = P.subs[e];
        if (s.h == h && sub_matches(sub_view(P.arena, s.blob), v)) {
          if (nmatch++ == 0) e1 = e;
          idx0 = s.idx < idx0 ? s.idx : idx0;
        }
      }
      gran = nmatch * var_granules(v.nn, 0, v.np);
    }
  }
  uint32_t slot, vat;
  block_alloc2<256>(P.ob.n, nmatch, P.ob.var_n, gran, s_alloc, slot, vat);
  if (act && nmatch) {  // correlateMessage :107-124: one command per matching subscription
    const uint32_t g = var_granules(v.nn, 0, v.np);
    uint32_t left = nmatch;
    for (uint32_t e = e1; e != NO_ENTRY && left; e = P.sub_next[e]) {
      const SubEntry s = P.subs[e];
      if (s.h != h) continue;
      const SubView sb = sub_view(P.arena, s.blob);
      if (e != e1 && !sub_matches(sb, v)) continue;
      left--;
      if (slot >= P.ob.cap || (uint64_t)vat + g > P.ob.var_cap) { err |= DE_LOG_FULL; break; }
      // emission order = findSubscriptions' insertion order: the subscription's rank by store index among this
      // message's matches (a few bits: the outbox sort then covers the positions and little more), or, for a message
      // with many matches, its store index past the smallest of them (the same order; outbox_write refuses a span
      // past 2^24 entries instead of wrapping it)
      uint32_t em = 0;
      if (nmatch > 32) em = s.idx - idx0;
      else if (nmatch > 1)
        for (uint32_t e2 = e1; e2 != NO_ENTRY; e2 = P.sub_next[e2]) {
          const SubEntry s2 = P.subs[e2];
          if (s2.h == h && s2.idx < s.idx && sub_matches(sub_view(P.arena, s2.blob), v)) em++;
        }
      if (!outbox_write(P.ob, slot, vat, ZB_XCHG_CORRELATE, sb.wfp, sb.wfp, sb.token, s.wik, s.aik, pos, sb.elem, v.name,
                        v.nn, nullptr, 0, v.payload, v.np, em)) {
        err |= DE_UNSUPPORTED;
        break;
      }
      slot++;
      vat += g;
    }
  }
  if (act && acc && v.ttl > 0) {  // messageStore.addMessage (deadline = timeToLive + now)
    const uint64_t idx = P.msg_count + ((off >> PC_STORED) & PC_MASK);
    if (idx >= P.msg_cap) err |= DE_LOG_FULL;
    else {
      MsgEntry m;
      m.h = h; m.key = P.key_base + (int64_t)((off >> PC_ACC) & PC_MASK); m.pos = pos; m.deadline = v.ttl + P.clock;
      m.blob = d.payload; m.dead = 0;
      *(int64_t*)(P.arena + (uint64_t)d.payload * 8 + 16) = m.deadline;
      P.msgs[idx] = m;
      P.msg_next[idx] = atomicExch(&P.msg_head[h & P.msg_mask], (uint32_t)idx);
    }
  }
  flag_error(P, err);
}

// ------------------------------------------------------------------------------ DELETE
__global__ void __launch_bounds__(256) k_msg_delete(MsgParams P) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= P.n) return;
  const int64_t pos = P.base + j, fpos = P.out_base + j;
  zb_rec f = P.log[pos];
  f.kind = make_kind(ZB_VT_MESSAGE, ZB_RT_EVENT, false);  // writeFollowUpEvent(record.getKey(), DELETED, value)
  f.intent = 3;
  put_record(P, fpos, f, (uint32_t)(fpos - pos));
  // messageStore.removeMessage(key): entries are in key order
  int64_t lo = 0, hi = (int64_t)P.msg_count - 1;
  while (lo <= hi) {
    const int64_t mid = (lo + hi) >> 1;
    const int64_t k = P.msgs[mid].key;
    if (k == f.key) {
      P.msgs[mid].dead = 1;
      break;
    }
    if (k < f.key) lo = mid + 1;
    else hi = mid - 1;
  }
}

// ------------------------------------------------------------------------------ time to live
__global__ void __launch_bounds__(256) k_ttl_flags(MsgParams P) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i <= P.msg_count; i += stride)
    P.flags[i] = (i < P.msg_count && !P.msgs[i].dead && P.msgs[i].deadline <= P.now) ? 1u : 0u;
}
// writeFollowUpCommand(message.getKey(), DELETE, command) by the checker's own command writer (no source)
__global__ void __launch_bounds__(256) k_ttl_write(MsgParams P) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < P.msg_count; i += stride) {
    const MsgEntry m = P.msgs[i];
    if (m.dead || m.deadline > P.now) continue;
    zb_rec d;
    d.key = m.key;
    d.scope_key = -1;
    d.inst_key = -1;
    d.payload = m.blob;
    d.elem = NO_ELEM;
    d.intent = 2;  // DELETE
    d.kind = make_kind(ZB_VT_MESSAGE, ZB_RT_COMMAND, false);
    put_record(P, P.base + (int64_t)P.flag_off[i], d, 0);
  }
}

// ------------------------------------------------------------------------------ CORRELATE inbox
__global__ void __launch_bounds__(256) k_wis_inject(MsgParams P) {
  __shared__ uint64_t s_alloc64[256 / 64 + 1];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = i < P.n;
  const uint8_t* var = nullptr;
  zb_exchange_rec r{};
  if (act) r = delivered(P, i, var);
  const uint8_t* pl = var + r.name_len + r.ck_len;
  const uint32_t np = r.payload_len;
  const bool empty = act && (np == 0 || (np == 1 && pl[0] == 0xc0));  // DocumentValue: nil / empty -> {}
  const uint32_t blen = empty ? 1 : np;
  const uint64_t bbytes = act ? ((4 + (uint64_t)blen + 7) & ~7ull) : 0;
  const uint64_t bat = block_alloc64<256>((unsigned long long*)&P.hdr->arena_next, bbytes, s_alloc64);
  if (!act) return;
  uint32_t err = 0, ref = 0;
  uint8_t* b = nullptr;
  if (bat + bbytes > P.arena_cap) err |= DE_ARENA_FULL;
  else {
    b = P.arena + bat;
    ref = (uint32_t)(bat >> 3);
    WordWriter w(b);
    w.push(blen, 4);
    if (empty) w.push(0x80, 1);
    else w.bytes(pl, np);
    w.finish();
  }
  const int64_t pos = P.base + i;
  zb_rec d;
  d.key = pos;  // positionAsKey (SubscriptionApiCommandMessageHandler.java:144-149)
  d.scope_key = r.activity_instance_key;
  d.inst_key = r.workflow_instance_key;
  d.payload = ref;
  d.elem = r.elem;
  d.intent = 0;  // CORRELATE
  d.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE_SUBSCRIPTION, ZB_RT_COMMAND, false);
  put_record(P, pos, d, 0);
  // row_self (ElementInstanceIndex.getInstance(activityInstanceKey)): the row the subscription's token names when it
  // is live and holds the key -- rows are never reused and a key names at most one live row, so that row is the
  // instance. A token from another partition's numbering, or stale after this partition compacted its rows, is
  // counted instead: the host then sorts the keys and k_resolve searches the rows for them.
  const uint32_t t = r.token;
  const bool hit = t < P.rows && P.rmeta[t].state != 0 && P.rkeys[t].key == r.activity_instance_key;
  if (hit) P.links[pos] = 0xffffffff00000000ull | t;  // (the row-self half; no parent link)
  const uint64_t miss = __ballot(!hit);
  if (miss && (threadIdx.x & 63) == (uint32_t)(__ffsll((unsigned long long)__ballot(1)) - 1))
    atomicAdd(P.unresolved, (uint32_t)__popcll(miss));
  P.lookup_keys[i] = r.activity_instance_key;
  P.lookup_pos[i] = pos;
  flag_error(P, err);
}

// ------------------------------------------------------------------------------ outbox take
__global__ void k_outbox_sizes(Outbox ob, const uint32_t* idx, uint64_t n, uint32_t* sizes) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n) return;
  if (i == n) { sizes[n] = 0; return; }
  const zb_exchange_rec& r = ob.rec[idx[i]];
  sizes[i] = var_granules(r.name_len, r.ck_len, r.payload_len);
}
// first sorted index of every target partition (targets are the key's top 6 bits); first[parts] = n
__global__ void k_outbox_bounds(const uint64_t* keys, uint64_t n, uint64_t* first, int parts) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int t = (int)(keys[i] >> 58);
  const int tp = i == 0 ? -1 : (int)(keys[i - 1] >> 58);
  for (int q = tp + 1; q <= t && q < parts; q++) first[q] = i;
  if (i == n - 1)
    for (int q = t + 1; q <= parts; q++) first[q] = n;
}
// per target: (commands, variable granules)
__global__ void k_outbox_table(const uint64_t* first, const uint32_t* goff, int parts, uint64_t* table) {
  const int q = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (q >= parts) return;
  table[2 * q] = first[q + 1] - first[q];
  table[2 * q + 1] = (uint64_t)goff[first[q + 1]] - (uint64_t)goff[first[q]];
}
// sorted command i into its target's batch at dst + base[target]
__global__ void k_outbox_pack(Outbox ob, const uint32_t* idx, const uint64_t* keys, uint64_t n, const uint64_t* first,
                              const uint32_t* goff, const uint64_t* base, uint8_t* dst) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int q = (int)(keys[i] >> 58);
  const uint64_t f = first[q], cnt = first[q + 1] - f;
  uint8_t* bat = dst + base[q];
  const uint64_t var_bytes = 8 * ((uint64_t)goff[first[q + 1]] - (uint64_t)goff[f]);
  if (i == f) {
    ((uint64_t*)bat)[0] = cnt;
    ((uint64_t*)bat)[1] = ZB_XCHG_BATCH_HEADER + cnt * sizeof(zb_exchange_rec) + var_bytes;
  }
  zb_exchange_rec r = ob.rec[idx[i]];
  const uint64_t* src = (const uint64_t*)(ob.var + r.var_offset);
  r.var_offset = 8 * ((uint64_t)goff[i] - (uint64_t)goff[f]);
  ((zb_exchange_rec*)(bat + ZB_XCHG_BATCH_HEADER))[i - f] = r;
  uint64_t* vd = (uint64_t*)(bat + ZB_XCHG_BATCH_HEADER + cnt * sizeof(zb_exchange_rec) + r.var_offset);
  const uint32_t g = var_granules(r.name_len, r.ck_len, r.payload_len);
  for (uint32_t k = 0; k < g; k++) vd[k] = src[k];
}
// ---- zb_submit_publishes on the device. The blob layout is zb_msg.hpp's MsgView (no message id, deadline set
// when the message is stored); an empty or nil payload document becomes {} (PublishMessageProcessor: payload
// defaults to the empty document), anything but a map is the reference's "Document has invalid format" rejection
__global__ void k_pub_sizes(PubBuild p) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > p.n) return;
  if (i == p.n) { p.gran[i] = 0; return; }
  const uint64_t nc = p.ck_off[i + 1] - p.ck_off[i];
  const uint8_t* pl = p.pls + (p.pl_off[i] - p.pl_off[0]);
  uint64_t np = p.pl_off[i + 1] - p.pl_off[i];
  if (np == 0 || (np == 1 && pl[0] == 0xc0)) np = 1;
  else if (!((pl[0] & 0xf0) == 0x80 || pl[0] == 0xde || pl[0] == 0xdf)) atomicOr(p.err, 1u);
  if (nc > 0xffffffffull || np > 0xffffffffull) atomicOr(p.err + 1, 1u);
  p.gran[i] = (MSG_HDR + p.nn + nc + np + 7) >> 3;
}
__global__ void k_pub_build(PubBuild p) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  const uint64_t at = p.arena0 + p.goff[i] * 8;
  uint8_t* b = p.arena + at;
  const uint8_t* ck = p.cks + (p.ck_off[i] - p.ck_off[0]);
  const uint32_t nc = (uint32_t)(p.ck_off[i + 1] - p.ck_off[i]);
  const uint8_t* pl = p.pls + (p.pl_off[i] - p.pl_off[0]);
  uint32_t np = (uint32_t)(p.pl_off[i + 1] - p.pl_off[i]);
  const bool empty = np == 0 || (np == 1 && pl[0] == 0xc0);
  if (empty) np = 1;
  const uint32_t len = MSG_HDR - 4 + p.nn + nc + np;
  WordWriter w(b);  // MSG_HDR, then name, correlation key, payload (and the zero padding) as whole 8-byte words
  w.push((uint64_t)len | (uint64_t)p.nn << 32, 8);
  w.push((uint64_t)p.ttl, 8);
  w.push(0, 8);  // deadline: set when the message is stored
  w.push((uint64_t)nc | (uint64_t)np << 32, 8);
  w.push(0, 8);  // (no message id; pad)
  w.bytes(p.name, p.nn);
  w.bytes(ck, nc);
  if (empty) w.push(0x80, 1);
  else w.bytes(pl, np);
  w.finish();
  zb_rec r;
  r.key = -1; r.scope_key = -1; r.inst_key = -1;
  r.payload = (uint32_t)(at >> 3);
  r.elem = NO_ELEM; r.intent = 0;  // PUBLISH
  r.kind = make_kind(ZB_VT_MESSAGE, ZB_RT_COMMAND, false);
  p.out[i] = r;
  p.links[i] = ~0ull;
  p.srcd[i] = 0;             // (submitted: no source record)
  p.vlen[i] = VLEN_UNKNOWN;  // (the size pass measures it)
}

// the outbox order by counting: the keys of one take differ only in the bits of their spread (k_key_spread), and a
// take's keys are distinct (a source position emits one command per emission index), so a command's slot is the
// exclusive scan of the per-bucket counts over those bits -- one histogram, one scan, one scatter instead of the
// radix sort's passes. A bucket holds (commands << 40 | variable granules): one atomic gives a command both its slot
// and its variable bytes' place (equal keys, were there any, keep no particular order: neither did the outbox slots)
constexpr int CS_SHIFT = 40;
__global__ void __launch_bounds__(256) k_cs_hist(Outbox ob, uint64_t n, int begin, uint64_t mask,
                                                 unsigned long long* cnt) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const zb_exchange_rec& r = ob.rec[i];
  const uint32_t g = var_granules(r.name_len, r.ck_len, r.payload_len);
  atomicAdd(&cnt[(ob.keys[i] >> begin) & mask], (1ull << CS_SHIFT) | g);
}
// every command's slot in key order: its key and index (kout may be null), and with goff its variable granules' place
__global__ void __launch_bounds__(256) k_cs_scatter(Outbox ob, uint64_t n, int begin, uint64_t mask,
                                                    unsigned long long* off, uint64_t* kout, uint32_t* vout,
                                                    uint32_t* goff) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t k = ob.keys[i];
  uint64_t add = 1ull << CS_SHIFT;
  if (goff) {
    const zb_exchange_rec& r = ob.rec[i];
    add |= var_granules(r.name_len, r.ck_len, r.payload_len);
  }
  const uint64_t o = atomicAdd(&off[(k >> begin) & mask], add);
  const uint64_t p = o >> CS_SHIFT;
  if (kout) kout[p] = k;
  vout[p] = (uint32_t)i;
  if (goff) goff[p] = (uint32_t)(o & ((1ull << CS_SHIFT) - 1));
}
// a partition delivering to itself: its one exchange batch, written in key order (coalesced stores: the records and
// their variable bytes are read where the outbox holds them); the outbox is taken
__global__ void __launch_bounds__(256) k_local_pack(Outbox ob, const uint32_t* idx, const uint32_t* goff, uint64_t n,
                                                    uint64_t total, uint8_t* dst, uint32_t* taken_n,
                                                    uint32_t* taken_var) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) {  // the batch header; the outbox is taken (stream order: nothing in flight reads the counters)
    ((uint64_t*)dst)[0] = n;
    ((uint64_t*)dst)[1] = total;
    *taken_n = 0;
    *taken_var = 0;
  }
  if (i >= n) return;
  zb_exchange_rec r = ob.rec[idx[i]];
  const uint32_t g = var_granules(r.name_len, r.ck_len, r.payload_len);
  const uint64_t* src = (const uint64_t*)(ob.var + r.var_offset);
  r.var_offset = 8 * (uint64_t)goff[i];
  ((zb_exchange_rec*)(dst + ZB_XCHG_BATCH_HEADER))[i] = r;
  uint64_t* vd = (uint64_t*)(dst + ZB_XCHG_BATCH_HEADER + n * sizeof(zb_exchange_rec) + r.var_offset);
  for (uint32_t k = 0; k < g; k++) vd[k] = src[k];
}

__global__ void k_iota(uint32_t* p, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = (uint32_t)i;
}

// the key bits that differ between the keys of a sort: OR over i of keys[i] ^ keys[0] (the radix sort then runs over
// [lowest, highest] of them only). n_dev: the count is read on the device (min(*n_dev, n)), so that the host reads the
// spread in the same round trip as the count
__global__ void __launch_bounds__(256) k_key_spread(const uint64_t* keys, uint64_t n, unsigned long long* out,
                                                    const uint32_t* n_dev) {
  if (n_dev) n = std::min<uint64_t>(n, *n_dev);
  if (n == 0) return;
  __shared__ uint64_t s[4];
  const uint64_t k0 = keys[0];
  uint64_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    acc |= keys[i] ^ k0;
  for (int o = 32; o > 0; o >>= 1) acc |= (uint64_t)__shfl_xor((unsigned long long)acc, o, 64);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
  __syncthreads();
  // one atomic per workgroup (same-address atomics serialize)
  if (threadIdx.x == 0 && (s[0] | s[1] | s[2] | s[3])) atomicOr(out, (unsigned long long)(s[0] | s[1] | s[2] | s[3]));
}

static unsigned blocks(int64_t n) { return (unsigned)((n + 255) / 256); }
static unsigned grid_cap(uint64_t n) {
  const uint64_t g = (n + 255) / 256;
  return (unsigned)(g < 1 ? 1 : (g > 4096 ? 4096 : g));
}

void launch_pub_sizes(const PubBuild& p, hipStream_t s) {
  hipLaunchKernelGGL(k_pub_sizes, dim3(blocks((int64_t)p.n + 1)), dim3(256), 0, s, p);
}
void launch_pub_build(const PubBuild& p, hipStream_t s) {
  if (p.n) hipLaunchKernelGGL(k_pub_build, dim3(blocks((int64_t)p.n)), dim3(256), 0, s, p);
}
void launch_msg_open(const MsgParams& p, hipStream_t s) {
  if (p.n > 0) hipLaunchKernelGGL(k_msg_open, dim3(blocks(p.n)), dim3(256), 0, s, p);
}
void launch_pub_count(const MsgParams& p, hipStream_t s) {
  if (p.n > 0) hipLaunchKernelGGL(k_pub_count, dim3(blocks(p.n)), dim3(256), 0, s, p);
}
void launch_pub_emit(const MsgParams& p, hipStream_t s) {
  if (p.n > 0) hipLaunchKernelGGL(k_pub_emit, dim3(blocks(p.n)), dim3(256), 0, s, p);
}
void launch_msg_delete(const MsgParams& p, hipStream_t s) {
  if (p.n > 0) hipLaunchKernelGGL(k_msg_delete, dim3(blocks(p.n)), dim3(256), 0, s, p);
}
void launch_ttl_flags(const MsgParams& p, hipStream_t s) {
  hipLaunchKernelGGL(k_ttl_flags, dim3(grid_cap(p.msg_count + 1)), dim3(256), 0, s, p);
}
void launch_ttl_write(const MsgParams& p, hipStream_t s) {
  if (p.msg_count) hipLaunchKernelGGL(k_ttl_write, dim3(grid_cap(p.msg_count)), dim3(256), 0, s, p);
}
void launch_wis_inject(const MsgParams& p, hipStream_t s) {
  if (p.n > 0) hipLaunchKernelGGL(k_wis_inject, dim3(blocks(p.n)), dim3(256), 0, s, p);
}
void launch_outbox_sizes(const Outbox& ob, const uint32_t* idx, uint64_t n, uint32_t* sizes, hipStream_t s) {
  hipLaunchKernelGGL(k_outbox_sizes, dim3(blocks((int64_t)n + 1)), dim3(256), 0, s, ob, idx, n, sizes);
}
void launch_outbox_bounds(const uint64_t* keys, uint64_t n, uint64_t* first, int parts, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_outbox_bounds, dim3(blocks((int64_t)n)), dim3(256), 0, s, keys, n, first, parts);
}
void launch_outbox_table(const uint64_t* first, const uint32_t* goff, int parts, uint64_t* table, hipStream_t s) {
  hipLaunchKernelGGL(k_outbox_table, dim3(1), dim3(64), 0, s, first, goff, parts, table);
}
void launch_outbox_pack(const Outbox& ob, const uint32_t* idx, const uint64_t* keys, uint64_t n, const uint64_t* first,
                        const uint32_t* goff, const uint64_t* base, uint8_t* dst, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_outbox_pack, dim3(blocks((int64_t)n)), dim3(256), 0, s, ob, idx, keys, n, first, goff, base, dst);
}
void launch_cs_hist(const Outbox& ob, uint64_t n, int begin, int bits, unsigned long long* cnt, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_cs_hist, dim3(blocks((int64_t)n)), dim3(256), 0, s, ob, n, begin, (1ull << bits) - 1, cnt);
}
void launch_cs_scatter(const Outbox& ob, uint64_t n, int begin, int bits, unsigned long long* off, uint64_t* kout,
                       uint32_t* vout, uint32_t* goff, hipStream_t s) {
  if (n)
    hipLaunchKernelGGL(k_cs_scatter, dim3(blocks((int64_t)n)), dim3(256), 0, s, ob, n, begin, (1ull << bits) - 1, off,
                       kout, vout, goff);
}
void launch_local_pack(const Outbox& ob, const uint32_t* idx, const uint32_t* goff, uint64_t n, uint64_t total,
                       uint8_t* dst, uint32_t* taken_n, uint32_t* taken_var, hipStream_t s) {
  hipLaunchKernelGGL(k_local_pack, dim3(blocks((int64_t)n + 1)), dim3(256), 0, s, ob, idx, goff, n, total, dst, taken_n,
                     taken_var);
}
void launch_iota(uint32_t* p, uint64_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_iota, dim3(blocks((int64_t)n)), dim3(256), 0, s, p, n);
}
void launch_key_spread(const uint64_t* keys, uint64_t n, uint64_t* out, hipStream_t s, const uint32_t* n_dev) {
  if (n) hipLaunchKernelGGL(k_key_spread, dim3(std::min<uint64_t>((n + 1023) / 1024, 512)), dim3(256), 0, s, keys, n,
                           (unsigned long long*)out, n_dev);
}

}  // namespace zbg
