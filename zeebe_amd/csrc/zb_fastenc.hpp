// zb_fastenc.hpp — the drain write pass's fast value encoder (WORKFLOW_INSTANCE / JOB records into the LDS
// image). Included by zb_serialize.hip; compiled for the host only by tests/native.
#pragma once
#include <cstdint>
#include <vector>

#include "zb_device.hpp"

namespace zbg {

// The common records -- WORKFLOW_INSTANCE records of a deployed element and JOB records other than
// CANCEL(ED) -- are encoded into the LDS image with ALIGNED stores only: a b64 / b32 DS access off its
// natural alignment is replayed at 64 cycles per wave instruction on gfx950 (cdna_hip_programming.md, LDS
// alignment), which made a byte-addressed 8-byte writer LDS-bound. The writer keeps the bytes of the
// current 8-byte image slot in a register and stores the slot when it fills; the value's first slot (shared
// with the previous lane's value) and its last one (shared with the next lane's) are written at the end with
// naturally aligned b8 / b16 / b32 stores of exactly the value's bytes. Keys are immediates, integers are assembled in a register, strings are read
// from the LDS copy of the pool with aligned b64 reads, payload documents are copied as 8-byte words.
// Same bytes as encode_value: the GPU tests compare every value with the oracle's, and
// tests/test_fastenc_host.py fuzzes this on the host with guard bytes around each value.
// CHK: every slot store checks whether it is the value's first slot (values whose first bytes come from a
// variable-length run -- MESSAGE records -- cannot say which put completes it); without it a value's first put is
// marked FIRST and whole 8-byte.
// BF (branch-free; CHK false only): a slot store that must not happen goes to the lane's own 8-byte dummy slot instead
// (an image offset the caller reserves past the image, begin()): no divergent branch around the stores of put / seg
template <bool CHK = false, bool BF = false>
struct FastWT {
  static_assert(!(CHK && BF), "the checked writer branches");
  uint8_t* img;   // LDS image base (8-aligned)
  uint32_t pos;   // image offset of the next byte
  uint32_t head;  // image offset of the value's first byte
  uint64_t acc;   // the current slot's bytes below pos (low bytes first)
  uint64_t first; // the first slot's word (stored by end(): its bytes below head are the previous value's)
  uint32_t dummy; // (BF) this lane's dummy slot

  __device__ __forceinline__ void begin(uint8_t* base, uint32_t at, uint32_t dummy_slot = 0) {
    img = base;
    pos = head = at;
    acc = 0;
    first = 0;
    dummy = dummy_slot;
  }
  __device__ __forceinline__ uint32_t n() const { return pos - head; }
  // a whole image slot (CHK: the value's first slot is kept for end())
  __device__ __forceinline__ void st(uint32_t slot, uint64_t v) {
    if (CHK && (head & 7) && slot == (head & ~7u)) first = v;
    else *(uint64_t*)(img + slot) = v;
  }
  // bytes [b, e) of slot word v at image offset slot, with naturally aligned stores (0 <= b < e <= 8)
  __device__ __forceinline__ void part(uint32_t slot, uint64_t v, uint32_t b, uint32_t e) {
    if ((b & 1) && b < e) { img[slot + b] = (uint8_t)(v >> (8 * b)); b += 1; }
    if ((b & 2) && b + 2 <= e) { *(uint16_t*)(img + slot + b) = (uint16_t)(v >> (8 * b)); b += 2; }
    if ((b & 4) && b + 4 <= e) { *(uint32_t*)(img + slot + b) = (uint32_t)(v >> (8 * b)); b += 4; }
    // b is now 0 / 4-aligned (head part done) or the tail remains: [b, e) from the low end
    if (b + 4 <= e) { *(uint32_t*)(img + slot + b) = (uint32_t)(v >> (8 * b)); b += 4; }
    if (b + 2 <= e) { *(uint16_t*)(img + slot + b) = (uint16_t)(v >> (8 * b)); b += 2; }
    if (b < e) img[slot + b] = (uint8_t)(v >> (8 * b));
  }
  // append the low k bytes of v (1 <= k <= 8; v's other bytes zero). FIRST: the value's first put (8 bytes):
  // the slot it completes is the head slot, which end() stores; every later slot is the value's alone
  template <bool FIRST = false>
  __device__ __forceinline__ void put(uint64_t v, uint32_t k) {
    const uint32_t f = pos & 7;
    const uint64_t lo = acc | (v << (8 * f));
    const uint64_t hi = (v >> 1) >> (63 - 8 * f);  // the bytes past the slot (0 when f == 0)
    if (BF) {
      const bool full = f + k >= 8;
      if (FIRST) first = lo;  // (used by end() only when f != 0)
      *(uint64_t*)(img + ((full && !(FIRST && f)) ? pos - f : dummy)) = lo;
      acc = full ? hi : lo;
      pos += k;
      return;
    }
    if (f + k >= 8) {
      if (FIRST && f) first = lo;
      else st(pos - f, lo);
      acc = hi;
    } else {
      acc = lo;
    }
    pos += k;
  }
  // the first and the last slot's bytes (call once, after the last put; values of 16 bytes or more, so that
  // the two are different slots -- WORKFLOW_INSTANCE and JOB values are over 80 bytes)
  __device__ __forceinline__ void end() {
    if (head & 7) part(head & ~7u, first, head & 7, 8);
    if (pos & 7) part(pos & ~7u, acc, 0, pos & 7);
  }
  // instead of end() for a log frame's value (zb_frame.hpp): the value starts 8-aligned after the frame prefix, so its
  // first slot is its own; the last slot is stored whole, its bytes past the value zero (the frame's padding to 8)
  __device__ __forceinline__ void end_frame() {
    if (BF) {
      *(uint64_t*)(img + ((pos & 7) ? (pos & ~7u) : dummy)) = acc;
      return;
    }
    if (pos & 7) *(uint64_t*)(img + (pos & ~7u)) = acc;
  }
  // N - 1 literal bytes (may hold NULs), as immediates; FIRST: the value starts with them (N - 1 >= 8)
  template <bool FIRST = false, int N>
  __device__ __forceinline__ void lit(const char (&s)[N]) {
    constexpr int L = N - 1;
    static_assert(!FIRST || L >= 8, "the first put is a whole 8-byte chunk");
#pragma unroll
    for (int c = 0; c < L; c += 8) {
      uint64_t w = 0;
#pragma unroll
      for (int k = 0; k < 8; k++)
        if (c + k < L) w |= (uint64_t)(uint8_t)s[c + k] << (8 * k);
      if (FIRST && c == 0) put<true>(w, 8);
      else put(w, L - c < 8 ? L - c : 8);
    }
  }
  // MsgPackWriter.writeInteger (same ranges as W::integer): a fixint, or a header byte (0xcc..0xcf unsigned,
  // 0xd0..0xd3 signed, by width) and the low m = 1, 2, 4 or 8 bytes of v big-endian; one straight path
  __device__ __forceinline__ void ival(int64_t v) {
    const bool neg = v < 0;
    const uint64_t mag = neg ? ~(uint64_t)v : (uint64_t)v;  // signed ranges are [-2^(8m-1), 2^(8m-1))
    const bool fix = neg ? v >= -32 : v < 128;
    const uint32_t lg = neg ? (mag < 0x80u ? 0 : mag < 0x8000u ? 1 : mag < 0x80000000ull ? 2 : 3)
                            : (mag < 0x100u ? 0 : mag < 0x10000u ? 1 : mag < 0x100000000ull ? 2 : 3);
    const uint32_t m = 1u << lg;
    const uint64_t be = __builtin_bswap64((uint64_t)v << (64 - 8 * m));
    if (fix) { put((uint8_t)v, 1); return; }
    put(((neg ? 0xd0u : 0xccu) + lg) | be << 8, m < 8 ? m + 1 : 8);
    if (m == 8) put((uint8_t)v, 1);
  }
  // a key known to be -1, 0 or in [2^16, 2^32) (the template drain's short form): a fixint or 0xce + 4 bytes
  __device__ __forceinline__ void ival5(int64_t v) {
    const bool sp = (uint64_t)(v + 1) <= 1;
    put(sp ? (uint64_t)(uint8_t)v : (0xceull | (uint64_t)__builtin_bswap32((uint32_t)v) << 8), sp ? 1u : 5u);
  }
  // a constant run: c bytes at s (LDS, 8-aligned; the pool keeps SEG_PAD_LO readable bytes before its first run
  // and SEG_PAD_HI after its last); FIRST as in put. The byte shift between the run and the image is fixed for
  // the whole run, so image slot j is bytes [r, r + 8) of three consecutive run dwords p[2j..2j+2] (p: the run
  // read from a 4-aligned start chosen by the shift): two v_alignbyte and one aligned ds_write_b64 per slot. The
  // dwords are read eight at a time, issued together: the LDS latency is paid per four slots.
  template <bool FIRST = false>
  __device__ __forceinline__ void seg(const uint8_t* s, uint32_t c) {
    const uint32_t f = pos & 7, e = 8 - f, r = e & 3;
    const uint32_t* p = (const uint32_t*)(s + 4 * (e >> 2)) - 2;
    const uint32_t end = f + c, nf = end >> 3, rem = end & 7;
    const uint64_t own0 = f ? (~0ull << (8 * f)) : ~0ull;  // slot 0: the run's bytes (below them: acc)
    const uint32_t slot = pos - f;
    uint32_t x0 = p[0];
    if (BF) {  // every slot of the group stored (a slot past the run's whole slots: to the dummy); slot nf kept in acc
      uint64_t last = 0;
      for (uint32_t j = 0; j <= nf; j += 4) {
        uint32_t x[8];
#pragma unroll
        for (int k = 0; k < 8; k++) x[k] = p[2 * j + 1 + k];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint32_t jj = j + k;
          const uint32_t a = k ? x[2 * k - 1] : x0;
          uint64_t v = (uint64_t)__builtin_amdgcn_alignbyte(x[2 * k], a, r) |
                       (uint64_t)__builtin_amdgcn_alignbyte(x[2 * k + 1], x[2 * k], r) << 32;
          if (k == 0) v = jj == 0 ? (acc | (v & own0)) : v;
          if (FIRST && k == 0) first = jj == 0 ? v : first;
          const bool sto = jj < nf && !(FIRST && jj == 0 && f);
          *(uint64_t*)(img + (sto ? slot + 8 * jj : dummy)) = v;
          last = jj == nf ? v : last;
        }
        x0 = x[7];
      }
      acc = rem ? last & (~0ull >> (64 - 8 * rem)) : 0;
      pos += c;
      return;
    }
    for (uint32_t j = 0; j <= nf; j += 4) {
      uint32_t x[8];
#pragma unroll
      for (int k = 0; k < 8; k++) x[k] = p[2 * j + 1 + k];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t jj = j + k;
        if (jj > nf) break;
        const uint32_t a = k ? x[2 * k - 1] : x0;
        uint64_t v = (uint64_t)__builtin_amdgcn_alignbyte(x[2 * k], a, r) |
                     (uint64_t)__builtin_amdgcn_alignbyte(x[2 * k + 1], x[2 * k], r) << 32;
        if (jj == 0) v = acc | (v & own0);
        if (jj < nf) {
          if (FIRST && jj == 0 && f) first = v;
          else st(slot + 8 * jj, v);
        } else {
          acc = rem ? v & (~0ull >> (64 - 8 * rem)) : 0;
        }
      }
      x0 = x[7];
    }
    pos += c;
  }
  // n bytes (n > 0) of a register-resident run: v[i] = bytes [8i, 8i + 8) (bytes past n are masked off), n <= 8N;
  // the image shift is fixed for the run: slot i = acc | v[i] << 8f, then acc = v[i] >> (64 - 8f)
  template <int N>
  __device__ __forceinline__ void words(const uint64_t (&v)[N], uint32_t n) {
    const uint32_t f = pos & 7, sl = 8 * f, sr = 63 - sl;
    const uint32_t end = f + n, nf = end >> 3, rem = end & 7;
    const uint32_t slot = pos - f;
    if (BF) {  // all N slots: the ones past the run's whole slots to the dummy, slot nf's bytes kept in acc
#pragma unroll
      for (int i = 0; i < N; i++) {
        const uint64_t x = (uint32_t)(8 * i) < n ? v[i] : 0ull;
        const uint64_t o = acc | (x << sl);
        const bool full = (uint32_t)i < nf;
        *(uint64_t*)(img + (full ? slot + 8 * i : dummy)) = o;
        acc = full ? (x >> 1) >> sr : ((uint32_t)i == nf ? o : acc);
      }
      acc = rem ? acc & (~0ull >> (64 - 8 * rem)) : 0;
      pos += n;
      return;
    }
#pragma unroll
    for (int i = 0; i < N; i++) {
      if ((uint32_t)i > nf) break;
      const uint64_t x = (uint32_t)(8 * i) < n ? v[i] : 0ull;
      const uint64_t o = acc | (x << sl);
      if ((uint32_t)i < nf) {
        st(slot + 8 * i, o);
        acc = (x >> 1) >> sr;  // (f == 0: 0)
      } else {
        acc = o;
      }
    }
    acc = rem ? acc & (~0ull >> (64 - 8 * rem)) : 0;  // slot nf: the run's last bytes
    pos += n;
  }
  // MsgPackWriter.writeStringHeader / writeBinaryHeader
  __device__ __forceinline__ void str_hdr(uint32_t c) {
    if (c < 32) put(0xa0 | c, 1);
    else if (c < 256) put(0xd9 | (uint64_t)c << 8, 2);
    else if (c < 65536) put(0xda | (uint64_t)__builtin_bswap16((uint16_t)c) << 8, 3);
    else put(0xdb | (uint64_t)__builtin_bswap32(c) << 8, 5);
  }
  __device__ __forceinline__ void bin_hdr(uint32_t c) {
    if (c < 256) put(0xc4 | (uint64_t)c << 8, 2);
    else if (c < 65536) put(0xc5 | (uint64_t)__builtin_bswap16((uint16_t)c) << 8, 3);
    else put(0xc6 | (uint64_t)__builtin_bswap32(c) << 8, 5);
  }
  // n bytes at p in global memory, any alignment: whole 8-byte words around them are read (arena blobs are 8-aligned
  // and padded, and the arena has ARENA_SLACK readable bytes past its end)
  __device__ __forceinline__ void gbytes(const uint8_t* p, uint32_t n) {
    const uint32_t a = (uint32_t)((uintptr_t)p & 7);
    const uint64_t* q = (const uint64_t*)(p - a);
    uint64_t cur = q[0];
    for (uint32_t k = 0, j = 1; k < n; k += 8, j++) {
      const uint64_t nx = a + n > k + 8 ? q[j] : 0ull;  // (the word holding bytes past k + 8 - a, when there are any)
      const uint64_t x = a ? (cur >> (8 * a)) | (nx << (64 - 8 * a)) : cur;
      const uint32_t r = n - k;
      put(r < 8 ? x & (~0ull >> (64 - 8 * r)) : x, r < 8 ? r : 8);
      cur = nx;
    }
  }
};
using FastW = FastWT<false>;
using FastWB = FastWT<false, true>;

constexpr int SER_PRE = 6;  // payload document words prefetched per record (length + 44 bytes)
constexpr uint32_t ARENA_SLACK = 64;  // bytes allocated past the arena: SER_PRE words load unchecked

// The constant runs of an element's values, built at deploy time (build_value_segments) and copied into LDS
// by the write pass: a run is appended 8 bytes at a time from aligned LDS words instead of key by key.
//   WI_A  {0x87 "bpmnProcessId" pid "version" v "workflowKey" k "workflowInstanceKey"}   (per workflow)
//   WI_B  {"activityId" id "payload"}
//   JOB_A {0x87 "deadline" MIN "worker" "" "retries" r "type" t "headers" 0x86 "bpmnProcessId" pid
//          "workflowDefinitionVersion" v "workflowKey" k "workflowInstanceKey"}
//   JOB_B {"activityId" id "activityInstanceKey"}      JOB_C {"customHeaders" h "payload"}
//   WIS   {"messageName" name "payload"}               (elements that subscribe to a message)
// Each run starts 8-aligned in the segment pool and is zero-padded to 8 bytes.
enum { SEG_WI_A = 0, SEG_WI_B, SEG_JOB_A, SEG_JOB_B, SEG_JOB_C, SEG_WIS, SEG_N };
struct DevValSeg {
  uint16_t off8[SEG_N];  // offset / 8 in the segment pool
  uint16_t len[SEG_N];
};
static_assert(sizeof(DevValSeg) == 24, "DevValSeg is 24 bytes");
constexpr uint32_t SEG_PAD_LO = 16, SEG_PAD_HI = 48;  // readable bytes before the first run / after the last
constexpr uint32_t SEG_LDS_MAX = 16384;  // table (padded to 4 entries) + pool the fast passes copy into LDS

// the payload document [u32 len][bytes] as binary (MsgPackWriter.writeBinary): doc words W_j (8-aligned), the
// first SER_PRE already loaded (words past the document hold whatever follows it: only bytes past the payload
// come from them, and those are masked off); payload bytes [8k, 8k + 8) = W_k >> 32 | W_(k+1) << 32
template <bool CHK, bool BF>
__device__ __forceinline__ void fast_bin(FastWT<CHK, BF>& w, const uint64_t* dw, const uint64_t (&pre)[SER_PRE]) {
  const uint32_t plen = (uint32_t)pre[0];
  if (plen < 256) w.put(0xc4 | (uint64_t)plen << 8, 2);
  else if (plen < 65536) w.put(0xc5 | (uint64_t)__builtin_bswap16((uint16_t)plen) << 8, 3);
  else w.put(0xc6 | (uint64_t)__builtin_bswap32(plen) << 8, 5);
  if (plen == 0) return;
  constexpr uint32_t NPRE = 8 * (SER_PRE - 1);  // payload bytes in the prefetched words
  uint64_t v[SER_PRE - 1];
#pragma unroll
  for (int j = 1; j < SER_PRE; j++) v[j - 1] = (pre[j - 1] >> 32) | (pre[j] << 32);
  w.words(v, plen < NPRE ? plen : NPRE);
  if (plen > NPRE) {  // longer payloads: the rest from HBM (no load past the document)
    uint64_t cur = pre[SER_PRE - 1];
    for (uint32_t k = NPRE, j = SER_PRE; k < plen; k += 8, j++) {
      const uint64_t nx = k + 4 < plen ? dw[j] : 0;
      const uint64_t x = (cur >> 32) | (nx << 32);
      const uint32_t r = plen - k;
      w.put(r < 8 ? x & (~0ull >> (64 - 8 * r)) : x, r < 8 ? r : 8);
      cur = nx;
    }
  }
}

// the message-side records it takes too (encode_value's WORKFLOW_INSTANCE_SUBSCRIPTION / MESSAGE_SUBSCRIPTION / MESSAGE
// branches: fast_encode_msg); their lengths come from the size pass's dry run, not from a formula
__device__ __forceinline__ bool fast_msg_kind(const zb_rec& d) {
  if (d.kind & KIND_RAW) return false;
  const uint8_t vt = kind_vt(d.kind);
  return vt == ZB_VT_WORKFLOW_INSTANCE_SUBSCRIPTION || vt == ZB_VT_MESSAGE_SUBSCRIPTION || vt == ZB_VT_MESSAGE;
}
__device__ __forceinline__ bool fast_kind(const zb_rec& d) {
  if (d.kind & KIND_RAW) return false;
  const uint8_t vt = kind_vt(d.kind), rt = kind_rt(d.kind);
  if (vt == ZB_VT_WORKFLOW_INSTANCE)
    return !(d.intent == WI_CREATE && (rt == ZB_RT_COMMAND || rt == ZB_RT_COMMAND_REJECTION));
  return vt == ZB_VT_JOB && (d.intent | 1) != JI_CANCELED;
}

// encode_value's WORKFLOW_INSTANCE (non-submitted) and JOB branches from the constant runs of the record's
// element (tab / pool in LDS) and its variable fields: keys, payload
// L5: every key in ival5's range; FR: the value of a log frame (end_frame)
template <bool L5 = false, bool BF = false, bool FR = false>
__device__ __forceinline__ void fast_encode(FastWT<false, BF>& w, const zb_rec& d, const DevValSeg* tab, const uint8_t* segs,
                                            const uint64_t* dw, const uint64_t (&pre)[SER_PRE]) {
  const DevValSeg& t = tab[d.elem];
  if (kind_vt(d.kind) == ZB_VT_WORKFLOW_INSTANCE) {  // WorkflowInstanceRecord.java:39-60
    w.template seg<true>(segs + 8 * t.off8[SEG_WI_A], t.len[SEG_WI_A]);
    if (L5) w.ival5(d.inst_key); else w.ival(d.inst_key);
    w.seg(segs + 8 * t.off8[SEG_WI_B], t.len[SEG_WI_B]);
    fast_bin(w, dw, pre);
    w.lit("\xb0" "scopeInstanceKey");
    if (L5) w.ival5(d.scope_key); else w.ival(d.scope_key);
  } else {  // JobRecord.java:35-53 + JobHeaders.java:33-51
    w.template seg<true>(segs + 8 * t.off8[SEG_JOB_A], t.len[SEG_JOB_A]);
    if (L5) w.ival5(d.inst_key); else w.ival(d.inst_key);
    w.seg(segs + 8 * t.off8[SEG_JOB_B], t.len[SEG_JOB_B]);
    if (L5) w.ival5(d.scope_key); else w.ival(d.scope_key);
    w.seg(segs + 8 * t.off8[SEG_JOB_C], t.len[SEG_JOB_C]);
    fast_bin(w, dw, pre);
  }
  if (FR) w.end_frame();
  else w.end();
}

// The message-side values, from the record's blob (dw: its first word; zb_msg.hpp MsgView / SubView layouts) and,
// for a WORKFLOW_INSTANCE_SUBSCRIPTION, its element's message name run and the payload document. Checked stores: a
// MESSAGE value's first slot is completed inside its name.
template <bool FR = false>
__device__ __forceinline__ void fast_encode_msg(FastWT<true>& w, const zb_rec& d, const DevValSeg* tab,
                                                const uint8_t* segs, const uint64_t* dw,
                                                const uint64_t (&pre)[SER_PRE]) {
  const uint8_t vt = kind_vt(d.kind);
  const uint8_t* b = (const uint8_t*)dw;
  if (vt == ZB_VT_WORKFLOW_INSTANCE_SUBSCRIPTION) {  // WorkflowInstanceSubscriptionRecord.java:26-38
    const DevValSeg& t = tab[d.elem];
    w.lit("\x84" "\xb3" "workflowInstanceKey");
    w.ival(d.inst_key);
    w.lit("\xb3" "activityInstanceKey");
    w.ival(d.scope_key);
    w.seg(segs + 8 * t.off8[SEG_WIS], t.len[SEG_WIS]);
    fast_bin(w, dw, pre);
  } else if (vt == ZB_VT_MESSAGE_SUBSCRIPTION) {  // MessageSubscriptionRecord.java:26-41 (SubView: wfp, names at 24)
    const uint32_t nn = *(const uint32_t*)(b + 16), nc = *(const uint32_t*)(b + 20);
    w.lit("\x85" "\xbb" "workflowInstancePartitionId");
    w.ival(*(const int32_t*)(b + 4));
    w.lit("\xb3" "workflowInstanceKey");
    w.ival(d.inst_key);
    w.lit("\xb3" "activityInstanceKey");
    w.ival(d.scope_key);
    w.lit("\xab" "messageName");
    w.str_hdr(nn);
    w.gbytes(b + 24, nn);
    w.lit("\xae" "correlationKey");
    w.str_hdr(nc);
    w.gbytes(b + 24 + nn, nc);
  } else {  // MessageRecord.java:26-42 (MsgView: name, correlation key, payload, id from byte 40)
    const uint32_t nn = *(const uint32_t*)(b + 4), nc = *(const uint32_t*)(b + 24), np = *(const uint32_t*)(b + 28);
    const uint32_t nid = *(const uint32_t*)(b + 32);
    const uint8_t* name = b + 40;
    w.lit("\x85" "\xa4" "name");
    w.str_hdr(nn);
    w.gbytes(name, nn);
    w.lit("\xae" "correlationKey");
    w.str_hdr(nc);
    w.gbytes(name + nn, nc);
    w.lit("\xaa" "timeToLive");
    w.ival(*(const int64_t*)(b + 8));
    w.lit("\xa7" "payload");
    w.bin_hdr(np);
    w.gbytes(name + nn + nc, np);
    w.lit("\xa9" "messageId");
    w.str_hdr(nid);
    w.gbytes(name + nn + nc + np, nid);
  }
  if (FR) w.end_frame();
  else w.end();
}

// ---- host: the constant runs of every element's values (deploy time)
inline void seg_int(std::vector<uint8_t>& b, int64_t v) {  // MsgPackWriter.writeInteger
  auto be = [&](uint64_t x, int n) { for (int i = n - 1; i >= 0; i--) b.push_back((uint8_t)(x >> (8 * i))); };
  if (v < -(1LL << 5)) {
    if (v < -(1LL << 15)) {
      if (v < -(1LL << 31)) { b.push_back(0xd3); be((uint64_t)v, 8); }
      else { b.push_back(0xd2); be((uint64_t)v, 4); }
    } else if (v < -(1 << 7)) { b.push_back(0xd1); be((uint64_t)v, 2); }
    else { b.push_back(0xd0); be((uint64_t)v, 1); }
  } else if (v < (1 << 7)) b.push_back((uint8_t)v);
  else if (v < (1LL << 8)) { b.push_back(0xcc); be((uint64_t)v, 1); }
  else if (v < (1LL << 16)) { b.push_back(0xcd); be((uint64_t)v, 2); }
  else if (v < (1LL << 32)) { b.push_back(0xce); be((uint64_t)v, 4); }
  else { b.push_back(0xcf); be((uint64_t)v, 8); }
}
inline void seg_str(std::vector<uint8_t>& b, const uint8_t* s, uint32_t n) {  // MsgPackWriter.writeString
  if (n < 32) b.push_back((uint8_t)(0xa0 | n));
  else if (n < 256) { b.push_back(0xd9); b.push_back((uint8_t)n); }
  else if (n < 65536) { b.push_back(0xda); b.push_back((uint8_t)(n >> 8)); b.push_back((uint8_t)n); }
  else { b.push_back(0xdb); for (int i = 3; i >= 0; i--) b.push_back((uint8_t)(n >> (8 * i))); }
  b.insert(b.end(), s, s + n);
}
inline void seg_key(std::vector<uint8_t>& b, const char* k) {
  uint32_t n = 0;
  while (k[n]) n++;
  seg_str(b, (const uint8_t*)k, n);
}
// false: a run or the pool does not fit the 16-bit table fields
inline bool build_value_segments(const DevElem* elems, size_t n_elems, const DevWorkflow* wfs, size_t n_wfs,
                                 const uint8_t* pool, std::vector<DevValSeg>& tab, std::vector<uint8_t>& segs) {
  tab.assign(n_elems, DevValSeg{});
  segs.assign(SEG_PAD_LO, 0);  // (FastW::seg reads up to 8 bytes before a run)
  auto add = [&](const std::vector<uint8_t>& b, uint16_t& off8, uint16_t& len) {
    if (segs.size() / 8 > 0xffff || b.size() > 0xffff) return false;
    off8 = (uint16_t)(segs.size() / 8);
    len = (uint16_t)b.size();
    segs.insert(segs.end(), b.begin(), b.end());
    segs.resize((segs.size() + 7) & ~(size_t)7, 0);
    return true;
  };
  std::vector<uint16_t> wf_off(n_wfs), wf_len(n_wfs);
  for (size_t k = 0; k < n_wfs; k++) {  // WI_A, shared by a workflow's elements
    const DevWorkflow& wf = wfs[k];
    std::vector<uint8_t> b = {0x87};
    seg_key(b, "bpmnProcessId"); seg_str(b, pool + wf.pid_off, wf.pid_len);
    seg_key(b, "version"); seg_int(b, wf.version);
    seg_key(b, "workflowKey"); seg_int(b, wf.key);
    seg_key(b, "workflowInstanceKey");
    if (!add(b, wf_off[k], wf_len[k])) return false;
  }
  for (size_t i = 0; i < n_elems; i++) {
    const DevElem& e = elems[i];
    const DevWorkflow& wf = wfs[e.wf];
    DevValSeg& t = tab[i];
    t.off8[SEG_WI_A] = wf_off[e.wf];
    t.len[SEG_WI_A] = wf_len[e.wf];
    std::vector<uint8_t> b;
    seg_key(b, "activityId"); seg_str(b, pool + e.id_off, e.id_len); seg_key(b, "payload");
    if (!add(b, t.off8[SEG_WI_B], t.len[SEG_WI_B])) return false;
    if (e.kind == EK_CATCH) {  // (a message subscription: its WORKFLOW_INSTANCE_SUBSCRIPTION records)
      b.clear();
      seg_key(b, "messageName"); seg_str(b, pool + e.msg_off, e.msg_len); seg_key(b, "payload");
      if (!add(b, t.off8[SEG_WIS], t.len[SEG_WIS])) return false;
    }
    if (e.kind != EK_TASK) continue;  // only service tasks write JOB records
    b = {0x87};
    seg_key(b, "deadline"); seg_int(b, INT64_MIN);
    seg_key(b, "worker"); seg_str(b, nullptr, 0);
    seg_key(b, "retries"); seg_int(b, e.retries);
    seg_key(b, "type"); seg_str(b, pool + e.type_off, e.type_len);
    seg_key(b, "headers"); b.push_back(0x86);
    seg_key(b, "bpmnProcessId"); seg_str(b, pool + wf.pid_off, wf.pid_len);
    seg_key(b, "workflowDefinitionVersion"); seg_int(b, wf.version);
    seg_key(b, "workflowKey"); seg_int(b, wf.key);
    seg_key(b, "workflowInstanceKey");
    if (!add(b, t.off8[SEG_JOB_A], t.len[SEG_JOB_A])) return false;
    b.clear();
    seg_key(b, "activityId"); seg_str(b, pool + e.id_off, e.id_len); seg_key(b, "activityInstanceKey");
    if (!add(b, t.off8[SEG_JOB_B], t.len[SEG_JOB_B])) return false;
    b.clear();
    seg_key(b, "customHeaders");
    if (e.headers_off == NO_REF) b.push_back(0x80);  // JobRecord.NO_HEADERS
    else b.insert(b.end(), pool + e.headers_off, pool + e.headers_off + e.headers_len);
    seg_key(b, "payload");
    if (!add(b, t.off8[SEG_JOB_C], t.len[SEG_JOB_C])) return false;
  }
  segs.resize(segs.size() + SEG_PAD_HI, 0);  // (FastW::seg reads up to 40 bytes past a run)
  return true;
}

}  // namespace zbg
