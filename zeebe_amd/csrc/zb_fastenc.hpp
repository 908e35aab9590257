// zb_fastenc.hpp — the drain write pass's fast value encoder (WORKFLOW_INSTANCE / JOB records into the LDS
// image with 8-byte stores). Included by zb_serialize.hip; compiled for the host only by tests/native.
#pragma once
#include <cstdint>

#include "zb_device.hpp"

namespace zbg {

// The write pass's common records -- WORKFLOW_INSTANCE records of a deployed element and JOB records other
// than CANCEL(ED) -- are encoded into the LDS image with 8-byte stores (gfx950 LDS takes unaligned
// ds_write_b64): keys as immediates, integers assembled in a register, strings read from the LDS copy of the
// pool, payload documents copied as 8-byte words. A store may run up to 7 bytes past the field it writes:
// the fields after it (at least 8 bytes) overwrite them (same lane, LDS order). The value's trailing fields
// are written exactly, so nothing lands past the value (the next lane's record). Same bytes as encode_value:
// the GPU tests compare every value with the oracle's, tests/test_fastenc_host.py fuzzes this on the host
// (guard bytes after each value).
struct FastW {
  uint8_t* p;  // record start in the LDS image
  uint32_t n;
  __device__ __forceinline__ void st8(uint32_t o, uint64_t v) { __builtin_memcpy(p + o, &v, 8); }
  __device__ __forceinline__ void exact(uint32_t o, uint64_t v, uint32_t L) {  // the low L <= 8 bytes of v
    if (L == 8) { st8(o, v); return; }
    if (L & 4) { const uint32_t x = (uint32_t)v; __builtin_memcpy(p + o, &x, 4); v >>= 32; o += 4; }
    if (L & 2) { const uint16_t x = (uint16_t)v; __builtin_memcpy(p + o, &x, 2); v >>= 16; o += 2; }
    if (L & 1) p[o] = (uint8_t)v;
  }
  // N - 1 literal bytes (may hold NULs); EXACT: no store past them (the field after them may be 1 byte long)
  template <bool EXACT = false, int N>
  __device__ __forceinline__ void lit(const char (&s)[N]) {
    constexpr int L = N - 1;
#pragma unroll
    for (int c = 0; c < L; c += 8) {
      uint64_t w = 0;
#pragma unroll
      for (int k = 0; k < 8; k++)
        if (c + k < L) w |= (uint64_t)(uint8_t)s[c + k] << (8 * k);
      if (EXACT && L - c < 8) exact(n + c, w, L - c);
      else st8(n + c, w);
    }
    n += L;
  }
  // MsgPackWriter.writeInteger (same ranges as W::integer)
  __device__ __forceinline__ void ival(int64_t v, bool last = false) {
    uint64_t w;
    uint32_t L;
    if (v >= -32 && v < 128) { w = (uint8_t)v; L = 1; }
    else if (v >= 0) {
      if (v < 256) { w = 0xcc | (uint64_t)v << 8; L = 2; }
      else if (v < 65536) { w = 0xcd | (uint64_t)__builtin_bswap16((uint16_t)v) << 8; L = 3; }
      else if (v < (1LL << 32)) { w = 0xce | (uint64_t)__builtin_bswap32((uint32_t)v) << 8; L = 5; }
      else { w = 0xcf | __builtin_bswap64((uint64_t)v) << 8; L = 9; }
    } else {
      if (v >= -128) { w = 0xd0 | (uint64_t)(uint8_t)v << 8; L = 2; }
      else if (v >= -32768) { w = 0xd1 | (uint64_t)__builtin_bswap16((uint16_t)v) << 8; L = 3; }
      else if (v >= -(1LL << 31)) { w = 0xd2 | (uint64_t)__builtin_bswap32((uint32_t)v) << 8; L = 5; }
      else { w = 0xd3 | __builtin_bswap64((uint64_t)v) << 8; L = 9; }
    }
    if (L == 9) { st8(n, w); p[n + 8] = (uint8_t)v; }
    else if (last) exact(n, w, L);
    else st8(n, w);
    n += L;
  }
  __device__ __forceinline__ void raw(const uint8_t* s, uint32_t c) {  // s: LDS (reads may pass its end)
    for (uint32_t k = 0; k < c; k += 8) {
      uint64_t v;
      __builtin_memcpy(&v, s + k, 8);
      st8(n + k, v);
    }
    n += c;
  }
  __device__ __forceinline__ void str(const uint8_t* s, uint32_t c) {  // MsgPackWriter.writeString
    if (c < 32) { p[n] = (uint8_t)(0xa0 | c); n += 1; }
    else if (c < 256) { st8(n, 0xd9 | (uint64_t)c << 8); n += 2; }
    else if (c < 65536) { st8(n, 0xda | (uint64_t)__builtin_bswap16((uint16_t)c) << 8); n += 3; }
    else { st8(n, 0xdb | (uint64_t)__builtin_bswap32(c) << 8); n += 5; }
    raw(s, c);
  }
};

constexpr int SER_PRE = 6;  // payload document words prefetched per record (length + 44 bytes)

// the payload document [u32 len][bytes] as binary (MsgPackWriter.writeBinary): doc words W_j (8-aligned), the
// first SER_PRE already loaded; payload bytes [8k, 8k + 8) = W_k >> 32 | W_{k+1} << 32 (no read past the doc)
__device__ __forceinline__ void fast_bin(FastW& w, const uint64_t* dw, const uint64_t (&pre)[SER_PRE], bool last) {
  uint64_t cur = pre[0];
  const uint32_t plen = (uint32_t)cur;
  uint64_t h;
  uint32_t hl;
  if (plen < 256) { h = 0xc4 | (uint64_t)plen << 8; hl = 2; }
  else if (plen < 65536) { h = 0xc5 | (uint64_t)__builtin_bswap16((uint16_t)plen) << 8; hl = 3; }
  else { h = 0xc6 | (uint64_t)__builtin_bswap32(plen) << 8; hl = 5; }
  if (last) w.exact(w.n, h, hl);  // (a short last payload ends within the 8 bytes after the header)
  else w.st8(w.n, h);
  w.n += hl;
#pragma unroll
  for (int j = 1; j < SER_PRE; j++) {
    const uint32_t k = 8 * (j - 1);
    if (k < plen) {
      const uint64_t nx = k + 4 < plen ? pre[j] : 0;
      const uint64_t v = (cur >> 32) | (nx << 32);
      if (last && k + 8 > plen) w.exact(w.n + k, v, plen - k);
      else w.st8(w.n + k, v);
      cur = nx;
    }
  }
  for (uint32_t k = 8 * (SER_PRE - 1), j = SER_PRE; k < plen; k += 8, j++) {
    const uint64_t nx = k + 4 < plen ? dw[j] : 0;
    const uint64_t v = (cur >> 32) | (nx << 32);
    if (last && k + 8 > plen) w.exact(w.n + k, v, plen - k);
    else w.st8(w.n + k, v);
    cur = nx;
  }
  w.n += plen;
}

__device__ __forceinline__ bool fast_kind(const zb_rec& d) {
  if (d.kind & KIND_RAW) return false;
  const uint8_t vt = kind_vt(d.kind), rt = kind_rt(d.kind);
  if (vt == ZB_VT_WORKFLOW_INSTANCE)
    return !(d.intent == WI_CREATE && (rt == ZB_RT_COMMAND || rt == ZB_RT_COMMAND_REJECTION));
  return vt == ZB_VT_JOB && (d.intent | 1) != JI_CANCELED;
}

// encode_value's WORKFLOW_INSTANCE (non-submitted) and JOB branches; elems / wfs / pool in LDS
__device__ __forceinline__ void fast_encode(FastW& w, const zb_rec& d, const DevElem* elems, const DevWorkflow* wfs,
                                            const uint8_t* pool, const uint64_t* dw, const uint64_t (&pre)[SER_PRE]) {
  const DevElem& e = elems[d.elem];
  const DevWorkflow& wf = wfs[e.wf];
  if (kind_vt(d.kind) == ZB_VT_WORKFLOW_INSTANCE) {  // WorkflowInstanceRecord.java:39-60
    w.lit("\x87\xad" "bpmnProcessId");
    w.str(pool + wf.pid_off, wf.pid_len);
    w.lit("\xa7" "version");
    w.ival(wf.version);
    w.lit("\xab" "workflowKey");
    w.ival(wf.key);
    w.lit("\xb3" "workflowInstanceKey");
    w.ival(d.inst_key);
    w.lit("\xaa" "activityId");
    w.str(pool + e.id_off, e.id_len);
    w.lit("\xa7" "payload");
    fast_bin(w, dw, pre, false);
    w.lit<true>("\xb0" "scopeInstanceKey");  // (the value ends with a 1..9-byte integer)
    w.ival(d.scope_key, true);
  } else {  // JobRecord.java:35-53 + JobHeaders.java:33-51
    w.lit("\x87\xa8" "deadline" "\xd3\x80\x00\x00\x00\x00\x00\x00\x00" "\xa6" "worker" "\xa0" "\xa7" "retries");
    w.ival(e.retries);
    w.lit("\xa4" "type");
    w.str(pool + e.type_off, e.type_len);
    w.lit("\xa7" "headers" "\x86" "\xad" "bpmnProcessId");
    w.str(pool + wf.pid_off, wf.pid_len);
    w.lit("\xb9" "workflowDefinitionVersion");
    w.ival(wf.version);
    w.lit("\xab" "workflowKey");
    w.ival(wf.key);
    w.lit("\xb3" "workflowInstanceKey");
    w.ival(d.inst_key);
    w.lit("\xaa" "activityId");
    w.str(pool + e.id_off, e.id_len);
    w.lit("\xb3" "activityInstanceKey");
    w.ival(d.scope_key);
    w.lit("\xad" "customHeaders");
    if (e.headers_off == NO_REF) { w.p[w.n] = 0x80; w.n += 1; }  // JobRecord.NO_HEADERS
    else w.raw(pool + e.headers_off, e.headers_len);
    w.lit("\xa7" "payload");
    fast_bin(w, dw, pre, true);
  }
}

}  // namespace zbg
