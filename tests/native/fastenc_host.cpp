// TEST ONLY: compiles the drain write pass's fast value encoder (zeebe_amd/csrc/zb_fastenc.hpp) for the host
// so that its bytes -- and that it never stores past the value -- can be fuzzed on CPU
// (tests/test_fastenc_host.py). Nothing here is part of the product.
#include <cstdint>
#include <cstring>
#include <vector>
#define __device__
#define __host__
#define __forceinline__ inline
// v_alignbyte_b32: bytes [s, s + 4) of the little-endian pair (lo, hi), s = c mod 4
static inline uint32_t host_alignbyte(uint32_t hi, uint32_t lo, uint32_t c) {
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * (c & 3)));
}
#define __builtin_amdgcn_alignbyte host_alignbyte
#include "../../zeebe_amd/csrc/zb_fastenc.hpp"

using namespace zbg;

// Encodes one record with fast_encode into out + head (out 8-aligned, pre-filled by the caller with guard bytes).
// pool: element id / type / process id / headers bytes (offsets below); doc: [u32 len][payload], 8-aligned,
// padded to 8. Returns the encoded length (the caller checks out[n..cap) is still guard). BF: the branch-free
// writer (the template drain's), its dummy slot at image offset dummy.
template <bool BF>
static long fastenc_t(int vt, int intent, int64_t inst_key, int64_t scope_key, int64_t wf_key, int32_t version,
             int32_t retries, const uint8_t* pool_in, uint32_t pool_len, uint32_t pid_off, uint32_t pid_len,
             uint32_t id_off, uint32_t id_len, uint32_t type_off, uint32_t type_len, uint32_t hdr_off, uint32_t hdr_len,
             const uint64_t* doc, uint8_t* out, uint32_t head, uint32_t dummy) {
  static uint8_t pool[1 << 16];
  std::memset(pool, 0xcd, sizeof(pool));
  std::memcpy(pool, pool_in, pool_len);
  DevElem e{};
  e.kind = EK_TASK;  // (its JOB runs are built only for service tasks)
  e.wf = 0;
  e.id_off = id_off;
  e.id_len = (uint16_t)id_len;
  e.type_off = type_off;
  e.type_len = (uint16_t)type_len;
  e.headers_off = hdr_off;
  e.headers_len = hdr_len;
  e.retries = retries;
  DevWorkflow wf{};
  wf.key = wf_key;
  wf.version = version;
  wf.pid_off = pid_off;
  wf.pid_len = (uint16_t)pid_len;
  zb_rec d{};
  d.inst_key = inst_key;
  d.scope_key = scope_key;
  d.elem = 0;
  d.intent = (uint8_t)intent;
  d.kind = make_kind((uint8_t)vt, ZB_RT_EVENT, false);
  if (!fast_kind(d)) return -1;
  // the element's constant runs, as zb_deploy builds them (8-aligned copy: the device reads them from LDS)
  std::vector<DevValSeg> tab;
  std::vector<uint8_t> segs;
  if (!build_value_segments(&e, 1, &wf, 1, pool, tab, segs)) return -2;
  std::vector<uint64_t> seg_words((segs.size() + 7) / 8);
  std::memcpy(seg_words.data(), segs.data(), segs.size());
  uint64_t pre[SER_PRE];
  const uint32_t words = (4 + (uint32_t)doc[0] + 7) / 8;  // (doc[0] low half: the payload length)
  for (int j = 0; j < SER_PRE; j++) pre[j] = (uint32_t)j < words ? doc[j] : 0xa5a5a5a5a5a5a5a5ull;  // (next doc)
  FastWT<false, BF> w;
  w.begin(out, head, dummy);  // (out: 8-aligned image; the value starts at byte head of it)
  fast_encode(w, d, tab.data(), (const uint8_t*)seg_words.data(), doc, pre);
  return w.n();
}

extern "C" {
long fastenc(int vt, int intent, int64_t inst_key, int64_t scope_key, int64_t wf_key, int32_t version,
             int32_t retries, const uint8_t* pool_in, uint32_t pool_len, uint32_t pid_off, uint32_t pid_len,
             uint32_t id_off, uint32_t id_len, uint32_t type_off, uint32_t type_len, uint32_t hdr_off, uint32_t hdr_len,
             const uint64_t* doc, uint8_t* out, uint32_t head) {
  return fastenc_t<false>(vt, intent, inst_key, scope_key, wf_key, version, retries, pool_in, pool_len, pid_off, pid_len,
                          id_off, id_len, type_off, type_len, hdr_off, hdr_len, doc, out, head, 0);
}
long fastenc_bf(int vt, int intent, int64_t inst_key, int64_t scope_key, int64_t wf_key, int32_t version,
                int32_t retries, const uint8_t* pool_in, uint32_t pool_len, uint32_t pid_off, uint32_t pid_len,
                uint32_t id_off, uint32_t id_len, uint32_t type_off, uint32_t type_len, uint32_t hdr_off,
                uint32_t hdr_len, const uint64_t* doc, uint8_t* out, uint32_t head, uint32_t dummy) {
  return fastenc_t<true>(vt, intent, inst_key, scope_key, wf_key, version, retries, pool_in, pool_len, pid_off, pid_len,
                         id_off, id_len, type_off, type_len, hdr_off, hdr_len, doc, out, head, dummy);
}

// Encodes one message-side record (WORKFLOW_INSTANCE_SUBSCRIPTION / MESSAGE_SUBSCRIPTION / MESSAGE) with
// fast_encode_msg. blob: the record's arena blob (8-aligned, padded; a WIS record's payload document), msg: the
// element's message name (WIS). Returns the encoded length, -1 when the kind is not a fast message kind.
long fastenc_msg(int vt, int64_t inst_key, int64_t scope_key, const uint8_t* msg, uint32_t msg_len,
                 const uint64_t* blob, uint32_t blob_words, uint8_t* out, uint32_t head) {
  static uint8_t pool[1 << 16];
  std::memset(pool, 0xcd, sizeof(pool));
  std::memcpy(pool, msg, msg_len);
  DevElem e{};
  e.kind = EK_CATCH;
  e.wf = 0;
  e.msg_off = 0;
  e.msg_len = (uint16_t)msg_len;
  DevWorkflow wf{};
  zb_rec d{};
  d.inst_key = inst_key;
  d.scope_key = scope_key;
  d.elem = 0;
  d.kind = make_kind((uint8_t)vt, ZB_RT_EVENT, false);
  if (!fast_msg_kind(d)) return -1;
  std::vector<DevValSeg> tab;
  std::vector<uint8_t> segs;
  if (!build_value_segments(&e, 1, &wf, 1, pool, tab, segs)) return -2;
  std::vector<uint64_t> seg_words((segs.size() + 7) / 8);
  std::memcpy(seg_words.data(), segs.data(), segs.size());
  uint64_t pre[SER_PRE];
  for (int j = 0; j < SER_PRE; j++) pre[j] = (uint32_t)j < blob_words ? blob[j] : 0xa5a5a5a5a5a5a5a5ull;
  FastWT<true> w;
  w.begin(out, head);
  fast_encode_msg(w, d, tab.data(), (const uint8_t*)seg_words.data(), blob, pre);
  return w.n();
}
}
