// zb_serialize.hip — descriptor -> exact reference record value bytes (size, offsets, write; one pass or two).
//
// Value layouts (UnpackedObject.write: declared properties in declaration order, ObjectValue.java:140-153):
//   WorkflowInstanceRecord  broker-core/.../workflow/data/WorkflowInstanceRecord.java:39-60
//   JobRecord + JobHeaders  broker-core/.../job/data/JobRecord.java:35-53, JobHeaders.java:33-51
//   IncidentRecord          broker-core/.../incident/data/IncidentRecord.java (EnumProperty -> enum name string)
// Integer encoding is MsgPackWriter.writeInteger (msgpack-core/.../spec/MsgPackWriter.java:143-201).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "zb_devlib.hpp"
#include "zb_fastenc.hpp"
#include "zb_frame.hpp"
#include "zb_wavelib.hpp"
#include "zb_kernels.hpp"
#include "zb_msg.hpp"

namespace zbg {

struct W : Out {
  __device__ inline void integer(int64_t v) {
    if (v < -(1LL << 5)) {
      if (v < -(1LL << 15)) {
        if (v < -(1LL << 31)) { put(0xd3); for (int i = 7; i >= 0; i--) put((uint8_t)((uint64_t)v >> (8 * i))); }
        else { put(0xd2); for (int i = 3; i >= 0; i--) put((uint8_t)((uint32_t)v >> (8 * i))); }
      } else {
        if (v < -(1 << 7)) { put(0xd1); put((uint8_t)((uint16_t)v >> 8)); put((uint8_t)v); }
        else { put(0xd0); put((uint8_t)v); }
      }
    } else if (v < (1 << 7)) {
      put((uint8_t)v);
    } else if (v < (1LL << 16)) {
      if (v < (1 << 8)) { put(0xcc); put((uint8_t)v); }
      else { put(0xcd); put((uint8_t)(v >> 8)); put((uint8_t)v); }
    } else if (v < (1LL << 32)) {
      put(0xce); for (int i = 3; i >= 0; i--) put((uint8_t)(v >> (8 * i)));
    } else {
      put(0xcf); for (int i = 7; i >= 0; i--) put((uint8_t)((uint64_t)v >> (8 * i)));
    }
  }
  __device__ inline void key(const char* s) {
    uint32_t n = 0;
    while (s[n]) n++;
    str((const uint8_t*)s, n);
  }
  __device__ inline void bin(const uint8_t* s, uint32_t n) {
    if (n < 256) { put(0xc4); put((uint8_t)n); }
    else if (n < 65536) { put(0xc5); put((uint8_t)(n >> 8)); put((uint8_t)n); }
    else { put(0xc6); for (int i = 3; i >= 0; i--) put((uint8_t)(n >> (8 * i))); }
    if (dst && (((uintptr_t)s) & 3) == 0) {
      // arena documents: 4-byte aligned and padded to 8, so whole-word loads never leave the blob
      const uint32_t* w = (const uint32_t*)s;
      for (uint32_t k = 0; k < n; k += 4) {
        const uint32_t v = w[k >> 2];
        const uint32_t m = n - k < 4 ? n - k : 4;
        for (uint32_t b = 0; b < m; b++) dst[this->n + k + b] = (uint8_t)(v >> (8 * b));
      }
      this->n += n;
    } else {
      put_bytes(s, n);
    }
  }
  __device__ inline void cstr(const char* s) {  // append raw chars (message text)
    while (*s) put((uint8_t)*s++);
  }
};

__device__ const char* const TYPE_NAMES[9] = {"INTEGER", "FLOAT", "BOOLEAN", "NIL", "MAP", "ARRAY",
                                             "BINARY", "STRING", "EXTENSION"};
__device__ const char* const ERROR_TYPES[4] = {"UNKNOWN", "IO_MAPPING_ERROR", "JOB_NO_RETRIES", "CONDITION_ERROR"};

__device__ inline uint32_t dstrlen(const char* s) {
  uint32_t n = 0;
  while (s[n]) n++;
  return n;
}

// incident error message (JsonConditionInterpreter / ExclusiveSplitHandler / MappingProcessor texts)
__device__ inline void message(W& w, const SerParams& P, const uint8_t* det, bool size_only_hdr) {
  const uint8_t code = det[1], a = det[2], b = det[3];
  const uint16_t q = *(const uint16_t*)(det + 4);
  // compute length first (string header needs it)
  W m;
  m.dst = nullptr;
  m.n = 0;
  for (int pass = 0; pass < 2; pass++) {
    W& o = pass == 0 ? m : w;
    if (pass == 1) {
      uint32_t len = m.n;
      if (len < 32) o.put(0xa0 | len);
      else if (len < 256) { o.put(0xd9); o.put((uint8_t)len); }
      else { o.put(0xda); o.put((uint8_t)(len >> 8)); o.put((uint8_t)len); }
    }
    switch (code) {
      case EC_NO_FLOW: o.cstr("All conditions evaluated to false and no default flow is set."); break;
      case EC_PATH_NO_RESULT:
      case EC_PATH_MULTI: {
        const DevQuery& qq = P.queries[q];
        o.cstr("JSON path '");
        o.put_bytes(P.pool + qq.expr_off, qq.expr_len);
        o.cstr(code == EC_PATH_NO_RESULT ? "' has no result." : "' has more than one result.");
        break;
      }
      case EC_DIFF_TYPES:
        o.cstr("Cannot compare values of different types: ");
        o.cstr(TYPE_NAMES[a < 9 ? a : 8]);
        o.cstr(" and ");
        o.cstr(TYPE_NAMES[b < 9 ? b : 8]);
        break;
      case EC_CMP_TYPE: o.cstr("Cannot compare value of type: "); o.cstr(TYPE_NAMES[a < 9 ? a : 8]); break;
      case EC_NOT_NUMBER:
        o.cstr("Cannot compare values. Expected number but found: ");
        o.cstr(TYPE_NAMES[a < 9 ? a : 8]);
        break;
      case EC_MAPPING_NOT_MAP:
        o.cstr("Processing failed, since mapping will result in a non map object (json object).");
        break;
      case EC_MAPPING_NO_DATA: {  // MsgPackDocumentExtractor.executeLeafMapping :185-203
        const DevQuery& qq = P.queries[q];
        o.cstr("No data found for query ");
        o.put_bytes(P.pool + qq.expr_off, qq.expr_len);
        o.cstr(".");
        break;
      }
    }
  }
  (void)size_only_hdr;
}

__device__ inline const CmdRange* find_range(const SerParams& P, int64_t pos) {
  int lo = 0, hi = P.nranges - 1;
  while (lo <= hi) {
    int mid = (lo + hi) >> 1;
    const CmdRange& r = P.ranges[mid];
    if (pos < r.pos_begin) hi = mid - 1;
    else if (pos >= r.pos_end) lo = mid + 1;
    else return &r;
  }
  return nullptr;
}

__device__ __forceinline__ void encode_value(const SerParams& P, int64_t pos, const zb_rec& d, W& w) {
  const uint8_t vt = kind_vt(d.kind), rt = kind_rt(d.kind);
  if (d.kind & KIND_RAW) {  // zb_submit: the value as written, or the command value as the reference re-encodes it
    const uint8_t* doc = P.arena + (uint64_t)d.payload * 8;
    const uint32_t dl = *(const uint32_t*)doc;
    const uint8_t* raw = doc + ((4 + dl + 7) & ~7u);
    w.put_bytes(raw + 4, *(const uint32_t*)raw);
    return;
  }
  uint32_t plen = 0;
  const uint8_t* pl = nullptr;
  if (vt != ZB_VT_INCIDENT) {
    const uint8_t* p = P.arena + (uint64_t)d.payload * 8;
    plen = *(const uint32_t*)p;
    pl = p + 4;
  }
  if (vt == ZB_VT_WORKFLOW_INSTANCE) {
    w.map_hdr(7);
    const bool submitted = d.intent == WI_CREATE && (rt == ZB_RT_COMMAND || rt == ZB_RT_COMMAND_REJECTION);
    if (submitted) {
      const CmdRange* r = find_range(P, rt == ZB_RT_COMMAND ? pos : d.scope_key);
      w.key("bpmnProcessId");
      if (r) w.str(P.cmd_pool + r->pid_off, r->pid_len); else w.str(nullptr, 0);
      w.key("version"); w.integer(r ? r->version : -1);
      w.key("workflowKey"); w.integer(r ? r->workflow_key : -1);
      w.key("workflowInstanceKey"); w.integer(rt == ZB_RT_COMMAND ? -1 : d.inst_key);
      w.key("activityId"); w.str(nullptr, 0);
      w.key("payload"); w.bin(pl, plen);
      w.key("scopeInstanceKey"); w.integer(-1);
      return;
    }
    const DevElem& e = P.elems[d.elem];
    const DevWorkflow& wf = P.wfs[e.wf];
    w.key("bpmnProcessId"); w.str(P.pool + wf.pid_off, wf.pid_len);
    w.key("version"); w.integer(wf.version);
    w.key("workflowKey"); w.integer(wf.key);
    w.key("workflowInstanceKey"); w.integer(d.inst_key);
    w.key("activityId"); w.str(P.pool + e.id_off, e.id_len);
    w.key("payload"); w.bin(pl, plen);
    w.key("scopeInstanceKey"); w.integer(d.scope_key);
  } else if (vt == ZB_VT_JOB && (d.intent | 1) == JI_CANCELED) {  // CANCEL (12) or CANCELED (13)
    // TerminateServiceTaskHandler :37-58: a reset JobRecord with type "", headers without workflowKey
    const DevElem& e = P.elems[d.elem];
    const DevWorkflow& wf = P.wfs[e.wf];
    w.map_hdr(7);
    w.key("deadline"); w.integer(INT64_MIN);
    w.key("worker"); w.str(nullptr, 0);
    w.key("retries"); w.integer(-1);
    w.key("type"); w.str(nullptr, 0);
    w.key("headers");
    w.map_hdr(6);
    w.key("bpmnProcessId"); w.str(P.pool + wf.pid_off, wf.pid_len);
    w.key("workflowDefinitionVersion"); w.integer(wf.version);
    w.key("workflowKey"); w.integer(-1);
    w.key("workflowInstanceKey"); w.integer(d.inst_key);
    w.key("activityId"); w.str(P.pool + e.id_off, e.id_len);
    w.key("activityInstanceKey"); w.integer(d.scope_key);
    w.key("customHeaders"); w.put(0x80);
    w.key("payload"); w.bin((const uint8_t*)"\x80", 1);
  } else if (vt == ZB_VT_JOB) {
    const DevElem& e = P.elems[d.elem];
    const DevWorkflow& wf = P.wfs[e.wf];
    w.map_hdr(7);
    w.key("deadline"); w.integer(INT64_MIN);
    w.key("worker"); w.str(nullptr, 0);
    w.key("retries"); w.integer(e.retries);
    w.key("type"); w.str(P.pool + e.type_off, e.type_len);
    w.key("headers");
    w.map_hdr(6);
    w.key("bpmnProcessId"); w.str(P.pool + wf.pid_off, wf.pid_len);
    w.key("workflowDefinitionVersion"); w.integer(wf.version);
    w.key("workflowKey"); w.integer(wf.key);
    w.key("workflowInstanceKey"); w.integer(d.inst_key);
    w.key("activityId"); w.str(P.pool + e.id_off, e.id_len);
    w.key("activityInstanceKey"); w.integer(d.scope_key);
    w.key("customHeaders");
    if (e.headers_off == NO_REF) w.put(0x80);  // JobRecord.NO_HEADERS
    else w.put_bytes(P.pool + e.headers_off, e.headers_len);
    w.key("payload"); w.bin(pl, plen);
  } else if (vt == ZB_VT_INCIDENT) {
    const uint8_t* det = P.arena + (uint64_t)d.payload * 8 + 4;
    const DevElem& e = P.elems[d.elem];
    const DevWorkflow& wf = P.wfs[e.wf];
    w.map_hdr(9);
    w.key("errorType"); w.key(ERROR_TYPES[det[0] < 4 ? det[0] : 0]);
    w.key("errorMessage"); message(w, P, det, false);
    w.key("failureEventPosition"); w.integer(*(const int64_t*)(det + 12));
    w.key("bpmnProcessId"); w.str(P.pool + wf.pid_off, wf.pid_len);
    w.key("workflowInstanceKey"); w.integer(d.inst_key);
    w.key("activityId"); w.str(P.pool + e.id_off, e.id_len);
    w.key("activityInstanceKey"); w.integer(d.scope_key);
    w.key("jobKey"); w.integer(-1);
    w.key("payload"); w.bin((const uint8_t*)"\x80", 1);
  } else if (vt == ZB_VT_WORKFLOW_INSTANCE_SUBSCRIPTION) {  // WorkflowInstanceSubscriptionRecord.java:26-38
    const DevElem& e = P.elems[d.elem];
    w.map_hdr(4);
    w.key("workflowInstanceKey"); w.integer(d.inst_key);
    w.key("activityInstanceKey"); w.integer(d.scope_key);
    w.key("messageName"); w.str(P.pool + e.msg_off, e.msg_len);
    w.key("payload"); w.bin(pl, plen);
  } else if (vt == ZB_VT_MESSAGE_SUBSCRIPTION) {  // MessageSubscriptionRecord.java:26-41 (blob: zb_msg.hpp SubView)
    const SubView v = sub_view(P.arena, d.payload);
    w.map_hdr(5);
    w.key("workflowInstancePartitionId"); w.integer(v.wfp);
    w.key("workflowInstanceKey"); w.integer(d.inst_key);
    w.key("activityInstanceKey"); w.integer(d.scope_key);
    w.key("messageName"); w.str(v.name, v.nn);
    w.key("correlationKey"); w.str(v.ck, v.nc);
  } else if (vt == ZB_VT_MESSAGE) {  // MessageRecord.java:26-42 (blob: zb_msg.hpp MsgView)
    const MsgView v = msg_view(P.arena, d.payload);
    w.map_hdr(5);
    w.key("name"); w.str(v.name, v.nn);
    w.key("correlationKey"); w.str(v.ck, v.nc);
    w.key("timeToLive"); w.integer(v.ttl);
    w.key("payload"); w.bin(v.payload, v.np);
    w.key("messageId"); w.str(v.id, v.nid);
  }
}

// value size of record d. (Host-built value templates -- constant segments copied as whole words into the
// image -- were measured slower than this encoder on C3 10M: 8.9 vs 8.3 ms write pass, 1.40 G vs 1.06 G VALU
// instructions; the constant keys here compile to immediate stores. profiles/r02/pmc_c3g.json)
// The model tables the encoder reads per record (elements, workflows, the string pool) are a few hundred
// bytes for a typical deployment: every workgroup copies them into LDS once, which turns the
// descriptor -> element -> workflow -> string chain of dependent global loads into LDS reads.
constexpr uint32_t SER_MODEL_LDS = 4096;
__device__ __forceinline__ SerParams model_in_lds(const SerParams& P, uint8_t* sm, int nt) {
  if (!P.model_lds) return P;
  const uint32_t eb = (uint32_t)P.n_elems * (uint32_t)sizeof(DevElem), wb = (uint32_t)P.n_wfs * (uint32_t)sizeof(DevWorkflow);
  const uint32_t wo = (eb + 15) & ~15u, po = wo + ((wb + 15) & ~15u);
  for (uint32_t c = threadIdx.x; c < eb / 16; c += nt) ((uint4*)sm)[c] = ((const uint4*)P.elems)[c];
  for (uint32_t c = threadIdx.x; c < wb / 16; c += nt) ((uint4*)(sm + wo))[c] = ((const uint4*)P.wfs)[c];
  for (uint32_t c = threadIdx.x; c < P.pool_len; c += nt) sm[po + c] = P.pool[c];
  __syncthreads();
  SerParams Q = P;
  Q.elems = (const DevElem*)sm;
  Q.wfs = (const DevWorkflow*)(sm + wo);
  Q.pool = sm + po;
  return Q;
}

__device__ __forceinline__ uint32_t value_size(const SerParams& P, int64_t pos, const zb_rec& d) {
  W w;
  w.dst = nullptr;
  w.n = 0;
  encode_value(P, pos, d, w);
  return w.n;
}

// RejectionType: CREATE of an unknown workflow -> BAD_VALUE (0); CORRELATE of an absent activity, CANCEL /
// UPDATE_PAYLOAD of an instance that is not running -> NOT_APPLICABLE (1) (WorkflowInstanceStreamProcessor.java
// :477-479, :524-529, :571-573); job commands NOT_APPLICABLE but UPDATE_RETRIES with retries <= 0 BAD_VALUE
// (JobInstanceStreamProcessor.java:206-222; job_command keeps it in elem)
__device__ __forceinline__ uint8_t rejection_type(const zb_rec& d) {
  if (kind_rt(d.kind) != ZB_RT_COMMAND_REJECTION) return 255;
  const uint8_t vt = kind_vt(d.kind);
  if (vt == ZB_VT_WORKFLOW_INSTANCE && d.intent == WI_CREATE) return 0;
  if (vt == ZB_VT_JOB && d.intent == JI_UPDATE_RETRIES && (d.kind & KIND_RAW) && d.elem == 1) return 0;
  if (vt == ZB_VT_MESSAGE) return 0;  // a published message id (PublishMessageProcessor.java:77-84)
  return 1;
}

// ------------------------------------------------------------------------------ log frames (§8f rank 1)
// The frame layout and its 104-byte prefix: zb_frame.hpp (shared with the fast frame drains).

// rejection reasons of the commands this path rejects (WorkflowInstanceStreamProcessor.java:346-347, :527-529,
// :573, :478-479), of the job commands (JobInstanceStreamProcessor.java:155-158, :172-173, :186-187, :193,
// :215-220, :238) and of PUBLISH (PublishMessageProcessor.java:77-84: "message with id '%s' is already published",
// built around the message's id, reason 10)
__device__ const char* const REASONS[11] = {
    "", "Workflow is not deployed", "Workflow instance is not running", "activity is not active anymore",
    "Job is not in one of these states: CREATED, FAILED, TIMED_OUT", "Job is not in state: ACTIVATED, TIMED_OUT",
    "Job is not in state ACTIVATED", "Retries must be greater than 0", "Job is not in state FAILED",
    "Job does not exist", "message with id '"};
__device__ const char MSG_ID_TAIL[] = "' is already published";
__device__ __forceinline__ uint32_t reason_of(const zb_rec& d) {
  if (kind_rt(d.kind) != ZB_RT_COMMAND_REJECTION) return 0;
  const uint8_t vt = kind_vt(d.kind);
  if (vt == ZB_VT_WORKFLOW_INSTANCE) return d.intent == WI_CREATE ? 1 : 2;
  if (vt == ZB_VT_WORKFLOW_INSTANCE_SUBSCRIPTION) return 3;
  if (vt == ZB_VT_JOB) {
    switch (d.intent) {
      case JI_ACTIVATE: return 4;
      case JI_COMPLETE: return 5;
      case JI_FAIL: case JI_TIME_OUT: return 6;
      case JI_UPDATE_RETRIES: return rejection_type(d) == 0 ? 7 : 8;
      case JI_CANCEL: return 9;
    }
  }
  if (vt == ZB_VT_MESSAGE) return 10;
  return 0;
}
__device__ __forceinline__ uint32_t reason_len(const SerParams& P, const zb_rec& d, uint32_t r) {
  if (r == 10) return dstrlen(REASONS[10]) + msg_view(P.arena, d.payload).nid + dstrlen(MSG_ID_TAIL);
  return dstrlen(REASONS[r < 11 ? r : 0]);
}

__device__ __forceinline__ int64_t source_of(const SerParams& P, int64_t pos) {
  const uint32_t s = P.srcd[pos];
  return s ? pos - (int64_t)s : -1;
}

// frame of record d at log position pos into dst (8-aligned), or only its size (dst == nullptr); returns the
// aligned frame length
__device__ inline uint32_t encode_frame(const SerParams& P, int64_t pos, const zb_rec& d, uint8_t* dst) {
  const uint32_t rs = reason_of(d), rlen = reason_len(P, d, rs);
  W w;
  w.dst = dst ? dst + FRAME_PREFIX + rlen : nullptr;
  w.n = 0;
  encode_value(P, pos, d, w);
  const uint32_t framed = FRAME_PREFIX + rlen + w.n, fsize = (framed + 7) & ~7u;
  if (!dst) return fsize;
  const uint8_t vt = kind_vt(d.kind), rt = kind_rt(d.kind);
  const int64_t src = source_of(P, pos);
  uint32_t flags = 0;
  if (src >= 0) {
    const bool first = pos - 1 < P.log_begin || source_of(P, pos - 1) != src;
    const bool last = pos + 1 >= P.log_end || source_of(P, pos + 1) != src;
    flags = frame_flags(first, last);
  }
  uint64_t rid;
  uint32_t sid;
  frame_request(P.reqs, P.nreqs, frame_request_pos(pos, src, vt, rt, d.intent), rid, sid);
  uint64_t h[13];
  frame_words(h, FrameConst{P.stream_id, P.raft_term, P.timestamp}, framed, flags, pos, frame_producer(src, vt, rt, d.intent),
              src, d.key, rt, vt, d.intent, rejection_type(d), rlen, rid, sid);
  uint64_t* hd = (uint64_t*)dst;
#pragma unroll
  for (int j = 0; j < 13; j++) hd[j] = h[j];
  W r;
  r.dst = dst + FRAME_PREFIX;
  r.n = 0;
  if (rs) r.cstr(REASONS[rs < 11 ? rs : 0]);
  if (rs == 10) {
    const MsgView v = msg_view(P.arena, d.payload);
    r.put_bytes(v.id, v.nid);
    r.cstr(MSG_ID_TAIL);
  }
  for (uint32_t k = framed; k < fsize; k++) dst[k] = 0;
  return fsize;
}

// Size pass: value (or frame) length per record and the byte total of every 256-record tile (the write
// pass's tiles); the tile totals are scanned, each write-pass tile scans its own lengths. Values of the drain
// (len_in_vlen): the lengths the emitting kernels knew stay in vlen and only the measured ones are written
// there, so the pass reads 4 bytes per record and writes next to nothing. One 256-thread workgroup sizes
// SER_SIZE_TILES tiles (one per tile spent more on launching than on its 1 KB of lengths; 1024-thread
// workgroups cost occupancy: 0.73 ms vs 0.47 ms on C3 10M).
constexpr int SER_SIZE_TILES = 4;
template <bool FRAMES>
__global__ void __launch_bounds__(256) k_ser_size(SerParams P0) {
  __shared__ __attribute__((aligned(16))) uint8_t s_model[SER_MODEL_LDS];
  __shared__ unsigned long long s_sum[4 * SER_SIZE_TILES];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t n[SER_SIZE_TILES];
  bool measure[SER_SIZE_TILES], any = false;
#pragma unroll
  for (int j = 0; j < SER_SIZE_TILES; j++) {  // record i of tile j (coalesced 1 KB loads)
    const int64_t i = ((int64_t)blockIdx.x * SER_SIZE_TILES + j) * 256 + threadIdx.x;
    const bool live = i < P0.count;
    // the value length the emitting kernel knew, else the encoder's dry run (reads the record and its payload)
    n[j] = (live && P0.vlen) ? P0.vlen[P0.start + i] : VLEN_UNKNOWN;
    measure[j] = live && (n[j] == VLEN_UNKNOWN || P0.vlen_bad);  // (ZB_CFG_VLEN_CHECK: measure every record)
    any = any || measure[j];
    if (!live) n[j] = 0;
  }
  if (__syncthreads_or(any)) {  // the model tables go to LDS only for workgroups that encode
    const SerParams P = model_in_lds(P0, s_model, 256);
#pragma unroll 1
    for (int j = 0; j < SER_SIZE_TILES; j++) {
      if (!measure[j]) continue;
      const int64_t i = ((int64_t)blockIdx.x * SER_SIZE_TILES + j) * 256 + threadIdx.x;
      const int64_t pos = P.start + i;
      const zb_rec d = P.log[pos];
      // the fast encoder's records: the emit kernels' formula (element constant + key lengths + binary
      // payload); every other record, and every record under ZB_CFG_VLEN_CHECK, by the encoder's dry run
      const uint32_t m = (P.vconst && !P.vlen_bad && fast_kind(d))
          ? (kind_vt(d.kind) == ZB_VT_JOB ? P.vconst[d.elem].job : P.vconst[d.elem].wf) + mp_int_len(d.inst_key) +
                mp_int_len(d.scope_key) + mp_bin_len(*(const uint32_t*)(P.arena + (uint64_t)d.payload * 8))
          : value_size(P, pos, d);
      if (n[j] != VLEN_UNKNOWN && n[j] != m) atomicOr(P.vlen_bad, 1u);
      n[j] = FRAMES ? (FRAME_PREFIX + reason_len(P, d, reason_of(d)) + m + 7) & ~7u : m;
      if (P.len_in_vlen) P.vlen_out[pos] = n[j];
    }
  }
  const int64_t tiles = (P0.count + 255) / 256;
#pragma unroll
  for (int j = 0; j < SER_SIZE_TILES; j++) {
    const int64_t i = ((int64_t)blockIdx.x * SER_SIZE_TILES + j) * 256 + threadIdx.x;
    const bool live = i < P0.count;
    if (live && !measure[j] && FRAMES) {
      // a known value length (an emitting kernel's, or one a values drain measured and wrote back -- which
      // includes rejections): the frame adds the rejection reason of the record
      const zb_rec d = P0.log[P0.start + i];
      n[j] = (FRAME_PREFIX + reason_len(P0, d, reason_of(d)) + n[j] + 7) & ~7u;
    }
    if (live && !P0.len_in_vlen) P0.lengths[i] = n[j];
    unsigned long long y = n[j];
    for (int dd = 32; dd >= 1; dd >>= 1) y += __shfl_down(y, dd, 64);
    if (lane == 0) s_sum[4 * j + wv] = y;
  }
  if (!P0.tile_sums) return;
  __syncthreads();
  if (threadIdx.x < SER_SIZE_TILES) {
    const int64_t t = (int64_t)blockIdx.x * SER_SIZE_TILES + threadIdx.x;
    const int w = 4 * threadIdx.x;
    if (t < tiles) P0.tile_sums[t] = s_sum[w] + s_sum[w + 1] + s_sum[w + 2] + s_sum[w + 3];
    if (t == tiles) P0.tile_sums[t] = 0;  // the scan over tiles + 1 entries ends in the total
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && tiles % SER_SIZE_TILES == 0) P0.tile_sums[tiles] = 0;
}

// Write pass. Record i's value goes to out[offsets[i], offsets[i + 1]); the workgroup's records are one
// contiguous output range, so each thread encodes its value into an LDS image of that range (byte
// stores stay on chip) and the workgroup then streams the image out with 16-byte stores, aligned to
// the destination. A range larger than the image (large payloads) is encoded straight to HBM instead.
constexpr int SER_WG = 256;
constexpr int SER_IMG = 48 * 1024;  // three workgroups per CU

__device__ __forceinline__ zb_record_header record_header(const zb_rec& d, int64_t pos, uint32_t len, uint64_t off) {
  zb_record_header h;
  (void)pos;  // (implicit: start + index)
  h.key = d.key;
  h.record_type = kind_rt(d.kind);
  h.value_type = kind_vt(d.kind);
  h.intent = d.intent;
  h.rejection_type = rejection_type(d);
  h.value_length = len;
  h.value_offset = off;
  return h;
}

// streams image bytes [shift, shift + n) to out[o .. o + n) with 16-byte stores aligned to the destination
// (out + o - shift is 16-byte aligned)
__device__ __forceinline__ void stream_image(const uint8_t* img, uint8_t* out, uint64_t o, uint32_t shift, uint64_t n,
                                             bool nt) {
  uint8_t* dst = out + o - shift;
  const uint64_t lim = shift + n;  // image bytes [shift, lim) are ours
  const uint64_t full_lo = (shift + 15) & ~15ull, full_hi = lim & ~15ull;
  if (nt) {
    for (uint64_t c = full_lo + 16 * threadIdx.x; c < full_hi; c += 16 * SER_WG) {
      const uint4 v = *(const uint4*)(img + c);
      __builtin_nontemporal_store(v.x, (uint32_t*)(dst + c));
      __builtin_nontemporal_store(v.y, (uint32_t*)(dst + c) + 1);
      __builtin_nontemporal_store(v.z, (uint32_t*)(dst + c) + 2);
      __builtin_nontemporal_store(v.w, (uint32_t*)(dst + c) + 3);
    }
  } else {
    for (uint64_t c = full_lo + 16 * threadIdx.x; c < full_hi; c += 16 * SER_WG)
      *(uint4*)(dst + c) = *(const uint4*)(img + c);
  }
  const uint64_t head_end = full_lo < lim ? full_lo : lim;
  for (uint64_t c = shift + threadIdx.x; c < head_end; c += SER_WG) dst[c] = img[c];
  const uint64_t tail_lo = full_hi > head_end ? full_hi : head_end;
  for (uint64_t c = tail_lo + threadIdx.x; c < lim; c += SER_WG) dst[c] = img[c];
}

// Write pass: one workgroup per SER_WG-record tile. (A persistent grid with the next tile prefetched was
// measured slower -- 9.05 ms vs 8.32 ms on C3 10M, profiles/r02/ser_grid_sweep.txt -- and its loop cost the
// compiler 248 VGPRs.) A tile whose values exceed the image is written in windows: record k goes to window
// (off_k - o0) / ws with ws = image - longest value, so every window's records fit the image; the windows are
// encoded and streamed one after another (large values, e.g. C2's job records: 64 KB per tile). The phase loop
// lets the compiler spend 255 VGPRs unless told the LDS-bound occupancy (3 workgroups per CU): 168, no spills.
constexpr int SER_WINDOWS = 16;
template <bool FRAMES, bool NT>
__global__ void __launch_bounds__(SER_WG) __attribute__((amdgpu_waves_per_eu(3, 3))) k_ser_write(SerParams P0) {
  __shared__ __attribute__((aligned(16))) uint8_t img[SER_IMG + 16];
  __shared__ __attribute__((aligned(16))) uint8_t s_model[SER_MODEL_LDS + 16];  // (+16: 8-byte reads past the pool)
  __shared__ unsigned long long s_pay[SER_WG / 64];
  __shared__ unsigned long long s_wsum[SER_WG / 64];
  __shared__ uint32_t s_maxlen;
  __shared__ unsigned long long s_wlo[SER_WINDOWS], s_whi[SER_WINDOWS];
  const uint32_t tile = P0.tile_list_in ? P0.tile_list_in[blockIdx.x] : blockIdx.x;  // (the tiles k_ser_fast left)
  const int64_t base = (int64_t)tile * SER_WG;
  const int64_t i = base + threadIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool live = i < P0.count;
  // independent loads first; the model copy to LDS overlaps them
  zb_rec d{};
  uint64_t o0, o1, off = 0, nxt = 0, x = 0;
  uint32_t len = 0;
  if (P0.tile_offs) {  // tile offsets + lengths: this tile's exclusive scan in registers / LDS
    o0 = P0.tile_offs[tile];
    o1 = P0.tile_offs[tile + 1];
    if (live) len = P0.len_in_vlen ? P0.vlen[P0.start + i] : P0.lengths[i];
  } else {
    const int64_t last = (base + SER_WG < P0.count) ? base + SER_WG : P0.count;
    o0 = P0.offsets[base];
    o1 = P0.offsets[last];
    if (live) {
      off = P0.offsets[i];
      nxt = P0.offsets[i + 1];
    }
  }
  if (live) d = P0.log[P0.start + i];
  if (P0.tile_offs) {
    x = len;
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
      const uint64_t y = (uint64_t)__shfl_up((unsigned long long)x, k, 64);
      if (lane >= k) x += y;
    }
    if (lane == 63) s_wsum[wv] = x;
  }
  if (threadIdx.x == 0) s_maxlen = 0;
  const SerParams P = model_in_lds(P0, s_model, SER_WG);  // (ends in a barrier when the model goes to LDS)
  if (!P0.model_lds) __syncthreads();
  if (P.tile_offs) {
    uint64_t pre_w = 0;
#pragma unroll
    for (int k = 0; k < SER_WG / 64; k++)
      if (k < wv) pre_w += s_wsum[k];
    off = o0 + pre_w + x - len;
    nxt = off + len;
  }
  if (P.out_cap && o1 > P.out_cap) {  // does not fit: the host grows the buffer and runs the pass again
    if (threadIdx.x == 0) atomicOr(P.overflow, 1u);
    return;
  }
  if (!P.tile_offs) len = (uint32_t)(nxt - off);
  const uint32_t shift = (uint32_t)(((uintptr_t)(P.out + o0)) & 15);
  const bool staged = (o1 - o0) + shift <= (uint64_t)SER_IMG;
  uint64_t ws = 0;
  int nwin = 0;
  if (!staged) {
    if (live) atomicMax(&s_maxlen, len);
    if (threadIdx.x < SER_WINDOWS) { s_wlo[threadIdx.x] = ~0ull; s_whi[threadIdx.x] = 0; }
    __syncthreads();
    const uint32_t maxlen = s_maxlen;
    if (maxlen + 32 < (uint32_t)SER_IMG) {
      ws = (uint64_t)SER_IMG - 32 - maxlen;
      const uint64_t nw = (o1 - o0 + ws - 1) / ws;
      nwin = nw <= SER_WINDOWS ? (int)nw : 0;
    }
    if (nwin && live) {
      const int wk = (int)((off - o0) / ws);
      atomicMin(&s_wlo[wk], (unsigned long long)off);
      atomicMax(&s_whi[wk], (unsigned long long)nxt);
    }
    __syncthreads();
  }
  uint32_t pay = 0;
  const int64_t pos = P.start + i;
  if (live) {
    if (kind_vt(d.kind) != ZB_VT_INCIDENT && !(d.kind & KIND_RAW)) pay = *(const uint32_t*)(P.arena + (uint64_t)d.payload * 8);
    if (!FRAMES) {
      const zb_record_header h = record_header(d, pos, len, off);
      if (NT) {
        const uint64_t* hw = (const uint64_t*)&h;
        uint64_t* dh = (uint64_t*)(P.headers + i);
        for (int k = 0; k < (int)(sizeof(zb_record_header) / 8); k++) dh[k] = hw[k];  // (plain: L2 merges lines)
      } else {
        P.headers[i] = h;
      }
    }
  }
  if (P.totals) {
    unsigned long long y = pay;
    for (int dd = 32; dd >= 1; dd >>= 1) y += __shfl_down(y, dd, 64);
    if (lane == 0) s_pay[wv] = y;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long tt = 0;
      for (int k = 0; k < SER_WG / 64; k++) tt += s_pay[k];
      // one partial per workgroup, reduced by k_ser_sum: 400k same-address device atomics serialised the pass
      // (~2.4 ms of the empty pass on C3 10M, profiles/r02/ser_grid_sweep.txt)
      P.pay_part[tile] = tt;
    }
  }
  // the generic encoder in phases (one encode site keeps it inlined once): the whole tile staged, straight to
  // HBM, or one phase per window
  const int mywin = (nwin && live) ? (int)((off - o0) / ws) : -1;
  const int nph = nwin ? nwin : 1;
#pragma unroll 1
  for (int ph = 0; ph < nph; ph++) {
    uint64_t wlo = o0, whi = o1;
    uint32_t sh = shift;
    bool go = live;
    if (nwin) {
      wlo = s_wlo[ph];
      whi = s_whi[ph];
      if (wlo >= whi) continue;  // no value starts in this window (uniform)
      sh = (uint32_t)(((uintptr_t)(P.out + wlo)) & 15);
      go = mywin == ph;
    }
    const bool in_img = staged || nwin;
    const uint32_t lo = (uint32_t)(sh + (off - wlo));  // the record's image offset (staged / windowed)
    if (go) {
      uint8_t* dst = in_img ? img + lo : P.out + off;
      if (FRAMES) {
        (void)encode_frame(P, pos, d, dst);
      } else {
        W w;
        w.dst = dst;
        w.n = 0;
        encode_value(P, pos, d, w);
      }
    }
    if (in_img) {
      __syncthreads();
      stream_image(img, P.out, wlo, sh, whi - wlo, NT);
      __syncthreads();  // the image is reused by the next window
    }
  }
}

// payload-byte total of the write pass: every workgroup sums a slice of the per-tile partials, one atomic each
__global__ void __launch_bounds__(256) k_ser_sum(SerParams P, int64_t nparts) {
  __shared__ unsigned long long s[4];
  unsigned long long x = 0;
  for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < nparts; k += (int64_t)gridDim.x * 256) x += P.pay_part[k];
  for (int dd = 32; dd >= 1; dd >>= 1) x += __shfl_down(x, dd, 64);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = x;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd((unsigned long long*)&P.totals[1], s[0] + s[1] + s[2] + s[3]);
}


// Fast write pass, phase form (values + headers, no frames): one workgroup per 256-record tile as k_ser_write,
// but the LDS image holds ONE wave's records (64 values): the waves encode in turn and all four stream each
// wave's range out. It runs with a 40 KB image (3 workgroups per CU) over the tiles the wave-parallel pass
// (k_ser_wave, below) leaves because one of their values exceeds its image; tiles with a record the fast encoder
// does not take, or a wave range larger than 40 KB, go on to k_ser_write (tile_list).
constexpr int SER_FIMG_WIDE = 40 * 1024;
template <int IMG, bool LISTED>
__global__ void __launch_bounds__(SER_WG) __attribute__((amdgpu_waves_per_eu(3))) k_ser_fast(SerParams P0) {
  __shared__ __attribute__((aligned(16))) uint8_t img[IMG + 16];
  extern __shared__ __attribute__((aligned(16))) uint8_t s_model[];  // the constant runs (sized at launch)
  __shared__ unsigned long long s_wsum[SER_WG / 64], s_pay[SER_WG / 64];
  const uint32_t tile = LISTED ? P0.tile_list_in[blockIdx.x] : blockIdx.x;
  const int64_t base = (int64_t)tile * SER_WG;
  const int64_t i = base + threadIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool live = i < P0.count;
  const uint64_t o0 = P0.tile_offs[tile], o1 = P0.tile_offs[tile + 1];
  const uint32_t len = live ? (P0.len_in_vlen ? P0.vlen[P0.start + i] : P0.lengths[i]) : 0;
  zb_rec d{};
  if (live) d = P0.log[P0.start + i];
  const bool msg = live && fast_msg_kind(d);
  const bool fast = (live && fast_kind(d)) || msg;
  const uint64_t* dw = (const uint64_t*)(P0.arena + (uint64_t)d.payload * 8);
  uint64_t pre[SER_PRE];
#pragma unroll
  for (int j = 0; j < SER_PRE; j++)
    pre[j] = (fast && (uint64_t)d.payload * 8 + 8 * j + 8 <= P0.arena_bytes) ? dw[j] : 0;
  uint64_t x = len;
#pragma unroll
  for (int k = 1; k < 64; k <<= 1) {
    const uint64_t y = (uint64_t)__shfl_up((unsigned long long)x, k, 64);
    if (lane >= k) x += y;
  }
  if (lane == 63) s_wsum[wv] = x;
  // the elements' constant runs into LDS (their barrier is the vote's): table (4-byte words), pool (8-byte)
  const uint32_t tb = ((uint32_t)P0.n_elems * (uint32_t)sizeof(DevValSeg) + 15) & ~15u;
  for (uint32_t c = threadIdx.x; c < tb / 4; c += SER_WG) ((uint32_t*)s_model)[c] = ((const uint32_t*)P0.vsegs)[c];
  for (uint32_t c = threadIdx.x; c < P0.segpool_len / 8; c += SER_WG)
    ((uint64_t*)(s_model + tb))[c] = ((const uint64_t*)P0.segpool)[c];
  const bool all_fast = __syncthreads_and(fast || !live);
  bool fits = true;
#pragma unroll
  for (int k = 0; k < SER_WG / 64; k++) fits = fits && s_wsum[k] + 16 <= (uint64_t)IMG;
  if (P0.out_cap && o1 > P0.out_cap) {  // does not fit: the host grows the buffer and runs the pass again
    if (threadIdx.x == 0) atomicOr(P0.overflow, 1u);
    return;
  }
  if (!all_fast || !fits) {  // k_ser_write takes this tile
    if (threadIdx.x == 0) P0.tile_list[atomicAdd(P0.tile_list_n, 1u)] = tile;
    return;
  }
  uint64_t pw = 0;
#pragma unroll
  for (int k = 0; k < SER_WG / 64; k++)
    if (k < wv) pw += s_wsum[k];
  const uint64_t off = o0 + pw + x - len;
  if (live) {
    const zb_record_header h = record_header(d, P0.start + i, len, off);
    const uint64_t* hw = (const uint64_t*)&h;
    uint64_t* dh = (uint64_t*)(P0.headers + i);
    for (int k = 0; k < (int)(sizeof(zb_record_header) / 8); k++) dh[k] = hw[k];  // (plain: L2 merges lines)
  }
  if (P0.totals) {
    unsigned long long y = live ? (uint32_t)pre[0] : 0;
    for (int dd = 32; dd >= 1; dd >>= 1) y += __shfl_down(y, dd, 64);
    if (lane == 0) s_pay[wv] = y;
  }
  // phase k: wave k encodes its values into the image, then all four waves stream them out. Each wave runs
  // the phases before its own, its own (the encoder sits outside any loop: no constants hoisted into
  // registers for the whole kernel), then the rest -- the same barriers in the same order for every wave.
  auto stream_wave = [&](int k) {
    uint64_t lo = o0;
    for (int j = 0; j < k; j++) lo += s_wsum[j];
    const uint32_t sh = (uint32_t)(((uintptr_t)(P0.out + lo)) & 15);
    __syncthreads();
    stream_image(img, P0.out, lo, sh, s_wsum[k], true);
    __syncthreads();  // the image is reused by the next wave
  };
#pragma unroll 1
  for (int k = 0; k < wv; k++) stream_wave(k);
  if (live) {
    const uint64_t lo = o0 + pw;  // this wave's range starts at the tile start + the waves before it
    const uint32_t at = (uint32_t)(((uintptr_t)(P0.out + lo)) & 15) + (uint32_t)(off - lo);
    if (msg) {
      FastWT<true> w;
      w.begin(img, at);
      fast_encode_msg(w, d, (const DevValSeg*)s_model, s_model + tb, dw, pre);
    } else {
      FastW w;
      w.begin(img, at);
      fast_encode(w, d, (const DevValSeg*)s_model, s_model + tb, dw, pre);
    }
  }
  stream_wave(wv);
#pragma unroll 1
  for (int k = wv + 1; k < SER_WG / 64; k++) stream_wave(k);
  if (P0.totals && threadIdx.x == 0) P0.pay_part[tile] = s_pay[0] + s_pay[1] + s_pay[2] + s_pay[3];
}

// Fast write pass, wave-parallel form (the first pass of the descriptor drain): every wave has an image of its
// own and encodes its 64 records in rounds -- each lane its own record, the lanes whose values fit the image from
// the round's first byte -- then streams the round out; the four waves never wait for each other (the phase form
// above lets one wave encode at a time). A tile with a record the fast encoder does not take, or a single value
// larger than the image, goes to the next pass (tile_list: the 40 KB phase form, then k_ser_write; tile_list_slow:
// k_ser_write directly, for the tiles holding a record of a kind the fast encoder does not take).
constexpr uint32_t SER_WIMG = 11 * 1024 - 16;
// FRAMES (zb_serialize_frames): each lane's frame -- the 13 prefix words (zb_frame.hpp) and the value, padded to 8 --
// goes into the image at its 8-aligned offset; records with a rejection reason go to k_ser_write<true>
template <bool FRAMES>
__global__ void __launch_bounds__(SER_WG) __attribute__((amdgpu_waves_per_eu(3, 4))) k_ser_wave(SerParams P0) {
  // each wave's image, then its lanes' dummy slots (the branch-free writer's stores that must not land: FastWB)
  __shared__ __attribute__((aligned(16))) uint8_t s_img[SER_WG / 64][SER_WIMG + 16 + 8 * 64];
  extern __shared__ __attribute__((aligned(16))) uint8_t s_model[];  // the constant runs (sized at launch)
  __shared__ unsigned long long s_wsum[SER_WG / 64], s_pay[SER_WG / 64];
  const uint32_t tile = blockIdx.x;
  const int64_t base = (int64_t)tile * SER_WG;
  const int64_t i = base + threadIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool live = i < P0.count;
  const uint64_t o0 = P0.tile_offs[tile], o1 = P0.tile_offs[tile + 1];
  const uint32_t len = live ? (P0.len_in_vlen ? P0.vlen[P0.start + i] : P0.lengths[i]) : 0;
  zb_rec d{};
  if (live) d = P0.log[P0.start + i];
  const bool rej = FRAMES && kind_rt(d.kind) == ZB_RT_COMMAND_REJECTION;  // (frames: a rejection reason)
  const bool msg = live && !rej && fast_msg_kind(d);
  const bool fast = (live && !rej && fast_kind(d)) || msg;
  const uint64_t* dw = (const uint64_t*)(P0.arena + (uint64_t)d.payload * 8);
  uint64_t pre[SER_PRE];
#pragma unroll
  for (int j = 0; j < SER_PRE; j++)
    pre[j] = (fast && (uint64_t)d.payload * 8 + 8 * j + 8 <= P0.arena_bytes) ? dw[j] : 0;
  // frames: the record's source and its neighbours' (batch flags)
  int64_t src = -1;
  uint32_t fflags = 0;
  if (FRAMES && live) {
    const int64_t pos = P0.start + i;
    src = source_of(P0, pos);
    if (src >= 0) {
      const bool first = pos - 1 < P0.log_begin || source_of(P0, pos - 1) != src;
      const bool last = pos + 1 >= P0.log_end || source_of(P0, pos + 1) != src;
      fflags = frame_flags(first, last);
    }
  }
  uint64_t x = len;  // the wave's inclusive prefix of the value lengths
#pragma unroll
  for (int k = 1; k < 64; k <<= 1) {
    const uint64_t y = (uint64_t)__shfl_up((unsigned long long)x, k, 64);
    if (lane >= k) x += y;
  }
  if (lane == 63) s_wsum[wv] = x;
  // the elements' constant runs into LDS (their barrier is the vote's): table (4-byte words), pool (8-byte)
  const uint32_t tb = ((uint32_t)P0.n_elems * (uint32_t)sizeof(DevValSeg) + 15) & ~15u;
  for (uint32_t c = threadIdx.x; c < tb / 4; c += SER_WG) ((uint32_t*)s_model)[c] = ((const uint32_t*)P0.vsegs)[c];
  for (uint32_t c = threadIdx.x; c < P0.segpool_len / 8; c += SER_WG)
    ((uint64_t*)(s_model + tb))[c] = ((const uint64_t*)P0.segpool)[c];
  const bool all_fast = __syncthreads_and(!live || (fast && len + 16 <= SER_WIMG));
  if (P0.out_cap && o1 > P0.out_cap) {  // does not fit: the host grows the buffer and runs the pass again
    if (threadIdx.x == 0) atomicOr(P0.overflow, 1u);
    return;
  }
  if (!all_fast) {  // the next pass takes this tile: the 40 KB phase form if only a value's size is the reason
    const bool kinds = __syncthreads_and(!live || fast);
    if (threadIdx.x == 0) {
      if (kinds && !FRAMES) P0.tile_list[atomicAdd(P0.tile_list_n, 1u)] = tile;
      else P0.tile_list_slow[atomicAdd(P0.tile_list_n + 1, 1u)] = tile;  // (frames: k_ser_write<true>)
    }
    return;
  }
  uint64_t pw = 0;
#pragma unroll
  for (int k = 0; k < SER_WG / 64; k++)
    if (k < wv) pw += s_wsum[k];
  const uint64_t wlo = o0 + pw;  // this wave's range
  const uint32_t rel = (uint32_t)(x - len), incl = (uint32_t)x;  // this lane's value: [wlo + rel, wlo + incl)
  if (live && !FRAMES) {
    const zb_record_header h = record_header(d, P0.start + i, len, wlo + rel);
    const uint64_t* hw = (const uint64_t*)&h;
    uint64_t* dh = (uint64_t*)(P0.headers + i);
    for (int k = 0; k < (int)(sizeof(zb_record_header) / 8); k++) dh[k] = hw[k];  // (plain: L2 merges lines)
  }
  uint64_t rid = ~0ull;
  uint32_t sid = 0x80000000u;
  if (FRAMES && live && P0.nreqs) {
    const int64_t pos = P0.start + i;
    frame_request(P0.reqs, P0.nreqs, frame_request_pos(pos, src, kind_vt(d.kind), kind_rt(d.kind), d.intent), rid, sid);
  }
  if (P0.totals) {
    unsigned long long y = live ? (uint32_t)pre[0] : 0;
    for (int dd = 32; dd >= 1; dd >>= 1) y += __shfl_down(y, dd, 64);
    if (lane == 0) s_pay[wv] = y;
  }
  uint8_t* img = s_img[wv];
  const DevValSeg* tab = (const DevValSeg*)s_model;
  const uint8_t* segs = s_model + tb;
  // every key the wave's WORKFLOW_INSTANCE / JOB values carry is -1, 0 or in [2^16, 2^32): 5-byte integers (ival5)
  auto in5 = [](int64_t v) { return (uint64_t)(v + 1) <= 1 || (v >= 65536 && v < (1ll << 32)); };
  const bool l5 = __all(!live || msg || (in5(d.inst_key) && in5(d.scope_key)));
  constexpr uint32_t VO = FRAMES ? FRAME_PREFIX : 0u;  // the value's offset in the record's bytes
#pragma unroll 1
  for (int a = 0; a < 64;) {  // rounds: lanes [a, b) whose values fit the image from the round's first byte
    const uint32_t lo = __builtin_amdgcn_readlane(rel, a);
    const uint32_t sh = (uint32_t)(((uintptr_t)(P0.out + wlo + lo)) & 15);
    const bool fit = lane >= a && incl - lo + sh <= SER_WIMG;  // (lane a always fits: len + 16 <= the image)
    const uint64_t fm = __ballot(fit);
    const int b = 64 - __builtin_clzll(fm);
    if (fit && len) {
      const uint32_t at = sh + (rel - lo);
      uint32_t vn;
      if (msg) {
        FastWT<true> w;
        w.begin(img, at + VO);
        fast_encode_msg<FRAMES>(w, d, tab, segs, dw, pre);
        vn = w.n();
      } else {
        FastWB w;
        w.begin(img, at + VO, SER_WIMG + 16 + 8 * lane);
        if (l5) fast_encode<true, true, FRAMES>(w, d, tab, segs, dw, pre);
        else fast_encode<false, true, FRAMES>(w, d, tab, segs, dw, pre);
        vn = w.n();
      }
      if (FRAMES) {  // the prefix, once the value's length is known
        const uint8_t vt = kind_vt(d.kind), rt = kind_rt(d.kind);
        uint64_t h[13];
        frame_words(h, FrameConst{P0.stream_id, P0.raft_term, P0.timestamp}, FRAME_PREFIX + vn, fflags,
                    P0.start + i, frame_producer(src, vt, rt, d.intent), src, d.key, rt, vt, d.intent, 255, 0, rid, sid);
        frame_store_lds(img, at, h);
      }
    }
    const uint32_t hi = __builtin_amdgcn_readlane(incl, b - 1);
    wave_lds_sync();
    wave_stream(img, P0.out, wlo + lo, sh, hi - lo, lane);
    wave_lds_sync();  // the image is reused by the next round
    a = b;
  }
  __syncthreads();
  if (P0.totals && threadIdx.x == 0) P0.pay_part[tile] = s_pay[0] + s_pay[1] + s_pay[2] + s_pay[3];
}

// dynamic LDS of the fast passes: the segment table (whole 16-byte rows) + the segment pool
static uint32_t seg_lds_bytes(const SerParams& p) {
  return (((uint32_t)p.n_elems * (uint32_t)sizeof(DevValSeg) + 15) & ~15u) + p.segpool_len;
}
void launch_ser_fast(const SerParams& p, hipStream_t s) {
  if (p.count <= 0) return;
  const dim3 g((unsigned)((p.count + SER_WG - 1) / SER_WG));
  if (p.frames) hipLaunchKernelGGL(k_ser_wave<true>, g, dim3(SER_WG), seg_lds_bytes(p), s, p);
  else hipLaunchKernelGGL(k_ser_wave<false>, g, dim3(SER_WG), seg_lds_bytes(p), s, p);
}
void launch_ser_fast_wide(const SerParams& p, uint32_t n, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL((k_ser_fast<SER_FIMG_WIDE, true>), dim3(n), dim3(SER_WG), seg_lds_bytes(p), s, p);
}
void launch_ser_write_list(const SerParams& p, uint32_t n, hipStream_t s) {
  if (n == 0) return;
  if (p.frames) hipLaunchKernelGGL((k_ser_write<true, true>), dim3(n), dim3(SER_WG), 0, s, p);
  else if (p.nt) hipLaunchKernelGGL((k_ser_write<false, true>), dim3(n), dim3(SER_WG), 0, s, p);
  else hipLaunchKernelGGL((k_ser_write<false, false>), dim3(n), dim3(SER_WG), 0, s, p);
}
void launch_ser_sum(const SerParams& p, hipStream_t s) {
  const int64_t tiles = (p.count + SER_WG - 1) / SER_WG;
  if (p.count > 0 && p.totals)
    hipLaunchKernelGGL(k_ser_sum, dim3((unsigned)std::min<int64_t>(256, (tiles + 255) / 256)), dim3(256), 0, s, p, tiles);
}

// ------------------------------------------------------------------------------ single pass (zb_serialize)
// Size, offset and write in one launch: each 256-record tile sizes its values, scans them in LDS, gets
// its byte offset from its predecessors by decoupled look-back (tile ids in launch order from an atomic
// counter, so a tile only waits for tiles already running; status words are 8-byte agent-scope atomics
// on both sides, MI355X_MICROARCH.md "Valid forms"), then encodes into the LDS image and streams it out.
constexpr uint64_t TS_AGG = 1ull << 62, TS_INC = 2ull << 62, TS_VAL = (1ull << 44) - 1;

__device__ __forceinline__ uint64_t ts_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ts_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void __launch_bounds__(SER_WG) k_ser_fused(SerParams P0) {
  __shared__ __attribute__((aligned(16))) uint8_t img[SER_IMG + 16];
  __shared__ __attribute__((aligned(16))) uint8_t s_model[SER_MODEL_LDS];
  const SerParams P = model_in_lds(P0, s_model, SER_WG);
  __shared__ uint64_t s_wsum[SER_WG / 64];
  __shared__ unsigned long long s_pay[SER_WG / 64];
  __shared__ uint32_t s_tile;
  __shared__ uint64_t s_base;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x == 0) s_tile = atomicAdd(P.tile_ctr, 1u);
  __syncthreads();
  const uint32_t t = s_tile;
  const int64_t base = (int64_t)t * SER_WG;
  const int64_t i = base + threadIdx.x;
  zb_rec d{};
  uint32_t len = 0;
  if (i < P.count) {
    d = P.log[P.start + i];
    len = value_size(P, P.start + i, d);
  }
  // block exclusive scan of the lengths
  uint64_t x = len;
#pragma unroll
  for (int k = 1; k < 64; k <<= 1) {
    const uint64_t y = (uint64_t)__shfl_up((unsigned long long)x, k, 64);
    if (lane >= k) x += y;
  }
  if (lane == 63) s_wsum[wv] = x;
  __syncthreads();
  uint64_t pre = 0, agg = 0;
#pragma unroll
  for (int k = 0; k < SER_WG / 64; k++) {
    if (k < wv) pre += s_wsum[k];
    agg += s_wsum[k];
  }
  const uint64_t lo = pre + x - len;  // offset inside the tile
  const uint64_t tag = (uint64_t)(P.epoch & 0x3ffff) << 44;
  if (wv == 0) {  // decoupled look-back by the first wave
    uint64_t excl = 0;
    if (t == 0) {
      if (lane == 0) ts_store(P.tile_state, TS_INC | tag | agg);
    } else {
      if (lane == 0) ts_store(P.tile_state + t, TS_AGG | tag | agg);
      int64_t p = (int64_t)t - 1;
      for (;;) {
        const int64_t q = p - lane;
        uint64_t v = 0;
        bool inc = true;
        if (q >= 0) {
          uint64_t wd;
          do { wd = ts_load(P.tile_state + q); } while ((wd & ~(3ull << 62)) >> 44 != (tag >> 44) || !(wd >> 62));
          inc = (wd >> 62) == 2;
          v = wd & TS_VAL;
        }
        const uint64_t m = __ballot(inc);
        const int first = m ? __ffsll((unsigned long long)m) - 1 : 64;
        uint64_t s = lane <= first ? v : 0;
#pragma unroll
        for (int k = 32; k >= 1; k >>= 1) s += (uint64_t)__shfl_xor((unsigned long long)s, k, 64);
        excl += s;
        if (first < 64) break;
        p -= 64;
      }
      if (lane == 0) ts_store(P.tile_state + t, TS_INC | tag | (excl + agg));
    }
    if (lane == 0) {
      s_base = excl;
      if ((int64_t)(base + SER_WG) >= P.count && P.totals) P.totals[0] = excl + agg;  // the last tile
    }
  }
  __syncthreads();
  const uint64_t o0 = s_base;
  if (o0 + agg > P.out_cap) {  // does not fit: the host grows the buffer and runs the pass again
    if (threadIdx.x == 0) atomicOr(P.overflow, 1u);
    return;
  }
  const uint32_t shift = (uint32_t)(((uintptr_t)(P.out + o0)) & 15);
  const bool staged = agg + shift <= (uint64_t)SER_IMG;
  uint32_t pay = 0;
  if (i < P.count) {
    const int64_t pos = P.start + i;
    const uint64_t off = o0 + lo;
    W w;
    w.dst = staged ? img + shift + lo : P.out + off;
    w.n = 0;
    encode_value(P, pos, d, w);
    if (kind_vt(d.kind) != ZB_VT_INCIDENT && !(d.kind & KIND_RAW)) pay = *(const uint32_t*)(P.arena + (uint64_t)d.payload * 8);
    P.headers[i] = record_header(d, pos, len, off);
  }
  if (P.totals) {
    unsigned long long y = pay;
    for (int dd = 32; dd >= 1; dd >>= 1) y += __shfl_down(y, dd, 64);
    if (lane == 0) s_pay[wv] = y;
  }
  __syncthreads();
  if (P.totals && threadIdx.x == 0) {
    unsigned long long tt = 0;
    for (int k = 0; k < SER_WG / 64; k++) tt += s_pay[k];
    P.pay_part[t] = tt;  // reduced by k_ser_sum
  }
  if (!staged) return;
  uint8_t* dst = P.out + o0 - shift;
  const uint64_t lim = shift + agg;
  const uint64_t full_lo = (shift + 15) & ~15ull, full_hi = lim & ~15ull;
  for (uint64_t c = full_lo + 16 * threadIdx.x; c < full_hi; c += 16 * SER_WG)
    *(uint4*)(dst + c) = *(const uint4*)(img + c);
  const uint64_t head_end = full_lo < lim ? full_lo : lim;
  for (uint64_t c = shift + threadIdx.x; c < head_end; c += SER_WG) dst[c] = img[c];
  const uint64_t tail_lo = full_hi > head_end ? full_hi : head_end;
  for (uint64_t c = tail_lo + threadIdx.x; c < lim; c += SER_WG) dst[c] = img[c];
}

void launch_ser_fused(const SerParams& p, hipStream_t s) {
  if (p.count <= 0) return;
  const int64_t tiles = (p.count + SER_WG - 1) / SER_WG;
  hipLaunchKernelGGL(k_ser_fused, dim3((unsigned)tiles), dim3(SER_WG), 0, s, p);
  if (p.totals) hipLaunchKernelGGL(k_ser_sum, dim3((unsigned)std::min<int64_t>(256, (tiles + 255) / 256)), dim3(256), 0, s, p, tiles);
}

void launch_ser_size(const SerParams& p, hipStream_t s) {
  if (p.count <= 0) return;
  const int64_t work = p.count;
  constexpr int per = 256 * SER_SIZE_TILES;
  if (p.frames) hipLaunchKernelGGL(k_ser_size<true>, dim3((unsigned)((work + per - 1) / per)), dim3(256), 0, s, p);
  else hipLaunchKernelGGL(k_ser_size<false>, dim3((unsigned)((work + per - 1) / per)), dim3(256), 0, s, p);
}
void launch_ser_write(const SerParams& p, hipStream_t s) {
  if (p.count <= 0) return;
  const int64_t tiles = (p.count + SER_WG - 1) / SER_WG;
  if (p.frames) hipLaunchKernelGGL((k_ser_write<true, true>), dim3((unsigned)tiles), dim3(SER_WG), 0, s, p);
  else if (p.nt) hipLaunchKernelGGL((k_ser_write<false, true>), dim3((unsigned)tiles), dim3(SER_WG), 0, s, p);
  else hipLaunchKernelGGL((k_ser_write<false, false>), dim3((unsigned)tiles), dim3(SER_WG), 0, s, p);
  if (p.totals) hipLaunchKernelGGL(k_ser_sum, dim3((unsigned)std::min<int64_t>(256, (tiles + 255) / 256)), dim3(256), 0, s, p, tiles);
}

// ------------------------------------------------------------------------------ input injection
__global__ void k_inject(InjectParams P) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t base_ref = (uint32_t)(P.arena_base >> 3);
  for (int64_t i = tid; i < P.n; i += stride) {
    zb_rec d = P.staged[i];
    d.payload += base_ref;
    if (d.key == KEY_IS_POSITION) d.key = P.log_base + i;
    P.log[P.log_base + i] = d;
    P.links[P.log_base + i] = ~0ull;  // no rows yet
    P.srcd[P.log_base + i] = 0;       // written by another writer (client API, job processor, ...)
    P.vlen[P.log_base + i] = P.staged_vlen[i];
    P.cref[i] = d.payload;
  }
  const uint64_t nw = P.staged_bytes / 8;
  const uint64_t* src = (const uint64_t*)P.staged_arena;
  uint64_t* dst = (uint64_t*)(P.arena + P.arena_base);
  for (uint64_t i = tid; i < nw; i += stride) dst[i] = src[i];
}

__global__ void k_req_append(const StagedReq* in, uint64_t n, int64_t log_base, ReqMeta* out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const StagedReq r = in[i];
    out[i] = ReqMeta{log_base + r.idx, r.rid, r.sid, 0};
  }
}

void launch_req_append(const StagedReq* in, uint64_t n, int64_t log_base, ReqMeta* out, hipStream_t s) {
  if (n == 0) return;
  const uint64_t g = std::min<uint64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_req_append, dim3((unsigned)g), dim3(256), 0, s, in, n, log_base, out);
}

void launch_inject(const InjectParams& p, hipStream_t s) {
  int64_t work = p.n > (int64_t)(p.staged_bytes / 8) ? p.n : (int64_t)(p.staged_bytes / 8);
  int grid = (int)((work + 255) / 256);
  if (grid > 4096) grid = 4096;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(k_inject, dim3(grid), dim3(256), 0, s, p);
}

}  // namespace zbg
