// zb_wave.hip — the lockstep wave kernel (one launch per breadth-first generation of the log).
//
// One launch processes every record of generation g (log[begin, end)) and appends generation g+1
// at the log tail in exact reference log order: a record's follow-ups are contiguous and ordered
// by emission index, and records of generation g+1 are ordered by their parent's position
// (FIFO log processing == breadth-first waves). Keys come from an exclusive prefix
// sum of per-record "new key" counts in that order (KeyGenerator(1,5) / job KeyGenerator(2,5)).
//
// Structure (per workgroup of 256 threads, one record per thread, tiles claimed by a ticket):
//   1. process: decode descriptor, guards (BpmnStepProcessor.java:128-150), step handler
//      (BpmnStepProcessor.java:92-125 -> handlers) -> up to 4 output slots in registers, plus
//      counts (records, wf keys, job keys, rows, arena bytes); index mutations of existing rows
//   2. block scan of the 5 counts (wave64 shuffles + LDS)
//   3. decoupled look-back over predecessor tiles (8-byte {tag,value} granules, agent-scope
//      relaxed atomics: the granule IS the flag — cdna_hip_programming.md §6 G16 recipe R2)
//   4. write: keys, new rows (READY inserts), merged payloads, descriptors + row links
// The tile ticket makes every awaited predecessor a tile that a resident workgroup already owns,
// so the look-back cannot deadlock whatever the dispatch order.
#include <hip/hip_runtime.h>

#include "zb_devlib.hpp"
#include "zb_kernels.hpp"

namespace zbg {

constexpr int WG = 256;
constexpr int ITEMS = 2;           // records per thread per tile (item k of thread t = record k*WG + t)
constexpr int TILE = WG * ITEMS;
constexpr int MAX_SLOTS = 2;       // output records per item (one parent's batch emits <= 2 in every handler)

enum SlotFlags : uint8_t {
  SF_KEY_WF = 1,       // key = new wf key #ord
  SF_KEY_JOB = 2,      // key = new job key #ord
  SF_INST_WF = 4,      // inst_key = new wf key #ord (CREATE)
  SF_ROW_NEW = 8,      // row_self = new row #rord
  SF_ROW_INIT = 16,    // initialise that row as an ELEMENT_READY insert (ElementInstanceWriter.writeNewEvent)
  SF_PAY_MERGED = 32,  // payload = this thread's merge result
  SF_PAY_DETAIL = 64,  // payload = this thread's incident detail blob
  SF_COND_JOB = 128,   // GATEWAY_ACTIVATED of a conditional split: k_cond evaluates it before the next wave
};

struct Slot {
  zb_rec d;
  uint32_t rself, rscope;
  uint8_t flags, ord, rord, pad;
};

struct TState {
  Slot* s;  // this thread's MAX_SLOTS output slots, staged in LDS (dynamic indexing stays out of scratch)
  int ns, nwf, njob, nrow;
  uint32_t bytes;
  // one merge and one incident detail per thread at most
  bool merge;
  uint32_t m_src, m_tgt, m_len, m_bytes;
  bool detail;
  uint8_t d_type, d_code, d_a, d_b;
  uint16_t d_q;
  int64_t d_pos;
  uint32_t err, err_site;
  // stats
  uint32_t transitions, completed, created, merges;
  uint32_t merge_bytes, cond_bytes;
};

__device__ __forceinline__ void fail_at(TState& t, uint32_t flag, uint32_t site) {
  if (!t.err) t.err_site = site;
  t.err |= flag;
}

__device__ __forceinline__ const uint8_t* payload_ptr(const uint8_t* arena, uint32_t ref, uint32_t& len) {
  const uint8_t* p = arena + (uint64_t)ref * 8;
  len = *(const uint32_t*)p;
  return p + 4;
}

__device__ __forceinline__ uint32_t blob_bytes(uint32_t len) { return (4 + len + 7) & ~7u; }

__device__ __forceinline__ Slot& add_slot(TState& t) {
  if (t.ns >= MAX_SLOTS) { fail_at(t, DE_PROCESSING, 1); return t.s[MAX_SLOTS - 1]; }
  Slot& s = t.s[t.ns++];
  s.flags = 0; s.ord = 0; s.rord = 0;
  return s;
}

__device__ __forceinline__ void wf_event(TState& t, Slot& s, uint8_t intent, uint8_t cont) {
  s.d.intent = intent;
  s.d.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE, ZB_RT_EVENT, cont);
}

// ElementInstanceWriter.writeFollowUpEvent index side effects for a final state
__device__ __forceinline__ void remove_row(const WaveParams& P, uint32_t row) {
  RowMeta& m = P.rmeta[row];
  uint32_t parent = m.parent;
  m.state = 0;
  if (parent != NO_ROW) P.rmeta[parent].nchild -= 1;
}

__device__ void incident(TState& t, const zb_rec& rec, int64_t pos, uint8_t type, uint8_t code, uint8_t a,
                         uint8_t b, uint16_t q) {
  // BpmnStepContext.raiseIncident: IncidentIntent.CREATE command, key null
  Slot& s = add_slot(t);
  s.d.key = -1;
  s.d.scope_key = rec.key;  // activityInstanceKey = failing record's key
  s.d.inst_key = rec.inst_key;
  s.d.elem = rec.elem;
  s.d.intent = 0;
  s.d.kind = make_kind(ZB_VT_INCIDENT, ZB_RT_COMMAND, t.ns > 1);
  s.d.payload = 0;
  s.flags = SF_PAY_DETAIL;
  s.rself = NO_ROW;
  s.rscope = NO_ROW;
  t.detail = true;
  t.d_type = type; t.d_code = code; t.d_a = a; t.d_b = b; t.d_q = q; t.d_pos = pos;
  t.bytes += 24;  // [u32 len=16][type code a b][u16 q][pad][i64 position]
}

__device__ void bpmn_step(const WaveParams& P, const zb_rec& rec, int64_t pos, uint32_t rself, uint32_t rscope,
                          TState& t) {
  const uint8_t intent = rec.intent;
  // stateless records (SFT/SEO/EEO/GA) never have an element instance; GA's link carries a decision
  const bool stateless = intent == WI_SEQUENCE_FLOW_TAKEN || intent == WI_START_EVENT_OCCURRED ||
                         intent == WI_END_EVENT_OCCURRED || intent == WI_GATEWAY_ACTIVATED;
  const bool self_alive = !stateless && rself != NO_ROW && P.rmeta[rself].state != 0;
  const bool scope_alive = rscope != NO_ROW && P.rmeta[rscope].state != 0;
  if (!self_alive && !scope_alive) return;  // BpmnStepProcessor.java:244-247
  bool ok;
  switch (intent) {
    case WI_ELEMENT_READY: case WI_ELEMENT_ACTIVATED: case WI_ELEMENT_COMPLETING:
      if (!self_alive) { fail_at(t, DE_PROCESSING, 2); return; }  // NPE in noConcurrentTransitionGuard
      ok = P.rmeta[rself].state == intent;
      break;
    case WI_ELEMENT_COMPLETED: case WI_END_EVENT_OCCURRED: case WI_GATEWAY_ACTIVATED:
    case WI_START_EVENT_OCCURRED: case WI_SEQUENCE_FLOW_TAKEN:
      ok = scope_alive && P.rmeta[rscope].state == WI_ELEMENT_ACTIVATED;
      break;
    case WI_ELEMENT_TERMINATING: ok = true; break;
    case WI_ELEMENT_TERMINATED: ok = scope_alive && P.rmeta[rscope].state == WI_ELEMENT_TERMINATING; break;
    default: ok = false;
  }
  if (!ok) return;
  if (rec.elem == NO_ELEM) { fail_at(t, DE_PROCESSING, 3); return; }
  const DevElem el = P.elems[rec.elem];
  const uint8_t step = el.step[intent];
  if (step == ST_UNBOUND || step == ST_NONE) return;

  switch (step) {
    case ST_APPLY_INPUT_MAPPING: {  // InputMappingHandler (no mappings: io mappings are rejected at deploy)
      Slot& s = add_slot(t);
      s.d = rec;
      wf_event(t, s, WI_ELEMENT_ACTIVATED, t.ns > 1);
      s.rself = rself; s.rscope = rscope;
      RowMeta& m = P.rmeta[rself];
      m.state = WI_ELEMENT_ACTIVATED;
      m.payload = rec.payload;
      break;
    }
    case ST_APPLY_OUTPUT_MAPPING: {  // OutputMappingHandler :42-85, outputBehavior null -> merge
      if (!scope_alive) { fail_at(t, DE_PROCESSING, 4); return; }
      // The merge itself runs once, in the write phase, into an arena blob sized by the upper bound
      // |result| <= |source| + |target| + 3 (root header grows by <= 4, sub-headers / keys are
      // re-encoded minimally so never grow): no size pass on the hot path.
      const uint32_t tref = P.rmeta[rscope].payload;
      const uint32_t ns_ = *(const uint32_t*)(P.arena + (uint64_t)rec.payload * 8);
      const uint32_t nt_ = *(const uint32_t*)(P.arena + (uint64_t)tref * 8);
      if (t.merge) { fail_at(t, DE_UNSUPPORTED, 7); return; }
      t.merge = true;
      t.m_src = rec.payload; t.m_tgt = tref; t.m_len = ns_ + nt_ + 8;
      t.m_bytes = blob_bytes(t.m_len);
      t.bytes += t.m_bytes;
      Slot& s = add_slot(t);
      s.d = rec;
      wf_event(t, s, WI_ELEMENT_COMPLETED, t.ns > 1);
      s.flags |= SF_PAY_MERGED;
      s.rself = rself; s.rscope = rscope;
      remove_row(P, rself);
      break;
    }
    case ST_CREATE_JOB: {  // CreateJobHandler :33-56 -> JOB CREATE command, key null
      Slot& s = add_slot(t);
      s.d = rec;
      s.d.key = -1;
      s.d.scope_key = rec.key;  // headers.activityInstanceKey
      s.d.intent = JI_CREATE;
      s.d.kind = make_kind(ZB_VT_JOB, ZB_RT_COMMAND, t.ns > 1);
      s.rself = rself; s.rscope = rscope;
      break;
    }
    case ST_EXCLUSIVE_SPLIT: {  // ExclusiveSplitHandler :38-71, decision computed by k_cond (zb_aux.hip)
      // the GATEWAY_ACTIVATED record is stateless, so its row-self link carries the decision
      const uint32_t dec = rself;
      if (!(dec & COND_VALID)) { fail_at(t, DE_PROCESSING, 20); return; }
      if (dec & COND_UNSUPPORTED) { fail_at(t, DE_UNSUPPORTED, 21); return; }
      if (dec & COND_INCIDENT) {
        incident(t, rec, pos, 3 /*CONDITION_ERROR*/, (dec >> 27) & 7, (dec >> 23) & 15, (dec >> 19) & 15,
                 (uint16_t)(dec & 0xffff));
        break;
      }
      Slot& s = add_slot(t);
      s.d = rec;
      s.d.elem = (uint16_t)(dec & 0xffff);
      wf_event(t, s, WI_SEQUENCE_FLOW_TAKEN, t.ns > 1);
      s.flags |= SF_KEY_WF; s.ord = (uint8_t)t.nwf++;
      s.rself = NO_ROW; s.rscope = rscope;
      break;
    }
    case ST_CONSUME_TOKEN: {  // ConsumeTokenHandler :30-43
      if (!scope_alive) { fail_at(t, DE_PROCESSING, 9); return; }
      RowMeta& m = P.rmeta[rscope];
      const RowKeys k = P.rkeys[rscope];
      Slot& s = add_slot(t);
      s.d.key = k.key;
      s.d.scope_key = k.scope_key;
      s.d.inst_key = k.inst_key;
      s.d.elem = m.elem;
      s.d.payload = rec.payload;
      wf_event(t, s, WI_ELEMENT_COMPLETING, t.ns > 1);
      s.rself = rscope; s.rscope = m.parent;
      m.state = WI_ELEMENT_COMPLETING;
      m.payload = rec.payload;
      break;
    }
    case ST_TAKE_SEQUENCE_FLOW:
    case ST_ACTIVATE_GATEWAY:
    case ST_TRIGGER_END_EVENT: {
      Slot& s = add_slot(t);
      s.d = rec;
      uint8_t out_intent;
      if (step == ST_TAKE_SEQUENCE_FLOW) { s.d.elem = el.out0; out_intent = WI_SEQUENCE_FLOW_TAKEN; }
      else if (step == ST_ACTIVATE_GATEWAY) { s.d.elem = el.target; out_intent = WI_GATEWAY_ACTIVATED; }
      else { s.d.elem = el.target; out_intent = WI_END_EVENT_OCCURRED; }
      if (s.d.elem == NO_ELEM) { fail_at(t, DE_PROCESSING, 10); return; }
      wf_event(t, s, out_intent, t.ns > 1);
      s.flags |= SF_KEY_WF; s.ord = (uint8_t)t.nwf++;
      if (step == ST_ACTIVATE_GATEWAY && P.elems[s.d.elem].step[WI_GATEWAY_ACTIVATED] == ST_EXCLUSIVE_SPLIT)
        s.flags |= SF_COND_JOB;
      s.rself = NO_ROW; s.rscope = rscope;
      break;
    }
    case ST_START_STATEFUL_ELEMENT: {  // -> ELEMENT_READY(new key), index insert with parent = scope
      Slot& s = add_slot(t);
      s.d = rec;
      s.d.elem = el.target;
      wf_event(t, s, WI_ELEMENT_READY, t.ns > 1);
      s.flags |= SF_KEY_WF | SF_ROW_NEW | SF_ROW_INIT;
      s.ord = (uint8_t)t.nwf++;
      s.rord = (uint8_t)t.nrow++;
      s.rself = NO_ROW; s.rscope = scope_alive ? rscope : NO_ROW;
      if (scope_alive) P.rmeta[rscope].nchild += 1;
      break;
    }
    case ST_TRIGGER_START_EVENT: {  // TriggerStartEventHandler :30-39
      if (el.start == NO_ELEM) { fail_at(t, DE_PROCESSING, 11); return; }
      Slot& s = add_slot(t);
      s.d = rec;
      s.d.elem = el.start;
      s.d.scope_key = rec.key;
      wf_event(t, s, WI_START_EVENT_OCCURRED, t.ns > 1);
      s.flags |= SF_KEY_WF; s.ord = (uint8_t)t.nwf++;
      s.rself = NO_ROW; s.rscope = rself;
      break;
    }
    case ST_COMPLETE_PROCESS: {  // CompleteProcessHandler :28-35
      Slot& s = add_slot(t);
      s.d = rec;
      wf_event(t, s, WI_ELEMENT_COMPLETED, t.ns > 1);
      s.rself = rself; s.rscope = rscope;
      remove_row(P, rself);
      if (rec.key == rec.inst_key) t.completed += 1;
      break;
    }
    default:
      // message subscription, termination: not on the GPU path yet (flagged, never silently skipped)
      fail_at(t, DE_UNSUPPORTED, 12);
      break;
  }
}

__device__ void process_record(const WaveParams& P, const zb_rec& rec, int64_t pos, uint32_t rself,
                               uint32_t rscope, TState& t) {
  const uint8_t vt = kind_vt(rec.kind), rt = kind_rt(rec.kind);
  if (vt == ZB_VT_WORKFLOW_INSTANCE) {
    if (rt == ZB_RT_COMMAND) {
      if (rec.intent != WI_CREATE) { fail_at(t, DE_UNSUPPORTED, 13); return; }
      // CreateWorkflowInstanceEventProcessor :233-368: key first, then resolve (done at submit)
      const uint8_t ord = (uint8_t)t.nwf++;
      if (rec.elem == NO_ELEM) {
        Slot& s = add_slot(t);
        s.d = rec;
        s.d.scope_key = pos;  // command position -> serializer finds the submitted command value
        s.d.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE, ZB_RT_COMMAND_REJECTION, t.ns > 1);
        s.flags = SF_INST_WF;
        s.ord = ord;
        s.rself = NO_ROW; s.rscope = NO_ROW;
        return;
      }
      const uint8_t rord = (uint8_t)t.nrow++;
      for (int k = 0; k < 2; k++) {
        Slot& s = add_slot(t);
        s.d = rec;
        s.d.scope_key = -1;
        s.d.intent = k == 0 ? WI_CREATED : WI_ELEMENT_READY;
        s.d.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE, ZB_RT_EVENT, t.ns > 1);
        s.flags = SF_KEY_WF | SF_INST_WF | SF_ROW_NEW;
        s.ord = ord;
        s.rord = rord;
        s.rself = NO_ROW; s.rscope = NO_ROW;
      }
    } else if (rt == ZB_RT_EVENT) {
      if (rec.intent == WI_CREATED) {  // WorkflowInstanceCreatedEventProcessor: index insert (READY)
        if (rself == NO_ROW) { fail_at(t, DE_ROWS_FULL, 14); return; }
        RowMeta m;
        m.payload = rec.payload; m.parent = NO_ROW; m.elem = rec.elem; m.state = WI_ELEMENT_READY; m.flags = 0;
        m.nchild = 0;
        P.rmeta[rself] = m;
        P.rkeys[rself] = RowKeys{rec.key, rec.scope_key, rec.inst_key, 0};
        t.created += 1;
      } else if (rec.intent <= WI_ELEMENT_TERMINATED && rec.intent >= WI_START_EVENT_OCCURRED) {
        bpmn_step(P, rec, pos, rself, rscope, t);
      }
    }
  } else if (vt == ZB_VT_JOB) {
    if (rt == ZB_RT_COMMAND && rec.intent == JI_CREATE) {
      // canonical harness: JOB CREATED(k), JOB COMPLETED(k), k from the job key generator
      const uint8_t ord = (uint8_t)t.njob++;
      for (int k = 0; k < 2; k++) {
        Slot& s = add_slot(t);
        s.d = rec;
        s.d.intent = k == 0 ? JI_CREATED : JI_COMPLETED;
        s.d.kind = make_kind(ZB_VT_JOB, ZB_RT_EVENT, t.ns > 1);
        if (k == 1) s.d.payload = P.elems[rec.elem].job_payload;
        s.flags = SF_KEY_JOB;
        s.ord = ord;
        s.rself = rself; s.rscope = rscope;
      }
    } else if (rt == ZB_RT_EVENT && rec.intent == JI_CREATED) {  // JobCreatedProcessor :408-426
      if (rec.scope_key > 0 && rself != NO_ROW && P.rmeta[rself].state != 0) P.rkeys[rself].job_key = rec.key;
    } else if (rt == ZB_RT_EVENT && rec.intent == JI_COMPLETED) {  // JobCompletedEventProcessor :428-453
      if (rself == NO_ROW || P.rmeta[rself].state == 0) return;
      RowMeta& m = P.rmeta[rself];
      RowKeys& k = P.rkeys[rself];
      Slot& s = add_slot(t);
      s.d.key = rec.scope_key;
      s.d.scope_key = k.scope_key;
      s.d.inst_key = k.inst_key;
      s.d.elem = m.elem;
      s.d.payload = rec.payload;
      wf_event(t, s, WI_ELEMENT_COMPLETING, t.ns > 1);
      s.rself = rself; s.rscope = m.parent;
      m.state = WI_ELEMENT_COMPLETING;
      m.payload = rec.payload;
      k.job_key = -1;
    }
  }
}

// ------------------------------------------------------------------------------ scan helpers
// Tile counts packed like the status granules: a = rec << 28 | wf, b = job << 28 | row, c = bytes.
// Sums of packed values never carry between fields (per-wave totals < 2^28, checked on the host).
struct Cnt {
  uint64_t a, b, c;
};
__device__ __forceinline__ Cnt cnt_add(const Cnt& x, const Cnt& y) { return Cnt{x.a + y.a, x.b + y.b, x.c + y.c}; }
__device__ __forceinline__ uint64_t shfl_up64(uint64_t v, int d) {
  return (uint64_t)__shfl_up((unsigned long long)v, d, 64);
}
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int d) {
  return (uint64_t)__shfl_xor((unsigned long long)v, d, 64);
}
constexpr uint64_t F28 = 0xfffffffull;
constexpr uint64_t F56 = 0xffffffffffffffull;

__device__ __forceinline__ void publish(unsigned long long* st, int64_t tile, uint32_t tag, const Cnt& c) {
  const unsigned long long t8 = (unsigned long long)tag << 56;
  __hip_atomic_store(st + 3 * tile + 0, t8 | (c.a & F56), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(st + 3 * tile + 1, t8 | (c.b & F56), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(st + 3 * tile + 2, t8 | (c.c & F56), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------------------ the kernel
struct ItemInfo {  // per (thread, item) write-phase inputs, staged in LDS (32 B)
  uint32_t m_src, m_tgt, m_len, m_bytes;  // merge (m_bytes == 0: none)
  int64_t d_pos;                          // incident detail
  uint16_t d_q;
  uint8_t d_type, d_code, d_a, d_b, has_detail, ns;
};

__global__ void __launch_bounds__(WG) k_wave(WaveParams P) {
  __shared__ uint64_t s_a[ITEMS][WG / 64];  // per-wave totals of packed rec|wf|job|row (16 bit each)
  __shared__ uint64_t s_b[ITEMS][WG / 64];  // bytes
  __shared__ Cnt s_excl;                    // tile exclusive prefix
  __shared__ int64_t s_tile;
  __shared__ uint32_t s_err;
  __shared__ uint32_t s_stats[6];
  __shared__ Slot s_slots[WG * ITEMS * MAX_SLOTS];
  __shared__ ItemInfo s_info[WG * ITEMS];

  const WaveHdr* hin = P.hdr + (P.wave & 1);
  WaveHdr* hout = P.hdr + ((P.wave + 1) & 1);
  const int64_t begin = hin->begin, end = hin->end;
  const int64_t n = end - begin;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t epoch = (uint32_t)(P.wave % 127) + 1;

  if (blockIdx.x == 0 && threadIdx.x == 0) {
    P.tickets[(P.wave + 1) & 127] = 0;
    // the other parity's job lists were consumed by the aux kernels of wave - 1 (stream order); clear
    // them for wave + 1 (this wave's lists were cleared the same way by wave - 1 / zb_reset)
    P.merge_count[(P.wave + 1) & 1] = 0;
    P.cond_count[(P.wave + 1) & 1] = 0;
  }
  if (n <= 0) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *hout = *hin;
    return;
  }
  const int64_t ntiles = (n + TILE - 1) / TILE;
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd((unsigned long long*)&P.stats[6], 1ull);
  if (threadIdx.x < 6) s_stats[threadIdx.x] = 0;
  if (threadIdx.x == 0) s_err = 0;
  uint32_t st_trans = 0, st_completed = 0, st_created = 0, st_merges = 0, st_mbytes = 0, st_cbytes = 0;

  for (;;) {
    if (threadIdx.x == 0) s_tile = (int64_t)atomicAdd(P.tickets + (P.wave & 127), 1u);
    __syncthreads();
    const int64_t tile = s_tile;
    if (tile >= ntiles) break;

    // ---------------- 1. process (item k of this thread = record tile*TILE + k*WG + tid)
    uint64_t a[ITEMS], b[ITEMS];
    uint32_t err = 0, err_site = 0;
    int64_t err_pos = 0;
#pragma unroll 1
    for (int k = 0; k < ITEMS; k++) {
      TState t;
      t.s = s_slots + (threadIdx.x * ITEMS + k) * MAX_SLOTS;
      t.ns = t.nwf = t.njob = t.nrow = 0;
      t.bytes = 0; t.merge = false; t.detail = false; t.err = 0; t.err_site = 0;
      t.transitions = t.completed = t.created = t.merges = 0;
      t.merge_bytes = t.cond_bytes = 0;
      const int64_t r = begin + tile * TILE + k * WG + threadIdx.x;
      if (r < end) {
        const zb_rec rec = P.log[r];
        if (!kind_cont(rec.kind)) {
          // a thread owns its record plus the continuation records that follow it (one parent's batch)
          const uint64_t lk = P.links[r];
          process_record(P, rec, r, (uint32_t)lk, (uint32_t)(lk >> 32), t);
          for (int64_t q = r + 1; q < end && q < r + 4; q++) {
            const zb_rec rec2 = P.log[q];
            if (!kind_cont(rec2.kind)) break;
            const uint64_t lk2 = P.links[q];
            process_record(P, rec2, q, (uint32_t)lk2, (uint32_t)(lk2 >> 32), t);
          }
        }
      }
      ItemInfo inf;
      inf.m_src = t.m_src; inf.m_tgt = t.m_tgt; inf.m_len = t.m_len; inf.m_bytes = t.merge ? t.m_bytes : 0;
      inf.d_pos = t.d_pos; inf.d_q = t.d_q; inf.d_type = t.d_type; inf.d_code = t.d_code; inf.d_a = t.d_a;
      inf.d_b = t.d_b; inf.has_detail = t.detail; inf.ns = (uint8_t)t.ns;
      s_info[threadIdx.x * ITEMS + k] = inf;
      a[k] = (uint64_t)t.ns | ((uint64_t)t.nwf << 16) | ((uint64_t)t.njob << 32) | ((uint64_t)t.nrow << 48);
      b[k] = t.bytes;
      if (t.err && !err) { err_site = t.err_site; err_pos = r; }
      err |= t.err;
      st_created += t.created; st_merges += t.merges; st_mbytes += t.merge_bytes; st_cbytes += t.cond_bytes;
      st_completed += t.completed;
    }

    // ---------------- 2. block scan, item-major order (all of item 0, then all of item 1)
    uint64_t ea[ITEMS], eb[ITEMS];
    uint64_t ta = 0, tb = 0;
#pragma unroll
    for (int k = 0; k < ITEMS; k++) {
      uint64_t ia = a[k], ib = b[k];
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        uint64_t ua = shfl_up64(ia, d), ub = shfl_up64(ib, d);
        if (lane >= d) { ia += ua; ib += ub; }
      }
      if (lane == 63) { s_a[k][wv] = ia; s_b[k][wv] = ib; }
      ea[k] = ia - a[k];
      eb[k] = ib - b[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < ITEMS; k++) {
      uint64_t wa = 0, wb = 0, ka = 0, kb = 0;
#pragma unroll
      for (int w = 0; w < WG / 64; w++) {
        if (w < wv) { wa += s_a[k][w]; wb += s_b[k][w]; }
        ka += s_a[k][w]; kb += s_b[k][w];
      }
      ea[k] += wa + ta;
      eb[k] += wb + tb;
      ta += ka;
      tb += kb;
    }
    const Cnt agg{((ta & 0xffff) << 28) | ((ta >> 16) & 0xffff), (((ta >> 32) & 0xffff) << 28) | (ta >> 48), tb};

    // ---------------- 3. decoupled look-back (wave 0), 256 predecessors per round trip
    if (wv == 0) {
      Cnt excl{0, 0, 0};
      if (tile == 0) {
        if (lane == 0) publish(P.status, 0, (epoch << 1) | 1, agg);
      } else {
        if (lane == 0) publish(P.status, tile, (epoch << 1) | 0, agg);
        int64_t base = tile - 1;
        uint32_t spins = 0;
        bool timeout = false;
        for (;;) {
          Cnt v[4];
          int first_local = 1 << 30;  // smallest window offset of a prefix this lane holds
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const int off = lane + 64 * j;
            const int64_t idx = base - off;
            v[j] = Cnt{0, 0, 0};
            if (idx < 0) { if (off < first_local) first_local = off; continue; }
            for (;;) {
              unsigned long long* g = P.status + 3 * idx;
              unsigned long long g0 = __hip_atomic_load(g + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              unsigned long long g1 = __hip_atomic_load(g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              unsigned long long g2 = __hip_atomic_load(g + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              uint32_t t0 = (uint32_t)(g0 >> 56), t1 = (uint32_t)(g1 >> 56), t2 = (uint32_t)(g2 >> 56);
              if (t0 == t1 && t1 == t2 && (t0 >> 1) == epoch) {
                v[j] = Cnt{g0 & F56, g1 & F56, g2 & F56};
                if ((t0 & 1) && off < first_local) first_local = off;
                break;
              }
              if (++spins > (1u << 24)) { timeout = true; if (off < first_local) first_local = off; break; }
              __builtin_amdgcn_s_sleep(1);
            }
          }
          // nearest predecessor holding an inclusive prefix (window offset), wave-wide minimum
          int first = first_local;
#pragma unroll
          for (int d = 32; d >= 1; d >>= 1) {
            int o = __shfl_xor(first, d, 64);
            first = o < first ? o : first;
          }
          Cnt c{0, 0, 0};
#pragma unroll
          for (int j = 0; j < 4; j++)
            if (lane + 64 * j <= first) c = cnt_add(c, v[j]);
#pragma unroll
          for (int d = 32; d >= 1; d >>= 1) {
            c.a += shfl_xor64(c.a, d); c.b += shfl_xor64(c.b, d); c.c += shfl_xor64(c.c, d);
          }
          excl = cnt_add(excl, c);
          if (first < 256) break;
          base -= 256;
        }
        if (__any(timeout) && lane == 0) atomicOr(&s_err, (uint32_t)DE_LOOKBACK_TIMEOUT);
        if (lane == 0) publish(P.status, tile, (epoch << 1) | 1, cnt_add(excl, agg));
      }
      if (lane == 0) s_excl = excl;
    }
    __syncthreads();
    const Cnt ex = s_excl;

    // ---------------- 4. write
#pragma unroll 1
    for (int k = 0; k < ITEMS; k++) {
      const ItemInfo inf = s_info[threadIdx.x * ITEMS + k];
      uint64_t out_rec = (uint64_t)end + (ex.a >> 28) + (ea[k] & 0xffff);
      const uint64_t wf0 = (ex.a & F28) + ((ea[k] >> 16) & 0xffff);
      const uint64_t job0 = (ex.b >> 28) + ((ea[k] >> 32) & 0xffff);
      const uint64_t row0 = (uint64_t)hin->rows_next + (ex.b & F28) + (ea[k] >> 48);
      uint64_t bump = (uint64_t)hin->arena_next + ex.c + eb[k];
      uint32_t merged_ref = 0, detail_ref = 0;
      if (inf.m_bytes) {
        // reserve the blob; k_merge (zb_aux.hip) fills it before the next wave reads any payload
        if (bump + inf.m_bytes > P.arena_cap) err |= DE_ARENA_FULL;
        else {
          merged_ref = (uint32_t)(bump >> 3);
          const uint32_t j = atomicAdd(P.merge_count + (P.wave & 1), 1u);
          if (j >= P.job_cap) err |= DE_LOG_FULL;
          else P.merge_jobs[(uint64_t)(P.wave & 1) * P.job_cap + j] = MergeJob{merged_ref, inf.m_src, inf.m_tgt, inf.m_len};
        }
        bump += inf.m_bytes;
      }
      if (inf.has_detail) {
        if (bump + 24 > P.arena_cap) err |= DE_ARENA_FULL;
        else {
          detail_ref = (uint32_t)(bump >> 3);
          uint8_t* dst = P.arena + bump;
          *(uint32_t*)dst = 16;
          dst[4] = inf.d_type; dst[5] = inf.d_code; dst[6] = inf.d_a; dst[7] = inf.d_b;
          *(uint16_t*)(dst + 8) = inf.d_q;
          *(int64_t*)(dst + 16) = inf.d_pos;
        }
        bump += 24;
      }
      const Slot* sl = s_slots + (threadIdx.x * ITEMS + k) * MAX_SLOTS;
      for (int i = 0; i < inf.ns; i++) {
        Slot s = sl[i];
        if (s.flags & SF_KEY_WF) s.d.key = hin->wf_next + 5 * (int64_t)(wf0 + s.ord);
        if (s.flags & SF_KEY_JOB) s.d.key = hin->job_next + 5 * (int64_t)(job0 + s.ord);
        if (s.flags & SF_INST_WF) s.d.inst_key = hin->wf_next + 5 * (int64_t)(wf0 + s.ord);
        if (s.flags & SF_PAY_MERGED) s.d.payload = merged_ref;
        if (s.flags & SF_PAY_DETAIL) s.d.payload = detail_ref;
        if (s.flags & SF_ROW_NEW) {
          const uint64_t row = row0 + s.rord;
          if (row >= P.row_cap) { err |= DE_ROWS_FULL; s.rself = NO_ROW; }
          else {
            s.rself = (uint32_t)row;
            if (s.flags & SF_ROW_INIT) {
              RowMeta m;
              m.payload = s.d.payload; m.parent = s.rscope; m.elem = s.d.elem; m.state = WI_ELEMENT_READY;
              m.flags = 0; m.nchild = 0;
              P.rmeta[row] = m;
              P.rkeys[row] = RowKeys{s.d.key, s.d.scope_key, s.d.inst_key, 0};
            }
          }
        }
        if (kind_vt(s.d.kind) == ZB_VT_WORKFLOW_INSTANCE && kind_rt(s.d.kind) == ZB_RT_EVENT) st_trans++;
        if (out_rec >= P.log_cap) { err |= DE_LOG_FULL; }
        else {
          P.log[out_rec] = s.d;
          P.links[out_rec] = (uint64_t)s.rself | ((uint64_t)s.rscope << 32);
          if (s.flags & SF_COND_JOB) {
            const uint32_t j = atomicAdd(P.cond_count + (P.wave & 1), 1u);
            if (j >= P.job_cap) err |= DE_LOG_FULL;
            else P.cond_jobs[(uint64_t)(P.wave & 1) * P.job_cap + j] = out_rec;
          }
        }
        out_rec++;
      }
    }
    if (err) {
      atomicOr(&s_err, err);
      // first failing record (lowest position) and the code site that flagged it
      atomicMin((unsigned long long*)P.err_info, ((unsigned long long)err_pos << 8) | (err_site & 0xff));
    }
    if (tile == ntiles - 1 && threadIdx.x == 0) {
      const Cnt tot = cnt_add(ex, agg);
      WaveHdr h = *hin;
      h.begin = end;
      h.end = end + (int64_t)(tot.a >> 28);
      h.wf_next = hin->wf_next + 5 * (int64_t)(tot.a & F28);
      h.job_next = hin->job_next + 5 * (int64_t)(tot.b >> 28);
      h.rows_next = hin->rows_next + (int64_t)(tot.b & F28);
      h.arena_next = hin->arena_next + (int64_t)tot.c;
      *hout = h;
    }
    __syncthreads();
  }
  // stats: block reduce -> one atomic per block per counter
  if (st_trans) atomicAdd(&s_stats[0], st_trans);
  if (st_completed) atomicAdd(&s_stats[1], st_completed);
  if (st_created) atomicAdd(&s_stats[2], st_created);
  if (st_merges) atomicAdd(&s_stats[3], st_merges);
  if (st_mbytes) atomicAdd(&s_stats[4], st_mbytes);
  if (st_cbytes) atomicAdd(&s_stats[5], st_cbytes);
  __syncthreads();
  if (threadIdx.x == 0) {
    if (s_err) atomicOr(P.err, s_err);
    for (int i = 0; i < 6; i++)
      if (s_stats[i]) atomicAdd((unsigned long long*)&P.stats[i], (unsigned long long)s_stats[i]);
  }
}

void launch_wave(const WaveParams& p, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(k_wave, dim3(grid), dim3(WG), 0, stream, p);
}

}  // namespace zbg
