// zb_wave.hip — one breadth-first generation (or a chunk of one) of the log per wave, as three
// launches with no inter-workgroup waiting anywhere:
//
//   k_process  per record: decode descriptor, guards (BpmnStepProcessor.java:128-150), step handler
//              (BpmnStepProcessor.java:92-125 -> handlers); index mutations of existing rows; the
//              follow-up records go to a staging slot pair, their counts (records, wf keys, job keys,
//              new rows, arena bytes, merge / condition jobs) to a count word, and the workgroup's
//              totals to block_agg (workgroup b owns one contiguous range of 256-record tiles).
//   k_scan     one workgroup: exclusive prefix of the workgroup totals, the next wave header, counters.
//   k_emit     per record: tile scan of the count words + the running workgroup prefix gives each follow-up its
//              log position, keys (KeyGenerator(1,5) / job KeyGenerator(2,5) ordinals), new rows
//              (ElementInstanceWriter.writeNewEvent inserts), reserved arena blobs and job-list entries.
//
// Follow-ups of a record are contiguous and ordered by emission index; follow-ups of the chunk are
// ordered by their parent's position (FIFO log processing == breadth-first waves), so the
// log, keys and rows come out exactly as the reference's sequential processor writes them.
#include <hip/hip_runtime.h>

#include "zb_devlib.hpp"
#include "zb_kernels.hpp"
#include "zb_msg.hpp"

namespace zbg {

constexpr int WG = WAVE_TILE;
constexpr int MAX_SLOTS = 2;  // output records per item (one parent's batch emits <= 2 in every handler)

enum SlotFlags : uint8_t {
  SF_KEY_WF = 1,       // key = new wf key #ord
  SF_KEY_JOB = 2,      // key = new job key #ord
  SF_INST_WF = 4,      // inst_key = new wf key #ord (CREATE)
  SF_ROW_NEW = 8,      // row_self = new row #rord
  SF_ROW_INIT = 16,    // initialise that row as an ELEMENT_READY insert (ElementInstanceWriter.writeNewEvent)
  SF_PAY_MERGED = 32,  // payload = this item's merge result
  SF_PAY_DETAIL = 64,  // payload = this item's incident detail blob
  SF_COND_JOB = 128,   // GATEWAY_ACTIVATED of a conditional split: k_cond evaluates it before the next wave
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
  // a parallel fork's expanded outputs (k_emit writes them after the staged slots)
  uint32_t nexp, exp_ord;
  uint32_t src_off;  // the record being processed, relative to the thread's first (the slots' source)
  // stats
  uint32_t transitions, completed, created, merges, canceled;
  uint32_t merge_bytes, cond_bytes;
  // a SUBSCRIBE_TO_INTERMEDIATE_MESSAGE step (SubscribeMessageHandler): k_subscribe does its side effect
  bool sub;
  int64_t sub_pos;
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
  s.pad = (uint8_t)t.src_off;
  s.plen = VLEN_UNKNOWN;
  return s;
}

// ---- value length hints (vlen) of the records a wave writes, so that the drain's size pass reads 4 bytes per
// record instead of every record's payload document: a follow-up carrying its source record's payload takes
// the source's payload length, recovered from the source's own hint (the inverse of the emit formula, the
// value's constant part + key lengths + bin header); the rest read the document's length word.
__device__ __forceinline__ uint32_t formula_base(const WaveParams& P, const zb_rec& d) {
  const ValueConst vc = P.vconst[d.elem];
  return (kind_vt(d.kind) == ZB_VT_JOB ? vc.job : vc.wf) + mp_int_len(d.inst_key) + mp_int_len(d.scope_key);
}
// (vl: the record's own hint, vlen[pos], loaded with the record: process_record's stores to the rows would otherwise
// keep the compiler from issuing the load before them, one more dependent round trip at the end of every record)
__device__ __forceinline__ uint32_t payload_len_of(const WaveParams& P, const zb_rec& rec, uint32_t vl) {
  if (kind_vt(rec.kind) == ZB_VT_INCIDENT) return VLEN_UNKNOWN;  // (payload: an incident detail blob)
  if (fast_kind(rec) && P.vconst) {
    const uint32_t v = vl;
    if (v != VLEN_UNKNOWN) {
      const uint32_t x = v - formula_base(P, rec);  // mp_bin_len(plen)
      return x <= 257 ? x - 2 : (x <= 65538 ? x - 3 : x - 5);
    }
  }
  return *(const uint32_t*)(P.arena + (uint64_t)rec.payload * 8);
}
// after process_record(rec at pos) staged slots [ns0, t.ns): their payload lengths
__device__ __forceinline__ void annotate_slots(const WaveParams& P, TState& t, int ns0, const zb_rec& rec, uint32_t vl) {
  uint32_t rl = VLEN_UNKNOWN;
  bool have = false;
  for (int k = ns0; k < t.ns; k++) {
    Slot& s = t.s[k];
    if (s.flags & (SF_PAY_MERGED | SF_PAY_DETAIL) || !fast_kind(s.d)) continue;
    if (s.d.payload == rec.payload && !(rec.kind & KIND_RAW)) {
      if (!have) { rl = payload_len_of(P, rec, vl); have = true; }
      s.plen = rl;
    } else {
      s.plen = *(const uint32_t*)(P.arena + (uint64_t)s.d.payload * 8);
    }
  }
}

__device__ __forceinline__ void wf_event(TState& t, Slot& s, uint8_t intent, uint8_t cont) {
  s.d.intent = intent;
  s.d.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE, ZB_RT_EVENT, cont);
}

// ElementInstanceWriter.writeFollowUpEvent index side effects for a final state
// (atomic: the tokens of a scope with parallel branches remove their children in the same wave)
__device__ __forceinline__ void remove_row(const WaveParams& P, uint32_t row) {
  RowMeta& m = P.rmeta[row];
  uint32_t parent = m.parent;
  m.state = 0;
  if (parent != NO_ROW) atomicSub(&P.rmeta[parent].nchild, 1);
}

__device__ __forceinline__ bool can_terminate(uint8_t state) {  // WorkflowInstanceLifecycle.canTerminate
  return state == WI_ELEMENT_READY || state == WI_ELEMENT_ACTIVATED || state == WI_ELEMENT_COMPLETING;
}

// the blob after a submitted record's payload document holds its verbatim value (KIND_RAW); the copy
// of the document after that one is followed by the command value as the reference re-encodes it
// (zb_submit arena layout: [doc][raw value][doc][re-encoded value], each [u32 len][bytes] 8-aligned)
__device__ __forceinline__ uint32_t next_blob(const uint8_t* arena, uint32_t ref) {
  const uint32_t len = *(const uint32_t*)(arena + (uint64_t)ref * 8);
  return ref + ((4 + len + 7) >> 3);
}
__device__ __forceinline__ uint32_t derived_ref(const uint8_t* arena, uint32_t ref) {
  return next_blob(arena, next_blob(arena, ref));
}

// a WORKFLOW_INSTANCE event carrying an indexed element instance's value (row) with the given intent
__device__ __forceinline__ Slot& row_event(const WaveParams& P, TState& t, uint32_t row, uint8_t intent) {
  const RowMeta m = P.rmeta[row];
  const RowKeys k = P.rkeys[row];
  Slot& s = add_slot(t);
  s.d.key = k.key;
  s.d.scope_key = k.scope_key;
  s.d.inst_key = k.inst_key;
  s.d.elem = m.elem;
  s.d.payload = m.payload;
  wf_event(t, s, intent, t.ns > 1);
  s.rself = row; s.rscope = m.parent;
  return s;
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

// k_map's outcome for the record at pos (zb_aux.hip)
__device__ __forceinline__ uint64_t map_outcome(const WaveParams& P, int64_t pos) {
  return P.mapres[pos - P.hdr[P.wave & 1].begin];
}
// true: a result document (ref in the low bits); otherwise the IO_MAPPING_ERROR incident is raised
// (BpmnStepContext.raiseIncident) or the processor fails
__device__ bool map_ok(TState& t, const zb_rec& rec, int64_t pos, uint64_t mr) {
  const uint64_t st = mr & (15ull << 60);
  if (st == MR_OK) return true;
  if (st == MR_INCIDENT) incident(t, rec, pos, 1 /*IO_MAPPING_ERROR*/, (uint8_t)(mr >> 48), 0, 0, (uint16_t)(mr >> 32));
  else if (st == MR_UNSUPPORTED) fail_at(t, DE_UNSUPPORTED, 30);
  else fail_at(t, DE_PROCESSING, 31);  // MappingProcessor threw something else (or no outcome)
  return false;
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
  const DevElem& el = P.elems[rec.elem];
  const uint8_t step = el.step[intent];
  if (step == ST_UNBOUND || step == ST_NONE) return;

  switch (step) {
    case ST_APPLY_INPUT_MAPPING: {  // InputMappingHandler :39-70 (mappings: extract, done by k_map)
      uint32_t pay = rec.payload;
      if (el.n_in) {
        const uint64_t mr = map_outcome(P, pos);
        if (!map_ok(t, rec, pos, mr)) return;
        pay = (uint32_t)mr;
      }
      Slot& s = add_slot(t);
      s.d = rec;
      s.d.payload = pay;
      wf_event(t, s, WI_ELEMENT_ACTIVATED, t.ns > 1);
      s.rself = rself; s.rscope = rscope;
      RowMeta& m = P.rmeta[rself];
      m.state = WI_ELEMENT_ACTIVATED;
      m.payload = pay;
      break;
    }
    case ST_APPLY_OUTPUT_MAPPING: {  // OutputMappingHandler :42-85, outputBehavior null -> merge
      if (!scope_alive) { fail_at(t, DE_PROCESSING, 4); return; }
      const uint8_t ob = (el.flags >> OB_SHIFT) & 3;
      if (ob == OB_NONE || el.n_out_map || ob == OB_OVERWRITE) {
        // none: the flow scope's payload; mappings / overwrite: the document k_map produced
        uint32_t pay = P.rmeta[rscope].payload;
        if (ob != OB_NONE) {
          const uint64_t mr = map_outcome(P, pos);
          if (!map_ok(t, rec, pos, mr)) return;
          pay = (uint32_t)mr;
        }
        Slot& s = add_slot(t);
        s.d = rec;
        s.d.payload = pay;
        wf_event(t, s, WI_ELEMENT_COMPLETED, t.ns > 1);
        s.rself = rself; s.rscope = rscope;
        remove_row(P, rself);
        break;
      }
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
      if (P.has_parallel) {
        // EXTENSION (C4): k_pre took this token off the scope; the scope completes on its last token, i.e.
        // when the count reached 0 and this is the wave's last consumer in log order
        const RowAux& a = P.raux[rscope];
        if (a.tokens < 0) { fail_at(t, DE_PROCESSING, 40); return; }
        if (a.tokens != 0 || a.consume_pos != pos) return;
      }
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
      if (scope_alive) atomicAdd(&P.rmeta[rscope].nchild, 1);
      break;
    }
    case ST_TRIGGER_START_EVENT: {  // TriggerStartEventHandler :30-39
      if (el.start == NO_ELEM) { fail_at(t, DE_PROCESSING, 11); return; }
      if (P.has_parallel && self_alive) {  // EXTENSION (C4): the start event's token
        RowAux a;
        a.tokens = 1; a.first = NO_ROW; a.join_cnt[0] = a.join_cnt[1] = 0;
        a.consume_pos = 0; a.join_pos[0] = a.join_pos[1] = 0; a.mark = 0;
        P.raux[rself] = a;
      }
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
    case ST_SUBSCRIBE_TO_INTERMEDIATE_MESSAGE: {  // SubscribeMessageHandler :77-141: a side effect, no record
      // the correlation-key query and the open-subscription command run in k_subscribe, after this wave's
      // k_process (no record of this step depends on them; a failure stops the partition either way)
      if (t.sub) { fail_at(t, DE_UNSUPPORTED, 35); return; }
      t.sub = true;
      t.sub_pos = pos;
      break;
    }
    case ST_PARALLEL_SPLIT: {  // EXTENSION (C4): one SEQUENCE_FLOW_TAKEN per outgoing flow (k_emit writes them)
      if (el.n_out == 0 || el.n_out > MAX_FANOUT || t.nexp) { fail_at(t, DE_UNSUPPORTED, 41); return; }
      t.nexp = el.n_out;
      t.exp_ord = (uint32_t)t.nwf;
      t.nwf += el.n_out;
      break;
    }
    case ST_PARALLEL_MERGE: {  // EXTENSION (C4): the wave's last arrival (log order) that completes the arity fires
      if (!scope_alive || el.target == NO_ELEM) { fail_at(t, DE_PROCESSING, 42); return; }
      const DevElem& g = P.elems[el.target];
      RowAux& a = P.raux[rscope];
      if (a.join_pos[g.join_slot] != pos) return;
      const uint32_t cnt = a.join_cnt[g.join_slot];
      if (cnt < g.m_in) return;
      if (cnt > g.m_in) { fail_at(t, DE_UNSUPPORTED, 43); return; }  // a flow taken twice before the join fired
      a.join_cnt[g.join_slot] = 0;
      Slot& s = add_slot(t);
      s.d = rec;
      s.d.elem = el.target;
      wf_event(t, s, WI_GATEWAY_ACTIVATED, t.ns > 1);
      s.flags |= SF_KEY_WF; s.ord = (uint8_t)t.nwf++;
      s.rself = NO_ROW; s.rscope = rscope;
      break;
    }
    case ST_TERMINATE_CONTAINED_INSTANCES: {  // TerminateContainedElementsHandler :31-53
      if (!self_alive) { fail_at(t, DE_PROCESSING, 44); return; }
      if (P.rmeta[rself].nchild == 0) {
        Slot& s = add_slot(t);
        s.d = rec;
        wf_event(t, s, WI_ELEMENT_TERMINATED, t.ns > 1);
        s.rself = rself; s.rscope = rscope;
        remove_row(P, rself);
        if (rec.key == rec.inst_key) t.canceled += 1;
      } else {
        const RowAux& a = P.raux[rself];
        const uint32_t child = a.mark == P.epoch ? a.first : NO_ROW;
        if (child == NO_ROW) { fail_at(t, DE_PROCESSING, 45); return; }
        if (can_terminate(P.rmeta[child].state)) {
          row_event(P, t, child, WI_ELEMENT_TERMINATING);
          P.rmeta[child].state = WI_ELEMENT_TERMINATING;
        }
      }
      break;
    }
    case ST_TERMINATE_JOB_TASK:  // TerminateServiceTaskHandler :37-58: JOB CANCEL (key = job key) first
    case ST_TERMINATE_ELEMENT: {  // TerminateElementHandler :29-45
      if (step == ST_TERMINATE_JOB_TASK && self_alive && P.rkeys[rself].job_key > 0) {
        Slot& j = add_slot(t);
        j.d.key = P.rkeys[rself].job_key;
        j.d.scope_key = rec.key;  // headers.activityInstanceKey
        j.d.inst_key = rec.inst_key;
        j.d.elem = rec.elem;
        j.d.payload = 0;
        j.d.intent = JI_CANCEL;
        j.d.kind = make_kind(ZB_VT_JOB, ZB_RT_COMMAND, t.ns > 1);
        j.rself = NO_ROW; j.rscope = NO_ROW;
      }
      Slot& s = add_slot(t);
      s.d = rec;
      wf_event(t, s, WI_ELEMENT_TERMINATED, t.ns > 1);
      s.rself = rself; s.rscope = rscope;
      if (self_alive) remove_row(P, rself);
      break;
    }
    case ST_PROPAGATE_TERMINATION: {  // PropagateTerminationHandler :29-40 (the guard saw the scope TERMINATING)
      if (P.rmeta[rscope].nchild == 0) {
        const int64_t sk = P.rkeys[rscope].key;
        row_event(P, t, rscope, WI_ELEMENT_TERMINATED);
        remove_row(P, rscope);
        if (sk == P.rkeys[rscope].inst_key) t.canceled += 1;
      } else {
        // EXTENSION (several live tokens in the scope, C4): terminate the next child
        const RowAux& a = P.raux[rscope];
        const uint32_t child = a.mark == P.epoch ? a.first : NO_ROW;
        if (child == NO_ROW) { fail_at(t, DE_PROCESSING, 46); return; }
        if (can_terminate(P.rmeta[child].state)) {
          row_event(P, t, child, WI_ELEMENT_TERMINATING);
          P.rmeta[child].state = WI_ELEMENT_TERMINATING;
        }
      }
      break;
    }
    default:
      fail_at(t, DE_UNSUPPORTED, 12);  // never silently skipped
      break;
  }
}

// ---- the job stream processor (ZB_CFG_JOB_PROCESSOR): JobInstanceStreamProcessor.java:98-242 through
// CommandProcessorImpl (accept -> follow-up event with the command's value, a new key for a null command key;
// reject -> the command's value with its rejection). Job states live in the job table (P.jobs, by job key); all
// commands for one job in a tick arrive as one group (zb_submit), so the owning thread is the only one touching it.

__device__ void job_command(const WaveParams& P, const zb_rec& rec, uint32_t rself, uint32_t rscope, TState& t) {
  const uint8_t raw = rec.kind & KIND_RAW;
  Slot& s = add_slot(t);
  s.d = rec;
  if (raw) s.d.payload = derived_ref(P.arena, rec.payload);  // the command's value, as the reference re-encodes it
  s.rself = rself; s.rscope = rscope;  // (JOB events find the element instance through the activity key)
  if (rec.intent == JI_CREATE) {  // CreateJobProcessor :98-106 (a null key: the job key generator's next)
    s.d.intent = JI_CREATED;
    s.d.kind = make_kind(ZB_VT_JOB, ZB_RT_EVENT, t.ns > 1) | raw;
    s.flags = SF_KEY_JOB;  // k_emit assigns the key and marks the job CREATED
    s.ord = (uint8_t)t.njob++;
    return;
  }
  const int64_t j = job_find(P.jobs, rec.key);
  const uint8_t st = j >= 0 ? P.jobs.state[j] : JS_NONE;
  uint8_t ev = 0xff, next = st;
  bool bad_value = false;
  switch (rec.intent) {
    case JI_ACTIVATE:  // ActivateJobProcessor :108-160
      if (st == JS_CREATED || st == JS_FAILED || st == JS_TIMED_OUT) { ev = JI_ACTIVATED; next = JS_ACTIVATED; }
      break;
    case JI_COMPLETE:  // CompleteJobProcessor :162-175 (the state is deleted)
      if (st == JS_ACTIVATED || st == JS_TIMED_OUT) { ev = JI_COMPLETED; next = JS_NONE; }
      break;
    case JI_FAIL:      // FailJobProcessor :177-189
      if (st == JS_ACTIVATED) { ev = JI_FAILED; next = JS_FAILED; }
      break;
    case JI_TIME_OUT:  // TimeOutJobProcessor :191-204
      if (st == JS_ACTIVATED) { ev = JI_TIMED_OUT; next = JS_TIMED_OUT; }
      break;
    case JI_UPDATE_RETRIES:  // UpdateRetriesJobProcessor :206-222 (zb_submit: elem = value.retries > 0)
      if (st == JS_FAILED) {
        if (rec.elem == 1) ev = JI_RETRIES_UPDATED;
        else bad_value = true;
      }
      break;
    case JI_CANCEL:    // CancelJobProcessor :224-240
      if (st != JS_NONE) { ev = JI_CANCELED; next = JS_NONE; }
      break;
    default:  // no processor for this command
      t.ns--;
      return;
  }
  if (ev == 0xff) {  // reject: the reason follows the intent (and BAD_VALUE, kept in elem, for UPDATE_RETRIES)
    s.d.kind = make_kind(ZB_VT_JOB, ZB_RT_COMMAND_REJECTION, t.ns > 1) | raw;
    if (raw) s.d.elem = bad_value ? 1 : 0;
    return;
  }
  s.d.intent = ev;
  s.d.kind = make_kind(ZB_VT_JOB, ZB_RT_EVENT, t.ns > 1) | raw;
  if (j >= 0 && next != st) {
    if (next == JS_NONE) {  // JobStateController.deleteJobState: the slot becomes a tombstone
      P.jobs.state[j] = JS_NONE;
      __hip_atomic_store(P.jobs.keys + j, JOB_TOMB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      atomicAdd(P.jobs.tombs, 1u);
    } else {
      P.jobs.state[j] = next;
    }
  }
}

// (always inlined: as a call it takes the parameter block through scratch -- k_wave 128 -> 1104 B of scratch per lane)
__device__ __forceinline__ void process_record(const WaveParams& P, const zb_rec& rec, int64_t pos, uint32_t rself,
                               uint32_t rscope, TState& t) {
  const uint8_t vt = kind_vt(rec.kind), rt = kind_rt(rec.kind);
  if (vt == ZB_VT_WORKFLOW_INSTANCE) {
    if (rt == ZB_RT_COMMAND) {
      if (rec.intent == WI_CANCEL) {  // CancelWorkflowInstanceProcessor :511-555 (instance by command key)
        const bool can = rself != NO_ROW && can_terminate(P.rmeta[rself].state);
        if (!can) {  // writeRejection(command, NOT_APPLICABLE, "Workflow instance is not running")
          Slot& s = add_slot(t);
          s.d = rec;
          if (rec.kind & KIND_RAW) s.d.payload = derived_ref(P.arena, rec.payload);
          s.d.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE, ZB_RT_COMMAND_REJECTION, t.ns > 1) | (rec.kind & KIND_RAW);
          s.rself = NO_ROW; s.rscope = NO_ROW;
          return;
        }
        // getValue() is the live indexed object: setPayload(EMPTY) empties the index's copy too
        RowMeta& m = P.rmeta[rself];
        m.payload = 0;
        Slot& a = row_event(P, t, rself, WI_CANCELING);  // batch: CANCELING, ELEMENT_TERMINATING (command key)
        a.rself = NO_ROW; a.rscope = NO_ROW;
        row_event(P, t, rself, WI_ELEMENT_TERMINATING);
        m.state = WI_ELEMENT_TERMINATING;
        return;
      }
      if (rec.intent == WI_UPDATE_PAYLOAD) {  // UpdatePayloadProcessor :557-576 (instance by value key)
        const bool found = rself != NO_ROW && P.rmeta[rself].state != 0;
        Slot& s = add_slot(t);
        s.d = rec;
        if (rec.kind & KIND_RAW) s.d.payload = derived_ref(P.arena, rec.payload);  // command value, re-encoded
        s.rself = NO_ROW; s.rscope = NO_ROW;
        if (!found) {  // reject(NOT_APPLICABLE, "Workflow instance is not running")
          s.d.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE, ZB_RT_COMMAND_REJECTION, t.ns > 1) | (rec.kind & KIND_RAW);
          return;
        }
        P.rmeta[rself].payload = rec.payload;
        s.d.intent = WI_PAYLOAD_UPDATED;
        s.d.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE, ZB_RT_EVENT, t.ns > 1) | (rec.kind & KIND_RAW);
        if (rec.key < 0) { s.flags |= SF_KEY_WF; s.ord = (uint8_t)t.nwf++; }  // CommandProcessorImpl.accept :77-84
        return;
      }
      if (rec.intent != WI_CREATE) return;  // no processor registered for this key
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
    if (rt == ZB_RT_COMMAND && P.jobproc) {
      job_command(P, rec, rself, rscope, t);
    } else if (rt == ZB_RT_COMMAND && rec.intent == JI_CREATE) {
      if (!P.harness) return;  // the job stream processor answers from outside (zb_submit)
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
  } else if (vt == ZB_VT_WORKFLOW_INSTANCE_SUBSCRIPTION) {
    if (rt != ZB_RT_COMMAND || rec.intent != 0) return;  // CORRELATE
    // CorrelateWorkflowInstanceSubscription :463-508: the element instance by activityInstanceKey; the
    // delivered command carries the catch event's row (rows are never reused: row + key identify it)
    const bool found = rself != NO_ROW && rself < P.row_cap && P.rmeta[rself].state != 0 &&
                       P.rkeys[rself].key == rec.scope_key;
    const uint8_t raw = rec.kind & KIND_RAW;  // submitted through zb_submit: follow-ups re-encode its value
    if (!found) {  // writeRejection(record, NOT_APPLICABLE, "activity is not active anymore")
      Slot& s = add_slot(t);
      s.d = rec;
      if (raw) s.d.payload = derived_ref(P.arena, rec.payload);
      s.d.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE_SUBSCRIPTION, ZB_RT_COMMAND_REJECTION, t.ns > 1) | raw;
      s.rself = NO_ROW; s.rscope = NO_ROW;
      return;
    }
    RowMeta& m = P.rmeta[rself];
    const RowKeys k = P.rkeys[rself];
    Slot& a = add_slot(t);  // batch: CORRELATED(record key), ELEMENT_COMPLETING(activityInstanceKey)
    a.d = rec;
    if (raw) a.d.payload = derived_ref(P.arena, rec.payload);
    a.d.intent = 1;
    a.d.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE_SUBSCRIPTION, ZB_RT_EVENT, t.ns > 1) | raw;
    a.rself = NO_ROW; a.rscope = NO_ROW;
    Slot& b = add_slot(t);
    b.d.key = rec.scope_key;
    b.d.scope_key = k.scope_key;
    b.d.inst_key = k.inst_key;
    b.d.elem = m.elem;
    b.d.payload = rec.payload;  // value.setPayload(subscription.getPayload())
    wf_event(t, b, WI_ELEMENT_COMPLETING, t.ns > 1);
    b.rself = rself; b.rscope = m.parent;
    m.state = WI_ELEMENT_COMPLETING;
    m.payload = rec.payload;
  }
}

// the next wave's subscribe-step counters (one thread)
__device__ __forceinline__ void clear_sub_counts(const WaveParams& P) {
  for (int s = 0; s < SUB_STRIPES; s++) P.sub_count[((P.wave + 1) & 1) * SUB_STRIPES + s] = 0;
}

// The open-subscription command of a SUBSCRIBE step (SubscribeMessageHandler :77-141,
// SubscriptionCommandSender.openMessageSubscription :83-103): the correlation key extracted from the
// element instance's payload, routed to abs(hash(correlationKey) % P), ordered by the catch event's log
// position. One thread per subscribe step of the wave (k_process listed them).
__global__ void __launch_bounds__(256) k_subscribe(WaveParams P) {
  __shared__ uint32_t s_alloc[2 * (256 / 64) + 2];
  const uint64_t scap = P.job_cap / SUB_STRIPES;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
#pragma unroll 1
  for (int s = 0; s < SUB_STRIPES; s++) {
  const uint64_t n = std::min<uint64_t>(P.sub_count[(P.wave & 1) * SUB_STRIPES + s], scap);
  const uint64_t* jobs = P.sub_jobs + s * scap;
  // (uniform trip count per workgroup: block_alloc2 below is a workgroup-wide operation)
  for (uint64_t j0 = (uint64_t)blockIdx.x * 256; j0 < n; j0 += stride) {
    const uint64_t j = j0 + threadIdx.x;
    const bool act = j < n;
    uint32_t err = 0, site = 0, ck_len = 0, gran = 0, rself = NO_ROW;
    int64_t pos = 0;
    zb_rec rec{};
    const uint8_t* ck = nullptr;
    uint8_t ckbuf[8];
    const DevElem* el = nullptr;
    if (act) {
      pos = (int64_t)jobs[j];
      rec = P.log[pos];
      rself = (uint32_t)P.links[pos];
      el = &P.elems[rec.elem];
      const uint8_t* pp = P.arena + (uint64_t)rec.payload * 8;
      const uint32_t len = *(const uint32_t*)pp;
      QueryResult q;
      Tok tk;
      if (!run_query(pp + 4, len, P.queries[el->ck_query], P.filters, P.pool, q)) { err = DE_UNSUPPORTED; site = 30; }
      // extractCorrelationKey :121-141: exactly one result, a string or a long, else the processor fails
      else if (q.count != 1) { err = DE_PROCESSING; site = 31; }
      else if (!read_tok(pp + 4 + q.pos, q.len, tk)) { err = DE_PROCESSING; site = 32; }
      else if (tk.type == TT_STRING) {
        ck_len = tk.len;
        ck = pp + 4 + q.pos + tk.hdr;
      } else if (tk.type == TT_INTEGER) {  // QueryResult.getLongAsBuffer: 8 bytes, native (little-endian) order
        ck_len = 8;
        for (int i = 0; i < 8; i++) ckbuf[i] = (uint8_t)((uint64_t)tk.ival >> (8 * i));
        ck = ckbuf;
      } else {
        err = DE_PROCESSING; site = 34;  // "Failed to extract correlation-key: wrong type"
      }
      if (!err) gran = var_granules(el->msg_len, ck_len, 0);
    }
    uint32_t slot, vat;
    block_alloc2<256>(P.obx.n, act && !err ? 1u : 0u, P.obx.var_n, gran, s_alloc, slot, vat);
    if (act && !err) {
      if (slot >= P.obx.cap || (uint64_t)vat + gran > P.obx.var_cap) { err = DE_LOG_FULL; site = 36; }
      else {
        const int32_t target = subscription_partition(ck, ck_len, P.partition_count);
        if (!outbox_write(P.obx, slot, vat, ZB_XCHG_OPEN, target, P.partition_id, rself, rec.inst_key, rec.key, pos,
                          rec.elem, P.pool + el->msg_off, el->msg_len, ck, ck_len, nullptr, 0, 0)) {
          err = DE_UNSUPPORTED; site = 37;
        }
      }
    }
    if (err) {
      atomicOr(P.err, err);
      atomicMin((unsigned long long*)P.err_info, ((unsigned long long)pos << 8) | site);
    }
  }
  }
}

// ------------------------------------------------------------------------------ helpers
__device__ __forceinline__ uint64_t shfl_up64(uint64_t v, int d) {
  return (uint64_t)__shfl_up((unsigned long long)v, d, 64);
}
__device__ __forceinline__ uint64_t shfl_down64(uint64_t v, int d) {
  return (uint64_t)__shfl_down((unsigned long long)v, d, 64);
}

struct Chunk {
  int64_t begin, end, n;  // [begin, end) records processed by this wave
};
__device__ __forceinline__ Chunk wave_chunk(const WaveParams& P, const WaveHdr* h) {
  const int64_t b = h->begin, g = gen_limit(P, h);
  const int64_t e = chunk_end(P, b, g);
  return Chunk{b, e, e - b};
}
// contiguous tile range of workgroup b (identical in k_process and k_emit)
__device__ __forceinline__ void block_tiles(const Chunk& c, int64_t& t0, int64_t& t1) {
  const int64_t ntiles = (c.n + WG - 1) / WG;
  t0 = (int64_t)blockIdx.x * ntiles / gridDim.x;
  t1 = (int64_t)(blockIdx.x + 1) * ntiles / gridDim.x;
}

// A batch's records are processed by the thread of its first record, in order (the later ones may read
// what the earlier ones wrote to the index: CREATED + READY, JOB CREATED + COMPLETED). A parallel fork's
// SEQUENCE_FLOW_TAKEN batch is the exception: its flows touch only their own new element instances (and
// the scope's counters, atomically), so each is a record of its own.
__device__ __forceinline__ bool grouped(const zb_rec& r) {
  return kind_cont(r.kind) && !(r.intent == WI_SEQUENCE_FLOW_TAKEN && kind_vt(r.kind) == ZB_VT_WORKFLOW_INSTANCE);
}

// ------------------------------------------------------------------------------ k_process
__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(4, 8))) k_process(WaveParams P) {
  __shared__ Slot s_slots[WG * MAX_SLOTS];
  __shared__ uint64_t s_red[WG / 64][6];  // (6 packed totals)
  const WaveHdr* hin = P.hdr + (P.wave & 1);
  const Chunk c = wave_chunk(P, hin);
  if (c.n <= 0) return;
  const int64_t gen_end = gen_limit(P, hin);  // (the batch tails read below)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int64_t t0, t1;
  block_tiles(c, t0, t1);
  // this thread's totals over the workgroup's tiles: packed 16-bit fields (<= 2 per record per tile, and
  // a workgroup owns at most wave_cap / WG / grid tiles), bytes separately
  uint64_t acc_a = 0;  // rec | wf << 16 | job << 32 | row << 48
  uint64_t acc_b = 0;  // merges | conds << 16 | transitions << 32 | completed << 48
  uint64_t acc_bytes = 0;
  uint32_t acc_created = 0;

  for (int64_t tile = t0; tile < t1; tile++) {
    const int64_t i = tile * WG + threadIdx.x;  // wave-relative index
    const int64_t r = c.begin + i;
    if (r >= c.end) continue;
    TState t;
    t.s = s_slots + threadIdx.x * MAX_SLOTS;
    t.ns = t.nwf = t.njob = t.nrow = 0;
    t.bytes = 0; t.merge = false; t.detail = false; t.err = 0; t.err_site = 0;
    t.transitions = t.completed = t.created = t.merges = t.canceled = 0;
    t.merge_bytes = t.cond_bytes = 0;
    t.sub = false;
    t.nexp = 0; t.exp_ord = 0; t.src_off = 0;
    uint32_t nconds = 0;
    const zb_rec rec = P.log[r];
    if (!grouped(rec)) {
      // a thread owns its record plus the continuation records that follow it (one parent's batch);
      // a batch never spans generations, so its tail may lie past a chunk end (skipped there as cont)
      const uint64_t lk = P.links[r];
      const uint32_t vl = P.vlen[r];
      process_record(P, rec, r, (uint32_t)lk, (uint32_t)(lk >> 32), t);
      annotate_slots(P, t, 0, rec, vl);
      for (int64_t q = r + 1; q < gen_end && q < r + 4; q++) {
        const zb_rec rec2 = P.log[q];
        if (!grouped(rec2)) break;
        const uint64_t lk2 = P.links[q];
        const uint32_t vl2 = P.vlen[q];
        t.src_off = (uint32_t)(q - r);
        const int ns0 = t.ns;
        process_record(P, rec2, q, (uint32_t)lk2, (uint32_t)(lk2 >> 32), t);
        annotate_slots(P, t, ns0, rec2, vl2);
      }
    }
    // stage the follow-ups and the count word
    Slot* dst = P.stage + (uint64_t)i * MAX_SLOTS;
    for (int k = 0; k < t.ns; k++) {
      const Slot sl = t.s[k];
      dst[k] = sl;
      nconds += (sl.flags & SF_COND_JOB) ? 1 : 0;
      if (kind_vt(sl.d.kind) == ZB_VT_WORKFLOW_INSTANCE && kind_rt(sl.d.kind) == ZB_RT_EVENT) t.transitions++;
    }
    if (t.merge || t.detail) {
      ItemInfo inf;
      inf.m_src = t.m_src; inf.m_tgt = t.m_tgt; inf.m_len = t.m_len; inf.m_bytes = t.merge ? t.m_bytes : 0;
      inf.d_pos = t.d_pos; inf.d_q = t.d_q; inf.d_type = t.d_type; inf.d_code = t.d_code; inf.d_a = t.d_a;
      inf.d_b = t.d_b; inf.has_detail = t.detail; inf.ns = (uint8_t)t.ns;
      P.info[i] = inf;
    }
    t.transitions += t.nexp;  // a fork's SEQUENCE_FLOW_TAKEN events
    const uint32_t nwf_staged = (uint32_t)t.nwf - t.nexp;
    P.cw[i] = (uint64_t)t.ns | ((uint64_t)nwf_staged << CW_NWF) | ((uint64_t)t.njob << CW_NJOB) |
              ((uint64_t)t.nrow << CW_NROW) | ((uint64_t)(t.merge ? 1 : 0) << CW_MERGE) |
              ((uint64_t)(t.detail ? 1 : 0) << CW_DETAIL) | ((uint64_t)nconds << CW_NCOND) |
              ((uint64_t)t.nexp << CW_NEXP) | ((uint64_t)t.bytes << 32);
    acc_a += (uint64_t)(t.ns + t.nexp) | ((uint64_t)t.nwf << 16) | ((uint64_t)t.njob << 32) |
             ((uint64_t)t.nrow << 48);
    acc_b += (uint64_t)(t.merge ? 1 : 0) | ((uint64_t)nconds << 16) | ((uint64_t)t.transitions << 32) |
             ((uint64_t)t.completed << 48);
    acc_bytes += t.bytes;
    acc_created += t.created | (t.canceled << 16);
    if (__ballot(t.sub)) {  // wave-uniform: this tile's subscribe steps, in the wave's job list (its stripe)
      const uint32_t s = blockIdx.x % SUB_STRIPES;
      const uint64_t scap = P.job_cap / SUB_STRIPES;
      const uint32_t slot = wave_alloc(P.sub_count + (P.wave & 1) * SUB_STRIPES + s, t.sub ? 1u : 0u);
      if (t.sub) {
        if (slot < scap) P.sub_jobs[s * scap + slot] = (uint64_t)t.sub_pos;
        else fail_at(t, DE_LOG_FULL, 36);
      }
    }
    if (t.err) {
      atomicOr(P.err, t.err);
      // first failing record (lowest position) and the code site that flagged it
      atomicMin((unsigned long long*)P.err_info, ((unsigned long long)r << 8) | (t.err_site & 0xff));
    }
  }
  // workgroup totals: unpack to 32-bit lanes sums, wave reduction, 4 partials through LDS
  uint64_t v[6] = {acc_a & 0xffffffffull, acc_a >> 32, acc_b & 0xffffffffull, acc_b >> 32, acc_bytes,
                   (uint64_t)acc_created};
  // 16-bit fields of a thread's totals never overflow (<= 65 * tiles per workgroup), but the sum over
  // 256 threads can: widen each 16-bit pair into two 32-bit halves first
  uint64_t w[11];
  w[0] = v[0] & 0xffff; w[1] = v[0] >> 16; w[2] = v[1] & 0xffff; w[3] = v[1] >> 16;
  w[4] = v[2] & 0xffff; w[5] = v[2] >> 16; w[6] = v[3] & 0xffff; w[7] = v[3] >> 16;
  w[8] = v[4]; w[9] = v[5] & 0xffff; w[10] = v[5] >> 16;
  uint64_t pk[6] = {w[0] | (w[1] << 32), w[2] | (w[3] << 32), w[4] | (w[5] << 32), w[6] | (w[7] << 32),
                    w[8], w[9] | (w[10] << 32)};
#pragma unroll
  for (int f = 0; f < 6; f++) {
    uint64_t x = pk[f];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += shfl_down64(x, d);
    pk[f] = x;
  }
  if (lane == 0) {
#pragma unroll
    for (int f = 0; f < 6; f++) s_red[wv][f] = pk[f];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t a[6];
#pragma unroll
    for (int f = 0; f < 6; f++) a[f] = s_red[0][f] + s_red[1][f] + s_red[2][f] + s_red[3][f];
    BlockAgg g;
    g.rec = (uint32_t)a[0]; g.wf = (uint32_t)(a[0] >> 32);
    g.job = (uint32_t)a[1]; g.row = (uint32_t)(a[1] >> 32);
    g.merges = (uint32_t)a[2]; g.conds = (uint32_t)(a[2] >> 32);
    g.transitions = (uint32_t)a[3]; g.completed = (uint32_t)(a[3] >> 32);
    g.bytes = a[4];
    g.created = (uint32_t)a[5]; g.canceled = (uint32_t)(a[5] >> 32);
    P.block_agg[blockIdx.x] = g;
  }
}

// ------------------------------------------------------------------------------ k_pre
// Scope-wide counters of the chunk, before k_process decides anything (only when the model has parallel
// gateways or a cancellation is in flight). Token effects are order-independent sums, so they are
// applied here with atomics and every decision in k_process reads the chunk's final counts plus the
// max log position of the records that touched them -- which reproduces the sequential outcome: a scope
// completes / a join fires exactly at its last consumer / arrival in log order.
// Guards are the BpmnStepProcessor ones (scope ACTIVATED); k_process has not run yet, so they read the
// state every record of the chunk sees in the reference (no record of the chunk changes them first).
__global__ void __launch_bounds__(WG) k_pre(WaveParams P) {
  const WaveHdr* hin = P.hdr + (P.wave & 1);
  const Chunk c = wave_chunk(P, hin);
  const int64_t stride = (int64_t)gridDim.x * WG;
  for (int64_t r = c.begin + (int64_t)blockIdx.x * WG + threadIdx.x; r < c.end; r += stride) {
    const zb_rec rec = P.log[r];
    if (kind_vt(rec.kind) != ZB_VT_WORKFLOW_INSTANCE || kind_rt(rec.kind) != ZB_RT_EVENT) continue;
    const uint8_t it = rec.intent;
    if (it != WI_END_EVENT_OCCURRED && it != WI_ELEMENT_COMPLETED && it != WI_SEQUENCE_FLOW_TAKEN &&
        it != WI_GATEWAY_ACTIVATED && it != WI_ELEMENT_TERMINATING && it != WI_ELEMENT_TERMINATED)
      continue;
    if (rec.elem == NO_ELEM) continue;
    const uint64_t lk = P.links[r];
    const uint32_t rself = (uint32_t)lk, rscope = (uint32_t)(lk >> 32);
    const DevElem& el = P.elems[rec.elem];
    const uint8_t step = el.step[it];
    const bool scope_alive = rscope != NO_ROW && P.rmeta[rscope].state != 0;
    const uint8_t sst = scope_alive ? P.rmeta[rscope].state : 0;
    if (P.has_parallel && sst == WI_ELEMENT_ACTIVATED) {
      RowAux& a = P.raux[rscope];
      if (step == ST_CONSUME_TOKEN && (it == WI_END_EVENT_OCCURRED || it == WI_ELEMENT_COMPLETED)) {
        atomicSub(&a.tokens, 1);
        atomicMax((unsigned long long*)&a.consume_pos, (unsigned long long)r);
      } else if (step == ST_PARALLEL_MERGE && it == WI_SEQUENCE_FLOW_TAKEN && el.target != NO_ELEM) {
        const uint32_t slot = P.elems[el.target].join_slot;
        atomicAdd(&a.join_cnt[slot], 1u);
        atomicMax((unsigned long long*)&a.join_pos[slot], (unsigned long long)r);
      } else if (step == ST_PARALLEL_SPLIT && it == WI_GATEWAY_ACTIVATED) {
        atomicAdd(&a.tokens, (int32_t)el.n_out - (int32_t)(el.m_in > 1 ? el.m_in : 1));
      }
    }
    if (P.term) {
      // the first live child of a scope being terminated (TerminateContainedElementsHandler :31-53 children.get(0)):
      // the smallest live row of its children list (rows are allocated in insertion order). Every record of the chunk
      // that asks for a scope's first child computes the same row from the state before the chunk (k_process has not
      // run), so the stores agree.
      uint32_t row = NO_ROW;
      if (it == WI_ELEMENT_TERMINATING && step == ST_TERMINATE_CONTAINED_INSTANCES && rself != NO_ROW &&
          P.rmeta[rself].state != 0 && P.rmeta[rself].nchild > 0)
        row = rself;
      else if (it == WI_ELEMENT_TERMINATED && step == ST_PROPAGATE_TERMINATION && sst == WI_ELEMENT_TERMINATING &&
               P.rmeta[rscope].nchild > 0)
        row = rscope;
      if (row != NO_ROW) {
        uint32_t first = NO_ROW;
        uint64_t n = 0;
        for (uint32_t ch = P.rlink[row].c_head; ch != NO_ROW && n < P.row_cap; ch = P.rlink[ch].c_next, n++) {
          if (!ZB_DCHECK(ch < P.row_cap, "row %u child %u\n", row, ch)) break;
          const RowMeta cm = P.rmeta[ch];
          if (cm.state != 0 && cm.parent == row && ch < first) first = ch;
        }
        P.raux[row].first = first;
        P.raux[row].mark = P.epoch;
      }
    }
  }
}

// ------------------------------------------------------------------------------ k_scan
constexpr int SCAN_WG = 1024;

__device__ __forceinline__ void agg_fields(const BlockAgg& g, uint64_t* x) {
  x[0] += g.rec; x[1] += g.wf; x[2] += g.job; x[3] += g.row; x[4] += g.bytes;
  x[5] += g.merges; x[6] += g.conds; x[7] += g.transitions; x[8] += g.completed;
  x[9] += g.created; x[10] += g.canceled;
}

__global__ void __launch_bounds__(SCAN_WG) k_scan(WaveParams P) {
  __shared__ uint64_t s_w[SCAN_WG / 64][11];
  const WaveHdr* hin = P.hdr + (P.wave & 1);
  WaveHdr* hout = P.hdr + ((P.wave + 1) & 1);
  const Chunk c = wave_chunk(P, hin);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // workgroup aggregates [k0, k1) per scan thread
  const int per = (P.grid + SCAN_WG - 1) / SCAN_WG;
  const int k0 = threadIdx.x * per, k1 = k0 + per < P.grid ? k0 + per : P.grid;
  // fields: rec wf job row bytes merges conds | transitions completed created canceled (reduced only)
  uint64_t x[11] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  if (c.n > 0)
    for (int k = k0; k < k1; k++) agg_fields(P.block_agg[k], x);
  uint64_t ex[11];
#pragma unroll
  for (int f = 0; f < 11; f++) {
    uint64_t y = x[f];
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t u = shfl_up64(y, d);
      if (lane >= d) y += u;
    }
    ex[f] = y - x[f];
    if (lane == 63) s_w[wv][f] = y;
  }
  __syncthreads();
  if (c.n > 0) {
#pragma unroll
    for (int f = 0; f < 7; f++) {
      uint64_t pre = 0;
      for (int w = 0; w < wv; w++) pre += s_w[w][f];
      ex[f] += pre;
    }
    for (int k = k0; k < k1; k++) {
      const BlockAgg g = P.block_agg[k];
      P.block_off[k] = BlockOff{ex[0], ex[1], ex[2], ex[3], ex[4], (uint32_t)ex[5], (uint32_t)ex[6]};
      ex[0] += g.rec; ex[1] += g.wf; ex[2] += g.job; ex[3] += g.row; ex[4] += g.bytes;
      ex[5] += g.merges; ex[6] += g.conds;
    }
  }
  if (threadIdx.x == 0) {
    uint64_t tot[11];
    for (int f = 0; f < 11; f++) {
      tot[f] = 0;
      for (int w = 0; w < SCAN_WG / 64; w++) tot[f] += s_w[w][f];
    }
    WaveHdr h = *hin;
    if (c.n > 0) {
      h.begin = c.end;
      h.end = hin->end + (int64_t)tot[0];
      h.gen_end = (c.end == hin->gen_end) ? h.end : hin->gen_end;
      h.wf_next = hin->wf_next + 5 * (int64_t)tot[1];
      h.job_next = hin->job_next + 5 * (int64_t)tot[2];
      h.rows_next = hin->rows_next + (int64_t)tot[3];
      h.arena_next = hin->arena_next + (int64_t)tot[4];
      P.stats[0] += tot[7];
      P.stats[1] += tot[8];
      P.stats[2] += tot[9];
      P.stats[6] += 1;
      P.stats[7] += tot[10];
      uint32_t err = 0;
      if ((uint64_t)h.end > P.log_cap) err |= DE_LOG_FULL;
      if ((uint64_t)h.rows_next > P.row_cap) err |= DE_ROWS_FULL;
      if ((uint64_t)h.arena_next > P.arena_cap) err |= DE_ARENA_FULL;
      if (tot[5] > P.job_cap || tot[6] > P.job_cap) err |= DE_LOG_FULL;
      if (err) atomicOr(P.err, err);
    }
    *hout = h;
    P.merge_count[P.wave & 1] = c.n > 0 ? (uint32_t)tot[5] : 0;
    if (P.sub_count) clear_sub_counts(P);  // the next wave's subscribe list
    P.cond_count[P.wave & 1] = c.n > 0 ? (uint32_t)tot[6] : 0;
  }
}

// ------------------------------------------------------------------------------ emit (k_emit, k_wave)
// Writes the follow-ups of wave item i at their final positions: staged slots sl[0, ns) get their keys
// (KeyGenerator ordinals wf0 / job0 + slot ordinal), rows (row0 + ordinal; ELEMENT_READY inserts initialise the
// row), merge result / incident detail blobs (reserved at bump) and job-list entries; a parallel fork's
// SEQUENCE_FLOW_TAKEN records follow (EXTENSION, C4). Every base already includes the item's exclusive offset.
__device__ __forceinline__ void emit_item(const WaveParams& P, const Chunk& c, int64_t i, uint64_t w, const Slot* sl,
                                          const ItemInfo& inf, uint64_t out_rec, uint64_t wf0, uint64_t job0,
                                          uint64_t row0, uint64_t bump, uint64_t merge_j, uint64_t cond_j,
                                          int64_t wf_next, int64_t job_next, uint64_t par) {
  const int ns = (int)(w & 7);
  const uint64_t nexp = (w >> CW_NEXP) & 63;
  uint32_t err = 0;
  uint32_t merged_ref = 0, detail_ref = 0;
  if (w & ((1ull << CW_MERGE) | (1ull << CW_DETAIL))) {
    if (inf.m_bytes) {
      // reserve the blob; k_merge (zb_aux.hip) fills it before the next wave reads any payload
      if (bump + inf.m_bytes > P.arena_cap) err |= DE_ARENA_FULL;
      else {
        merged_ref = (uint32_t)(bump >> 3);
        if (merge_j < P.job_cap) {
          int64_t mpos = -1;  // the slot that carries the result
          for (int k = 0; k < ns; k++)
            if (sl[k].flags & SF_PAY_MERGED) mpos = (int64_t)out_rec + k;
          P.merge_jobs[par + merge_j] = MergeJob{merged_ref, inf.m_src, inf.m_tgt, inf.m_len, mpos};
        }
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
  }
  for (int k = 0; k < ns; k++) {
    Slot s = sl[k];
    if (s.flags & SF_KEY_WF) s.d.key = wf_next + 5 * (int64_t)(wf0 + s.ord);
    if (s.flags & SF_KEY_JOB) {
      s.d.key = job_next + 5 * (int64_t)(job0 + s.ord);
      // the job stream processor's CREATED: the job exists from here on (JobStateController.putJobState)
      if (P.jobproc && s.d.intent == JI_CREATED) {
        const int64_t j = job_insert(P.jobs, s.d.key);
        if (j >= 0) P.jobs.state[j] = JS_CREATED;
        else err |= DE_ROWS_FULL;  // job table full
      }
    }
    if (s.flags & SF_INST_WF) s.d.inst_key = wf_next + 5 * (int64_t)(wf0 + s.ord);
    if (s.flags & SF_PAY_MERGED) s.d.payload = merged_ref;
    if (s.flags & SF_PAY_DETAIL) s.d.payload = detail_ref;
    if (s.flags & SF_ROW_NEW) {
      const uint64_t row = row0 + s.rord;
      if (row >= P.row_cap) { err |= DE_ROWS_FULL; s.rself = NO_ROW; }
      else {
        s.rself = (uint32_t)row;
        RowMeta m;
        RowKeys k;
        uint32_t c_next = NO_ROW;
        if (s.flags & SF_ROW_INIT) {
          m.payload = s.d.payload; m.parent = s.rscope; m.elem = s.d.elem; m.state = WI_ELEMENT_READY;
          m.flags = 0; m.nchild = 0;
          k = RowKeys{s.d.key, s.d.scope_key, s.d.inst_key, 0};
          // ElementInstance.children.add: into the flow scope's list (read from the next wave on)
          if (s.rscope != NO_ROW) c_next = atomicExch(&P.rlink[s.rscope].c_head, (uint32_t)row);
        } else {
          // a CREATE's row: the instance enters the index when its CREATED event is processed (next wave), and
          // until then the row reads as free (state 0, no parent, no children), whatever the memory held before
          m.payload = 0; m.parent = NO_ROW; m.elem = NO_ELEM; m.state = 0; m.flags = 0; m.nchild = 0;
          k = RowKeys{0, 0, 0, 0};
        }
        P.rmeta[row] = m;
        P.rkeys[row] = k;
        P.rlink[row] = RowLink{NO_ROW, c_next};
      }
    }
    if (out_rec >= P.log_cap) { err |= DE_LOG_FULL; }
    else {
      P.log[out_rec] = s.d;
      P.links[out_rec] = (uint64_t)s.rself | ((uint64_t)s.rscope << 32);
      P.srcd[out_rec] = (uint32_t)(out_rec - (uint64_t)(c.begin + i + s.pad));
      P.vlen[out_rec] = (s.plen != VLEN_UNKNOWN && P.vconst) ? formula_base(P, s.d) + mp_bin_len(s.plen) : VLEN_UNKNOWN;
      if (s.flags & SF_COND_JOB) {
        if (cond_j < P.job_cap) P.cond_jobs[par + cond_j] = out_rec;
        cond_j++;
      }
    }
    out_rec++;
  }
  if (nexp) {  // EXTENSION (C4): a parallel fork, one SEQUENCE_FLOW_TAKEN per outgoing flow, keys in order
    const int64_t r = c.begin + i;
    const zb_rec g = P.log[r];
    const uint32_t rscope = (uint32_t)(P.links[r] >> 32);
    const DevElem& ge = P.elems[g.elem];
    const uint64_t kord = wf0 + ((w >> CW_NWF) & 7);
    for (uint32_t j = 0; j < (uint32_t)nexp; j++) {
      zb_rec d = g;
      d.elem = P.cond_flows[ge.out_begin + j];
      d.key = wf_next + 5 * (int64_t)(kord + j);
      d.intent = WI_SEQUENCE_FLOW_TAKEN;
      d.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE, ZB_RT_EVENT, ns + j > 0);
      if (out_rec >= P.log_cap) { err |= DE_LOG_FULL; }
      else {
        P.log[out_rec] = d;
        P.links[out_rec] = (uint64_t)NO_ROW | ((uint64_t)rscope << 32);
        P.srcd[out_rec] = (uint32_t)(out_rec - (uint64_t)r);
        P.vlen[out_rec] = VLEN_UNKNOWN;
      }
      out_rec++;
    }
  }
  if (err) atomicOr(P.err, err);  // capacity overflow: the wave's results are void, the host stops
}

// ------------------------------------------------------------------------------ k_emit
__global__ void __launch_bounds__(WG) k_emit(WaveParams P) {
  __shared__ uint64_t s_a[WG / 64], s_b[WG / 64];
  const WaveHdr* hin = P.hdr + (P.wave & 1);
  const Chunk c = wave_chunk(P, hin);
  if (c.n <= 0) return;
  int64_t t0, t1;
  block_tiles(c, t0, t1);
  if (t0 >= t1) return;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t end = hin->end, wf_next = hin->wf_next, job_next = hin->job_next;
  const uint64_t rows_next = (uint64_t)hin->rows_next, arena_next = (uint64_t)hin->arena_next;
  const uint64_t par = (uint64_t)(P.wave & 1) * P.job_cap;
  const BlockOff bo = P.block_off[blockIdx.x];
  // running workgroup offsets (tile prefix): outputs, wf keys, job keys, rows, bytes, merges, conds
  uint64_t c_rec = bo.rec, c_wf = bo.wf, c_job = bo.job, c_row = bo.row, c_bytes = bo.bytes;
  uint64_t c_merge = bo.merges, c_cond = bo.conds;

  for (int64_t tile = t0; tile < t1; tile++) {
    const int64_t i = tile * WG + threadIdx.x;
    const uint64_t w = (c.begin + i < c.end) ? P.cw[i] : 0;
    // packed block scan: a = outputs | wf << 16 | job << 32 | row << 48, b = bytes | merges << 40 | conds << 52
    const uint64_t nexp = (w >> CW_NEXP) & 63;
    const uint64_t a0 = ((w & 7) + nexp) | ((((w >> CW_NWF) & 7) + nexp) << 16) | (((w >> CW_NJOB) & 7) << 32) |
                        (((w >> CW_NROW) & 7) << 48);
    const uint64_t b0 = (w >> 32) | (((w >> CW_MERGE) & 1) << 40) | (((w >> CW_NCOND) & 7) << 52);
    uint64_t a = a0, b = b0;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t ua = shfl_up64(a, d), ub = shfl_up64(b, d);
      if (lane >= d) { a += ua; b += ub; }
    }
    __syncthreads();  // s_a / s_b reuse across tiles
    if (lane == 63) { s_a[wv] = a; s_b[wv] = b; }
    __syncthreads();
    uint64_t ta = 0, tb = 0;
#pragma unroll
    for (int k = 0; k < WG / 64; k++) {
      if (k < wv) { a += s_a[k]; b += s_b[k]; }
      ta += s_a[k]; tb += s_b[k];
    }
    a -= a0;
    b -= b0;
    const uint64_t r_rec = c_rec, r_wf = c_wf, r_job = c_job, r_row = c_row, r_bytes = c_bytes;
    const uint64_t r_merge = c_merge, r_cond = c_cond;
    c_rec += ta & 0xffff; c_wf += (ta >> 16) & 0xffff; c_job += (ta >> 32) & 0xffff; c_row += ta >> 48;
    c_bytes += tb & 0xffffffffffull; c_merge += (tb >> 40) & 0xfff; c_cond += tb >> 52;
    const int ns = (int)(w & 7);
    if (ns == 0 && nexp == 0 && !((w >> CW_DETAIL) & 1)) continue;
    uint64_t out_rec = (uint64_t)end + r_rec + (a & 0xffff);
    const uint64_t wf0 = r_wf + ((a >> 16) & 0xffff);
    const uint64_t job0 = r_job + ((a >> 32) & 0xffff);
    const uint64_t row0 = rows_next + r_row + (a >> 48);
    uint64_t bump = arena_next + r_bytes + (b & 0xffffffffffull);
    const uint64_t merge_j = r_merge + ((b >> 40) & 0xfff);
    uint64_t cond_j = r_cond + (b >> 52);
    ItemInfo inf{};
    if (w & ((1ull << CW_MERGE) | (1ull << CW_DETAIL))) inf = P.info[i];
    emit_item(P, c, i, w, P.stage + (uint64_t)i * MAX_SLOTS, inf, out_rec, wf0, job0, row0, bump, merge_j, cond_j,
              wf_next, job_next, par);
  }
}

// ------------------------------------------------------------------------------ k_wave (fused)
// k_process + k_scan + k_emit in one launch: each 256-record tile is processed (follow-ups staged in LDS),
// scanned in LDS, gets its offsets from its predecessors, and writes its follow-ups straight from LDS -- no count
// words, staging slots or side information round-trip through HBM (the three-kernel form that does: C2 1M stepping
// 28.1 against 20.5 ms, profiles/r05/wave_exp_split_r05a.txt), and no single-workgroup scan between the passes.
// The grid is persistent (every workgroup resident, tiles dealt round-robin in increasing order): round k is tiles
// [kG, (k+1)G), and a tile only ever waits for tiles of its own or an earlier round, which are already running.
// On a GPU shared with other processes not every workgroup of the grid is resident, and round-robin tiles then wait
// for workgroups that are never dispatched (profiles/r06/c4_8rank_samedevice_r06aq.err.txt): with ZB_CFG_SHARED_GPU
// (tile_claim set) tiles are claimed from a counter instead, in increasing order, so every smaller tile is held by a
// running workgroup and the hand-off progresses whatever the device keeps resident. The claims are one contended
// device-scope atomic per tile -- C2 wave-only 16.5 -> 25.2 ms per step (profiles/r06/ab_tile_claim_r06ar.txt) --
// so the product default is the round-robin deal. The next tile is claimed when the current one starts.
//
// Offsets (a hierarchical hand-off instead of a decoupled look-back: the look-back walked 8.8 rounds of 8
// predecessors per tile, 55 % of tile time, because the tiles of a round all finish processing together and
// inclusive prefixes then trickle forward one round of loads at a time, profiles/r04/phases_c2w_r04f.txt). Within
// a round the tiles form groups of LB_GROUP:
//   * every tile publishes its aggregate, packed into two granules (lbA);
//   * a tile's exclusive prefix inside its group is the sum of its group predecessors' aggregates -- one load per
//     lane of the first wave, all at once; the group's last tile publishes the group total (lbG) right away;
//   * the sum of the earlier groups of the round: their totals, read by the second wave at the same time;
//   * the round's base (lbR): published by the last tile of the previous round.
// So a tile waits for the slowest tile of its group, then ~2 dependent round trips -- no chain along the round.
//
// Hand-off state: 8-byte granules {tag, value} written and read by agent-scope atomics (the data is its own
// flag, cdna_hip_programming.md Guideline 16 R2). Aggregates carry an 8-bit tag (lb_seq, the host zeroes lbA when it
// wraps); group totals and round bases one granule per field with a 32-bit epoch tag. Waiting is bounded in time
// (the constant-rate wall clock, not a spin count: a resident predecessor that the scheduler time-slices out keeps
// its waiters spinning without progress for as long as it is descheduled): a hand-off that has not arrived after
// LB_TIMEOUT_TICKS sets DE_TIMEOUT, the wave's results are void and the host stops the partition -- it never hangs
// the device.
constexpr int LB_FIELDS = 8;   // group totals / round bases: rec wf job row bytes_lo bytes_hi merges conds
constexpr int LB_GROUP = 64;   // tiles per group (one lane each)
constexpr uint64_t LB_TIMEOUT_TICKS = 400000000ull;  // 4 s of the 100 MHz wall clock per hand-off, then DE_TIMEOUT

__device__ __forceinline__ uint32_t lb_tag(int64_t epoch, uint32_t kind) {
  return (uint32_t)((((uint64_t)epoch + 1) << 1) | kind);
}
// a tile aggregate: a = rec:17 wf:17 job:11 row:11, b = merges:9 conds:11 bytes:36, each under the 8-bit tag
__device__ __forceinline__ uint64_t lb_pack_a(uint32_t tag8, uint64_t ta) {
  return ((uint64_t)tag8 << 56) | ((ta & 0xffff) << 39) | (((ta >> 16) & 0xffff) << 22) |
         (((ta >> 32) & 0x7ff) << 11) | ((ta >> 48) & 0x7ff);
}
// field f of a tile aggregate (the tile scan's packed totals; bytes, field 4, are handled by the callers)
__device__ __forceinline__ uint64_t lb_field(uint64_t ta, uint64_t merges, uint64_t conds, int f) {
  return f == 0 ? (ta & 0xffff) : f == 1 ? ((ta >> 16) & 0xffff) : f == 2 ? ((ta >> 32) & 0xffff) :
         f == 3 ? (ta >> 48) : f == 6 ? merges : f == 7 ? conds : 0;
}
__device__ __forceinline__ uint64_t lb_pack_b(uint32_t tag8, uint64_t tbytes, uint64_t merges, uint64_t conds) {
  return ((uint64_t)tag8 << 56) | (merges << 47) | (conds << 36) | tbytes;
}

// wait until every granule this lane reads carries its tag (n: granules, 0..2); false: timed out / another tile did
template <int N>
__device__ __forceinline__ bool lb_wait(uint32_t* err, const uint64_t* const (&g)[N], const uint32_t (&tag)[N],
                                        int shift, bool active, uint64_t (&v)[N], uint64_t t_start) {
  bool timeout = false;
  if (active) {
    for (uint32_t spins = 0;; spins++) {
      bool ok = true;
#pragma unroll
      for (int k = 0; k < N; k++) {
        v[k] = __hip_atomic_load(g[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok &= (uint32_t)(v[k] >> shift) == tag[k];
      }
      if (ok) break;
      if ((spins & 255) == 255 &&
          (wall_clock64() - t_start > LB_TIMEOUT_TICKS ||
           (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & DE_TIMEOUT))) {
        timeout = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  return !__ballot(timeout);
}

template <bool CLAIM>  // ZB_CFG_SHARED_GPU: tiles claimed from P.tile_claim (a kernel of its own, so the default path
                       // carries none of the claim code; C2 wave-only within 1-2 % of the round-6 head either way,
                       // profiles/r06/ab_shared_gpu_optin_r06au.txt)
__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(4, 8))) k_wave(WaveParams P) {
  __shared__ Slot s_slots[WG * MAX_SLOTS];
  __shared__ uint64_t s_a[WG / 64], s_b[WG / 64];
  __shared__ uint64_t s_st[WG / 64][2];  // transitions | completed << 32, created | canceled << 32
  __shared__ uint64_t s_ex[LB_FIELDS];   // the tile's exclusive prefix
  __shared__ uint64_t s_part[3][LB_FIELDS];  // its parts: in the group, earlier groups of the round, the round base
  __shared__ int s_void;                 // a hand-off timed out: the tile's prefix is unknown, nothing is emitted
  __shared__ uint32_t s_tile;            // ZB_CFG_SHARED_GPU: the workgroup's next claimed tile
  constexpr bool claim = CLAIM;
  if (claim && blockIdx.x == 0 && threadIdx.x == 0) *P.tile_claim_next = 0;  // (the next launch starts after this one ends)
  const WaveHdr* hin = P.hdr + (P.wave & 1);
  WaveHdr* hout = P.hdr + ((P.wave + 1) & 1);
  const Chunk c = wave_chunk(P, hin);
  if (c.n <= 0) {  // nothing in this wave (the batch outran quiescence): carry the header forward
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      *hout = *hin;
      P.merge_count[P.wave & 1] = 0;
      P.cond_count[P.wave & 1] = 0;
      if (P.sub_count) clear_sub_counts(P);
    }
    return;
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t ntiles = (c.n + WG - 1) / WG;
  const int64_t gen_end = gen_limit(P, hin);  // (the batch tails read below)
  const int64_t end = hin->end, wf_next = hin->wf_next, job_next = hin->job_next;
  const uint64_t rows_next = (uint64_t)hin->rows_next, arena_next = (uint64_t)hin->arena_next;
  const uint64_t par = (uint64_t)(P.wave & 1) * P.job_cap;
  const int64_t G = gridDim.x;
  const int64_t GPR = (G + LB_GROUP - 1) / LB_GROUP;  // groups per round
  const uint32_t tag8 = P.lb_tag8, tag_grp = lb_tag(P.epoch, 0), tag_rnd = lb_tag(P.epoch, 1);
  uint64_t* const lbA = P.lookback;
  uint64_t* const lbG = P.lookback + 2 * P.lb_tiles;
  uint64_t* const lbR = lbG + (uint64_t)LB_FIELDS * (P.lb_tiles + 512);
  // the workgroup's statistics (transitions, completed, created, canceled): summed over its tiles, added to the
  // partition counters once at the end (they are not part of the scan)
  uint64_t wg_sa = 0, wg_sb = 0;

#ifdef ZB_PHASES
  uint64_t ph_t = wall_clock64(), ph[4] = {0, 0, 0, 0};  // process, hand-off, emit, hand-off spins (first wave)
#define ZB_PHASE(k) do { const uint64_t ph_n = wall_clock64(); ph[k] += ph_n - ph_t; ph_t = ph_n; } while (0)
#else
#define ZB_PHASE(k) do { } while (0)
#endif
  // (the tile index stays wave-uniform, in scalar registers: read from LDS it would take vector registers and make
  //  every offset computed from it per-lane work -- C2 wave-only 16.6 -> 17.8 ms)
  int64_t tile = blockIdx.x;
  if (claim) {
    if (threadIdx.x == 0) s_tile = atomicAdd(P.tile_claim, 1u);
    __syncthreads();
    tile = (int64_t)__builtin_amdgcn_readfirstlane(s_tile);
  }
  [[maybe_unused]] int64_t ntl = 0;  // tiles this workgroup processed (ZB_PHASES)
  while (tile < ntiles) {
    ntl++;
    // the next claim: in flight while this tile loads its records (s_tile is rewritten after the tile scan's barrier)
    uint32_t next_claim = 0;
    if (claim && threadIdx.x == 0) next_claim = atomicAdd(P.tile_claim, 1u);
    const int64_t i = tile * WG + threadIdx.x;  // wave-relative index
    const int64_t r = c.begin + i;
    // ---- process (k_process)
    TState t;
    t.s = s_slots + threadIdx.x * MAX_SLOTS;
    t.ns = t.nwf = t.njob = t.nrow = 0;
    t.bytes = 0; t.merge = false; t.detail = false; t.err = 0; t.err_site = 0;
    t.transitions = t.completed = t.created = t.merges = t.canceled = 0;
    t.merge_bytes = t.cond_bytes = 0;
    t.sub = false;
    t.nexp = 0; t.exp_ord = 0; t.src_off = 0;
    uint32_t nconds = 0;
    if (threadIdx.x == 0) s_void = 0;  // (ordered before every wave's hand-off by the tile scan's barrier)
    if (r < c.end) {
      const zb_rec rec = P.log[r];
      const uint64_t lk = P.links[r];
      const uint32_t vl = P.vlen[r];
      if (!grouped(rec)) {
        process_record(P, rec, r, (uint32_t)lk, (uint32_t)(lk >> 32), t);
        annotate_slots(P, t, 0, rec, vl);
        for (int64_t q = r + 1; q < gen_end && q < r + 4; q++) {
          const zb_rec rec2 = P.log[q];
          if (!grouped(rec2)) break;
          const uint64_t lk2 = P.links[q];
          const uint32_t vl2 = P.vlen[q];
          t.src_off = (uint32_t)(q - r);
          const int ns0 = t.ns;
          process_record(P, rec2, q, (uint32_t)lk2, (uint32_t)(lk2 >> 32), t);
          annotate_slots(P, t, ns0, rec2, vl2);
        }
      }
    }
    for (int k = 0; k < t.ns; k++) {
      const Slot& sl = t.s[k];
      nconds += (sl.flags & SF_COND_JOB) ? 1 : 0;
      if (kind_vt(sl.d.kind) == ZB_VT_WORKFLOW_INSTANCE && kind_rt(sl.d.kind) == ZB_RT_EVENT) t.transitions++;
    }
    t.transitions += t.nexp;  // a fork's SEQUENCE_FLOW_TAKEN events
    const uint64_t nwf_staged = (uint64_t)t.nwf - t.nexp;
    const uint64_t w = (uint64_t)t.ns | (nwf_staged << CW_NWF) | ((uint64_t)t.njob << CW_NJOB) |
                       ((uint64_t)t.nrow << CW_NROW) | ((uint64_t)(t.merge ? 1 : 0) << CW_MERGE) |
                       ((uint64_t)(t.detail ? 1 : 0) << CW_DETAIL) | ((uint64_t)nconds << CW_NCOND) |
                       ((uint64_t)t.nexp << CW_NEXP) | ((uint64_t)t.bytes << 32);
    if (t.merge || t.detail) {  // (global, not LDS: 8 KB of LDS per workgroup cost a resident workgroup per CU)
      ItemInfo inf;
      inf.m_src = t.m_src; inf.m_tgt = t.m_tgt; inf.m_len = t.m_len; inf.m_bytes = t.merge ? t.m_bytes : 0;
      inf.d_pos = t.d_pos; inf.d_q = t.d_q; inf.d_type = t.d_type; inf.d_code = t.d_code; inf.d_a = t.d_a;
      inf.d_b = t.d_b; inf.has_detail = t.detail; inf.ns = (uint8_t)t.ns;
      P.info[i] = inf;
    }
    if (__ballot(t.sub)) {  // wave-uniform: this tile's subscribe steps, in the wave's job list (its stripe)
      const uint32_t s = blockIdx.x % SUB_STRIPES;
      const uint64_t scap = P.job_cap / SUB_STRIPES;
      const uint32_t slot = wave_alloc(P.sub_count + (P.wave & 1) * SUB_STRIPES + s, t.sub ? 1u : 0u);
      if (t.sub) {
        if (slot < scap) P.sub_jobs[s * scap + slot] = (uint64_t)t.sub_pos;
        else fail_at(t, DE_LOG_FULL, 36);
      }
    }
    if (t.err) {
      atomicOr(P.err, t.err);
      atomicMin((unsigned long long*)P.err_info, ((unsigned long long)r << 8) | (t.err_site & 0xff));
    }
    // ---- tile scan (packed as in k_emit): a = outputs | wf << 16 | job << 32 | row << 48,
    //      b = bytes | merges << 40 | conds << 52
    const uint64_t nexp = (w >> CW_NEXP) & 63;
    const uint64_t a0 = ((w & 7) + nexp) | ((((w >> CW_NWF) & 7) + nexp) << 16) | (((w >> CW_NJOB) & 7) << 32) |
                        (((w >> CW_NROW) & 7) << 48);
    const uint64_t b0 = (w >> 32) | (((w >> CW_MERGE) & 1) << 40) | (((w >> CW_NCOND) & 7) << 52);
    uint64_t a = a0, b = b0;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t ua = shfl_up64(a, d), ub = shfl_up64(b, d);
      if (lane >= d) { a += ua; b += ub; }
    }
    uint64_t st0 = (uint64_t)t.transitions | ((uint64_t)t.completed << 32);
    uint64_t st1 = (uint64_t)t.created | ((uint64_t)t.canceled << 32);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) { st0 += shfl_down64(st0, d); st1 += shfl_down64(st1, d); }
    if (lane == 63) { s_a[wv] = a; s_b[wv] = b; }
    if (lane == 0) { s_st[wv][0] = st0; s_st[wv][1] = st1; }
    __syncthreads();
    ZB_PHASE(0);  // process + tile scan
    uint64_t ta = 0, tb = 0;
#pragma unroll
    for (int k = 0; k < WG / 64; k++) {
      if (k < wv) { a += s_a[k]; b += s_b[k]; }
      ta += s_a[k]; tb += s_b[k];
    }
    a -= a0;
    b -= b0;
    // ---- offsets: this tile's place in its round (k) and group (gi, position u)
    const int64_t k = tile / G, j = tile - k * G;
    const int64_t gi = j / LB_GROUP, u = j % LB_GROUP;
    const int64_t t_grp0 = tile - u;  // the group's first tile
    const bool last_of_chunk = tile == ntiles - 1;
    const bool last_of_group = u == LB_GROUP - 1 || j == G - 1 || last_of_chunk;
    const uint64_t gg = (uint64_t)(k * GPR + gi);  // the group's index among the wave's groups
    if (claim && threadIdx.x == 0) s_tile = next_claim;  // (every thread has read this tile's index)
    const uint64_t t_start = wall_clock64();
    if (wv == 0) {
      // the aggregate, published first (lane 0), then this tile's exclusive prefix within its group
      const uint64_t tbytes = tb & 0xffffffffffull;
      const uint64_t tmerge = (tb >> 40) & 0xfff, tcond = tb >> 52;
      if (lane == 0) {
        const uint64_t tb36 = tbytes < (1ull << 36) ? tbytes : (1ull << 36) - 1;
        if (tbytes != tb36) atomicOr(P.err, (uint32_t)DE_ARENA_FULL);  // (a tile's blobs past 64 GB: no arena holds them)
        __hip_atomic_store(lbA + 2 * tile, lb_pack_a(tag8, ta), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(lbA + 2 * tile + 1, lb_pack_b(tag8, tb36, tmerge, tcond), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        wg_sa += s_st[0][0] + s_st[1][0] + s_st[2][0] + s_st[3][0];
        wg_sb += s_st[0][1] + s_st[1][1] + s_st[2][1] + s_st[3][1];
      }
      const uint64_t* gp[2] = {lbA + 2 * (t_grp0 + lane), lbA + 2 * (t_grp0 + lane) + 1};
      const uint32_t tg[2] = {tag8, tag8};
      uint64_t v[2] = {0, 0};
      const bool ok = lb_wait<2>(P.err, gp, tg, 56, lane < u, v, t_start);
      uint64_t x0 = 0, x1 = 0, x2 = 0, x3 = 0;  // rec | wf << 32, job | row << 32, merges | conds << 32, bytes
      if (lane < u) {
        x0 = ((v[0] >> 39) & 0x1ffff) | (((v[0] >> 22) & 0x1ffff) << 32);
        x1 = ((v[0] >> 11) & 0x7ff) | ((v[0] & 0x7ff) << 32);
        x2 = ((v[1] >> 47) & 0x1ff) | (((v[1] >> 36) & 0x7ff) << 32);
        x3 = v[1] & ((1ull << 36) - 1);
      }
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) {
        x0 += __shfl_xor(x0, d, 64); x1 += __shfl_xor(x1, d, 64);
        x2 += __shfl_xor(x2, d, 64); x3 += __shfl_xor(x3, d, 64);
      }
      // lane f < 8: field f of the exclusive prefix within the group (bytes whole in field 4, field 5 zero)
      const uint64_t e = lane == 0 ? (uint32_t)x0 : lane == 1 ? x0 >> 32 : lane == 2 ? (uint32_t)x1 :
                         lane == 3 ? x1 >> 32 : lane == 4 ? x3 : lane == 6 ? (uint32_t)x2 : lane == 7 ? x2 >> 32 : 0;
      if (!ok && lane == 0) s_void = 1;
      if (lane < LB_FIELDS) s_part[0][lane] = ok ? e : 0;
      if (ok && last_of_group && lane < LB_FIELDS) {  // the group's total, for the later groups of the round
        const uint64_t own = lane == 4 ? tbytes : lane == 5 ? 0 : lb_field(ta, tmerge, tcond, lane);
        const uint64_t tot = e + own;
        const uint32_t val = lane == 4 ? (uint32_t)tot : lane == 5 ? (uint32_t)((x3 + tbytes) >> 32) : (uint32_t)tot;
        __hip_atomic_store(lbG + gg * LB_FIELDS + lane, ((uint64_t)tag_grp << 32) | val, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    } else if (wv == 1) {
      // the totals of the round's earlier groups: lane = 8 * group + field, 8 groups per pass
      uint64_t acc = 0;
      bool ok = true;
      for (int64_t base = 0; base < gi && ok; base += 64 / LB_FIELDS) {
        const int64_t q = base + lane / LB_FIELDS;
        const uint64_t* gp[1] = {lbG + (uint64_t)(k * GPR + q) * LB_FIELDS + lane % LB_FIELDS};
        const uint32_t tg[1] = {tag_grp};
        uint64_t v[1] = {0};
        ok = lb_wait<1>(P.err, gp, tg, 32, q < gi, v, t_start);
        uint64_t x = q < gi ? (uint32_t)v[0] : 0;
#pragma unroll
        for (int d = LB_FIELDS; d < 64; d <<= 1) x += __shfl_xor(x, d, 64);
        acc += x;
      }
      // bytes travel as two 32-bit granules (fields 4, 5): recombine the carry
      const uint64_t lo = __shfl(acc, 4, 64), hi = __shfl(acc, 5, 64);
      if (!ok && lane == 0) s_void = 1;
      if (lane < LB_FIELDS) s_part[1][lane] = !ok ? 0 : lane == 4 ? lo + (hi << 32) : lane == 5 ? 0 : acc;
    } else if (wv == 2) {
      // the round's base, published by the previous round's last tile
      const uint64_t* gp[1] = {lbR + (uint64_t)k * LB_FIELDS + lane % LB_FIELDS};
      const uint32_t tg[1] = {tag_rnd};
      uint64_t v[1] = {0};
      const bool ok = lb_wait<1>(P.err, gp, tg, 32, k > 0 && lane < LB_FIELDS, v, t_start);
      const uint64_t x = k > 0 ? (uint32_t)v[0] : 0;
      const uint64_t hi = __shfl(x, 5, 64);
      if (!ok && lane == 0) s_void = 1;
      if (lane < LB_FIELDS) s_part[2][lane] = !ok ? 0 : lane == 4 ? x + (hi << 32) : lane == 5 ? 0 : x;
    }
    __syncthreads();
    if (wv == 0) {
      const uint64_t tbytes = tb & 0xffffffffffull;
      const uint64_t own = lane == 4 ? tbytes : lane == 5 ? 0 : lb_field(ta, (tb >> 40) & 0xfff, tb >> 52, lane);
      const uint64_t ex = lane < LB_FIELDS ? s_part[0][lane] + s_part[1][lane] + s_part[2][lane] : 0;
      const uint64_t inc = ex + own;
      const uint64_t t0 = __shfl(inc, 0, 64), t1 = __shfl(inc, 1, 64), t2 = __shfl(inc, 2, 64);
      const uint64_t t3 = __shfl(inc, 3, 64), t4 = __shfl(inc, 4, 64), t6 = __shfl(inc, 6, 64);
      const uint64_t t7 = __shfl(inc, 7, 64);
      if (s_void) {
        if (lane == 0) atomicOr(P.err, (uint32_t)DE_TIMEOUT);  // (the host fails the wave: nothing is written from a
      } else {                                                 //  partial prefix; the other tiles stop waiting too)
        if (lane < LB_FIELDS) s_ex[lane] = ex;
        // the last tile of a round hands the next round its base
        if (j == G - 1 && !last_of_chunk && lane < LB_FIELDS) {
          const uint32_t val = lane == 4 ? (uint32_t)t4 : lane == 5 ? (uint32_t)(t4 >> 32) : (uint32_t)inc;
          __hip_atomic_store(lbR + (uint64_t)(k + 1) * LB_FIELDS + lane, ((uint64_t)tag_rnd << 32) | val,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // the chunk's last tile: totals -> next wave header, counters, job counts (k_scan's job)
        if (last_of_chunk && lane == 0) {
          WaveHdr h = *hin;
          h.begin = c.end;
          h.end = hin->end + (int64_t)t0;
          h.gen_end = (c.end == hin->gen_end) ? h.end : hin->gen_end;
          h.wf_next = hin->wf_next + 5 * (int64_t)t1;
          h.job_next = hin->job_next + 5 * (int64_t)t2;
          h.rows_next = hin->rows_next + (int64_t)t3;
          h.arena_next = hin->arena_next + (int64_t)t4;
          P.stats[6] += 1;
          uint32_t err = 0;
          if ((uint64_t)h.end > P.log_cap) err |= DE_LOG_FULL;
          if ((uint64_t)h.rows_next > P.row_cap) err |= DE_ROWS_FULL;
          if ((uint64_t)h.arena_next > P.arena_cap) err |= DE_ARENA_FULL;
          if (t6 > P.job_cap || t7 > P.job_cap) err |= DE_LOG_FULL;
          if (err) atomicOr(P.err, err);
          *hout = h;
                P.merge_count[P.wave & 1] = (uint32_t)t6;
          P.cond_count[P.wave & 1] = (uint32_t)t7;
          if (P.sub_count) clear_sub_counts(P);  // the next wave's subscribe list
        }
      }
    }
    __syncthreads();
    ZB_PHASE(1);  // hand-off (+ the chunk's header on the last tile)
    // ---- emit (k_emit) straight from the LDS slots
    const uint64_t we = w;
    const int ns = (int)(we & 7);
    if (!s_void && r < c.end && (ns || ((we >> CW_NEXP) & 63) || ((we >> CW_DETAIL) & 1))) {
      const uint64_t out_rec = (uint64_t)end + s_ex[0] + (a & 0xffff);
      const uint64_t wf0 = s_ex[1] + ((a >> 16) & 0xffff);
      const uint64_t job0 = s_ex[2] + ((a >> 32) & 0xffff);
      const uint64_t row0 = rows_next + s_ex[3] + (a >> 48);
      const uint64_t bump = arena_next + s_ex[4] + (b & 0xffffffffffull);
      const uint64_t merge_j = s_ex[6] + ((b >> 40) & 0xfff);
      const uint64_t cond_j = s_ex[7] + (b >> 52);
      ItemInfo inf{};
      if (we & ((1ull << CW_MERGE) | (1ull << CW_DETAIL))) inf = P.info[i];
      emit_item(P, c, i, we, s_slots + threadIdx.x * MAX_SLOTS, inf, out_rec, wf0, job0, row0, bump, merge_j, cond_j,
                wf_next, job_next, par);
    }
    __syncthreads();  // LDS slots and scan scratch are reused by the next tile
    ZB_PHASE(2);  // emit
    tile = claim ? (int64_t)__builtin_amdgcn_readfirstlane(s_tile) : tile + G;
  }
  if (threadIdx.x == 0 && (wg_sa | wg_sb)) {  // (into the workgroup's bank: launch_stat_fold)
    unsigned long long* bank = (unsigned long long*)(P.stats + 8 + 8 * (blockIdx.x % STAT_BANKS));
    atomicAdd(bank + 0, (unsigned long long)(uint32_t)wg_sa);  // transitions
    atomicAdd(bank + 1, (unsigned long long)(wg_sa >> 32));    // completed instances
    atomicAdd(bank + 2, (unsigned long long)(uint32_t)wg_sb);  // created
    atomicAdd(bank + 3, (unsigned long long)(wg_sb >> 32));    // canceled
  }
#ifdef ZB_PHASES
  if (threadIdx.x == 0 && P.phase) {
    for (int k = 0; k < 3; k++) atomicAdd(P.phase + k, (unsigned long long)ph[k]);
    atomicAdd(P.phase + 4, (unsigned long long)ntl);
    atomicAdd(P.phase + 3, (unsigned long long)ntl);
  }
#endif
#undef ZB_PHASE
}


// ------------------------------------------------------------------------------ k_conflict
// The chunk of a generation that holds records of conflicting instances (WaveParams.conf_*) ends at the first
// record, in log order, of such an instance whose earlier record is in the generation's unprocessed range: two
// passes over [begin, gen_end) (the first position of each instance, then the smallest later one). A batch's
// continuation records are processed with their head, in order, by one thread: only heads count.
__device__ __forceinline__ int64_t conf_slot(const WaveParams& P, int64_t key) {
  if (key < 0) return -1;
  uint64_t s = ((uint64_t)key * 0x9E3779B97F4A7C15ull >> 32) & P.conf_mask;
  for (uint64_t n = 0; n <= P.conf_mask; n++, s = (s + 1) & P.conf_mask) {
    const int64_t k = P.conf_keys[s];
    if (k == key) return (int64_t)s;
    if (k == INT64_MIN) return -1;
  }
  return -1;
}
template <bool SPLIT>
__global__ void __launch_bounds__(256) k_conflict(WaveParams P) {
  const WaveHdr* hin = P.hdr + (P.wave & 1);
  const int64_t b = hin->begin, g = gen_limit(P, hin);
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t r = b + (int64_t)blockIdx.x * 256 + threadIdx.x; r < g; r += stride) {
    const zb_rec rec = P.log[r];
    if (grouped(rec)) continue;
    const int64_t s = conf_slot(P, conflict_key(rec.inst_key, rec.key, rec.kind));
    if (s < 0) continue;
    if (!SPLIT) atomicMin((unsigned long long*)(P.conf_first + s), (unsigned long long)r);
    else if (r > P.conf_first[s]) atomicMin((unsigned long long*)P.conf_split, (unsigned long long)r);
  }
}
void launch_conflict(const WaveParams& p, hipStream_t stream) {
  hipLaunchKernelGGL((k_conflict<false>), dim3(512), dim3(256), 0, stream, p);
  hipLaunchKernelGGL((k_conflict<true>), dim3(512), dim3(256), 0, stream, p);
}

__global__ void __launch_bounds__(64) k_stat_fold(uint64_t* stats) {
  uint64_t* bank = stats + 8 + 8 * threadIdx.x;
  uint64_t x[4];
#pragma unroll
  for (int f = 0; f < 4; f++) {
    x[f] = bank[f];
    bank[f] = 0;
  }
#pragma unroll
  for (int f = 0; f < 4; f++)
    for (int d = 32; d >= 1; d >>= 1) x[f] += __shfl_xor(x[f], d, 64);
  if (threadIdx.x == 0) {
    stats[0] += x[0];
    stats[1] += x[1];
    stats[2] += x[2];
    stats[7] += x[3];
  }
}
void launch_stat_fold(uint64_t* stats, hipStream_t stream) {
  static_assert(STAT_BANKS == 64, "one lane per bank");
  hipLaunchKernelGGL(k_stat_fold, dim3(1), dim3(64), 0, stream, stats);
}

void launch_wave(const WaveParams& p, int grid, hipStream_t stream) {
  if (p.tile_claim) hipLaunchKernelGGL(k_wave<true>, dim3(grid), dim3(WG), 0, stream, p);
  else hipLaunchKernelGGL(k_wave<false>, dim3(grid), dim3(WG), 0, stream, p);
}
int wave_resident_per_cu() {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_wave<false>, WG, 0) != hipSuccess) return 0;
  return n;
}

void launch_pre(const WaveParams& p, hipStream_t stream) {
  hipLaunchKernelGGL(k_pre, dim3(p.grid), dim3(WG), 0, stream, p);
}
void launch_process(const WaveParams& p, hipStream_t stream) {
  hipLaunchKernelGGL(k_process, dim3(p.grid), dim3(WG), 0, stream, p);
}
void launch_scan(const WaveParams& p, hipStream_t stream) {
  hipLaunchKernelGGL(k_scan, dim3(1), dim3(SCAN_WG), 0, stream, p);
}
void launch_emit(const WaveParams& p, hipStream_t stream) {
  hipLaunchKernelGGL(k_emit, dim3(p.grid), dim3(WG), 0, stream, p);
}
void launch_subscribe(const WaveParams& p, hipStream_t stream) {
  // five workgroups per CU (82 VGPRs): the correlation-key queries of a wave that opens 1M subscriptions are
  // latency-bound (C5: 426 us on one workgroup per CU); a wave without subscribe steps exits at the count
  hipLaunchKernelGGL(k_subscribe, dim3(1280), dim3(256), 0, stream, p);
}

}  // namespace zbg
