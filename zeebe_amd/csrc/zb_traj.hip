// zb_traj.hip — run-to-quiescence of a batch of independent workflow instances ("trajectory" path).
//
// Why this is exact. The reference processes its log FIFO, one record at a time
// (StreamProcessorController.java:296-414), so a batch of CREATE commands written to an idle
// partition is processed in breadth-first generations, and inside a generation records are ordered
// by their parent's position. By induction from generation 0 (the CREATEs, in instance order) every
// generation is instance-major: instance i's records of generation g are contiguous and come after
// those of instances < i. Workflow instances without message correlation never read each other's
// state, so instance i's sequence of generations ("trajectory") depends only on its own records and
// element instances. What couples instances is the log position and the keys: the partition's
// KeyGenerator(1, 5) / job KeyGenerator(2, 5) (KeyGenerator.java:28-60) hand out keys in processing
// order, so the key and position of a follow-up emitted while processing generation g are
//     base(g) + (follow-ups emitted by instances < i in generation g) + (emission index).
//
// So one thread owns one instance and keeps its element instances and its current generation in
// registers; the only cross-instance quantity is a per-(generation, workgroup) count:
//   k_traj<false>   (count)  step every instance to quiescence; per generation write the
//                            workgroup's (records, wf keys, job keys) totals.
//   k_traj_scan              per generation: exclusive prefix of the workgroup totals.
//   k_traj_base              prefix of the generation totals: absolute position / key bases.
//   k_traj<true>    (emit)   step again; per generation a workgroup scan places every follow-up at
//                            its final log position with its final keys; merges and condition
//                            incidents write their payload blobs; live element instances are
//                            written to the partition's SoA rows at the end.
//   k_traj_commit            new wave header (log end, key generators, allocators).
// The count pass writes nothing but the totals, so when an instance needs something this path does
// not implement (more than TR element instances or TF records per generation, message
// subscriptions, a processing failure) it raises a flag and the host runs the general wave path
// (zb_wave.hip) on the same injected log instead — both are gfx950 kernels, nothing runs on the CPU.
//
// Handlers mirror bpmn_step/process_record in zb_wave.hip (same reference citations); the two paths
// are checked against each other and the oracle by tests/test_gpu_parity.py.
#include <hip/hip_runtime.h>

#include "zb_devlib.hpp"
#include "zb_kernels.hpp"
#include "zb_wavelib.hpp"
#include "zb_xlock.hpp"
#include "zb_tmpl.hpp"

namespace zbg {

constexpr int TWG = TRAJ_WG;

constexpr uint8_t LN = 0xff;  // no local row

// The control fields of a DevElem (zb_device.hpp layout), as dword loads through the constant
// address space: seven independent s_load_dword with a uniform element index, no byte loads, no
// stack copy for the dynamically indexed step table.
struct ElemCtl {
  uint32_t st[3];  // step[0..11]                                   (dwords 1..3)
  uint32_t ot;     // out0 | target << 16                           (dword 4)
  uint32_t sd;     // start | dflt << 16                            (dword 5)
  uint32_t cc;     // cond_begin | cond_count << 16                 (dword 6)
  __device__ __forceinline__ uint8_t step(uint32_t intent) const {
    const uint32_t w = intent < 4 ? st[0] : (intent < 8 ? st[1] : st[2]);
    return (uint8_t)(w >> ((intent & 3) * 8));
  }
  __device__ __forceinline__ uint16_t out0() const { return (uint16_t)ot; }
  __device__ __forceinline__ uint16_t target() const { return (uint16_t)(ot >> 16); }
  __device__ __forceinline__ uint16_t start() const { return (uint16_t)sd; }
  __device__ __forceinline__ uint16_t dflt() const { return (uint16_t)(sd >> 16); }
  __device__ __forceinline__ uint16_t cond_begin() const { return (uint16_t)cc; }
  __device__ __forceinline__ uint16_t cond_count() const { return (uint16_t)(cc >> 16); }
};
static_assert(offsetof(DevElem, step) == 4 && offsetof(DevElem, out0) == 16 && offsetof(DevElem, target) == 18 &&
                  offsetof(DevElem, start) == 20 && offsetof(DevElem, dflt) == 22 &&
                  offsetof(DevElem, cond_begin) == 24 && offsetof(DevElem, cond_count) == 26 &&
                  offsetof(DevElem, job_payload) == 40 && sizeof(DevElem) == 80,
              "ElemCtl mirrors the DevElem layout");
__device__ __forceinline__ uint32_t elem_dword(const TrajParams& P, uint32_t e, uint32_t d) {
  return K((const uint32_t*)P.elems)[(uint64_t)e * (sizeof(DevElem) / 4) + d];
}
__device__ __forceinline__ ElemCtl elem_ctl(const TrajParams& P, uint32_t e) {
  ElemCtl c;
  c.st[0] = elem_dword(P, e, 1); c.st[1] = elem_dword(P, e, 2); c.st[2] = elem_dword(P, e, 3);
  c.ot = elem_dword(P, e, 4); c.sd = elem_dword(P, e, 5); c.cc = elem_dword(P, e, 6);
  return c;
}

enum TrajFlags : uint8_t {
  TK_WF = 1,         // key := new wf key #ord
  TK_JOB = 2,        // key := new job key #ord
  TK_INST = 4,       // the instance key := new wf key #ord (CREATE)
  TK_ROW_INIT = 8,   // initialise rself as an ELEMENT_READY insert (ElementInstanceWriter.writeNewEvent)
  TK_MERGED = 16,    // payload := this generation's merge result
  TK_DETAIL = 32,    // payload := this generation's incident detail blob
};

// trajectory-path error bits (count pass -> host falls back to the wave path)
// TE_XTREE: a merge needs the exact payload tree (zb_xmerge.hpp), which the wave pipeline runs: the batch falls back
enum TrajErr : uint32_t { TE_FALLBACK = 1u, TE_XTREE = 1u << 29, TE_REGEN = 1u << 30 };

// flat-merge staging in LDS (emit pass): per thread the two input blobs and the output blob
constexpr int FM_WORDS = 12;                  // 48-byte blob slots: documents of <= 44 bytes
constexpr int FM_BYTES = FM_WORDS * 4;
constexpr int FM_STRIDE = 3 * FM_WORDS + 1;   // odd stride: lanes at the same offset hit distinct banks
// Template emit (k_tmpl) packs the two inputs back to back: with ns + nt <= 4 * OUT_WORDS - 7 they take
// <= (ns + nt + 14) / 4 words. Uniform batches keep a 36-byte output blob (10 + 9 = 19 words per thread,
// odd: distinct banks; 19.5 KB per workgroup, eight workgroups per CU); class batches, whose CREATE
// payloads are larger, keep the 48-byte blob (13 + 12 = 25 words, six workgroups per CU).
template <bool CLS> struct TmLayout {
  static constexpr int OUT_WORDS = CLS ? 12 : 9;
  static constexpr int IN_WORDS = (4 * OUT_WORDS - 7 + 14) / 4;
  static constexpr int STRIDE = IN_WORDS + OUT_WORDS;
};

// Condition documents are staged into the same per-thread LDS slot before the json-el VM runs: the
// VM reads its document token by token (dependent byte loads), which from HBM costs a memory
// latency per token; the staging copy issues all of its 8-byte loads back to back instead.
constexpr int CD_BYTES = (FM_STRIDE - 1) * 4;  // [u32 len][document] of documents <= 140 bytes
__device__ __forceinline__ void stage_copy(const uint8_t* pp, uint32_t len, uint32_t* slot) {
  const uint2* g = (const uint2*)pp;  // arena blobs are 8-aligned and padded to 8 bytes
  const uint32_t n8 = (len + 4 + 7) / 8;
#pragma unroll 1
  for (uint32_t c = 0; c < n8; c += 8) {
    uint2 v[8];
#pragma unroll
    for (uint32_t k = 0; k < 8; k++)
      if (c + k < n8) v[k] = g[c + k];
#pragma unroll
    for (uint32_t k = 0; k < 8; k++)
      if (c + k < n8) { slot[2 * (c + k)] = v[k].x; slot[2 * (c + k) + 1] = v[k].y; }
  }
}
__device__ __forceinline__ const uint8_t* stage_doc(const uint8_t* pp, uint32_t len, uint32_t* slot) {
  if (slot == nullptr || len + 4 > (uint32_t)CD_BYTES) return pp + 4;
  stage_copy(pp, len, slot);
  return (const uint8_t*)slot + 4;
}

struct TRec {
  uint32_t key, scope_key;
  uint32_t payload;
  uint16_t elem;
  uint8_t intent, kind;
  uint8_t rself, rscope, flags, ord;
};

// Per-instance state lives in ext-vector registers: a dynamic index becomes an extract / insert
// element (selects), never an address, so nothing is spilled to scratch.
typedef uint32_t u32x4 __attribute__((ext_vector_type(TR)));
typedef int32_t i32x4 __attribute__((ext_vector_type(TR)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(TF)));

// One generation of one instance (<= TF records), structure of vectors
struct Gen {
  u32x2 key, sk;
  u32x2 pay;
  u32x2 m0;  // elem | intent << 16 | kind << 24
  u32x2 m1;  // rself | rscope << 8 | flags << 16 | ord << 24
  __device__ __forceinline__ TRec get(int k) const {
    TRec r;
    r.key = key[k]; r.scope_key = sk[k]; r.payload = pay[k];
    const uint32_t a = m0[k], b = m1[k];
    r.elem = (uint16_t)a; r.intent = (uint8_t)(a >> 16); r.kind = (uint8_t)(a >> 24);
    r.rself = (uint8_t)b; r.rscope = (uint8_t)(b >> 8); r.flags = (uint8_t)(b >> 16); r.ord = (uint8_t)(b >> 24);
    return r;
  }
  __device__ __forceinline__ void set(int k, const TRec& r) {
    key[k] = r.key; sk[k] = r.scope_key; pay[k] = r.payload;
    m0[k] = (uint32_t)r.elem | ((uint32_t)r.intent << 16) | ((uint32_t)r.kind << 24);
    m1[k] = (uint32_t)r.rself | ((uint32_t)r.rscope << 8) | ((uint32_t)r.flags << 16) | ((uint32_t)r.ord << 24);
  }
};

// One workflow instance: its element instances (local rows) and its current generation.
struct Inst {
  u32x4 rkey, rjob;  // key ordinals (the row's scope key is its parent's key)
  u32x4 rpay;
  u32x4 rmeta;  // elem | state << 16 | parent << 24
  i32x4 rnch;
  uint32_t used, to_free;
  uint32_t inst_key;
  uint32_t ckey, crow;  // class batch: outcome key of the instance's class, its agg / mgen row
  Gen cur, nx;
  int nc, nn, nwf, njob;
  // this generation's payload work: one merge and one incident detail at most
  bool merge, detail;
  uint32_t m_src, m_tgt, m_len;
  uint8_t d_code, d_a, d_b;
  uint16_t d_q;
  int64_t d_pos;
  uint32_t err;
  // stats (emit pass)
  uint32_t transitions, completed, created, merges, cond_bytes;
  uint64_t merge_bytes;

  __device__ __forceinline__ uint8_t state(int r) const { return (uint8_t)(rmeta[r] >> 16); }
  __device__ __forceinline__ uint16_t elem(int r) const { return (uint16_t)rmeta[r]; }
  __device__ __forceinline__ uint8_t parent(int r) const { return (uint8_t)(rmeta[r] >> 24); }
  __device__ __forceinline__ bool alive(int r) const { return r != LN && state(r) != 0; }
  __device__ __forceinline__ uint32_t scope_of(int r) const {
    const int p = parent(r);
    return p == LN ? NOK : rkey[p];
  }
  __device__ __forceinline__ void set_state(int r, uint8_t s) {
    rmeta[r] = (rmeta[r] & 0xff00ffffu) | ((uint32_t)s << 16);
  }
  __device__ __forceinline__ void set_meta(int r, uint16_t el, uint8_t st, uint8_t par) {
    rmeta[r] = (uint32_t)el | ((uint32_t)st << 16) | ((uint32_t)par << 24);
  }
  __device__ __forceinline__ int alloc() {
    const uint32_t freebits = ~used & ((1u << TR) - 1);
    if (!freebits) { err |= TE_FALLBACK; return LN; }
    const int r = __builtin_ctz(freebits);
    used |= 1u << r;
    set_meta(r, NO_ELEM, 0, LN);
    rnch[r] = 0;
    return r;
  }
  // ElementInstanceWriter: remove on a final state; the slot is reused from the next generation on
  __device__ __forceinline__ void remove(int r) {
    const int p = parent(r);
    set_state(r, 0);
    if (p != LN) rnch[p] -= 1;
    to_free |= 1u << r;
  }
  __device__ __forceinline__ void push(const TRec& s) {
    if (nn >= TF) { err |= TE_FALLBACK; return; }
    nx.set(nn, s);
    nn++;
  }
};

__device__ __forceinline__ int64_t wf_key(const TrajParams& P, uint32_t o) {
  return o == NOK ? -1 : P.wf_start + 5 * (int64_t)o;
}
__device__ __forceinline__ int64_t job_key(const TrajParams& P, uint32_t o) {
  return o == NOK ? -1 : P.job_start + 5 * (int64_t)o;
}

__device__ __forceinline__ uint32_t tblob_bytes(uint32_t len) { return (4 + len + 7) & ~7u; }

// upper bound of the length of the document behind a symbolic payload ref (trace count pass)
__device__ __forceinline__ uint32_t sym_bound(const TrajParams& P, uint32_t sym, uint32_t row) {
  if (sym == PAY_CREATE) return P.max_create;
  if (sym & PAY_MERGE) return P.mgen[row + (sym & 0xffff)].stride - 4;
  return arena_len(P.arena, sym);
}

__device__ __forceinline__ void t_incident(Inst& I, const TRec& rec, int64_t pos, uint8_t code, uint8_t a, uint8_t b, uint16_t q) {
  // BpmnStepContext.raiseIncident: IncidentIntent.CREATE command, key null, CONDITION_ERROR
  TRec s;
  s.key = NOK;
  s.scope_key = rec.key;  // activityInstanceKey = failing record's key
  s.payload = 0;
  s.elem = rec.elem;
  s.intent = 0;
  s.kind = make_kind(ZB_VT_INCIDENT, ZB_RT_COMMAND, I.nn > 0);
  s.rself = LN; s.rscope = LN; s.flags = TK_DETAIL; s.ord = 0;
  if (I.detail) { I.err |= TE_FALLBACK; return; }
  I.detail = true;
  I.d_code = code; I.d_a = a; I.d_b = b; I.d_q = q; I.d_pos = pos;
  I.push(s);
}

// bpmn_step (zb_wave.hip) on local rows: BpmnStepProcessor.java:92-251 guards + step handlers.
// COND: exclusive splits are evaluated here (else they send the batch to the wave pipeline).
template <bool EMIT, bool COND>
__device__ __forceinline__ void t_step(const TrajParams& P, Inst& I, const TRec& rec, int64_t pos, uint32_t* slot) {
  // (rec's control fields are wave-uniform in a uniform batch: t_record scalarized them)
  const uint8_t intent = rec.intent;
  const bool stateless = intent == WI_SEQUENCE_FLOW_TAKEN || intent == WI_START_EVENT_OCCURRED ||
                         intent == WI_END_EVENT_OCCURRED || intent == WI_GATEWAY_ACTIVATED;
  const int rself = rec.rself, rscope = rec.rscope;
  const bool self_alive = !stateless && I.alive(rself);
  const bool scope_alive = I.alive(rscope);
  if (!self_alive && !scope_alive) return;  // BpmnStepProcessor.java:244-247
  bool ok;
  switch (intent) {
    case WI_ELEMENT_READY: case WI_ELEMENT_ACTIVATED: case WI_ELEMENT_COMPLETING:
      if (!self_alive) { I.err |= TE_FALLBACK; return; }
      ok = I.state(rself) == intent;
      break;
    case WI_ELEMENT_COMPLETED: case WI_END_EVENT_OCCURRED: case WI_GATEWAY_ACTIVATED:
    case WI_START_EVENT_OCCURRED: case WI_SEQUENCE_FLOW_TAKEN:
      ok = scope_alive && I.state(rscope) == WI_ELEMENT_ACTIVATED;
      break;
    case WI_ELEMENT_TERMINATING: ok = true; break;
    case WI_ELEMENT_TERMINATED: ok = scope_alive && I.state(rscope) == WI_ELEMENT_TERMINATING; break;
    default: ok = false;
  }
  if (!ok) return;
  if (rec.elem == NO_ELEM) { I.err |= TE_FALLBACK; return; }
  const ElemCtl el = elem_ctl(P, rec.elem);  // scalar loads when rec.elem is wave-uniform
  const uint8_t step = el.step(intent);
  if (step == ST_UNBOUND || step == ST_NONE) return;

  TRec s = rec;
  s.flags = 0; s.ord = 0;
  switch (step) {
    case ST_APPLY_INPUT_MAPPING: {  // InputMappingHandler (no io mappings)
      s.intent = WI_ELEMENT_ACTIVATED;
      s.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE, ZB_RT_EVENT, I.nn > 0);
      I.set_state(rself, WI_ELEMENT_ACTIVATED);
      I.rpay[rself] = rec.payload;
      I.push(s);
      break;
    }
    case ST_APPLY_OUTPUT_MAPPING: {  // OutputMappingHandler :42-85, outputBehavior null -> merge
      if (!scope_alive || I.merge) { I.err |= TE_FALLBACK; return; }
      I.merge = true;
      I.m_src = rec.payload;
      I.m_tgt = I.rpay[rscope];
      if (EMIT) I.m_len = arena_len(P.arena, I.m_src) + arena_len(P.arena, I.m_tgt) + 8;
      s.intent = WI_ELEMENT_COMPLETED;
      s.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE, ZB_RT_EVENT, I.nn > 0);
      s.flags = TK_MERGED;
      s.rself = LN;
      I.remove(rself);
      I.push(s);
      break;
    }
    case ST_CREATE_JOB: {  // CreateJobHandler :33-56 -> JOB CREATE command, key null
      s.key = NOK;
      s.scope_key = rec.key;  // headers.activityInstanceKey
      s.intent = JI_CREATE;
      s.kind = make_kind(ZB_VT_JOB, ZB_RT_COMMAND, I.nn > 0);
      I.push(s);
      break;
    }
    case ST_EXCLUSIVE_SPLIT: {  // ExclusiveSplitHandler :38-71 (first true condition, else default)
      if constexpr (!COND) {
        // class batch: the outcome is a digit of the class key (k_cls_classify evaluated this split's
        // conditions on the CREATE payload, which is the scope payload here: no merge precedes a split)
        uint32_t o = 0xffffffffu;
        const uint32_t cc = el.cond_count();
        // (a class batch's count pass is its trace, with symbolic payloads: it checks that the split reads
        // the CREATE payload, since k_cls_classify never saw a merge result)
        if (P.cls && (EMIT || rec.payload == PAY_CREATE))
          for (int k = 0; k < P.nsplits; k++)
            if (P.split_elem[k] == rec.elem) o = (I.ckey / P.split_stride[k]) % (cc + 2);
        uint16_t chosen = NO_ELEM;
        if (o < cc) chosen = K(P.cond_flows)[el.cond_begin() + o];
        else if (o == cc) chosen = el.dflt();
        // errors and missing defaults raise incidents: those batches take the per-instance path
        if (chosen == NO_ELEM) { I.err |= TE_FALLBACK; return; }
        I.cond_bytes += 1;  // trace: split visits (k_traj_commit: x CREATE payload bytes of the class)
        s.elem = chosen;
        s.intent = WI_SEQUENCE_FLOW_TAKEN;
        s.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE, ZB_RT_EVENT, I.nn > 0);
        s.flags = TK_WF; s.ord = (uint8_t)I.nwf++;
        s.rself = LN;
        I.push(s);
        break;
      } else {
        const uint8_t* pp = P.arena + (uint64_t)rec.payload * 8;
        const uint32_t len = *(const uint32_t*)pp;
        const uint8_t* doc = stage_doc(pp, len, slot);
        uint16_t chosen = NO_ELEM;
        CondOut co{0, 0, 0, 0};
        bool unsup = false;
        for (uint32_t c = 0; c < el.cond_count(); c++) {
          const uint16_t flow = K(P.cond_flows)[el.cond_begin() + c];
          const bool res = eval_condition(K(P.elems)[flow].cond_prog, P.code, doc, len, P.consts, P.queries,
                                          P.filters, P.pool, co, unsup);
          if (unsup || co.err) break;
          if (res) { chosen = flow; break; }
        }
        I.cond_bytes += len;
        if (unsup) { I.err |= TE_FALLBACK; return; }
        if (co.err) { t_incident(I, rec, pos, co.err & 7, co.a & 15, co.b & 15, co.q); break; }
        if (chosen == NO_ELEM) chosen = el.dflt();
        if (chosen == NO_ELEM) { t_incident(I, rec, pos, EC_NO_FLOW, 0, 0, 0); break; }
        s.elem = chosen;
        s.intent = WI_SEQUENCE_FLOW_TAKEN;
        s.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE, ZB_RT_EVENT, I.nn > 0);
        s.flags = TK_WF; s.ord = (uint8_t)I.nwf++;
        s.rself = LN;
        I.push(s);
        break;
      }
    }
    case ST_CONSUME_TOKEN: {  // ConsumeTokenHandler :30-43
      if (!scope_alive) { I.err |= TE_FALLBACK; return; }
      s.key = I.rkey[rscope];
      s.scope_key = I.scope_of(rscope);
      s.elem = I.elem(rscope);
      s.payload = rec.payload;
      s.intent = WI_ELEMENT_COMPLETING;
      s.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE, ZB_RT_EVENT, I.nn > 0);
      s.rself = (uint8_t)rscope;
      s.rscope = I.parent(rscope);
      I.set_state(rscope, WI_ELEMENT_COMPLETING);
      I.rpay[rscope] = rec.payload;
      I.push(s);
      break;
    }
    case ST_TAKE_SEQUENCE_FLOW:
    case ST_ACTIVATE_GATEWAY:
    case ST_TRIGGER_END_EVENT: {
      uint8_t out_intent;
      if (step == ST_TAKE_SEQUENCE_FLOW) { s.elem = el.out0(); out_intent = WI_SEQUENCE_FLOW_TAKEN; }
      else if (step == ST_ACTIVATE_GATEWAY) { s.elem = el.target(); out_intent = WI_GATEWAY_ACTIVATED; }
      else { s.elem = el.target(); out_intent = WI_END_EVENT_OCCURRED; }
      if (s.elem == NO_ELEM) { I.err |= TE_FALLBACK; return; }
      s.intent = out_intent;
      s.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE, ZB_RT_EVENT, I.nn > 0);
      s.flags = TK_WF; s.ord = (uint8_t)I.nwf++;
      s.rself = LN;
      I.push(s);
      break;
    }
    case ST_START_STATEFUL_ELEMENT: {  // -> ELEMENT_READY(new key), index insert with parent = scope
      const int row = I.alloc();
      if (row == LN) return;
      s.elem = el.target();
      s.intent = WI_ELEMENT_READY;
      s.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE, ZB_RT_EVENT, I.nn > 0);
      s.flags = TK_WF | TK_ROW_INIT; s.ord = (uint8_t)I.nwf++;
      s.rself = (uint8_t)row;
      s.rscope = scope_alive ? (uint8_t)rscope : LN;
      if (scope_alive) I.rnch[rscope] += 1;
      I.push(s);
      break;
    }
    case ST_TRIGGER_START_EVENT: {  // TriggerStartEventHandler :30-39
      if (el.start() == NO_ELEM) { I.err |= TE_FALLBACK; return; }
      s.elem = el.start();
      s.scope_key = rec.key;
      s.intent = WI_START_EVENT_OCCURRED;
      s.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE, ZB_RT_EVENT, I.nn > 0);
      s.flags = TK_WF; s.ord = (uint8_t)I.nwf++;
      s.rscope = (uint8_t)rself;
      s.rself = LN;
      I.push(s);
      break;
    }
    case ST_COMPLETE_PROCESS: {  // CompleteProcessHandler :28-35
      s.intent = WI_ELEMENT_COMPLETED;
      s.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE, ZB_RT_EVENT, I.nn > 0);
      s.rself = LN;
      I.remove(rself);
      if (rec.key == I.inst_key) I.completed += 1;  // (statistics: emit pass / trace)
      I.push(s);
      break;
    }
    default:  // message subscriptions, termination: general wave path
      I.err |= TE_FALLBACK;
      break;
  }
}

// process_record (zb_wave.hip) on local rows
template <bool EMIT, bool COND, bool UNI>
__device__ __forceinline__ void t_record(const TrajParams& P, Inst& I, const TRec& rec_in, int64_t pos,
                                         uint32_t* slot) {
  TRec rec = rec_in;
  if (UNI) {  // control fields are the same in every lane: keep them in SGPRs (scalar branches, s_load)
    rec.elem = (uint16_t)__builtin_amdgcn_readfirstlane(rec.elem);
    rec.intent = (uint8_t)__builtin_amdgcn_readfirstlane(rec.intent);
    rec.kind = (uint8_t)__builtin_amdgcn_readfirstlane(rec.kind);
    rec.rself = (uint8_t)__builtin_amdgcn_readfirstlane(rec.rself);
    rec.rscope = (uint8_t)__builtin_amdgcn_readfirstlane(rec.rscope);
    rec.flags = (uint8_t)__builtin_amdgcn_readfirstlane(rec.flags);
    rec.ord = (uint8_t)__builtin_amdgcn_readfirstlane(rec.ord);
  }
  const uint8_t vt = kind_vt(rec.kind), rt = kind_rt(rec.kind);
  if (vt == ZB_VT_WORKFLOW_INSTANCE) {
    if (rt == ZB_RT_COMMAND) {
      if (rec.intent != WI_CREATE) { I.err |= TE_FALLBACK; return; }
      // CreateWorkflowInstanceEventProcessor :233-368: key first, then resolve (done at submit)
      const uint8_t ord = (uint8_t)I.nwf++;
      TRec s = rec;
      s.ord = ord;
      if (rec.elem == NO_ELEM) {
        s.scope_key = NOK;  // written as the command position (the serializer finds the command value)
        s.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE, ZB_RT_COMMAND_REJECTION, I.nn > 0);
        s.flags = TK_INST;
        s.rself = LN; s.rscope = LN;
        I.push(s);
        return;
      }
      const int row = I.alloc();  // inserted when CREATED is processed
      if (row == LN) return;
      s.scope_key = NOK;
      s.flags = TK_WF | TK_INST;
      s.rself = (uint8_t)row; s.rscope = LN;
      s.intent = WI_CREATED;
      s.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE, ZB_RT_EVENT, I.nn > 0);
      I.push(s);
      s.intent = WI_ELEMENT_READY;
      s.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE, ZB_RT_EVENT, I.nn > 0);
      I.push(s);
    } else if (rt == ZB_RT_EVENT) {
      if (rec.intent == WI_CREATED) {  // WorkflowInstanceCreatedEventProcessor: index insert (READY)
        const int r = rec.rself;
        if (r == LN) { I.err |= TE_FALLBACK; return; }
        I.set_meta(r, rec.elem, WI_ELEMENT_READY, LN);
        I.rpay[r] = rec.payload;
        I.rkey[r] = rec.key;
        I.rjob[r] = JOB_ZERO;
        I.rnch[r] = 0;
        I.created += 1;
      } else if (rec.intent <= WI_ELEMENT_TERMINATED && rec.intent >= WI_START_EVENT_OCCURRED) {
        t_step<EMIT, COND>(P, I, rec, pos, slot);
      }
    }
  } else if (vt == ZB_VT_JOB) {
    if (rt == ZB_RT_COMMAND && rec.intent == JI_CREATE) {
      // canonical harness: JOB CREATED(k), JOB COMPLETED(k), k from the job key generator
      const uint8_t ord = (uint8_t)I.njob++;
      TRec s = rec;
      s.flags = TK_JOB; s.ord = ord;
      s.intent = JI_CREATED;
      s.kind = make_kind(ZB_VT_JOB, ZB_RT_EVENT, I.nn > 0);
      I.push(s);
      s.intent = JI_COMPLETED;
      s.kind = make_kind(ZB_VT_JOB, ZB_RT_EVENT, I.nn > 0);
      s.payload = elem_dword(P, rec.elem, 10);  // DevElem.job_payload
      I.push(s);
    } else if (rt == ZB_RT_EVENT && rec.intent == JI_CREATED) {  // JobCreatedProcessor :408-426
      if (rec.scope_key != NOK && I.alive(rec.rself)) I.rjob[rec.rself] = rec.key;
    } else if (rt == ZB_RT_EVENT && rec.intent == JI_COMPLETED) {  // JobCompletedEventProcessor :428-453
      const int r = rec.rself;
      if (!I.alive(r)) return;
      TRec s;
      s.key = rec.scope_key;
      s.scope_key = I.scope_of(r);
      s.elem = I.elem(r);
      s.payload = rec.payload;
      s.intent = WI_ELEMENT_COMPLETING;
      s.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE, ZB_RT_EVENT, I.nn > 0);
      s.rself = (uint8_t)r;
      s.rscope = I.parent(r);
      s.flags = 0; s.ord = 0;
      I.set_state(r, WI_ELEMENT_COMPLETING);
      I.rpay[r] = rec.payload;
      I.rjob[r] = NOK;
      I.push(s);
    }
  }
  // other value types (incident commands): not registered on the workflow stream processor
}

// ------------------------------------------------------------------------------ workgroup scans
__device__ __forceinline__ uint64_t tshfl_up(uint64_t v, int d) {
  return (uint64_t)__shfl_up((unsigned long long)v, d, 64);
}

// exclusive scan of (a, b) over the 256 threads of the workgroup; returns the totals in ta / tb
__device__ __forceinline__ void block_scan2(uint64_t& a, uint64_t& b, uint64_t& ta, uint64_t& tb,
                                            uint64_t (*s)[2]) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t a0 = a, b0 = b;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t ua = tshfl_up(a, d), ub = tshfl_up(b, d);
    if (lane >= d) { a += ua; b += ub; }
  }
  if (lane == 63) { s[wv][0] = a; s[wv][1] = b; }
  __syncthreads();
  ta = 0; tb = 0;
#pragma unroll
  for (int k = 0; k < TWG / 64; k++) {
    const uint64_t xa = s[k][0], xb = s[k][1];
    if (k < wv) { a += xa; b += xb; }
    ta += xa; tb += xb;
  }
  a -= a0;
  b -= b0;
  __syncthreads();  // s reused by the next call
}

// Default output merge of the documents behind refs src (job / message payload) and tgt (scope payload)
// into the blob at arena byte offset at (capacity m_len): LDS-staged flat-map fast path; a non-flat
// document sets TE_REGEN (first pass) or runs the general indexer / merger (GEN rerun).
// PK_OUT / PK_IN != 0: packed layout (inputs back to back in PK_IN words, output blob of PK_OUT words)
// tree (template emit): a pair the structural merge refuses is left to k_tmpl_xtree (*tree set, the blob unwritten)
// instead of sending the batch to the wave pipeline (TE_XTREE)
template <bool GEN, int PK_OUT = 0, int PK_IN = 0>
__device__ __forceinline__ void merge_into(const TrajParams& P, uint32_t src, uint32_t tgt, uint32_t m_len, uint64_t at,
                                           uint32_t* reg, uint32_t& err, uint32_t& ns, uint32_t& nt, uint32_t& olen,
                                           bool* tree = nullptr) {
  constexpr bool PACKED = PK_OUT != 0;
  constexpr uint32_t OUT_BYTES = PACKED ? 4 * PK_OUT : FM_BYTES;
  constexpr uint32_t OUT_OFF = PACKED ? PK_IN : 2 * FM_WORDS;
  const uint32_t* gs = (const uint32_t*)(P.arena + (uint64_t)src * 8);
  const uint32_t* gt = (const uint32_t*)(P.arena + (uint64_t)tgt * 8);
  ns = gs[0];
  nt = gt[0];
  uint32_t* gd = (uint32_t*)(P.arena + at);
  olen = 0;
  bool done = false;
  if (ns + nt + 3 <= OUT_BYTES - 4) {
    // flat fast path on LDS copies of the two documents
    const uint32_t ws = PACKED ? (ns + 7) / 4 : FM_WORDS;
    for (uint32_t k = 0; k < (ns + 7) / 4; k++) reg[k] = gs[k];
    for (uint32_t k = 0; k < (nt + 7) / 4; k++) reg[ws + k] = gt[k];
    uint8_t* lo = (uint8_t*)(reg + OUT_OFF);
    done = merge_flat((const uint8_t*)reg + 4, ns, (const uint8_t*)(reg + ws) + 4, nt, lo + 4, OUT_BYTES - 4, olen);
    if (done) {
      reg[OUT_OFF] = olen;
      for (uint32_t k = 0; k < (olen + 7) / 4; k++) gd[k] = reg[OUT_OFF + k];
    }
  } else {
    // larger flat documents: the same fast path straight on the arena
    done = merge_flat((const uint8_t*)gs + 4, ns, (const uint8_t*)gt + 4, nt, (uint8_t*)gd + 4, m_len, olen);
    if (done) gd[0] = olen;
  }
  if (!done) {
    if constexpr (GEN) {
      Out o{(uint8_t*)gd + 4, 0};
      bool unsup = false;
      const bool ok = merge_docs((const uint8_t*)gs + 4, ns, (const uint8_t*)gt + 4, nt, o, unsup);
      olen = o.n;
      if (o.n > m_len) err |= DE_UNSUPPORTED;  // (never for a document merge_docs takes: as k_merge_gen)
      // shapes the structural merge refuses: the exact tree (zb_xmerge.hpp) -- in k_tmpl_xtree after the template
      // emit (a grid of XLANE_COUNT lanes, one lane workspace each; in the emit itself a batch of 1M lanes would queue
      // for the XLANE_GROUPS lane groups: 38 ms per 1M-instance tick, profiles/r05/exact_tree_r05k.txt), or, for the
      // per-instance path, on the wave pipeline
      if (!ok || unsup) {
        if (tree) *tree = true;
        else err |= TE_XTREE;
      } else {
        gd[0] = olen;
      }
    } else {
      err |= TE_REGEN;
    }
  }
}

// inclusive scan over the 64 lanes of a wave
__device__ __forceinline__ uint64_t wave_scan(uint64_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t u = tshfl_up(v, d);
    if (lane >= d) v += u;
  }
  return v;
}

// ------------------------------------------------------------------------------ k_traj
// EMIT: emit pass (else count pass). UNI: uniform batch (see TrajParams::uni): every instance has the
// same per-generation counts, so positions and keys are affine in the instance index and the
// generation loop needs no workgroup synchronisation at all. COND: exclusive splits supported.
// GEN: the general merge (merge_docs) backs up the flat fast path; without it a non-flat merge
// makes the pass set ctl->regen and the host-side launch sequence reruns the pass with GEN.
// TRACE (count pass of a uniform batch, one instance): payload refs are symbolic (PAY_CREATE, PAY_MERGE | w,
// literal refs) so that each generation's merge gets a result bound valid for every instance of the
// batch (MergeGen); the emit pass then places instance i's result at mbase(w) + i * stride(w).
// CLS (with TRACE): class batch trace, lane c traces the representative of class c.
template <bool EMIT, bool UNI, bool COND, bool GEN, bool TRACE, bool CLS>
__global__ void __launch_bounds__(TWG) k_traj(TrajParams P) {
  __shared__ uint64_t s_scan[TWG / 64][2];
  __shared__ uint64_t s_abase;
  __shared__ uint32_t s_merge[(EMIT || COND) ? TWG * FM_STRIDE : 1];
  uint32_t* const slot = COND ? s_merge + threadIdx.x * FM_STRIDE : nullptr;  // condition documents
  TrajCtl* ctl = P.ctl;
  if (EMIT && ctl->flag) return;
  if (EMIT && GEN && !ctl->regen) return;
  const int nwg = gridDim.x;
  int64_t inst = (int64_t)blockIdx.x * TWG + threadIdx.x;
  // lanes past the batch follow lane 0's control in a uniform batch: they must not write anything
  bool active = inst < P.n;
  uint32_t cls = 0;
  if (CLS) {  // class trace: lane c traces the representative of class c
    const ClsPlan* pl = P.plan;
    const uint32_t ncls = __builtin_amdgcn_readfirstlane(pl->nc);
    cls = threadIdx.x;
    active = cls < ncls;
    inst = active ? pl->rep[cls] : 0;
  }

  Inst I;
  I.used = 0; I.to_free = 0;
  I.rkey = 0; I.rjob = 0; I.rpay = 0; I.rmeta = 0; I.rnch = 0;
  I.cur.key = 0; I.cur.sk = 0; I.cur.pay = 0; I.cur.m0 = 0; I.cur.m1 = 0;
  I.nx = I.cur;
  I.inst_key = NOK;
  I.nc = 0; I.nn = 0; I.nwf = 0; I.njob = 0;
  I.merge = false; I.detail = false; I.m_src = I.m_tgt = I.m_len = 0;
  I.d_code = I.d_a = I.d_b = 0; I.d_q = 0; I.d_pos = 0;
  I.err = 0;
  I.transitions = I.completed = I.created = I.merges = I.cond_bytes = 0;
  I.merge_bytes = 0;
  I.ckey = CLS ? P.plan->key[cls & (CLS_MAX - 1)] : 0;
  I.crow = CLS ? cls * CLS_ROW : 0;
  int64_t fpos = P.log_base + inst;  // log position of the first record of the current generation
  if ((CLS && TRACE) ? active : inst < P.n) {
    const zb_rec d = P.log[fpos];
    TRec r;
    r.key = NOK; r.scope_key = NOK; r.payload = TRACE ? PAY_CREATE : d.payload; r.elem = d.elem;  // a CREATE
    r.intent = d.intent;
    r.kind = d.kind; r.rself = LN; r.rscope = LN; r.flags = 0; r.ord = 0;
    I.cur.set(0, r);
    I.nc = 1;
  }

  int w = 0;
  const int W = UNI ? (int)P.wcount[cls] : 0;
  int wl = 0;  // generations in which this instance had records (trace)
  while (UNI ? (w < W) : __syncthreads_or(I.nc > 0)) {
    if (!UNI && w >= P.wcap) {  // more generations than the count buffers hold
      if (!EMIT && threadIdx.x == 0) atomicOr(&ctl->flag, TE_FALLBACK);
      return;
    }
    // ---- uniform batch: every lane of the wave follows the same trajectory, so the control half of the
    // state (record kinds, intents, elements, row links, row states) is the same in all lanes; read it
    // from the first lane so that the compiler keeps it in SGPRs and every branch below is scalar.
    // Per-lane data (keys, payload refs) stays in VGPRs.
    if (UNI) {
#pragma unroll
      for (int k = 0; k < TF; k++) {
        I.cur.m0[k] = __builtin_amdgcn_readfirstlane(I.cur.m0[k]);
        I.cur.m1[k] = __builtin_amdgcn_readfirstlane(I.cur.m1[k]);
      }
#pragma unroll
      for (int k = 0; k < TR; k++) {
        I.rmeta[k] = __builtin_amdgcn_readfirstlane(I.rmeta[k]);
        I.rnch[k] = __builtin_amdgcn_readfirstlane(I.rnch[k]);
      }
      I.nc = __builtin_amdgcn_readfirstlane(I.nc);
      I.used = __builtin_amdgcn_readfirstlane(I.used);
    }
    if (I.nc > 0) wl = w + 1;
    // ---- process this generation (log order inside the instance)
    int cut = 0;  // follow-ups [0, cut) come from the generation's first record, the rest from its second
#pragma unroll 1
    for (int k = 0; k < I.nc; k++) {
      t_record<EMIT, COND, UNI>(P, I, I.cur.get(k), fpos + k, slot);
      if (k == 0) cut = I.nn;
    }
    // ---- place the follow-ups
    uint64_t a = (uint64_t)I.nn | ((uint64_t)I.nwf << 16) | ((uint64_t)I.njob << 32);
    uint64_t bytes = 0;
    if (EMIT && active) bytes = (I.merge ? tblob_bytes(I.m_len) : 0) + (I.detail ? 24 : 0);
    const uint64_t a_own = a;  // (block_scan2 turns a into the exclusive prefix)
    uint64_t ta = 0, tb = 0;
    if (!UNI) block_scan2(a, bytes, ta, tb, s_scan);
    int64_t pos0;
    uint32_t kwf, kjob;  // key ordinals of this instance's first new wf / job key
    if (UNI) {
      // positions and keys are affine in the instance index; the arena is allocated per wave
      const uint64_t c = kload(P.agg, (uint64_t)w);
      const TrajBase wb = kload(P.wbase, (uint64_t)w);
      pos0 = wb.pos + inst * (int64_t)(c & 0xffff);
      kwf = (uint32_t)(wb.wf + inst * (int64_t)((c >> 16) & 0xffff));
      kjob = (uint32_t)(wb.job + inst * (int64_t)(c >> 32));
      if (EMIT && I.merge) {
        // this instance's merge slot of generation w (MergeGen: the stride bounds every instance's result)
        const MergeGen g = kload(P.mgen, (uint64_t)w);
        tb = (uint64_t)wb.mbase + (uint64_t)inst * g.stride;
        bytes = 0;
        if (!g.has || tblob_bytes(I.m_len) > g.stride) { I.err |= DE_UNSUPPORTED; tb = P.arena_cap; }
      }
    } else if (!EMIT) {
      if (TRACE) {  // one traced instance per lane (lane = class): its own counts
        if (active) P.agg[(uint64_t)I.crow + w] = a_own;
      } else if (threadIdx.x == 0) {
        P.agg[(uint64_t)w * nwg + blockIdx.x] = ta;
      }
      pos0 = 0;
      if (TRACE) {  // symbolic keys: resolved per instance by the template emit pass
        kwf = SYMK_WF | ((uint32_t)w << 4);
        kjob = SYMK_JOB | ((uint32_t)w << 4);
      } else {
        kwf = (uint32_t)((a >> 16) & 0xffff);  // placeholder ordinals: nothing in the count depends on key values
        kjob = (uint32_t)(a >> 32);
      }
    } else {
      const TrajBase wb = P.wbase[w];
      const uint4 off = P.woff[(uint64_t)w * nwg + blockIdx.x];
      pos0 = wb.pos + off.x + (int64_t)(a & 0xffff);
      kwf = (uint32_t)(wb.wf + off.y + ((a >> 16) & 0xffff));
      kjob = (uint32_t)(wb.job + off.z + (a >> 32));
      if (tb) {
        if (threadIdx.x == 0) s_abase = atomicAdd((unsigned long long*)&ctl->arena_next, (unsigned long long)tb);
        __syncthreads();
      }
    }
    uint32_t merged_ref = 0, detail_ref = 0;
    if (TRACE && active) {
      MergeGen g{0, 0, 0, 0};
      if (I.merge) {
        g.src = I.m_src; g.tgt = I.m_tgt; g.has = 1;
        const uint32_t bound = sym_bound(P, I.m_src, I.crow) + sym_bound(P, I.m_tgt, I.crow) + 8;  // emit reserves |s| + |t| + 8
        g.stride = tblob_bytes(bound);
        merged_ref = PAY_MERGE | (uint32_t)w;
        I.merges += 1;
      }
      P.mgen[I.crow + w] = g;
    }
    if (EMIT && active && (I.merge || I.detail)) {
      uint64_t at = (UNI ? tb : s_abase) + bytes;
      if (I.merge) {
        const uint32_t mb = tblob_bytes(I.m_len);
        if (at + mb > P.arena_cap) I.err |= DE_ARENA_FULL;
        else {
          uint32_t ns = 0, nt = 0, olen = 0;
          merge_into<GEN>(P, I.m_src, I.m_tgt, I.m_len, at, s_merge + threadIdx.x * FM_STRIDE, I.err, ns, nt, olen);
          merged_ref = (uint32_t)(at >> 3);
          I.merges += 1;
          I.merge_bytes += ns + nt + olen;
        }
        at += mb;
      }
      if (I.detail) {
        if (at + 24 > P.arena_cap) I.err |= DE_ARENA_FULL;
        else {
          detail_ref = (uint32_t)(at >> 3);
          uint8_t* dst = P.arena + at;
          *(uint32_t*)dst = 16;
          dst[4] = 3;  // CONDITION_ERROR
          dst[5] = I.d_code; dst[6] = I.d_a; dst[7] = I.d_b;
          *(uint16_t*)(dst + 8) = I.d_q;
          *(int64_t*)(dst + 16) = I.d_pos;
        }
      }
    }
    // keys, row inserts, log writes
#pragma unroll
    for (int k = 0; k < TF; k++) {
      if (k < I.nn) {
        TRec s = I.nx.get(k);
        if (s.flags & TK_WF) s.key = kwf + s.ord;
        if (s.flags & TK_JOB) s.key = kjob + s.ord;
        if (s.flags & TK_INST) I.inst_key = kwf + s.ord;
        if (s.flags & TK_MERGED) s.payload = merged_ref;
        if (s.flags & TK_DETAIL) s.payload = detail_ref;
        if (s.flags & TK_ROW_INIT) {
          const int r = s.rself;
          I.set_meta(r, s.elem, WI_ELEMENT_READY, s.rscope);
          I.rpay[r] = s.payload;
          I.rkey[r] = s.key;
          I.rjob[r] = JOB_ZERO;
          I.rnch[r] = 0;
        }
        if (TRACE && active) {  // the trajectory's record, symbolic
          if (s.flags & TK_DETAIL) I.err |= TE_FALLBACK;  // incidents are never templated
          TmplRec t;
          t.key = s.key;
          t.scope = kind_rt(s.kind) == ZB_RT_COMMAND_REJECTION ? SYM_CMDPOS : s.scope_key;
          t.inst = I.inst_key;
          t.payload = s.payload;
          t.elem = s.elem; t.intent = s.intent; t.kind = s.kind;
          t.pad[0] = k < cut ? 0 : 1;  // source: the instance's record of the previous generation
          t.pad[1] = t.pad[2] = 0;
          P.tmpl[((uint64_t)I.crow + w) * TF + k] = t;
          if (kind_vt(s.kind) == ZB_VT_WORKFLOW_INSTANCE && kind_rt(s.kind) == ZB_RT_EVENT) I.transitions++;
        }
        s.flags = 0;
        I.cur.set(k, s);
        if (EMIT && active) {
          zb_rec d;
          const bool job_event = kind_vt(s.kind) == ZB_VT_JOB && kind_rt(s.kind) == ZB_RT_EVENT;
          d.key = job_event ? job_key(P, s.key) : wf_key(P, s.key);
          d.scope_key = kind_rt(s.kind) == ZB_RT_COMMAND_REJECTION ? P.log_base + inst : wf_key(P, s.scope_key);
          d.inst_key = wf_key(P, I.inst_key);
          d.payload = s.payload;
          d.elem = s.elem; d.intent = s.intent; d.kind = s.kind;
          if (pos0 + k < (int64_t)P.log_cap) {
            P.log[pos0 + k] = d;
            P.srcd[pos0 + k] = (uint32_t)(pos0 + k - (fpos + (k < cut ? 0 : 1)));
            P.vlen[pos0 + k] = VLEN_UNKNOWN;
          } else I.err |= DE_LOG_FULL;
          if (kind_vt(s.kind) == ZB_VT_WORKFLOW_INSTANCE && kind_rt(s.kind) == ZB_RT_EVENT) I.transitions++;
        }
      }
    }
    fpos = pos0;
    I.nc = I.nn;
    I.nn = 0; I.nwf = 0; I.njob = 0;
    I.merge = false; I.detail = false;
    I.used &= ~I.to_free;
    I.to_free = 0;
    w++;
  }

  if (!EMIT) {
    if (TRACE) {
      if (active) {
        P.wcount[cls] = (uint32_t)wl;
        // the template emit writes no element-instance rows: every traced instance must end
#pragma unroll
        for (int k = 0; k < TR; k++)
          if (((I.used >> k) & 1) && I.alive(k)) I.err |= TE_FALLBACK;
        uint32_t* cs = P.cstat + (uint64_t)cls * TSTAT;
        cs[0] = I.transitions; cs[1] = I.completed; cs[2] = I.created; cs[3] = I.merges; cs[4] = I.cond_bytes;
      }
      if (threadIdx.x == 0) atomicMax(&ctl->wmax, (uint32_t)w);
    } else if (threadIdx.x == 0) {
      P.wcount[blockIdx.x] = (uint32_t)w;
      atomicMax(&ctl->wmax, (uint32_t)w);
    }
    if (I.err) atomicOr(&ctl->flag, TE_FALLBACK);
    return;
  }

  // ---- live element instances -> partition rows (instances stopped by an incident keep theirs)
  if (!active) I.used = 0;
  uint32_t live = 0;
#pragma unroll
  for (int k = 0; k < TR; k++)
    if (((I.used >> k) & 1) && I.alive(k)) live |= 1u << k;
  uint64_t a = (uint64_t)__builtin_popcount(live), bz = 0, ta, tb;
  block_scan2(a, bz, ta, tb, s_scan);
  if (ta) {
    if (threadIdx.x == 0) s_abase = atomicAdd((unsigned long long*)&ctl->rows_next, (unsigned long long)ta);
    __syncthreads();
    const uint64_t r0 = s_abase + a;
    u32x4 gid = NO_ROW;
    uint32_t n = 0;
#pragma unroll
    for (int k = 0; k < TR; k++)
      if ((live >> k) & 1) gid[k] = (uint32_t)(r0 + n++);
    // the children lists (RowLink.c_head / c_next): every row of the instance is this thread's, parents included
    u32x4 head = NO_ROW, next = NO_ROW;
#pragma unroll
    for (int k = 0; k < TR; k++) {
      const int par = (int)(I.rmeta[k] >> 24);
      if (((live >> k) & 1) && par != LN) {
#pragma unroll
        for (int q = 0; q < TR; q++)
          if (q == par) { next[k] = head[q]; head[q] = gid[k]; }
      }
    }
#pragma unroll
    for (int k = 0; k < TR; k++) {
      if (!((live >> k) & 1)) continue;
      if (gid[k] >= P.row_cap) { I.err |= DE_ROWS_FULL; continue; }
      const uint32_t meta = I.rmeta[k];
      const int par = (int)(meta >> 24);
      RowMeta m;
      m.payload = I.rpay[k];
      m.parent = par == LN ? NO_ROW : gid[par];
      m.elem = (uint16_t)meta;
      m.state = (uint8_t)(meta >> 16);
      m.flags = 0;
      m.nchild = I.rnch[k];
      const uint32_t jk = I.rjob[k];
      P.rmeta[gid[k]] = m;
      P.rkeys[gid[k]] = RowKeys{wf_key(P, I.rkey[k]), wf_key(P, I.scope_of(k)), wf_key(P, I.inst_key),
                                jk == JOB_ZERO ? 0 : job_key(P, jk)};
      P.rlink[gid[k]] = RowLink{head[k], next[k]};
    }
  }
  // ---- statistics
  if (!active) I.transitions = I.completed = I.created = I.merges = I.cond_bytes = 0, I.merge_bytes = 0;
  uint64_t s0 = (uint64_t)I.transitions | ((uint64_t)I.completed << 32);
  uint64_t s1 = (uint64_t)I.created | ((uint64_t)I.merges << 32);
  block_scan2(s0, s1, ta, tb, s_scan);
  uint64_t s2 = I.merge_bytes, s3 = I.cond_bytes, tc, td;
  block_scan2(s2, s3, tc, td, s_scan);
  if (threadIdx.x == 0) {  // per-workgroup partials (no same-address atomics): k_traj_commit reduces them
    uint64_t* ws = P.wstats + (uint64_t)blockIdx.x * 6;
    ws[0] = ta & 0xffffffffu; ws[1] = ta >> 32; ws[2] = tb & 0xffffffffu; ws[3] = tb >> 32; ws[4] = tc; ws[5] = td;
  }
  if (!active) I.err = 0;
  if (I.err & TE_REGEN) atomicOr(&ctl->regen, 1u);
  if (I.err & TE_XTREE) atomicOr(&ctl->flag, TE_FALLBACK);  // (nothing commits: the wave pipeline runs the batch)
  const uint32_t derr = I.err & ~(uint32_t)(TE_FALLBACK | TE_REGEN | TE_XTREE);
  if (I.err & TE_FALLBACK) atomicOr(&ctl->derr, (uint32_t)DE_PROCESSING);  // count and emit passes disagree
  if (derr) atomicOr(&ctl->derr, derr);
}

// ------------------------------------------------------------------------------ scans
// one workgroup per generation w: exclusive prefix over workgroups of agg[w][.]
__global__ void __launch_bounds__(1024) k_traj_scan(TrajParams P) {
  __shared__ uint64_t s_w[16][3];
  const TrajCtl* ctl = P.ctl;
  const uint32_t w = blockIdx.x;
  if (ctl->flag || w >= ctl->wmax) return;
  const int nwg = P.nwg;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t carry[3] = {0, 0, 0};
  for (int base = 0; base < nwg; base += 1024) {
    const int b = base + threadIdx.x;
    uint64_t v = 0;
    if (b < nwg && w < P.wcount[b]) v = P.agg[(uint64_t)w * nwg + b];
    uint64_t x[3] = {v & 0xffff, (v >> 16) & 0xffff, v >> 32};
    uint64_t ex[3];
#pragma unroll
    for (int f = 0; f < 3; f++) {
      uint64_t y = x[f];
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint64_t u = tshfl_up(y, d);
        if (lane >= d) y += u;
      }
      ex[f] = y - x[f];
      if (lane == 63) s_w[wv][f] = y;
    }
    __syncthreads();
    uint64_t tot[3] = {0, 0, 0};
#pragma unroll
    for (int f = 0; f < 3; f++) {
      for (int k = 0; k < 16; k++) {
        if (k < wv) ex[f] += s_w[k][f];
        tot[f] += s_w[k][f];
      }
      ex[f] += carry[f];
    }
    if (b < nwg) P.woff[(uint64_t)w * nwg + b] = make_uint4((uint32_t)ex[0], (uint32_t)ex[1], (uint32_t)ex[2], 0);
#pragma unroll
    for (int f = 0; f < 3; f++) carry[f] += tot[f];
    __syncthreads();
  }
  if (threadIdx.x == 0) P.wtot[w] = make_uint4((uint32_t)carry[0], (uint32_t)carry[1], (uint32_t)carry[2], 0);
}

// one workgroup: generation bases (log position of generation w+1, key generator values at w)
__global__ void __launch_bounds__(1024) k_traj_base(TrajParams P) {
  __shared__ uint64_t s_w[16][4];
  __shared__ uint64_t s_carry[4];
  TrajCtl* ctl = P.ctl;
  if (ctl->flag) return;
  const uint32_t W = ctl->wmax;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool uni = P.uni != 0 || P.cls != 0;  // per-class counts (one class: uniform batch)
  const uint32_t ncls = P.cls ? P.plan->nc : 1;
  if (threadIdx.x < 4) s_carry[threadIdx.x] = 0;
  __syncthreads();
  for (uint32_t base = 0; base < W; base += 1024) {
    const uint32_t w = base + threadIdx.x;
    uint64_t x[4] = {0, 0, 0, 0};
    if (w < W) {
      if (uni) {  // generation totals: class counts x class sizes; merge slots: stride x class size
        for (uint32_t c = 0; c < ncls; c++) {
          const uint64_t m = P.cls ? (uint64_t)P.plan->n[c] : (uint64_t)P.uni;
          const MergeGen g = P.mgen[(uint64_t)c * CLS_ROW + w];
          if (g.has) x[3] += (uint64_t)g.stride * m;
          const uint64_t a = P.agg[(uint64_t)c * CLS_ROW + w];
          x[0] += (a & 0xffff) * m; x[1] += ((a >> 16) & 0xffff) * m; x[2] += (a >> 32) * m;
        }
      } else {
        const uint4 t = P.wtot[w];
        x[0] = t.x; x[1] = t.y; x[2] = t.z;
      }
    }
    uint64_t ex[4];
#pragma unroll
    for (int f = 0; f < 4; f++) {
      uint64_t y = x[f];
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint64_t u = tshfl_up(y, d);
        if (lane >= d) y += u;
      }
      ex[f] = y - x[f];
      if (lane == 63) s_w[wv][f] = y;
    }
    __syncthreads();
    uint64_t tot[4] = {0, 0, 0, 0};
#pragma unroll
    for (int f = 0; f < 4; f++) {
      for (int k = 0; k < 16; k++) {
        if (k < wv) ex[f] += s_w[k][f];
        tot[f] += s_w[k][f];
      }
      ex[f] += s_carry[f];
    }
    if (w < W) {
      TrajBase b;
      b.pos = P.log_base + P.n + (int64_t)ex[0];
      b.wf = (int64_t)ex[1];  // key ordinals (zb_traj.hip keys are wf_start / job_start + 5 * ordinal)
      b.job = (int64_t)ex[2];
      b.mbase = (int64_t)(ctl->arena_start + ex[3]);
      P.wbase[w] = b;
    }
    __syncthreads();
    if (threadIdx.x < 4) s_carry[threadIdx.x] += tot[threadIdx.x];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (uni) ctl->arena_next = ctl->arena_start + s_carry[3];  // every merge slot of the batch
    ctl->end = P.log_base + P.n + (int64_t)s_carry[0];
    ctl->wf_next = P.wf_start + 5 * (int64_t)s_carry[1];
    ctl->job_next = P.job_start + 5 * (int64_t)s_carry[2];
    if ((uint64_t)ctl->end > P.log_cap) ctl->flag |= TE_FALLBACK;  // the wave path reports the capacity error
  }
}

// a non-flat merge stopped the first emit pass: restart the allocators and statistics for the rerun
__global__ void k_traj_regen(TrajParams P) {
  TrajCtl* ctl = P.ctl;
  if (ctl->flag || !ctl->regen) return;
  if (!P.uni && !P.cls) ctl->arena_next = ctl->arena_start;  // (uniform batch: merge slots fixed by k_traj_base)
  ctl->rows_next = ctl->rows_start;
  ctl->derr = 0;
}

constexpr int COMMIT_WG = 1024;
__global__ void __launch_bounds__(COMMIT_WG) k_traj_commit(TrajParams P) {
  __shared__ uint64_t s_st[COMMIT_WG / 64][6];
  const TrajCtl* ctl = P.ctl;
  if (ctl->flag) return;
  uint64_t st[6] = {0, 0, 0, 0, 0, 0};
  // the emit workgroups' statistics (a deferred batch's emit wrote none: every workgroup's are zero)
  if (!ctl->defer)
    for (int b = threadIdx.x; b < P.nwg_e; b += blockDim.x)
#pragma unroll
      for (int f = 0; f < 6; f++) st[f] += P.wstats[(uint64_t)b * 6 + f];
#pragma unroll
  for (int f = 0; f < 6; f++) {
    uint64_t x = st[f];
    for (int d = 32; d >= 1; d >>= 1) x += (uint64_t)__shfl_down((unsigned long long)x, d, 64);
    if ((threadIdx.x & 63) == 0) s_st[threadIdx.x >> 6][f] = x;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  for (int f = 0; f < 6; f++)
    for (int k = 0; k < COMMIT_WG / 64; k++) P.stats[f] += s_st[k][f];
  if (P.uni || P.cls) {  // template emit: per-class traced statistics x class sizes
    const uint32_t nc = P.cls ? P.plan->nc : 1;
    for (uint32_t c = 0; c < nc; c++) {
      const uint64_t m = P.cls ? (uint64_t)P.plan->n[c] : (uint64_t)P.uni;
      const uint32_t* cs = P.cstat + (uint64_t)c * TSTAT;
      P.stats[0] += m * cs[0];  // transitions
      P.stats[1] += m * cs[1];  // completed instances
      P.stats[2] += m * cs[2];  // created
      P.stats[3] += m * cs[3];  // merges
      if (P.cls) P.stats[5] += (uint64_t)cs[4] * P.plan->lensum[c];  // condition payload bytes
    }
  }
  if (ctl->derr) atomicOr(P.err, ctl->derr);
  WaveHdr h = *P.hdr;
  h.begin = h.end = h.gen_end = ctl->end;
  h.wf_next = ctl->wf_next;
  h.job_next = ctl->job_next;
  h.rows_next = (int64_t)ctl->rows_next;
  h.arena_next = (int64_t)ctl->arena_next;
  *P.hdr = h;
  P.stats[6] += ctl->wmax;
  if ((uint64_t)ctl->rows_next > P.row_cap) atomicOr(P.err, (uint32_t)DE_ROWS_FULL);
  if ((uint64_t)ctl->arena_next > P.arena_cap) atomicOr(P.err, (uint32_t)DE_ARENA_FULL);
}

// ------------------------------------------------------------------------------ class batches
// A batch whose CREATEs all address one process, in a model whose exclusive splits never read a merge
// result (zb_engine: traj_model_ok), evaluates every condition on the instance's CREATE payload, so
// the outcome of every split is fixed when the instance is created. The outcome key is the mixed-radix
// vector of the outcomes of all the model's splits (digit: index of the first true condition,
// cond_count = none -> default flow, cond_count + 1 = evaluation error); instances with equal keys
// follow the same trajectory. Each class runs like a uniform batch: one traced representative, emit
// waves holding a single class (scalar control), and positions, keys and merge slots linear in
// before_c(i), the number of class-c instances that precede instance i.
//   k_cls_classify  key of every instance (conditions on an LDS copy of the CREATE payload), key histogram
//   k_cls_plan      dense classes of the keys present (more than CLS_MAX: per-instance path)
//   k_cls_masks     per 64-instance group and class: ballot; per workgroup and class: count
//   k_cls_scan      per class: exclusive prefix of the workgroup counts
//   k_cls_perm      per group and class: instances before the group; emit slot -> instance
//   k_traj<TRACE, CLS> one lane per class: per-generation counts and merge bounds of its representative
// load_operand (zb_devlib.hpp) for the sweep below: constants and query descriptors through the scalar
// cache; only the [ROOT, MAP_KEY] fast query form (any other path -> unsupported: the batch takes the
// per-instance path, which runs the general json-path executor).
__device__ __forceinline__ bool load_operand_k(const TrajParams& P, bool is_path, uint32_t idx, const uint8_t* doc,
                                               uint32_t n, Operand& o, CondOut& out, bool& unsupported) {
  if (!is_path) {
    const DevConst c = kload(P.consts, idx);
    o.type = c.type; o.bval = c.bval; o.ival = c.ival; o.fval = c.fval; o.s = P.pool + c.str_off; o.slen = c.str_len;
    return true;
  }
  const DevQuery q = kload(P.queries, idx);
  if (!q.fast) { unsupported = true; return false; }
  const DevFilter f = kload(P.filters, q.first + 1);
  QueryResult r;
  if (!query_fast(doc, n, P.pool + f.key_off, f.key_len, r)) { unsupported = true; return false; }
  if (r.count == 0) { out.err = EC_PATH_NO_RESULT; out.q = (uint16_t)idx; return false; }
  if (r.count > 1) { out.err = EC_PATH_MULTI; out.q = (uint16_t)idx; return false; }
  Tok t;
  if (!read_tok(doc + r.pos, r.len, t)) { unsupported = true; return false; }
  o.type = t.type; o.bval = t.bval; o.ival = t.ival; o.fval = t.fval;
  o.s = doc + r.pos + t.hdr; o.slen = t.len;
  return true;
}

// The operands of every split condition in one scan of the CREATE payload: query_fast ([ROOT, MAP_KEY k]: every
// top-level value under key k) for all the model's condition keys at once. The scan (token walk, value skips,
// the container-key check) does not depend on the key, so each key's (count, first result) -- and whether the
// scan is unsupported -- is what query_fast gives for that key alone. The first result of each key is decoded
// where the walk reads it (the token load_operand reads), so the VM's path operands are register moves.
// n <= 16 bytes at p (the LDS copy of a document, any alignment) as two little-endian words, the bytes past n zero:
// five dword reads from the 4-aligned address below p and v_alignbyte, instead of a dependent read per byte
// (reads up to 19 bytes past p: the slot's padding or the next slot, masked off)
__device__ __forceinline__ void lds_words16(const uint8_t* p, uint32_t n, uint64_t& w0, uint64_t& w1) {
  const uint32_t a = (uint32_t)(uintptr_t)p & 3;
  const uint32_t* q = (const uint32_t*)(p - a);
  const uint32_t d0 = q[0], d1 = q[1], d2 = q[2], d3 = q[3], d4 = q[4];
  const uint64_t lo = (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, a) | (uint64_t)__builtin_amdgcn_alignbyte(d2, d1, a) << 32;
  const uint64_t hi = (uint64_t)__builtin_amdgcn_alignbyte(d3, d2, a) | (uint64_t)__builtin_amdgcn_alignbyte(d4, d3, a) << 32;
  w0 = n >= 8 ? lo : (lo & ((1ull << (8 * n)) - 1));
  w1 = n >= 16 ? hi : (n <= 8 ? 0ull : (hi & ((1ull << (8 * (n - 8))) - 1)));
}

struct Extract {  // per condition key: its first result, decoded
  uint32_t meta[CLS_QMAX];  // result count (saturating at 255) | token type << 8 | boolean << 16
  uint32_t sp[CLS_QMAX];    // string / binary bytes: document offset | length << 16 (the LDS copy holds <= 96 bytes)
  uint64_t num[CLS_QMAX];   // integer, or the double's bits
  bool ok;
};
__device__ __forceinline__ void extract_fast(const TrajParams& P, const uint8_t* d, uint32_t n, Extract& x) {
#pragma unroll
  for (int j = 0; j < CLS_QMAX; j++) { x.meta[j] = 0; x.sp[j] = 0; x.num[j] = 0; }
  Tok t;
  if (!read_tok(d, n, t)) { x.ok = n == 0; return; }
  x.ok = true;
  if (t.type != TT_MAP) return;  // root filter needs a container; arrays give no key matches
  uint32_t pos = t.total;
  for (uint32_t i = 0; i < t.len; i++) {
    Tok k, v;
    if (pos >= n || !read_tok(d + pos, n - pos, k)) { x.ok = false; return; }
    const uint32_t kpos = pos;
    pos += k.total;
    // the value: its first token (the operand's token), then the rest of a container
    if (pos >= n || !read_tok(d + pos, n - pos, v)) { x.ok = false; return; }
    const uint32_t vend = (v.type == TT_MAP || v.type == TT_ARRAY) ? skip_value(d, n, pos) : pos + v.total;
    if (vend == 0xffffffffu) { x.ok = false; return; }
    if (k.type == TT_STRING) {
      // the key's bytes as two words (keys of at most 16 bytes; longer ones byte by byte against the pool)
      uint64_t kw0 = 0, kw1 = 0;
      if (k.len <= 16) lds_words16(d + kpos + k.hdr, k.len, kw0, kw1);
#pragma unroll
      for (int j = 0; j < CLS_QMAX; j++) {
        if (j < P.cls_nq && k.len == P.cls_key_len[j] &&
            (k.len <= 16 ? (kw0 == P.cls_key_w[j][0] && kw1 == P.cls_key_w[j][1])
                         : bytes_eq(d + kpos + k.hdr, P.pool + P.cls_key_off[j], k.len))) {
          const uint32_t c = x.meta[j] & 255;
          if (c == 0) {
            x.meta[j] = (uint32_t)v.type << 8 | (v.bval ? 1u : 0u) << 16;
            x.sp[j] = (pos + v.hdr) | v.len << 16;
            x.num[j] = v.type == TT_FLOAT ? (uint64_t)__double_as_longlong(v.fval) : (uint64_t)v.ival;
          }
          x.meta[j] = (x.meta[j] & ~255u) | (c < 255 ? c + 1 : 255);
        }
      }
    } else if (k.type == TT_MAP || k.type == TT_ARRAY) {
      x.ok = false;  // container map keys: the reference's traversal would descend; not supported here
      return;
    }
    pos = vend;
  }
}
// load_operand_k with the query results taken from the extraction: a path operand names its extraction slot
// (P.cls_code), a wave-uniform index
__device__ __forceinline__ bool load_operand_x(const TrajParams& P, bool is_path, uint32_t idx, const uint8_t* doc,
                                               const Extract& x, Operand& o, CondOut& out, bool& unsupported) {
  if (!is_path) {
    const DevConst c = kload(P.consts, idx);
    o.type = c.type; o.bval = c.bval; o.ival = c.ival; o.fval = c.fval; o.s = P.pool + c.str_off; o.slen = c.str_len;
    return true;
  }
  if (!x.ok) { unsupported = true; return false; }
  const uint32_t j = __builtin_amdgcn_readfirstlane(idx);
  uint32_t meta = 0, sp = 0;
  uint64_t num = 0;
#pragma unroll
  for (int jj = 0; jj < CLS_QMAX; jj++)  // (a scalar compare: no dynamically indexed register array)
    if ((uint32_t)jj == j) { meta = x.meta[jj]; sp = x.sp[jj]; num = x.num[jj]; }
  const uint32_t cnt = meta & 255;
  if (cnt == 0) { out.err = EC_PATH_NO_RESULT; out.q = (uint16_t)j; return false; }
  if (cnt > 1) { out.err = EC_PATH_MULTI; out.q = (uint16_t)j; return false; }
  o.type = (uint8_t)(meta >> 8);
  o.bval = (meta >> 16) & 1;
  o.ival = (int64_t)num;
  o.fval = __longlong_as_double((long long)num);
  o.s = doc + (sp & 0xffff);
  o.slen = sp >> 16;
  return true;
}

// a string operand's bytes (<= 16) as two words: a path operand from the document's LDS copy, a constant from the
// deploy-time table
__device__ __forceinline__ void str_words(const TrajParams& P, bool is_path, uint32_t idx, const Operand& o,
                                          uint64_t& w0, uint64_t& w1) {
  if (is_path) {
    lds_words16(o.s, o.slen, w0, w1);
  } else {
    w0 = K(P.const_w)[2 * (uint64_t)idx];
    w1 = K(P.const_w)[2 * (uint64_t)idx + 1];
  }
}

// One comparison of the json-el VM (eval_condition, zb_devlib.hpp) on the extraction (EXT) or the document: 0 false,
// 1 true, 2 an error (out / unsupported say which), with eval_condition's operand loading and type rules.
template <bool EXT>
__device__ __forceinline__ int eval_atom(const TrajParams& P, uint32_t w0, uint32_t w1, const uint8_t* doc, uint32_t n,
                                         const Extract& ext, CondOut& out, bool& unsupported) {
  const uint32_t op = (w0 >> 8) & 0xf;
  Operand x, y;
  const bool lx = EXT ? load_operand_x(P, (w0 >> 12) & 1, w1 & 0xffff, doc, ext, x, out, unsupported)
                      : load_operand_k(P, (w0 >> 12) & 1, w1 & 0xffff, doc, n, x, out, unsupported);
  const bool ly = lx && (EXT ? load_operand_x(P, (w0 >> 13) & 1, w1 >> 16, doc, ext, y, out, unsupported)
                             : load_operand_k(P, (w0 >> 13) & 1, w1 >> 16, doc, n, y, out, unsupported));
  if (!lx || !ly) return 2;
  bool r;
  if (op == OP_EQ || op == OP_NE) {
    bool eq = false;
    if (x.type == TT_NIL) eq = y.type == TT_NIL;
    else if (y.type == TT_NIL) eq = false;
    else {
      if (!same_type(x, y, out)) return 2;
      switch (x.type) {
        case TT_STRING:
          if (EXT && x.slen == y.slen && x.slen <= 16) {  // as words: a path operand's bytes from the LDS document,
            uint64_t a0, a1, b0, b1;                       // a constant's precomputed
            str_words(P, (w0 >> 12) & 1, w1 & 0xffff, x, a0, a1);
            str_words(P, (w0 >> 13) & 1, w1 >> 16, y, b0, b1);
            eq = a0 == b0 && a1 == b1;
          } else {
            eq = x.slen == y.slen && bytes_eq(x.s, y.s, x.slen);
          }
          break;
        case TT_BOOLEAN: eq = x.bval == y.bval; break;
        case TT_INTEGER: eq = x.ival == y.ival; break;
        case TT_FLOAT: eq = x.fval == y.fval; break;
        default: out.err = EC_CMP_TYPE; out.a = x.type; return 2;
      }
    }
    r = (op == OP_EQ) ? eq : !eq;
  } else {
    if (!same_type(x, y, out)) return 2;
    if (x.type != TT_INTEGER && x.type != TT_FLOAT) { out.err = EC_NOT_NUMBER; out.a = x.type; return 2; }
    if (x.type == TT_INTEGER) {
      r = op == OP_LT ? x.ival < y.ival : op == OP_LE ? x.ival <= y.ival : op == OP_GT ? x.ival > y.ival
                                                                                     : x.ival >= y.ival;
    } else {
      r = op == OP_LT ? x.fval < y.fval : op == OP_LE ? x.fval <= y.fval : op == OP_GT ? x.fval > y.fval
                                                                                     : x.fval >= y.fval;
    }
  }
  return r ? 1 : 0;
}

// The json-el VM (eval_condition, zb_devlib.hpp) as one wave-uniform sweep over the program: every lane
// runs the same program and its jumps only go forward (zb_model.cpp emit), so instruction pc is
// fetched once per wave through the scalar cache and executed by the lanes whose own pc is there.
// Same results, errors and short-circuit behaviour as eval_condition.
template <bool EXT>
__device__ __forceinline__ bool eval_condition_sweep(const TrajParams& P, uint32_t pc0, const uint8_t* doc, uint32_t n,
                                                     const Extract& ext, CondOut& out, bool& unsupported) {
  bool r = false, done = false;
  uint32_t mine = pc0;
  out.err = 0;
  const uint32_t* code = EXT ? P.cls_code : P.code;
  for (uint32_t pc = pc0; pc < pc0 + 4096; pc++) {
    const uint32_t w0 = K(code)[2 * pc], w1 = K(code)[2 * pc + 1];
    const uint32_t opc = w0 & 0xff;
    if (opc == PC_END) return done ? false : r;
    if (done || mine != pc) continue;
    if (opc == PC_JF || opc == PC_JT) {
      mine = (opc == PC_JF ? !r : r) ? (w0 >> 16) : pc + 1;
      continue;
    }
    mine = pc + 1;
    const int o = eval_atom<EXT>(P, w0, w1, doc, n, ext, out, unsupported);
    if (o == 2) {
      done = true;
      continue;
    }
    r = o == 1;
  }
  unsupported = true;
  return false;
}

// outcome key of one CREATE payload: every split of the model, digit = first true condition / none / error
template <bool EXT>
__device__ __forceinline__ uint32_t outcome_key(const TrajParams& P, const uint8_t* doc, uint32_t len) {
  Extract ext;
  if (EXT) extract_fast(P, doc, len, ext);
  if (EXT && P.cls_natoms) {  // the outcome table: every comparison once, then one lookup
    // (the comparisons' code words all loaded up front: one scalar load round trip, not one per comparison)
    const int na = P.cls_natoms;
    uint32_t aw[2 * CLS_TABLE_ATOMS];
#pragma unroll
    for (int a = 0; a < 2 * CLS_TABLE_ATOMS; a++) aw[a] = a < 2 * na ? K(P.cls_atom_w)[a] : 0u;
    uint32_t idx = 0, mul = 1;
#pragma unroll
    for (int a = 0; a < CLS_TABLE_ATOMS; a++) {
      if (a >= na) break;
      CondOut co{0, 0, 0, 0};
      bool unsup = false;
      idx += (uint32_t)eval_atom<true>(P, aw[2 * a], aw[2 * a + 1], doc, len, ext, co, unsup) * mul;
      mul *= 3;
    }
    return P.cls_table[idx];
  }
  uint32_t key = 0;
  for (int k = 0; k < P.nsplits; k++) {
    const ElemCtl el = elem_ctl(P, P.split_elem[k]);
    const uint32_t cc = el.cond_count();
    uint32_t o = cc;
    for (uint32_t c = 0; c < cc; c++) {
      CondOut co{0, 0, 0, 0};
      bool unsup = false;
      const uint16_t flow = K(P.cond_flows)[el.cond_begin() + c];
      const uint32_t prog = K(P.elems)[flow].cond_prog;
      const bool res = eval_condition_sweep<EXT>(P, prog, doc, len, ext, co, unsup);
      if (unsup || co.err) { o = cc + 1; break; }
      if (res) { o = c; break; }
    }
    key += o * P.split_stride[k];
  }
  return key;
}

// classify: per-thread document slot [u32 len][document], an odd stride in words: 25 (documents <= 92 bytes) or, when
// every staged CREATE payload fits 44 bytes (P.max_create; C3's are <= 38), 13 -- the slots are what bounds the
// occupancy (25: 5 workgroups per CU by LDS, 13: 8, at 64 VGPRs), and the kernel is latency-bound on its two dependent
// loads per instance.
// INJ: the batch's injection (k_inject's per-record work: descriptor, links, source, value length, CREATE ref) in the
// same thread, which then classifies from the ref it just computed -- the stores of the injection overlap the loads of
// the classification, and the ref is not written and read back (the documents are in place: no staged bytes to copy)
template <int CL_STRIDE, bool INJ>
__global__ void __launch_bounds__(TWG) k_cls_classify(TrajParams P, InjectParams I) {
  __shared__ uint32_t s_doc[TWG * CL_STRIDE];
  __shared__ uint32_t s_hist[256], s_rep[256];
  __shared__ unsigned long long s_len[256];
  const int t = threadIdx.x;
  s_hist[t] = 0;
  s_rep[t] = 0xffffffffu;
  s_len[t] = 0;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * TWG + t;
  uint32_t mkey = 0, mlen = 0;
  if (i < P.n) {
    uint32_t ref;
    if (INJ) {
      zb_rec d = I.staged[i];
      d.payload += (uint32_t)(I.arena_base >> 3);
      if (d.key == KEY_IS_POSITION) d.key = I.log_base + i;
      I.log[I.log_base + i] = d;
      I.links[I.log_base + i] = ~0ull;  // no rows yet
      I.srcd[I.log_base + i] = 0;       // written by another writer (client API, job processor, ...)
      I.vlen[I.log_base + i] = I.staged_vlen[i];
      I.cref[i] = d.payload;
      ref = d.payload;
    } else {
      ref = P.cref ? P.cref[i] : P.log[P.log_base + i].payload;
    }
    const uint8_t* pp = P.arena + (uint64_t)ref * 8;
    const uint32_t len = *(const uint32_t*)pp;
    // the VM inlined on the LDS copy (LDS loads per token); a document too large for the copy gets the
    // error outcome at every split (its class, when it reaches one, sends the batch to the per-instance path)
    uint32_t key = 0;
    if (((len + 11) & ~7u) <= CL_STRIDE * 4) {  // (stage_copy writes whole 8-byte words)
      stage_copy(pp, len, s_doc + t * CL_STRIDE);
      const uint8_t* doc = (const uint8_t*)(s_doc + t * CL_STRIDE) + 4;
      key = P.cls_nq ? outcome_key<true>(P, doc, len) : outcome_key<false>(P, doc, len);
    } else {
      for (int k = 0; k < P.nsplits; k++) key += (elem_ctl(P, P.split_elem[k]).cond_count() + 1) * P.split_stride[k];
    }
    P.ikey[i] = (uint8_t)key;
    P.clen[i] = len;  // (the template drain's size pass reads 4 bytes per instance instead of two dependent loads)
    mkey = key & 255;
    mlen = len;
  }
  // key histogram: one leader per distinct key of the wave adds the wave's count, first instance and payload
  // bytes (LDS atomics of 64 lanes on a few addresses serialize)
  uint64_t act = __ballot(i < P.n);
  while (act) {
    const int l = __ffsll((unsigned long long)act) - 1;
    const uint32_t k0 = __shfl(mkey, l, 64);
    const bool in = i < P.n && mkey == k0;
    const uint64_t m = __ballot(in);
    unsigned long long y = in ? (unsigned long long)mlen : 0ull;
    for (int d = 32; d >= 1; d >>= 1) y += __shfl_xor(y, d, 64);
    if ((t & 63) == l) {  // (the first lane of the key: the smallest instance)
      atomicAdd(&s_hist[k0], (uint32_t)__builtin_popcountll(m));
      atomicMin(&s_rep[k0], (uint32_t)i);
      atomicAdd(&s_len[k0], y);
    }
    act &= ~m;
  }
  __syncthreads();
  if (s_hist[t]) {
    // banked: same-address atomics from every workgroup would serialize at the memory side
    const uint32_t hb = (blockIdx.x % CLS_HB) * 256 + t;
    atomicAdd(&P.khist[hb], s_hist[t]);
    atomicMin(&P.krep[hb], s_rep[t]);
    atomicAdd((unsigned long long*)&P.klen[hb], s_len[t]);
  }
}

__global__ void __launch_bounds__(256) k_cls_plan(TrajParams P) {
  __shared__ uint32_t s_w[4];
  ClsPlan* pl = P.plan;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  uint32_t cnt = 0, rep = 0xffffffffu;
  uint64_t lsum = 0;
  for (int b = 0; b < CLS_HB; b++) {
    cnt += P.khist[b * 256 + t];
    rep = min(rep, P.krep[b * 256 + t]);
    lsum += P.klen[b * 256 + t];
    // the banks back to their empty state for the next batch (allocated empty: grow_class_buffers; only k_cls_classify
    // adds to them, and this launch follows it in every class run)
    P.khist[b * 256 + t] = 0;
    P.krep[b * 256 + t] = 0xffffffffu;
    P.klen[b * 256 + t] = 0;
  }
  const uint64_t m = __ballot(cnt > 0);
  if (lane == 0) s_w[wv] = (uint32_t)__builtin_popcountll(m);
  __syncthreads();
  uint32_t cid = (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1));
  for (int k = 0; k < wv; k++) cid += s_w[k];
  const uint32_t nc = s_w[0] + s_w[1] + s_w[2] + s_w[3];
  pl->cid[t] = (cnt > 0 && cid < CLS_MAX) ? (uint8_t)cid : 0xff;
  if (cnt > 0 && cid < CLS_MAX) {
    pl->key[cid] = (uint32_t)t;
    pl->n[cid] = cnt;
    pl->rep[cid] = rep;
    pl->lensum[cid] = lsum;
  }
  __syncthreads();
  if (t == 0) {
    if (nc == 0 || nc > CLS_MAX) {
      atomicOr(&P.ctl->flag, TE_FALLBACK);
      pl->nc = 0;
      return;
    }
    pl->nc = nc;
  }
}

__global__ void __launch_bounds__(TWG) k_cls_masks(TrajParams P) {
  __shared__ uint32_t s_cnt[TWG / 64][CLS_MAX];
  if (P.ctl->flag) return;
  const ClsPlan* pl = P.plan;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint32_t nc = __builtin_amdgcn_readfirstlane(pl->nc);
  const int64_t i = (int64_t)blockIdx.x * TWG + t;
  const uint32_t c = i < P.n ? pl->cid[P.ikey[i]] : 0xffu;
  const uint64_t grp = ((uint64_t)blockIdx.x * (TWG / 64) + wv) * CLS_MAX;
  // (the template drain's size formula: per class the CREATE payloads' binary lengths and byte counts)
  // (32-bit DPP sums: a deferred batch's values fit the drain's 11 KB wave image, so a wave's sum is below 2^20; a
  // batch that does not fit leaves the template drain, whatever these say)
  const uint32_t cl = i < P.n ? P.clen[i] : 0u;
  const uint32_t bl = mp_bin_len(cl);
  for (uint32_t k = 0; k < nc; k++) {
    const uint64_t m = __ballot(c == k);
    const uint32_t g = wave_incl_scan(c == k ? bl : 0u), q = wave_incl_scan(c == k ? cl : 0u);
    if (lane == 63) {
      P.cg[2 * (grp + k)] = g;
      P.cg[2 * (grp + k) + 1] = q;
    }
    if (lane == 0) {
      P.cmask[grp + k] = m;
      s_cnt[wv][k] = (uint32_t)__builtin_popcountll(m);
    }
  }
  __syncthreads();
  if ((uint32_t)t < nc) {
    uint32_t sum = 0;
    for (int v = 0; v < TWG / 64; v++) sum += s_cnt[v][t];
    P.wgcnt[(uint64_t)t * P.nwg + blockIdx.x] = sum;
  }
}

// one workgroup per class: exclusive prefix over workgroups of wgcnt[c][.]
__global__ void __launch_bounds__(1024) k_cls_scan(TrajParams P) {
  __shared__ uint32_t s_w[16];
  const uint32_t c = blockIdx.x;
  if (P.ctl->flag || c >= P.plan->nc) return;
  const int nwg = P.nwg;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t carry = 0;
  const uint32_t* in = P.wgcnt + (uint64_t)c * nwg;
  uint32_t* out = P.wgoff + (uint64_t)c * nwg;
  for (int base = 0; base < nwg; base += 1024) {
    const int b = base + threadIdx.x;
    const uint32_t x = b < nwg ? in[b] : 0;
    uint32_t y = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t u = __shfl_up(y, d, 64);
      if (lane >= d) y += u;
    }
    if (lane == 63) s_w[wv] = y;
    __syncthreads();
    uint32_t ex = y - x + carry, tot = 0;
    for (int k = 0; k < 16; k++) {
      if (k < wv) ex += s_w[k];
      tot += s_w[k];
    }
    if (b < nwg) out[b] = ex;
    carry += tot;
    __syncthreads();
  }
}

__global__ void __launch_bounds__(TWG) k_cls_perm(TrajParams P) {
  if (P.ctl->flag) return;
  const ClsPlan* pl = P.plan;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint32_t nc = __builtin_amdgcn_readfirstlane(pl->nc);
  const uint64_t grp0 = (uint64_t)blockIdx.x * (TWG / 64) * CLS_MAX;
  const uint64_t grp = grp0 + (uint64_t)wv * CLS_MAX;
  const int64_t i = (int64_t)blockIdx.x * TWG + t;
  const uint32_t c = i < P.n ? pl->cid[P.ikey[i]] : 0xffu;
  uint32_t mine = 0;
  for (uint32_t k = 0; k < nc; k++) {
    uint32_t off = P.wgoff[(uint64_t)k * P.nwg + blockIdx.x];
    for (int v = 0; v < wv; v++) off += (uint32_t)__builtin_popcountll(P.cmask[grp0 + (uint64_t)v * CLS_MAX + k]);
    if (lane == 0) P.woffw[grp + k] = off;
    if (k == c) mine = off + (uint32_t)__builtin_popcountll(P.cmask[grp + k] & ((1ull << lane) - 1));
  }
  if (c < nc) {  // slot in the (block, class) segment: rank among the block's class-c instances
    const uint32_t blk = blockIdx.x / CLS_BLK_WG;
    const uint32_t first = P.wgoff[(uint64_t)c * P.nwg + (uint64_t)blk * CLS_BLK_WG];
    P.perm[P.segs[(uint64_t)blk * CLS_MAX + c] + mine - first] = (uint32_t)i;
  }
}

// Emit slots are laid out block by block (CLS_BLK_WG instance workgroups), and inside a block class by
// class, each (block, class) segment padded to whole waves: a wave holds one class, and the waves that
// write one region of the log run close together in time (k_tmpl maps blocks to XCDs contiguously).
// One workgroup: exclusive prefix of the padded segment sizes; class of every emit wave.
__global__ void __launch_bounds__(1024) k_cls_segs(TrajParams P) {
  __shared__ uint32_t s_w[16];
  ClsPlan* pl = P.plan;
  if (P.ctl->flag) return;
  const uint32_t nc = pl->nc, nwg = (uint32_t)P.nwg;
  const uint32_t E = (uint32_t)P.nblk * nc;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t carry = 0;
  for (uint32_t base = 0; base < E; base += 1024) {
    const uint32_t e = base + threadIdx.x;
    uint32_t x = 0, b = 0, c = 0;
    if (e < E) {
      b = e / nc;
      c = e % nc;
      const uint32_t w0 = b * CLS_BLK_WG, w1 = w0 + CLS_BLK_WG;
      const uint32_t lo = P.wgoff[(uint64_t)c * nwg + w0];
      const uint32_t hi = w1 < nwg ? P.wgoff[(uint64_t)c * nwg + w1] : pl->n[c];
      x = (hi - lo + 63) & ~63u;
    }
    uint32_t y = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t u = __shfl_up(y, d, 64);
      if (lane >= d) y += u;
    }
    if (lane == 63) s_w[wv] = y;
    __syncthreads();
    uint32_t ex = y - x + carry, tot = 0;
    for (int k = 0; k < 16; k++) {
      if (k < wv) ex += s_w[k];
      tot += s_w[k];
    }
    if (e < E) {
      P.segs[(uint64_t)b * CLS_MAX + c] = ex;
      for (uint32_t j = 0; j < x / 64; j++) P.wcls[ex / 64 + j] = c;
    }
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) pl->slots = carry;
}

// ------------------------------------------------------------------------------ template emit
template <bool CLS, bool GEN>
__global__ void __launch_bounds__(TWG) k_tmpl(TrajParams P) {
  using TL = TmLayout<CLS>;
  __shared__ uint32_t s_merge[TWG * TL::STRIDE];
  __shared__ uint64_t s_scan[TWG / 64][2];
  TrajCtl* ctl = P.ctl;
  if (ctl->flag) return;
  if (GEN && !ctl->regen) return;
  if (ctl->defer && !P.materialize) {  // deferred batch (zb_tdrain.hip): no descriptors now, no merge bytes
    if (threadIdx.x < 6) P.wstats[(uint64_t)blockIdx.x * 6 + threadIdx.x] = 0;
    return;
  }
  int64_t inst = (int64_t)blockIdx.x * TWG + threadIdx.x;
  bool active = inst < P.n;
  uint32_t cls = 0;
  TmplLane L;
  L.ncls = 1;
  if (CLS) {
    const ClsPlan* pl = P.plan;
    L.ncls = __builtin_amdgcn_readfirstlane(pl->nc);
    // XCD-aware: workgroups are dispatched round-robin over the 8 XCDs; give each XCD a contiguous
    // range of emit slots (blocks), so that the partial lines of one log region meet in one L2
    const uint32_t G = gridDim.x;  // a multiple of 8
    const uint32_t lwg = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
    const uint32_t sl = lwg * TWG + threadIdx.x;
    const uint32_t slots = __builtin_amdgcn_readfirstlane(pl->slots);
    uint32_t pi = 0xffffffffu;
    cls = 0;
    if (__builtin_amdgcn_readfirstlane(sl) < slots) {  // (slots come in whole waves)
      cls = __builtin_amdgcn_readfirstlane(P.wcls[sl >> 6]);
      pi = P.perm[sl];
    }
    active = pi != 0xffffffffu;
    const uint32_t p0 = __builtin_amdgcn_readfirstlane(pi);  // lane 0 of a segment wave is never padding
    inst = active ? pi : (p0 != 0xffffffffu ? p0 : pl->rep[0]);
    const uint64_t grp = (uint64_t)(inst >> 6) * CLS_MAX;
    const uint64_t lt = (1ull << (inst & 63)) - 1;
#pragma unroll
    for (int c = 0; c < CLS_MAX; c++)
      L.before[c] = c < (int)L.ncls ? P.woffw[grp + c] + (uint32_t)__builtin_popcountll(P.cmask[grp + c] & lt) : 0;
  } else {
    if (!active) inst = 0;  // (follows instance 0, writes nothing)
#pragma unroll
    for (int c = 0; c < CLS_MAX; c++) L.before[c] = c == 0 ? (uint32_t)inst : 0;
  }
  const uint32_t crow = cls * CLS_ROW;
  const int W = (int)P.wcount[cls];
  const uint32_t create_ref = P.log[P.log_base + inst].payload;
  uint32_t err = 0;
  uint64_t merge_bytes = 0;
  uint32_t pc_sym = PAY_CREATE, pc_ref = create_ref;  // last resolved payload symbol
  // payload lengths for the value lengths (vlen): the CREATE payload's is read once per instance
  const uint32_t create_len = arena_len(P.arena, create_ref);
  uint32_t pc_len = create_len;
  uint32_t* reg = s_merge + threadIdx.x * TL::STRIDE;
  int64_t prev0 = P.log_base + inst;  // the instance's first record of the previous generation (the CREATE)
  int xg = 0x7fffffff;  // the first generation whose merge k_tmpl_xtree finishes (every later merge of it too)

#pragma unroll 1
  for (int w = 0; w < W; w++) {
    const TrajBase wb = kload(P.wbase, (uint64_t)w);
    int64_t po = 0, pw = 0, pj = 0;
#pragma unroll
    for (int c = 0; c < CLS_MAX; c++) {
      if (c >= (int)L.ncls) break;
      const uint64_t n = kload(P.agg, (uint64_t)c * CLS_ROW + w);
      po += (int64_t)L.before[c] * (int64_t)(n & 0xffff);
      pw += (int64_t)L.before[c] * (int64_t)((n >> 16) & 0xffff);
      pj += (int64_t)L.before[c] * (int64_t)(n >> 32);
    }
    const int64_t pos0 = wb.pos + po, kwf = wb.wf + pw, kjob = wb.job + pj;
    const uint32_t nrec = (uint32_t)(kload(P.agg, (uint64_t)crow + w) & 0xffff);
    // this generation's merge: source / target resolved, result into the instance's slot
    const MergeGen g = kload(P.mgen, (uint64_t)crow + w);
    uint32_t merged_ref = 0, merged_len = 0;
    if (g.has) {
      uint32_t src = g.src, tgt = g.tgt;
      if (src == PAY_CREATE) src = create_ref;
      else if (src & PAY_MERGE) src = (uint32_t)(tmpl_mslot(P, L, src & 0xffff) >> 3);
      if (tgt == pc_sym) tgt = pc_ref;
      else if (tgt == PAY_CREATE) tgt = create_ref;
      else if (tgt & PAY_MERGE) tgt = (uint32_t)(tmpl_mslot(P, L, tgt & 0xffff) >> 3);
      const uint64_t at = tmpl_mslot(P, L, (uint32_t)w);
      merged_ref = (uint32_t)(at >> 3);
      merged_len = 0;
      if (active && w > xg) {  // (a pending chain: k_tmpl_xtree merges it, in order)
        merged_len = VLEN_UNKNOWN;
      } else if (active) {
        const uint32_t m_len = arena_len(P.arena, src) + arena_len(P.arena, tgt) + 8;
        if (tblob_bytes(m_len) > g.stride) err |= DE_UNSUPPORTED;
        else if (at + g.stride > P.arena_cap) err |= DE_ARENA_FULL;
        else {
          uint32_t ns = 0, nt = 0, olen = 0;
          bool tree = false;
          merge_into<GEN, TL::OUT_WORDS, TL::IN_WORDS>(P, src, tgt, m_len, at, reg, err, ns, nt, olen,
                                                        P.xq ? &tree : nullptr);
          if (tree) {
            xg = w;
            merged_len = VLEN_UNKNOWN;
            P.xq[atomicAdd(&ctl->xq_n, 1u)] = (uint64_t)inst | (uint64_t)w << 40;
          } else {
            merge_bytes += ns + nt + olen;
            merged_len = olen;
          }
        }
      }
    }
#pragma unroll 1
    for (uint32_t k = 0; k < nrec; k++) {
      const TmplRec t = kload(P.tmpl, ((uint64_t)crow + w) * TF + k);
      zb_rec d;
      d.key = tmpl_key(P, L, t.key, (uint32_t)w, kwf, kjob);
      d.scope_key = t.scope == SYM_CMDPOS ? P.log_base + inst : tmpl_key(P, L, t.scope, (uint32_t)w, kwf, kjob);
      d.inst_key = tmpl_key(P, L, t.inst, (uint32_t)w, kwf, kjob);
      uint32_t pay = t.payload, plen;
      if (pay == (PAY_MERGE | (uint32_t)w)) { pay = merged_ref; plen = merged_len; }
      else if (pay == pc_sym) { pay = pc_ref; plen = pc_len; }
      else if (pay == PAY_CREATE) { pay = create_ref; plen = create_len; }
      else if (pay & PAY_MERGE) {
        const uint32_t r = (uint32_t)(tmpl_mslot(P, L, pay & 0xffff) >> 3);
        const bool pend = (int)(pay & 0xffff) >= xg;  // (k_tmpl_xtree writes it: no length yet)
        plen = (active && !pend) ? arena_len(P.arena, r) : (pend ? VLEN_UNKNOWN : 0);
        pc_sym = pay;
        pc_ref = r;
        pc_len = plen;
        pay = r;
      } else {
        plen = arena_len(P.arena, pay);  // a static blob (shared by every instance: cached)
      }
      if (t.payload & PAY_MERGE) { pc_sym = t.payload; pc_ref = pay; pc_len = plen; }
      d.payload = pay;
      d.elem = t.elem; d.intent = t.intent; d.kind = t.kind;
      if (active) {
        if (pos0 + k < (int64_t)P.log_cap) {
          P.log[pos0 + k] = d;
          P.srcd[pos0 + k] = (uint32_t)(pos0 + k - (prev0 + t.pad[0]));
          // the value's length (zb_serialize.hip encode_value) from the element's constants and the variable fields
          // (a pending merge result's length is not known yet: the drain's size pass measures it)
          const uint8_t vt = kind_vt(d.kind), rt = kind_rt(d.kind);
          uint32_t vl = VLEN_UNKNOWN;
          if (plen != VLEN_UNKNOWN && !(d.kind & KIND_RAW) && ((vt == ZB_VT_WORKFLOW_INSTANCE && rt == ZB_RT_EVENT) ||
                                                              (vt == ZB_VT_JOB && (d.intent | 1) != JI_CANCELED))) {
            const ValueConst vc = kload(P.vconst, (uint64_t)d.elem);
            vl = (vt == ZB_VT_JOB ? vc.job : vc.wf) + mp_int_len(d.inst_key) + mp_int_len(d.scope_key) + mp_bin_len(plen);
          }
          P.vlen[pos0 + k] = vl;
        } else err |= DE_LOG_FULL;
      }
    }
    prev0 = pos0;
  }
  // statistics: everything but the merge bytes is a per-class constant (k_traj_commit)
  uint64_t s0 = active ? merge_bytes : 0, s1 = 0, t0, t1;
  block_scan2(s0, s1, t0, t1, s_scan);
  if (threadIdx.x == 0) {
    uint64_t* ws = P.wstats + (uint64_t)blockIdx.x * 6;
    ws[0] = ws[1] = ws[2] = ws[3] = ws[5] = 0;
    ws[4] = t0;
  }
  if (!active) err = 0;
  if (err & TE_REGEN) atomicOr(&ctl->regen, 1u);
  if (err & TE_XTREE) atomicOr(&ctl->flag, TE_FALLBACK);  // (nothing commits: the wave pipeline runs the batch)
  const uint32_t derr = err & ~(uint32_t)(TE_FALLBACK | TE_REGEN | TE_XTREE);
  if (derr) atomicOr(&ctl->derr, derr);
}

// Class batches in instance order (the default): lane = instance, as the log orders them, each lane
// following its own class's trace (the loops run to the wave's longest class; lanes of other classes are
// masked). In generation w the wave's 64 instances own ONE contiguous log range (pos0(i + 1) = pos0(i) +
// records of i), so each lane stages its descriptors / source deltas / value lengths in the wave's slice of
// the merge workspace and the wave writes the range out with whole-line 16-byte stores. The class-uniform
// emit (k_tmpl<true>, class-uniform order) wrote each record from its own lane: a wave's lanes sit among the
// other classes' instances, every store instruction touched ~64 partly written lines, and the L2 write
// requests, not HBM, bounded the launch (profiles/r02/tmpl_store_exp.txt).
template <bool GEN>
__global__ void __launch_bounds__(TWG) k_tmpl_io(TrajParams P) {
  using TL = TmLayout<true>;
  static_assert(64 * TL::STRIDE * 4 >= 64 * TF * (32 + 4 + 4), "staging fits the wave's merge workspace");
  __shared__ uint32_t s_merge[TWG * TL::STRIDE];
  __shared__ uint64_t s_scan[TWG / 64][2];
  TrajCtl* ctl = P.ctl;
  if (ctl->flag) return;
  if (GEN && !ctl->regen) return;
  if (ctl->defer && !P.materialize) {  // deferred batch (zb_tdrain.hip): no descriptors now, no merge bytes
    if (threadIdx.x < 6) P.wstats[(uint64_t)blockIdx.x * 6 + threadIdx.x] = 0;
    return;
  }
  const int lane = threadIdx.x & 63;
  int64_t inst = (int64_t)blockIdx.x * TWG + threadIdx.x;
  const bool active = inst < P.n;
  if (!active) inst = P.n - 1;  // (follows the last instance, writes nothing)
  TmplLane L;
  L.ncls = __builtin_amdgcn_readfirstlane(P.plan->nc);
  uint32_t cls = 0;
  cls = tmpl_lane_io(P, inst, L);
  const uint32_t crow = cls * CLS_ROW;
  const int W = active ? (int)P.wcount[cls] : 0;
  int Wmax = W;
  for (int d = 32; d >= 1; d >>= 1) Wmax = max(Wmax, __shfl_xor(Wmax, d, 64));
  const uint32_t create_ref = P.log[P.log_base + inst].payload;
  uint32_t err = 0;
  uint64_t merge_bytes = 0;
  uint32_t pc_sym = PAY_CREATE, pc_ref = create_ref;  // last resolved payload symbol
  const uint32_t create_len = arena_len(P.arena, create_ref);
  uint32_t pc_len = create_len;
  uint32_t* reg = s_merge + threadIdx.x * TL::STRIDE;
  uint8_t* stage = (uint8_t*)(s_merge + (threadIdx.x & ~63) * TL::STRIDE);  // the wave's slice
  zb_rec* s_desc = (zb_rec*)stage;
  uint32_t* s_srcd = (uint32_t*)(stage + 64 * TF * 32);
  uint32_t* s_vlen = s_srcd + 64 * TF;
  int64_t prev0 = P.log_base + inst;  // the instance's first record of the previous generation (the CREATE)
  int xg = 0x7fffffff;  // the first generation whose merge k_tmpl_xtree finishes (every later merge of it too)

#pragma unroll 1
  for (int w = 0; w < Wmax; w++) {
    const bool live = w < W;
    const TrajBase wb = kload(P.wbase, (uint64_t)w);
    int64_t po = 0, pw = 0, pj = 0;
#pragma unroll
    for (int c = 0; c < CLS_MAX; c++) {
      if (c >= (int)L.ncls) break;
      const uint64_t n = kload(P.agg, (uint64_t)c * CLS_ROW + w);
      po += (int64_t)L.before[c] * (int64_t)(n & 0xffff);
      pw += (int64_t)L.before[c] * (int64_t)((n >> 16) & 0xffff);
      pj += (int64_t)L.before[c] * (int64_t)(n >> 32);
    }
    const int64_t pos0 = wb.pos + po, kwf = wb.wf + pw, kjob = wb.job + pj;
    const uint32_t nrec = live ? (uint32_t)(P.agg[(uint64_t)crow + w] & 0xffff) : 0;
    uint32_t merged_ref = 0, merged_len = 0;
    const MergeGen g = live ? P.mgen[(uint64_t)crow + w] : MergeGen{};
    if (g.has) {
      uint32_t src = g.src, tgt = g.tgt;
      if (src == PAY_CREATE) src = create_ref;
      else if (src & PAY_MERGE) src = (uint32_t)(tmpl_mslot(P, L, src & 0xffff) >> 3);
      if (tgt == pc_sym) tgt = pc_ref;
      else if (tgt == PAY_CREATE) tgt = create_ref;
      else if (tgt & PAY_MERGE) tgt = (uint32_t)(tmpl_mslot(P, L, tgt & 0xffff) >> 3);
      const uint64_t at = tmpl_mslot(P, L, (uint32_t)w);
      merged_ref = (uint32_t)(at >> 3);
      if (w > xg) {  // (a pending chain: k_tmpl_xtree merges it, in order)
        merged_len = VLEN_UNKNOWN;
      } else {
        const uint32_t m_len = arena_len(P.arena, src) + arena_len(P.arena, tgt) + 8;
        if (tblob_bytes(m_len) > g.stride) err |= DE_UNSUPPORTED;
        else if (at + g.stride > P.arena_cap) err |= DE_ARENA_FULL;
        else {
          uint32_t ns = 0, nt = 0, olen = 0;
          bool tree = false;
          merge_into<GEN, TL::OUT_WORDS, TL::IN_WORDS>(P, src, tgt, m_len, at, reg, err, ns, nt, olen,
                                                        P.xq ? &tree : nullptr);
          if (tree) {
            xg = w;
            merged_len = VLEN_UNKNOWN;
            P.xq[atomicAdd(&ctl->xq_n, 1u)] = (uint64_t)inst | (uint64_t)w << 40;
          } else {
            merge_bytes += ns + nt + olen;
            merged_len = olen;
          }
        }
      }
    }
    // the wave's range of this generation: [base, base + span)
    uint32_t span = nrec;
    for (int d = 32; d >= 1; d >>= 1) span += __shfl_xor(span, d, 64);
    const int64_t base = __shfl(pos0, 0, 64);  // lane 0 is an active instance whenever span > 0
    const uint32_t rel = (uint32_t)(pos0 - base);
#pragma unroll 1
    for (uint32_t k = 0; k < nrec; k++) {
      const TmplRec t = P.tmpl[((uint64_t)crow + w) * TF + k];
      zb_rec d;
      d.key = tmpl_key(P, L, t.key, (uint32_t)w, kwf, kjob);
      d.scope_key = t.scope == SYM_CMDPOS ? P.log_base + inst : tmpl_key(P, L, t.scope, (uint32_t)w, kwf, kjob);
      d.inst_key = tmpl_key(P, L, t.inst, (uint32_t)w, kwf, kjob);
      uint32_t pay = t.payload, plen;
      if (pay == (PAY_MERGE | (uint32_t)w)) { pay = merged_ref; plen = merged_len; }
      else if (pay == pc_sym) { pay = pc_ref; plen = pc_len; }
      else if (pay == PAY_CREATE) { pay = create_ref; plen = create_len; }
      else if (pay & PAY_MERGE) {
        const uint32_t r = (uint32_t)(tmpl_mslot(P, L, pay & 0xffff) >> 3);
        plen = (int)(pay & 0xffff) >= xg ? VLEN_UNKNOWN : arena_len(P.arena, r);  // (pending: k_tmpl_xtree writes it)
        pc_sym = pay;
        pc_ref = r;
        pc_len = plen;
        pay = r;
      } else {
        plen = arena_len(P.arena, pay);  // a static blob (shared by every instance: cached)
      }
      if (t.payload & PAY_MERGE) { pc_sym = t.payload; pc_ref = pay; pc_len = plen; }
      d.payload = pay;
      d.elem = t.elem; d.intent = t.intent; d.kind = t.kind;
      // the value's length (zb_serialize.hip encode_value) from the element's constants and the variable fields
      // (a pending merge result's length is not known yet: the drain's size pass measures it)
      const uint8_t vt = kind_vt(d.kind), rt = kind_rt(d.kind);
      uint32_t vl = VLEN_UNKNOWN;
      if (plen != VLEN_UNKNOWN && !(d.kind & KIND_RAW) && ((vt == ZB_VT_WORKFLOW_INSTANCE && rt == ZB_RT_EVENT) ||
                                                          (vt == ZB_VT_JOB && (d.intent | 1) != JI_CANCELED))) {
        const ValueConst vc = kload(P.vconst, (uint64_t)d.elem);
        vl = (vt == ZB_VT_JOB ? vc.job : vc.wf) + mp_int_len(d.inst_key) + mp_int_len(d.scope_key) + mp_bin_len(plen);
      }
      s_desc[rel + k] = d;
      s_srcd[rel + k] = (uint32_t)(pos0 + k - (prev0 + t.pad[0]));
      s_vlen[rel + k] = vl;
    }
    if (live) prev0 = pos0;
    // the wave's range out in whole lines (records past the log's capacity are an error, not written)
    if (span) {
      uint32_t fit = span;
      if (base + span > (int64_t)P.log_cap) {
        fit = base < (int64_t)P.log_cap ? (uint32_t)((int64_t)P.log_cap - base) : 0;
        err |= DE_LOG_FULL;
      }
      uint4* dst = (uint4*)(P.log + base);
      for (uint32_t c = lane; c < 2 * fit; c += 64) dst[c] = ((const uint4*)s_desc)[c];
      for (uint32_t c = lane; c < fit; c += 64) {
        P.srcd[base + c] = s_srcd[c];
        P.vlen[base + c] = s_vlen[c];
      }
    }
  }
  // statistics: everything but the merge bytes is a per-class constant (k_traj_commit)
  uint64_t s0 = active ? merge_bytes : 0, s1 = 0, t0, t1;
  block_scan2(s0, s1, t0, t1, s_scan);
  if (threadIdx.x == 0) {
    uint64_t* ws = P.wstats + (uint64_t)blockIdx.x * 6;
    ws[0] = ws[1] = ws[2] = ws[3] = ws[5] = 0;
    ws[4] = t0;
  }
  if (!active) err &= DE_LOG_FULL;  // (the range copy is the wave's: an inactive lane may see its overflow)
  if (err & TE_REGEN) atomicOr(&ctl->regen, 1u);
  if (err & TE_XTREE) atomicOr(&ctl->flag, TE_FALLBACK);  // (nothing commits: the wave pipeline runs the batch)
  const uint32_t derr = err & ~(uint32_t)(TE_FALLBACK | TE_REGEN | TE_XTREE);
  if (derr) atomicOr(&ctl->derr, derr);
}

// The exact tree for the merge chains the template emit left (zb_xmerge.hpp; as k_merge_gen on the wave pipeline): the
// GEN pass queued every instance whose merge the structural merge refused (P.xq: instance | first generation << 40)
// and wrote its descriptors with the merge slots' refs. Here each queued instance runs its merges from that generation
// on, in generation order (a later merge may read an earlier one's result): the structural merge first, the exact tree
// where it refuses (MsgPackDocumentIndexer.java:136-283, MsgPackTree.java:141-166). One lane per queued instance over a
// grid of XLANE_COUNT lanes, so each wave holds one lane group of workspaces at a time (x_run, wave-uniform calls).
template <bool CLS>
__global__ void __launch_bounds__(256) k_tmpl_xtree(TrajParams P) {
  __shared__ unsigned long long s_b[4];
  const TrajCtl* ctl = P.ctl;
  if (ctl->flag) return;
  const uint32_t n = ctl->xq_n;
  if (n == 0) return;
  uint32_t err = 0;
  unsigned long long bytes = 0;
  const uint32_t stride = gridDim.x * blockDim.x;
  const uint32_t rounds = (n + stride - 1) / stride;  // (every lane of a wave walks the same rounds)
  for (uint32_t rd = 0; rd < rounds; rd++) {
    const uint32_t q = rd * stride + blockIdx.x * blockDim.x + threadIdx.x;
    const bool act = q < n;
    const uint64_t ent = act ? P.xq[q] : 0;
    const int64_t inst = (int64_t)(ent & ((1ull << 40) - 1));
    const int xg = (int)(ent >> 40);
    TmplLane L;
    uint32_t cls = 0;
    if (CLS) {
      L.ncls = __builtin_amdgcn_readfirstlane(P.plan->nc);
      cls = tmpl_lane_io(P, inst, L);
    } else {
      L.ncls = 1;
#pragma unroll
      for (int c = 0; c < CLS_MAX; c++) L.before[c] = c == 0 ? (uint32_t)inst : 0;
    }
    const int W = act ? (int)P.wcount[cls] : 0;
    int Wmax = W;
    for (int d = 32; d >= 1; d >>= 1) Wmax = max(Wmax, __shfl_xor(Wmax, d, 64));
    const uint32_t create_ref = act ? P.log[P.log_base + inst].payload : 0u;
    for (int w = 0; w < Wmax; w++) {
      const MergeGen g = (act && w >= xg && w < W) ? P.mgen[(uint64_t)cls * CLS_ROW + w] : MergeGen{};
      bool need = false;
      const uint8_t *sp = nullptr, *tp = nullptr;
      uint8_t* dst = nullptr;
      uint32_t ns = 0, nt = 0, cap = 0, olen = 0;
      if (g.has) {
        uint32_t src = g.src, tgt = g.tgt;  // (resolved as the emit does: its pc_sym cache names the same refs)
        if (src == PAY_CREATE) src = create_ref;
        else if (src & PAY_MERGE) src = (uint32_t)(tmpl_mslot(P, L, src & 0xffff) >> 3);
        if (tgt == PAY_CREATE) tgt = create_ref;
        else if (tgt & PAY_MERGE) tgt = (uint32_t)(tmpl_mslot(P, L, tgt & 0xffff) >> 3);
        sp = P.arena + (uint64_t)src * 8;
        tp = P.arena + (uint64_t)tgt * 8;
        ns = *(const uint32_t*)sp;
        nt = *(const uint32_t*)tp;
        cap = ns + nt + 8;
        const uint64_t at = tmpl_mslot(P, L, (uint32_t)w);
        dst = P.arena + at;
        if (tblob_bytes(cap) > g.stride) {
          err |= DE_UNSUPPORTED;
        } else if (at + g.stride > P.arena_cap) {
          err |= DE_ARENA_FULL;
        } else if (w == xg) {  // (the GEN pass's structural merge refused this very pair: straight to the tree)
          need = true;
        } else {
          Out o{dst + 4, 0};
          bool unsup = false;
          const bool ok = merge_docs(sp + 4, ns, tp + 4, nt, o, unsup);
          olen = o.n;
          if (o.n > cap) err |= DE_UNSUPPORTED;
          need = (!ok || unsup) && o.n <= cap;
          if (!need && o.n <= cap) {
            *(uint32_t*)dst = olen;
            bytes += ns + nt + olen;
          }
        }
      }
      x_run(XSlabs{P.xslab, P.xlocks, P.xlane}, need, [&](const XWs& ws, bool fin) {
        Out o{dst + 4, 0};
        const int st = x_merge(ws, sp + 4, ns, tp + 4, nt, o, cap);
        if (st == X_UNSUP && !fin) return st;
        if (st == X_OK) {
          if (o.n == 1 && dst[4] == 0xc0) dst[4] = 0x80;  // an empty tree: DocumentValue.wrap turns nil into {}
          olen = o.n;
        } else {
          // X_NOT_MAP (a non-map root) would be an incident, which a merge already emitted cannot become
          err |= st == X_FAIL ? DE_BAD_PAYLOAD : DE_UNSUPPORTED;
        }
        return st;
      });
      if (need) {
        *(uint32_t*)dst = olen;
        bytes += ns + nt + olen;
      }
    }
  }
  if (err) atomicOr(P.err, err);
  for (int d = 32; d >= 1; d >>= 1) bytes += __shfl_down(bytes, d, 64);
  if ((threadIdx.x & 63) == 0) s_b[threadIdx.x >> 6] = bytes;
  __syncthreads();
  if (threadIdx.x == 0 && (s_b[0] | s_b[1] | s_b[2] | s_b[3]))
    atomicAdd((unsigned long long*)P.stats + 4, s_b[0] + s_b[1] + s_b[2] + s_b[3]);  // merge bytes
}

// conditions are compiled into the count / emit kernels only when the model has exclusive splits
// (a uniform batch never has any), keeping the condition VM's call frame out of the other variants
void launch_traj_count(const TrajParams& p, hipStream_t s) {
  if (p.cond) hipLaunchKernelGGL((k_traj<false, false, true, false, false, false>), dim3(p.nwg), dim3(TWG), 0, s, p);
  else hipLaunchKernelGGL((k_traj<false, false, false, false, false, false>), dim3(p.nwg), dim3(TWG), 0, s, p);
}
// uniform batch: count one representative instance (the first CREATE), one workgroup
void launch_traj_count_uniform(const TrajParams& p, hipStream_t s) {
  TrajParams q = p;
  q.n = 1;
  q.nwg = 1;
  hipLaunchKernelGGL((k_traj<false, false, false, false, true, false>), dim3(1), dim3(TWG), 0, s, q);
}
// class batch: classify, plan, group masks, offsets, emit permutation, one traced representative per class
void launch_traj_count_classes(const TrajParams& p, const InjectParams* inj, hipStream_t s) {
  const InjectParams ip = inj ? *inj : InjectParams{};
  const bool small = ((p.max_create + 11) & ~7u) <= 13 * 4;
  if (inj && small) hipLaunchKernelGGL((k_cls_classify<13, true>), dim3(p.nwg), dim3(TWG), 0, s, p, ip);
  else if (inj) hipLaunchKernelGGL((k_cls_classify<25, true>), dim3(p.nwg), dim3(TWG), 0, s, p, ip);
  else if (small) hipLaunchKernelGGL((k_cls_classify<13, false>), dim3(p.nwg), dim3(TWG), 0, s, p, ip);
  else hipLaunchKernelGGL((k_cls_classify<25, false>), dim3(p.nwg), dim3(TWG), 0, s, p, ip);
  hipLaunchKernelGGL(k_cls_plan, dim3(1), dim3(256), 0, s, p);
  hipLaunchKernelGGL(k_cls_masks, dim3(p.nwg), dim3(TWG), 0, s, p);
  hipLaunchKernelGGL(k_cls_scan, dim3(CLS_MAX), dim3(1024), 0, s, p);
  if (!p.io) {  // the class-uniform emit's slot layout
    hipLaunchKernelGGL(k_cls_segs, dim3(1), dim3(1024), 0, s, p);
    hipLaunchKernelGGL(k_cls_perm, dim3(p.nwg), dim3(TWG), 0, s, p);
  }
  hipLaunchKernelGGL((k_traj<false, false, false, false, true, true>), dim3(1), dim3(TWG), 0, s, p);
}
void launch_traj_scan(const TrajParams& p, hipStream_t s) {
  if (!p.uni && !p.cls) hipLaunchKernelGGL(k_traj_scan, dim3(p.wcap), dim3(1024), 0, s, p);
  hipLaunchKernelGGL(k_traj_base, dim3(1), dim3(1024), 0, s, p);
}
void launch_traj_emit(const TrajParams& p, hipStream_t s, hipEvent_t* ev_main) {
  const dim3 g(p.nwg), b(TWG);
  auto mark = [&](int i) {
    if (ev_main) (void)hipEventRecord(ev_main[i], s);
  };
  if ((p.cls || p.uni) && p.defer_ok && !p.materialize) launch_tmpl_decide(p, s);
  if (p.cls && p.io) {  // instance order (default)
    mark(0);
    hipLaunchKernelGGL((k_tmpl_io<false>), g, b, 0, s, p);
    mark(1);
    hipLaunchKernelGGL(k_traj_regen, dim3(1), dim3(1), 0, s, p);
    hipLaunchKernelGGL((k_tmpl_io<true>), g, b, 0, s, p);
  } else if (p.cls) {
    const dim3 ge(p.nwg_e);
    mark(0);
    hipLaunchKernelGGL((k_tmpl<true, false>), ge, b, 0, s, p);
    mark(1);
    hipLaunchKernelGGL(k_traj_regen, dim3(1), dim3(1), 0, s, p);
    hipLaunchKernelGGL((k_tmpl<true, true>), ge, b, 0, s, p);
  } else if (p.uni) {
    mark(0);
    hipLaunchKernelGGL((k_tmpl<false, false>), g, b, 0, s, p);
    mark(1);
    hipLaunchKernelGGL(k_traj_regen, dim3(1), dim3(1), 0, s, p);
    hipLaunchKernelGGL((k_tmpl<false, true>), g, b, 0, s, p);
  } else if (p.cond) {
    mark(0);
    hipLaunchKernelGGL((k_traj<true, false, true, false, false, false>), g, b, 0, s, p);
    mark(1);
    hipLaunchKernelGGL(k_traj_regen, dim3(1), dim3(1), 0, s, p);
    hipLaunchKernelGGL((k_traj<true, false, true, true, false, false>), g, b, 0, s, p);
  } else {
    mark(0);
    hipLaunchKernelGGL((k_traj<true, false, false, false, false, false>), g, b, 0, s, p);
    mark(1);
    hipLaunchKernelGGL(k_traj_regen, dim3(1), dim3(1), 0, s, p);
    hipLaunchKernelGGL((k_traj<true, false, false, true, false, false>), g, b, 0, s, p);
  }
  if (!p.materialize) hipLaunchKernelGGL(k_traj_commit, dim3(1), dim3(COMMIT_WG), 0, s, p);
  if (p.xq && (p.uni || p.cls) && !p.materialize) {  // the merge chains the template emit queued for the exact tree (none: exits at once)
    if (p.cls) hipLaunchKernelGGL(k_tmpl_xtree<true>, dim3(XLANE_COUNT / 256), dim3(256), 0, s, p);
    else hipLaunchKernelGGL(k_tmpl_xtree<false>, dim3(XLANE_COUNT / 256), dim3(256), 0, s, p);
  }
}

}  // namespace zbg
