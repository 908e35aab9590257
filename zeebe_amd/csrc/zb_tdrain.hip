// zb_tdrain.hip — the drain of a deferred template batch: record values + headers encoded straight from the
// traced class trajectories and each instance's rank, with no descriptors in between.
//
// A uniform or class batch on the trajectory path (zb_traj.hip) is fully described by its traces (TmplRec per
// class and generation), the generation bases (TrajBase) and, per instance, its class and the class-c instances
// before it (TmplLane). k_tmpl turns that into 32-byte descriptors (+ source deltas and value-length hints) that
// the drain (zb_serialize.hip) reads back: on C3 10M, 3.3 GB written by k_tmpl as 6.8 GB of partial lines and
// 7.8 GB read back by k_ser_fast per step (profiles/r02). When the batch's records are all of the kinds the fast
// encoder takes and no generation merges payloads, zb_step leaves the batch deferred (TrajCtl.defer) and
// zb_serialize of exactly its records runs this drain instead:
//   k_tdrain_size   one lane per instance (instance order = log order inside every generation): per generation
//                   the value bytes of the wave's records -> wbytes[w][wave]
//   (hipcub)        exclusive scan over wbytes, generation-major = log order -> byte offset of every wave range
//   k_tdrain_write  the same lanes again: headers of the wave's records; per generation the four waves of a
//                   workgroup take turns encoding their values with the fast encoder (zb_fastenc.hpp) into the
//                   workgroup's LDS image, which all 256 lanes stream out with 16-byte stores
// The CREATE payload -- the payload of every record the instance writes -- is read once per lane, not once per
// record. Anything else (zb_step, frames, descriptors, a partial range, compaction) materializes the batch
// first with k_tmpl, so every other API sees the descriptors it always saw.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "zb_fastenc.hpp"
#include "zb_frame.hpp"
#include "zb_tmpl.hpp"
#include "zb_wavelib.hpp"

namespace zbg {

constexpr int TD_WG = TRAJ_WG;  // 256 lanes = 256 instances, four waves
// each wave's image: one round of the wave's records of a generation (64 records of C3, ~10 KB); a lane whose
// records alone exceed it sends the batch to the descriptor path (ZB_EAGAIN). 4 x 11 KB + the tables (~8 KB for
// C3): three workgroups per CU, as the 135 VGPRs allow (measured: 7 KB images, four workgroups, 2 rounds per
// generation: 1.3x the time)
constexpr uint32_t TD_IMG = 11 * 1024 - 16;

// The batch's tables in LDS (every lookup of the generation loop is an LDS read, not a dependent global load):
//   agg[c][w]  records | wf keys << 16 | job keys << 32 of class c in generation w (one instance)
//   wbase[w]   generation bases (log position, key ordinals)
//   tmpl[c][w][k] traced records,  vconst[e] value-length constants of element e
struct TdTab {
  const uint64_t* agg;
  const TrajBase* wbase;
  const TmplRec* tmpl;
  const ValueConst* vconst;
  uint32_t wmax;
};
struct TdLayout {
  uint32_t tab, pool, agg, wbase, tmpl, vconst, total;  // byte offsets in dynamic LDS (16-aligned) and the size
};
__host__ __device__ __forceinline__ uint32_t td_r16(uint32_t x) { return (x + 15) & ~15u; }
__host__ __device__ __forceinline__ TdLayout td_layout(const TDrainParams& d, bool model) {
  TdLayout l;
  l.tab = 0;
  const uint32_t tb = model ? td_r16((uint32_t)d.n_elems * (uint32_t)sizeof(DevValSeg)) : 0u;  // DevValSeg table
  l.pool = l.tab + tb;
  l.agg = l.pool + (model ? td_r16(d.segpool_len) : 0u);
  l.wbase = l.agg + td_r16(d.nc * d.wmax * 8u);
  l.tmpl = l.wbase + td_r16(d.wmax * (uint32_t)sizeof(TrajBase));
  l.vconst = l.tmpl + td_r16(d.nc * d.wmax * (uint32_t)TF * (uint32_t)sizeof(TmplRec));
  l.total = l.vconst + td_r16((uint32_t)d.n_elems * (uint32_t)sizeof(ValueConst));
  return l;
}
// copies the tables (and, for the write pass, the value segments) into LDS; ends in a barrier
__device__ __forceinline__ TdTab td_load_tables(const TDrainParams& D, uint8_t* sm, bool model) {
  const TdLayout l = td_layout(D, model);
  const TrajParams& P = D.t;
  const int t = threadIdx.x;
  if (model) {
    const uint32_t tb = td_r16((uint32_t)D.n_elems * (uint32_t)sizeof(DevValSeg));  // (padded to 4 entries at deploy)
    for (uint32_t c = t; c < tb / 4; c += TD_WG) ((uint32_t*)(sm + l.tab))[c] = ((const uint32_t*)D.vsegs)[c];
    for (uint32_t c = t; c < D.segpool_len / 8; c += TD_WG) ((uint64_t*)(sm + l.pool))[c] = ((const uint64_t*)D.segpool)[c];
  }
  uint64_t* agg = (uint64_t*)(sm + l.agg);
  for (uint32_t c = t; c < D.nc * D.wmax; c += TD_WG)
    agg[c] = P.agg[(uint64_t)(c / D.wmax) * CLS_ROW + c % D.wmax];
  TrajBase* wb = (TrajBase*)(sm + l.wbase);
  for (uint32_t c = t; c < D.wmax; c += TD_WG) wb[c] = P.wbase[c];
  uint4* tm = (uint4*)(sm + l.tmpl);  // TmplRec: two 16-byte halves
  for (uint32_t c = t; c < D.nc * D.wmax * TF * 2; c += TD_WG) {
    const uint32_t r = c / 2, h = c & 1, k = r % TF, cw = r / TF;
    const uint64_t src = ((uint64_t)(cw / D.wmax) * CLS_ROW + cw % D.wmax) * TF + k;
    tm[c] = ((const uint4*)(P.tmpl + src))[h];
  }
  ValueConst* vc = (ValueConst*)(sm + l.vconst);
  for (uint32_t c = t; c < (uint32_t)D.n_elems; c += TD_WG) vc[c] = P.vconst[c];
  __syncthreads();
  TdTab T;
  T.agg = agg; T.wbase = wb; T.tmpl = (const TmplRec*)tm; T.vconst = vc; T.wmax = D.wmax;
  return T;
}

// key ordinal base of generation g for this instance: wf (f = 1) or job (f = 2) counter (tmpl_kbase on the tables)
__device__ __forceinline__ int64_t td_kbase(const TdTab& T, const TmplLane& L, uint32_t g, int f) {
  const TrajBase wb = T.wbase[g];
  int64_t k = f == 1 ? wb.wf : wb.job;
#pragma unroll
  for (int c = 0; c < CLS_MAX; c++) {
    if (c >= (int)L.ncls) break;
    const uint64_t n = T.agg[c * T.wmax + g];
    k += (int64_t)L.before[c] * (int64_t)(f == 1 ? ((n >> 16) & 0xffff) : (n >> 32));
  }
  return k;
}
// kwf0: the instance's wf key ordinal base of generation 0 (its process instance key: the workflowInstanceKey and
// the flow scope of most records), computed once per lane
__device__ __forceinline__ int64_t td_key(const TrajParams& P, const TdTab& T, const TmplLane& L, uint32_t sym,
                                          uint32_t w, int64_t kwf, int64_t kjob, int64_t kwf0) {
  if (sym == NOK) return -1;
  if (sym == JOB_ZERO) return 0;
  const uint32_t g = (sym >> 4) & 0xfff, ord = sym & 15;
  if (sym & SYMK_WF) return P.wf_start + 5 * ((g == w ? kwf : g == 0 ? kwf0 : td_kbase(T, L, g, 1)) + ord);
  return P.job_start + 5 * ((g == w ? kjob : td_kbase(T, L, g, 2)) + ord);
}

// td_kbase / td_key for a wave whose every key / position lies in [2^16, 2^32) or is -1 / 0 (the size pass's short
// form): the same values in 32-bit arithmetic (exact: every result is below 2^32)
__device__ __forceinline__ uint32_t td_kbase32(const TdTab& T, const TmplLane& L, uint32_t g, int f) {
  const TrajBase wb = T.wbase[g];
  uint32_t k = (uint32_t)(f == 1 ? wb.wf : wb.job);
#pragma unroll
  for (int c = 0; c < CLS_MAX; c++) {
    if (c >= (int)L.ncls) break;
    const uint64_t n = T.agg[c * T.wmax + g];
    k += L.before[c] * (f == 1 ? (uint32_t)((n >> 16) & 0xffff) : (uint32_t)(n >> 32));
  }
  return k;
}
__device__ __forceinline__ int64_t td_key5(const TrajParams& P, const TdTab& T, const TmplLane& L, uint32_t sym,
                                           uint32_t w, int64_t kwf, int64_t kjob, int64_t kwf0) {
  if (sym == NOK) return -1;
  if (sym == JOB_ZERO) return 0;
  const uint32_t g = (sym >> 4) & 0xfff, ord = sym & 15;
  if (sym & SYMK_WF)
    return (int64_t)((uint32_t)P.wf_start +
                     5u * ((g == w ? (uint32_t)kwf : g == 0 ? (uint32_t)kwf0 : td_kbase32(T, L, g, 1)) + ord));
  return (int64_t)((uint32_t)P.job_start + 5u * ((g == w ? (uint32_t)kjob : td_kbase32(T, L, g, 2)) + ord));
}
// msgpack length of such a key: -1 / 0 are fixints, the rest 0xce + 4 bytes
__device__ __forceinline__ uint32_t td_klen5(int64_t v) { return (uint64_t)(v + 1) <= 1 ? 1u : 5u; }

// one instance's generation w: log position and key bases (linear in the class ranks), record count
struct TdGen {
  int64_t pos0, kwf, kjob;
  uint32_t nrec;
};
__device__ __forceinline__ TdGen td_gen(const TdTab& T, const TmplLane& L, uint32_t cls, int w, bool live) {
  const TrajBase wb = T.wbase[w];
  int64_t po = 0, pw = 0, pj = 0;
#pragma unroll
  for (int c = 0; c < CLS_MAX; c++) {
    if (c >= (int)L.ncls) break;
    const uint64_t n = T.agg[c * T.wmax + w];
    po += (int64_t)L.before[c] * (int64_t)(n & 0xffff);
    pw += (int64_t)L.before[c] * (int64_t)((n >> 16) & 0xffff);
    pj += (int64_t)L.before[c] * (int64_t)(n >> 32);
  }
  TdGen G;
  G.pos0 = wb.pos + po;
  G.kwf = wb.wf + pw;
  G.kjob = wb.job + pj;
  G.nrec = live ? (uint32_t)(T.agg[cls * T.wmax + w] & 0xffff) : 0;
  return G;
}
// td_gen for a whole wave of consecutive instances: the first lane's bases by the linear formula, computed from
// its class ranks in scalar registers (agg and the generation bases through the scalar cache), every other
// lane's as the first lane's plus an exclusive scan of the lanes' own counts (instance i's records follow those
// of the instances before it in every generation). b0: the first lane's class ranks, nc classes.
__device__ __forceinline__ TdGen td_gen_wave(const TrajParams& P, const TdTab& T, const uint32_t (&b0)[CLS_MAX],
                                             uint32_t nc, uint32_t cls, int w, bool live) {
  const TrajBase wb = kload(P.wbase, (uint64_t)w);
  int64_t po = 0, pw = 0, pj = 0;
#pragma unroll
  for (int c = 0; c < CLS_MAX; c++) {
    if (c >= (int)nc) break;
    const uint64_t n = kload(P.agg, (uint64_t)c * CLS_ROW + (uint64_t)w);
    po += (int64_t)b0[c] * (int64_t)(n & 0xffff);
    pw += (int64_t)b0[c] * (int64_t)((n >> 16) & 0xffff);
    pj += (int64_t)b0[c] * (int64_t)(n >> 32);
  }
  const uint64_t own = T.agg[cls * T.wmax + w];  // (what td_gen's dot product counts for this lane's class)
  const uint32_t x = (uint32_t)(own & 0xff) | (uint32_t)((own >> 16) & 0xfff) << 8 | (uint32_t)((own >> 32) & 0xfff) << 20;
  const uint32_t ex = wave_incl_scan(x) - x;  // (per instance <= TF records and <= 15 keys of each kind)
  TdGen G;
  G.pos0 = wb.pos + po + (ex & 0xff);
  G.kwf = wb.wf + pw + ((ex >> 8) & 0xfff);
  G.kjob = wb.job + pj + (ex >> 20);
  G.nrec = live ? (uint32_t)(own & 0xffff) : 0;
  return G;
}

// The first SER_PRE words of a static payload blob (a trace's literal ref, the same for every lane of its class)
// through the scalar cache, one scalar load sequence per distinct ref of the wave: inside the write pass's
// generation loop a vector load would wait for every store the wave issued before it (vmcnt counts loads and
// stores together, in order), i.e. for the previous generation's whole image stream. `mine`: this lane's record
// has a static payload, ref; the other lanes' pre is left as it is.
template <int N>
__device__ __forceinline__ void td_static_pre(const uint8_t* arena, bool mine, uint32_t ref, uint64_t (&pre)[N]) {
  uint64_t need = __ballot(mine);
  while (need) {
    const uint32_t r = __builtin_amdgcn_readlane(ref, __builtin_ctzll(need));
    const cptr<uint64_t> src = K((const uint64_t*)(arena + (uint64_t)r * 8));
    uint64_t w[N];
#pragma unroll
    for (int j = 0; j < N; j++) w[j] = src[j];  // (ARENA_SLACK: never past the allocation)
    const bool take = mine && ref == r;
#pragma unroll
    for (int j = 0; j < N; j++) pre[j] = take ? w[j] : pre[j];  // (a select: in a branch on ref == r the compiler
    need &= ~__ballot(take);                                     //  turns the loads into vector ones)
  }
}

// record k of the instance's generation w, resolved from the class trace; vl: its value length (the
// encoder's, by the formula), plen: its payload document's length
template <bool SCALAR_STATIC = false, bool L5 = false>
__device__ __forceinline__ zb_rec td_record(const TrajParams& P, const TdTab& T, const TmplLane& L, uint32_t cls, int w,
                                            uint32_t k, const TdGen& G, int64_t inst, uint32_t create_ref,
                                            uint32_t create_len, int64_t kwf0, uint32_t& vl, uint32_t& plen) {
  const TmplRec t = T.tmpl[(cls * T.wmax + w) * TF + k];
  zb_rec d;
  if (L5) {
    d.key = td_key5(P, T, L, t.key, (uint32_t)w, G.kwf, G.kjob, kwf0);
    d.scope_key = t.scope == SYM_CMDPOS ? P.log_base + inst : td_key5(P, T, L, t.scope, (uint32_t)w, G.kwf, G.kjob, kwf0);
    d.inst_key = td_key5(P, T, L, t.inst, (uint32_t)w, G.kwf, G.kjob, kwf0);
  } else {
    d.key = td_key(P, T, L, t.key, (uint32_t)w, G.kwf, G.kjob, kwf0);
    d.scope_key = t.scope == SYM_CMDPOS ? P.log_base + inst : td_key(P, T, L, t.scope, (uint32_t)w, G.kwf, G.kjob, kwf0);
    d.inst_key = td_key(P, T, L, t.inst, (uint32_t)w, G.kwf, G.kjob, kwf0);
  }
  // (k_tmpl_decide: no merge results in a deferred batch -- the CREATE payload or a static blob)
  const bool cr = t.payload == PAY_CREATE;
  d.payload = cr ? create_ref : t.payload;
  if (SCALAR_STATIC) {  // (the write pass: a static blob's length word through the scalar cache)
    uint64_t w0[1] = {0};
    td_static_pre(P.arena, !cr, d.payload, w0);  // (the active lanes: a waterfall over their refs)
    plen = cr ? create_len : (uint32_t)w0[0];
  } else {
    plen = cr ? create_len : arena_len(P.arena, d.payload);
  }
  d.elem = t.elem; d.intent = t.intent; d.kind = t.kind;
  const ValueConst vc = T.vconst[d.elem];
  vl = (kind_vt(d.kind) == ZB_VT_JOB ? vc.job : vc.wf) +
       (L5 ? td_klen5(d.inst_key) + td_klen5(d.scope_key) : mp_int_len(d.inst_key) + mp_int_len(d.scope_key)) +
       mp_bin_len(plen);
  return d;
}

// lane setup shared by both passes: class, ranks, CREATE payload
struct TdLane {
  TmplLane L;
  uint32_t cls, W, create_ref, create_len;
  int64_t inst, kwf0;
  bool active;
};
// need_ref: the CREATE payload's arena ref (the write pass reads the document); a class batch's payload lengths come
// from k_cls_classify's per-instance array, so the size pass reads 4 bytes per instance and no descriptor
__device__ __forceinline__ TdLane td_lane(const TrajParams& P, const TdTab& T, int64_t tile, bool need_ref) {
  TdLane t;
  t.inst = tile * TD_WG + threadIdx.x;
  t.active = t.inst < P.n;
  if (!t.active) t.inst = P.n - 1;  // (follows the last instance, writes nothing)
  t.cls = 0;
  if (P.cls) {
    t.L.ncls = __builtin_amdgcn_readfirstlane(P.plan->nc);
    t.cls = tmpl_lane_io(P, t.inst, t.L);
  } else {
    t.L.ncls = 1;
#pragma unroll
    for (int c = 0; c < CLS_MAX; c++) t.L.before[c] = c == 0 ? (uint32_t)t.inst : 0;
  }
  t.W = t.active ? P.wcount[t.cls] : 0;  // generations of the instance's class (rows beyond it are not its)
  t.create_ref = (need_ref || !P.clen) ? (P.cref ? P.cref[t.inst] : P.log[P.log_base + t.inst].payload) : 0u;
  t.create_len = P.clen ? P.clen[t.inst] : arena_len(P.arena, t.create_ref);
  t.kwf0 = td_kbase(T, t.L, 0, 1);
  return t;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {  // (lane 63: the wave's total)
  return wave_incl_scan(x);
}

// msgpack length of a symbolic key / position (td_key) known to be -1, 0 or in [2^16, 2^32)
__device__ __forceinline__ uint32_t td_len5(uint32_t sym) { return (sym == NOK || sym == JOB_ZERO) ? 1u : 5u; }

// Both passes: one workgroup per tile of 256 instances (a persistent grid that copies the tables once per
// workgroup measured slower: 0.39 -> 0.55 ms for the size pass on C3 10M)
// a record's bytes in the drain: its value, or (FR) its frame -- prefix + value, padded to 8 (no rejection reasons in a
// deferred batch)
template <bool FR>
__device__ __forceinline__ uint32_t td_bytes(uint32_t vl) { return FR ? (FRAME_PREFIX + vl + 7) & ~7u : vl; }

template <bool FR>
__global__ void __launch_bounds__(TD_WG) k_tdrain_size(TDrainParams D) {
  extern __shared__ __attribute__((aligned(16))) uint8_t s_tab[];
  __shared__ unsigned long long s_pay[TD_WG / 64];
  const TrajParams& P = D.t;
  const TdTab T = td_load_tables(D, s_tab, false);
  const int lane = threadIdx.x & 63;
  uint64_t pay = 0;
  {
    const int64_t tile = blockIdx.x;
    const TdLane L = td_lane(P, T, tile, false);
    const uint64_t wave = (uint64_t)tile * (TD_WG / 64) + (threadIdx.x >> 6);
    // Short form: when the wave's smallest key and position (its first lane's generation-0 bases, which every
    // later key of the wave exceeds) are >= 2^16 and the batch's largest is below 2^32, every key / position the
    // wave's records carry encodes in 5 bytes (MsgPackWriter.writeInteger): the lengths follow from the traces
    // alone, without resolving a single key. Otherwise (the first 13k keys of a partition) td_record resolves each.
    const bool lo_ok = P.wf_start + 5 * L.kwf0 >= 65536 && P.log_base + L.inst >= 65536 &&
                       (!D.jobs || P.job_start + 5 * td_kbase(T, L.L, 0, 2) >= 65536);
    const bool len5 = D.len5_ok && __builtin_amdgcn_readlane(lo_ok ? 1 : 0, 0);
#pragma unroll 1
    for (int w = 0; w < (int)D.wmax; w++) {
      uint32_t mine = 0;
      if (len5) {
        const uint32_t nrec = w < (int)L.W ? (uint32_t)(T.agg[L.cls * T.wmax + w] & 0xffff) : 0u;
#pragma unroll
        for (int k = 0; k < TF; k++) {
          if ((uint32_t)k >= nrec) break;
          const TmplRec t = T.tmpl[(L.cls * T.wmax + w) * TF + k];
          const uint32_t plen = t.payload == PAY_CREATE ? L.create_len : arena_len(P.arena, t.payload);
          const ValueConst vc = T.vconst[t.elem];
          mine += td_bytes<FR>((kind_vt(t.kind) == ZB_VT_JOB ? vc.job : vc.wf) + td_len5(t.inst) + td_len5(t.scope) +
                               mp_bin_len(plen));
          pay += plen;
        }
      } else {
        const TdGen G = td_gen(T, L.L, L.cls, w, w < (int)L.W);
#pragma unroll 1
        for (uint32_t k = 0; k < G.nrec; k++) {
          uint32_t vl, plen;
          (void)td_record(P, T, L.L, L.cls, w, k, G, L.inst, L.create_ref, L.create_len, L.kwf0, vl, plen);
          mine += td_bytes<FR>(vl);
          pay += plen;
        }
      }
      const uint32_t b = wave_sum(mine);
      if (lane == 63) D.wbytes[(uint64_t)w * D.nwave + wave] = b;
    }
  }
  // payload bytes of the drained records (zb_serialize_stats.payload_bytes): one partial per workgroup
  unsigned long long y = pay;
  for (int d = 32; d >= 1; d >>= 1) y += __shfl_down(y, d, 64);
  if (lane == 0) s_pay[threadIdx.x >> 6] = y;
  __syncthreads();
  if (threadIdx.x == 0) D.pay_part[blockIdx.x] = s_pay[0] + s_pay[1] + s_pay[2] + s_pay[3];
}

// The sizes of a class batch whose every key / position encodes in 5 bytes, with no record resolved: a class-c
// instance's value bytes in generation w are the class's constant part (per record: element constant + 5-byte keys,
// a static payload's binary) plus, per record that carries the CREATE payload, that payload as binary -- so a wave's
// bytes are sum_c (instances of c) x const[c][w] + creates[c][w] x (the wave's class-c CREATE binary lengths), from
// k_cls_masks' per-wave class masks and sums. One thread per instance workgroup (its four waves), workgroups
// [wg0, nwg); what k_tdrain_size writes: wbytes[w][wave] and the workgroup's payload bytes.
__global__ void __launch_bounds__(256) k_tdrain_sizes(TDrainParams D, uint32_t wg0) {
  __shared__ uint32_t s_cs[TD_MAX_CW], s_m[TD_MAX_CW], s_sp[TD_MAX_CW];
  const TrajParams& P = D.t;
  const uint32_t nc = D.nc, W = D.wmax;
  for (uint32_t e = threadIdx.x; e < nc * W; e += 256) {
    const uint32_t c = e / W, w = e % W;
    const uint64_t row = (uint64_t)c * CLS_ROW + w;
    const uint32_t nrec = w < P.wcount[c] ? (uint32_t)(P.agg[row] & 0xffff) : 0u;
    uint32_t cs = 0, m = 0, sp = 0;
    for (uint32_t k = 0; k < nrec && k < (uint32_t)TF; k++) {
      const TmplRec t = P.tmpl[row * TF + k];
      const ValueConst vc = P.vconst[t.elem];
      cs += (kind_vt(t.kind) == ZB_VT_JOB ? vc.job : vc.wf) + td_len5(t.inst) + td_len5(t.scope);
      if (t.payload == PAY_CREATE) {
        m += 1;
      } else {
        const uint32_t pl = arena_len(P.arena, t.payload);
        cs += mp_bin_len(pl);
        sp += pl;
      }
    }
    s_cs[e] = cs;
    s_m[e] = m;
    s_sp[e] = sp;
  }
  __syncthreads();
  const uint64_t g = (uint64_t)wg0 + (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= (uint64_t)P.nwg) return;
  uint64_t pay = 0;
  for (int v = 0; v < TD_WG / 64; v++) {
    const uint64_t wave = g * (TD_WG / 64) + v, grp = wave * CLS_MAX;
    uint32_t n[CLS_MAX];
    uint32_t gb[CLS_MAX], pb[CLS_MAX];
#pragma unroll
    for (int c = 0; c < CLS_MAX; c++) {
      const bool in = c < (int)nc;
      n[c] = in ? (uint32_t)__builtin_popcountll(P.cmask[grp + c]) : 0u;
      gb[c] = in ? P.cg[2 * (grp + c)] : 0u;
      pb[c] = in ? P.cg[2 * (grp + c) + 1] : 0u;
    }
    for (uint32_t w = 0; w < W; w++) {
      uint64_t b = 0;
#pragma unroll
      for (int c = 0; c < CLS_MAX; c++) {
        if (c >= (int)nc) break;
        const uint32_t e = c * W + w;
        b += (uint64_t)n[c] * s_cs[e] + (uint64_t)s_m[e] * gb[c];
        pay += (uint64_t)s_m[e] * pb[c] + (uint64_t)n[c] * s_sp[e];
      }
      D.wbytes[(uint64_t)w * D.nwave + wave] = b;
    }
  }
  D.pay_part[g] = pay;
}

// FR: log frames (zb_serialize_frames): each record's 13 prefix words (zb_frame.hpp) go into the image before its value,
// which the writer ends with the frame's zero padding; no headers. A record's source is its parent in the instance's
// previous generation (TmplRec.pad[0], as k_tmpl writes srcd), the first generation's the instance's CREATE; a batch
// (same source, contiguous) is at most the instance's TF records of one generation.
template <uint32_t IMG, bool FR>
__global__ void __launch_bounds__(TD_WG) __attribute__((amdgpu_waves_per_eu(3, 4))) k_tdrain_write(TDrainParams D) {
  // each wave's image, then its lanes' dummy slots (the branch-free writer's stores that must not land: FastWB)
  __shared__ __attribute__((aligned(16))) uint8_t s_img[TD_WG / 64][IMG + 16 + 8 * 64];
  extern __shared__ __attribute__((aligned(16))) uint8_t s_tab[];  // value segments + the batch's tables
  const TrajParams& P = D.t;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const TdTab T = td_load_tables(D, s_tab, true);
  const TdLayout lay = td_layout(D, true);
  const DevValSeg* tab = (const DevValSeg*)(s_tab + lay.tab);
  const uint8_t* segs = s_tab + lay.pool;
  uint8_t* img = s_img[wv];
  uint32_t bad = 0;
#ifdef ZB_PHASES  // (measurement build: wall-clock ticks per phase, summed by lane 0 of every wave)
  uint64_t ph_t = wall_clock64(), ph[4] = {0, 0, 0, 0}, ph_g = 0;
#define TD_PHASE(k) do { const uint64_t ph_n = wall_clock64(); ph[k] += ph_n - ph_t; ph_t = ph_n; } while (0)
#else
#define TD_PHASE(k) do { } while (0)
#endif
  {
    const int64_t tile = blockIdx.x;
    const TdLane L = td_lane(P, T, tile, true);
    // the instance's CREATE payload document, read once: every record of a deferred batch carries it or a static blob
    const uint64_t* cdw = (const uint64_t*)(P.arena + (uint64_t)L.create_ref * 8);
    uint64_t cpre[SER_PRE];
#pragma unroll
    for (int j = 0; j < SER_PRE; j++) cpre[j] = cdw[j];  // (ARENA_SLACK: never past the allocation)
    // the loads retired here, before the first store: an empty asm that redefines the words makes the compiler wait
    // for them once, instead of at the generation loop's first use of them, where the wait (vmcnt) would also take
    // every store issued so far
#pragma unroll
    for (int j = 0; j < SER_PRE; j++) asm volatile("" : "+v"(cpre[j]));
    // frames: request metadata of the instance's CREATE (its CREATED event carries it), the instance's records of the
    // previous generation (sources)
    uint64_t rid = ~0ull;
    uint32_t sid = 0x80000000u;
    if (FR && D.nreqs) {
      if (D.req_dense) {
        rid = D.reqs[L.inst].request_id;
        sid = (uint32_t)D.reqs[L.inst].request_stream_id;
      } else {
        frame_request(D.reqs, D.nreqs, P.log_base + L.inst, rid, sid);
      }
      asm volatile("" : "+v"(rid), "+v"(sid));  // (retired before the first store, as the payload words)
    }
    int64_t prev0 = P.log_base + L.inst;
    const FrameConst fcst{D.stream_id, D.raft_term, D.timestamp};
    // the wave's first lane's class ranks (td_gen_wave)
    uint32_t b0[CLS_MAX];
#pragma unroll
    for (int c = 0; c < CLS_MAX; c++) b0[c] = __builtin_amdgcn_readlane(L.L.before[c], 0);
    const uint32_t nc = __builtin_amdgcn_readfirstlane(L.L.ncls);
    const uint64_t swave = (uint64_t)tile * (TD_WG / 64) + __builtin_amdgcn_readfirstlane(wv);
    // this wave's value range of generation w: woffs[w][wave .. wave + 1], read one generation ahead (scalar loads)
    uint64_t nbase = K(D.woffs)[swave], nend = K(D.woffs)[swave + 1];
    // L5: every key / position of the wave in [2^16, 2^32) (k_tdrain_size's short form): 32-bit keys, 5-byte integers
    auto gen_loop = [&](auto l5) {
    constexpr bool L5 = decltype(l5)::value;
#pragma unroll 1
    for (int w = 0; w < (int)D.wmax; w++) {
      const uint64_t wbase = nbase, wend = nend;
      if (w + 1 < (int)D.wmax) {
        nbase = K(D.woffs)[(uint64_t)(w + 1) * D.nwave + swave];
        nend = K(D.woffs)[(uint64_t)(w + 1) * D.nwave + swave + 1];
      }
      if (wend == wbase) continue;  // (uniform: no record of this wave in generation w)
      if (wend > D.out_cap) {  // does not fit: the host grows the buffer and runs the pass again
        if (lane == 0) atomicOr(D.flags, 1u);
        continue;
      }
      const TdGen G = td_gen_wave(P, T, b0, nc, L.cls, w, w < (int)L.W);
      uint32_t vl0 = 0, vl1 = 0;
      zb_rec d0{}, d1{};
      {
        uint32_t plen;
        if (G.nrec > 0) d0 = td_record<true, L5>(P, T, L.L, L.cls, w, 0, G, L.inst, L.create_ref, L.create_len, L.kwf0, vl0, plen);
        if (G.nrec > 1) d1 = td_record<true, L5>(P, T, L.L, L.cls, w, 1, G, L.inst, L.create_ref, L.create_len, L.kwf0, vl1, plen);
      }
      const uint32_t f0 = G.nrec > 0 ? td_bytes<FR>(vl0) : 0u, f1 = G.nrec > 1 ? td_bytes<FR>(vl1) : 0u;
      const uint32_t mine = f0 + f1;
      const uint32_t incl = wave_incl_scan(mine);
      const uint32_t rel = incl - mine;  // this lane's values: [wbase + rel, wbase + incl)
      // the size pass's byte total of the wave (a formula for most waves: k_tdrain_sizes) must be what the records
      // encode to; a mismatch writes nothing and sends the batch to the descriptor drain instead of past its range
      if (wbase + (uint64_t)__builtin_amdgcn_readlane(incl, 63) != wend) {
        bad = 1;
        continue;
      }
#ifdef ZB_PHASES
      ph_g++;
#endif
      TD_PHASE(0);
      // headers: key, types / intent / rejection, length, offset (the position is implicit: start + index)
#pragma unroll
      for (int k = 0; k < TF; k++) {
        if (FR || (uint32_t)k >= G.nrec) break;
        const zb_rec& d = k ? d1 : d0;
        uint64_t* dh = (uint64_t*)(D.headers + (G.pos0 + k - D.start));
        const uint64_t meta = (uint64_t)kind_rt(d.kind) | (uint64_t)kind_vt(d.kind) << 8 | (uint64_t)d.intent << 16 |
                              255ull << 24 | (uint64_t)(k ? vl1 : vl0) << 32;  // (no rejections: k_tmpl_decide)
        // plain stores: a header line is written by three stores of every lane (24-byte stride), which L2 merges into
        // whole lines; as non-temporal stores they reached HBM as partial lines (write pass 4.55 -> 4.25 ms same box)
        if (!FR) {
          dh[0] = (uint64_t)d.key;
          dh[1] = meta;
          dh[2] = wbase + rel + (k ? vl0 : 0);
        }
      }
      TD_PHASE(1);
      // rounds: lanes [a, b) whose values fit the image from the round's first byte; each lane encodes its own
      // records (no redistribution: a generation of C3 is one round of every lane)
#pragma unroll 1
      for (int a = 0; a < 64;) {
        const uint32_t lo = __builtin_amdgcn_readlane(rel, a);  // the round's first byte
        const uint32_t sh = (uint32_t)(((uintptr_t)(D.out + wbase + lo)) & 15);
        const bool fit = lane >= a && incl - lo + sh <= IMG;  // (a suffix of lanes >= a fails: incl grows)
        const uint64_t fm = __ballot(fit);
        const int b = fm ? 64 - __builtin_clzll(fm) : a;
        if (b == a) {  // one instance's records exceed the image: the host takes the descriptor path
          bad = 1;
          break;
        }
        if (fit && mine) {
          // frames: the sources of the instance's records (TmplRec.pad[0]: its parent's index in the previous generation)
          uint32_t sp0 = 0, sp1 = 0;
          if (FR) {
            const TmplRec* tr = T.tmpl + (L.cls * T.wmax + w) * TF;
            sp0 = tr[0].pad[0];
            sp1 = G.nrec > 1 ? tr[1].pad[0] : sp0 + 1;
          }
#pragma unroll 1
          for (uint32_t k = 0; k < G.nrec; k++) {
            const zb_rec d = k ? d1 : d0;
            const bool cr = d.payload == L.create_ref;
            const uint64_t* dw = cr ? cdw : (const uint64_t*)(P.arena + (uint64_t)d.payload * 8);
            uint64_t pre[SER_PRE];
#pragma unroll
            for (int j = 0; j < SER_PRE; j++) pre[j] = cpre[j];
            td_static_pre(P.arena, !cr, d.payload, pre);  // a static blob: through the scalar cache
            const uint32_t at = sh + (rel - lo) + (k ? f0 : 0);
            const uint32_t vl = k ? vl1 : vl0;
            FastWB fw;
            fw.begin(img, at + (FR ? FRAME_PREFIX : 0u), IMG + 16 + 8 * lane);
            fast_encode<L5, true, FR>(fw, d, tab, segs, dw, pre);
            if (fw.n() != vl) bad = 1;  // the formula and the encoder disagree: never silently
            if (FR) {
              const int64_t src = prev0 + (k ? sp1 : sp0);
              const bool pair = G.nrec > 1 && sp0 == sp1;  // (the instance's two records share their source)
              const uint8_t vt = kind_vt(d.kind), rt = kind_rt(d.kind);
              const bool req = vt == ZB_VT_WORKFLOW_INSTANCE && rt == ZB_RT_EVENT && d.intent == WI_CREATED;
              uint64_t h[13];
              frame_words(h, fcst, FRAME_PREFIX + vl, frame_flags(k == 0 || !pair, k == 1 || !pair), G.pos0 + k,
                          frame_producer(src, vt, rt, d.intent), src, d.key, rt, vt, d.intent, 255, 0,
                          req ? rid : ~0ull, req ? sid : 0x80000000u);
              frame_store_lds(img, at, h);
            }
          }
        }
        const uint32_t hi = __builtin_amdgcn_readlane(incl, b - 1);
        TD_PHASE(2);
        wave_lds_sync();
        wave_stream(img, D.out, wbase + lo, sh, hi - lo, lane);
        wave_lds_sync();  // the image is reused by the next round
        TD_PHASE(3);
        a = b;
      }
      if (G.nrec) prev0 = G.pos0;
    }
    };
    const bool lo_ok = P.wf_start + 5 * L.kwf0 >= 65536 && P.log_base + L.inst >= 65536 &&
                       (!D.jobs || P.job_start + 5 * td_kbase(T, L.L, 0, 2) >= 65536);
    if (D.len5_ok && __builtin_amdgcn_readlane(lo_ok ? 1 : 0, 0)) gen_loop(std::true_type{});
    else gen_loop(std::false_type{});
  }
  if (bad) atomicOr(D.flags + 1, 1u);
#ifdef ZB_PHASES
  if (lane == 0 && D.phase) {
    for (int k = 0; k < 4; k++) atomicAdd(D.phase + k, (unsigned long long)ph[k]);
    atomicAdd(D.phase + 4, 1ull);
    atomicAdd(D.phase + 5, (unsigned long long)ph_g);
  }
#endif
#undef TD_PHASE
}

// payload-byte total over the per-workgroup partials
__global__ void __launch_bounds__(256) k_tdrain_sum(TDrainParams D, int64_t nparts) {
  __shared__ unsigned long long s[4];
  unsigned long long x = 0;
  for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < nparts; k += (int64_t)gridDim.x * 256) x += D.pay_part[k];
  for (int dd = 32; dd >= 1; dd >>= 1) x += __shfl_down(x, dd, 64);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = x;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd((unsigned long long*)D.totals + 1, s[0] + s[1] + s[2] + s[3]);
}

// Decides, after the trace and the generation bases, whether the batch may stay deferred: every traced record
// is a WORKFLOW_INSTANCE event or a JOB record other than CANCEL(ED) (the fast encoder's kinds and the value-
// length formula's), no generation merges payloads (the records' payloads are the CREATE payload or static
// blobs), and the host allows it (TrajParams.defer_ok: value segments deployed, ZB_CFG_NO_DEFER).
__global__ void __launch_bounds__(256) k_tmpl_decide(TrajParams P) {
  __shared__ uint32_t s_bad;
  TrajCtl* ctl = P.ctl;
  if (ctl->flag) return;
  if (threadIdx.x == 0) s_bad = 0;
  __syncthreads();
  const uint32_t nc = P.cls ? P.plan->nc : 1;
  for (uint32_t c = 0; c < nc; c++) {
    const uint32_t W = P.wcount[c];
    for (uint32_t w = threadIdx.x; w < W; w += blockDim.x) {
      const uint64_t row = (uint64_t)c * CLS_ROW + w;
      uint32_t bad = P.mgen[row].has ? 1u : 0u;
      const uint32_t nrec = (uint32_t)(P.agg[row] & 0xffff);
      for (uint32_t k = 0; k < nrec && k < (uint32_t)TF; k++) {
        const TmplRec t = P.tmpl[row * TF + k];
        const uint8_t vt = kind_vt(t.kind), rt = kind_rt(t.kind);
        const bool ok = !(t.kind & KIND_RAW) &&
                        ((vt == ZB_VT_WORKFLOW_INSTANCE && rt == ZB_RT_EVENT) ||
                         (vt == ZB_VT_JOB && rt != ZB_RT_COMMAND_REJECTION && (t.intent | 1) != JI_CANCELED)) &&
                        (t.payload == PAY_CREATE || !(t.payload & PAY_MERGE));
        if (!ok) bad = 1;
      }
      if (bad) atomicOr(&s_bad, 1u);
    }
  }
  __syncthreads();
  // the drain keeps the tables in LDS (TD_MAX_GEN, TD_MAX_CW)
  const bool fits = ctl->wmax <= TD_MAX_GEN && nc * ctl->wmax <= TD_MAX_CW;
  if (threadIdx.x == 0) ctl->defer = (s_bad || !fits || !P.defer_ok) ? 0u : 1u;
}

void launch_tmpl_decide(const TrajParams& p, hipStream_t s) {
  hipLaunchKernelGGL(k_tmpl_decide, dim3(1), dim3(256), 0, s, p);
}

void launch_tdrain_size(const TDrainParams& d, uint32_t wg0, hipStream_t s) {
  if (wg0 && d.frames) hipLaunchKernelGGL(k_tdrain_size<true>, dim3(wg0), dim3(TD_WG), td_layout(d, false).total, s, d);
  else if (wg0) hipLaunchKernelGGL(k_tdrain_size<false>, dim3(wg0), dim3(TD_WG), td_layout(d, false).total, s, d);
  const uint64_t rest = (uint64_t)d.t.nwg - wg0;
  if (rest) hipLaunchKernelGGL(k_tdrain_sizes, dim3((unsigned)((rest + 255) / 256)), dim3(256), 0, s, d, wg0);
}
void launch_tdrain_write(const TDrainParams& d, hipStream_t s) {
  if (d.frames)
    hipLaunchKernelGGL((k_tdrain_write<TD_IMG, true>), dim3((unsigned)d.t.nwg), dim3(TD_WG), td_layout(d, true).total, s, d);
  else
    hipLaunchKernelGGL((k_tdrain_write<TD_IMG, false>), dim3((unsigned)d.t.nwg), dim3(TD_WG), td_layout(d, true).total, s, d);
  hipLaunchKernelGGL(k_tdrain_sum, dim3((unsigned)std::min<int64_t>(256, (d.t.nwg + 255) / 256)), dim3(256), 0, s, d,
                     (int64_t)d.t.nwg);
}

}  // namespace zbg
