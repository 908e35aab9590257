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
//   k_tdrain_write  the same lanes again: headers of the wave's records, values encoded with the fast encoder
//                   (zb_fastenc.hpp) into the wave's LDS image and streamed out with 16-byte stores
// The CREATE payload -- the payload of every record the instance writes -- is read once per lane, not once per
// record. Anything else (zb_step, frames, descriptors, a partial range, compaction) materializes the batch
// first with k_tmpl, so every other API sees the descriptors it always saw.
#include <hip/hip_runtime.h>

#include "zb_fastenc.hpp"
#include "zb_tmpl.hpp"

namespace zbg {

constexpr int TD_WG = TRAJ_WG;  // 256 lanes = 256 instances, four waves
constexpr uint32_t TD_IMG = 6 * 1024 - 16;  // per-wave image: 6 KB slices, four per workgroup (+ the model)

// one instance's generation w: log position and key bases (linear in the class ranks), record count
struct TdGen {
  int64_t pos0, kwf, kjob;
  uint32_t nrec;
};
__device__ __forceinline__ TdGen td_gen(const TrajParams& P, const TmplLane& L, uint32_t crow, int w, bool live) {
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
  TdGen G;
  G.pos0 = wb.pos + po;
  G.kwf = wb.wf + pw;
  G.kjob = wb.job + pj;
  G.nrec = live ? (uint32_t)(P.agg[(uint64_t)crow + w] & 0xffff) : 0;
  return G;
}
// record k of the instance's generation w, resolved from the class trace; *vl: its value length (the
// encoder's, by the formula), *plen: its payload document's length
__device__ __forceinline__ zb_rec td_record(const TrajParams& P, const TmplLane& L, uint32_t crow, int w, uint32_t k,
                                            const TdGen& G, int64_t inst, uint32_t create_ref, uint32_t create_len,
                                            uint32_t& vl, uint32_t& plen) {
  const TmplRec t = P.tmpl[((uint64_t)crow + w) * TF + k];
  zb_rec d;
  d.key = tmpl_key(P, L, t.key, (uint32_t)w, G.kwf, G.kjob);
  d.scope_key = t.scope == SYM_CMDPOS ? P.log_base + inst : tmpl_key(P, L, t.scope, (uint32_t)w, G.kwf, G.kjob);
  d.inst_key = tmpl_key(P, L, t.inst, (uint32_t)w, G.kwf, G.kjob);
  // (k_tmpl_decide: no merge results in a deferred batch -- the CREATE payload or a static blob)
  const bool cr = t.payload == PAY_CREATE;
  d.payload = cr ? create_ref : t.payload;
  plen = cr ? create_len : arena_len(P.arena, d.payload);
  d.elem = t.elem; d.intent = t.intent; d.kind = t.kind;
  const ValueConst vc = kload(P.vconst, (uint64_t)d.elem);
  vl = (kind_vt(d.kind) == ZB_VT_JOB ? vc.job : vc.wf) + mp_int_len(d.inst_key) + mp_int_len(d.scope_key) +
       mp_bin_len(plen);
  return d;
}

// lane setup shared by both passes: class, ranks, CREATE payload
struct TdLane {
  TmplLane L;
  uint32_t crow, W, create_ref, create_len;
  int64_t inst;
  bool active;
};
__device__ __forceinline__ TdLane td_lane(const TrajParams& P) {
  TdLane t;
  t.inst = (int64_t)blockIdx.x * TD_WG + threadIdx.x;
  t.active = t.inst < P.n;
  if (!t.active) t.inst = P.n - 1;  // (follows the last instance, writes nothing)
  uint32_t cls = 0;
  if (P.cls) {
    t.L.ncls = __builtin_amdgcn_readfirstlane(P.plan->nc);
    cls = tmpl_lane_io(P, t.inst, t.L);
  } else {
    t.L.ncls = 1;
#pragma unroll
    for (int c = 0; c < CLS_MAX; c++) t.L.before[c] = c == 0 ? (uint32_t)t.inst : 0;
  }
  t.crow = cls * CLS_ROW;
  t.W = t.active ? P.wcount[cls] : 0;
  t.create_ref = P.log[P.log_base + t.inst].payload;
  t.create_len = arena_len(P.arena, t.create_ref);
  return t;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
  return x;
}

__global__ void __launch_bounds__(TD_WG) k_tdrain_size(TDrainParams D) {
  const TrajParams& P = D.t;
  const TdLane T = td_lane(P);
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * (TD_WG / 64) + (threadIdx.x >> 6);
  uint64_t pay = 0;
#pragma unroll 1
  for (int w = 0; w < (int)D.wmax; w++) {
    const TdGen G = td_gen(P, T.L, T.crow, w, w < (int)T.W);
    uint32_t mine = 0;
#pragma unroll 1
    for (uint32_t k = 0; k < G.nrec; k++) {
      uint32_t vl, plen;
      (void)td_record(P, T.L, T.crow, w, k, G, T.inst, T.create_ref, T.create_len, vl, plen);
      mine += vl;
      pay += plen;
    }
    const uint32_t b = wave_sum(mine);
    if (lane == 0) D.wbytes[(uint64_t)w * D.nwave + wave] = b;
  }
  // payload bytes of the drained records (zb_serialize_stats.payload_bytes): one partial per workgroup
  __shared__ unsigned long long s_pay[TD_WG / 64];
  unsigned long long y = pay;
  for (int d = 32; d >= 1; d >>= 1) y += __shfl_down(y, d, 64);
  if (lane == 0) s_pay[threadIdx.x >> 6] = y;
  __syncthreads();
  if (threadIdx.x == 0) D.pay_part[blockIdx.x] = s_pay[0] + s_pay[1] + s_pay[2] + s_pay[3];
}

// LDS writes of other lanes of the wave are visible to this lane's later reads (and the reverse)
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// image bytes [shift, shift + n) -> out[o, o + n): 16-byte non-temporal stores aligned to the destination,
// bytes at the two ends (shared with the neighbouring ranges) one at a time
__device__ __forceinline__ void wave_stream(const uint8_t* img, uint8_t* out, uint64_t o, uint32_t shift, uint32_t n,
                                            int lane) {
  uint8_t* dst = out + o - shift;
  const uint32_t lim = shift + n;
  const uint32_t full_lo = (shift + 15) & ~15u, full_hi = lim & ~15u;
  for (uint32_t c = full_lo + 16 * lane; c < full_hi; c += 16 * 64) {
    const uint4 v = *(const uint4*)(img + c);
    __builtin_nontemporal_store(v.x, (uint32_t*)(dst + c));
    __builtin_nontemporal_store(v.y, (uint32_t*)(dst + c) + 1);
    __builtin_nontemporal_store(v.z, (uint32_t*)(dst + c) + 2);
    __builtin_nontemporal_store(v.w, (uint32_t*)(dst + c) + 3);
  }
  const uint32_t head_end = full_lo < lim ? full_lo : lim;
  for (uint32_t c = shift + lane; c < head_end; c += 64) dst[c] = img[c];
  const uint32_t tail_lo = full_hi > head_end ? full_hi : head_end;
  for (uint32_t c = tail_lo + lane; c < lim; c += 64) dst[c] = img[c];
}

__global__ void __launch_bounds__(TD_WG) __attribute__((amdgpu_waves_per_eu(4, 4))) k_tdrain_write(TDrainParams D) {
  __shared__ __attribute__((aligned(16))) uint8_t s_img[TD_WG / 64][TD_IMG + 16];
  extern __shared__ __attribute__((aligned(16))) uint8_t s_model[];  // the constant runs (sized at launch)
  const TrajParams& P = D.t;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t wave = (uint64_t)blockIdx.x * (TD_WG / 64) + wv;
  const TdLane T = td_lane(P);
  // the CREATE payload's first words (length + 44 bytes), once per instance
  const uint64_t* cdw = (const uint64_t*)(P.arena + (uint64_t)T.create_ref * 8);
  uint64_t cpre[SER_PRE];
#pragma unroll
  for (int j = 0; j < SER_PRE; j++)
    cpre[j] = (uint64_t)T.create_ref * 8 + 8 * j + 8 <= P.arena_cap ? cdw[j] : 0;
  // the elements' constant runs into LDS: table (4-byte words), pool (8-byte words)
  const uint32_t tb = ((uint32_t)D.n_elems * (uint32_t)sizeof(DevValSeg) + 15) & ~15u;
  for (uint32_t c = threadIdx.x; c < tb / 4; c += TD_WG) ((uint32_t*)s_model)[c] = ((const uint32_t*)D.vsegs)[c];  // (padded)
  for (uint32_t c = threadIdx.x; c < D.segpool_len / 8; c += TD_WG)
    ((uint64_t*)(s_model + tb))[c] = ((const uint64_t*)D.segpool)[c];
  __syncthreads();
  const DevValSeg* tab = (const DevValSeg*)s_model;
  const uint8_t* segs = s_model + tb;
  uint8_t* img = s_img[wv];
  uint32_t bad = 0;
  int64_t hdr_key[TF];
  uint32_t hdr_meta[TF], hdr_len[TF];
#pragma unroll 1
  for (int w = 0; w < (int)D.wmax; w++) {
    const uint64_t wbase = D.woffs[(uint64_t)w * D.nwave + wave];
    const uint64_t wend = D.woffs[(uint64_t)w * D.nwave + wave + 1];
    if (wend == wbase) continue;  // (uniform: no record of this wave in generation w)
    const TdGen G = td_gen(P, T.L, T.crow, w, w < (int)T.W);
    uint32_t mine = 0;
#pragma unroll 1
    for (uint32_t k = 0; k < G.nrec; k++) {  // value lengths first (the wave's offsets), headers with them
      uint32_t vl, plen;
      const zb_rec d = td_record(P, T.L, T.crow, w, k, G, T.inst, T.create_ref, T.create_len, vl, plen);
      hdr_key[k & 1] = d.key;  // (TF == 2)
      hdr_meta[k & 1] = (uint32_t)kind_rt(d.kind) | (uint32_t)kind_vt(d.kind) << 8 | (uint32_t)d.intent << 16 |
                        255u << 24;  // (k_tmpl_decide: no rejections in a deferred batch)
      hdr_len[k & 1] = vl;
      mine += vl;
    }
    uint32_t incl = mine;
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
      const uint32_t y = __shfl_up(incl, k, 64);
      if (lane >= k) incl += y;
    }
    const uint64_t off = wbase + incl - mine;  // this lane's values: [off, off + mine)
    if (wend > D.out_cap) {  // does not fit: the host grows the buffer and runs the pass again
      if (lane == 0) atomicOr(D.flags, 1u);
      continue;
    }
    // headers (position implicit: start + index): key, types / intent / rejection, length, offset
    uint64_t hoff = off;
#pragma unroll 1
    for (uint32_t k = 0; k < G.nrec; k++) {
      uint64_t* dh = (uint64_t*)(D.headers + (G.pos0 + k - D.start));
      __builtin_nontemporal_store((uint64_t)hdr_key[k & 1], dh);
      __builtin_nontemporal_store((uint64_t)hdr_meta[k & 1] | (uint64_t)hdr_len[k & 1] << 32, dh + 1);
      __builtin_nontemporal_store(hoff, dh + 2);
      hoff += hdr_len[k & 1];
    }
    // windows of whole lanes that fit the image, in lane order (the lanes' ranges are consecutive)
    bool done = mine == 0;
    if (!done && mine + 16 > TD_IMG) {  // one instance's records exceed the image: the host takes the generic path
      bad = 1;
      done = true;
    }
#pragma unroll 1
    while (true) {
      const uint64_t pend = __ballot(!done);
      if (!pend) break;
      const int first = __ffsll((unsigned long long)pend) - 1;
      const uint64_t wlo = __shfl(off, first, 64);
      const uint32_t sh = (uint32_t)(((uintptr_t)(D.out + wlo)) & 15);
      const bool go = !done && (off + mine - wlo) + sh <= TD_IMG;
      uint64_t hi = go ? off + mine : 0;
      for (int d = 32; d >= 1; d >>= 1) {
        const uint64_t y = (uint64_t)__shfl_xor((unsigned long long)hi, d, 64);
        hi = y > hi ? y : hi;
      }
      if (go) {
        uint32_t at = sh + (uint32_t)(off - wlo);
#pragma unroll 1
        for (uint32_t k = 0; k < G.nrec; k++) {
          uint32_t vl, plen;
          const zb_rec d = td_record(P, T.L, T.crow, w, k, G, T.inst, T.create_ref, T.create_len, vl, plen);
          const bool cr = d.payload == T.create_ref;  // else a static blob (shared by every instance: cached)
          const uint64_t* dw = (const uint64_t*)(P.arena + (uint64_t)d.payload * 8);
          uint64_t pre[SER_PRE];
#pragma unroll
          for (int j = 0; j < SER_PRE; j++)
            pre[j] = cr ? cpre[j] : ((uint64_t)d.payload * 8 + 8 * j + 8 <= P.arena_cap ? dw[j] : 0);
          FastW fw;
          fw.begin(img, at);
          fast_encode(fw, d, tab, segs, dw, pre);
          if (fw.n() != vl) bad = 1;  // the formula and the encoder disagree: never silently
          at += vl;
        }
      }
      wave_lds_sync();
      wave_stream(img, D.out, wlo, sh, (uint32_t)(hi - wlo), lane);
      wave_lds_sync();  // the image is reused by the next window
      done = done || go;
    }
  }
  if (bad) atomicOr(D.flags + 1, 1u);
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
// blobs), and the host allows it (TrajParams.defer_ok: value segments deployed, ZB_TMPL_DEFER).
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
  if (threadIdx.x == 0) ctl->defer = (s_bad || !P.defer_ok) ? 0u : 1u;
}

void launch_tmpl_decide(const TrajParams& p, hipStream_t s) {
  hipLaunchKernelGGL(k_tmpl_decide, dim3(1), dim3(256), 0, s, p);
}

uint32_t tdrain_lds_bytes(const TDrainParams& d) {
  return (((uint32_t)d.n_elems * (uint32_t)sizeof(DevValSeg) + 15) & ~15u) + d.segpool_len;
}
void launch_tdrain_size(const TDrainParams& d, hipStream_t s) {
  hipLaunchKernelGGL(k_tdrain_size, dim3((unsigned)d.t.nwg), dim3(TD_WG), 0, s, d);
}
void launch_tdrain_write(const TDrainParams& d, hipStream_t s) {
  hipLaunchKernelGGL(k_tdrain_write, dim3((unsigned)d.t.nwg), dim3(TD_WG), tdrain_lds_bytes(d), s, d);
  hipLaunchKernelGGL(k_tdrain_sum, dim3((unsigned)std::min<int64_t>(256, (d.t.nwg + 255) / 256)), dim3(256), 0, s, d,
                     (int64_t)d.t.nwg);
}

}  // namespace zbg
