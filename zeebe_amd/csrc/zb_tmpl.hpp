// zb_tmpl.hpp — resolving a traced class trajectory (TmplRec) for one instance: shared by the template emit
// (k_tmpl, zb_traj.hip), which writes the records as descriptors, and the template drain (zb_tdrain.hip),
// which encodes them straight into record values + headers.
#pragma once
#include <hip/hip_runtime.h>

#include "zb_kernels.hpp"

namespace zbg {

// Read-only tables (the deployed model; per-generation bases written by earlier launches) accessed
// through the constant address space: with a wave-uniform index (every control decision of a
// uniform batch) the backend emits scalar loads (s_load, scalar cache) instead of vector loads on
// the generation loop's dependence chain.
template <class T>
using cptr = const T __attribute__((address_space(4)))*;
template <class T>
__device__ __forceinline__ cptr<T> K(const T* p) { return (cptr<T>)p; }
// element i of a read-only array of dword-multiple structs through the constant address space
template <class T>
__device__ __forceinline__ T kload(const T* p, uint64_t i) {
  static_assert(sizeof(T) % 4 == 0, "dword-multiple struct");
  T out;
  const cptr<uint32_t> src = (cptr<uint32_t>)(p + i);
  uint32_t* d = (uint32_t*)&out;
#pragma unroll
  for (int k = 0; k < (int)(sizeof(T) / 4); k++) d[k] = src[k];
  return out;
}

// Keys inside a trajectory are 32-bit ordinals of the partition's generators within the batch:
// wf key = wf_start + 5 * ordinal, job key = job_start + 5 * ordinal (every key a batch record
// carries is created by the batch); NOK stands for the null key -1.
constexpr uint32_t NOK = 0xffffffffu;
constexpr uint32_t JOB_ZERO = 0xfffffffeu;  // row job key 0 (no job created yet)
// symbolic keys of a trace (TmplRec): tag | generation << 4 | ordinal
constexpr uint32_t SYMK_WF = 0x80000000u, SYMK_JOB = 0x40000000u;
constexpr uint32_t SYM_CMDPOS = 0xfffffffdu;

__device__ __forceinline__ uint32_t arena_len(const uint8_t* arena, uint32_t ref) {
  return *(const uint32_t*)(arena + (uint64_t)ref * 8);
}

// symbolic payload refs of a trace (literal refs are static blobs below 2^28)
constexpr uint32_t PAY_MERGE = 0x80000000u;   // | generation: that generation's merge result
constexpr uint32_t PAY_CREATE = 0xC0000000u;  // the instance's CREATE payload

// Uniform and class batches: every instance of class c follows the traced trajectory of c (TmplRec,
// symbolic), so the emit pass instantiates it instead of stepping the state machine again: per
// generation (a scalar loop) the instance's log position and key bases are linear in before_c(i).
struct TmplLane {
  uint32_t before[CLS_MAX];
  uint32_t ncls;
};
// key ordinal base of generation g for this instance: wf (f = 1) or job (f = 2) counter
__device__ __forceinline__ int64_t tmpl_kbase(const TrajParams& P, const TmplLane& L, uint32_t g, int f) {
  const TrajBase wb = kload(P.wbase, (uint64_t)g);
  int64_t k = f == 1 ? wb.wf : wb.job;
#pragma unroll
  for (int c = 0; c < CLS_MAX; c++) {
    if (c >= (int)L.ncls) break;
    const uint64_t n = kload(P.agg, (uint64_t)c * CLS_ROW + g);
    k += (int64_t)L.before[c] * (int64_t)(f == 1 ? ((n >> 16) & 0xffff) : (n >> 32));
  }
  return k;
}
// arena byte offset of this instance's merge slot of generation g
__device__ __forceinline__ uint64_t tmpl_mslot(const TrajParams& P, const TmplLane& L, uint32_t g) {
  int64_t pm = kload(P.wbase, (uint64_t)g).mbase;
#pragma unroll
  for (int c = 0; c < CLS_MAX; c++) {
    if (c >= (int)L.ncls) break;
    const MergeGen m = kload(P.mgen, (uint64_t)c * CLS_ROW + g);
    if (m.has) pm += (int64_t)L.before[c] * (int64_t)m.stride;
  }
  return (uint64_t)pm;
}
// a symbolic key: -1, or the partition key of the ordinal-th key created in its generation
__device__ __forceinline__ int64_t tmpl_key(const TrajParams& P, const TmplLane& L, uint32_t sym, uint32_t w,
                                            int64_t kwf, int64_t kjob) {
  if (sym == NOK) return -1;
  if (sym == JOB_ZERO) return 0;
  const uint32_t g = (sym >> 4) & 0xfff, ord = sym & 15;
  if (sym & SYMK_WF) return P.wf_start + 5 * ((g == w ? kwf : tmpl_kbase(P, L, g, 1)) + ord);
  return P.job_start + 5 * ((g == w ? kjob : tmpl_kbase(P, L, g, 2)) + ord);
}

// Instance-order lanes of a class batch (lane = instance, as the log orders every generation): the class of
// instance `inst` and, per class c, the class-c instances before it -- its workgroup's offset (k_cls_scan),
// the waves of the workgroup before it, the lanes of its wave before it.
__device__ __forceinline__ uint32_t tmpl_lane_io(const TrajParams& P, int64_t inst, TmplLane& L) {
  uint32_t cls = 0;
  const uint64_t grp = (uint64_t)(inst >> 6) * CLS_MAX;
  const uint64_t wg = (uint64_t)(inst / TRAJ_WG), grp0 = wg * (TRAJ_WG / 64) * CLS_MAX;
  const int wvi = (int)((inst % TRAJ_WG) >> 6);
  const uint32_t bit = (uint32_t)(inst & 63);
  const uint64_t lt = (1ull << bit) - 1;
#pragma unroll
  for (int c = 0; c < CLS_MAX; c++) {
    if (c >= (int)L.ncls) { L.before[c] = 0; continue; }
    const uint64_t m = P.cmask[grp + c];
    uint32_t off = P.wgoff[(uint64_t)c * P.nwg + wg];
    for (int v = 0; v < wvi; v++) off += (uint32_t)__builtin_popcountll(P.cmask[grp0 + (uint64_t)v * CLS_MAX + c]);
    L.before[c] = off + (uint32_t)__builtin_popcountll(m & lt);
    if ((m >> bit) & 1) cls = (uint32_t)c;
  }
  return cls;
}

}  // namespace zbg
