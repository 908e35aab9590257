// zb_aux.hip — the two payload kernels that run between waves, off the state-machine kernel:
//   k_merge: default output merges reserved by k_wave (OutputMappingHandler :42-85 ->
//            MappingProcessor.merge, json-path/.../mapping/MappingProcessor.java:143-170)
//   k_cond:  exclusive-gateway condition evaluation for GATEWAY_ACTIVATED records emitted by the
//            wave (ExclusiveSplitHandler :38-71 -> JsonConditionInterpreter.eval); the decision is
//            a pure function of (gateway, payload), both fixed when the record is written, so
//            evaluating right after the writing wave is the same as at processing time.
// Both walk a compact job list (one entry per merge / split) with a grid-stride loop, so their
// register-heavy byte parsers never limit the occupancy of k_wave.
#include <hip/hip_runtime.h>

#include "zb_devlib.hpp"
#include "zb_kernels.hpp"

namespace zbg {

// sum over the 256 threads of a workgroup, valid in thread 0 (statistics: one device atomic per workgroup
// instead of one per thread -- same-address device atomics serialise)
__device__ __forceinline__ unsigned long long wg_sum256(unsigned long long x, unsigned long long* s4) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_down(x, d, 64);
  if ((threadIdx.x & 63) == 0) s4[threadIdx.x >> 6] = x;
  __syncthreads();
  const unsigned long long t = s4[0] + s4[1] + s4[2] + s4[3];
  __syncthreads();
  return t;
}

__global__ void __launch_bounds__(256) k_merge(WaveParams P) {
  __shared__ unsigned long long s4[4];
  const uint32_t n = P.merge_count[P.wave & 1];
  const MergeJob* jobs = P.merge_jobs + (uint64_t)(P.wave & 1) * P.job_cap;
  uint32_t err = 0;
  unsigned long long merges = 0, bytes = 0;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const MergeJob j = jobs[i];
    const uint8_t* sp = P.arena + (uint64_t)j.src * 8;
    const uint8_t* tp = P.arena + (uint64_t)j.tgt * 8;
    const uint32_t ns = *(const uint32_t*)sp, nt = *(const uint32_t*)tp;
    uint8_t* dst = P.arena + (uint64_t)j.dst * 8;
    Out o{dst + 4, 0};
    bool unsup = false;
    if (!merge_docs(sp + 4, ns, tp + 4, nt, o, unsup)) err |= DE_BAD_PAYLOAD;
    else if (unsup || o.n > j.cap) err |= DE_UNSUPPORTED;
    *(uint32_t*)dst = o.n;
    merges += 1;
    bytes += ns + nt + o.n;
  }
  if (err) atomicOr(P.err, err);
  merges = wg_sum256(merges, s4);
  bytes = wg_sum256(bytes, s4);
  if (threadIdx.x == 0 && merges) {
    atomicAdd((unsigned long long*)&P.stats[3], merges);
    atomicAdd((unsigned long long*)&P.stats[4], bytes);
  }
}

__global__ void __launch_bounds__(256) k_cond(WaveParams P) {
  __shared__ unsigned long long s4[4];
  const uint32_t n = P.cond_count[P.wave & 1];
  const uint64_t* jobs = P.cond_jobs + (uint64_t)(P.wave & 1) * P.job_cap;
  unsigned long long bytes = 0;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint64_t r = jobs[i];
    const zb_rec rec = P.log[r];
    const DevElem& el = P.elems[rec.elem];
    const uint8_t* pp = P.arena + (uint64_t)rec.payload * 8;
    const uint32_t len = *(const uint32_t*)pp;
    const uint8_t* doc = pp + 4;
    uint32_t dec = COND_VALID;
    uint16_t chosen = NO_ELEM;
    CondOut co{0, 0, 0, 0};
    bool unsup = false;
    for (uint32_t c = 0; c < el.cond_count; c++) {
      const uint16_t flow = P.cond_flows[el.cond_begin + c];
      const bool res =
          eval_condition(P.elems[flow].cond_prog, P.code, doc, len, P.consts, P.queries, P.filters, P.pool, co, unsup);
      if (unsup || co.err) break;
      if (res) { chosen = flow; break; }
    }
    bytes += len;
    if (unsup) dec |= COND_UNSUPPORTED;
    else if (co.err)
      dec |= COND_INCIDENT | ((uint32_t)(co.err & 7) << 27) | ((uint32_t)(co.a & 15) << 23) |
             ((uint32_t)(co.b & 15) << 19) | co.q;
    else {
      if (chosen == NO_ELEM) chosen = el.dflt;
      if (chosen == NO_ELEM) dec |= COND_INCIDENT | ((uint32_t)EC_NO_FLOW << 27);
      else dec |= chosen;
    }
    uint32_t* link = (uint32_t*)(P.links + r);
    link[0] = dec;  // row-self half of the link; the scope half stays
  }
  bytes = wg_sum256(bytes, s4);
  if (threadIdx.x == 0 && bytes) atomicAdd((unsigned long long*)&P.stats[5], bytes);
}

void launch_merge(const WaveParams& p, hipStream_t s) {
  hipLaunchKernelGGL(k_merge, dim3(1024), dim3(256), 0, s, p);
}
void launch_cond(const WaveParams& p, hipStream_t s) {
  hipLaunchKernelGGL(k_cond, dim3(1024), dim3(256), 0, s, p);
}

}  // namespace zbg
