// zb_aux.hip — the payload kernels that run around a wave, off the state-machine kernel:
//   k_map:   explicit io-mappings of the records a wave is about to process (below)
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
#include "zb_xlock.hpp"

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

// the ELEMENT_COMPLETED record carrying a merge result: its value length hint
__device__ __forceinline__ void merge_hint(const WaveParams& P, const MergeJob& j, uint32_t olen) {
  if (j.pos >= 0 && (uint64_t)j.pos < P.log_cap && P.vconst) {  // (a slot past the window was not written)
    const zb_rec d = P.log[j.pos];
    const ValueConst vc = P.vconst[d.elem];
    P.vlen[j.pos] = vc.wf + mp_int_len(d.inst_key) + mp_int_len(d.scope_key) + mp_bin_len(olen);
  }
}

// The wave's default output merges (OutputMappingHandler.java:42-85 -> MappingProcessor.merge), in two
// kernels: k_merge takes every merge of flat documents (merge_flat: scalar values under fixstr keys, the payload
// shape of nearly every workflow) -- small in registers and without a workspace, so the job list streams at full
// occupancy -- and queues the rest for k_merge_gen, the general indexer / merger (merge_docs, a per-thread node
// workspace), which for most waves finds its queue empty.
// small documents are merged in an LDS copy: the flat merge re-reads its documents byte by byte, and a byte read
// from LDS costs a fraction of one from global memory (the workflows' payloads are a few keys: C2's merges are
// {orderId, step} documents of ~20 bytes)
constexpr int KM_WORDS = 12;                 // 48-byte document slots: documents of <= 44 bytes
constexpr int KM_STRIDE = 3 * KM_WORDS + 1;  // source, target, result; odd stride: distinct banks per lane

__global__ void __launch_bounds__(256) k_merge(WaveParams P) {
  __shared__ unsigned long long s4[4];
  __shared__ uint32_t s_m[256 * KM_STRIDE];
  if (wave_void(P)) return;
  const uint32_t n = (uint32_t)std::min<uint64_t>(P.merge_count[P.wave & 1], P.job_cap);
  const MergeJob* jobs = P.merge_jobs + (uint64_t)(P.wave & 1) * P.job_cap;
  uint32_t* slow_n = P.merge_slow_count + (P.wave & 1);
  uint32_t* reg = s_m + threadIdx.x * KM_STRIDE;
  unsigned long long merges = 0, bytes = 0;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const MergeJob j = jobs[i];
    const uint32_t* gs = (const uint32_t*)(P.arena + (uint64_t)j.src * 8);
    const uint32_t* gt = (const uint32_t*)(P.arena + (uint64_t)j.tgt * 8);
    const uint32_t ns = gs[0], nt = gt[0];
    uint8_t* dst = P.arena + (uint64_t)j.dst * 8;
    uint32_t olen = 0;
    bool done;
    if (ns + nt + 3 <= 4 * KM_WORDS - 4) {  // (the result is at most ns + nt + 3 bytes)
      for (uint32_t k = 0; k < (ns + 7) / 4; k++) reg[k] = gs[k];
      for (uint32_t k = 0; k < (nt + 7) / 4; k++) reg[KM_WORDS + k] = gt[k];
      uint8_t* lo = (uint8_t*)(reg + 2 * KM_WORDS);
      done = merge_flat((const uint8_t*)reg + 4, ns, (const uint8_t*)(reg + KM_WORDS) + 4, nt, lo + 4,
                        4 * KM_WORDS - 4, olen);
      if (done) {
        reg[2 * KM_WORDS] = olen;
        for (uint32_t k = 0; k < (olen + 7) / 4; k++) ((uint32_t*)dst)[k] = reg[2 * KM_WORDS + k];
      }
    } else {
      done = merge_flat((const uint8_t*)gs + 4, ns, (const uint8_t*)gt + 4, nt, dst + 4, j.cap, olen);
      if (done) *(uint32_t*)dst = olen;
    }
    if (done) {
      merge_hint(P, j, olen);
      merges += 1;
      bytes += ns + nt + olen;
    } else {
      P.merge_slow[atomicAdd(slow_n, 1u)] = i;
    }
  }
  merges = wg_sum256(merges, s4);
  bytes = wg_sum256(bytes, s4);
  if (threadIdx.x == 0 && merges) {
    atomicAdd((unsigned long long*)&P.stats[3], merges);
    atomicAdd((unsigned long long*)&P.stats[4], bytes);
  }
}

__global__ void __launch_bounds__(256) k_merge_gen(WaveParams P) {
  __shared__ unsigned long long s4[4];
  const uint32_t n = P.merge_slow_count[P.wave & 1];
  const MergeJob* jobs = P.merge_jobs + (uint64_t)(P.wave & 1) * P.job_cap;
  if (blockIdx.x == 0 && threadIdx.x == 0) P.merge_slow_count[(P.wave + 1) & 1] = 0;  // the next wave's queue
  if (n == 0 || wave_void(P)) return;
  uint32_t err = 0;
  unsigned long long merges = 0, bytes = 0;
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) {
    const MergeJob j = jobs[P.merge_slow[q]];
    const uint8_t* sp = P.arena + (uint64_t)j.src * 8;
    const uint8_t* tp = P.arena + (uint64_t)j.tgt * 8;
    const uint32_t ns = *(const uint32_t*)sp, nt = *(const uint32_t*)tp;
    uint8_t* dst = P.arena + (uint64_t)j.dst * 8;
    Out o{dst + 4, 0};
    bool unsup = false;
    const bool ok = merge_docs(sp + 4, ns, tp + 4, nt, o, unsup);
    // the shapes merge_docs refuses (and documents it cannot read, which the reference's indexer reads up to the
    // first bad token) take the exact tree
    uint32_t olen = o.n;
    // (|result| <= ns + nt + 3 <= cap for every document merge_docs takes; a first pass past the blob would already
    // have overwritten its neighbour, so it fails the partition instead of going on through the exact tree)
    if (o.n > j.cap) err |= DE_UNSUPPORTED;
    x_run(XSlabs{P.xslab, P.xlocks, P.xlane}, (!ok || unsup) && o.n <= j.cap, [&](const XWs& ws, bool fin) {
      Out w{dst + 4, 0};
      const int st = x_merge(ws, sp + 4, ns, tp + 4, nt, w, j.cap);
      if (st == X_UNSUP && !fin) return st;
      if (st == X_OK) {
        if (w.n == 1 && dst[4] == 0xc0) dst[4] = 0x80;  // an empty tree: DocumentValue.wrap turns nil into {}
        olen = w.n;
      } else {
        // X_NOT_MAP (a non-map root) would be an incident, which a merge k_wave already emitted cannot become
        err |= st == X_FAIL ? DE_BAD_PAYLOAD : DE_UNSUPPORTED;
      }
      return st;
    });
    *(uint32_t*)dst = olen;
    merge_hint(P, j, olen);
    merges += 1;
    bytes += ns + nt + olen;
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
  if (wave_void(P)) return;
  const uint32_t n = (uint32_t)std::min<uint64_t>(P.cond_count[P.wave & 1], P.job_cap);
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

// k_map: explicit io-mappings of the chunk's records, before the wave processes them (InputMappingHandler
// :39-70 -> MappingProcessor.extract; OutputMappingHandler :42-85 -> MappingProcessor.merge with the element's
// output mappings, or with none into {} for outputBehavior overwrite). One thread per record of the chunk (plus
// the batch tails that reach past its end); a READY / COMPLETING record of a mapped element that will pass its
// guard gets its result document in a fresh arena blob (size pass, one 8-byte atomic on the wave header's
// arena pointer, write pass) or the MappingException that becomes its IO_MAPPING_ERROR incident; k_process
// reads the outcome from mapres. The guard and the flow scope's payload are read before the wave changes
// anything, which is what the record's own turn in log order sees: only the record's own thread changes its
// row, and a flow scope's value changes only with records of the scope itself.
__global__ void __launch_bounds__(256) k_map(WaveParams P) {
  WaveHdr* hin = P.hdr + (P.wave & 1);
  const int64_t b = hin->begin, g = gen_limit(P, hin);
  const int64_t cend = chunk_end(P, b, g);
  const int64_t lim = cend + 3 < g ? cend + 3 : g;  // a batch's tail may lie past the chunk end
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  MNode* ws = P.map_ws + tid * MAP_NODES;
  uint32_t err = 0;
  for (int64_t r = b + (int64_t)tid; r < lim; r += (int64_t)gridDim.x * blockDim.x) {
    uint64_t res = 0;
    const zb_rec rec = P.log[r];
    if (kind_vt(rec.kind) == ZB_VT_WORKFLOW_INSTANCE && kind_rt(rec.kind) == ZB_RT_EVENT && rec.elem != NO_ELEM) {
      const DevElem& el = P.elems[rec.elem];
      const uint8_t ob = (el.flags >> OB_SHIFT) & 3;
      const bool in = rec.intent == WI_ELEMENT_READY && el.n_in && el.step[WI_ELEMENT_READY] == ST_APPLY_INPUT_MAPPING;
      const bool out = rec.intent == WI_ELEMENT_COMPLETING && el.step[WI_ELEMENT_COMPLETING] == ST_APPLY_OUTPUT_MAPPING &&
                       (el.n_out_map || ob == OB_OVERWRITE);
      const uint64_t lk = P.links[r];
      const uint32_t rself = (uint32_t)lk, rscope = (uint32_t)(lk >> 32);
      if ((in || out) && rself != NO_ROW && P.rmeta[rself].state == rec.intent && (in || rscope != NO_ROW)) {
        const uint8_t* sp = P.arena + (uint64_t)rec.payload * 8;
        const uint32_t ns = *(const uint32_t*)sp;
        const uint8_t* tp = nullptr;
        uint32_t nt = 0;
        if (out) {
          tp = P.arena + (ob == OB_OVERWRITE ? 0 : (uint64_t)P.rmeta[rscope].payload * 8);  // ref 0: {}
          nt = *(const uint32_t*)tp;
          tp += 4;
        }
        const uint16_t first = in ? el.map_in : el.map_out;
        const uint32_t nm = in ? el.n_in : el.n_out_map;
        uint16_t fq = 0;
        int st;
        Out o{nullptr, 0};
        bool unsup = false;
        if (nm) st = map_documents(sp + 4, ns, tp, nt, P.maps + first, nm, P.segs, P.queries, P.filters, P.pool, ws, o, fq);
        else st = !merge_docs(sp + 4, ns, tp, nt, o, unsup) ? MAP_UNSUPPORTED : (unsup ? MAP_UNSUPPORTED : MAP_OK);
        // what the node-table mapper / structural merge refuse: the exact tree, size pass, arena, write pass
        x_run(XSlabs{P.xslab, P.xlocks, P.xlane}, st == MAP_UNSUPPORTED, [&](const XWs& ws, bool fin) {
          Out z{nullptr, 0};
          uint16_t xq = 0;
          int xs = nm ? x_map(ws, sp + 4, ns, tp, nt, P.maps + first, nm, P.segs, P.queries, P.filters,
                              P.pool, z, 0x7fffffffu, xq)
                      : x_merge(ws, sp + 4, ns, tp, nt, z, 0x7fffffffu);
          if (xs == X_UNSUP && !fin) return xs;
          if (xs == X_OK) {
            const uint64_t bytes = (4 + z.n + 7) & ~7ull;
            const uint64_t at = atomicAdd((unsigned long long*)&hin->arena_next, (unsigned long long)bytes);
            if (at + bytes > P.arena_cap) {
              err |= DE_ARENA_FULL;
            } else {
              Out w{P.arena + at + 4, 0};
              xs = nm ? x_map(ws, sp + 4, ns, tp, nt, P.maps + first, nm, P.segs, P.queries, P.filters,
                              P.pool, w, 0x7fffffffu, xq)
                      : x_merge(ws, sp + 4, ns, tp, nt, w, 0x7fffffffu);
              if (w.n == 1 && P.arena[at + 4] == 0xc0) P.arena[at + 4] = 0x80;  // nil -> {} (DocumentValue.wrap)
              *(uint32_t*)(P.arena + at) = w.n;
              res = MR_OK | (at >> 3);
            }
            st = MAP_DONE;
          } else if (xs == X_NO_DATA) {
            st = MAP_ERR_NO_DATA;
            fq = xq;
          } else {
            st = xs == X_NOT_MAP ? MAP_ERR_NOT_MAP : xs == X_FAIL ? MAP_FAIL : MAP_UNSUPPORTED;
          }
          return xs;
        });
        if (st == MAP_DONE) {
        } else if (st == MAP_OK) {
          const uint64_t bytes = (4 + o.n + 7) & ~7ull;
          const uint64_t at = atomicAdd((unsigned long long*)&hin->arena_next, (unsigned long long)bytes);
          if (at + bytes > P.arena_cap) {
            err |= DE_ARENA_FULL;
          } else {
            Out w{P.arena + at + 4, 0};
            if (nm) st = map_documents(sp + 4, ns, tp, nt, P.maps + first, nm, P.segs, P.queries, P.filters, P.pool, ws, w, fq);
            else (void)merge_docs(sp + 4, ns, tp, nt, w, unsup);
            *(uint32_t*)(P.arena + at) = w.n;
            res = MR_OK | (at >> 3);
          }
        } else if (st == MAP_ERR_NO_DATA) {
          res = MR_INCIDENT | ((uint64_t)EC_MAPPING_NO_DATA << 48) | ((uint64_t)fq << 32);
        } else if (st == MAP_ERR_NOT_MAP) {
          res = MR_INCIDENT | ((uint64_t)EC_MAPPING_NOT_MAP << 48);
        } else {
          res = st == MAP_FAIL ? MR_FAIL : MR_UNSUPPORTED;
        }
      }
    }
    P.mapres[r - b] = res;
  }
  if (err) atomicOr(P.err, err);
}

void launch_map(const WaveParams& p, hipStream_t s) {
  hipLaunchKernelGGL(k_map, dim3(MAP_GRID), dim3(256), 0, s, p);
}

void launch_merge(const WaveParams& p, hipStream_t s) {
  hipLaunchKernelGGL(k_merge, dim3(1024), dim3(256), 0, s, p);
  // (the general merge's queue is empty for flat payloads -- nearly every wave -- and the launch exits at once; a full
  // queue of exact-tree merges keeps every lane workspace busy: XLANE_COUNT lanes, latency-bound per lane)
  hipLaunchKernelGGL(k_merge_gen, dim3(XLANE_COUNT / 256), dim3(256), 0, s, p);
}
void launch_cond(const WaveParams& p, hipStream_t s) {
  hipLaunchKernelGGL(k_cond, dim3(1024), dim3(256), 0, s, p);
}

}  // namespace zbg
