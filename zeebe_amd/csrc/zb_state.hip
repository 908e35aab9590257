// zb_state.hip — element-instance index lookups and read-back over the SoA rows.
//
//   k_resolve     submitted records -> the row of the element instance their key names
//                 (ElementInstanceIndex.getInstance, ElementInstanceIndex.java:40-44): one pass over
//                 the allocated rows, each live row binary-searches its key among the batch's sorted
//                 lookup keys. Rows are never reused and a key names at most one live row.
//   k_live_rows   live rows -> (key, row) pairs for zb_read_instances / snapshots.
//   k_row_descs   rows in key order -> WORKFLOW_INSTANCE descriptors of their indexed values, which the
//                 serializer (zb_serialize.hip) turns into WorkflowInstanceRecord bytes.
#include <hip/hip_runtime.h>

#include "zb_kernels.hpp"

namespace zbg {

__global__ void __launch_bounds__(256) k_resolve(ResolveParams P) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x; r < P.rows; r += stride) {
    if (P.rmeta[r].state == 0) continue;
    const int64_t key = P.rkeys[r].key;
    // lower bound of key in the sorted lookup keys
    int64_t lo = 0, hi = P.n;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (P.keys[mid] < key) lo = mid + 1;
      else hi = mid;
    }
    for (int64_t i = lo; i < P.n && P.keys[i] == key; i++) {
      uint32_t* link = (uint32_t*)(P.links + P.pos_base + P.pos[i]);
      link[0] = (uint32_t)r;  // row-self half
    }
  }
}

__global__ void __launch_bounds__(256) k_live_rows(LiveParams P) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x; r < P.rows; r += stride) {
    if (P.rmeta[r].state == 0) continue;
    const uint32_t slot = atomicAdd(P.count, 1u);
    if (slot < P.cap) {
      P.keys[slot] = P.rkeys[r].key;
      P.row_of[slot] = (uint32_t)r;
    }
  }
}

__global__ void __launch_bounds__(256) k_row_descs(LiveParams P) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= P.n) return;
  const uint32_t r = P.row_of[i];
  const RowMeta m = P.rmeta[r];
  const RowKeys k = P.rkeys[r];
  zb_rec d;
  d.key = k.key;
  d.scope_key = k.scope_key;
  d.inst_key = k.inst_key;
  d.payload = m.payload;
  d.elem = m.elem;
  d.intent = m.state;
  d.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE, ZB_RT_EVENT, false);
  P.descs[i] = d;
  InstHead h;
  h.key = k.key;
  h.parent_key = m.parent == NO_ROW ? -1 : P.rkeys[m.parent].key;
  h.job_key = k.job_key;
  h.state = m.state;
  P.heads[i] = h;
}

__global__ void __launch_bounds__(64) k_status(StatusCopy c) {
  for (int k = 0; k < c.count; k++)
    for (uint32_t i = threadIdx.x; i < c.words[k]; i += 64) c.dst[k][i] = c.src[k][i];
}

void launch_resolve(const ResolveParams& p, hipStream_t s) {
  if (p.rows == 0 || p.n == 0) return;
  const uint64_t g = (p.rows + 255) / 256;
  hipLaunchKernelGGL(k_resolve, dim3((unsigned)(g < 4096 ? g : 4096)), dim3(256), 0, s, p);
}
void launch_live_rows(const LiveParams& p, hipStream_t s) {
  if (p.rows == 0) return;
  const uint64_t g = (p.rows + 255) / 256;
  hipLaunchKernelGGL(k_live_rows, dim3((unsigned)(g < 4096 ? g : 4096)), dim3(256), 0, s, p);
}
void launch_row_descs(const LiveParams& p, hipStream_t s) {
  if (p.n == 0) return;
  hipLaunchKernelGGL(k_row_descs, dim3((unsigned)((p.n + 255) / 256)), dim3(256), 0, s, p);
}

void launch_status(const StatusCopy& c, hipStream_t s) {
  if (c.count) hipLaunchKernelGGL(k_status, dim3(1), dim3(64), 0, s, c);
}

}  // namespace zbg
