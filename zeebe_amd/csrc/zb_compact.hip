// zb_compact.hip — keeping a partition's device state proportional to what is live, so that one engine
// runs for the partition's lifetime:
//
//   element-instance rows   ElementInstanceIndex.removeInstance (ElementInstanceIndex.java:54-64) frees an
//                           instance on COMPLETED / TERMINATED (ElementInstanceWriter.java:96). Rows are
//                           allocated by a bump pointer in log order (k_emit), so a dead row is reclaimed by
//                           compaction at a quiescent point: the live rows move to the front in index order
//                           (order = insertion order, which TerminateContainedElementsHandler's children.get(0)
//                           relies on) and every row reference is renamed (the flow-scope parent links).
//   payload arena           bump-allocated msgpack blobs; compaction marks the blobs reachable from the roots
//                           (live rows' payloads, the records of the log window the caller has not released,
//                           the message stores) in a granule bitmap, ranks every marked 8-byte granule by a
//                           scan of per-word popcounts and moves it to its rank (through a scratch copy), then
//                           renames the roots' refs with the same rank function. Blobs that travel together
//                           (a submitted record's [payload document][verbatim value]) stay adjacent.
//   job states              JobStateController's map (JobInstanceStreamProcessor.java:70-242) as an open-
//                           addressing table keyed by job key; removals leave tombstones that the rebuild
//                           kernels drop.
//
// All of it runs between ticks (the partition is quiescent: no record is unprocessed, so no record link
// names a row, and no deferred job holds an arena ref).
#include <hip/hip_runtime.h>

#include "zb_kernels.hpp"
#include "zb_msg.hpp"

namespace zbg {

// ------------------------------------------------------------------------------ rows
__global__ void __launch_bounds__(256) k_row_flags(CompactParams P) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x; r <= P.rows; r += stride)
    P.row_flag[r] = (r < P.rows && P.rmeta[r].state != 0) ? 1u : 0u;
}

// live row r -> scratch slot row_new[r], parent renamed; RowAux's first-child request is per wave (reset)
__global__ void __launch_bounds__(256) k_row_gather(CompactParams P) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x; r < P.rows; r += stride) {
    RowMeta m = P.rmeta[r];
    if (m.state == 0) continue;
    const uint32_t n = P.row_new[r];
    if (m.parent != NO_ROW) m.parent = (m.parent < P.rows && P.rmeta[m.parent].state != 0) ? P.row_new[m.parent] : NO_ROW;
    P.m2[n] = m;
    P.k2[n] = P.rkeys[r];  // (links: k_row_relink)
    RowAux a = P.raux[r];
    a.first = NO_ROW;
    a.mark = 0;
    P.a2[n] = a;
  }
}

// the children lists of the compacted rows [0, live_rows): every row with a parent links itself into it
__global__ void __launch_bounds__(256) k_row_relink(CompactParams P) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x; r < P.live_rows; r += stride) {
    const uint32_t p = P.rmeta[r].parent;
    if (p != NO_ROW && ZB_DCHECK(p < P.live_rows, "row %llu parent %u\n", (unsigned long long)r, p))
      P.rlink[r].c_next = atomicExch(&P.rlink[p].c_head, (uint32_t)r);
  }
}

// ------------------------------------------------------------------------------ arena
__device__ __forceinline__ void mark_granules(const CompactParams& P, uint64_t g, uint64_t n) {
  while (n) {
    const uint64_t w = g >> 6, b = g & 63;
    const uint64_t take = (64 - b) < n ? (64 - b) : n;
    const uint64_t mask = (take == 64 ? ~0ull : ((1ull << take) - 1)) << b;
    atomicOr((unsigned long long*)(P.bits + w), (unsigned long long)mask);
    g += take;
    n -= take;
  }
}

// bitmap index of a granule: [static, arena_next) and [arena_top, arena_end) back to back (the free gap between them
// has no bits)
__device__ __forceinline__ uint64_t bit_of(const CompactParams& P, uint64_t ref) {
  const uint64_t g = ref - P.static_refs, lo = P.arena_next / 8 - P.static_refs;
  return g < lo ? g : g - (P.arena_top - P.arena_next) / 8;
}
// a byte range of an allocated blob: in [static, arena_next) or in the staged documents' [arena_top, arena_end)
__device__ __forceinline__ bool arena_span(const CompactParams& P, uint64_t b0, uint64_t b1) {
  return (b0 >= P.static_refs * 8 && b1 <= P.arena_next) || (b0 >= P.arena_top && b1 <= P.arena_end);
}
// mark `blobs` consecutive blobs from ref (refs below the static region are never moved). A blob is
// [u32 len][len bytes] padded to 8; one whose length runs past its region -- a ref that does not point at a blob
// header -- marks nothing and flags the partition (the bitmap covers the allocated regions only)
__device__ __forceinline__ void mark_ref(const CompactParams& P, uint32_t ref, int blobs) {
  for (int k = 0; k < blobs; k++) {
    if (!arena_span(P, (uint64_t)ref * 8, (uint64_t)ref * 8 + 8)) return;
    const uint32_t len = *(const uint32_t*)(P.arena + (uint64_t)ref * 8);
    const uint64_t n = (4 + (uint64_t)len + 7) >> 3;
    if (!arena_span(P, (uint64_t)ref * 8, ((uint64_t)ref + n) * 8)) {
      atomicOr(P.err, (uint32_t)DE_CORRUPT);
      return;
    }
    mark_granules(P, bit_of(P, ref), n);
    ref += (uint32_t)n;
  }
}

// blobs a log record references: KIND_RAW records their [document][verbatim / re-encoded value] pair
// (zb_serialize.hip encode_value), the rest one blob (document, incident detail, message / subscription blob)
__device__ __forceinline__ int record_blobs(const zb_rec& d) { return (d.kind & KIND_RAW) ? 2 : 1; }

__global__ void __launch_bounds__(256) k_mark(CompactParams P) {
  const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x, stride = (uint64_t)gridDim.x * 256;
  for (uint64_t r = tid; r < P.live_rows; r += stride) mark_ref(P, P.rmeta[r].payload, 1);
  const uint64_t nwin = (uint64_t)(P.win_end - P.win_begin);
  for (uint64_t i = tid; i < nwin; i += stride) {
    const zb_rec d = P.log[P.win_begin + (int64_t)i];
    mark_ref(P, d.payload, record_blobs(d));
  }
  for (uint64_t i = tid; i < P.msg_count; i += stride)
    if (!P.msgs[i].dead) mark_ref(P, P.msgs[i].blob, 1);
  for (uint64_t i = tid; i < P.sub_count; i += stride) mark_ref(P, P.subs[i].blob, 1);
}

__global__ void __launch_bounds__(256) k_word_pop(CompactParams P) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x; w <= P.words; w += stride)
    P.word_pop[w] = w < P.words ? (uint32_t)__popcll((unsigned long long)P.bits[w]) : 0u;
}

// a ref's position after compaction: the static region stays, a dynamic granule goes to its rank among the
// marked ones
__device__ __forceinline__ uint32_t renamed(const CompactParams& P, uint32_t ref) {
  if (!arena_span(P, (uint64_t)ref * 8, (uint64_t)ref * 8 + 8)) return ref;
  const uint64_t g = bit_of(P, ref);
  const uint64_t w = g >> 6, b = g & 63;
  const uint64_t below = b ? (P.bits[w] & ((1ull << b) - 1)) : 0;
  return (uint32_t)(P.static_refs + P.word_off[w] + (uint64_t)__popcll((unsigned long long)below));
}

// every marked granule to its rank in the scratch copy (granule-per-thread: coalesced reads, ranks increase
// with g so the writes stay nearly coalesced)
__global__ void __launch_bounds__(256) k_arena_gather(CompactParams P) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  const uint64_t* src = (const uint64_t*)(P.arena + P.static_refs * 8);
  uint64_t* dst = (uint64_t*)P.scratch;
  const uint64_t ng = P.words * 64;
  const uint64_t lo = P.arena_next / 8 - P.static_refs, gap = (P.arena_top - P.arena_next) / 8;
  for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < ng; g += stride) {
    const uint64_t w = g >> 6, b = g & 63;
    const uint64_t word = P.bits[w];
    if (!((word >> b) & 1)) continue;
    const uint64_t below = b ? (word & ((1ull << b) - 1)) : 0;
    dst[P.word_off[w] + (uint64_t)__popcll((unsigned long long)below)] = src[g < lo ? g : g + gap];
  }
}

__global__ void __launch_bounds__(256) k_rename(CompactParams P) {
  const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x, stride = (uint64_t)gridDim.x * 256;
  for (uint64_t r = tid; r < P.live_rows; r += stride) P.rmeta[r].payload = renamed(P, P.rmeta[r].payload);
  const uint64_t nwin = (uint64_t)(P.win_end - P.win_begin);
  for (uint64_t i = tid; i < nwin; i += stride) {
    zb_rec* d = P.log + P.win_begin + (int64_t)i;
    d->payload = renamed(P, d->payload);
  }
  for (uint64_t i = tid; i < P.msg_count; i += stride)
    if (!P.msgs[i].dead) P.msgs[i].blob = renamed(P, P.msgs[i].blob);
  for (uint64_t i = tid; i < P.sub_count; i += stride) P.subs[i].blob = renamed(P, P.subs[i].blob);
}

// ------------------------------------------------------------------------------ job states
// live entries of the table -> list (any order: the table is a set), then the table is cleared and refilled
__global__ void __launch_bounds__(256) k_job_collect(JobTable T, int64_t* keys_out, uint8_t* st_out, uint32_t* n_out) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s <= T.mask; s += stride) {
    const int64_t k = T.keys[s];
    if (k == JOB_EMPTY || k == JOB_TOMB) continue;
    const uint32_t i = atomicAdd(n_out, 1u);
    keys_out[i] = k;
    st_out[i] = T.state[s];
  }
}
__global__ void __launch_bounds__(256) k_job_clear(JobTable T) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s <= T.mask; s += stride) {
    T.keys[s] = JOB_EMPTY;
    T.state[s] = JS_NONE;
  }
}
__global__ void __launch_bounds__(256) k_job_fill(JobTable T, const int64_t* keys, const uint8_t* st, uint32_t n,
                                                  uint32_t* err) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const int64_t s = job_insert(T, keys[i]);
    if (s < 0) atomicOr(err, (uint32_t)DE_ROWS_FULL);
    else T.state[s] = st[i];
  }
}

// ------------------------------------------------------------------------------ message stores
// MessageDataStore.removeMessage leaves a dead entry; compaction keeps the live ones in insertion order and the
// chains are rebuilt from them (the walk order never shows: matches are ordered by log position / index)
__global__ void __launch_bounds__(256) k_msg_flags(CompactParams P) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i <= P.msg_count; i += stride)
    P.row_flag[i] = (i < P.msg_count && !P.msgs[i].dead) ? 1u : 0u;
}
__global__ void __launch_bounds__(256) k_msg_gather(CompactParams P, MsgEntry* out) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < P.msg_count; i += stride)
    if (!P.msgs[i].dead) out[P.row_new[i]] = P.msgs[i];
}
// chains of entries [0, n) rebuilt in index order (a later entry is pushed later: the head is the newest)
__global__ void __launch_bounds__(256) k_chain_clear(uint32_t* head, uint64_t nheads) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < nheads; i += stride) head[i] = NO_ENTRY;
}
template <class E>
__global__ void __launch_bounds__(256) k_chain_build(const E* ent, uint64_t n, uint32_t* head, uint32_t* next,
                                                     uint64_t mask) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
    next[i] = atomicExch(&head[ent[i].h & mask], (uint32_t)i);
}

static unsigned grid_for(uint64_t n) {
  const uint64_t g = (n + 255) / 256;
  return (unsigned)(g < 1 ? 1 : (g > 4096 ? 4096 : g));
}

void launch_row_flags(const CompactParams& p, hipStream_t s) {
  hipLaunchKernelGGL(k_row_flags, dim3(grid_for(p.rows + 1)), dim3(256), 0, s, p);
}
void launch_row_gather(const CompactParams& p, hipStream_t s) {
  if (p.rows) hipLaunchKernelGGL(k_row_gather, dim3(grid_for(p.rows)), dim3(256), 0, s, p);
}
void launch_row_relink(const CompactParams& p, hipStream_t s) {
  if (p.live_rows) hipLaunchKernelGGL(k_row_relink, dim3(grid_for(p.live_rows)), dim3(256), 0, s, p);
}
void launch_mark(const CompactParams& p, hipStream_t s) {
  uint64_t n = p.live_rows;
  const uint64_t nwin = (uint64_t)(p.win_end - p.win_begin);
  if (nwin > n) n = nwin;
  if (p.msg_count > n) n = p.msg_count;
  if (p.sub_count > n) n = p.sub_count;
  if (n) hipLaunchKernelGGL(k_mark, dim3(grid_for(n)), dim3(256), 0, s, p);
}
void launch_word_pop(const CompactParams& p, hipStream_t s) {
  hipLaunchKernelGGL(k_word_pop, dim3(grid_for(p.words + 1)), dim3(256), 0, s, p);
}
void launch_arena_gather(const CompactParams& p, hipStream_t s) {
  if (p.words) hipLaunchKernelGGL(k_arena_gather, dim3(grid_for(p.words * 64)), dim3(256), 0, s, p);
}
void launch_rename(const CompactParams& p, hipStream_t s) {
  uint64_t n = p.live_rows;
  const uint64_t nwin = (uint64_t)(p.win_end - p.win_begin);
  if (nwin > n) n = nwin;
  if (p.msg_count > n) n = p.msg_count;
  if (p.sub_count > n) n = p.sub_count;
  if (n) hipLaunchKernelGGL(k_rename, dim3(grid_for(n)), dim3(256), 0, s, p);
}
void launch_job_collect(const JobTable& t, int64_t* keys, uint8_t* st, uint32_t* n, hipStream_t s) {
  hipLaunchKernelGGL(k_job_collect, dim3(grid_for(t.mask + 1)), dim3(256), 0, s, t, keys, st, n);
}
void launch_job_clear(const JobTable& t, hipStream_t s) {
  hipLaunchKernelGGL(k_job_clear, dim3(grid_for(t.mask + 1)), dim3(256), 0, s, t);
}
void launch_job_fill(const JobTable& t, const int64_t* keys, const uint8_t* st, uint32_t n, uint32_t* err, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_job_fill, dim3(grid_for(n)), dim3(256), 0, s, t, keys, st, n, err);
}
void launch_msg_flags(const CompactParams& p, hipStream_t s) {
  hipLaunchKernelGGL(k_msg_flags, dim3(grid_for(p.msg_count + 1)), dim3(256), 0, s, p);
}
void launch_msg_gather(const CompactParams& p, MsgEntry* out, hipStream_t s) {
  if (p.msg_count) hipLaunchKernelGGL(k_msg_gather, dim3(grid_for(p.msg_count)), dim3(256), 0, s, p, out);
}
void launch_chains(const MsgEntry* msgs, uint64_t nm, uint32_t* mh, uint32_t* mn, const SubEntry* subs, uint64_t ns,
                   uint32_t* sh, uint32_t* sn, uint64_t mask, hipStream_t s) {
  hipLaunchKernelGGL(k_chain_clear, dim3(grid_for(mask + 1)), dim3(256), 0, s, mh, mask + 1);
  hipLaunchKernelGGL(k_chain_clear, dim3(grid_for(mask + 1)), dim3(256), 0, s, sh, mask + 1);
  if (nm) hipLaunchKernelGGL(k_chain_build<MsgEntry>, dim3(grid_for(nm)), dim3(256), 0, s, msgs, nm, mh, mn, mask);
  if (ns) hipLaunchKernelGGL(k_chain_build<SubEntry>, dim3(grid_for(ns)), dim3(256), 0, s, subs, ns, sh, sn, mask);
}

}  // namespace zbg
