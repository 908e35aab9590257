// zb_engine.hip — host side of libzbgpu.so: the C ABI of include/zb_engine.h.
//
// One handle = one partition on one HIP device with one stream. zb_step launches one wave
// kernel per breadth-first generation, in batches of WAVES_PER_SYNC launches between host
// checks of the device wave header (quiescence = empty generation). No CPU fallback exists:
// every record is processed by the gfx950 kernels, and anything they do not implement is
// reported as ZB_EUNSUPPORTED.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <string>
#include <vector>

#include "zb_kernels.hpp"
#include "zb_model.hpp"
#include "zb_msg.hpp"

using namespace zbg;

namespace {

constexpr int WAVES_PER_SYNC = 16;
constexpr int EV_PER_WAVE = 4;  // before k_process, after k_process, after k_emit, after the aux kernels
constexpr uint64_t STATIC_ARENA_BYTES = 1ull << 20;  // {} at ref 0 + harness job completion payloads
constexpr uint64_t TRAJ_BUDGET_BYTES = 256ull << 20;  // per-(generation, workgroup) counts of the trajectory path
constexpr int TRAJ_MAX_GENERATIONS = CLS_ROW;
constexpr int TRAJ_WAVE_CAP = 8192;                   // k_traj_scan grid bound (one workgroup per generation)

template <class T>
struct DevVec {
  T* p = nullptr;
  size_t n = 0;
  void free() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  hipError_t upload(const std::vector<T>& v, hipStream_t s) {
    if (v.size() > n || !p) {
      free();
      size_t cap = v.empty() ? 1 : v.size();
      hipError_t e = hipMalloc(&p, cap * sizeof(T));
      if (e != hipSuccess) return e;
      n = cap;
    }
    if (v.empty()) return hipSuccess;
    return hipMemcpyAsync(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s);
  }
};

}  // namespace

struct zb_engine {
  zb_config cfg{};
  hipStream_t stream = nullptr;
  std::string err;

  ModelTables model;
  DevVec<DevElem> d_elems;
  DevVec<DevWorkflow> d_wfs;
  DevVec<uint16_t> d_cond;
  DevVec<uint32_t> d_code;
  DevVec<DevConst> d_consts;
  DevVec<DevQuery> d_queries;
  DevVec<DevFilter> d_filters;
  DevVec<uint8_t> d_pool;

  // device state
  zb_rec* log = nullptr;
  uint64_t* links = nullptr;
  RowMeta* rmeta = nullptr;
  RowKeys* rkeys = nullptr;
  uint8_t* arena = nullptr;
  WaveHdr* hdr = nullptr;
  uint32_t* derr = nullptr;
  uint64_t* dstats = nullptr;
  // wave staging (k_process -> k_scan -> k_emit), wave_cap records
  uint64_t wave_cap = 0;
  uint64_t* cw = nullptr;
  Slot* stage = nullptr;
  ItemInfo* info = nullptr;
  BlockAgg* block_agg = nullptr;
  BlockOff* block_off = nullptr;
  uint64_t* derr_info = nullptr;
  MergeJob* merge_jobs = nullptr;
  uint64_t* cond_jobs = nullptr;
  uint32_t* job_counts = nullptr;  // [0..1] merge counts, [2..3] cond counts
  uint64_t job_cap = 0;
  WaveHdr* h_hdr_pinned = nullptr;  // pinned mirror for D2H polling
  uint32_t* h_err_pinned = nullptr;

  int64_t wave = 0;
  WaveHdr host_hdr{};
  bool has_merges = false, has_splits = false;
  bool failed = false;

  // static arena region (ref 0 = {}, harness payloads)
  std::vector<uint8_t> static_blobs;

  // staged input
  std::vector<zb_rec> staged;
  std::vector<uint8_t> staged_arena;
  struct PendingRange {
    int64_t first, last;  // staged indices
    int64_t workflow_key;
    int32_t version;
    uint32_t pid_off;
    uint16_t pid_len;
  };
  std::vector<PendingRange> pending_ranges;
  DevVec<zb_rec> d_staged;
  DevVec<uint8_t> d_staged_arena;
  bool staged_uploaded = false;
  bool staged_pending = false;  // the staged batch has not been injected yet (zb_reset(keep) re-arms it)
  uint16_t staged_elem = NO_ELEM;  // process element of the staged CREATEs ...
  bool staged_uniform = true;      // ... when they all address the same one
  uint32_t staged_max_len = 1;     // longest staged CREATE payload (uniform batch merge bounds)

  // submitted command ranges (serialization of CREATE commands / rejections)
  std::vector<CmdRange> ranges;
  std::vector<uint8_t> cmd_pool;
  DevVec<CmdRange> d_ranges;
  DevVec<uint8_t> d_cmd_pool;

  // trajectory path buffers (zb_traj.hip), grown on demand
  bool traj_model_ok = true;     // false when merges can precede condition evaluation (see zb_traj.hip)
  uint64_t traj_entries = 0;     // capacity of agg / woff in (generation, workgroup) entries
  uint64_t* t_agg = nullptr;
  uint4* t_woff = nullptr;
  uint32_t* t_wcount = nullptr;
  uint64_t t_nwg_cap = 0;
  uint4* t_wtot = nullptr;
  TrajBase* t_wbase = nullptr;
  TrajCtl* t_ctl = nullptr;
  MergeGen* t_mgen = nullptr;     // [TRAJ_MAX_GENERATIONS] uniform batch merge slots
  uint64_t* t_wstats = nullptr;   // [t_nwg_cap + CLS_MAX][6] emit statistics per workgroup
  TrajCtl* h_ctl_pinned = nullptr;
  // class batches (zb_traj.hip k_cls_*): the model's exclusive splits as outcome-key digits
  bool cls_ok = false;            // split outcome keys fit 8 bits and CLS_MAX_SPLITS splits
  int nsplits = 0;
  uint32_t split_elem[CLS_MAX_SPLITS] = {}, split_stride[CLS_MAX_SPLITS] = {};
  ClsPlan* c_plan = nullptr;
  uint64_t cls_cap = 0;           // instances the class buffers hold
  uint8_t* c_ikey = nullptr;
  uint32_t *c_khist = nullptr, *c_krep = nullptr;  // [CLS_HB][256] each (one allocation with c_klen)
  uint64_t* c_klen = nullptr;                       // [CLS_HB][256]
  TmplRec* t_tmpl = nullptr;     // [CLS_MAX][CLS_ROW][TF] traced records (uniform / class batches)
  uint32_t* t_cstat = nullptr;   // [CLS_MAX][TSTAT]
  uint64_t* c_mask = nullptr;
  uint32_t *c_woffw = nullptr, *c_wgcnt = nullptr, *c_wgoff = nullptr, *c_perm = nullptr;
  uint32_t *c_segs = nullptr, *c_wcls = nullptr;

  // message correlation (zb_msg.hip): outboxes [0] open-subscription, [1] correlate
  zb_exchange_rec* obox[2] = {nullptr, nullptr};
  uint64_t* okeys[2] = {nullptr, nullptr};
  uint32_t* on = nullptr;  // [2] device counters
  uint64_t ocap = 0;
  // message stores (MessageSubscriptionDataStore / MessageDataStore), allocated on first use
  SubEntry* subs = nullptr;
  uint32_t *sub_head = nullptr, *sub_next = nullptr;
  MsgEntry* msgs = nullptr;
  uint32_t *msg_head = nullptr, *msg_next = nullptr;
  uint64_t store_cap = 0, head_mask = 0, sub_count = 0, msg_count = 0;
  int64_t msg_key_next = 0;  // message KeyGenerator(0, 1) (MessageService.java:91)
  bool has_catch = false;
  // RCCL communicator over the partitions of the node (zb_comm_*)
  ncclComm_t comm = nullptr;
  uint64_t* d_xcounts = nullptr;  // [2 * 64] send / receive counts

  // timing
  std::vector<hipEvent_t> ev;
};

namespace {

int fail(zb_engine* e, int code, const std::string& msg) {
  e->err = msg;
  return code;
}

#define HIPCHECK(e, call)                                                              \
  do {                                                                                 \
    hipError_t _r = (call);                                                            \
    if (_r != hipSuccess) return fail((e), ZB_EDEVICE, std::string(#call) + ": " + hipGetErrorString(_r)); \
  } while (0)

uint32_t add_blob(std::vector<uint8_t>& arena, const uint8_t* p, uint32_t n) {
  size_t off = arena.size();
  size_t total = (4 + (size_t)n + 7) & ~(size_t)7;
  arena.resize(off + total, 0);
  std::memcpy(arena.data() + off, &n, 4);
  if (n) std::memcpy(arena.data() + off + 4, p, n);
  return (uint32_t)(off >> 3);
}

int upload_model(zb_engine* e) {
  HIPCHECK(e, e->d_elems.upload(e->model.elems, e->stream));
  HIPCHECK(e, e->d_wfs.upload(e->model.workflows, e->stream));
  HIPCHECK(e, e->d_cond.upload(e->model.cond_flows, e->stream));
  HIPCHECK(e, e->d_code.upload(e->model.code, e->stream));
  HIPCHECK(e, e->d_consts.upload(e->model.consts, e->stream));
  HIPCHECK(e, e->d_queries.upload(e->model.queries, e->stream));
  HIPCHECK(e, e->d_filters.upload(e->model.filters, e->stream));
  HIPCHECK(e, e->d_pool.upload(e->model.pool, e->stream));
  if (e->static_blobs.size() > STATIC_ARENA_BYTES) return fail(e, ZB_ENOMEM, "static payload region full");
  HIPCHECK(e, hipMemcpyAsync(e->arena, e->static_blobs.data(), e->static_blobs.size(), hipMemcpyHostToDevice,
                             e->stream));
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  return ZB_OK;
}

WaveParams wave_params(zb_engine* e) {
  WaveParams p;
  p.log = e->log;
  p.links = e->links;
  p.rmeta = e->rmeta;
  p.rkeys = e->rkeys;
  p.arena = e->arena;
  p.elems = e->d_elems.p;
  p.wfs = e->d_wfs.p;
  p.cond_flows = e->d_cond.p;
  p.code = e->d_code.p;
  p.consts = e->d_consts.p;
  p.queries = e->d_queries.p;
  p.filters = e->d_filters.p;
  p.pool = e->d_pool.p;
  p.hdr = e->hdr;
  p.cw = e->cw;
  p.stage = e->stage;
  p.info = e->info;
  p.block_agg = e->block_agg;
  p.block_off = e->block_off;
  p.wave_cap = e->wave_cap;
  p.err = e->derr;
  p.err_info = e->derr_info;
  p.merge_jobs = e->merge_jobs;
  p.merge_count = e->job_counts;
  p.cond_jobs = e->cond_jobs;
  p.cond_count = e->job_counts + 2;
  p.job_cap = e->job_cap;
  p.stats = e->dstats;
  p.log_cap = e->cfg.log_capacity;
  p.row_cap = e->cfg.row_capacity;
  p.arena_cap = e->cfg.arena_bytes;
  p.wave = e->wave;
  p.obox = e->obox[0];
  p.okeys = e->okeys[0];
  p.on = e->on;
  p.ocap = e->ocap;
  p.partition_id = e->cfg.partition_id;
  p.partition_count = e->cfg.partition_count;
  return p;
}

int check_device_errors(zb_engine* e, uint32_t flags) {
  if (!flags) return ZB_OK;
  e->failed = true;
  std::string m = "device error flags:";
  if (flags & DE_LOG_FULL) m += " log-capacity";
  if (flags & DE_ROWS_FULL) m += " row-capacity";
  if (flags & DE_ARENA_FULL) m += " arena-capacity";
  if (flags & DE_UNSUPPORTED) m += " unsupported-shape";
  if (flags & DE_PROCESSING) m += " processing-failure";
  if (flags & DE_BAD_PAYLOAD) m += " malformed-payload";
  uint64_t info = ~0ull;
  if (hipMemcpy(&info, e->derr_info, sizeof(info), hipMemcpyDeviceToHost) == hipSuccess && info != ~0ull)
    m += " (first at log position " + std::to_string(info >> 8) + ", site " + std::to_string(info & 0xff) + ")";
  int code = ZB_EPROCESSING;
  if (flags & (DE_LOG_FULL | DE_ROWS_FULL | DE_ARENA_FULL)) code = ZB_ENOMEM;
  else if (flags & DE_UNSUPPORTED) code = ZB_EUNSUPPORTED;
  return fail(e, code, m);
}

// Trajectory path (zb_traj.hip) for a batch of n CREATE commands injected at log_base on an idle
// partition. Returns 1 when the batch ran to quiescence, 0 when the count pass asked for the wave
// pipeline (nothing but scratch counts was written), <0 on a device error.
// emit slots of a class batch: instances + the padding of every (block, class) segment
uint64_t cls_slot_bound(uint64_t n, uint64_t nwg) {
  const uint64_t nblk = (nwg + CLS_BLK_WG - 1) / CLS_BLK_WG;
  return n + 64 * CLS_MAX * nblk;
}

int grow_class_buffers(zb_engine* e, uint64_t n, uint64_t nwg) {
  if (n <= e->cls_cap) return ZB_OK;
  void* ps[] = {e->c_ikey, e->c_khist, e->c_mask, e->c_woffw, e->c_wgcnt, e->c_wgoff, e->c_perm, e->c_segs, e->c_wcls};
  for (void* q : ps)
    if (q) (void)hipFree(q);
  e->c_ikey = nullptr; e->c_khist = e->c_krep = nullptr; e->c_klen = nullptr; e->c_mask = nullptr;
  e->c_woffw = e->c_wgcnt = e->c_wgoff = e->c_perm = e->c_segs = e->c_wcls = nullptr;
  e->cls_cap = 0;
  const uint64_t groups = nwg * (TRAJ_WG / 64);
  HIPCHECK(e, hipMalloc(&e->c_ikey, n));
  HIPCHECK(e, hipMalloc(&e->c_khist, CLS_HB * 256 * (2 * sizeof(uint32_t) + sizeof(uint64_t))));
  e->c_krep = e->c_khist + CLS_HB * 256;
  e->c_klen = (uint64_t*)(e->c_khist + 2 * CLS_HB * 256);
  HIPCHECK(e, hipMalloc(&e->c_mask, groups * CLS_MAX * sizeof(uint64_t)));
  HIPCHECK(e, hipMalloc(&e->c_woffw, groups * CLS_MAX * sizeof(uint32_t)));
  HIPCHECK(e, hipMalloc(&e->c_wgcnt, nwg * CLS_MAX * sizeof(uint32_t)));
  HIPCHECK(e, hipMalloc(&e->c_wgoff, nwg * CLS_MAX * sizeof(uint32_t)));
  const uint64_t nblk = (nwg + CLS_BLK_WG - 1) / CLS_BLK_WG;
  const uint64_t slots = cls_slot_bound(n, nwg);
  HIPCHECK(e, hipMalloc(&e->c_perm, slots * sizeof(uint32_t)));
  HIPCHECK(e, hipMalloc(&e->c_segs, nblk * CLS_MAX * sizeof(uint32_t)));
  HIPCHECK(e, hipMalloc(&e->c_wcls, (slots / 64 + 1) * sizeof(uint32_t)));
  if (!e->c_plan) HIPCHECK(e, hipMalloc(&e->c_plan, sizeof(ClsPlan)));
  e->cls_cap = nwg * TRAJ_WG;
  return ZB_OK;
}

int run_trajectory(zb_engine* e, int64_t log_base, int64_t n, zb_step_stats& st, bool allow_tmpl) {
  const uint64_t nwg = (uint64_t)((n + TRAJ_WG - 1) / TRAJ_WG);
  const uint64_t per_entry = sizeof(uint64_t) + sizeof(uint4);
  uint64_t wcap = std::min<uint64_t>(TRAJ_MAX_GENERATIONS, (TRAJ_BUDGET_BYTES / per_entry) / nwg);
  if (wcap < 8 || nwg > 0x7fffffffull) return 0;
  if (wcap * nwg > e->traj_entries) {
    if (e->t_agg) (void)hipFree(e->t_agg);
    if (e->t_woff) (void)hipFree(e->t_woff);
    e->t_agg = nullptr; e->t_woff = nullptr; e->traj_entries = 0;
    const uint64_t ent = TRAJ_BUDGET_BYTES / per_entry;
    HIPCHECK(e, hipMalloc(&e->t_agg, ent * sizeof(uint64_t)));
    HIPCHECK(e, hipMalloc(&e->t_woff, ent * sizeof(uint4)));
    e->traj_entries = ent;
  }
  if (nwg > e->t_nwg_cap) {
    if (e->t_wcount) (void)hipFree(e->t_wcount);
    if (e->t_wstats) (void)hipFree(e->t_wstats);
    e->t_wcount = nullptr;
    e->t_wstats = nullptr;
    HIPCHECK(e, hipMalloc(&e->t_wcount, (nwg + CLS_MAX) * sizeof(uint32_t)));
    // (class batches emit over up to nwg + nwg / 8 + 8 workgroups)
    HIPCHECK(e, hipMalloc(&e->t_wstats, (2 * nwg + 64) * 6 * sizeof(uint64_t)));
    e->t_nwg_cap = nwg;
  }
  TrajCtl c{};
  c.arena_next = c.arena_start = (uint64_t)e->host_hdr.arena_next;
  c.rows_next = c.rows_start = (uint64_t)e->host_hdr.rows_next;
  *e->h_ctl_pinned = c;
  HIPCHECK(e, hipMemcpyAsync(e->t_ctl, e->h_ctl_pinned, sizeof(TrajCtl), hipMemcpyHostToDevice, e->stream));
  TrajParams p{};
  p.log = e->log;
  p.arena = e->arena;
  p.rmeta = e->rmeta;
  p.rkeys = e->rkeys;
  p.elems = e->d_elems.p;
  p.cond_flows = e->d_cond.p;
  p.code = e->d_code.p;
  p.consts = e->d_consts.p;
  p.queries = e->d_queries.p;
  p.filters = e->d_filters.p;
  p.pool = e->d_pool.p;
  p.log_base = log_base;
  p.n = n;
  p.wf_start = e->host_hdr.wf_next;
  p.job_start = e->host_hdr.job_next;
  p.nwg = (int32_t)nwg;
  p.wcap = (int32_t)wcap;
  // Without exclusive splits nothing in a trajectory depends on payload values, so a batch whose
  // CREATEs all address one process has one trajectory shape: count it on the first instance.
  p.uni = (allow_tmpl && !e->has_splits && e->staged_uniform) ? n : 0;
  p.cond = e->has_splits ? 1 : 0;
  // With exclusive splits whose conditions only ever read the CREATE payload, the batch splits into a
  // few trajectory classes (k_cls_*); each runs like a uniform batch. More classes than CLS_MAX, or a
  // class whose trajectory raises an incident, sends the batch to the per-instance count pass below.
  p.cls = (allow_tmpl && e->has_splits && e->staged_uniform && e->cls_ok) ? 1 : 0;
  p.nwg_e = (int32_t)nwg;
  if (p.cls) {
    int grc = grow_class_buffers(e, (uint64_t)n, nwg);
    if (grc != ZB_OK) return grc;
    // every (block, class) segment padded to whole waves; a multiple of 8 workgroups (XCD mapping)
    p.nwg_e = (int32_t)(((cls_slot_bound((uint64_t)n, nwg) + TRAJ_WG - 1) / TRAJ_WG + 7) & ~7ull);
    p.nblk = (int32_t)((nwg + CLS_BLK_WG - 1) / CLS_BLK_WG);
    p.segs = e->c_segs;
    p.wcls = e->c_wcls;
    HIPCHECK(e, hipMemsetAsync(e->c_perm, 0xff, cls_slot_bound((uint64_t)n, nwg) * sizeof(uint32_t), e->stream));
    p.nsplits = e->nsplits;
    for (int k = 0; k < CLS_MAX_SPLITS; k++) {
      p.split_elem[k] = e->split_elem[k];
      p.split_stride[k] = e->split_stride[k];
    }
    p.plan = e->c_plan;
    p.ikey = e->c_ikey;
    p.khist = e->c_khist;
    p.klen = e->c_klen;
    p.krep = e->c_krep;
    p.cmask = e->c_mask;
    p.woffw = e->c_woffw;
    p.wgcnt = e->c_wgcnt;
    p.wgoff = e->c_wgoff;
    p.perm = e->c_perm;
    HIPCHECK(e, hipMemsetAsync(e->c_khist, 0, CLS_HB * 256 * sizeof(uint32_t), e->stream));
    HIPCHECK(e, hipMemsetAsync(e->c_klen, 0, CLS_HB * 256 * sizeof(uint64_t), e->stream));
    HIPCHECK(e, hipMemsetAsync(e->c_krep, 0xff, CLS_HB * 256 * sizeof(uint32_t), e->stream));
  }
  p.agg = e->t_agg;
  p.wcount = e->t_wcount;
  p.woff = e->t_woff;
  p.wtot = e->t_wtot;
  p.wbase = e->t_wbase;
  p.ctl = e->t_ctl;
  p.mgen = e->t_mgen;
  p.tmpl = e->t_tmpl;
  p.cstat = e->t_cstat;
  p.wstats = e->t_wstats;
  p.max_create = e->staged_max_len;
  p.hdr = e->hdr + (e->wave & 1);
  p.err = e->derr;
  p.stats = e->dstats;
  p.log_cap = e->cfg.log_capacity;
  p.row_cap = e->cfg.row_capacity;
  p.arena_cap = e->cfg.arena_bytes;
  hipEvent_t* ev = e->ev.data();
  HIPCHECK(e, hipEventRecord(ev[0], e->stream));
  if (p.cls) launch_traj_count_classes(p, e->stream);
  else if (p.uni) launch_traj_count_uniform(p, e->stream);
  else launch_traj_count(p, e->stream);
  HIPCHECK(e, hipEventRecord(ev[1], e->stream));
  launch_traj_scan(p, e->stream);
  launch_traj_emit(p, e->stream, &ev[3]);
  HIPCHECK(e, hipEventRecord(ev[2], e->stream));
  HIPCHECK(e, hipGetLastError());
  HIPCHECK(e, hipMemcpyAsync(e->h_ctl_pinned, e->t_ctl, sizeof(TrajCtl), hipMemcpyDeviceToHost, e->stream));
  HIPCHECK(e, hipMemcpyAsync(e->h_hdr_pinned, e->hdr + (e->wave & 1), sizeof(WaveHdr), hipMemcpyDeviceToHost,
                             e->stream));
  HIPCHECK(e, hipMemcpyAsync(e->h_err_pinned, e->derr, sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  float ms0 = 0, ms1 = 0, ms_main = 0;
  HIPCHECK(e, hipEventElapsedTime(&ms0, ev[0], ev[1]));
  HIPCHECK(e, hipEventElapsedTime(&ms1, ev[1], ev[2]));
  HIPCHECK(e, hipEventElapsedTime(&ms_main, ev[3], ev[4]));
  st.main_emit_kernel_ms += ms_main;
  st.process_kernel_ms += ms0;
  st.emit_kernel_ms += ms1;
  st.wave_kernel_ms += ms0 + ms1;
  st.launches += p.cls ? 11 : p.uni ? 6 : 7;
  if (p.cls && getenv("ZB_DEBUG_CLS")) {  // class batch internals (debugging aid)
    ClsPlan pl;
    uint32_t wc[CLS_MAX];
    (void)hipMemcpy(&pl, e->c_plan, sizeof(pl), hipMemcpyDeviceToHost);
    (void)hipMemcpy(wc, e->t_wcount, sizeof(wc), hipMemcpyDeviceToHost);
    const TrajCtl& c2 = *e->h_ctl_pinned;
    fprintf(stderr, "zb cls: flag=%u wmax=%u end=%ld nc=%u slots=%u\n", c2.flag, c2.wmax, (long)c2.end, pl.nc, pl.slots);
    for (uint32_t c = 0; c < pl.nc && c < CLS_MAX; c++) {
      std::vector<uint64_t> a(c2.wmax);
      if (c2.wmax) (void)hipMemcpy(a.data(), e->t_agg + (uint64_t)c * CLS_ROW, c2.wmax * 8, hipMemcpyDeviceToHost);
      fprintf(stderr, "  class %u key=%u n=%u rep=%u W=%u agg:", c, pl.key[c], pl.n[c], pl.rep[c], wc[c]);
      for (auto x : a) fprintf(stderr, " %lx", (unsigned long)x);
      fprintf(stderr, "\n");
    }
  }
  if (e->h_ctl_pinned->flag) {
    // nothing but scratch counts was written: run the batch per instance (or on the wave pipeline)
    if ((p.cls || p.uni) && e->traj_model_ok) return run_trajectory(e, log_base, n, st, false);
    return 0;
  }
  e->host_hdr = e->h_hdr_pinned[0];
  int rc = check_device_errors(e, *e->h_err_pinned);
  if (rc != ZB_OK) return rc;
  st.path = p.cls ? 2 : 1;
  return 1;
}

// outboxes: one record per element-instance row at most (a subscription per catch event instance;
// a correlation per subscription and publish)
int ensure_outbox(zb_engine* e) {
  if (e->on) return ZB_OK;
  e->ocap = std::max<uint64_t>(e->cfg.row_capacity, 1024);
  for (int k = 0; k < 2; k++) {
    HIPCHECK(e, hipMalloc(&e->obox[k], e->ocap * sizeof(zb_exchange_rec)));
    HIPCHECK(e, hipMalloc(&e->okeys[k], e->ocap * sizeof(uint64_t)));
  }
  HIPCHECK(e, hipMalloc(&e->on, 2 * sizeof(uint32_t)));
  HIPCHECK(e, hipMemsetAsync(e->on, 0, 2 * sizeof(uint32_t), e->stream));
  return ZB_OK;
}

int ensure_stores(zb_engine* e) {
  int rc = ensure_outbox(e);
  if (rc != ZB_OK) return rc;
  if (e->subs) return ZB_OK;
  e->store_cap = std::max<uint64_t>(e->cfg.row_capacity, 1024);
  uint64_t heads = 1;
  while (heads < 2 * e->store_cap) heads <<= 1;
  e->head_mask = heads - 1;
  HIPCHECK(e, hipMalloc(&e->subs, e->store_cap * sizeof(SubEntry)));
  HIPCHECK(e, hipMalloc(&e->sub_next, e->store_cap * sizeof(uint32_t)));
  HIPCHECK(e, hipMalloc(&e->sub_head, heads * sizeof(uint32_t)));
  HIPCHECK(e, hipMalloc(&e->msgs, e->store_cap * sizeof(MsgEntry)));
  HIPCHECK(e, hipMalloc(&e->msg_next, e->store_cap * sizeof(uint32_t)));
  HIPCHECK(e, hipMalloc(&e->msg_head, heads * sizeof(uint32_t)));
  HIPCHECK(e, hipMemsetAsync(e->sub_head, 0xff, heads * sizeof(uint32_t), e->stream));
  HIPCHECK(e, hipMemsetAsync(e->msg_head, 0xff, heads * sizeof(uint32_t), e->stream));
  return ZB_OK;
}

MsgParams msg_params(zb_engine* e) {
  MsgParams p{};
  p.log = e->log;
  p.links = e->links;
  p.arena = e->arena;
  p.subs = e->subs; p.sub_head = e->sub_head; p.sub_next = e->sub_next;
  p.sub_mask = e->head_mask; p.sub_count = e->sub_count; p.sub_cap = e->store_cap;
  p.msgs = e->msgs; p.msg_head = e->msg_head; p.msg_next = e->msg_next;
  p.msg_mask = e->head_mask; p.msg_count = e->msg_count; p.msg_cap = e->store_cap;
  p.obox = e->obox[1]; p.okeys = e->okeys[1]; p.on = e->on + 1; p.ocap = e->ocap;
  p.err = e->derr;
  return p;
}

// the partition must be idle for a message-side batch (canonical schedule, zeebe_amd/cluster.py)
int require_idle(zb_engine* e) {
  if (e->failed) return fail(e, ZB_EPROCESSING, "partition stopped after a processing failure: " + e->err);
  if (e->host_hdr.begin != e->host_hdr.end || (e->staged_pending && !e->staged.empty()))
    return fail(e, ZB_EINVAL, "partition not quiescent: step it before delivering or publishing");
  return ZB_OK;
}

int finish_batch(zb_engine* e) {
  HIPCHECK(e, hipMemcpyAsync(e->hdr + (e->wave & 1), &e->host_hdr, sizeof(WaveHdr), hipMemcpyHostToDevice, e->stream));
  HIPCHECK(e, hipGetLastError());
  HIPCHECK(e, hipMemcpyAsync(e->h_err_pinned, e->derr, sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  return check_device_errors(e, *e->h_err_pinned);
}

}  // namespace

extern "C" {

int zb_engine_create(const zb_config* cfg, zb_engine** out) {
  if (!cfg || !out) return ZB_EINVAL;
  *out = nullptr;
  auto* e = new zb_engine();
  e->cfg = *cfg;
  if (e->cfg.log_capacity == 0) e->cfg.log_capacity = 1ull << 22;
  if (e->cfg.row_capacity == 0) e->cfg.row_capacity = 1ull << 20;
  if (e->cfg.arena_bytes == 0) e->cfg.arena_bytes = 64ull << 20;
  if (e->cfg.arena_bytes < 2 * STATIC_ARENA_BYTES) e->cfg.arena_bytes = 2 * STATIC_ARENA_BYTES;
  if (e->cfg.partition_count <= 0) e->cfg.partition_count = 1;
  if (e->cfg.log_capacity >= (1ull << 40) || e->cfg.row_capacity >= 0xffffffffull ||
      e->cfg.arena_bytes >= (8ull << 32)) {
    delete e;
    return ZB_EINVAL;
  }
  auto cleanup = [&](int code) {
    zb_engine_destroy(e);
    return code;
  };
  if (hipSetDevice(cfg->device) != hipSuccess) return cleanup(ZB_EDEVICE);
  if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) return cleanup(ZB_EDEVICE);
  const uint64_t L = e->cfg.log_capacity;
  e->wave_cap = e->cfg.wave_records ? e->cfg.wave_records : std::min<uint64_t>(L, 1ull << 22);
  e->wave_cap = (e->wave_cap + WAVE_TILE - 1) / WAVE_TILE * WAVE_TILE;
  if (hipMalloc(&e->log, L * sizeof(zb_rec)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->links, L * sizeof(uint64_t)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->rmeta, e->cfg.row_capacity * sizeof(RowMeta)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->rkeys, e->cfg.row_capacity * sizeof(RowKeys)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->arena, e->cfg.arena_bytes) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->hdr, 2 * sizeof(WaveHdr)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->cw, e->wave_cap * sizeof(uint64_t)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->stage, e->wave_cap * 2 * sizeof(Slot)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->info, e->wave_cap * sizeof(ItemInfo)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->block_agg, WAVE_GRID * sizeof(BlockAgg)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->block_off, WAVE_GRID * sizeof(BlockOff)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->derr, sizeof(uint32_t)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->dstats, 8 * sizeof(uint64_t)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->derr_info, sizeof(uint64_t)) != hipSuccess) return cleanup(ZB_ENOMEM);
  e->job_cap = std::min<uint64_t>(L, 1ull << 26);
  if (hipMalloc(&e->merge_jobs, 2 * e->job_cap * sizeof(MergeJob)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->cond_jobs, 2 * e->job_cap * sizeof(uint64_t)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->job_counts, 4 * sizeof(uint32_t)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipHostMalloc(&e->h_hdr_pinned, 2 * sizeof(WaveHdr)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipHostMalloc(&e->h_err_pinned, sizeof(uint32_t)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipHostMalloc(&e->h_ctl_pinned, sizeof(TrajCtl)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->t_ctl, sizeof(TrajCtl)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->t_wtot, TRAJ_WAVE_CAP * sizeof(uint4)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->t_wbase, TRAJ_WAVE_CAP * sizeof(TrajBase)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->t_mgen, CLS_MAX * CLS_ROW * sizeof(MergeGen)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->t_tmpl, (size_t)CLS_MAX * CLS_ROW * TF * sizeof(TmplRec)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->t_cstat, CLS_MAX * TSTAT * sizeof(uint32_t)) != hipSuccess) return cleanup(ZB_ENOMEM);
  e->ev.resize(EV_PER_WAVE * WAVES_PER_SYNC);
  for (auto& x : e->ev)
    if (hipEventCreate(&x) != hipSuccess) return cleanup(ZB_EDEVICE);
  const uint8_t empty = 0x80;
  add_blob(e->static_blobs, &empty, 1);  // ref 0 = {} (DocumentValue.EMPTY_DOCUMENT)
  if (hipMemcpy(e->arena, e->static_blobs.data(), e->static_blobs.size(), hipMemcpyHostToDevice) != hipSuccess)
    return cleanup(ZB_EDEVICE);
  int rc = zb_reset(e, 0);
  if (rc != ZB_OK) return cleanup(rc);
  *out = e;
  return ZB_OK;
}

void zb_engine_destroy(zb_engine* e) {
  if (!e) return;
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  for (auto& x : e->ev)
    if (x) (void)hipEventDestroy(x);
  void* ps[] = {e->log, e->links, e->rmeta, e->rkeys, e->arena, e->hdr, e->derr, e->dstats, e->derr_info,
                e->merge_jobs, e->cond_jobs, e->job_counts, e->cw, e->stage, e->info, e->block_agg, e->block_off,
                e->t_agg, e->t_woff, e->t_wcount, e->t_wtot, e->t_wbase, e->t_ctl, e->t_mgen, e->t_wstats,
                e->c_plan, e->c_ikey, e->c_khist, e->c_mask, e->c_woffw, e->c_wgcnt, e->c_wgoff, e->c_perm,
                e->t_tmpl, e->t_cstat, e->c_segs, e->c_wcls};
  for (void* p : ps)
    if (p) (void)hipFree(p);
  if (e->comm) (void)ncclCommDestroy(e->comm);
  void* ms[] = {e->obox[0], e->obox[1], e->okeys[0], e->okeys[1], e->on, e->subs, e->sub_head, e->sub_next,
                e->msgs, e->msg_head, e->msg_next, e->d_xcounts};
  for (void* p : ms)
    if (p) (void)hipFree(p);
  if (e->h_hdr_pinned) (void)hipHostFree(e->h_hdr_pinned);
  if (e->h_err_pinned) (void)hipHostFree(e->h_err_pinned);
  if (e->h_ctl_pinned) (void)hipHostFree(e->h_ctl_pinned);
  e->d_elems.free(); e->d_wfs.free(); e->d_cond.free(); e->d_code.free(); e->d_consts.free();
  e->d_queries.free(); e->d_filters.free(); e->d_pool.free(); e->d_staged.free(); e->d_staged_arena.free();
  e->d_ranges.free(); e->d_cmd_pool.free();
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
}

const char* zb_last_error(const zb_engine* e) { return e ? e->err.c_str() : "null engine"; }

int zb_reset(zb_engine* e, int keep_staged) {
  if (!e) return ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  e->wave = 0;
  e->failed = false;
  WaveHdr h{};
  h.begin = h.end = h.gen_end = 0;
  h.wf_next = 1;   // KeyGenerator.createWorkflowInstanceKeyGenerator: (1, 5)
  h.job_next = 2;  // KeyGenerator.createJobKeyGenerator: (2, 5)
  h.rows_next = 0;
  h.arena_next = (int64_t)STATIC_ARENA_BYTES;
  e->host_hdr = h;
  HIPCHECK(e, hipMemcpyAsync(e->hdr, &h, sizeof(h), hipMemcpyHostToDevice, e->stream));
  HIPCHECK(e, hipMemsetAsync(e->derr, 0, sizeof(uint32_t), e->stream));
  HIPCHECK(e, hipMemsetAsync(e->derr_info, 0xff, sizeof(uint64_t), e->stream));
  HIPCHECK(e, hipMemsetAsync(e->job_counts, 0, 4 * sizeof(uint32_t), e->stream));
  HIPCHECK(e, hipMemsetAsync(e->dstats, 0, 8 * sizeof(uint64_t), e->stream));
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  e->ranges.clear();
  e->cmd_pool.clear();
  if (!keep_staged) {
    e->staged.clear();
    e->staged_arena.clear();
    e->pending_ranges.clear();
    e->staged_uploaded = false;
  }
  e->staged_pending = !e->staged.empty();
  e->sub_count = e->msg_count = 0;
  e->msg_key_next = 0;
  if (e->on) HIPCHECK(e, hipMemsetAsync(e->on, 0, 2 * sizeof(uint32_t), e->stream));
  if (e->subs) {
    HIPCHECK(e, hipMemsetAsync(e->sub_head, 0xff, (e->head_mask + 1) * sizeof(uint32_t), e->stream));
    HIPCHECK(e, hipMemsetAsync(e->msg_head, 0xff, (e->head_mask + 1) * sizeof(uint32_t), e->stream));
  }
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  return ZB_OK;
}

int zb_deploy(zb_engine* e, int64_t workflow_key, int32_t version, const uint8_t* xml, size_t len) {
  if (!e || !xml) return ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  std::string msg;
  int rc = compile_deployment(e->model, std::string((const char*)xml, len), workflow_key, version, msg);
  if (rc != ZB_OK) return fail(e, rc, msg);
  for (const DevElem& el : e->model.elems) {
    if (el.step[WI_ELEMENT_COMPLETING] == ST_APPLY_OUTPUT_MAPPING) e->has_merges = true;
    if (el.step[WI_GATEWAY_ACTIVATED] == ST_EXCLUSIVE_SPLIT) e->has_splits = true;
    if (el.kind == EK_CATCH) e->has_catch = true;
  }
  if (e->has_catch) {
    int orc = ensure_outbox(e);
    if (orc != ZB_OK) return orc;
  }
  // the trajectory count pass skips payload merges, so conditions must never read a merge result
  e->traj_model_ok = !(e->has_merges && e->has_splits);
  // class batches: every split of the model is one digit (radix conditions + 2) of an 8-bit outcome key
  e->nsplits = 0;
  e->cls_ok = true;
  uint32_t stride = 1;
  for (size_t i = 0; i < e->model.elems.size() && e->cls_ok; i++) {
    const DevElem& el = e->model.elems[i];
    if (el.step[WI_GATEWAY_ACTIVATED] != ST_EXCLUSIVE_SPLIT) continue;
    const uint32_t radix = (uint32_t)el.cond_count + 2;
    if (e->nsplits == CLS_MAX_SPLITS || (uint64_t)stride * radix > 256) { e->cls_ok = false; break; }
    e->split_elem[e->nsplits] = (uint32_t)i;
    e->split_stride[e->nsplits] = stride;
    e->nsplits++;
    stride *= radix;
  }
  if (!e->cls_ok) e->nsplits = 0;
  return upload_model(e);
}

int zb_set_job_completion_payload(zb_engine* e, int64_t workflow_key, const char* activity_id, const uint8_t* payload,
                                  size_t len) {
  if (!e || !activity_id) return ZB_EINVAL;
  int wfi = -1;
  for (size_t i = 0; i < e->model.workflows.size(); i++)
    if (e->model.workflows[i].key == workflow_key) wfi = (int)i;
  if (wfi < 0) return fail(e, ZB_EINVAL, "unknown workflow key");
  bool found = false;
  uint32_t ref = 0;
  if (len > 0 && !(len == 1 && payload[0] == 0xc0)) {
    if ((payload[0] & 0xf0) != 0x80 && payload[0] != 0xde && payload[0] != 0xdf)
      return fail(e, ZB_EINVAL, "job payload must be a msgpack map");
    ref = add_blob(e->static_blobs, payload, (uint32_t)len);
  }
  for (size_t i = 0; i < e->model.elems.size(); i++) {
    DevElem& el = e->model.elems[i];
    if (el.wf == wfi && el.kind == EK_TASK && e->model.elem_ids[i] == activity_id) {
      el.job_payload = ref;
      found = true;
    }
  }
  if (!found) return fail(e, ZB_EINVAL, "no service task with that id");
  return upload_model(e);
}

int zb_submit_creates(zb_engine* e, const char* pid, int32_t version, int64_t workflow_key, size_t n,
                      const uint8_t* payloads, const uint64_t* offsets) {
  if (!e || (n > 0 && (!payloads || !offsets)) || !pid) return ZB_EINVAL;
  // resolve like CreateWorkflowInstanceEventProcessor (all workflows are deployed locally)
  uint16_t pelem = NO_ELEM;
  const std::string spid(pid);
  const auto& W = e->model.workflows;
  if (workflow_key > 0) {
    for (auto& w : W)
      if (w.key == workflow_key) pelem = w.process_elem;
  } else if (version > 0) {
    for (auto& w : W)
      if (w.version == version && e->model.str(w.pid_off, w.pid_len) == spid) pelem = w.process_elem;
  } else {
    int32_t best = INT32_MIN;
    for (auto& w : W)
      if (e->model.str(w.pid_off, w.pid_len) == spid && w.version > best) { best = w.version; pelem = w.process_elem; }
  }
  if (!e->staged_pending) {  // the previous batch was injected: start a new one
    e->staged.clear();
    e->staged_arena.clear();
    e->pending_ranges.clear();
    e->staged_uploaded = false;
  }
  if (e->staged.empty()) {
    e->staged_elem = pelem;
    e->staged_uniform = true;
    e->staged_max_len = 1;
  } else if (n > 0 && pelem != e->staged_elem) {
    e->staged_uniform = false;
  }
  zb_engine::PendingRange pr;
  pr.first = (int64_t)e->staged.size();
  pr.last = pr.first + (int64_t)n;
  pr.workflow_key = workflow_key;
  pr.version = version;
  pr.pid_off = (uint32_t)e->cmd_pool.size();
  pr.pid_len = (uint16_t)spid.size();
  e->cmd_pool.insert(e->cmd_pool.end(), spid.begin(), spid.end());
  e->staged.reserve(e->staged.size() + n);
  for (size_t i = 0; i < n; i++) {
    const uint8_t* p = payloads + offsets[i];
    uint64_t len = offsets[i + 1] - offsets[i];
    uint32_t ref;
    if (len == 0 || (len == 1 && p[0] == 0xc0)) {
      const uint8_t empty = 0x80;  // DocumentValue: nil / empty -> {}
      ref = add_blob(e->staged_arena, &empty, 1);
    } else {
      uint8_t b = p[0];
      if (!((b & 0xf0) == 0x80 || b == 0xde || b == 0xdf))
        return fail(e, ZB_EINVAL, "Document has invalid format. On root level an object is only allowed.");
      ref = add_blob(e->staged_arena, p, (uint32_t)len);
      e->staged_max_len = std::max<uint32_t>(e->staged_max_len, (uint32_t)len);
    }
    zb_rec d;
    d.key = -1;
    d.scope_key = -1;
    d.inst_key = -1;
    d.payload = ref;
    d.elem = pelem;
    d.intent = WI_CREATE;
    d.kind = make_kind(ZB_VT_WORKFLOW_INSTANCE, ZB_RT_COMMAND, false);
    e->staged.push_back(d);
  }
  e->pending_ranges.push_back(pr);
  e->staged_uploaded = false;
  e->staged_pending = true;
  return ZB_OK;
}

int zb_step(zb_engine* e, uint32_t max_waves, zb_step_stats* stats) {
  if (!e) return ZB_EINVAL;
  if (e->failed) return fail(e, ZB_EPROCESSING, "partition stopped after a processing failure: " + e->err);
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  auto t0 = std::chrono::steady_clock::now();
  zb_step_stats st{};
  bool try_traj = false;
  int64_t traj_base = 0, traj_n = 0;
  // ---- inject staged input at the log tail (engine is quiescent between steps)
  if (e->staged_pending && !e->staged.empty()) {
    // an idle partition fed only CREATE commands runs as independent trajectories (zb_traj.hip)
    try_traj = !(e->cfg.flags & ZB_CFG_WAVE_ONLY) && max_waves == 0 &&
               (e->traj_model_ok || (e->cls_ok && e->staged_uniform)) &&
               e->host_hdr.begin == e->host_hdr.end;
    traj_base = e->host_hdr.end;
    traj_n = (int64_t)e->staged.size();
    const int64_t n = (int64_t)e->staged.size();
    if ((uint64_t)(e->host_hdr.end + n) > e->cfg.log_capacity) return fail(e, ZB_ENOMEM, "log capacity");
    if ((uint64_t)e->host_hdr.arena_next + e->staged_arena.size() > e->cfg.arena_bytes)
      return fail(e, ZB_ENOMEM, "arena capacity");
    if (!e->staged_uploaded) {
      HIPCHECK(e, e->d_staged.upload(e->staged, e->stream));
      HIPCHECK(e, e->d_staged_arena.upload(e->staged_arena, e->stream));
      e->staged_uploaded = true;
    }
    InjectParams ip;
    ip.log = e->log;
    ip.links = e->links;
    ip.arena = e->arena;
    ip.staged = e->d_staged.p;
    ip.staged_arena = e->d_staged_arena.p;
    ip.n = n;
    ip.log_base = e->host_hdr.end;
    ip.arena_base = (uint64_t)e->host_hdr.arena_next;
    ip.staged_bytes = e->staged_arena.size();
    launch_inject(ip, e->stream);
    for (auto& pr : e->pending_ranges) {
      CmdRange r{};
      r.pos_begin = ip.log_base + pr.first;
      r.pos_end = ip.log_base + pr.last;
      r.workflow_key = pr.workflow_key;
      r.version = pr.version;
      r.pid_off = pr.pid_off;
      r.pid_len = pr.pid_len;
      e->ranges.push_back(r);
    }
    if (e->host_hdr.begin == e->host_hdr.gen_end) e->host_hdr.gen_end = e->host_hdr.end + n;
    e->host_hdr.end += n;
    e->host_hdr.arena_next += (int64_t)e->staged_arena.size();
    HIPCHECK(e, hipMemcpyAsync(e->hdr + (e->wave & 1), &e->host_hdr, sizeof(WaveHdr), hipMemcpyHostToDevice,
                               e->stream));
    e->staged_pending = false;
  }
  const int64_t processed_from = e->host_hdr.begin;
  const int64_t written_from = e->host_hdr.end;
  uint64_t stats_before[8];
  HIPCHECK(e, hipMemcpy(stats_before, e->dstats, sizeof(stats_before), hipMemcpyDeviceToHost));
  uint32_t launched = 0;
  bool quiescent = e->host_hdr.begin == e->host_hdr.end;
  if (try_traj && !quiescent) {
    int rc = run_trajectory(e, traj_base, traj_n, st, true);
    if (rc < 0) return rc;
    quiescent = e->host_hdr.begin == e->host_hdr.end;
  }
  while (!quiescent && (max_waves == 0 || launched < max_waves)) {
    int batch = WAVES_PER_SYNC;
    if (max_waves) batch = std::min<int>(batch, (int)(max_waves - launched));
    for (int i = 0; i < batch; i++) {
      WaveParams p = wave_params(e);
      hipEvent_t* ev = &e->ev[EV_PER_WAVE * i];
      HIPCHECK(e, hipEventRecord(ev[0], e->stream));
      launch_process(p, e->stream);
      HIPCHECK(e, hipEventRecord(ev[1], e->stream));
      launch_scan(p, e->stream);
      launch_emit(p, e->stream);
      HIPCHECK(e, hipEventRecord(ev[2], e->stream));
      // payload kernels for this wave's deferred work (only when the model can produce any)
      if (e->has_merges) launch_merge(p, e->stream);
      if (e->has_splits) launch_cond(p, e->stream);
      HIPCHECK(e, hipEventRecord(ev[3], e->stream));
      e->wave++;
    }
    HIPCHECK(e, hipGetLastError());
    HIPCHECK(e, hipMemcpyAsync(e->h_hdr_pinned, e->hdr + (e->wave & 1), sizeof(WaveHdr), hipMemcpyDeviceToHost,
                               e->stream));
    HIPCHECK(e, hipMemcpyAsync(e->h_err_pinned, e->derr, sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
    HIPCHECK(e, hipStreamSynchronize(e->stream));
    for (int i = 0; i < batch; i++) {
      const hipEvent_t* ev = &e->ev[EV_PER_WAVE * i];
      float ms0 = 0, ms1 = 0, ms2 = 0;
      HIPCHECK(e, hipEventElapsedTime(&ms0, ev[0], ev[1]));
      HIPCHECK(e, hipEventElapsedTime(&ms1, ev[1], ev[2]));
      HIPCHECK(e, hipEventElapsedTime(&ms2, ev[2], ev[3]));
      st.process_kernel_ms += ms0;
      st.emit_kernel_ms += ms1;
      st.aux_kernel_ms += ms2;
      st.wave_kernel_ms += ms0 + ms1 + ms2;
    }
    launched += batch;
    st.launches += batch;
    e->host_hdr = e->h_hdr_pinned[0];
    int rc = check_device_errors(e, *e->h_err_pinned);
    if (rc != ZB_OK) return rc;
    quiescent = e->host_hdr.begin == e->host_hdr.end;
  }
  uint64_t stats_after[8];
  HIPCHECK(e, hipMemcpy(stats_after, e->dstats, sizeof(stats_after), hipMemcpyDeviceToHost));
  st.records_processed = (uint64_t)(e->host_hdr.begin - processed_from);
  st.records_written = (uint64_t)(e->host_hdr.end - written_from);
  st.transitions = stats_after[0] - stats_before[0];
  st.completed_instances = stats_after[1] - stats_before[1];
  st.merges = stats_after[3] - stats_before[3];
  st.merge_bytes = stats_after[4] - stats_before[4];
  st.condition_payload_bytes = stats_after[5] - stats_before[5];
  st.waves = stats_after[6] - stats_before[6];
  st.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (stats) *stats = st;
  if (!quiescent) return ZB_EAGAIN;
  return ZB_OK;
}

int64_t zb_log_size(zb_engine* e) { return e ? e->host_hdr.end : -1; }

int zb_read_descriptors(zb_engine* e, int64_t start, int64_t count, zb_rec* out) {
  if (!e || start < 0 || count < 0 || start + count > e->host_hdr.end || (!out && count)) return ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  HIPCHECK(e, hipMemcpyAsync(out, e->log + start, count * sizeof(zb_rec), hipMemcpyDeviceToHost, e->stream));
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  return ZB_OK;
}

int zb_drain(zb_engine* e, int64_t start, int64_t count, zb_record_header* headers, uint8_t* values,
             size_t values_cap, size_t* values_len) {
  if (!e || start < 0 || count < 0 || start + count > e->host_hdr.end) return ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  if (count == 0) {
    if (values_len) *values_len = 0;
    return ZB_OK;
  }
  HIPCHECK(e, e->d_ranges.upload(e->ranges, e->stream));
  HIPCHECK(e, e->d_cmd_pool.upload(e->cmd_pool, e->stream));
  uint64_t* d_len = nullptr;
  uint64_t* d_off = nullptr;
  void* d_tmp = nullptr;
  size_t tmp_bytes = 0;
  zb_record_header* d_hdrs = nullptr;
  uint8_t* d_out = nullptr;
  int rc = ZB_OK;
  auto cleanup = [&]() {
    if (d_len) (void)hipFree(d_len);
    if (d_off) (void)hipFree(d_off);
    if (d_tmp) (void)hipFree(d_tmp);
    if (d_hdrs) (void)hipFree(d_hdrs);
    if (d_out) (void)hipFree(d_out);
  };
  SerParams sp{};
  sp.log = e->log;
  sp.arena = e->arena;
  sp.elems = e->d_elems.p;
  sp.wfs = e->d_wfs.p;
  sp.queries = e->d_queries.p;
  sp.pool = e->d_pool.p;
  sp.ranges = e->d_ranges.p;
  sp.nranges = (int32_t)e->ranges.size();
  sp.cmd_pool = e->d_cmd_pool.p;
  sp.start = start;
  sp.count = count;
  do {
    if (hipMalloc(&d_len, (count + 1) * sizeof(uint64_t)) != hipSuccess ||
        hipMalloc(&d_off, (count + 1) * sizeof(uint64_t)) != hipSuccess) { rc = fail(e, ZB_ENOMEM, "drain buffers"); break; }
    if (hipMemsetAsync(d_len, 0, (count + 1) * sizeof(uint64_t), e->stream) != hipSuccess) { rc = ZB_EDEVICE; break; }
    sp.lengths = (uint32_t*)nullptr;
    // size pass writes 32-bit lengths into the low half of a 64-bit array
    SerParams sz = sp;
    sz.lengths = (uint32_t*)d_off;  // scratch
    launch_ser_size(sz, e->stream);
    // widen to 64-bit for the scan: reuse a tiny conversion via hipcub TransformInputIterator
    hipcub::TransformInputIterator<uint64_t, hipcub::CastOp<uint64_t>, const uint32_t*> it(
        (const uint32_t*)d_off, hipcub::CastOp<uint64_t>());
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, it, d_len, (int)count, e->stream) != hipSuccess) {
      rc = fail(e, ZB_EDEVICE, "scan sizing");
      break;
    }
    if (hipMalloc(&d_tmp, tmp_bytes + 16) != hipSuccess) { rc = fail(e, ZB_ENOMEM, "scan temp"); break; }
    if (hipcub::DeviceScan::ExclusiveSum(d_tmp, tmp_bytes, it, d_len, (int)count, e->stream) != hipSuccess) {
      rc = fail(e, ZB_EDEVICE, "scan");
      break;
    }
    uint64_t last_off = 0;
    uint32_t last_len = 0;
    if (hipMemcpyAsync(&last_off, d_len + count - 1, 8, hipMemcpyDeviceToHost, e->stream) != hipSuccess ||
        hipMemcpyAsync(&last_len, ((uint32_t*)d_off) + count - 1, 4, hipMemcpyDeviceToHost, e->stream) != hipSuccess ||
        hipStreamSynchronize(e->stream) != hipSuccess) { rc = fail(e, ZB_EDEVICE, "drain size"); break; }
    const uint64_t total = last_off + last_len;
    if (values_len) *values_len = total;
    if (!values || !headers || values_cap < total) { rc = ZB_ENOMEM; break; }
    if (hipMalloc(&d_out, total + 1) != hipSuccess || hipMalloc(&d_hdrs, count * sizeof(zb_record_header)) != hipSuccess) {
      rc = fail(e, ZB_ENOMEM, "drain output");
      break;
    }
    SerParams wr = sp;
    wr.offsets = d_len;
    wr.out = d_out;
    wr.headers = d_hdrs;
    launch_ser_write(wr, e->stream);
    if (hipMemcpyAsync(values, d_out, total, hipMemcpyDeviceToHost, e->stream) != hipSuccess ||
        hipMemcpyAsync(headers, d_hdrs, count * sizeof(zb_record_header), hipMemcpyDeviceToHost, e->stream) !=
            hipSuccess ||
        hipStreamSynchronize(e->stream) != hipSuccess) { rc = fail(e, ZB_EDEVICE, "drain copy"); break; }
  } while (0);
  cleanup();
  return rc;
}

int zb_submit_publishes(zb_engine* e, const char* name, int64_t ttl, size_t n, const uint8_t* cks,
                        const uint64_t* ck_offsets, const uint8_t* payloads, const uint64_t* payload_offsets) {
  if (!e || !name || (n > 0 && (!cks || !ck_offsets || !payloads || !payload_offsets))) return ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  int rc = require_idle(e);
  if (rc != ZB_OK) return rc;
  if (n == 0) return ZB_OK;
  rc = ensure_stores(e);
  if (rc != ZB_OK) return rc;
  const uint64_t nn = std::strlen(name);
  if (nn > 0xffff) return fail(e, ZB_EINVAL, "message name too long");
  const int per = ttl > 0 ? 1 : 2;
  const int64_t base = e->host_hdr.end;
  if ((uint64_t)(base + (int64_t)n * (1 + per)) > e->cfg.log_capacity) return fail(e, ZB_ENOMEM, "log capacity");
  if ((uint64_t)base + n * (1 + per) >= (1ull << 34)) return fail(e, ZB_EUNSUPPORTED, "log position beyond the outbox order key");
  if (e->msg_count + (ttl > 0 ? n : 0) > e->store_cap) return fail(e, ZB_ENOMEM, "message store capacity");
  // PUBLISH commands (null key) and their message blobs, built on the host and uploaded once
  std::vector<zb_rec> recs(n);
  std::vector<uint8_t> blobs;
  const uint64_t arena0 = (uint64_t)e->host_hdr.arena_next;
  for (size_t i = 0; i < n; i++) {
    const uint8_t* ck = cks + ck_offsets[i];
    const uint64_t nc = ck_offsets[i + 1] - ck_offsets[i];
    const uint8_t* pl = payloads + payload_offsets[i];
    uint64_t np = payload_offsets[i + 1] - payload_offsets[i];
    static const uint8_t EMPTY = 0x80;
    if (np == 0 || (np == 1 && pl[0] == 0xc0)) { pl = &EMPTY; np = 1; }  // DocumentValue: nil / empty -> {}
    else if (!((pl[0] & 0xf0) == 0x80 || pl[0] == 0xde || pl[0] == 0xdf))
      return fail(e, ZB_EINVAL, "Document has invalid format. On root level an object is only allowed.");
    if (nc > 0xffff) return fail(e, ZB_EINVAL, "correlation key too long");
    const size_t off = blobs.size();
    const uint32_t len = (uint32_t)(16 + nn + nc + np);
    blobs.resize(off + ((4 + len + 7) & ~(size_t)7), 0);
    uint8_t* b = blobs.data() + off;
    std::memcpy(b, &len, 4);
    std::memcpy(b + 4, &ttl, 8);
    const uint16_t n16 = (uint16_t)nn, c16 = (uint16_t)nc;
    const uint32_t p32 = (uint32_t)np;
    std::memcpy(b + 12, &n16, 2);
    std::memcpy(b + 14, &c16, 2);
    std::memcpy(b + 16, &p32, 4);
    std::memcpy(b + 20, name, nn);
    std::memcpy(b + 20 + nn, ck, nc);
    std::memcpy(b + 20 + nn + nc, pl, np);
    zb_rec& d = recs[i];
    d.key = -1; d.scope_key = -1; d.inst_key = -1;
    d.payload = (uint32_t)((arena0 + off) >> 3);
    d.elem = NO_ELEM; d.intent = 0;  // PUBLISH
    d.kind = make_kind(ZB_VT_MESSAGE, ZB_RT_COMMAND, false);
  }
  if (arena0 + blobs.size() > e->cfg.arena_bytes) return fail(e, ZB_ENOMEM, "arena capacity");
  HIPCHECK(e, hipMemcpyAsync(e->log + base, recs.data(), n * sizeof(zb_rec), hipMemcpyHostToDevice, e->stream));
  HIPCHECK(e, hipMemcpyAsync(e->arena + arena0, blobs.data(), blobs.size(), hipMemcpyHostToDevice, e->stream));
  HIPCHECK(e, hipMemsetAsync(e->links + base, 0xff, n * sizeof(uint64_t), e->stream));
  MsgParams p = msg_params(e);
  p.n = (int64_t)n;
  p.base = base;
  p.ttl = ttl;
  p.key_base = e->msg_key_next;
  launch_msg_publish(p, e->stream);
  e->msg_key_next += (int64_t)n;
  if (ttl > 0) e->msg_count += n;
  e->host_hdr.end = base + (int64_t)n * (1 + per);
  e->host_hdr.begin = e->host_hdr.gen_end = e->host_hdr.end;
  e->host_hdr.arena_next += (int64_t)blobs.size();
  return finish_batch(e);
}

int zb_inbox_submit(zb_engine* e, int kind, const zb_exchange_rec* src, size_t n, int src_on_device) {
  if (!e || (n > 0 && !src) || (kind != ZB_XCHG_OPEN && kind != ZB_XCHG_CORRELATE)) return ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  int rc = require_idle(e);
  if (rc != ZB_OK) return rc;
  if (n == 0) return ZB_OK;
  rc = ensure_stores(e);
  if (rc != ZB_OK) return rc;
  const int64_t base = e->host_hdr.end;
  const uint64_t recs = kind == ZB_XCHG_OPEN ? 2 * n : n;
  const uint64_t stride = kind == ZB_XCHG_OPEN ? SUB_BLOB : WIS_BLOB;
  if ((uint64_t)base + recs > e->cfg.log_capacity) return fail(e, ZB_ENOMEM, "log capacity");
  if ((uint64_t)base + recs >= (1ull << 34)) return fail(e, ZB_EUNSUPPORTED, "log position beyond the outbox order key");
  if ((uint64_t)e->host_hdr.arena_next + n * stride > e->cfg.arena_bytes) return fail(e, ZB_ENOMEM, "arena capacity");
  if (kind == ZB_XCHG_OPEN && (e->sub_count + n > e->store_cap || e->sub_count + n >= (1ull << 24)))
    return fail(e, ZB_ENOMEM, "subscription store capacity");
  const zb_exchange_rec* dsrc = src;
  zb_exchange_rec* tmp = nullptr;
  if (!src_on_device) {
    HIPCHECK(e, hipMalloc(&tmp, n * sizeof(zb_exchange_rec)));
    HIPCHECK(e, hipMemcpyAsync(tmp, src, n * sizeof(zb_exchange_rec), hipMemcpyHostToDevice, e->stream));
    dsrc = tmp;
  }
  MsgParams p = msg_params(e);
  p.in = dsrc;
  p.n = (int64_t)n;
  p.base = base;
  p.arena_base = (uint64_t)e->host_hdr.arena_next;
  if (kind == ZB_XCHG_OPEN) {
    launch_msg_open(p, e->stream);  // processed at once: OPEN commands + OPENED events
    e->sub_count += n;
    e->host_hdr.end = base + (int64_t)recs;
    e->host_hdr.begin = e->host_hdr.gen_end = e->host_hdr.end;
  } else {
    launch_wis_inject(p, e->stream);  // CORRELATE commands: the next zb_step processes them
    e->host_hdr.end = base + (int64_t)recs;
    e->host_hdr.gen_end = e->host_hdr.end;
  }
  e->host_hdr.arena_next += (int64_t)(n * stride);
  rc = finish_batch(e);
  if (tmp) (void)hipFree(tmp);
  return rc;
}

int zb_outbox_count(zb_engine* e, int kind, uint64_t* n) {
  if (!e || !n || (kind != ZB_XCHG_OPEN && kind != ZB_XCHG_CORRELATE)) return ZB_EINVAL;
  *n = 0;
  if (!e->on) return ZB_OK;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  uint32_t c = 0;
  HIPCHECK(e, hipMemcpyAsync(&c, e->on + (kind - 1), sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  *n = c;
  return ZB_OK;
}

int zb_outbox_take(zb_engine* e, int kind, zb_exchange_rec* dst, size_t cap, int dst_on_device, uint64_t* counts,
                   uint64_t* n_out) {
  if (!e || !counts || !n_out || (kind != ZB_XCHG_OPEN && kind != ZB_XCHG_CORRELATE)) return ZB_EINVAL;
  const int P = e->cfg.partition_count;
  if (P > 64) return fail(e, ZB_EUNSUPPORTED, "more than 64 partitions");
  for (int q = 0; q < P; q++) counts[q] = 0;
  uint64_t n = 0;
  int rc = zb_outbox_count(e, kind, &n);
  if (rc != ZB_OK) return rc;
  *n_out = n;
  if (n == 0) return ZB_OK;
  if (n > cap || !dst) return fail(e, ZB_ENOMEM, "outbox destination too small");
  if (n > e->ocap) return fail(e, ZB_ENOMEM, "outbox overflow");
  const int k = kind - 1;
  // sort (key, index) pairs: target partition, source position, emission order
  uint64_t* keys_out = nullptr;
  uint32_t *idx_in = nullptr, *idx_out = nullptr;
  uint64_t* first = nullptr;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  zb_exchange_rec* staging = nullptr;
  auto cleanup = [&]() {
    void* ps[] = {keys_out, idx_in, idx_out, first, tmp, staging};
    for (void* q : ps)
      if (q) (void)hipFree(q);
  };
  do {
    if (hipMalloc(&keys_out, n * 8) != hipSuccess || hipMalloc(&idx_in, n * 4) != hipSuccess ||
        hipMalloc(&idx_out, n * 4) != hipSuccess || hipMalloc(&first, (P + 1) * 8) != hipSuccess) {
      rc = fail(e, ZB_ENOMEM, "outbox sort buffers");
      break;
    }
    launch_iota(idx_in, n, e->stream);
    if (hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, e->okeys[k], keys_out, idx_in, idx_out, (int)n, 0, 64,
                                           e->stream) != hipSuccess ||
        hipMalloc(&tmp, tmp_bytes + 16) != hipSuccess ||
        hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, e->okeys[k], keys_out, idx_in, idx_out, (int)n, 0, 64,
                                           e->stream) != hipSuccess) {
      rc = fail(e, ZB_EDEVICE, "outbox sort");
      break;
    }
    zb_exchange_rec* out = dst;
    if (!dst_on_device) {
      if (hipMalloc(&staging, n * sizeof(zb_exchange_rec)) != hipSuccess) { rc = fail(e, ZB_ENOMEM, "outbox staging"); break; }
      out = staging;
    }
    launch_outbox_gather(e->obox[k], idx_out, out, n, e->stream);
    launch_outbox_bounds(keys_out, n, first, P, e->stream);
    std::vector<uint64_t> h_first(P, 0);
    if (hipMemcpyAsync(h_first.data(), first, P * 8, hipMemcpyDeviceToHost, e->stream) != hipSuccess ||
        (!dst_on_device && hipMemcpyAsync(dst, staging, n * sizeof(zb_exchange_rec), hipMemcpyDeviceToHost, e->stream) !=
                               hipSuccess) ||
        hipMemsetAsync(e->on + k, 0, sizeof(uint32_t), e->stream) != hipSuccess ||
        hipStreamSynchronize(e->stream) != hipSuccess) {
      rc = fail(e, ZB_EDEVICE, "outbox copy");
      break;
    }
    for (int q = 0; q < P; q++) counts[q] = (q + 1 < P ? h_first[q + 1] : n) - h_first[q];
  } while (0);
  cleanup();
  return rc;
}

#define NCCLCHECK(e, call)                                                                      \
  do {                                                                                          \
    ncclResult_t _r = (call);                                                                   \
    if (_r != ncclSuccess) return fail((e), ZB_EDEVICE, std::string(#call) + ": " + ncclGetErrorString(_r)); \
  } while (0)

int zb_comm_unique_id(uint8_t id[128]) {
  if (!id) return ZB_EINVAL;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return ZB_EDEVICE;
  std::memcpy(id, &u, sizeof(u));
  return ZB_OK;
}

int zb_comm_init(zb_engine* e, const uint8_t id[128], int nranks, int rank) {
  if (!e || !id || nranks != e->cfg.partition_count || rank != e->cfg.partition_id || nranks > 64) return ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  NCCLCHECK(e, ncclCommInitRank(&e->comm, nranks, u, rank));
  HIPCHECK(e, hipMalloc(&e->d_xcounts, 2 * 64 * sizeof(uint64_t)));
  return ensure_outbox(e);
}

int zb_comm_pending(zb_engine* e, uint64_t global[2]) {
  if (!e || !global || !e->comm) return ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  uint64_t local[2] = {0, 0};
  for (int k = 0; k < 2; k++) {
    int rc = zb_outbox_count(e, k + 1, &local[k]);
    if (rc != ZB_OK) return rc;
  }
  HIPCHECK(e, hipMemcpyAsync(e->d_xcounts, local, sizeof(local), hipMemcpyHostToDevice, e->stream));
  NCCLCHECK(e, ncclAllReduce(e->d_xcounts, e->d_xcounts, 2, ncclUint64, ncclSum, e->comm, e->stream));
  HIPCHECK(e, hipMemcpyAsync(global, e->d_xcounts, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, e->stream));
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  return ZB_OK;
}

int zb_comm_exchange(zb_engine* e, int kind, uint64_t* received) {
  if (!e || !received || !e->comm || (kind != ZB_XCHG_OPEN && kind != ZB_XCHG_CORRELATE)) return ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  const int P = e->cfg.partition_count;
  *received = 0;
  uint64_t n = 0;
  int rc = zb_outbox_count(e, kind, &n);
  if (rc != ZB_OK) return rc;
  zb_exchange_rec* send = nullptr;
  zb_exchange_rec* recv = nullptr;
  auto cleanup = [&]() {
    if (send) (void)hipFree(send);
    if (recv) (void)hipFree(recv);
  };
  std::vector<uint64_t> sc(P, 0), rcv(P, 0);
  if (hipMalloc(&send, std::max<uint64_t>(n, 1) * sizeof(zb_exchange_rec)) != hipSuccess) {
    cleanup();
    return fail(e, ZB_ENOMEM, "exchange send buffer");
  }
  uint64_t got = 0;
  rc = zb_outbox_take(e, kind, send, std::max<uint64_t>(n, 1), 1, sc.data(), &got);
  if (rc != ZB_OK) { cleanup(); return rc; }
  // 1. counts: every rank learns how many commands each source sends it
  if (hipMemcpyAsync(e->d_xcounts, sc.data(), P * 8, hipMemcpyHostToDevice, e->stream) != hipSuccess) {
    cleanup();
    return fail(e, ZB_EDEVICE, "exchange counts upload");
  }
  ncclResult_t nr = ncclGroupStart();
  for (int q = 0; q < P && nr == ncclSuccess; q++) {
    nr = ncclSend(e->d_xcounts + q, 1, ncclUint64, q, e->comm, e->stream);
    if (nr == ncclSuccess) nr = ncclRecv(e->d_xcounts + 64 + q, 1, ncclUint64, q, e->comm, e->stream);
  }
  if (nr == ncclSuccess) nr = ncclGroupEnd();
  if (nr != ncclSuccess) { cleanup(); return fail(e, ZB_EDEVICE, std::string("exchange counts: ") + ncclGetErrorString(nr)); }
  if (hipMemcpyAsync(rcv.data(), e->d_xcounts + 64, P * 8, hipMemcpyDeviceToHost, e->stream) != hipSuccess ||
      hipStreamSynchronize(e->stream) != hipSuccess) {
    cleanup();
    return fail(e, ZB_EDEVICE, "exchange counts download");
  }
  uint64_t total = 0;
  for (int q = 0; q < P; q++) total += rcv[q];
  if (hipMalloc(&recv, std::max<uint64_t>(total, 1) * sizeof(zb_exchange_rec)) != hipSuccess) {
    cleanup();
    return fail(e, ZB_ENOMEM, "exchange receive buffer");
  }
  // 2. records: slices by target out, by source in (source-rank order = canonical delivery order)
  nr = ncclGroupStart();
  uint64_t so = 0, ro = 0;
  for (int q = 0; q < P && nr == ncclSuccess; q++) {
    if (sc[q]) nr = ncclSend(send + so, sc[q] * sizeof(zb_exchange_rec), ncclUint8, q, e->comm, e->stream);
    if (nr == ncclSuccess && rcv[q]) nr = ncclRecv(recv + ro, rcv[q] * sizeof(zb_exchange_rec), ncclUint8, q, e->comm, e->stream);
    so += sc[q];
    ro += rcv[q];
  }
  if (nr == ncclSuccess) nr = ncclGroupEnd();
  if (nr != ncclSuccess) { cleanup(); return fail(e, ZB_EDEVICE, std::string("exchange records: ") + ncclGetErrorString(nr)); }
  if (hipStreamSynchronize(e->stream) != hipSuccess) { cleanup(); return fail(e, ZB_EDEVICE, "exchange sync"); }
  rc = total ? zb_inbox_submit(e, kind, recv, total, 1) : ZB_OK;
  cleanup();
  if (rc == ZB_OK) *received = total;
  return rc;
}

int zb_counters(zb_engine* e, int64_t out[8]) {
  if (!e || !out) return ZB_EINVAL;
  uint64_t s[8];
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  HIPCHECK(e, hipMemcpy(s, e->dstats, sizeof(s), hipMemcpyDeviceToHost));
  out[0] = (int64_t)s[2];
  out[1] = (int64_t)s[1];
  out[2] = 0;
  out[3] = e->host_hdr.wf_next;
  out[4] = e->host_hdr.job_next;
  out[5] = e->host_hdr.rows_next;
  out[6] = e->host_hdr.arena_next;
  out[7] = e->host_hdr.end;
  return ZB_OK;
}

}  // extern "C"
