// zb_engine.hip — host side of libzbgpu.so: the C ABI of include/zb_engine.h.
//
// One handle = one partition on one HIP device with one stream. zb_step launches one wave
// kernel per breadth-first generation, in batches of WAVES_PER_SYNC launches between host
// checks of the device wave header (quiescence = empty generation). No CPU fallback exists:
// every record is processed by the gfx950 kernels, and anything they do not implement is
// reported as ZB_EUNSUPPORTED.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rocprim/device/device_radix_sort.hpp>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "zb_devlib.hpp"
#include "zb_xmerge.hpp"
#include "zb_kernels.hpp"
#include "zb_model.hpp"
#include "zb_msg.hpp"

using namespace zbg;

namespace {

constexpr int WAVES_PER_SYNC = 16;      // the first batch; each later batch of the step doubles, up to
constexpr int WAVES_PER_SYNC_MAX = 64;  // (long chains: fewer host round trips, at most one batch of empty waves)
constexpr int TRAJ_RETRY = 15;  // batches that go straight to the wave pipeline after a trajectory fallback
constexpr int JOB_COUNTS = 8 + 2 * SUB_STRIPES;  // merge / cond / (unused) / slow-merge counts, the subscribe stripes
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

// a PUBLISH batch resident in p_in (zb_upload_publishes): byte offsets of its pieces
struct PubUpload {
  bool valid;
  uint64_t n;
  uint32_t nn;
  int64_t ttl;
  uint64_t a_ck, a_cko, a_pl, a_plo, a_name;
  uint64_t gran;  // the batch's blob granules (8 bytes), scanned at upload
};

struct zb_engine {
  zb_config cfg{};
  hipStream_t stream = nullptr;
  int32_t ncu = 256;            // compute units of the device
  int32_t wave_fused_grid = 0;  // k_wave: resident workgroups (0 = three-kernel pipeline; ZB_CFG_WAVE_SPLIT forces it)
  uint64_t* lookback = nullptr; // k_wave hand-off granules (WaveParams.lookback)
  uint64_t lb_tiles = 0;
  uint64_t lb_seq = 0;          // k_wave launches (aggregate tags: 1 + lb_seq % 255)
  std::string err;

  ModelTables model;
  DevVec<DevElem> d_elems;
  DevVec<DevWorkflow> d_wfs;
  DevVec<uint16_t> d_cond;
  DevVec<uint32_t> d_code;
  DevVec<uint32_t> d_cls_code;  // the program with the split conditions' path operands as extraction slots
  DevVec<uint32_t> d_cls_atom;  // outcome table (k_cls_classify): the conditions' comparisons (their code words)
  DevVec<uint8_t> d_cls_table;  //   and the class key of every combination of their outcomes
  int cls_natoms = 0;
  DevVec<DevConst> d_consts;
  DevVec<uint64_t> d_const_w;  // [consts][2] the bytes of string constants of at most 16 bytes (classify)
  DevVec<DevQuery> d_queries;
  DevVec<DevFilter> d_filters;
  DevVec<uint8_t> d_pool;
  DevVec<DevMapping> d_maps;
  DevVec<DevSeg> d_segs;
  bool has_io = false;          // some element has a zeebe:ioMapping (k_map runs, no trajectory path)
  uint64_t* mapres = nullptr;   // k_map outcomes [wave_cap + 8]
  MNode* map_ws = nullptr;      // k_map tree workspaces
  int ser_mode = 0;              // 0 = two passes (size, scan, write), 1 = single pass (look-back, ZB_CFG_SINGLE_PASS_DRAIN)

  // device state. The log arrays hold the window [win_base, win_base + log_capacity) of absolute positions;
  // log / links / srcd / vlen are biased pointers (index = absolute position) into the *_mem allocations, so
  // every kernel indexes by position and the window moves by re-biasing (rebase_log)
  zb_rec* log = nullptr;
  uint64_t* links = nullptr;
  uint32_t* srcd = nullptr;     // per record: position - source position (0: none), for log frames
  uint32_t* vlen = nullptr;     // per record: serialized value length if the emitting kernel knew it
  zb_rec* log_mem = nullptr;
  uint64_t* links_mem = nullptr;
  uint32_t* srcd_mem = nullptr;
  uint32_t* vlen_mem = nullptr;
  int64_t win_base = 0;         // first position the device log holds (earlier ones were released / not restored)
  int64_t released = 0;         // zb_log_release: the caller appended everything below
  DevVec<ValueConst> d_vconst;  // per element: constant parts of its WORKFLOW_INSTANCE / JOB values
  DevVec<DevValSeg> d_vsegs;    // per element: its values' constant runs (fast drain passes)
  DevVec<uint8_t> d_segpool;
  uint32_t segpool_len = 0;
  bool seg_ok = false;          // the runs fit the fast passes' LDS
  uint32_t* vlen_bad = nullptr; // ZB_CFG_VLEN_CHECK: the size pass checks every known length (device flag)
  uint8_t* row_mem = nullptr;   // element-instance rows: the three planes below, one allocation
  RowMeta* rmeta = nullptr;     // [row_capacity]
  RowKeys* rkeys = nullptr;     // [row_capacity]
  RowLink* rlink = nullptr;     // [row_capacity]
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
  uint32_t* job_counts = nullptr;  // [0..1] merge counts, [2..3] cond counts, [4..5] unused,
                                   // [6..7] merges left to the general merger, [8..] subscribe counts [2][SUB_STRIPES]
  uint32_t* merge_slow = nullptr;  // [job_cap] indices of those merges
  unsigned long long* phase = nullptr;  // (ZB_PHASES measurement build) k_wave phase sums
  PubUpload pub_up{};                   // a PUBLISH batch uploaded by zb_upload_publishes, not processed yet
  uint8_t* xslab = nullptr;        // exact payload tree workspaces (zb_xmerge.hpp), with a model that merges / maps
  uint32_t* xlocks = nullptr;
  uint8_t* xlane = nullptr;        // per-thread exact-tree workspaces (XLANE_COUNT x XLANE_BYTES), with xslab
  bool xpool_held = false;         // xslab / xlocks / xlane are the device's shared set (xpool_acquire)
  uint64_t* sub_jobs = nullptr;    // [job_cap] subscribe steps of a wave (models with message catch events)
  uint64_t job_cap = 0;
  WaveHdr* h_hdr_pinned = nullptr;  // pinned mirror for D2H polling
  uint32_t* h_err_pinned = nullptr;

  int64_t wave = 0;
  WaveHdr host_hdr{};
  bool has_merges = false, has_splits = false;
  bool has_tasks = false;  // some deployed element is a service task (writes JOB CREATE commands)
  bool failed = false;

  // static arena region (ref 0 = {}, harness payloads)
  std::vector<uint8_t> static_blobs;

  // staged input
  std::vector<zb_rec> staged;
  std::vector<uint32_t> staged_vlen;   // value length of each staged record (VLEN_UNKNOWN: measured at drain)
  DevVec<uint32_t> d_staged_vlen;
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
  // Staged CREATE documents are uploaded in place, into the top of the arena (k_inject references them, no copy):
  // the device allocators grow [STATIC, arena_next) up to arena_top, and [arena_top, arena_bytes) holds the
  // documents of staged batches, newest lowest. Compaction moves the live ones down with everything else.
  uint64_t arena_top = 0;        // the device allocators' ceiling (arena_bytes when no documents are in place)
  bool staged_in_place = false;  // the uploaded batch's documents are at [staged_base, staged_top)
  uint64_t staged_base = 0, staged_top = 0;
  bool staged_pending = false;  // the staged batch has not been injected yet (zb_reset(keep) re-arms it)
  uint16_t staged_elem = NO_ELEM;  // process element of the staged CREATEs ...
  bool staged_uniform = true;      // ... when they all address the same one
  uint32_t staged_max_len = 1;     // longest staged CREATE payload (uniform batch merge bounds)

  // request metadata: of staged records (staged index), then of injected ones (log position, sorted)
  using StagedReq = zbg::StagedReq;
  std::vector<StagedReq> staged_reqs;
  DevVec<StagedReq> d_staged_reqs;  // (uploaded with the staged batch)
  bool staged_reqs_uploaded = false;
  // request metadata of the injected commands, device-resident and sorted by position (k_req_append at each injection,
  // no host copy): entries [req_lo, req_n) are live; one run per injection (its positions and entries)
  ReqMeta* d_req = nullptr;
  uint64_t req_cap = 0, req_lo = 0, req_n = 0;
  struct ReqRun { int64_t first, last; uint64_t lo, n; };
  std::vector<ReqRun> req_runs;

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
  uint64_t* t_xq = nullptr;        // the template emit's exact-tree queue (TrajParams.xq), one entry per instance
  uint64_t t_xq_cap = 0;
  MergeGen* t_mgen = nullptr;     // [TRAJ_MAX_GENERATIONS] uniform batch merge slots
  uint64_t* t_wstats = nullptr;   // [t_nwg_cap + CLS_MAX][6] emit statistics per workgroup
  TrajCtl* h_ctl_pinned = nullptr;
  uint64_t* h_stats_pinned = nullptr;  // [0..7] counters before a step, [8..15] after, [16] a class batch's ClsPlan.nc,
                                       // [17] sort_pairs' key spread, [18] the waves counter before a wave loop,
                                       // [19..20] the outbox counts (zb_outbox_count)
  // class batches (zb_traj.hip k_cls_*): the model's exclusive splits as outcome-key digits
  bool cls_ok = false;            // split outcome keys fit 8 bits and CLS_MAX_SPLITS splits
  int nsplits = 0;
  int cls_nq = 0;                 // distinct fast queries of the split conditions (k_cls_classify extraction)
  uint16_t cls_q[CLS_QMAX] = {};
  uint32_t cls_key_off[CLS_QMAX] = {}, cls_key_len[CLS_QMAX] = {};
  uint64_t cls_key_w[CLS_QMAX][2] = {};
  uint32_t split_elem[CLS_MAX_SPLITS] = {}, split_stride[CLS_MAX_SPLITS] = {};
  ClsPlan* c_plan = nullptr;
  uint64_t cls_cap = 0;           // instances the class buffers hold
  uint8_t* c_ikey = nullptr;
  uint32_t* c_clen = nullptr;
  uint32_t* d_cref = nullptr;  // [cref_cap] the last injected batch's payload refs (k_inject), at log position cref_base
  uint64_t cref_cap = 0;
  int64_t cref_base = -1;
  uint32_t *c_khist = nullptr, *c_krep = nullptr;  // [CLS_HB][256] each (one allocation with c_klen)
  uint64_t* c_klen = nullptr;                       // [CLS_HB][256]
  TmplRec* t_tmpl = nullptr;     // [CLS_MAX][CLS_ROW][TF] traced records (uniform / class batches)
  uint32_t* t_cstat = nullptr;   // [CLS_MAX][TSTAT]
  uint64_t* c_mask = nullptr;
  uint32_t* c_cg = nullptr;     // [groups][CLS_MAX][2] CREATE payload bytes per wave and class (k_cls_masks)
  uint32_t *c_woffw = nullptr, *c_wgcnt = nullptr, *c_wgoff = nullptr, *c_perm = nullptr;
  uint32_t *c_segs = nullptr, *c_wcls = nullptr;

  // message correlation (zb_msg.hip): outboxes [0] open-subscription, [1] correlate
  zb_exchange_rec* obox[2] = {nullptr, nullptr};
  uint64_t* okeys[2] = {nullptr, nullptr};
  uint8_t* ovar[2] = {nullptr, nullptr};  // their commands' variable bytes
  uint32_t* on = nullptr;  // [4] device counters: commands of [0] / [1], byte-section granules of [0] / [1]
  int64_t ob_pos_base[2] = {0, 0};  // Outbox.pos_base of [0] / [1]: the processing frontier at its last take
  uint64_t ocap = 0, ovar_cap = 0;        // commands, granules
  int64_t clock_ms = 0;                   // zb_set_clock (ActorClock of the message stream processor)
  // message batches / delivered exchange batches
  uint8_t* m_prior = nullptr;
  uint8_t* p_in = nullptr;        // zb_submit_publishes: the caller's keys / payloads / offsets on the device
  uint64_t p_in_cap = 0;
  uint64_t* p_gran = nullptr;     // [n + 1] blob granules, [n + 1] their scan, error flags
  uint64_t p_gran_cap = 0;
  uint64_t m_prior_cap = 0;
  uint64_t* m_cnt = nullptr;
  uint64_t m_cnt_cap = 0;
  void* m_tmp = nullptr;
  uint64_t m_tmp_cap = 0;
  uint8_t* in_buf = nullptr;
  uint64_t in_buf_cap = 0;
  DevVec<uint64_t> d_slices;
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
  bool comm_broken = false;       // an RCCL call failed: the communicator is not used again
  uint64_t* d_xcounts = nullptr;  // [4 * 64]: (count, status) pairs sent to / received from every rank
  // persistent exchange buffers, bytes (grown geometrically, never freed per round)
  uint8_t* xsend = nullptr;
  uint8_t* xrecv = nullptr;
  uint64_t xsend_cap = 0, xrecv_cap = 0;
  // outbox sort buffers, sized to the outbox capacity once
  uint64_t* ob_keys = nullptr;
  uint32_t *ob_idx_in = nullptr, *ob_idx_out = nullptr;
  uint64_t* ob_first = nullptr;  // [65]
  uint32_t *ob_sizes = nullptr, *ob_goff = nullptr;
  uint64_t *ob_table = nullptr, *ob_base = nullptr;
  void* ob_tmp = nullptr;  // (scan scratch)
  size_t ob_tmp_bytes = 0;
  uint32_t ob_counts_read[2] = {0, 0};  // both outbox command counts at the last zb_outbox_count
  // the outbox counters (commands, granules) in h_stats_pinned[19..20] are current: copied in the round trip that
  // ended the last work able to change them (a wave batch, a delivery, a message batch), so zb_outbox_count
  // needs no round trip of its own; cleared by everything that enqueues such work
  bool ob_counts_valid = false;
  // non-empty waves of the last wave loop, per kind of input (a partition that alternates kinds -- C5: CREATE batches,
  // then the correlations delivered to its inbox -- settles each kind in its own count): 1 staged CREATEs only,
  // 2 other staged records, 3 records already in the log (inbox deliveries)
  int wave_hint[4] = {0, 0, 0, 0};
  int traj_skip = 0;     // batches left that skip the trajectory attempt after a fallback (zb_step)     // non-empty waves of the last step's wave loop (its first batch, zb_step)
  int ob_plan_kind = 0;  // the outbox kind outbox_plan sorted and sized last (0: none)
  uint64_t ob_plan_n = 0, ob_plan_total = 0, ob_plan_base[64] = {};
  uint8_t* ob_staging = nullptr;
  uint64_t ob_staging_cap = 0;

  // scope-wide row state (RowAux), first-live-child requests, wave epoch
  RowAux* raux = nullptr;
  int64_t epoch = 1;
  bool has_parallel = false;
  bool term = false;               // a CANCEL was injected: terminations may run until quiescence
  // zb_submit: per staged record, the key whose element-instance row it needs (INT64_MIN: none)
  std::vector<int64_t> staged_lookup;
  bool staged_only_creates = true;
  bool staged_has_cancel = false;
  // per-tick race rules of zb_submit (include/zb_engine.h)
  std::unordered_map<int64_t, uint8_t> tick_inst;  // workflow instance -> 1: scope command, 2: other records
  std::unordered_set<int64_t> tick_aik;
  std::unordered_set<int64_t> tick_jobs;   // job keys with commands in the staged tick (one group each)
  std::unordered_set<int64_t> tick_conflicts;  // workflow instances whose staged records race (serialised by chunks)
  DevVec<int64_t> d_conf_keys;             // their open-addressing table (uploaded with the batch)
  int64_t* conf_first = nullptr;           // [conf_cap] + conf_split
  uint64_t conf_cap = 0, conf_mask = 0, staged_conf = 0;
  bool conf_active = false;                // the injected tick has conflicting instances: k_conflict every wave
  JobTable jobs{};                         // ZB_CFG_JOB_PROCESSOR: job states by job key (open addressing)
  // compaction (zb_compact.hip): scratch grown on demand, lifetime totals
  uint32_t *c_flag = nullptr, *c_new = nullptr;  // scan input / output (live rows, live messages)
  uint64_t c_flag_cap = 0, c_new_cap = 0;
  void* c_tmp = nullptr;
  size_t c_tmp_cap = 0;
  uint8_t* c_scratch = nullptr;                  // live rows / live arena granules / live messages
  uint64_t c_scratch_cap = 0;
  uint64_t* c_bits = nullptr;                    // arena granule bitmap
  uint64_t c_bits_cap = 0;
  uint32_t *c_pop = nullptr, *c_off = nullptr;   // per-word popcounts and their scan
  uint64_t c_pop_cap = 0, c_off_cap = 0;
  uint32_t* c_count = nullptr;                   // device counter (job rebuild)
  uint64_t rows_total = 0, arena_total = 0, records_total = 0, compactions = 0;  // lifetime allocation totals
  uint64_t rows_mark = 0, arena_mark = 0;  // rows / arena bytes live after the last compaction (maintain)
  // inbox CORRELATE resolution by activity instance key (zb_inbox_submit)
  int64_t *x_keys = nullptr, *x_pos = nullptr, *x_keys2 = nullptr, *x_pos2 = nullptr;
  uint32_t* d_unresolved = nullptr;  // delivered CORRELATEs whose token named no live row of their key (running count)
  // a class batch's injection, left to the classification kernel (run_trajectory), or to zb_step if that never ran
  bool inject_deferred = false;
  InjectParams inject_ip{};
  bool traj_stats_fresh = false;  // the last trajectory run's read-back holds the counters (h_stats_pinned + 8)
  // the outbox's counting sort: per bucket (commands << 40 | variable granules), their exclusive scan
  unsigned long long *cs_cnt = nullptr, *cs_off = nullptr;
  void* cs_tmp = nullptr;
  uint64_t cs_cap = 0, cs_tmp_cap = 0;
  bool ob_plan_cs = false;  // the plan is a local batch from the counting sort (outbox_emit: k_local_pack)
  uint32_t unresolved_seen = 0;
  uint64_t x_cap = 0;
  DevVec<int64_t> d_lookup_keys, d_lookup_pos;    // zb_submit lookups of the staged batch: key, staged index
  uint64_t staged_nlook = 0;
  uint64_t staged_lookup_spread = 0;  // OR of key ^ first key over the staged lookups (upload_staged)
  int64_t *look_keys = nullptr, *look_idx = nullptr;  // sorted on the device by zb_step
  uint64_t look_cap = 0;
  // radix sorts of (key, value) pairs (sort_pairs): scratch and the spread of the keys
  uint8_t* sort_tmp = nullptr;
  uint64_t sort_tmp_cap = 0;
  uint64_t* d_spread = nullptr;
  // drain buffers (zb_serialize), grown on demand and reused
  uint64_t dr_cap = 0, dr_val_cap = 0, dr_tmp_cap = 0;
  uint32_t* dr_len = nullptr;  // value lengths
  uint64_t *dr_off = nullptr, *dr_tiles = nullptr, *dr_pay = nullptr, *dr_tsum = nullptr;  // tile offsets / states / ...
  uint8_t* h_stage = nullptr;    // pinned staging of host-built uploads (zb_submit_publishes)
  size_t h_stage_cap = 0;
  uint32_t* dr_list = nullptr;   // tiles the first fast pass leaves to the wide one
  uint32_t* dr_list2 = nullptr;  // tiles for k_ser_write (left by either fast pass)
  uint32_t dr_wide_tiles = 0;    // tiles the last drain's wide fast pass encoded
  uint32_t dr_slow_tiles = 0;    // how many tiles the last drain ran through k_ser_write
  bool dr_split = false;         // the last drain ran k_ser_fast + k_ser_write (events 2-4, 5-3)
  int ser_fast = 1;              // 0 (ZB_CFG_GENERIC_DRAIN): every tile through k_ser_write
  bool wave_events = false;      // ZB_CFG_WAVE_EVENTS: timing events around every wave's kernels
  int tmpl_io = 0;               // ZB_CFG_INSTANCE_ORDER: class batches emitted in instance order (k_tmpl_io)
  zb_record_header* dr_hdr = nullptr;
  uint8_t* dr_val = nullptr;
  bool dr_frames = false;       // the drain batch holds log frames (no headers)
  void* dr_tmp = nullptr;
  uint64_t* dr_total = nullptr;   // [0] value bytes, [1] payload bytes (device)
  uint64_t* h_dr_total = nullptr; // pinned mirror
  int64_t dr_count = 0;           // records of the batch in the drain buffers
  uint64_t dr_bytes = 0;
  uint64_t dr_epoch = 0;          // look-back tags of the single-pass serializer
  hipEvent_t dr_ev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};

  // deferred template batch (zb_tdrain.hip): a uniform / class batch whose descriptors k_tmpl has not written;
  // zb_serialize of exactly [seg_begin, seg_end) encodes it from the traces, anything else materializes it
  int tmpl_defer = 1;             // 0 (ZB_CFG_NO_DEFER): always write the descriptors in zb_step
  bool seg_pending = false;
  int64_t seg_begin = 0, seg_end = 0;
  uint32_t seg_wmax = 0, seg_nc = 1;
  int64_t seg_key_end = 0;  // every key and position the deferred batch's records carry is below this
  bool seg_jobs = false;    // the deferred batch created job keys
  TrajParams seg_p{};
  uint64_t* td_wbytes = nullptr;  // [wmax * nwave + 1] (u64: hipcub's scan accumulates in the input type)
  uint64_t* td_woffs = nullptr;
  uint64_t td_cap = 0;
  void* td_tmp = nullptr;
  size_t td_tmp_cap = 0;
  uint64_t* td_pay = nullptr;     // [nwg]
  uint64_t td_pay_cap = 0;
  uint32_t* td_flags = nullptr;   // [2]

  // timing
  std::vector<hipEvent_t> ev;
  // pinned upload ring (upload_async)
  uint8_t* h_up = nullptr;
  uint64_t h_up_cap = 0, h_up_off = 0;
};

namespace {

// Host -> device copy of n bytes through the engine's pinned upload ring. A copy from pageable memory makes the
// host wait until the GPU has run it (a staged, synchronous round trip: ~20-40 us each, a dozen per C5 step); from
// the ring it is only stream-ordered. The ring wraps after a stream synchronisation (every earlier copy out of it
// has run by then); a copy larger than the ring goes the pageable way.
hipError_t upload_async(zb_engine* e, void* dst, const void* src, size_t n) {
  if (n == 0) return hipSuccess;
  if (!e->h_up || n > e->h_up_cap) return hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, e->stream);
  if (e->h_up_off + n > e->h_up_cap) {
    const hipError_t r = hipStreamSynchronize(e->stream);
    if (r != hipSuccess) return r;
    e->h_up_off = 0;
  }
  uint8_t* at = e->h_up + e->h_up_off;
  std::memcpy(at, src, n);
  e->h_up_off = (e->h_up_off + n + 63) & ~63ull;
  return hipMemcpyAsync(dst, at, n, hipMemcpyHostToDevice, e->stream);
}
template <class T>
hipError_t upload_vec(zb_engine* e, DevVec<T>& d, const std::vector<T>& v) {
  if (v.size() > d.n || !d.p) {
    d.free();
    const size_t cap = v.empty() ? 1 : v.size();
    const hipError_t r = hipMalloc(&d.p, cap * sizeof(T));
    if (r != hipSuccess) return r;
    d.n = cap;
  }
  return upload_async(e, d.p, v.data(), v.size() * sizeof(T));
}

// stream-ordered read-back of a few device words into pinned host memory with one launch (k_status) instead of one
// copy per item; valid on the host after the stream's next synchronisation
struct StatusReads {
  StatusCopy c{};
  void add(void* host, const void* dev, size_t bytes) {
    if (c.count >= StatusCopy::MAX) std::abort();  // (a programming error: the call sites are fixed)
    c.src[c.count] = (const uint32_t*)dev;
    c.dst[c.count] = (uint32_t*)host;
    c.words[c.count] = (uint32_t)(bytes / 4);
    c.count++;
  }
  hipError_t launch(hipStream_t s) const {
    launch_status(c, s);
    return hipGetLastError();
  }
};

// The exact-tree workspaces (zb_xmerge.hpp) of one device, shared by every engine on it: slabs and lane groups are held
// under device-wide locks (zb_xlock.hpp), so the partitions of one GPU need one set, not 4 GiB each. Taken by the first
// engine whose model merges or maps, freed with the last. Lanes that cannot be allocated leave the engines on the big-slab
// path (XTree with lanes == nullptr) instead of failing the deploy.
struct XPool {
  uint8_t* slab = nullptr;
  uint32_t* locks = nullptr;
  uint8_t* lane = nullptr;
  int refs = 0;
};
std::mutex g_xpool_mu;
std::map<int, XPool> g_xpool;

int fail(zb_engine* e, int code, const std::string& msg);

int xpool_acquire(zb_engine* e) {
  if (e->xpool_held) return ZB_OK;
  std::lock_guard<std::mutex> g(g_xpool_mu);
  XPool& x = g_xpool[e->cfg.device];
  if (!x.refs) {
    if (hipMalloc(&x.slab, (size_t)XSLAB_COUNT * XSLAB_BYTES) != hipSuccess ||
        hipMalloc(&x.locks, XLOCK_COUNT * sizeof(uint32_t)) != hipSuccess ||
        hipMemset(x.locks, 0, XLOCK_COUNT * sizeof(uint32_t)) != hipSuccess) {
      if (x.slab) (void)hipFree(x.slab);
      if (x.locks) (void)hipFree(x.locks);
      x = XPool{};
      return fail(e, ZB_ENOMEM, "exact payload tree slabs");
    }
    if (hipMalloc(&x.lane, (size_t)XLANE_COUNT * XLANE_BYTES) != hipSuccess) {
      (void)hipGetLastError();
      x.lane = nullptr;  // (the slab path)
    }
  }
  x.refs++;
  e->xslab = x.slab;
  e->xlocks = x.locks;
  e->xlane = x.lane;
  e->xpool_held = true;
  return ZB_OK;
}

void xpool_release(zb_engine* e) {
  if (!e->xpool_held) return;
  std::lock_guard<std::mutex> g(g_xpool_mu);
  XPool& x = g_xpool[e->cfg.device];
  if (--x.refs == 0) {
    (void)hipDeviceSynchronize();  // (another engine's stream may still run a merge on it: none left now)
    if (x.slab) (void)hipFree(x.slab);
    if (x.locks) (void)hipFree(x.locks);
    if (x.lane) (void)hipFree(x.lane);
    x = XPool{};
  }
  e->xslab = nullptr;
  e->xlocks = nullptr;
  e->xlane = nullptr;
  e->xpool_held = false;
}

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
  {  // string constants as two little-endian words (k_cls_classify compares strings of <= 16 bytes as words)
    std::vector<uint64_t> w(2 * std::max<size_t>(e->model.consts.size(), 1), 0);
    for (size_t i = 0; i < e->model.consts.size(); i++) {
      const DevConst& c = e->model.consts[i];
      if (c.type != TT_STRING || c.str_len > 16) continue;
      for (uint32_t b = 0; b < c.str_len; b++)
        w[2 * i + b / 8] |= (uint64_t)e->model.pool[c.str_off + b] << (8 * (b % 8));
    }
    HIPCHECK(e, e->d_const_w.upload(w, e->stream));
  }
  HIPCHECK(e, e->d_queries.upload(e->model.queries, e->stream));
  HIPCHECK(e, e->d_filters.upload(e->model.filters, e->stream));
  HIPCHECK(e, e->d_pool.upload(e->model.pool, e->stream));
  HIPCHECK(e, e->d_maps.upload(e->model.maps, e->stream));
  {  // constant parts of the values an element's records carry (zb_serialize.hip encode_value)
    std::vector<ValueConst> vc(e->model.elems.size());
    for (size_t i = 0; i < vc.size(); i++) {
      const DevElem& el = e->model.elems[i];
      const DevWorkflow& wf = e->model.workflows[el.wf];
      const uint32_t pid = mp_str_len(wf.pid_len), id = mp_str_len(el.id_len);
      vc[i].wf = 1 + 14 + pid + 8 + mp_int_len(wf.version) + 12 + mp_int_len(wf.key) + 20 + 11 + id + 8 + 17;
      vc[i].job = 1 + 9 + 9 + 7 + 1 + 8 + mp_int_len(el.retries) + 5 + mp_str_len(el.type_len) + 8 + 1 + 14 + pid +
                  26 + mp_int_len(wf.version) + 12 + mp_int_len(wf.key) + 20 + 11 + id + 20 + 14 +
                  (el.headers_off == NO_REF ? 1 : el.headers_len) + 8;
    }
    HIPCHECK(e, e->d_vconst.upload(vc, e->stream));
    // the fast drain passes' constant runs (zb_fastenc.hpp); the table padded to whole 16-byte LDS copies
    std::vector<DevValSeg> tab;
    std::vector<uint8_t> segs;
    e->seg_ok = build_value_segments(e->model.elems.data(), e->model.elems.size(), e->model.workflows.data(),
                                     e->model.workflows.size(), e->model.pool.data(), tab, segs);
    tab.resize((tab.size() + 3) & ~(size_t)3, DevValSeg{});
    e->seg_ok = e->seg_ok && tab.size() * sizeof(DevValSeg) + segs.size() <= SEG_LDS_MAX;
    e->segpool_len = (uint32_t)segs.size();
    HIPCHECK(e, e->d_vsegs.upload(tab, e->stream));
    HIPCHECK(e, e->d_segpool.upload(segs, e->stream));
  }
  HIPCHECK(e, e->d_segs.upload(e->model.segs, e->stream));
  if (e->static_blobs.size() > STATIC_ARENA_BYTES) return fail(e, ZB_ENOMEM, "static payload region full");
  HIPCHECK(e, hipMemcpyAsync(e->arena, e->static_blobs.data(), e->static_blobs.size(), hipMemcpyHostToDevice,
                             e->stream));
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  return ZB_OK;
}

// one outbox of the partition (kind ZB_XCHG_OPEN / _CORRELATE)
Outbox outbox(zb_engine* e, int kind) {
  Outbox o{};
  const int k = kind - 1;
  o.rec = e->obox[k];
  o.keys = e->okeys[k];
  o.n = e->on ? e->on + k : nullptr;
  o.cap = e->ocap;
  o.var = e->ovar[k];
  o.var_n = e->on ? e->on + 2 + k : nullptr;
  o.var_cap = e->ovar_cap;
  o.pos_base = e->ob_pos_base[k];
  return o;
}

WaveParams wave_params(zb_engine* e) {
  WaveParams p;
  p.log = e->log;
  p.links = e->links;
  p.srcd = e->srcd;
  p.vlen = e->vlen;
  p.rmeta = e->rmeta;
  p.rkeys = e->rkeys;
  p.rlink = e->rlink;
  p.arena = e->arena;
  p.elems = e->d_elems.p;
  p.wfs = e->d_wfs.p;
  p.cond_flows = e->d_cond.p;
  p.code = e->d_code.p;
  p.consts = e->d_consts.p;
  p.queries = e->d_queries.p;
  p.filters = e->d_filters.p;
  p.pool = e->d_pool.p;
  p.vconst = e->d_vconst.p;
  p.maps = e->d_maps.p;
  p.segs = e->d_segs.p;
  p.mapres = e->mapres;
  p.map_ws = e->map_ws;
  p.hdr = e->hdr;
  p.cw = e->cw;
  p.stage = e->stage;
  p.info = e->info;
  p.block_agg = e->block_agg;
  p.block_off = e->block_off;
  p.lookback = e->lookback;
  p.lb_tiles = e->lb_tiles;
  p.wave_cap = e->wave_cap;
  p.err = e->derr;
  p.err_info = e->derr_info;
  p.merge_jobs = e->merge_jobs;
  p.merge_count = e->job_counts;
  p.merge_slow = e->merge_slow;
  p.merge_slow_count = e->job_counts + 6;
  p.xslab = e->xslab;
  p.xlocks = e->xlocks;
  p.xlane = e->xlane;
  p.phase = e->phase;
  p.cond_jobs = e->cond_jobs;
  p.cond_count = e->job_counts + 2;
  p.sub_jobs = e->sub_jobs;
  p.sub_count = e->job_counts + 8;  // [2][SUB_STRIPES]
  p.job_cap = e->job_cap;
  p.stats = e->dstats;
  p.log_cap = (uint64_t)e->win_base + e->cfg.log_capacity;  // absolute: the window's end
  p.row_cap = e->cfg.row_capacity;
  p.arena_cap = e->arena_top;  // (the allocators' ceiling: staged documents above it)
  p.wave = e->wave;
  p.obx = outbox(e, ZB_XCHG_OPEN);
  p.partition_id = e->cfg.partition_id;
  p.partition_count = e->cfg.partition_count;
  p.raux = e->raux;
  p.has_parallel = e->has_parallel ? 1 : 0;
  p.harness = (e->cfg.flags & (ZB_CFG_EXTERNAL_JOBS | ZB_CFG_JOB_PROCESSOR)) ? 0 : 1;
  p.jobproc = (e->cfg.flags & ZB_CFG_JOB_PROCESSOR) ? 1 : 0;
  p.jobs = e->jobs;
  p.term = e->term ? 1 : 0;
  p.epoch = e->epoch;
  p.conflicts = e->conf_active ? 1 : 0;
  p.conf_keys = e->d_conf_keys.p;
  p.conf_first = e->conf_first;
  p.conf_split = e->conf_first ? e->conf_first + e->conf_cap : nullptr;
  p.conf_mask = e->conf_mask;
  // about four 256-record tiles per workgroup for the generation last seen by the host, 256..1024 workgroups
  // (C2 wave-only, 1M records per wave: 1024 workgroups 32.5 ms/step, 2048 33.0, 512 34.3, one tile per
  // workgroup 44.6 -- per-workgroup fixed costs; profiles/r02/grid_sweep.txt); a generation that grows inside
  // the batch is still covered, with more tiles per workgroup
  {
    const int64_t gen = std::max<int64_t>(e->host_hdr.gen_end - e->host_hdr.begin, e->host_hdr.end - e->host_hdr.begin);
    const int64_t chunk = std::min<int64_t>(gen, (int64_t)e->wave_cap);
    const int64_t g = ((chunk + WAVE_TILE - 1) / WAVE_TILE + 3) / 4;
    p.grid = (int32_t)std::max<int64_t>(256, std::min<int64_t>(g, 1024));
  }
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
  if (flags & DE_TIMEOUT) m += " hand-off-timeout";
  if (flags & DE_CORRUPT) m += " corrupt-arena-reference";
  uint64_t info = ~0ull;
  if (hipMemcpy(&info, e->derr_info, sizeof(info), hipMemcpyDeviceToHost) == hipSuccess && info != ~0ull)
    m += " (first at log position " + std::to_string(info >> 8) + ", site " + std::to_string(info & 0xff) + ")";
  int code = ZB_EPROCESSING;
  if (flags & (DE_LOG_FULL | DE_ROWS_FULL | DE_ARENA_FULL)) code = ZB_ENOMEM;
  else if (flags & DE_UNSUPPORTED) code = ZB_EUNSUPPORTED;
  if (flags & (DE_TIMEOUT | DE_CORRUPT)) code = ZB_EDEVICE;
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
  void* ps[] = {e->c_ikey, e->c_clen, e->c_khist, e->c_mask, e->c_woffw, e->c_wgcnt, e->c_wgoff, e->c_perm, e->c_segs,
                e->c_wcls, e->c_cg};
  for (void* q : ps)
    if (q) (void)hipFree(q);
  e->c_ikey = nullptr; e->c_clen = nullptr; e->c_khist = e->c_krep = nullptr; e->c_klen = nullptr; e->c_mask = nullptr;
  e->c_woffw = e->c_wgcnt = e->c_wgoff = e->c_perm = e->c_segs = e->c_wcls = nullptr;
  e->c_cg = nullptr;
  e->cls_cap = 0;
  const uint64_t groups = nwg * (TRAJ_WG / 64);
  // per-instance arrays hold cls_cap = nwg * TRAJ_WG entries: a later batch of up to that many instances reuses them
  const uint64_t cap = nwg * TRAJ_WG;
  HIPCHECK(e, hipMalloc(&e->c_ikey, cap));
  HIPCHECK(e, hipMalloc(&e->c_clen, cap * sizeof(uint32_t)));
  HIPCHECK(e, hipMalloc(&e->c_khist, CLS_HB * 256 * (2 * sizeof(uint32_t) + sizeof(uint64_t))));
  e->c_krep = e->c_khist + CLS_HB * 256;
  e->c_klen = (uint64_t*)(e->c_khist + 2 * CLS_HB * 256);
  HIPCHECK(e, hipMemsetAsync(e->c_khist, 0, CLS_HB * 256 * sizeof(uint32_t), e->stream));
  HIPCHECK(e, hipMemsetAsync(e->c_klen, 0, CLS_HB * 256 * sizeof(uint64_t), e->stream));
  HIPCHECK(e, hipMemsetAsync(e->c_krep, 0xff, CLS_HB * 256 * sizeof(uint32_t), e->stream));
  HIPCHECK(e, hipMalloc(&e->c_mask, groups * CLS_MAX * sizeof(uint64_t)));
  HIPCHECK(e, hipMalloc(&e->c_cg, groups * CLS_MAX * 2 * sizeof(uint32_t)));
  HIPCHECK(e, hipMalloc(&e->c_woffw, groups * CLS_MAX * sizeof(uint32_t)));
  HIPCHECK(e, hipMalloc(&e->c_wgcnt, nwg * CLS_MAX * sizeof(uint32_t)));
  HIPCHECK(e, hipMalloc(&e->c_wgoff, nwg * CLS_MAX * sizeof(uint32_t)));
  const uint64_t nblk = (nwg + CLS_BLK_WG - 1) / CLS_BLK_WG;
  const uint64_t slots = cls_slot_bound(cap, nwg);  // (for any batch of up to cap instances)
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
  p.vconst = e->d_vconst.p;
  p.srcd = e->srcd;
  p.vlen = e->vlen;
  p.arena = e->arena;
  p.rmeta = e->rmeta;
  p.rkeys = e->rkeys;
  p.rlink = e->rlink;
  p.elems = e->d_elems.p;
  p.cond_flows = e->d_cond.p;
  p.code = e->d_code.p;
  p.cls_code = e->d_cls_code.p;
  p.consts = e->d_consts.p;
  p.queries = e->d_queries.p;
  p.filters = e->d_filters.p;
  p.pool = e->d_pool.p;
  p.log_base = log_base;
  p.n = n;
  // (the batch k_inject just wrote: its CREATE payload refs as a compact array)
  p.cref = (e->d_cref && e->cref_base == log_base && (uint64_t)n <= e->cref_cap) ? e->d_cref : nullptr;
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
    // instance-order emit (k_tmpl_io) over the instance workgroups; otherwise class-uniform emit, every
    // (block, class) segment padded to whole waves, a multiple of 8 workgroups (XCD mapping)
    // (a batch the drain may take from its traces skips the class-uniform slot layout: if it is emitted after all,
    // now or when materialized, the emit runs in instance order)
    const bool may_defer = e->tmpl_defer && e->seg_ok && e->d_vsegs.p && e->d_vconst.p;
    p.io = e->tmpl_io || may_defer;
    if (!p.io) p.nwg_e = (int32_t)(((cls_slot_bound((uint64_t)n, nwg) + TRAJ_WG - 1) / TRAJ_WG + 7) & ~7ull);
    p.nblk = (int32_t)((nwg + CLS_BLK_WG - 1) / CLS_BLK_WG);
    p.segs = e->c_segs;
    p.wcls = e->c_wcls;
    if (!p.io) HIPCHECK(e, hipMemsetAsync(e->c_perm, 0xff, cls_slot_bound((uint64_t)n, nwg) * sizeof(uint32_t), e->stream));
    p.nsplits = e->nsplits;
    p.cls_nq = e->cls_nq;
    p.cls_natoms = e->cls_natoms;
    p.cls_atom_w = e->d_cls_atom.p;
    p.cls_table = e->d_cls_table.p;
    for (int j = 0; j < CLS_QMAX; j++) {
      p.cls_q[j] = e->cls_q[j];
      p.cls_key_off[j] = e->cls_key_off[j];
      p.cls_key_len[j] = e->cls_key_len[j];
      p.cls_key_w[j][0] = e->cls_key_w[j][0];
      p.cls_key_w[j][1] = e->cls_key_w[j][1];
    }
    p.const_w = e->d_const_w.p;
    for (int k = 0; k < CLS_MAX_SPLITS; k++) {
      p.split_elem[k] = e->split_elem[k];
      p.split_stride[k] = e->split_stride[k];
    }
    p.plan = e->c_plan;
    p.ikey = e->c_ikey;
    p.clen = e->c_clen;
    p.khist = e->c_khist;
    p.klen = e->c_klen;
    p.krep = e->c_krep;
    p.cmask = e->c_mask;
    p.cg = e->c_cg;
    p.woffw = e->c_woffw;
    p.wgcnt = e->c_wgcnt;
    p.wgoff = e->c_wgoff;
    p.perm = e->c_perm;
    // (the key banks are empty here: allocated so, and k_cls_plan empties them after every classification)
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
  p.log_cap = (uint64_t)e->win_base + e->cfg.log_capacity;  // absolute: the window's end
  p.xslab = e->xslab;
  p.xlocks = e->xlocks;
  p.xlane = e->xlane;
  if (e->has_merges && e->xslab) {  // (a model that merges: refused pairs go to k_tmpl_xtree)
    if ((uint64_t)n > e->t_xq_cap) {
      if (e->t_xq) (void)hipFree(e->t_xq);
      e->t_xq = nullptr;
      e->t_xq_cap = 0;
      HIPCHECK(e, hipMalloc(&e->t_xq, (uint64_t)n * sizeof(uint64_t)));
      e->t_xq_cap = (uint64_t)n;
    }
    p.xq = e->t_xq;
  }
  p.row_cap = e->cfg.row_capacity;
  p.arena_cap = e->arena_top;  // (the allocators' ceiling: staged documents above it)
  p.defer_ok = (e->tmpl_defer && e->seg_ok && e->d_vsegs.p && e->d_vconst.p && (p.cls || p.uni)) ? 1 : 0;
  hipEvent_t* ev = e->ev.data();
  HIPCHECK(e, hipEventRecord(ev[0], e->stream));
  if (p.cls) {
    const bool inj = e->inject_deferred && e->inject_ip.log_base == log_base && e->inject_ip.n == n;
    launch_traj_count_classes(p, inj ? &e->inject_ip : nullptr, e->stream);
    if (inj) e->inject_deferred = false;
  }
  else if (p.uni) launch_traj_count_uniform(p, e->stream);
  else launch_traj_count(p, e->stream);
  HIPCHECK(e, hipEventRecord(ev[1], e->stream));
  launch_traj_scan(p, e->stream);
  launch_traj_emit(p, e->stream, &ev[3]);
  HIPCHECK(e, hipEventRecord(ev[2], e->stream));
  HIPCHECK(e, hipGetLastError());
  {
    StatusReads r;
    r.add(e->h_ctl_pinned, e->t_ctl, sizeof(TrajCtl));
    r.add(e->h_hdr_pinned, e->hdr + (e->wave & 1), sizeof(WaveHdr));
    r.add(e->h_err_pinned, e->derr, sizeof(uint32_t));
    if (p.cls) r.add(e->h_stats_pinned + 16, e->c_plan, sizeof(uint32_t));
    // (and the counters: a step the trajectory run makes quiescent needs no round trip of its own for them, zb_step)
    r.add(e->h_stats_pinned + 8, e->dstats, 8 * sizeof(uint64_t));
    if (e->on) r.add(e->h_stats_pinned + 19, e->on, 4 * sizeof(uint32_t));
    HIPCHECK(e, r.launch(e->stream));
  }
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  e->traj_stats_fresh = true;
  if (e->on) e->ob_counts_valid = true;
  float ms0 = 0, ms1 = 0, ms_main = 0;
  HIPCHECK(e, hipEventElapsedTime(&ms0, ev[0], ev[1]));
  HIPCHECK(e, hipEventElapsedTime(&ms1, ev[1], ev[2]));
  HIPCHECK(e, hipEventElapsedTime(&ms_main, ev[3], ev[4]));
  st.main_emit_kernel_ms += ms_main;
  st.process_kernel_ms += ms0;
  st.emit_kernel_ms += ms1;
  st.wave_kernel_ms += ms0 + ms1;
  st.launches += p.cls ? 11 : p.uni ? 6 : 7;
#ifdef ZB_CHECKED
  if (p.cls && getenv("ZB_DEBUG_CLS")) {  // class batch internals (debugging aid of the guard-band build)
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
#endif
  if (e->h_ctl_pinned->flag) {
    // nothing but scratch counts was written: run the batch per instance (or on the wave pipeline)
    if ((p.cls || p.uni) && e->traj_model_ok) return run_trajectory(e, log_base, n, st, false);
    return 0;
  }
  e->host_hdr = e->h_hdr_pinned[0];
  int rc = check_device_errors(e, *e->h_err_pinned);
  if (rc != ZB_OK) return rc;
  st.path = p.cls ? 2 : 1;
  if (e->h_ctl_pinned->defer) {  // descriptors not written: zb_serialize encodes the batch from its traces
    e->seg_pending = true;
    e->seg_begin = log_base + n;
    e->seg_end = e->host_hdr.end;
    e->seg_wmax = e->h_ctl_pinned->wmax;
    e->seg_key_end = std::max(std::max(e->host_hdr.wf_next, e->host_hdr.job_next), e->host_hdr.end);
    e->seg_jobs = e->host_hdr.job_next != p.job_start;
    e->seg_p = p;
    e->seg_nc = 1;
    if (p.cls) e->seg_nc = (uint32_t)e->h_stats_pinned[16];  // ClsPlan.nc (copied with the trajectory's results)
  }
  return 1;
}

// outboxes: one record per element-instance row at most (a subscription per catch event instance;
// a correlation per subscription and publish)
int ensure_outbox(zb_engine* e) {
  if (e->on) return ZB_OK;
  e->ocap = std::max<uint64_t>(e->cfg.row_capacity, 1024);
  // byte sections: 192 bytes per command on average (name + correlation key or payload), at least 64 MiB
  e->ovar_cap = std::max<uint64_t>(e->ocap * 24, 8ull << 20);
  for (int k = 0; k < 2; k++) {
    HIPCHECK(e, hipMalloc(&e->obox[k], e->ocap * sizeof(zb_exchange_rec)));
    HIPCHECK(e, hipMalloc(&e->okeys[k], e->ocap * sizeof(uint64_t)));
    HIPCHECK(e, hipMalloc(&e->ovar[k], e->ovar_cap * 8));
  }
  HIPCHECK(e, hipMalloc(&e->on, 4 * sizeof(uint32_t)));
  HIPCHECK(e, hipMemsetAsync(e->on, 0, 4 * sizeof(uint32_t), e->stream));
  e->ob_counts_valid = false;
  if (!e->sub_jobs) HIPCHECK(e, hipMalloc(&e->sub_jobs, e->job_cap * sizeof(uint64_t)));
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


// the partition must be idle for a message-side batch (canonical schedule, zeebe_amd/cluster.py)
// Radix sort of (key, value) pairs by 64-bit keys, stable, into kout / vout. Only the key bits that differ
// between the keys are sorted (k_key_spread; the others are equal in every key): the outbox keys (target, source
// position, emission) and the instance keys of a tick span ~25 of their 64 bits, so Onesweep makes 4 passes
// instead of 8. Always Onesweep: rocprim's default takes its merge sort below 2^20 pairs, which made 21 launches
// and ~190 us of a 1M-pair outbox on MI355X (C5 kernel trace, round 4). Signed keys: the sign flip of the radix
// order is the same in every key, so the differing bits are those of the raw keys.
using OnesweepSort = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                                rocprim::default_config, 0>;
// spread_known: the spread is already in h_stats_pinned[17] (the caller launched k_key_spread and read it back with
// a round trip of its own)
template <class K, class V>
int sort_pairs(zb_engine* e, const K* kin, K* kout, const V* vin, V* vout, uint64_t n, const char* what,
               bool spread_known = false) {
  static_assert(sizeof(K) == 8, "64-bit keys");
  if (n == 0) return ZB_OK;
  if (n > (uint64_t)INT32_MAX) return fail(e, ZB_EUNSUPPORTED, std::string(what) + ": more than 2^31 keys");
  if (!spread_known) {
    HIPCHECK(e, hipMemsetAsync(e->d_spread, 0, sizeof(uint64_t), e->stream));
    launch_key_spread((const uint64_t*)kin, n, e->d_spread, e->stream);
    HIPCHECK(e, hipMemcpyAsync(e->h_stats_pinned + 17, e->d_spread, sizeof(uint64_t), hipMemcpyDeviceToHost,
                               e->stream));
    HIPCHECK(e, hipStreamSynchronize(e->stream));
  }
  const uint64_t spread = e->h_stats_pinned[17];
  if (spread == 0) {  // one key (or all equal): the input order
    HIPCHECK(e, hipMemcpyAsync(kout, kin, n * sizeof(K), hipMemcpyDeviceToDevice, e->stream));
    HIPCHECK(e, hipMemcpyAsync(vout, vin, n * sizeof(V), hipMemcpyDeviceToDevice, e->stream));
    return ZB_OK;
  }
  const unsigned begin = (unsigned)__builtin_ctzll(spread), end = 64u - (unsigned)__builtin_clzll(spread);
  size_t need = 0;
  if (rocprim::radix_sort_pairs<OnesweepSort>(nullptr, need, kin, kout, vin, vout, (size_t)n, begin, end,
                                              e->stream) != hipSuccess)
    return fail(e, ZB_EDEVICE, std::string(what) + ": sort sizing");
  if (need + 16 > e->sort_tmp_cap) {
    HIPCHECK(e, hipStreamSynchronize(e->stream));
    if (e->sort_tmp) (void)hipFree(e->sort_tmp);
    e->sort_tmp = nullptr;
    e->sort_tmp_cap = 0;
    const uint64_t c = std::max<uint64_t>(need + need / 2 + 16, 1 << 20);
    HIPCHECK(e, hipMalloc(&e->sort_tmp, c));
    e->sort_tmp_cap = c;
  }
  size_t have = e->sort_tmp_cap;
  if (rocprim::radix_sort_pairs<OnesweepSort>(e->sort_tmp, have, kin, kout, vin, vout, (size_t)n, begin, end,
                                              e->stream) != hipSuccess)
    return fail(e, ZB_EDEVICE, std::string(what) + ": sort");
  return ZB_OK;
}

int require_idle(zb_engine* e) {
  if (e->failed) return fail(e, ZB_EPROCESSING, "partition stopped after a processing failure: " + e->err);
  if (e->host_hdr.begin != e->host_hdr.end || (e->staged_pending && !e->staged.empty()))
    return fail(e, ZB_EINVAL, "partition not quiescent: step it before delivering or publishing");
  return ZB_OK;
}

int finish_batch(zb_engine* e) {
  HIPCHECK(e, upload_async(e, e->hdr + (e->wave & 1), &e->host_hdr, sizeof(WaveHdr)));
  HIPCHECK(e, hipGetLastError());
  {
    StatusReads r;
    r.add(e->h_err_pinned, e->derr, sizeof(uint32_t));
    // (a message batch's correlations are in the outbox: the exchange decision reads the counters from here)
    if (e->on) r.add(e->h_stats_pinned + 19, e->on, 4 * sizeof(uint32_t));
    HIPCHECK(e, r.launch(e->stream));
  }
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  e->ob_counts_valid = e->on != nullptr;
  return check_device_errors(e, *e->h_err_pinned);
}

// ---- the long-running partition: log window, compaction of rows / arena / stores / job states

// biased views of the log arrays: element [pos] of the view is array index pos - win_base
template <class T>
T* biased(T* mem, int64_t base) {
  return (T*)((uintptr_t)mem - (uintptr_t)base * sizeof(T));
}
void rebias(zb_engine* e) {
  e->log = biased(e->log_mem, e->win_base);
  e->links = biased(e->links_mem, e->win_base);
  e->srcd = biased(e->srcd_mem, e->win_base);
  e->vlen = biased(e->vlen_mem, e->win_base);
}

// Records the caller released move out of the window: [released, end) go to the front of the arrays (the
// partition is quiescent: nothing below end is unprocessed). Chunks of at most (released - win_base) records,
// front to back, never overlap a source not yet copied.
// request metadata of released records: the runs wholly below the window go (a run the window cuts stays whole: its
// entries below the window are never looked up); an empty table starts again at entry 0
void drop_requests(zb_engine* e) {
  size_t k = 0;
  while (k < e->req_runs.size() && e->req_runs[k].last < e->win_base) k++;
  e->req_runs.erase(e->req_runs.begin(), e->req_runs.begin() + k);
  if (e->req_runs.empty()) e->req_lo = e->req_n = 0;
  else e->req_lo = e->req_runs.front().lo;
}

// the staged batch's request metadata appended to the device table (positions log_base + staged index)
int append_requests(zb_engine* e, int64_t log_base) {
  const uint64_t m = e->staged_reqs.size();
  if (!m) return ZB_OK;
  if (!e->staged_reqs_uploaded) {
    HIPCHECK(e, e->d_staged_reqs.upload(e->staged_reqs, e->stream));
    e->staged_reqs_uploaded = true;
  }
  if (e->req_n + m > e->req_cap) {  // grow, keeping only the live entries
    const uint64_t live = e->req_n - e->req_lo;
    const uint64_t cap = std::max<uint64_t>(2 * (live + m), 1024);
    ReqMeta* p = nullptr;
    HIPCHECK(e, hipMalloc(&p, cap * sizeof(ReqMeta)));
    if (live) HIPCHECK(e, hipMemcpyAsync(p, e->d_req + e->req_lo, live * sizeof(ReqMeta), hipMemcpyDeviceToDevice, e->stream));
    HIPCHECK(e, hipStreamSynchronize(e->stream));
    if (e->d_req) (void)hipFree(e->d_req);
    e->d_req = p;
    e->req_cap = cap;
    for (auto& r : e->req_runs) r.lo -= e->req_lo;
    e->req_n = live;
    e->req_lo = 0;
  }
  launch_req_append(e->d_staged_reqs.p, m, log_base, e->d_req + e->req_n, e->stream);
  e->req_runs.push_back(zb_engine::ReqRun{log_base + e->staged_reqs.front().idx, log_base + e->staged_reqs.back().idx,
                                          e->req_n, m});
  e->req_n += m;
  return ZB_OK;
}

int rebase_log(zb_engine* e) {
  const int64_t from = std::min(e->released, e->host_hdr.end);
  if (from <= e->win_base) return ZB_OK;
  const int64_t keep = e->host_hdr.end - from, shift = from - e->win_base;
  for (int64_t o = 0; o < keep; o += shift) {
    const int64_t n = std::min(shift, keep - o);
    HIPCHECK(e, hipMemcpyAsync(e->log_mem + o, e->log_mem + shift + o, n * sizeof(zb_rec), hipMemcpyDeviceToDevice, e->stream));
    HIPCHECK(e, hipMemcpyAsync(e->links_mem + o, e->links_mem + shift + o, n * sizeof(uint64_t), hipMemcpyDeviceToDevice, e->stream));
    HIPCHECK(e, hipMemcpyAsync(e->srcd_mem + o, e->srcd_mem + shift + o, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, e->stream));
    HIPCHECK(e, hipMemcpyAsync(e->vlen_mem + o, e->vlen_mem + shift + o, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, e->stream));
  }
  e->win_base = from;
  rebias(e);
  // submitted-command ranges and request metadata of released records are no longer needed by the drain
  e->ranges.erase(std::remove_if(e->ranges.begin(), e->ranges.end(),
                                 [&](const CmdRange& r) { return r.pos_end <= e->win_base; }), e->ranges.end());
  drop_requests(e);
  // the process-id strings they name: only those of the remaining (and the staged) ranges are kept
  std::vector<uint8_t> pool;
  auto keep_str = [&](uint32_t& off, uint16_t len) {
    const uint32_t at = (uint32_t)pool.size();
    pool.insert(pool.end(), e->cmd_pool.begin() + off, e->cmd_pool.begin() + off + len);
    off = at;
  };
  for (auto& r : e->ranges) keep_str(r.pid_off, r.pid_len);
  for (auto& r : e->pending_ranges) keep_str(r.pid_off, r.pid_len);
  e->cmd_pool.swap(pool);
  return ZB_OK;
}

template <class T>
int grow(zb_engine* e, T** p, uint64_t* cap, uint64_t n) {
  if (n <= *cap && *p) return ZB_OK;
  HIPCHECK(e, hipStreamSynchronize(e->stream));  // (queued work may still use the old buffer)
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  const uint64_t c = std::max<uint64_t>(n + n / 4, 1024);
  HIPCHECK(e, hipMalloc(p, c * sizeof(T)));
  *cap = c;
  return ZB_OK;
}

// exclusive scan of in[0, n] into out; returns the total (out[n], in[n] being 0)
int scan_u32(zb_engine* e, const uint32_t* in, uint32_t* out, uint64_t n, uint64_t* total) {
  if (n + 1 > (uint64_t)INT32_MAX) return fail(e, ZB_EUNSUPPORTED, "compaction over more than 2^31 entries");
  size_t tmp = 0;
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, in, out, (int)(n + 1), e->stream) != hipSuccess)
    return fail(e, ZB_EDEVICE, "compaction scan sizing");
  if (tmp > e->c_tmp_cap) {
    HIPCHECK(e, hipStreamSynchronize(e->stream));
    if (e->c_tmp) (void)hipFree(e->c_tmp);
    e->c_tmp = nullptr;
    e->c_tmp_cap = 0;
    HIPCHECK(e, hipMalloc(&e->c_tmp, tmp + tmp / 4 + 16));
    e->c_tmp_cap = tmp + tmp / 4;
  }
  tmp = e->c_tmp_cap;
  if (hipcub::DeviceScan::ExclusiveSum(e->c_tmp, tmp, in, out, (int)(n + 1), e->stream) != hipSuccess)
    return fail(e, ZB_EDEVICE, "compaction scan");
  uint32_t t = 0;
  HIPCHECK(e, hipMemcpyAsync(&t, out + n, sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  *total = t;
  return ZB_OK;
}

// the scan scratch for scans of up to n + 1 entries, reserved ahead (scan_u32 grows it otherwise)
int scan_reserve(zb_engine* e, uint64_t n) {
  if (n + 1 > (uint64_t)INT32_MAX) return ZB_OK;  // (scan_u32 refuses such a scan itself)
  size_t tmp = 0;
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)(n + 1),
                                       e->stream) != hipSuccess)
    return fail(e, ZB_EDEVICE, "compaction scan sizing");
  if (tmp <= e->c_tmp_cap && e->c_tmp) return ZB_OK;
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  if (e->c_tmp) (void)hipFree(e->c_tmp);
  e->c_tmp = nullptr;
  e->c_tmp_cap = 0;
  HIPCHECK(e, hipMalloc(&e->c_tmp, tmp + tmp / 4 + 16));
  e->c_tmp_cap = tmp + tmp / 4;
  return ZB_OK;
}

// The compaction buffers that scale with the capacities' index space, sized once when the engine is created: rows
// and messages (flags and their scan), the dynamic arena's granule words (bitmap, popcounts, their scan) and the
// scan scratch for the largest scan -- a few bytes per row and per 64 arena granules. Grown per compaction instead, a
// partition that keeps growing freed and reallocated them -- each a device-wide synchronisation -- at nearly every
// compaction (C2 steady state: 3.2 ms ticks against 1.1 ms). The gather scratch (the live rows or the live dynamic
// arena, up to the whole arena) is reserve_gather's, at the first compaction.
int reserve_compaction(zb_engine* e) {
  const uint64_t nflag = std::max<uint64_t>(e->cfg.row_capacity, 1024) + 1;  // (rows; the stores hold as many)
  const uint64_t words_cap = ((e->cfg.arena_bytes - STATIC_ARENA_BYTES) / 8 + 63) / 64 + 1;
  int rc = grow(e, &e->c_flag, &e->c_flag_cap, nflag);
  if (rc == ZB_OK) rc = grow(e, &e->c_new, &e->c_new_cap, nflag);
  if (rc == ZB_OK) rc = grow(e, &e->c_bits, &e->c_bits_cap, words_cap);
  if (rc == ZB_OK) rc = grow(e, &e->c_pop, &e->c_pop_cap, words_cap + 1);
  if (rc == ZB_OK) rc = grow(e, &e->c_off, &e->c_off_cap, words_cap + 1);
  if (rc == ZB_OK) rc = scan_reserve(e, std::max(nflag, words_cap + 1));
  return rc;
}

// The gather scratch: reserved at the partition's first compaction for its capacities (the row table, the dynamic
// arena) -- grown on demand it was reallocated, each time a device-wide synchronisation, at the first compactions of a
// growing partition (C2 steady state: 0.6-1.2 ms of a 1.6-2.0 ms compaction). An engine that never compacts holds
// none. (At creation, for every engine, it doubled a large partition's device memory.)
int reserve_gather(zb_engine* e) {
  const uint64_t row_bytes = sizeof(RowMeta) + sizeof(RowKeys) + sizeof(RowAux);
  const uint64_t full = std::max<uint64_t>(e->cfg.row_capacity * row_bytes, e->cfg.arena_bytes - STATIC_ARENA_BYTES);
  if (e->c_scratch && e->c_scratch_cap >= full) return ZB_OK;
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  if (e->c_scratch) (void)hipFree(e->c_scratch);
  e->c_scratch = nullptr;
  e->c_scratch_cap = 0;
  HIPCHECK(e, hipMalloc(&e->c_scratch, full));
  e->c_scratch_cap = full;
  return ZB_OK;
}

CompactParams compact_params(zb_engine* e) {
  CompactParams c{};
  c.rmeta = e->rmeta; c.rkeys = e->rkeys; c.rlink = e->rlink; c.raux = e->raux;
  c.rows = (uint64_t)e->host_hdr.rows_next;
  c.live_rows = c.rows;
  c.row_flag = e->c_flag; c.row_new = e->c_new;
  c.arena = e->arena;
  c.static_refs = STATIC_ARENA_BYTES / 8;
  c.arena_next = (uint64_t)e->host_hdr.arena_next;
  c.arena_top = e->arena_top;
  c.arena_end = e->cfg.arena_bytes;
  c.log = e->log;
  c.win_begin = e->win_base;
  c.win_end = e->host_hdr.end;
  c.msgs = e->msgs; c.msg_count = e->msgs ? e->msg_count : 0;
  c.subs = e->subs; c.sub_count = e->subs ? e->sub_count : 0;
  c.err = e->derr;
  return c;
}

// Compaction of a quiescent partition: dead element-instance rows, removed messages, unreachable arena
// blobs and job-table tombstones are dropped; everything live keeps its order (zb_compact.hip).
int compact_state(zb_engine* e) {
#ifdef ZB_PHASES  // (measurement build: host time per compaction phase, waits at its round trips included)
  auto ct0 = std::chrono::steady_clock::now();
  double ct[8] = {0};
  int cti = 0;
#define ZB_CT() do { auto n_ = std::chrono::steady_clock::now(); \
    ct[cti++ & 7] = std::chrono::duration<double, std::milli>(n_ - ct0).count(); ct0 = n_; } while (0)
#else
#define ZB_CT() do { } while (0)
#endif
  const uint64_t rows = (uint64_t)e->host_hdr.rows_next;
  int rc = reserve_compaction(e);  // (no-op: zb_engine_create reserved them)
  if (rc == ZB_OK) rc = reserve_gather(e);
  if (rc != ZB_OK) return rc;
  // 1. rows: live ones to the front (index order kept), parents renamed
  CompactParams c = compact_params(e);
  uint64_t live = 0;
  if (rows) {
    launch_row_flags(c, e->stream);
    rc = scan_u32(e, e->c_flag, e->c_new, rows, &live);
    if (rc != ZB_OK) return rc;
    const uint64_t row_bytes = ROW_BYTES + sizeof(RowAux);
    rc = grow(e, &e->c_scratch, &e->c_scratch_cap, std::max<uint64_t>(live, 1) * row_bytes);
    if (rc != ZB_OK) return rc;
    c.row_new = e->c_new;
    c.m2 = (RowMeta*)e->c_scratch;
    c.k2 = (RowKeys*)(e->c_scratch + live * sizeof(RowMeta));
    c.a2 = (RowAux*)(e->c_scratch + live * (sizeof(RowMeta) + sizeof(RowKeys)));
    launch_row_gather(c, e->stream);
    if (live) {
      HIPCHECK(e, hipMemcpyAsync(e->rmeta, c.m2, live * sizeof(RowMeta), hipMemcpyDeviceToDevice, e->stream));
      HIPCHECK(e, hipMemcpyAsync(e->rkeys, c.k2, live * sizeof(RowKeys), hipMemcpyDeviceToDevice, e->stream));
      HIPCHECK(e, hipMemcpyAsync(e->raux, c.a2, live * sizeof(RowAux), hipMemcpyDeviceToDevice, e->stream));
      c.live_rows = live;  // the children lists of the renamed rows, relinked
      HIPCHECK(e, hipMemsetAsync(e->rlink, 0xff, live * sizeof(RowLink), e->stream));  // (NO_ROW)
      launch_row_relink(c, e->stream);
    }
  }
  e->host_hdr.rows_next = (int64_t)live;
  ZB_CT();  // rows
  // 2. message store: removed messages dropped, chains rebuilt (subscriptions are never removed)
  if (e->msgs && e->msg_count) {
    c = compact_params(e);
    launch_msg_flags(c, e->stream);
    uint64_t live_msgs = 0;
    rc = scan_u32(e, e->c_flag, e->c_new, e->msg_count, &live_msgs);
    if (rc != ZB_OK) return rc;
    if (live_msgs != e->msg_count) {
      rc = grow(e, &e->c_scratch, &e->c_scratch_cap, std::max<uint64_t>(live_msgs, 1) * sizeof(MsgEntry));
      if (rc != ZB_OK) return rc;
      launch_msg_gather(c, (MsgEntry*)e->c_scratch, e->stream);
      if (live_msgs)
        HIPCHECK(e, hipMemcpyAsync(e->msgs, e->c_scratch, live_msgs * sizeof(MsgEntry), hipMemcpyDeviceToDevice, e->stream));
      e->msg_count = live_msgs;
      launch_chains(e->msgs, e->msg_count, e->msg_head, e->msg_next, e->subs, e->sub_count, e->sub_head, e->sub_next,
                    e->head_mask, e->stream);
    }
  }
  ZB_CT();  // messages
  // 3. arena: blobs reachable from live rows, the unreleased log window and the stores. A batch uploaded in place
  // but not injected yet (no record references it) is not part of it: it goes to the very top of the arena
  // afterwards (through the scratch when it has to move), so that the allocators get everything below it back.
  c = compact_params(e);
  c.live_rows = live;
  const bool pend = e->staged_in_place && e->staged_pending;
  const uint64_t pb = pend ? e->staged_top - e->staged_base : 0;  // its bytes
  const bool pend_moves = pend && e->staged_base != e->cfg.arena_bytes - pb;
  // (the bitmap spans the staged documents at the top too, after the allocated bytes: they move down with the rest)
  const uint64_t dyn = (uint64_t)e->host_hdr.arena_next - STATIC_ARENA_BYTES + (e->cfg.arena_bytes - e->arena_top);
  const uint64_t words = (dyn / 8 + 63) / 64;
  uint64_t granules = 0;
  if (words) {
    rc = grow(e, &e->c_bits, &e->c_bits_cap, words);
    if (rc == ZB_OK) rc = grow(e, &e->c_pop, &e->c_pop_cap, words + 1);
    if (rc == ZB_OK) rc = grow(e, &e->c_off, &e->c_off_cap, words + 1);
    if (rc != ZB_OK) return rc;
    HIPCHECK(e, hipMemsetAsync(e->c_bits, 0, words * sizeof(uint64_t), e->stream));
    c.bits = e->c_bits; c.word_pop = e->c_pop; c.word_off = e->c_off; c.words = words;
    launch_mark(c, e->stream);
    launch_word_pop(c, e->stream);
    rc = scan_u32(e, e->c_pop, e->c_off, words, &granules);
    if (rc != ZB_OK) return rc;
    ZB_CT();  // arena marking
  }
  const bool room = STATIC_ARENA_BYTES + granules * 8 + pb <= e->cfg.arena_bytes;
  rc = grow(e, &e->c_scratch, &e->c_scratch_cap, std::max<uint64_t>(granules * 8 + (pend_moves && room ? pb : 0), 8));
  if (rc != ZB_OK) return rc;
  if (pend_moves && room)  // (stashed before the live bytes are copied back over the region it may lie in)
    HIPCHECK(e, hipMemcpyAsync(e->c_scratch + granules * 8, e->arena + e->staged_base, pb, hipMemcpyDeviceToDevice,
                               e->stream));
  if (words) {
    c.scratch = e->c_scratch;
    launch_arena_gather(c, e->stream);
    launch_rename(c, e->stream);
    if (granules)
      HIPCHECK(e, hipMemcpyAsync(e->arena + STATIC_ARENA_BYTES, e->c_scratch, granules * 8, hipMemcpyDeviceToDevice, e->stream));
    e->host_hdr.arena_next = (int64_t)(STATIC_ARENA_BYTES + granules * 8);
  }
  if (pend && room) {
    if (pend_moves)
      HIPCHECK(e, hipMemcpyAsync(e->arena + e->cfg.arena_bytes - pb, e->c_scratch + granules * 8, pb,
                                 hipMemcpyDeviceToDevice, e->stream));
    e->staged_base = e->cfg.arena_bytes - pb;
    e->staged_top = e->cfg.arena_bytes;
    e->arena_top = e->staged_base;
  } else {
    e->arena_top = e->cfg.arena_bytes;
    if (e->staged_in_place) {  // (no room beside the live bytes: the step that injects it uploads it again)
      e->staged_in_place = false;
      e->staged_uploaded = false;
    }
  }
  ZB_CT();  // arena gather
  // 4. job table: tombstones dropped (live entries collected, table cleared, refilled)
  if (e->jobs.keys) {
    uint32_t tombs = 0;
    HIPCHECK(e, hipMemcpyAsync(&tombs, e->jobs.tombs, sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
    HIPCHECK(e, hipStreamSynchronize(e->stream));
    if (tombs) {
      const uint64_t slots = e->jobs.mask + 1;
      rc = grow(e, &e->c_scratch, &e->c_scratch_cap, slots * (sizeof(int64_t) + 1));
      if (rc != ZB_OK) return rc;
      if (!e->c_count) HIPCHECK(e, hipMalloc(&e->c_count, sizeof(uint32_t)));
      HIPCHECK(e, hipMemsetAsync(e->c_count, 0, sizeof(uint32_t), e->stream));
      int64_t* keys = (int64_t*)e->c_scratch;
      uint8_t* st = e->c_scratch + slots * sizeof(int64_t);
      launch_job_collect(e->jobs, keys, st, e->c_count, e->stream);
      uint32_t n = 0;
      HIPCHECK(e, hipMemcpyAsync(&n, e->c_count, sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
      HIPCHECK(e, hipStreamSynchronize(e->stream));
      launch_job_clear(e->jobs, e->stream);
      launch_job_fill(e->jobs, keys, st, n, e->derr, e->stream);
      HIPCHECK(e, hipMemsetAsync(e->jobs.tombs, 0, sizeof(uint32_t), e->stream));
    }
  }
  e->compactions++;
  e->rows_mark = (uint64_t)e->host_hdr.rows_next;  // what survived: the next trigger is relative to it
  e->arena_mark = (uint64_t)e->host_hdr.arena_next;
  ZB_CT();  // job table
  rc = finish_batch(e);  // the device wave header takes the new allocators
  ZB_CT();  // the last round trip
#ifdef ZB_PHASES
  fprintf(stderr, "compaction ms: rows %.3f msgs %.3f mark %.3f gather %.3f jobs %.3f finish %.3f\n", ct[0], ct[1], ct[2],
          ct[3], ct[4], ct[5]);
#endif
#undef ZB_CT
  return rc;
}

// A deferred template batch gets its descriptors (+ source deltas, value-length hints) written by the emit
// pass it skipped; the batch's buffers (traces, class plan, generation bases) are still those of the last
// trajectory run (every zb_step settles the deferred batch before a new run).
int materialize(zb_engine* e) {
  if (!e->seg_pending) return ZB_OK;
  e->seg_pending = false;
  TrajParams p = e->seg_p;
  p.materialize = 1;
  launch_traj_emit(p, e->stream, nullptr);
  HIPCHECK(e, hipGetLastError());
  HIPCHECK(e, hipMemcpyAsync(e->h_ctl_pinned, e->t_ctl, sizeof(TrajCtl), hipMemcpyDeviceToHost, e->stream));
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  return check_device_errors(e, e->h_ctl_pinned->derr);
}
// before anything reads the log window or reuses the trajectory buffers: a deferred batch that was released
// (appended by the caller) is dropped, any other is materialized
int settle_deferred(zb_engine* e) {
  if (!e->seg_pending) return ZB_OK;
  if (e->released >= e->seg_end) {
    e->seg_pending = false;
    return ZB_OK;
  }
  return materialize(e);
}

// Between ticks: the released part of the log leaves the window, and the state is compacted when a region has
// used half of the room the last compaction left it (or always, force) -- so a partition whose live state fits
// its capacities runs indefinitely, and a compaction that frees little is not repeated at every tick (each one
// is paid for by at least half the free room having been allocated since the last).
int maintain(zb_engine* e, bool force) {
  if (e->failed || e->host_hdr.begin != e->host_hdr.end) return ZB_OK;  // only at quiescence
  int rc = settle_deferred(e);
  if (rc != ZB_OK) return rc;
  rc = rebase_log(e);
  if (rc != ZB_OK) return rc;
  const uint64_t rm = std::min<uint64_t>(e->rows_mark, e->cfg.row_capacity);
  const uint64_t am = std::max<uint64_t>(std::min<uint64_t>(e->arena_mark, e->cfg.arena_bytes), STATIC_ARENA_BYTES);
  const uint64_t ru = (uint64_t)e->host_hdr.rows_next;
  // the arena: allocated bytes + the documents of injected batches at the top; a batch uploaded in place but not
  // injected yet is neither (compaction cannot reclaim it: it is the capacity the rest has to live beside)
  const bool pend = e->staged_in_place && e->staged_pending;
  const uint64_t pend_bytes = pend ? e->staged_top - e->staged_base : 0;
  const uint64_t au = (uint64_t)e->host_hdr.arena_next + (e->cfg.arena_bytes - (pend ? e->staged_top : e->arena_top));
  const uint64_t rc_ = e->cfg.row_capacity, ac = e->cfg.arena_bytes - pend_bytes;
  const uint64_t am_ = std::min(am, ac);
  // (and whenever less than an eighth is left: then compacting is the only way on)
  const bool rows_half = ru > rm + (rc_ - rm) / 2 || rc_ - std::min(ru, rc_) < rc_ / 8;
  const bool arena_half = au > am_ + (ac - am_) / 2 || ac - std::min(au, ac) < (ac - STATIC_ARENA_BYTES) / 8;
  bool jobs_half = false;
  if (e->jobs.keys && !force && !rows_half && !arena_half) {
    uint32_t tombs = 0;
    HIPCHECK(e, hipMemcpyAsync(&tombs, e->jobs.tombs, sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
    HIPCHECK(e, hipStreamSynchronize(e->stream));
    jobs_half = tombs > (e->jobs.mask + 1) / 4;
  }
  if (force || rows_half || arena_half || jobs_half) return compact_state(e);
  return ZB_OK;
}

}  // namespace

extern "C" {

int zb_engine_create(const zb_config* cfg, zb_engine** out) {
  if (!cfg || !out) return ZB_EINVAL;
  *out = nullptr;
  auto* e = new zb_engine();
  e->cfg = *cfg;
  const int32_t fl = e->cfg.flags;
  e->ser_mode = (fl & ZB_CFG_SINGLE_PASS_DRAIN) ? 1 : 0;
  e->ser_fast = (fl & ZB_CFG_GENERIC_DRAIN) ? 0 : 1;
  e->tmpl_io = (fl & ZB_CFG_INSTANCE_ORDER) ? 1 : 0;
  e->tmpl_defer = (fl & ZB_CFG_NO_DEFER) ? 0 : 1;
  e->wave_events = (fl & ZB_CFG_WAVE_EVENTS) != 0;
  if (e->cfg.log_capacity == 0) e->cfg.log_capacity = 1ull << 22;
  if (e->cfg.row_capacity == 0) e->cfg.row_capacity = 1ull << 20;
  if (e->cfg.arena_bytes == 0) e->cfg.arena_bytes = 64ull << 20;
  if (e->cfg.arena_bytes < 2 * STATIC_ARENA_BYTES) e->cfg.arena_bytes = 2 * STATIC_ARENA_BYTES;
  e->cfg.arena_bytes &= ~7ull;  // (whole 8-byte granules: refs are granule indexes, documents sit at its top)
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
  {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, cfg->device) == hipSuccess && ncu > 0)
      e->ncu = ncu;
  }
  {
    const int per_cu = (e->cfg.flags & ZB_CFG_WAVE_SPLIT) ? 0 : wave_resident_per_cu();
    // the occupancy limit less one workgroup per eight CUs: every workgroup of the persistent grid is resident
    // with room to spare, so no tile waits on a workgroup that is not running. (A grid of (per_cu - 1) per CU left
    // a quarter of the wave slots idle: C2 1M wave-only stepping 19.8 ms at 768 workgroups, 17.9 at 1024.)
    e->wave_fused_grid = per_cu > 1 ? per_cu * e->ncu - std::max(1, e->ncu / 8) : (per_cu == 1 ? e->ncu : 0);
  }
  const uint64_t L = e->cfg.log_capacity;
  e->wave_cap = e->cfg.wave_records ? e->cfg.wave_records : std::min<uint64_t>(L, 1ull << 22);
  e->wave_cap = (e->wave_cap + WAVE_TILE - 1) / WAVE_TILE * WAVE_TILE;
  if (hipMalloc(&e->log_mem, L * sizeof(zb_rec)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->links_mem, L * sizeof(uint64_t)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->srcd_mem, L * sizeof(uint32_t)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->vlen_mem, L * sizeof(uint32_t)) != hipSuccess) return cleanup(ZB_ENOMEM);
  rebias(e);
  if ((e->cfg.flags & ZB_CFG_VLEN_CHECK) && hipMalloc(&e->vlen_bad, sizeof(uint32_t)) != hipSuccess)
    return cleanup(ZB_ENOMEM);
  // job states: open addressing at load <= 1/2 for row_capacity live jobs
  if (e->cfg.flags & ZB_CFG_JOB_PROCESSOR) {
    uint64_t slots = 1024;
    while (slots < 2 * e->cfg.row_capacity) slots <<= 1;
    e->jobs.mask = slots - 1;
    if (hipMalloc(&e->jobs.keys, slots * sizeof(int64_t)) != hipSuccess ||
        hipMalloc(&e->jobs.state, slots) != hipSuccess || hipMalloc(&e->jobs.tombs, sizeof(uint32_t)) != hipSuccess)
      return cleanup(ZB_ENOMEM);
  }
  if (hipMalloc(&e->row_mem, e->cfg.row_capacity * ROW_BYTES) != hipSuccess) return cleanup(ZB_ENOMEM);
  e->rmeta = (RowMeta*)e->row_mem;
  e->rkeys = (RowKeys*)(e->row_mem + e->cfg.row_capacity * sizeof(RowMeta));
  e->rlink = (RowLink*)(e->row_mem + e->cfg.row_capacity * (sizeof(RowMeta) + sizeof(RowKeys)));
  // (+ ARENA_SLACK: the drain's encoders load a payload document's first words without a bounds check)
  if (hipMalloc(&e->arena, e->cfg.arena_bytes + ARENA_SLACK) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->hdr, 2 * sizeof(WaveHdr)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->cw, e->wave_cap * sizeof(uint64_t)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->stage, e->wave_cap * 2 * sizeof(Slot)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->info, e->wave_cap * sizeof(ItemInfo)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->block_agg, WAVE_GRID_MAX * sizeof(BlockAgg)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->block_off, WAVE_GRID_MAX * sizeof(BlockOff)) != hipSuccess) return cleanup(ZB_ENOMEM);
  {
    e->lb_tiles = e->wave_cap / WAVE_TILE + 1;
    // (+ 1: the two k_wave tile counters)
    const size_t lb = (2 * e->lb_tiles + 8 * (e->lb_tiles + 512) + 8 * (e->lb_tiles + 2) + 1) * sizeof(uint64_t);
    if (hipMalloc(&e->lookback, lb) != hipSuccess) return cleanup(ZB_ENOMEM);
    if (hipMemset(e->lookback, 0, lb) != hipSuccess) return cleanup(ZB_EDEVICE);
  }
  if (hipMalloc(&e->derr, sizeof(uint32_t)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->dstats, STAT_WORDS * sizeof(uint64_t)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->derr_info, sizeof(uint64_t)) != hipSuccess) return cleanup(ZB_ENOMEM);
  e->job_cap = std::min<uint64_t>(L, 1ull << 26);
  if (hipMalloc(&e->merge_jobs, 2 * e->job_cap * sizeof(MergeJob)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->cond_jobs, 2 * e->job_cap * sizeof(uint64_t)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->job_counts, JOB_COUNTS * sizeof(uint32_t)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->merge_slow, e->job_cap * sizeof(uint32_t)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipHostMalloc(&e->h_hdr_pinned, 2 * sizeof(WaveHdr)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipHostMalloc(&e->h_err_pinned, 2 * sizeof(uint32_t)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipHostMalloc(&e->h_ctl_pinned, sizeof(TrajCtl)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipHostMalloc(&e->h_stats_pinned, 21 * sizeof(uint64_t)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipHostMalloc(&e->h_up, 1 << 20) != hipSuccess) return cleanup(ZB_ENOMEM);
  e->h_up_cap = 1 << 20;
  if (hipMalloc(&e->d_spread, sizeof(uint64_t)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->t_ctl, sizeof(TrajCtl)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->t_wtot, TRAJ_WAVE_CAP * sizeof(uint4)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->t_wbase, TRAJ_WAVE_CAP * sizeof(TrajBase)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->t_mgen, CLS_MAX * CLS_ROW * sizeof(MergeGen)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->t_tmpl, (size_t)CLS_MAX * CLS_ROW * TF * sizeof(TmplRec)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->t_cstat, CLS_MAX * TSTAT * sizeof(uint32_t)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMalloc(&e->raux, e->cfg.row_capacity * sizeof(RowAux)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMemset(e->raux, 0, e->cfg.row_capacity * sizeof(RowAux)) != hipSuccess) return cleanup(ZB_EDEVICE);
#ifdef ZB_PHASES
  if (hipMalloc(&e->phase, 16 * sizeof(unsigned long long)) != hipSuccess) return cleanup(ZB_ENOMEM);
  if (hipMemset(e->phase, 0, 16 * sizeof(unsigned long long)) != hipSuccess) return cleanup(ZB_EDEVICE);
#endif
  e->ev.resize(EV_PER_WAVE * WAVES_PER_SYNC_MAX);
  for (auto& x : e->ev)
    if (hipEventCreate(&x) != hipSuccess) return cleanup(ZB_EDEVICE);
  const uint8_t empty = 0x80;
  add_blob(e->static_blobs, &empty, 1);  // ref 0 = {} (DocumentValue.EMPTY_DOCUMENT)
  if (hipMemcpy(e->arena, e->static_blobs.data(), e->static_blobs.size(), hipMemcpyHostToDevice) != hipSuccess)
    return cleanup(ZB_EDEVICE);
  int rc = zb_reset(e, 0);
  if (rc == ZB_OK) rc = reserve_compaction(e);
  if (rc != ZB_OK) return cleanup(rc);
  *out = e;
  return ZB_OK;
}

void zb_engine_destroy(zb_engine* e) {
  if (!e) return;
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  for (auto& x : e->ev)
    if (x) (void)hipEventDestroy(x);
  void* ps[] = {e->vlen_mem, e->vlen_bad, e->jobs.keys, e->jobs.state, e->jobs.tombs, e->c_flag, e->c_new, e->c_tmp,
                e->c_scratch, e->c_bits, e->c_pop, e->c_off, e->c_count, e->x_keys, e->x_pos, e->x_keys2, e->x_pos2,
                e->sort_tmp, e->d_spread, e->mapres, e->map_ws, e->log_mem, e->links_mem, e->srcd_mem, e->row_mem, e->arena, e->hdr, e->derr, e->dstats, e->derr_info,
                e->merge_jobs, e->merge_slow, e->cond_jobs, e->job_counts, e->sub_jobs, e->cw, e->stage, e->info, e->block_agg, e->block_off, e->lookback,
                e->t_agg, e->t_woff, e->t_wcount, e->t_wtot, e->t_wbase, e->t_ctl, e->t_mgen, e->t_wstats, e->t_xq,
                e->c_plan, e->c_ikey, e->c_clen, e->d_cref, e->c_khist, e->c_mask, e->c_cg, e->c_woffw, e->c_wgcnt, e->c_wgoff, e->c_perm,
                e->t_tmpl, e->t_cstat, e->c_segs, e->c_wcls, e->raux, e->look_keys, e->look_idx,
                e->conf_first, e->phase};
  for (void* p : ps)
    if (p) (void)hipFree(p);
  xpool_release(e);
  if (e->comm) (void)ncclCommDestroy(e->comm);
  void* ms[] = {e->obox[0], e->obox[1], e->okeys[0], e->okeys[1], e->ovar[0], e->ovar[1], e->on, e->subs, e->sub_head,
                e->sub_next, e->msgs, e->msg_head, e->msg_next, e->d_xcounts, e->xsend, e->xrecv, e->ob_keys, e->ob_idx_in,
                e->ob_idx_out, e->ob_first, e->ob_sizes, e->ob_goff, e->ob_table, e->ob_base, e->ob_tmp, e->ob_staging,
                e->m_prior, e->m_cnt, e->m_tmp, e->in_buf, e->p_in, e->p_gran, e->d_unresolved, e->cs_cnt, e->cs_off,
                e->cs_tmp};
  for (void* p : ms)
    if (p) (void)hipFree(p);
  if (e->h_hdr_pinned) (void)hipHostFree(e->h_hdr_pinned);
  if (e->h_err_pinned) (void)hipHostFree(e->h_err_pinned);
  if (e->h_ctl_pinned) (void)hipHostFree(e->h_ctl_pinned);
  if (e->h_stats_pinned) (void)hipHostFree(e->h_stats_pinned);
  if (e->h_up) (void)hipHostFree(e->h_up);
  e->d_elems.free(); e->d_wfs.free(); e->d_cond.free(); e->d_code.free(); e->d_cls_code.free(); e->d_cls_atom.free(); e->d_cls_table.free(); e->d_consts.free(); e->d_const_w.free();
  e->d_queries.free(); e->d_filters.free(); e->d_pool.free(); e->d_staged.free(); e->d_staged_arena.free();
  e->d_ranges.free(); e->d_cmd_pool.free(); e->d_lookup_keys.free(); e->d_lookup_pos.free();
  e->d_maps.free();
  e->d_segs.free();
  e->d_vconst.free();
  e->d_vsegs.free();
  e->d_segpool.free();
  e->d_staged_vlen.free();
  e->d_staged_reqs.free();
  if (e->d_req) (void)hipFree(e->d_req);
  e->d_slices.free();
  void* dr[] = {e->dr_len, e->dr_off, e->dr_hdr, e->dr_val, e->dr_tmp, e->dr_total, e->dr_tiles, e->dr_pay, e->dr_tsum,
                e->dr_list, e->dr_list2};
  for (void* p : dr)
    if (p) (void)hipFree(p);
  if (e->h_dr_total) (void)hipHostFree(e->h_dr_total);
  if (e->h_stage) (void)hipHostFree(e->h_stage);
  for (auto& x : e->dr_ev)
    if (x) (void)hipEventDestroy(x);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
}

#ifdef ZB_PHASES
// the measurement build's k_wave phase sums since the engine was created (wall-clock ticks of 10 ns, summed over
// workgroups): [0] process + tile scan, [1] look-back, [2] emit, [3] tiles, [4] look-back rounds
int zb_phase_times(zb_engine* e, unsigned long long* out5) {
  if (!e || !out5) return ZB_EINVAL;
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  HIPCHECK(e, hipMemcpy(out5, e->phase, 5 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return ZB_OK;
}
// k_tdrain_write's phase sums (ticks of 10 ns summed over waves): [0] generation setup (bases, records, scan),
// [1] headers, [2] encode, [3] image stream (with its two wave syncs), [4] waves, [5] generations
int zb_tdrain_phase_times(zb_engine* e, unsigned long long* out6) {
  if (!e || !out6) return ZB_EINVAL;
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  HIPCHECK(e, hipMemcpy(out6, e->phase + 8, 6 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return ZB_OK;
}
#endif

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
  HIPCHECK(e, hipMemsetAsync(e->job_counts, 0, JOB_COUNTS * sizeof(uint32_t), e->stream));
  HIPCHECK(e, hipMemsetAsync(e->dstats, 0, STAT_WORDS * sizeof(uint64_t), e->stream));  // (banks too)
  if (e->jobs.keys) {
    HIPCHECK(e, hipMemsetAsync(e->jobs.keys, 0, (e->jobs.mask + 1) * sizeof(int64_t), e->stream));  // JOB_EMPTY
    HIPCHECK(e, hipMemsetAsync(e->jobs.state, 0, e->jobs.mask + 1, e->stream));
    HIPCHECK(e, hipMemsetAsync(e->jobs.tombs, 0, sizeof(uint32_t), e->stream));
  }
  e->win_base = e->released = 0;
  e->seg_pending = false;  // (the log is empty again)
  rebias(e);
  e->rows_total = e->arena_total = e->records_total = e->compactions = 0;
  e->rows_mark = 0;
  e->arena_mark = STATIC_ARENA_BYTES;
  // (a kept batch's documents stay where they were uploaded; everything above them is free again)
  const bool keep_docs = keep_staged && e->staged_uploaded && e->staged_in_place;
  e->arena_top = keep_docs ? e->staged_base : e->cfg.arena_bytes;
  if (keep_docs) e->staged_top = e->cfg.arena_bytes;
  else e->staged_in_place = false;
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  e->ranges.clear();
  e->cmd_pool.clear();
  e->req_runs.clear();
  e->req_lo = e->req_n = 0;
  if (!keep_staged) {
    e->staged_reqs.clear();
    e->staged_reqs_uploaded = false;
    e->staged.clear();
    e->staged_vlen.clear();
    e->staged_arena.clear();
    e->pending_ranges.clear();
    e->staged_lookup.clear();
    e->staged_only_creates = true;
    e->staged_has_cancel = false;
    e->tick_inst.clear();
    e->tick_aik.clear();
    e->tick_jobs.clear();
    e->staged_uploaded = false;
    // (the wave hints stay: a reset starts the log again, not a new workload -- the next tick of the same model
    // settles in as many waves, as it would on a partition that never resets; zb_deploy clears them)
  }
  e->term = false;
  e->conf_active = false;
  e->staged_pending = !e->staged.empty();
  e->sub_count = e->msg_count = 0;
  e->msg_key_next = 0;
  if (e->on) HIPCHECK(e, hipMemsetAsync(e->on, 0, 4 * sizeof(uint32_t), e->stream));
  e->ob_counts_valid = false;
  e->ob_pos_base[0] = e->ob_pos_base[1] = 0;
  e->clock_ms = 0;
  if (e->subs) {
    HIPCHECK(e, hipMemsetAsync(e->sub_head, 0xff, (e->head_mask + 1) * sizeof(uint32_t), e->stream));
    HIPCHECK(e, hipMemsetAsync(e->msg_head, 0xff, (e->head_mask + 1) * sizeof(uint32_t), e->stream));
  }
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  return ZB_OK;
}

int zb_validate_deployment(const uint8_t* xml, size_t len, char* err, size_t err_cap) {
  if (!xml) return ZB_EINVAL;
  ModelTables t;
  std::string msg;
  const int rc = compile_deployment(t, std::string((const char*)xml, len), 1, 1, msg);
  if (err && err_cap) {
    const size_t n = std::min(msg.size(), err_cap - 1);
    std::memcpy(err, msg.data(), n);
    err[n] = 0;
  }
  return rc;
}

int zb_deploy(zb_engine* e, int64_t workflow_key, int32_t version, const uint8_t* xml, size_t len) {
  if (!e || !xml) return ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  std::string msg;
  int rc = compile_deployment(e->model, std::string((const char*)xml, len), workflow_key, version, msg);
  if (rc != ZB_OK) return fail(e, rc, msg);
  for (int& h : e->wave_hint) h = 0;  // (the last tick's wave count says nothing about the new model's ticks)
  for (const DevElem& el : e->model.elems) {
    if (el.step[WI_ELEMENT_COMPLETING] == ST_APPLY_OUTPUT_MAPPING) e->has_merges = true;
    if (el.step[WI_GATEWAY_ACTIVATED] == ST_EXCLUSIVE_SPLIT) e->has_splits = true;
    if (el.kind == EK_CATCH) e->has_catch = true;
    if (el.kind == EK_PAR) e->has_parallel = true;
    if (el.flags & EF_IO) e->has_io = true;
    if (el.kind == EK_TASK || el.step[WI_ELEMENT_ACTIVATED] == ST_CREATE_JOB) e->has_tasks = true;
  }
  if (e->has_io && !e->mapres) {
    HIPCHECK(e, hipMalloc(&e->mapres, (e->wave_cap + 8) * sizeof(uint64_t)));
    HIPCHECK(e, hipMalloc(&e->map_ws, (size_t)MAP_GRID * 256 * MAP_NODES * sizeof(MNode)));
  }
  if (e->has_io || e->has_merges) {  // payloads the structural merge / mapper refuse: the device's shared workspaces
    const int xrc = xpool_acquire(e);
    if (xrc != ZB_OK) return xrc;
  }
  if (e->has_catch) {
    int orc = ensure_outbox(e);
    if (orc != ZB_OK) return orc;
  }
  // the trajectory count pass skips payload merges, so conditions must never read a merge result
  e->traj_model_ok = !(e->has_merges && e->has_splits) && !e->has_io;
  e->traj_skip = 0;  // (a new model: try the trajectory path again)
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
  // the condition queries the class path extracts in one scan: every path operand of every split's conditions,
  // all of the [ROOT, MAP_KEY k] form, at most CLS_QMAX distinct (else each operand runs its own query)
  e->cls_nq = 0;
  bool ext_ok = e->cls_ok;
  for (int k = 0; k < e->nsplits && ext_ok; k++) {
    const DevElem& el = e->model.elems[e->split_elem[k]];
    for (uint32_t c = 0; c < el.cond_count && ext_ok; c++) {
      const DevElem& flow = e->model.elems[e->model.cond_flows[el.cond_begin + c]];
      if (flow.cond_prog == NO_REF) continue;
      for (uint32_t pc = flow.cond_prog; 2 * pc + 1 < e->model.code.size(); pc++) {
        const uint32_t w0 = e->model.code[2 * pc], w1 = e->model.code[2 * pc + 1];
        if ((w0 & 0xff) == PC_END) break;
        if ((w0 & 0xff) != PC_CMP) continue;
        for (int side = 0; side < 2 && ext_ok; side++) {
          if (!((w0 >> (12 + side)) & 1)) continue;
          const uint16_t q = (uint16_t)(side ? w1 >> 16 : w1 & 0xffff);
          const DevQuery& dq = e->model.queries[q];
          if (!dq.fast) { ext_ok = false; break; }
          bool seen = false;
          for (int j = 0; j < e->cls_nq; j++) seen = seen || e->cls_q[j] == q;
          if (seen) continue;
          if (e->cls_nq == CLS_QMAX) { ext_ok = false; break; }
          const DevFilter& f = e->model.filters[dq.first + 1];
          e->cls_q[e->cls_nq] = q;
          e->cls_key_off[e->cls_nq] = f.key_off;
          e->cls_key_len[e->cls_nq] = f.key_len;
          e->cls_key_w[e->cls_nq][0] = e->cls_key_w[e->cls_nq][1] = 0;
          for (uint32_t b = 0; b < f.key_len && b < 16; b++)
            e->cls_key_w[e->cls_nq][b / 8] |= (uint64_t)e->model.pool[f.key_off + b] << (8 * (b % 8));
          e->cls_nq++;
        }
      }
    }
  }
  if (!ext_ok) e->cls_nq = 0;
  // k_cls_classify runs the split conditions on the extracted operands: their path operand fields name the
  // extraction slot instead of the query (a wave-uniform index into the extraction)
  std::vector<uint32_t> cc = e->model.code;
  if (e->cls_nq) {
    for (int k = 0; k < e->nsplits; k++) {
      const DevElem& el = e->model.elems[e->split_elem[k]];
      for (uint32_t c = 0; c < el.cond_count; c++) {
        const DevElem& flow = e->model.elems[e->model.cond_flows[el.cond_begin + c]];
        if (flow.cond_prog == NO_REF) continue;
        for (uint32_t pc = flow.cond_prog; 2 * pc + 1 < cc.size(); pc++) {
          const uint32_t w0 = cc[2 * pc];
          if ((w0 & 0xff) == PC_END) break;
          if ((w0 & 0xff) != PC_CMP) continue;
          uint32_t w1 = e->model.code[2 * pc + 1];
          for (int side = 0; side < 2; side++) {
            if (!((w0 >> (12 + side)) & 1)) continue;
            const uint16_t q = (uint16_t)(side ? w1 >> 16 : w1 & 0xffff);
            uint32_t j = 0;
            while ((int)j < e->cls_nq && e->cls_q[j] != q) j++;
            w1 = side ? ((w1 & 0xffffu) | j << 16) : ((w1 & 0xffff0000u) | j);
          }
          cc[2 * pc + 1] = w1;
        }
      }
    }
  }
  HIPCHECK(e, e->d_cls_code.upload(cc, e->stream));
  // The outcome table: with at most CLS_TABLE_ATOMS comparisons in the split conditions, the class key is a function
  // of their outcomes (false / true / error), which the conditions' programs give by this walk -- the control flow of
  // eval_condition_sweep: forward jumps on the last result, an error ends the condition (its split's digit: cc + 1)
  e->cls_natoms = 0;
  if (e->cls_nq) {
    std::vector<uint32_t> atoms;
    bool ok = true;
    for (int k = 0; k < e->nsplits && ok; k++) {
      const DevElem& el = e->model.elems[e->split_elem[k]];
      for (uint32_t c = 0; c < el.cond_count && ok; c++) {
        const DevElem& flow = e->model.elems[e->model.cond_flows[el.cond_begin + c]];
        if (flow.cond_prog == NO_REF) { ok = false; break; }
        for (uint32_t pc = flow.cond_prog; ; pc++) {
          if (2 * pc + 1 >= cc.size()) { ok = false; break; }
          const uint32_t op = cc[2 * pc] & 0xff;
          if (op == PC_END) break;
          if (op == PC_CMP && std::find(atoms.begin(), atoms.end(), pc) == atoms.end()) atoms.push_back(pc);
        }
      }
    }
    if (ok && !atoms.empty() && atoms.size() <= CLS_TABLE_ATOMS) {
      uint32_t entries = 1;
      for (size_t a = 0; a < atoms.size(); a++) entries *= 3;
      std::vector<uint8_t> table(entries);
      std::vector<uint8_t> out(atoms.size());
      for (uint32_t idx = 0; idx < entries && ok; idx++) {
        for (size_t a = 0, v = idx; a < atoms.size(); a++, v /= 3) out[a] = (uint8_t)(v % 3);
        uint32_t key = 0;
        for (int k = 0; k < e->nsplits; k++) {
          const DevElem& el = e->model.elems[e->split_elem[k]];
          uint32_t o = el.cond_count;
          for (uint32_t c = 0; c < el.cond_count; c++) {
            const DevElem& flow = e->model.elems[e->model.cond_flows[el.cond_begin + c]];
            int res = 0;  // 0 false, 1 true, 2 error
            bool r = false;
            for (uint32_t pc = flow.cond_prog; 2 * pc + 1 < cc.size();) {
              const uint32_t w0 = cc[2 * pc], opc = w0 & 0xff;
              if (opc == PC_END) { res = r ? 1 : 0; break; }
              if (opc == PC_JF || opc == PC_JT) {
                pc = ((opc == PC_JF) ? !r : r) ? (w0 >> 16) : pc + 1;
                continue;
              }
              const uint8_t v = out[std::find(atoms.begin(), atoms.end(), pc) - atoms.begin()];
              if (v == 2) { res = 2; break; }
              r = v == 1;
              pc++;
            }
            if (res == 2) { o = el.cond_count + 1; break; }
            if (res == 1) { o = c; break; }
          }
          key += o * e->split_stride[k];
        }
        if (key > 255) ok = false;
        table[idx] = (uint8_t)key;
      }
      if (ok) {
        std::vector<uint32_t> aw;  // (the code words themselves: no dependent load of the pc on the device)
        for (uint32_t pc : atoms) { aw.push_back(cc[2 * pc]); aw.push_back(cc[2 * pc + 1]); }
        HIPCHECK(e, e->d_cls_atom.upload(aw, e->stream));
        HIPCHECK(e, e->d_cls_table.upload(table, e->stream));
        e->cls_natoms = (int)atoms.size();
      }
    }
  }
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

}  // extern "C"

// resolve a CREATE's workflow like CreateWorkflowInstanceEventProcessor (all workflows are deployed locally):
// workflow_key > 0 by key, else version > 0 by (process id, version), else the latest version
uint16_t resolve_process(const zb_engine* e, const std::string& spid, int32_t version, int64_t workflow_key) {
  uint16_t pelem = NO_ELEM;
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
  return pelem;
}

bool is_doc(const uint8_t* p, uint64_t len) {  // DocumentValue: nil / empty -> {}, else a map
  if (len == 0 || (len == 1 && p[0] == 0xc0)) return true;
  const uint8_t b = p[0];
  return (b & 0xf0) == 0x80 || b == 0xde || b == 0xdf;
}

// the staged batch of the last zb_step was injected: start a new one
void begin_staging(zb_engine* e) {
  if (e->staged_pending) return;
  e->staged_in_place = false;  // (the injected batch's documents belong to the arena's top region now)
  e->staged_reqs.clear();
  e->staged_reqs_uploaded = false;
  e->staged.clear();
  e->staged_vlen.clear();
  e->staged_arena.clear();
  e->pending_ranges.clear();
  e->staged_lookup.clear();
  e->staged_only_creates = true;
  e->staged_has_cancel = false;
  e->tick_inst.clear();
  e->tick_aik.clear();
  e->tick_jobs.clear();
  e->tick_conflicts.clear();
  e->staged_uploaded = false;
}

// the staged batch on the device: descriptors, value lengths, arena bytes, and the (key, staged index) pairs of
// the records that name an element instance (ElementInstanceIndex.getInstance), sorted by zb_step on the device
int upload_staged(zb_engine* e) {
  if (e->staged_uploaded) return ZB_OK;
  HIPCHECK(e, e->d_staged.upload(e->staged, e->stream));
  if (!e->staged_reqs.empty() && !e->staged_reqs_uploaded) {
    HIPCHECK(e, e->d_staged_reqs.upload(e->staged_reqs, e->stream));
    e->staged_reqs_uploaded = true;
  }
  HIPCHECK(e, e->d_staged_vlen.upload(e->staged_vlen, e->stream));
  // the documents: in place at the top of the arena when they fit above the allocators' bytes (an earlier upload
  // of this same batch gives its room back first), else into a staging buffer that k_inject copies from
  if (e->staged_in_place) e->arena_top = e->staged_top;
  e->staged_in_place = false;
  const uint64_t sb = e->staged_arena.size();  // (whole granules: add_blob)
  if (sb && e->arena_top >= (uint64_t)e->host_hdr.arena_next + sb) {
    e->staged_top = e->arena_top;
    e->staged_base = e->arena_top - sb;
    HIPCHECK(e, hipMemcpyAsync(e->arena + e->staged_base, e->staged_arena.data(), sb, hipMemcpyHostToDevice, e->stream));
    e->arena_top = e->staged_base;
    e->staged_in_place = true;
  } else {
    HIPCHECK(e, e->d_staged_arena.upload(e->staged_arena, e->stream));
  }
  e->staged_nlook = 0;
  if (!e->staged_only_creates) {  // (CREATE-only batches name no element instance)
    std::vector<int64_t> lk, li;
    uint64_t spread = 0;  // (the device sort's key bits, known here: zb_step needs no round trip for them)
    for (size_t i = 0; i < e->staged_lookup.size(); i++)
      if (e->staged_lookup[i] != INT64_MIN) {
        lk.push_back(e->staged_lookup[i]);
        li.push_back((int64_t)i);
        spread |= (uint64_t)lk.back() ^ (uint64_t)lk[0];
      }
    e->staged_lookup_spread = spread;
    if (!lk.empty()) {
      HIPCHECK(e, e->d_lookup_keys.upload(lk, e->stream));
      HIPCHECK(e, e->d_lookup_pos.upload(li, e->stream));
      HIPCHECK(e, hipStreamSynchronize(e->stream));  // (the host vectors die here)
    }
    e->staged_nlook = lk.size();
  }
  e->staged_conf = e->tick_conflicts.size();
  if (e->staged_conf) {  // open addressing at load <= 1/2
    uint64_t cap = 64;
    while (cap < 2 * e->staged_conf) cap <<= 1;
    std::vector<int64_t> tab(cap, INT64_MIN);
    for (int64_t k : e->tick_conflicts) {
      uint64_t h = ((uint64_t)k * 0x9E3779B97F4A7C15ull >> 32) & (cap - 1);
      while (tab[h] != INT64_MIN) h = (h + 1) & (cap - 1);
      tab[h] = k;
    }
    HIPCHECK(e, e->d_conf_keys.upload(tab, e->stream));
    if (cap > e->conf_cap) {
      HIPCHECK(e, hipStreamSynchronize(e->stream));
      if (e->conf_first) (void)hipFree(e->conf_first);
      e->conf_first = nullptr;
      HIPCHECK(e, hipMalloc(&e->conf_first, (cap + 1) * sizeof(int64_t)));
      e->conf_cap = cap;
    }
    e->conf_mask = cap - 1;
    HIPCHECK(e, hipStreamSynchronize(e->stream));  // (the host table dies here)
  }
  e->staged_uploaded = true;
  return ZB_OK;
}

extern "C" {

int zb_upload_staged(zb_engine* e) {
  if (!e) return ZB_EINVAL;
  if (!e->staged_pending || e->staged.empty()) return ZB_OK;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  return upload_staged(e);
}

int zb_submit_creates(zb_engine* e, const char* pid, int32_t version, int64_t workflow_key, size_t n,
                      const uint8_t* payloads, const uint64_t* offsets) {
  if (!e || (n > 0 && (!payloads || !offsets)) || !pid) return ZB_EINVAL;
  // validate everything before any staged state changes (all-or-nothing)
  for (size_t i = 0; i < n; i++) {
    if (offsets[i + 1] < offsets[i] || offsets[i + 1] - offsets[i] > 0xffffffffull) return fail(e, ZB_EINVAL, "bad payload offsets");
    if (!is_doc(payloads + offsets[i], offsets[i + 1] - offsets[i]))
      return fail(e, ZB_EINVAL, "Document has invalid format. On root level an object is only allowed.");
  }
  const std::string spid(pid);
  if (spid.size() > 0xffff) return fail(e, ZB_EINVAL, "bpmn process id too long");
  const uint16_t pelem = resolve_process(e, spid, version, workflow_key);
  begin_staging(e);
  e->staged_uploaded = false;  // the device copy (if any) no longer matches
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
  e->staged_lookup.reserve(e->staged_lookup.size() + n);
  for (size_t i = 0; i < n; i++) {
    const uint8_t* p = payloads + offsets[i];
    uint64_t len = offsets[i + 1] - offsets[i];
    uint32_t ref;
    if (len == 0 || (len == 1 && p[0] == 0xc0)) {
      const uint8_t empty = 0x80;  // DocumentValue: nil / empty -> {}
      ref = add_blob(e->staged_arena, &empty, 1);
    } else {
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
    // the command's value (zb_serialize.hip encode_value, submitted CREATE): pid / version / workflowKey of
    // the call, instance / scope keys -1, activityId ""
    const uint32_t plen = (len == 0 || (len == 1 && p[0] == 0xc0)) ? 1u : (uint32_t)len;
    e->staged_vlen.push_back(1 + 14 + mp_str_len((uint32_t)spid.size()) + 8 + mp_int_len(version) + 12 +
                             mp_int_len(workflow_key) + 20 + 1 + 11 + 1 + 8 + mp_bin_len(plen) + 17 + 1);
    e->staged_lookup.push_back(INT64_MIN);
  }
  e->pending_ranges.push_back(pr);
  e->staged_pending = true;
  return ZB_OK;
}

}  // extern "C"

// ---- zb_submit: host-side decoding of reference record values (UnpackedObject.wrap, ObjectValue.java:93-131)
namespace {

struct MpIn {
  const uint8_t* p;
  size_t n, o = 0;
  bool ok = true;
  uint8_t u8() { if (o >= n) { ok = false; return 0; } return p[o++]; }
  uint64_t be(int k) { uint64_t v = 0; for (int i = 0; i < k; i++) v = (v << 8) | u8(); return v; }
  uint32_t map_hdr() {
    uint8_t h = u8();
    if ((h & 0xf0) == 0x80) return h & 0x0f;
    if (h == 0xde) return (uint32_t)be(2);
    if (h == 0xdf) return (uint32_t)be(4);
    ok = false;
    return 0;
  }
  bool str(const uint8_t*& s, uint32_t& len) {
    uint8_t h = u8();
    if ((h & 0xe0) == 0xa0) len = h & 0x1f;
    else if (h == 0xd9) len = (uint32_t)be(1);
    else if (h == 0xda) len = (uint32_t)be(2);
    else if (h == 0xdb) len = (uint32_t)be(4);
    else { ok = false; return false; }
    if (o + len > n) { ok = false; return false; }
    s = p + o; o += len;
    return true;
  }
  bool bin(const uint8_t*& s, uint32_t& len) {
    uint8_t h = u8();
    if (h == 0xc4) len = (uint32_t)be(1);
    else if (h == 0xc5) len = (uint32_t)be(2);
    else if (h == 0xc6) len = (uint32_t)be(4);
    else { ok = false; return false; }
    if (o + len > n) { ok = false; return false; }
    s = p + o; o += len;
    return true;
  }
  int64_t integer() {
    uint8_t h = u8();
    if (h <= 0x7f) return h;
    if (h >= 0xe0) return (int8_t)h;
    switch (h) {
      case 0xcc: return (int64_t)be(1);
      case 0xcd: return (int64_t)be(2);
      case 0xce: return (int64_t)be(4);
      case 0xcf: return (int64_t)be(8);
      case 0xd0: return (int8_t)be(1);
      case 0xd1: return (int16_t)be(2);
      case 0xd2: return (int32_t)be(4);
      case 0xd3: return (int64_t)be(8);
    }
    ok = false;
    return 0;
  }
  void skip(int64_t count = 1) {  // MsgPackReader.skipValues
    while (count > 0 && ok) {
      uint8_t b = u8();
      if (b <= 0x7f || b >= 0xe0 || b == 0xc0 || b == 0xc2 || b == 0xc3) {
      } else if ((b & 0xf0) == 0x80) count += (int64_t)(b & 0x0f) * 2;
      else if ((b & 0xf0) == 0x90) count += (b & 0x0f);
      else if ((b & 0xe0) == 0xa0) o += (b & 0x1f);
      else switch (b) {
        case 0xd0: case 0xcc: o += 1; break;
        case 0xd1: case 0xcd: o += 2; break;
        case 0xd2: case 0xce: case 0xca: o += 4; break;
        case 0xd3: case 0xcf: case 0xcb: o += 8; break;
        case 0xc4: case 0xd9: o += be(1); break;
        case 0xc5: case 0xda: o += be(2); break;
        case 0xc6: case 0xdb: o += be(4); break;
        case 0xd4: o += 2; break;
        case 0xd5: o += 3; break;
        case 0xd6: o += 5; break;
        case 0xd7: o += 9; break;
        case 0xd8: o += 17; break;
        case 0xc7: o += 1 + be(1); break;
        case 0xc8: o += 1 + be(2); break;
        case 0xc9: o += 1 + be(4); break;
        case 0xdc: count += be(2); break;
        case 0xdd: count += be(4); break;
        case 0xde: count += (int64_t)be(2) * 2; break;
        case 0xdf: count += (int64_t)be(4) * 2; break;
        default: ok = false;
      }
      if (o > n) ok = false;
      count--;
    }
  }
  bool key_is(const uint8_t* k, uint32_t kl, const char* s) { return kl == strlen(s) && memcmp(k, s, kl) == 0; }
};

// the declared properties a submitted value carries (defaults as in the reference records)
struct Decoded {
  std::string bpmn_process_id, message_name, activity_id;
  int64_t version = -1, workflow_key = -1, wik = -1, aik = -1, scope = -1;
  const uint8_t* payload = nullptr;
  uint32_t payload_len = 0;
  // JobRecord / JobHeaders (JobRecord.java:35-53, JobHeaders.java:33-51)
  int64_t deadline = INT64_MIN, retries = -1;
  std::string worker, type;
  const uint8_t* custom_headers = nullptr;  // PackedProperty, raw
  uint32_t custom_headers_len = 0;
};

bool decode_value(uint8_t vt, const uint8_t* v, size_t n, Decoded& d) {
  if (n == 0) return true;
  MpIn in{v, n};
  const uint32_t props = in.map_hdr();
  for (uint32_t i = 0; i < props && in.ok; i++) {
    const uint8_t* k; uint32_t kl;
    if (!in.str(k, kl)) return false;
    const uint8_t* s; uint32_t sl;
    if (in.key_is(k, kl, "payload")) {
      if (!in.bin(d.payload, d.payload_len)) return false;
    } else if (vt == ZB_VT_WORKFLOW_INSTANCE && in.key_is(k, kl, "bpmnProcessId")) {
      if (!in.str(s, sl)) return false;
      d.bpmn_process_id.assign((const char*)s, sl);
    } else if (vt == ZB_VT_WORKFLOW_INSTANCE && in.key_is(k, kl, "version")) d.version = in.integer();
    else if (vt == ZB_VT_WORKFLOW_INSTANCE && in.key_is(k, kl, "workflowKey")) d.workflow_key = in.integer();
    else if (vt != ZB_VT_JOB && in.key_is(k, kl, "workflowInstanceKey")) d.wik = in.integer();
    else if (vt == ZB_VT_WORKFLOW_INSTANCE && in.key_is(k, kl, "scopeInstanceKey")) d.scope = in.integer();
    else if (vt == ZB_VT_WORKFLOW_INSTANCE_SUBSCRIPTION && in.key_is(k, kl, "activityInstanceKey")) d.aik = in.integer();
    else if (vt == ZB_VT_WORKFLOW_INSTANCE_SUBSCRIPTION && in.key_is(k, kl, "messageName")) {
      if (!in.str(s, sl)) return false;
      d.message_name.assign((const char*)s, sl);
    } else if (vt == ZB_VT_WORKFLOW_INSTANCE && in.key_is(k, kl, "activityId")) {
      if (!in.str(s, sl)) return false;
      d.activity_id.assign((const char*)s, sl);
    } else if (vt == ZB_VT_JOB && in.key_is(k, kl, "headers")) {  // JobHeaders.java:33-51
      const uint32_t hp = in.map_hdr();
      for (uint32_t j = 0; j < hp && in.ok; j++) {
        const uint8_t* hk; uint32_t hkl;
        if (!in.str(hk, hkl)) return false;
        if (in.key_is(hk, hkl, "workflowInstanceKey")) d.wik = in.integer();
        else if (in.key_is(hk, hkl, "activityInstanceKey")) d.aik = in.integer();
        else if (in.key_is(hk, hkl, "workflowKey")) d.workflow_key = in.integer();
        else if (in.key_is(hk, hkl, "workflowDefinitionVersion")) d.version = in.integer();
        else if (in.key_is(hk, hkl, "bpmnProcessId")) {
          if (!in.str(s, sl)) return false;
          d.bpmn_process_id.assign((const char*)s, sl);
        } else if (in.key_is(hk, hkl, "activityId")) {
          if (!in.str(s, sl)) return false;
          d.activity_id.assign((const char*)s, sl);
        } else in.skip();
      }
    } else if (vt == ZB_VT_JOB && in.key_is(k, kl, "deadline")) d.deadline = in.integer();
    else if (vt == ZB_VT_JOB && in.key_is(k, kl, "retries")) d.retries = in.integer();
    else if (vt == ZB_VT_JOB && (in.key_is(k, kl, "worker") || in.key_is(k, kl, "type"))) {
      const bool w = in.key_is(k, kl, "worker");
      if (!in.str(s, sl)) return false;
      (w ? d.worker : d.type).assign((const char*)s, sl);
    } else if (vt == ZB_VT_JOB && in.key_is(k, kl, "customHeaders")) {
      const size_t st = in.o;
      in.skip();
      d.custom_headers = v + st;
      d.custom_headers_len = (uint32_t)(in.o - st);
    } else in.skip();
  }
  return in.ok && in.o == n;
}

// MsgPackWriter.writeInteger (MsgPackWriter.java:143-201)
void put_int(std::vector<uint8_t>& b, int64_t v) {
  auto be = [&](uint64_t x, int k) { for (int i = k - 1; i >= 0; i--) b.push_back((uint8_t)(x >> (8 * i))); };
  if (v < -(1LL << 5)) {
    if (v < -(1LL << 15)) { if (v < -(1LL << 31)) { b.push_back(0xd3); be((uint64_t)v, 8); } else { b.push_back(0xd2); be((uint64_t)v, 4); } }
    else if (v < -(1 << 7)) { b.push_back(0xd1); be((uint64_t)v, 2); }
    else { b.push_back(0xd0); be((uint64_t)v, 1); }
  } else if (v < (1 << 7)) b.push_back((uint8_t)v);
  else if (v < (1LL << 8)) { b.push_back(0xcc); be((uint64_t)v, 1); }
  else if (v < (1LL << 16)) { b.push_back(0xcd); be((uint64_t)v, 2); }
  else if (v < (1LL << 32)) { b.push_back(0xce); be((uint64_t)v, 4); }
  else { b.push_back(0xcf); be((uint64_t)v, 8); }
}
void put_str(std::vector<uint8_t>& b, const std::string& s) {
  const size_t n = s.size();
  if (n < 32) b.push_back((uint8_t)(0xa0 | n));
  else if (n < 256) { b.push_back(0xd9); b.push_back((uint8_t)n); }
  else if (n < 65536) { b.push_back(0xda); b.push_back((uint8_t)(n >> 8)); b.push_back((uint8_t)n); }
  else { b.push_back(0xdb); for (int i = 3; i >= 0; i--) b.push_back((uint8_t)(n >> (8 * i))); }
  b.insert(b.end(), s.begin(), s.end());
}
void put_bin(std::vector<uint8_t>& b, const uint8_t* p, uint32_t n) {
  if (n < 256) { b.push_back(0xc4); b.push_back((uint8_t)n); }
  else if (n < 65536) { b.push_back(0xc5); b.push_back((uint8_t)(n >> 8)); b.push_back((uint8_t)n); }
  else { b.push_back(0xc6); for (int i = 3; i >= 0; i--) b.push_back((uint8_t)(n >> (8 * i))); }
  b.insert(b.end(), p, p + n);
}

// the command value as the reference writes it back (CommandProcessorImpl.accept / writeRejection:
// record.getValue() re-encoded: declared properties in order, ObjectValue.java:140-153)
std::vector<uint8_t> reencode(uint8_t vt, const Decoded& d, const uint8_t* doc, uint32_t doc_len) {
  std::vector<uint8_t> b;
  if (vt == ZB_VT_WORKFLOW_INSTANCE) {  // WorkflowInstanceRecord.java:39-60
    b.push_back(0x87);
    put_str(b, "bpmnProcessId"); put_str(b, d.bpmn_process_id);
    put_str(b, "version"); put_int(b, d.version);
    put_str(b, "workflowKey"); put_int(b, d.workflow_key);
    put_str(b, "workflowInstanceKey"); put_int(b, d.wik);
    put_str(b, "activityId"); put_str(b, d.activity_id);
    put_str(b, "payload"); put_bin(b, doc, doc_len);
    put_str(b, "scopeInstanceKey"); put_int(b, d.scope);
  } else if (vt == ZB_VT_JOB) {  // JobRecord.java:35-53 with JobHeaders.java:33-51
    b.push_back(0x87);
    put_str(b, "deadline"); put_int(b, d.deadline);
    put_str(b, "worker"); put_str(b, d.worker);
    put_str(b, "retries"); put_int(b, d.retries);
    put_str(b, "type"); put_str(b, d.type);
    put_str(b, "headers");
    b.push_back(0x86);
    put_str(b, "bpmnProcessId"); put_str(b, d.bpmn_process_id);
    put_str(b, "workflowDefinitionVersion"); put_int(b, d.version);
    put_str(b, "workflowKey"); put_int(b, d.workflow_key);
    put_str(b, "workflowInstanceKey"); put_int(b, d.wik);
    put_str(b, "activityId"); put_str(b, d.activity_id);
    put_str(b, "activityInstanceKey"); put_int(b, d.aik);
    put_str(b, "customHeaders");
    if (d.custom_headers) b.insert(b.end(), d.custom_headers, d.custom_headers + d.custom_headers_len);
    else b.push_back(0x80);  // JobRecord.NO_HEADERS
    put_str(b, "payload"); put_bin(b, doc, doc_len);
  } else {  // WorkflowInstanceSubscriptionRecord.java:26-38
    b.push_back(0x84);
    put_str(b, "workflowInstanceKey"); put_int(b, d.wik);
    put_str(b, "activityInstanceKey"); put_int(b, d.aik);
    put_str(b, "messageName"); put_str(b, d.message_name);
    put_str(b, "payload"); put_bin(b, doc, doc_len);
  }
  return b;
}

}  // namespace

extern "C" {

int zb_submit(zb_engine* e, const zb_rec_desc* recs, size_t n, const uint8_t* values, size_t values_len) {
  if (!e || (n > 0 && (!recs || (!values && values_len)))) return ZB_EINVAL;
  if (e->failed) return fail(e, ZB_EPROCESSING, "partition stopped after a processing failure: " + e->err);
  struct Prep {
    zb_rec d;
    int64_t lookup = INT64_MIN, inst = INT64_MIN, aik = INT64_MIN;
    bool scope_cmd = false, pair = false, cancel = false, create = false, job_cmd = false;
    uint16_t pelem = NO_ELEM;
    std::string pid;
    int64_t wkey = -1;
    int32_t version = -1;
    const uint8_t* raw = nullptr;
    uint32_t raw_len = 0;
    const uint8_t* doc = nullptr;
    uint32_t doc_len = 0;
    std::vector<uint8_t> canon;
  };
  std::vector<Prep> prep(n);
  static const uint8_t EMPTY = 0x80;
  // 1. decode + validate (nothing staged on any error)
  for (size_t i = 0; i < n; i++) {
    const zb_rec_desc& r = recs[i];
    if (r.value_offset > values_len || r.value_length > values_len - r.value_offset)
      return fail(e, ZB_EINVAL, "record " + std::to_string(i) + ": value out of range");
    Prep& p = prep[i];
    p.raw = values + r.value_offset;
    p.raw_len = r.value_length;
    Decoded dv;
    const uint8_t vt = r.value_type, rt = r.record_type, it = r.intent;
    const bool wf_cmd = vt == ZB_VT_WORKFLOW_INSTANCE && rt == ZB_RT_COMMAND;
    const bool job_ev = vt == ZB_VT_JOB && rt == ZB_RT_EVENT && (it == JI_CREATED || it == JI_COMPLETED);
    const bool corr = vt == ZB_VT_WORKFLOW_INSTANCE_SUBSCRIPTION && rt == ZB_RT_COMMAND && it == 0;
    // the job stream processor's commands (JobInstanceStreamProcessor.java:76-84), with ZB_CFG_JOB_PROCESSOR
    const bool job_cmd = vt == ZB_VT_JOB && rt == ZB_RT_COMMAND && (e->cfg.flags & ZB_CFG_JOB_PROCESSOR) &&
                         (it == JI_CREATE || it == JI_ACTIVATE || it == JI_COMPLETE || it == JI_FAIL ||
                          it == JI_TIME_OUT || it == JI_UPDATE_RETRIES || it == JI_CANCEL);
    if (!(wf_cmd && (it == WI_CREATE || it == WI_CANCEL || it == WI_UPDATE_PAYLOAD)) && !job_ev && !corr && !job_cmd)
      return fail(e, ZB_EUNSUPPORTED, "record " + std::to_string(i) + ": no workflow processor is registered for "
                                      "(recordType, valueType, intent) = (" + std::to_string(rt) + ", " +
                                      std::to_string(vt) + ", " + std::to_string(it) + ")");
    if (!decode_value(vt, p.raw, p.raw_len, dv))
      return fail(e, ZB_EINVAL, "record " + std::to_string(i) + ": malformed msgpack value");
    p.doc = dv.payload ? dv.payload : &EMPTY;
    p.doc_len = dv.payload ? dv.payload_len : 1;
    if (p.doc_len == 0 || (p.doc_len == 1 && p.doc[0] == 0xc0)) { p.doc = &EMPTY; p.doc_len = 1; }
    if (!is_doc(p.doc, p.doc_len))
      return fail(e, ZB_EINVAL, "record " + std::to_string(i) + ": Document has invalid format. On root level an object is only allowed.");
    zb_rec& d = p.d;
    d.key = r.key;
    d.scope_key = -1;
    d.inst_key = -1;
    d.payload = 0;
    d.elem = NO_ELEM;
    d.intent = it;
    d.kind = (uint8_t)(make_kind(vt, rt, false) | KIND_RAW);
    if (wf_cmd && it == WI_CREATE) {
      p.create = true;
      if (dv.bpmn_process_id.size() > 0xffff) return fail(e, ZB_EINVAL, "bpmn process id too long");
      p.pid = dv.bpmn_process_id;
      p.version = (int32_t)dv.version;
      p.wkey = dv.workflow_key;
      d.elem = resolve_process(e, p.pid, p.version, p.wkey);
      d.key = -1;
    } else if (wf_cmd) {
      p.scope_cmd = true;
      p.cancel = it == WI_CANCEL;
      p.lookup = p.cancel ? r.key : dv.wik;
      p.inst = p.lookup;
      // (a CANCEL names its instance by the command key; its descriptor carries it for k_conflict -- the
      // command's own value is written verbatim, so the descriptor's instance key is not serialized)
      d.inst_key = p.cancel ? r.key : dv.wik;
      p.canon = reencode(vt, dv, p.doc, p.doc_len);
    } else if (job_cmd) {
      if (it == JI_CREATE && r.key >= 0)
        return fail(e, ZB_EUNSUPPORTED, "record " + std::to_string(i) + ": JOB CREATE with a key (job keys come from "
                                        "the partition's job key generator)");
      p.job_cmd = true;
      p.lookup = dv.aik;
      p.inst = conflict_key(dv.wik, r.key, d.kind);  // (a job without workflow headers: by its job key)
      d.scope_key = dv.aik;
      d.inst_key = dv.wik;
      if (it == JI_UPDATE_RETRIES) d.elem = dv.retries > 0 ? 1 : 0;  // (job_command reads it)
      p.canon = reencode(vt, dv, p.doc, p.doc_len);
    } else if (job_ev) {
      p.lookup = dv.aik;
      p.inst = dv.wik;
      p.aik = dv.aik;
      d.scope_key = dv.aik;  // headers.activityInstanceKey
      d.inst_key = dv.wik;
    } else {  // CORRELATE: key = its log position (positionAsKey)
      p.lookup = dv.aik;
      p.inst = dv.wik;
      p.aik = dv.aik;
      d.key = KEY_IS_POSITION;
      d.scope_key = dv.aik;
      d.inst_key = dv.wik;
      p.canon = reencode(vt, dv, p.doc, p.doc_len);
    }
  }
  // 2. races of one tick (include/zb_engine.h), against what is staged already: records of one workflow instance
  // that a lockstep wave could not process as the reference's processor does -- one after the other, each seeing
  // what the earlier ones did -- make the instance a conflicting one; zb_step then cuts every generation of the
  // tick before the next record of such an instance (k_conflict), which restores that order for it.
  if (!e->staged_pending) { e->tick_inst.clear(); e->tick_aik.clear(); e->tick_jobs.clear(); e->tick_conflicts.clear(); }
  std::unordered_map<int64_t, uint8_t> inst = e->staged_pending ? e->tick_inst : std::unordered_map<int64_t, uint8_t>();
  std::unordered_set<int64_t> aiks = e->staged_pending ? e->tick_aik : std::unordered_set<int64_t>();
  std::unordered_set<int64_t> tick_jobs = e->staged_pending ? e->tick_jobs : std::unordered_set<int64_t>();
  std::unordered_set<int64_t> confl = e->staged_pending ? e->tick_conflicts : std::unordered_set<int64_t>();
  const zb_rec* prev_staged = (e->staged_pending && !e->staged.empty()) ? &e->staged.back() : nullptr;
  for (size_t i = 0; i < n; i++) {
    Prep& p = prep[i];
    if (p.create) continue;
    const zb_rec* prev = i > 0 ? &prep[i - 1].d : prev_staged;
    // JOB CREATED directly followed by its JOB COMPLETED: one batch, processed in order by one thread
    if (recs[i].value_type == ZB_VT_JOB && recs[i].intent == JI_COMPLETED && prev && kind_vt(prev->kind) == ZB_VT_JOB &&
        prev->intent == JI_CREATED && prev->key == recs[i].key && prev->scope_key == p.d.scope_key) {
      p.pair = true;
      p.d.kind |= 0x40;
      continue;
    }
    // a job's commands of one tick: two consecutive ones form one group, processed in order by one thread (a
    // group's records share that thread's MAX_SLOTS (2) output slots); any other repeat is a conflict
    if (p.job_cmd && p.d.key >= 0) {
      if (prev && kind_vt(prev->kind) == ZB_VT_JOB && kind_rt(prev->kind) == ZB_RT_COMMAND && prev->key == p.d.key &&
          !(prev->kind & 0x40) && !confl.count(p.inst)) {
        p.d.kind |= 0x40;
        continue;
      }
      if (!tick_jobs.insert(p.d.key).second) confl.insert(p.inst);
    }
    uint8_t& f = inst[p.inst];
    if ((f & 1) || (p.scope_cmd && f)) confl.insert(p.inst);
    f |= p.scope_cmd ? 1 : 2;
    if (p.aik != INT64_MIN && !aiks.insert(p.aik).second) confl.insert(p.inst);
  }
  // 3. stage
  begin_staging(e);
  e->staged_uploaded = false;
  e->tick_inst.swap(inst);
  e->tick_aik.swap(aiks);
  e->tick_jobs.swap(tick_jobs);
  e->tick_conflicts.swap(confl);
  for (size_t i = 0; i < n; i++) {
    Prep& p = prep[i];
    // arena: [payload document][verbatim value] (+ [document][re-encoded command value])
    p.d.payload = add_blob(e->staged_arena, p.doc, p.doc_len);
    add_blob(e->staged_arena, p.raw, p.raw_len);
    if (!p.canon.empty()) {
      add_blob(e->staged_arena, p.doc, p.doc_len);
      add_blob(e->staged_arena, p.canon.data(), (uint32_t)p.canon.size());
    }
    if (p.create) {
      if (e->staged.empty()) { e->staged_elem = p.d.elem; e->staged_uniform = true; e->staged_max_len = 1; }
      else if (p.d.elem != e->staged_elem) e->staged_uniform = false;
      e->staged_max_len = std::max<uint32_t>(e->staged_max_len, p.doc_len);
      zb_engine::PendingRange pr;
      pr.first = (int64_t)e->staged.size();
      pr.last = pr.first + 1;
      pr.workflow_key = p.wkey;
      pr.version = p.version;
      pr.pid_off = (uint32_t)e->cmd_pool.size();
      pr.pid_len = (uint16_t)p.pid.size();
      e->cmd_pool.insert(e->cmd_pool.end(), p.pid.begin(), p.pid.end());
      e->pending_ranges.push_back(pr);
    } else {
      e->staged_only_creates = false;
      if (p.cancel) e->staged_has_cancel = true;
    }
    e->staged.push_back(p.d);
    e->staged_vlen.push_back(p.raw_len);  // KIND_RAW: the value as written
    e->staged_lookup.push_back(p.lookup == INT64_MIN ? INT64_MIN : p.lookup);
  }
  if (n) e->staged_pending = true;
  return ZB_OK;
}

int zb_step(zb_engine* e, uint32_t max_waves, zb_step_stats* stats) {
  if (!e) return ZB_EINVAL;
  if (e->failed) return fail(e, ZB_EPROCESSING, "partition stopped after a processing failure: " + e->err);
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  auto t0 = std::chrono::steady_clock::now();
#ifdef ZB_PHASES  // (measurement build: host time per part of the step, waits at its round trips included)
  auto sp0 = t0;
  double sp[6] = {0};
#define ZB_SP(k) do { auto n_ = std::chrono::steady_clock::now(); \
    sp[k] += std::chrono::duration<double, std::milli>(n_ - sp0).count(); sp0 = n_; } while (0)
#else
#define ZB_SP(k) do { } while (0)
#endif
  zb_step_stats st{};
  bool try_traj = false;
  {
    int mrc = settle_deferred(e);  // (a new trajectory run reuses the deferred batch's buffers)
    if (mrc != ZB_OK) return mrc;
    mrc = maintain(e, false);  // released records leave the window; compaction when a region is half full
    if (mrc != ZB_OK) return mrc;
  }
  ZB_SP(0);  // settle / maintain (compaction)
  const int64_t rows_before = e->host_hdr.rows_next, arena_before = e->host_hdr.arena_next;
  const int64_t end_before = e->host_hdr.end;  // records appended by this call: injected input + follow-ups
  int64_t traj_base = 0, traj_n = 0;
  const int hint_key = (e->staged_pending && !e->staged.empty()) ? (e->staged_only_creates ? 1 : 2) : 3;
  const bool injecting = e->staged_pending && !e->staged.empty();
  if (!injecting && e->host_hdr.begin == e->host_hdr.end) {  // nothing to process: no kernel, no round trip
    st.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (stats) *stats = st;
    e->term = false;
    e->conf_active = false;
    return ZB_OK;
  }
  e->ob_counts_valid = false;  // (the waves below may write the outbox)
  // ---- inject staged input at the log tail (engine is quiescent between steps)
  if (injecting) {
    if (!e->staged_only_creates && e->host_hdr.begin != e->host_hdr.end)
      return fail(e, ZB_EINVAL, "records other than CREATE are injected into a quiescent partition only: "
                                "step it to quiescence first");
    // an idle partition fed only CREATE commands runs as independent trajectories (zb_traj.hip) -- no parallel
    // gateways, and either the canonical job harness or no service task in any deployed model: the workflow
    // processor writes the same records for a CREATE whichever job processor shares the log
    // (WorkflowInstanceStreamProcessor.java:233-368; JobInstanceStreamProcessor is a separate registration,
    // JobInstanceStreamProcessor.java:77-83), so a model without service tasks never meets the job mode
    // (the general wave pipeline covers everything else)
    const bool job_mode_ok = !(e->cfg.flags & (ZB_CFG_EXTERNAL_JOBS | ZB_CFG_JOB_PROCESSOR)) || !e->has_tasks;
    try_traj = !(e->cfg.flags & ZB_CFG_WAVE_ONLY) && job_mode_ok && max_waves == 0 &&
               e->staged_only_creates && !e->has_parallel && !e->has_io &&
               (e->traj_model_ok || (e->cls_ok && e->staged_uniform)) &&
               e->host_hdr.begin == e->host_hdr.end;
    traj_base = e->host_hdr.end;
    traj_n = (int64_t)e->staged.size();
    const int64_t n = (int64_t)e->staged.size();
    if ((uint64_t)(e->host_hdr.end + n - e->win_base) > e->cfg.log_capacity)
      return fail(e, ZB_ENOMEM, "log capacity (release drained records with zb_log_release)");
    {
      const int urc = upload_staged(e);  // (already done by zb_upload_staged, or by an earlier step of a kept batch)
      if (urc != ZB_OK) return urc;
    }
    if (!e->staged_in_place && (uint64_t)e->host_hdr.arena_next + e->staged_arena.size() > e->arena_top)
      return fail(e, ZB_ENOMEM, "arena capacity");
    InjectParams ip;
    ip.log = e->log;
    ip.links = e->links;
    ip.srcd = e->srcd;
    ip.vlen = e->vlen;
    ip.staged_vlen = e->d_staged_vlen.p;
    ip.arena = e->arena;
    ip.staged = e->d_staged.p;
    ip.staged_arena = e->d_staged_arena.p;
    ip.n = n;
    ip.log_base = e->host_hdr.end;
    // documents in place: only the refs are rebased (the batch's documents are referenced where they lie)
    ip.arena_base = e->staged_in_place ? e->staged_base : (uint64_t)e->host_hdr.arena_next;
    ip.staged_bytes = e->staged_in_place ? 0 : e->staged_arena.size();
    if ((uint64_t)n > e->cref_cap) {
      if (e->d_cref) (void)hipFree(e->d_cref);
      e->d_cref = nullptr;
      e->cref_cap = 0;
      HIPCHECK(e, hipMalloc(&e->d_cref, (uint64_t)n * sizeof(uint32_t)));
      e->cref_cap = (uint64_t)n;
    }
    ip.cref = e->d_cref;
    e->cref_base = ip.log_base;
    // a batch headed for the class path (run_trajectory: classify, then trace the classes) is injected by the
    // classification kernel itself, one thread per CREATE (k_cls_classify<.., true>); anything else by k_inject
    const bool fuse = try_traj && e->traj_skip == 0 && e->has_splits && e->staged_uniform && e->cls_ok &&
                      ip.staged_bytes == 0 && e->staged_nlook == 0;
    if (fuse) {
      e->inject_ip = ip;
      e->inject_deferred = true;
    } else {
      launch_inject(ip, e->stream);
    }
    // records naming an element instance by key: its row (ElementInstanceIndex.getInstance); the (key, index)
    // pairs were uploaded with the batch and are sorted here, on the device
    if (e->staged_nlook) {
      const uint64_t m = e->staged_nlook;
      if (m > (uint64_t)INT32_MAX) return fail(e, ZB_EUNSUPPORTED, "more than 2^31 staged lookups");
      if (m > e->look_cap) {
        HIPCHECK(e, hipStreamSynchronize(e->stream));
        if (e->look_keys) (void)hipFree(e->look_keys);
        if (e->look_idx) (void)hipFree(e->look_idx);
        e->look_keys = e->look_idx = nullptr;
        e->look_cap = 0;
        const uint64_t c = std::max<uint64_t>(m + m / 4, 1024);
        HIPCHECK(e, hipMalloc(&e->look_keys, c * sizeof(int64_t)));
        HIPCHECK(e, hipMalloc(&e->look_idx, c * sizeof(int64_t)));
        e->look_cap = c;
      }
      e->h_stats_pinned[17] = e->staged_lookup_spread;  // (computed on the host by upload_staged)
      int rc = sort_pairs(e, (const int64_t*)e->d_lookup_keys.p, e->look_keys, (const int64_t*)e->d_lookup_pos.p,
                          e->look_idx, m, "lookup", true);
      if (rc != ZB_OK) return rc;
      ResolveParams rp{};
      rp.rmeta = e->rmeta; rp.rkeys = e->rkeys; rp.rows = (uint64_t)e->host_hdr.rows_next;
      rp.keys = e->look_keys; rp.pos = e->look_idx; rp.pos_base = ip.log_base; rp.n = (int64_t)m;
      rp.links = e->links;
      launch_resolve(rp, e->stream);
    }
    if (e->staged_has_cancel) e->term = true;
    if (e->staged_conf) e->conf_active = true;  // (until the tick is quiescent)
    {
      const int qrc = append_requests(e, ip.log_base);
      if (qrc != ZB_OK) return qrc;
    }
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
    if (e->staged_in_place) e->arena_total += e->staged_arena.size();  // (allocated at the top, not by arena_next)
    else e->host_hdr.arena_next += (int64_t)e->staged_arena.size();
    HIPCHECK(e, upload_async(e, e->hdr + (e->wave & 1), &e->host_hdr, sizeof(WaveHdr)));
    e->staged_pending = false;
  }
  ZB_SP(1);  // inject, lookups
  const int64_t processed_from = e->host_hdr.begin;
  const int64_t written_from = e->host_hdr.end;
  // counters before / after the step: stream-ordered copies into pinned memory, read after the step's last sync
  uint64_t* stats_before = e->h_stats_pinned;
  uint64_t* stats_after = e->h_stats_pinned + 8;
  HIPCHECK(e, hipMemcpyAsync(stats_before, e->dstats, 8 * sizeof(uint64_t), hipMemcpyDeviceToHost, e->stream));
  uint32_t launched = 0;
  bool quiescent = e->host_hdr.begin == e->host_hdr.end;
  // A batch the trajectory path falls back from (a message subscription, a termination, ... on some instance's
  // path) costs a class attempt and a per-instance attempt before the wave pipeline runs it (C5: ~0.35 ms of a
  // 6.6 ms step); after a fallback the next TRAJ_RETRY batches of the model go straight to the wave pipeline.
  if (try_traj && e->traj_skip > 0) {
    e->traj_skip--;
    try_traj = false;
  }
  e->traj_stats_fresh = false;
  if (try_traj && !quiescent) {
    int rc = run_trajectory(e, traj_base, traj_n, st, true);
    if (e->inject_deferred) {  // (run_trajectory returned before its classification: inject here, stream-ordered)
      e->inject_deferred = false;
      launch_inject(e->inject_ip, e->stream);
    }
    if (rc < 0) return rc;
    if (rc == 0) e->traj_skip = TRAJ_RETRY;
    quiescent = e->host_hdr.begin == e->host_hdr.end;
  }
  if (e->inject_deferred) {  // (not reached in practice: the fuse condition implies the trajectory run above)
    e->inject_deferred = false;
    launch_inject(e->inject_ip, e->stream);
  }
  ZB_SP(2);  // trajectory
  // the first batch: as many waves as the last wave loop over the same kind of input had (a tick of the same workload
  // settles in as many waves, and each launch past quiescence costs ~20 us of empty kernels), else WAVES_PER_SYNC
  const bool loop = !quiescent && (max_waves == 0 || launched < max_waves);
  bool stats_fresh = quiescent && e->traj_stats_fresh;  // (the trajectory run read the counters back at its end)
  if (loop) HIPCHECK(e, hipMemcpyAsync(e->h_stats_pinned + 18, e->dstats + 6, sizeof(uint64_t), hipMemcpyDeviceToHost,
                                       e->stream));  // (the waves counter before the loop)
  // batches follow the hint until it is used up (C2: 148 waves as 64 + 64 + 20, not 64 + 16 + 32 + 64 with 28 empty
  // waves), then -- the tick needs a few more -- 4, doubling; without a hint WAVES_PER_SYNC, doubling
  const int hint = e->wave_hint[hint_key];
  int next_batch = hint > 0 ? std::min<int>(hint, WAVES_PER_SYNC_MAX) : WAVES_PER_SYNC;
  int grow = hint > 0 ? 4 : WAVES_PER_SYNC;
  while (!quiescent && (max_waves == 0 || launched < max_waves)) {
    int batch = next_batch;
    if (max_waves) batch = std::min<int>(batch, (int)(max_waves - launched));
    // timing events cost ~5 us of stream time each between kernels (C2: 4 per wave = 2.9 ms of a 41 ms
    // step): per wave only with ZB_CFG_WAVE_EVENTS (process / emit / aux split), else one pair per batch
    const bool per_wave = e->wave_events;
    if (!per_wave) HIPCHECK(e, hipEventRecord(e->ev[0], e->stream));
    for (int i = 0; i < batch; i++) {
      WaveParams p = wave_params(e);
      hipEvent_t* ev = &e->ev[EV_PER_WAVE * i];
      if (per_wave) HIPCHECK(e, hipEventRecord(ev[0], e->stream));
      if (p.conflicts) {  // the chunk ends before the next record of a conflicting instance
        HIPCHECK(e, hipMemsetAsync(e->conf_first, 0x7f, (e->conf_mask + 1) * sizeof(int64_t), e->stream));
        HIPCHECK(e, hipMemsetAsync(p.conf_split, 0x7f, sizeof(int64_t), e->stream));
        launch_conflict(p, e->stream);
      }
      if (p.has_parallel || p.term) launch_pre(p, e->stream);  // scope-wide counters / first live children
      if (e->has_io) launch_map(p, e->stream);  // io-mapping results of the chunk's records
      if (e->wave_fused_grid) {  // process + scan + emit in one launch (k_wave)
        // tile aggregates carry an 8-bit tag: when it wraps, no granule may hold a tag of an earlier launch
        if (e->lb_seq % 255 == 0 && e->lb_seq)
          HIPCHECK(e, hipMemsetAsync(e->lookback, 0, 2 * e->lb_tiles * sizeof(uint64_t), e->stream));
        p.lb_tag8 = (uint32_t)(1 + e->lb_seq % 255);
        uint32_t* const claims = (uint32_t*)(e->lookback + 2 * e->lb_tiles + 8 * (e->lb_tiles + 512) + 8 * (e->lb_tiles + 2));
        const bool shared = (e->cfg.flags & ZB_CFG_SHARED_GPU) != 0;
        p.tile_claim = shared ? claims + (e->lb_seq & 1) : nullptr;
        p.tile_claim_next = shared ? claims + ((e->lb_seq + 1) & 1) : nullptr;
        e->lb_seq++;
        launch_wave(p, e->wave_fused_grid, e->stream);
        if (per_wave) HIPCHECK(e, hipEventRecord(ev[1], e->stream));
        if (per_wave) HIPCHECK(e, hipEventRecord(ev[2], e->stream));
      } else {
        launch_process(p, e->stream);
        if (per_wave) HIPCHECK(e, hipEventRecord(ev[1], e->stream));
        launch_scan(p, e->stream);
        launch_emit(p, e->stream);
        if (per_wave) HIPCHECK(e, hipEventRecord(ev[2], e->stream));
      }
      // payload kernels for this wave's deferred work (only when the model can produce any)
      if (e->has_catch) launch_subscribe(p, e->stream);  // this wave's subscribe steps (outbox)
      if (e->has_merges) launch_merge(p, e->stream);
      if (e->has_splits) launch_cond(p, e->stream);
      if (per_wave) HIPCHECK(e, hipEventRecord(ev[3], e->stream));
      e->wave++;
      e->epoch++;
    }
    if (e->wave_fused_grid) launch_stat_fold(e->dstats, e->stream);  // k_wave's statistics banks -> the counters
    if (!per_wave) HIPCHECK(e, hipEventRecord(e->ev[1], e->stream));
    HIPCHECK(e, hipGetLastError());
    {
      StatusReads r;
      r.add(e->h_hdr_pinned, e->hdr + (e->wave & 1), sizeof(WaveHdr));
      r.add(e->h_err_pinned, e->derr, sizeof(uint32_t));
      // (the counters too: after the batch that ends the loop they need no round trip of their own)
      r.add(stats_after, e->dstats, 8 * sizeof(uint64_t));
      // (and the outbox counters: the exchange decision after a quiescent step needs no round trip of its own)
      if (e->on) r.add(e->h_stats_pinned + 19, e->on, 4 * sizeof(uint32_t));
      HIPCHECK(e, r.launch(e->stream));
    }
    HIPCHECK(e, hipStreamSynchronize(e->stream));
    e->ob_counts_valid = e->on != nullptr;
    stats_fresh = true;
    if (per_wave) {
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
    } else {  // the batch as a whole (kernel boundaries included), reported as the process share
      float ms = 0;
      HIPCHECK(e, hipEventElapsedTime(&ms, e->ev[0], e->ev[1]));
      st.process_kernel_ms += ms;
      st.wave_kernel_ms += ms;
    }
    launched += batch;
    st.launches += batch;
    if (hint > (int)launched) {
      next_batch = std::min<int>(hint - (int)launched, WAVES_PER_SYNC_MAX);
    } else {
      next_batch = grow;
      grow = std::min(2 * grow, WAVES_PER_SYNC_MAX);
    }
    e->host_hdr = e->h_hdr_pinned[0];
    int rc = check_device_errors(e, *e->h_err_pinned);
    if (rc != ZB_OK) return rc;
    quiescent = e->host_hdr.begin == e->host_hdr.end;
  }
  ZB_SP(3);  // wave loop
  if (!stats_fresh) {
    StatusReads r;
    r.add(stats_after, e->dstats, 8 * sizeof(uint64_t));
    if (e->on) r.add(e->h_stats_pinned + 19, e->on, 4 * sizeof(uint32_t));
    HIPCHECK(e, r.launch(e->stream));
    HIPCHECK(e, hipStreamSynchronize(e->stream));
    e->ob_counts_valid = e->on != nullptr;
  }
  if (loop && quiescent) e->wave_hint[hint_key] = (int)(stats_after[6] - e->h_stats_pinned[18]);  // its non-empty waves
  st.records_processed = (uint64_t)(e->host_hdr.begin - processed_from);
  st.records_written = (uint64_t)(e->host_hdr.end - written_from);
  st.transitions = stats_after[0] - stats_before[0];
  st.completed_instances = stats_after[1] - stats_before[1];
  st.merges = stats_after[3] - stats_before[3];
  st.merge_bytes = stats_after[4] - stats_before[4];
  st.condition_payload_bytes = stats_after[5] - stats_before[5];
  st.waves = stats_after[6] - stats_before[6];
  e->rows_total += (uint64_t)std::max<int64_t>(0, e->host_hdr.rows_next - rows_before);
  e->arena_total += (uint64_t)std::max<int64_t>(0, e->host_hdr.arena_next - arena_before);
  e->records_total += (uint64_t)(e->host_hdr.end - end_before);
  st.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  ZB_SP(4);  // tail
#ifdef ZB_PHASES
  if (launched) fprintf(stderr, "step ms: maintain %.3f inject %.3f traj %.3f waves %.3f tail %.3f (%u launches)\n",
                        sp[0], sp[1], sp[2], sp[3], sp[4], launched);
#endif
#undef ZB_SP
  if (stats) *stats = st;
  if (!quiescent) return ZB_EAGAIN;
  e->term = false;  // every termination chain has ended
  e->conf_active = false;
  return ZB_OK;
}

int64_t zb_log_size(zb_engine* e) { return e ? e->host_hdr.end : -1; }

int zb_read_source_positions(zb_engine* e, int64_t start, int64_t count, int64_t* out) {
  if (!e || start < e->win_base || count < 0 || start + count > e->host_hdr.end || (!out && count)) return ZB_EINVAL;
  if (count == 0) return ZB_OK;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  int rc = materialize(e);
  if (rc != ZB_OK) return rc;
  std::vector<uint32_t> d((size_t)count);
  HIPCHECK(e, hipMemcpyAsync(d.data(), e->srcd + start, count * sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  for (int64_t i = 0; i < count; i++) out[i] = d[(size_t)i] ? start + i - (int64_t)d[(size_t)i] : -1;
  return ZB_OK;
}

int zb_read_descriptors(zb_engine* e, int64_t start, int64_t count, zb_rec* out) {
  if (!e || start < e->win_base || count < 0 || start + count > e->host_hdr.end || (!out && count)) return ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  int rc = materialize(e);
  if (rc != ZB_OK) return rc;
  HIPCHECK(e, hipMemcpyAsync(out, e->log + start, count * sizeof(zb_rec), hipMemcpyDeviceToHost, e->stream));
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  return ZB_OK;
}

static int serialize(zb_engine* e, int64_t start, int64_t count, const zb_frame_config* fc, zb_serialize_stats* stats);

int zb_serialize(zb_engine* e, int64_t start, int64_t count, zb_serialize_stats* stats) {
  return serialize(e, start, count, nullptr, stats);
}

int zb_serialize_frames(zb_engine* e, int64_t start, int64_t count, const zb_frame_config* fc,
                        zb_serialize_stats* stats) {
  if (!fc) return ZB_EINVAL;
  return serialize(e, start, count, fc, stats);
}

int zb_set_request_metadata(zb_engine* e, size_t n, const uint64_t* request_ids, const int32_t* request_stream_ids) {
  if (!e || (n && (!request_ids || !request_stream_ids))) return ZB_EINVAL;
  // only records staged since the last injection (e->staged holds them while staged_pending): after zb_step the
  // indices would name records of the batch already in the log
  if (n && !e->staged_pending) return fail(e, ZB_EINVAL, "no staged records: request metadata goes with zb_submit*");
  if (n > e->staged.size()) return fail(e, ZB_EINVAL, "more request metadata than staged records");
  const int64_t first = (int64_t)(e->staged.size() - n);
  // (staged indices only grow between injections: the list stays sorted unless a range is set twice)
  for (size_t i = 0; i < n; i++) {
    const int64_t idx = first + (int64_t)i;
    if (!e->staged_reqs.empty() && e->staged_reqs.back().idx >= idx)
      return fail(e, ZB_EINVAL, "request metadata already set for these records");
    e->staged_reqs.push_back(zb_engine::StagedReq{idx, request_ids[i], request_stream_ids[i], 0});
    e->staged_reqs_uploaded = false;
  }
  return ZB_OK;
}

// zb_serialize of exactly a deferred template batch: k_tdrain_size -> scan -> k_tdrain_write (zb_tdrain.hip).
// ZB_EAGAIN: the batch needs the descriptor path (an instance's records exceed the wave image, or a value length
// disagreed with the encoder -- never silently).
static int serialize_deferred(zb_engine* e, int64_t start, int64_t count, const zb_frame_config* fc,
                              zb_serialize_stats& st) {
  const TrajParams& p = e->seg_p;
  const uint64_t nwave = (uint64_t)p.nwg * (TRAJ_WG / 64);
  const uint64_t ent = (uint64_t)e->seg_wmax * nwave + 1;
  if (ent > (uint64_t)INT32_MAX) return ZB_EAGAIN;
  if (ent > e->td_cap) {
    if (e->td_wbytes) (void)hipFree(e->td_wbytes);
    if (e->td_woffs) (void)hipFree(e->td_woffs);
    if (e->td_tmp) (void)hipFree(e->td_tmp);
    e->td_wbytes = nullptr; e->td_woffs = nullptr; e->td_tmp = nullptr; e->td_cap = 0;
    const uint64_t cap = ent + ent / 4 + 1024;
    HIPCHECK(e, hipMalloc(&e->td_wbytes, cap * sizeof(uint64_t)));
    HIPCHECK(e, hipMalloc(&e->td_woffs, cap * sizeof(uint64_t)));
    size_t tmp = 0;
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, e->td_wbytes, e->td_woffs, (int)cap, e->stream) != hipSuccess)
      return fail(e, ZB_EDEVICE, "template drain scan sizing");
    HIPCHECK(e, hipMalloc(&e->td_tmp, tmp + 16));
    e->td_tmp_cap = tmp;
    e->td_cap = cap;
  }
  if ((uint64_t)p.nwg > e->td_pay_cap) {
    if (e->td_pay) (void)hipFree(e->td_pay);
    e->td_pay = nullptr;
    HIPCHECK(e, hipMalloc(&e->td_pay, (uint64_t)p.nwg * sizeof(uint64_t)));
    e->td_pay_cap = (uint64_t)p.nwg;
  }
  if (!e->td_flags) HIPCHECK(e, hipMalloc(&e->td_flags, 4 * sizeof(uint32_t)));
  TDrainParams d{};
  d.t = p;
  d.headers = e->dr_hdr;
  d.start = start;
  d.wmax = e->seg_wmax;
  d.nwave = (uint32_t)nwave;
  d.wbytes = e->td_wbytes;
  d.woffs = e->td_woffs;
  d.pay_part = e->td_pay;
  d.totals = e->dr_total;
  d.flags = e->td_flags;
  d.vsegs = e->d_vsegs.p;
  d.segpool = e->d_segpool.p;
  d.segpool_len = e->segpool_len;
  d.n_elems = (int32_t)e->model.elems.size();
  d.nc = e->seg_nc;
  d.len5_ok = e->seg_key_end <= (int64_t)UINT32_MAX ? 1u : 0u;
  d.jobs = e->seg_jobs ? 1u : 0u;
#ifdef ZB_PHASES
  d.phase = e->phase ? e->phase + 8 : nullptr;
#endif
  if (fc) {  // log frames: no headers; the request metadata of the batch's CREATE commands [log_base, log_base + n)
    d.frames = 1;
    d.stream_id = fc->stream_id;
    d.raft_term = fc->raft_term;
    d.timestamp = fc->timestamp;
    for (const auto& r : e->req_runs)  // the batch's own run covers every CREATE: entry i is instance i's
      if (r.first == p.log_base && r.last == p.log_base + p.n - 1 && (int64_t)r.n == p.n) {
        d.reqs = e->d_req + r.lo;
        d.nreqs = p.n;
        d.req_dense = 1;
      }
    if (!d.req_dense && e->req_n > e->req_lo) {  // otherwise a search of the whole table
      d.reqs = e->d_req + e->req_lo;
      d.nreqs = (int64_t)(e->req_n - e->req_lo);
    }
  }
  float ms_size = 0, ms_scan = 0, ms_write = 0;
  for (int attempt = 0; attempt < 2; attempt++) {
    d.out = e->dr_val;
    d.out_cap = e->dr_val_cap;
    HIPCHECK(e, hipMemsetAsync(e->dr_total, 0, 4 * sizeof(uint64_t), e->stream));
    HIPCHECK(e, hipMemsetAsync(e->td_flags, 0, 4 * sizeof(uint32_t), e->stream));
    HIPCHECK(e, hipMemsetAsync(e->td_wbytes + (ent - 1), 0, sizeof(uint64_t), e->stream));
    HIPCHECK(e, hipEventRecord(e->dr_ev[0], e->stream));
    // a class batch without job keys: the workgroups whose every key encodes in 5 bytes get their sizes from the
    // per-wave class counts and CREATE payload sums (k_tdrain_sizes); the first ones (keys / positions below 2^16)
    // resolve every record (k_tdrain_size)
    uint32_t wg0 = (uint32_t)p.nwg;
    if (p.cls && !d.jobs && d.len5_ok && !d.frames) {  // (frame padding is not linear in the payload lengths)
      const int64_t thr = std::max<int64_t>(65536 - p.log_base, (65536 - p.wf_start + 4) / 5);
      wg0 = (uint32_t)std::min<int64_t>(p.nwg, (std::max<int64_t>(thr, 0) + TRAJ_WG - 1) / TRAJ_WG);
    }
    launch_tdrain_size(d, wg0, e->stream);
    HIPCHECK(e, hipEventRecord(e->dr_ev[1], e->stream));
    size_t tmp = e->td_tmp_cap;
    if (hipcub::DeviceScan::ExclusiveSum(e->td_tmp, tmp, e->td_wbytes, e->td_woffs, (int)ent, e->stream) != hipSuccess)
      return fail(e, ZB_EDEVICE, "template drain scan");
    HIPCHECK(e, hipMemcpyAsync(e->dr_total, e->td_woffs + (ent - 1), sizeof(uint64_t), hipMemcpyDeviceToDevice, e->stream));
    HIPCHECK(e, hipEventRecord(e->dr_ev[2], e->stream));
    launch_tdrain_write(d, e->stream);
    HIPCHECK(e, hipEventRecord(e->dr_ev[3], e->stream));
    HIPCHECK(e, hipGetLastError());
    HIPCHECK(e, hipMemcpyAsync(e->h_dr_total, e->dr_total, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, e->stream));
    HIPCHECK(e, hipMemcpyAsync(e->h_dr_total + 2, e->td_flags, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
    HIPCHECK(e, hipStreamSynchronize(e->stream));
    const uint32_t* fl = (const uint32_t*)(e->h_dr_total + 2);
    if (fl[1]) return ZB_EAGAIN;
    if (!fl[0]) break;
    if (attempt == 1) return fail(e, ZB_EDEVICE, "drain buffer overflow after growing it");
    (void)hipFree(e->dr_val);
    e->dr_val = nullptr;
    e->dr_val_cap = 0;
    const uint64_t cap = e->h_dr_total[0] + e->h_dr_total[0] / 4 + (64ull << 20);
    HIPCHECK(e, hipMalloc(&e->dr_val, cap));
    e->dr_val_cap = cap;
  }
  HIPCHECK(e, hipEventElapsedTime(&ms_size, e->dr_ev[0], e->dr_ev[1]));
  HIPCHECK(e, hipEventElapsedTime(&ms_scan, e->dr_ev[1], e->dr_ev[2]));
  HIPCHECK(e, hipEventElapsedTime(&ms_write, e->dr_ev[2], e->dr_ev[3]));
  st.records = (uint64_t)count;
  st.value_bytes = e->h_dr_total[0];
  st.payload_bytes = e->h_dr_total[1];
  st.size_kernel_ms = ms_size;
  st.scan_ms = ms_scan;
  st.write_kernel_ms = ms_write;
  st.generic_tiles = 0;
  st.template_drain = 1;
  e->dr_slow_tiles = 0;
  e->dr_split = false;
  return ZB_OK;
}

static int serialize(zb_engine* e, int64_t start, int64_t count, const zb_frame_config* fc, zb_serialize_stats* stats) {
  if (!e || start < e->win_base || count < 0 || start + count > e->host_hdr.end) return ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  auto t0 = std::chrono::steady_clock::now();
  zb_serialize_stats st{};
  e->dr_count = 0;
  e->dr_bytes = 0;
  if (count == 0) {
    if (stats) *stats = st;
    return ZB_OK;
  }
  if (!e->dr_ev[0])
    for (auto& x : e->dr_ev) HIPCHECK(e, hipEventCreate(&x));
  if (!e->dr_total) {
    HIPCHECK(e, hipMalloc(&e->dr_total, 4 * sizeof(uint64_t)));  // [0] bytes [1] payload bytes [2] ctr|overflow
    HIPCHECK(e, hipHostMalloc(&e->h_dr_total, 4 * sizeof(uint64_t)));
  }
  if ((uint64_t)count > e->dr_cap) {
    void* ps[] = {e->dr_len, e->dr_off, e->dr_hdr, e->dr_tmp, e->dr_tiles, e->dr_pay, e->dr_tsum, e->dr_list, e->dr_list2};
    for (void* q : ps)
      if (q) (void)hipFree(q);
    e->dr_off = e->dr_tiles = e->dr_pay = e->dr_tsum = nullptr; e->dr_len = e->dr_list = e->dr_list2 = nullptr;
    e->dr_hdr = nullptr;
    e->dr_tmp = nullptr;
    e->dr_cap = e->dr_tmp_cap = 0;
    const uint64_t cap = (uint64_t)count + (uint64_t)count / 4 + 1024;
    if (cap + 1 > (uint64_t)INT32_MAX) return fail(e, ZB_EUNSUPPORTED, "more than 2^31 records in one drain");
    HIPCHECK(e, hipMalloc(&e->dr_hdr, cap * sizeof(zb_record_header)));
    HIPCHECK(e, hipMalloc(&e->dr_tiles, (cap / 256 + 2) * sizeof(uint64_t)));  // single pass: tile states
    HIPCHECK(e, hipMalloc(&e->dr_pay, (cap / 256 + 2) * sizeof(uint64_t)));    // payload bytes per tile
    HIPCHECK(e, hipMemset(e->dr_tiles, 0, (cap / 256 + 2) * sizeof(uint64_t)));
    // two passes: value lengths (u32 per record) and byte totals per 256-record tile -> tile offsets
    HIPCHECK(e, hipMalloc(&e->dr_len, cap * sizeof(uint32_t)));
    HIPCHECK(e, hipMalloc(&e->dr_tsum, (cap / 256 + 2) * sizeof(uint64_t)));
    HIPCHECK(e, hipMalloc(&e->dr_off, (cap / 256 + 2) * sizeof(uint64_t)));
    HIPCHECK(e, hipMalloc(&e->dr_list, (cap / 256 + 2) * sizeof(uint32_t)));
    HIPCHECK(e, hipMalloc(&e->dr_list2, (cap / 256 + 2) * sizeof(uint32_t)));
    size_t tmp = 0;
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, e->dr_tsum, e->dr_off, (int)(cap / 256 + 2), e->stream) != hipSuccess)
      return fail(e, ZB_EDEVICE, "scan sizing");
    HIPCHECK(e, hipMalloc(&e->dr_tmp, tmp + 16));
    e->dr_tmp_cap = tmp;
    e->dr_cap = cap;
  }
  if (e->dr_val_cap == 0) {  // first estimate; grown from the exact total if it overflows
    const uint64_t cap = (uint64_t)count * 200 + (64ull << 20);
    HIPCHECK(e, hipMalloc(&e->dr_val, cap));
    e->dr_val_cap = cap;
  }
  if (e->seg_pending) {  // a deferred template batch: encoded from its traces, or materialized first
    if (start == e->seg_begin && count == e->seg_end - e->seg_begin) {
      const int rc = serialize_deferred(e, start, count, fc, st);
      if (rc == ZB_OK) {
        e->dr_count = count;
        e->dr_bytes = st.value_bytes;
        e->dr_frames = fc != nullptr;
        st.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (stats) *stats = st;
        return ZB_OK;
      }
      if (rc != ZB_EAGAIN) return rc;
      st = zb_serialize_stats{};
    }
    const int rc = materialize(e);
    if (rc != ZB_OK) return rc;
  }
  HIPCHECK(e, upload_vec(e, e->d_ranges, e->ranges));
  HIPCHECK(e, upload_vec(e, e->d_cmd_pool, e->cmd_pool));
  SerParams sp{};
  sp.nt = 1;
  if (fc) {
    sp.frames = 1;
    sp.stream_id = fc->stream_id;
    sp.raft_term = fc->raft_term;
    sp.timestamp = fc->timestamp;
    sp.log_begin = e->win_base;
    sp.log_end = e->host_hdr.end;
    sp.reqs = e->req_n > e->req_lo ? e->d_req + e->req_lo : nullptr;
    sp.nreqs = (int64_t)(e->req_n - e->req_lo);
  }
  sp.log = e->log;
  sp.srcd = e->srcd;
  sp.vlen = e->vlen;
  sp.vlen_bad = e->vlen_bad;
  sp.arena = e->arena;
  sp.arena_bytes = e->cfg.arena_bytes;
  sp.vconst = e->d_vconst.p;
  sp.vsegs = e->d_vsegs.p;
  sp.segpool = e->d_segpool.p;
  sp.segpool_len = e->segpool_len;
  sp.seg_lds = e->seg_ok ? 1 : 0;
  sp.elems = e->d_elems.p;
  sp.wfs = e->d_wfs.p;
  sp.queries = e->d_queries.p;
  sp.pool = e->d_pool.p;
  sp.ranges = e->d_ranges.p;
  sp.nranges = (int32_t)e->ranges.size();
  sp.cmd_pool = e->d_cmd_pool.p;
  sp.start = start;
  sp.count = count;
  sp.totals = e->dr_total;
  sp.tile_state = e->dr_tiles;
  sp.pay_part = e->dr_pay;
  sp.n_elems = (int32_t)e->model.elems.size();
  sp.n_wfs = (int32_t)e->model.workflows.size();
  sp.pool_len = (uint32_t)e->model.pool.size();
  {
    const uint64_t need = ((sp.n_elems * sizeof(DevElem) + 15) & ~15ull) + ((sp.n_wfs * sizeof(DevWorkflow) + 15) & ~15ull) +
                          sp.pool_len;
    sp.model_lds = (need <= 4096 && e->d_elems.p && e->d_wfs.p && e->d_pool.p) ? 1 : 0;
  }
  sp.tile_ctr = (uint32_t*)(e->dr_total + 2);
  sp.overflow = (uint32_t*)(e->dr_total + 2) + 1;
  sp.headers = e->dr_hdr;
  float ms_size = 0, ms_scan = 0, ms_write = 0;
  for (int attempt = 0; attempt < 2; attempt++) {
    sp.out = e->dr_val;
    sp.out_cap = e->dr_val_cap;
    HIPCHECK(e, hipMemsetAsync(e->dr_total, 0, 4 * sizeof(uint64_t), e->stream));
    e->dr_split = false;
    if (e->ser_mode == 1 && !fc) {  // one pass: decoupled look-back over 256-record tiles (values only)
      if ((++e->dr_epoch & 0x3ffff) == 0) {  // tile-state tags wrap: clear them once
        HIPCHECK(e, hipMemsetAsync(e->dr_tiles, 0, (e->dr_cap / 256 + 2) * sizeof(uint64_t), e->stream));
        ++e->dr_epoch;
      }
      sp.epoch = (uint32_t)e->dr_epoch;
      HIPCHECK(e, hipEventRecord(e->dr_ev[0], e->stream));
      HIPCHECK(e, hipEventRecord(e->dr_ev[1], e->stream));
      HIPCHECK(e, hipEventRecord(e->dr_ev[2], e->stream));
      launch_ser_fused(sp, e->stream);
      HIPCHECK(e, hipEventRecord(e->dr_ev[3], e->stream));
    } else {  // two passes: sizes -> exclusive scan -> write (no host round trip: capacity checked on the device)
      if (e->vlen_bad) HIPCHECK(e, hipMemsetAsync(e->vlen_bad, 0, sizeof(uint32_t), e->stream));
      const int64_t tiles = (count + 255) / 256;
      SerParams sz = sp;
      sz.lengths = e->dr_len;
      // values: lengths in vlen (measured ones filled in); frames: lengths[]
      sz.len_in_vlen = fc ? 0 : 1;
      sz.vlen_out = e->vlen;
      sz.tile_sums = e->dr_tsum;  // tiles + 1 entries, the last one 0: the scan's last output is the total
      HIPCHECK(e, hipEventRecord(e->dr_ev[0], e->stream));
      launch_ser_size(sz, e->stream);
      HIPCHECK(e, hipEventRecord(e->dr_ev[1], e->stream));
      size_t tmp = e->dr_tmp_cap;
      if (hipcub::DeviceScan::ExclusiveSum(e->dr_tmp, tmp, e->dr_tsum, e->dr_off, (int)(tiles + 1), e->stream) != hipSuccess)
        return fail(e, ZB_EDEVICE, "drain scan");
      HIPCHECK(e, hipMemcpyAsync(e->dr_total, e->dr_off + tiles, sizeof(uint64_t), hipMemcpyDeviceToDevice, e->stream));
      HIPCHECK(e, hipEventRecord(e->dr_ev[2], e->stream));
      SerParams wr = sp;
      wr.lengths = e->dr_len;
      wr.len_in_vlen = sz.len_in_vlen;
      wr.tile_offs = e->dr_off;
      e->dr_split = e->ser_fast && sp.seg_lds && sp.arena_bytes;
      if (e->dr_split) {  // k_ser_fast, then k_ser_write over the tiles it left
        // pass 1 over every tile (k_ser_wave, 11 KB per wave) -> list A (a value over its image) and list B (a
        // record kind the fast encoder does not take); pass 2 over A (40 KB phase form) -> more of list B;
        // k_ser_write over B. Frames: k_ser_wave<true> (prefix + value + padding per lane), every tile it leaves
        // (a rejection reason, a kind it does not take, a frame over its image) in list B for k_ser_write<true>
        uint32_t* cnt = (uint32_t*)(e->dr_total + 3);  // [0] list A, [1] list B (zeroed with dr_total)
        wr.tile_list = e->dr_list;
        wr.tile_list_slow = e->dr_list2;
        wr.tile_list_n = cnt;
        launch_ser_fast(wr, e->stream);
        HIPCHECK(e, hipEventRecord(e->dr_ev[4], e->stream));
        HIPCHECK(e, hipMemcpyAsync(e->h_dr_total + 3, e->dr_total + 3, sizeof(uint64_t), hipMemcpyDeviceToHost, e->stream));
        HIPCHECK(e, hipStreamSynchronize(e->stream));
        const uint32_t nA = ((const uint32_t*)(e->h_dr_total + 3))[0];
        uint32_t nB = ((const uint32_t*)(e->h_dr_total + 3))[1];
        HIPCHECK(e, hipEventRecord(e->dr_ev[5], e->stream));  // (the host round trips are not write-pass time)
        const uint32_t nB1 = nB;
        if (nA) {
          SerParams w2 = wr;
          w2.tile_list_in = e->dr_list;
          w2.tile_list = e->dr_list2;  // (appended after pass 1's entries)
          w2.tile_list_n = cnt + 1;
          launch_ser_fast_wide(w2, nA, e->stream);
          HIPCHECK(e, hipMemcpyAsync(e->h_dr_total + 3, e->dr_total + 3, sizeof(uint64_t), hipMemcpyDeviceToHost, e->stream));
          HIPCHECK(e, hipStreamSynchronize(e->stream));
          nB = ((const uint32_t*)(e->h_dr_total + 3))[1];
        }
        if (nB) {
          SerParams w3 = wr;
          w3.tile_list_in = e->dr_list2;
          launch_ser_write_list(w3, nB, e->stream);
        }
        e->dr_slow_tiles = nB;
        e->dr_wide_tiles = nA - (nB - nB1);
        launch_ser_sum(wr, e->stream);
      } else {
        e->dr_slow_tiles = (uint32_t)tiles;
        launch_ser_write(wr, e->stream);
      }
      HIPCHECK(e, hipEventRecord(e->dr_ev[3], e->stream));
    }
    HIPCHECK(e, hipMemcpyAsync(e->h_dr_total, e->dr_total, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, e->stream));
    HIPCHECK(e, hipStreamSynchronize(e->stream));
    HIPCHECK(e, hipGetLastError());
    if (e->vlen_bad) {  // ZB_CFG_VLEN_CHECK: an emitting kernel's value length disagreed with the encoder
      uint32_t bad = 0;
      HIPCHECK(e, hipMemcpy(&bad, e->vlen_bad, sizeof(bad), hipMemcpyDeviceToHost));
      if (bad) return fail(e, ZB_EDEVICE, "value length hint differs from the serialized value (ZB_CFG_VLEN_CHECK)");
    }
    const uint32_t overflow = ((const uint32_t*)(e->h_dr_total + 2))[1];
    if (!overflow) break;
    if (attempt == 1) return fail(e, ZB_EDEVICE, "drain buffer overflow after growing it");
    (void)hipFree(e->dr_val);
    e->dr_val = nullptr;
    e->dr_val_cap = 0;
    const uint64_t cap = e->h_dr_total[0] + e->h_dr_total[0] / 4 + (64ull << 20);
    HIPCHECK(e, hipMalloc(&e->dr_val, cap));
    e->dr_val_cap = cap;
  }
  HIPCHECK(e, hipEventElapsedTime(&ms_size, e->dr_ev[0], e->dr_ev[1]));
  HIPCHECK(e, hipEventElapsedTime(&ms_scan, e->dr_ev[1], e->dr_ev[2]));
  if (e->dr_split) {  // fast pass + generic pass over its leftovers, without the host round trip between them
    float a = 0, b = 0;
    HIPCHECK(e, hipEventElapsedTime(&a, e->dr_ev[2], e->dr_ev[4]));
    HIPCHECK(e, hipEventElapsedTime(&b, e->dr_ev[5], e->dr_ev[3]));
    ms_write = a + b;
  } else {
    HIPCHECK(e, hipEventElapsedTime(&ms_write, e->dr_ev[2], e->dr_ev[3]));
  }
  e->dr_count = count;
  e->dr_bytes = e->h_dr_total[0];
  e->dr_frames = fc != nullptr;
  st.records = (uint64_t)count;
  st.value_bytes = e->h_dr_total[0];
  st.payload_bytes = e->h_dr_total[1];
  st.size_kernel_ms = ms_size;
  st.scan_ms = ms_scan;
  st.write_kernel_ms = ms_write;
  st.generic_tiles = e->ser_mode == 1 && !fc ? 0 : e->dr_slow_tiles;
  st.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (stats) *stats = st;
  return ZB_OK;
}

int zb_drain_copy(zb_engine* e, zb_record_header* headers, uint8_t* values, uint64_t value_off, size_t values_len) {
  if (!e || value_off > e->dr_bytes || values_len > e->dr_bytes - value_off || (values_len && !values)) return ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  if (headers && e->dr_frames) return fail(e, ZB_EINVAL, "the drain batch holds log frames: no headers");
  if (headers && e->dr_count)
    HIPCHECK(e, hipMemcpyAsync(headers, e->dr_hdr, e->dr_count * sizeof(zb_record_header), hipMemcpyDeviceToHost, e->stream));
  if (values_len) HIPCHECK(e, hipMemcpyAsync(values, e->dr_val + value_off, values_len, hipMemcpyDeviceToHost, e->stream));
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  return ZB_OK;
}

void* zb_pinned_alloc(size_t bytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes ? bytes : 1) != hipSuccess) return nullptr;
  return p;
}
void zb_pinned_free(void* p) {
  if (p) (void)hipHostFree(p);
}

int zb_drain(zb_engine* e, int64_t start, int64_t count, zb_record_header* headers, uint8_t* values,
             size_t values_cap, size_t* values_len) {
  zb_serialize_stats st{};
  int rc = zb_serialize(e, start, count, &st);
  if (rc != ZB_OK) return rc;
  if (values_len) *values_len = st.value_bytes;
  if (count == 0) return ZB_OK;
  if (!values || !headers || values_cap < st.value_bytes) return ZB_ENOMEM;
  return zb_drain_copy(e, headers, values, 0, st.value_bytes);
}

// pinned host staging for uploads built on the host (grown on demand; the stream is drained before reuse)
static uint8_t* host_stage(zb_engine* e, size_t bytes) {
  if (hipStreamSynchronize(e->stream) != hipSuccess) return nullptr;
  if (bytes > e->h_stage_cap) {
    if (e->h_stage) (void)hipHostFree(e->h_stage);
    e->h_stage = nullptr;
    e->h_stage_cap = 0;
    const size_t cap = bytes + bytes / 4 + (1 << 20);
    if (hipHostMalloc(&e->h_stage, cap) != hipSuccess) return nullptr;
    e->h_stage_cap = cap;
  }
  return e->h_stage;
}

}  // extern "C"

// ---- the message stream processor and the partition exchange (host side; kernels in zb_msg.hip)
namespace {

// MESSAGE commands ready for the device: descriptors (payload = the message blob's ref relative to the batch's
// blob area; KIND_RAW commands have their verbatim value blob right after it) and the blob area
struct MsgBatch {
  std::vector<zb_rec> recs;
  std::vector<uint8_t> blobs;
  std::vector<uint8_t> prior;  // PUBLISH: an earlier command of the batch has the same (name, ck, id) and ttl > 0
};

// message blob (zb_msg.hpp MsgView): [u32 len][u32 nn][i64 ttl][i64 deadline][u32 nc][u32 np][u32 nid][u32 pad]
// [name][ck][payload][id]
uint32_t add_msg_blob(std::vector<uint8_t>& a, const uint8_t* name, uint32_t nn, const uint8_t* ck, uint32_t nc,
                      int64_t ttl, const uint8_t* pl, uint32_t np, const uint8_t* id, uint32_t nid) {
  const size_t off = a.size();
  const uint32_t len = MSG_HDR - 4 + nn + nc + np + nid;
  a.resize(off + ((4 + (size_t)len + 7) & ~(size_t)7), 0);
  uint8_t* b = a.data() + off;
  const int64_t deadline = 0;  // set when the message is stored
  std::memcpy(b, &len, 4);
  std::memcpy(b + 4, &nn, 4);
  std::memcpy(b + 8, &ttl, 8);
  std::memcpy(b + 16, &deadline, 8);
  std::memcpy(b + 24, &nc, 4);
  std::memcpy(b + 28, &np, 4);
  std::memcpy(b + 32, &nid, 4);
  uint8_t* d = b + MSG_HDR;
  if (nn) std::memcpy(d, name, nn);
  if (nc) std::memcpy(d + nn, ck, nc);
  if (np) std::memcpy(d + nn + nc, pl, np);
  if (nid) std::memcpy(d + nn + nc + np, id, nid);
  return (uint32_t)(off >> 3);
}

MsgParams msg_params(zb_engine* e) {
  MsgParams p{};
  p.log = e->log; p.links = e->links; p.srcd = e->srcd; p.vlen = e->vlen;
  p.arena = e->arena;
  p.hdr = e->hdr + (e->wave & 1);
  p.arena_cap = e->arena_top;  // (the allocators' ceiling: staged documents above it)
  p.subs = e->subs; p.sub_head = e->sub_head; p.sub_next = e->sub_next;
  p.sub_mask = e->head_mask; p.sub_count = e->sub_count; p.sub_cap = e->store_cap;
  p.msgs = e->msgs; p.msg_head = e->msg_head; p.msg_next = e->msg_next;
  p.msg_mask = e->head_mask; p.msg_count = e->msg_count; p.msg_cap = e->store_cap;
  p.ob = outbox(e, ZB_XCHG_CORRELATE);  // the message side sends correlations
  p.err = e->derr;
  p.clock = e->clock_ms;
  return p;
}

// the device header after message-side kernels that allocate blobs with atomics (arena_next)
int pull_header(zb_engine* e) {
  HIPCHECK(e, hipMemcpyAsync(e->h_hdr_pinned, e->hdr + (e->wave & 1), sizeof(WaveHdr), hipMemcpyDeviceToHost, e->stream));
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  e->host_hdr.arena_next = e->h_hdr_pinned[0].arena_next;
  return ZB_OK;
}

int grow_dev(zb_engine* e, uint8_t** p, uint64_t* cap, uint64_t bytes) {
  if (bytes <= *cap && *p) return ZB_OK;
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  const uint64_t c = std::max<uint64_t>(bytes + bytes / 2, 1 << 20);
  HIPCHECK(e, hipMalloc(p, c));
  *cap = c;
  return ZB_OK;
}

// exclusive scan of u64 in[0, n] into out (in[n] = 0); returns out[n]
int scan_u64(zb_engine* e, uint64_t* in, uint64_t* out, uint64_t n, uint64_t* total) {
  if (n + 1 > (uint64_t)INT32_MAX) return fail(e, ZB_EUNSUPPORTED, "more than 2^31 commands in one batch");
  HIPCHECK(e, hipMemsetAsync(in + n, 0, sizeof(uint64_t), e->stream));
  size_t tmp = 0;
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, in, out, (int)(n + 1), e->stream) != hipSuccess)
    return fail(e, ZB_EDEVICE, "scan sizing");
  int rc = grow_dev(e, (uint8_t**)&e->m_tmp, &e->m_tmp_cap, tmp + 16);
  if (rc != ZB_OK) return rc;
  tmp = e->m_tmp_cap;
  if (hipcub::DeviceScan::ExclusiveSum(e->m_tmp, tmp, in, out, (int)(n + 1), e->stream) != hipSuccess)
    return fail(e, ZB_EDEVICE, "scan");
  HIPCHECK(e, hipMemcpyAsync(total, out + n, sizeof(uint64_t), hipMemcpyDeviceToHost, e->stream));
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  return ZB_OK;
}

// Appends the batch's commands at the log tail and processes them in order, runs of one intent in lockstep
// (PUBLISH: count, scan, emit; DELETE: emit). Follow-ups come after all the commands, in command order (FIFO).
// the outbox order keys of commands from records up to `end` fit their position field (zb_msg.hpp outbox_key)
bool outbox_span_ok(const zb_engine* e, int64_t end) {
  return (uint64_t)(end - std::min(e->ob_pos_base[0], e->ob_pos_base[1])) < (1ull << OB_REL_BITS);
}

// capacity checks of a message batch of n commands (publishes of them) with blob_bytes of blobs
int check_message_batch(zb_engine* e, uint64_t n, uint64_t publishes, uint64_t blob_bytes) {
  const int64_t base = e->host_hdr.end;
  // upper bounds first: every command writes at most 3 records (itself, PUBLISHED, DELETED)
  if ((uint64_t)(base - e->win_base) + 3 * n > e->cfg.log_capacity)
    return fail(e, ZB_ENOMEM, "log capacity (release drained records with zb_log_release)");
  if (!outbox_span_ok(e, base + 3 * (int64_t)n))
    return fail(e, ZB_EUNSUPPORTED, "more than 2^34 log positions since the outbox was last taken");
  if (e->msg_count + publishes > e->store_cap) return fail(e, ZB_ENOMEM, "message store capacity");
  if ((uint64_t)e->host_hdr.arena_next + blob_bytes > e->arena_top) return fail(e, ZB_ENOMEM, "arena capacity");
  return ZB_OK;
}

// the commands of a message batch are in the log at [end, end + n), their blobs at the arena tail (blob_bytes),
// the intra-batch prior flags in m_prior: process them in runs of one intent (runs: [i0, i1) with its intent)
int process_uploaded_messages(zb_engine* e, uint64_t n, uint64_t blob_bytes,
                              const std::vector<std::pair<uint64_t, uint8_t>>& runs, int uniform_out = 0);

int process_messages(zb_engine* e, const MsgBatch& b) {
  const uint64_t n = b.recs.size();
  if (n == 0) return ZB_OK;
  const int64_t base = e->host_hdr.end;
  uint64_t publishes = 0;
  for (const zb_rec& r : b.recs) publishes += r.intent == 0 ? 1 : 0;
  int rc0 = check_message_batch(e, n, publishes, b.blobs.size());
  if (rc0 != ZB_OK) return rc0;
  const uint64_t arena0 = (uint64_t)e->host_hdr.arena_next;
  // commands + blobs (refs made absolute on the host), one upload through pinned staging
  uint8_t* stage = host_stage(e, n * sizeof(zb_rec) + b.blobs.size() + n);
  if (!stage) return fail(e, ZB_ENOMEM, "pinned staging memory");
  zb_rec* recs = (zb_rec*)stage;
  for (uint64_t i = 0; i < n; i++) {
    recs[i] = b.recs[i];
    recs[i].payload += (uint32_t)(arena0 >> 3);
  }
  std::memcpy(stage + n * sizeof(zb_rec), b.blobs.data(), b.blobs.size());
  std::memcpy(stage + n * sizeof(zb_rec) + b.blobs.size(), b.prior.data(), n);
  int rc = grow_dev(e, &e->m_prior, &e->m_prior_cap, n);
  if (rc != ZB_OK) return rc;
  HIPCHECK(e, hipMemcpyAsync(e->log + base, recs, n * sizeof(zb_rec), hipMemcpyHostToDevice, e->stream));
  HIPCHECK(e, hipMemcpyAsync(e->arena + arena0, stage + n * sizeof(zb_rec), b.blobs.size(), hipMemcpyHostToDevice, e->stream));
  HIPCHECK(e, hipMemcpyAsync(e->m_prior, stage + n * sizeof(zb_rec) + b.blobs.size(), n, hipMemcpyHostToDevice, e->stream));
  std::vector<std::pair<uint64_t, uint8_t>> runs;
  for (uint64_t i0 = 0; i0 < n;) {
    const uint8_t intent = b.recs[i0].intent;
    uint64_t i1 = i0 + 1;
    while (i1 < n && b.recs[i1].intent == intent) i1++;
    runs.emplace_back(i1, intent);
    i0 = i1;
  }
  return process_uploaded_messages(e, n, b.blobs.size(), runs);
}

// uniform_out (zb_publish_uploaded): every command is a PUBLISH without a message id -- none can be rejected
// (MessageDataStore.hasMessage needs an id), each writes uniform_out records (PUBLISHED, + DELETED when ttl <= 0: 2)
// and is stored iff uniform_out == 1 -- so the per-command counts and their scan are the closed form i * uniform_out
// (no count pass, no round trip); k_pub_build already initialized the commands' links / sources / lengths
int process_uploaded_messages(zb_engine* e, uint64_t n, uint64_t blob_bytes,
                              const std::vector<std::pair<uint64_t, uint8_t>>& runs, int uniform_out) {
  const int64_t base = e->host_hdr.end;
  e->ob_counts_valid = false;  // (k_pub_emit writes correlations; finish_batch reads the counters back)
  int rc = uniform_out ? ZB_OK : grow_dev(e, (uint8_t**)&e->m_cnt, &e->m_cnt_cap, 2 * (n + 1) * sizeof(uint64_t));
  if (rc != ZB_OK) return rc;
  if (!uniform_out) {
    HIPCHECK(e, hipMemsetAsync(e->links + base, 0xff, n * sizeof(uint64_t), e->stream));
    HIPCHECK(e, hipMemsetAsync(e->srcd + base, 0, n * sizeof(uint32_t), e->stream));  // written by other writers
    // (the verbatim value of a submitted command is its serialized length: the size pass measures the rest)
    HIPCHECK(e, hipMemsetAsync(e->vlen + base, 0xff, n * sizeof(uint32_t), e->stream));
  }
  e->host_hdr.arena_next += (int64_t)blob_bytes;
  e->arena_total += blob_bytes;
  int64_t out = base + (int64_t)n;  // the next follow-up position
  size_t run = 0;
  for (uint64_t i0 = 0; i0 < n;) {
    while (runs[run].first <= i0) run++;
    const uint8_t intent = runs[run].second;
    const uint64_t i1 = std::min<uint64_t>(runs[run].first, i0 + (1u << 20));  // (the count packing: 2^21)
    MsgParams p = msg_params(e);
    p.base = base + (int64_t)i0;
    p.n = (int64_t)(i1 - i0);
    p.out_base = out;
    if (intent == 0 && uniform_out) {
      const uint64_t m = i1 - i0;
      p.key_base = e->msg_key_next;
      p.uni_out = uniform_out;
      launch_pub_emit(p, e->stream);
      out += (int64_t)(m * (uint64_t)uniform_out);
      e->msg_key_next += (int64_t)m;
      if (uniform_out == 1) e->msg_count += m;
    } else if (intent == 0) {  // PUBLISH
      p.prior = e->m_prior + i0;
      p.cnt = e->m_cnt;
      p.cnt_off = e->m_cnt + (n + 1);
      p.key_base = e->msg_key_next;
      launch_pub_count(p, e->stream);
      uint64_t tot = 0;
      rc = scan_u64(e, e->m_cnt, e->m_cnt + (n + 1), i1 - i0, &tot);
      if (rc != ZB_OK) return rc;
      launch_pub_emit(p, e->stream);
      const uint64_t mask = (1ull << 21) - 1;
      out += (int64_t)(tot & mask);
      e->msg_key_next += (int64_t)((tot >> 21) & mask);
      e->msg_count += (tot >> 42) & mask;
    } else {  // DELETE
      launch_msg_delete(p, e->stream);
      out += (int64_t)(i1 - i0);
    }
    i0 = i1;
  }
  e->records_total += (uint64_t)(out - base);
  e->host_hdr.end = out;
  e->host_hdr.begin = e->host_hdr.gen_end = e->host_hdr.end;
  return finish_batch(e);
}

// MessageRecord (MessageRecord.java:26-42) of a submitted MESSAGE command
bool decode_message(const uint8_t* v, size_t n, std::string& name, std::string& ck, int64_t& ttl, const uint8_t*& pl,
                    uint32_t& np, std::string& id) {
  ttl = 0;
  pl = nullptr;
  np = 0;
  if (n == 0) return true;
  MpIn in{v, n};
  const uint32_t props = in.map_hdr();
  for (uint32_t i = 0; i < props && in.ok; i++) {
    const uint8_t* k; uint32_t kl;
    if (!in.str(k, kl)) return false;
    const uint8_t* s; uint32_t sl;
    if (in.key_is(k, kl, "name")) { if (!in.str(s, sl)) return false; name.assign((const char*)s, sl); }
    else if (in.key_is(k, kl, "correlationKey")) { if (!in.str(s, sl)) return false; ck.assign((const char*)s, sl); }
    else if (in.key_is(k, kl, "messageId")) { if (!in.str(s, sl)) return false; id.assign((const char*)s, sl); }
    else if (in.key_is(k, kl, "timeToLive")) ttl = in.integer();
    else if (in.key_is(k, kl, "payload")) { if (!in.bin(pl, np)) return false; }
    else in.skip();
  }
  return in.ok && in.o == n;
}

// the intra-batch part of MessageDataStore.hasMessage: command i follows a command with the same (name,
// correlation key, message id) and ttl > 0 (which stores it unless it is rejected itself -- then so is i)
struct PriorIds {
  std::unordered_set<std::string> seen;
  uint8_t check(const std::string& name, const std::string& ck, const std::string& id, int64_t ttl) {
    if (id.empty()) return 0;
    std::string k;
    k.reserve(name.size() + ck.size() + id.size() + 16);
    auto put = [&](const std::string& s) { const uint64_t l = s.size(); k.append((const char*)&l, 8); k += s; };
    put(name); put(ck); put(id);
    const uint8_t hit = seen.count(k) ? 1 : 0;
    if (ttl > 0) seen.insert(k);
    return hit;
  }
};

// delivered batches in device memory at buf (slices: command count and byte offset of each batch)
int deliver(zb_engine* e, int kind, const uint8_t* buf, const std::vector<uint64_t>& counts,
            const std::vector<uint64_t>& offs, uint64_t* delivered) {
  uint64_t n = 0;
  std::vector<uint64_t> first;
  std::vector<uint64_t> off;
  for (size_t s = 0; s < counts.size(); s++) {
    if (!counts[s]) continue;
    first.push_back(n);
    off.push_back(offs[s]);
    n += counts[s];
  }
  if (delivered) *delivered = n;
  if (n == 0) return ZB_OK;
  const int64_t base = e->host_hdr.end;
  const uint64_t recs = kind == ZB_XCHG_OPEN ? 2 * n : n;
  if ((uint64_t)(base - e->win_base) + recs > e->cfg.log_capacity) return fail(e, ZB_ENOMEM, "log capacity");
  if (!outbox_span_ok(e, base + (int64_t)recs))
    return fail(e, ZB_EUNSUPPORTED, "more than 2^34 log positions since the outbox was last taken");
  if (kind == ZB_XCHG_OPEN && (e->sub_count + n > e->store_cap || e->sub_count + n >= (1ull << 32)))
    return fail(e, ZB_ENOMEM, "subscription store capacity");
  std::vector<uint64_t> table(first);
  table.insert(table.end(), off.begin(), off.end());
  HIPCHECK(e, upload_vec(e, e->d_slices, table));
  MsgParams p = msg_params(e);
  p.in = buf;
  p.nslices = (int32_t)first.size();
  p.slice_first = e->d_slices.p;
  p.slice_off = e->d_slices.p + first.size();
  p.n = (int64_t)n;
  p.base = base;
  const int64_t arena_before = e->host_hdr.arena_next;
  e->ob_counts_valid = false;  // (k_msg_open writes correlations; read back below)
  if (kind == ZB_XCHG_OPEN) {
    launch_msg_open(p, e->stream);  // processed at once: OPEN commands + OPENED events
    e->sub_count += n;
    e->host_hdr.end = base + (int64_t)recs;
    e->host_hdr.begin = e->host_hdr.gen_end = e->host_hdr.end;
  } else {
    // CORRELATE commands: the next zb_step processes them; the element instance each names is looked up by its
    // activity instance key (ElementInstanceIndex.getInstance). k_wis_inject takes the row the subscription's token
    // names when that row still holds the key (live); the others -- a foreign or stale token -- are counted, and only
    // then are the keys sorted and the rows searched (k_resolve, below)
    if (!e->d_unresolved) {
      HIPCHECK(e, hipMalloc(&e->d_unresolved, sizeof(uint32_t)));
      HIPCHECK(e, hipMemsetAsync(e->d_unresolved, 0, sizeof(uint32_t), e->stream));
      e->unresolved_seen = 0;
    }
    if (n > e->x_cap) {
      HIPCHECK(e, hipStreamSynchronize(e->stream));
      void* xs[] = {e->x_keys, e->x_pos, e->x_keys2, e->x_pos2};
      for (void* q : xs)
        if (q) (void)hipFree(q);
      e->x_keys = e->x_pos = e->x_keys2 = e->x_pos2 = nullptr;
      e->x_cap = 0;
      const uint64_t c = std::max<uint64_t>(n + n / 2, 1024);
      HIPCHECK(e, hipMalloc(&e->x_keys, c * 8));
      HIPCHECK(e, hipMalloc(&e->x_pos, c * 8));
      HIPCHECK(e, hipMalloc(&e->x_keys2, c * 8));
      HIPCHECK(e, hipMalloc(&e->x_pos2, c * 8));
      e->x_cap = c;
    }
    if (n > (uint64_t)INT32_MAX) return fail(e, ZB_EUNSUPPORTED, "more than 2^31 delivered commands");
    p.lookup_keys = e->x_keys;
    p.lookup_pos = e->x_pos;
    p.rmeta = e->rmeta;
    p.rkeys = e->rkeys;
    p.rows = (uint64_t)e->host_hdr.rows_next;
    p.unresolved = e->d_unresolved;
    launch_wis_inject(p, e->stream);
    e->host_hdr.end = base + (int64_t)recs;
    e->host_hdr.gen_end = e->host_hdr.end;
  }
  // blobs were allocated on the device header: its arena pointer and the error word in one round trip (with the
  // outbox counters and the unresolved count), then the host's header (log range) back to the device, stream-ordered
  // before the next step's kernels
  uint32_t* unres = e->h_err_pinned + 1;
  {
    StatusReads r;
    r.add(e->h_hdr_pinned, e->hdr + (e->wave & 1), sizeof(WaveHdr));
    r.add(e->h_err_pinned, e->derr, sizeof(uint32_t));
    if (e->on) r.add(e->h_stats_pinned + 19, e->on, 4 * sizeof(uint32_t));
    if (kind != ZB_XCHG_OPEN) r.add(unres, e->d_unresolved, sizeof(uint32_t));
    HIPCHECK(e, r.launch(e->stream));
  }
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  e->ob_counts_valid = e->on != nullptr;
  e->host_hdr.arena_next = e->h_hdr_pinned[0].arena_next;
  int rc = check_device_errors(e, *e->h_err_pinned);
  if (rc != ZB_OK) return rc;
  if (kind != ZB_XCHG_OPEN && *unres != e->unresolved_seen) {  // (a running count: no reset between deliveries)
    e->unresolved_seen = *unres;
    rc = sort_pairs(e, e->x_keys, e->x_keys2, e->x_pos, e->x_pos2, n, "inbox");
    if (rc != ZB_OK) return rc;
    ResolveParams rp{};
    rp.rmeta = e->rmeta; rp.rkeys = e->rkeys; rp.rows = (uint64_t)e->host_hdr.rows_next;
    rp.keys = e->x_keys2; rp.pos = e->x_pos2; rp.pos_base = 0; rp.n = (int64_t)n;
    rp.links = e->links;
    launch_resolve(rp, e->stream);  // (every key of the delivery: the token rows it finds again are the same rows)
  }
  e->records_total += recs;
  e->arena_total += (uint64_t)(e->host_hdr.arena_next - arena_before);
  HIPCHECK(e, upload_async(e, e->hdr + (e->wave & 1), &e->host_hdr, sizeof(WaveHdr)));
  return ZB_OK;
}

// an exchange batch header [count][total bytes] inside the avail bytes left: the records fit the batch (no overflow
// in count * 64), the total is 8-aligned
bool batch_header_ok(const uint64_t h[2], size_t avail) {
  if (h[1] < ZB_XCHG_BATCH_HEADER || h[1] > avail || (h[1] & 7)) return false;
  return h[0] <= (h[1] - ZB_XCHG_BATCH_HEADER) / sizeof(zb_exchange_rec);
}

// every record's variable bytes [name][correlation key][payload] lie inside its batch's byte section, and a
// CORRELATE names a catch element of this partition's model (the inbox kernels read both without a bounds check)
bool batch_records_ok(const zb_exchange_rec* r, uint64_t cnt, uint64_t total, int kind, size_t n_elems) {
  const uint64_t var_bytes = total - ZB_XCHG_BATCH_HEADER - cnt * sizeof(zb_exchange_rec);
  for (uint64_t i = 0; i < cnt; i++) {
    const uint64_t need = (uint64_t)r[i].name_len + r[i].ck_len + r[i].payload_len;  // (< 2^34: no overflow)
    if (r[i].var_offset > var_bytes || need > var_bytes - r[i].var_offset) return false;
    if (kind == ZB_XCHG_CORRELATE && r[i].elem >= n_elems) return false;
  }
  return true;
}

// batches laid out back to back (host memory): (count, byte offset) of each, from their headers, every record checked
bool parse_batches(const uint8_t* p, size_t bytes, int kind, size_t n_elems, std::vector<uint64_t>& counts,
                   std::vector<uint64_t>& offs) {
  size_t o = 0;
  while (o < bytes) {
    if (bytes - o < ZB_XCHG_BATCH_HEADER) return false;
    uint64_t h[2];
    std::memcpy(h, p + o, sizeof(h));
    if (!batch_header_ok(h, bytes - o)) return false;
    std::vector<zb_exchange_rec> r(h[0]);
    if (h[0]) std::memcpy(r.data(), p + o + ZB_XCHG_BATCH_HEADER, h[0] * sizeof(zb_exchange_rec));
    if (!batch_records_ok(r.data(), h[0], h[1], kind, n_elems)) return false;
    counts.push_back(h[0]);
    offs.push_back(o);
    o += h[1];
  }
  return true;
}

}  // namespace

extern "C" {

int zb_set_clock(zb_engine* e, int64_t now_ms) {
  if (!e) return ZB_EINVAL;
  e->clock_ms = now_ms;
  return ZB_OK;
}

int zb_submit_messages(zb_engine* e, const zb_rec_desc* recs, size_t n, const uint8_t* values, size_t values_len) {
  if (!e || (n > 0 && (!recs || (!values && values_len)))) return ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  int rc = require_idle(e);
  if (rc != ZB_OK) return rc;
  if (n == 0) return ZB_OK;
  MsgBatch b;
  b.recs.reserve(n);
  b.prior.reserve(n);
  PriorIds prior;
  static const uint8_t EMPTY = 0x80;
  for (size_t i = 0; i < n; i++) {  // decode + validate everything first (nothing changes on an error)
    const zb_rec_desc& r = recs[i];
    if (r.value_offset > values_len || r.value_length > values_len - r.value_offset)
      return fail(e, ZB_EINVAL, "record " + std::to_string(i) + ": value out of range");
    if (r.value_type != ZB_VT_MESSAGE || r.record_type != ZB_RT_COMMAND || (r.intent != 0 && r.intent != 2))
      return fail(e, ZB_EUNSUPPORTED, "record " + std::to_string(i) + ": no message processor is registered for "
                                      "(recordType, valueType, intent) = (" + std::to_string(r.record_type) + ", " +
                                      std::to_string(r.value_type) + ", " + std::to_string(r.intent) + ")");
    const uint8_t* v = values + r.value_offset;
    std::string name, ck, id;
    int64_t ttl = 0;
    const uint8_t* pl = nullptr;
    uint32_t np = 0;
    if (!decode_message(v, r.value_length, name, ck, ttl, pl, np, id))
      return fail(e, ZB_EINVAL, "record " + std::to_string(i) + ": malformed msgpack value");
    if (!pl || np == 0 || (np == 1 && pl[0] == 0xc0)) { pl = &EMPTY; np = 1; }  // DocumentValue: nil -> {}
    if (!is_doc(pl, np))
      return fail(e, ZB_EINVAL, "record " + std::to_string(i) + ": Document has invalid format. On root level an object is only allowed.");
    zb_rec d{};
    d.key = r.intent == 0 ? -1 : r.key;  // PUBLISH: a client command has no key
    d.scope_key = -1;
    d.inst_key = -1;
    d.payload = add_msg_blob(b.blobs, (const uint8_t*)name.data(), (uint32_t)name.size(), (const uint8_t*)ck.data(),
                             (uint32_t)ck.size(), ttl, pl, np, (const uint8_t*)id.data(), (uint32_t)id.size());
    add_blob(b.blobs, v, (uint32_t)r.value_length);  // the verbatim value (KIND_RAW)
    d.elem = NO_ELEM;
    d.intent = r.intent;
    d.kind = (uint8_t)(make_kind(ZB_VT_MESSAGE, ZB_RT_COMMAND, false) | KIND_RAW);
    b.recs.push_back(d);
    b.prior.push_back(r.intent == 0 ? prior.check(name, ck, id, ttl) : 0);
  }
  rc = ensure_stores(e);
  if (rc == ZB_OK) rc = maintain(e, false);
  if (rc != ZB_OK) return rc;
  return process_messages(e, b);
}

}  // extern "C"
namespace {
// the device-side view of an uploaded PUBLISH batch (zb_upload_publishes: p_in holds the caller's bytes as they are)
PubBuild pub_build_params(zb_engine* e, const PubUpload& u) {
  PubBuild pb{};
  pb.cks = e->p_in + u.a_ck;
  pb.ck_off = (const uint64_t*)(e->p_in + u.a_cko);
  pb.pls = e->p_in + u.a_pl;
  pb.pl_off = (const uint64_t*)(e->p_in + u.a_plo);
  pb.name = e->p_in + u.a_name;
  pb.nn = u.nn;
  pb.ttl = u.ttl;
  pb.n = u.n;
  pb.gran = e->p_gran;
  pb.goff = e->p_gran + (u.n + 1);
  pb.err = (uint32_t*)(e->p_gran + 2 * (u.n + 1));
  return pb;
}
}  // namespace
extern "C" {

int zb_upload_publishes(zb_engine* e, const char* name, int64_t ttl, size_t n, const uint8_t* cks,
                        const uint64_t* ck_offsets, const uint8_t* payloads, const uint64_t* payload_offsets) {
  if (!e || !name || (n > 0 && (!cks || !ck_offsets || !payloads || !payload_offsets))) return ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  e->pub_up.valid = false;
  if (n == 0) return ZB_OK;
  const uint32_t nn = (uint32_t)std::strlen(name);
  int rc = ensure_stores(e);
  if (rc != ZB_OK) return rc;
  // The caller's correlation keys / payloads go up as they are (one pinned staging copy, by up to 8 host
  // threads for large batches); the commands and message blobs are built on the device (k_pub_sizes / scan /
  // k_pub_build, zb_msg.hip) when the batch is processed -- all-or-nothing: nothing reaches the log or the arena
  // before the checks pass.
  const uint64_t ckb = ck_offsets[n] - ck_offsets[0], plb = payload_offsets[n] - payload_offsets[0];
  const uint64_t offb = (n + 1) * sizeof(uint64_t);
  const uint64_t a_ck = 0, a_cko = (ckb + 15) & ~15ull, a_pl = a_cko + offb, a_plo = a_pl + ((plb + 15) & ~15ull);
  const uint64_t a_name = a_plo + offb, total = a_name + ((nn + 16) & ~15ull);
  uint8_t* stage = host_stage(e, total);
  if (!stage) return fail(e, ZB_ENOMEM, "pinned staging memory");
  {
    struct Piece { uint8_t* dst; const uint8_t* src; uint64_t n; };
    const Piece pieces[5] = {{stage + a_ck, cks + ck_offsets[0], ckb}, {stage + a_cko, (const uint8_t*)ck_offsets, offb},
                             {stage + a_pl, payloads + payload_offsets[0], plb},
                             {stage + a_plo, (const uint8_t*)payload_offsets, offb}, {stage + a_name, (const uint8_t*)name, nn}};
    const size_t nth = total >= (16u << 20) ? std::min<size_t>(8, std::max(1u, std::thread::hardware_concurrency())) : 1;
    auto body = [&](size_t t) {  // byte range [t, t + 1) / nth of every piece
      for (const Piece& q : pieces) {
        const uint64_t lo = q.n * t / nth, hi = q.n * (t + 1) / nth;
        if (hi > lo) std::memcpy(q.dst + lo, q.src + lo, hi - lo);
      }
    };
    std::vector<std::thread> ths;
    for (size_t t = 1; t < nth; t++) ths.emplace_back(body, t);
    body(0);
    for (auto& th : ths) th.join();
  }
  rc = grow_dev(e, &e->p_in, &e->p_in_cap, total);
  if (rc == ZB_OK) rc = grow_dev(e, (uint8_t**)&e->p_gran, &e->p_gran_cap, 2 * (n + 1) * sizeof(uint64_t) + 16);
  if (rc == ZB_OK) rc = grow_dev(e, &e->m_prior, &e->m_prior_cap, n);
  if (rc != ZB_OK) return rc;
  HIPCHECK(e, hipMemcpyAsync(e->p_in, stage, total, hipMemcpyHostToDevice, e->stream));
  // the batch checked and its blobs sized now (k_pub_sizes, scan): processing it needs no round trip for them
  PubUpload u{true, n, nn, ttl, a_ck, a_cko, a_pl, a_plo, a_name, 0};
  PubBuild pb = pub_build_params(e, u);
  HIPCHECK(e, hipMemsetAsync(pb.err, 0, 2 * sizeof(uint32_t), e->stream));
  launch_pub_sizes(pb, e->stream);
  uint32_t herr[2] = {0, 0};
  HIPCHECK(e, hipMemcpyAsync(herr, pb.err, sizeof(herr), hipMemcpyDeviceToHost, e->stream));
  rc = scan_u64(e, e->p_gran, e->p_gran + (n + 1), n, &u.gran);  // (sets gran[n] = 0 first; its round trip covers
  if (rc != ZB_OK) return rc;                                      // the upload and the error words too)
  if (herr[0]) return fail(e, ZB_EINVAL, "Document has invalid format. On root level an object is only allowed.");
  if (herr[1]) return fail(e, ZB_EINVAL, "correlation key or payload too long");
  e->pub_up = u;
  return ZB_OK;
}

int zb_publish_uploaded(zb_engine* e) {
  if (!e) return ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  if (!e->pub_up.valid) return fail(e, ZB_EINVAL, "no uploaded publish batch (zb_upload_publishes)");
  int rc = require_idle(e);
  if (rc != ZB_OK) return rc;
  rc = maintain(e, false);
  if (rc != ZB_OK) return rc;
  const PubUpload u = e->pub_up;
  e->pub_up.valid = false;
  const uint64_t n = u.n;
  rc = check_message_batch(e, n, n, u.gran * 8);
  if (rc != ZB_OK) return rc;
  PubBuild pb = pub_build_params(e, u);
  pb.arena = e->arena;
  pb.arena0 = (uint64_t)e->host_hdr.arena_next;
  pb.out = e->log + e->host_hdr.end;
  pb.links = e->links + e->host_hdr.end;
  pb.srcd = e->srcd + e->host_hdr.end;
  pb.vlen = e->vlen + e->host_hdr.end;
  launch_pub_build(pb, e->stream);
  std::vector<std::pair<uint64_t, uint8_t>> runs{{n, (uint8_t)0}};
  return process_uploaded_messages(e, n, u.gran * 8, runs, u.ttl > 0 ? 1 : 2);
}

int zb_submit_publishes(zb_engine* e, const char* name, int64_t ttl, size_t n, const uint8_t* cks,
                        const uint64_t* ck_offsets, const uint8_t* payloads, const uint64_t* payload_offsets) {
  if (!e || !name || (n > 0 && (!cks || !ck_offsets || !payloads || !payload_offsets))) return ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  int rc = require_idle(e);
  if (rc != ZB_OK) return rc;
  if (n == 0) return ZB_OK;
  rc = zb_upload_publishes(e, name, ttl, n, cks, ck_offsets, payloads, payload_offsets);
  return rc == ZB_OK ? zb_publish_uploaded(e) : rc;
}

int zb_expire_messages(zb_engine* e, int64_t now_ms, uint64_t* n_deleted) {
  if (!e) return ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  if (n_deleted) *n_deleted = 0;
  int rc = require_idle(e);
  if (rc != ZB_OK) return rc;
  if (!e->msgs || e->msg_count == 0) return ZB_OK;
  rc = maintain(e, false);
  if (rc != ZB_OK) return rc;
  const uint64_t m = e->msg_count;
  rc = grow(e, &e->c_flag, &e->c_flag_cap, m + 1);
  if (rc == ZB_OK) rc = grow(e, &e->c_new, &e->c_new_cap, m + 1);
  if (rc != ZB_OK) return rc;
  MsgParams p = msg_params(e);
  p.now = now_ms;
  p.flags = e->c_flag;
  launch_ttl_flags(p, e->stream);
  uint64_t k = 0;
  rc = scan_u32(e, e->c_flag, e->c_new, m, &k);
  if (rc != ZB_OK) return rc;
  if (k == 0) return ZB_OK;
  const int64_t base = e->host_hdr.end;
  if ((uint64_t)(base - e->win_base) + 2 * k > e->cfg.log_capacity) return fail(e, ZB_ENOMEM, "log capacity");
  p.base = base;
  p.flag_off = e->c_new;
  launch_ttl_write(p, e->stream);  // the checker's DELETE commands at [base, base + k)
  MsgParams d = msg_params(e);
  d.base = base;
  d.n = (int64_t)k;
  d.out_base = base + (int64_t)k;
  launch_msg_delete(d, e->stream);  // ... and their processing
  e->host_hdr.end = base + 2 * (int64_t)k;
  e->host_hdr.begin = e->host_hdr.gen_end = e->host_hdr.end;
  e->records_total += 2 * k;
  if (n_deleted) *n_deleted = k;
  return finish_batch(e);
}

int zb_inbox_submit(zb_engine* e, int kind, const uint8_t* batches, size_t bytes, int on_device) {
  if (!e || (bytes > 0 && !batches) || (kind != ZB_XCHG_OPEN && kind != ZB_XCHG_CORRELATE)) return ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  int rc = require_idle(e);
  if (rc != ZB_OK) return rc;
  if (bytes == 0) return ZB_OK;
  std::vector<uint64_t> counts, offs;
  const size_t n_elems = e->model.elems.size();
  if (on_device) {  // batch headers and records read one batch after another, checked as for host batches
    size_t o = 0;
    std::vector<zb_exchange_rec> r;
    while (o < bytes) {
      uint64_t h[2];
      if (bytes - o < sizeof(h)) return fail(e, ZB_EINVAL, "malformed exchange batches");
      HIPCHECK(e, hipMemcpy(h, batches + o, sizeof(h), hipMemcpyDeviceToHost));
      if (!batch_header_ok(h, bytes - o)) return fail(e, ZB_EINVAL, "malformed exchange batches");
      r.resize(h[0]);
      if (h[0])
        HIPCHECK(e, hipMemcpy(r.data(), batches + o + ZB_XCHG_BATCH_HEADER, h[0] * sizeof(zb_exchange_rec),
                              hipMemcpyDeviceToHost));
      if (!batch_records_ok(r.data(), h[0], h[1], kind, n_elems))
        return fail(e, ZB_EINVAL, "malformed exchange batches: a record's variable bytes or element out of range");
      counts.push_back(h[0]);
      offs.push_back(o);
      o += h[1];
    }
  } else if (!parse_batches(batches, bytes, kind, n_elems, counts, offs)) {
    return fail(e, ZB_EINVAL, "malformed exchange batches");
  }
  rc = ensure_stores(e);
  if (rc == ZB_OK) rc = maintain(e, false);
  if (rc != ZB_OK) return rc;
  const uint8_t* dbuf = batches;
  if (!on_device) {
    rc = grow_dev(e, &e->in_buf, &e->in_buf_cap, bytes);
    if (rc != ZB_OK) return rc;
    HIPCHECK(e, hipMemcpyAsync(e->in_buf, batches, bytes, hipMemcpyHostToDevice, e->stream));
    dbuf = e->in_buf;
  }
  return deliver(e, kind, dbuf, counts, offs, nullptr);
}

int zb_outbox_count(zb_engine* e, int kind, uint64_t* n) {
  if (!e || !n || (kind != ZB_XCHG_OPEN && kind != ZB_XCHG_CORRELATE)) return ZB_EINVAL;
  *n = 0;
  if (!e->on) return ZB_OK;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  uint32_t* c = (uint32_t*)(e->h_stats_pinned + 19);  // (pinned: commands OPEN, CORRELATE, granules OPEN, CORRELATE)
  if (!e->ob_counts_valid) {
    StatusReads r;
    r.add(c, e->on, 4 * sizeof(uint32_t));
    HIPCHECK(e, r.launch(e->stream));
    HIPCHECK(e, hipStreamSynchronize(e->stream));
    e->ob_counts_valid = true;
  }
  for (int k = 1; k <= 2; k++)
    if ((uint64_t)c[k - 1] > e->ocap || (uint64_t)c[k + 1] > e->ovar_cap)
      return fail(e, ZB_ENOMEM, "outbox overflow (commands or their variable bytes)");
  *n = c[kind - 1];
  e->ob_counts_read[0] = c[0];
  e->ob_counts_read[1] = c[1];
  // an empty outbox takes the processing frontier as its order-key base now, not only at its next take: every command
  // it receives from here on comes from a record at or after it (a kind that stays empty for long would otherwise keep
  // an old base, and a later command -- or the span check of a message batch -- would meet the 2^34 relative-key limit)
  for (int k = 0; k < 2; k++)
    if (c[k] == 0) e->ob_pos_base[k] = std::max(e->ob_pos_base[k], e->host_hdr.begin);
  return ZB_OK;
}

}  // extern "C"

namespace {
// outbox_plan sorts the outbox of `kind` by (target, source position, emission) and sizes one exchange batch per
// target: per-target byte sizes into bytes_per_target, *total = their sum (the outbox is left as it is).
// outbox_emit then lays the planned batches out at dst (device, target order) and takes the outbox: one sort per
// exchange.
// local: one partition delivering to its own inbox -- the batch sizes are needed only as a capacity bound, so the
// per-target table is not read back (one host round trip less per exchange)
int outbox_plan(zb_engine* e, int kind, uint64_t* bytes_per_target, uint64_t* counts, uint64_t* n_out, uint64_t* total,
                bool local = false) {
  const int P = e->cfg.partition_count;
  if (P > 64) return fail(e, ZB_EUNSUPPORTED, "more than 64 partitions");
  for (int q = 0; q < P; q++) bytes_per_target[q] = counts[q] = 0;
  *total = 0;
  e->ob_plan_kind = 0;
  const int k = kind - 1;
  if (e->on && e->ob_counts_valid && ((const uint32_t*)(e->h_stats_pinned + 19))[k] == 0)  // (nothing to take)
    return zb_outbox_count(e, kind, n_out);
  // the key spread of the sort below, over the device-side count: read back in the count's round trip
  if (e->on) {  // (the counters read again, in the spread's round trip)
    HIPCHECK(e, hipMemsetAsync(e->d_spread, 0, sizeof(uint64_t), e->stream));
    launch_key_spread(e->okeys[k], e->ocap, e->d_spread, e->stream, e->on + k);
    StatusReads r;
    r.add(e->h_stats_pinned + 17, e->d_spread, sizeof(uint64_t));
    r.add(e->h_stats_pinned + 19, e->on, 4 * sizeof(uint32_t));
    HIPCHECK(e, r.launch(e->stream));
    HIPCHECK(e, hipStreamSynchronize(e->stream));
    e->ob_counts_valid = true;
  }
  uint64_t n = 0;
  int rc = zb_outbox_count(e, kind, &n);
  if (rc != ZB_OK) return rc;
  *n_out = n;
  if (n == 0) return ZB_OK;
  if (!e->ob_keys) {  // sort buffers, allocated once at the outbox capacity
    const uint64_t c = e->ocap;
    if (hipMalloc(&e->ob_keys, c * 8) != hipSuccess || hipMalloc(&e->ob_idx_in, c * 4) != hipSuccess ||
        hipMalloc(&e->ob_idx_out, c * 4) != hipSuccess || hipMalloc(&e->ob_first, 65 * 8) != hipSuccess ||
        hipMalloc(&e->ob_sizes, (c + 1) * 4) != hipSuccess || hipMalloc(&e->ob_goff, (c + 1) * 4) != hipSuccess ||
        hipMalloc(&e->ob_table, 2 * 64 * 8) != hipSuccess || hipMalloc(&e->ob_base, 64 * 8) != hipSuccess)
      return fail(e, ZB_ENOMEM, "outbox sort buffers");
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, e->ob_tmp_bytes, e->ob_sizes, e->ob_goff, (int)(c + 1), e->stream) !=
        hipSuccess)
      return fail(e, ZB_ENOMEM, "outbox scan scratch");
    if (hipMalloc(&e->ob_tmp, e->ob_tmp_bytes + 16) != hipSuccess) return fail(e, ZB_ENOMEM, "outbox scan scratch");
  }
  // the sort: by counting when the keys' spread is narrow and dense enough (a tick's commands: a position range a
  // few times the command count), else the radix sort over the spread's bits
  const uint64_t spread = e->h_stats_pinned[17];
  const int cs_begin = spread ? __builtin_ctzll(spread) : 0;
  const int cs_bits = spread ? 64 - __builtin_clzll(spread) - cs_begin : 0;
  const Outbox ob = outbox(e, kind);
  e->ob_plan_cs = false;
  // (a bucket packs commands << 40 | granules: fewer than 2^24 commands and 2^40 granules per take)
  const uint64_t var_gran = ((const uint32_t*)(e->h_stats_pinned + 19))[kind + 1];
  if (spread && cs_bits <= 24 && (1ull << cs_bits) <= 32 * n && n < (1ull << 24) && var_gran < (1ull << 40)) {
    const uint64_t nb = 1ull << cs_bits;
    size_t tmp = 0;
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, e->cs_cnt, e->cs_off, (int)nb, e->stream) != hipSuccess)
      return fail(e, ZB_EDEVICE, "outbox count scan sizing");
    if (nb > e->cs_cap || tmp + 16 > e->cs_tmp_cap) {
      HIPCHECK(e, hipStreamSynchronize(e->stream));
      void* ps[] = {e->cs_cnt, e->cs_off, e->cs_tmp};
      for (void* q : ps)
        if (q) (void)hipFree(q);
      e->cs_cnt = e->cs_off = nullptr;
      e->cs_tmp = nullptr;
      e->cs_cap = e->cs_tmp_cap = 0;
      HIPCHECK(e, hipMalloc(&e->cs_cnt, nb * 8));
      HIPCHECK(e, hipMalloc(&e->cs_off, nb * 8));
      HIPCHECK(e, hipMalloc(&e->cs_tmp, tmp + 16));
      e->cs_cap = nb;
      e->cs_tmp_cap = tmp + 16;
    }
    HIPCHECK(e, hipMemsetAsync(e->cs_cnt, 0, nb * 8, e->stream));
    launch_cs_hist(ob, n, cs_begin, cs_bits, e->cs_cnt, e->stream);
    size_t have = e->cs_tmp_cap;
    if (hipcub::DeviceScan::ExclusiveSum(e->cs_tmp, have, e->cs_cnt, e->cs_off, (int)nb, e->stream) != hipSuccess)
      return fail(e, ZB_EDEVICE, "outbox count scan");
    if (local && P == 1) {  // the slots and variable places come out of the scatter (outbox_emit: k_local_pack)
      launch_cs_scatter(ob, n, cs_begin, cs_bits, e->cs_off, nullptr, e->ob_idx_out, e->ob_goff, e->stream);
      const uint32_t* c = (const uint32_t*)(e->h_stats_pinned + 19);
      counts[0] = n;
      bytes_per_target[0] = ZB_XCHG_BATCH_HEADER + n * sizeof(zb_exchange_rec) + 8 * (uint64_t)c[kind + 1];
      *total = bytes_per_target[0];
      e->ob_plan_cs = true;
      e->ob_plan_kind = kind;
      e->ob_plan_n = n;
      e->ob_plan_total = *total;
      return ZB_OK;
    }
    launch_cs_scatter(ob, n, cs_begin, cs_bits, e->cs_off, e->ob_keys, e->ob_idx_out, nullptr, e->stream);
  } else {
    launch_iota(e->ob_idx_in, n, e->stream);
    rc = sort_pairs(e, (const uint64_t*)e->okeys[k], e->ob_keys, (const uint32_t*)e->ob_idx_in, e->ob_idx_out, n,
                    "outbox", true);
    if (rc != ZB_OK) return rc;
  }
  launch_outbox_sizes(ob, e->ob_idx_out, n, e->ob_sizes, e->stream);
  size_t tmp_bytes = e->ob_tmp_bytes;
  if (hipcub::DeviceScan::ExclusiveSum(e->ob_tmp, tmp_bytes, e->ob_sizes, e->ob_goff, (int)(n + 1), e->stream) != hipSuccess)
    return fail(e, ZB_EDEVICE, "outbox scan");
  launch_outbox_bounds(e->ob_keys, n, e->ob_first, P, e->stream);
  if (local && P == 1) {  // (the command count and variable granules came with the count's round trip)
    const uint32_t* c = (const uint32_t*)(e->h_stats_pinned + 19);
    counts[0] = n;
    bytes_per_target[0] = ZB_XCHG_BATCH_HEADER + n * sizeof(zb_exchange_rec) + 8 * (uint64_t)c[kind + 1];
    e->ob_plan_base[0] = 0;
    *total = bytes_per_target[0];
    e->ob_plan_kind = kind;
    e->ob_plan_n = n;
    e->ob_plan_total = *total;
    return ZB_OK;
  }
  launch_outbox_table(e->ob_first, e->ob_goff, P, e->ob_table, e->stream);
  uint64_t table[128];
  HIPCHECK(e, hipMemcpyAsync(table, e->ob_table, 2 * P * 8, hipMemcpyDeviceToHost, e->stream));
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  uint64_t o = 0;
  for (int q = 0; q < P; q++) {
    counts[q] = table[2 * q];
    bytes_per_target[q] = counts[q] ? ZB_XCHG_BATCH_HEADER + counts[q] * sizeof(zb_exchange_rec) + 8 * table[2 * q + 1] : 0;
    e->ob_plan_base[q] = o;
    o += bytes_per_target[q];
  }
  *total = o;
  e->ob_plan_kind = kind;
  e->ob_plan_n = n;
  e->ob_plan_total = o;
  return ZB_OK;
}

int outbox_emit(zb_engine* e, int kind, uint8_t* dst, uint64_t cap) {
  if (e->ob_plan_kind != kind) return fail(e, ZB_EDEVICE, "outbox emit without a plan");
  e->ob_plan_kind = 0;
  if (e->ob_plan_total > cap) return fail(e, ZB_ENOMEM, "outbox destination too small");
  const int P = e->cfg.partition_count;
  const int k = kind - 1;
  if (e->ob_plan_cs) {  // one batch in the counting sort's order; the pack also takes the outbox
    launch_local_pack(outbox(e, kind), e->ob_idx_out, e->ob_goff, e->ob_plan_n, e->ob_plan_total, dst, e->on + k,
                      e->on + 2 + k, e->stream);
  } else {
    HIPCHECK(e, upload_async(e, e->ob_base, e->ob_plan_base, P * 8));
    launch_outbox_pack(outbox(e, kind), e->ob_idx_out, e->ob_keys, e->ob_plan_n, e->ob_first, e->ob_goff, e->ob_base,
                       dst, e->stream);
    HIPCHECK(e, hipMemsetAsync(e->on + k, 0, sizeof(uint32_t), e->stream));      // the outbox is taken
    HIPCHECK(e, hipMemsetAsync(e->on + 2 + k, 0, sizeof(uint32_t), e->stream));  // (and its byte section)
  }
  if (e->ob_counts_valid) {  // (the other kind's counters are untouched: the read-back copy stays current)
    uint32_t* c = (uint32_t*)(e->h_stats_pinned + 19);
    c[k] = c[2 + k] = 0;
  }
  // the commands written from here on come from records at or after the processing frontier
  e->ob_pos_base[k] = e->host_hdr.begin;
  return ZB_OK;  // (stream-ordered: the exchange's sends / the local delivery follow on the same stream)
}
}  // namespace

extern "C" {

int zb_outbox_take(zb_engine* e, int kind, uint8_t* dst, size_t cap, int dst_on_device, uint64_t* bytes_per_target,
                   uint64_t* n_out, uint64_t* total) {
  if (!e || !bytes_per_target || !n_out || !total || (kind != ZB_XCHG_OPEN && kind != ZB_XCHG_CORRELATE))
    return ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  uint64_t counts[64];
  int rc = outbox_plan(e, kind, bytes_per_target, counts, n_out, total);
  if (rc != ZB_OK || *n_out == 0) return rc;
  if (!dst || cap < *total) return ZB_ENOMEM;
  uint8_t* out = dst;
  if (!dst_on_device) {
    rc = grow_dev(e, &e->ob_staging, &e->ob_staging_cap, *total);
    if (rc != ZB_OK) return rc;
    out = e->ob_staging;
  }
  rc = outbox_emit(e, kind, out, dst_on_device ? cap : e->ob_staging_cap);
  if (rc != ZB_OK) return rc;
  if (!dst_on_device) HIPCHECK(e, hipMemcpyAsync(dst, e->ob_staging, *total, hipMemcpyDeviceToHost, e->stream));
  HIPCHECK(e, hipStreamSynchronize(e->stream));  // (the batches are complete on return)
  return ZB_OK;
}

#define NCCLCHECK(e, call)                                                                      \
  do {                                                                                          \
    ncclResult_t _r = (call);                                                                   \
    if (_r != ncclSuccess) return fail((e), ZB_EDEVICE, std::string(#call) + ": " + ncclGetErrorString(_r)); \
  } while (0)

const char* zb_rccl_library(void) {
  static std::string path;
  Dl_info info{};
  if (path.empty() && dladdr((void*)&ncclCommInitRank, &info) && info.dli_fname) path = info.dli_fname;
  return path.c_str();
}

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
  e->comm_broken = false;
  HIPCHECK(e, hipMalloc(&e->d_xcounts, 8 * 64 * sizeof(uint64_t)));
  int rc = ensure_outbox(e);
  if (rc != ZB_OK) return rc;
  // exchange buffers for the common case up front (grown later only if a round needs more)
  rc = grow_dev(e, &e->xsend, &e->xsend_cap, 16ull << 20);
  if (rc == ZB_OK) rc = grow_dev(e, &e->xrecv, &e->xrecv_cap, 16ull << 20);
  return rc;
}

}  // extern "C"

namespace {
// an RCCL failure leaves the communicator unusable (peers may be inside the same collective): abort it so
// that no later call blocks on it, and fail this and every later exchange on this engine
int comm_fail(zb_engine* e, const std::string& what, ncclResult_t r) {
  e->comm_broken = true;
  if (e->comm) (void)ncclCommAbort(e->comm);
  e->comm = nullptr;
  return fail(e, ZB_EDEVICE, what + ": " + ncclGetErrorString(r));
}
}  // namespace

extern "C" {

// a single partition without ZB_CFG_RCCL_SELF exchanges with itself on the device: it needs no communicator
static bool comm_local(const zb_engine* e) {
  return e->cfg.partition_count == 1 && !(e->cfg.flags & ZB_CFG_RCCL_SELF);
}

int zb_comm_pending(zb_engine* e, uint64_t global[2]) {
  if (!e || !global) return ZB_EINVAL;
  if (!e->comm && !comm_local(e))
    return e->comm_broken ? fail(e, ZB_EDEVICE, "communicator aborted after an earlier failure") : ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  uint64_t local[2] = {0, 0};
  int rc0 = zb_outbox_count(e, ZB_XCHG_OPEN, &local[0]);  // (one read of both counts)
  if (rc0 != ZB_OK) return rc0;
  local[1] = e->ob_counts_read[1];
  if (e->cfg.partition_count == 1 && !(e->cfg.flags & ZB_CFG_RCCL_SELF)) {  // no peer: the sum is the local count
    global[0] = local[0];
    global[1] = local[1];
    return ZB_OK;
  }
  HIPCHECK(e, hipMemcpyAsync(e->d_xcounts, local, sizeof(local), hipMemcpyHostToDevice, e->stream));
  ncclResult_t nr = ncclAllReduce(e->d_xcounts, e->d_xcounts, 2, ncclUint64, ncclSum, e->comm, e->stream);
  if (nr != ncclSuccess) return comm_fail(e, "pending counts", nr);
  HIPCHECK(e, hipMemcpyAsync(global, e->d_xcounts, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, e->stream));
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  return ZB_OK;
}

// Collective on every rank, whatever happens locally: a rank whose local work fails still takes part in
// both agreement steps (sending zero sizes and its status), so every rank returns the same error instead
// of one rank leaving the collective and its peers blocking in ncclSend / ncclRecv. In the guard-band test build
// only (zb_checked.hpp), ZB_FAIL_EXCHANGE=<rank> makes that rank's local step fail.
int zb_comm_exchange(zb_engine* e, int kind, uint64_t* received) {
  if (!e || !received || (kind != ZB_XCHG_OPEN && kind != ZB_XCHG_CORRELATE)) return ZB_EINVAL;
  if (!e->comm && !comm_local(e))
    return e->comm_broken ? fail(e, ZB_EDEVICE, "communicator aborted after an earlier failure") : ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  const int P = e->cfg.partition_count;
  *received = 0;
  // 0. local: the outbox as one batch per target into the persistent send buffer
  uint64_t sb[64] = {}, sc[64] = {}, n = 0, total = 0;
  int local = ZB_OK;
#ifdef ZB_CHECKED
  if (const char* f = std::getenv("ZB_FAIL_EXCHANGE"))  // (before the outbox is taken: a retry still has it)
    if (*f && atoi(f) == e->cfg.partition_id) local = fail(e, ZB_EDEVICE, "injected local failure (ZB_FAIL_EXCHANGE)");
#endif
  const bool self = P == 1 && !(e->cfg.flags & ZB_CFG_RCCL_SELF);
  if (local == ZB_OK) local = outbox_plan(e, kind, sb, sc, &n, &total, self);
  if (local == ZB_OK && n) local = grow_dev(e, &e->xsend, &e->xsend_cap, total);
  if (local == ZB_OK && n) local = outbox_emit(e, kind, e->xsend, e->xsend_cap);
  if (P == 1 && !(e->cfg.flags & ZB_CFG_RCCL_SELF)) {  // no peer: the batch is this partition's own inbox
    if (local != ZB_OK || n == 0) return local;
    std::vector<uint64_t> rcounts{sc[0]}, roffs{0};
    int rc = require_idle(e);
    if (rc == ZB_OK) rc = ensure_stores(e);
    if (rc == ZB_OK) rc = maintain(e, false);
    if (rc == ZB_OK) rc = deliver(e, kind, e->xsend, rcounts, roffs, received);
    return rc;
  }
  if (local != ZB_OK) for (int q = 0; q < P; q++) sb[q] = sc[q] = 0;
  const std::string local_err = local != ZB_OK ? e->err : std::string();
  // 1. agreement + sizes: every rank sends every peer (bytes, commands, status) for it; always posted
  std::vector<uint64_t> tri(4 * 64, 0);
  for (int q = 0; q < P; q++) { tri[4 * q] = sb[q]; tri[4 * q + 1] = sc[q]; tri[4 * q + 2] = (uint64_t)(uint32_t)local; }
  if (hipMemcpyAsync(e->d_xcounts, tri.data(), 4 * P * 8, hipMemcpyHostToDevice, e->stream) != hipSuccess)
    local = local != ZB_OK ? local : ZB_EDEVICE;  // the sizes may be stale: the status still travels below
  ncclResult_t nr = ncclGroupStart();
  for (int q = 0; q < P && nr == ncclSuccess; q++) {
    nr = ncclSend(e->d_xcounts + 4 * q, 4, ncclUint64, q, e->comm, e->stream);
    if (nr == ncclSuccess) nr = ncclRecv(e->d_xcounts + 256 + 4 * q, 4, ncclUint64, q, e->comm, e->stream);
  }
  if (nr == ncclSuccess) nr = ncclGroupEnd();
  if (nr != ncclSuccess) return comm_fail(e, "exchange sizes", nr);
  std::vector<uint64_t> rtri(4 * 64, 0);
  if (hipMemcpyAsync(rtri.data(), e->d_xcounts + 256, 4 * P * 8, hipMemcpyDeviceToHost, e->stream) != hipSuccess ||
      hipStreamSynchronize(e->stream) != hipSuccess)
    return comm_fail(e, "exchange sizes download", ncclSystemError);
  int peer_failed = -1;
  uint64_t rbytes = 0;
  std::vector<uint64_t> rcounts(P), roffs(P);
  for (int q = 0; q < P; q++) {
    roffs[q] = rbytes;
    rcounts[q] = rtri[4 * q + 1];
    rbytes += rtri[4 * q];
    if (rtri[4 * q + 2] != 0 && peer_failed < 0) peer_failed = q;
  }
  // 2. the receive side may fail locally too: agree once more (max of the statuses) before any byte moves
  if (peer_failed < 0 && local == ZB_OK && rbytes) local = grow_dev(e, &e->xrecv, &e->xrecv_cap, rbytes);
  uint64_t st = (local != ZB_OK || peer_failed >= 0) ? 1 : 0;
  if (hipMemcpyAsync(e->d_xcounts + 448, &st, 8, hipMemcpyHostToDevice, e->stream) != hipSuccess)
    return comm_fail(e, "exchange status upload", ncclSystemError);
  nr = ncclAllReduce(e->d_xcounts + 448, e->d_xcounts + 448, 1, ncclUint64, ncclMax, e->comm, e->stream);
  if (nr != ncclSuccess) return comm_fail(e, "exchange status", nr);
  if (hipMemcpyAsync(&st, e->d_xcounts + 448, 8, hipMemcpyDeviceToHost, e->stream) != hipSuccess ||
      hipStreamSynchronize(e->stream) != hipSuccess)
    return comm_fail(e, "exchange status download", ncclSystemError);
  if (st != 0) {
    if (local != ZB_OK) return fail(e, local, "exchange: " + (local_err.empty() ? std::string("receive buffer") : local_err));
    if (peer_failed >= 0)
      return fail(e, ZB_EDEVICE, "exchange: partition " + std::to_string(peer_failed) + " failed locally");
    return fail(e, ZB_EDEVICE, "exchange: a peer failed to size its receive buffer");
  }
  // 3. batches: one per (source, target) pair; received in source-rank order = canonical delivery order
  nr = ncclGroupStart();
  uint64_t so = 0;
  for (int q = 0; q < P && nr == ncclSuccess; q++) {
    if (sb[q]) nr = ncclSend(e->xsend + so, sb[q], ncclUint8, q, e->comm, e->stream);
    if (nr == ncclSuccess && rtri[4 * q]) nr = ncclRecv(e->xrecv + roffs[q], rtri[4 * q], ncclUint8, q, e->comm, e->stream);
    so += sb[q];
  }
  if (nr == ncclSuccess) nr = ncclGroupEnd();
  if (nr != ncclSuccess) return comm_fail(e, "exchange records", nr);
  if (hipStreamSynchronize(e->stream) != hipSuccess) return comm_fail(e, "exchange sync", ncclSystemError);
  // 4. delivery is local (no further collective in this call)
  int rc = ZB_OK;
  if (rbytes) {
    rc = require_idle(e);
    if (rc == ZB_OK) rc = ensure_stores(e);
    if (rc == ZB_OK) rc = maintain(e, false);
    if (rc == ZB_OK) rc = deliver(e, kind, e->xrecv, rcounts, roffs, received);
  }
  return rc;
}

int zb_log_release(zb_engine* e, int64_t position) {
  if (!e) return ZB_EINVAL;
  // only processed records can leave the window (the engine still reads the unprocessed ones)
  if (position > e->host_hdr.begin) return fail(e, ZB_EINVAL, "cannot release unprocessed records");
  e->released = std::max(e->released, position);
  return ZB_OK;
}

int zb_log_start(zb_engine* e, int64_t position) {
  if (!e) return ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  if (e->failed) return fail(e, ZB_EPROCESSING, "partition stopped after a processing failure: " + e->err);
  if (e->host_hdr.begin != e->host_hdr.end) return fail(e, ZB_EINVAL, "partition not quiescent");
  if (e->staged_pending && !e->staged.empty()) return fail(e, ZB_EINVAL, "staged input not injected yet");
  if (position < e->host_hdr.end) return fail(e, ZB_EINVAL, "log positions only grow");
  if (std::max(e->released, e->win_base) < e->host_hdr.end) return fail(e, ZB_EINVAL, "unreleased records in the window");
  if (e->on) {  // queued exchange commands carry order keys relative to the old base: take them first
    uint64_t n_open = 0, n_corr = 0;
    int rc = zb_outbox_count(e, ZB_XCHG_OPEN, &n_open);
    if (rc == ZB_OK) rc = zb_outbox_count(e, ZB_XCHG_CORRELATE, &n_corr);
    if (rc != ZB_OK) return rc;
    if (n_open || n_corr) return fail(e, ZB_EINVAL, "untaken exchange commands in the outbox: exchange them first");
  }
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  e->host_hdr.begin = e->host_hdr.end = e->host_hdr.gen_end = position;
  e->win_base = e->released = position;
  e->ob_pos_base[0] = e->ob_pos_base[1] = position;
  e->ranges.clear();
  e->req_runs.clear();
  e->req_lo = e->req_n = 0;
  e->cmd_pool.clear();
  rebias(e);
  HIPCHECK(e, upload_async(e, e->hdr + (e->wave & 1), &e->host_hdr, sizeof(WaveHdr)));
  HIPCHECK(e, hipStreamSynchronize(e->stream));
  return ZB_OK;
}

int zb_compact(zb_engine* e) {
  if (!e) return ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  if (e->failed) return fail(e, ZB_EPROCESSING, "partition stopped after a processing failure: " + e->err);
  if (e->host_hdr.begin != e->host_hdr.end) return fail(e, ZB_EINVAL, "partition not quiescent");
  return maintain(e, true);
}

int zb_read_memory_stats(zb_engine* e, zb_memory_stats* out) {
  if (!e || !out) return ZB_EINVAL;
  zb_memory_stats m{};
  m.log_window_begin = e->win_base;
  m.log_end = e->host_hdr.end;
  m.log_capacity = e->cfg.log_capacity;
  m.rows_allocated = (uint64_t)e->host_hdr.rows_next;
  m.row_capacity = e->cfg.row_capacity;
  m.arena_used = (uint64_t)e->host_hdr.arena_next + (e->cfg.arena_bytes - e->arena_top);
  m.arena_bytes = e->cfg.arena_bytes;
  m.records_total = e->records_total;
  m.rows_total = e->rows_total;
  m.arena_total = e->arena_total;
  m.compactions = e->compactions;
  *out = m;
  return ZB_OK;
}

int zb_counters(zb_engine* e, int64_t out[8]) {
  if (!e || !out) return ZB_EINVAL;
  uint64_t s[8];
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  HIPCHECK(e, hipMemcpy(s, e->dstats, sizeof(s), hipMemcpyDeviceToHost));
  out[0] = (int64_t)s[2];
  out[1] = (int64_t)s[1];
  out[2] = (int64_t)s[7];
  out[3] = e->host_hdr.wf_next;
  out[4] = e->host_hdr.job_next;
  out[5] = e->host_hdr.rows_next;
  out[6] = e->host_hdr.arena_next;
  out[7] = e->host_hdr.end;
  return ZB_OK;
}

}  // extern "C"

// ---- element-instance index read-back and snapshots
namespace {

int require_quiescent(zb_engine* e) {
  if (e->failed) return fail(e, ZB_EPROCESSING, "partition stopped after a processing failure: " + e->err);
  if (e->host_hdr.begin != e->host_hdr.end) return fail(e, ZB_EINVAL, "partition not quiescent");
  return ZB_OK;
}

}  // namespace

extern "C" {

int zb_read_instances(zb_engine* e, uint8_t* buf, size_t cap, size_t* len, uint64_t* count) {
  if (!e || !len) return ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  const uint64_t rows = (uint64_t)e->host_hdr.rows_next;
  *len = 0;
  if (count) *count = 0;
  if (rows == 0) return ZB_OK;
  uint32_t* d_count = nullptr;
  int64_t* d_keys = nullptr;
  uint32_t* d_rows = nullptr;
  zb_rec* d_descs = nullptr;
  InstHead* d_heads = nullptr;
  uint64_t *d_len = nullptr, *d_off = nullptr;
  uint8_t* d_out = nullptr;
  zb_record_header* d_hdrs = nullptr;
  void* d_tmp = nullptr;
  int rc = ZB_OK;
  auto cleanup = [&]() {
    void* ps[] = {d_count, d_keys, d_rows, d_descs, d_heads, d_len, d_off, d_out, d_hdrs, d_tmp};
    for (void* q : ps)
      if (q) (void)hipFree(q);
  };
  do {
    if (hipMalloc(&d_count, 4) != hipSuccess || hipMalloc(&d_keys, rows * 8) != hipSuccess ||
        hipMalloc(&d_rows, rows * 4) != hipSuccess) { rc = fail(e, ZB_ENOMEM, "read_instances buffers"); break; }
    if (hipMemsetAsync(d_count, 0, 4, e->stream) != hipSuccess) { rc = ZB_EDEVICE; break; }
    LiveParams lp{};
    lp.rmeta = e->rmeta; lp.rkeys = e->rkeys; lp.rows = rows; lp.count = d_count; lp.cap = rows;
    lp.keys = d_keys; lp.row_of = d_rows;
    launch_live_rows(lp, e->stream);
    uint32_t live = 0;
    if (hipMemcpyAsync(&live, d_count, 4, hipMemcpyDeviceToHost, e->stream) != hipSuccess ||
        hipStreamSynchronize(e->stream) != hipSuccess) { rc = fail(e, ZB_EDEVICE, "read_instances count"); break; }
    if (count) *count = live;
    if (live == 0) break;
    // key order (ElementInstanceIndex is a hash map; the dump is canonicalised by key)
    std::vector<int64_t> keys(live);
    std::vector<uint32_t> rws(live);
    if (hipMemcpy(keys.data(), d_keys, live * 8, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(rws.data(), d_rows, live * 4, hipMemcpyDeviceToHost) != hipSuccess) { rc = ZB_EDEVICE; break; }
    std::vector<uint32_t> ord(live);
    for (uint32_t i = 0; i < live; i++) ord[i] = i;
    std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return keys[a] < keys[b]; });
    std::vector<uint32_t> sorted_rows(live);
    for (uint32_t i = 0; i < live; i++) sorted_rows[i] = rws[ord[i]];
    if (hipMemcpy(d_rows, sorted_rows.data(), live * 4, hipMemcpyHostToDevice) != hipSuccess) { rc = ZB_EDEVICE; break; }
    if (hipMalloc(&d_descs, live * sizeof(zb_rec)) != hipSuccess || hipMalloc(&d_heads, live * sizeof(InstHead)) != hipSuccess ||
        hipMalloc(&d_len, (live + 1) * 8) != hipSuccess || hipMalloc(&d_off, (live + 1) * 8) != hipSuccess ||
        hipMalloc(&d_hdrs, live * sizeof(zb_record_header)) != hipSuccess) { rc = fail(e, ZB_ENOMEM, "read_instances"); break; }
    lp.n = live; lp.descs = d_descs; lp.heads = d_heads;
    launch_row_descs(lp, e->stream);
    // values: the serializer over the descriptors (size pass, scan, write pass)
    SerParams sp{};
    sp.log = d_descs; sp.arena = e->arena; sp.arena_bytes = e->cfg.arena_bytes; sp.elems = e->d_elems.p; sp.wfs = e->d_wfs.p;
    sp.queries = e->d_queries.p; sp.pool = e->d_pool.p; sp.ranges = nullptr; sp.nranges = 0;
    sp.cmd_pool = nullptr; sp.start = 0; sp.count = live;
    SerParams sz = sp;
    sz.lengths = (uint32_t*)d_off;
    launch_ser_size(sz, e->stream);
    std::vector<uint32_t> lens(live);
    if (hipMemcpyAsync(lens.data(), d_off, live * 4, hipMemcpyDeviceToHost, e->stream) != hipSuccess ||
        hipStreamSynchronize(e->stream) != hipSuccess) { rc = ZB_EDEVICE; break; }
    std::vector<uint64_t> offs(live + 1, 0);
    for (uint32_t i = 0; i < live; i++) offs[i + 1] = offs[i] + lens[i];
    const uint64_t total = offs[live];
    *len = (size_t)(total + (uint64_t)live * sizeof(InstHead));
    if (!buf || cap < *len) { rc = ZB_ENOMEM; break; }
    if (hipMalloc(&d_out, total + 1) != hipSuccess ||
        hipMemcpy(d_len, offs.data(), (live + 1) * 8, hipMemcpyHostToDevice) != hipSuccess) { rc = ZB_ENOMEM; break; }
    SerParams wr = sp;
    wr.offsets = d_len; wr.out = d_out; wr.headers = d_hdrs;
    launch_ser_write(wr, e->stream);
    std::vector<InstHead> heads(live);
    std::vector<uint8_t> vals(total);
    if (hipMemcpyAsync(heads.data(), d_heads, live * sizeof(InstHead), hipMemcpyDeviceToHost, e->stream) != hipSuccess ||
        (total && hipMemcpyAsync(vals.data(), d_out, total, hipMemcpyDeviceToHost, e->stream) != hipSuccess) ||
        hipStreamSynchronize(e->stream) != hipSuccess) { rc = fail(e, ZB_EDEVICE, "read_instances copy"); break; }
    size_t o = 0;
    for (uint32_t i = 0; i < live; i++) {
      InstHead h = heads[i];
      h.value_len = lens[i];
      std::memcpy(buf + o, &h, sizeof(h));
      o += sizeof(h);
      std::memcpy(buf + o, vals.data() + offs[i], lens[i]);
      o += lens[i];
    }
  } while (0);
  cleanup();
  return rc;
}

}  // extern "C"

namespace {
constexpr uint64_t SNAP_MAGIC = 0x32504e53425a4755ull;  // "UGZBSNP2"
// A snapshot holds the live state only (taken right after a forced compaction): the element-instance rows
// [0, live) (state, keys and scope state; the children links are rebuilt on restore), the arena's dynamic region [STATIC, arena_next) (the static region comes with the deployments),
// the live job states as (key, state) pairs, and the store entries (chains are rebuilt on restore).
struct SnapHead {
  uint64_t magic;
  uint64_t model_hash;    // deployments the snapshot was taken with (zb_restore checks)
  WaveHdr hdr;
  uint64_t stats[8];
  int64_t epoch, msg_key_next;
  uint64_t sub_count, msg_count;
  uint64_t rows, arena_dyn;
  uint64_t jobs;          // live job states (ZB_CFG_JOB_PROCESSOR)
  uint64_t records_total, rows_total, arena_total;
};

uint64_t model_hash(const zb_engine* e) {  // FNV-1a over the deployed tables
  uint64_t h = 1469598103934665603ull;
  auto mix = [&](const void* p, size_t n) {
    const uint8_t* b = (const uint8_t*)p;
    for (size_t i = 0; i < n; i++) { h ^= b[i]; h *= 1099511628211ull; }
  };
  mix(e->model.elems.data(), e->model.elems.size() * sizeof(DevElem));
  mix(e->model.workflows.data(), e->model.workflows.size() * sizeof(DevWorkflow));
  mix(e->model.pool.data(), e->model.pool.size());
  mix(e->static_blobs.data(), e->static_blobs.size());
  return h;
}

size_t snap_bytes(const SnapHead& h) {
  return sizeof(h) + h.rows * (sizeof(RowMeta) + sizeof(RowKeys) + sizeof(RowAux)) + h.arena_dyn +
         h.jobs * (sizeof(int64_t) + 1) + h.sub_count * sizeof(SubEntry) + h.msg_count * sizeof(MsgEntry);
}
}  // namespace

extern "C" {

int zb_snapshot(zb_engine* e, uint8_t* buf, size_t cap, size_t* len) {
  if (!e || !len) return ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  int rc = require_quiescent(e);
  if (rc != ZB_OK) return rc;
  if (e->staged_pending && !e->staged.empty()) return fail(e, ZB_EINVAL, "staged input not injected yet");
  rc = maintain(e, true);  // live state only
  if (rc != ZB_OK) return rc;
  SnapHead h{};
  h.magic = SNAP_MAGIC;
  h.model_hash = model_hash(e);
  h.hdr = e->host_hdr;
  HIPCHECK(e, hipMemcpy(h.stats, e->dstats, sizeof(h.stats), hipMemcpyDeviceToHost));
  h.epoch = e->epoch;
  h.msg_key_next = e->msg_key_next;
  h.sub_count = e->subs ? e->sub_count : 0;
  h.msg_count = e->msgs ? e->msg_count : 0;
  h.rows = (uint64_t)e->host_hdr.rows_next;
  h.arena_dyn = (uint64_t)e->host_hdr.arena_next - STATIC_ARENA_BYTES;
  h.records_total = e->records_total; h.rows_total = e->rows_total; h.arena_total = e->arena_total;
  // live job states: collected on the device (the table itself is sized by capacity)
  if (e->jobs.keys) {
    const uint64_t slots = e->jobs.mask + 1;
    rc = grow(e, &e->c_scratch, &e->c_scratch_cap, slots * (sizeof(int64_t) + 1));
    if (rc != ZB_OK) return rc;
    if (!e->c_count) HIPCHECK(e, hipMalloc(&e->c_count, sizeof(uint32_t)));
    HIPCHECK(e, hipMemsetAsync(e->c_count, 0, sizeof(uint32_t), e->stream));
    launch_job_collect(e->jobs, (int64_t*)e->c_scratch, e->c_scratch + slots * sizeof(int64_t), e->c_count, e->stream);
    uint32_t n = 0;
    HIPCHECK(e, hipMemcpyAsync(&n, e->c_count, sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
    HIPCHECK(e, hipStreamSynchronize(e->stream));
    h.jobs = n;
  }
  const size_t need = snap_bytes(h);
  *len = need;
  if (!buf || cap < need) return ZB_ENOMEM;
  uint8_t* o = buf;
  std::memcpy(o, &h, sizeof(h)); o += sizeof(h);
  auto get = [&](const void* src, size_t n) -> bool {
    if (n && hipMemcpy(o, src, n, hipMemcpyDeviceToHost) != hipSuccess) return false;
    o += n;
    return true;
  };
  bool ok = get(e->rmeta, h.rows * sizeof(RowMeta)) && get(e->rkeys, h.rows * sizeof(RowKeys)) &&
            get(e->raux, h.rows * sizeof(RowAux)) && get(e->arena + STATIC_ARENA_BYTES, h.arena_dyn);
  if (!ok) return fail(e, ZB_EDEVICE, "snapshot copy");
  if (h.jobs) {
    const uint64_t slots = e->jobs.mask + 1;
    ok = get(e->c_scratch, h.jobs * sizeof(int64_t)) && get(e->c_scratch + slots * sizeof(int64_t), h.jobs);
    if (!ok) return fail(e, ZB_EDEVICE, "snapshot copy (job states)");
  }
  ok = get(e->subs, h.sub_count * sizeof(SubEntry)) && get(e->msgs, h.msg_count * sizeof(MsgEntry));
  if (!ok) return fail(e, ZB_EDEVICE, "snapshot copy (message stores)");
  return ZB_OK;
}

int zb_restore(zb_engine* e, const uint8_t* buf, size_t len) {
  if (!e || !buf || len < sizeof(SnapHead)) return ZB_EINVAL;
  HIPCHECK(e, hipSetDevice(e->cfg.device));
  SnapHead h;
  std::memcpy(&h, buf, sizeof(h));
  if (h.magic != SNAP_MAGIC) return fail(e, ZB_EINVAL, "not a zb snapshot");
  e->seg_pending = false;  // (the restored log replaces it)
  if (h.model_hash != model_hash(e)) return fail(e, ZB_EINVAL, "snapshot was taken with other deployments");
  if (len < snap_bytes(h)) return fail(e, ZB_EINVAL, "truncated snapshot");
  if (h.rows > e->cfg.row_capacity || STATIC_ARENA_BYTES + h.arena_dyn > e->cfg.arena_bytes)
    return fail(e, ZB_ENOMEM, "snapshot exceeds this engine's capacities");
  if (h.jobs && !e->jobs.keys)
    return fail(e, ZB_EINVAL, "snapshot holds job states: restore into an engine with ZB_CFG_JOB_PROCESSOR");
  if (e->jobs.keys && h.jobs > (e->jobs.mask + 1) / 2) return fail(e, ZB_ENOMEM, "snapshot job states exceed the job table");
  int rc = zb_reset(e, 0);
  if (rc != ZB_OK) return rc;
  if (h.sub_count || h.msg_count) {
    rc = ensure_stores(e);
    if (rc != ZB_OK) return rc;
    if (h.sub_count > e->store_cap || h.msg_count > e->store_cap)
      return fail(e, ZB_ENOMEM, "snapshot message stores exceed this engine's store capacity");
  }
  const uint8_t* o = buf + sizeof(h);
  auto put = [&](void* dst, size_t n) -> bool {
    if (n && hipMemcpy(dst, o, n, hipMemcpyHostToDevice) != hipSuccess) return false;
    o += n;
    return true;
  };
  bool ok = put(e->rmeta, h.rows * sizeof(RowMeta)) && put(e->rkeys, h.rows * sizeof(RowKeys)) &&
            put(e->raux, h.rows * sizeof(RowAux)) && put(e->arena + STATIC_ARENA_BYTES, h.arena_dyn);
  if (!ok) return fail(e, ZB_EDEVICE, "restore copy");
  if (h.rows) {  // the children lists are not in the snapshot: rebuilt from the parents (as after a compaction)
    CompactParams c = compact_params(e);
    c.live_rows = h.rows;
    HIPCHECK(e, hipMemsetAsync(e->rlink, 0xff, h.rows * sizeof(RowLink), e->stream));
    launch_row_relink(c, e->stream);
  }
  if (h.jobs) {
    rc = grow(e, &e->c_scratch, &e->c_scratch_cap, h.jobs * (sizeof(int64_t) + 1));
    if (rc != ZB_OK) return rc;
    ok = put(e->c_scratch, h.jobs * sizeof(int64_t)) && put(e->c_scratch + h.jobs * sizeof(int64_t), h.jobs);
    if (!ok) return fail(e, ZB_EDEVICE, "restore copy (job states)");
    launch_job_fill(e->jobs, (const int64_t*)e->c_scratch, e->c_scratch + h.jobs * sizeof(int64_t), (uint32_t)h.jobs,
                    e->derr, e->stream);
  }
  if (h.sub_count || h.msg_count) {
    ok = put(e->subs, h.sub_count * sizeof(SubEntry)) && put(e->msgs, h.msg_count * sizeof(MsgEntry));
    if (!ok) return fail(e, ZB_EDEVICE, "restore copy (message stores)");
    launch_chains(e->msgs, h.msg_count, e->msg_head, e->msg_next, e->subs, h.sub_count, e->sub_head, e->sub_next,
                  e->head_mask, e->stream);
  }
  e->host_hdr = h.hdr;
  e->host_hdr.begin = e->host_hdr.gen_end = e->host_hdr.end;
  // the log itself lives in the logstream, not in the snapshot: the window starts empty at its end
  e->win_base = e->released = e->host_hdr.end;
  e->ob_pos_base[0] = e->ob_pos_base[1] = e->host_hdr.end;
  rebias(e);
  e->epoch = std::max(e->epoch, h.epoch);
  e->msg_key_next = h.msg_key_next;
  e->sub_count = h.sub_count; e->msg_count = h.msg_count;
  e->records_total = h.records_total; e->rows_total = h.rows_total; e->arena_total = h.arena_total;
  e->rows_mark = h.rows;  // (a snapshot holds live state only)
  e->arena_mark = STATIC_ARENA_BYTES + h.arena_dyn;
  e->wave = 0;  // (and the per-wave job queues of both parities empty, whatever wave ran last)
  HIPCHECK(e, hipMemsetAsync(e->job_counts, 0, JOB_COUNTS * sizeof(uint32_t), e->stream));
  HIPCHECK(e, hipMemcpy(e->dstats, h.stats, sizeof(h.stats), hipMemcpyHostToDevice));
  return finish_batch(e);
}

}  // extern "C"
