// zb_kernels.hpp — kernel parameter blocks and launchers shared by zb_engine.cpp and the .hip files.
#pragma once
#include <hip/hip_runtime.h>

#include "zb_device.hpp"

namespace zbg {

// A deferred default output merge: k_wave reserves the result blob (upper-bound sized), k_merge fills it.
struct MergeJob {
  uint32_t dst;   // result blob ref (arena offset / 8)
  uint32_t src;   // source (job / message payload) ref
  uint32_t tgt;   // target (flow scope payload) ref
  uint32_t cap;   // bytes reserved after the 4-byte length word
};

// k_cond decision word, stored in the row-self link of a GATEWAY_ACTIVATED record
constexpr uint32_t COND_VALID = 1u << 31;
constexpr uint32_t COND_INCIDENT = 1u << 30;
constexpr uint32_t COND_UNSUPPORTED = 1u << 17;
// flow: [15:0] chosen sequence flow elem; incident: [29:27] code [26:23] a [22:19] b [15:0] query

constexpr int WAVE_TILE = 256;   // records per tile (one per thread of a 256-thread workgroup)
constexpr int WAVE_GRID = 1024;  // workgroups of k_process / k_emit; workgroup b owns tiles [b*T/G, (b+1)*T/G)

// One staged output record of k_process (48 B): descriptor + row links + what k_emit fills in.
struct Slot {
  zb_rec d;
  uint32_t rself, rscope;
  uint8_t flags, ord, rord, pad;
  uint32_t pad2;
};
static_assert(sizeof(Slot) == 48, "Slot is 48 bytes");

// Per-record side information of k_process, written only when a merge or an incident detail exists.
struct ItemInfo {
  uint32_t m_src, m_tgt, m_len, m_bytes;  // merge (m_bytes == 0: none)
  int64_t d_pos;                          // incident detail
  uint16_t d_q;
  uint8_t d_type, d_code, d_a, d_b, has_detail, ns;
};
static_assert(sizeof(ItemInfo) == 32, "ItemInfo is 32 bytes");

// Per-workgroup totals of k_process (each workgroup owns one contiguous range of 256-record tiles,
// the same range in k_emit), and their exclusive prefix computed by k_scan.
struct BlockAgg {
  uint64_t bytes;
  uint32_t rec, wf, job, row, merges, conds;
  uint32_t transitions, completed, created, pad;
};
static_assert(sizeof(BlockAgg) == 48, "BlockAgg is 48 bytes");
struct BlockOff {
  uint64_t rec, wf, job, row, bytes;
  uint32_t merges, conds;
};
static_assert(sizeof(BlockOff) == 48, "BlockOff is 48 bytes");

// Count word of one record (k_process -> k_emit): bits [0,3) outputs, [3,6) wf keys, [6,9) job keys,
// [9,12) new rows, 12 merge, 13 incident detail, [14,17) condition jobs, [32,64) arena bytes.
constexpr int CW_NWF = 3, CW_NJOB = 6, CW_NROW = 9, CW_MERGE = 12, CW_DETAIL = 13, CW_NCOND = 14;

struct WaveParams {
  zb_rec* log;
  uint64_t* links;        // per record: row_self | row_scope << 32
  RowMeta* rmeta;
  RowKeys* rkeys;
  uint8_t* arena;
  const DevElem* elems;
  const DevWorkflow* wfs;
  const uint16_t* cond_flows;
  const uint32_t* code;
  const DevConst* consts;
  const DevQuery* queries;
  const DevFilter* filters;
  const uint8_t* pool;
  WaveHdr* hdr;            // [2], double buffered
  uint32_t* err;           // sticky DevErr flags
  uint64_t* err_info;      // min over failing records of (position << 8 | site)
  uint64_t* stats;         // [8] transitions, completed, created, merges, merge_bytes, cond_bytes, waves
  // wave staging (indexed by record - begin; wave_cap records)
  uint64_t* cw;            // count words
  Slot* stage;             // [wave_cap][2] output slots
  ItemInfo* info;          // [wave_cap] side info (sparse)
  BlockAgg* block_agg;     // [WAVE_GRID]
  BlockOff* block_off;     // [WAVE_GRID]
  MergeJob* merge_jobs;    // [2][job_cap], by wave parity
  uint32_t* merge_count;   // [2]
  uint64_t* cond_jobs;     // [2][job_cap] record indices of conditional GATEWAY_ACTIVATED records
  uint32_t* cond_count;    // [2]
  uint64_t job_cap;
  uint64_t log_cap, row_cap, arena_cap, wave_cap;
  int64_t wave;
  // open-subscription outbox (SUBSCRIBE_TO_INTERMEDIATE_MESSAGE side effects), zb_msg.hpp
  zb_exchange_rec* obox;
  uint64_t* okeys;
  uint32_t* on;
  uint64_t ocap;
  int32_t partition_id, partition_count;
};

// message stores (zb_msg.hip): MessageSubscriptionDataStore / MessageDataStore entries
struct SubEntry {   // 48 B
  uint64_t h;       // name_ck_hash(messageName, correlationKey)
  int64_t wik, aik;
  int64_t pos;      // log position of the OPEN command
  uint32_t blob;    // subscription blob ref (wfp, elem, token, name, correlation key)
  uint32_t idx;     // insertion index
};
struct MsgEntry {   // 32 B, messages stored with ttl > 0
  uint64_t h;
  int64_t key;
  int64_t pos;      // log position of the PUBLISH command
  uint32_t blob;    // message blob ref
  uint32_t pad;
};
struct MsgParams {
  zb_rec* log;
  uint64_t* links;
  uint8_t* arena;
  const zb_exchange_rec* in;  // delivered commands (k_msg_open, k_wis_inject)
  int64_t n, base;            // batch size, log position of its first command
  uint64_t arena_base;        // byte offset of the batch's blobs
  SubEntry* subs;
  uint32_t *sub_head, *sub_next;
  uint64_t sub_mask, sub_count, sub_cap;
  MsgEntry* msgs;
  uint32_t *msg_head, *msg_next;
  uint64_t msg_mask, msg_count, msg_cap;
  int64_t ttl, key_base;      // publish batch
  zb_exchange_rec* obox;      // correlate outbox
  uint64_t* okeys;
  uint32_t* on;
  uint64_t ocap;
  uint32_t* err;
};

void launch_msg_open(const MsgParams& p, hipStream_t stream);
void launch_msg_publish(const MsgParams& p, hipStream_t stream);
void launch_wis_inject(const MsgParams& p, hipStream_t stream);
void launch_outbox_gather(const zb_exchange_rec* src, const uint32_t* idx, zb_exchange_rec* dst, uint64_t n,
                          hipStream_t stream);
void launch_outbox_bounds(const uint64_t* keys, uint64_t n, uint64_t* first, int parts, hipStream_t stream);
void launch_iota(uint32_t* p, uint64_t n, hipStream_t stream);


void launch_process(const WaveParams& p, hipStream_t stream);
void launch_scan(const WaveParams& p, hipStream_t stream);
void launch_emit(const WaveParams& p, hipStream_t stream);
void launch_merge(const WaveParams& p, hipStream_t stream);
void launch_cond(const WaveParams& p, hipStream_t stream);

// submitted CREATE commands: one range per zb_submit_creates call (serialization of their values)
struct CmdRange {
  int64_t pos_begin, pos_end;
  int64_t workflow_key;
  int32_t version;
  uint16_t pid_len;
  uint16_t pad;
  uint32_t pid_off;       // in the engine's command string pool (device copy in SerParams.cmd_pool)
  uint32_t pad2;
};

struct SerParams {
  const zb_rec* log;
  const uint8_t* arena;
  const DevElem* elems;
  const DevWorkflow* wfs;
  const DevQuery* queries;
  const uint8_t* pool;
  const CmdRange* ranges;
  int32_t nranges;
  const uint8_t* cmd_pool;
  int64_t start, count;
  const uint64_t* offsets;  // exclusive offsets of value bytes (count+1), write pass
  uint32_t* lengths;        // size pass output
  uint8_t* out;
  zb_record_header* headers;
};

void launch_ser_size(const SerParams& p, hipStream_t stream);
void launch_ser_write(const SerParams& p, hipStream_t stream);

struct InjectParams {
  zb_rec* log;
  uint64_t* links;
  uint8_t* arena;
  const zb_rec* staged;
  const uint8_t* staged_arena;
  int64_t n;
  int64_t log_base;       // where the staged records go
  uint64_t arena_base;    // byte offset in the arena for the staged payload blobs
  uint64_t staged_bytes;
};

void launch_inject(const InjectParams& p, hipStream_t stream);

// ---- trajectory path (zb_traj.hip): a batch of CREATEs on an idle partition, run to quiescence
constexpr int TRAJ_WG = 256;  // instances per workgroup (one per thread)
constexpr int TR = 4;         // element instances per workflow instance held in registers
constexpr int TF = 2;         // records per workflow instance per generation
constexpr int CLS_MAX = 8;          // trajectory classes of a class batch
constexpr int CLS_MAX_SPLITS = 8;   // exclusive splits a class key covers
constexpr int CLS_ROW = 4096;       // agg / mgen row of one class (>= generations of a batch)
constexpr int CLS_BLK_WG = 16;      // instance workgroups per emit block (class segments per block)
constexpr int CLS_HB = 64;          // key histogram banks (workgroup b adds into bank b % CLS_HB)

// One record of a traced trajectory (uniform / class batch), with symbolic keys and payload refs that
// the template emit pass (k_tmpl) resolves per instance: keys SYMK_WF / SYMK_JOB | generation << 4 |
// ordinal (the ordinal-th key the instance creates in that generation), NOK, or SYM_CMDPOS (the CREATE
// command's log position); payloads PAY_CREATE, PAY_MERGE | generation, or a literal (static) ref.
struct TmplRec {
  uint32_t key, scope, inst, payload;
  uint16_t elem;
  uint8_t intent, kind;
  uint32_t pad[3];
};
constexpr int TSTAT = 8;  // per-class trace statistics: transitions, completed, created, merges, split visits

// Class batch (zb_traj.hip): dense classes of the outcome keys present in the batch.
struct ClsPlan {
  uint32_t nc, slots;       // classes; emit slots (every (block, class) segment padded to a multiple of 64)
  uint32_t key[CLS_MAX];    // outcome key of class c
  uint32_t n[CLS_MAX];      // instances of class c
  uint32_t rep[CLS_MAX];    // representative (first) instance of class c
  uint64_t lensum[CLS_MAX]; // CREATE payload bytes of the instances of class c (condition statistics)
  uint8_t cid[256];         // key -> class (0xff: absent)
};

struct TrajCtl {
  uint32_t flag;       // != 0: the count pass met something this path does not do -> wave path
  uint32_t wmax;       // generations of the batch
  uint64_t arena_next; // payload arena bump pointer (emit pass)
  uint64_t rows_next;  // row allocator (live element instances at the end)
  int64_t end, wf_next, job_next;  // log end and key generators after the batch (k_traj_base)
  uint64_t arena_start, rows_start;  // allocator values before the emit pass (a rerun restarts there)
  uint32_t regen;      // the emit pass met a non-flat merge: rerun it with the general merge
  uint32_t derr;       // DevErr flags of the (last) emit pass
  uint64_t st[6];      // emit pass statistics: transitions, completed, created, merges, merge bytes, cond bytes
};
struct TrajBase {      // generation w: log position of its follow-ups, key generator values
  int64_t pos, wf, job, mbase;  // mbase: arena byte offset of the batch's merge results of generation w
};

// Uniform batch (zb_traj.hip): the representative instance's default output merge of generation w,
// with symbolic source / target payloads (PAY_CREATE, PAY_MERGE | w', literal refs) and the slot
// stride that bounds every instance's result. The emit pass writes instance i's merge result of
// generation w at wbase[w].mbase + i * stride: no arena allocation (no atomic) on the hot path.
struct MergeGen {
  uint32_t src, tgt, stride, has;
};

struct TrajParams {
  zb_rec* log;
  uint8_t* arena;
  RowMeta* rmeta;
  RowKeys* rkeys;
  const DevElem* elems;
  const uint16_t* cond_flows;
  const uint32_t* code;
  const DevConst* consts;
  const DevQuery* queries;
  const DevFilter* filters;
  const uint8_t* pool;
  int64_t log_base, n;   // the batch: CREATE commands at [log_base, log_base + n)
  int64_t wf_start, job_start;
  int32_t cond;          // the model has exclusive splits (condition VM compiled into the kernels)
  int32_t cls;           // class batch (uniform process, exclusive splits on CREATE payloads): see ClsPlan
  int64_t uni;           // > 0: uniform batch of `uni` instances whose trajectories are data-independent;
                         // agg[w] holds one instance's counts (count pass over instance 0 only)
  int32_t nwg, wcap;     // workgroups, generations the count buffers hold
  uint64_t* agg;         // [wcap][nwg] workgroup totals: records | wf keys << 16 | job keys << 32
  uint32_t* wcount;      // [nwg] generations processed by each workgroup
  uint4* woff;           // [wcap][nwg] exclusive prefix of agg over workgroups
  uint4* wtot;           // [wcap] generation totals
  TrajBase* wbase;       // [wcap]
  TrajCtl* ctl;
  WaveHdr* hdr;          // the partition's current wave header (committed at the end)
  uint32_t* err;
  uint64_t* stats;
  uint64_t log_cap, row_cap, arena_cap;
  MergeGen* mgen;        // [wcap] uniform batch: per-generation merge slots (written by the count pass)
  uint64_t* wstats;      // [nwg][6] emit-pass statistics per workgroup (reduced by k_traj_commit)
  uint32_t max_create;   // longest CREATE payload of the batch (merge result bounds)
  int32_t nwg_e;         // emit-pass workgroups (class batch: class segments are padded)
  // class batch: the model's exclusive splits (element, key stride, radix = conditions + 2)
  int32_t nsplits, pad3;
  uint32_t split_elem[CLS_MAX_SPLITS], split_stride[CLS_MAX_SPLITS];
  ClsPlan* plan;
  uint8_t* ikey;         // [n] outcome key of every instance
  uint32_t* khist;       // [CLS_HB][256] instances per key
  uint32_t* krep;        // [CLS_HB][256] first instance per key
  uint64_t* cmask;       // [n / 64][CLS_MAX] per 64-instance group: ballot of the instances of class c
  uint32_t* woffw;       // [n / 64][CLS_MAX] instances of class c before the group
  uint32_t* wgcnt;       // [CLS_MAX][nwg] instances of class c in workgroup b
  uint32_t* wgoff;       // [CLS_MAX][nwg] exclusive prefix of wgcnt over workgroups
  uint32_t* perm;        // [slots] emit slot -> instance (~0: padding)
  uint32_t* segs;        // [nblk][CLS_MAX] first emit slot of the class-c segment of block b
  uint32_t* wcls;        // [slots / 64] class of every emit wave
  int32_t nblk, pad4;    // blocks of CLS_BLK_WG instance workgroups
  uint64_t* klen;        // [CLS_HB][256] CREATE payload bytes per key
  TmplRec* tmpl;         // [CLS_MAX][CLS_ROW][TF] traced records per class and generation
  uint32_t* cstat;       // [CLS_MAX][TSTAT] traced statistics per class
};

void launch_traj_count(const TrajParams& p, hipStream_t stream);
void launch_traj_count_uniform(const TrajParams& p, hipStream_t stream);
void launch_traj_count_classes(const TrajParams& p, hipStream_t stream);
void launch_traj_scan(const TrajParams& p, hipStream_t stream);
// ev_main (optional, 2 events): recorded around the main emit launch only
void launch_traj_emit(const TrajParams& p, hipStream_t stream, hipEvent_t* ev_main = nullptr);

}  // namespace zbg
