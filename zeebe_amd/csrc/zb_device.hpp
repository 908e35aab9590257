// zb_device.hpp — data layout shared by the host model compiler and the gfx950 kernels.
//
// Everything the wave kernels read is a flat, 8-byte-aligned table in HBM:
//   * DevElem[]      one 64-byte row per flow element of every deployed workflow (activityId index)
//   * DevWorkflow[]  workflow key / version / process element
//   * code[]         exclusive-gateway condition programs (json-el compiled to a jump program)
//   * DevConst[]     condition constants; DevQuery[]/DevFilter[] compiled json-path queries
//   * pool[]         byte pool: element ids, job types, message names, filter keys, string constants
#pragma once
#include <cstdint>

#include "../../include/zb_engine.h"

// ZB_DCHECK(cond, fmt, ...): a device-side bounds check of the guard-band build (ZB_CHECKED, zb_checked.hpp): a
// failed check prints its site and values and evaluates to false, so the caller skips the access instead of
// faulting; in the product build it is the constant true and costs nothing.
#ifdef ZB_CHECKED
#define ZB_DCHECK(cond, ...) \
  ((cond) ? true : (printf("ZB_DCHECK %s:%d: %s: ", __FILE__, __LINE__, #cond), printf(__VA_ARGS__), false))
#else
#define ZB_DCHECK(cond, ...) true
#endif

namespace zbg {

constexpr uint16_t NO_ELEM = 0xffff;
constexpr uint32_t NO_ROW = 0xffffffffu;
constexpr uint32_t NO_REF = 0xffffffffu;

// element kinds (FlowElementHandler.java:46-57 factories + the process)
enum Kind : uint8_t { EK_PROCESS = 0, EK_START = 1, EK_END = 2, EK_TASK = 3, EK_SUB = 4, EK_XOR = 5, EK_CATCH = 6,
                      EK_FLOW = 7,
                      EK_PAR = 8 };  // parallel gateway: EXTENSION (C4), rejected by the reference

// BpmnStep.java:20-54 (same order)
enum Step : uint8_t {
  ST_NONE = 0, ST_TAKE_SEQUENCE_FLOW, ST_CONSUME_TOKEN, ST_EXCLUSIVE_SPLIT, ST_CREATE_JOB, ST_APPLY_INPUT_MAPPING,
  ST_APPLY_OUTPUT_MAPPING, ST_ACTIVATE_GATEWAY, ST_SUBSCRIBE_TO_INTERMEDIATE_MESSAGE, ST_START_STATEFUL_ELEMENT,
  ST_TRIGGER_END_EVENT, ST_TRIGGER_START_EVENT, ST_TERMINATE_CONTAINED_INSTANCES, ST_TERMINATE_JOB_TASK,
  ST_TERMINATE_ELEMENT, ST_PROPAGATE_TERMINATION, ST_CANCEL_PROCESS, ST_COMPLETE_PROCESS,
  // EXTENSION (C4): GATEWAY_ACTIVATED of a parallel gateway forks; a flow into a join is an arrival
  ST_PARALLEL_SPLIT, ST_PARALLEL_MERGE,
  ST_UNBOUND = 255
};
constexpr int MAX_FANOUT = 63;  // outgoing flows of a parallel gateway (count word field)
constexpr int JOIN_SLOTS = 2;   // parallel joins directly inside one scope (RowAux counters)

// WorkflowInstanceIntent.java:18-38
enum WfIntent : uint8_t {
  WI_CREATE = 0, WI_CREATED = 1, WI_START_EVENT_OCCURRED = 2, WI_END_EVENT_OCCURRED = 3, WI_SEQUENCE_FLOW_TAKEN = 4,
  WI_GATEWAY_ACTIVATED = 5, WI_ELEMENT_READY = 6, WI_ELEMENT_ACTIVATED = 7, WI_ELEMENT_COMPLETING = 8,
  WI_ELEMENT_COMPLETED = 9, WI_ELEMENT_TERMINATING = 10, WI_ELEMENT_TERMINATED = 11, WI_CANCEL = 12,
  WI_CANCELING = 13, WI_UPDATE_PAYLOAD = 14, WI_PAYLOAD_UPDATED = 15
};
enum JobIntentG : uint8_t { JI_CREATE = 0, JI_CREATED = 1, JI_ACTIVATE = 2, JI_ACTIVATED = 3, JI_COMPLETE = 4,
                           JI_COMPLETED = 5, JI_TIME_OUT = 6, JI_TIMED_OUT = 7, JI_FAIL = 8, JI_FAILED = 9,
                           JI_UPDATE_RETRIES = 10, JI_RETRIES_UPDATED = 11, JI_CANCEL = 12, JI_CANCELED = 13 };
// job states of the job stream processor (JobStateController), one byte per job key ordinal ((key - 2) / 5)
enum JobStateG : uint8_t { JS_NONE = 0, JS_CREATED = 1, JS_ACTIVATED = 2, JS_FAILED = 3, JS_TIMED_OUT = 4 };

// record kind byte: [3:0] value type, [5:4] record type, 6 second record of a batch, 7 KIND_RAW: the value
// is serialized verbatim from the blob that follows the payload document blob (records submitted through
// zb_submit, and the follow-ups the reference writes as the re-encoded command value)
constexpr uint8_t KIND_RAW = 0x80;
__host__ __device__ inline uint8_t make_kind(uint8_t vt, uint8_t rt, bool cont) {
  return (uint8_t)(vt | (rt << 4) | (cont ? 0x40 : 0));
}
__host__ __device__ inline uint8_t kind_vt(uint8_t k) { return k & 0x0f; }
__host__ __device__ inline uint8_t kind_rt(uint8_t k) { return (k >> 4) & 0x03; }
__host__ __device__ inline bool kind_cont(uint8_t k) { return (k & 0x40) != 0; }

// What k_conflict serialises a tick's racing records by (zb_submit marks the racing ones): the workflow instance;
// a job command of a job with no workflow headers (JobHeaders.workflowInstanceKey -1, JobHeaders.java:33-51) races
// only with that job's own commands, so it is keyed by its job key, tagged apart from instance keys. -1: none.
constexpr int64_t CONF_JOB_TAG = 1ll << 62;
__host__ __device__ inline int64_t conflict_key(int64_t inst_key, int64_t key, uint8_t kind) {
  if (inst_key >= 0) return inst_key;
  if (kind_vt(kind) == ZB_VT_JOB && kind_rt(kind) == ZB_RT_COMMAND && key >= 0) return key | CONF_JOB_TAG;
  return -1;
}

struct DevElem {              // 72 bytes
  uint8_t kind;
  uint8_t flags;              // bit0: has io mapping (rejected at deploy for now)
  uint16_t wf;                // workflow index
  uint8_t step[12];           // by WF intent 0..11
  uint16_t out0;              // first executable outgoing flow (TakeSequenceFlowHandler uses get(0))
  uint16_t target;            // sequence flow target
  uint16_t start;             // container start event
  uint16_t dflt;              // exclusive gateway default flow
  uint16_t cond_begin;        // exclusive gateway: conditioned flows in executable order (cond_flows[])
  uint16_t cond_count;
  uint16_t ck_query;          // intermediate message catch: correlation key query
  uint16_t n_out;             // number of executable outgoing flows
  uint32_t cond_prog;         // sequence flow: condition program offset in code[] (NO_REF = none)
  int32_t retries;            // service task
  uint32_t job_payload;       // service task: harness completion payload ref (0 = {})
  uint32_t id_off;            // element id (activityId) in pool
  uint16_t id_len;
  uint16_t type_len;          // job type length
  uint32_t type_off;          // job type in pool
  uint32_t headers_off;       // encoded custom headers in pool (raw msgpack)
  uint32_t headers_len;
  uint32_t msg_off;           // message name in pool
  uint16_t msg_len;
  uint16_t out_begin;         // parallel gateway: its outgoing flows in executable order (flows[])
  uint8_t m_in;               // parallel gateway: incoming sequence flows (join arity)
  uint8_t join_slot;          // parallel join: its counter slot in the scope's RowAux
  uint16_t map_in;            // first input mapping (DevMapping) of the element's zeebe:ioMapping
  uint16_t map_out;           // first output mapping
  uint8_t n_in, n_out_map;    // input / output mappings
};
static_assert(sizeof(DevElem) == 80, "DevElem layout is 80 bytes");

struct DevWorkflow {          // 32 bytes
  int64_t key;
  int32_t version;
  uint16_t process_elem;
  uint16_t pid_len;           // bpmnProcessId
  uint32_t pid_off;
  uint32_t pad[3];
};
static_assert(sizeof(DevWorkflow) == 32, "DevWorkflow must stay 32 bytes");

// ---- json-path (JsonPathQueryCompiler filter ids) ----
enum FilterId : uint8_t { F_ROOT = 0, F_MAP_KEY = 1, F_INDEX = 2, F_WILDCARD = 3 };
struct DevFilter {            // 16 bytes
  uint8_t id;
  uint8_t pad;
  uint16_t key_len;
  int32_t index;
  uint32_t key_off;
  uint32_t pad2;
};
struct DevQuery {             // 16 bytes
  uint16_t first;             // index of first filter
  uint16_t count;
  uint16_t expr_len;          // expression text (for incident messages, host side)
  uint16_t fast;              // 1: [ROOT, MAP_KEY k] -> top-level lookup fast path
  uint32_t expr_off;
  uint32_t pad;
};

// ---- value lengths (msgpack sizes of MsgPackWriter.writeInteger / writeString / writeBinary) ----
// The emit kernels that know a record's payload length write the length of its serialized value (vlen),
// so that the drain's size pass does not re-read every payload from HBM (VLEN_UNKNOWN: the size pass
// encodes the value to measure it).
constexpr uint32_t VLEN_UNKNOWN = 0xffffffffu;
__host__ __device__ inline uint32_t mp_int_len(int64_t v) {
  if (v < -(1LL << 5)) return v < -(1LL << 15) ? (v < -(1LL << 31) ? 9 : 5) : (v < -(1LL << 7) ? 3 : 2);
  if (v < (1LL << 7)) return 1;
  if (v < (1LL << 16)) return v < (1LL << 8) ? 2 : 3;
  return v < (1LL << 32) ? 5 : 9;
}
__host__ __device__ inline uint32_t mp_str_len(uint32_t n) { return (n < 32 ? 1 : n < 256 ? 2 : n < 65536 ? 3 : 5) + n; }
__host__ __device__ inline uint32_t mp_bin_len(uint32_t n) { return (n < 256 ? 2 : n < 65536 ? 3 : 5) + n; }
// per element: the constant part of a WORKFLOW_INSTANCE event value and of a JOB record value it writes
// (zb_serialize.hip encode_value); + mp_int_len(workflowInstanceKey) + mp_int_len(scope / activity instance
// key) + mp_bin_len(payload length)
struct ValueConst {
  uint32_t wf, job;
};

// ---- explicit io-mappings (Mapping.java: source query -> target path) ----
struct DevMapping {           // 8 bytes
  uint16_t query;             // DevQuery of the source expression
  uint16_t nseg;              // target path segments: the LITERAL / ROOT_OBJECT tokens of JsonPathTokenizer
  uint32_t seg;               // first segment in segs[]
};
struct DevSeg {               // 8 bytes: segment text in the pool
  uint32_t off, len;
};
// DevElem.flags: bit 0 has io mapping; bits 1-2 output behaviour (ZeebeOutputBehavior; 0 = unset = merge)
constexpr uint8_t EF_IO = 1, OB_SHIFT = 1, OB_UNSET = 0, OB_NONE = 1, OB_MERGE = 2, OB_OVERWRITE = 3;

// ---- json-el constants / program ----
enum TokType : uint8_t { TT_INTEGER = 0, TT_FLOAT = 1, TT_BOOLEAN = 2, TT_NIL = 3, TT_MAP = 4, TT_ARRAY = 5,
                         TT_BINARY = 6, TT_STRING = 7, TT_EXTENSION = 8 };
struct DevConst {             // 24 bytes
  uint8_t type;
  uint8_t bval;
  uint16_t str_len;
  uint32_t str_off;
  int64_t ival;
  double fval;
};
enum CmpOp : uint8_t { OP_EQ = 0, OP_NE, OP_LT, OP_LE, OP_GT, OP_GE };
enum Opcode : uint8_t { PC_CMP = 1, PC_JF = 2, PC_JT = 3, PC_END = 4 };
// one instruction = 2 x uint32:
//   w0: [7:0] opcode  [11:8] cmp op  [12] lhs is path  [13] rhs is path  [31:16] jump target (instr index)
//   w1: [15:0] lhs index (const or query)  [31:16] rhs index

// incident detail codes (host formats the reference's error messages)
enum ErrCode : uint8_t {
  EC_NO_FLOW = 1,        // "All conditions evaluated to false and no default flow is set."
  EC_PATH_NO_RESULT = 2, // "JSON path '%s' has no result."
  EC_PATH_MULTI = 3,     // "JSON path '%s' has more than one result."
  EC_DIFF_TYPES = 4,     // "Cannot compare values of different types: %s and %s"
  EC_CMP_TYPE = 5,       // "Cannot compare value of type: %s"
  EC_NOT_NUMBER = 6,     // "Cannot compare values. Expected number but found: %s"
  EC_MAPPING_NOT_MAP = 7, // "Processing failed, since mapping will result in a non map object (json object)."
  EC_MAPPING_NO_DATA = 8  // "No data found for query %s." (MsgPackDocumentExtractor.executeLeafMapping)
};

// device error flags (sticky, host checks after each batch of waves)
enum DevErr : uint32_t {
  DE_LOG_FULL = 1u, DE_ROWS_FULL = 2u, DE_ARENA_FULL = 4u, DE_UNSUPPORTED = 8u, DE_PROCESSING = 16u,
  DE_BAD_PAYLOAD = 64u, DE_TIMEOUT = 128u,
  DE_CORRUPT = 256u  // a reference names a blob that runs past the arena's allocated bytes (compaction)
};

// Per-wave header (double buffered: wave w reads hdr[w&1], k_scan of wave w writes hdr[(w+1)&1]).
// A wave processes the chunk [begin, min(gen_end, begin + wave_cap)) of the current breadth-first
// generation [begin, gen_end) and appends its follow-ups at the log tail `end`. Processing a
// generation in chunks is still FIFO order: every follow-up lands after the whole generation.
struct WaveHdr {
  int64_t begin;               // first unprocessed record
  int64_t end;                 // log tail (records [0, end) exist)
  int64_t gen_end;             // end of the generation being processed (begin <= gen_end <= end)
  int64_t wf_next, job_next;   // key generators (next key)
  int64_t rows_next;           // row allocator
  int64_t arena_next;          // payload arena bump pointer (bytes)
  int64_t pad[9];
};
static_assert(sizeof(WaveHdr) == 128, "WaveHdr is 128 bytes");
static_assert(sizeof(zb_record_header) == 24, "zb_record_header is 24 bytes (the drain writes one per record)");

// An element instance (ElementInstance.java:30-111) is a row of three planes, each its own array indexed by row: its
// state (RowMeta, 16 B), its keys (RowKeys, 32 B) and its place among its flow scope's children (RowLink, 8 B). The
// wave pipeline's record processing reads the state of the instances it steps, which are mostly consecutive rows:
// 16-byte entries put eight of them in a 128-byte line. (One 64-byte line per row, all planes together, measured
// slower on C2: every touched instance cost a whole line)
struct RowMeta {
  uint32_t payload;
  uint32_t parent;
  uint16_t elem;
  uint8_t state;               // WF intent of the indexed state; 0 = no instance
  uint8_t flags;
  int32_t nchild;
};
struct RowKeys {
  int64_t key, scope_key, inst_key, job_key;
};
// children: ElementInstance.children as an intrusive list -- c_head the last inserted child, c_next the sibling inserted
// before it (any order: concurrent inserts of one wave link in arrival order). TerminateContainedElementsHandler's
// children.get(0) is the first live child in insertion order, which is the smallest live row index of the list (rows
// are allocated in insertion order); removed children stay linked (k_pre skips them) until compaction relinks.
struct RowLink {
  uint32_t c_head, c_next;
};
static_assert(sizeof(RowMeta) == 16 && sizeof(RowKeys) == 32 && sizeof(RowLink) == 8, "row planes");
constexpr uint64_t ROW_BYTES = sizeof(RowMeta) + sizeof(RowKeys) + sizeof(RowLink);  // one row, all planes
// Scope-wide state touched only by scope operations (never on the chain-stepping hot path):
// EXTENSION token / join counters of a scope with parallel gateways, and the first
// live child of a scope being terminated (TerminateContainedElementsHandler :31-53 children.get(0)).
struct RowAux {
  int32_t tokens;              // live tokens of the scope (+ merged arrivals pending their GATEWAY_ACTIVATED)
  uint32_t first;              // min live child row (k_pre, from RowLink.c_head), valid when mark == the wave's epoch
  uint32_t join_cnt[JOIN_SLOTS];
  int64_t consume_pos;         // max log position of a CONSUME_TOKEN on this scope (k_pre)
  int64_t join_pos[JOIN_SLOTS];// max log position of an arrival per join slot (k_pre)
  int64_t mark;                // epoch of the wave that asked for `first`
};
static_assert(sizeof(RowAux) == 48, "RowAux is 48 bytes");

}  // namespace zbg
