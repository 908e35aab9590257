/*
 * zb_engine.h — C ABI of the MI355X batched BPMN stepping core (libzbgpu.so).
 *
 * This is the drop-in boundary for the reference's workflow-instance stepping path: a thin
 * JNI/FFI shim registered as the reference's TypedRecordProcessor for the same
 * (recordType, valueType, intent) keys as
 *   broker-core/src/main/java/io/zeebe/broker/workflow/processor/WorkflowInstanceStreamProcessor.java:103-169
 * forwards the records of one processing tick into zb_submit_*, calls zb_step, and appends the
 * records returned by zb_drain to the log (INTEGRATION.md shows the binding).
 *
 * Conventions:
 *   - plain C types only, caller-owned buffers, int status codes (0 ok, <0 error); nothing throws
 *     across the ABI and no pointer passed in is retained after the call returns;
 *   - one handle = one partition = one HIP device + one HIP stream; a handle is thread-affine
 *     (the reference runs one actor per stream processor, StreamProcessorController.java:39);
 *   - records come back in exact reference log order (FIFO == breadth-first waves),
 *     with keys from the partition's KeyGenerator(1, 5) / job KeyGenerator(2, 5)
 *     (broker-core/.../logstreams/processor/KeyGenerator.java:28-60).
 */
#ifndef ZB_ENGINE_H
#define ZB_ENGINE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------------------------- */
#define ZB_OK 0
#define ZB_EINVAL (-1)        /* bad argument */
#define ZB_ENOMEM (-2)        /* device capacity (log / element rows / payload arena) exhausted */
#define ZB_EUNSUPPORTED (-3)  /* model or payload shape the GPU path does not implement (never a silent fallback) */
#define ZB_EDEPLOY (-4)       /* deployment resource rejected (parse / transform / condition compile error) */
#define ZB_EDEVICE (-5)       /* HIP runtime error */
#define ZB_EAGAIN (-6)        /* stepping stopped at max_waves before quiescence; call zb_step again */
#define ZB_EPROCESSING (-7)   /* processing failure: the partition stops (StreamProcessorController.onFailure) */

/* ---- protocol enums (protocol/src/main/resources/protocol.xml:31-67, protocol intent classes) -- */
#define ZB_VT_JOB 0
#define ZB_VT_WORKFLOW_INSTANCE 5
#define ZB_VT_INCIDENT 6
#define ZB_VT_MESSAGE 10
#define ZB_VT_MESSAGE_SUBSCRIPTION 11
#define ZB_VT_WORKFLOW_INSTANCE_SUBSCRIPTION 12
#define ZB_RT_EVENT 0
#define ZB_RT_COMMAND 1
#define ZB_RT_COMMAND_REJECTION 2

/* zb_config.flags */
#define ZB_CFG_WAVE_ONLY 1    /* always use the general wave pipeline (never the trajectory path) */
#define ZB_CFG_EXTERNAL_JOBS 2 /* no canonical job harness: JOB CREATE commands wait for the job stream
                                  processor's JOB CREATED / JOB COMPLETED events, submitted with zb_submit */
#define ZB_CFG_JOB_PROCESSOR 4 /* the job stream processor runs on the GPU too (JobInstanceStreamProcessor.java:70-242):
                                 JOB commands (the workflow's CREATE / CANCEL, a worker's ACTIVATE / COMPLETE /
                                 FAIL / TIME_OUT / UPDATE_RETRIES through zb_submit) are processed at their log
                                 position with per-job states; implies no harness (as ZB_CFG_EXTERNAL_JOBS) */
/* Diagnostic / measurement flags (never needed for correct output; the defaults are the product configuration): */
#define ZB_CFG_VLEN_CHECK 8       /* the drain's size pass checks every value length an emitting kernel wrote
                                     against the encoder's dry run (a mismatch fails zb_serialize with ZB_EDEVICE) */
#define ZB_CFG_GENERIC_DRAIN 16   /* every drain tile through the generic encoder (k_ser_write): the reference pass
                                     the fast passes are compared with */
#define ZB_CFG_NO_DEFER 32        /* trajectory batches always write their descriptors in zb_step (no template drain) */
#define ZB_CFG_INSTANCE_ORDER 64  /* class batches are emitted in instance order (k_tmpl_io) even when not deferred */
#define ZB_CFG_WAVE_EVENTS 128    /* timing events around every wave's kernels (zb_step_stats process / emit / aux) */
#define ZB_CFG_WAVE_SPLIT 256     /* the three-kernel wave pipeline (k_process, k_scan, k_emit) instead of k_wave */
#define ZB_CFG_SINGLE_PASS_DRAIN 512 /* values drained in one pass with decoupled look-back (measured slower) */
#define ZB_CFG_RCCL_SELF 1024     /* a one-partition engine still exchanges through its RCCL communicator (both agreement
                                     collectives and ncclSend / ncclRecv to itself: the P > 1 code path); without it a
                                     single partition hands its outbox to its own inbox on the device */
#define ZB_CFG_SHARED_GPU 2048    /* the GPU is shared with other processes' engines: the wave pipeline's persistent
                                     kernel claims its tiles from a counter, so its hand-off progresses when only part
                                     of its grid is resident (without it, engines of several processes stepping on one
                                     GPU at once can time out their hand-off, DE_TIMEOUT; the claims cost one contended
                                     atomic per tile) */

typedef struct zb_engine zb_engine;

typedef struct zb_config {
  int32_t device;           /* HIP device ordinal */
  int32_t partition_id;
  int32_t partition_count;
  int32_t flags;            /* ZB_CFG_* bits */
  uint64_t log_capacity;    /* max records in the device log (32 B descriptor + 8 B row links each) */
  uint64_t row_capacity;    /* max element-instance rows (SoA planes: RowMeta 16 + RowKeys 32 + RowLink 8 + RowAux 48 B) */
  uint64_t arena_bytes;     /* payload arena (msgpack documents, 8-byte aligned blobs) */
  uint64_t wave_records;    /* max records processed per wave (chunk of a generation); 0 = min(log_capacity, 2^22) */
} zb_config;

/* The 32-byte record descriptor kept in HBM for every record of the log. */
typedef struct zb_rec {
  int64_t key;        /* record key (-1 = null key) */
  int64_t scope_key;  /* WF: value.scopeInstanceKey; JOB: headers.activityInstanceKey; INCIDENT: activityInstanceKey */
  int64_t inst_key;   /* value.workflowInstanceKey */
  uint32_t payload;   /* payload ref (arena offset / 8); INCIDENT: detail ref */
  uint16_t elem;      /* global element index (value.activityId); 0xffff = none */
  uint8_t intent;
  uint8_t kind;       /* bits 0-3 value type, bits 4-5 record type, bit 6 = 2nd record of a batch */
} zb_rec;

/* Serialized record as handed back for log append (the layout of zb_rec_desc, the submit input, with the
 * rejection type in its pad byte). value bytes are the exact msgpack value (UnpackedObject.write) of the
 * reference record. Header i of a drained batch [start, start + count) is the record at log position
 * start + i; source positions, batch flags and the SBE metadata are in the log frames
 * (zb_serialize_frames). 24 bytes: the drain writes one per record, so every byte is HBM traffic. */
typedef struct zb_record_header {
  int64_t key;
  uint8_t record_type;
  uint8_t value_type;
  uint8_t intent;
  uint8_t rejection_type; /* 255 = none */
  uint32_t value_length;
  uint64_t value_offset;  /* into the value buffer passed to zb_drain */
} zb_record_header;

typedef struct zb_step_stats {
  uint64_t waves;              /* wave kernels that processed >= 1 record */
  uint64_t launches;           /* wave kernels launched (incl. the final empty one) */
  uint64_t records_processed;
  uint64_t records_written;
  uint64_t transitions;        /* WORKFLOW_INSTANCE events written (streamprocessor_events_count{written}, WF only) */
  uint64_t completed_instances;/* process-level ELEMENT_COMPLETED written */
  uint64_t merges;             /* default output merges performed */
  uint64_t merge_bytes;        /* sum of (job + scope + result) payload bytes of those merges */
  uint64_t condition_payload_bytes; /* payload bytes read by exclusive-gateway evaluations */
  double wave_kernel_ms;       /* device time of all wave kernels (HIP events on the engine stream) */
  double wall_ms;              /* host wall time of the zb_step call */
  double process_kernel_ms;    /* k_process share of wave_kernel_ms (trajectory: count pass; wave pipeline without
                                  ZB_CFG_WAVE_EVENTS: all of it, timed per batch of waves) */
  double emit_kernel_ms;       /* k_scan + k_emit share (trajectory: scans + emit pass) */
  double aux_kernel_ms;        /* k_merge + k_cond share */
  uint64_t path;               /* 0: wave pipeline, 1: trajectory path (zb_traj.hip) ran the step,
                                  2: trajectory path as a class batch (k_cls_*: split outcomes fixed at creation) */
  double main_emit_kernel_ms;  /* trajectory path: the main emit launch alone (k_tmpl / k_traj<emit>), the
                                  dominant kernel priced by bench.py's roofline; 0 on the wave pipeline */
} zb_step_stats;

/* One partition-to-partition command (SubscriptionCommandSender.java:83-128) exchanged between partitions
 * (zeebe_amd/cluster.py; RCCL over xGMI between GPUs):
 *   ZB_XCHG_OPEN:      OpenMessageSubscriptionCommand, workflow partition -> abs(hash(ck) % P)
 *   ZB_XCHG_CORRELATE: CorrelateWorkflowInstanceSubscriptionCommand, message partition -> workflow partition
 * A 64-byte header; its variable fields follow in the byte section of the batch that carries it, so message
 * names, correlation keys and payload documents have no length limit. token / elem are the workflow partition's
 * element-instance row (a hint: a delivered CORRELATE finds its element instance by activity instance key) and
 * catch element. */
#define ZB_XCHG_OPEN 1
#define ZB_XCHG_CORRELATE 2
typedef struct zb_exchange_rec {
  int32_t kind;
  int32_t target_partition;
  int32_t wf_partition;          /* workflowInstancePartitionId */
  uint32_t token;
  int64_t workflow_instance_key;
  int64_t activity_instance_key;
  int64_t source_position;       /* log position of the record whose processing produced it */
  uint16_t elem;                 /* catch element (workflow partition's model) */
  uint16_t pad;
  uint32_t name_len;             /* messageName */
  uint32_t ck_len;               /* correlationKey (ZB_XCHG_OPEN) */
  uint32_t payload_len;          /* message payload document (ZB_XCHG_CORRELATE) */
  uint64_t var_offset;           /* [name][correlation key][payload] at this offset of the batch's byte section */
} zb_exchange_rec;
/* An exchange batch -- the commands one partition sends one other partition in a round -- is one contiguous,
 * 8-byte aligned block: [uint64 count][uint64 total bytes][count x zb_exchange_rec][byte section]; each
 * record's variable bytes are padded to 8. A delivery is a sequence of batches (one per sending partition, in
 * partition order). */
#define ZB_XCHG_BATCH_HEADER 16

/* ---- lifecycle ------------------------------------------------------------------------- */
int zb_engine_create(const zb_config* cfg, zb_engine** out);
void zb_engine_destroy(zb_engine* e);
const char* zb_last_error(const zb_engine* e);
/* Clears records, element instances, payloads and key generators (deployments stay).
 * keep_staged != 0 keeps the staged input batch so that it is injected again by the next zb_step. */
int zb_reset(zb_engine* e, int keep_staged);

/* ---- deployment (WorkflowCache.addWorkflow + BpmnTransformer) -------------------------- */
/* Host-only (no device, no engine): transforms a BPMN 2.0 XML resource exactly as zb_deploy would --
 * BpmnTransformer + json-el / json-path compilation -- and reports why it would be rejected
 * (DeploymentCreateEventProcessor.java:91-151 validation / transformation). Returns ZB_OK,
 * ZB_EDEPLOY or ZB_EUNSUPPORTED; err (may be NULL) receives the message. */
int zb_validate_deployment(const uint8_t* bpmn_xml, size_t len, char* err, size_t err_cap);
/* Deploys every executable process of a BPMN 2.0 XML resource; process i gets workflow_key + i. */
int zb_deploy(zb_engine* e, int64_t workflow_key, int32_t version, const uint8_t* bpmn_xml, size_t len);
/* Canonical job harness: payload of the JOB COMPLETED event appended for every
 * JOB CREATE command of the given service task (default: empty document). */
int zb_set_job_completion_payload(zb_engine* e, int64_t workflow_key, const char* activity_id,
                                  const uint8_t* payload, size_t len);

/* ---- input --------------------------------------------------------------------------- */
/* Stages n WORKFLOW_INSTANCE CREATE commands (ExecuteCommandRequest, ClientApiMessageHandler.java:147-162)
 * addressed like the reference's CreateWorkflowInstanceEventProcessor: workflow_key > 0 by key,
 * else version > 0 by (bpmn_process_id, version), else latest version of bpmn_process_id.
 * payloads: concatenated msgpack documents, offsets[i]..offsets[i+1] (n+1 entries). */
int zb_submit_creates(zb_engine* e, const char* bpmn_process_id, int32_t version, int64_t workflow_key,
                      size_t n, const uint8_t* payloads, const uint64_t* offsets);

/* General record input: the records a JNI shim forwards for the 18 (recordType, valueType, intent) keys
 * WorkflowInstanceStreamProcessor registers (WorkflowInstanceStreamProcessor.java:103-169), as the log
 * holds them: metadata + the reference msgpack value (UnpackedObject.write). The engine decodes each
 * value, keeps its bytes verbatim for the log, and injects the batch at the log tail at the next
 * zb_step, in submission order. Accepted:
 *   COMMAND WORKFLOW_INSTANCE CREATE          (CreateWorkflowInstanceEventProcessor :224-368)
 *   COMMAND WORKFLOW_INSTANCE CANCEL          (CancelWorkflowInstanceProcessor :511-555; key = instance key)
 *   COMMAND WORKFLOW_INSTANCE UPDATE_PAYLOAD  (UpdatePayloadProcessor :557-576)
 *   EVENT   JOB CREATED / COMPLETED           (JobCreatedProcessor :408-426, JobCompletedEventProcessor :428-453)
 *   COMMAND WORKFLOW_INSTANCE_SUBSCRIPTION CORRELATE (:455-509; its key becomes its log position)
 * Any order is accepted, as the reference's processor accepts it: records of one workflow instance that would
 * race inside one lockstep wave (a CANCEL or UPDATE_PAYLOAD next to other records of its instance, two records
 * of one activity instance other than a JOB CREATED directly followed by its JOB COMPLETED, a job's commands
 * that are not two consecutive ones) make the instance a conflicting one for the tick, and zb_step cuts every
 * generation of the tick before the next record of such an instance, so each is processed after the ones before
 * it in log order, as the reference does. Records other than CREATE are injected only into a quiescent
 * partition. All-or-nothing: on error nothing is staged. */
typedef struct zb_rec_desc {
  int64_t key;            /* record key (-1 = null) */
  uint8_t record_type;    /* ZB_RT_* */
  uint8_t value_type;     /* ZB_VT_* */
  uint8_t intent;
  uint8_t pad;
  uint32_t value_length;
  uint64_t value_offset;  /* into the values buffer */
} zb_rec_desc;
int zb_submit(zb_engine* e, const zb_rec_desc* recs, size_t n, const uint8_t* values, size_t values_len);

/* Uploads the staged input batch to the device now (zb_step does it otherwise): a caller overlaps the PCIe
 * transfer of the next tick's input with the current tick's drain, and keeps it out of the tick. */
int zb_upload_staged(zb_engine* e);

/* ---- stepping ------------------------------------------------------------------------ */
/* Injects staged input at the log tail and runs lockstep waves until quiescence (ZB_OK) or
 * max_waves (ZB_EAGAIN). stats may be NULL. */
int zb_step(zb_engine* e, uint32_t max_waves, zb_step_stats* stats);

/* ---- the message stream processor (config 5; MessageService.java:90-129) --------------------------- */
/* ActorClock.currentTimeMillis() for the records processed from now on: a stored message's deadline is
 * timeToLive + now (MessageDataStore.Message). */
int zb_set_clock(zb_engine* e, int64_t now_ms);
/* MESSAGE commands as the log holds them (ClientApiMessageHandler.java:90-162 for PUBLISH; the time-to-live
 * checker's DELETE): metadata + the reference MessageRecord value (MessageRecord.java:26-42: name,
 * correlationKey, timeToLive, payload, messageId), kept verbatim for the log. Appended and processed at once
 * by the message stream processor, in order (runs of one intent are processed in lockstep):
 *   COMMAND MESSAGE PUBLISH (key -1)  PublishMessageProcessor.java:58-124: a messageId already published with
 *                                     the same name and correlation key -> BAD_VALUE rejection; else PUBLISHED
 *                                     (+ DELETED when timeToLive <= 0, else stored) and a correlate command per
 *                                     matching subscription in the outbox
 *   COMMAND MESSAGE DELETE (key = message key)  DeleteMessageProcessor.java:36-45: DELETED, message removed
 * The partition must be quiescent with nothing staged. */
int zb_submit_messages(zb_engine* e, const zb_rec_desc* recs, size_t n, const uint8_t* values, size_t values_len);
/* Bulk PUBLISH commands with one message name and time-to-live and no message id, built by the engine
 * (correlation keys / payloads concatenated, n+1 offsets each): same processing as zb_submit_messages. */
int zb_submit_publishes(zb_engine* e, const char* message_name, int64_t ttl, size_t n, const uint8_t* cks,
                        const uint64_t* ck_offsets, const uint8_t* payloads, const uint64_t* payload_offsets);
/* zb_submit_publishes in two parts: the batch goes to HBM (zb_upload_publishes; any partition state, returns when
 * the data is resident, checked -- a payload that is not a map or nil, a key or payload over 4 GB: ZB_EINVAL here -- and
 * its message blobs sized) and is processed later (zb_publish_uploaded; quiescent, nothing staged; without message ids
 * every command is accepted, so its record counts need no count pass) -- so a broker overlaps the next batch's PCIe copy
 * with the current tick. Another upload replaces a batch not processed yet. */
int zb_upload_publishes(zb_engine* e, const char* message_name, int64_t ttl, size_t n, const uint8_t* cks,
                        const uint64_t* ck_offsets, const uint8_t* payloads, const uint64_t* payload_offsets);
int zb_publish_uploaded(zb_engine* e);
/* MessageTimeToLiveChecker.run (MessageTimeToLiveChecker.java:44-68) at now_ms: a DELETE command for every
 * stored message with deadline <= now_ms, in store order, then their processing. *n_deleted = commands written. */
int zb_expire_messages(zb_engine* e, int64_t now_ms, uint64_t* n_deleted);
/* Exchange batches from other partitions, in delivery order (zeebe_amd/cluster.py schedule); batches is a
 * device pointer when on_device != 0. ZB_XCHG_OPEN commands are appended as MESSAGE_SUBSCRIPTION OPEN commands
 * and processed at once (OpenMessageSubscriptionProcessor.java:56-92); ZB_XCHG_CORRELATE commands are appended
 * as WORKFLOW_INSTANCE_SUBSCRIPTION CORRELATE commands (key = log position,
 * SubscriptionApiCommandMessageHandler.java:131-151), processed by the next zb_step
 * (WorkflowInstanceStreamProcessor.java:455-509). The partition must be quiescent with nothing staged. */
int zb_inbox_submit(zb_engine* e, int kind, const uint8_t* batches, size_t bytes, int on_device);
/* Pending outgoing commands of a kind (side effects of processed records). */
int zb_outbox_count(zb_engine* e, int kind, uint64_t* n);
/* Takes every pending command of a kind, ordered by (target partition, source position, emission order), as one
 * exchange batch per target partition with commands, back to back in target order, into dst (cap bytes; device
 * pointer when dst_on_device != 0). bytes_per_target[partition_count]: each target's batch size (0: none).
 * *total = bytes needed; with dst NULL or cap too small nothing is taken (ZB_ENOMEM unless nothing is pending). */
int zb_outbox_take(zb_engine* e, int kind, uint8_t* dst, size_t cap, int dst_on_device, uint64_t* bytes_per_target,
                   uint64_t* n_out, uint64_t* total);

/* Partition-to-partition exchange over RCCL (xGMI between the GPUs of a node): one communicator
 * per engine, rank = partition id. zb_comm_unique_id on one rank; the 128-byte id travels to the
 * others out of band (zeebe_amd/cluster.py uses the torch.distributed control plane). */
int zb_comm_unique_id(uint8_t id[128]);
/* The RCCL library file the communicator runs on (the engine links /opt/rocm/lib/librccl.so; a process that
 * loaded another copy of the library first -- e.g. torch's -- resolves to that one: load libzbgpu.so first). */
const char* zb_rccl_library(void);
int zb_comm_init(zb_engine* e, const uint8_t id[128], int nranks, int rank);
/* A single partition (partition_count 1, no ZB_CFG_RCCL_SELF) needs no zb_comm_init: its exchange delivers its outbox
 * to its own inbox on the device, without a collective.
 * Collective: global[k] = sum over ranks of the pending commands of kind k+1 (ZB_XCHG_OPEN, _CORRELATE). */
int zb_comm_pending(zb_engine* e, uint64_t global[2]);
/* Collective: every rank takes its pending commands of `kind` (zb_outbox_take order), sends each target
 * its batch (ncclSend / ncclRecv in one group), and delivers what it receives in source-rank order
 * (zb_inbox_submit). *received = commands delivered to this rank.
 * Failure protocol: a rank whose local work fails (outbox read, buffer growth) still takes part in the
 * (count, status) all-to-all and the status all-reduce that precede the record exchange, so every rank
 * returns an error in the same call and none is left blocking in ncclSend / ncclRecv. A failing RCCL
 * call aborts the communicator (ncclCommAbort); later exchanges on the engine fail with ZB_EDEVICE.
 * Exchange and sort buffers persist across calls (no allocation per round in the steady state). */
int zb_comm_exchange(zb_engine* e, int kind, uint64_t* received);

/* ---- output -------------------------------------------------------------------------- */
int64_t zb_log_size(zb_engine* e);
/* Source event position of records [start, start+count) (LogEntryDescriptor sourceEventPosition: the record
 * whose processing wrote it, TypedStreamWriterImpl / TypedCommandWriterImpl.configureSourceContext), -1 for
 * records another writer appended (client commands, zb_submit). */
int zb_read_source_positions(zb_engine* e, int64_t start, int64_t count, int64_t* out);
/* Copies raw descriptors [start, start+count) to host. */
int zb_read_descriptors(zb_engine* e, int64_t start, int64_t count, zb_rec* out);
/* Serializes records [start, start+count) on the GPU into reference value bytes and copies them
 * back: headers[count], value bytes into values (capacity values_cap); *values_len = bytes needed.
 * If values_cap is too small nothing is copied and ZB_ENOMEM is returned with *values_len set.
 * = zb_serialize + zb_drain_copy. */
int zb_drain(zb_engine* e, int64_t start, int64_t count, zb_record_header* headers, uint8_t* values,
             size_t values_cap, size_t* values_len);

/* The two halves of zb_drain. zb_serialize writes the headers and value bytes of records
 * [start, start+count) into the engine's device-resident drain buffers (reused between calls; the
 * batch stays there until the next zb_serialize); zb_drain_copy copies that batch, or a byte range
 * of its values, to host memory (pinned memory gives the full PCIe rate). */
typedef struct zb_serialize_stats {
  uint64_t records;
  uint64_t value_bytes;        /* serialized record values */
  uint64_t payload_bytes;      /* payload documents copied into them (msgpack bin) */
  double size_kernel_ms;       /* size pass (0: sizes, offsets and values in one pass) */
  double scan_ms;              /* exclusive scan of the sizes (0 in the single-pass serializer) */
  double write_kernel_ms;      /* write pass (headers + values; the whole single pass): the drain's kernel */
  double wall_ms;
  uint64_t generic_tiles;      /* 256-record tiles the generic write pass encoded (the rest: the fast pass) */
  uint64_t template_drain;     /* 1: a deferred trajectory batch, encoded from its traces (no descriptors) */
} zb_serialize_stats;
int zb_serialize(zb_engine* e, int64_t start, int64_t count, zb_serialize_stats* stats);
/* headers: NULL or room for the batch's headers; values: NULL or values_len bytes from value byte
 * value_off of the batch. */
int zb_drain_copy(zb_engine* e, zb_record_header* headers, uint8_t* values, uint64_t value_off, size_t values_len);
/* Log frames: zb_serialize_frames serializes records [start, start+count) into the
 * drain buffer as the byte stream the reference's log writers append to the dispatcher buffer
 * (LogStreamBatchWriterImpl.java:222-268, LogStreamWriterImpl.java:150-205): per record a
 * DataFrameDescriptor header (DataFrameDescriptor.java:53-96; batch begin / end flags per
 * ClaimedFragmentBatch.commit), a LogEntryDescriptor header (LogEntryDescriptor.java:28-121), the SBE
 * RecordMetadata (RecordMetadata.java:96-128, protocol.xml:135-146) with the rejection reason, the value
 * and zero padding to 8 bytes. Positions are the engine's log positions (the dispatcher derives them from
 * the claim offset: the caller maps them). stats->value_bytes = frame bytes; zb_drain_copy(e, NULL, buf,
 * off, len) copies them. */
typedef struct zb_frame_config {
  int32_t stream_id;   /* dispatcher stream id = the log's partition id (LogStreamBatchWriterImpl.java:90) */
  int32_t raft_term;   /* LogStream.getTerm() */
  int64_t timestamp;   /* ActorClock.currentTimeMillis() of the tick, written into every frame */
} zb_frame_config;
int zb_serialize_frames(zb_engine* e, int64_t start, int64_t count, const zb_frame_config* fc,
                        zb_serialize_stats* stats);
/* Request metadata (RecordMetadata requestId / requestStreamId, ClientApiMessageHandler) of the last n
 * records staged by zb_submit / zb_submit_creates; CREATED and the CREATE rejection copy it from their
 * command (WorkflowInstanceStreamProcessor.java:254-257, :370-377). Frames only. */
int zb_set_request_metadata(zb_engine* e, size_t n, const uint64_t* request_ids, const int32_t* request_stream_ids);
/* Page-locked host memory for zb_drain_copy destinations (hipHostMalloc); NULL on failure. */
void* zb_pinned_alloc(size_t bytes);
void zb_pinned_free(void* p);
/* ---- a partition that runs indefinitely ------------------------------------------------------ */
/* The device log holds a window of log_capacity positions. The caller releases what it has appended to the
 * logstream (records below position; only processed ones): at the next call that appends (zb_step,
 * zb_submit_publishes, zb_inbox_submit) the window starts there, and released records can no longer be
 * drained. Positions stay absolute (LogStream positions are the caller's). */
int zb_log_release(zb_engine* e, int64_t position);
/* The partition's log continues at `position` (>= its current end): a processor that resumes on a logstream whose
 * earlier records it does not process (StreamProcessorController.java:296-414 reprocesses from a snapshot position;
 * LogEntryDescriptor.java:28-121 positions are 64-bit). Positions, source positions and position keys of everything
 * written afterwards follow from it. Only on an idle partition whose window is empty (everything written released)
 * and with nothing staged. */
int zb_log_start(zb_engine* e, int64_t position);
/* Compaction of a quiescent partition (also run automatically between ticks when the element-instance rows,
 * the payload arena or the job table are more than half full): element instances removed on COMPLETED /
 * TERMINATED free their rows (ElementInstanceIndex.removeInstance, ElementInstanceIndex.java:54-64), payload
 * blobs that no live row, unreleased record or stored message references are reclaimed, removed messages and
 * job states are dropped. Order-preserving: logs and state read back identically. */
int zb_compact(zb_engine* e);
typedef struct zb_memory_stats {
  int64_t log_window_begin, log_end;  /* positions [log_window_begin, log_end) are readable */
  uint64_t log_capacity;
  uint64_t rows_allocated, row_capacity;  /* rows in use (live + dead since the last compaction) */
  uint64_t arena_used, arena_bytes;
  uint64_t records_total, rows_total, arena_total;  /* lifetime totals written / allocated */
  uint64_t compactions;
} zb_memory_stats;
int zb_read_memory_stats(zb_engine* e, zb_memory_stats* out);

/* counters: [0] created [1] completed [2] canceled [3] next wf key [4] next job key
 *           [5] rows allocated [6] arena bytes used [7] log size */
int zb_counters(zb_engine* e, int64_t out[8]);

/* Live element instances (ElementInstanceIndex.java:25-65, ElementInstance.java:30-111) sorted by key,
 * packed as [i64 key][i64 flow scope (parent) key, -1 for none][i64 job key][u8 state (intent)][3 pad]
 * [u32 value length][value: the indexed WorkflowInstanceRecord]. *len = bytes needed; if cap is too
 * small nothing is copied and ZB_ENOMEM is returned. */
int zb_read_instances(zb_engine* e, uint8_t* buf, size_t cap, size_t* len, uint64_t* count);

/* Snapshot of a quiescent partition's processing state (ComposeableSerializableSnapshot.java:27-48:
 * element instances, key generators; plus payloads and message stores): element-instance rows, the
 * payload arena, wave header / key generators, statistics and message stores. Deployments are not in
 * it (the reference keeps them in the WorkflowCache): zb_restore requires the same deployments. The log
 * is not in it either: after zb_restore positions continue from the snapshot's log end and earlier
 * records cannot be drained. *len = bytes needed (ZB_ENOMEM if cap too small). */
int zb_snapshot(zb_engine* e, uint8_t* buf, size_t cap, size_t* len);
int zb_restore(zb_engine* e, const uint8_t* buf, size_t len);

#ifdef __cplusplus
}
#endif

#endif /* ZB_ENGINE_H */
