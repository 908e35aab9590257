// zb_frame.hpp — the 104-byte prefix of a log frame, shared by the generic frame encoder (encode_frame,
// zb_serialize.hip), the wave-parallel descriptor drain (k_ser_wave<true>) and the template drain
// (k_tdrain_write<.., true>), so that the three paths cannot drift apart.
//
// A record as LogStreamBatchWriterImpl.writeEventsToBuffer (:222-268) / LogStreamWriterImpl lay it into the
// dispatcher buffer: DataFrameDescriptor header (DataFrameDescriptor.java:53-96: framed length, version 0,
// batch flags, TYPE_MESSAGE, stream id), LogEntryDescriptor header (LogEntryDescriptor.java:28-121: version,
// position, raft term, producer id, source event position, key, timestamp, metadata length), RecordMetadata
// (RecordMetadata.java:96-128: SBE header {34, 200, 0, 1} + block + varData rejectionReason), the value, and
// zero padding to FRAME_ALIGNMENT 8. Frames start 8-aligned, so the prefix is 13 aligned 8-byte words.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "zb_kernels.hpp"  // (ReqMeta)

namespace zbg {

constexpr uint32_t FRAME_PREFIX = 12 + 48 + 8 + 34 + 2;
static_assert(FRAME_PREFIX == 13 * 8, "the prefix is 13 whole words");

// ClaimedFragmentBatch.commit :130-147: BEGIN on the first and END on the last fragment of a batch with more than
// one; a batch is the records one processed record wrote (contiguous, same source)
constexpr uint32_t FRAME_BEGIN = 0x80, FRAME_END = 0x40;
__host__ __device__ __forceinline__ uint32_t frame_flags(bool first, bool last) {
  return (first && last) ? 0u : first ? FRAME_BEGIN : (last ? FRAME_END : 0u);
}

// TypedStreamProcessor producer ids (StreamProcessorIds.java:23-39): harness job events 10 (the job processor),
// message partition records 90, everything else the workflow instance processor 70; records other writers
// appended keep the writer's default -1 (a MESSAGE DELETE command comes from the time-to-live checker's own
// command writer: producer id 0, TypedCommandWriterImpl never configured, MessageService.java:118-120)
__host__ __device__ __forceinline__ int32_t frame_producer(int64_t src, uint8_t vt, uint8_t rt, uint8_t intent) {
  return src < 0 ? ((vt == ZB_VT_MESSAGE && rt == ZB_RT_COMMAND && intent == 2) ? 0 : -1)
         : (vt == ZB_VT_JOB && rt != ZB_RT_COMMAND) ? 10
         : (vt == ZB_VT_MESSAGE || vt == ZB_VT_MESSAGE_SUBSCRIPTION) ? 90 : 70;
}

// the constant fields of a drain (zb_frame_config)
struct FrameConst {
  int32_t stream_id, raft_term;
  int64_t timestamp;
};

// the 13 prefix words of a frame: framed = prefix + rejection reason + value bytes (before the padding); rej the
// RejectionType (255: none), rlen the rejection reason's length; rid / sid the request metadata (~0 / 0x80000000:
// none)
__device__ __forceinline__ void frame_words(uint64_t (&h)[13], const FrameConst& fc, uint32_t framed, uint32_t flags,
                                            int64_t pos, int32_t producer, int64_t src, int64_t key, uint8_t rt,
                                            uint8_t vt, uint8_t intent, uint64_t rej, uint32_t rlen, uint64_t rid,
                                            uint32_t sid) {
  const uint64_t mlen = 8 + 34 + 2 + rlen;
  h[0] = (uint64_t)framed | (uint64_t)flags << 40;                          // length, version 0, flags, type 0
  h[1] = (uint64_t)(uint32_t)fc.stream_id;                                   // stream id, entry version, reserved
  h[2] = (uint64_t)pos;
  h[3] = (uint64_t)(uint32_t)fc.raft_term | (uint64_t)(uint32_t)producer << 32;
  h[4] = (uint64_t)src;
  h[5] = (uint64_t)key;
  h[6] = (uint64_t)fc.timestamp;
  h[7] = mlen | 34ull << 32 | 200ull << 48;                                   // metadata length | blockLength, templateId
  h[8] = 1ull << 16 | (uint64_t)rt << 32 | (uint64_t)(sid & 0xffffffu) << 40; // schemaId 0, version 1 | recordType
  h[9] = (uint64_t)(sid >> 24) | rid << 8;                                    // requestStreamId | requestId
  h[10] = (rid >> 56) | 0xffffffffffffff00ull;                                // | subscriptionId (null)
  h[11] = 0xffull | 1ull << 8 | (uint64_t)vt << 24 | (uint64_t)intent << 32 | 0xffffffull << 40;  // protocolVersion 1
  h[12] = 0xffffffffffull | rej << 40 | (uint64_t)rlen << 48;                  // incidentKey (null) | rejectionType
}

// the command whose request metadata a frame carries: a submitted command's own (no source), its CREATED / CREATE
// rejection's (the CREATE command); -1: none
__host__ __device__ __forceinline__ int64_t frame_request_pos(int64_t pos, int64_t src, uint8_t vt, uint8_t rt,
                                                              uint8_t intent) {
  if (src < 0) return pos;
  if (vt == ZB_VT_WORKFLOW_INSTANCE &&
      ((rt == ZB_RT_EVENT && intent == WI_CREATED) || (rt == ZB_RT_COMMAND_REJECTION && intent == WI_CREATE)))
    return src;
  return -1;
}

// the 13 prefix words into an LDS image at an 8-aligned offset: six 16-byte stores and one 8-byte store, without a
// divergent branch on the offset's alignment (the odd word is the first when the offset is 8 mod 16, else the last)
__device__ __forceinline__ void frame_store_lds(uint8_t* img, uint32_t at, const uint64_t (&h)[13]) {
  const bool o = (at & 8) != 0;
  *(uint64_t*)(img + at + (o ? 0u : 96u)) = o ? h[0] : h[12];
  uint4* q = (uint4*)(img + at + (o ? 8u : 0u));
#pragma unroll
  for (int j = 0; j < 6; j++) {
    const uint64_t a = o ? h[1 + 2 * j] : h[2 * j], b = o ? h[2 + 2 * j] : h[2 * j + 1];
    q[j] = uint4{(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)};
  }
}

// request metadata of the record at pos whose request is the command at q (q < 0: none) in a sorted table
__device__ __forceinline__ void frame_request(const ReqMeta* reqs, int64_t nreqs, int64_t q, uint64_t& rid, uint32_t& sid) {
  rid = ~0ull;
  sid = 0x80000000u;
  if (q < 0 || nreqs <= 0) return;
  int64_t lo = 0, hi = nreqs - 1;
  while (lo <= hi) {
    const int64_t mid = (lo + hi) >> 1;
    const int64_t p = reqs[mid].pos;
    if (p == q) {
      rid = reqs[mid].request_id;
      sid = (uint32_t)reqs[mid].request_stream_id;
      return;
    }
    if (p < q) lo = mid + 1; else hi = mid - 1;
  }
}

}  // namespace zbg
