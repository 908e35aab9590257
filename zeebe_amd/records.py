"""Reference record values as msgpack bytes, and the protocol enums the boundary speaks.

``zb_submit`` (include/zb_engine.h) takes records the way the reference's log holds them: record
type, value type, intent, key and the msgpack value written by ``UnpackedObject.write`` (declared
properties in declaration order, ObjectValue.java:140-153; integers by MsgPackWriter.writeInteger,
MsgPackWriter.java:143-201). These encoders produce the values other writers of the partition log
put there: the client API (CREATE / CANCEL / UPDATE_PAYLOAD commands,
ClientApiMessageHandler.java:90-162), the job stream processor (JOB CREATED / COMPLETED events,
JobInstanceStreamProcessor.java:98-180) and the subscription API (WORKFLOW_INSTANCE_SUBSCRIPTION
CORRELATE, SubscriptionApiCommandMessageHandler.java:112-151).
"""
from __future__ import annotations

import struct

from .workloads import mp_int, mp_str

# protocol.xml:31-67
RT_EVENT, RT_COMMAND, RT_REJECTION = 0, 1, 2
VT_JOB, VT_WORKFLOW_INSTANCE, VT_INCIDENT, VT_MESSAGE, VT_MESSAGE_SUBSCRIPTION, VT_WIS = 0, 5, 6, 10, 11, 12

# WorkflowInstanceIntent.java:18-38
(WI_CREATE, WI_CREATED, WI_START_EVENT_OCCURRED, WI_END_EVENT_OCCURRED, WI_SEQUENCE_FLOW_TAKEN,
 WI_GATEWAY_ACTIVATED, WI_ELEMENT_READY, WI_ELEMENT_ACTIVATED, WI_ELEMENT_COMPLETING, WI_ELEMENT_COMPLETED,
 WI_ELEMENT_TERMINATING, WI_ELEMENT_TERMINATED, WI_CANCEL, WI_CANCELING, WI_UPDATE_PAYLOAD,
 WI_PAYLOAD_UPDATED) = range(16)
WI_NAMES = ["CREATE", "CREATED", "START_EVENT_OCCURRED", "END_EVENT_OCCURRED", "SEQUENCE_FLOW_TAKEN",
            "GATEWAY_ACTIVATED", "ELEMENT_READY", "ELEMENT_ACTIVATED", "ELEMENT_COMPLETING", "ELEMENT_COMPLETED",
            "ELEMENT_TERMINATING", "ELEMENT_TERMINATED", "CANCEL", "CANCELING", "UPDATE_PAYLOAD", "PAYLOAD_UPDATED"]
# JobIntent.java:18-37
JI_CREATE, JI_CREATED, JI_ACTIVATE, JI_ACTIVATED, JI_COMPLETE, JI_COMPLETED = 0, 1, 2, 3, 4, 5
JI_TIME_OUT, JI_TIMED_OUT, JI_FAIL, JI_FAILED, JI_UPDATE_RETRIES, JI_RETRIES_UPDATED = 6, 7, 8, 9, 10, 11
JI_CANCEL, JI_CANCELED = 12, 13
JI_NAMES = ["CREATE", "CREATED", "ACTIVATE", "ACTIVATED", "COMPLETE", "COMPLETED", "TIME_OUT", "TIMED_OUT", "FAIL",
            "FAILED", "UPDATE_RETRIES", "RETRIES_UPDATED", "CANCEL", "CANCELED"]
RT_NAMES = ["EVENT", "COMMAND", "COMMAND_REJECTION"]
# WorkflowInstanceSubscriptionIntent.java:19-20
WIS_CORRELATE, WIS_CORRELATED = 0, 1

INSTANT_NULL = -(1 << 63)  # Protocol.INSTANT_NULL_VALUE
EMPTY_DOCUMENT = b"\x80"


def mp_bin(b: bytes) -> bytes:
    n = len(b)
    if n < 256:
        return b"\xc4" + bytes([n]) + b
    if n < 65536:
        return b"\xc5" + struct.pack(">H", n) + b
    return b"\xc6" + struct.pack(">I", n) + b


def _map(n: int) -> bytes:
    return bytes([0x80 | n]) if n < 16 else b"\xde" + struct.pack(">H", n)


def _doc(payload) -> bytes:
    """DocumentValue: nil / empty -> {} (DocumentValue.java:35-55)."""
    if payload is None or payload == b"" or payload == b"\xc0":
        return EMPTY_DOCUMENT
    return payload


def wf_record(bpmn_process_id: str = "", version: int = -1, workflow_key: int = -1,
              workflow_instance_key: int = -1, activity_id: str = "", payload: bytes = EMPTY_DOCUMENT,
              scope_instance_key: int = -1) -> bytes:
    """WorkflowInstanceRecord (WorkflowInstanceRecord.java:39-60)."""
    return (_map(7) + mp_str("bpmnProcessId") + mp_str(bpmn_process_id) + mp_str("version") + mp_int(version)
            + mp_str("workflowKey") + mp_int(workflow_key) + mp_str("workflowInstanceKey")
            + mp_int(workflow_instance_key) + mp_str("activityId") + mp_str(activity_id)
            + mp_str("payload") + mp_bin(_doc(payload)) + mp_str("scopeInstanceKey") + mp_int(scope_instance_key))


def job_record(type: str = "", retries: int = -1, worker: str = "", deadline: int = INSTANT_NULL,
               bpmn_process_id: str = "", version: int = -1, workflow_key: int = -1,
               workflow_instance_key: int = -1, activity_id: str = "", activity_instance_key: int = -1,
               custom_headers: bytes = EMPTY_DOCUMENT, payload: bytes = EMPTY_DOCUMENT) -> bytes:
    """JobRecord + JobHeaders (JobRecord.java:35-53, JobHeaders.java:33-51)."""
    headers = (_map(6) + mp_str("bpmnProcessId") + mp_str(bpmn_process_id)
               + mp_str("workflowDefinitionVersion") + mp_int(version) + mp_str("workflowKey") + mp_int(workflow_key)
               + mp_str("workflowInstanceKey") + mp_int(workflow_instance_key) + mp_str("activityId")
               + mp_str(activity_id) + mp_str("activityInstanceKey") + mp_int(activity_instance_key))
    return (_map(7) + mp_str("deadline") + mp_int(deadline) + mp_str("worker") + mp_str(worker)
            + mp_str("retries") + mp_int(retries) + mp_str("type") + mp_str(type) + mp_str("headers") + headers
            + mp_str("customHeaders") + custom_headers + mp_str("payload") + mp_bin(_doc(payload)))


def wis_record(workflow_instance_key: int = -1, activity_instance_key: int = -1, message_name: str = "",
               payload: bytes = EMPTY_DOCUMENT) -> bytes:
    """WorkflowInstanceSubscriptionRecord (WorkflowInstanceSubscriptionRecord.java:26-38)."""
    return (_map(4) + mp_str("workflowInstanceKey") + mp_int(workflow_instance_key) + mp_str("activityInstanceKey")
            + mp_int(activity_instance_key) + mp_str("messageName") + mp_str(message_name) + mp_str("payload")
            + mp_bin(_doc(payload)))


def _props(value: bytes) -> dict:
    """Top-level properties of a msgpack map -> raw value bytes of each (no re-encoding)."""
    import msgpack

    u = msgpack.Unpacker(raw=False)
    u.feed(value)
    n = u.read_map_header()
    out = {}
    for _ in range(n):
        k = u.unpack()
        start = u.tell()
        u.skip()
        out[k] = value[start:u.tell()]
    return out


def job_event(create_value: bytes, payload=None) -> bytes:
    """The value of a JOB event the job stream processor writes for a JOB CREATE command: the command's
    JobRecord (CreateJobProcessor accepts it as is, JobInstanceStreamProcessor.java:98-106), with the
    completing worker's payload (JobInstanceStreamProcessor.java:166-180) when given -- the shape
    WorkflowInstanceStreamProcessorTest.java:206-211 writes."""
    if payload is None:
        return create_value
    p = _props(create_value)
    out = _map(len(p))
    for k, raw in p.items():
        out += mp_str(k) + (mp_bin(_doc(payload)) if k == "payload" else raw)
    return out


# ---- log frames (zb_serialize_frames): DataFrameDescriptor.java:53-96 + LogEntryDescriptor.java:28-121 +
# RecordMetadata (protocol.xml:135-146; SBE message header + 34-byte block + varData rejectionReason)
FRAME_ALIGNMENT = 8
FLAG_BATCH_BEGIN, FLAG_BATCH_END = 0x80, 0x40
_DF = struct.Struct("<iBBhi")                 # framed length, version, flags, type, stream id
_LE = struct.Struct("<hhqiiqqqhh")            # version, reserved, position, raft term, producer id,
                                              # source event position, key, timestamp, metadata length, unused
_SBE = struct.Struct("<HHHHBiQQHBBQB")        # blockLength templateId schemaId version | recordType
                                              # requestStreamId requestId subscriptionId protocolVersion
                                              # valueType intent incidentKey rejectionType


def parse_frames(buf) -> list:
    """Log frames -> list of dicts (one per record), as a log reader (LoggedEventImpl) sees them."""
    buf = bytes(buf)
    out, off = [], 0
    while off < len(buf):
        framed, ver, flags, typ, stream = _DF.unpack_from(buf, off)
        le = off + _DF.size
        (_, _, pos, term, producer, src, key, ts, mlen, _) = _LE.unpack_from(buf, le)
        mo = le + _LE.size
        (blen, tmpl, schema, sver, rt, rsid, rid, sub, pver, vt, it, ik, rj) = _SBE.unpack_from(buf, mo)
        rlen = struct.unpack_from("<H", buf, mo + 8 + blen)[0]
        reason = buf[mo + 8 + blen + 2:mo + 8 + blen + 2 + rlen]
        value = buf[mo + mlen:off + framed]
        out.append(dict(framed_length=framed, version=ver, flags=flags, type=typ, stream_id=stream, position=pos,
                        raft_term=term, producer_id=producer, source_position=src, key=key, timestamp=ts,
                        metadata_length=mlen, block_length=blen, template_id=tmpl, schema_id=schema,
                        schema_version=sver, record_type=rt, request_stream_id=rsid, request_id=rid,
                        subscription_id=sub, protocol_version=pver, value_type=vt, intent=it, incident_key=ik,
                        rejection_type=rj, rejection_reason=reason, value=value))
        off += (framed + FRAME_ALIGNMENT - 1) & ~(FRAME_ALIGNMENT - 1)
    return out


def build_frame(f: dict) -> bytes:
    """The inverse of parse_frames for one record (fields as parse_frames returns them; framed_length and
    metadata_length are recomputed): what LogStreamBatchWriterImpl.writeEventsToBuffer (:222-268) writes into a
    claimed fragment, padded to FRAME_ALIGNMENT."""
    reason = bytes(f.get("rejection_reason", b""))
    value = bytes(f["value"])
    mlen = 8 + 34 + 2 + len(reason)
    framed = _DF.size + _LE.size + mlen + len(value)
    out = bytearray(_DF.pack(framed, 0, f.get("flags", 0), 0, f.get("stream_id", 0)))
    out += _LE.pack(0, 0, f["position"], f.get("raft_term", 0), f["producer_id"], f["source_position"], f["key"],
                    f.get("timestamp", 0), mlen, 0)
    out += _SBE.pack(34, 200, 0, 1, f["record_type"], f.get("request_stream_id", -(1 << 31)), f.get("request_id", (1 << 64) - 1),
                     f.get("subscription_id", (1 << 64) - 1), f.get("protocol_version", 1), f["value_type"],
                     f["intent"], f.get("incident_key", (1 << 64) - 1), f.get("rejection_type", 255))
    out += struct.pack("<H", len(reason)) + reason + value
    out += b"\0" * (-len(out) % FRAME_ALIGNMENT)
    return bytes(out)
