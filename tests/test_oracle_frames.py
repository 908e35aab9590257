"""The oracle's log frames: the bytes LogStreamBatchWriterImpl / LogStreamWriterImpl lay
into the dispatcher buffer for every record the stepping path writes.

Pinned by the reference's own tests where they speak about bytes:
* ClaimedFragmentBatchTest.java:114-140, :206-229 -- a committed batch of two fragments carries BATCH_BEGIN on
  the first and BATCH_END on the last, a single-fragment batch no flags; the frame length field is
  framedLength(fragment) = fragment + DataFrameDescriptor.HEADER_LENGTH (12); fragments are 8-aligned;
  type TYPE_MESSAGE; stream id as claimed (LogStreamBatchWriterImpl.java:90: the partition id);
* LogEntryDescriptor.java:64-121 offsets (48-byte header: version, reserved, position, raft term, producer id,
  source event position, key, timestamp, metadata length, unused);
* LogStreamBatchWriterTest.java:236-286: each event's metadata block is written as given (here RecordMetadata).
The RecordMetadata block layout (protocol.xml:135-146, SBE 1.5.6 sequential offsets, 34-byte block) and the
producer ids (StreamProcessorIds.java:23-39) follow the source: no reference test pins their bytes (parity
unpinned).
"""
import struct

import msgpack

from oracle import zbref
from zeebe_amd import records as R, workloads


def _run(cfg="c1", n=3, request=None):
    c = workloads.CONFIGS[cfg]
    o = zbref.Oracle()
    o.deploy(c["workflow"]().to_xml(), 100, 1)
    for act, p in c["job_payloads"]().items():
        o.set_job_payload(100, act, p)
    for i, p in enumerate(workloads.split(*c["payloads"](n))):
        o.create(c["process"], p)
        if request:
            o.set_request(o.log_size() - 1, *request(i))
    o.run()
    return o


def test_frame_layout_matches_records():
    o = _run("c1", 3)
    recs = o.records()
    buf = o.frames(stream_id=7, raft_term=3, timestamp=1234567)
    fr = R.parse_frames(buf)
    assert len(fr) == len(recs)
    off = 0
    for f, r in zip(fr, recs):
        assert off % R.FRAME_ALIGNMENT == 0
        mlen = 8 + 34 + 2 + len(f["rejection_reason"])
        assert f["metadata_length"] == mlen
        assert f["framed_length"] == 12 + 48 + mlen + len(r.value)  # framedLength(fragment)
        assert (f["version"], f["type"], f["stream_id"], f["raft_term"], f["timestamp"]) == (0, 0, 7, 3, 1234567)
        assert (f["position"], f["key"], f["source_position"]) == (r.position, r.key, r.source_position)
        assert (f["record_type"], f["value_type"], f["intent"], f["rejection_type"]) == \
               (r.record_type, r.value_type, r.intent, r.rejection_type)
        assert (f["block_length"], f["template_id"], f["schema_id"], f["schema_version"]) == (34, 200, 0, 1)
        assert f["protocol_version"] == 1
        assert f["subscription_id"] == 2 ** 64 - 1 and f["incident_key"] == 2 ** 64 - 1
        assert f["value"] == r.value
        pad = buf[off + f["framed_length"]:off + ((f["framed_length"] + 7) & ~7)]
        assert pad == b"\0" * len(pad)
        off += (f["framed_length"] + 7) & ~7
    assert off == len(buf)


def test_batch_flags_and_producers():
    o = _run("c1", 2)
    recs, fr = o.records(), R.parse_frames(o.frames())
    by_src = {}
    for r in recs:
        by_src.setdefault(r.source_position, []).append(r.position)
    for r, f in zip(recs, fr):
        group = by_src[r.source_position] if r.source_position >= 0 else [r.position]
        if len(group) == 1:  # ClaimedFragmentBatchTest.shouldCommitSingleFragmentBatch: no flags
            assert f["flags"] == 0
        elif r.position == group[0]:
            assert f["flags"] == R.FLAG_BATCH_BEGIN
        elif r.position == group[-1]:
            assert f["flags"] == R.FLAG_BATCH_END
        else:
            assert f["flags"] == 0
        if r.source_position < 0:  # submitted by the client API: LogStreamWriterImpl defaults
            assert f["producer_id"] == -1
        elif r.value_type == R.VT_JOB and r.record_type == R.RT_EVENT:
            assert f["producer_id"] == 10  # the job processor (harness)
        else:
            assert f["producer_id"] == 70  # WORKFLOW_INSTANCE_PROCESSOR_ID
    # CREATE -> CREATED + ELEMENT_READY is one batch (acceptCommand :357-365)
    created = [f for f in fr if f["value_type"] == R.VT_WORKFLOW_INSTANCE and f["intent"] == R.WI_CREATED]
    assert created and all(f["flags"] == R.FLAG_BATCH_BEGIN for f in created)


def test_request_metadata_follows_create():
    o = _run("c1", 2, request=lambda i: (1000 + i, 40 + i))
    fr = R.parse_frames(o.frames())
    null_id, null_sid = 2 ** 64 - 1, -(2 ** 31)
    for f in fr:
        if f["value_type"] == R.VT_WORKFLOW_INSTANCE and f["intent"] in (R.WI_CREATE, R.WI_CREATED):
            inst = 0 if f["intent"] == R.WI_CREATE and f["position"] == 0 else None
            assert f["request_id"] in (1000, 1001) and f["request_stream_id"] in (40, 41), f
            if inst is not None:
                assert (f["request_id"], f["request_stream_id"]) == (1000, 40)
        else:  # RecordMetadata.reset on every other write
            assert (f["request_id"], f["request_stream_id"]) == (null_id, null_sid), f


def test_rejection_reason_in_metadata():
    o = zbref.Oracle()
    o.create("missing", b"\x80")
    o.submit(R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_CANCEL, 99, b"\x80")
    o.run()
    fr = R.parse_frames(o.frames())
    rej = [f for f in fr if f["record_type"] == R.RT_REJECTION]
    assert [(f["intent"], f["rejection_type"], f["rejection_reason"]) for f in rej] == [
        (R.WI_CREATE, 0, b"Workflow is not deployed"), (R.WI_CANCEL, 1, b"Workflow instance is not running")]
    for f in rej:
        assert f["metadata_length"] == 44 + len(f["rejection_reason"])
        assert f["producer_id"] == 70 and f["flags"] == 0
    assert [f["rejection_type"] for f in fr if f["record_type"] != R.RT_REJECTION] == [255] * (len(fr) - 2)


def test_message_processor_frames():
    o = zbref.Oracle()
    o.publish(b"order", b"k1", b"\x80", 0)  # ttl 0: PUBLISHED + DELETED in one batch
    o.run()
    fr = R.parse_frames(o.frames())
    ev = [f for f in fr if f["record_type"] == R.RT_EVENT]
    assert [f["flags"] for f in ev] == [R.FLAG_BATCH_BEGIN, R.FLAG_BATCH_END]
    assert all(f["producer_id"] == 90 for f in ev)
    assert msgpack.unpackb(ev[0]["value"], raw=False)["name"] == "order"
    assert struct.unpack_from("<i", o.frames(), 0)[0] == fr[0]["framed_length"]
