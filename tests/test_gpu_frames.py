"""Log frames on the GPU (zb_serialize_frames) vs the oracle's, byte for byte.

Every GPU parity test already compares the frames of its whole log (tests/frames_check.py); these cases add
the request metadata of client commands (zb_set_request_metadata: CREATED and the CREATE rejection copy it,
WorkflowInstanceStreamProcessor.java:254-257, :370-377) on both pipelines, and frame invariants at a size
the oracle is not run on.
"""
import pytest

from frames_check import FRAME_CFG, assert_frames_equal
from oracle import zbref
from zeebe_amd import records as R, workloads

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("wave_only", [False, True])
def test_request_metadata(wave_only):
    from zeebe_amd.engine import Engine

    cfg = workloads.CONFIGS["c1"]
    xml = cfg["workflow"]().to_xml()
    payloads = workloads.split(*cfg["payloads"](40))
    o = zbref.Oracle()
    e = Engine(wave_only=wave_only)
    for x in (o, e):
        x.deploy(xml, 100, 1)
        for act, p in cfg["job_payloads"]().items():
            x.set_job_payload(100, act, p)
    ids = [5000 + 7 * i for i in range(len(payloads))]
    sids = [i % 3 for i in range(len(payloads))]
    for i, p in enumerate(payloads):
        o.create(cfg["process"], p)
        if i % 2 == 0:  # every other command carries request metadata
            o.set_request(o.log_size() - 1, ids[i], sids[i])
    e.create(cfg["process"], payloads)
    # request metadata of the last n staged records: here all of them, nulls where the oracle has none
    e.set_request_metadata([ids[i] if i % 2 == 0 else 2 ** 64 - 1 for i in range(len(payloads))],
                           [sids[i] if i % 2 == 0 else -(2 ** 31) for i in range(len(payloads))])
    # a command for a process that is not deployed: its rejection copies the request metadata too
    o.create("missing", b"\x80")
    o.set_request(o.log_size() - 1, 99, 9)
    e.create("missing", [b"\x80"])
    e.set_request_metadata([99], [9])
    o.run()
    st = e.step()
    assert st["quiescent"]
    assert_frames_equal(o, e)
    fr = R.parse_frames(e.frames(0, None, **FRAME_CFG))
    created = [f for f in fr if f["value_type"] == R.VT_WORKFLOW_INSTANCE and f["intent"] == R.WI_CREATED]
    assert [f["request_id"] for f in created[:2]] == [5000, 2 ** 64 - 1]
    rej = [f for f in fr if f["record_type"] == R.RT_REJECTION]
    assert [(f["request_id"], f["request_stream_id"], f["rejection_reason"]) for f in rej] == \
           [(99, 9, b"Workflow is not deployed")]
    e.close()


def test_frames_c2_properties():
    """C2 at 20k instances (trajectory template path): frame framing, batch flags and sources as invariants."""
    from zeebe_amd.engine import Engine

    n = 20000
    cfg = workloads.CONFIGS["c2"]
    e = Engine(log_capacity=1 << 23, row_capacity=1 << 20, arena_bytes=1 << 28)
    e.deploy(cfg["workflow"]().to_xml(), 100, 1)
    for act, p in cfg["job_payloads"]().items():
        e.set_job_payload(100, act, p)
    blob, offs = cfg["payloads"](n)
    e.create_packed(cfg["process"], blob, offs)
    st = e.step()
    assert st["quiescent"] and st["path"] in (1, 2)
    total = e.log_size()
    buf = e.frames(0, None, **FRAME_CFG)
    fr = R.parse_frames(buf)
    assert len(fr) == total == 169 * n  # CREATE, 108 WF events, 20 JOB CREATE, 40 harness job events
    recs = e.records()
    for f, r in zip(fr, recs):
        assert (f["position"], f["source_position"], f["key"], f["value"]) == \
               (r.position, r.source_position, r.key, r.value)
    # sources: every non-submitted record's source precedes it; batches are runs of one source
    runs = {}
    for f in fr:
        if f["source_position"] >= 0:
            assert f["source_position"] < f["position"]
            runs.setdefault(f["source_position"], []).append(f)
        else:
            assert f["flags"] == 0 and f["producer_id"] == -1
    for src, fs in runs.items():
        assert [g["position"] for g in fs] == list(range(fs[0]["position"], fs[0]["position"] + len(fs)))
        if len(fs) == 1:
            assert fs[0]["flags"] == 0
        else:
            assert fs[0]["flags"] == R.FLAG_BATCH_BEGIN and fs[-1]["flags"] == R.FLAG_BATCH_END
    e.close()


def test_frames_after_values_drain_with_rejections(monkeypatch):
    """records() then frames() over one log holding rejections: the values drain writes the measured
    value lengths back into the engine's length hints, and the frames size pass must still add each rejection's
    reason. Product configuration (no ZB_CFG_VLEN_CHECK): the size pass trusts the hints."""
    from zeebe_amd.engine import Engine

    cfg = workloads.CONFIGS["c1"]
    xml = cfg["workflow"]().to_xml()
    o = zbref.Oracle()
    e = Engine(external_jobs=True)
    o.set_harness(False)
    for x in (o, e):
        x.deploy(xml, 100, 1)
    payloads = workloads.split(*cfg["payloads"](30))
    for p in payloads:
        o.create(cfg["process"], p)
    o.create("missing", b"\x80")  # CREATE rejection
    e.create(cfg["process"], payloads)
    e.create("missing", [b"\x80"])
    o.run()
    assert e.step()["quiescent"]
    pos = o.log_size()
    # CANCEL of instances that do not exist / UPDATE_PAYLOAD of one that does not: NOT_APPLICABLE rejections
    recs = [(R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_CANCEL, 7777 + 5 * i, b"\x80") for i in range(3)]
    recs.append((R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_UPDATE_PAYLOAD, -1, R.wf_record(workflow_instance_key=999)))
    recs.append((R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_CANCEL, 1, b"\x80"))
    for r in recs:
        o.submit(*r)
    e.submit_records(recs)
    o.run()
    assert e.step()["quiescent"]
    ref, got = o.records(), e.records()  # the values drain first (writes the measured lengths back)
    assert [(r.key, r.record_type, r.intent, r.value) for r in ref] == [(r.key, r.record_type, r.intent, r.value)
                                                                        for r in got]
    assert sum(1 for r in got if r.record_type == R.RT_REJECTION) >= 5
    assert_frames_equal(o, e)
    assert_frames_equal(o, e, pos)
    e.close()
