"""The oracle's cancel / terminate path, submitted records (external job processor) and the C4
parallel-gateway extension.

Cancel sequences are pinned by CancelWorkflowInstanceTest.java (transcribed into
tests/golden/reference_vectors.json "cancels"). Parallel gateways are an EXTENSION the reference rejects
at deployment (FlowElementValidator.java:36-58): their semantics are checked here as
properties, parity unpinned.
"""
import msgpack
import pytest

from oracle import zbref
from zeebe_amd import bpmn, records as R, workloads

WFN = R.WI_NAMES


def _wf(rec):
    return msgpack.unpackb(rec.value, raw=False)


def _job_creates(o, start=0):
    return [r for r in o.records(start) if r.value_type == R.VT_JOB and r.record_type == R.RT_COMMAND
            and r.intent == R.JI_CREATE]


def run_cancel_case(o, case):
    """Drive one CancelWorkflowInstanceTest case on an engine with the partition interface of
    zbref.Oracle / zeebe_amd.engine.Engine (harness off); returns the log position of the CANCEL."""
    o.deploy(case["xml"], 100, 1)
    o.set_harness(False)
    o.create(case["process"], bytes.fromhex(case["payload"]))
    o.run()
    if case["job_created"]:
        (jc,) = _job_creates(o)
        o.submit(R.RT_EVENT, R.VT_JOB, R.JI_CREATED, 2, R.job_event(jc.value))
        o.run()
    pos = o.log_size()
    o.submit(R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_CANCEL, 1, b"\x80")  # TestTopicClient: empty value
    o.run()
    return pos


@pytest.mark.parametrize("idx", range(4))
def test_cancel_sequences(vectors, idx):
    case = vectors["cancels"][idx]
    o = zbref.Oracle()
    pos = run_cancel_case(o, case)
    recs = o.records(pos)
    wf = [(_wf(r).get("activityId") if r.record_type != R.RT_COMMAND else None, WFN[r.intent])
          for r in recs if r.value_type == R.VT_WORKFLOW_INSTANCE]
    assert wf == [tuple(x) for x in case["expect"]]
    term = [r for r in recs if r.value_type == R.VT_WORKFLOW_INSTANCE and r.intent == R.WI_ELEMENT_TERMINATED]
    terminating = {r.key: r.position for r in recs
                   if r.value_type == R.VT_WORKFLOW_INSTANCE and r.intent == R.WI_ELEMENT_TERMINATING}
    # the process instance's TERMINATED carries the payload the CANCEL emptied on the indexed value
    proc = term[-1]
    assert proc.key == 1 and _wf(proc)["payload"] == b"\x80"
    if case["name"] == "cancel_intermediate_catch_event":
        ce = term[0]
        assert ce.source_position == terminating[ce.key]
    if "expect_job_cancel_headers" in case:
        (jc,) = [r for r in recs if r.value_type == R.VT_JOB and r.intent == R.JI_CANCEL]
        assert jc.record_type == R.RT_COMMAND and jc.key == 2
        task_terminating = [r for r in recs if r.value_type == R.VT_WORKFLOW_INSTANCE
                            and r.intent == R.WI_ELEMENT_TERMINATING and _wf(r)["activityId"] == "task"][0]
        assert jc.source_position == task_terminating.position
        h = msgpack.unpackb(jc.value, raw=False)["headers"]
        for k, v in case["expect_job_cancel_headers"].items():
            assert h[k] == v
        assert h["workflowInstanceKey"] == 1
    assert o.counters()["canceled"] == 1
    assert o.instances() == []


def test_cancel_rejections():
    o = zbref.Oracle()
    o.submit(R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_CANCEL, 77, b"\x80")
    o.run()
    (c, rej) = o.records()
    assert rej.record_type == R.RT_REJECTION and rej.rejection_type == 1 and rej.key == 77
    # UPDATE_PAYLOAD of an unknown instance: NOT_APPLICABLE rejection of the (re-encoded) command
    o.submit(R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_UPDATE_PAYLOAD, -1, R.wf_record(workflow_instance_key=5))
    o.run()
    assert o.records()[-1].record_type == R.RT_REJECTION


def test_update_payload_then_complete():
    """UpdatePayloadProcessor :557-576: the instance's indexed payload is replaced; the task's completion merges
    into the updated scope payload (OutputMappingHandler :56-75)."""
    xml = workloads.CONFIGS["c1"]["workflow"]().to_xml()
    o = zbref.Oracle()
    o.deploy(xml, 100, 1)
    o.set_harness(False)
    o.create("process", msgpack.packb({"orderId": 1}))
    o.run()
    (jc,) = _job_creates(o)
    new = msgpack.packb({"orderId": 2, "extra": True})
    o.submit(R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_UPDATE_PAYLOAD, 1,
             R.wf_record(workflow_instance_key=1, payload=new))
    o.run()
    assert o.records()[-1].intent == R.WI_PAYLOAD_UPDATED
    inst = {k: v for k, _, _, _, v in o.instances()}
    assert msgpack.unpackb(_wfv(inst[1])["payload"]) == {"orderId": 2, "extra": True}
    o.submit(R.RT_EVENT, R.VT_JOB, R.JI_CREATED, 2, R.job_event(jc.value))
    o.submit(R.RT_EVENT, R.VT_JOB, R.JI_COMPLETED, 2, R.job_event(jc.value, msgpack.packb({"done": 1})))
    o.run()
    done = [r for r in o.records() if r.value_type == R.VT_WORKFLOW_INSTANCE and r.intent == R.WI_ELEMENT_COMPLETED
            and _wf(r)["activityId"] == "task"][0]
    assert msgpack.unpackb(_wf(done)["payload"]) == {"orderId": 2, "extra": True, "done": 1}
    assert o.counters()["completed"] == 1


def _wfv(v):
    return msgpack.unpackb(v, raw=False)


def test_submitted_records_kept_verbatim():
    """Records written by other writers stay in the log as written (the job events' bytes)."""
    xml = workloads.CONFIGS["c1"]["workflow"]().to_xml()
    o = zbref.Oracle()
    o.deploy(xml, 100, 1)
    o.set_harness(False)
    o.create("process", b"\x80")
    o.run()
    (jc,) = _job_creates(o)
    ev = R.job_event(jc.value, msgpack.packb({"x": 1}))
    o.submit(R.RT_EVENT, R.VT_JOB, R.JI_COMPLETED, 2, ev)
    o.run()
    assert [r.value for r in o.records() if r.value_type == R.VT_JOB and r.intent == R.JI_COMPLETED] == [ev]
    # job key was never set (no JOB CREATED): completion still completes the activity
    assert o.counters()["completed"] == 1


def test_instances_dump_mid_flight():
    xml = workloads.CONFIGS["c4twin"]["workflow"]().to_xml()
    o = zbref.Oracle()
    o.deploy(xml, 100, 1)
    o.set_harness(False)
    for i in range(3):
        o.create("subs", msgpack.packb({"orderId": i}))
    o.run()
    inst = o.instances()
    # per instance: the process, sub1 (child of the process) and task1 (child of sub1), all ACTIVATED
    assert len(inst) == 9
    by = {k: (pk, st, _wfv(v)["activityId"]) for k, pk, jk, st, v in inst}
    for k, (pk, st, aid) in by.items():
        assert st == R.WI_ELEMENT_ACTIVATED
        if aid == "subs":
            assert pk == -1
        elif aid == "sub1":
            assert by[pk][2] == "subs"
        else:
            assert aid == "task1" and by[pk][2] == "sub1"


# ------------------------------------------------------------------------------ C4 extension
def _c4(n, fanout=8, subprocesses=True):
    xml = bpmn.parallel_workflow(fanout, subprocesses=subprocesses).to_xml()
    o = zbref.Oracle()
    o.deploy(xml, 100, 1)
    for k in range(1, fanout + 1):
        o.set_job_payload(100, "task%d" % k, b"\x81" + workloads.mp_str("sub") + workloads.mp_int(k))
    for i in range(n):
        o.create("par", msgpack.packb({"orderId": i}))
    o.run()
    return o


def test_parallel_fork_join_properties():
    n, F = 5, 8
    o = _c4(n, F)
    recs = o.records()
    wf = [r for r in recs if r.value_type == R.VT_WORKFLOW_INSTANCE and r.record_type == R.RT_EVENT]
    by_inst = {}
    for r in wf:
        by_inst.setdefault(_wf(r)["workflowInstanceKey"], []).append(r)
    assert len(by_inst) == n
    for ik, rs in by_inst.items():
        ids = [(_wf(r)["activityId"], r.intent) for r in rs]
        # one fork activation emits F flows, in executable (reverse document) order, as one batch
        ga = [r for r in rs if r.intent == R.WI_GATEWAY_ACTIVATED]
        assert [_wf(r)["activityId"] for r in ga] == ["fork", "join"]
        forks = [r for r in rs if r.source_position == ga[0].position]
        assert [_wf(r)["activityId"] for r in forks] == ["b%d" % k for k in range(F, 0, -1)]
        # the join fires once, on the last arrival (in log order) of its F incoming flows
        arrivals = [r for r in rs if r.intent == R.WI_SEQUENCE_FLOW_TAKEN and _wf(r)["activityId"].startswith("j")]
        assert len(arrivals) == F and ga[1].source_position == max(a.position for a in arrivals)
        # every sub process completes; the process completes exactly once, after the join
        assert sum(1 for a, it in ids if a.startswith("sub") and it == R.WI_ELEMENT_COMPLETED) == F
        assert ids[-1] == ("par", R.WI_ELEMENT_COMPLETED)
        assert sum(1 for a, it in ids if a == "par" and it == R.WI_ELEMENT_COMPLETED) == 1
    c = o.counters()
    assert c["completed"] == n and c["live_instances"] == 0


def test_parallel_without_join_consumes_tokens():
    """Branches ending at their own end events: the scope completes when its last token is consumed."""
    b = bpmn.Bpmn.create_executable_process("p").start_event("s").parallel_gateway("fork")
    b.sequence_flow_id("a").end_event("ea")
    b.move_to_node("fork").sequence_flow_id("b").service_task("t", type="t").end_event("eb")
    xml = b.done().to_xml()
    o = zbref.Oracle()
    o.deploy(xml, 100, 1)
    o.create("p", b"\x80")
    o.run()
    wf = [(_wf(r)["activityId"], r.intent) for r in o.records()
          if r.value_type == R.VT_WORKFLOW_INSTANCE and r.record_type == R.RT_EVENT]
    assert wf.count(("p", R.WI_ELEMENT_COMPLETING)) == 1 and wf[-1] == ("p", R.WI_ELEMENT_COMPLETED)
    # the process completes after the second end event, not the first
    ends = [i for i, x in enumerate(wf) if x[1] == R.WI_END_EVENT_OCCURRED]
    assert len(ends) == 2 and wf.index(("p", R.WI_ELEMENT_COMPLETING)) > ends[1]
    assert o.counters()["completed"] == 1


def test_parallel_cancel_terminates_every_branch():
    """Cancel with several live tokens (EXTENSION): children terminate one after another."""
    xml = bpmn.parallel_workflow(3, subprocesses=False).to_xml()
    o = zbref.Oracle()
    o.deploy(xml, 100, 1)
    o.set_harness(False)
    o.create("par", b"\x80")
    o.run()
    assert len(o.instances()) == 4
    pos = o.log_size()
    o.submit(R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_CANCEL, 1, b"\x80")
    o.run()
    wf = [(_wf(r).get("activityId"), WFN[r.intent]) for r in o.records(pos)
          if r.value_type == R.VT_WORKFLOW_INSTANCE and r.record_type == R.RT_EVENT]
    assert wf[:2] == [("par", "CANCELING"), ("par", "ELEMENT_TERMINATING")]
    assert sum(1 for x in wf if x[1] == "ELEMENT_TERMINATED") == 4 and wf[-1] == ("par", "ELEMENT_TERMINATED")
    assert o.instances() == [] and o.counters()["canceled"] == 1
