"""The oracle's job stream processor (JobInstanceStreamProcessor.java:70-242), pinned on the
JobInstanceStreamProcessorTest sequences transcribed into tests/golden/reference_vectors.json ("job_sequences"),
plus the rejection reasons, the new-key rule for CREATE and UPDATE_RETRIES (not covered by that test class)."""
import msgpack

from oracle import zbref
from zeebe_amd import records as R

JOB = R.job_record(type="foo")                                     # job() :481-487
ACTIVATED = R.job_record(type="foo", worker="bar", deadline=1234)  # activatedJob(deadline) :489-497


def run_sequence(o, seq, key=None):
    o.set_job_processor(True)
    key = seq["key"] if key is None else key
    for batch in seq["batches"]:
        for intent in batch:
            value = JOB if intent in ("CREATE",) or (intent == "CANCEL" and seq["name"] == "cancel_created_job") \
                else ACTIVATED
            o.submit(R.RT_COMMAND, R.VT_JOB, R.JI_NAMES.index(intent), key, value)
        o.run()
    return [r for r in o.records() if r.value_type == R.VT_JOB]


def test_job_sequences(vectors):
    assert len(vectors["job_sequences"]) == 12
    for seq in vectors["job_sequences"]:
        recs = run_sequence(zbref.Oracle(), seq)
        got = [[R.RT_NAMES[r.record_type], R.JI_NAMES[r.intent]] for r in recs]
        assert got == seq["expect"], seq["name"]
        assert all(r.key == 1 for r in recs)


def test_rejection_reasons_and_values():
    o = zbref.Oracle()
    o.set_job_processor(True)
    for intent in (R.JI_ACTIVATE, R.JI_COMPLETE, R.JI_FAIL, R.JI_TIME_OUT, R.JI_UPDATE_RETRIES, R.JI_CANCEL):
        o.submit(R.RT_COMMAND, R.VT_JOB, intent, 7, ACTIVATED)
    o.run()
    fr = R.parse_frames(o.frames())
    rej = [(f["intent"], f["rejection_type"], f["rejection_reason"].decode()) for f in fr
           if f["record_type"] == R.RT_REJECTION]
    assert rej == [
        (R.JI_ACTIVATE, 1, "Job is not in one of these states: CREATED, FAILED, TIMED_OUT"),
        (R.JI_COMPLETE, 1, "Job is not in state: ACTIVATED, TIMED_OUT"),
        (R.JI_FAIL, 1, "Job is not in state ACTIVATED"),
        (R.JI_TIME_OUT, 1, "Job is not in state ACTIVATED"),
        (R.JI_UPDATE_RETRIES, 1, "Job is not in state FAILED"),
        (R.JI_CANCEL, 1, "Job does not exist")]
    assert all(f["producer_id"] == 10 for f in fr if f["record_type"] == R.RT_REJECTION)
    # the rejection carries the command's value (writeRejection(command, ...))
    vals = [r.value for r in o.records() if r.record_type == R.RT_REJECTION]
    assert all(msgpack.unpackb(v, raw=False)["worker"] == "bar" for v in vals)


def test_update_retries():
    o = zbref.Oracle()
    o.set_job_processor(True)
    for intent in (R.JI_CREATE, R.JI_ACTIVATE, R.JI_FAIL):
        o.submit(R.RT_COMMAND, R.VT_JOB, intent, 4, ACTIVATED)
        o.run()
    o.submit(R.RT_COMMAND, R.VT_JOB, R.JI_UPDATE_RETRIES, 4, R.job_record(type="foo", retries=0))
    o.submit(R.RT_COMMAND, R.VT_JOB, R.JI_UPDATE_RETRIES, 4, R.job_record(type="foo", retries=2))
    o.run()
    tail = [(r.record_type, r.intent, r.rejection_type) for r in o.records()[-4:]]
    assert tail == [(R.RT_COMMAND, R.JI_UPDATE_RETRIES, 255), (R.RT_COMMAND, R.JI_UPDATE_RETRIES, 255),
                    (R.RT_REJECTION, R.JI_UPDATE_RETRIES, 0), (R.RT_EVENT, R.JI_RETRIES_UPDATED, 255)]


def test_workflow_job_through_the_processor():
    """A service task's JOB CREATE gets its key from the job key generator (2, 7, ...), CREATED reaches the
    workflow processor, and a worker's ACTIVATE + COMPLETE complete the task with the COMPLETE payload."""
    from zeebe_amd import bpmn, workloads

    cfg = workloads.CONFIGS["c1"]
    o = zbref.Oracle()
    o.deploy(cfg["workflow"]().to_xml(), 100, 1)
    o.set_job_processor(True)
    for p in workloads.split(*cfg["payloads"](2)):
        o.create(cfg["process"], p)
    o.run()
    creates = [r for r in o.records() if r.value_type == R.VT_JOB and r.record_type == R.RT_COMMAND]
    created = [r for r in o.records() if r.value_type == R.VT_JOB and r.intent == R.JI_CREATED]
    assert [r.key for r in created] == [2, 7] and len(creates) == 2
    for r in created:
        o.submit(R.RT_COMMAND, R.VT_JOB, R.JI_ACTIVATE, r.key, R.job_event(r.value))
    o.run()
    for r in created:
        o.submit(R.RT_COMMAND, R.VT_JOB, R.JI_COMPLETE, r.key, R.job_event(r.value, b"\x81\xa4done\xc3"))
    o.run()
    assert o.counters()["completed"] == 2
    del bpmn
