"""GPU engine vs the oracle on the paths beyond the CREATE-batch configs, through the C ABI:

* records submitted with zb_submit (the job stream processor's JOB CREATED / COMPLETED events with
  per-instance payloads, CANCEL, UPDATE_PAYLOAD, CORRELATE) with the harness off (ZB_CFG_EXTERNAL_JOBS);
* cancellation / termination (CancelWorkflowInstanceTest sequences, mid-task and mid-subprocess);
* C4 parallel fork / join (EXTENSION, parity with the oracle's definition);
* the final element-instance state (zb_read_instances vs the oracle's ElementInstanceIndex);
* snapshot -> restore -> continue equals an uninterrupted run.

Every log record is compared bit-exact (position, key, record / value type, intent, value bytes).
"""
import msgpack
import pytest

from frames_check import assert_frames_equal
from oracle import zbref
from zeebe_amd import bpmn, records as R, workloads

pytestmark = pytest.mark.gpu


def _engine(**kw):
    from zeebe_amd.engine import Engine

    kw.setdefault("log_capacity", 1 << 20)
    kw.setdefault("row_capacity", 1 << 18)
    return Engine(**kw)


def compare_logs(o, e, start=0):
    ref, got = o.records(start), e.records(start)
    assert len(got) == len(ref), (len(got), len(ref))
    for a, b in zip(ref, got):
        assert (a.position, a.source_position, a.key, a.record_type, a.value_type, a.intent) == \
               (b.position, b.source_position, b.key, b.record_type, b.value_type, b.intent), (a, b)
        if b.record_type == R.RT_REJECTION:
            assert a.rejection_type == b.rejection_type, (a, b)
        assert a.value == b.value, (a.position, msgpack.unpackb(a.value, raw=False), msgpack.unpackb(b.value, raw=False))
    assert_frames_equal(o, e, start)
    return ref


def compare_instances(o, e):
    ref, got = o.instances(), e.instances()
    assert len(got) == len(ref), (len(got), len(ref))
    for a, b in zip(ref, got):
        assert a[:4] == b[:4], (a, b)
        assert a[4] == b[4], (msgpack.unpackb(a[4], raw=False), msgpack.unpackb(b[4], raw=False))
    return ref


class Pair:
    """Drives the oracle and the GPU engine through the same inputs (the canonical schedule)."""

    def __init__(self, xml, external=False, wave_only=False, wf_key=100, **cap):
        self.o = zbref.Oracle()
        self.e = _engine(external_jobs=external, wave_only=wave_only, **cap)
        self.o.deploy(xml, wf_key, 1)
        self.e.deploy(xml, wf_key, 1)
        if external:
            self.o.set_harness(False)
        self.jobs_seen = 0
        self.job_key = {}

    def job_payload(self, act, p, wf_key=100):
        self.o.set_job_payload(wf_key, act, p)
        self.e.set_job_payload(wf_key, act, p)

    def create(self, process, payloads):
        for p in payloads:
            self.o.create(process, p)
        self.e.create(process, payloads)

    def submit(self, recs):
        for r in recs:
            self.o.submit(*r)
        self.e.submit_records(recs)

    def run(self):
        self.o.run()
        st = self.e.step()
        assert st["quiescent"], st
        return st

    def new_job_creates(self):
        """JOB CREATE commands written since the last call, with the job key the job stream processor
        would give them (KeyGenerator(2, 5) in order, JobInstanceStreamProcessor.java:76)."""
        out = []
        for r in self.o.records():
            if r.value_type == R.VT_JOB and r.record_type == R.RT_COMMAND and r.intent == R.JI_CREATE:
                if r.position not in self.job_key:
                    self.job_key[r.position] = 2 + 5 * len(self.job_key)
                    out.append((self.job_key[r.position], r))
        return out

    def check(self, start=0):
        compare_logs(self.o, self.e, start)
        compare_instances(self.o, self.e)
        oc, ec = self.o.counters(), self.e.counters()
        assert (ec["created"], ec["completed"], ec["canceled"], ec["next_wf_key"]) == \
               (oc["created"], oc["completed"], oc["canceled"], oc["next_wf_key"]), (oc, ec)


def job_events(creates, payload_of=None, created=True, completed=True):
    recs = []
    for key, rec in creates:
        if created:
            recs.append((R.RT_EVENT, R.VT_JOB, R.JI_CREATED, key, R.job_event(rec.value)))
        if completed:
            pl = payload_of(key, rec) if payload_of else None
            recs.append((R.RT_EVENT, R.VT_JOB, R.JI_COMPLETED, key, R.job_event(rec.value, pl)))
    return recs


# ------------------------------------------------------------------------------ C4 (EXTENSION)
@pytest.mark.parametrize("n,fanout,subs", [(3, 2, False), (7, 8, True), (1000, 8, True)])
def test_parallel_fork_join(n, fanout, subs):
    xml = bpmn.parallel_workflow(fanout, subprocesses=subs).to_xml()
    pr = Pair(xml, log_capacity=n * 400 + 4096, row_capacity=n * 40 + 1024, arena_bytes=(64 << 20) + n * 4096)
    for k in range(1, fanout + 1):
        pr.job_payload("task%d" % k, b"\x81" + workloads.mp_str("sub") + workloads.mp_int(k))
    blob, offs = workloads.order_payloads(n)
    pr.create("par", workloads.split(blob, offs))
    st = pr.run()
    assert st["path"] == 0  # parallel gateways run on the wave pipeline
    pr.check()
    assert st["completed_instances"] == n


def test_parallel_branches_consume_tokens():
    b = bpmn.Bpmn.create_executable_process("p").start_event("s").parallel_gateway("fork")
    b.sequence_flow_id("a").end_event("ea")
    b.move_to_node("fork").sequence_flow_id("b").service_task("t", type="t").end_event("eb")
    b.move_to_node("fork").sequence_flow_id("c").service_task("u", type="u").service_task("v", type="v").end_event("ec")
    pr = Pair(b.done().to_xml())
    pr.create("p", [msgpack.packb({"i": i}) for i in range(50)])
    pr.run()
    pr.check()
    assert pr.e.counters()["completed"] == 50


def test_parallel_with_external_jobs_and_cancel():
    """Jobs completed per branch in separate ticks, then the rest cancelled while several tokens are live."""
    xml = bpmn.parallel_workflow(4, subprocesses=True).to_xml()
    pr = Pair(xml, external=True)
    pr.create("par", [msgpack.packb({"orderId": i}) for i in range(20)])
    pr.run()
    creates = pr.new_job_creates()
    assert len(creates) == 80
    # tick 2: two branches of every instance complete (distinct activity instances: no race)
    done = [c for c in creates if msgpack.unpackb(c[1].value, raw=False)["headers"]["activityId"] in ("task1", "task3")]
    pr.submit(job_events(done, lambda k, r: msgpack.packb({"job": k})))
    pr.run()
    pr.check()
    # tick 3: cancel half of the instances (several live sub processes each)
    pos = pr.o.log_size()
    pr.submit([(R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_CANCEL, 1 + 5 * i, b"\x80") for i in range(0, 20, 2)])
    pr.run()
    pr.check(pos)
    # tick 4: the remaining jobs of the others complete -> their instances complete
    rest = [c for c in creates if c not in done
            and msgpack.unpackb(c[1].value, raw=False)["headers"]["workflowInstanceKey"] % 10 == 6]
    pr.submit(job_events(rest, lambda k, r: msgpack.packb({"late": k})))
    pr.run()
    pr.check()
    assert pr.e.counters()["completed"] == 10 and pr.e.counters()["canceled"] == 10


# ------------------------------------------------------------------------------ cancel (reference sequences)
@pytest.mark.parametrize("idx", range(4))
def test_cancel_reference_sequences(vectors, idx):
    case = vectors["cancels"][idx]
    pr = Pair(case["xml"], external=True)
    pr.create(case["process"], [bytes.fromhex(case["payload"])])
    pr.run()
    if case["job_created"]:
        pr.submit(job_events(pr.new_job_creates(), completed=False))
        pr.run()
    pr.check()
    pos = pr.o.log_size()
    pr.submit([(R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_CANCEL, 1, b"\x80")])
    pr.run()
    ref = compare_logs(pr.o, pr.e, pos)
    wf = [(msgpack.unpackb(r.value, raw=False).get("activityId") if r.record_type != R.RT_COMMAND else None,
           R.WI_NAMES[r.intent]) for r in ref if r.value_type == R.VT_WORKFLOW_INSTANCE]
    assert wf == [tuple(x) for x in case["expect"]]
    pr.check()
    assert pr.e.instances() == []


@pytest.mark.parametrize("wave_only", [False, True])
def test_cancel_mid_task_and_mid_subprocess(wave_only):
    """C4 twin (8 sub processes in sequence): instances at different tasks when cancelled; some cancels
    reject (already completed / unknown key)."""
    cfg = workloads.CONFIGS["c4twin"]
    pr = Pair(cfg["workflow"]().to_xml(), external=True, wave_only=wave_only)
    n = 60
    blob, offs = cfg["payloads"](n)
    pr.create(cfg["process"], workloads.split(blob, offs))
    pr.run()
    # advance instance i through i % 9 tasks (9 = completed) with per-instance payloads
    for step in range(8):
        creates = pr.new_job_creates()
        adv = [c for c in creates
               if (msgpack.unpackb(c[1].value, raw=False)["headers"]["workflowInstanceKey"] - 1) // 5 % 9 > step]
        if not adv:
            break
        pr.submit(job_events(adv, lambda k, r: msgpack.packb({"step": k, "w": r.position})))
        pr.run()
        pr.check()
    pos = pr.o.log_size()
    cancels = [(R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_CANCEL, 1 + 5 * i, b"\x80") for i in range(n)]
    cancels.append((R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_CANCEL, 123456789, b"\x80"))
    pr.submit(cancels)
    pr.run()
    pr.check(pos)
    assert pr.e.instances() == []


# ------------------------------------------------------------------------------ submitted records
def test_per_instance_job_payloads_chain():
    """A 3-task chain driven by the job stream processor's events with per-instance, per-task payloads."""
    xml = bpmn.chain_workflow(3).to_xml()
    pr = Pair(xml, external=True)
    n = 400
    blob, offs = workloads.order_payloads(n)
    pr.create("chain", workloads.split(blob, offs))
    pr.run()
    for t in range(3):
        creates = pr.new_job_creates()
        assert len(creates) == n
        pr.submit(job_events(creates, lambda k, r: msgpack.packb({"t%d" % t: k, "nested": {"k": [k, t]}})))
        pr.run()
        pr.check()
    assert pr.e.counters()["completed"] == n


def test_update_payload_and_rejections():
    cfg = workloads.CONFIGS["c1"]
    pr = Pair(cfg["workflow"]().to_xml(), external=True)
    pr.create("process", [msgpack.packb({"orderId": i}) for i in range(10)])
    pr.run()
    creates = pr.new_job_creates()
    ups = [(R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_UPDATE_PAYLOAD, -1 if i % 2 else 1 + 5 * i,
            R.wf_record(workflow_instance_key=1 + 5 * i, payload=msgpack.packb({"updated": i})))
           for i in range(0, 10, 2)]
    ups.append((R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_UPDATE_PAYLOAD, -1, R.wf_record(workflow_instance_key=999)))
    ups.append((R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_CANCEL, 998, b"\x80"))
    pr.submit(ups)
    pr.run()
    pr.check()
    pr.submit(job_events(creates, lambda k, r: msgpack.packb({"done": k})))
    pr.run()
    pr.check()


def test_submitted_correlate():
    """WORKFLOW_INSTANCE_SUBSCRIPTION CORRELATE from the subscription API, through zb_submit."""
    xml = bpmn.message_workflow().to_xml()
    pr = Pair(xml)
    pr.create("msg", [msgpack.packb({"orderId": "o-%d" % i}) for i in range(8)])
    pr.run()
    inst = {k: msgpack.unpackb(v, raw=False)["activityId"] for k, _, _, _, v in pr.o.instances()}
    waits = sorted(k for k, a in inst.items() if a == "wait")
    recs = [(R.RT_COMMAND, R.VT_WIS, R.WIS_CORRELATE, -1,
             R.wis_record(workflow_instance_key=1 + 5 * i, activity_instance_key=a, message_name="order",
                          payload=msgpack.packb({"paid": i})))
            for i, a in enumerate(waits[:5])]
    recs.append((R.RT_COMMAND, R.VT_WIS, R.WIS_CORRELATE, -1,
                 R.wis_record(workflow_instance_key=1, activity_instance_key=424242, message_name="order")))
    pr.submit(recs)
    pr.run()
    pr.check()
    assert pr.e.counters()["completed"] == 5


def test_submit_validation():
    from zeebe_amd.engine import ZbError

    cfg = workloads.CONFIGS["c1"]
    pr = Pair(cfg["workflow"]().to_xml(), external=True)
    pr.create("process", [b"\x80"])
    pr.run()
    e = pr.e
    n0 = e.log_size()
    with pytest.raises(ZbError):  # no workflow processor for JOB ACTIVATED
        e.submit_records([(R.RT_EVENT, R.VT_JOB, R.JI_ACTIVATED, 2, R.job_record())])
    # (a CANCEL and an UPDATE_PAYLOAD of one instance in one tick are accepted and serialised: test_gpu_races.py)
    with pytest.raises(ZbError):  # malformed value
        e.submit_records([(R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_CANCEL, 1, b"\x81\xa1")])
    # nothing was staged by the failed calls
    assert e.step()["records_processed"] == 0 and e.log_size() == n0


def test_submitted_creates_verbatim():
    """CREATE commands through zb_submit: the log keeps the client's bytes; unknown processes reject."""
    cfg = workloads.CONFIGS["c1"]
    pr = Pair(cfg["workflow"]().to_xml())
    for act, p in cfg["job_payloads"]().items():
        pr.job_payload(act, p)
    recs = [(R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_CREATE, -1,
             R.wf_record(bpmn_process_id="process", payload=msgpack.packb({"i": i}))) for i in range(5)]
    recs.append((R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_CREATE, -1, R.wf_record(bpmn_process_id="nope")))
    recs.append((R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_CREATE, -1,
                 R.wf_record(bpmn_process_id="process", version=1)))
    pr.submit(recs)
    pr.run()
    pr.check()


# ------------------------------------------------------------------------------ snapshot / restore
def test_snapshot_restore_continue():
    cfg = workloads.CONFIGS["c4twin"]
    xml = cfg["workflow"]().to_xml()
    n = 50
    blob, offs = cfg["payloads"](n)

    def drive(pr, stop_after=None):
        pr.create(cfg["process"], workloads.split(blob, offs))
        pr.run()
        for step in range(8):
            if stop_after is not None and step == stop_after:
                return
            creates = pr.new_job_creates()
            pr.submit(job_events(creates, lambda k, r: msgpack.packb({"s": k})))
            pr.run()

    full = Pair(xml, external=True)
    drive(full)
    part = Pair(xml, external=True)
    drive(part, stop_after=3)
    snap = part.e.snapshot()
    pos = part.e.log_size()
    part.e.close()
    from zeebe_amd.engine import Engine

    part.e = Engine(external_jobs=True, log_capacity=1 << 20, row_capacity=1 << 18)
    part.e.deploy(xml, 100, 1)
    part.e.restore(snap)
    assert part.e.log_size() == pos
    compare_instances(part.o, part.e)
    for step in range(3, 8):
        creates = part.new_job_creates()
        part.submit(job_events(creates, lambda k, r: msgpack.packb({"s": k})))
        part.run()
    compare_logs(full.o, part.e, pos)  # the restored engine continues exactly like the uninterrupted run
    compare_instances(full.o, part.e)
    assert part.e.counters()["completed"] == n
