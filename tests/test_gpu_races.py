"""Records of one workflow instance that race inside a tick (include/zb_engine.h, zb_submit): the reference's
processor takes them one after the other in log order (WorkflowInstanceStreamProcessor.java:511-576 guards,
BpmnStepProcessor.java:128-150), so the engine must give the same records as processing them sequentially. zb_submit
marks such instances as conflicting and zb_step cuts every generation of the tick before the next record of one of
them (k_conflict, zb_wave.hip); the other instances of the tick stay in lockstep.

Every case is compared with the oracle (a sequential restatement) at every tick: records (positions, source
positions, keys, values), log frames, element-instance state and key generators.
"""
import msgpack
import pytest

from frames_check import assert_frames_equal
from oracle import zbref
from zeebe_amd import records as R, workloads

pytestmark = pytest.mark.gpu


def _compare(o, e, start):
    ref, got = o.records(start), e.records(start)
    assert len(got) == len(ref), (len(got), len(ref))
    for a, b in zip(ref, got):
        assert (a.position, a.source_position, a.key, a.record_type, a.value_type, a.intent, a.rejection_type) == \
               (b.position, b.source_position, b.key, b.record_type, b.value_type, b.intent, b.rejection_type), (a, b)
        assert a.value == b.value, (a.position, msgpack.unpackb(a.value, raw=False), msgpack.unpackb(b.value, raw=False))
    assert_frames_equal(o, e, start)
    assert o.instances() == e.instances()
    oc, ec = o.counters(), e.counters()
    assert (ec["created"], ec["completed"], ec["canceled"], ec["next_wf_key"], ec["next_job_key"]) == \
           (oc["created"], oc["completed"], oc["canceled"], oc["next_wf_key"], oc["next_job_key"]), (oc, ec)
    return len(ref)


class Pair:
    """The oracle and the engine fed the same records in the same order (external job processor: job keys 2 + 5j
    in JOB CREATE order)."""

    def __init__(self, xmls, job_processor=False):
        from zeebe_amd.engine import Engine

        self.o = zbref.Oracle()
        if job_processor:
            self.o.set_job_processor(True)
        else:
            self.o.set_harness(False)
        self.e = Engine(external_jobs=not job_processor, job_processor=job_processor, log_capacity=1 << 18,
                        row_capacity=1 << 15, arena_bytes=16 << 20)
        for k, xml in xmls.items():
            self.o.deploy(xml, k, 1)
            self.e.deploy(xml, k, 1)
        self.scan = 0
        self.jobs = []  # (key, JOB CREATE / CREATED record value, workflow instance key)

    def tick(self, creates=(), recs=(), by_one=False):
        start = self.e.log_size()
        assert start == self.o.log_size()
        for process, payloads in creates:
            for p in payloads:
                self.o.create(process, p)
            self.e.create(process, payloads)
        for r in recs:
            self.o.submit(*r)
        if by_one:  # (several zb_submit calls: the conflict rules apply across them)
            for r in recs:
                self.e.submit_records([r])
        elif recs:
            self.e.submit_records(list(recs))
        self.o.run()
        st = self.e.step()
        assert st["quiescent"], st
        n = _compare(self.o, self.e, start)
        self.e.release(self.e.log_size())
        for r in self.o.records(self.scan):
            if r.value_type == R.VT_JOB and r.intent == (R.JI_CREATED if self.job_processor_mode() else R.JI_CREATE) \
                    and r.record_type == (R.RT_EVENT if self.job_processor_mode() else R.RT_COMMAND):
                wik = msgpack.unpackb(r.value, raw=False)["headers"]["workflowInstanceKey"]
                key = r.key if self.job_processor_mode() else 2 + 5 * len(self.jobs)
                self.jobs.append((key, r.value, wik))
        self.scan = self.o.log_size()
        return n

    def job_processor_mode(self):
        return bool(self.e._flags & 4)

    def job_of(self, wik, last=True):
        js = [j for j in self.jobs if j[2] == wik]
        return js[-1] if last else js[0]

    def roots(self):
        return [k for k, parent, *_ in self.e.instances() if parent == -1]


def _created(j):
    return (R.RT_EVENT, R.VT_JOB, R.JI_CREATED, j[0], R.job_event(j[1]))


def _completed(j, pl=None):
    return (R.RT_EVENT, R.VT_JOB, R.JI_COMPLETED, j[0], R.job_event(j[1], pl or msgpack.packb({"done": j[0]})))


def _cancel(wik):
    return (R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_CANCEL, wik, b"\x80")


def _update(wik, doc):
    return (R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_UPDATE_PAYLOAD, wik,
            R.wf_record(workflow_instance_key=wik, payload=msgpack.packb(doc)))


@pytest.mark.parametrize("by_one", [False, True])
def test_racing_records_in_one_tick(by_one):
    c1, c4t, c2 = workloads.CONFIGS["c1"], workloads.CONFIGS["c4twin"], workloads.CONFIGS["c2"]
    p = Pair({100: c1["workflow"]().to_xml(), 200: c4t["workflow"]().to_xml(), 300: c2["workflow"]().to_xml()})
    pays = lambda n, b: [msgpack.packb({"orderId": b + i, "blob": "q" * ((b + i) % 23)}) for i in range(n)]  # noqa
    p.tick([("process", pays(12, 0)), ("subs", pays(12, 100)), ("chain", pays(40, 200))])
    roots = p.roots()
    assert len(roots) == 64
    a, b, c, d, f, g, h, k = roots[:8]
    quiet = roots[8:]
    # tick 1: every race the lockstep wave cannot take, next to many quiet instances completing their jobs
    recs = [_cancel(a), _created(p.job_of(a)), _completed(p.job_of(a)),          # cancel, then its job completes
            _created(p.job_of(b)), _completed(p.job_of(b)), _cancel(b),          # job completes, then cancel
            _cancel(c), _cancel(c),                                              # cancelled twice
            _update(d, {"u": 1}), _created(p.job_of(d)), _completed(p.job_of(d)),  # update, then completion
            _created(p.job_of(f)), _completed(p.job_of(f)), _update(f, {"u": 2}),  # completion, then update
            _update(g, {"u": 3}), _update(g, {"u": 4}),                          # two updates
            _created(p.job_of(h))]                                               # created, 20 records ...
    recs += [_created(p.job_of(q)) for q in quiet[:20]]
    recs += [_completed(p.job_of(h))]                                             # ... completed later
    recs += [_completed(p.job_of(q)) for q in quiet[:20]]
    recs += [_update(k, {"u": 5}), _cancel(k), _update(k, {"u": 6})]            # update, cancel, update
    recs += [_created(p.job_of(q)) for q in quiet[20:]] + [_completed(p.job_of(q)) for q in quiet[20:]]
    n = p.tick(recs=recs, by_one=by_one)
    assert n > 200
    # tick 2: the survivors race again (completion + cancel of the same instances), plus new instances
    roots = p.roots()
    recs = []
    for i, r in enumerate(roots[:10]):
        j = p.job_of(r)
        recs += [_created(j), _cancel(r), _completed(j)] if i % 2 else [_update(r, {"v": i}), _created(j), _completed(j)]
    p.tick([("chain", pays(10, 900))], recs, by_one=by_one)
    # tick 3: nothing races (the conflict set of the last tick must not linger)
    roots = p.roots()
    p.tick(recs=[x for r in roots[:10] for x in (_created(p.job_of(r)), _completed(p.job_of(r)))])


def test_duplicate_job_completion_fails_like_the_reference():
    """Two JOB COMPLETED events for one job in a tick: both pass JobCompletedEventProcessor (the activity is still
    ACTIVATED when each is processed) and both write ELEMENT_COMPLETING; the second COMPLETING finds no element
    instance and the reference's noConcurrentTransitionGuard throws a NullPointerException
    (BpmnStepProcessor.java:128-150), which fails the processor. The engine fails the step the same way rather
    than writing records the reference never writes."""
    from zeebe_amd.engine import ZbError

    c1 = workloads.CONFIGS["c1"]
    p = Pair({100: c1["workflow"]().to_xml()})
    p.tick([("process", [msgpack.packb({"orderId": i}) for i in range(4)])])
    j = p.job_of(p.roots()[1])
    recs = [_created(j), _completed(j), _completed(j, msgpack.packb({"again": 1}))]
    for r in recs:
        p.o.submit(*r)
    with pytest.raises(zbref.ZbrefError, match="noConcurrentTransitionGuard"):
        p.o.run()
    p.e.submit_records(recs)
    with pytest.raises(ZbError):
        p.e.step()


def test_racing_job_commands():
    """The job stream processor on the GPU (ZB_CFG_JOB_PROCESSOR): more than two commands for a job in one tick, and a
    job's commands separated by other records (JobInstanceStreamProcessor.java:70-242, processed in log order)."""
    c1 = workloads.CONFIGS["c1"]
    p = Pair({100: c1["workflow"]().to_xml()}, job_processor=True)
    p.tick([("process", [msgpack.packb({"orderId": i}) for i in range(16)])])
    jobs = list(p.jobs)

    def act(j, worker="w"):
        v = msgpack.unpackb(R.job_event(j[1]), raw=False)
        v.update(worker=worker, deadline=10 ** 12)
        return (R.RT_COMMAND, R.VT_JOB, R.JI_ACTIVATE, j[0], msgpack.packb(v))

    def comp(j, doc):
        v = msgpack.unpackb(R.job_event(j[1], msgpack.packb(doc)), raw=False)
        return (R.RT_COMMAND, R.VT_JOB, R.JI_COMPLETE, j[0], msgpack.packb(v))

    def fail(j):
        v = msgpack.unpackb(R.job_event(j[1]), raw=False)
        v.update(retries=0)
        return (R.RT_COMMAND, R.VT_JOB, R.JI_FAIL, j[0], msgpack.packb(v))

    recs = []
    for i, j in enumerate(jobs):
        if i % 4 == 0:    # activate, complete, complete again (rejected)
            recs += [act(j), comp(j, {"a": i}), comp(j, {"b": i})]
        elif i % 4 == 1:  # activate, fail, then activate again
            recs += [act(j), fail(j), act(j, "x")]
        elif i % 4 == 2:  # activate ... (others) ... complete
            recs.append(act(j))
        else:
            recs += [act(j), comp(j, {"c": i})]
    recs += [comp(j, {"late": i}) for i, j in enumerate(jobs) if i % 4 == 2]
    p.tick(recs=recs)
    p.tick(recs=[act(j) for i, j in enumerate(jobs) if i % 4 == 1])


def test_racing_commands_of_jobs_without_headers():
    """Jobs created by JOB CREATE commands with no workflow headers (JobHeaders.workflowInstanceKey -1,
    JobHeaders.java:33-51) under the job stream processor: their commands race only with the same job's commands, so
    zb_submit keys them by job key (conflict_key, zb_device.hpp) and k_conflict cuts the generation before the next
    command of such a job. Before that key, two commands of one such job that were not next to each other ran in one
    lockstep wave against the same job state (JobInstanceStreamProcessor.java:70-242 takes them in log order)."""
    c1 = workloads.CONFIGS["c1"]
    p = Pair({100: c1["workflow"]().to_xml()}, job_processor=True)
    creates = [(R.RT_COMMAND, R.VT_JOB, R.JI_CREATE, -1, R.job_record(type="ext%d" % i, retries=3)) for i in range(8)]
    p.tick([("process", [msgpack.packb({"orderId": i}) for i in range(8)])], recs=creates)
    free = [j for j in p.jobs if j[2] == -1]
    bound = [j for j in p.jobs if j[2] != -1]
    assert len(free) == 8 and len(bound) == 8

    def cmd(intent, j, **kw):
        v = msgpack.unpackb(j[1], raw=False)
        v.update(kw)
        return (R.RT_COMMAND, R.VT_JOB, intent, j[0], msgpack.packb(v))

    recs = [cmd(R.JI_ACTIVATE, j, worker="w", deadline=10 ** 12) for j in free + bound]  # every job activated ...
    recs += [cmd(R.JI_COMPLETE, j) for j in free[:4]]                                   # ... then completed
    recs += [cmd(R.JI_FAIL, j, retries=0) for j in free[4:]]                            # ... or failed
    recs += [cmd(R.JI_COMPLETE, j) for j in bound]
    recs += [cmd(R.JI_UPDATE_RETRIES, j, retries=2) for j in free[4:]]                   # failed -> retries updated
    recs += [cmd(R.JI_ACTIVATE, j, worker="x", deadline=10 ** 12) for j in free]        # rejected for the completed
    p.tick(recs=recs)
    p.tick(recs=[cmd(R.JI_CANCEL, j) for j in free] + [cmd(R.JI_CANCEL, j) for j in free[:2]])
