"""The steady-state workload of `bench.py --config c2 --steady` (bench_steady.py, the `extras.c2_steady` line) under
parity: the same schedule -- a live population of 20-task chain instances waiting on jobs; per tick JOB CREATED +
JOB COMPLETED events for a quarter of the pending jobs (the completing worker's payload merged into the instance),
the CREATE commands that keep the population near its size and CANCEL commands for waiting instances -- with the
external job processor (WorkflowInstanceStreamProcessor.java:408-576: JobCreatedProcessor, JobCompletedEventProcessor,
CancelWorkflowInstanceProcessor).

* test_steady_schedule_vs_oracle: a few thousand live instances for 10 ticks, through capacities that make the engine
  compact, every tick compared with the oracle (positions, source positions, keys, values, log frames,
  element-instance state, counters).
* test_steady_schedule_properties_1m: the bench's own size (1M live instances) for 4 ticks: per tick the records
  written, the transitions, the completed / created / cancelled instances and the next tick's pending jobs equal
  what the schedule predicts from per-event figures the oracle gives for one instance of each event kind.
"""
import numpy as np
import pytest

import bench_steady as S
from oracle import zbref
from test_gpu_long_running import _compare_tick
from zeebe_amd import bpmn, records as R

pytestmark = pytest.mark.gpu


def _inputs_to_oracle(o, pay, descs, vals):
    for p in pay:
        o.create("chain", p)
    for d in descs:
        o.submit(int(d["record_type"]), int(d["value_type"]), int(d["intent"]), int(d["key"]),
                 vals[int(d["value_offset"]):int(d["value_offset"]) + int(d["value_length"])])


def _inputs_to_engine(e, pay, descs, vals):
    offs = np.zeros(len(pay) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(p) for p in pay], dtype=np.uint64)
    e.create_packed("chain", b"".join(pay), offs)
    if len(descs):
        e.submit_packed(descs, vals)
    e.upload_staged()


def test_steady_schedule_vs_oracle():
    from zeebe_amd.engine import Engine

    live, ticks = 4000, 10
    # rows / arena / log sized well below what the run allocates: the engine compacts on the way
    e = Engine(log_capacity=1 << 17, row_capacity=16384, arena_bytes=(4 << 20), external_jobs=True)
    o = zbref.Oracle()
    o.set_harness(False)
    xml = bpmn.chain_workflow(S.TASKS).to_xml()
    e.deploy(xml, 100, 1)
    o.deploy(xml, 100, 1)
    w = S.JobWorld(live, cancels=live // 100)
    pay = [b"\x81\xa7orderId" + S._mp_int(i) for i in range(live)]
    _inputs_to_oracle(o, pay, [], b"")
    _inputs_to_engine(e, pay, [], b"")
    o.run()
    st = e.step()
    assert st["quiescent"], st
    _compare_tick(o, e, 0)
    w.harvest_oracle(o, 0)
    e.release(e.log_size())
    written = 0
    for t in range(ticks):
        start = e.log_size()
        assert start == o.log_size()
        pay, descs, vals, n_done, n_cancel, n_create = w.inputs()
        assert n_done > 0 and n_cancel > 0 and n_create > 0
        _inputs_to_oracle(o, pay, descs, vals)
        _inputs_to_engine(e, pay, descs, vals)
        o.run()
        st = e.step()
        assert st["quiescent"], st
        written += _compare_tick(o, e, start)
        w.harvest_oracle(o, start)
        e.release(e.log_size())
    m = e.memory_stats()
    assert m["compactions"] >= 1, m  # (the tick after a compaction was compared like the others)
    assert written > 10 * 16384 // 4, written
    e.close()
    o.close()


def _per_event_figures():
    """(records written, transitions, completed instances) the oracle writes for one event of each kind of the
    schedule, on a partition holding one waiting instance: a job completion at task k < TASKS and at the last task,
    a CREATE (to its first job), a CANCEL of an instance waiting on a job."""
    xml = bpmn.chain_workflow(S.TASKS).to_xml()

    def fresh():
        o = zbref.Oracle()
        o.set_harness(False)
        o.deploy(xml, 100, 1)
        return o

    def delta(o, f, n_in):  # (the log also holds the n_in submitted records; the engine's records_written does not)
        c0, n0 = o.counters(), o.log_size()
        f()
        o.run()
        c1 = o.counters()
        return (o.log_size() - n0 - n_in, c1["transitions"] - c0["transitions"], c1["completed"] - c0["completed"])

    out = {}
    o = fresh()
    out["create"] = delta(o, lambda: o.create("chain", b"\x81\xa7orderId\x01"), 1)
    w = S.JobWorld(1, cancels=0)
    w.harvest_oracle(o, 0)
    job = 0
    for k in range(1, S.TASKS + 1):  # walk the instance through every task
        wik, aik, task, v = w.pending.pop()
        assert task == k
        key = 2 + 5 * job
        job += 1
        cut = v.rfind(b"\xa7payload")
        doc = b"\x81" + bytes([0xa0 + len("t%d" % task)]) + b"t%d" % task + S._mp_int(task)
        n0 = o.log_size()
        d = delta(o, lambda: (o.submit(R.RT_EVENT, R.VT_JOB, R.JI_CREATED, key, v),
                              o.submit(R.RT_EVENT, R.VT_JOB, R.JI_COMPLETED, key,
                                       v[:cut] + b"\xa7payload\xc4" + bytes([len(doc)]) + doc)), 2)
        out.setdefault("done_last" if k == S.TASKS else "done", set()).add(d)
        w.harvest_oracle(o, n0)
    o2 = fresh()
    o2.create("chain", b"\x81\xa7orderId\x01")
    o2.run()
    w2 = S.JobWorld(1, cancels=0)
    w2.harvest_oracle(o2, 0)
    out["cancel"] = delta(o2, lambda: o2.submit(R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_CANCEL, w2.pending[0][0],
                                                b"\x80"), 1)
    assert len(out["done"]) == 1 and len(out["done_last"]) == 1, out  # the same figures at every task
    out["done"], out["done_last"] = out["done"].pop(), out["done_last"].pop()
    return out


def test_steady_schedule_properties_1m():
    from zeebe_amd.engine import Engine

    fig = _per_event_figures()
    live = 1_000_000
    recs_tick = live // S.FRACTION * 8 + (live // (S.FRACTION * S.TASKS)) * 12 + S.CANCELS * 10
    e = Engine(log_capacity=max(live * 12, 4 * recs_tick), row_capacity=4 * live + (1 << 20),
               arena_bytes=live * 1200 + (256 << 20), external_jobs=True)
    e.deploy(bpmn.chain_workflow(S.TASKS).to_xml(), 100, 1)
    w = S.JobWorld(live)
    pay = [b"\x81\xa7orderId" + S._mp_int(i) for i in range(live)]
    offs = np.zeros(live + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(p) for p in pay], dtype=np.uint64)
    e.create_packed("chain", b"".join(pay), offs)
    st = e.step()
    assert st["quiescent"] and st["records_written"] == live * fig["create"][0], st
    w.harvest(e, live, e.log_size() - live)
    assert len(w.pending) == live
    e.release(e.log_size())
    for t in range(4):
        pend = [p[2] for p in w.pending]
        pay, descs, vals, n_done, n_cancel, n_create = w.inputs()
        last = sum(1 for i, k in enumerate(pend) if (i + t) % S.FRACTION == 0 and k == S.TASKS)
        start = e.log_size()
        _inputs_to_engine(e, pay, descs, vals)
        c0 = e.counters()
        st = e.step()
        c1 = e.counters()
        assert st["quiescent"], st
        n_in = n_create + len(descs)
        exp = [n_create * fig["create"][i] + (n_done - last) * fig["done"][i] + last * fig["done_last"][i] +
               n_cancel * fig["cancel"][i] for i in range(3)]
        assert st["records_written"] == exp[0], (t, st["records_written"], exp)
        assert st["transitions"] == exp[1] and st["completed_instances"] == exp[2], (t, st, exp)
        assert c1["created"] - c0["created"] == n_create and c1["canceled"] - c0["canceled"] == n_cancel, (c0, c1)
        before = len(w.pending)
        w.harvest(e, start + n_in, e.log_size() - start - n_in)
        assert len(w.pending) - before == n_create + n_done - last, (t, len(w.pending), before)  # new JOB CREATEs
        assert len(set(p[0] for p in w.pending)) == len(w.pending)  # one pending job per waiting instance
        e.release(e.log_size())
    e.close()
