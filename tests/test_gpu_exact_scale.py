"""The exact payload tree under contention at scale: >= 100k merges in one tick whose documents the structural merge
refuses, so that every wave of the tick, on every XCD, queues for the lane groups of zb_xlock.hpp (held without
agent-scope fences: a workspace is only ever written through its XCD's L2).

Every result byte is checked against the reference merge of the same pair (oracle zbref_merge:
MsgPackDocumentIndexer.java:136-283, MsgPackTree.java:141-166, MsgPackDocumentTreeWriter), and a strided sample of the
instances against the oracle engine record for record (values, keys, positions, frames).
  * canonical harness: one job completion payload with a duplicate key, 120k CREATE payloads of mixed odd shapes
    (duplicate keys, '[' / ']' keys, nested maps and arrays): on the trajectory path and on the wave pipeline;
  * external job processor: 120k JOB COMPLETED events of one tick, each with an odd payload of its own (the wave
    pipeline's k_merge_gen).
"""
import ctypes
import random

import msgpack
import numpy as np
import pytest

from oracle import zbref
from test_gpu_parity import _compare, _run_both
from test_xmerge_host import M, enc, odd_map
from zeebe_amd import bpmn, records as R

pytestmark = pytest.mark.gpu

N = 120_000
DUP_JOB = enc(M([("step", 1), ("a[b]", M([("x", 1)])), ("step", 2)]))  # source of every harness merge


def _model():
    return bpmn.Bpmn.create_executable_process("p").start_event("s").service_task("t", type="t").end_event("e").done()


class _Ref:
    """zbref_merge with one output buffer (the reference merge of a (source, target) pair)."""

    def __init__(self):
        self.out = ctypes.create_string_buffer(1 << 20)
        self.err = ctypes.create_string_buffer(1024)

    def __call__(self, src, tgt):
        n = zbref.lib().zbref_merge(src, len(src), tgt, len(tgt), self.out, 1 << 20, self.err, 1024)
        return None if n < 0 else self.out.raw[:n]


def _documents(n, seed, ref, partner=None):
    """n odd maps (target documents, or with `partner` the sources merged into partner[i]) that the reference merges
    without failing; every one holds a duplicate key or a bracket key, so the structural merge refuses it."""
    r = random.Random(seed)
    pool = [odd_map(r, 2) for _ in range(4096)]  # shapes, made distinct per document by the keys appended below
    docs, want = [], []
    for i in range(n):
        while True:
            m = M(pool[i % len(pool)] if r.random() < 0.9 else odd_map(r, 2))
            m.append(("k", i))
            m.append(("k[%d]" % (i % 7), M([("v", i)])) if i % 2 else ("k", -i))
            d = enc(m)
            src, tgt = (d, partner[i]) if partner is not None else (DUP_JOB, d)
            out = ref(src, tgt)
            # (the engine reserves |source| + |target| + 8 bytes per result -- DESIGN.md §4 Exact payload tree: only id
            # collisions that duplicate a subtree exceed it, and those fail the step with ZB_EUNSUPPORTED)
            if out is not None and len(out) + 4 <= len(src) + len(tgt) + 8:
                break
        docs.append(d)
        want.append(out)
    return docs, want


def _drain(e, start, count):
    from zeebe_amd.engine import HEADER_DTYPE

    ser = e.serialize(start, count)
    vals = np.empty(max(ser["value_bytes"], 1), dtype=np.uint8)
    hdrs = np.empty(count, dtype=HEADER_DTYPE)
    e.drain_copy(vals.ctypes.data, 0, ser["value_bytes"], hdrs.ctypes.data)
    return hdrs, vals.tobytes()


def _task_completions(e, start, count):
    """{workflow instance key: payload} of the task's ELEMENT_COMPLETED records in [start, start + count)."""
    h, v = _drain(e, start, count)
    sel = np.nonzero((h["value_type"] == R.VT_WORKFLOW_INSTANCE) & (h["record_type"] == R.RT_EVENT) &
                     (h["intent"] == R.WI_ELEMENT_COMPLETED))[0]
    out = {}
    for j in sel:
        o, n = int(h["value_offset"][j]), int(h["value_length"][j])
        rec = msgpack.unpackb(v[o:o + n], raw=False)
        if rec["activityId"] == "t":
            out[rec["workflowInstanceKey"]] = rec["payload"]
    return out


_HARNESS_DOCS = []


@pytest.mark.parametrize("path", ["traj", "wave"])
def test_exact_tree_harness_at_scale(path):
    from zeebe_amd.engine import Engine

    if not _HARNESS_DOCS:  # (both paths merge the same documents)
        _HARNESS_DOCS.append(_documents(N, 31, _Ref()))
    docs, want = _HARNESS_DOCS[0]
    e = Engine(wave_only=path == "wave", log_capacity=N * 20, row_capacity=N * 4, arena_bytes=N * 2048 + (64 << 20))
    e.deploy(_model().to_xml(), 100, 1)
    e.set_job_payload(100, "t", DUP_JOB)
    e.create("p", docs)
    st = e.step()
    assert st["quiescent"] and st["merges"] == N and st["completed_instances"] == N, st
    got = _task_completions(e, N, e.log_size() - N)
    e.close()
    assert len(got) == N
    bad = [i for i in range(N) if got.get(1 + 5 * i) != want[i]]  # instance i's key: its CREATE is processed i-th
    assert not bad, (len(bad), bad[:5])
    # record-for-record against the oracle engine on a strided sample of the shapes
    sample = [docs[i] for i in range(0, N, N // 97)]
    o, e2, _ = _run_both(_model().to_xml(), "p", sample, {"t": DUP_JOB}, path=path, log_capacity=1 << 16,
                         row_capacity=1 << 12, arena_bytes=64 << 20)
    _compare(o, e2)
    e2.close()


def test_exact_tree_external_completions_at_scale():
    from zeebe_amd.engine import Engine

    ref = _Ref()
    r = random.Random(7)
    creates = [enc(M([("orderId", i), ("tags", [i % 3, "x"]), ("a", M([("b", i % 5)]))])) for i in range(N)]
    pls, want = _documents(N, 43, ref, partner=creates)
    e = Engine(external_jobs=True, log_capacity=N * 24, row_capacity=N * 4, arena_bytes=N * 4096 + (64 << 20))
    e.deploy(_model().to_xml(), 100, 1)
    e.create("p", creates)
    assert e.step()["quiescent"]
    h, v = _drain(e, 0, e.log_size())
    jobs = np.nonzero((h["value_type"] == R.VT_JOB) & (h["intent"] == R.JI_CREATE) & (h["record_type"] == R.RT_COMMAND))[0]
    assert len(jobs) == N
    recs, inst = [], []
    order = list(range(N))
    r.shuffle(order)  # completions in an order of their own (the external job processor's)
    job_vals = []
    for j in jobs:
        o, n = int(h["value_offset"][j]), int(h["value_length"][j])
        job_vals.append(v[o:o + n])
    for k in order:
        val = job_vals[k]
        wik = msgpack.unpackb(val, raw=False)["headers"]["workflowInstanceKey"]
        i = (wik - 1) // 5
        key = 2 + 5 * k
        recs.append((R.RT_EVENT, R.VT_JOB, R.JI_CREATED, key, R.job_event(val)))
        recs.append((R.RT_EVENT, R.VT_JOB, R.JI_COMPLETED, key, R.job_event(val, pls[i])))
        inst.append(i)
    start = e.log_size()
    e.submit_records(recs)
    st = e.step()
    assert st["quiescent"] and st["merges"] == N and st["completed_instances"] == N, st
    got = _task_completions(e, start, e.log_size() - start)
    e.close()
    bad = [i for i in range(N) if got.get(1 + 5 * i) != want[i]]
    assert not bad, (len(bad), bad[:5])
    # the oracle engine on a strided sample: the same completions, record for record
    from test_gpu_races import Pair

    p = Pair({100: _model().to_xml()})
    sample = list(range(0, N, N // 61))
    p.tick([("p", [creates[i] for i in sample])])
    roots = p.roots()
    tick = []
    for s, wik in zip(sample, roots):
        j = p.job_of(wik)
        tick.append((R.RT_EVENT, R.VT_JOB, R.JI_CREATED, j[0], R.job_event(j[1])))
        tick.append((R.RT_EVENT, R.VT_JOB, R.JI_COMPLETED, j[0], R.job_event(j[1], pls[s])))
    assert p.tick(recs=tick) > 0
