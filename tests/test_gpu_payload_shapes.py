"""Payload shapes the kernels' structural merge and node-table mapper refuse, on the GPU, vs the oracle bit for bit.

The reference merges and maps any document (MsgPackDocumentIndexer.java:136-283, MsgPackTree.java:84-166): duplicate
keys (the last value, at the first key's position), keys holding '[' / ']' (its string node ids "$[a][b]" collide
with other paths, and the collisions show in the output), non-string keys below the root (the processor fails),
any depth, any number of nodes. merge_docs / merge_flat / map_documents cover the usual shapes; everything else goes
to the exact tree (zeebe_amd/csrc/zb_xmerge.hpp, a workspace slab per lane through zb_xlock.hpp) from k_merge_gen,
k_map and the trajectory path's merge. Cases:
  * the default output merge on both pipelines (canonical job harness: job payload into the CREATE payload);
  * 300 job completions with odd payloads in one tick (external job processor): hundreds of lanes of one wave
    queue for the 32 slabs;
  * explicit output / input mappings over documents with bracket keys and more than 256 nodes.
Host-side fuzzing of the same source against the oracle: tests/test_xmerge_host.py.
"""
import random

import msgpack
import pytest

from test_gpu_parity import _compare, _run_both
from test_gpu_races import Pair, _completed, _created
from test_xmerge_host import M, deep, enc, odd_map, oracle_merge
from oracle import zbref
from zeebe_amd import bpmn, workloads

pytestmark = pytest.mark.gpu


def _task_model():
    return bpmn.Bpmn.create_executable_process("p").start_event("s").service_task("t", type="t").end_event("e").done()


CASES = [
    (M([("a", 1), ("a", 2), ("b", M([("c", 1), ("c", [1, 2])]))]), M([("b", M([("c", 9)])), ("z", 1), ("z", 2)])),
    (M([("a", M([("b", 2)])), ("q", 1)]), M([("a[b]", 1)])),                    # distinct ids "$[a][b]", "$[a[b]]"
    (M([("a][b", 0)]), M([("a", M([("b", "shared")]))])),                       # one id for two paths: "$[a][b]"
    (M([("x", M([("0", "m"), ("2", 7)]))]), M([("x", [1, 2, M([("0", 5)])])])),  # index / key "0"
    (deep(40), deep(37, "leaf")),                                               # deeper than 16
    (M([("n%d" % i, i) for i in range(0, 300, 3)]), M([("n%d" % i, M([("v", i)])) for i in range(300)])),
]


@pytest.mark.parametrize("path", ["traj", "wave"])
def test_default_merge_odd_shapes(path):
    xml = _task_model().to_xml()
    r = random.Random(17)
    cases = CASES + [(odd_map(r, 3), odd_map(r, 3)) for _ in range(6)]
    for tgt, src in cases:
        o, e, st = _run_both(xml, "p", [enc(tgt)] * 3, {"t": enc(src)}, path=path,
                             log_capacity=1 << 14, row_capacity=1 << 10, arena_bytes=16 << 20)
        _compare(o, e)
        e.close()


def test_default_merge_odd_shapes_fails_like_the_reference():
    """A non-string key below the root: the reference's indexer throws, the processor fails -- so does the engine
    (and the oracle), instead of writing anything made up."""
    from zeebe_amd.engine import ZbError

    xml = _task_model().to_xml()
    o = zbref.Oracle()
    o.deploy(xml, 100, 1)
    o.set_job_payload(100, "t", enc(M([("a", M([(1, 2)]))])))
    o.create("p", enc(M([("a", 1)])))
    with pytest.raises(Exception):
        o.run()
    for path in ("traj", "wave"):
        from zeebe_amd.engine import Engine

        e = Engine(wave_only=path == "wave", log_capacity=1 << 12, row_capacity=1 << 10, arena_bytes=8 << 20)
        e.deploy(xml, 100, 1)
        e.set_job_payload(100, "t", enc(M([("a", M([(1, 2)]))])))
        e.create("p", [enc(M([("a", 1)]))])
        with pytest.raises(ZbError):
            e.step()
        e.close()


def test_many_exact_merges_in_one_wave():
    c1 = workloads.CONFIGS["c1"]
    p = Pair({100: c1["workflow"]().to_xml()})
    r = random.Random(23)
    creates = [enc(M([("orderId", i), ("k", i), ("k", -i), ("x[%d]" % (i % 3), M([("y", i)]))])) for i in range(300)]
    p.tick([("process", creates)])
    roots = p.roots()
    recs = []
    for i, wik in enumerate(roots):
        j = p.job_of(wik)
        recs.append(_created(j))
        pl = enc(M([("k", "late"), ("x", M([(str(i % 3), "collide")])), ("k", 1)]))
        if i % 2:  # a random odd document, as long as the reference merges it (some make its writer throw)
            while True:
                pl = enc(odd_map(r, 3))
                if not isinstance(oracle_merge(pl, creates[i]), str):
                    break
        recs.append(_completed(j, pl))
    n = p.tick(recs=recs)
    assert n > 600


def _mapped(outputs, inputs=()):
    return (bpmn.Bpmn.create_executable_process("m").start_event("s")
            .service_task("t", type="t", inputs=list(inputs), outputs=list(outputs)).end_event("e").done())


def test_mappings_over_odd_documents():
    """Explicit mappings where map_documents stops: bracket keys in the documents, more than 256 nodes."""
    from zeebe_amd.engine import Engine

    big = M([("k%d" % i, M([("v", i), ("w", [i, i + 1])])) for i in range(120)])  # > 256 nodes
    models = [
        _mapped([("$.res", "$.out")]),
        _mapped([("$.res", "$.k3.v"), ("$.res2", "$.n")], inputs=[("$.k1", "$.k1"), ("$.a[b]", "$.ab")]),
        _mapped([("$", "$.all")]),
    ]
    creates = [
        M(list(big) + [("a[b]", 1), ("a", M([("b", 2)]))]),
        M([("a[b]", M([("c", 1)])), ("a", M([("b", M([("c", 2)]))])), ("k1", 1)]),
        M([("k1", 1), ("k1", 2), ("z]", [1, 2])]),
    ]
    jobs = [
        M([("res", deep(33)), ("res2", M([("q[1]", 1)]))]),
        M([("res", 1), ("res2", big)]),
    ]
    from zeebe_amd.engine import ZbError

    outcomes = {"ok": 0, "fail": 0}
    for model in models:
        xml = model.to_xml()
        for job in jobs:
            for c in creates:
                o, e = zbref.Oracle(), Engine(log_capacity=1 << 14, row_capacity=1 << 10, arena_bytes=16 << 20)
                for x in (o, e):
                    x.deploy(xml, 100, 1)
                    x.set_job_payload(100, "t", enc(job))
                o.create("m", enc(c))
                e.create("m", [enc(c)])
                try:
                    o.run()
                except zbref.ZbrefError:  # e.g. a duplicate key matched twice by a source query: the processor fails
                    with pytest.raises(ZbError):
                        e.step()
                    outcomes["fail"] += 1
                else:
                    st = e.step()
                    assert st["quiescent"]
                    _compare(o, e)
                    assert o.instances() == e.instances()
                    outcomes["ok"] += 1
                e.close()
    assert outcomes["ok"] >= 12 and outcomes["fail"] >= 1, outcomes
