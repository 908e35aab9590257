"""Class batches (zb_traj.hip k_cls_*) vs the oracle, record for record.

A batch of CREATEs for one process whose exclusive splits read only the CREATE payload is split into
trajectory classes by the outcome of every split, and each class runs like a uniform batch. These
cases check the class path itself (stat path == 2) and each way out of it: more classes than CLS_MAX
and incidents go to the per-instance trajectory path (path == 1), a split that reads a merge result goes
to the wave pipeline (path == 0). Every case is compared with the oracle bit for bit.
"""
import random

import msgpack
import pytest

from frames_check import assert_frames_equal

from oracle import zbref
from zeebe_amd import bpmn, workloads

pytestmark = pytest.mark.gpu


def _run(xml, process, payloads, job_payloads=None, wave_only=False, **cap):
    from zeebe_amd.engine import Engine

    o = zbref.Oracle()
    o.deploy(xml, 100, 1)
    e = Engine(wave_only=wave_only, **cap)
    e.deploy(xml, 100, 1)
    for act, p in (job_payloads or {}).items():
        o.set_job_payload(100, act, p)
        e.set_job_payload(100, act, p)
    for p in payloads:
        o.create(process, p)
    e.create(process, payloads)
    o.run()
    st = e.step()
    assert st["quiescent"]
    ref, got = o.records(), e.records()
    assert len(got) == len(ref), (len(got), len(ref))
    for a, b in zip(ref, got):
        assert (a.position, a.key, a.record_type, a.value_type, a.intent) == \
               (b.position, b.key, b.record_type, b.value_type, b.intent), (a, b)
        assert a.value == b.value, (a.position, msgpack.unpackb(a.value, raw=False),
                                    msgpack.unpackb(b.value, raw=False))
    assert_frames_equal(o, e)
    oc, ec = o.counters(), e.counters()
    assert (ec["next_wf_key"], ec["next_job_key"], ec["completed"]) == \
           (oc["next_wf_key"], oc["next_job_key"], oc["completed"])
    e.close()
    return st


@pytest.mark.parametrize("n", [1, 5, 63, 64, 65, 3000])
def test_c3_classes(n):
    cfg = workloads.CONFIGS["c3"]
    blob, offs = cfg["payloads"](n)
    st = _run(cfg["workflow"]().to_xml(), cfg["process"], workloads.split(blob, offs))
    assert st["path"] == 2
    assert st["completed_instances"] == n


def _xor_tasks():
    # split first, then a service task on every branch: merges follow the split (class batch)
    b = bpmn.Bpmn.create_executable_process("xt").start_event("s").exclusive_gateway("x")
    b.sequence_flow_id("fa").condition("$.v < 10").service_task("ta", type="a").end_event("ea")
    b.move_to_node("x").sequence_flow_id("fb").condition("$.v >= 10 && $.w == true").service_task(
        "tb", type="b").service_task("tb2", type="b2").end_event("eb")
    return b.move_to_node("x").default_flow().sequence_flow_id("fc").end_event("ec").done()


def test_split_then_tasks():
    rng = random.Random(7)
    payloads = [msgpack.packb({"v": rng.randrange(20), "w": rng.random() < 0.5, "id": i}) for i in range(700)]
    jp = {"ta": msgpack.packb({"a": 1}), "tb": msgpack.packb({"b": "x" * 9}), "tb2": msgpack.packb({"v": -1})}
    st = _run(_xor_tasks().to_xml(), "xt", payloads, jp)
    assert st["path"] == 2
    st_w = _run(_xor_tasks().to_xml(), "xt", payloads, jp, wave_only=True)
    assert st_w["path"] == 0
    for k in ("transitions", "completed_instances", "merges", "merge_bytes", "condition_payload_bytes"):
        assert st[k] == st_w[k], k


def test_merge_before_split():
    # a task's merge result feeds the split: the class trace refuses it, the wave pipeline runs the batch
    b = bpmn.Bpmn.create_executable_process("ms").start_event("s").service_task("t", type="t").exclusive_gateway("x")
    b.sequence_flow_id("f1").condition("$.k > 3").end_event("e1")
    m = b.move_to_node("x").default_flow().sequence_flow_id("f2").end_event("e2").done()
    payloads = [msgpack.packb({"k": i % 7}) for i in range(200)]
    st = _run(m.to_xml(), "ms", payloads, {"t": msgpack.packb({"j": 1})})
    assert st["path"] == 0


def test_more_classes_than_cls_max():
    # four splits on four keys (radix 4 each -> 256 keys): random payloads give far more than 8 classes
    b = bpmn.Bpmn.create_executable_process("many").start_event("s")
    for k in range(4):
        g = b.exclusive_gateway("g%d" % k)
        g.sequence_flow_id("c%da" % k).condition("$.k%d < 3" % k).end_event("e%da" % k)
        g.move_to_node("g%d" % k).sequence_flow_id("c%db" % k).condition("$.k%d < 6" % k).end_event("e%db" % k)
        b = g.move_to_node("g%d" % k).default_flow().sequence_flow_id("d%d" % k)
    m = b.end_event("end").done()
    rng = random.Random(3)
    payloads = [msgpack.packb({"k%d" % k: rng.randrange(9) for k in range(4)}) for _ in range(1500)]
    st = _run(m.to_xml(), "many", payloads)
    assert st["path"] == 1


def test_few_of_many_keys():
    # the same model with payloads that only ever produce 3 distinct keys stays on the class path
    b = bpmn.Bpmn.create_executable_process("many").start_event("s")
    for k in range(4):
        g = b.exclusive_gateway("g%d" % k)
        g.sequence_flow_id("c%da" % k).condition("$.k%d < 3" % k).end_event("e%da" % k)
        g.move_to_node("g%d" % k).sequence_flow_id("c%db" % k).condition("$.k%d < 6" % k).end_event("e%db" % k)
        b = g.move_to_node("g%d" % k).default_flow().sequence_flow_id("d%d" % k)
    m = b.end_event("end").done()
    shapes = [{"k0": 1, "k1": 0, "k2": 0, "k3": 0}, {"k0": 8, "k1": 8, "k2": 4, "k3": 0},
              {"k0": 7, "k1": 7, "k2": 7, "k3": 7}]
    payloads = [msgpack.packb(shapes[(i * 7) % 3]) for i in range(999)]
    st = _run(m.to_xml(), "many", payloads)
    assert st["path"] == 2


def test_incident_class_falls_back():
    # no default flow: payloads where every condition is false raise an incident (per-instance path)
    b = bpmn.Bpmn.create_executable_process("inc").start_event("s").exclusive_gateway("x")
    b.sequence_flow_id("f1").condition("$.a == 1").end_event("e1")
    m = b.move_to_node("x").sequence_flow_id("f2").condition("$.a == 2").end_event("e2").done()
    payloads = [msgpack.packb({"a": i % 3}) for i in range(300)]
    st = _run(m.to_xml(), "inc", payloads)
    assert st["path"] == 1


@pytest.mark.parametrize("consts", [("", "a", "abcdefg"), ("abcdefgh", "abcdefghi", "abcdefghijklmno"),
                                    ("abcdefghijklmnop", "abcdefghijklmnopq", "abcdefghijklmnopqrst")])
def test_string_conditions_and_long_keys(consts):
    # k_cls_classify compares condition keys and string constants of at most 16 bytes as words (lds_words16) and
    # longer ones byte by byte: constants of 0 .. 20 bytes, a key of 18 bytes, values equal to the constant, one byte
    # shorter / longer, differing in the last byte or in case; three splits (8 classes: the class path runs)
    long_key = "a_key_of_18_bytes_"
    keys = ["s0", "s1", long_key]
    b = bpmn.Bpmn.create_executable_process("strs").start_event("s")
    for k, c in enumerate(consts):
        g = b.exclusive_gateway("g%d" % k)
        g.sequence_flow_id("m%d" % k).condition("$.%s == '%s'" % (keys[k], c)).end_event("e%d" % k)
        b = g.move_to_node("g%d" % k).default_flow().sequence_flow_id("d%d" % k)
    m = b.end_event("end").done()
    r = random.Random(len(consts[0]))

    def val(c):
        return r.choice([c, c, c[:-1] if c else "x", c + "z", (c[:-1] + "Z") if c else "", c.upper()])

    payloads = [msgpack.packb({keys[k]: val(consts[k]) for k in range(3)}) for _ in range(2000)]
    st = _run(m.to_xml(), "strs", payloads)
    assert st["path"] == 2


@pytest.mark.parametrize("io", [False, True])
def test_growing_class_batches_on_one_engine(io):
    """Class batches of growing and shrinking sizes on one engine: 10, 200, 256 (one trajectory workgroup), 300 and
    512 (two), 4100 (17 workgroups: two emit blocks of CLS_BLK_WG = 16), then 3000 (12, reusing the larger buffers).
    The class buffers allocated for an earlier batch serve every later one of at most their capacity (the slot
    arrays of the class-uniform emit -- ZB_CFG_NO_DEFER without ZB_CFG_INSTANCE_ORDER -- are sized for the
    workgroups' capacity and the block count, not for the batch that allocated them)."""
    from zeebe_amd.engine import CFG_INSTANCE_ORDER, CFG_NO_DEFER, Engine

    cfg = workloads.CONFIGS["c3"]
    xml = cfg["workflow"]().to_xml()
    o = zbref.Oracle()
    o.deploy(xml, 100, 1)
    e = Engine(flags=CFG_NO_DEFER | (CFG_INSTANCE_ORDER if io else 0))
    e.deploy(xml, 100, 1)
    for n in (10, 200, 256, 300, 512, 4100, 3000):
        blob, offs = cfg["payloads"](n)
        pays = workloads.split(blob, offs)
        for p in pays:
            o.create(cfg["process"], p)
        e.create(cfg["process"], pays)
        o.run()
        st = e.step()
        assert st["quiescent"] and st["path"] == 2
    ref, got = o.records(), e.records()
    assert len(got) == len(ref)
    for a, b in zip(ref, got):
        assert (a.position, a.key, a.intent, a.value) == (b.position, b.key, b.intent, b.value), a.position
    e.close()


def _short_circuit_model():
    b = bpmn.Bpmn.create_executable_process("sc").start_event("s").exclusive_gateway("g")
    b.sequence_flow_id("f1").condition("$.a < 5 && $.b == 'x'").end_event("e1")
    b.move_to_node("g").sequence_flow_id("f2").condition("$.a >= 5 || $.c > 1.5").end_event("e2")
    return b.move_to_node("g").default_flow().sequence_flow_id("f3").end_event("e3").done()


@pytest.mark.parametrize("errors", [False, True])
def test_outcome_table_short_circuit(errors):
    # k_cls_classify's outcome table (every comparison once, the class key looked up): short-circuit && / ||, and
    # comparisons whose operand is missing or of another type (an error only where the program reaches it: `$.b`
    # is never read when `$.a < 5` is false)
    rng = random.Random(3)
    payloads = []
    for i in range(900):
        d = {"a": rng.randrange(10), "b": rng.choice(["x", "y"]), "c": rng.choice([1.0, 2.0])}
        if errors:
            r = rng.random()
            if r < 0.1:
                del d["b"]
            elif r < 0.2:
                d["b"] = 7
            elif r < 0.3:
                del d["c"]
            elif r < 0.35:
                d["a"] = "s"
        payloads.append(msgpack.packb(d))
    st = _run(_short_circuit_model().to_xml(), "sc", payloads)
    if not errors:
        assert st["path"] == 2  # (with errors: incident classes send the batch to the per-instance path)
