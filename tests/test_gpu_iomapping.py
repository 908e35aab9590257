"""Explicit io-mappings on the GPU (k_map + the wave pipeline) vs the oracle, bit for bit.

* every WorkflowTaskIOMappingTest case (tests/golden/reference_vectors.json "io_workflows", whose expected
  payloads / incident messages test_oracle_iomapping.py pins on the oracle): input mappings, output mappings,
  outputBehavior none / merge / overwrite, IO_MAPPING_ERROR incidents;
* a batch of instances through a sub process and tasks with input and output mappings, with payloads that
  make some mappings fail (incidents) and some succeed.
Records, log frames and the final element-instance state are compared with the oracle.
"""
import random

import msgpack
import pytest

from frames_check import assert_frames_equal
from oracle import zbref
from test_oracle_iomapping import check_io_outcome, io_workflow
from zeebe_amd import bpmn

pytestmark = pytest.mark.gpu


def _compare(o, e):
    ref, got = o.records(), e.records()
    assert len(got) == len(ref), (len(got), len(ref))
    for a, b in zip(ref, got):
        assert (a.position, a.key, a.record_type, a.value_type, a.intent) == \
               (b.position, b.key, b.record_type, b.value_type, b.intent), (a, b)
        assert a.value == b.value, (a.position, msgpack.unpackb(a.value, raw=False),
                                    msgpack.unpackb(b.value, raw=False))
    assert_frames_equal(o, e)
    oi, ei = o.instances(), e.instances()
    assert oi == ei
    return got


def test_io_workflow_vectors(vectors):
    from zeebe_amd.engine import Engine

    for v in vectors["io_workflows"]:
        xml = io_workflow(v).to_xml()
        o, e = zbref.Oracle(), Engine()
        for x in (o, e):
            x.deploy(xml, 100, 1)
            x.set_job_payload(100, "service", bytes.fromhex(v["complete"]))
        create = bytes.fromhex(v["create"]) if v["create"] else b""
        o.create("process", create)
        e.create("process", [create])
        o.run()
        st = e.step()
        assert st["quiescent"] and st["path"] == 0, v["name"]
        got = _compare(o, e)
        check_io_outcome(v, got)
        e.close()


def _mapped_model():
    sub = bpmn.Bpmn.create_executable_process("io").start_event("s").sub_process("sub")
    sub.zeebe_input("$.order", "$.o").zeebe_input("$.customer.id", "$.cid")
    sub.zeebe_output("$.o.total", "$.total").zeebe_output("$.res", "$.result.sub")
    sub.embedded_sub_process().start_event("ss").service_task(
        "t1", type="a", inputs=[("$.o.items[0]", "$.first"), ("$.cid", "$.c")],
        outputs=[("$.price", "$.o.total"), ("$.flag", "$.res")]).end_event("se").sub_process_done()
    b = sub.service_task("t2", type="b", outputs=[("$.x", "$.x")], output_behavior="overwrite")
    b = b.service_task("t3", type="c", output_behavior="none")
    return b.end_event("e").done()


def test_mapped_batch():
    from zeebe_amd.engine import Engine

    xml = _mapped_model().to_xml()
    rng = random.Random(5)
    payloads = []
    for i in range(600):
        doc = {"order": {"items": [rng.randrange(100) for _ in range(rng.randrange(0, 3))], "n": i},
               "customer": {"id": "c%d" % i}, "keep": i}
        if i % 7 == 0:
            del doc["customer"]  # input mapping of the sub process fails: no data for $.customer.id
        payloads.append(msgpack.packb(doc))
    o, e = zbref.Oracle(), Engine(log_capacity=1 << 18, row_capacity=1 << 16)
    for x in (o, e):
        x.deploy(xml, 100, 1)
        x.set_job_payload(100, "t1", msgpack.packb({"price": 12.5, "flag": True}))
        x.set_job_payload(100, "t2", msgpack.packb({"x": [1, 2], "y": 0}))
        x.set_job_payload(100, "t3", msgpack.packb({"z": 1}))
    for p in payloads:
        o.create("io", p)
    e.create("io", payloads)
    o.run()
    st = e.step()
    assert st["quiescent"] and st["path"] == 0
    got = _compare(o, e)
    incidents = [r for r in got if r.value_type == 6]
    assert incidents and len(incidents) < len(payloads)
    e.close()
