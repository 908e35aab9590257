"""The drain's two write passes give the same bytes.

zb_serialize runs the fast pass (k_ser_fast: per-wave LDS image, the fast WORKFLOW_INSTANCE / JOB encoder)
over every 256-record tile and hands the tiles it cannot take (other record kinds, a wave's values over its
image) to the generic pass (k_ser_write). ZB_CFG_GENERIC_DRAIN sends every tile through the generic pass, whose
bytes every other GPU test compares with the oracle. Here the two drains of the same log must agree byte for
byte -- values and the 40-byte record headers -- on logs that mix the cases: C3 (all tiles fast), C2 with
job payloads large enough that tiles overflow the fast image, and the CREATE commands (generic records) at
the head of every log.
"""
import ctypes
import os

import msgpack
import pytest

from zeebe_amd import bpmn, workloads

pytestmark = pytest.mark.gpu


def _drain(make, fast, vlen_check=None, **engine_args):
    from zeebe_amd.engine import CFG_GENERIC_DRAIN, CFG_VLEN_CHECK, Engine, zb_record_header

    flags = (0 if fast else CFG_GENERIC_DRAIN) | (CFG_VLEN_CHECK if vlen_check else 0)
    e = Engine(flags=flags, **engine_args)
    make(e)
    st = e.step()
    assert st["quiescent"]
    n = e.log_size()
    ser = e.serialize(0, n)
    vals = ctypes.create_string_buffer(max(ser["value_bytes"], 1))
    hdrs = (zb_record_header * n)()
    e.drain_copy(ctypes.addressof(vals), 0, ser["value_bytes"], ctypes.addressof(hdrs))
    e.close()
    return ser, vals.raw[:ser["value_bytes"]], bytes(hdrs)


def _compare(make, expect_generic_all=False):
    sf, vf, hf = _drain(make, True)
    sg, vg, hg = _drain(make, False)
    tiles = (sf["records"] + 255) // 256
    assert sg["generic_tiles"] == tiles
    assert sf["value_bytes"] == sg["value_bytes"] and sf["payload_bytes"] == sg["payload_bytes"]
    assert vf == vg
    assert hf == hg
    if not expect_generic_all:
        assert sf["generic_tiles"] < tiles
    return sf


def test_c3_fast_drain_matches_generic():
    cfg = workloads.CONFIGS["c3"]
    blob, offs = cfg["payloads"](20000)

    def make(e):
        e.deploy(cfg["workflow"]().to_xml(), 100, 1)
        e.create_packed(cfg["process"], blob, offs)

    sf = _compare(make)
    assert sf["generic_tiles"] <= 79  # only the tiles holding the 20k CREATE commands (generic records)


def test_c2_large_job_payloads_fast_drain_matches_generic():
    # job payloads of 40..400 bytes: the merged instance payloads grow along the chain, so later tiles
    # outgrow the one-wave image and go to the generic pass; JOB records take the fast JOB encoder
    wf = bpmn.chain_workflow(6)
    blob, offs = workloads.order_payloads(3000)
    jp = {"t%d" % k: msgpack.packb({"k%d" % k: "x" * (40 * k * k // 3)}) for k in range(1, 7)}

    def make(e):
        e.deploy(wf.to_xml(), 100, 1)
        for act, p in jp.items():
            e.set_job_payload(100, act, p)
        e.create_packed("chain", blob, offs)

    _compare(make)


def test_mixed_kinds_fast_drain_matches_generic():
    # incidents (no default flow) interleave generic records with fast ones inside tiles
    b = bpmn.Bpmn.create_executable_process("inc").start_event("s").exclusive_gateway("x")
    b.sequence_flow_id("f1").condition("$.a == 1").end_event("e1")
    m = b.move_to_node("x").sequence_flow_id("f2").condition("$.a == 2").end_event("e2").done()
    payloads = [msgpack.packb({"a": i % 3, "pad": "p" * (i % 50)}) for i in range(3000)]

    def make(e):
        e.deploy(m.to_xml(), 100, 1)
        e.create("inc", payloads)

    _compare(make)


def test_message_kinds_fast_drain_matches_generic():
    """Message correlation on one partition (its outbox delivered to its own inbox): WORKFLOW_INSTANCE_SUBSCRIPTION,
    MESSAGE_SUBSCRIPTION and MESSAGE records (fast_encode_msg) interleaved with WORKFLOW_INSTANCE ones in every tile,
    published messages that correlate, that are stored and that expire."""
    from zeebe_amd import cluster

    xml = (bpmn.Bpmn.create_executable_process("wf").start_event()
           .intermediate_catch_event("catch-event", message="order canceled", correlation_key="$.orderId")
           .sequence_flow_id("to-end").end_event().done().to_xml())

    def make(e):
        e.deploy(xml, 100, 1)
        c = cluster.LocalCluster([e])
        e.create("wf", [msgpack.packb({"orderId": "order-%d" % i, "pad": "p" * (i % 40)}) for i in range(3000)])
        c.settle()
        c.publish(b"order canceled", [b"order-%d" % i for i in range(0, 3000, 2)],
                  [msgpack.packb({"n": i, "s": "x" * (i % 70)}) for i in range(0, 3000, 2)])
        c.publish(b"order canceled", [b"nobody-%d" % i for i in range(200)], [b"\x80"] * 200)
        c.publish(b"order canceled", [b"late-%d" % i for i in range(100)], [b"\x80"] * 100, ttl=0)

    sf = _compare(make)
    assert sf["generic_tiles"] * 4 < (sf["records"] + 255) // 256  # (tiles with submitted commands stay generic)


def test_size_pass_formula_matches_encoder():
    # records without a length from their emitting kernel (the wave pipeline writes none) are sized by the
    # size pass: WORKFLOW_INSTANCE / JOB records by the emit kernels' formula, unless ZB_CFG_VLEN_CHECK, which
    # runs the encoder's dry run on every record. Both must give the same drain, byte for byte.
    wf = bpmn.chain_workflow(4)
    blob, offs = workloads.order_payloads(2000)
    jp = {"t%d" % k: msgpack.packb({"k%d" % k: "y" * (7 * k)}) for k in range(1, 5)}

    def make(e):
        e.deploy(wf.to_xml(), 100, 1)
        for act, p in jp.items():
            e.set_job_payload(100, act, p)
        e.create_packed("chain", blob, offs)

    a = _drain(make, True, vlen_check=False, wave_only=True)
    b = _drain(make, True, vlen_check=True, wave_only=True)
    assert a[0]["value_bytes"] == b[0]["value_bytes"]
    assert a[1] == b[1] and a[2] == b[2]


# ---- the template drain (zb_tdrain.hip): a uniform / class batch left without descriptors by zb_step, encoded
# straight from its traces by zb_serialize of exactly its records; vs the descriptor path (ZB_CFG_NO_DEFER)
def _template_drain(make, defer):
    from zeebe_amd.engine import CFG_NO_DEFER, Engine, zb_record_header

    e = Engine(log_capacity=1 << 22, row_capacity=1 << 16, arena_bytes=64 << 20, flags=0 if defer else CFG_NO_DEFER)
    n = make(e)
    st = e.step()
    assert st["quiescent"] and st["path"] in (1, 2), st
    L = e.log_size()
    ser = e.serialize(n, L - n)
    vals = ctypes.create_string_buffer(max(ser["value_bytes"], 1))
    hdrs = (zb_record_header * (L - n))()
    e.drain_copy(ctypes.addressof(vals), 0, ser["value_bytes"], ctypes.addressof(hdrs))
    out = dict(ser=ser, values=vals.raw[:ser["value_bytes"]], headers=bytes(hdrs))
    # then the descriptors (materialized on demand) and the records API
    out["desc"] = bytes(e.descriptors(0, L))
    out["records"] = e.records(n)
    out["counters"] = e.counters()
    e.close()
    return out


def _simple_workflow():
    return bpmn.Bpmn.create_executable_process("simple").start_event().end_event().done().to_xml()


@pytest.mark.parametrize("shape", ["c3", "c3_100k", "uniform"])
def test_template_drain_matches_descriptor_drain(shape):
    """c3_200k: past the first 65536 instances (keys / positions >= 2^16) the size pass takes the class formula
    (k_tdrain_sizes) instead of resolving every record (k_tdrain_size): both parts in one batch."""
    if shape.startswith("c3"):
        cfg = workloads.CONFIGS["c3"]
        n_inst = 100000 if shape == "c3_100k" else 30000
        blob, offs = workloads.xor_payloads_np(n_inst)

        def make(e):
            e.deploy(cfg["workflow"]().to_xml(), 100, 1)
            e.create_packed(cfg["process"], blob, offs)
            return n_inst
    else:
        blob, offs = workloads.order_payloads(7000)

        def make(e):
            e.deploy(_simple_workflow(), 100, 1)
            e.create_packed("simple", blob, offs)
            return 7000

    a = _template_drain(make, True)
    b = _template_drain(make, False)
    assert a["ser"]["template_drain"] == 1 and b["ser"]["template_drain"] == 0
    assert a["ser"]["value_bytes"] == b["ser"]["value_bytes"] and a["ser"]["payload_bytes"] == b["ser"]["payload_bytes"]
    assert a["values"] == b["values"]
    assert a["headers"] == b["headers"]
    assert a["desc"] == b["desc"]
    assert a["records"] == b["records"]
    assert a["counters"] == b["counters"]


def test_template_drain_not_taken_for_merges_or_partial_ranges():
    """C1's canonical harness merges job payloads: the batch is not deferred. A deferred batch serialized from
    another start, or as frames, is materialized first and drained from its descriptors."""
    cfg = workloads.CONFIGS["c1"]
    from zeebe_amd.engine import Engine

    e = Engine(log_capacity=1 << 20, row_capacity=1 << 14, arena_bytes=32 << 20)
    e.deploy(cfg["workflow"]().to_xml(), 100, 1)
    blob, offs = workloads.order_payloads(2000)
    e.create_packed(cfg["process"], blob, offs)
    assert e.step()["quiescent"]
    assert e.serialize(2000, e.log_size() - 2000)["template_drain"] == 0
    e.close()
    c3 = workloads.CONFIGS["c3"]
    blob, offs = c3["payloads"](5000)
    e = Engine(log_capacity=1 << 20, row_capacity=1 << 14, arena_bytes=32 << 20)
    e.deploy(c3["workflow"]().to_xml(), 100, 1)
    e.create_packed(c3["process"], blob, offs)
    assert e.step()["quiescent"]
    L = e.log_size()
    whole = e.records(0)  # from 0: includes the CREATE commands -> materialized, descriptor drain
    assert e.serialize(5000, L - 5000)["template_drain"] == 0  # (no longer deferred)
    assert [r.position for r in whole] == list(range(L))
    e.close()
