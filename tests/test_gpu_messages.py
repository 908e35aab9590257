"""Message correlation on the GPU (config 5 shape): GPU partitions vs oracle partitions, record for record.

Both clusters run the same canonical schedule (zeebe_amd.cluster.LocalCluster): several GPU engines
share cuda:0 here (one per partition); the oracle partitions are the checker. Every record of every
partition's log is compared: position, key, record / value type, intent, rejection type and the full
msgpack value bytes.
"""
import msgpack
import pytest

from frames_check import assert_frames_equal
from oracle import zbref
from zeebe_amd import bpmn, cluster

pytestmark = pytest.mark.gpu


def catch_workflow():
    # IntermediateMessageCatchEventTest.java:59-66
    return (bpmn.Bpmn.create_executable_process("wf").start_event()
            .intermediate_catch_event("catch-event", message="order canceled", correlation_key="$.orderId")
            .sequence_flow_id("to-end").end_event().done().to_xml())


def clusters(P, xml, n_log=1 << 20):
    from zeebe_amd.engine import Engine

    gpu = [Engine(device=0, partition_id=p, partition_count=P, log_capacity=n_log, row_capacity=1 << 18,
                  arena_bytes=256 << 20) for p in range(P)]
    ref = [zbref.OraclePartition(p, P) for p in range(P)]
    for x in gpu + ref:
        x.deploy(xml, 100, 1)
    return gpu, ref, cluster.LocalCluster(gpu), cluster.LocalCluster(ref)


def compare(gpu, ref):
    for p, (g, o) in enumerate(zip(gpu, ref)):
        a, b = o.records(), g.records()
        assert len(a) == len(b), (p, len(a), len(b))
        for x, y in zip(a, b):
            assert (x.position, x.key, x.record_type, x.value_type, x.intent) == \
                   (y.position, y.key, y.record_type, y.value_type, y.intent), (p, x, y)
            if x.record_type == 2:
                assert x.rejection_type == y.rejection_type, (p, x, y)
            assert x.value == y.value, (p, x.position, msgpack.unpackb(x.value, raw=False),
                                        msgpack.unpackb(y.value, raw=False))
        assert_frames_equal(o, g)


def both(fn, gpu, ref):
    fn(gpu)
    fn(ref)


@pytest.mark.parametrize("P", [1, 3])
def test_correlation_round_trip(P):
    gpu, ref, cg, co = clusters(P, catch_workflow())
    n = 60
    for i in range(n):
        gpu[i % P].create("wf", [msgpack.packb({"orderId": "order-%d" % i})])
        ref[i % P].create("wf", msgpack.packb({"orderId": "order-%d" % i}))
    cg.settle()
    co.settle()
    compare(gpu, ref)
    cks = [b"order-%d" % i for i in range(n)]
    pls = [msgpack.packb({"foo": i}) for i in range(n)]
    cg.publish(b"order canceled", cks, pls)
    co.publish(b"order canceled", cks, pls)
    compare(gpu, ref)
    assert sum(g.counters()["completed"] for g in gpu) == n


def test_published_first_ttl_duplicates_and_rejections():
    P = 3
    gpu, ref, cg, co = clusters(P, catch_workflow())
    for c in (cg, co):
        # shouldNotCorrelateMessageAfterTTL :264-279 shape, then a stored message for order-1
        c.publish(b"order canceled", [b"order-0"], [msgpack.packb({"nr": "first"})], ttl=0)
        c.publish(b"order canceled", [b"order-0", b"order-1"],
                  [msgpack.packb({"nr": "second"}), msgpack.packb({"nr": "x"})], ttl=10000)
    for i, key in enumerate(["order-0", "order-1", "order-2", "order-2", "order-3"]):
        gpu[i % P].create("wf", [msgpack.packb({"orderId": key})])
        ref[i % P].create("wf", msgpack.packb({"orderId": key}))
    cg.settle()
    co.settle()
    compare(gpu, ref)
    # correlate to all subscriptions of order-2; order-2 again -> CORRELATE rejections (activity gone)
    for c in (cg, co):
        c.publish(b"order canceled", [b"order-2", b"order-3"], [b"\x80", msgpack.packb({"a": [1, 2]})])
        c.publish(b"order canceled", [b"order-2"], [msgpack.packb({"again": True})], ttl=0)
    compare(gpu, ref)
    recs = [r for p in ref for r in p.records() if r.value_type == 12 and r.record_type == 2]
    assert recs, "expected CORRELATE rejections"


@pytest.mark.parametrize("P", [1, 3])
def test_one_message_many_subscriptions(P):
    """One PUBLISH matching many open subscriptions: its CORRELATE commands leave in findSubscriptions' insertion
    order (the outbox orders them by their rank among the message's matches, up to 32, and by the store index
    beyond), interleaved with other messages' correlations."""
    gpu, ref, cg, co = clusters(P, catch_workflow())
    keys = ["shared"] * 45 + ["five"] * 5 + ["order-%d" % i for i in range(10)]
    for i, key in enumerate(keys):
        gpu[i % P].create("wf", [msgpack.packb({"orderId": key})])
        ref[i % P].create("wf", msgpack.packb({"orderId": key}))
    cg.settle()
    co.settle()
    compare(gpu, ref)
    cks = [b"order-3", b"shared", b"five", b"order-7"]
    pls = [msgpack.packb({"m": i}) for i in range(len(cks))]
    cg.publish(b"order canceled", cks, pls)
    co.publish(b"order canceled", cks, pls)
    compare(gpu, ref)
    assert sum(g.counters()["completed"] for g in gpu) == 45 + 5 + 2


def test_outbox_single_target_counting_sort():
    """Every command of an outbox for one target partition: the keys' spread then leaves out the target bits and the
    take sorts by counting (k_cs_hist / k_cs_scatter) on the outbox path (zb_outbox_take, P > 1) -- the OPEN commands of
    each workflow partition, and the CORRELATE commands of one message partition to one workflow partition, many of them
    one message's matches (emission indexes 0..44 at one source position)."""
    P = 3
    cks = [k for k in ("key-%d" % i for i in range(400)) if cluster.subscription_partition(k.encode(), P) == 0]
    shared, single = cks[0], cks[1:21]
    keys = [shared] * 45 + single
    gpu, ref, cg, co = clusters(P, catch_workflow())
    for i, key in enumerate(keys):  # every instance on partition 1, every subscription on partition 0
        gpu[1].create("wf", [msgpack.packb({"orderId": key})])
        ref[1].create("wf", msgpack.packb({"orderId": key}))
    cg.settle()
    co.settle()
    compare(gpu, ref)
    # one message first (its 45 correlations share a source position: the keys differ in the emission bits only),
    # then several (positions and emission 0)
    for c in (cg, co):
        c.publish(b"order canceled", [shared.encode()], [msgpack.packb({"m": 0})])
    compare(gpu, ref)
    pub = [k.encode() for k in single[::2]]
    pls = [msgpack.packb({"m": i + 1}) for i in range(len(pub))]
    cg.publish(b"order canceled", pub, pls)
    co.publish(b"order canceled", pub, pls)
    compare(gpu, ref)
    assert sum(g.counters()["completed"] for g in gpu) == 45 + len(pub)


def test_correlate_with_stale_and_foreign_tokens():
    """A delivered CORRELATE takes the row its token names only when that row is live and holds its activity instance
    key; a foreign token (NO_TOKEN) or another instance's row is counted and resolved by the sorted key search
    (k_resolve) -- the records must be those of the oracle, which resolves every command by key."""
    import numpy as np

    from zeebe_amd.engine import Engine

    n = 90
    e = Engine(device=0, partition_id=0, partition_count=1, log_capacity=1 << 16, row_capacity=1 << 12)
    o = zbref.OraclePartition(0, 1)
    co = cluster.LocalCluster([o])
    for x in (e, o):
        x.deploy(catch_workflow(), 100, 1)
    for i in range(n):
        e.create("wf", [msgpack.packb({"orderId": "order-%d" % i})])
        o.create("wf", msgpack.packb({"orderId": "order-%d" % i}))
    e.run()
    buf, _ = e.outbox(cluster.KIND_OPEN)
    e.inbox(cluster.KIND_OPEN, buf)
    e.run()
    co.settle()
    cks = [b"order-%d" % i for i in range(n)]
    pls = [msgpack.packb({"paid": i}) for i in range(n)]
    e.publish(b"order canceled", cks, pls)
    co.publish(b"order canceled", cks, pls)
    buf, _ = e.outbox(cluster.KIND_CORRELATE)
    b = bytearray(np.asarray(buf, dtype=np.uint8).tobytes())
    cnt = int.from_bytes(b[0:8], "little")
    assert cnt == n
    toks = [int.from_bytes(b[16 + 64 * j + 12:16 + 64 * j + 16], "little") for j in range(cnt)]
    for j in range(cnt):
        t = 0xFFFFFFFF if j % 3 == 0 else toks[(j + 1) % cnt] if j % 3 == 1 else toks[j]
        b[16 + 64 * j + 12:16 + 64 * j + 16] = t.to_bytes(4, "little")
    e.inbox(cluster.KIND_CORRELATE, b)
    e.run()
    compare([e], [o])
    assert e.counters()["completed"] == n
    e.close()


def test_integer_correlation_key():
    # extractCorrelationKey: a long becomes its 8 little-endian bytes (hash routing and store key)
    P = 3
    xml = (bpmn.Bpmn.create_executable_process("wf").start_event()
           .intermediate_catch_event("catch-event", message="paid", correlation_key="$.id")
           .end_event().done().to_xml())
    gpu, ref, cg, co = clusters(P, xml)
    for i in range(12):
        gpu[i % P].create("wf", [msgpack.packb({"id": 1000 + i})])
        ref[i % P].create("wf", msgpack.packb({"id": 1000 + i}))
    cg.settle()
    co.settle()
    compare(gpu, ref)
    cks = [int(1000 + i).to_bytes(8, "little", signed=True) for i in range(12)]
    for c in (cg, co):
        c.publish(b"paid", cks, [msgpack.packb({"ok": i}) for i in range(12)])
    compare(gpu, ref)
    assert sum(g.counters()["completed"] for g in gpu) == 12


def test_c5_scale_properties():
    """4 partitions on one GPU, 200k instances: every instance completes, every log has the C5 shape."""
    from zeebe_amd.engine import Engine

    P, n = 4, 200_000
    xml = bpmn.message_workflow().to_xml()
    gpu = [Engine(device=0, partition_id=p, partition_count=P, log_capacity=n * 8, row_capacity=n,
                  arena_bytes=(n // P) * 1024 + (64 << 20)) for p in range(P)]
    for g in gpu:
        g.deploy(xml, 100, 1)
    for p in range(P):
        payloads = [msgpack.packb({"orderId": "order-%d" % i}) for i in range(p, n, P)]
        gpu[p].create("msg", payloads)
    c = cluster.LocalCluster(gpu)
    c.settle()
    assert sum(g.pending(1) + g.pending(2) for g in gpu) == 0
    cks = [b"order-%d" % i for i in range(n)]
    c.publish(b"order", cks, [msgpack.packb({"paid": True})] * n)
    assert sum(g.counters()["completed"] for g in gpu) == n
    # per instance: CREATE + 13 WORKFLOW_INSTANCE events + WIS CORRELATE / CORRELATED;
    # per message PUBLISH + PUBLISHED; per subscription OPEN + OPENED
    total = sum(g.log_size() for g in gpu)
    assert total == n * (1 + 13 + 2) + n * 2 + n * 2, total


@pytest.mark.parametrize("rccl_self", [True, False])
def test_rccl_exchange_single_rank(rccl_self):
    """DistCluster with the engine's own RCCL communicator (world size 1 here: the one-GPU box) against the oracle:
    with ZB_CFG_RCCL_SELF the exchange goes through the agreement collectives and ncclSend / ncclRecv to self (the
    P > 1 code path), without it the one partition delivers its outbox to its own inbox on the device."""
    import os
    import socket

    import torch.distributed as dist
    from zeebe_amd.engine import CFG_RCCL_SELF, Engine

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        e = Engine(device=0, partition_id=0, partition_count=1, log_capacity=1 << 20, row_capacity=1 << 18,
                   flags=CFG_RCCL_SELF if rccl_self else 0)
        o = zbref.OraclePartition(0, 1)
        for x in (e, o):
            x.deploy(catch_workflow(), 100, 1)
        n = 50
        e.create("wf", [msgpack.packb({"orderId": "order-%d" % i}) for i in range(n)])
        for i in range(n):
            o.create("wf", msgpack.packb({"orderId": "order-%d" % i}))
        dc = cluster.DistCluster(e)
        assert dc.rccl
        co = cluster.LocalCluster([o])
        dc.settle()
        co.settle()
        cks = [b"order-%d" % i for i in range(n)]
        pls = [msgpack.packb({"n": i}) for i in range(n)]
        dc.publish(b"order canceled", cks, pls)
        co.publish(b"order canceled", cks, pls)
        compare([e], [o])
        assert e.counters()["completed"] == n
    finally:
        dist.destroy_process_group()


# ------------------------------------------------------------------------------ the whole message partition
def _msg_value(name, ck, ttl, payload=b"\x80", message_id=b""):
    """MessageRecord (MessageRecord.java:26-42) as the client API writes it."""
    return msgpack.packb({"name": name, "correlationKey": ck, "timeToLive": ttl, "payload": payload,
                          "messageId": message_id})


def _submit_messages(gpu, ref, msgs, P):
    """MESSAGE commands (intent, key, name, ck, ttl, payload, id) routed to abs(hash(ck) % P) as a client would."""
    by = [[] for _ in range(P)]
    for intent, key, name, ck, ttl, payload, mid in msgs:
        q = cluster.subscription_partition(ck.encode(), P)
        by[q].append((intent, key, _msg_value(name, ck, ttl, payload, mid)))
    for q in range(P):
        if by[q]:
            gpu[q].submit_messages(by[q])
            for intent, key, value in by[q]:
                ref[q].submit(1, 10, intent, key, value)


def test_message_ids_delete_ttl_and_large_fields():
    """PublishMessageProcessor's messageId rejection (against the store and inside one batch), DELETE commands,
    the time-to-live checker removing stored messages at a clock, per-command names and TTLs, 4 KB payloads and
    200-byte correlation keys / message names through the variable-length exchange, at P = 1 and P = 3."""
    for P in (1, 3):
        name = "m" * 150
        xml = (bpmn.Bpmn.create_executable_process("wf").start_event()
               .intermediate_catch_event("catch", message=name, correlation_key="$.k").end_event().done().to_xml())
        gpu, ref, cg, co = clusters(P, xml)
        for x in gpu + ref:
            x.set_clock(1000)
        big = msgpack.packb({"blob": "z" * 4000, "n": 1})
        cks = ["c%03d-" % i + "x" * 195 for i in range(12)]
        # t=1000: stored messages (ttl 500 / 5000), a duplicate id in the batch, an empty id (never a duplicate),
        # ttl 0 (deleted at once), another name
        msgs = [(0, -1, name, cks[0], 500, big, "id-0"), (0, -1, name, cks[0], 500, big, "id-0"),
                (0, -1, name, cks[1], 5000, msgpack.packb({"v": 1}), "id-1"), (0, -1, name, cks[2], 0, big, ""),
                (0, -1, name, cks[2], 0, big, ""), (0, -1, "other", cks[3], 700, big, "id-0"),
                (0, -1, name, cks[4], 5000, msgpack.packb({"v": 4}), "")]
        _submit_messages(gpu, ref, msgs, P)
        co.settle()
        cg.settle()
        compare(gpu, ref)
        # the same ids again (rejected: already stored) and a DELETE of a stored message (key from the log)
        stored = [r for p in ref for r in p.records() if r.value_type == 10 and r.intent == 1]
        victim = [r for r in stored if msgpack.unpackb(r.value, raw=False)["correlationKey"] == cks[4]][0]
        msgs = [(0, -1, name, cks[0], 500, big, "id-0"), (0, -1, name, cks[1], 10, big, "id-1"),
                (2, victim.key, name, cks[4], 5000, msgpack.packb({"v": 4}), "")]
        _submit_messages(gpu, ref, msgs, P)
        co.settle()
        cg.settle()
        compare(gpu, ref)
        # instances subscribe: cks[1] correlates with its stored message; cks[4]'s was deleted; cks[5] waits
        for i, ck in enumerate([cks[1], cks[4], cks[5], cks[0]]):
            gpu[i % P].create("wf", [msgpack.packb({"k": ck})])
            ref[i % P].create("wf", msgpack.packb({"k": ck}))
        cg.settle()
        co.settle()
        compare(gpu, ref)
        # the time-to-live checker at t=1600: id-0 (deadline 1500) and "other" (1700? no: 1700 > 1600) expire
        for q in range(P):
            n_g = gpu[q].expire_messages(1600)
            n_o = ref[q].check_ttl(1600)
            assert n_g == n_o
        co.settle()
        cg.settle()
        compare(gpu, ref)
        # a message for the waiting instance, published after the clock moved on
        for x in gpu + ref:
            x.set_clock(9000)
        _submit_messages(gpu, ref, [(0, -1, name, cks[5], 100, big, "late")], P)
        co.settle()
        cg.settle()
        compare(gpu, ref)
        for q in range(P):
            assert gpu[q].expire_messages(20000) == ref[q].check_ttl(20000)
        co.settle()
        cg.settle()
        compare(gpu, ref)
        assert sum(g.counters()["completed"] for g in gpu) == sum(o.counters()["completed"] for o in ref) >= 3
        rej = [r for p in ref for r in p.records() if r.value_type == 10 and r.record_type == 2]
        assert len(rej) >= 3
        for g in gpu:
            g.close()


def _xbatch(recs, var=b""):
    """One exchange batch (include/zb_engine.h): [count][total bytes][count x 64-byte zb_exchange_rec][byte section]."""
    import struct

    body = b"".join(struct.pack("<iiiIqqqHHIIIQ", *r) for r in recs) + var
    body += b"\0" * (-len(body) % 8)
    return struct.pack("<QQ", len(recs), 16 + len(body)) + body


def test_inbox_rejects_malformed_batches():
    """zb_inbox_submit checks every batch before anything reaches the device: a count whose records do
    not fit the batch (incl. a count * 64 that overflows), a record whose variable bytes run past the batch's byte
    section, an offset past it, a CORRELATE naming an element the model does not have -- each ZB_EINVAL, with the
    log unchanged; a well-formed batch is then accepted."""
    import struct

    from zeebe_amd.engine import Engine, ZbError

    e = Engine(device=0, partition_id=0, partition_count=1, log_capacity=1 << 16, row_capacity=1 << 12)
    e.deploy(catch_workflow(), 100, 1)
    e.create("wf", [msgpack.packb({"orderId": "order-1"})])
    e.run()
    n0 = e.log_size()
    name, ck = b"order canceled", b"order-1"
    ok_open = (1, 0, 0, 0, 1, 6, 3, 1, 0, len(name), len(ck), 0, 0)
    good = _xbatch([ok_open], name + ck)
    bad = [
        struct.pack("<QQ", 1 << 58, 16 + 64) + good[16:16 + 64],                   # count * 64 overflows
        struct.pack("<QQ", 2, len(good)) + good[16:],                              # two records do not fit
        _xbatch([(1, 0, 0, 0, 1, 6, 3, 1, 0, len(name), 4096, 0, 0)], name + ck),  # ck runs past the section
        _xbatch([(1, 0, 0, 0, 1, 6, 3, 1, 0, len(name), len(ck), 0, 1 << 40)], name + ck),  # offset past it
    ]
    for b in bad:
        with pytest.raises(ZbError, match="ZB_EINVAL"):
            e.inbox(cluster.KIND_OPEN, bytearray(b))
    with pytest.raises(ZbError, match="ZB_EINVAL"):  # CORRELATE of an element the model does not have
        e.inbox(cluster.KIND_CORRELATE, bytearray(_xbatch([(2, 0, 0, 0, 1, 6, 3, 60000, 0, len(name), 0, 1, 0)],
                                                          name + b"\x80")))
    assert e.log_size() == n0
    e.inbox(cluster.KIND_OPEN, bytearray(good))  # (OPEN + OPENED)
    assert e.log_size() == n0 + 2
    e.close()


def _exchange_failure_protocol():
    """(body of test_rccl_exchange_failure_protocol, run in a process that loaded the guard-band build)"""
    import os
    import socket

    import torch.distributed as dist
    from zeebe_amd.engine import CFG_RCCL_SELF, Engine, ZbError, checked_violations

    assert checked_violations() is not None, "the failure hook exists only in the guard-band build"
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        e = Engine(device=0, partition_id=0, partition_count=1, log_capacity=1 << 20, row_capacity=1 << 18,
                   flags=CFG_RCCL_SELF)  # (the P > 1 code path: collectives and send / recv to self)
        e.deploy(catch_workflow(), 100, 1)
        e.create("wf", [msgpack.packb({"orderId": "order-%d" % i}) for i in range(20)])
        dc = cluster.DistCluster(e)
        e.run()
        assert e.comm_pending()[0] == 20
        os.environ["ZB_FAIL_EXCHANGE"] = "0"
        try:
            with pytest.raises(ZbError, match="injected local failure"):
                e.comm_exchange(cluster.KIND_OPEN)
        finally:
            del os.environ["ZB_FAIL_EXCHANGE"]
        assert e.comm_pending()[0] == 20  # nothing was taken
        dc.settle()
        dc.publish(b"order canceled", [b"order-%d" % i for i in range(20)], [b"\x80"] * 20)
        assert e.counters()["completed"] == 20
        assert checked_violations()[0] == 0
        e.close()
    finally:
        dist.destroy_process_group()


def test_rccl_exchange_failure_protocol():
    """A rank whose local part of zb_comm_exchange fails (injected before its outbox is taken) returns an error from
    the collective instead of hanging; the next exchange goes through and the run completes. The injection hook
    (ZB_FAIL_EXCHANGE) exists only in the guard-band test build (zeebe_amd/csrc/zb_checked.hpp), never in the
    product library, so the case runs in a child process that loads that build."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, ZB_CHECKED_LIBRARY="1", PYTHONPATH=os.pathsep.join([root, os.path.join(root, "tests")]))
    code = "import test_gpu_messages as t; t._exchange_failure_protocol(); print('exchange failure protocol ok')"
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "exchange failure protocol ok" in r.stdout, (r.returncode, r.stdout[-2000:],
                                                                              r.stderr[-4000:])


@pytest.mark.parametrize("P", [1, 3])
def test_positions_past_2_34(P):
    """Log positions are 64-bit and never rebased (LogEntryDescriptor.java:28-121; positionAsKey,
    SubscriptionApiCommandMessageHandler.java:146): partitions whose logs continue at and across 2^34 (zb_log_start; the
    oracle with the same position base) correlate exactly as at position 0 -- the outbox order keys hold positions
    relative to the outbox's last take (zb_msg.hpp outbox_key), so a tick straddling 2^34 orders its exchange as any
    other. Covers CORRELATE keys (= positions), source positions, log frames and a message matching more than 32
    subscriptions (the emission index by store-index span)."""
    gpu, ref, cg, co = clusters(P, catch_workflow())
    bases = [(1 << 34) - 40 + p * ((1 << 35) + 7) for p in range(P)]  # partition 0 crosses 2^34 in its first tick
    for g, o, b in zip(gpu, ref, bases):
        g.log_start(b)
        o.set_position_base(b)
        assert g.log_size() == o.log_size() == b
    keys = ["shared"] * 40 + ["order-%d" % i for i in range(30)]
    for i, key in enumerate(keys):
        gpu[i % P].create("wf", [msgpack.packb({"orderId": key})])
        ref[i % P].create("wf", msgpack.packb({"orderId": key}))
    cg.settle()
    co.settle()
    cks = [b"order-%d" % i for i in range(0, 30, 2)] + [b"shared"] + [b"order-%d" % i for i in range(1, 30, 2)]
    pls = [msgpack.packb({"m": i}) for i in range(len(cks))]
    cg.publish(b"order canceled", cks, pls)
    co.publish(b"order canceled", cks, pls)
    for p, (g, o, b) in enumerate(zip(gpu, ref, bases)):
        a, c = o.records(b), g.records(b)
        assert len(a) == len(c) and len(a) > 0, (p, len(a), len(c))
        assert a[-1].position >= (1 << 34), (p, a[-1].position)
        for x, y in zip(a, c):
            assert (x.position, x.source_position, x.key, x.record_type, x.value_type, x.intent) == \
                   (y.position, y.source_position, y.key, y.record_type, y.value_type, y.intent), (p, x, y)
            assert x.value == y.value, (p, x.position)
        assert_frames_equal(o, g, b)
    assert sum(g.counters()["completed"] for g in gpu) == len(keys)
