"""Message correlation across partitions: the oracle against the reference's known answers.

Expected values are transcribed from
broker-core/src/test/java/io/zeebe/broker/workflow/IntermediateMessageCatchEventTest.java (file:line
per test), run through zeebe_amd.cluster's canonical schedule (LocalCluster in one process,
DistCluster over gloo with world size 2). CPU only.
"""
import os
import socket

import msgpack
import pytest

from oracle import zbref
from zeebe_amd import bpmn, cluster

P = 3  # IntermediateMessageCatchEventTest runs on "zeebe.unit-test.increased.partitions.cfg.toml"
WF_PARTITION = 0


def workflow_xml():
    # IntermediateMessageCatchEventTest.java:59-66
    return (bpmn.Bpmn.create_executable_process("wf").start_event()
            .intermediate_catch_event("catch-event", message="order canceled", correlation_key="$.orderId")
            .sequence_flow_id("to-end").end_event().done().to_xml())


def make_cluster(partitions=P):
    parts = [zbref.OraclePartition(p, partitions) for p in range(partitions)]
    for p in parts:
        p.deploy(workflow_xml(), 100, 1)
    return parts, cluster.LocalCluster(parts)


def create(parts, payload, partition=WF_PARTITION):
    parts[partition].create("wf", msgpack.packb(payload))


def wf_events(part):
    out = []
    for r in part.records():
        if r.value_type == 5:
            out.append((r, msgpack.unpackb(r.value, raw=False)))
    return out


def all_records(parts):
    return [(i, r) for i, p in enumerate(parts) for r in p.records()]


WF_INTENTS = ["CREATE", "CREATED", "START_EVENT_OCCURRED", "END_EVENT_OCCURRED", "SEQUENCE_FLOW_TAKEN",
              "GATEWAY_ACTIVATED", "ELEMENT_READY", "ELEMENT_ACTIVATED", "ELEMENT_COMPLETING", "ELEMENT_COMPLETED",
              "ELEMENT_TERMINATING", "ELEMENT_TERMINATED", "CANCEL", "CANCELING"]


def test_hash_routing_matches_reference_vectors(vectors):
    # SubscriptionUtilTest.java:29-43 and the oracle's C restatement agree with cluster.java_hash
    for s, h in vectors["hashes"]:
        assert cluster.java_hash(s.encode()) == h == zbref.subscription_hash(s.encode())
    for s in ("order-123", "order-456", "ü-non-ascii", "x" * 40):
        b = s.encode()
        assert cluster.java_hash(b) == zbref.subscription_hash(b)
        assert cluster.subscription_partition(b, 7) == abs(zbref.subscription_hash(b) % 7 if zbref.subscription_hash(b) >= 0
                                                           else -((-zbref.subscription_hash(b)) % 7))


def test_lifecycle_with_message_published_first():
    # testWorkflowInstanceLifeCycle :94-117
    parts, c = make_cluster()
    c.publish(b"order canceled", [b"order-123"], [b"\x80"])
    create(parts, {"orderId": "order-123"})
    c.settle()
    intents = [WF_INTENTS[r.intent] for r, _ in wf_events(parts[WF_PARTITION])][:11]
    assert intents == ["CREATE", "CREATED", "ELEMENT_READY", "ELEMENT_ACTIVATED", "START_EVENT_OCCURRED",
                       "SEQUENCE_FLOW_TAKEN", "ELEMENT_READY", "ELEMENT_ACTIVATED", "ELEMENT_COMPLETING",
                       "ELEMENT_COMPLETED", "SEQUENCE_FLOW_TAKEN"]


def test_open_message_subscription_value():
    # shouldOpenMessageSubscription :120-139 (containsExactly)
    parts, c = make_cluster()
    create(parts, {"orderId": "order-123"})
    c.settle()
    wf = wf_events(parts[WF_PARTITION])
    wik = wf[1][0].key
    activated = [r for r, v in wf if v["activityId"] == "catch-event" and WF_INTENTS[r.intent] == "ELEMENT_ACTIVATED"][0]
    target = cluster.subscription_partition(b"order-123", P)
    opened = [r for r in parts[target].records() if r.value_type == 11 and r.record_type == 0 and r.intent == 1]
    assert len(opened) == 1
    assert msgpack.unpackb(opened[0].value, raw=False) == {
        "workflowInstancePartitionId": WF_PARTITION, "workflowInstanceKey": wik,
        "activityInstanceKey": activated.key, "messageName": "order canceled", "correlationKey": "order-123"}
    # the command's key is its log position (positionAsKey) and the event keeps it
    assert opened[0].key == [r for r in parts[target].records() if r.value_type == 11][0].position


@pytest.mark.parametrize("published_first", [False, True])
def test_correlate_and_merge_payload(published_first):
    # shouldCorrelateMessageIfEnteredBefore :175-198, shouldCorrelateMessageIfPublishedBefore :201-222
    parts, c = make_cluster()
    if published_first:
        c.publish(b"order canceled", [b"order-123"], [msgpack.packb({"foo": "bar"})])
    create(parts, {"orderId": "order-123"})
    c.settle()
    if not published_first:
        c.publish(b"order canceled", [b"order-123"], [msgpack.packb({"foo": "bar"})])
    done = [v for r, v in wf_events(parts[WF_PARTITION])
            if v["activityId"] == "catch-event" and WF_INTENTS[r.intent] == "ELEMENT_COMPLETED"]
    assert len(done) == 1
    assert done[0]["bpmnProcessId"] == "wf" and done[0]["version"] == 1
    assert msgpack.unpackb(done[0]["payload"], raw=False) == {"orderId": "order-123", "foo": "bar"}
    # shouldContinueInstanceAfteMessageIsCorrelated :225-243
    assert any(v["activityId"] == "to-end" for r, v in wf_events(parts[WF_PARTITION]))
    assert parts[WF_PARTITION].counters()["completed"] == 1


def test_correlate_with_zero_ttl():
    # shouldCorrelateMessageWithZeroTTL :246-261: the message is deleted at once, but correlates
    parts, c = make_cluster()
    create(parts, {"orderId": "order-123"})
    c.settle()
    c.publish(b"order canceled", [b"order-123"], [msgpack.packb({"foo": "bar"})], ttl=0)
    assert parts[WF_PARTITION].counters()["completed"] == 1
    target = cluster.subscription_partition(b"order-123", P)
    intents = [(r.record_type, r.intent) for r in parts[target].records() if r.value_type == 10]
    assert intents == [(1, 0), (0, 1), (0, 3)]  # PUBLISH, PUBLISHED, DELETED


def test_no_correlation_after_ttl():
    # shouldNotCorrelateMessageAfterTTL :264-279
    parts, c = make_cluster()
    c.publish(b"order canceled", [b"order-123"], [msgpack.packb({"nr": "first"})], ttl=0)
    c.publish(b"order canceled", [b"order-123"], [msgpack.packb({"nr": "second"})], ttl=10000)
    create(parts, {"orderId": "order-123"})
    c.settle()
    done = [v for r, v in wf_events(parts[WF_PARTITION])
            if v["activityId"] == "catch-event" and WF_INTENTS[r.intent] == "ELEMENT_COMPLETED"]
    assert msgpack.unpackb(done[0]["payload"], raw=False) == {"orderId": "order-123", "nr": "second"}


def test_correlate_by_correlation_key_and_to_all_subscriptions():
    # shouldCorrelateMessageByCorrelationKey :282-307, shouldCorrelateMessageToAllSubscriptions :310-332
    parts, c = make_cluster()
    create(parts, {"orderId": "order-123"})
    create(parts, {"orderId": "order-456"})
    create(parts, {"orderId": "order-123"})
    c.settle()
    c.publish(b"order canceled", [b"order-123", b"order-456"],
              [msgpack.packb({"foo": "bar"}), msgpack.packb({"foo": "baz"})])
    done = {}
    for r, v in wf_events(parts[WF_PARTITION]):
        if v["activityId"] == "catch-event" and WF_INTENTS[r.intent] == "ELEMENT_COMPLETED":
            done[v["workflowInstanceKey"]] = msgpack.unpackb(v["payload"], raw=False)
    assert sorted(done.values(), key=str) == sorted([
        {"orderId": "order-123", "foo": "bar"}, {"orderId": "order-456", "foo": "baz"},
        {"orderId": "order-123", "foo": "bar"}], key=str)


def test_correlated_record_value():
    # shouldCorrelateWorkflowInstanceSubscription :335-363 (containsExactly, 4 entries)
    parts, c = make_cluster()
    create(parts, {"orderId": "order-123"})
    c.settle()
    wf = wf_events(parts[WF_PARTITION])
    wik = wf[1][0].key
    aik = [r for r, v in wf if v["activityId"] == "catch-event" and WF_INTENTS[r.intent] == "ELEMENT_ACTIVATED"][0].key
    payload = msgpack.packb({"foo": "bar"})
    c.publish(b"order canceled", [b"order-123"], [payload])
    recs = [r for r in parts[WF_PARTITION].records() if r.value_type == 12]
    assert [(r.record_type, r.intent) for r in recs] == [(1, 0), (0, 1)]
    assert recs[1].key == recs[0].key == recs[0].position
    assert msgpack.unpackb(recs[1].value, raw=False) == {
        "workflowInstanceKey": wik, "activityInstanceKey": aik, "messageName": "order canceled", "payload": payload}


def test_reject_correlate_after_cancel():
    # shouldRejectCorrelateCommand :366-398
    parts, c = make_cluster()
    create(parts, {"orderId": "order-123"})
    c.settle()
    wf = wf_events(parts[WF_PARTITION])
    wik = wf[1][0].key
    aik = [r for r, v in wf if v["activityId"] == "catch-event" and WF_INTENTS[r.intent] == "ELEMENT_ACTIVATED"][0].key
    parts[WF_PARTITION].cancel(wik)
    c.settle()
    c.publish(b"order canceled", [b"order-123"], [b"\x80"])
    rej = [r for r in parts[WF_PARTITION].records() if r.value_type == 12 and r.record_type == 2]
    assert len(rej) == 1 and rej[0].intent == 0 and rej[0].rejection_type == 1  # NOT_APPLICABLE
    v = msgpack.unpackb(rej[0].value, raw=False)
    assert v["workflowInstanceKey"] == wik and v["activityInstanceKey"] == aik


# ---------------------------------------------------------------- DistCluster over gloo (world size 2)
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _c5_inputs(n):
    cks = [b"order-%d" % i for i in range(n)]
    return cks, [msgpack.packb({"paid": True})] * n


def _dist_worker(rank, world, port, n, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = zbref.OraclePartition(rank, world)
    p.deploy(workflow_xml(), 100, 1)
    cks, pls = _c5_inputs(n)
    for i in range(rank, n, world):  # round-robin CREATE dispatch
        p.create("wf", msgpack.packb({"orderId": cks[i].decode()}))
    dc = cluster.DistCluster(p)
    dc.settle()
    dc.publish(b"order canceled", cks, pls)
    q.put((rank, p.dump(), p.counters()["completed"]))
    dist.barrier()
    dist.destroy_process_group()


def test_dist_cluster_gloo_matches_local_cluster():
    import torch.multiprocessing as mp

    n, world = 40, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dist_worker, args=(r, world, port, n, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    got = {}
    for _ in range(world):
        rank, dump, completed = q.get(timeout=120)
        got[rank] = (dump, completed)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    # the same schedule in one process
    parts, c = make_cluster(world)
    cks, pls = _c5_inputs(n)
    for i in range(n):
        parts[i % world].create("wf", msgpack.packb({"orderId": cks[i].decode()}))
    c.settle()
    c.publish(b"order canceled", cks, pls)
    for r in range(world):
        assert got[r][0] == parts[r].dump()
    assert sum(got[r][1] for r in range(world)) == n
