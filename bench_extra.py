"""bench.py --config c5: message correlation across partitions (the default run is C3, bench.py).

C5: start -> message catch ("order", $.orderId) -> end, instances round-robin over the
    partitions (one per GPU); phase 1 runs the CREATEs to quiescence (subscriptions opened on partition
    abs(hash % P)), phase 2 publishes one message per orderId (TTL 1 h, payload {"paid": true}) and runs
    to quiescence. The engines exchange the subscription / correlation commands over RCCL
    (zeebe_amd.cluster.DistCluster). One step = both phases; transitions = WORKFLOW_INSTANCE events.
"""
import json
import os
import time

import numpy as np

HBM_PEAK_GBS = 8000.0
BYTES_PER_TRANSITION = 96


def _routing(cks, world):
    """abs(javaHash(ck) % P) for many keys at once (SubscriptionUtil.java:30-38), vectorized by length."""
    out = np.zeros(len(cks), dtype=np.int64)
    by_len = {}
    for i, c in enumerate(cks):
        by_len.setdefault(len(c), []).append(i)
    for L, idx in by_len.items():
        a = np.frombuffer(b"".join(cks[i] for i in idx), dtype=np.int8).reshape(len(idx), L).astype(np.int64)
        h = np.zeros(len(idx), dtype=np.int64)
        for j in range(L):
            h = (h * 31 + a[:, j]) & 0xFFFFFFFF
        h = np.where(h >= (1 << 31), h - (1 << 32), h)
        out[np.asarray(idx)] = np.abs(np.fmod(h, world))
    return out


def _emit(out, rank):
    if rank == 0:
        print(json.dumps(out))


def cpu_baseline_c5(world, n_sample):
    """The oracle (C++ restatement) on a bounded C5 sample: `world` oracle partitions, each stepped on its own
    thread, with the exchange rounds of zeebe_amd.cluster.LocalCluster restated in C++ (oracle/zbref.cpp
    zbref_c5_bench: no Python in the timed region), timed from the first CREATE to the quiescence after the
    publishes. The reference's message and subscription stores are ArrayLists scanned per command
    (MessageDataStore.java:37-56, MessageSubscriptionDataStore.java:47-55) and the oracle keeps them so, which makes
    the CPU cost grow with the per-partition sample: the sample size is stated."""
    from oracle import zbref
    from zeebe_amd import bpmn

    P = max(world, 1)
    wall, tr, comp, rounds = zbref.c5_bench(P, n_sample, bpmn.message_workflow().to_xml())
    from bench import cpu_model

    return {"value": tr / wall, "unit": "transitions/s", "cores": P, "kind": "port",
            "sample": "C5, %d instances on each of %d oracle partitions, one thread per partition, exchange rounds in "
                      "C++ (%d rounds): %.2f s, %d transitions" % (n_sample, P, rounds, wall, tr),
            "cpu_model": cpu_model(), "completed_instances_per_s": comp / wall}


def run_c5(a, rank, world, local_rank, dist, barrier, reduce_max, reduce_sum):
    import msgpack

    from zeebe_amd import bpmn, cluster
    from zeebe_amd.engine import Engine, rccl_library

    n = a.instances  # per partition
    N = n * world
    eng = Engine(device=0 if a.same_device else local_rank, partition_id=rank, partition_count=world,
                 log_capacity=n * 24, row_capacity=4 * n + 1024, arena_bytes=n * 640 + (64 << 20))
    eng.deploy(bpmn.message_workflow().to_xml(), 100, 1)
    # instance i -> partition i % P (round-robin CREATE dispatch)
    mine = range(rank, N, world)
    create_payloads = [msgpack.packb({"orderId": "order-%d" % i}) for i in mine]
    cks = [b"order-%d" % i for i in range(N)]
    route = _routing(cks, world)
    my_msgs = [cks[i] for i in np.nonzero(route == rank)[0]]
    paid = msgpack.packb({"paid": True})
    dc = cluster.DistCluster(eng)
    # the PUBLISH commands, packed once like the staged CREATEs (input preparation, not processing)
    ck_off = np.zeros(len(my_msgs) + 1, dtype=np.uint64)
    ck_off[1:] = np.cumsum([len(c) for c in my_msgs])
    pl_off = np.arange(len(my_msgs) + 1, dtype=np.uint64) * len(paid)
    ck_blob, pl_blob = b"".join(my_msgs), paid * len(my_msgs)
    tot = dict(records=0, value_bytes=0, transitions=0, ser_ms=0.0)

    def step():
        eng.reset()
        # the tick's input in HBM before the timed region (bench contract): the staged CREATE commands and the
        # PUBLISH batch (zb_upload_staged / zb_upload_publishes; a broker overlaps them with the previous tick)
        eng.create("msg", create_payloads)
        eng.upload_staged()
        if my_msgs:
            eng.upload_publishes_packed(b"order", ck_blob, ck_off, pl_blob, pl_off, 3600000)
        t = time.perf_counter()
        dc.settle()
        if my_msgs:
            eng.publish_uploaded()
        dc.settle()
        ser = eng.serialize(0, eng.log_size())  # the drain: every record the partition's log holds after the step
        dt = time.perf_counter() - t
        return dt, ser

    for _ in range(a.warmup):
        step()
    barrier()
    el = 0.0
    step_ms = []
    for _ in range(a.steps):
        barrier()
        dt, ser = step()
        step_ms.append(reduce_max(dt) * 1e3)
        el += step_ms[-1] / 1e3
        tot["records"] += ser["records"]
        tot["value_bytes"] += ser["value_bytes"]
        tot["ser_ms"] += ser["write_kernel_ms"] + ser["size_kernel_ms"]
    completed = reduce_sum(eng.counters()["completed"])
    assert completed == N, (completed, N)
    tr = 13 * N * a.steps  # 13 WORKFLOW_INSTANCE events per instance
    path_bytes = (BYTES_PER_TRANSITION * 13 + 2 * len(paid)) * N  # + P per correlation-key extraction / merge (approx.)
    ms = el * 1e3 / a.steps
    out = {"metric": "BPMN element transitions/sec (+ completed instances/sec) per node; % HBM roofline",
           "value": tr / el, "unit": "transitions/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
           "ms_per_step": ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "int64", "data": "synthetic (SURVEY §8d C5: orderId 'order-<i>', payload {paid: true})",
           "config": {"workload": "C5: message catch correlated across partitions (RCCL exchange), "
                                  "%d instances per GPU" % n, "instances_per_gpu": n, "partitions": world,
                      "parallelism": "partition-per-gpu", "exchange": "RCCL ncclSend/ncclRecv (engine)" if world > 1 else
                      "one partition: its outbox is its own inbox, on the device (no peer to exchange with)",
                      "timed_step": "CREATE injection to quiescence, exchange rounds, publish to quiescence, "
                                    "zb_serialize of every record of the partition's log (values + headers, in HBM); "
                                    "the CREATE and PUBLISH inputs are uploaded before the timed region"},
           "completed_instances_per_s": N * a.steps / el,
           "step_ms": [round(x, 3) for x in step_ms],
           "drained_records_per_step_rank0": tot["records"] / a.steps,
           "rccl_library": rccl_library(),
           "roofline": {"bound": "hbm", "achieved": path_bytes / (ms / 1e3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": path_bytes / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, "traffic": None,
                        "kernel": "whole step (host-driven exchange rounds; no single dominant kernel)",
                        "alg_bytes_model": "SURVEY §8d: 96 B per transition + payload terms, all partitions",
                        "path_frac": path_bytes / (ms / 1e3) / 1e9 / HBM_PEAK_GBS},
           "note": "excludes payload generation and hash routing of the published keys (input preparation)"}
    # HBM bytes of the step's kernels (every zbg / rocprim kernel of a PMC run of one step: FETCH_SIZE x2 + WRITE_SIZE,
    # separate rocprofv3 --pmc passes; the runtime's fill / copy kernels of the untimed reset and uploads excluded)
    from bench import ROOT, _pmc_file, load_traffic_step

    traffic = load_traffic_step("c5_%d" % n, ("zbg::", "void zbg::", "void rocprim::"))
    if traffic:
        out["roofline"]["traffic"] = traffic
        out["roofline"]["traffic_note"] = ("HBM bytes per step of every engine kernel (zbg / rocprim) from rocprofv3 "
                                           "FETCH_SIZE x2 + WRITE_SIZE (%s)" % os.path.relpath(_pmc_file("c5_%d" % n),
                                                                                                 ROOT))
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        # the shape of this line (one partition, its outbox delivered to its own inbox) on one core, and the node's
        # shape (P partitions exchanging, one core each) beside it
        one = cpu_baseline_c5(1, a.cpu_sample or 8000)
        one["multi_partition"] = cpu_baseline_c5(8 if a.cpu_partitions == 0 else a.cpu_partitions, a.cpu_sample or 8000)
        out["cpu_baseline"] = one
    _emit(out, rank)
