"""The fast log-frame drains against the generic frame encoder, byte for byte, in the job modes the integration binds.

zb_serialize_frames (the frames the broker appends through LogStreamBatchWriter) has three paths:
  * a deferred trajectory batch: the template drain writes one frame per record straight from the class traces
    (k_tdrain_write<.., true>: the 104-byte prefix of zb_frame.hpp + the value + zero padding);
  * descriptors (ZB_CFG_NO_DEFER here; the wave pipeline in general): the wave-parallel fast encoder k_ser_wave<true>;
  * the generic encoder k_ser_write<true> (ZB_CFG_GENERIC_DRAIN), the reference pass of the two above.
C3 (exclusive gateways, no service task) runs on the trajectory path in every job mode: the workflow processor writes
the same records for a CREATE whichever job processor shares the log (WorkflowInstanceStreamProcessor.java:233-368).
Request metadata: on every CREATE (the dense table), or on half of them (the sorted-search form).
The oracle checks frames and values of the integration mode at a size it runs in seconds.
"""
import msgpack
import numpy as np
import pytest

from frames_check import FRAME_CFG, assert_frames_equal
from oracle import zbref
from zeebe_amd import bpmn, records as R, workloads

pytestmark = pytest.mark.gpu

N = 100_000


def _c3(n, mode, flags, reqs):
    from zeebe_amd.engine import Engine

    e = Engine(log_capacity=n * 16, row_capacity=1 << 20, arena_bytes=n * 64 + (64 << 20), flags=flags,
               external_jobs=mode == "ext", job_processor=mode == "jobproc")
    e.deploy(bpmn.xor_workflow().to_xml(), 100, 1)
    blob, offs = workloads.xor_payloads_np(n)
    h = n // 2
    if reqs == "half":  # metadata on the second half only: the sorted-search form
        e.create_packed("xor", blob[:offs[h]], offs[:h + 1])
        e.create_packed("xor", blob[offs[h]:], offs[h:] - offs[h])
        m = n - h
    else:
        e.create_packed("xor", blob, offs)
        m = n
    e.set_request_metadata([1000 + 3 * i for i in range(m)], [i % 5 for i in range(m)])
    st = e.step()
    assert st["quiescent"] and st["completed_instances"] == n
    L = e.log_size()
    ser = e.serialize_frames(n, L - n, **FRAME_CFG)  # the records the tick wrote (the broker appends them)
    buf = np.empty(max(ser["value_bytes"], 1), dtype=np.uint8)
    e.drain_copy(buf.ctypes.data, 0, ser["value_bytes"])
    e.close()
    return st, ser, buf[:ser["value_bytes"]], L


@pytest.mark.parametrize("mode,reqs", [("harness", "all"), ("ext", "all"), ("jobproc", "half"), ("ext", "half")])
def test_fast_frames_equal_generic_c3(mode, reqs):
    from zeebe_amd.engine import CFG_GENERIC_DRAIN, CFG_NO_DEFER

    st, ser, tmpl, L = _c3(N, mode, 0, reqs)
    assert st["path"] == 2 and ser["template_drain"] == 1  # the integration mode takes the trajectory path
    st2, ser2, wave, L2 = _c3(N, mode, CFG_NO_DEFER, reqs)
    assert ser2["template_drain"] == 0 and ser2["generic_tiles"] == 0  # every tile through k_ser_wave<true>
    st3, ser3, gen, L3 = _c3(N, mode, CFG_NO_DEFER | CFG_GENERIC_DRAIN, reqs)
    assert L == L2 == L3 and ser["records"] == ser3["records"] == L - N
    assert ser["value_bytes"] == ser2["value_bytes"] == ser3["value_bytes"]
    assert np.array_equal(wave, gen)
    assert np.array_equal(tmpl, gen)
    # the first generation (CREATED + ELEMENT_READY of every instance, sourced by its CREATE): request metadata
    off = 0
    for _ in range(2 * N):
        off += (int(tmpl[off:off + 4].view("<u4")[0]) + 7) & ~7
    fr = R.parse_frames(tmpl[:off].tobytes())
    created = [f for f in fr if f["value_type"] == R.VT_WORKFLOW_INSTANCE and f["intent"] == R.WI_CREATED]
    assert len(created) == N
    for f in created:
        i = f["source_position"]  # the CREATE at position i is instance i's command
        if reqs == "all" or i >= N // 2:
            j = i if reqs == "all" else i - N // 2
            assert (f["request_id"], f["request_stream_id"]) == (1000 + 3 * j, j % 5)
        else:
            assert f["request_id"] == 2 ** 64 - 1


@pytest.mark.parametrize("mode", ["ext", "jobproc"])
def test_integration_mode_frames_vs_oracle(mode):
    """C3 in the integration's job modes at 3000 instances: the template drain's frames of the tick equal the oracle's,
    and so do the whole log's frames and values (materialized: k_ser_wave<true>)."""
    from zeebe_amd.engine import Engine

    n = 3000
    xml = bpmn.xor_workflow().to_xml()
    o = zbref.Oracle()
    o.set_harness(False)
    e = Engine(external_jobs=mode == "ext", job_processor=mode == "jobproc")
    for x in (o, e):
        x.deploy(xml, 100, 1)
    payloads = workloads.split(*workloads.xor_payloads(n))
    for i, p in enumerate(payloads):
        o.create("xor", p)
        o.set_request(o.log_size() - 1, 7 + i, i % 3)
    e.create("xor", payloads)
    e.set_request_metadata([7 + i for i in range(n)], [i % 3 for i in range(n)])
    o.run()
    st = e.step()
    assert st["quiescent"] and st["path"] == 2
    assert_frames_equal(o, e, n)  # exactly the deferred batch: the template drain
    assert_frames_equal(o, e)  # the whole log (materialized descriptors)
    ref, got = o.records(), e.records()
    assert [(r.key, r.record_type, r.intent, r.value) for r in ref] == \
           [(r.key, r.record_type, r.intent, r.value) for r in got]
    e.close()


def test_wave_pipeline_frames_fast_equal_generic():
    """C2 on the wave pipeline with external jobs (the integration's other mode): CREATE tick, then a tick of job events
    for every pending job; the frames of each tick through k_ser_wave<true> equal k_ser_write<true>'s."""
    from zeebe_amd.engine import CFG_GENERIC_DRAIN, Engine

    n = 20000
    cfg = workloads.CONFIGS["c2"]
    xml = cfg["workflow"]().to_xml()
    outs = []
    for flags in (0, CFG_GENERIC_DRAIN):
        e = Engine(log_capacity=1 << 23, row_capacity=1 << 21, arena_bytes=1 << 28, external_jobs=True, flags=flags)
        e.deploy(xml, 100, 1)
        e.create_packed(cfg["process"], *cfg["payloads"](n))
        assert e.step()["quiescent"]
        ticks = [e.frames(0, None, **FRAME_CFG)]
        recs = e.records()
        jobs = [r for r in recs if r.value_type == R.VT_JOB and r.intent == R.JI_CREATE]
        assert len(jobs) == n
        start = e.log_size()
        evs = []
        for k, r in enumerate(jobs):  # the external job processor's events (keys of its own generator)
            key = (1 << 40) + 5 * k
            evs.append((R.RT_EVENT, R.VT_JOB, R.JI_CREATED, key, R.job_event(r.value)))
            evs.append((R.RT_EVENT, R.VT_JOB, R.JI_COMPLETED, key,
                        R.job_event(r.value, msgpack.packb({"job": k, "note": "x" * (k % 300)}))))
        e.submit_records(evs)
        assert e.step()["quiescent"]
        ticks.append(e.frames(start, None, **FRAME_CFG))
        e.close()
        outs.append(ticks)
    assert outs[0] == outs[1]
