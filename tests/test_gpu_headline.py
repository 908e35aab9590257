"""The bench's headline step (C3, 10M instances, BASELINE.json configs[2]) byte-checked in the configuration that
produces the number: product configuration (no diagnostic flags), the batch left without descriptors by zb_step and drained
from its traces (zb_tdrain.hip).

  * the template drain's values and record headers equal the generic encoder's over the descriptors
    (ZB_CFG_NO_DEFER: k_tmpl writes them; ZB_CFG_GENERIC_DRAIN: every tile through k_ser_write), byte for byte, for all
    ~101.7M records;
  * a strided sample of instances: every record's value equals the reference's bytes for that instance -- the
    oracle runs the instance alone, its keys are mapped onto the keys the 10M run gave the same records (in
    order), and the values re-encoded with those keys (msgpack's minimal encodings = MsgPackWriter's).
"""
import ctypes

import msgpack
import numpy as np
import pytest

from oracle import zbref
from zeebe_amd import bpmn, workloads

pytestmark = pytest.mark.gpu

N = 10_000_000


def _run(monkeypatch, fast):
    from zeebe_amd.engine import CFG_GENERIC_DRAIN, CFG_NO_DEFER, Engine

    e = Engine(log_capacity=N * 16, row_capacity=1 << 20, arena_bytes=N * 64 + (64 << 20),
               flags=0 if fast else CFG_GENERIC_DRAIN | CFG_NO_DEFER)
    e.deploy(bpmn.xor_workflow().to_xml(), 100, 1)
    blob, offs = workloads.xor_payloads_np(N)
    e.create_packed("xor", blob, offs)
    del blob
    st = e.step()
    assert st["quiescent"] and st["path"] == 2 and st["completed_instances"] == N
    L = e.log_size()
    ser = e.serialize(N, L - N)  # the bench's drain: the records the tick wrote
    return e, ser, L


def _copy(e, ser, count):
    from zeebe_amd.engine import zb_record_header

    vals = np.empty(ser["value_bytes"], dtype=np.uint8)
    hdrs = (zb_record_header * count)()
    e.drain_copy(vals.ctypes.data, 0, ser["value_bytes"], ctypes.addressof(hdrs))
    return vals, np.frombuffer(hdrs, dtype=np.uint8).copy()


def test_headline_template_drain_equals_generic_and_reference(monkeypatch):
    e, ser, L = _run(monkeypatch, True)
    count = L - N
    assert ser["template_drain"] == 1 and ser["generic_tiles"] == 0  # drained from the traces
    vals, hdrs = _copy(e, ser, count)
    # per-instance check on a strided sample (the descriptors: materialized on demand)
    from test_gpu_properties import descriptors

    d = descriptors(e, N, count)
    e.close()
    H = np.frombuffer(hdrs.tobytes(), dtype=np.dtype([("key", "<i8"), ("rt", "u1"), ("vt", "u1"), ("intent", "u1"),
                                                       ("rej", "u1"), ("len", "<u4"), ("off", "<u8")]))
    sample = list(range(0, N, N // 37))[:37] + [N - 1]
    keys = 1 + 5 * np.array(sample, dtype=np.int64)  # instance keys: the CREATEs are processed in order
    for i, ik in zip(sample, keys):
        payload = workloads.split(*workloads.xor_payloads(1, start=i))[0]
        o = zbref.Oracle()
        o.deploy(bpmn.xor_workflow().to_xml(), 100, 1)
        o.create("xor", payload)
        o.run()
        ref = [r for r in o.records() if r.record_type == 0]  # its events (the CREATE command is not drained)
        idx = np.nonzero(d["inst_key"] == ik)[0]
        assert len(idx) == len(ref), (i, len(idx), len(ref))
        kmap = {}
        for r, j in zip(ref, idx):
            if r.key in kmap:
                assert kmap[r.key] == H["key"][j], (i, r)
            kmap.setdefault(r.key, int(H["key"][j]))
            assert (H["intent"][j], H["vt"][j], H["rt"][j]) == (r.intent, r.value_type, r.record_type), (i, r)
            v = msgpack.unpackb(r.value, raw=False)
            for f in ("workflowInstanceKey", "scopeInstanceKey"):
                if v.get(f, -1) >= 0:
                    v[f] = kmap[v[f]]
            want = msgpack.packb(v, use_bin_type=True)
            got = vals[H["off"][j]:H["off"][j] + H["len"][j]].tobytes()
            assert got == want, (i, r.intent, msgpack.unpackb(got, raw=False), v)
    del d
    # the generic encoder over the same log: identical bytes
    e2, ser2, L2 = _run(monkeypatch, False)
    assert ser2["template_drain"] == 0
    assert L2 == L and ser2["value_bytes"] == ser["value_bytes"] and ser2["payload_bytes"] == ser["payload_bytes"]
    vals2, hdrs2 = _copy(e2, ser2, count)
    e2.close()
    assert np.array_equal(hdrs, hdrs2)
    step = 1 << 28
    for o in range(0, len(vals), step):
        assert np.array_equal(vals[o:o + step], vals2[o:o + step]), o
