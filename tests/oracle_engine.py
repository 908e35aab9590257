"""Test infrastructure: a CPU stand-in for zeebe_amd.engine.Engine in the controller emulation (tests/
controller_sim.py), so that the stream-processor protocol (zeebe_amd/stream_processor.py) runs without a GPU.

It is the oracle (oracle/zbref.cpp, the sequential restatement of the reference) behind the engine's interface:
a tick's staged records are submitted and run to quiescence; the per-tick race rules of zb_submit
(zeebe_amd/csrc/zb_engine.hip, "race rules of one tick"; include/zb_engine.h) are restated so that ticks split
where the GPU engine splits them; snapshot / restore replay the tick history into a fresh oracle. Never product
code: the GPU variant of the same tests runs the real engine.
"""
from __future__ import annotations

import base64
import json

import msgpack

from oracle import zbref
from zeebe_amd import records as R
from zeebe_amd.engine import ZB_EUNSUPPORTED, ZbError


def _race_keys(rec):
    """(workflow instance, activity instance, scope command) of a non-CREATE record, as zb_submit decodes them."""
    rt, vt, it, key, value = rec
    v = msgpack.unpackb(value, raw=False) if value else {}
    if vt == R.VT_WORKFLOW_INSTANCE and rt == R.RT_COMMAND:
        return (key if it == R.WI_CANCEL else v.get("workflowInstanceKey", -1)), None, True
    if vt == R.VT_JOB:
        h = v.get("headers", {})
        return h.get("workflowInstanceKey", -1), h.get("activityInstanceKey", -1), False
    return v.get("workflowInstanceKey", -1), v.get("activityInstanceKey", -1), False  # CORRELATE


class OracleEngine:
    def __init__(self, deployments, external_jobs=True):
        self.deployments = list(deployments)  # (xml, workflow key)
        self.external_jobs = external_jobs
        self.history = []  # ticks: [(rec, request id, request stream id)]
        self._new()

    def _new(self):
        self.o = zbref.Oracle()
        self.o.set_harness(not self.external_jobs)
        for xml, k in self.deployments:
            self.o.deploy(xml, k, 1)
        self.staged = []
        self.inst, self.aiks = {}, set()

    def submit_records(self, recs):
        for rec in recs:
            rt, vt, it, key, value = rec
            if not (vt == R.VT_WORKFLOW_INSTANCE and rt == R.RT_COMMAND and it == R.WI_CREATE):
                prev = self.staged[-1][0] if self.staged else None
                pair = (vt == R.VT_JOB and it == R.JI_COMPLETED and prev is not None and prev[1] == R.VT_JOB and
                        prev[2] == R.JI_CREATED and prev[3] == key and _race_keys(prev)[1] == _race_keys(rec)[1])
                if not pair:
                    inst, aik, scope = _race_keys(rec)
                    f = self.inst.get(inst, 0)
                    if (f & 1) or (scope and f):
                        raise ZbError(ZB_EUNSUPPORTED, "workflow instance %d races in this tick" % inst)
                    if aik is not None and aik in self.aiks:
                        raise ZbError(ZB_EUNSUPPORTED, "activity instance %d races in this tick" % aik)
                    self.inst[inst] = f | (1 if scope else 2)
                    if aik is not None:
                        self.aiks.add(aik)
            self.staged.append([rec, None, None])

    def set_request_metadata(self, rids, sids):
        for k, (rid, sid) in enumerate(zip(rids, sids)):
            st = self.staged[len(self.staged) - len(rids) + k]
            st[1], st[2] = rid, sid

    def _run_tick(self, tick):
        base = self.o.log_size()
        for i, (rec, rid, sid) in enumerate(tick):
            self.o.submit(*rec)
            if rid is not None:
                self.o.set_request(base + i, rid, sid)
        self.o.run()

    def step(self):
        tick, self.staged = self.staged, []
        self.inst, self.aiks = {}, set()
        self._run_tick(tick)
        self.history.append(tick)
        return {"quiescent": True}

    def log_size(self):
        return self.o.log_size()

    def frames(self, start, count, **cfg):
        return self.o.frames(start, start + count, **cfg)

    def release(self, position):
        pass

    def snapshot(self) -> bytes:
        enc = lambda t: [[list(rec[:4]) + [base64.b64encode(rec[4]).decode()], rid, sid] for rec, rid, sid in t]  # noqa
        return json.dumps([enc(t) for t in self.history]).encode()

    def restore(self, snap: bytes):
        self.o.close()
        self._new()
        self.history = []
        for t in json.loads(snap):
            tick = [((r[0], r[1], r[2], r[3], base64.b64decode(r[4])), rid, sid) for r, rid, sid in t]
            self._run_tick(tick)
            self.history.append(tick)

    def close(self):
        self.o.close()
