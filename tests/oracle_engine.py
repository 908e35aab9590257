"""Test infrastructure: a CPU stand-in for zeebe_amd.engine.Engine in the controller emulation (tests/
controller_sim.py), so that the stream-processor protocol (zeebe_amd/stream_processor.py) runs without a GPU.

It is the oracle (oracle/zbref.cpp, the sequential restatement of the reference) behind the engine's interface:
a tick's staged records are submitted and run to quiescence (like zb_submit, it takes records of one instance that
race in any order: the engine serialises them, the oracle is sequential anyway); snapshot / restore replay the tick
history into a fresh oracle. Never product code: the GPU variant of the same tests runs the real engine.
"""
from __future__ import annotations

import base64
import json

from oracle import zbref


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

    def submit_records(self, recs):
        for rec in recs:
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
