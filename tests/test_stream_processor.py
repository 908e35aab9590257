"""The engine behind the reference's stream-processor surface (zeebe_amd/stream_processor.py), driven
by an emulation of the partition log and of StreamProcessorController (tests/controller_sim.py):

* clients append CREATE commands (with request ids) and CANCELs; an emulated job processor answers every JOB CREATE
  command the engine writes with JOB CREATED and, later, JOB COMPLETED events (producer id 10) -- some of them for
  instances being cancelled in the same tick (the engine serialises such records), some for instances already gone;
  more CREATEs arrive while the processor is writing a tick's follow-ups;
* the follow-ups go to the log as one batch per processed record, with source positions mapped to log positions and
  the reference's producer ids and batch flags; the processor skips them when it reads them back;
* snapshots are taken between records (with inputs staged, in the middle of a reconciliation); the broker is killed
  between ticks and in the middle of writing a tick; the restarted processor restores the snapshot, reconciles the
  follow-ups the dead one wrote (regenerating them without writing and matching each, field by field) and writes
  the ones it had not written yet.

Checks: the log of a run with crashes is byte-identical to the log of the same schedule without them (no record
written twice, none lost, every reprocessed tick regenerated identically), and every tick's follow-ups equal the
oracle's for the same inputs (keys, values, types, request ids, producer ids, batch flags, mapped source positions).
The CPU variant runs the protocol over a CPU stand-in of the engine (tests/oracle_engine.py); the GPU variant runs
the HIP engine.
"""
import msgpack
import pytest

from controller_sim import Controller, Crash, Log, SnapshotStorage
from oracle import zbref
from zeebe_amd import records as R, workloads
from zeebe_amd.stream_processor import GpuStreamProcessor

C1, C4T = workloads.CONFIGS["c1"], workloads.CONFIGS["c4twin"]
DEPLOY = [(C1["workflow"]().to_xml(), 100), (C4T["workflow"]().to_xml(), 200)]
CLIENT, JOBS = -1, 10  # producer ids of the client API writer and of the job processor


class World:
    """The other writers of the partition, reacting to the log only (so a run with crashes sees the same)."""

    def __init__(self, log: Log, mid_creates=(), crash_batches=()):
        self.log = log
        self.request = 1000
        self.scan = 0
        self.jobs = []          # (job key, JOB CREATE value) in creation order
        self.pending = []       # jobs created, not completed yet
        self.mid = set(mid_creates)
        self.crash = set(crash_batches)
        self.batches = 0
        self.n = 0
        log.after_batch = self.after_batch

    def create(self, process, payload):
        wf = R.wf_record(bpmn_process_id=process, payload=payload)
        self.request += 1
        self.log.append([dict(key=-1, record_type=R.RT_COMMAND, value_type=R.VT_WORKFLOW_INSTANCE, intent=R.WI_CREATE,
                              value=wf, request_id=self.request, request_stream_id=7)], -1, CLIENT)

    def cancel(self, wik):
        self.log.append([dict(key=wik, record_type=R.RT_COMMAND, value_type=R.VT_WORKFLOW_INSTANCE,
                              intent=R.WI_CANCEL, value=b"\x80")], -1, CLIENT)

    def after_batch(self, log, evs):
        if evs[0]["producer_id"] != 70:
            return
        self.batches += 1
        if self.batches in self.mid:  # a client command arrives while the processor writes
            self.create("subs", msgpack.packb({"orderId": 5000 + self.batches}))
        if self.batches in self.crash:
            self.crash.discard(self.batches)
            raise Crash()

    def live_instances(self):
        live = {}
        for ev in self.log.events:
            if ev["value_type"] == R.VT_WORKFLOW_INSTANCE and ev["record_type"] == R.RT_EVENT:
                if ev["intent"] == R.WI_CREATED:
                    live[ev["key"]] = 1
                elif ev["intent"] in (R.WI_ELEMENT_COMPLETED, R.WI_ELEMENT_TERMINATED):
                    live.pop(ev["key"], None)
        return sorted(live)

    def job_round(self, r):
        """The job processor: JOB CREATED for every new JOB CREATE command (keys 2 + 5j), JOB COMPLETED for three
        of every four jobs created in earlier rounds and for the first new one (right behind its CREATED)."""
        new = []
        for ev in self.log.events[self.scan:]:
            if ev["value_type"] == R.VT_JOB and ev["record_type"] == R.RT_COMMAND and ev["intent"] == R.JI_CREATE:
                key = 2 + 5 * len(self.jobs)
                self.jobs.append((key, ev["value"]))
                new.append((key, ev["value"], ev["position"]))
        self.scan = len(self.log.events)
        done = [j for i, j in enumerate(self.pending) if (i + r) % 4]
        self.pending = [j for i, j in enumerate(self.pending) if not (i + r) % 4]
        for i, (key, v, pos) in enumerate(new):
            self.log.append([dict(key=key, record_type=R.RT_EVENT, value_type=R.VT_JOB, intent=R.JI_CREATED,
                                  value=R.job_event(v))], pos, JOBS)
            if i == 0:
                self._complete(key, v, r)
            else:
                self.pending.append((key, v, pos))
        for key, v, _ in done:
            self._complete(key, v, r)

    def _complete(self, key, v, r):
        pl = msgpack.packb({"round": r, "job": key, "note": "x" * (key % 37)})
        self.log.append([dict(key=key, record_type=R.RT_EVENT, value_type=R.VT_JOB, intent=R.JI_COMPLETED,
                              value=R.job_event(v, pl))], -1, JOBS)


def run_schedule(make_engine, rounds=9, snapshot_every=0, crash_rounds=(), crash_batches=(), mid_creates=(),
                 max_tick=1 << 16):
    log = Log()
    world = World(log, mid_creates, crash_batches)
    storage = SnapshotStorage()
    stats = dict(incarnations=1, reprocessed=0, ticks=[], reconciled=0, resumed=0, written=0)

    def collect(c):
        stats["ticks"] += c.sp.ticks
        stats["reprocessed"] += c.reprocessed
        for k in ("reconciled", "resumed", "written"):
            stats[k] += c.sp.stats[k]

    def make_processor(writer, has_next):
        return GpuStreamProcessor(make_engine, writer, has_next, engine_producers=(70,), max_tick=max_tick)

    def start():
        c = Controller(log, storage, make_processor, snapshot_every=snapshot_every)
        c.open()
        return c

    ctl = start()

    def settle():
        nonlocal ctl
        while True:
            try:
                ctl.run()
                return
            except Crash:
                collect(ctl)
                ctl.close()
                stats["incarnations"] += 1
                ctl = start()

    settle()
    inst = 0
    for r in range(rounds):
        for i in range(6):
            process = "process" if (inst + i) % 2 == 0 else "subs"
            world.create(process, msgpack.packb({"orderId": inst + i, "blob": "p" * ((inst + i) % 29)}))
        inst += 6
        if r % 3 == 2:
            for wik in world.live_instances()[:2]:
                world.cancel(wik)
        world.job_round(r)
        settle()
        if r in crash_rounds:  # killed between ticks (after the round's last snapshot, if any)
            collect(ctl)
            ctl.close()
            stats["incarnations"] += 1
            ctl = start()
            settle()
    collect(ctl)
    ctl.close()
    return log, stats


def check_against_oracle(log: Log, ticks):
    """Every engine tick's follow-ups in the log equal the oracle's for the same inputs."""
    o = zbref.Oracle()
    o.set_harness(False)
    for xml, k in DEPLOY:
        o.deploy(xml, k, 1)
    by_pos = {ev["position"]: ev for ev in log.events}
    outs = [ev for ev in log.events if ev["producer_id"] == 70]
    k_out = 0
    for t in ticks:
        base = o.log_size()
        omap = {}
        for i, p in enumerate(t["inputs"]):
            ev = by_pos[p]
            o.submit(ev["record_type"], ev["value_type"], ev["intent"], ev["key"], ev["value"])
            if ev["request_id"] != (1 << 64) - 1:
                o.set_request(base + i, ev["request_id"], ev["request_stream_id"])
            omap[base + i] = p
        o.run()
        n = len(t["inputs"])
        ref = R.parse_frames(o.frames(base + n, -1))
        assert len(ref) == t["outputs"], (len(ref), t["outputs"])
        for f in ref:
            g = outs[k_out]
            k_out += 1
            for fld in ("key", "record_type", "value_type", "intent", "rejection_type", "rejection_reason",
                        "request_id", "request_stream_id", "producer_id", "value", "flags"):
                assert f[fld] == g[fld], (fld, f[fld], g[fld], g["position"])
            assert omap[f["source_position"]] == g["source_position"], (f["source_position"], g["position"])
            omap[f["position"]] = g["position"]
    assert k_out == len(outs)  # every follow-up in the log belongs to exactly one tick
    return k_out


def _engine_cpu():
    from oracle_engine import OracleEngine

    return OracleEngine(DEPLOY)


def _engine_gpu():
    from zeebe_amd.engine import Engine

    e = Engine(external_jobs=True, log_capacity=1 << 16, row_capacity=1 << 12, arena_bytes=4 << 20)
    for xml, k in DEPLOY:
        e.deploy(xml, k, 1)
    return e


def _protocol(make_engine):
    ref_log, ref = run_schedule(make_engine, mid_creates=(3, 17, 40))
    n = check_against_oracle(ref_log, ref["ticks"])
    assert n > 300 and len(ref["ticks"]) >= 9 and ref["written"] == n
    # snapshots every 23 records, killed between ticks after rounds 2 and 5, and in the middle of writing the
    # follow-ups of three ticks: the same log, byte for byte
    log, st = run_schedule(make_engine, snapshot_every=23, crash_rounds=(2, 5), crash_batches=(11, 52, 90),
                           mid_creates=(3, 17, 40))
    assert st["incarnations"] == 6 and st["reprocessed"] > 0 and st["reconciled"] > 0 and st["resumed"] > 0
    assert bytes(log.buf) == bytes(ref_log.buf)
    assert st["written"] <= n  # (the batches being written when a crash hit are in the log but not counted)
    # killed with no snapshot at all: everything is reconciled from the start of the log
    log2, st2 = run_schedule(make_engine, crash_rounds=(4,), crash_batches=(30,), mid_creates=(3, 17, 40))
    assert bytes(log2.buf) == bytes(ref_log.buf) and st2["reconciled"] > 0
    # ticks capped at 4 inputs (replay must close them at the same input)
    cap_log, cap = run_schedule(make_engine, mid_creates=(3, 17, 40), max_tick=4)
    check_against_oracle(cap_log, cap["ticks"])
    log3, _ = run_schedule(make_engine, snapshot_every=17, crash_rounds=(3,), crash_batches=(25, 61),
                           mid_creates=(3, 17, 40), max_tick=4)
    assert bytes(log3.buf) == bytes(cap_log.buf)


def test_stream_processor_protocol_cpu():
    _protocol(_engine_cpu)


@pytest.mark.gpu
def test_stream_processor_protocol_gpu():
    _protocol(_engine_gpu)
