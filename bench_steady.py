"""bench.py --config c2 --steady: the partition in steady state -- the general wave pipeline over live state, the
way a broker runs it once instances wait on workers -- with the drain inside the step.

Workload (SURVEY §8d C2 shape, north_star's "job creation/completion for service tasks"): the 20-service-task chain
with external job handling (ZB_CFG_EXTERNAL_JOBS: the reference's JobInstanceStreamProcessor stays the job
processor; its JOB CREATED / COMPLETED events are the engine's input, JobCreatedProcessor / JobCompletedEventProcessor,
WorkflowInstanceStreamProcessor.java:408-453). Tick 0 creates the live population (default 1,000,000 instances, each
then waiting on its first job). Every later tick carries, as records other writers put on the log:
  * JOB CREATED + JOB COMPLETED events for a quarter of the pending jobs (rotating; the completing worker's payload
    {"t<k>": k} is merged into the instance: default output mapping);
  * new CREATE commands, as many as instances are expected to finish per tick (live / (4 x 20)), so the population
    stays near its size;
  * 1,000 CANCEL commands for waiting instances (their tasks are terminated and JOB CANCEL commands written).
One step = zb_step of the tick to quiescence + zb_serialize of every record the tick wrote (values + headers, in
HBM); the tick's input records are staged and uploaded before the timed region (zb_upload_staged), as a broker
overlaps the next tick's input with the current tick's drain. The job processor's side (turning the tick's JOB
CREATE commands into the next tick's events) runs on the host between ticks, untimed; the window is released
(zb_log_release) and the state compacted by the engine as it fills.
"""
import time

import numpy as np

from zeebe_amd import records as R

TASKS = 20
FRACTION = 4  # a quarter of the pending jobs complete per tick
CANCELS = 1000


def _mp_int(v):
    from zeebe_amd.workloads import mp_int

    return mp_int(v)


class JobWorld:
    """The other writers: the job processor (job keys 2 + 5j, KeyGenerator.createJobKeyGenerator) with its
    workers, and clients creating / cancelling instances."""

    def __init__(self, live, cancels=CANCELS):
        self.live = live
        self.cancels = cancels
        self.pending = []    # [wik, aik, task index, JOB CREATE value bytes] of every waiting instance
        self.next_job = 0
        self.tick = 0
        self.created = 0

    def harvest_oracle(self, o, start):
        """The same from the oracle's records (the sequential restatement writes the identical log)."""
        import msgpack

        for r in o.records(start):
            if r.value_type == R.VT_JOB and r.record_type == R.RT_COMMAND and r.intent == R.JI_CREATE:
                h = msgpack.unpackb(r.value, raw=False)["headers"]
                self.pending.append([h["workflowInstanceKey"], h["activityInstanceKey"], int(h["activityId"][1:]),
                                     r.value])

    def harvest(self, eng, start, count, ser=None):
        """The tick's JOB CREATE commands, from its drained records (ser: the zb_serialize of exactly that range,
        already in the engine's drain buffers)."""
        if count == 0:
            return
        from zeebe_amd.engine import HEADER_DTYPE

        d = eng.descriptors(start, count)
        if ser is None:
            ser = eng.serialize(start, count)
        hdr = np.empty(count, dtype=HEADER_DTYPE)
        vals = np.empty(max(ser["value_bytes"], 1), dtype=np.uint8)
        eng.drain_copy(vals.ctypes.data, 0, ser["value_bytes"], headers_ptr=hdr.ctypes.data)
        sel = np.nonzero((hdr["record_type"] == R.RT_COMMAND) & (hdr["value_type"] == R.VT_JOB) &
                         (hdr["intent"] == R.JI_CREATE))[0]
        raw = vals.tobytes()
        off, ln = hdr["value_offset"][sel], hdr["value_length"][sel]
        wik, aik = d["inst_key"][sel], d["scope_key"][sel]
        for k in range(len(sel)):
            v = raw[off[k]:off[k] + ln[k]]
            a = v.find(b"\xaaactivityId")  # activityId "t<k>"
            task = int(v[a + 12:a + 12 + (v[a + 11] & 31)][1:])
            self.pending.append([int(wik[k]), int(aik[k]), task, v])

    def inputs(self):
        """(CREATE payloads, zb_rec_desc records, value bytes) of the next tick."""
        from zeebe_amd.engine import DESC_DTYPE

        t = self.tick
        self.tick += 1
        done = [p for i, p in enumerate(self.pending) if (i + t) % FRACTION == 0]
        rest = [p for i, p in enumerate(self.pending) if (i + t) % FRACTION != 0]
        cancel, self.pending = rest[:self.cancels], rest[self.cancels:]
        n_create = max(1, self.live // (FRACTION * TASKS))
        pay = [b"\x81\xa7orderId" + _mp_int(self.created + i) for i in range(n_create)]
        self.created += n_create
        m = 2 * len(done) + len(cancel)
        descs = np.zeros(m, dtype=DESC_DTYPE)
        parts, pos = [], 0
        recs = []
        for wik, aik, task, v in done:
            key = 2 + 5 * self.next_job
            self.next_job += 1
            cut = v.rfind(b"\xa7payload")
            doc = b"\x81" + bytes([0xa0 + len("t%d" % task)]) + b"t%d" % task + _mp_int(task)
            completed = v[:cut] + b"\xa7payload" + b"\xc4" + bytes([len(doc)]) + doc
            recs.append((key, R.RT_EVENT, R.VT_JOB, R.JI_CREATED, v))
            recs.append((key, R.RT_EVENT, R.VT_JOB, R.JI_COMPLETED, completed))
        for wik, aik, task, v in cancel:
            recs.append((wik, R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_CANCEL, b"\x80"))
        for i, (key, rt, vt, it, v) in enumerate(recs):
            descs[i] = (key, rt, vt, it, 0, len(v), pos)
            parts.append(v)
            pos += len(v)
        return pay, descs, b"".join(parts), len(done), len(cancel), n_create


def run_steady(a, rank, world, local_rank, barrier, steps, warmup, live=1_000_000):
    from zeebe_amd import bpmn
    from zeebe_amd.engine import Engine

    recs_tick = live // FRACTION * 8 + (live // (FRACTION * TASKS)) * 12 + CANCELS * 10
    # (per tick ~290K rows and ~130 MB of documents become garbage: the partition compacts about every fifth tick.
    # Measured with 9M rows / a 5 GB arena instead: 2 compactions in 24 ticks but 2.2 ms each against 0.85 -- the
    # mark / gather passes span every allocated byte -- and 1.32 ms per tick either way)
    eng = Engine(device=0 if a.same_device else local_rank, partition_id=rank, partition_count=world,
                 log_capacity=max(live * 12, 4 * recs_tick), row_capacity=4 * live + (1 << 20),
                 arena_bytes=(live * 1200) + (256 << 20), external_jobs=True)
    eng.deploy(bpmn.chain_workflow(TASKS).to_xml(), 100, 1)
    w = JobWorld(live)
    # tick 0: the live population
    pay = [b"\x81\xa7orderId" + _mp_int(live * 4096 + rank * live + i) for i in range(live)]
    offs = np.zeros(live + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(p) for p in pay], dtype=np.uint64)
    start = eng.log_size()
    eng.create_packed("chain", b"".join(pay), offs)
    del pay
    st = eng.step()
    assert st["quiescent"], st
    w.harvest(eng, start + live, eng.log_size() - start - live)
    eng.release(eng.log_size())

    tot = dict(transitions=0, completed=0, written=0, merges=0, merge_bytes=0, cond_bytes=0, kernel_ms=0.0,
               process_ms=0.0, emit_ms=0.0, aux_ms=0.0, main_ms=0.0, launches=0, waves=0, step_s=0.0, drain_s=0.0,
               ser_write_ms=0.0, ser_size_ms=0.0, value_bytes=0, payload_bytes=0, drained=0, path=0, generic_tiles=0,
               template_drain=0, create_bytes=0, instances=live, inputs=0, completions=0, cancels=0, creates=0,
               elapsed=0.0, live_rows=0, tick_ms=[])

    def one_tick(timed):
        pay, descs, vals, n_done, n_cancel, n_create = w.inputs()
        offs = np.zeros(len(pay) + 1, dtype=np.uint64)
        offs[1:] = np.cumsum([len(p) for p in pay], dtype=np.uint64)
        start = eng.log_size()
        eng.create_packed("chain", b"".join(pay), offs)
        eng.submit_packed(descs, vals)
        eng.upload_staged()
        n_in = len(pay) + len(descs)
        barrier()
        t0 = time.perf_counter()
        st = eng.step()
        t1 = time.perf_counter()
        ser = eng.serialize(start + n_in, eng.log_size() - start - n_in)  # the records the tick wrote
        t2 = time.perf_counter()
        assert st["quiescent"], st
        if timed:
            tot["tick_ms"].append((t2 - t0) * 1e3)
            tot["elapsed"] += t2 - t0
            tot["step_s"] += t1 - t0
            tot["drain_s"] += t2 - t1
            for k, s in (("transitions", "transitions"), ("completed", "completed_instances"),
                         ("written", "records_written"), ("merges", "merges"), ("merge_bytes", "merge_bytes"),
                         ("cond_bytes", "condition_payload_bytes"), ("kernel_ms", "wave_kernel_ms"),
                         ("process_ms", "process_kernel_ms"), ("emit_ms", "emit_kernel_ms"),
                         ("aux_ms", "aux_kernel_ms"), ("launches", "launches"), ("waves", "waves")):
                tot[k] += st[s]
            tot["ser_write_ms"] += ser["write_kernel_ms"]
            tot["ser_size_ms"] += ser["size_kernel_ms"]
            tot["value_bytes"] += ser["value_bytes"]
            tot["payload_bytes"] += ser["payload_bytes"]
            tot["drained"] += ser["records"]
            tot["generic_tiles"] += ser["generic_tiles"]
            tot["inputs"] += n_in
            tot["completions"] += n_done
            tot["cancels"] += n_cancel
            tot["creates"] += n_create
        w.harvest(eng, start + n_in, eng.log_size() - start - n_in, ser)
        eng.release(eng.log_size())

    for _ in range(warmup):
        one_tick(False)
    for _ in range(steps):
        one_tick(True)
    m = eng.memory_stats()
    tot["live_rows"] = m["rows_allocated"]
    tot["compactions"] = m["compactions"]
    tot["pending_jobs"] = len(w.pending)
    tot["desc"] = ("C2 steady state: %d-service-task chain, %d live instances per GPU, external job processor; per "
                   "tick JOB CREATED + COMPLETED for 1/%d of the pending jobs (payload merges), ~%d new CREATEs and "
                   "%d CANCELs, the tick's records drained in the step" % (TASKS, live, FRACTION,
                                                                          live // (FRACTION * TASKS), CANCELS))
    eng.close()
    return tot


def cpu_baseline_steady(live, ticks):
    """The oracle (sequential C++ restatement) driven by the same schedule on a bounded sample: `live` instances,
    then `ticks` ticks of the same mix; timed from the first input of the first tick to quiescence of the last."""
    from oracle import zbref
    from zeebe_amd import bpmn

    o = zbref.Oracle()
    o.set_harness(False)
    o.deploy(bpmn.chain_workflow(TASKS).to_xml(), 100, 1)
    for i in range(live):
        o.create("chain", b"\x81\xa7orderId" + _mp_int(i))
    o.run()
    w = JobWorld(live)

    def harvest(start):
        w.harvest_oracle(o, start)

    harvest(0)
    c0 = o.counters()
    elapsed = 0.0
    for _ in range(ticks):
        pay, descs, vals, _, _, _ = w.inputs()
        start = o.log_size()
        t0 = time.perf_counter()
        for p in pay:
            o.create("chain", p)
        for d in descs:
            o.submit(int(d["record_type"]), int(d["value_type"]), int(d["intent"]), int(d["key"]),
                     vals[int(d["value_offset"]):int(d["value_offset"]) + int(d["value_length"])])
        o.run()
        elapsed += time.perf_counter() - t0
        harvest(start)
    c1 = o.counters()
    o.close()
    tr = c1["transitions"] - c0["transitions"]
    return {"value": tr / elapsed, "unit": "transitions/s", "cores": 1, "kind": "port",
            "sample": "C2 steady state, %d live instances, %d ticks of the same mix (1/%d of the pending jobs "
                      "completed per tick, creates, %d cancels) by oracle/zbref, 1 thread: %.2f s, %d transitions"
                      % (live, ticks, FRACTION, CANCELS, elapsed, tr)}
