"""The GPU core behind the reference's stream-processor plugin surface: the host-side mirror of what a maintainer
registers for a partition with ``StreamProcessorServiceFactory.Builder.processor(...)``.

The reference interfaces it follows (read as text in /root/reference):

* ``StreamProcessor`` (logstreams/.../processor/StreamProcessor.java:23-50): ``onEvent(LoggedEvent)`` returns the
  ``EventProcessor`` for a record or null (the controller then skips it, StreamProcessorController.java:339-344);
  ``getStateResource`` is the snapshot of the processor's state; ``onRecovered`` ends reprocessing.
* ``EventProcessor`` (EventProcessor.java:21-58): ``processEvent`` (state only), ``writeEvent(writer)`` returns the
  position of the last record written, 0 for none, < 0 to be called again; ``updateState``.
* ``StreamProcessorController`` (StreamProcessorController.java): recovery restores the snapshot (:156-175), takes
  ``lastSourceEventPosition`` = the largest source position among the records this processor's id wrote after the
  snapshot (:189-211), reprocesses the records up to it with ``processEvent`` + ``updateState`` only (:213-279),
  then reads, processes and writes (:296-414).
* ``LogStreamBatchWriter`` (LogStreamBatchWriter.java): one ``sourceRecordPosition`` and ``producerId`` per batch,
  ``event().key().metadataWriter().value().done()`` per record, ``tryWrite`` claims one fragment batch whose entries
  get consecutive fragment positions and returns the last (LogStreamBatchWriterImpl.java:195-268). The reference's
  ``TypedStreamWriterImpl`` writes the follow-ups of one processed record as one such batch.

How the engine maps onto it. The engine processes a *tick* of input records -- the records other writers put on the
log that the workflow processor consumes (client CREATE / CANCEL / UPDATE_PAYLOAD commands, the job processor's JOB
CREATED / COMPLETED events, the subscription API's CORRELATE commands) -- to quiescence and returns every follow-up
in reference FIFO order, each with the engine position of the record that produced it (``zb_serialize_frames``).
The processor therefore does not process its own follow-ups when it reads them back:

* live: an input's ``processEvent`` stages it; the tick closes when the reader has caught up (or ``max_tick``
  inputs are staged; records of one instance may race inside a tick, the engine serialises them). The tick's
  follow-ups are written as one batch per processed record -- source position mapped from engine to log positions,
  producer id of the processor the reference would have written it with (70 workflow, 10 job, 90 message) -- so the
  log holds the bytes the reference writes, batch flags included.
* the filter: a record the processor wrote itself in this incarnation is not processed again (its EventProcessor
  only closes a tick that has become due: the controller calls ``writeEvent`` for processed records only).
* recovery: the snapshot holds the engine's live state (``zb_snapshot``), the staged inputs and any unfinished
  reconciliation. A follow-up an earlier incarnation wrote after the snapshot is *reconciled*, not processed. Its
  tick's inputs are recovered from the log by the rule a live tick closes with: every input precedes its tick's
  first follow-up, and a live tick closes on its last input once the reader has caught up (so it holds every staged
  input before its first follow-up), or on its ``max_tick``-th. The engine steps them without writing, and each follow-up it regenerates is matched, field by field,
  against the record already in the log; the generation-1 follow-ups (source = an input) are read before the tick
  is formed. An earlier incarnation that died while writing leaves a prefix: the rest is written once the reader
  has caught up. In the broker, another writer's command claimed between the reader catching up and the tick's
  first claim would sit before the first follow-up without being part of the tick; reconciliation then reports a
  ``ReconcileError`` (the partition stops, as the controller's onFailure does) instead of writing a different log.

``engine_factory()`` returns a fresh engine with the partition's workflows deployed (the GPU ``Engine`` in the
product; the controller emulation in tests/ also drives a CPU stand-in through the same interface).
"""
from __future__ import annotations

import base64
import json
from collections import deque
from typing import Callable, Dict, List, Optional

from . import records as R

WORKFLOW_INSTANCE_PROCESSOR_ID = 70  # StreamProcessorIds.java:35
JOB_QUEUE_PROCESSOR_ID = 10          # StreamProcessorIds.java:23
MESSAGE_PROCESSOR_ID = 90            # StreamProcessorIds.java:39

# the input keys: (recordType, valueType, intent) the workflow processor consumes that other writers produce
# (WorkflowInstanceStreamProcessor.java:103-169; the other keys it registers are its own follow-ups)
INPUT_KEYS = {
    (R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_CREATE),
    (R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_CANCEL),
    (R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_UPDATE_PAYLOAD),
    (R.RT_EVENT, R.VT_JOB, R.JI_CREATED),
    (R.RT_EVENT, R.VT_JOB, R.JI_COMPLETED),
    (R.RT_COMMAND, R.VT_WIS, R.WIS_CORRELATE),
}
NULL_REQUEST_ID = (1 << 64) - 1
NULL_REQUEST_STREAM = -(1 << 31)
# the fields a re-read follow-up must carry for the engine's regenerated one to be the same record
_MATCH = ("key", "record_type", "value_type", "intent", "rejection_type", "rejection_reason", "request_id",
          "request_stream_id", "producer_id", "value")


class ReconcileError(RuntimeError):
    """A follow-up in the log differs from the one the engine regenerates on replay (the partition must stop, as
    StreamProcessorController.onFailure does for a reprocessing failure, :229-232)."""


def _key(ev: dict):
    return ev["record_type"], ev["value_type"], ev["intent"]


class _Staged:
    """EventProcessor of an input record: processEvent stages it; writeEvent closes the tick when it is due."""

    def __init__(self, sp: "GpuStreamProcessor", ev: dict):
        self.sp, self.ev = sp, ev

    def process_event(self):
        self.sp.pending.append(self.ev)

    def execute_side_effects(self) -> bool:
        return True

    def write_event(self, writer=None) -> int:
        # (the controller's writer is stamped with this record's position and the processor id,
        # StreamProcessorController.java:368-373; the follow-ups go through the processor's own batch writer, as
        # TypedStreamWriterImpl's do, with the source position and producer id of each processed record)
        return self.sp._maybe_close()

    def update_state(self):
        pass


class _Own(_Staged):
    """EventProcessor of a follow-up this incarnation wrote: nothing to process (the engine produced it)."""

    def process_event(self):
        pass


class _Reconciled(_Staged):
    """EventProcessor of a follow-up an earlier incarnation wrote: matched against the engine's regenerated one."""

    def process_event(self):
        self.sp._reconcile(self.ev)


class GpuStreamProcessor:
    def __init__(self, engine_factory: Callable[[], object], writer, has_next: Callable[[], bool],
                 engine_producers=(WORKFLOW_INSTANCE_PROCESSOR_ID,), processor_id: int = WORKFLOW_INSTANCE_PROCESSOR_ID,
                 max_tick: int = 1 << 16, frame_cfg: Optional[dict] = None):
        self.engine_factory = engine_factory
        self.writer = writer                   # a LogStreamBatchWriter on the partition's log
        self.has_next = has_next               # StreamProcessorContext.getLogStreamReader().hasNext()
        self.engine_producers = set(engine_producers)
        self.processor_id = processor_id
        self.max_tick = max_tick
        self.frame_cfg = dict(frame_cfg or {})
        self.engine = engine_factory()
        self.pending: List[dict] = []          # staged inputs (log order)
        self.expect: deque = deque()           # regenerated follow-ups not yet matched against the log
        self.run: List[dict] = []              # re-read generation-1 follow-ups whose tick is not formed yet
        self.emap: Dict[int, int] = {}         # engine position -> log position (the current tick's records)
        self.seen_upto = -1                    # engine-written records up to here are in the engine's state
        self.recovering = True                 # until the reader first catches up: no live tick is closed while
                                               # an earlier incarnation's follow-ups may still be unread
        self.ticks: List[dict] = []            # observers (tests): inputs of every engine tick, replayed or not
        self.stats = {"reconciled": 0, "resumed": 0, "written": 0}

    # ---- StreamProcessor
    def on_event(self, ev: dict):
        """The processor's filter and dispatch: null for records it does not process."""
        if ev["producer_id"] in self.engine_producers:
            if ev["position"] <= self.seen_upto:
                return _Own(self, ev)  # the engine processed it when it produced it
            return _Reconciled(self, ev)
        if _key(ev) in INPUT_KEYS:
            return _Staged(self, ev)
        return None

    def on_recovered(self):
        """End of reprocessing: a tick whose reconciliation the log leaves open is completed once caught up (in
        the broker a job submitted on the processor's actor, StreamProcessorContext.getActorControl)."""
        self._maybe_close()

    def snapshot(self) -> bytes:
        """getStateResource: the engine's live state + the staged inputs and the unfinished reconciliation."""
        b64 = lambda b: base64.b64encode(b).decode()  # noqa: E731
        fr = lambda f: {**{k: v for k, v in f.items() if not isinstance(v, bytes)},  # noqa: E731
                        "value": b64(f["value"]), "rejection_reason": b64(f["rejection_reason"])}
        return json.dumps({"engine": b64(self.engine.snapshot()), "pending": [fr(x) for x in self.pending],
                           "expect": [fr(x) for x in self.expect], "run": [fr(x) for x in self.run],
                           "emap": sorted(self.emap.items()), "seen_upto": self.seen_upto}).encode()

    def recover(self, snap: bytes):
        d = json.loads(snap)
        unb = lambda s: base64.b64decode(s)  # noqa: E731
        fr = lambda f: {**f, "value": unb(f["value"]), "rejection_reason": unb(f["rejection_reason"])}  # noqa: E731
        self.engine.restore(unb(d["engine"]))
        self.pending = [fr(x) for x in d["pending"]]
        self.expect = deque(fr(x) for x in d["expect"])
        self.run = [fr(x) for x in d["run"]]
        self.emap = {int(a): int(b) for a, b in d["emap"]}
        self.seen_upto = int(d["seen_upto"])
        self.recovering = True

    def close(self):
        self.engine.close()

    # ---- ticks
    def _step(self, inputs: List[dict]) -> List[dict]:
        """Runs the inputs through the engine as one tick (records of one instance may race in any order: zb_submit
        marks the instance and zb_step serialises its records); returns the follow-ups (frames with engine
        positions) and maps the inputs' engine positions to their log positions."""
        base = self.engine.log_size()
        n = len(inputs)
        for ev in inputs:
            self.engine.submit_records([(ev["record_type"], ev["value_type"], ev["intent"], ev["key"], ev["value"])])
            if ev["request_id"] != NULL_REQUEST_ID:
                self.engine.set_request_metadata([ev["request_id"]], [ev["request_stream_id"]])
        st = self.engine.step()
        if not st["quiescent"]:
            raise RuntimeError("engine did not reach quiescence")
        end = self.engine.log_size()
        for k, ev in enumerate(inputs):
            self.emap[base + k] = ev["position"]
        frames = R.parse_frames(self.engine.frames(base + n, end - base - n, **self.frame_cfg)) if end > base + n \
            else []
        for f in frames:  # a CORRELATE's key is its log position (positionAsKey, SubscriptionApiCommandMessageHandler
            src = f["source_position"]  # .java:146): the engine gives it, and its follow-ups, its engine position
            if f["value_type"] == R.VT_WIS and base <= src < base + n and f["key"] == src:
                f["key"] = inputs[src - base]["key"]
        self.engine.release(end)  # (the frames are on the host; the device window moves on)
        self.ticks.append({"inputs": [ev["position"] for ev in inputs], "engine_base": base, "outputs": len(frames)})
        return frames

    def _write(self, frames: List[dict]) -> int:
        """One batch per processed record (consecutive follow-ups of one source), source / producer of the batch."""
        writer = self.writer
        last = 0
        j = 0
        while j < len(frames):
            src = frames[j]["source_position"]
            k = j
            while k < len(frames) and frames[k]["source_position"] == src:
                k += 1
            batch = frames[j:k]
            producers = {f["producer_id"] for f in batch}
            assert len(producers) == 1, producers
            writer.reset()
            writer.source_record_position(self.emap[src] if src >= 0 else -1).producer_id(producers.pop())
            for f in batch:
                writer.event(f)
            positions = writer.try_write()
            for f, p in zip(batch, positions):
                self.emap[f["position"]] = p
            last = positions[-1]
            self.seen_upto = last
            self.stats["written"] += len(batch)
            j = k
        return last

    def _maybe_close(self) -> int:
        caught_up = not self.has_next()
        while self.run and caught_up and not self.expect:  # the log ends inside generation 1 of a tick an
            self._form_tick()                                # earlier incarnation wrote
        pos = 0
        if self.expect:
            if not caught_up:
                return 0
            rest = list(self.expect)  # an earlier incarnation died while writing this tick: write the rest
            self.expect.clear()
            self.stats["resumed"] += len(rest)
            pos = self._write(rest)
            self.emap.clear()
            caught_up = not self.has_next()
        if caught_up:
            self.recovering = False
        if not self.recovering and self.pending and (caught_up or len(self.pending) >= self.max_tick):
            inputs, self.pending = self.pending, []
            frames = self._step(inputs)
            pos = self._write(frames) or pos
            self.emap.clear()
        return pos

    # ---- reconciliation of follow-ups an earlier incarnation wrote
    def _reconcile(self, ev: dict):
        if not self.expect:
            staged = {x["position"] for x in self.pending}
            if ev["source_position"] in staged:
                self.run.append(ev)  # generation 1 of a tick: its inputs are not known yet
                return
            if not self.run:
                raise ReconcileError("follow-up at %d: its tick's inputs are not in the log after the snapshot"
                                     % ev["position"])
            self._form_tick()
            while self.run and not self.expect:
                self._form_tick()
        self._match(ev)

    def _form_tick(self):
        """The tick whose generation-1 follow-ups are in run: every staged input before its first follow-up, at most
        max_tick -- exactly the inputs a live tick closes with (on its last input once the reader has caught up, or
        on its max_tick-th). (Inputs with no follow-up of their own, such as a JOB CREATED, are among them: moving
        one into another tick could change the order in which the tick's racing records are serialised.)"""
        first = self.run[0]["position"]
        k = min(sum(1 for x in self.pending if x["position"] < first), self.max_tick)
        if k == 0:
            raise ReconcileError("follow-up at %d: its tick's inputs are not in the log after the snapshot" % first)
        inputs, self.pending = self.pending[:k], self.pending[k:]
        self.expect = deque(self._step(inputs))
        run, self.run = self.run, []
        for i, r in enumerate(run):
            if not self.expect:  # (the tick wrote generation 1 only: the rest of the run is the next tick's)
                self.run = run[i:]
                return
            self._match(r)

    def _match(self, ev: dict):
        if not self.expect:
            raise ReconcileError("follow-up at %d has no counterpart in the replayed tick" % ev["position"])
        f = self.expect.popleft()
        diff = {k: (f[k], ev[k]) for k in _MATCH if f[k] != ev[k]}
        src = f["source_position"]
        mapped = self.emap.get(src, -1) if src >= 0 else -1
        if mapped != ev["source_position"]:
            diff["source_position"] = (mapped, ev["source_position"])
        if diff:
            raise ReconcileError("follow-up at %d differs from the replayed one: %s" % (ev["position"], diff))
        self.emap[f["position"]] = ev["position"]
        self.seen_upto = max(self.seen_upto, ev["position"])
        self.stats["reconciled"] += 1
        if not self.expect:
            self.emap.clear()
