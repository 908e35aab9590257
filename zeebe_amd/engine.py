"""Python binding of libzbgpu.so (ctypes over the C ABI in include/zb_engine.h).

The product path: every call goes to the HIP engine. If the shared library is missing this module
raises at import time -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import struct
from typing import List, NamedTuple, Optional, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libzbgpu.so")
# ZB_CHECKED_LIBRARY=1 (tests only): the guard-band build of the same sources (zeebe_amd/csrc/zb_checked.hpp), which
# reports every out-of-bounds device write per kernel launch -- a test instrument, never the product library
if os.environ.get("ZB_CHECKED_LIBRARY") == "1":
    LIB_PATH = os.path.join(_HERE, "libzbgpu_checked.so")
# ZB_PHASES_LIBRARY=1 (measurement only): the phase-timing build (-DZB_PHASES): k_wave's time per phase of its tiles
if os.environ.get("ZB_PHASES_LIBRARY") == "1":
    LIB_PATH = os.path.join(_HERE, "libzbgpu_phases.so")

CFG_WAVE_ONLY = 1  # zb_config.flags: never take the trajectory path
CFG_EXTERNAL_JOBS = 2  # zb_config.flags: no canonical job harness (job events come through zb_submit)
CFG_JOB_PROCESSOR = 4  # zb_config.flags: the job stream processor runs on the GPU (job commands through zb_submit)
# diagnostic / measurement flags (include/zb_engine.h; the defaults are the product configuration)
CFG_VLEN_CHECK = 8  # the drain's size pass checks every value-length hint against the encoder
CFG_GENERIC_DRAIN = 16  # every drain tile through the generic encoder (the reference pass of the fast ones)
CFG_NO_DEFER = 32  # trajectory batches write their descriptors in zb_step (no template drain)
CFG_INSTANCE_ORDER = 64  # class batches emitted in instance order even when not deferred
CFG_WAVE_EVENTS = 128  # timing events around every wave's kernels
CFG_WAVE_SPLIT = 256  # three-kernel wave pipeline instead of the fused k_wave
CFG_SINGLE_PASS_DRAIN = 512  # one-pass (look-back) value drain
CFG_RCCL_SELF = 1024  # a one-partition engine exchanges through RCCL anyway (tests of the P > 1 path on one GPU)
CFG_SHARED_GPU = 2048  # the GPU is shared with other processes' engines: the wave kernel claims its tiles

ZB_OK, ZB_EINVAL, ZB_ENOMEM, ZB_EUNSUPPORTED, ZB_EDEPLOY, ZB_EDEVICE, ZB_EAGAIN, ZB_EPROCESSING = \
    0, -1, -2, -3, -4, -5, -6, -7
_NAMES = {0: "ZB_OK", -1: "ZB_EINVAL", -2: "ZB_ENOMEM", -3: "ZB_EUNSUPPORTED", -4: "ZB_EDEPLOY",
          -5: "ZB_EDEVICE", -6: "ZB_EAGAIN", -7: "ZB_EPROCESSING"}


class ZbError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__("%s: %s" % (_NAMES.get(code, code), msg))
        self.code = code


class zb_config(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("partition_id", ctypes.c_int32),
                ("partition_count", ctypes.c_int32), ("flags", ctypes.c_int32),
                ("log_capacity", ctypes.c_uint64), ("row_capacity", ctypes.c_uint64),
                ("arena_bytes", ctypes.c_uint64), ("wave_records", ctypes.c_uint64)]


class zb_rec(ctypes.Structure):
    _fields_ = [("key", ctypes.c_int64), ("scope_key", ctypes.c_int64), ("inst_key", ctypes.c_int64),
                ("payload", ctypes.c_uint32), ("elem", ctypes.c_uint16), ("intent", ctypes.c_uint8),
                ("kind", ctypes.c_uint8)]


class zb_rec_desc(ctypes.Structure):
    _fields_ = [("key", ctypes.c_int64), ("record_type", ctypes.c_uint8), ("value_type", ctypes.c_uint8),
                ("intent", ctypes.c_uint8), ("pad", ctypes.c_uint8), ("value_length", ctypes.c_uint32),
                ("value_offset", ctypes.c_uint64)]


class zb_record_header(ctypes.Structure):  # header i of a drained batch: the record at position start + i
    _fields_ = [("key", ctypes.c_int64), ("record_type", ctypes.c_uint8), ("value_type", ctypes.c_uint8),
                ("intent", ctypes.c_uint8), ("rejection_type", ctypes.c_uint8), ("value_length", ctypes.c_uint32),
                ("value_offset", ctypes.c_uint64)]


class zb_step_stats(ctypes.Structure):
    _fields_ = [("waves", ctypes.c_uint64), ("launches", ctypes.c_uint64),
                ("records_processed", ctypes.c_uint64), ("records_written", ctypes.c_uint64),
                ("transitions", ctypes.c_uint64), ("completed_instances", ctypes.c_uint64),
                ("merges", ctypes.c_uint64), ("merge_bytes", ctypes.c_uint64),
                ("condition_payload_bytes", ctypes.c_uint64), ("wave_kernel_ms", ctypes.c_double),
                ("wall_ms", ctypes.c_double), ("process_kernel_ms", ctypes.c_double),
                ("emit_kernel_ms", ctypes.c_double), ("aux_kernel_ms", ctypes.c_double),
                ("path", ctypes.c_uint64), ("main_emit_kernel_ms", ctypes.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class zb_frame_config(ctypes.Structure):
    _fields_ = [("stream_id", ctypes.c_int32), ("raft_term", ctypes.c_int32), ("timestamp", ctypes.c_int64)]


class zb_serialize_stats(ctypes.Structure):
    _fields_ = [("records", ctypes.c_uint64), ("value_bytes", ctypes.c_uint64), ("payload_bytes", ctypes.c_uint64),
                ("size_kernel_ms", ctypes.c_double), ("scan_ms", ctypes.c_double),
                ("write_kernel_ms", ctypes.c_double), ("wall_ms", ctypes.c_double),
                ("generic_tiles", ctypes.c_uint64), ("template_drain", ctypes.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class zb_memory_stats(ctypes.Structure):
    _fields_ = [("log_window_begin", ctypes.c_int64), ("log_end", ctypes.c_int64), ("log_capacity", ctypes.c_uint64),
                ("rows_allocated", ctypes.c_uint64), ("row_capacity", ctypes.c_uint64),
                ("arena_used", ctypes.c_uint64), ("arena_bytes", ctypes.c_uint64),
                ("records_total", ctypes.c_uint64), ("rows_total", ctypes.c_uint64), ("arena_total", ctypes.c_uint64),
                ("compactions", ctypes.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class Record(NamedTuple):
    position: int
    source_position: int
    key: int
    record_type: int
    value_type: int
    intent: int
    rejection_type: int
    value: bytes


_INST = struct.Struct("<qqqB3xI")  # zb_read_instances record header
# zb_rec_desc / zb_record_header as numpy records (submit_packed, bulk drains)
DESC_DTYPE = [("key", "<i8"), ("record_type", "u1"), ("value_type", "u1"), ("intent", "u1"), ("pad", "u1"),
              ("value_length", "<u4"), ("value_offset", "<u8")]
HEADER_DTYPE = [("key", "<i8"), ("record_type", "u1"), ("value_type", "u1"), ("intent", "u1"),
                ("rejection_type", "u1"), ("value_length", "<u4"), ("value_offset", "<u8")]

_lib = None


class _Absent:
    def __init__(self, name):
        self.name, self.argtypes, self.restype = name, None, None

    def __call__(self, *a):
        raise RuntimeError("%s is not in this library" % self.name)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("libzbgpu.so not built (%s): run __graft_entry__.build()" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        if os.environ.get("ZB_AB_LIBRARY") == "1":
            # (same-box A/B of an earlier round's library, tools/gpu/wave_ab.sh: the entry points it lacks fail when
            # called instead of when the binding is set up; the product library exports every one, test_abi.py)
            for name in EXPORTED_SYMBOLS:
                if not hasattr(L, name):
                    setattr(L, name, _Absent(name))
        vp = ctypes.c_void_p
        L.zb_engine_create.argtypes = [ctypes.POINTER(zb_config), ctypes.POINTER(vp)]
        L.zb_engine_destroy.argtypes = [vp]
        L.zb_last_error.restype = ctypes.c_char_p
        L.zb_last_error.argtypes = [vp]
        L.zb_reset.argtypes = [vp, ctypes.c_int]
        L.zb_deploy.argtypes = [vp, ctypes.c_int64, ctypes.c_int32, ctypes.c_char_p, ctypes.c_size_t]
        L.zb_set_job_completion_payload.argtypes = [vp, ctypes.c_int64, ctypes.c_char_p, ctypes.c_char_p,
                                                    ctypes.c_size_t]
        L.zb_submit_creates.argtypes = [vp, ctypes.c_char_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t,
                                        ctypes.c_void_p, ctypes.c_void_p]
        L.zb_step.argtypes = [vp, ctypes.c_uint32, ctypes.POINTER(zb_step_stats)]
        L.zb_upload_staged.argtypes = [vp]
        L.zb_log_size.restype = ctypes.c_int64
        L.zb_log_size.argtypes = [vp]
        L.zb_read_descriptors.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p]
        L.zb_read_source_positions.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p]
        L.zb_drain.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
        L.zb_counters.argtypes = [vp, ctypes.POINTER(ctypes.c_int64)]
        u64p = ctypes.POINTER(ctypes.c_uint64)
        L.zb_submit_publishes.argtypes = [vp, ctypes.c_char_p, ctypes.c_int64, ctypes.c_size_t, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.zb_upload_publishes.argtypes = [vp, ctypes.c_char_p, ctypes.c_int64, ctypes.c_size_t, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.zb_publish_uploaded.argtypes = [vp]
        L.zb_inbox_submit.argtypes = [vp, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        L.zb_outbox_count.argtypes = [vp, ctypes.c_int, u64p]
        L.zb_outbox_take.argtypes = [vp, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, u64p, u64p, u64p]
        L.zb_submit_messages.argtypes = [vp, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
        L.zb_set_clock.argtypes = [vp, ctypes.c_int64]
        L.zb_expire_messages.argtypes = [vp, ctypes.c_int64, u64p]
        L.zb_comm_unique_id.argtypes = [ctypes.c_char_p]
        L.zb_comm_init.argtypes = [vp, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
        L.zb_comm_pending.argtypes = [vp, u64p]
        L.zb_comm_exchange.argtypes = [vp, ctypes.c_int, u64p]
        szp = ctypes.POINTER(ctypes.c_size_t)
        L.zb_submit.argtypes = [vp, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
        L.zb_validate_deployment.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
        L.zb_serialize.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(zb_serialize_stats)]
        L.zb_drain_copy.argtypes = [vp, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_size_t]
        L.zb_serialize_frames.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(zb_frame_config),
                                          ctypes.POINTER(zb_serialize_stats)]
        L.zb_set_request_metadata.argtypes = [vp, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
        L.zb_rccl_library.restype = ctypes.c_char_p
        L.zb_rccl_library.argtypes = []
        L.zb_pinned_alloc.restype = ctypes.c_void_p
        L.zb_pinned_alloc.argtypes = [ctypes.c_size_t]
        L.zb_pinned_free.argtypes = [ctypes.c_void_p]
        L.zb_read_instances.argtypes = [vp, ctypes.c_void_p, ctypes.c_size_t, szp, u64p]
        L.zb_snapshot.argtypes = [vp, ctypes.c_void_p, ctypes.c_size_t, szp]
        L.zb_log_release.argtypes = [vp, ctypes.c_int64]
        L.zb_log_start.argtypes = [vp, ctypes.c_int64]
        L.zb_compact.argtypes = [vp]
        L.zb_read_memory_stats.argtypes = [vp, ctypes.POINTER(zb_memory_stats)]
        L.zb_restore.argtypes = [vp, ctypes.c_void_p, ctypes.c_size_t]
        if hasattr(L, "zb_checked_violations"):  # (the guard-band build only)
            L.zb_checked_violations.restype = ctypes.c_ulonglong
            L.zb_checked_violations.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
        _lib = L
    return _lib


EXPORTED_SYMBOLS = ["zb_engine_create", "zb_engine_destroy", "zb_last_error", "zb_reset", "zb_deploy",
                    "zb_set_job_completion_payload", "zb_submit_creates", "zb_step", "zb_log_size",
                    "zb_read_descriptors", "zb_drain", "zb_counters", "zb_submit_publishes", "zb_upload_publishes",
                    "zb_publish_uploaded", "zb_inbox_submit",
                    "zb_outbox_count", "zb_outbox_take", "zb_comm_unique_id", "zb_comm_init", "zb_comm_pending",
                    "zb_comm_exchange", "zb_submit", "zb_read_instances", "zb_snapshot", "zb_restore",
                    "zb_validate_deployment", "zb_serialize", "zb_drain_copy", "zb_pinned_alloc", "zb_pinned_free",
                    "zb_serialize_frames", "zb_set_request_metadata", "zb_read_source_positions",
                    "zb_log_release", "zb_log_start", "zb_compact", "zb_read_memory_stats", "zb_submit_messages", "zb_set_clock",
                    "zb_expire_messages", "zb_rccl_library", "zb_upload_staged"]


def checked_violations():
    """(violations, launches checked) of the guard-band build, or None for the product library."""
    L = lib()
    if not hasattr(L, "zb_checked_violations"):
        return None
    n = ctypes.c_ulonglong(0)
    v = L.zb_checked_violations(ctypes.byref(n))
    return int(v), int(n.value)


def validate_deployment(xml):
    """Host-only: (status, message) of transforming a deployment resource as zb_deploy would."""
    if isinstance(xml, str):
        xml = xml.encode()
    err = ctypes.create_string_buffer(4096)
    rc = lib().zb_validate_deployment(xml, len(xml), err, 4096)
    return rc, err.value.decode("utf-8", "replace")


class Engine:
    """One partition of the GPU stepping core (one HIP device + stream)."""

    def __init__(self, device: int = 0, partition_id: int = 0, partition_count: int = 1,
                 log_capacity: int = 1 << 22, row_capacity: int = 1 << 20, arena_bytes: int = 64 << 20,
                 wave_records: int = 0, wave_only: bool = False, external_jobs: bool = False,
                 job_processor: bool = False, flags: int = 0):
        """flags: further zb_config.flags bits (the CFG_* diagnostic / measurement flags above)."""
        self._L = lib()
        flags = int(flags) | (CFG_WAVE_ONLY if wave_only else 0) | (CFG_EXTERNAL_JOBS if external_jobs else 0) | \
            (CFG_JOB_PROCESSOR if job_processor else 0)
        external_jobs = external_jobs or job_processor
        cfg = zb_config(device, partition_id, partition_count, flags, log_capacity, row_capacity, arena_bytes,
                        wave_records)
        h = ctypes.c_void_p()
        self._device, self._parts = device, partition_count
        self._external = external_jobs
        self._flags = flags
        rc = self._L.zb_engine_create(ctypes.byref(cfg), ctypes.byref(h))
        if rc != ZB_OK:
            raise ZbError(rc, "zb_engine_create failed")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._L.zb_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int):
        if rc != ZB_OK:
            raise ZbError(rc, self._L.zb_last_error(self._h).decode("utf-8", "replace"))
        return rc

    def reset(self, keep_staged: bool = False):
        self._check(self._L.zb_reset(self._h, 1 if keep_staged else 0))

    def deploy(self, xml, workflow_key: int, version: int = 1):
        if isinstance(xml, str):
            xml = xml.encode()
        self._check(self._L.zb_deploy(self._h, workflow_key, version, xml, len(xml)))

    def set_job_payload(self, workflow_key: int, activity_id: str, payload: bytes):
        self._check(self._L.zb_set_job_completion_payload(self._h, workflow_key, activity_id.encode(), payload,
                                                          len(payload)))

    def create(self, process_id: str, payloads: Sequence[bytes], version: int = -1, workflow_key: int = -1):
        import numpy as np

        n = len(payloads)
        offs = np.zeros(n + 1, dtype=np.uint64)
        if n:
            offs[1:] = np.cumsum([len(p) for p in payloads], dtype=np.uint64)
        blob = b"".join(payloads)
        buf = ctypes.create_string_buffer(blob, max(len(blob), 1))
        self._check(self._L.zb_submit_creates(self._h, process_id.encode(), version, workflow_key, n, buf,
                                              offs.ctypes.data))

    def create_packed(self, process_id: str, blob: bytes, offsets, version: int = -1, workflow_key: int = -1):
        """Bulk form: offsets is a uint64 numpy array of n+1 entries into blob."""
        buf = ctypes.create_string_buffer(blob, max(len(blob), 1))
        n = len(offsets) - 1
        self._check(self._L.zb_submit_creates(self._h, process_id.encode(), version, workflow_key, n, buf,
                                              offsets.ctypes.data))

    def submit_records(self, recs):
        """zb_submit: recs = [(record_type, value_type, intent, key, value bytes), ...] in log order."""
        n = len(recs)
        arr = (zb_rec_desc * max(n, 1))()
        blob = bytearray()
        for i, (rt, vt, it, key, value) in enumerate(recs):
            arr[i] = zb_rec_desc(key, rt, vt, it, 0, len(value), len(blob))
            blob += value
        buf = ctypes.create_string_buffer(bytes(blob), max(len(blob), 1))
        self._check(self._L.zb_submit(self._h, arr, n, buf, len(blob)))

    def submit_packed(self, descs, values: bytes):
        """zb_submit over prepared arrays: descs a numpy array of zb_rec_desc records (DESC_DTYPE), values the
        concatenated value bytes they index."""
        import numpy as np

        descs = np.ascontiguousarray(descs, dtype=DESC_DTYPE)
        buf = ctypes.create_string_buffer(bytes(values), max(len(values), 1))
        self._check(self._L.zb_submit(self._h, descs.ctypes.data, len(descs), buf, len(values)))

    def upload_staged(self):
        """zb_upload_staged: the staged input batch to the device now (not inside the next zb_step)."""
        self._check(self._L.zb_upload_staged(self._h))

    def set_job_processor(self, on: bool):
        """The job stream processor is fixed at creation (job_processor=...): only checks it matches."""
        if bool(on) != bool(self._flags & CFG_JOB_PROCESSOR):
            raise ValueError("the job stream processor is chosen at engine creation (job_processor)")

    def set_harness(self, on: bool):
        """The job harness is fixed at creation (external_jobs=...): only checks it matches."""
        if bool(on) == self._external:
            raise ValueError("the canonical job harness is chosen at engine creation (external_jobs)")

    def submit(self, record_type: int, value_type: int, intent: int, key: int, value: bytes):
        """One record (the oracle's submit signature)."""
        self.submit_records([(record_type, value_type, intent, key, value)])

    def instances(self):
        """Live element instances sorted by key: [(key, parent_key, job_key, state, value bytes)]."""
        need = ctypes.c_size_t(0)
        cnt = ctypes.c_uint64(0)
        rc = self._L.zb_read_instances(self._h, None, 0, ctypes.byref(need), ctypes.byref(cnt))
        if rc not in (ZB_OK, ZB_ENOMEM):
            self._check(rc)
        if need.value == 0:
            return []
        buf = ctypes.create_string_buffer(need.value)
        self._check(self._L.zb_read_instances(self._h, buf, need.value, ctypes.byref(need), ctypes.byref(cnt)))
        raw, out, off = buf.raw, [], 0
        while off < len(raw):
            key, pk, jk, st, n = _INST.unpack_from(raw, off)
            off += _INST.size
            out.append((key, pk, jk, st, raw[off:off + n]))
            off += n
        return out

    def snapshot(self) -> bytes:
        need = ctypes.c_size_t(0)
        rc = self._L.zb_snapshot(self._h, None, 0, ctypes.byref(need))
        if rc not in (ZB_OK, ZB_ENOMEM):
            self._check(rc)
        buf = ctypes.create_string_buffer(max(need.value, 1))
        self._check(self._L.zb_snapshot(self._h, buf, need.value, ctypes.byref(need)))
        return buf.raw[:need.value]

    def restore(self, snap: bytes):
        buf = ctypes.create_string_buffer(snap, max(len(snap), 1))
        self._check(self._L.zb_restore(self._h, buf, len(snap)))

    def step(self, max_waves: int = 0) -> dict:
        st = zb_step_stats()
        rc = self._L.zb_step(self._h, max_waves, ctypes.byref(st))
        if rc not in (ZB_OK, ZB_EAGAIN):
            self._check(rc)
        d = st.as_dict()
        d["quiescent"] = rc == ZB_OK
        return d

    def serialize(self, start: int, count: int) -> dict:
        """zb_serialize: records [start, start+count) -> the engine's device-resident drain buffers."""
        st = zb_serialize_stats()
        self._check(self._L.zb_serialize(self._h, start, count, ctypes.byref(st)))
        return st.as_dict()

    def serialize_frames(self, start: int, count: int, stream_id: int = 0, raft_term: int = 0,
                         timestamp: int = 0) -> dict:
        """zb_serialize_frames: records [start, start+count) -> log frames in the device-resident drain buffer."""
        fc = zb_frame_config(stream_id, raft_term, timestamp)
        st = zb_serialize_stats()
        self._check(self._L.zb_serialize_frames(self._h, start, count, ctypes.byref(fc), ctypes.byref(st)))
        return st.as_dict()

    def frames(self, start: int = 0, count: Optional[int] = None, stream_id: int = 0, raft_term: int = 0,
               timestamp: int = 0) -> bytes:
        """The log frames of records [start, start+count), copied to host memory."""
        if count is None:
            count = self.log_size() - start
        st = self.serialize_frames(start, count, stream_id, raft_term, timestamp)
        n = st["value_bytes"]
        buf = ctypes.create_string_buffer(max(n, 1))
        if n:
            self._check(self._L.zb_drain_copy(self._h, None, buf, 0, n))
        return buf.raw[:n]

    def set_request_metadata(self, request_ids, request_stream_ids):
        """Request metadata of the last len(request_ids) staged records (zb_set_request_metadata)."""
        n = len(request_ids)
        ids = (ctypes.c_uint64 * max(n, 1))(*request_ids)
        sids = (ctypes.c_int32 * max(n, 1))(*request_stream_ids)
        self._check(self._L.zb_set_request_metadata(self._h, n, ids, sids))

    def set_request_metadata_np(self, request_ids, request_stream_ids):
        """set_request_metadata from numpy arrays (uint64 / int32), without per-element conversion."""
        import numpy as np

        ids = np.ascontiguousarray(request_ids, dtype=np.uint64)
        sids = np.ascontiguousarray(request_stream_ids, dtype=np.int32)
        assert len(ids) == len(sids)
        self._check(self._L.zb_set_request_metadata(self._h, len(ids), ids.ctypes.data, sids.ctypes.data))

    def drain_copy(self, dst_ptr: int, value_off: int, nbytes: int, headers_ptr=None):
        """zb_drain_copy into caller memory (an address, e.g. from pinned_alloc)."""
        self._check(self._L.zb_drain_copy(self._h, headers_ptr, dst_ptr, value_off, nbytes))

    def log_size(self) -> int:
        return self._L.zb_log_size(self._h)

    def release(self, position: int):
        """zb_log_release: records below position were appended by the caller; they leave the device window."""
        self._check(self._L.zb_log_release(self._h, position))

    def log_start(self, position: int):
        """zb_log_start: the (idle, fully released) partition's log continues at position."""
        self._check(self._L.zb_log_start(self._h, position))

    def compact(self):
        """zb_compact: drop dead element-instance rows, unreachable payload blobs, removed messages / job states."""
        self._check(self._L.zb_compact(self._h))

    def phase_times(self):
        """(measurement build ZB_PHASES_LIBRARY=1 only) k_wave's wall-clock ticks (10 ns) per phase, summed over its
        workgroups: process + tile scan, look-back, emit, and the tiles processed."""
        out = (ctypes.c_ulonglong * 5)()
        self._L.zb_phase_times.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        self._check(self._L.zb_phase_times(self._h, out))
        return dict(process=out[0], lookback=out[1], emit=out[2], tiles=out[3], rounds=out[4])

    def tdrain_phase_times(self):
        """(measurement build ZB_PHASES_LIBRARY=1 only) k_tdrain_write's wall-clock ticks (10 ns) per phase, summed over
        its waves: generation setup, headers, encode, image stream; and the waves and generations counted."""
        out = (ctypes.c_ulonglong * 6)()
        self._L.zb_tdrain_phase_times.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        self._check(self._L.zb_tdrain_phase_times(self._h, out))
        return dict(setup=out[0], headers=out[1], encode=out[2], stream=out[3], waves=out[4], gens=out[5])

    def memory_stats(self) -> dict:
        m = zb_memory_stats()
        self._check(self._L.zb_read_memory_stats(self._h, ctypes.byref(m)))
        return m.as_dict()

    def descriptors(self, start: int = 0, count: Optional[int] = None):
        import numpy as np

        if count is None:
            count = self.log_size() - start
        arr = (zb_rec * max(count, 1))()
        self._check(self._L.zb_read_descriptors(self._h, start, count, arr))
        dt = np.dtype([("key", "<i8"), ("scope_key", "<i8"), ("inst_key", "<i8"), ("payload", "<u4"),
                       ("elem", "<u2"), ("intent", "u1"), ("kind", "u1")])
        return np.frombuffer(bytes(arr)[:count * 32], dtype=dt)

    def records(self, start: int = 0, count: Optional[int] = None) -> List[Record]:
        if count is None:
            count = self.log_size() - start
        if count <= 0:
            return []
        hdrs = (zb_record_header * count)()
        need = ctypes.c_size_t(0)
        rc = self._L.zb_drain(self._h, start, count, hdrs, None, 0, ctypes.byref(need))
        if rc not in (ZB_OK, ZB_ENOMEM):
            self._check(rc)
        buf = ctypes.create_string_buffer(max(need.value, 1))
        self._check(self._L.zb_drain(self._h, start, count, hdrs, buf, need.value, ctypes.byref(need)))
        raw = buf.raw
        src = (ctypes.c_int64 * count)()
        self._check(self._L.zb_read_source_positions(self._h, start, count, src))
        out = []
        for i, h in enumerate(hdrs):
            v = raw[h.value_offset:h.value_offset + h.value_length]
            out.append(Record(start + i, src[i], h.key, h.record_type, h.value_type, h.intent, h.rejection_type, v))
        return out

    # ---- partition interface of zeebe_amd.cluster (message correlation, config 5)
    def run(self) -> dict:
        """Step to quiescence (StreamProcessorController loop until no unprocessed record is left)."""
        st = self.step()
        assert st["quiescent"]
        return st

    def pending(self, kind: int) -> int:
        n = ctypes.c_uint64(0)
        self._check(self._L.zb_outbox_count(self._h, kind, ctypes.byref(n)))
        return n.value

    def outbox(self, kind: int):
        """All pending commands of a kind, sorted by (target, source position, emission), as exchange batches (one
        per target partition with commands, back to back; include/zb_engine.h) in a host uint8 array + the byte
        size of each target's batch. (Between GPUs the engines exchange device-resident outboxes over RCCL
        themselves: comm_exchange().)"""
        import numpy as np

        sizes = (ctypes.c_uint64 * max(self._parts, 1))()
        got, total = ctypes.c_uint64(0), ctypes.c_uint64(0)
        rc = self._L.zb_outbox_take(self._h, kind, None, 0, 0, sizes, ctypes.byref(got), ctypes.byref(total))
        if rc not in (ZB_OK, ZB_ENOMEM):
            self._check(rc)
        if got.value == 0:
            return np.zeros(0, dtype=np.uint8), [0] * self._parts
        buf = np.zeros(total.value, dtype=np.uint8)
        self._check(self._L.zb_outbox_take(self._h, kind, buf.ctypes.data, total.value, 0, sizes, ctypes.byref(got),
                                           ctypes.byref(total)))
        return buf, [int(sizes[q]) for q in range(self._parts)]

    def inbox(self, kind: int, buf):
        """Exchange batches delivered by other partitions (host uint8 array, delivery order)."""
        import numpy as np

        a = np.ascontiguousarray(np.asarray(buf, dtype=np.uint8))
        if len(a):
            self._check(self._L.zb_inbox_submit(self._h, kind, a.ctypes.data, len(a), 0))

    # ---- RCCL exchange between engines of different processes (one partition per GPU)
    @staticmethod
    def comm_unique_id() -> bytes:
        buf = ctypes.create_string_buffer(128)
        rc = lib().zb_comm_unique_id(buf)
        if rc != ZB_OK:
            raise ZbError(rc, "zb_comm_unique_id failed")
        return buf.raw

    def comm_init(self, unique_id: bytes, nranks: int, rank: int):
        self._check(self._L.zb_comm_init(self._h, unique_id, nranks, rank))

    def needs_communicator(self) -> bool:
        """A single partition delivers its outbox to its own inbox on the device: no RCCL communicator (unless
        CFG_RCCL_SELF asks for the collective path anyway)."""
        return self._parts > 1 or bool(self._flags & CFG_RCCL_SELF)

    def comm_pending(self):
        g = (ctypes.c_uint64 * 2)()
        self._check(self._L.zb_comm_pending(self._h, g))
        return int(g[0]), int(g[1])

    def comm_exchange(self, kind: int) -> int:
        n = ctypes.c_uint64(0)
        self._check(self._L.zb_comm_exchange(self._h, kind, ctypes.byref(n)))
        return n.value

    def publish(self, name: bytes, correlation_keys, payloads, ttl: int = 3600000):
        """MESSAGE PUBLISH commands, one message name and time-to-live for the batch."""
        import numpy as np

        if isinstance(name, str):
            name = name.encode()
        n = len(correlation_keys)
        ck_off = np.zeros(n + 1, dtype=np.uint64)
        pl_off = np.zeros(n + 1, dtype=np.uint64)
        if n:
            ck_off[1:] = np.cumsum([len(c) for c in correlation_keys])
            pl_off[1:] = np.cumsum([len(p) for p in payloads])
        self.publish_packed(name, b"".join(correlation_keys), ck_off, b"".join(payloads), pl_off, ttl)

    def publish_packed(self, name: bytes, ck_blob: bytes, ck_off, pl_blob: bytes, pl_off, ttl: int = 3600000):
        """publish() with the batch already packed: message i has correlation key ck_blob[ck_off[i]:ck_off[i+1]]
        and payload pl_blob[pl_off[i]:pl_off[i+1]] (offsets: n + 1 uint64, numpy)."""
        import numpy as np

        if isinstance(name, str):
            name = name.encode()
        ck_off = np.ascontiguousarray(ck_off, dtype=np.uint64)
        pl_off = np.ascontiguousarray(pl_off, dtype=np.uint64)
        n = len(ck_off) - 1
        self._check(self._L.zb_submit_publishes(self._h, name, ttl, n, ck_blob, ck_off.ctypes.data, pl_blob,
                                                pl_off.ctypes.data))

    def upload_publishes_packed(self, name: bytes, ck_blob: bytes, ck_off, pl_blob: bytes, pl_off,
                                ttl: int = 3600000):
        """zb_upload_publishes: publish_packed's batch to HBM now, processed by publish_uploaded()."""
        import numpy as np

        if isinstance(name, str):
            name = name.encode()
        ck_off = np.ascontiguousarray(ck_off, dtype=np.uint64)
        pl_off = np.ascontiguousarray(pl_off, dtype=np.uint64)
        n = len(ck_off) - 1
        self._check(self._L.zb_upload_publishes(self._h, name, ttl, n, ck_blob, ck_off.ctypes.data, pl_blob,
                                                pl_off.ctypes.data))

    def publish_uploaded(self):
        """zb_publish_uploaded: the uploaded PUBLISH batch's commands, processed."""
        self._check(self._L.zb_publish_uploaded(self._h))

    def submit_messages(self, recs):
        """zb_submit_messages: recs = [(intent, key, MessageRecord value bytes), ...] (MESSAGE commands: PUBLISH 0,
        DELETE 2), appended and processed at once."""
        n = len(recs)
        arr = (zb_rec_desc * max(n, 1))()
        blob = bytearray()
        for i, (intent, key, value) in enumerate(recs):
            arr[i] = zb_rec_desc(key, 1, 10, intent, 0, len(value), len(blob))
            blob += value
        buf = ctypes.create_string_buffer(bytes(blob), max(len(blob), 1))
        self._check(self._L.zb_submit_messages(self._h, arr, n, buf, len(blob)))

    def set_clock(self, now_ms: int):
        self._check(self._L.zb_set_clock(self._h, now_ms))

    def expire_messages(self, now_ms: int) -> int:
        """MessageTimeToLiveChecker at now_ms: DELETE commands for the expired messages, processed."""
        n = ctypes.c_uint64(0)
        self._check(self._L.zb_expire_messages(self._h, now_ms, ctypes.byref(n)))
        return n.value

    def counters(self) -> dict:
        arr = (ctypes.c_int64 * 8)()
        self._check(self._L.zb_counters(self._h, arr))
        return dict(created=arr[0], completed=arr[1], canceled=arr[2], next_wf_key=arr[3], next_job_key=arr[4],
                    rows=arr[5], arena_bytes=arr[6], log_size=arr[7])


def rccl_library() -> str:
    """The file of the RCCL library the engine's communicator runs on (zb_rccl_library: dladdr of ncclCommInitRank)."""
    return lib().zb_rccl_library().decode("utf-8", "replace")


def pinned_alloc(nbytes: int) -> int:
    p = lib().zb_pinned_alloc(nbytes)
    if not p:
        raise MemoryError("zb_pinned_alloc(%d) failed" % nbytes)
    return p


def pinned_free(p: int):
    lib().zb_pinned_free(p)
