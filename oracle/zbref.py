"""ctypes binding of the zbref oracle (ORACLE / TEST INFRASTRUCTURE ONLY).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker
and the CPU baseline. The product path (zeebe_amd) never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import struct
import subprocess
from typing import List, NamedTuple, Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libzbref.so")


def build() -> str:
    subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, i64, i32, sz = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_size_t
        cp, u8p = ctypes.c_char_p, ctypes.c_char_p
        L.zbref_new.restype = vp
        L.zbref_new.argtypes = [ctypes.c_int, ctypes.c_int]
        L.zbref_free.argtypes = [vp]
        L.zbref_last_error.restype = cp
        L.zbref_last_error.argtypes = [vp]
        L.zbref_deploy.argtypes = [vp, cp, sz, i64, i32]
        L.zbref_set_job_payload.argtypes = [vp, i64, cp, u8p, sz]
        L.zbref_submit_create.argtypes = [vp, cp, i32, i64, u8p, sz]
        L.zbref_submit_cancel.argtypes = [vp, i64]
        L.zbref_submit_creates.argtypes = [vp, cp, i32, i64, sz, ctypes.c_void_p, ctypes.c_void_p]
        L.zbref_set_harness.argtypes = [vp, ctypes.c_int]
        L.zbref_set_job_processor.argtypes = [vp, ctypes.c_int]
        L.zbref_submit_record.argtypes = [vp, ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint8, i64, u8p, sz]
        L.zbref_dump_instances.restype = i64
        L.zbref_dump_instances.argtypes = [vp, ctypes.c_void_p, sz]
        L.zbref_submit_correlate.argtypes = [vp, i64, i64, cp, u8p, sz]
        L.zbref_submit_open.argtypes = [vp, i32, i64, i64, u8p, sz, u8p, sz]
        L.zbref_submit_publish.argtypes = [vp, u8p, sz, u8p, sz, i64, u8p, sz, u8p, sz]
        L.zbref_set_clock.argtypes = [vp, i64]
        L.zbref_check_ttl.argtypes = [vp, i64]
        L.zbref_check_ttl.restype = i64
        L.zbref_side_effect_count.restype = i64
        L.zbref_side_effect_count.argtypes = [vp]
        L.zbref_side_effect_get.argtypes = [vp, i64, ctypes.POINTER(i32), ctypes.POINTER(i64), ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
        L.zbref_clear_side_effects.argtypes = [vp]
        L.zbref_run.restype = i64
        L.zbref_run.argtypes = [vp, i64]
        L.zbref_log_size.restype = i64
        L.zbref_log_size.argtypes = [vp]
        L.zbref_dump_log.restype = i64
        L.zbref_dump_log.argtypes = [vp, i64, i64, ctypes.c_void_p, sz]
        L.zbref_counters.argtypes = [vp, ctypes.POINTER(i64)]
        L.zbref_side_effects.restype = i64
        L.zbref_side_effects.argtypes = [vp, i64, ctypes.POINTER(i64), ctypes.POINTER(i32), ctypes.c_void_p, sz]
        L.zbref_eval_condition.argtypes = [cp, u8p, sz, ctypes.c_char_p, sz]
        L.zbref_eval_condition_seq.argtypes = [cp, u8p, ctypes.POINTER(ctypes.c_uint32), ctypes.c_int,
                                               ctypes.POINTER(ctypes.c_int)]
        L.zbref_merge.restype = i64
        L.zbref_merge.argtypes = [u8p, sz, u8p, sz, ctypes.c_void_p, sz, ctypes.c_char_p, sz]
        L.zbref_map.restype = i64
        L.zbref_map.argtypes = [u8p, sz, u8p, sz, ctypes.c_char_p, ctypes.c_void_p, sz, ctypes.c_char_p, sz]
        L.zbref_query.argtypes = [cp, u8p, sz, ctypes.POINTER(i32), ctypes.c_int, ctypes.c_char_p, sz]
        L.zbref_jp_tokens.restype = ctypes.c_int
        L.zbref_jp_tokens.argtypes = [cp, ctypes.POINTER(i32), ctypes.c_int]
        L.zbref_jp_compile.restype = ctypes.c_int
        L.zbref_jp_compile.argtypes = [cp, ctypes.POINTER(i32), ctypes.POINTER(i32), ctypes.c_int, ctypes.POINTER(i32),
                                       ctypes.c_char_p, sz]
        L.zbref_read_token.restype = ctypes.c_int
        L.zbref_read_token.argtypes = [u8p, sz, ctypes.POINTER(i64), ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i32),
                                       ctypes.c_char_p, sz]
        L.zbref_traverse.restype = ctypes.c_int
        L.zbref_traverse.argtypes = [u8p, sz, ctypes.POINTER(i32), ctypes.c_char_p, sz]
        L.zbref_set_position_base.argtypes = [vp, i64]
        L.zbref_tree_dump.restype = i64
        L.zbref_tree_dump.argtypes = [u8p, sz, cp, ctypes.c_int, ctypes.c_void_p, sz, ctypes.c_char_p, sz]
        L.zbref_subscription_hash.restype = i32
        L.zbref_subscription_hash.argtypes = [u8p, sz]
        L.zbref_encode_int.restype = i64
        L.zbref_encode_int.argtypes = [i64, ctypes.c_void_p]
        L.zbref_encode_float.restype = i64
        L.zbref_encode_float.argtypes = [ctypes.c_double, ctypes.c_void_p]
        L.zbref_set_request.argtypes = [vp, i64, ctypes.c_uint64, i32]
        L.zbref_frames.restype = i64
        L.zbref_frames.argtypes = [vp, i64, i64, i32, i32, i64, ctypes.c_void_p, sz]
        L.zbref_run_timed.restype = ctypes.c_double
        L.zbref_run_timed.argtypes = [vp, ctypes.POINTER(i64)]
        _lib = L
    return _lib


_HDR = struct.Struct("<qqqBBBBI")  # zbref_record


class Record(NamedTuple):
    position: int
    source_position: int
    key: int
    record_type: int
    value_type: int
    intent: int
    rejection_type: int
    value: bytes


def parse_log(buf: bytes) -> List[Record]:
    out = []
    off = 0
    while off < len(buf):
        pos, src, key, rt, vt, it, rj, vlen = _HDR.unpack_from(buf, off)
        off += _HDR.size
        out.append(Record(pos, src, key, rt, vt, it, rj, bytes(buf[off:off + vlen])))
        off += vlen
    return out


_INST = struct.Struct("<qqqB3xI")


def parse_instances(buf: bytes):
    """[i64 key][i64 parent key][i64 job key][u8 state][3 pad][u32 n][value] records (zb_read_instances layout)."""
    out, off = [], 0
    while off < len(buf):
        key, pk, jk, st, n = _INST.unpack_from(buf, off)
        off += _INST.size
        out.append((key, pk, jk, st, bytes(buf[off:off + n])))
        off += n
    return out


class ZbrefError(RuntimeError):
    pass


class Oracle:
    """One partition of the sequential reference restatement."""

    def __init__(self, partition_id: int = 0, partition_count: int = 1):
        self._L = lib()
        self._h = self._L.zbref_new(partition_id, partition_count)

    def close(self):
        if self._h:
            self._L.zbref_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _err(self) -> str:
        return self._L.zbref_last_error(self._h).decode("utf-8", "replace")

    def deploy(self, xml: bytes, workflow_key: int, version: int = 1):
        if isinstance(xml, str):
            xml = xml.encode()
        if self._L.zbref_deploy(self._h, xml, len(xml), workflow_key, version) != 0:
            raise ZbrefError(self._err())

    def set_job_payload(self, workflow_key: int, activity_id: str, payload: bytes):
        self._L.zbref_set_job_payload(self._h, workflow_key, activity_id.encode(), payload, len(payload))

    def create(self, process_id: str, payload: bytes = b"\x80", version: int = -1, workflow_key: int = -1):
        if self._L.zbref_submit_create(self._h, process_id.encode(), version, workflow_key, payload, len(payload)):
            raise ZbrefError(self._err())

    def create_packed(self, process_id: str, blob: bytes, offsets, version: int = -1, workflow_key: int = -1):
        """Bulk create: offsets is a uint64 numpy array of n+1 entries into blob."""
        buf = ctypes.create_string_buffer(blob, max(len(blob), 1))
        if self._L.zbref_submit_creates(self._h, process_id.encode(), version, workflow_key, len(offsets) - 1, buf,
                                        offsets.ctypes.data):
            raise ZbrefError(self._err())

    def cancel(self, key: int):
        self._L.zbref_submit_cancel(self._h, key)

    def set_position_base(self, base: int):
        """The log's first position (the engine's zb_log_start): positions, source positions, position keys follow."""
        if self._L.zbref_set_position_base(self._h, base):
            raise ZbrefError("position base on a non-empty log")

    def set_harness(self, on: bool):
        """Canonical job harness on (default) / off (JOB CREATE commands wait for submitted job events)."""
        self._L.zbref_set_harness(self._h, 1 if on else 0)

    def set_job_processor(self, on: bool):
        """The job stream processor (JobInstanceStreamProcessor) processes JOB commands on this log (harness off)."""
        self._L.zbref_set_job_processor(self._h, 1 if on else 0)

    def submit(self, record_type: int, value_type: int, intent: int, key: int, value: bytes):
        """A record written by another writer, as its reference msgpack value (kept verbatim in the log)."""
        if self._L.zbref_submit_record(self._h, record_type, value_type, intent, key, value, len(value)):
            raise ZbrefError(self._err())

    def instances(self):
        """Live element instances (ElementInstanceIndex) sorted by key:
        list of (key, parent_key, job_key, state, value bytes)."""
        need = self._L.zbref_dump_instances(self._h, None, 0)
        buf = ctypes.create_string_buffer(max(need, 1))
        self._L.zbref_dump_instances(self._h, buf, need)
        return parse_instances(buf.raw[:need])

    def correlate(self, wf_instance_key: int, activity_instance_key: int, message_name, payload: bytes):
        """WORKFLOW_INSTANCE_SUBSCRIPTION CORRELATE command (key = its log position)."""
        if isinstance(message_name, str):
            message_name = message_name.encode()
        self._L.zbref_submit_correlate(self._h, wf_instance_key, activity_instance_key, message_name, payload,
                                       len(payload))

    def open_subscription(self, wf_partition: int, wf_instance_key: int, activity_instance_key: int,
                          message_name: bytes, correlation_key: bytes):
        """MESSAGE_SUBSCRIPTION OPEN command (key = its log position)."""
        self._L.zbref_submit_open(self._h, wf_partition, wf_instance_key, activity_instance_key, message_name,
                                  len(message_name), correlation_key, len(correlation_key))

    def publish(self, name: bytes, correlation_key: bytes, payload: bytes = b"\x80", ttl: int = 0,
                message_id: bytes = b""):
        """MESSAGE PUBLISH command (null key)."""
        self._L.zbref_submit_publish(self._h, name, len(name), correlation_key, len(correlation_key), ttl, payload,
                                     len(payload), message_id, len(message_id))

    def set_clock(self, now_ms: int):
        """ActorClock.currentTimeMillis() for the records processed from now on (message deadlines)."""
        self._L.zbref_set_clock(self._h, now_ms)

    def check_ttl(self, now_ms: int) -> int:
        """MessageTimeToLiveChecker.run at now_ms: DELETE commands for the expired messages (run() processes
        them). Returns how many were written."""
        return self._L.zbref_check_ttl(self._h, now_ms)

    def take_side_effects(self):
        """Side effects since the last call, in emission order, as dicts (kind 1 open, 2 correlate)."""
        n = self._L.zbref_side_effect_count(self._h)
        out = []
        ints = (ctypes.c_int32 * 3)()
        keys = (ctypes.c_int64 * 2)()
        lens = (ctypes.c_uint64 * 3)()
        bufs = [ctypes.create_string_buffer(4096) for _ in range(3)]
        for i in range(n):
            self._L.zbref_side_effect_get(self._h, i, ints, keys, bufs[0], bufs[1], bufs[2], lens)
            name, ck, payload = (bufs[k].raw[:lens[k]] for k in range(3))
            out.append(dict(kind=ints[0], partition=ints[1], wf_partition=ints[2], wik=keys[0], aik=keys[1],
                            name=name, ck=ck, payload=payload))
        self._L.zbref_clear_side_effects(self._h)
        return out

    def run(self, max_records: int = -1) -> int:
        n = self._L.zbref_run(self._h, max_records)
        if n < 0:
            raise ZbrefError(self._err())
        return n

    def run_timed(self):
        n = ctypes.c_int64()
        t = self._L.zbref_run_timed(self._h, ctypes.byref(n))
        if n.value < 0:
            raise ZbrefError(self._err())
        return n.value, t

    def log_size(self) -> int:
        return self._L.zbref_log_size(self._h)

    def records(self, start: int = 0, end: int = -1) -> List[Record]:
        need = self._L.zbref_dump_log(self._h, start, end, None, 0)
        buf = ctypes.create_string_buffer(max(need, 1))
        self._L.zbref_dump_log(self._h, start, end, buf, need)
        return parse_log(buf.raw[:need])

    def dump(self, start: int = 0, end: int = -1) -> bytes:
        need = self._L.zbref_dump_log(self._h, start, end, None, 0)
        buf = ctypes.create_string_buffer(max(need, 1))
        self._L.zbref_dump_log(self._h, start, end, buf, need)
        return buf.raw[:need]

    def set_request(self, position: int, request_id: int, request_stream_id: int):
        """Request metadata (requestId, requestStreamId) of the submitted command at `position`."""
        if self._L.zbref_set_request(self._h, position, request_id, request_stream_id):
            raise ZbrefError("no record at position %d" % position)

    def frames(self, start: int = 0, end: int = -1, stream_id: int = 0, raft_term: int = 0,
               timestamp: int = 0) -> bytes:
        """Log frames of records [start, end) as the reference's log writers lay them into the dispatcher
        buffer (DataFrameDescriptor + LogEntryDescriptor + RecordMetadata + value, 8-aligned)."""
        need = self._L.zbref_frames(self._h, start, end, stream_id, raft_term, timestamp, None, 0)
        buf = ctypes.create_string_buffer(max(need, 1))
        self._L.zbref_frames(self._h, start, end, stream_id, raft_term, timestamp, buf, need)
        return buf.raw[:need]

    def counters(self) -> dict:
        arr = (ctypes.c_int64 * 7)()
        self._L.zbref_counters(self._h, arr)
        return dict(created=arr[0], completed=arr[1], canceled=arr[2], live_instances=arr[3],
                    next_wf_key=arr[4], next_job_key=arr[5], transitions=arr[6])

    def side_effects(self):
        n = self._L.zbref_side_effects(self._h, -1, None, None, None, 0)
        out = []
        for i in range(n):
            keys = (ctypes.c_int64 * 2)()
            part = ctypes.c_int32()
            buf = ctypes.create_string_buffer(4096)
            ln = self._L.zbref_side_effects(self._h, i, keys, ctypes.byref(part), buf, 4096)
            out.append((keys[0], keys[1], part.value, buf.raw[:ln]))
        return out


def eval_condition(expr: str, doc: bytes):
    """Returns True/False, or raises ValueError(compile msg) / RuntimeError(eval msg)."""
    err = ctypes.create_string_buffer(4096)
    r = lib().zbref_eval_condition(expr.encode(), doc, len(doc), err, 4096)
    if r == -1:
        raise ValueError(err.value.decode())
    if r == -2:
        raise RuntimeError(err.value.decode())
    return bool(r)


def merge(source: bytes, target: bytes) -> bytes:
    out = ctypes.create_string_buffer(65536)
    err = ctypes.create_string_buffer(4096)
    n = lib().zbref_merge(source, len(source), target, len(target), out, 65536, err, 4096)
    if n < 0:
        raise RuntimeError(err.value.decode())
    return out.raw[:n]


class MappingError(Exception):
    """MappingException (json-path/.../mapping/MappingException.java): becomes an IO_MAPPING_ERROR incident."""


def map_documents(source: bytes, mappings, target: Optional[bytes] = None) -> bytes:
    """MappingProcessor.extract(source, mappings) (target None) or .merge(source, target, mappings)."""
    spec = "".join("%s\t%s\n" % (a, b) for a, b in mappings).encode()
    out = ctypes.create_string_buffer(1 << 20)
    err = ctypes.create_string_buffer(4096)
    n = lib().zbref_map(source, len(source), target, len(target) if target is not None else 0, spec, out, 1 << 20,
                        err, 4096)
    if n == -1:
        raise MappingError(err.value.decode())
    if n < 0:
        raise RuntimeError(err.value.decode())
    return out.raw[:n]


def query(path: str, doc: bytes):
    out = (ctypes.c_int32 * 256)()
    err = ctypes.create_string_buffer(4096)
    n = lib().zbref_query(path.encode(), doc, len(doc), out, 128, err, 4096)
    if n < 0:
        raise ValueError(err.value.decode())
    return [doc[out[2 * i]:out[2 * i] + out[2 * i + 1]] for i in range(min(n, 128))]


JP_TOKENS = ["START_INPUT", "END_INPUT", "ROOT_OBJECT", "CHILD_OPERATOR", "RECURSION_OPERATOR", "WILDCARD",
             "SUBSCRIPT_OPERATOR_BEGIN", "SUBSCRIPT_OPERATOR_END", "CHILD_BRACKET_OPERATOR_BEGIN",
             "CHILD_BRACKET_OPERATOR_END", "LITERAL"]  # zbref_jsonpath.hpp JpToken order
MP_TYPES = ["INTEGER", "FLOAT", "BOOLEAN", "NIL", "MAP", "ARRAY", "BINARY", "STRING", "EXTENSION", "NEVER_USED"]


def jp_tokens(expr: str):
    """JsonPathTokenizer.tokenize: [(token name, position, length)]."""
    out = (ctypes.c_int32 * 768)()
    n = lib().zbref_jp_tokens(expr.encode(), out, 256)
    return [(JP_TOKENS[out[3 * i]], out[3 * i + 1], out[3 * i + 2]) for i in range(min(n, 256))]


def jp_compile(expr: str):
    """JsonPathQueryCompiler.compile: ([(filter id, index)], None) or (None, (invalid position, error reason))."""
    ids, idx, pos = (ctypes.c_int32 * 256)(), (ctypes.c_int32 * 256)(), ctypes.c_int32()
    err = ctypes.create_string_buffer(512)
    n = lib().zbref_jp_compile(expr.encode(), ids, idx, 256, ctypes.byref(pos), err, 512)
    if n < 0:
        return None, (pos.value, err.value.decode())
    return [(ids[i], idx[i]) for i in range(n)], None


def read_token(b: bytes):
    """MsgPackReader.readToken: dict(type, int, float, bool, size, value, consumed), or the exception message."""
    iv, fv, out = ctypes.c_int64(), ctypes.c_double(), (ctypes.c_int32 * 6)()
    err = ctypes.create_string_buffer(512)
    if lib().zbref_read_token(b, len(b), ctypes.byref(iv), ctypes.byref(fv), out, err, 512) < 0:
        return err.value.decode()
    return {"type": MP_TYPES[out[0]], "int": iv.value, "float": fv.value, "bool": bool(out[1]), "size": out[2],
            "value": b[out[3]:out[3] + out[4]] if out[3] >= 0 else None, "consumed": out[5]}


def traverse(doc: bytes):
    """MsgPackTraverser.traverse: (True, None) or (False, (invalid position, error message))."""
    pos = ctypes.c_int32()
    err = ctypes.create_string_buffer(512)
    if lib().zbref_traverse(doc, len(doc), ctypes.byref(pos), err, 512):
        return True, None
    return False, (pos.value, err.value.decode())


def query_positions(path: str, doc: bytes):
    """MsgPackQueryExecutor results as (position, length) pairs."""
    out = (ctypes.c_int32 * 256)()
    err = ctypes.create_string_buffer(4096)
    n = lib().zbref_query(path.encode(), doc, len(doc), out, 128, err, 4096)
    if n < 0:
        raise ValueError(err.value.decode())
    return [(out[2 * i], out[2 * i + 1]) for i in range(min(n, 128))]


def parse_tree_dump(buf: bytes) -> dict:
    """A tree dump (zbref_tree_dump / devlib_xtree_dump) -> {id: (type, [children], leaf bytes or None)}."""
    out = {}
    for line in buf.split(b"\n"):
        if not line:
            continue
        ty, nid, ch, leaf = line.split(b"\0")
        out[nid.decode()] = (ty.decode(), [c.decode() for c in ch.split(b"\x1e")] if ch else [],
                             bytes.fromhex(leaf.decode()) if leaf else None)
    return out


def tree(doc: bytes, mappings=None) -> dict:
    """MsgPackDocumentIndexer.index(doc) (mappings None) or MsgPackDocumentExtractor.extract(mappings) of doc, as
    parse_tree_dump gives it; a failure raises MappingError / RuntimeError with the processor's message."""
    spec = "".join("%s\t%s\n" % m for m in (mappings or [])).encode()
    err = ctypes.create_string_buffer(4096)
    need = lib().zbref_tree_dump(doc, len(doc), spec, 1 if mappings else 0, None, 0, err, 4096)
    if need < 0:
        raise (MappingError if need == -1 else RuntimeError)(err.value.decode())
    buf = ctypes.create_string_buffer(need)
    lib().zbref_tree_dump(doc, len(doc), spec, 1 if mappings else 0, buf, need, err, 4096)
    return parse_tree_dump(buf.raw[:need])


def subscription_hash(b: bytes) -> int:
    return lib().zbref_subscription_hash(b, len(b))


def encode_int(v: int) -> bytes:
    buf = ctypes.create_string_buffer(16)
    n = lib().zbref_encode_int(v, buf)
    return buf.raw[:n]


def encode_float(v: float) -> bytes:
    buf = ctypes.create_string_buffer(16)
    n = lib().zbref_encode_float(v, buf)
    return buf.raw[:n]


def c5_bench(partitions: int, per_partition: int, xml: str):
    """zbref_c5_bench: the C5 schedule over `partitions` oracle partitions, one thread each, exchange in C++.
    Returns (wall seconds, transitions, completed instances, exchange rounds)."""
    out = (ctypes.c_double * 4)()
    x = xml.encode()
    lib().zbref_c5_bench.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_char_p, ctypes.c_size_t,
                                     ctypes.POINTER(ctypes.c_double)]
    if lib().zbref_c5_bench(partitions, per_partition, x, len(x), out) != 0:
        raise ZbrefError("c5 bench failed")
    return out[0], int(out[1]), int(out[2]), int(out[3])


class OraclePartition(Oracle):
    """An oracle partition with the partition interface of zeebe_amd.cluster (LocalCluster / DistCluster):
    side effects become exchange records (zb_exchange_rec layout) sorted by target partition, stable in
    emission order."""

    def __init__(self, partition_id: int = 0, partition_count: int = 1):
        super().__init__(partition_id, partition_count)
        self.partition_id, self.partition_count = partition_id, partition_count
        self._fx = []

    def _harvest(self):
        self._fx.extend(self.take_side_effects())

    def pending(self, kind: int) -> int:
        self._harvest()
        return sum(1 for f in self._fx if f["kind"] == kind)

    def outbox(self, kind: int):
        from zeebe_amd import cluster

        self._harvest()
        mine = [f for f in self._fx if f["kind"] == kind]
        self._fx = [f for f in self._fx if f["kind"] != kind]
        return cluster.pack(mine, self.partition_count)  # one batch per target, emission order within it

    def inbox(self, kind: int, buf):
        from zeebe_amd import cluster

        for r in cluster.unpack(buf.cpu().numpy() if hasattr(buf, "cpu") else buf):
            if kind == cluster.KIND_OPEN:
                self.open_subscription(r["wf_partition"], r["wik"], r["aik"], r["name"], r["ck"])
            else:
                self.correlate(r["wik"], r["aik"], r["name"], r["payload"])

    def publish_batch(self, name: bytes, cks, payloads, ttl: int):
        for ck, pl in zip(cks, payloads):
            Oracle.publish(self, name, ck, pl, ttl)

    def publish(self, name, cks, payloads=None, ttl: int = 3600000, message_id: bytes = b""):
        """Cluster form: publish(name, [ck...], [payload...], ttl); single form: publish(name, ck, payload, ttl)."""
        if isinstance(cks, (bytes, bytearray)):
            return Oracle.publish(self, name, cks, payloads if payloads is not None else b"\x80", ttl, message_id)
        self.publish_batch(name, cks, payloads, ttl)
