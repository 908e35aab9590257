"""Synthetic inputs for BASELINE.json's configurations.

Shared by the parity tests and bench.py. Payloads are msgpack documents built with the
reference writer's encoding rules (MsgPackWriter.java:143-305: minimal integers, fixstr keys);
all generators are deterministic (counter-based Philox4x32-10, seed 42, counter = instance index).
"""
from __future__ import annotations

import struct
from typing import List, Tuple

import numpy as np

from . import bpmn


def mp_int(v: int) -> bytes:
    """MsgPackWriter.writeInteger (signed semantics)."""
    if v < -(1 << 5):
        if v < -(1 << 15):
            return b"\xd3" + struct.pack(">q", v) if v < -(1 << 31) else b"\xd2" + struct.pack(">i", v)
        return b"\xd1" + struct.pack(">h", v) if v < -(1 << 7) else b"\xd0" + struct.pack(">b", v)
    if v < (1 << 7):
        return struct.pack(">b", v) if v < 0 else bytes([v])
    if v < (1 << 16):
        return b"\xcc" + bytes([v]) if v < (1 << 8) else b"\xcd" + struct.pack(">H", v)
    return b"\xce" + struct.pack(">I", v) if v < (1 << 32) else b"\xcf" + struct.pack(">q", v)


def mp_str(s: str) -> bytes:
    b = s.encode()
    n = len(b)
    if n < 32:
        return bytes([0xa0 | n]) + b
    if n < 256:
        return b"\xd9" + bytes([n]) + b
    return b"\xda" + struct.pack(">H", n) + b


def order_payloads(n: int, start: int = 0) -> Tuple[bytes, np.ndarray]:
    """{"orderId": i} for i in [start, start+n): packed blob + uint64 offsets (n+1)."""
    head = b"\x81" + mp_str("orderId")
    parts = [head + mp_int(i) for i in range(start, start + n)]
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(p) for p in parts], dtype=np.uint64)
    return b"".join(parts), offs


def order_string_payloads(n: int, start: int = 0) -> Tuple[bytes, np.ndarray]:
    """C5: {"orderId": "order-<i>"}."""
    head = b"\x81" + mp_str("orderId")
    parts = [head + mp_str("order-%d" % i) for i in range(start, start + n)]
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(p) for p in parts], dtype=np.uint64)
    return b"".join(parts), offs


REGIONS = ("EU", "US", "APAC")


def philox4x32(counter: np.ndarray, key: int) -> np.ndarray:
    """Philox4x32-10 (Salmon et al., SC'11) of the 128-bit counters (i, 0, 0, 0), key (key, 0): (n, 4) uint32.
    Counter-based: instance i's values depend on i alone, so any partitioning of the instances generates the
    same payload for the same instance (stream = instance index)."""
    m0, m1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
    mask = np.uint64(0xFFFFFFFF)
    c0 = counter.astype(np.uint64) & mask
    c1 = (counter.astype(np.uint64) >> np.uint64(32)) & mask
    c2 = np.zeros_like(c0)
    c3 = np.zeros_like(c0)
    k0, k1 = np.uint64(key & 0xFFFFFFFF), np.uint64(0)
    for _ in range(10):
        p0 = m0 * c0
        p1 = m1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & mask
        hi1, lo1 = p1 >> np.uint64(32), p1 & mask
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = (k0 + np.uint64(0x9E3779B9)) & mask
        k1 = (k1 + np.uint64(0xBB67AE85)) & mask
    return np.stack([c0, c1, c2, c3], axis=1).astype(np.uint32)


def xor_fields(n: int, seed: int = 42, start: int = 0):
    """C3 payload fields of instances [start, start + n): amount U[0,2000), region index U{0,1,2}, score U[0,1)
    (53-bit float64), from Philox4x32-10 with counter = instance index, key = seed."""
    r = philox4x32(np.arange(start, start + n, dtype=np.uint64), seed).astype(np.uint64)
    amount = (r[:, 0] % np.uint64(2000)).astype(np.int64)
    region = (r[:, 1] % np.uint64(3)).astype(np.int64)
    score = ((r[:, 2] >> np.uint64(11)) << np.uint64(32) | r[:, 3]).astype(np.float64)  # 21 + 32 bits
    score = score / float(1 << 53)
    return amount, region, score


def xor_payloads(n: int, seed: int = 42, start: int = 0) -> Tuple[bytes, np.ndarray]:
    """C3: {"amount": U[0,2000), "region": EU|US|APAC, "score": U[0,1) float64} (Philox4x32-10, seed 42, counter =
    instance index), encoded with the reference writer's rules (float32 iff exactly representable)."""
    amount, region, score = xor_fields(n, seed, start)
    ka, kr, ks = mp_str("amount"), mp_str("region"), mp_str("score")
    regs = [mp_str(r) for r in REGIONS]
    parts = []
    for a, r, s in zip(amount.tolist(), region.tolist(), score.tolist()):
        f = struct.pack(">f", s)
        sv = b"\xca" + f if struct.unpack(">f", f)[0] == s else b"\xcb" + struct.pack(">d", s)
        parts.append(b"\x83" + ka + mp_int(a) + kr + regs[r] + ks + sv)
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(p) for p in parts], dtype=np.uint64)
    return b"".join(parts), offs


def xor_payloads_np(n: int, seed: int = 42, start: int = 0) -> Tuple[bytes, np.ndarray]:
    """xor_payloads, vectorized (same bytes): rows of at most 48 bytes assembled column-wise, then packed."""
    amount, region, score = xor_fields(n, seed, start)
    W = 48
    buf = np.zeros((n, W), dtype=np.uint8)
    ln = np.zeros(n, dtype=np.int64)

    def put_const(b: bytes):
        a = np.frombuffer(b, dtype=np.uint8)
        cols = ln[:, None] + np.arange(len(a))[None, :]
        buf[np.arange(n)[:, None], cols] = a[None, :]
        ln[:] += len(a)

    def put_rows(vals: np.ndarray, width: np.ndarray):
        # vals: (n, k) bytes, width: per-row count used
        k = vals.shape[1]
        rows = np.repeat(np.arange(n), k)
        cols = (ln[:, None] + np.arange(k)[None, :]).ravel()
        keep = (np.arange(k)[None, :] < width[:, None]).ravel()
        buf[rows[keep], cols[keep]] = vals.ravel()[keep]
        ln[:] += width

    put_const(b"\x83" + mp_str("amount"))
    # mp_int for 0 <= a < 2000: fixint (<128), 0xcc uint8 (<256), 0xcd uint16
    a = amount.astype(np.int64)
    v = np.zeros((n, 3), dtype=np.uint8)
    w = np.where(a < 128, 1, np.where(a < 256, 2, 3))
    v[:, 0] = np.where(a < 128, a, np.where(a < 256, 0xcc, 0xcd))
    v[:, 1] = np.where(a < 256, a & 0xff, a >> 8)
    v[:, 2] = a & 0xff
    put_rows(v, w)
    put_const(mp_str("region"))
    regs = [mp_str(r) for r in REGIONS]
    rv = np.zeros((n, max(len(r) for r in regs)), dtype=np.uint8)
    rw = np.zeros(n, dtype=np.int64)
    for k, r in enumerate(regs):
        m = region == k
        rv[m, :len(r)] = np.frombuffer(r, dtype=np.uint8)
        rw[m] = len(r)
    put_rows(rv, rw)
    put_const(mp_str("score"))
    f32 = score.astype(np.float32)
    exact = f32.astype(np.float64) == score
    sv = np.zeros((n, 9), dtype=np.uint8)
    sv[:, 0] = np.where(exact, 0xca, 0xcb)
    b32 = f32.astype(">f4").view(np.uint8).reshape(n, 4)
    b64 = score.astype(">f8").view(np.uint8).reshape(n, 8)
    sv[:, 1:9] = b64
    sv[exact, 1:5] = b32[exact]
    put_rows(sv, np.where(exact, 5, 9))
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(ln, dtype=np.uint64)
    mask = np.arange(W)[None, :] < ln[:, None]
    return buf[mask].tobytes(), offs


def split(blob: bytes, offs: np.ndarray) -> List[bytes]:
    o = offs.tolist()
    return [blob[o[i]:o[i + 1]] for i in range(len(o) - 1)]


CONFIGS = {
    "c1": dict(workflow=bpmn.config1_workflow, process="process", payloads=order_payloads,
               job_payloads=lambda: {"task": b"\x81" + mp_str("done") + b"\xc3"}),
    "c2": dict(workflow=lambda: bpmn.chain_workflow(20), process="chain", payloads=order_payloads,
               job_payloads=lambda: {"t%d" % k: b"\x81" + mp_str("step") + mp_int(k) for k in range(1, 21)}),
    "c3": dict(workflow=bpmn.xor_workflow, process="xor", payloads=xor_payloads, job_payloads=lambda: {}),
    "c4": dict(workflow=lambda: bpmn.parallel_workflow(8), process="par", payloads=order_payloads,
               job_payloads=lambda: {"task%d" % k: b"\x81" + mp_str("sub") + mp_int(k) for k in range(1, 9)}),
    "c4twin": dict(workflow=lambda: bpmn.subprocess_chain_workflow(8), process="subs", payloads=order_payloads,
                   job_payloads=lambda: {"task%d" % k: b"\x81" + mp_str("sub") + mp_int(k) for k in range(1, 9)}),
}
