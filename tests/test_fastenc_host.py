"""Fuzz the drain write pass's fast value encoder (zeebe_amd/csrc/zb_fastenc.hpp) on CPU.

tests/native/fastenc_host.cpp compiles the encoder for the host. Each value is checked two ways:
  * its bytes equal the reference layout (WorkflowInstanceRecord.java:39-60, JobRecord.java:35-53 +
    JobHeaders.java:33-51, MsgPackWriter integer / string / binary encodings), built here with msgpack;
  * no store lands outside the value: the image is filled with guard bytes and the value starts at every
    offset mod 8; on the GPU the bytes around a value belong to the neighbouring lanes' records (the
    encoder stores whole aligned 8-byte slots inside the value, exact aligned pieces at its two ends).
"""
import ctypes
import os
import random
import struct
import subprocess

import msgpack
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
NATIVE = os.path.join(HERE, "native")
CSRC = os.path.join(HERE, "..", "zeebe_amd", "csrc")
VT_JOB, VT_WI = 0, 5
VT_MSG, VT_MSG_SUB, VT_WIS = 10, 11, 12
GUARD = 0xEE


@pytest.fixture(scope="module")
def lib():
    src = os.path.join(NATIVE, "fastenc_host.cpp")
    so = os.path.join(NATIVE, "libfastenc_host.so")
    deps = [src] + [os.path.join(CSRC, f) for f in ("zb_fastenc.hpp", "zb_device.hpp")]
    if not os.path.exists(so) or os.path.getmtime(so) < max(os.path.getmtime(f) for f in deps):
        subprocess.check_call(["g++", "-O1", "-std=c++17", "-fPIC", "-shared", "-o", so, src])
    L = ctypes.CDLL(so)
    L.fastenc.restype = ctypes.c_long
    L.fastenc.argtypes = ([ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32,
                           ctypes.c_int32, ctypes.c_char_p] + [ctypes.c_uint32] * 9 + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32])
    L.fastenc_bf.restype = ctypes.c_long
    L.fastenc_bf.argtypes = L.fastenc.argtypes + [ctypes.c_uint32]
    L.fastenc_msg.restype = ctypes.c_long
    L.fastenc_msg.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_char_p, ctypes.c_uint32,
                              ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32]
    return L


def rand_int(r):
    return r.choice([0, 1, -1, 127, 128, -32, -33, 255, 256, 65535, 65536, 2 ** 32 - 1, 2 ** 32, 2 ** 63 - 1,
                     -128, -129, -32768, -32769, -2 ** 31, -2 ** 31 - 1, -2 ** 63, r.randint(-2 ** 63, 2 ** 63 - 1),
                     r.randint(-70000, 70000), r.randint(0, 2 ** 40)])


def rand_str(r):
    return "".join(r.choice("abcxyz_-0") for _ in range(r.choice([0, 1, 5, 7, 8, 9, 15, 31, 32, 33, 40, 255, 256, 300])))


def encode(lib, vt, intent, inst, scope, wfkey, version, retries, pid, act, jtype, headers, payload, head=0, bf=False):
    """bf: the branch-free writer (the template drain's); its dummy slot is the 8 bytes past the checked image."""
    pool = b""
    offs = {}
    for name, v in (("pid", pid), ("act", act), ("type", jtype), ("hdr", headers or b"")):
        offs[name] = len(pool)
        pool += v
    doc = struct.pack("<I", len(payload)) + payload
    doc += b"\0" * (-len(doc) % 8) + b"\xa5" * 64  # padded to 8, then whatever follows in the arena
    dbuf = ctypes.create_string_buffer(doc, len(doc))
    cap = (2048 + len(payload) + len(pool) + 7) // 8 * 8
    out = (ctypes.c_uint64 * (cap // 8 + 1))()  # 8-aligned image (+ the dummy slot)
    ctypes.memset(out, GUARD, cap)
    args = (vt, intent, inst, scope, wfkey, version, retries, pool, len(pool), offs["pid"], len(pid),
            offs["act"], len(act), offs["type"], len(jtype), offs["hdr"] if headers else 0xFFFFFFFF,
            len(headers or b""), dbuf, out, head)
    n = lib.fastenc_bf(*args, cap) if bf else lib.fastenc(*args)
    raw = bytes(out)[:cap]
    assert n > 0
    assert all(b == GUARD for b in raw[:head]), "store before the value start (the previous lane's bytes)"
    assert all(b == GUARD for b in raw[head + n:]), "store past the value end"
    return raw[head:head + n]


def expect_wi(pid, version, wfkey, inst, act, payload, scope):
    return msgpack.packb({"bpmnProcessId": pid.decode(), "version": version, "workflowKey": wfkey,
                          "workflowInstanceKey": inst, "activityId": act.decode(), "payload": payload,
                          "scopeInstanceKey": scope}, use_bin_type=True)


def expect_job(pid, version, wfkey, inst, act, payload, scope, retries, jtype, headers):
    # JobRecord: deadline, worker, retries, type, headers (JobHeaders: 6 properties), customHeaders, payload
    head = msgpack.packb({"deadline": -2 ** 63, "worker": "", "retries": retries, "type": jtype.decode(),
                          "headers": {"bpmnProcessId": pid.decode(), "workflowDefinitionVersion": version,
                                      "workflowKey": wfkey, "workflowInstanceKey": inst, "activityId": act.decode(),
                                      "activityInstanceKey": scope}, "customHeaders": {}}, use_bin_type=True)
    # customHeaders are raw pre-encoded msgpack from the pool ({} = 0x80 when there are none), payload last
    assert head.startswith(b"\x86") and head.endswith(b"\xadcustomHeaders\x80")
    head = head[:-1] + (headers if headers else b"\x80")
    return b"\x87" + head[1:] + msgpack.packb("payload") + msgpack.packb(payload, use_bin_type=True)


@pytest.mark.parametrize("bf", [False, True])
def test_fast_encoder_fuzz(lib, bf):
    r = random.Random(11)
    for it in range(3000):
        pid, act, jtype = (rand_str(r).encode() for _ in range(3))
        payload = bytes(r.randrange(256) for _ in range(r.choice([0, 1, 2, 3, 4, 5, 6, 7, 8, 11, 12, 13, 35, 43, 44,
                                                                   45, 48, 52, 100, 255, 256, 300, 70000])))
        inst, scope, wfkey = rand_int(r), rand_int(r), rand_int(r)
        version, retries = (max(-2 ** 31, min(2 ** 31 - 1, rand_int(r))) for _ in range(2))
        headers = r.choice([None, msgpack.packb({"k": "v" * r.randrange(20)})])
        if it % 2 == 0:
            got = encode(lib, VT_WI, 4, inst, scope, wfkey, version, retries, pid, act, jtype, headers, payload,
                         head=r.randrange(24), bf=bf)
            assert got == expect_wi(pid, version, wfkey, inst, act, payload, scope), it
        else:
            got = encode(lib, VT_JOB, 5, inst, scope, wfkey, version, retries, pid, act, jtype, headers, payload,
                         head=r.randrange(24), bf=bf)
            assert got == expect_job(pid, version, wfkey, inst, act, payload, scope, retries, jtype, headers), it


def test_fast_kind_excludes_cancel(lib):
    # JOB CANCEL / CANCELED (a reset record) and submitted CREATEs stay on the generic encoder
    for intent in (12, 13):
        n = lib.fastenc(VT_JOB, intent, 1, 1, 1, 1, 3, b"x", 1, 0, 1, 0, 1, 0, 1, 0xFFFFFFFF, 0,
                        ctypes.create_string_buffer(16), ctypes.create_string_buffer(256), 0)
        assert n == -1


def encode_msg(lib, vt, inst, scope, msg, blob, head):
    """One message-side value through fast_encode_msg (checked stores): bytes, and nothing stored outside them."""
    blob = blob + b"\0" * (-len(blob) % 8) + b"\xa5" * 64  # padded to 8, then whatever follows in the arena
    bbuf = ctypes.create_string_buffer(blob, len(blob))
    cap = (4096 + len(blob) + 7) // 8 * 8
    out = (ctypes.c_uint64 * (cap // 8))()
    ctypes.memset(out, GUARD, cap)
    n = lib.fastenc_msg(vt, inst, scope, msg, len(msg), bbuf, len(blob) // 8, out, head)
    raw = bytes(out)
    assert n > 0
    assert all(b == GUARD for b in raw[:head]), "store before the value start (the previous lane's bytes)"
    assert all(b == GUARD for b in raw[head + n:]), "store past the value end"
    return raw[head:head + n]


def test_fast_encoder_message_kinds_fuzz(lib):
    """WorkflowInstanceSubscriptionRecord.java:26-38, MessageSubscriptionRecord.java:26-41, MessageRecord.java:26-42
    (the layouts encode_value writes), from the arena blobs zb_msg.hpp reads (SubView / MsgView)."""
    r = random.Random(17)
    for it in range(3000):
        inst, scope = rand_int(r), rand_int(r)
        head = r.randrange(24)
        kind = it % 3
        if kind == 0:
            msg = rand_str(r).encode()
            payload = bytes(r.randrange(256) for _ in range(r.choice([0, 1, 7, 8, 9, 43, 44, 45, 100, 300, 70000])))
            blob = struct.pack("<I", len(payload)) + payload
            got = encode_msg(lib, VT_WIS, inst, scope, msg, blob, head)
            want = msgpack.packb({"workflowInstanceKey": inst, "activityInstanceKey": scope, "messageName": msg.decode(),
                                  "payload": payload}, use_bin_type=True)
        elif kind == 1:
            name, ck = rand_str(r).encode(), rand_str(r).encode()
            wfp = r.choice([0, 1, 7, 127, 128, 255, 256, 65535, 65536, 2 ** 31 - 1])
            blob = struct.pack("<IiIH2xII", 24 + len(name) + len(ck), wfp, r.randrange(2 ** 32), r.randrange(2 ** 16),
                               len(name), len(ck)) + name + ck
            got = encode_msg(lib, VT_MSG_SUB, inst, scope, b"", blob, head)
            want = msgpack.packb({"workflowInstancePartitionId": wfp, "workflowInstanceKey": inst,
                                  "activityInstanceKey": scope, "messageName": name.decode(),
                                  "correlationKey": ck.decode()}, use_bin_type=True)
        else:
            name, ck, mid = rand_str(r).encode(), rand_str(r).encode(), rand_str(r).encode()
            payload = bytes(r.randrange(256) for _ in range(r.choice([0, 1, 5, 8, 13, 64, 255, 256, 1000])))
            ttl = rand_int(r)
            blob = (struct.pack("<IIqqIII4x", 40 + len(name) + len(ck) + len(payload) + len(mid), len(name), ttl,
                                r.randrange(2 ** 40), len(ck), len(payload), len(mid)) + name + ck + payload + mid)
            got = encode_msg(lib, VT_MSG, inst, scope, b"", blob, head)
            want = msgpack.packb({"name": name.decode(), "correlationKey": ck.decode(), "timeToLive": ttl,
                                  "payload": payload, "messageId": mid.decode()}, use_bin_type=True)
        assert got == want, (it, kind, head)
