"""Fuzz the kernels' per-thread byte routines (merge, json-path) against the oracle on CPU.

tests/native/devlib_host.cpp compiles zeebe_amd/csrc/zb_devlib.hpp for the host (test only); the
same source runs inside the HIP kernels, so logic bugs show up here without a GPU.
"""
import ctypes
import os
import random
import struct
import subprocess

import msgpack
import pytest

from oracle import zbref

HERE = os.path.dirname(os.path.abspath(__file__))
NATIVE = os.path.join(HERE, "native")


@pytest.fixture(scope="module")
def devlib():
    src = os.path.join(NATIVE, "devlib_host.cpp")
    so = os.path.join(NATIVE, "libdevlib_host.so")
    hdrs = [os.path.join(HERE, "..", "zeebe_amd", "csrc", f) for f in ("zb_devlib.hpp", "zb_model.cpp", "zb_model.hpp",
                                                                        "zb_device.hpp")]
    if not os.path.exists(so) or os.path.getmtime(so) < max([os.path.getmtime(src)] + [os.path.getmtime(h) for h in hdrs]):
        subprocess.check_call(["g++", "-O1", "-std=c++17", "-fPIC", "-shared", "-I/opt/rocm/include", "-o", so, src])
    L = ctypes.CDLL(so)
    L.devlib_merge.restype = ctypes.c_long
    L.devlib_merge.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p,
                               ctypes.c_uint32]
    L.devlib_query.restype = ctypes.c_long
    return L


def rand_value(r, depth):
    k = r.random()
    if depth > 0 and k < 0.2:
        return {rand_key(r): rand_value(r, depth - 1) for _ in range(r.randint(0, 4))}
    if depth > 0 and k < 0.35:
        return [rand_value(r, depth - 1) for _ in range(r.randint(0, 4))]
    return r.choice([None, True, False, r.randint(-2 ** 40, 2 ** 40), r.randint(-200, 300), r.random() * 100,
                     "s" * r.randint(0, 40), b"\x01\x02"])


def rand_key(r):
    return r.choice(["a", "b", "c", "d", "0", "1", "2", "key", "x" * 33])


def rand_doc(r, depth=3):
    return {rand_key(r): rand_value(r, depth) for _ in range(r.randint(0, 5))}


def dev_merge(L, src, tgt):
    out = ctypes.create_string_buffer(1 << 16)
    n = L.devlib_merge(src, len(src), tgt, len(tgt), out, 1 << 16)
    return n, out.raw[:max(n, 0)]


def test_merge_fuzz_vs_oracle(devlib):
    r = random.Random(7)
    checked = unsupported = 0
    for _ in range(3000):
        s, t = rand_doc(r), rand_doc(r)
        if r.random() < 0.3:  # overlapping keys with mixed shapes
            for k in list(s)[:2]:
                t[k] = rand_value(r, 2)
        sb, tb = msgpack.packb(s), msgpack.packb(t)
        n, got = dev_merge(devlib, sb, tb)
        if n == -2:
            unsupported += 1
            continue
        assert n >= 0, (s, t, n)
        ref = zbref.merge(sb, tb)
        ref = b"\x80" if ref == b"\xc0" else ref
        assert got == ref, (s, t, got.hex(), ref.hex())
        checked += 1
    assert unsupported == 0
    assert checked > 2900


def test_merge_byte_vectors(devlib, vectors):
    for v in vectors["merges"]:
        sb, tb = bytes.fromhex(v["source"]), bytes.fromhex(v["target"])
        n, got = dev_merge(devlib, sb, tb)
        assert n >= 0
        ref = zbref.merge(sb, tb)
        assert got == (b"\x80" if ref == b"\xc0" else ref)


def _filters(path):
    """Compile a simple path the way JsonPathQueryCompiler does (for the fuzz only: $.a.b, $.a[1], $.*)."""
    ids, idx, keys, koff, klen = [0], [0], b"", [0], [0]
    i = 1
    toks = path[1:].replace("[", ".").replace("]", "").split(".")[1:] if path != "$" else []
    for t in toks:
        if t == "*":
            ids.append(3); idx.append(0); koff.append(0); klen.append(0)
        elif t.isdigit():
            ids.append(2); idx.append(int(t)); koff.append(0); klen.append(0)
        else:
            ids.append(1); idx.append(0); koff.append(len(keys)); klen.append(len(t)); keys += t.encode()
    return ids, idx, keys, koff, klen


def test_query_fuzz_vs_oracle(devlib):
    r = random.Random(11)
    paths = ["$.a", "$.b", "$.key", "$.a.b", "$.a.c", "$.a[1]", "$.b[0]", "$.*", "$.a.*", "$.0"]
    for _ in range(3000):
        doc = msgpack.packb(rand_doc(r))
        for p in paths:
            ids, idx, keys, koff, klen = _filters(p)
            nf = len(ids)
            A = lambda t, v: (t * len(v))(*v)  # noqa: E731
            out = (ctypes.c_uint32 * 2)()
            fast = 1 if (nf == 2 and ids[1] == 1) else 0
            for use_fast in ({fast, 0} if fast else {0}):
                cnt = devlib.devlib_query(doc, len(doc), bytes(ids), A(ctypes.c_int32, idx), keys or b"\0",
                                          A(ctypes.c_uint32, koff), A(ctypes.c_uint32, klen), nf, use_fast, out)
                ref = zbref.query(p, doc)
                assert cnt == len(ref), (p, msgpack.unpackb(doc, raw=False), cnt, len(ref), use_fast)
                if cnt:
                    assert doc[out[0]:out[0] + out[1]] == ref[0], (p, doc.hex())


def _flat_doc(r):
    keys = ["a", "b", "c", "orderId", "step", "done", "k" * 31, "0", ""]
    vals = [None, True, False, 0, 1, -1, 127, 128, -33, 255, 256, 65535, 65536, -129, -40000, 2 ** 31, -2 ** 31 - 1,
            2 ** 40, -2 ** 40, 0.5, 1e300, "", "x", "y" * 31, "z" * 32, "w" * 200, b"\x00", b"\x01" * 40]
    return {r.choice(keys): r.choice(vals) for _ in range(r.randint(0, 6))}


def test_flat_merge_matches_general(devlib):
    """merge_flat (the kernels' fast path) is byte-identical to merge_docs wherever it accepts the input."""
    devlib.devlib_merge_flat.restype = ctypes.c_long
    devlib.devlib_merge_flat.argtypes = devlib.devlib_merge.argtypes
    r = random.Random(7)
    accepted = 0
    for it in range(6000):
        src, tgt = _flat_doc(r), _flat_doc(r)
        if it % 10 == 0:
            tgt = r.choice([{}, None])
        if it % 13 == 0:
            src = r.choice([{}, None])
        sb = b"" if src is None and it % 2 else msgpack.packb(src)
        tb = msgpack.packb(tgt)
        if it % 17 == 0:  # non-flat shapes must be declined
            sb = msgpack.packb({"n": {"x": 1}})
        cap = len(sb) + len(tb) + 8
        out_f = ctypes.create_string_buffer(cap + 1)
        out_g = ctypes.create_string_buffer(cap + 1)
        nf = devlib.devlib_merge_flat(sb, len(sb), tb, len(tb), out_f, cap)
        ng = devlib.devlib_merge(sb, len(sb), tb, len(tb), out_g, cap)
        if nf == -5:
            continue
        accepted += 1
        assert ng >= 0, (src, tgt, ng)
        assert out_f.raw[:nf] == out_g.raw[:ng], (src, tgt)
    assert accepted > 3000


# ---- explicit io-mappings (map_documents) vs the oracle's MappingProcessor restatement, with the tables built by
# the product's deploy-time compilers (zb_model.cpp compile_mapping)
def dev_map(L, src, tgt, mappings):
    spec = "".join("%s\t%s\n" % m for m in mappings).encode()
    out = ctypes.create_string_buffer(1 << 16)
    err = ctypes.create_string_buffer(512)
    fq = ctypes.c_uint32()
    n = L.devlib_map_text(src, len(src), tgt, len(tgt) if tgt is not None else 0, spec, out, 1 << 16,
                          ctypes.byref(fq), err, 512)
    return n, out.raw[:max(n, 0)], fq.value


def _oracle_map(src, tgt, mappings):
    try:
        return 0, zbref.map_documents(src, mappings, tgt)
    except zbref.MappingError as e:
        return 1, str(e)
    except RuntimeError as e:
        return 2, str(e)


def test_mapping_fuzz_vs_oracle(devlib):
    devlib.devlib_map_text.restype = ctypes.c_long
    r = random.Random(23)
    sources = ["$", "$.a", "$.b", "$.key", "$.a.b", "$.a.c", "$.a[1]", "$.b[0]", "$.0", "$.c"]
    targets = ["$", "$.a", "$.b", "$.n", "$.a.b", "$.a.x", "$.n.m", "$.a[0]", "$.n[1]", "$.a.0", "$.b.c.d",
               "$.x[0].y"]
    checked = {0: 0, 1: 0, 2: 0}
    unsupported = 0
    for it in range(4000):
        s = rand_doc(r)
        t = rand_doc(r) if it % 4 else None
        present = ["$." + k for k in s if k.isalnum() and not k.isdigit()] + ["$"]
        ms = [(r.choice(present) if r.random() < 0.7 else r.choice(sources), r.choice(targets))
              for _ in range(r.randint(1, 3))]
        sb = msgpack.packb(s)
        tb = msgpack.packb(t) if t is not None else None
        n, got, fq = dev_map(devlib, sb, tb, ms)
        kind, ref = _oracle_map(sb, tb, ms)
        if n == -14:
            unsupported += 1
            continue
        ctx = (s, t, ms, n, kind, ref)
        if kind == 0:
            assert n >= 0 and got == ref, ctx
        elif kind == 1:
            if ref.startswith("No data found for query "):
                assert n == -11 and ref == "No data found for query %s." % ms[fq][0], ctx
            else:
                assert n == -12 and ref.startswith("Processing failed, since mapping"), ctx
        else:
            assert n == -13, ctx
        checked[kind] += 1
    assert unsupported < 40, unsupported
    assert checked[0] > 1000 and checked[1] > 200 and checked[2] > 0, checked


def test_mapping_reference_vectors(devlib, vectors):
    """Every MappingExtractParameterizedTest / MappingMergeParameterizedTest row (transcribed into
    reference_vectors.json) through the kernels' engine: the same document or the same failure as the oracle,
    which test_oracle_iomapping.py pins on the rows' expected JSON."""
    devlib.devlib_map_text.restype = ctypes.c_long
    ran = unsupported = 0
    for kind in ("mapping_extracts", "mapping_merges"):
        for row in vectors[kind]:
            ms = [tuple(m) for m in row["mappings"]]
            if not ms:  # no mappings: the kernels run the default merge (test_merge_* above)
                continue
            src = bytes.fromhex(row["source"])
            tgt = bytes.fromhex(row["target"]) if "target" in row else None
            n, got, _ = dev_map(devlib, src, tgt, ms)
            if n == -20:  # the deploy-time compiler rejects the path (the reference's would too)
                continue
            if n == -14:
                unsupported += 1
                continue
            okind, ref = _oracle_map(src, tgt, ms)
            if okind == 0:
                assert n >= 0 and got == ref, (row, n)
            else:
                assert n in (-11, -12, -13), (row, n, ref)
            ran += 1
    assert ran >= 90 and unsupported <= 6, (ran, unsupported)
