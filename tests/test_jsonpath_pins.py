"""Pin the json-path tokenizer / compiler, the query walker and the msgpack token reader -- the oracle's
restatement AND the product's own code (zb_model.cpp compile_filters / compile_query, zb_devlib.hpp run_query /
read_tok, built for the host by tests/native/devlib_host.cpp) -- on the reference's own tests, transcribed into
tests/golden/reference_vectors.json by tests/golden/make_reference_vectors.py:

  jsonpath_tokens   json-path/src/test/java/io/zeebe/msgpack/jsonpath/JsonPathTokenizerTest.java:28-124
  jsonpath_compile  json-path/.../jsonpath/JsonPathQueryCompilerTest.java:31-79
  jsonpath_invalid  json-path/.../jsonpath/JsonPathQueryValidationTest.java:29-38
  queries           json-path/.../jsonpath/JsonPathTest.java:39-104, .../query/MsgPackQueryProcessorTest.java:38-146,
                    .../query/MsgPackQueryValueFormatsTest.java:39-116, .../query/MsgPackTraverserTest.java:111-228
  traversal_errors  .../query/MsgPackTraverserTest.java:230-256
  read_tokens       msgpack-core/src/test/java/io/zeebe/msgpack/spec/MsgPackReadTokenTest.java:55-241

The device query entry (run_query) is the one every exclusive-gateway condition operand and every correlation key
extraction (k_subscribe) goes through. CPU only.
"""
import ctypes
import struct

import pytest

from oracle import zbref
from test_devlib_host import devlib  # noqa: F401  (module fixture: the host build of the kernels' routines)

TOK_TYPES = ["INTEGER", "FLOAT", "BOOLEAN", "NIL", "MAP", "ARRAY", "BINARY", "STRING", "EXTENSION"]  # zb_device.hpp


def dev_compile(L, expr):
    ids, idx = (ctypes.c_int32 * 64)(), (ctypes.c_int32 * 64)()
    err = ctypes.create_string_buffer(256)
    L.devlib_compile_path.restype = ctypes.c_long
    n = L.devlib_compile_path(expr.encode(), ids, idx, 64, err, 256)
    if n < 0:
        return None, err.value.decode()
    return [ids[i] for i in range(n)], None


def dev_query(L, expr, doc):
    out = (ctypes.c_uint32 * 2)()
    L.devlib_query_text.restype = ctypes.c_long
    n = L.devlib_query_text(expr.encode(), doc, len(doc), out)
    return n, (out[0], out[1])


def dev_token(L, b):
    iv, fv, out = ctypes.c_int64(), ctypes.c_double(), (ctypes.c_int32 * 5)()
    L.devlib_read_token.restype = ctypes.c_long
    if L.devlib_read_token(b, len(b), ctypes.byref(iv), ctypes.byref(fv), out) < 0:
        return None
    ty, hdr, ln = TOK_TYPES[out[0]], out[3], out[2]
    return {"type": ty, "int": iv.value, "float": fv.value, "bool": bool(out[1]),
            "size": ln if ty in ("MAP", "ARRAY") else 0,
            "value": b[hdr:hdr + ln] if ty in ("STRING", "BINARY") else None, "consumed": out[4]}


def test_tokenizer_oracle(vectors):
    for v in vectors["jsonpath_tokens"]:
        assert [list(t) for t in zbref.jp_tokens(v["expr"])] == v["tokens"], v["expr"]


def test_compiler_filter_instances(vectors, devlib):  # noqa: F811
    for v in vectors["jsonpath_compile"]:
        got, err = zbref.jp_compile(v["expr"])
        assert err is None and [f[0] for f in got] == v["filter_ids"], (v, got, err)
        ids, err = dev_compile(devlib, v["expr"])
        assert err is None and ids == v["filter_ids"], (v, ids, err)


def test_compiler_rejects_invalid_paths(vectors, devlib):  # noqa: F811
    for v in vectors["jsonpath_invalid"]:
        got, err = zbref.jp_compile(v["expr"])
        assert got is None and err == (v["position"], v["error"]), (v, err)
        # (the product reports the reason -- a deployment fails with it -- not the position)
        ids, msg = dev_compile(devlib, v["expr"])
        assert ids is None and msg == v["error"], (v, msg)


def test_query_results(vectors, devlib):  # noqa: F811
    for v in vectors["queries"]:
        doc = bytes.fromhex(v["doc"])
        res = [tuple(r) for r in v["results"]]
        assert zbref.query_positions(v["path"], doc) == res, v
        n, first = dev_query(devlib, v["path"], doc)
        assert n == len(res), (v, n)
        if res:
            assert first == res[0], (v, first)
        if "value" in v:
            assert doc[res[0][0]:res[0][0] + res[0][1]].hex() == v["value"], v
        if "type" in v:  # QueryResult.isString / isLong ... as the product's reader types the single result
            t = dev_token(devlib, doc[first[0]:first[0] + first[1]])
            assert t["type"] == v["type"], (v, t)
            if "long_buffer" in v:  # getLongAsBuffer: 8 bytes, native order (k_subscribe's integer correlation key)
                assert struct.pack("<q", t["int"]).hex() == v["long_buffer"], v


def test_traversal_stops_at_unsupported_token(vectors, devlib):  # noqa: F811
    for v in vectors["traversal_errors"]:
        doc = bytes.fromhex(v["doc"])
        assert zbref.traverse(doc) == (False, (v["position"], v["error"]))
        assert dev_token(devlib, doc[:v["position"]]) is not None
        assert dev_token(devlib, doc[v["position"]:]) is None  # the kernels' reader refuses the same token
        assert zbref.read_token(doc[v["position"]:]) == v["error"]


@pytest.mark.parametrize("side", ["oracle", "product"])
def test_read_token(vectors, devlib, side):  # noqa: F811
    for v in vectors["read_tokens"]:
        b = bytes.fromhex(v["bytes"])
        t = zbref.read_token(b) if side == "oracle" else dev_token(devlib, b)
        assert isinstance(t, dict), (v, t)
        assert t["type"] == v["type"] and t["consumed"] == len(b), (v, t)
        for k in ("int", "size", "bool", "float"):
            if k in v:
                assert t[k] == v[k], (v["name"], k, t[k], v[k])
        if "value" in v:
            assert t["value"].hex() == v["value"], (v, t)
