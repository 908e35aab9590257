"""Pin the payload tree -- the oracle's restatement (oracle/zbref_mapping.hpp) AND the product's exact tree
(zeebe_amd/csrc/zb_xmerge.hpp, built for the host by tests/native/devlib_host.cpp) -- on the reference's own tree
tests, transcribed into tests/golden/reference_vectors.json (`trees`, `tree_writes`) by
tests/golden/make_reference_vectors.py:

  json-path/src/test/java/io/zeebe/msgpack/mapping/MsgPackDocumentIndexerTest.java:47-223  (node ids, child sets,
                                                                                            leaf bytes)
  json-path/.../mapping/MsgPackDocumentExtractorTest.java:41-219                           (extraction trees, error)
  json-path/.../mapping/MsgPackTreeTest.java:36-84                                          (through the extractor)
  json-path/.../mapping/MsgPackDocumentTreeWriterTest.java:33-70                            (index + write)

Before this file the exact tree was only fuzzed against the oracle, both being restatements of the same Java; the
assertions here are the reference's. CPU only.
"""
import ctypes
import json
import os

import msgpack
import pytest

from oracle import zbref
from test_devlib_host import devlib  # noqa: F401

HERE = os.path.dirname(os.path.abspath(__file__))


def dev_tree(L, doc, mappings=None):
    spec = "".join("%s\t%s\n" % tuple(m) for m in (mappings or [])).encode()
    L.devlib_xtree_dump.restype = ctypes.c_long
    L.devlib_xtree_dump.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p,
                                    ctypes.c_uint32]
    mode = 1 if mappings else 0
    n = L.devlib_xtree_dump(doc, len(doc), spec, mode, None, 0)
    if n < 0:
        return n
    buf = ctypes.create_string_buffer(n)
    L.devlib_xtree_dump(doc, len(doc), spec, mode, buf, n)
    return zbref.parse_tree_dump(buf.raw[:n])


def check(tree, expect, ctx):
    for kind, nid, want in expect:
        assert nid in tree, (ctx, nid, sorted(tree))
        ty, children, leaf = tree[nid]
        if kind == "leaf":  # assertThatIsLeafNode: isLeaf(id) and writeLeafMapping's bytes
            assert leaf is not None and leaf.hex() == want, (ctx, nid, leaf, want)
        else:  # assertThatIsMapNode / assertThatIsArrayNode: the type and the child set
            assert ty == {"map": "M", "array": "A"}[kind], (ctx, nid, ty)
            assert len(children) == len(want) and set(children) == set(want), (ctx, nid, children, want)


def test_trees_oracle(vectors):
    for v in vectors["trees"]:
        doc = bytes.fromhex(v["doc"])
        ms = [tuple(m) for m in v["mappings"]] if v["mappings"] else None
        if "error" in v:
            with pytest.raises(RuntimeError, match=v["error"]):
                zbref.tree(doc, ms)
            continue
        check(zbref.tree(doc, ms), v["expect"], v["src"])


def test_trees_exact_tree(vectors, devlib):  # noqa: F811
    for v in vectors["trees"]:
        doc = bytes.fromhex(v["doc"])
        ms = v["mappings"]
        got = dev_tree(devlib, doc, ms)
        if "error" in v:  # IllegalStateException (not a MappingException): X_FAIL, the processor fails
            assert got == -101, (v["src"], got)
            continue
        assert isinstance(got, dict), (v["src"], got)
        check(got, v["expect"], v["src"])
        # and node for node the oracle's tree: types, child order (LinkedHashSet), leaf bytes
        assert got == zbref.tree(doc, [tuple(m) for m in ms] if ms else None), v["src"]


def test_tree_writer_round_trip(vectors, devlib):  # noqa: F811
    for v in vectors["tree_writes"]:
        with open(os.path.join(HERE, "golden", v["json_file"]), "rb") as f:
            js = json.loads(f.read())
        doc = msgpack.packb(js)
        assert len(doc) > 64  # (shouldWriteMsgPackTreeWhenWriterHasSmallInitSize)
        ref = zbref.merge(doc, b"")  # MappingProcessor.extract without mappings: index, then write the tree
        assert len(ref) == len(doc) and msgpack.unpackb(ref) == js
        out = ctypes.create_string_buffer(1 << 16)
        fq, err = ctypes.c_uint32(), ctypes.create_string_buffer(256)
        devlib.devlib_xmerge.restype = ctypes.c_long
        n = devlib.devlib_xmerge(doc, len(doc), b"", 0, b"", 0, out, 1 << 16, ctypes.byref(fq), err, 256, -1)
        assert n == len(doc) and out.raw[:n] == ref
