"""The PRODUCT's json-el / json-path compiler and condition VM pinned on the reference's own vectors.

tests/golden/reference_vectors.json holds the reference's known answers (JsonConditionInterpreterTest
:35-93, JsonConditionTest :34-141, JsonConditionParserTest :29-58, JsonConditionParserFailureMessageTest
:33-49). Here they go through the product, not the oracle:

* CPU (not gpu): every valid expression deploys and every invalid one is rejected by the product's
  deployment transformer (zb_validate_deployment: the same code zb_deploy runs);
* GPU: one exclusive gateway per expression, one workflow instance per vector document; the branch
  taken by the device VM (or the CONDITION_ERROR incident and its message) must be the reference's
  expected result -- and the whole log bit-exact against the oracle.
"""
import msgpack
import pytest

from zeebe_amd import bpmn, engine


def gateway_model(expr: str, pid: str = "cond"):
    """start -> xor {flow "t" [expr] -> end "et"; default "f" -> end "ef"}: EXCLUSIVE_SPLIT binding."""
    b = bpmn.Bpmn.create_executable_process(pid).start_event("s").exclusive_gateway("x")
    b.sequence_flow_id("t").condition(expr).end_event("et")
    return b.move_to_node("x").default_flow().sequence_flow_id("f").end_event("ef").done()


def test_product_accepts_reference_valid_expressions(vectors):
    exprs = set(vectors["parser_valid"]) | {v["expr"] for v in vectors["conditions"]} | \
        {v["expr"] for v in vectors["condition_errors"]}
    for expr in sorted(exprs):
        rc, msg = engine.validate_deployment(gateway_model(expr).to_xml())
        assert rc in (engine.ZB_OK, engine.ZB_EUNSUPPORTED), (expr, rc, msg)
        if rc == engine.ZB_EUNSUPPORTED:  # only the documented refusal (|integer constant| >= 2^53)
            assert "2^53" in msg, (expr, msg)


def test_product_rejects_reference_invalid_expressions(vectors):
    for expr, ref_msg in vectors["parser_failures"]:
        if expr == "":
            continue  # an empty <conditionExpression/> is no condition at all in the BPMN resource
        rc, msg = engine.validate_deployment(gateway_model(expr).to_xml())
        assert rc == engine.ZB_EDEPLOY, (expr, rc, msg)
        # the reference's failure message (scala-parser-combinators: furthest failure, later at a tie)
        assert msg.startswith(ref_msg), (expr, ref_msg, msg)


def test_product_string_literal_lexing():
    """JavaTokenParsers.stringLiteral / the single-quoted alternative: control characters, unknown escapes
    and a double quote inside single quotes are rejected; the legal escapes are kept raw."""
    ok = ["$.a == 'x\\\\y'", "$.a == 'x\\ty'", '$.a == "it\'s"', "$.a == 'u\\u00e9'", '$.a == "q\\"q"']
    bad = ["$.a == 'x\\qy'", "$.a == 'a\"b'", "$.a == 'x\x01y'", '$.a == "x\x7fy"', "$.a == 'u\\u00g9'"]
    for expr in ok:
        rc, msg = engine.validate_deployment(gateway_model(expr).to_xml())
        assert rc == engine.ZB_OK, (expr, msg)
    for expr in bad:
        if "\x01" in expr or "\x7f" in expr:
            # not representable in XML 1.0 text: build the resource with a character reference
            xml = gateway_model("$.a == 'PLACEHOLDER'").to_xml().replace("PLACEHOLDER", expr[8:-1].replace(
                "\x01", "&#1;").replace("\x7f", "&#127;"))
        else:
            xml = gateway_model(expr).to_xml()
        rc, msg = engine.validate_deployment(xml)
        assert rc == engine.ZB_EDEPLOY, (expr, rc, msg)


def _by_expr(vectors):
    groups = {}
    for v in vectors["conditions"] + vectors["condition_errors"]:
        groups.setdefault(v["expr"], []).append(v)
    return groups


@pytest.mark.gpu
def test_device_vm_on_reference_vectors(vectors):
    from oracle import zbref
    from zeebe_amd.engine import Engine

    groups = _by_expr(vectors)
    checked = 0
    for gi, (expr, vs) in enumerate(sorted(groups.items())):
        xml = gateway_model(expr).to_xml()
        rc, msg = engine.validate_deployment(xml)
        if rc == engine.ZB_EUNSUPPORTED:
            continue
        e = Engine(log_capacity=1 << 14, row_capacity=1 << 12, arena_bytes=8 << 20, wave_only=(gi % 2 == 1))
        e.deploy(xml, 100, 1)
        o = zbref.Oracle()
        o.deploy(xml, 100, 1)
        docs = [bytes.fromhex(v["doc"]) for v in vs]
        e.create("cond", docs)
        for d in docs:
            o.create("cond", d)
        assert e.step()["quiescent"]
        o.run()
        got, ref = e.records(), o.records()
        assert [(r.key, r.record_type, r.value_type, r.intent, r.value) for r in got] == \
               [(r.key, r.record_type, r.value_type, r.intent, r.value) for r in ref], expr
        # per instance: the end event reached, or the incident raised
        outcome = {}
        for r in got:
            v = msgpack.unpackb(r.value, raw=False)
            if r.value_type == 5 and r.intent == 3:  # END_EVENT_OCCURRED
                outcome[v["workflowInstanceKey"]] = v["activityId"] == "et"
            elif r.value_type == 6:  # IncidentIntent.CREATE
                outcome[v["workflowInstanceKey"]] = ("error", v["errorMessage"])
        for i, v in enumerate(vs):
            res = outcome[1 + 5 * i]
            if "error" in v:
                assert res[0] == "error" and v["error"] in res[1], (expr, v, res)
            else:
                assert res == v["expected"], (expr, v, res)
            checked += 1
        e.close()
    assert checked >= 60
