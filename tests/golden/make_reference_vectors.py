"""Generate tests/golden/reference_vectors.json: the reference's own known-answer vectors.

Every expected value below is TRANSCRIBED from the reference test named next to it (inputs are
re-encoded with python-msgpack the way the reference tests encode them with Jackson's msgpack
mapper: minimal ints, float64 doubles, str keys). Nothing here is produced by running the oracle;
the oracle is checked against this file (tests/test_oracle_golden.py) and then serves as the
checker of the GPU engine.

Run:  python tests/golden/make_reference_vectors.py
"""
import json
import math
import os
import sys

import msgpack

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from zeebe_amd import bpmn  # noqa: E402


def mp(obj) -> str:
    return msgpack.packb(obj, use_bin_type=True).hex()


def jl(s: str):
    """The reference tests write JSON with single quotes (JSON_MAPPER ALLOW_SINGLE_QUOTES)."""
    return json.loads(s.replace("'", '"'))


def conditions():
    # json-el/src/test/java/io/zeebe/msgpack/el/JsonConditionInterpreterTest.java:35-93
    nan, inf = float("nan"), float("inf")
    v = [
        ("$.foo == 'bar'", {"foo": "bar"}, True), ("$.foo == 'bar'", {"foo": "baz"}, False),
        ("$.foo == true", {"foo": True}, True), ("$.foo == true", {"foo": False}, False),
        ("$.foo == 3", {"foo": 3}, True), ("$.foo == 3", {"foo": 4}, False),
        ("$.foo == 2.5", {"foo": 2.5}, True), ("$.foo == 2.5", {"foo": 2.6}, False),
        ("$.foo == 2", {"foo": 2.0}, True), ("$.foo == 2.0", {"foo": 2}, True),
        ("$.foo == null", {"foo": None}, True), ("$.foo == null", {"foo": "bar"}, False),
        ("$.foo == $.bar", {"foo": "a", "bar": "a"}, True), ("$.foo == $.bar", {"foo": "a", "bar": "b"}, False),
        ("$.foo != 'bar'", {"foo": "baz"}, True), ("$.foo != 'bar'", {"foo": "bar"}, False),
        ("$.foo != null", {"foo": "bar"}, True), ("$.foo != null", {"foo": None}, False),
        ("$.foo < 5", {"foo": 4}, True), ("$.foo < 5", {"foo": 5}, False),
        ("$.foo <= 5", {"foo": 5}, True), ("$.foo <= 5", {"foo": 6}, False),
        ("$.foo <= 5.0", {"foo": 4.8}, True), ("$.foo <= 5.0", {"foo": 5}, True),
        ("$.foo <= 5.0", {"foo": 5.1}, False),
        ("$.foo > 5", {"foo": 6}, True), ("$.foo > 5", {"foo": 5}, False),
        ("$.foo >= 5", {"foo": 5}, True), ("$.foo >= 5", {"foo": 4}, False),
        ("$.foo < $.bar", {"foo": 1, "bar": 2}, True), ("$.foo < $.bar", {"foo": 2, "bar": 2}, False),
        ("$.foo == 1 || $.foo == 2", {"foo": 1}, True), ("$.foo == 1 || $.foo == 2", {"foo": 2}, True),
        ("$.foo == 1 || $.foo == 2", {"foo": 3}, False),
        ("$.foo == 1 || $.foo == 2 || $.foo == 3", {"foo": 3}, True),
        ("$.foo == 1 || $.foo == 2 || $.foo == 3", {"foo": 4}, False),
        ("$.foo > 2 && $.foo > 3", {"foo": 4}, True), ("$.foo > 2 && $.foo > 3", {"foo": 3}, False),
        ("$.foo > 2 && $.foo > 3", {"foo": 2}, False),
        ("$.foo > 2 && $.foo > 3 && $.foo > 4", {"foo": 5}, True),
        ("$.foo > 2 && $.foo > 3 && $.foo > 4", {"foo": 4}, False),
        ("$.foo == 1 || $.foo > 2 && $.foo > 3", {"foo": 4}, True),
        ("$.foo == 1 || $.foo > 2 && $.foo > 3", {"foo": 1}, True),
        ("$.foo == 1 || $.foo > 2 && $.foo > 3", {"foo": 2}, False),
        ("$.foo == 1 || $.foo > 2 && $.foo > 3", {"foo": 3}, False),
        ("($.foo == 1 || $.foo > 2) && $.foo > 3", {"foo": 4}, True),
        ("($.foo == 1 || $.foo > 2) && $.foo > 3", {"foo": 1}, False),
        ("($.foo == 1 || $.foo > 2) && $.foo > 3", {"foo": 2}, False),
        ("($.foo == 1 || $.foo > 2) && $.foo > 3", {"foo": 3}, False),
        ("$.foo < 5", {"foo": nan}, False), ("$.foo > 5", {"foo": nan}, False),
        ("$.foo < 5", {"foo": inf}, False), ("$.foo > 5", {"foo": inf}, True),
        ("$.foo < 5", {"foo": -inf}, True), ("$.foo > 5", {"foo": -inf}, False),
    ]
    return [{"expr": e, "doc": mp(d), "expected": r} for e, d, r in v]


def condition_errors():
    # json-el/src/test/java/io/zeebe/msgpack/el/JsonConditionTest.java:34-141
    return [
        {"expr": "$.foo == $.bar || $.foo > 2 || $.bar <= 2", "doc": mp({"foo": 2, "bar": 2}), "expected": True},
        {"expr": "$.foo == $.bar || $.foo > 2 || $.bar <= 2", "doc": mp({"foo": 2, "bar": 3}), "expected": False},
        {"expr": "$.foo > 3", "doc": mp({"foo": "bar"}),
         "error": "Cannot compare values of different types: STRING and INTEGER"},
        {"expr": "$.foo > 3", "doc": mp({"bar": 4}), "error": "JSON path '$.foo' has no result"},
        {"expr": "$.foo > 3", "doc": mp({"foo": None}),
         "error": "Cannot compare values of different types: NIL and INTEGER"},
        {"expr": "$.foo == $.bar", "doc": mp({"foo": [1, 2, 3], "bar": [4, 5, 6]}),
         "error": "Cannot compare value of type: ARRAY"},
        {"expr": "$.foo == $.bar", "doc": mp({"foo": {"a": 1}, "bar": {"b": 2}}),
         "error": "Cannot compare value of type: MAP"},
        {"expr": "$.foo < $.bar", "doc": mp({"foo": "a", "bar": "b"}),
         "error": "Cannot compare values. Expected number but found: STRING"},
    ]


def parser_valid():
    # json-el/src/test/java/io/zeebe/msgpack/el/JsonConditionParserTest.java:29-58
    return ["$.foo == 'bar'", '$.foo == "bar"', "$.foo == true", "$.foo == 21", "$.foo == 2.5", "$.foo == $.bar",
            "$.foo.bar == true", "$.foo[1] == true", "'foo' == 'bar'", "$.foo != 'bar'", "$.foo < 100",
            "$.foo <= -100", "$.foo > 2.5", "$.foo >= 2.5", "$.foo >= .5", "$.foo >= -.5", "$.foo >= $.bar",
            "2 < 4", "$.foo > 2 && $.foo < 4", "$.foo > 2 && $.foo < 4 && $.bar > 12", "$.foo > 2 || $.bar < 4",
            "$.foo > 2 || $.bar < 4 || $.foobar == 21", "$.foo > 2 && $.foo < 4 || $.bar == 6", "($.foo == 2)",
            "$.foo > 2 && ($.foo < 4 || $.bar == 6)"]


def parser_failures():
    # json-el/src/test/java/io/zeebe/msgpack/el/JsonConditionParserFailureMessageTest.java:33-49
    # and JsonConditionTest.shouldReportParseFailure (:61-68)
    return [
        ["", "expression is empty"],
        ["foo", "expected comparison, disjunction or conjunction."],
        ["$.foo", "expected comparison operator ('==', '!=', '<', '<=', '>', '>=')"],
        ["$.foo ==", "expected literal (JSON path, string, number, boolean, null)"],
        ["$.foo < 'bar'", "expected number or JSON path"],
        ["$.foo < true", "expected number or JSON path"],
        ["$.foo == { 'a': 2 }", "expected literal (JSON path, string, number, boolean, null)"],
        ["$.foo == [1, 2, 3]", "expected literal (JSON path, string, number, boolean, null)"],
        ["$.foo + 3", "expected comparison operator ('==', '!=', '<', '<=', '>', '>=')"],
        ["$.foo or $.bar", "expected comparison operator ('==', '!=', '<', '<=', '>', '>=')"],
        ["$.foo < 3 &&", "expected comparison"],
        ["$.foo < 3 ||", "expected comparison"],
        ["($.foo < 3", "`)' expected but end of source found"],
        ["$.foo.. < 3", "Unexpected json-path"],
        ["$.foo < NaN", "expected number or JSON path"],
        ["$.foo < Infinity", "expected number or JSON path"],
        ["$.foo < -Infinity", "expected number or JSON path"],
    ]


def merges():
    # json-path/src/test/java/io/zeebe/msgpack/mapping/MappingMergeParameterizedTest.java:42-180
    # (the rows whose mapping column is null = default top-level merge; compared as JSON trees)
    nested = ("{'arr':[{'obj':{'value':'x', 'otherArr':[{'test':'hallo'}, {'obj':{'arr':[0, 1]}} ]}}, "
              "{'otherValue':1}], 'ab':{'b':{'value':'y'}}}")
    rows = [
        ("{'hallo':'twsewas','int':1}", "{'foo':'bar','int':3}", "{'hallo':'twsewas','foo':'bar','int':1}"),
        ("{'foo':'bar','int':1,'obj':{'test':'ok'},'array':[1,2,3]}",
         "{'foo':'bar','int':3,'obj':{'test':'ok'},'array':[1],'test':'value'}",
         "{'foo':'bar','int':1,'obj':{'test':'ok'},'array':[1,2,3],'test':'value'}"),
        (nested, "{'foo':'bar','int':3,'obj':{'test':'ok'},'array':[1],'test':'value'}",
         nested[:-1] + ",'foo':'bar','int':3,'obj':{'test':'ok'},'array':[1],'test':'value'}"),
        (nested, "{'foo':'bar','int':3,'ab':{'c':{'value':'z'}},'array':[1],'test':'value'}",
         nested[:-1] + ",'foo':'bar','int':3,'array':[1],'test':'value'}"),
        # MappingMergeTest.shouldMergeTwiceWithoutMappings :181-220
        ("{'test':'thisValue'}", "{'arr':[0, 1], 'obj':{'int':1}, 'test':'value'}",
         "{'arr':[0, 1], 'obj':{'int':1}, 'test':'thisValue'}"),
        ("{'other':[2, 3]}", "{'arr':[0, 1], 'obj':{'int':1}, 'test':'thisValue'}",
         "{'arr':[0, 1], 'obj':{'int':1}, 'test':'thisValue', 'other':[2, 3]}"),
    ]
    out = [{"source": mp(jl(s)), "target": mp(jl(t)), "expected_json": jl(e)} for s, t, e in rows]
    # MappingMergeTest :221-264 byte-exact nil / empty cases
    out += [
        {"source": "c0", "target": "80", "expected_hex": "80"},
        {"source": "80", "target": "c0", "expected_hex": "80"},
        {"source": "c0", "target": "c0", "expected_hex": "c0"},
    ]
    # WorkflowTaskIOMappingTest.shouldUseWFPayloadIfCompleteWithNoPayload :569-590 (byte exact) and
    # MsgPackUtil.JSON_DOCUMENT/OTHER_DOCUMENT/MERGED_OTHER_WITH_JSON_DOCUMENT
    # (broker-core/src/test/java/io/zeebe/broker/test/MsgPackUtil.java:31-34)
    jd = jl("{'string':'value', 'jsonObject':{'testAttr':'test'}}")
    od = jl("{'string':'bar', 'otherObject':{'testAttr':'test'}}")
    out += [
        {"source": "80", "target": mp(jd), "expected_hex": mp(jd)},
        {"source": mp(od), "target": mp(jd),
         "expected_json": jl("{'string':'bar', 'jsonObject':{'testAttr':'test'}, 'otherObject':{'testAttr':'test'}}")},
        {"source": mp(jd), "target": mp(jd), "expected_json": jd},
    ]
    return out


def writer():
    # msgpack-core/src/test/java/io/zeebe/msgpack/spec/MsgPackWriterTest.java:43-120
    ints = [(5, "05"), ((1 << 8) - 1, "ccff"), ((1 << 16) - 1, "cdffff"), ((1 << 32) - 1, "ceffffffff"),
            ((1 << 63) - 1, "cf7fffffffffffffff"), (-(1 << 7), "d080"), (-(1 << 15), "d18000"),
            (-(1 << 31), "d280000000"), (-(1 << 63), "d38000000000000000"), (-1, "ff"), (-32, "e0"),
            (-33, "d0df"), (127, "7f"), (128, "cc80")]
    floats = [(123.0, "ca42f60000"), (1.7976931348623157e308, "cb7fefffffffffffff")]
    return {"ints": ints, "floats": floats}


def hashes():
    # protocol/src/test/java/io/zeebe/protocol/SubscriptionUtilTest.java:29-43
    return [["a", 97], ["b", 98], ["c", 99], ["", 0]]


WF = {"CREATE": 0, "CREATED": 1, "START_EVENT_OCCURRED": 2, "END_EVENT_OCCURRED": 3, "SEQUENCE_FLOW_TAKEN": 4,
      "GATEWAY_ACTIVATED": 5, "ELEMENT_READY": 6, "ELEMENT_ACTIVATED": 7, "ELEMENT_COMPLETING": 8,
      "ELEMENT_COMPLETED": 9, "ELEMENT_TERMINATING": 10, "ELEMENT_TERMINATED": 11, "CANCEL": 12, "CANCELING": 13,
      "UPDATE_PAYLOAD": 14, "PAYLOAD_UPDATED": 15}


def workflows():
    B = bpmn.Bpmn
    out = []
    # WorkflowInstanceFunctionalTest.testWorkflowInstanceStatesWithServiceTask :518-556
    m = (B.create_executable_process("process").start_event("a").service_task("b", type="foo")
         .end_event("c").done())
    out.append({"name": "states_with_service_task", "xml": m.to_xml(), "process": "process",
                "instances": [{"payload": "80"}], "job_payloads": {},
                "expect_wf_intents": ["CREATE", "CREATED", "ELEMENT_READY", "ELEMENT_ACTIVATED",
                                      "START_EVENT_OCCURRED", "SEQUENCE_FLOW_TAKEN", "ELEMENT_READY",
                                      "ELEMENT_ACTIVATED", "ELEMENT_COMPLETING", "ELEMENT_COMPLETED",
                                      "SEQUENCE_FLOW_TAKEN", "END_EVENT_OCCURRED", "ELEMENT_COMPLETING",
                                      "ELEMENT_COMPLETED"]})
    # :558-597
    m = (B.create_executable_process("workflow").start_event().exclusive_gateway("xor")
         .sequence_flow_id("s1").condition("$.foo < 5").end_event("a").move_to_last_exclusive_gateway()
         .default_flow().sequence_flow_id("s2").end_event("b").done())
    out.append({"name": "states_with_exclusive_gateway", "xml": m.to_xml(), "process": "workflow",
                "instances": [{"payload": mp({"foo": 4})}], "job_payloads": {},
                "expect_wf_intents": ["CREATE", "CREATED", "ELEMENT_READY", "ELEMENT_ACTIVATED",
                                      "START_EVENT_OCCURRED", "SEQUENCE_FLOW_TAKEN", "GATEWAY_ACTIVATED",
                                      "SEQUENCE_FLOW_TAKEN", "END_EVENT_OCCURRED", "ELEMENT_COMPLETING",
                                      "ELEMENT_COMPLETED"]})
    # shouldSpitOnExclusiveGateway :351-393 (end event reached per payload)
    m = (B.create_executable_process("workflow").start_event().exclusive_gateway("xor")
         .sequence_flow_id("s1").condition("$.foo < 5").end_event("a").move_to_last_gateway()
         .sequence_flow_id("s2").condition("$.foo >= 5 && $.foo < 10").end_event("b")
         .move_to_last_exclusive_gateway().default_flow().sequence_flow_id("s3").end_event("c").done())
    out.append({"name": "split_on_exclusive_gateway", "xml": m.to_xml(), "process": "workflow",
                "instances": [{"payload": mp({"foo": 4})}, {"payload": mp({"foo": 8})},
                              {"payload": mp({"foo": 12})}], "job_payloads": {},
                "expect_end_event": ["a", "b", "c"]})
    # shouldJoinOnExclusiveGateway :395-442 (flows taken per instance)
    m = (B.create_executable_process("workflow").start_event().exclusive_gateway("split")
         .sequence_flow_id("s1").condition("$.foo < 5").exclusive_gateway("joinRequest")
         .move_to_last_exclusive_gateway().default_flow().sequence_flow_id("s2").connect_to("joinRequest")
         .end_event("end").done())
    out.append({"name": "join_on_exclusive_gateway", "xml": m.to_xml(), "process": "workflow",
                "instances": [{"payload": mp({"foo": 4})}, {"payload": mp({"foo": 8})}], "job_payloads": {},
                "expect_flows_contain": [["s1"], ["s2"]], "expect_flows_exclude": [["s2"], ["s1"]]})
    # EmbeddedSubProcessTest.shouldCompleteEmbeddedSubProcess :132-165 (+ scope keys :123-128)
    sp = (B.create_executable_process("process").start_event("start").sequence_flow_id("flow1")
          .sub_process("subProcess"))
    (sp.embedded_sub_process().start_event("subProcessStart").sequence_flow_id("subProcessFlow1")
     .service_task("subProcessTask", type="type").sequence_flow_id("subProcessFlow2").end_event("subProcessEnd"))
    m = sp.sequence_flow_id("flow2").end_event("end").done()
    seq = [("CREATED", "process"), ("ELEMENT_READY", "process"), ("ELEMENT_ACTIVATED", "process"),
           ("START_EVENT_OCCURRED", "start"), ("SEQUENCE_FLOW_TAKEN", "flow1"), ("ELEMENT_READY", "subProcess"),
           ("ELEMENT_ACTIVATED", "subProcess"), ("START_EVENT_OCCURRED", "subProcessStart"),
           ("SEQUENCE_FLOW_TAKEN", "subProcessFlow1"), ("ELEMENT_READY", "subProcessTask"),
           ("ELEMENT_ACTIVATED", "subProcessTask"), ("ELEMENT_COMPLETING", "subProcessTask"),
           ("ELEMENT_COMPLETED", "subProcessTask"), ("SEQUENCE_FLOW_TAKEN", "subProcessFlow2"),
           ("END_EVENT_OCCURRED", "subProcessEnd"), ("ELEMENT_COMPLETING", "subProcess"),
           ("ELEMENT_COMPLETED", "subProcess"), ("SEQUENCE_FLOW_TAKEN", "flow2"), ("END_EVENT_OCCURRED", "end"),
           ("ELEMENT_COMPLETING", "process"), ("ELEMENT_COMPLETED", "process")]
    out.append({"name": "embedded_sub_process", "xml": m.to_xml(), "process": "process",
                "instances": [{"payload": mp({"key": "val"})}], "job_payloads": {},
                "expect_wf_events": [list(x) for x in seq],
                "expect_scope_checks": True})
    # shouldCompleteNestedSubProcess :293-344
    outer = B.create_executable_process("process").start_event().sub_process("outerSubProcess")
    inner_start = outer.embedded_sub_process().start_event()
    inner_sp = inner_start.sub_process("innerSubProcess")
    inner_sp.embedded_sub_process().start_event().service_task("task", type="type").end_event()
    inner_sp.end_event()
    m = outer.end_event().done()
    seq = [("ELEMENT_READY", "outerSubProcess"), ("ELEMENT_ACTIVATED", "outerSubProcess"),
           ("ELEMENT_READY", "innerSubProcess"), ("ELEMENT_ACTIVATED", "innerSubProcess"),
           ("ELEMENT_READY", "task"), ("ELEMENT_ACTIVATED", "task"), ("ELEMENT_COMPLETING", "task"),
           ("ELEMENT_COMPLETED", "task"), ("ELEMENT_COMPLETING", "innerSubProcess"),
           ("ELEMENT_COMPLETED", "innerSubProcess"), ("ELEMENT_COMPLETING", "outerSubProcess"),
           ("ELEMENT_COMPLETED", "outerSubProcess")]
    out.append({"name": "nested_sub_process", "xml": m.to_xml(), "process": "process",
                "instances": [{"payload": "80"}], "job_payloads": {},
                "expect_filtered_events": [list(x) for x in seq],
                "filter_ids": ["innerSubProcess", "outerSubProcess", "task"]})
    # WorkflowTaskIOMappingTest.shouldNotSeePayloadOfWorkflowInstanceBefore :462-495
    jd = jl("{'string':'value', 'jsonObject':{'testAttr':'test'}}")
    m = (B.create_executable_process("process").start_event().service_task("service", type="external")
         .end_event().done())
    out.append({"name": "io_payload_isolation", "xml": m.to_xml(), "process": "process",
                "instances": [{"payload": mp(jd), "job_payload": mp(jd)},
                              {"payload": "80", "job_payload": mp({"foo": "bar"})}],
                "expect_task_completed_payload_json": [jd, {"foo": "bar"}]})
    # shouldUseWFPayloadIfCompleteWithNoPayload :569-590 (byte exact)
    out.append({"name": "io_no_job_payload_byte_exact", "xml": m.to_xml(), "process": "process",
                "instances": [{"payload": mp(jd), "job_payload": "80"}],
                "expect_task_completed_payload_hex": [mp(jd)]})
    return out


def cancels():
    """CancelWorkflowInstanceTest.java:49-260: workflow events from the CANCEL command on, as (activityId,
    intent); activityId None for the command. The instance is cancelled while its task waits for a job
    (job_created: the job stream processor has written JOB CREATED first) or its catch event waits."""
    B = bpmn.Bpmn
    wf = (B.create_executable_process("process").start_event().service_task("task", type="test", retries=5)
          .end_event().done())
    sp = B.create_executable_process("process").start_event().sub_process("subProcess")
    sp.embedded_sub_process().start_event().service_task("task", type="test", retries=5).end_event()
    sub = sp.end_event().done()
    catch = (B.create_executable_process("wf").start_event()
             .intermediate_catch_event("catch-event", message="msg", correlation_key="$.id").done())
    C = "CANCEL"
    return [
        # shouldCancelWorkflowInstance :81-124
        {"name": "cancel_workflow_instance", "xml": wf.to_xml(), "process": "process", "payload": "80",
         "job_created": False,
         "expect": [[None, C], ["process", "CANCELING"], ["process", "ELEMENT_TERMINATING"],
                    ["task", "ELEMENT_TERMINATING"], ["task", "ELEMENT_TERMINATED"],
                    ["process", "ELEMENT_TERMINATED"]]},
        # shouldCancelWorkflowInstanceWithEmbeddedSubProcess :126-156
        {"name": "cancel_with_embedded_sub_process", "xml": sub.to_xml(), "process": "process", "payload": "80",
         "job_created": False,
         "expect": [[None, C], ["process", "CANCELING"], ["process", "ELEMENT_TERMINATING"],
                    ["subProcess", "ELEMENT_TERMINATING"], ["task", "ELEMENT_TERMINATING"],
                    ["task", "ELEMENT_TERMINATED"], ["subProcess", "ELEMENT_TERMINATED"],
                    ["process", "ELEMENT_TERMINATED"]]},
        # shouldCancelIntermediateCatchEvent :184-214 (TERMINATED's source = TERMINATING's position)
        {"name": "cancel_intermediate_catch_event", "xml": catch.to_xml(), "process": "wf",
         "payload": mp({"id": "123"}), "job_created": False,
         "expect": [[None, C], ["wf", "CANCELING"], ["wf", "ELEMENT_TERMINATING"],
                    ["catch-event", "ELEMENT_TERMINATING"], ["catch-event", "ELEMENT_TERMINATED"],
                    ["wf", "ELEMENT_TERMINATED"]]},
        # shouldCancelJobForActivity :216-245: JOB CANCEL command (key = job key) written with the task's
        # TERMINATED, source = the task's TERMINATING; headers carry the instance / process / version / activity
        {"name": "cancel_job_for_activity", "xml": wf.to_xml(), "process": "process", "payload": "80",
         "job_created": True,
         "expect": [[None, C], ["process", "CANCELING"], ["process", "ELEMENT_TERMINATING"],
                    ["task", "ELEMENT_TERMINATING"], ["task", "ELEMENT_TERMINATED"],
                    ["process", "ELEMENT_TERMINATED"]],
         "expect_job_cancel_headers": {"bpmnProcessId": "process", "workflowDefinitionVersion": 1,
                                       "activityId": "task"}},
    ]



# ------------------------------------------------------------------------------ explicit io-mappings
REF = "/root/reference"
MAPPING_TESTS = "json-path/src/test/java/io/zeebe/msgpack/mapping"


class _JavaRows:
    """Reads the rows of a JUnit `parameters()` table (`new Object[][] { {...}, ... }`) from the reference
    test source: Java string literals (concatenated with +), null, createMapping(src, tgt),
    createMappings().mapping(src, tgt)...build(), and the largeJsonDocument.json resource."""

    def __init__(self, text, res_dir):
        self.s = text
        self.i = text.index("new Object[][]")
        self.i = text.index("{", self.i) + 1
        self.res_dir = res_dir

    def ws(self):
        while self.i < len(self.s):
            if self.s[self.i].isspace():
                self.i += 1
            elif self.s.startswith("//", self.i):
                self.i = self.s.index("\n", self.i)
            else:
                break

    def string(self):
        assert self.s[self.i] == '"'
        j = self.i + 1
        out = []
        while self.s[j] != '"':
            if self.s[j] == "\\":
                out.append(self.s[j + 1])
                j += 2
            else:
                out.append(self.s[j])
                j += 1
        self.i = j + 1
        return "".join(out)

    def value(self):
        self.ws()
        if self.s.startswith("null", self.i):
            self.i += 4
            return None
        if self.s[self.i] == '"':
            v = self.string()
            while True:
                self.ws()
                if self.s[self.i] == "+":
                    self.i += 1
                    self.ws()
                    v += self.string()
                else:
                    return v
        if self.s.startswith("createMappings()", self.i):
            self.i += len("createMappings()")
            ms = []
            while True:
                self.ws()
                if self.s.startswith(".mapping(", self.i):
                    self.i += len(".mapping(")
                    self.ws()
                    a = self.string()
                    self.ws(); assert self.s[self.i] == ","; self.i += 1; self.ws()
                    b = self.string()
                    self.ws(); assert self.s[self.i] == ")"; self.i += 1
                    ms.append([a, b])
                elif self.s.startswith(".build()", self.i):
                    self.i += len(".build()")
                    return ms
                else:
                    raise ValueError(self.s[self.i:self.i + 40])
        if self.s.startswith("createMapping(", self.i):
            self.i += len("createMapping(")
            self.ws()
            a = self.string()
            self.ws(); assert self.s[self.i] == ","; self.i += 1; self.ws()
            b = self.string()
            self.ws(); assert self.s[self.i] == ")"; self.i += 1
            return [[a, b]]
        if self.s.startswith("new String(", self.i):
            k = self.s.index('getResource("', self.i) + len('getResource("')
            name = self.s[k:self.s.index('"', k)]
            self.i = self.s.index(".toURI())))", self.i) + len(".toURI())))")
            with open(os.path.join(self.res_dir, name)) as f:
                return f.read()
        raise ValueError(self.s[self.i:self.i + 60])

    def rows(self):
        out = []
        while True:
            self.ws()
            if self.s[self.i] == "}":
                return out
            assert self.s[self.i] == "{", self.s[self.i:self.i + 40]
            self.i += 1
            row = []
            while True:
                row.append(self.value())
                self.ws()
                if self.s[self.i] == ",":
                    self.i += 1
                    self.ws()
                    if self.s[self.i] == "}":
                        self.i += 1
                        break
                    continue
                assert self.s[self.i] == "}", self.s[self.i:self.i + 40]
                self.i += 1
                break
            out.append(row)
            self.ws()
            if self.s[self.i] == ",":
                self.i += 1


def _java_rows(name):
    with open(os.path.join(REF, MAPPING_TESTS, name)) as f:
        text = f.read()
    return _JavaRows(text, os.path.join(REF, "json-path/src/test/resources/io/zeebe/msgpack/mapping")).rows()


def _tree(s):
    """JSON_MAPPER.readTree with ALLOW_SINGLE_QUOTES; Jackson ignores a trailing '}' after the root value."""
    return json.JSONDecoder().raw_decode(s.replace("'", '"'))[0]


def mapping_extracts():
    # json-path/src/test/java/io/zeebe/msgpack/mapping/MappingExtractParameterizedTest.java:40-230 (all rows),
    # MappingExtractTest.java:51-79 (exceptions), :81-113 (extract twice); compared as JSON trees
    out = [{"source": mp(_tree(src)), "mappings": ms or [], "expected_json": _tree(exp)}
           for src, ms, exp in _java_rows("MappingExtractParameterizedTest.java")]
    out += [
        {"source": "80", "mappings": [["$.foo", "$"]], "error": "No data found for query $.foo."},
        {"source": mp({"foo": "bar"}), "mappings": [["$.foo", "$"]],
         "error": "Processing failed, since mapping will result in a non map object (json object)."},
        {"source": mp(_tree("{'arr':[{'deepObj':{'value':123}}, 1], 'obj':{'int':1}, 'test':'value'}")),
         "mappings": [["$.arr[0]", "$"]], "expected_json": {"deepObj": {"value": 123}}},
        {"source": mp({"deepObj": {"value": 123}}), "mappings": [["$.deepObj", "$"]], "expected_json": {"value": 123}},
    ]
    return out


def mapping_merges():
    # json-path/src/test/java/io/zeebe/msgpack/mapping/MappingMergeParameterizedTest.java:40-420 (all rows;
    # the mapping-less ones are also in `merges`), MappingMergeTest.java:70-100 (exceptions)
    out = [{"source": mp(_tree(src)), "target": mp(_tree(tgt)), "mappings": ms or [], "expected_json": _tree(exp)}
           for src, tgt, ms, exp in _java_rows("MappingMergeParameterizedTest.java")]
    out += [
        {"source": "80", "target": "80", "mappings": [["$.foo", "$"]], "error": "No data found for query $.foo."},
        {"source": mp({"foo": "bar"}), "target": mp({"foo": "bar"}), "mappings": [["$.foo", "$"]],
         "error": "Processing failed, since mapping will result in a non map object (json object)."},
    ]
    return out


def io_workflows():
    # broker-core/src/test/java/io/zeebe/broker/workflow/WorkflowTaskIOMappingTest.java: start -> service task
    # "service" (type "external") -> end. create / complete payloads: MsgPackUtil.JSON_DOCUMENT (MSGPACK_PAYLOAD),
    # OTHER_DOCUMENT (OTHER_PAYLOAD); a completion without payload completes with {} . Expected: the JOB CREATE
    # payload, the task's ELEMENT_COMPLETED payload, or the incident's errorMessage (IO_MAPPING_ERROR).
    jd = "{'string':'value', 'jsonObject':{'testAttr':'test'}}"
    od = "{'string':'bar', 'otherObject':{'testAttr':'test'}}"
    merged = "{'string':'bar', 'jsonObject':{'testAttr':'test'}, 'otherObject':{'testAttr':'test'}}"
    rows = [
        # name, inputs, outputs, behavior, create, complete, job payload, completed payload, incident
        ("shouldCreateTwoNewObjectsViaInputMapping :90-113", [["$.string", "$.newFoo"], ["$.jsonObject", "$.newObj"]],
         [], None, jd, None, "{'newFoo':'value', 'newObj':{'testAttr':'test'}}", None, None),
        ("shouldCreateIncidentForNoMatchOnInputMapping :134-156", [["$.notExisting", "$"]], [], None, jd, None, None,
         None, "No data found for query $.notExisting."),
        ("shouldCreateIncidentForNonMatchingAndMatchingValueOnInputMapping :158-183",
         [["$.notExisting", "$.nullVal"], ["$.string", "$.existing"]], [], None, jd, None, None, None,
         "No data found for query $.notExisting."),
        ("shouldUseOutputMappingWithNoWorkflowPayload :232-254", [], [["$.string", "$.foo"]], None, None, od, None,
         "{'foo':'bar'}", None),
        ("shouldUseNoneOutputBehaviorWithoutCompletePayload :256-279", [], [], "none", jd, None, None, jd, None),
        ("shouldUseNoneOutputBehaviorAndCompletePayload :281-304", [], [], "none", jd, od, None, jd, None),
        ("shouldUseOverwriteOutputBehaviorWithoutCompletePayload :306-329", [], [], "overwrite", jd, None, None,
         "{}", None),
        ("shouldUseOverwriteOutputBehaviorAndCompletePayload :331-354", [], [], "overwrite", jd, od, None, od, None),
        ("shouldUseOverwriteOutputBehaviorWithOutputMappingAndCompletePayload :356-383", [], [["$.string", "$.foo"]],
         "overwrite", jd, od, None, "{'foo':'bar'}", None),
        ("shouldCreateIncidentOnOverwriteOutputBehaviorWithOutputMappingAndWithoutCompletedPayload :385-414", [],
         [["$.string", "$.foo"]], "overwrite", jd, None, None, None, "No data found for query $.string."),
        ("shouldNotSeePayloadOfWorkflowInstanceBeforeOnOutputMapping :497-538 (first instance)", [],
         [["$", "$.taskPayload"]], None, jd, jd, None,
         "{'string':'value', 'jsonObject':{'testAttr':'test'},'taskPayload':{'string':'value', "
         "'jsonObject':{'testAttr':'test'}}}", None),
        ("shouldUseDefaultOutputMappingIfOnlyInputMappingSpecified :540-566", [["$", "$"]], [], None, jd, od, None,
         merged, None),
        ("shouldUseOutputMappingToAddObjectsToWorkflowPayload :591-620", [],
         [["$.string", "$.newFoo"], ["$.jsonObject", "$.newObj"]], None, jd, jd, None,
         "{'newFoo':'value', 'newObj':{'testAttr':'test'}, 'string':'value', 'jsonObject':{'testAttr':'test'}}",
         None),
        ("shouldCreateIncidentForNotMatchingOnOutputMapping :622-648", [], [["$.notExisting", "$.notExist"]], None,
         jd, jd, None, None, "No data found for query $.notExisting."),
        ("shouldUseInOutMapping :650-690", [["$.jsonObject", "$"]], [["$.testAttr", "$.result"]], None, jd,
         "{'testAttr':123}", "{'testAttr':'test'}",
         "{'string':'value', 'jsonObject':{'testAttr':'test'}, 'result':123}", None),
    ]
    out = []
    for name, ins, outs, beh, create, complete, job, done, inc in rows:
        out.append({"name": name, "inputs": ins, "outputs": outs, "behavior": beh,
                    "create": mp(_tree(create)) if create else None,
                    "complete": mp(_tree(complete)) if complete else "80",
                    "job_payload_json": _tree(job) if job else None,
                    "completed_payload_json": _tree(done) if done else None,
                    "incident": inc})
    return out

def job_sequences():
    """JobInstanceStreamProcessorTest.java:59-462: commands written to the job stream processor, in batches
    that reach the log before the processor sees any of them (the tests' blockAfterJobEvent / unblock), and
    the job records the log ends up with as (recordType, intent). Values: job() = JobRecord{type "foo"},
    activated = JobRecord{type "foo", worker "bar", deadline} (:481-497). Key 1 for every command."""
    C, E, R = "COMMAND", "EVENT", "COMMAND_REJECTION"

    def seq(name, batches, expect):
        return {"name": name, "key": 1, "batches": batches, "expect": [[t, i] for t, i in expect]}

    return [
        seq("complete_expired_job", [["CREATE"], ["ACTIVATE"], ["TIME_OUT"], ["COMPLETE"]],   # :59-97
            [(C, "CREATE"), (E, "CREATED"), (C, "ACTIVATE"), (E, "ACTIVATED"), (C, "TIME_OUT"), (E, "TIMED_OUT"),
             (C, "COMPLETE"), (E, "COMPLETED")]),
        seq("activate_only_once", [["CREATE"], ["ACTIVATE", "ACTIVATE"]],                     # :99-131
            [(C, "CREATE"), (E, "CREATED"), (C, "ACTIVATE"), (C, "ACTIVATE"), (E, "ACTIVATED"), (R, "ACTIVATE")]),
        seq("reject_activation_job_not_found", [["ACTIVATE"]],                                # :133-155
            [(C, "ACTIVATE"), (R, "ACTIVATE")]),
        seq("expire_activation_only_once", [["CREATE"], ["ACTIVATE"], ["TIME_OUT", "TIME_OUT"]],  # :157-194
            [(C, "CREATE"), (E, "CREATED"), (C, "ACTIVATE"), (E, "ACTIVATED"), (C, "TIME_OUT"), (C, "TIME_OUT"),
             (E, "TIMED_OUT"), (R, "TIME_OUT")]),
        seq("reject_expire_if_created", [["CREATE"], ["TIME_OUT"]],                           # :200-226
            [(C, "CREATE"), (E, "CREATED"), (C, "TIME_OUT"), (R, "TIME_OUT")]),
        seq("reject_expire_if_completed", [["CREATE"], ["ACTIVATE"], ["COMPLETE", "TIME_OUT"]],  # :228-265
            [(C, "CREATE"), (E, "CREATED"), (C, "ACTIVATE"), (E, "ACTIVATED"), (C, "COMPLETE"), (C, "TIME_OUT"),
             (E, "COMPLETED"), (R, "TIME_OUT")]),
        seq("reject_expire_if_failed", [["CREATE"], ["ACTIVATE"], ["FAIL", "TIME_OUT"]],      # :267-304
            [(C, "CREATE"), (E, "CREATED"), (C, "ACTIVATE"), (E, "ACTIVATED"), (C, "FAIL"), (C, "TIME_OUT"),
             (E, "FAILED"), (R, "TIME_OUT")]),
        seq("reject_expire_job_not_found", [["TIME_OUT"]],                                    # :306-326
            [(C, "TIME_OUT"), (R, "TIME_OUT")]),
        seq("cancel_created_job", [["CREATE"], ["CANCEL"]],                                   # :328-353
            [(C, "CREATE"), (E, "CREATED"), (C, "CANCEL"), (E, "CANCELED")]),
        seq("cancel_activated_job", [["CREATE"], ["ACTIVATE"], ["CANCEL"]],                   # :355-386
            [(C, "CREATE"), (E, "CREATED"), (C, "ACTIVATE"), (E, "ACTIVATED"), (C, "CANCEL"), (E, "CANCELED")]),
        seq("cancel_failed_job", [["CREATE"], ["ACTIVATE"], ["FAIL"], ["CANCEL"]],            # :388-424
            [(C, "CREATE"), (E, "CREATED"), (C, "ACTIVATE"), (E, "ACTIVATED"), (C, "FAIL"), (E, "FAILED"),
             (C, "CANCEL"), (E, "CANCELED")]),
        seq("reject_cancel_if_completed", [["CREATE"], ["ACTIVATE"], ["COMPLETE"], ["CANCEL"]],  # :426-462
            [(C, "CREATE"), (E, "CREATED"), (C, "ACTIVATE"), (E, "ACTIVATED"), (C, "COMPLETE"), (E, "COMPLETED"),
             (C, "CANCEL"), (R, "CANCEL")]),
    ]


# ---- json-path and msgpack reader (SURVEY §8c pins for the query walker every condition and correlation key uses)
def jsonpath_tokens():
    # json-path/src/test/java/io/zeebe/msgpack/jsonpath/JsonPathTokenizerTest.java:28-124 (token, position, length)
    return [
        {"expr": "$.key1.key2[index]", "tokens": [
            ["START_INPUT", 0, 18], ["ROOT_OBJECT", 0, 1], ["CHILD_OPERATOR", 1, 1], ["LITERAL", 2, 4],
            ["CHILD_OPERATOR", 6, 1], ["LITERAL", 7, 4], ["SUBSCRIPT_OPERATOR_BEGIN", 11, 1], ["LITERAL", 12, 5],
            ["SUBSCRIPT_OPERATOR_END", 17, 1], ["END_INPUT", 0, 18]]},
        {"expr": "$['key1.key2'].test[index]", "tokens": [
            ["START_INPUT", 0, 26], ["ROOT_OBJECT", 0, 1], ["CHILD_BRACKET_OPERATOR_BEGIN", 1, 2], ["LITERAL", 3, 9],
            ["CHILD_BRACKET_OPERATOR_END", 12, 2], ["CHILD_OPERATOR", 14, 1], ["LITERAL", 15, 4],
            ["SUBSCRIPT_OPERATOR_BEGIN", 19, 1], ["LITERAL", 20, 5], ["SUBSCRIPT_OPERATOR_END", 25, 1],
            ["END_INPUT", 0, 26]]},
        {"expr": "$.a[b].c", "tokens": [
            ["START_INPUT", 0, 8], ["ROOT_OBJECT", 0, 1], ["CHILD_OPERATOR", 1, 1], ["LITERAL", 2, 1],
            ["SUBSCRIPT_OPERATOR_BEGIN", 3, 1], ["LITERAL", 4, 1], ["SUBSCRIPT_OPERATOR_END", 5, 1],
            ["CHILD_OPERATOR", 6, 1], ["LITERAL", 7, 1], ["END_INPUT", 0, 8]]},
    ]


def jsonpath_compile():
    # JsonPathQueryCompilerTest.java:31-79: the filter id of every filter instance (0 root, 1 map value with key,
    # 2 array index, 3 wildcard); :81-96 the query keeps its expression (checked by the compiler tests as is)
    return [{"expr": "$.key1.key2[1].key3", "filter_ids": [0, 1, 1, 2, 1]},
            {"expr": "$.*", "filter_ids": [0, 3]}]


def jsonpath_invalid():
    # JsonPathQueryValidationTest.java:29-38: (path, invalid position, error reason)
    return [{"expr": "$..", "position": 1, "error": "Unexpected json-path token RECURSION_OPERATOR"},
            {"expr": "foo", "position": 0, "error": "Unexpected json-path token LITERAL"},
            {"expr": "$.foo.$", "position": 6, "error": "Unexpected json-path token ROOT_OBJECT"},
            {"expr": "$.[foo", "position": 2, "error": "Unexpected json-path token SUBSCRIPT_OPERATOR_BEGIN"}]


def _mpj_long(v):
    """msgpack-java MessagePacker.packLong: the smallest format of the value."""
    import struct
    if -32 <= v < 128:
        return struct.pack("b", v)
    if v >= 0:
        for fmt, code, lim in ((">B", 0xcc, 1 << 8), (">H", 0xcd, 1 << 16), (">I", 0xce, 1 << 32)):
            if v < lim:
                return bytes([code]) + struct.pack(fmt, v)
        return b"\xcf" + struct.pack(">Q", v)
    for fmt, code, lim in ((">b", 0xd0, 1 << 7), (">h", 0xd1, 1 << 15), (">i", 0xd2, 1 << 31)):
        if v >= -lim:
            return bytes([code]) + struct.pack(fmt, v)
    return b"\xd3" + struct.pack(">q", v)


def queries():
    """Query results as (position, length) pairs, with the type of a single result where the test asserts one."""
    import struct
    foo = bytes.fromhex("a3666f6f")
    nt = bytes.fromhex("ae") + b"NOT_THE_TARGET"
    out = [
        # JsonPathTest.java:39-104 (Jackson msgpack of {"foo": "bar"})
        {"src": "JsonPathTest :39-104", "path": "$.foo", "doc": mp({"foo": "bar"}), "results": [[5, 4]],
         "type": "STRING", "value": "a3626172"},
        # MsgPackQueryProcessorTest.java:38-146
        {"src": "MsgPackQueryProcessorTest :38-43, :86-93", "path": "$.foo", "doc": "80", "results": [],
         "single_error": "no result found"},
        {"src": "MsgPackQueryProcessorTest :45-62", "path": "$.foo", "doc": "81a3666f6fa3626172", "results": [[5, 4]],
         "type": "STRING", "value": "a3626172"},
        {"src": "MsgPackQueryProcessorTest :64-84", "path": "$.foo", "doc": "81a3666f6f01", "results": [[5, 1]],
         "type": "INTEGER", "long_buffer": struct.pack("<q", 1).hex()},
        {"src": "MsgPackQueryProcessorTest :95-110", "path": "$.*", "doc": "82a17800a17901", "results": [[3, 1], [6, 1]],
         "single_error": "found more than one result"},
        {"src": "MsgPackQueryProcessorTest :112-146", "path": "$.foo", "doc": "81a3666f6fc2", "results": [[5, 1]],
         "type": "BOOLEAN", "string_error": "expected String but found 'BOOLEAN'",
         "long_error": "expected Long but found 'BOOLEAN'"},
        # MsgPackTraverserTest.java:111-155 ($.foo[1].bar), :157-191 ($.target), :193-228 ($.*)
        {"src": "MsgPackTraverserTest :111-155", "path": "$.foo[1].bar",
         "doc": (b"\x82" + nt + nt + foo + b"\x92" + nt + b"\x82" + nt + nt + bytes.fromhex("a3626172") +
                 b"\xaaTHE_TARGET").hex(), "results": [[86, 11]]},
        {"src": "MsgPackTraverserTest :157-191", "path": "$.target",
         "doc": (b"\x82" + foo + foo + b"\xa6target\x81" + foo + foo).hex(), "results": [[16, 9]]},
        {"src": "MsgPackTraverserTest :193-228", "path": "$.*",
         "doc": (b"\x82\xa4key1\xa4val1\xa4key2\xa4val2").hex(), "results": [[6, 5], [16, 5]]},
    ]
    # MsgPackQueryValueFormatsTest.java:39-116: {"foo": value} -> the value's bytes (msgpack-java encodings)
    vals = [foo, b"\xc3", b"\xc2", b"\xcb" + struct.pack(">d", 1.444), b"\xca" + struct.pack(">f", 1.555),
            _mpj_long(1 << 4), _mpj_long(-(1 << 2)), _mpj_long(1 << 7), _mpj_long(1 << 14), _mpj_long(1 << 29),
            _mpj_long((1 << 31) - 1 + 10), b"\xc0", _mpj_long(123)]
    for v in vals:
        out.append({"src": "MsgPackQueryValueFormatsTest :39-116", "path": "$.foo", "doc": (b"\x81" + foo + v).hex(),
                    "results": [[5, len(v)]], "value": v.hex()})
    return out


def traversal_errors():
    # MsgPackTraverserTest.java:230-256: a valid string followed by 0xc7 (ext 8, unsupported)
    return [{"doc": "a3666f6fc7", "position": 4, "error": "Unsupported token format"}]


def read_tokens():
    # msgpack-core/src/test/java/io/zeebe/msgpack/spec/MsgPackReadTokenTest.java:55-241 (the reader consumes the
    # whole input in every row)
    import struct
    r = [("positive fixint", "7f", "INTEGER", {"int": 0x7f}), ("fixmap", "8f", "MAP", {"size": 15}),
         ("fixarray", "9f", "ARRAY", {"size": 15}), ("fixstr", "a122", "STRING", {"value": "22"}),
         ("nil", "c0", "NIL", {}), ("false", "c2", "BOOLEAN", {"bool": False}), ("true", "c3", "BOOLEAN", {"bool": True}),
         ("bin 8", "c40122", "BINARY", {"value": "22"}), ("bin 16", "c5000122", "BINARY", {"value": "22"}),
         ("bin 32", "c60000000122", "BINARY", {"value": "22"}),
         ("float 32", "ca" + struct.pack(">f", 123123.12).hex(), "FLOAT",
          {"float": struct.unpack(">f", struct.pack(">f", 123123.12))[0]}),
         ("float 64", "cb" + struct.pack(">d", 123123.123).hex(), "FLOAT", {"float": 123123.123}),
         ("uint 8", "ccff", "INTEGER", {"int": (1 << 8) - 1}), ("uint 16", "cdffff", "INTEGER", {"int": (1 << 16) - 1}),
         ("uint 32", "ceffffffff", "INTEGER", {"int": (1 << 32) - 1}),
         ("uint 64", "cf7fffffffffffffff", "INTEGER", {"int": (1 << 63) - 1}),
         ("int 8", "d080", "INTEGER", {"int": -128}), ("int 16", "d18000", "INTEGER", {"int": -32768}),
         ("int 32", "d280000000", "INTEGER", {"int": -(1 << 31)}),
         ("int 64", "d38000000000000000", "INTEGER", {"int": -(1 << 63)}),
         ("str 8", "d90122", "STRING", {"value": "22"}), ("str 16", "da000122", "STRING", {"value": "22"}),
         ("str 32", "db0000000122", "STRING", {"value": "22"}),
         ("array 16", "dcffff", "ARRAY", {"size": 0xffff}), ("array 32", "dd7fffffff", "ARRAY", {"size": (1 << 31) - 1}),
         ("map 16", "deffff", "MAP", {"size": 0xffff}), ("map 32", "df00ffffff", "MAP", {"size": 0x00ffffff}),
         ("negative fixint", "e0", "INTEGER", {"int": -32})]
    return [dict(name=n, bytes=b, type=t, **a) for n, b, t, a in r]


# ---- the payload tree (MsgPackDocumentIndexer / MsgPackTree / MsgPackDocumentExtractor / MsgPackDocumentTreeWriter):
# the pins of the exact tree (zeebe_amd/csrc/zb_xmerge.hpp) and of the oracle's zbref_mapping.hpp
def _nid(*names):
    """MappingTestUtil.constructNodeId: "$" + "[name]"..."""
    return names[0] + "".join("[%s]" % n for n in names[1:])


def _mapping_payload():
    """MappingTestUtil.java:36-80 JSON_PAYLOAD (MSG_PACK_BYTES; a HashMap, so its key order is not part of any test)."""
    return {"string": "value", "boolean": False, "integer": 1024, "long": (1 << 63) - 1, "double": 0.3,
            "array": [0, 1, 2, 3], "jsonObject": {"testAttr": "test"}}


def trees():
    """Each row: a document, the mappings of an extraction (none: the document is indexed), and the assertions of the
    test on the resulting tree: ["map" | "array", node id, its children (as a set)] or ["leaf", node id, the leaf's
    msgpack bytes] (assertThatIsMapNode / assertThatIsArrayNode / assertThatIsLeafNode, MappingTestUtil.java:85-117),
    or the failure message."""
    P = _mapping_payload()
    doc = mp(P)
    keys = list(P)
    rows = []
    # json-path/src/test/java/io/zeebe/msgpack/mapping/MsgPackDocumentIndexerTest.java:47-102
    rows.append({"src": "MsgPackDocumentIndexerTest.shouldIndexDocument :47-102", "doc": doc, "mappings": None,
                 "expect": [["map", "$", keys], ["map", _nid("$", "jsonObject"), ["testAttr"]],
                            ["array", _nid("$", "array"), ["0", "1", "2", "3"]],
                            ["leaf", _nid("$", "string"), mp("value")], ["leaf", _nid("$", "boolean"), mp(False)],
                            ["leaf", _nid("$", "integer"), mp(1024)], ["leaf", _nid("$", "long"), mp((1 << 63) - 1)],
                            ["leaf", _nid("$", "double"), mp(0.3)]] +
                           [["leaf", _nid("$", "array", str(i)), mp(i)] for i in range(4)] +
                           [["leaf", _nid("$", "jsonObject", "testAttr"), mp("test")]]})
    d2 = _tree("{'first': { 'range': [0, 2], 'friends': [-1, {'id': 0, 'name': 'Rodriguez Richards'}],"
               "'greeting': 'Hello, Bauer! You have 7 unread messages.', 'favoriteFruit': 'apple'}}")
    f = ("$", "first")
    rows.append({"src": "MsgPackDocumentIndexerTest.shouldIndexDocumentWithMoreArrays :104-161", "doc": mp(d2),
                 "mappings": None,
                 "expect": [["map", "$", ["first"]], ["map", _nid(*f), ["range", "friends", "greeting", "favoriteFruit"]],
                            ["array", _nid(*f, "range"), ["0", "1"]], ["leaf", _nid(*f, "range", "0"), mp(0)],
                            ["leaf", _nid(*f, "range", "1"), mp(2)], ["array", _nid(*f, "friends"), ["0", "1"]],
                            ["leaf", _nid(*f, "friends", "0"), mp(-1)],
                            ["map", _nid(*f, "friends", "1"), ["id", "name"]],
                            ["leaf", _nid(*f, "friends", "1", "id"), mp(0)],
                            ["leaf", _nid(*f, "friends", "1", "name"), mp("Rodriguez Richards")],
                            ["leaf", _nid(*f, "greeting"), mp("Hello, Bauer! You have 7 unread messages.")],
                            ["leaf", _nid(*f, "favoriteFruit"), mp("apple")]]})
    d3 = _tree("{'friends': [{'id': 0, 'name': 'Rodriguez Richards'}, {'id': 0, 'name': 'Rodriguez Richards'}]}")
    rows.append({"src": "MsgPackDocumentIndexerTest.shouldIndexDocumentWitObjectArray :163-199", "doc": mp(d3),
                 "mappings": None,
                 "expect": [["map", "$", ["friends"]], ["array", _nid("$", "friends"), ["0", "1"]]] +
                           [e for i in ("0", "1") for e in (
                               ["map", _nid("$", "friends", i), ["id", "name"]],
                               ["leaf", _nid("$", "friends", i, "id"), mp(0)],
                               ["leaf", _nid("$", "friends", i, "name"), mp("Rodriguez Richards")])]})
    rows.append({"src": "MsgPackDocumentIndexerTest.shouldIndexDocumentWitArrayAndObjectWithIndex :201-223",
                 "doc": mp(_tree("{'a':['foo'], 'a0':{'b':'c'}}")), "mappings": None,
                 "expect": [["map", "$", ["a", "a0"]], ["array", _nid("$", "a"), ["0"]],
                            ["leaf", _nid("$", "a", "0"), mp("foo")], ["map", _nid("$", "a0"), ["b"]],
                            ["leaf", _nid("$", "a0", "b"), mp("c")]]})
    # MsgPackDocumentExtractorTest.java:41-219
    ja = mp({"testAttr": "test"})
    ex = [
        (":41-53 shouldExtractHoleDocument", [["$", "$"]], [["leaf", "$", doc]]),
        (":55-68 shouldExtractHoleDocumentAndCreateNewObject", [["$", "$.old"]],
         [["map", "$", ["old"]], ["leaf", _nid("$", "old"), doc]]),
        (":70-84 shouldExtractHoleDocumentAndCreateNewDeepObject", [["$", "$.old.test"]],
         [["map", "$", ["old"]], ["map", _nid("$", "old"), ["test"]], ["leaf", _nid("$", "old", "test"), doc]]),
        (":86-104 shouldCreateOrRenameObject", [["$.jsonObject", "$.testObj"]],
         [["map", "$", ["testObj"]], ["leaf", _nid("$", "testObj"), ja]]),
        (":106-124 shouldCreateObjectOnRoot", [["$.jsonObject", "$"]], [["leaf", "$", ja]]),
        (":126-145 shouldCreateValueOnArrayIndex", [["$.array[1]", "$.array[0]"]],
         [["map", "$", ["array"]], ["array", _nid("$", "array"), ["0"]], ["leaf", _nid("$", "array", "0"), mp(1)]]),
        (":147-169 shouldCreateValueOnArrayIndexObject", [["$.array[1]", "$.array[0].test"]],
         [["map", "$", ["array"]], ["array", _nid("$", "array"), ["0"]], ["map", _nid("$", "array", "0"), ["test"]],
          ["leaf", _nid("$", "array", "0", "test"), mp(1)]]),
        (":171-202 shouldExtractWithMoreMappings",
         [["$.boolean", "$.newBoolean"], ["$.array", "$.newArray"], ["$.jsonObject", "$.newObject"]],
         [["map", "$", ["newBoolean", "newArray", "newObject"]], ["leaf", _nid("$", "newBoolean"), mp(False)],
          ["leaf", _nid("$", "newArray"), mp([0, 1, 2, 3])], ["leaf", _nid("$", "newObject"), ja]]),
    ]
    for name, ms, exp in ex:
        rows.append({"src": "MsgPackDocumentExtractorTest" + name, "doc": doc, "mappings": ms, "expect": exp})
    rows.append({"src": "MsgPackDocumentExtractorTest :204-219 shouldThrowExceptionIfMappingMatchesTwice",
                 "doc": mp(_tree("{'foo':'bar', 'foa':'baz'}")), "mappings": [["$.*", "$"]],
                 "error": "JSON path mapping has more than one matching source."})
    # MsgPackTreeTest.java:36-84, through the extractor: a leaf of the whole document, and a leaf that reads the
    # extract document (setExtractDocument) rather than the underlying one
    inner = {"aObject": {"test": "test"}, "string": "stringValue"}
    rows.append({"src": "MsgPackTreeTest :36-47 shouldUseUnderlyingDocument (as extract $ -> $)", "doc": doc,
                 "mappings": [["$", "$"]], "expect": [["leaf", "$", doc]]})
    rows.append({"src": "MsgPackTreeTest :49-84 shouldDifferBetweenUnderlyingAndExtractDocument (as extract "
                        "$.aObject -> $)", "doc": mp(inner), "mappings": [["$.aObject", "$"]],
                 "expect": [["leaf", "$", mp({"test": "test"})]]})
    return rows


def tree_writes():
    """MsgPackDocumentTreeWriterTest.java:33-70: index the test resource largeJsonDocument.json (Jackson msgpack of its
    JSON tree) and write the tree: the result has the document's length and JSON value. The resource is copied as data
    to tests/golden/mapping_largeJsonDocument.json."""
    src = os.path.join(REF, "json-path/src/test/resources/io/zeebe/msgpack/mapping/largeJsonDocument.json")
    with open(src, "rb") as f:
        text = f.read()
    with open(os.path.join(HERE, "mapping_largeJsonDocument.json"), "wb") as f:
        f.write(text)
    return [{"src": "MsgPackDocumentTreeWriterTest :33-70", "json_file": "mapping_largeJsonDocument.json"}]


def main():
    data = {
        "conditions": conditions(),
        "condition_errors": condition_errors(),
        "parser_valid": parser_valid(),
        "parser_failures": parser_failures(),
        "merges": merges(),
        "writer": writer(),
        "hashes": hashes(),
        "workflows": workflows(),
        "cancels": cancels(),
        "mapping_extracts": mapping_extracts(),
        "mapping_merges": mapping_merges(),
        "io_workflows": io_workflows(),
        "job_sequences": job_sequences(),
        "wf_intents": WF,
        "jsonpath_tokens": jsonpath_tokens(),
        "jsonpath_compile": jsonpath_compile(),
        "jsonpath_invalid": jsonpath_invalid(),
        "queries": queries(),
        "traversal_errors": traversal_errors(),
        "read_tokens": read_tokens(),
        "trees": trees(),
        "tree_writes": tree_writes(),
    }
    with open(os.path.join(HERE, "reference_vectors.json"), "w") as f:
        json.dump(data, f, indent=1, allow_nan=False, default=str)
    print("wrote", os.path.join(HERE, "reference_vectors.json"))


if __name__ == "__main__":
    main()
