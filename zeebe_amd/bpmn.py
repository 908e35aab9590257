"""Fluent BPMN 2.0 builder that emits deployment XML (the input format of ``zb_deploy``).

This mirrors the reference's model API ``Bpmn.createExecutableProcess(...)`` builder
(``bpmn-model/src/main/java/io/zeebe/model/bpmn/Bpmn.java`` and
``bpmn-model/src/main/java/io/zeebe/model/bpmn/builder/AbstractFlowNodeBuilder.java:65-150``)
closely enough that the *document order* of the generated XML matches the reference builder:

* a sequence flow is created lazily: ``sequence_flow_id()`` / ``condition()`` / ``default_flow()``
  create it *before* the target node (``getCurrentSequenceFlowBuilder`` ->
  ``createSibling(SequenceFlow)``, ``AbstractFlowNodeBuilder.java:65-71``); otherwise it is created
  right after the target in ``connectTargetWithSequenceFlow`` (``:103-109``);
* ``<outgoing>`` / ``<incoming>`` reference children are appended in connect order
  (``SequenceFlowBuilder.from/to``).

Document order matters: the transformer visits siblings in reverse document order
(``ModelWalker.java:59-63``), which fixes each node's executable outgoing-flow order.

The builder is a convenience for tests and the benchmark; the engine itself consumes plain BPMN
XML, so hand-written deployment resources work too.
"""
from __future__ import annotations

from typing import List, Optional
from xml.sax.saxutils import escape, quoteattr

BPMN_NS = "http://www.omg.org/spec/BPMN/20100524/MODEL"
ZEEBE_NS = "http://camunda.org/schema/zeebe/1.0"


class _Node:
    def __init__(self, tag: str, ident: Optional[str], attrs=None):
        self.tag = tag
        self.id = ident
        self.attrs = dict(attrs or {})
        self.children: List[_Node] = []
        self.text: Optional[str] = None
        self.parent: Optional[_Node] = None

    def add(self, child: "_Node") -> "_Node":
        child.parent = self
        self.children.append(child)
        return child

    def to_xml(self, out: List[str], indent: str = "") -> None:
        attrs = ""
        if self.id is not None:
            attrs += " id=" + quoteattr(self.id)
        for k, v in self.attrs.items():
            attrs += " %s=%s" % (k, quoteattr(str(v)))
        if not self.children and self.text is None:
            out.append("%s<%s%s/>" % (indent, self.tag, attrs))
            return
        if self.text is not None and not self.children:
            out.append("%s<%s%s>%s</%s>" % (indent, self.tag, attrs, escape(self.text), self.tag))
            return
        out.append("%s<%s%s>" % (indent, self.tag, attrs))
        for c in self.children:
            c.to_xml(out, indent + "  ")
        out.append("%s</%s>" % (indent, self.tag))


class BpmnModel:
    """A built model: ``.to_xml()`` gives the deployment resource bytes."""

    def __init__(self, definitions: _Node):
        self.definitions = definitions

    def to_xml(self) -> str:
        out = ['<?xml version="1.0" encoding="UTF-8" standalone="no"?>']
        self.definitions.to_xml(out)
        return "\n".join(out) + "\n"

    def to_bytes(self) -> bytes:
        return self.to_xml().encode("utf-8")


class _Ctx:
    def __init__(self, process_id: str):
        self.definitions = _Node(
            "bpmn:definitions",
            "definitions",
            {"xmlns:bpmn": BPMN_NS, "xmlns:zeebe": ZEEBE_NS, "targetNamespace": "http://bpmn.io/schema/bpmn"},
        )
        self.process = self.definitions.add(_Node("bpmn:process", process_id, {"isExecutable": "true"}))
        self.by_id = {process_id: self.process}
        self.counter = 0

    def gen_id(self, prefix: str) -> str:
        self.counter += 1
        return "%s_%d" % (prefix, self.counter)


class FlowNodeBuilder:
    """Builder positioned on one flow node (mirrors ``AbstractFlowNodeBuilder``)."""

    def __init__(self, ctx: _Ctx, node: _Node):
        self._ctx = ctx
        self._node = node
        self._flow: Optional[_Node] = None
        self._flow_default = False

    # ---- sequence flow attributes (create the flow lazily, before the target) ----
    def _current_flow(self) -> _Node:
        if self._flow is None:
            self._flow = self._node.parent.add(_Node("bpmn:sequenceFlow", self._ctx.gen_id("sequenceFlow")))
            self._ctx.by_id[self._flow.id] = self._flow
        return self._flow

    def sequence_flow_id(self, ident: str) -> "FlowNodeBuilder":
        flow = self._current_flow()
        del self._ctx.by_id[flow.id]
        flow.id = ident
        self._ctx.by_id[ident] = flow
        return self

    def condition(self, expression: str) -> "FlowNodeBuilder":
        flow = self._current_flow()
        c = flow.add(_Node("bpmn:conditionExpression", None))
        c.text = expression
        return self

    def default_flow(self) -> "FlowNodeBuilder":
        self._current_flow()
        self._flow_default = True
        return self

    # ---- connecting ----
    def _connect(self, target: _Node) -> None:
        flow = self._current_flow()
        flow.attrs["sourceRef"] = self._node.id
        flow.attrs["targetRef"] = target.id
        self._node.add(_Node("bpmn:outgoing", None)).text = flow.id
        target.add(_Node("bpmn:incoming", None)).text = flow.id
        if self._flow_default:
            self._node.attrs["default"] = flow.id
        self._flow = None
        self._flow_default = False

    def _target(self, tag: str, ident: Optional[str], prefix: str) -> _Node:
        ident = ident or self._ctx.gen_id(prefix)
        node = self._node.parent.add(_Node(tag, ident))
        self._ctx.by_id[ident] = node
        self._connect(node)
        return node

    def service_task(self, ident: Optional[str] = None, type: Optional[str] = None, retries: Optional[int] = None,
                     headers=None, inputs=None, outputs=None, output_behavior: Optional[str] = None):
        node = self._target("bpmn:serviceTask", ident, "serviceTask")
        b = FlowNodeBuilder(self._ctx, node)
        if type is not None:
            b.zeebe_task_type(type, retries)
        if headers:
            for k, v in headers:
                b.zeebe_task_header(k, v)
        for s, t in inputs or []:
            b.zeebe_input(s, t)
        for s, t in outputs or []:
            b.zeebe_output(s, t)
        if output_behavior is not None:
            b.zeebe_output_behavior(output_behavior)
        return b

    def end_event(self, ident: Optional[str] = None) -> "FlowNodeBuilder":
        return FlowNodeBuilder(self._ctx, self._target("bpmn:endEvent", ident, "endEvent"))

    def exclusive_gateway(self, ident: Optional[str] = None) -> "FlowNodeBuilder":
        return FlowNodeBuilder(self._ctx, self._target("bpmn:exclusiveGateway", ident, "exclusiveGateway"))

    def parallel_gateway(self, ident: Optional[str] = None) -> "FlowNodeBuilder":
        return FlowNodeBuilder(self._ctx, self._target("bpmn:parallelGateway", ident, "parallelGateway"))

    def intermediate_catch_event(self, ident: Optional[str] = None, message: Optional[str] = None,
                                 correlation_key: Optional[str] = None) -> "FlowNodeBuilder":
        node = self._target("bpmn:intermediateCatchEvent", ident, "intermediateCatchEvent")
        b = FlowNodeBuilder(self._ctx, node)
        if message is not None:
            b.message(message, correlation_key)
        return b

    def sub_process(self, ident: Optional[str] = None) -> "SubProcessBuilder":
        return SubProcessBuilder(self._ctx, self._target("bpmn:subProcess", ident, "subProcess"))

    def connect_to(self, ident: str) -> "FlowNodeBuilder":
        target = self._ctx.by_id[ident]
        self._connect(target)
        return FlowNodeBuilder(self._ctx, target)

    # ---- navigation ----
    def move_to_node(self, ident: str) -> "FlowNodeBuilder":
        return FlowNodeBuilder(self._ctx, self._ctx.by_id[ident])

    def _find_last_gateway(self, tags) -> "FlowNodeBuilder":
        # AbstractFlowNodeBuilder.findLastGateway :326-339: walk unique previous nodes backwards
        node = self._node
        while True:
            prev = [n for n in self._all_nodes() if n.tag == "bpmn:sequenceFlow"
                    and n.attrs.get("targetRef") == node.id]
            if len(prev) != 1:
                raise ValueError("Unable to determine an unique previous gateway of %s" % node.id)
            node = self._ctx.by_id[prev[0].attrs["sourceRef"]]
            if node.tag in tags:
                return FlowNodeBuilder(self._ctx, node)

    def move_to_last_gateway(self) -> "FlowNodeBuilder":
        return self._find_last_gateway(("bpmn:exclusiveGateway", "bpmn:parallelGateway"))

    def move_to_last_exclusive_gateway(self) -> "FlowNodeBuilder":
        return self._find_last_gateway(("bpmn:exclusiveGateway",))

    def _all_nodes(self) -> List[_Node]:
        out: List[_Node] = []

        def walk(n: _Node):
            out.append(n)
            for c in n.children:
                walk(c)

        walk(self._ctx.process)
        return out

    # ---- zeebe extensions ----
    def _ext(self) -> _Node:
        for c in self._node.children:
            if c.tag == "bpmn:extensionElements":
                return c
        ext = _Node("bpmn:extensionElements", None)
        ext.parent = self._node
        self._node.children.insert(0, ext)
        return ext

    def _ext_single(self, tag: str) -> _Node:
        ext = self._ext()
        for c in ext.children:
            if c.tag == tag:
                return c
        return ext.add(_Node(tag, None))

    def zeebe_task_type(self, type: str, retries: Optional[int] = None) -> "FlowNodeBuilder":
        td = self._ext_single("zeebe:taskDefinition")
        td.attrs["type"] = type
        if retries is not None:
            td.attrs["retries"] = str(retries)
        return self

    def zeebe_task_header(self, key: str, value: str) -> "FlowNodeBuilder":
        th = self._ext_single("zeebe:taskHeaders")
        th.add(_Node("zeebe:header", None, {"key": key, "value": value}))
        return self

    def zeebe_input(self, source: str, target: str) -> "FlowNodeBuilder":
        self._ext_single("zeebe:ioMapping").add(_Node("zeebe:input", None, {"source": source, "target": target}))
        return self

    def zeebe_output(self, source: str, target: str) -> "FlowNodeBuilder":
        self._ext_single("zeebe:ioMapping").add(_Node("zeebe:output", None, {"source": source, "target": target}))
        return self

    def zeebe_output_behavior(self, behavior: str) -> "FlowNodeBuilder":
        self._ext_single("zeebe:ioMapping").attrs["zeebe:outputBehavior"] = behavior
        return self

    def message(self, name: str, correlation_key: Optional[str]) -> "FlowNodeBuilder":
        defs = self._ctx.definitions
        msg_id = self._ctx.gen_id("message")
        msg = _Node("bpmn:message", msg_id, {"name": name})
        # messages live at definitions level, before the process (Message created as child of definitions)
        defs.children.insert(0, msg)
        msg.parent = defs
        if correlation_key is not None:
            ext = msg.add(_Node("bpmn:extensionElements", None))
            ext.add(_Node("zeebe:subscription", None, {"correlationKey": correlation_key}))
        self._node.add(_Node("bpmn:messageEventDefinition", self._ctx.gen_id("messageEventDefinition"),
                             {"messageRef": msg_id}))
        return self

    def done(self) -> BpmnModel:
        return BpmnModel(self._ctx.definitions)

    @property
    def id(self) -> str:
        return self._node.id


class SubProcessBuilder(FlowNodeBuilder):
    def embedded_sub_process(self) -> "EmbeddedBuilder":
        return EmbeddedBuilder(self._ctx, self._node, self)


class EmbeddedBuilder:
    def __init__(self, ctx: _Ctx, sub: _Node, owner: SubProcessBuilder):
        self._ctx = ctx
        self._sub = sub
        self._owner = owner

    def start_event(self, ident: Optional[str] = None) -> "FlowNodeBuilder":
        ident = ident or self._ctx.gen_id("startEvent")
        node = self._sub.add(_Node("bpmn:startEvent", ident))
        self._ctx.by_id[ident] = node
        return _ScopedBuilder(self._ctx, node, self._owner)


class _ScopedBuilder(FlowNodeBuilder):
    """Flow-node builder inside an embedded sub process; ``sub_process_done()`` returns to it."""

    def __init__(self, ctx, node, owner):
        super().__init__(ctx, node)
        self._owner = owner

    def _wrap(self, b: FlowNodeBuilder):
        if isinstance(b, SubProcessBuilder):
            return b
        s = _ScopedBuilder(self._ctx, b._node, self._owner)
        return s

    def service_task(self, *a, **k):
        return self._wrap(super().service_task(*a, **k))

    def end_event(self, *a, **k):
        return self._wrap(super().end_event(*a, **k))

    def exclusive_gateway(self, *a, **k):
        return self._wrap(super().exclusive_gateway(*a, **k))

    def parallel_gateway(self, *a, **k):
        return self._wrap(super().parallel_gateway(*a, **k))

    def intermediate_catch_event(self, *a, **k):
        return self._wrap(super().intermediate_catch_event(*a, **k))

    def connect_to(self, ident):
        return self._wrap(super().connect_to(ident))

    def move_to_node(self, ident):
        return self._wrap(super().move_to_node(ident))

    def move_to_last_exclusive_gateway(self):
        return self._wrap(super().move_to_last_exclusive_gateway())

    def move_to_last_gateway(self):
        return self._wrap(super().move_to_last_gateway())

    def sub_process_done(self) -> SubProcessBuilder:
        return self._owner


class ProcessBuilder:
    def __init__(self, process_id: str):
        self._ctx = _Ctx(process_id)

    def start_event(self, ident: Optional[str] = None) -> FlowNodeBuilder:
        ident = ident or self._ctx.gen_id("startEvent")
        node = self._ctx.process.add(_Node("bpmn:startEvent", ident))
        self._ctx.by_id[ident] = node
        return FlowNodeBuilder(self._ctx, node)


class Bpmn:
    @staticmethod
    def create_executable_process(process_id: str) -> ProcessBuilder:
        return ProcessBuilder(process_id)


# ---------------------------------------------------------------------------------------------
# Workflows used by BASELINE.json's configs
# ---------------------------------------------------------------------------------------------

def config1_workflow() -> BpmnModel:
    """C1: start -> flow1 -> service task "task" (type "task", retries 3) -> flow2 -> end."""
    return (Bpmn.create_executable_process("process").start_event("start")
            .sequence_flow_id("flow1").service_task("task", type="task", retries=3)
            .sequence_flow_id("flow2").end_event("end").done())


def chain_workflow(n_tasks: int = 20, process_id: str = "chain") -> BpmnModel:
    """C2: start -> t1 -> ... -> tN -> end, task k has job type "t<k>"."""
    b = Bpmn.create_executable_process(process_id).start_event("start")
    for k in range(1, n_tasks + 1):
        b = b.sequence_flow_id("f%d" % k).service_task("t%d" % k, type="t%d" % k)
    return b.sequence_flow_id("f%d" % (n_tasks + 1)).end_event("end").done()


def xor_workflow(process_id: str = "xor") -> BpmnModel:
    """C3: two exclusive gateways with json-el conditions (conditioned flows declared first)."""
    b = Bpmn.create_executable_process(process_id).start_event("start").sequence_flow_id("f0")
    g1 = b.exclusive_gateway("g1")
    g2 = g1.sequence_flow_id("f1").condition("$.amount < 1000 && $.region == 'EU'").exclusive_gateway("g2")
    g2.sequence_flow_id("f3").condition("$.amount < 100").end_event("endA1")
    g2.move_to_node("g2").default_flow().sequence_flow_id("f4").end_event("endA2")
    g1b = g1.move_to_node("g1")
    g1b.sequence_flow_id("f2").condition("$.score >= 0.5").end_event("endB")
    return g1.move_to_node("g1").default_flow().sequence_flow_id("f5").end_event("endC").done()


def subprocess_chain_workflow(n_sub: int = 8, process_id: str = "subs") -> BpmnModel:
    """C4 parity twin: n embedded sub processes in sequence, each start -> task_k -> end."""
    b = Bpmn.create_executable_process(process_id).start_event("start")
    for k in range(1, n_sub + 1):
        sp = b.sequence_flow_id("in%d" % k).sub_process("sub%d" % k)
        inner = sp.embedded_sub_process().start_event("s%d_start" % k)
        inner = inner.sequence_flow_id("s%d_f1" % k).service_task("task%d" % k, type="task%d" % k)
        inner.sequence_flow_id("s%d_f2" % k).end_event("s%d_end" % k)
        b = sp
    return b.sequence_flow_id("out").end_event("end").done()


def message_workflow(process_id: str = "msg") -> BpmnModel:
    """C5: start -> intermediate message catch ("order", $.orderId) -> end."""
    return (Bpmn.create_executable_process(process_id).start_event("start")
            .intermediate_catch_event("wait", message="order", correlation_key="$.orderId")
            .end_event("end").done())


def parallel_workflow(fanout: int = 8, process_id: str = "par", subprocesses: bool = True) -> BpmnModel:
    """C4 (EXTENSION): start -> fork (parallel) -> fanout x [sub_k {start -> task_k -> end}] ->
    join (parallel) -> end. With subprocesses=False each branch is the service task alone."""
    fork = Bpmn.create_executable_process(process_id).start_event("start").sequence_flow_id("in").parallel_gateway("fork")
    for k in range(1, fanout + 1):
        b = fork.move_to_node("fork").sequence_flow_id("b%d" % k)
        if subprocesses:
            sp = b.sub_process("sub%d" % k)
            inner = sp.embedded_sub_process().start_event("s%d_start" % k)
            inner.sequence_flow_id("s%d_f1" % k).service_task("task%d" % k, type="task%d" % k) \
                .sequence_flow_id("s%d_f2" % k).end_event("s%d_end" % k)
            b = sp
        else:
            b = b.service_task("task%d" % k, type="task%d" % k)
        b = b.sequence_flow_id("j%d" % k)
        if k == 1:
            join = b.parallel_gateway("join")
            join.sequence_flow_id("out").end_event("end")
        else:
            b.connect_to("join")
    return fork.done()
