"""The oracle's explicit io-mappings pinned on the reference's own vectors (tests/golden/reference_vectors.json):

* mapping_extracts: MappingExtractParameterizedTest.java (every row) + MappingExtractTest.java exceptions;
* mapping_merges:   MappingMergeParameterizedTest.java (every row) + MappingMergeTest.java exceptions;
* io_workflows:     WorkflowTaskIOMappingTest.java, start -> service task -> end with zeebe:ioMapping: the JOB CREATE
                    payload, the task's ELEMENT_COMPLETED payload, or the IO_MAPPING_ERROR incident message.

The reference compares documents as JSON trees (key order unpinned); so do these tests.
"""
import msgpack
import pytest

from oracle import zbref
from zeebe_amd import bpmn


def _tree(doc: bytes):
    return msgpack.unpackb(doc, raw=False, strict_map_key=False)


def test_extract_vectors(vectors):
    for v in vectors["mapping_extracts"]:
        src = bytes.fromhex(v["source"])
        if "error" in v:
            with pytest.raises(zbref.MappingError, match=v["error"].replace("$", r"\$").replace(".", r"\.").replace("(", r"\(").replace(")", r"\)")):
                zbref.map_documents(src, v["mappings"])
            continue
        assert _tree(zbref.map_documents(src, v["mappings"])) == v["expected_json"], v


def test_merge_vectors(vectors):
    for v in vectors["mapping_merges"]:
        src, tgt = bytes.fromhex(v["source"]), bytes.fromhex(v["target"])
        if "error" in v:
            with pytest.raises(zbref.MappingError) as ei:
                zbref.map_documents(src, v["mappings"], tgt)
            assert str(ei.value) == v["error"]
            continue
        assert _tree(zbref.map_documents(src, v["mappings"], tgt)) == v["expected_json"], v


def io_workflow(v, pid="process"):
    """The WorkflowTaskIOMappingTest model: start -> service task "service" (type "external") -> end."""
    return bpmn.Bpmn.create_executable_process(pid).start_event("start").service_task(
        "service", type="external", inputs=v["inputs"] or None, outputs=v["outputs"] or None,
        output_behavior=v["behavior"]).end_event("end").done()


def run_oracle_io(v):
    o = zbref.Oracle()
    o.deploy(io_workflow(v).to_xml(), 100, 1)
    o.set_job_payload(100, "service", bytes.fromhex(v["complete"]))
    o.create("process", bytes.fromhex(v["create"]) if v["create"] else b"")
    o.run()
    return o


def check_io_outcome(v, records):
    job_create = [r for r in records if r.value_type == 0 and r.intent == 0]
    completed = [r for r in records if r.value_type == 5 and r.intent == 9 and
                 msgpack.unpackb(r.value, raw=False)["activityId"] == "service"]
    incidents = [r for r in records if r.value_type == 6]
    if v["incident"]:
        assert len(incidents) == 1 and not completed, v["name"]
        val = msgpack.unpackb(incidents[0].value, raw=False)
        assert val["errorType"] == "IO_MAPPING_ERROR" and val["errorMessage"] == v["incident"], (v["name"], val)
        return
    assert not incidents, v["name"]
    if v["job_payload_json"] is not None:
        assert _tree(msgpack.unpackb(job_create[0].value, raw=False)["payload"]) == v["job_payload_json"], v["name"]
    if v["completed_payload_json"] is not None:
        assert len(completed) == 1, v["name"]
        assert _tree(msgpack.unpackb(completed[0].value, raw=False)["payload"]) == v["completed_payload_json"], v["name"]


def test_io_workflow_vectors(vectors):
    for v in vectors["io_workflows"]:
        check_io_outcome(v, run_oracle_io(v).records())


def test_io_mapping_deploy_validation():
    bad = [
        dict(inputs=[["$.a", "$"], ["$.b", "$.c"]], outputs=None, behavior=None),  # root target + another input
        dict(inputs=None, outputs=[["$.a", "$"], ["$.b", "$.c"]], behavior=None),
        dict(inputs=None, outputs=[["$.a", "$.b"]], behavior="none"),  # none + outputs
        dict(inputs=[["$.a.*", "$.b"]], outputs=None, behavior=None),  # prohibited path
        dict(inputs=[["foo", "$.b"]], outputs=None, behavior=None),  # invalid json path
    ]
    for b in bad:
        o = zbref.Oracle()
        v = {"inputs": b["inputs"], "outputs": b["outputs"], "behavior": b["behavior"]}
        with pytest.raises(Exception):
            o.deploy(io_workflow(v).to_xml(), 100, 1)
