"""The product's deploy-time handling of zeebe:ioMapping (zb_model.cpp, through the host-only
zb_validate_deployment): every WorkflowTaskIOMappingTest model deploys, and the invalid ones fail with the
oracle's message (ZeebeIoMappingValidator, ZeebeExpressionValidator.validateJsonPath). CPU only."""
import pytest

from oracle import zbref
from test_oracle_iomapping import io_workflow
from zeebe_amd import engine

BAD = [
    dict(inputs=[["$.a", "$"], ["$.b", "$.c"]], outputs=None, behavior=None),
    dict(inputs=None, outputs=[["$.a", "$"], ["$.b", "$.c"]], behavior=None),
    dict(inputs=None, outputs=[["$.a", "$.b"]], behavior="none"),
    dict(inputs=[["$.a.*", "$.b"]], outputs=None, behavior=None),
    dict(inputs=[["foo", "$.b"]], outputs=None, behavior=None),
    dict(inputs=[["$.a", "$.b[1,2]"]], outputs=None, behavior=None),
]


def test_io_workflows_deploy(vectors):
    for v in vectors["io_workflows"]:
        rc, msg = engine.validate_deployment(io_workflow(v).to_xml())
        assert rc == 0, (v["name"], msg)


@pytest.mark.parametrize("b", BAD)
def test_invalid_io_mappings_rejected_like_the_oracle(b):
    xml = io_workflow(b).to_xml()
    o = zbref.Oracle()
    with pytest.raises(zbref.ZbrefError) as ei:
        o.deploy(xml, 100, 1)
    rc, msg = engine.validate_deployment(xml)
    assert rc == -4, (rc, msg)
    assert msg == str(ei.value)
