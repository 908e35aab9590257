import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# GPU tests run the product configuration (the drain's size pass trusts the value lengths the emitting kernels
# wrote); tests/test_gpu_parity.py runs every case a second time with ZB_VLEN_CHECK=1, where the size pass
# checks each of those lengths against the encoder's dry run
os.environ.pop("ZB_VLEN_CHECK", None)
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box via gpurun)")


@pytest.fixture(autouse=True)
def _guard_bands(request):
    """Under the guard-band build (ZB_CHECKED_LIBRARY=1, GPU tests): a test fails when any kernel launched during
    it wrote outside its buffer (zeebe_amd/csrc/zb_checked.hpp)."""
    if os.environ.get("ZB_CHECKED_LIBRARY") != "1" or request.node.get_closest_marker("gpu") is None:
        yield
        return
    from zeebe_amd import engine

    before = engine.checked_violations()
    yield
    after = engine.checked_violations()
    assert before is not None and after is not None, "ZB_CHECKED_LIBRARY=1 but the guard-band build is not loaded"
    assert after[0] == before[0], "guard-band violations during the test: %d (see stderr / ZB_CHECKED_TRACE)" % (
        after[0] - before[0])


@pytest.fixture(scope="session")
def vectors():
    import json

    with open(os.path.join(ROOT, "tests", "golden", "reference_vectors.json")) as f:
        return json.load(f)
