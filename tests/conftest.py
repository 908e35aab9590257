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


@pytest.fixture(scope="session")
def vectors():
    import json

    with open(os.path.join(ROOT, "tests", "golden", "reference_vectors.json")) as f:
        return json.load(f)
