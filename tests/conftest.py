import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (REPO, os.path.join(REPO, "oracle"), HERE, os.path.join(REPO, "ali-fmm-and-ray-tracing_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    cache = {}

    def load(name):
        if name not in cache:
            cache[name] = np.load(os.path.join(HERE, "golden", name + ".npz"))
        return cache[name]

    return load


@pytest.fixture(scope="session")
def envelope():
    """Measured parity errors of this run (name -> value), written to gpurun_out/parity_envelope.json
    at the end of the session: the evidence the thresholds in test_gpu_parity.py are set against."""
    import json

    rec = {}
    yield rec
    if rec:
        os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
        with open(os.path.join(REPO, "gpurun_out", "parity_envelope.json"), "w") as f:
            json.dump(rec, f, indent=1, sort_keys=True)
