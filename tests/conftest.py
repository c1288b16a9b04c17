import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return np.load(os.path.join(GOLDEN, name + ".npz"))
    return load


@pytest.fixture
def tune():
    """Kernel switches for one test (include/svc_hip.h, svc_ctx_set_config "tune.<name>"): tune(target, name=value, ...)
    on an SVCEngine, or with target None on the op-level entry points' context. Every context touched is reset to its
    creation-time switches when the test ends."""
    from svc_inference_pipeline_amd import _lib
    touched = {}

    def set_(target, **kv):
        if target is None:
            _lib.tune(None, **kv)
        else:
            target.tune(**kv)
        touched[id(target)] = target

    yield set_
    for target in touched.values():
        if target is None:
            _lib.tune(None, reset=1)
        elif target._ctx:  # (an engine the test closed itself has nothing left to reset)
            target.tune(reset=1)
