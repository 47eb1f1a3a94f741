import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rnnt-inference_amd"))
sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden", "golden.npz")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP engine compute calls)")


@pytest.fixture(scope="session")
def golden():
    return dict(np.load(GOLDEN, allow_pickle=False))


@pytest.fixture(scope="session")
def ckpt():
    from rnnt_amd import synthetic
    return synthetic.make_checkpoint(synthetic.DEFAULT_SEED)


@pytest.fixture(scope="session")
def pm_golden(ckpt, golden):
    """int8 + bf16 PreparedModel quantised with the reference's own calibrated amax."""
    from rnnt_amd import weights
    return weights.prepare_model(ckpt, golden["calib_amax"], bf16=True)


@pytest.fixture(scope="session")
def pm_f32(ckpt, golden):
    from rnnt_amd import weights
    return weights.prepare_model(ckpt, golden["calib_amax"], bf16=False)


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as o
    o.lib()
    return o
