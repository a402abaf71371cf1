import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(autouse=True)
def _fresh_session():
    import tensorflow_distributed_example_amd as tde
    tde.backend.clear_session()
    tde.backend.set_random_seed(0)
    yield
    tde.backend.set_global_policy(None)


@pytest.fixture
def bf16_policy():
    """Run the test under the mixed_bfloat16 policy (the bf16 MFMA kernel forms)."""
    import tensorflow_distributed_example_amd as tde
    tde.backend.set_global_policy("mixed_bfloat16")
    yield
    tde.backend.set_global_policy(None)


@pytest.fixture
def fp32_policy():
    import tensorflow_distributed_example_amd as tde
    tde.backend.set_global_policy("float32")
    yield
    tde.backend.set_global_policy(None)


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
