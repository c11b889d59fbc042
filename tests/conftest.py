import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    # torch (and its HIP runtime) before any test module can load the native
    # extension at collection time: two HIP runtimes in one process leave the
    # second one with 0 visible devices
    import torch  # noqa: F401

    config.addinivalue_line("markers", "gpu: needs an MI355X (run via gpurun)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def C():
    import torch  # noqa: F401  (shared HIP runtime must load first)

    from seldon_core_amd import native

    return native()


@pytest.fixture(scope="session")
def has_gpu():
    import torch

    return torch.cuda.is_available()


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="needs a GPU")
    for item in items:
        if "gpu" in item.keywords and config.getoption("-m") not in ("gpu",):
            item.add_marker(skip)
