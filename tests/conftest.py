import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: multi-process or long-running test")
    config.addinivalue_line("markers", "strict_native: stock GPU kernels raise (ops._policy)")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True)
def _stock_oracle_mode(request):
    """GPU tests compare the native kernels against fp32 PyTorch oracles, which
    run through the same layers on stock kernels: the explicit oracle mode of
    ``ops._policy`` (outside it a GPU tensor that leaves native coverage
    raises).  Tests marked ``strict_native`` run with it OFF."""
    if "strict_native" in request.keywords:
        yield
        return
    from distributed_ml_pytorch_amd.ops._policy import stock_allowed

    with stock_allowed(True):
        yield
