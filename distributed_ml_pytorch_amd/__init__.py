"""distributed_ml_pytorch_amd — MI355X-native asynchronous-SGD (Downpour) training engine.

Capabilities of bkpcoding/distributed_ML_pytorch (parameter-server ASGD with
push/pull every N steps, the asgd.optim API, the example CLI and launcher),
re-designed for AMD Instinct MI355X (gfx950): flat parameter arenas, fused
HIP kernels, RCCL over xGMI, plus sharded-PS ASGD and bucketed sync DP.
"""
__version__ = "0.1.0"

from . import models, ops, parallel, utils  # noqa: F401
