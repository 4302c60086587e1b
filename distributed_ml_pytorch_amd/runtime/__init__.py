"""Process bootstrap and the training engine."""
from .dist import DistInfo, init_distributed, shutdown  # noqa: F401
from .trainer import TrainConfig, Worker, run_training  # noqa: F401
