from distributed_ml_pytorch_amd.parallel.asgd import DownpourSGD  # noqa: F401
