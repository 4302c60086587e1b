from distributed_ml_pytorch_amd.parallel.asgd import Asynchronous, DownpourSGD  # noqa: F401
