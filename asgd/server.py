from distributed_ml_pytorch_amd.parallel.server import ParameterServer, make_ps_groups  # noqa: F401
