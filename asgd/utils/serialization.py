from distributed_ml_pytorch_amd.utils.serialization import (  # noqa: F401
    ravel_model_params, unravel_model_params)
