"""Serialization, data, metrics and checkpoint utilities."""
from . import checkpoint, data, metrics, serialization  # noqa: F401
from .serialization import ravel_model_params, unravel_model_params  # noqa: F401
