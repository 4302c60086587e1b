"""Reference-compatible import surface: ``asgd.optim``, ``asgd.server``, ``asgd.utils``.

The reference package ``asgd`` (/root/reference/asgd) is importable under the same
names here; everything is implemented in ``distributed_ml_pytorch_amd``.
"""
