"""The reference example's models (LeNet, AlexNet), importable as in the reference."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_ml_pytorch_amd.models import MLP, AlexNet, LeNet, resnet18, resnet50, vit_b16  # noqa: E402,F401
