#!/usr/bin/env python
"""Distbelief training example: same flags and roles as the reference's example/main.py.

    python example/main.py --no-distributed                       # plain SGD (make single)
    python example/main.py --no-distributed --cuda                # on one MI355X (make gpu)
    python example/main.py --rank 0 --world-size 3 --server       # PS (make server)
    python example/main.py --rank 1 --world-size 3                # worker (make first)
    python -m distributed_ml_pytorch_amd.launch --nproc 3 -- example/main.py --model lenet
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_ml_pytorch_amd.cli import main  # noqa: E402

if __name__ == "__main__":
    main(sys.argv[1:])
