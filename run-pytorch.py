#!/usr/bin/env python
"""Job submission: the reference submitted example/main.py to AzureML with no
arguments (run-pytorch.py:7-19).  Here the job runs on this node: 1 parameter
server + N workers (one per GPU with --gpus), with every argument forwarded.

    python run-pytorch.py --nproc 3 -- --model lenet --epochs 1
    python run-pytorch.py --nproc 8 --gpus -- --model resnet18 --ps sharded
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_ml_pytorch_amd.launch import main  # noqa: E402

if __name__ == "__main__":
    argv = sys.argv[1:]
    if "--" in argv:
        i = argv.index("--")
        argv = argv[:i] + [os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                        "example", "main.py"), "--"] + argv[i + 1:]
    main(argv)
