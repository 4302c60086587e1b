#!/usr/bin/env python
"""Point-to-point demo (the reference's pytorch_p2p_ex.py): rank 0 sends a tensor to rank 1.

CPU/gloo by default; ``--rccl`` sends a GPU tensor over RCCL instead (needs 2 GPUs).
Every send is waited on (the reference pattern, kept explicit here).
"""
import argparse
import os

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def run(rank, size, use_rccl):
    dev = torch.device("cuda", rank) if use_rccl else torch.device("cpu")
    tensor = torch.zeros(1, device=dev)
    if rank == 0:
        tensor += 1
        dist.send(tensor=tensor, dst=1)
    else:
        dist.recv(tensor=tensor, src=0)
    print("Rank ", rank, " has data ", tensor[0].item(), flush=True)


def init_process(rank, size, use_rccl, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if use_rccl:
        torch.cuda.set_device(rank)
    dist.init_process_group("nccl" if use_rccl else "gloo", rank=rank, world_size=size)
    try:
        run(rank, size, use_rccl)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--rccl", action="store_true")
    ap.add_argument("--port", type=int, default=29500)
    a = ap.parse_args()
    mp.set_start_method("spawn")
    procs = [mp.Process(target=init_process, args=(r, 2, a.rccl, a.port)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join()
