"""Local multi-process launcher (replaces the reference's AzureML ``run-pytorch.py``).

The reference submits ``example/main.py`` to an AzureML compute target without
forwarding any arguments (/root/reference/run-pytorch.py:10-16) and
otherwise relies on three hand-started shells (Makefile:13-20).  This launcher
starts ``--nproc`` ranks on this node (one per GPU with ``--gpus``), sets the
env:// rendezvous (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR=127.0.0.1 /
MASTER_PORT), forwards every argument, streams output with a rank prefix,
and tears the whole job down if any rank fails.

    python -m distributed_ml_pytorch_amd.launch --nproc 3 -- example/main.py --model lenet
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import threading
import time

from .runtime.dist import apply_hw_queue_policy


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _pump(prefix: str, stream, out):
    for line in iter(stream.readline, b""):
        out.write(f"[{prefix}] {line.decode(errors='replace')}")
        out.flush()


def launch(script: str, script_args, nproc: int, gpus: bool = False, port: int | None = None,
           python: str = sys.executable, env_extra: dict | None = None,
           timeout: float | None = None) -> int:
    port = port or free_port()
    procs = []
    threads = []
    for r in range(nproc):
        env = dict(os.environ)
        env.update({"RANK": str(r), "WORLD_SIZE": str(nproc), "LOCAL_RANK": str(r),
                    "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if gpus:
            # every rank runs several HIP streams (PS links, push/pull side
            # stream, RCCL): one queue policy for all (profiles/hw_queue_policy_r5.txt)
            apply_hw_queue_policy(nproc, env)
        if env_extra:
            env.update(env_extra)
        args = [python, script, *script_args, "--rank", str(r), "--world-size", str(nproc),
                "--master", "127.0.0.1", "--port", str(port)]
        if gpus and "--cuda" not in script_args:
            args.append("--cuda")
        p = subprocess.Popen(args, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                             start_new_session=True)
        procs.append(p)
        t = threading.Thread(target=_pump, args=(f"rank{r}", p.stdout, sys.stdout), daemon=True)
        t.start()
        threads.append(t)
    deadline = time.monotonic() + timeout if timeout else None
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            failed = [c for c in codes if c not in (None, 0)]
            if failed:
                rc = failed[0]
                break
            if all(c == 0 for c in codes):
                break
            if deadline and time.monotonic() > deadline:
                rc = 124
                break
            time.sleep(0.1)
    finally:
        if rc != 0:
            for p in procs:
                if p.poll() is None:
                    try:
                        os.killpg(p.pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
            for p in procs:
                try:
                    p.wait(timeout=10)
                except subprocess.TimeoutExpired:
                    os.killpg(p.pid, signal.SIGKILL)
        for t in threads:
            t.join(timeout=5)
    return rc


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--nproc", type=int, default=3, help="ranks (central PS: 1 PS + nproc-1 workers)")
    ap.add_argument("--gpus", action="store_true", help="one rank per GPU (adds --cuda)")
    ap.add_argument("--port", type=int, default=None)
    ap.add_argument("--timeout", type=float, default=None)
    ap.add_argument("script", nargs="?", default=None)
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    script = a.script or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                      "example", "main.py")
    args = [x for x in a.args if x != "--"]
    sys.exit(launch(script, args, a.nproc, a.gpus, a.port, timeout=a.timeout))


if __name__ == "__main__":
    main()
