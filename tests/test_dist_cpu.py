"""Multi-process tests of the distributed runtime on CPU (gloo, localhost ranks).

The reference's only "cluster" test pattern is localhost processes over gloo
(pytorch_p2p_ex.py:18-36); these tests use it to cover the PS protocol, the
sharded PS, sync DP, messaging, the launcher and the p2p demo.
"""
import os
import socket
import subprocess
import sys
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _run(fn, world, *args):
    port = _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_entry, args=(fn, r, world, port, q, args)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, res = q.get(timeout=240)
        out[r] = res
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0, f"rank exited with {p.exitcode}"
    for r, res in out.items():
        if isinstance(res, BaseException) or (isinstance(res, str) and res.startswith("ERR")):
            raise AssertionError(f"rank {r}: {res}")
    return out


def _entry(fn, rank, world, port, q, args):
    try:
        _init(rank, world, port)
        res = fn(rank, world, *args)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, res))
    except BaseException as e:  # report to the parent instead of hanging it
        import traceback

        q.put((rank, "ERR " + traceback.format_exc()))


# ---------------------------------------------------------------- central PS
def _ps_topology(rank, world):
    from distributed_ml_pytorch_amd.runtime.dist import DistInfo
    from distributed_ml_pytorch_amd.runtime.trainer import TrainConfig, run_training

    cfg = TrainConfig(model="mlp", n_train=512, n_test=128, test_batch_size=128, batch_size=32,
                      epochs=1, lr=0.05, n_push=3, n_pull=4, mode="asgd", ps="central",
                      cuda=False, log_interval=0, evaluate=True, verbose=False,
                      log_dir=tempfile.mkdtemp())
    info = DistInfo(rank, world, rank, "gloo", torch.device("cpu"))
    res = run_training(cfg, info)
    return {k: v for k, v in res.items() if isinstance(v, (int, float, str, dict))}


def test_central_ps_one_server_two_workers():
    out = _run(_ps_topology, 3)
    ps = out[0]
    assert ps["role"] == "ps"
    steps = 512 // 32
    # each worker: 1 init ParameterUpdate, ceil(steps/n_push) pushes, ceil(steps/n_pull) pulls
    assert ps["counts"]["ParameterUpdate"] == 2
    assert ps["counts"]["GradientUpdate"] == 2 * -(-steps // 3)
    assert ps["counts"]["ParameterRequest"] == 2 * -(-steps // 4)
    assert ps["version"] == ps["counts"]["GradientUpdate"]
    for r in (1, 2):
        assert out[r]["role"] == "worker" and out[r]["steps"] == steps
        assert out[r]["test_accuracy"] > 0.3       # learnable synthetic task


def _ps_delta_scale(rank, world):
    from distributed_ml_pytorch_amd.parallel.server import ParameterServer

    out = {}
    for mode, expect in (("sum", 1.0), ("mean", 1.0 / 3), (0.25, 0.25)):
        ps = ParameterServer(numel=10, workers=[1, 2, 3], delta_scale=mode)
        before = ps.shard[:10].clone()
        d = torch.arange(10, dtype=torch.float32)
        ps._apply(d)
        out[str(mode)] = float((ps.shard[:10] - before - expect * d).abs().max())
    return out


def test_ps_delta_scale_sum_mean_float():
    """Central PS push combine: the reference's raw sum (1.0), the mean over its
    workers (1/W) or a given factor, applied to every pushed delta."""
    out = _run(_ps_delta_scale, 1)
    assert all(v < 1e-6 for v in out[0].values()), out


# --------------------------------------------------------------- sharded PS
def _sharded(rank, world):
    from distributed_ml_pytorch_amd.models import build_model
    from distributed_ml_pytorch_amd.parallel.asgd import Asynchronous
    from distributed_ml_pytorch_amd.parallel.clients import ShardedPSClient

    torch.manual_seed(100 + rank)           # different init per rank: broadcast fixes it
    m, _, _ = build_model("mlp")
    opt = Asynchronous(m.parameters(), lr=0.1, n_push=2, n_pull=2, model=m,
                       client=ShardedPSClient(staleness=0))
    p0 = opt.arena.p32.clone()
    gathered = [torch.zeros_like(p0) for _ in range(world)]
    dist.all_gather(gathered, p0)
    assert all(torch.equal(g, gathered[0]) for g in gathered), "init not broadcast"
    torch.manual_seed(rank)
    deltas = []
    for step in range(4):
        x, y = torch.randn(8, 1, 28, 28), torch.randint(0, 10, (8,))
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        deltas.append(-0.1 * opt.arena.g32.clone())
        opt.step()
    opt.finish()
    # after step 2 (push at idx 2, pull at idx 2 with staleness 0) every rank holds
    # p0 + sum over ranks of their pushed deltas; steps 3 add local-only updates.
    mine = torch.stack(deltas[:3]).sum(0)
    tot = mine.clone()
    dist.all_reduce(tot)
    expect_after_pull = p0 + tot
    local_after = expect_after_pull + deltas[3]
    err = float((opt.arena.p32 - local_after).abs().max())
    return err


def test_sharded_ps_collective_push_pull():
    out = _run(_sharded, 2)
    for r, err in out.items():
        assert err < 1e-5, (r, err)


# ----------------------------------------------------------------- sync DP
def _ddp(rank, world, bucket_mb=0.25, steps=1, momentum=0.0):
    from distributed_ml_pytorch_amd.models import build_model
    from distributed_ml_pytorch_amd.parallel.arena import attach_arena
    from distributed_ml_pytorch_amd.parallel.ddp import BucketedAllReduce, FusedSGD

    torch.manual_seed(0)
    m, _, _ = build_model("mlp")
    arena = attach_arena(m, shadow_dtype=None)
    ddp = BucketedAllReduce(arena, bucket_mb=bucket_mb)
    opt = FusedSGD(list(m.parameters()), arena, lr=0.1, momentum=momentum,
                   grad_scale=1.0 / world)
    g = torch.Generator().manual_seed(7)
    batches = [(torch.randn(8 * world, 1, 28, 28, generator=g),
                torch.randint(0, 10, (8 * world,), generator=g)) for _ in range(steps)]
    for xs, ys in batches:
        x, y = xs[rank * 8:(rank + 1) * 8], ys[rank * 8:(rank + 1) * 8]
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        ddp.synchronize()
        opt.step()
    # single-process oracle: stock torch.optim.SGD on the full batch
    torch.manual_seed(0)
    ref, _, _ = build_model("mlp")
    ropt = torch.optim.SGD(ref.parameters(), lr=0.1, momentum=momentum)
    for xs, ys in batches:
        ropt.zero_grad()
        torch.nn.functional.cross_entropy(ref(xs), ys).backward()
        ropt.step()
    got = arena.ravel()
    exp = torch.cat([p.detach().reshape(-1) for p in ref.parameters()])
    return {"err": float((got - exp).abs().max()), "buckets": ddp.num_buckets}


def test_bucketed_allreduce_matches_full_batch_sgd():
    out = _run(_ddp, 2)
    for r, res in out.items():
        assert res["err"] < 1e-5, (r, res)
        assert res["buckets"] >= 2          # 0.25 MB buckets -> several per 2 MB model


@pytest.mark.slow
@pytest.mark.parametrize("bucket_mb", [0.1, 4.0])
def test_bucketed_allreduce_4ranks_momentum_matches_full_batch(bucket_mb):
    """4 gloo ranks, several steps with momentum, many small buckets vs one
    bucket: identical to single-process SGD on the concatenated batch."""
    out = _run(_ddp, 4, bucket_mb, 3, 0.9)
    for r, res in out.items():
        assert res["err"] < 2e-5, (r, res)
        assert (res["buckets"] >= 3) == (bucket_mb < 1), res


# --------------------------------------------------------------- messaging
def _messaging(rank, world):
    from distributed_ml_pytorch_amd.parallel import messaging as M

    workers = dist.new_group(list(range(1, world)))
    if rank == 0:
        got = []

        class L(M.MessageListener):
            def receive(self, sender, code, parameter):
                got.append((sender, code.name, None if parameter is None else float(parameter.sum())))

        lst = L(numel=4)
        lst.run()   # returns on Shutdown
        return got
    M.send_message(M.MessageCode.GradientUpdate, torch.ones(4) * rank, dst=0, step=3)
    M.send_message(M.MessageCode.ParameterRequest, torch.ones(4), dst=0)   # payload dropped
    M.SENDS.drain()
    dist.barrier(group=workers)          # every worker's messages are out
    if rank == world - 1:
        M.send_message(M.MessageCode.Shutdown, None, dst=0)
        M.SENDS.drain()
    return "ok"


def test_messaging_header_payload_and_listener():
    out = _run(_messaging, 3)
    got = out[0]
    grads = sorted(g for g in got if g[1] == "GradientUpdate")
    reqs = [g for g in got if g[1] == "ParameterRequest"]
    assert grads == [(1, "GradientUpdate", 4.0), (2, "GradientUpdate", 8.0)]
    assert sorted(r[0] for r in reqs) == [1, 2] and all(r[2] is None for r in reqs)


# --------------------------------------------------------- launcher / demos
def test_p2p_demo_script():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "pytorch_p2p_ex.py"), "--port",
                        str(_port())], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Rank  1  has data  1.0" in r.stdout


def test_launcher_runs_reference_topology(tmp_path):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "run-pytorch.py"), "--nproc", "3",
                        "--timeout", "200", "--", "--model", "mlp", "--epochs", "1",
                        "--n-train", "256", "--n-test", "64", "--test-batch-size", "64",
                        "--log-interval", "0", "--log-dir", str(tmp_path / "log")],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-2000:])
    assert os.path.exists(tmp_path / "log" / "node1.csv")
    assert os.path.exists(tmp_path / "log" / "node2.csv")
    assert "[ps] finished" in r.stdout


def test_bench_two_ranks_sharded_ps_cpu():
    """bench.py under torch.distributed.run with 2 gloo ranks: one JSON line from
    rank 0 and every rank leaves the time-to-target phase together."""
    import json

    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--model", "lenet", "--batch", "16", "--n-push", "2", "--n-pull", "2",
           "--ttl-target", "2.2", "--ttl-max-steps", "60"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 3 and out["value"] > 0
    assert out["config"]["global_batch"] == 32
    assert "sharded" in out["config"]["parallelism"]


# ------------------------------------------------------ PS worker liveness
def _liveness(rank, world):
    import time

    from distributed_ml_pytorch_amd.parallel import messaging as M
    from distributed_ml_pytorch_amd.parallel.server import ParameterServer

    n = 64
    if rank == 0:
        ps = ParameterServer(numel=n, worker_timeout=1.0)
        t0 = time.monotonic()
        st = ps.run()
        st["secs"] = time.monotonic() - t0
        st["shard"] = ps.parameters()[:4].tolist()
        return st
    tr = M.SendTracker()
    M.send_message(M.MessageCode.ParameterUpdate, torch.zeros(n), tracker=tr)
    if rank == 2:
        # hangs from the PS's point of view: one push, then silence, no Shutdown
        M.send_message(M.MessageCode.GradientUpdate, torch.ones(n), tracker=tr)
        tr.drain()
        return "silent"
    for i in range(8):
        time.sleep(0.3)
        M.send_message(M.MessageCode.GradientUpdate, torch.full((n,), 0.5), step=i, tracker=tr)
    M.send_message(M.MessageCode.Shutdown, tracker=tr)
    tr.drain()
    return "ok"


def test_ps_drops_silent_worker_and_keeps_serving():
    """a worker that goes silent (no Shutdown) is dropped after
    ``worker_timeout`` while the PS keeps applying the live worker's pushes and
    then exits cleanly -- the reference's PS would block in recv forever."""
    out = _run(_liveness, 3)
    ps = out[0]
    assert ps["dropped"] == [2]
    assert ps["counts"]["GradientUpdate"] == 9 and ps["version"] == 9
    assert ps["shard"] == [5.0] * 4          # 0 + 1 (silent worker) + 8 x 0.5
    assert ps["secs"] < 60


def _bucket_calibration(rank, world):
    from distributed_ml_pytorch_amd.parallel.ddp import calibrate_bucket_mb

    pick, table = calibrate_bucket_mb(None, "cpu", candidates=(0.25, 0.5, 1.0), reps=2)
    return pick, table


def test_sync_dp_bucket_is_measured_and_agreed():
    """SURVEY §5.8 / VERDICT r5: the sync-DP bucket is measured on the live group (all-reduce
    timings of candidate sizes, MAX-reduced so every rank decides the same), not a constant."""
    out = _run(_bucket_calibration, 3)
    picks = {r: res[0] for r, res in out.items()}
    tables = {r: res[1] for r, res in out.items()}
    assert len(set(picks.values())) == 1, picks
    assert all(t == tables[0] for t in tables.values()), tables
    assert [row[0] for row in tables[0]] == [0.25, 0.5, 1.0]
    assert picks[0] in (0.25, 0.5, 1.0) and all(row[2] > 0 for row in tables[0])
