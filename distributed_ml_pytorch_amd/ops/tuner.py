"""Per-shape kernel selection by measurement ("measure, don't guess").

The conv kernels are compiled for several tile configurations
(``_native.conv_configs()``).  The first time a (pass, shape) is seen, every
eligible configuration is timed with HIP events on the current stream and the
fastest is cached for the process.  Tuning never runs while a stream is being
captured into a graph (the heuristic default is used then) and can be
disabled with ``DMP_CONV_TUNE=0``.

* ``DMP_CONV_TUNE_SEED=a.json[:b.json]``: READ-ONLY picks loaded at start-up
  (``bench.py`` points it at the committed ``tuning/mi355x_tune_cache.json``,
  measured with more rounds than a cold start can afford: deterministic picks
  and no tuning at start-up).  Never written: shapes missing from it are tuned
  in memory only.
* ``DMP_CONV_TUNE_CACHE=path.json``: a read-write cache persisted across
  processes.  New picks are MERGED into the file under an exclusive lock, so
  concurrent ranks of one node do not drop each other's entries.  Regenerating
  the committed seed is an explicit step (``scripts/gpu_make_tune_cache.sh``
  copies it, tunes into the copy, and the copy is committed by hand).
"""
from __future__ import annotations

import json
import os
import threading

try:
    import fcntl
except ImportError:  # pragma: no cover - non-POSIX
    fcntl = None

import torch

_lock = threading.RLock()   # a candidate may tune an inner kernel (1x1 conv -> GEMM)


class KernelTuner:
    def __init__(self):
        self.cache: dict[tuple, int] = {}
        self.timings: dict[tuple, dict] = {}
        self.enabled = os.environ.get("DMP_CONV_TUNE", "1") != "0"
        self.path = os.environ.get("DMP_CONV_TUNE_CACHE")
        self.reps = int(os.environ.get("DMP_CONV_TUNE_REPS", "5"))
        self.rounds = int(os.environ.get("DMP_CONV_TUNE_ROUNDS", "2"))
        self.spin = int(os.environ.get("DMP_CONV_TUNE_SPIN", "2000000"))   # GPU cycles
        self.new: dict[tuple, int] = {}     # picks made by this process
        for seed in filter(None, os.environ.get("DMP_CONV_TUNE_SEED", "").split(os.pathsep)):
            self.cache.update(self._read(seed))
        if self.path:
            self.cache.update(self._read(self.path))

    @staticmethod
    def _read(path) -> dict:
        try:
            with open(path) as f:
                return {tuple(json.loads(k)): int(v) for k, v in json.load(f).items()}
        except (OSError, ValueError):
            return {}

    def best(self, key: tuple, runner, candidates) -> int:
        got = self.cache.get(key)
        if got is not None:
            return got
        if not self.enabled or not candidates or torch.cuda.is_current_stream_capturing():
            return -1
        with _lock:
            if key in self.cache:
                return self.cache[key]
            # every candidate is warmed once, then timed in `rounds` interleaved
            # passes (min over passes): one cold or clock-ramping pass must not
            # decide the pick
            for c in candidates:
                runner(c)
            times = {c: float("inf") for c in candidates}
            for _ in range(self.rounds):
                for c in candidates:
                    a = torch.cuda.Event(enable_timing=True)
                    b = torch.cuda.Event(enable_timing=True)
                    # the GPU spins while the host enqueues the reps, so they run
                    # back-to-back: a ~10 us kernel is otherwise timed at the
                    # host's launch rate and every candidate looks the same
                    torch.cuda._sleep(self.spin)
                    a.record()
                    for _ in range(self.reps):
                        runner(c)
                    b.record()
                    b.synchronize()
                    times[c] = min(times[c], a.elapsed_time(b) / self.reps)
            best = min(times, key=times.get)
            self.cache[key] = best
            self.new[key] = best
            self.timings[key] = times
            if self.path:
                self._save()
            return best

    def _save(self):
        """Merge this process's picks into the cache file: read-merge-replace under
        an exclusive lock on a side file, so concurrent ranks of one node keep
        each other's entries (entries already on disk win for their keys only if
        this process did not tune them)."""
        try:
            os.makedirs(os.path.dirname(os.path.abspath(self.path)), exist_ok=True)
            with open(self.path + ".lock", "a") as lk:
                if fcntl is not None:
                    fcntl.flock(lk, fcntl.LOCK_EX)
                merged = self._read(self.path)
                merged.update(self.new)
                tmp = f"{self.path}.{os.getpid()}.tmp"
                with open(tmp, "w") as f:
                    json.dump({json.dumps(list(k)): v for k, v in sorted(
                        merged.items(), key=lambda kv: json.dumps(list(kv[0])))}, f, indent=0)
                os.replace(tmp, self.path)
        except OSError:
            pass

    def report(self) -> list[dict]:
        out = []
        for k, times in self.timings.items():
            best = self.cache[k]
            out.append({"key": list(k), "best": best, "best_ms": times[best],
                        "worst_ms": max(times.values())})
        return out


TUNER = KernelTuner()
