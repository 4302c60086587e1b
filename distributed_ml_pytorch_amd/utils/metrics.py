"""Per-iteration training log + throughput meters (reference §5.5).

The reference appends ``{timestamp, iteration, training_loss[, test_loss,
test_accuracy]}`` per iteration and writes a pandas CSV to
``log/{single,gpu,node<rank>}.csv`` (/root/reference/example/main.py:76-105),
crashing when ``log/`` does not exist.  Same schema here, plus
``epoch``, ``samples_per_sec`` and free-form extras; the directory is created.
GPU losses are accumulated as tensors and only synchronised at log points,
so logging never stalls the step pipeline (the reference synced every step
with ``loss.item()``, main.py:79).
"""
from __future__ import annotations

import csv
import os
import time
from datetime import datetime

import torch

BASE_FIELDS = ["index", "timestamp", "epoch", "iteration", "training_loss", "test_loss",
               "test_accuracy", "samples_per_sec"]


class IterationLog:
    def __init__(self):
        self.rows: list[dict] = []
        self._pending: list[tuple[dict, torch.Tensor]] = []

    def append(self, epoch: int, iteration: int, loss, **extra):
        row = {"timestamp": datetime.now().isoformat(sep=" "), "epoch": epoch,
               "iteration": iteration, **extra}
        if isinstance(loss, torch.Tensor):
            self._pending.append((row, loss.detach()))
        else:
            row["training_loss"] = float(loss)
        self.rows.append(row)
        return row

    def flush_pending(self):
        if not self._pending:
            return
        vals = torch.stack([t.float().reshape(()) for _, t in self._pending]).tolist()
        for (row, _), v in zip(self._pending, vals):
            row["training_loss"] = v
        self._pending.clear()

    def last(self) -> dict:
        self.flush_pending()
        return self.rows[-1] if self.rows else {}

    def to_csv(self, path: str):
        self.flush_pending()
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        fields = list(BASE_FIELDS)
        for r in self.rows:
            for k in r:
                if k not in fields:
                    fields.append(k)
        with open(path, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=fields)
            w.writeheader()
            for i, r in enumerate(self.rows):
                w.writerow({"index": i, **r})
        return path


def log_path(no_distributed: bool, cuda: bool, rank: int | None, log_dir: str = "log") -> str:
    if no_distributed:
        return os.path.join(log_dir, "gpu.csv" if cuda else "single.csv")
    return os.path.join(log_dir, f"node{rank}.csv")


class Throughput:
    """Wall-clock samples/sec with optional device synchronisation."""

    def __init__(self, sync_cuda: bool = False):
        self.sync_cuda = sync_cuda
        self.reset()

    def reset(self):
        if self.sync_cuda:
            torch.cuda.synchronize()
        self.t0 = time.perf_counter()
        self.samples = 0

    def add(self, n: int):
        self.samples += n

    def rate(self) -> float:
        if self.sync_cuda:
            torch.cuda.synchronize()
        dt = time.perf_counter() - self.t0
        return self.samples / dt if dt > 0 else 0.0


class _Phase:
    __slots__ = ("timer", "name", "t")

    def __init__(self, timer, name):
        self.timer, self.name = timer, name

    def __enter__(self):
        self.t = time.perf_counter()
        return self

    def __exit__(self, *a):
        dt = time.perf_counter() - self.t
        tm = self.timer
        tm.totals[self.name] = tm.totals.get(self.name, 0.0) + dt
        tm.counts[self.name] = tm.counts.get(self.name, 0) + 1
        return False


class StepTimer:
    """Host-side time per named step phase (compute, push, pull-issue,
    land).  The GPU work of these phases is asynchronous; the host times say how
    long the CPU spends issuing them (what an eager step costs beyond the GPU), and
    the PS clients add device-side span times of their side-stream collectives
    (``push_device_ms`` / ``pull_device_ms`` in their stats)."""

    def __init__(self):
        self.totals: dict[str, float] = {}
        self.counts: dict[str, int] = {}

    def time(self, name: str):
        return _Phase(self, name)

    def reset(self):
        self.totals.clear()
        self.counts.clear()

    def summary(self) -> dict:
        return {k: {"total_s": round(v, 6), "count": self.counts[k],
                    "mean_ms": round(1e3 * v / max(self.counts[k], 1), 4)}
                for k, v in self.totals.items()}


class ClockSampler:
    """Graphics clock (MHz) and socket power (W) of one GPU, sampled by a host
    thread through amdsmi while a timed window runs, so box-to-box variance in a
    benchmark line is visible next to the number (a throttled box reads lower
    sclk).  These are the SMU's reported values, not the in-kernel clock
    (MI355X_MICROARCH.md, DVFS give-back item 6); every failure (no amdsmi, no
    permission, no matching device) yields ``None`` instead of an exception."""

    def __init__(self, device_index: int = 0, period_s: float = 0.004):
        self.period = period_s
        self.device_index = device_index
        self._h = None
        self._smi = None
        self._thr = None
        self._stop = None
        self.samples: list[tuple[float, float | None]] = []
        try:
            import amdsmi

            amdsmi.amdsmi_init()
            self._smi = amdsmi
            hs = amdsmi.amdsmi_get_processor_handles()
            self._h = self._match(hs)
        except Exception:
            self._h = None

    def _match(self, hs):
        if not hs:
            return None
        try:   # same PCI bus as the torch device when torch reports one
            props = torch.cuda.get_device_properties(self.device_index)
            bus = getattr(props, "pci_bus_id", None)
            if bus is not None:
                for h in hs:
                    bdf = self._smi.amdsmi_get_gpu_device_bdf(h)
                    if int(bdf.split(":")[1], 16) == int(bus):
                        return h
        except Exception:
            pass
        return hs[0] if len(hs) == 1 else hs[min(self.device_index, len(hs) - 1)]

    def _read(self, extra: bool = False):
        """(sclk, socket power[, mclk, fabric clock, hotspot temperature]) -- the extra
        three only when ``extra`` (every 4th sample: they explain box-to-box spread
        that sclk alone does not, e.g. a lower memory clock)."""
        smi = self._smi
        clk = smi.amdsmi_get_clock_info(self._h, smi.AmdSmiClkType.SYS)["clk"]
        pw = None
        try:
            p = smi.amdsmi_get_power_info(self._h)
            pw = p.get("current_socket_power")
            if not isinstance(pw, (int, float)) or pw <= 0:
                pw = p.get("average_socket_power")
            pw = float(pw) if isinstance(pw, (int, float)) and pw > 0 else None
        except Exception:
            pass
        mclk = fclk = temp = None
        if extra:
            for kind, attr in ((smi.AmdSmiClkType.MEM, "m"), (smi.AmdSmiClkType.DF, "f")):
                try:
                    v = float(smi.amdsmi_get_clock_info(self._h, kind)["clk"])
                    if attr == "m":
                        mclk = v
                    else:
                        fclk = v
                except Exception:
                    pass
            try:
                temp = float(smi.amdsmi_get_temp_metric(self._h, smi.AmdSmiTemperatureType.HOTSPOT,
                                                        smi.AmdSmiTemperatureMetric.CURRENT))
            except Exception:
                pass
        return float(clk), pw, mclk, fclk, temp

    def start(self):
        if self._h is None:
            return self
        import threading

        self.samples = []
        self._stop = threading.Event()

        def loop():
            k = 0
            while not self._stop.is_set():
                try:
                    self.samples.append(self._read(extra=k % 4 == 0))
                except Exception:
                    return
                k += 1
                self._stop.wait(self.period)

        self._thr = threading.Thread(target=loop, daemon=True)
        self._thr.start()
        return self

    def stop(self) -> dict | None:
        if self._thr is None:
            return None
        self._stop.set()
        self._thr.join(timeout=1.0)
        self._thr = None
        clks = [x[0] for x in self.samples if x[0] and x[0] > 0]
        pws = [x[1] for x in self.samples if x[1]]
        if not clks:
            return None
        out = {"samples": len(clks), "sclk_mhz_mean": round(sum(clks) / len(clks), 1),
               "sclk_mhz_min": min(clks), "sclk_mhz_max": max(clks)}
        if pws:
            out["power_w_mean"] = round(sum(pws) / len(pws), 1)
            out["power_w_max"] = max(pws)
        for i, name in ((2, "mclk_mhz_mean"), (3, "fclk_mhz_mean"), (4, "hotspot_c_mean")):
            v = [x[i] for x in self.samples if len(x) > i and x[i] is not None]
            if v:
                out[name] = round(sum(v) / len(v), 1)
        return out


def classification_report(conf: torch.Tensor, names=None, digits: int = 2) -> str:
    """Per-class precision / recall / F1 / support from a [C, C] confusion matrix
    (rows = true class), laid out like sklearn's ``classification_report`` that the
    reference prints on its verbose evaluation (/root/reference/example/main.py:127-131)."""
    conf = conf.to(torch.float64)
    c = conf.shape[0]
    names = list(names) if names is not None else [str(i) for i in range(c)]
    tp = conf.diag()
    support = conf.sum(1)
    predicted = conf.sum(0)
    prec = torch.where(predicted > 0, tp / predicted.clamp_min(1), torch.zeros_like(tp))
    rec = torch.where(support > 0, tp / support.clamp_min(1), torch.zeros_like(tp))
    f1 = torch.where(prec + rec > 0, 2 * prec * rec / (prec + rec).clamp_min(1e-30),
                     torch.zeros_like(tp))
    total = float(support.sum())
    width = max(max(len(n) for n in names), len("weighted avg"), digits)
    head = " " * width + "".join(f"{h:>10}" for h in ("precision", "recall", "f1-score",
                                                      "support"))
    lines = [head, ""]
    fmt = "{:>%d}" % width + ("{:>10.%df}" % digits) * 3 + "{:>10}"
    for i in range(c):
        lines.append(fmt.format(names[i], float(prec[i]), float(rec[i]), float(f1[i]),
                                int(support[i])))
    lines.append("")
    acc = float(tp.sum()) / total if total else 0.0
    lines.append(("{:>%d}" % width).format("accuracy") + " " * 20
                 + ("{:>10.%df}" % digits).format(acc) + f"{int(total):>10}")
    lines.append(fmt.format("macro avg", float(prec.mean()), float(rec.mean()),
                            float(f1.mean()), int(total)))
    w = support / total if total else support
    lines.append(fmt.format("weighted avg", float((prec * w).sum()), float((rec * w).sum()),
                            float((f1 * w).sum()), int(total)))
    return "\n".join(lines)
