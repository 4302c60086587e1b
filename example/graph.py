#!/usr/bin/env python
"""Plot train/test curves from the per-iteration CSV logs (the reference's missing
example/graph.py, Makefile:9-11).  Writes docs/train_time.png and docs/test_time.png
(matplotlib optional: without it, prints a text summary)."""
import csv
import glob
import os
import sys


def load(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main(log_dir="log", out_dir="docs"):
    files = sorted(glob.glob(os.path.join(log_dir, "*.csv")))
    if not files:
        print(f"no logs under {log_dir}/")
        return 1
    series = {os.path.basename(p)[:-4]: load(p) for p in files}
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:
        for name, rows in series.items():
            last = rows[-1]
            print(f"{name}: {len(rows)} iterations, final training_loss={last.get('training_loss')}")
        return 0
    os.makedirs(out_dir, exist_ok=True)
    for key, fname in (("training_loss", "train_time.png"), ("test_loss", "test_time.png")):
        plt.figure()
        for name, rows in series.items():
            ys = [(i, float(r[key])) for i, r in enumerate(rows) if r.get(key) not in (None, "")]
            if ys:
                plt.plot([a for a, _ in ys], [b for _, b in ys], label=name)
        plt.xlabel("iteration")
        plt.ylabel(key)
        plt.legend()
        plt.savefig(os.path.join(out_dir, fname))
    return 0


if __name__ == "__main__":
    sys.exit(main(*sys.argv[1:]))
