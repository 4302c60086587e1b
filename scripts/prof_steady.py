#!/usr/bin/env python
"""Steady-state per-step kernel breakdown from a rocprofv3 kernel_trace.csv.

Step boundaries are the dispatches of a once-per-step kernel (default: the fused
ASGD optimizer).  The last ``--steps`` complete steps are summarised: wall time
per step (boundary to boundary), busy kernel time, and the top kernels by time
per step.  Tuning sweeps and graph capture at the start of the run are excluded.
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    return n[:110]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="asgd_fused_step")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(marks) < a.steps + 1:
        raise SystemExit(f"only {len(marks)} marker dispatches")
    lo, hi = marks[-a.steps - 1], marks[-1]
    win = rows[lo + 1:hi + 1]
    t0 = int(rows[lo]["End_Timestamp"])
    t1 = int(rows[hi]["End_Timestamp"])
    wall = (t1 - t0) / 1e3 / a.steps
    per = defaultdict(float)
    cnt = defaultdict(int)
    fam = defaultdict(float)
    for r in win:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 / a.steps
        k = short(r["Kernel_Name"])
        per[k] += d
        cnt[k] += 1
        fam[re.sub(r"<.*", "", k)] += d
    busy = sum(per.values())
    print(f"steady state over last {a.steps} steps: wall {wall:.1f} us/step, kernel busy "
          f"{busy:.1f} us/step ({100 * busy / wall:.1f}%), {len(win) / a.steps:.0f} dispatches/step")
    print(f"{'us/step':>9} {'%':>6} {'calls':>6}  kernel")
    for k, v in sorted(per.items(), key=lambda kv: -kv[1])[:a.top]:
        print(f"{v:9.1f} {100 * v / busy:6.2f} {cnt[k] / a.steps:6.1f}  {k}")
    print("\nby family:")
    for k, v in sorted(fam.items(), key=lambda kv: -kv[1])[:20]:
        print(f"{v:9.1f} us {100 * v / busy:6.2f}%  {k}")


if __name__ == "__main__":
    main()
