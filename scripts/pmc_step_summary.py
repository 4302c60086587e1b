#!/usr/bin/env python
"""Per-kernel MFMA work and HBM traffic of one training step from rocprofv3 --pmc runs of the
bench (counter_collection.csv of each pass), joined with the per-kernel device time of a
steady-state profile (scripts/prof_steady.py output, no counters: the PMC runs serialise
dispatches).  Every MFMA in csrc/ is v_mfma_f32_16x16x32_bf16 = 16384 FLOP per wave instruction.
    python scripts/pmc_step_summary.py --steady profiles/resnet18_steady_state_r6_closing.txt \\
        --step-kernel asgd_fused_step_kernel A.csv B.csv C.csv"""
import argparse
import csv
import re
from collections import defaultdict


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0].strip()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steady", required=True)
    ap.add_argument("--step-kernel", default="asgd_fused_step_kernel")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("csvs", nargs="+")
    a = ap.parse_args()
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for p in a.csvs:
        for r in csv.DictReader(open(p)):
            k = short(r["Kernel_Name"])
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(k, p)].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    steps_per_pass = {}
    for p in a.csvs:
        steps_per_pass[p] = max(1, sum(len(v) for (k, q), v in disp.items()
                                       if q == p and a.step_kernel in k))
    # per-step value of each counter: divide by the step count of the pass that measured it
    per = defaultdict(dict)
    for (k, p), _ in disp.items():
        pass
    counters_pass = {}
    for p in a.csvs:
        for r in csv.DictReader(open(p)):
            counters_pass[r["Counter_Name"]] = p
    for k, cs in tot.items():
        for c, v in cs.items():
            per[k][c] = v / steps_per_pass[counters_pass[c]]
    times = {}
    for line in open(a.steady):
        m = re.match(r"\s*([\d.]+)\s+[\d.]+\s+[\d.]+\s+(.*)$", line)
        if m and "dmp::" in m.group(2) or (m and "__amd" in m.group(2)):
            times[short(m.group(2))] = times.get(short(m.group(2)), 0.0) + float(m.group(1))
    rows = []
    for k, t in times.items():
        c = per.get(k, {})
        fl = c.get("SQ_INSTS_MFMA", 0.0) * 16384
        by = c.get("FETCH_SIZE", 0.0) * 1024 + c.get("WRITE_SIZE", 0.0) * 1024
        rows.append((t, k, fl, by))
    rows.sort(reverse=True)
    T = sum(r[0] for r in rows)
    F = sum(r[2] for r in rows)
    B = sum(r[3] for r in rows)
    print(f"step: {T:.1f} us of kernels, {F / 1e12:.3f} TFLOP on MFMA ({F / T / 1e6:.0f} TF/s), "
          f"{B / 1e9:.2f} GB HBM (fetch + write) ({B / T / 1e6:.2f} TB/s)")
    print(f"{'us/step':>8} {'TF/s':>6} {'%peak':>6} {'TB/s':>6}  kernel (MFMA TF/s at 2.5 PF dense bf16 peak; HBM TB/s)")
    for t, k, fl, by in rows[:a.top]:
        tf = fl / t / 1e6 if t else 0.0
        print(f"{t:8.1f} {tf:6.0f} {100 * tf / 2500:6.1f} {by / t / 1e6 if t else 0:6.2f}  {k[:100]}")


if __name__ == "__main__":
    main()
