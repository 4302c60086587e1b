#!/usr/bin/env python
"""Every dispatch of ONE steady-state step, in launch order, from a rocprofv3
kernel_trace.csv: start offset, duration, gap to the previous dispatch and the
kernel (step boundary = the once-per-step marker kernel, default the fused
optimizer).  Shows which launches are latency-bound (short kernels on small
tensors) and where the gaps are."""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="asgd_fused_step")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    lo, hi = marks[-2], marks[-1]
    t0 = int(rows[lo]["End_Timestamp"])
    prev = t0
    tot = gaps = 0.0
    print(f"{'start':>8} {'dur':>7} {'gap':>6}  kernel (grid)")
    for r in rows[lo + 1:hi + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        d, gp = (e - s) / 1e3, (s - prev) / 1e3
        tot += d
        gaps += max(gp, 0.0)
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:90]
        grid = r.get("Grid_Size", r.get("Grid_Size_X", ""))
        print(f"{(s - t0) / 1e3:8.1f} {d:7.1f} {gp:6.1f}  {n} ({grid})")
        prev = e
    print(f"busy {tot:.1f} us, gaps {gaps:.1f} us, wall {(prev - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
