#!/usr/bin/env python
"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time, grouped families."""
import csv
import re
import sys
from collections import defaultdict


def family(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    n = re.sub(r"<.*", "", n)
    if n.startswith("igemm_") or "conv" in n.lower() and "dmp::" not in n:
        return "miopen:" + n.split("_")[0] + "_" + n.split("_")[1]
    return n


def main(path):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"total kernel time {tot / 1e6:.3f} ms over {sum(int(r['Calls']) for r in rows)} dispatches")
    print(f"{'ms':>9} {'%':>6} {'calls':>6} {'avg_us':>9}  kernel")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:40]:
        print(f"{float(r['TotalDurationNs']) / 1e6:9.3f} {float(r['Percentage']):6.2f} "
              f"{int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.2f}  {r['Name'][:120]}")
    fam = defaultdict(float)
    for r in rows:
        fam[family(r["Name"])] += float(r["TotalDurationNs"])
    print("\nby family:")
    for k, v in sorted(fam.items(), key=lambda kv: -kv[1])[:25]:
        print(f"{v / 1e6:9.3f} ms {100 * v / tot:6.2f}%  {k[:100]}")


if __name__ == "__main__":
    main(sys.argv[1])
