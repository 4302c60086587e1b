#!/usr/bin/env python
"""Summarise rocprofv3 --pmc counter_collection.csv files: per kernel, median over dispatches."""
import csv
import statistics
import sys
from collections import defaultdict


def main(paths):
    show_all = "--all" in paths
    paths = [p for p in paths if p != "--all"]
    for path in paths:
        rows = list(csv.DictReader(open(path)))
        per = defaultdict(lambda: defaultdict(list))
        for r in rows:
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:90]
            per[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        print(f"== {path}")
        for k, cs in per.items():
            if not show_all and "conv" not in k and "wgrad" not in k:
                continue
            vals = {c: statistics.median(v) for c, v in cs.items()}
            print(f"  {k}")
            print("    " + "  ".join(f"{c}={v:.4g}" for c, v in sorted(vals.items())))
            if "SQ_VALU_MFMA_BUSY_CYCLES" in vals and "SQ_BUSY_CYCLES" in vals:
                print(f"    MFMA busy / SQ busy = {vals['SQ_VALU_MFMA_BUSY_CYCLES'] / max(vals['SQ_BUSY_CYCLES'], 1):.3f}")
            if "SQ_INSTS_VALU" in vals and "SQ_INSTS_MFMA" in vals:
                print(f"    VALU/MFMA = {vals['SQ_INSTS_VALU'] / max(vals['SQ_INSTS_MFMA'], 1):.2f}  "
                      f"LDS/MFMA = {vals.get('SQ_INSTS_LDS', 0) / max(vals['SQ_INSTS_MFMA'], 1):.2f}")
            if "TCC_HIT_sum" in vals and "TCC_MISS_sum" in vals:
                print(f"    L2 hit rate = {vals['TCC_HIT_sum'] / max(vals['TCC_HIT_sum'] + vals['TCC_MISS_sum'], 1):.3f}")
            if "SQ_WAVE_CYCLES" in vals and "SQ_WAIT_ANY" in vals:
                wc = max(vals["SQ_WAVE_CYCLES"], 1)
                print(f"    of wave cycles: waiting (vmcnt/lgkmcnt/barrier) {vals['SQ_WAIT_ANY'] / wc:.3f}"
                      f"  issue-stalled {vals.get('SQ_WAIT_INST_ANY', 0) / wc:.3f}"
                      f"  issuing {vals.get('SQ_ACTIVE_INST_ANY', 0) / wc:.3f}")
            if "SQ_LDS_BANK_CONFLICT" in vals and "SQ_LDS_IDX_ACTIVE" in vals:
                print(f"    LDS bank conflict / active = {vals['SQ_LDS_BANK_CONFLICT'] / max(vals['SQ_LDS_IDX_ACTIVE'], 1):.3f}")


if __name__ == "__main__":
    main(sys.argv[1:])
