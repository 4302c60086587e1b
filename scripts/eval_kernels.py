#!/usr/bin/env python
"""Kernel census of an inference-forward rocprofv3 run (kernel_stats.csv):
total time per kernel and a verdict on library / ATen compute kernels
(hipBLASLt ``Cijk_*``, MIOpen, ``at::native`` other than fills / copies)."""
import csv
import sys

LIB = ("Cijk_", "miopen", "MIOpen", "igemm_", "naive_conv", "gridwise_")
ATEN = "at::native::"
# fills / copies, and the random input generation of the driver script itself
BENIGN = ("FillFunctor", "copy_kernel", "direct_copy", "CatArrayBatchedCopy", "rocclr_copyBuffer",
          "distribution_elementwise")


def main(path):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    lib, aten = [], []
    print(f"total {tot / 1e6:.3f} ms, {sum(int(r['Calls']) for r in rows)} dispatches")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        n = r["Name"]
        tag = ""
        if "dmp::" not in n and any(k in n for k in LIB):
            lib.append(n)
            tag = "  <-- LIBRARY"
        elif ATEN in n and not any(k in n for k in BENIGN):
            aten.append(n)
            tag = "  <-- ATen compute"
        print(f"{float(r['TotalDurationNs']) / 1e6:9.3f} ms {int(r['Calls']):5d}  {n[:110]}{tag}")
    print(f"library kernels: {len(lib)}; ATen compute kernels: {len(aten)}")


if __name__ == "__main__":
    main(sys.argv[1])
