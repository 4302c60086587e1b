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


def per_forward(trace, marker="softmax_xent"):
    """Dispatches of ONE timed forward: between the last two loss-kernel dispatches
    of a kernel_trace.csv (each forward ends in exactly one)."""
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    if len(marks) < 2:
        print(f"per-forward census: only {len(marks)} '{marker}' dispatches")
        return
    win = rows[marks[-2] + 1:marks[-1] + 1]
    cnt, dur = {}, {}
    for r in win:
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:100]
        cnt[n] = cnt.get(n, 0) + 1
        dur[n] = dur.get(n, 0.0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f"\nONE forward (last timed): {len(win)} dispatches, busy {sum(dur.values()):.1f} us")
    for n in sorted(cnt, key=lambda k: -dur[k]):
        print(f"{dur[n]:9.1f} us {cnt[n]:4d}  {n}")
    bn = sum(c for n, c in cnt.items() if "bn_" in n)
    cp = sum(c for n, c in cnt.items() if "copyBuffer" in n or "copy_kernel" in n)
    print(f"per forward: BatchNorm kernels {bn}, copies {cp}")


if __name__ == "__main__":
    main(sys.argv[1])
    if len(sys.argv) > 2:
        per_forward(sys.argv[2])
