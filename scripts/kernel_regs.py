#!/usr/bin/env python
"""Register / spill / occupancy table of the kernels in one HIP source (device-only
compile with -Rpass-analysis=kernel-resource-usage).  Usage:
python scripts/kernel_regs.py distributed_ml_pytorch_amd/csrc/conv.hip [name-substring ...]"""
import re
import subprocess
import sys
from pathlib import Path

CSRC = Path(__file__).resolve().parents[1] / "distributed_ml_pytorch_amd" / "csrc"


def main():
    src = sys.argv[1]
    pats = sys.argv[2:]
    out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                          "--cuda-device-only", "-c", "-DDMP_ABLATE=0", "-I", str(CSRC), src, "-o",
                          "/dev/null", "-Rpass-analysis=kernel-resource-usage"],
                         capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|VGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
        if not m:
            continue
        k, v = m.group(1), m.group(2)
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    for r in rows:
        if pats and not any(p in r["name"] for p in pats):
            continue
        print(f"{r.get('VGPRs', '?'):>4} v {r.get('AGPRs', '?'):>4} a  spill {r.get('VGPRs Spill', '?'):>4}  "
              f"occ {r.get('Occupancy [waves/SIMD]', '?'):>2}  {r['name']}")


if __name__ == "__main__":
    main()
