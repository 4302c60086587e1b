#!/bin/bash
# ping-pong halo wgrad (variant 8): numerics over every config, then R18 timings (stride 1 and 2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r4r && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_conv_gpu.py -k "halo_conv_configs or stride2" > gpurun_out/r4r/tests.log 2>&1
rc=$?; grep -E "FAIL|^E |passed|failed" gpurun_out/r4r/tests.log | head -20; echo "tests rc=$rc"; [[ $rc == 0 ]] || exit $rc
SHAPES=r18 timeout -k 10 400 python -u scripts/wgrad_r50_bench.py > gpurun_out/r4r/w18.log 2>&1 || exit $?
STRIDE=2 SHAPES=r18s2 timeout -k 10 400 python -u scripts/wgrad_r50_bench.py > gpurun_out/r4r/w18s2.log 2>&1 || exit $?
for f in w18 w18s2; do python3 - gpurun_out/r4r/$f.log <<'PY'
import re, sys
for ln in open(sys.argv[1]):
    if not ln.startswith("C="):
        continue
    head = ln.split("|")[0].strip()
    ent = dict((int(k), float(v.split("(")[0])) for k, v in re.findall(r"(\d+):([\d.]+\([^)]*\))", ln.split("|")[1]))
    pp = {k: v for k, v in ent.items() if k % 1000 >= 96 and k >= 1000}
    old = {k: v for k, v in ent.items() if not (k % 1000 >= 96 and k >= 1000)}
    bo = min(old, key=old.get); bp = min(pp, key=pp.get) if pp else None
    print(head[:60], f"| best old {bo} {old[bo]:.1f} us | best pingpong {bp} {pp.get(bp, float('nan')):.1f} us")
PY
done
