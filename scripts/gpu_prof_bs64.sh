set -u
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/p64 && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p64/prof -o r18b64 -- python3 bench.py --batch 64 --steps 40 --warmup 10 --ttl-target 0 --ref-batch 0 > gpurun_out/p64/prof.log 2>&1 || exit $?
python3 scripts/prof_steady.py gpurun_out/p64/prof/r18b64_kernel_trace.csv --steps 30 --top 60 > gpurun_out/p64/steady.txt && rm -f gpurun_out/p64/prof/*.csv
head -45 gpurun_out/p64/steady.txt
