cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python scripts/conv_ablate.py --shape 256,64,32,32,64,3,1,1 > gpurun_out/ablate_l1.txt 2>&1 || exit $?
timeout -k 10 300 python scripts/conv_ablate.py --shape 256,256,8,8,256,3,1,1 > gpurun_out/ablate_l3.txt 2>&1 || exit $?
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/pmc -o l1 -- python3 scripts/conv_ablate.py --shape 256,64,32,32,64,3,1,1 > gpurun_out/pmc.log 2>&1; echo pmc rc=$?
cat gpurun_out/ablate_l1.txt gpurun_out/ablate_l3.txt
