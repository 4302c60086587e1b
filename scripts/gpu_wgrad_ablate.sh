cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
: > gpurun_out/wgrad_ablate.txt
for sh in 256,64,32,32,64,3,1,1 256,128,16,16,128,3,1,1 256,256,8,8,256,3,1,1 256,512,4,4,512,3,1,1 256,64,32,32,128,3,2,1; do
  timeout -k 10 200 python scripts/conv_ablate.py --wgrad-only --shape $sh >> gpurun_out/wgrad_ablate.txt 2>&1 || exit $?
done
cat gpurun_out/wgrad_ablate.txt
