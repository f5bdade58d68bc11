cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 900 gpurun_out/pytest_gpu.log python -m pytest tests -m gpu -q -p no:cacheprovider &&
tail -3 gpurun_out/pytest_gpu.log &&
tools/gpu_step.sh 900 gpurun_out/ab2.log python tools/ab_spmm.py --scale 10 --rounds 4 --variants res:256:256,res:128:128,res:512:512 &&
tools/gpu_step.sh 600 gpurun_out/ab2_bf16.log python tools/ab_spmm.py --scale 10 --rounds 3 --dtype bf16 --variants res:256:256 &&
grep -A7 '"res' gpurun_out/ab2.log; grep -A7 '"res' gpurun_out/ab2_bf16.log
