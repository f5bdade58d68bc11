cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 900 gpurun_out/pytest_gpu.log python -m pytest tests -m gpu -q -p no:cacheprovider &&
tail -2 gpurun_out/pytest_gpu.log &&
tools/gpu_step.sh 900 gpurun_out/ab3.log python tools/ab_spmm.py --scale 10 --rounds 4 --variants res:256:256:4,res:256:256:8,res:256:256:16 &&
tools/gpu_step.sh 900 gpurun_out/ab3_bf16.log python tools/ab_spmm.py --scale 10 --rounds 4 --dtype bf16 --variants res:256:256:4,res:256:256:8,res:256:256:16 &&
grep -A3 '"res' gpurun_out/ab3.log; grep -A3 '"res' gpurun_out/ab3_bf16.log
