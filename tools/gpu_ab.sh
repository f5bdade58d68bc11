cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 900 gpurun_out/pytest_gpu.log python -m pytest tests -m gpu -q -p no:cacheprovider -x &&
tools/gpu_step.sh 900 gpurun_out/ab1.log python tools/ab_spmm.py --scale 10 --rounds 4 &&
tools/gpu_step.sh 600 gpurun_out/ab_bf16.log python tools/ab_spmm.py --scale 10 --rounds 3 --dtype bf16 --variants res:256:256 &&
tail -3 gpurun_out/pytest_gpu.log; cat gpurun_out/ab1.log | tail -40; tail -12 gpurun_out/ab_bf16.log
