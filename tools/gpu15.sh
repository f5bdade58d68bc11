cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -2 gpurun_out/pytest_gpu.log &&
tools/gpu_step.sh 600 gpurun_out/ab_bf16.log python tools/ab_spmm.py --scale 10 --rounds 3 --dtype bf16 --variants res:256:256:0:off,res:256:256:0:on &&
tools/gpu_step.sh 600 gpurun_out/ab_f32.log python tools/ab_spmm.py --scale 10 --rounds 3 --variants res:256:256:0:off,res:256:256:0:on &&
tools/gpu_step.sh 600 gpurun_out/bench.log python bench.py --no-cpu-baseline &&
tools/gpu_step.sh 600 gpurun_out/bench_bf16.log python bench.py --dtype bf16 --no-cpu-baseline &&
grep -A6 '"res' gpurun_out/ab_bf16.log gpurun_out/ab_f32.log; tail -n 2 gpurun_out/bench.log gpurun_out/bench_bf16.log
