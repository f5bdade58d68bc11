cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 900 gpurun_out/pytest_gpu.log python -m pytest tests -m gpu -q -x -p no:cacheprovider &&
tail -2 gpurun_out/pytest_gpu.log &&
tools/gpu_step.sh 300 gpurun_out/ab_head.log python tools/ab_head.py && tail -2 gpurun_out/ab_head.log &&
tools/gpu_step.sh 900 gpurun_out/bench_mag.log python bench.py --no-cpu-baseline &&
tail -1 gpurun_out/bench_mag.log | cut -c1-200 && grep -o '"kernels_ms.*' gpurun_out/bench_mag.log
