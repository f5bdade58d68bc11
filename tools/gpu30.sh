cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -3 gpurun_out/pytest_gpu.log &&
tools/gpu_step.sh 600 gpurun_out/bench.log python bench.py --no-cpu-baseline &&
tools/gpu_step.sh 600 gpurun_out/bench_bf16.log python bench.py --dtype bf16 --no-cpu-baseline &&
tail -n 2 gpurun_out/bench.log gpurun_out/bench_bf16.log | grep -o '"ms_per_step": [0-9.]*\|"kernels_ms.*'
