# round-1 re-entry check: GPU parity suite, smoke, both bench lines at the current code
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread &&
tools/gpu_step.sh 300 gpurun_out/smoke.log python __graft_entry__.py smoke &&
tools/gpu_step.sh 600 gpurun_out/bench_full.log python bench.py &&
tools/gpu_step.sh 300 gpurun_out/bench_bf16.log python bench.py --dtype bf16 --no-cpu-baseline &&
tail -3 gpurun_out/pytest_gpu.log && tail -2 gpurun_out/smoke.log && tail -1 gpurun_out/bench_full.log && tail -1 gpurun_out/bench_bf16.log
