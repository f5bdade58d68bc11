cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider &&
tail -25 gpurun_out/pytest_gpu.log &&
tools/gpu_step.sh 600 gpurun_out/bench_ns_infer.log python bench.py --workload ns_infer --steps 5 --warmup 1 --no-cpu-baseline &&
tail -1 gpurun_out/bench_ns_infer.log | cut -c1-200
