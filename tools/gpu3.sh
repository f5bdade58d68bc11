cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 900 gpurun_out/pytest_gpu.log python -m pytest tests -m gpu -q -p no:cacheprovider &&
tools/gpu_step.sh 900 gpurun_out/prof_s10.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_s10 -o run -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline &&
tools/gpu_step.sh 900 gpurun_out/bench_s10.log python bench.py &&
tail -3 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/bench_s10.log
