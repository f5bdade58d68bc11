cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 300 gpurun_out/ab_dense.log python tools/ab_dense.py &&
tools/gpu_step.sh 900 gpurun_out/pytest_gpu.log python -m pytest tests -m gpu -q -p no:cacheprovider &&
tail -2 gpurun_out/pytest_gpu.log &&
tools/gpu_step.sh 900 gpurun_out/bench_mag.log python bench.py --no-cpu-baseline &&
tail -1 gpurun_out/bench_mag.log | cut -c1-600 &&
tools/gpu_step.sh 900 gpurun_out/prof_s10.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_s10 -o run -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline
