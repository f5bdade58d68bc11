cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 900 gpurun_out/pytest_gpu.log python -m pytest tests -m gpu -q -p no:cacheprovider &&
tools/gpu_step.sh 300 gpurun_out/smoke.log python __graft_entry__.py smoke &&
tools/gpu_step.sh 600 gpurun_out/bench_s1.log python bench.py --scale 1 --steps 5 --warmup 2 --no-cpu-baseline &&
tail -5 gpurun_out/pytest_gpu.log && tail -3 gpurun_out/smoke.log && tail -3 gpurun_out/bench_s1.log
