cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/pytest_drop.log python -u -m pytest tests/test_gpu_dropout.py -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider &&
tail -14 gpurun_out/pytest_drop.log &&
tools/gpu_step.sh 600 gpurun_out/bench_bf16.log python bench.py --dtype bf16 --no-cpu-baseline &&
tools/gpu_step.sh 600 gpurun_out/bench_dblp_bf16.log python bench.py --workload dblp --dtype bf16 --no-cpu-baseline &&
tools/gpu_step.sh 600 gpurun_out/bench_dblp.log python bench.py --workload dblp --no-cpu-baseline &&
tail -1 gpurun_out/bench_bf16.log | cut -c1-120
