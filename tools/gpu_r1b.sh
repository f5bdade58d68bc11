# new GPU tests (inference, extra layers) + ns_infer bench
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/pytest_new.log python -u -m pytest tests/test_gpu_infer.py tests/test_gpu_layers.py -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider &&
tail -30 gpurun_out/pytest_new.log &&
tools/gpu_step.sh 600 gpurun_out/bench_ns_infer.log python bench.py --workload ns_infer --steps 5 --warmup 1 --no-cpu-baseline &&
tail -3 gpurun_out/bench_ns_infer.log
