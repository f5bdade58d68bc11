# Round-3 re-entry check: NS engine / golden / DP tests (all cases reported), NS bench, then the whole -m gpu suite.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/t_ns.log python -u -m pytest tests/test_gpu_ns_engine.py tests/test_gpu_regnn_golden.py tests/test_gpu_ns_dp.py -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
grep -E "passed|failed|FAILED" gpurun_out/t_ns.log | tail -12 &&
tools/gpu_step.sh 300 gpurun_out/b_ns.log python bench.py --workload ns --no-full-batch --no-cpu-baseline &&
tail -2 gpurun_out/b_ns.log | head -1 | cut -c1-400 &&
tools/gpu_step.sh 900 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
grep -E "passed|failed|FAILED" gpurun_out/pytest_gpu.log | tail -12
