# multi-size group graphs from every start slot: NS tests, capture time / HBM, the default bench
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/t_ns.log python -u -m pytest tests/test_gpu_ns_engine.py tests/test_gpu_ns_dp.py -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
grep -E "passed|failed|FAILED" gpurun_out/t_ns.log | tail -8 &&
timeout -k 10 200 python tools/ns_mem.py 2>&1 | grep ahead &&
tools/gpu_step.sh 600 gpurun_out/b_default.log python bench.py &&
grep '^{' gpurun_out/b_default.log | cut -c1-300 &&
bash tools/ab_env.sh 2 REGNN_NS_AHEAD 4 8
