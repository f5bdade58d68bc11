# strided sampler with two targets per wave: NS parity tests, then A/B against one target per wave
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/t_ns.log python -u -m pytest tests/test_gpu_ns_engine.py tests/test_gpu_ns_typed.py tests/test_gpu_regnn_golden.py tests/test_gpu_ns.py tests/test_gpu_ns_dp.py -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
grep -E "passed|failed|FAILED" gpurun_out/t_ns.log | tail -8 &&
bash tools/ab_env.sh 3 REGNN_NS_HALF_WAVES 1 0 &&
AB_ARGS="--hidden 512 --steps 60" bash tools/ab_env.sh 2 REGNN_NS_HALF_WAVES 1 0
