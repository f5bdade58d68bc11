# NS tests (module pipelining), h512 A/B pipelined vs not, NS bench
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/t_ns.log python -u -m pytest tests/test_gpu_ns_engine.py tests/test_gpu_ns_typed.py tests/test_gpu_regnn_golden.py tests/test_gpu_ns_dp.py tests/test_gpu_ns.py tests/test_gpu_mag.py -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
grep -E "passed|failed|FAILED" gpurun_out/t_ns.log | tail -8 &&
AB_ARGS="--hidden 512 --steps 60" bash tools/ab_env.sh 2 REGNN_NS_MODULE_PIPELINE on off &&
tools/gpu_step.sh 300 gpurun_out/b_ns512.log python bench.py --workload ns --hidden 512 --no-full-batch --no-cpu-baseline &&
grep '^{' gpurun_out/b_ns512.log | cut -c1-260 &&
tools/gpu_step.sh 300 gpurun_out/b_epoch512.log python bench.py --workload ns_epoch --scale 1 --hidden 512 --no-cpu-baseline &&
grep '^{' gpurun_out/b_epoch512.log | cut -c1-300
