# NS tests (8-wave head, lean module hop), NS bench x3, h512 bench + trace
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/t_ns.log python -u -m pytest tests/test_gpu_ns_engine.py tests/test_gpu_regnn_golden.py tests/test_gpu_ns_typed.py tests/test_gpu_ns_dp.py -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
grep -E "passed|failed|FAILED" gpurun_out/t_ns.log | tail -8 &&
bash tools/ab_env.sh 3 REGNN_NS_SPLIT_JOIN on &&
AB_ARGS="--hidden 512 --steps 60" bash tools/ab_env.sh 2 REGNN_NS_MODULE_LEAN on off &&
tools/gpu_step.sh 300 gpurun_out/prof_ns512.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ns512 -o run -- python bench.py --workload ns --hidden 512 --no-full-batch --no-cpu-baseline --steps 30 &&
python tools/trace_window.py gpurun_out/prof_ns512/run_kernel_trace.csv ns_batch_kernel 30 > gpurun_out/ns512_window.txt; head -8 gpurun_out/ns512_window.txt
