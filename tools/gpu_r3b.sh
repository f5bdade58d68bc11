# NS two-layer step: its GPU tests, the ns bench line, a kernel trace window of 50 replayed steps
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 500 gpurun_out/t_ns2.log python -u -m pytest tests/test_gpu_ns_engine.py tests/test_gpu_regnn_golden.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
grep -E "passed|failed" gpurun_out/t_ns2.log | tail -3 &&
tools/gpu_step.sh 300 gpurun_out/b_ns2.log python bench.py --workload ns --no-full-batch --no-cpu-baseline &&
tail -1 gpurun_out/b_ns2.log | cut -c1-600 &&
tools/gpu_step.sh 300 gpurun_out/prof_ns2.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ns2 -o run -- python bench.py --workload ns --no-full-batch --no-cpu-baseline --steps 50 &&
python tools/trace_window.py gpurun_out/prof_ns2/run_kernel_trace.csv ns_batch_kernel 50 > gpurun_out/ns2_window.txt; head -30 gpurun_out/ns2_window.txt
