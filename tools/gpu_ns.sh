# NS engine: its GPU tests, then the default (ns) bench under rocprofv3 kernel-trace + stats.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 400 gpurun_out/t_ns.log python -u -m pytest tests/test_gpu_ns_engine.py tests/test_gpu_regnn_golden.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider &&
tail -4 gpurun_out/t_ns.log && grep -q " passed" gpurun_out/t_ns.log && ! grep -q "failed\|error" gpurun_out/t_ns.log &&
tools/gpu_step.sh 300 gpurun_out/b_ns.log python bench.py --workload ns --no-full-batch --no-cpu-baseline &&
tail -1 gpurun_out/b_ns.log &&
tools/gpu_step.sh 300 gpurun_out/prof_ns.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ns -o run -- python bench.py --workload ns --no-full-batch --no-cpu-baseline --steps 50 &&
python tools/trace_window.py gpurun_out/prof_ns/run_kernel_trace.csv ns_batch_kernel 50 > gpurun_out/ns_window.txt; head -40 gpurun_out/ns_window.txt
