# NS/module tests, h512 trace
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/t_ns.log python -u -m pytest tests/test_gpu_ns_engine.py tests/test_gpu_ns_typed.py tests/test_gpu_regnn_golden.py tests/test_gpu_mag.py tests/test_gpu_ns.py tests/test_gpu_gat_fused.py tests/test_gpu_layers.py -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
grep -E "passed|failed|FAILED" gpurun_out/t_ns.log | tail -8 &&
tools/gpu_step.sh 300 gpurun_out/prof_ns512.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ns512 -o run -- python bench.py --workload ns --hidden 512 --no-full-batch --no-cpu-baseline --steps 30 &&
python tools/trace_window.py gpurun_out/prof_ns512/run_kernel_trace.csv ns_batch_kernel 30 > gpurun_out/ns512_window.txt; head -12 gpurun_out/ns512_window.txt
