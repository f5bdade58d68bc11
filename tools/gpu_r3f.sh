# determinism probe, the whole -m gpu suite, h512 NS bench, NS kernel trace window
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 300 python tools/debug_gather2.py > gpurun_out/dbg_g2.txt 2>&1; tail -26 gpurun_out/dbg_g2.txt;
tools/gpu_step.sh 900 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
grep -E "passed|failed|FAILED" gpurun_out/pytest_gpu.log | tail -12 &&
tools/gpu_step.sh 300 gpurun_out/b_ns512.log python bench.py --workload ns --hidden 512 --no-full-batch --no-cpu-baseline &&
tail -2 gpurun_out/b_ns512.log | head -1 | cut -c1-300 && grep -o '"ns_kernels_ms.*' gpurun_out/b_ns512.log | cut -c1-1500 &&
tools/gpu_step.sh 300 gpurun_out/prof_ns.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ns -o run -- python bench.py --workload ns --no-full-batch --no-cpu-baseline --steps 50 &&
python tools/trace_window.py gpurun_out/prof_ns/run_kernel_trace.csv ns_batch_kernel 50 > gpurun_out/ns_window.txt; head -40 gpurun_out/ns_window.txt
