# NS PMC traffic for the current kernels, then the driver's default bench, kernel stats window
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
bash tools/gpu_pmc_ns.sh > gpurun_out/pmc_ns.out 2>&1 && tail -12 gpurun_out/pmc_ns.out &&
tools/gpu_step.sh 600 gpurun_out/b_default.log python bench.py &&
grep '^{' gpurun_out/b_default.log | cut -c1-200 &&
tools/gpu_step.sh 300 gpurun_out/prof_ns.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ns -o run -- python bench.py --workload ns --no-full-batch --no-cpu-baseline --steps 50 &&
python tools/trace_window.py gpurun_out/prof_ns/run_kernel_trace.csv ns_batch_kernel 50 timeline > gpurun_out/ns_window.txt; head -14 gpurun_out/ns_window.txt
