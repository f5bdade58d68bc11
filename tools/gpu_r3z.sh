# round-end measurements: NS PMC (re_nsm2 changed), the driver's default bench, NS kernel trace
# (window on agg0), hidden 512 and the mag-1x epoch
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
bash tools/gpu_pmc_ns.sh > gpurun_out/pmc_ns.out 2>&1 && tail -6 gpurun_out/pmc_ns.out &&
tools/gpu_step.sh 600 gpurun_out/b_default.log python bench.py &&
grep '^{' gpurun_out/b_default.log | cut -c1-240 &&
tools/gpu_step.sh 300 gpurun_out/prof_ns.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ns -o run -- python bench.py --workload ns --no-full-batch --no-cpu-baseline --steps 64 &&
python tools/trace_window.py gpurun_out/prof_ns/run_kernel_trace.csv agg0_kernel 48 timeline > gpurun_out/ns_window.txt; head -3 gpurun_out/ns_window.txt &&
tools/gpu_step.sh 300 gpurun_out/b_ns512.log python bench.py --workload ns --hidden 512 --no-full-batch --no-cpu-baseline &&
grep '^{' gpurun_out/b_ns512.log | cut -c1-200 &&
tools/gpu_step.sh 300 gpurun_out/b_epoch512.log python bench.py --workload ns_epoch --scale 1 --hidden 512 --no-cpu-baseline &&
grep '^{' gpurun_out/b_epoch512.log | cut -c1-300
