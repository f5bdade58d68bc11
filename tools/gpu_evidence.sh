# Round-end evidence for the NS step: PMC HBM traffic (tools/gpu_pmc_ns.sh) copied where bench.py
# reads it, the default bench line, a kernel trace of 50 graphed NS steps, and the hidden-512
# module path (bench line + trace window).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out || exit 1
bash tools/gpu_pmc_ns.sh && cp gpurun_out/pmc_ns_fp32.json profiles/pmc_ns_fp32.json || exit 1
tools/gpu_step.sh 600 gpurun_out/bench_full.log python bench.py || exit 1
tail -1 gpurun_out/bench_full.log | cut -c1-300
tools/gpu_step.sh 300 gpurun_out/prof_ns.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ns -o run -- python bench.py --workload ns --no-full-batch --no-cpu-baseline --steps 192 || exit 1
python tools/trace_window.py gpurun_out/prof_ns/run_kernel_trace.csv agg0w_kernel 128 timeline > gpurun_out/ns_window.txt
tools/gpu_step.sh 400 gpurun_out/b_h512.log python bench.py --workload ns --hidden 512 --no-full-batch --no-cpu-baseline || exit 1
tail -1 gpurun_out/b_h512.log | cut -c1-200
tools/gpu_step.sh 400 gpurun_out/prof_h512.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_h512 -o run -- python bench.py --workload ns --hidden 512 --no-full-batch --no-cpu-baseline --steps 30 || exit 1
python tools/trace_window.py gpurun_out/prof_h512/run_kernel_trace.csv ns_batch_kernel 30 > gpurun_out/h512_window.txt; head -3 gpurun_out/h512_window.txt
