# HBM at lookahead 4 / 8, then a kernel trace of the NS bench at lookahead 8 (window on agg0)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
REGNN_NS_AHEAD=4 timeout -k 10 200 python tools/ns_mem.py 2>&1 | grep ahead &&
REGNN_NS_AHEAD=8 timeout -k 10 200 python tools/ns_mem.py 2>&1 | grep ahead &&
export REGNN_NS_AHEAD=8 &&
tools/gpu_step.sh 300 gpurun_out/prof_ns.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ns -o run -- python bench.py --workload ns --no-full-batch --no-cpu-baseline --steps 64 &&
python tools/trace_window.py gpurun_out/prof_ns/run_kernel_trace.csv agg0_kernel 48 timeline > gpurun_out/ns_window.txt; cat gpurun_out/ns_window.txt
