# NS tests (determinism), phases of the two-layer step, h512 kernel trace, NS PMC traffic
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/t_ns.log python -u -m pytest tests/test_gpu_ns_engine.py tests/test_gpu_ns_typed.py -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
grep -E "passed|failed|FAILED" gpurun_out/t_ns.log | tail -8 &&
REGNN_LIB=$PWD/ab/libregnn_phases.so timeout -k 10 200 python tools/nsm2_phases.py > gpurun_out/phases_nopipe.txt 2>&1 && tail -30 gpurun_out/phases_nopipe.txt &&
REGNN_LIB=$PWD/ab/libregnn_phases.so timeout -k 10 200 python tools/nsm2_phases.py --pipeline > gpurun_out/phases_pipe.txt 2>&1 && tail -30 gpurun_out/phases_pipe.txt &&
tools/gpu_step.sh 300 gpurun_out/prof_ns512.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ns512 -o run -- python bench.py --workload ns --hidden 512 --no-full-batch --no-cpu-baseline --steps 30 &&
python tools/trace_window.py gpurun_out/prof_ns512/run_kernel_trace.csv ns_batch_kernel 30 > gpurun_out/ns512_window.txt; head -45 gpurun_out/ns512_window.txt &&
bash tools/gpu_pmc_ns.sh && cat gpurun_out/pmc_ns_fp32.json | head -50
