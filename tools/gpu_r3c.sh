cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 500 gpurun_out/t_ns3.log python -u -m pytest tests/test_gpu_ns_engine.py tests/test_gpu_regnn_golden.py tests/test_gpu_ns_dp.py -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
grep -E "passed|failed|FAILED" gpurun_out/t_ns3.log | tail -8 &&
REGNN_LIB=$PWD/ab/libregnn_phases.so timeout -k 10 200 python tools/nsm2_phases.py > gpurun_out/phases3.txt 2>&1 && tail -22 gpurun_out/phases3.txt &&
tools/gpu_step.sh 300 gpurun_out/b_ns3.log python bench.py --workload ns --no-full-batch --no-cpu-baseline &&
tail -2 gpurun_out/b_ns3.log | head -1 | cut -c1-300 &&
tools/gpu_step.sh 300 gpurun_out/prof_ns3.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ns3 -o run -- python bench.py --workload ns --no-full-batch --no-cpu-baseline --steps 50 &&
python tools/trace_window.py gpurun_out/prof_ns3/run_kernel_trace.csv ns_batch_kernel 50 > gpurun_out/ns3_window.txt; head -24 gpurun_out/ns3_window.txt
