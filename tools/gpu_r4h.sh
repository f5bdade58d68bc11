# NS tests, A/B vs r3 base, phases, h512 kernel-trace window
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/t_ns.log python -u -m pytest tests/test_gpu_ns_typed.py tests/test_gpu_ns_engine.py tests/test_gpu_ns.py tests/test_gpu_regnn_golden.py tests/test_gpu_ns_dp.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && tail -2 gpurun_out/t_ns.log &&
bash tools/ab_lib2.sh 2 base cur &&
REGNN_LIB=$PWD/ab/libregnn_phases.so timeout -k 10 200 python tools/nsm2_phases.py > gpurun_out/phases_nopipe.txt 2>&1; sed -n 3,12p gpurun_out/phases_nopipe.txt; tail -29 gpurun_out/phases_nopipe.txt | head -6 &&
tools/gpu_step.sh 300 gpurun_out/prof_ns512.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ns512 -o run -- python bench.py --workload ns --hidden 512 --no-full-batch --no-cpu-baseline --steps 30 &&
python tools/trace_window.py gpurun_out/prof_ns512/run_kernel_trace.csv ns_batch_kernel 30 > gpurun_out/ns512_window.txt; head -3 gpurun_out/ns512_window.txt
