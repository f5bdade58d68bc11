export TMPDIR=/tmp; mkdir -p gpurun_out
tools/gpu_step.sh 400 gpurun_out/t_ns.log python -u -m pytest tests/test_gpu_ns_engine.py tests/test_gpu_ns.py tests/test_gpu_mag.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider && tail -5 gpurun_out/t_ns.log &&
tools/gpu_step.sh 300 gpurun_out/prof_ns.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ns -o run -- python bench.py --workload ns --no-full-batch --no-cpu-baseline --steps 50 && tail -2 gpurun_out/prof_ns.log
