cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/bench_ns.log python bench.py --workload ns --steps 50 --warmup 5 --no-cpu-baseline &&
tools/gpu_step.sh 600 gpurun_out/prof_ns.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ns -o run -- python bench.py --workload ns --steps 50 --warmup 5 --no-cpu-baseline &&
tail -n 2 gpurun_out/bench_ns.log
