cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/prof_s1.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_s1 -o run -- python bench.py --scale 1 --steps 5 --warmup 2 --no-cpu-baseline &&
tools/gpu_step.sh 900 gpurun_out/bench_s10.log python bench.py &&
find gpurun_out/prof_s1 -name "*stats*" | head; tail -2 gpurun_out/bench_s10.log
