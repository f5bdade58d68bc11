cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/prof_fp32.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fp32 -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline
