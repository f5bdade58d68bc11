cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/prof_acm.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_acm -o run -- python bench.py --workload acm --steps 20 --warmup 3 --no-cpu-baseline &&
tools/gpu_step.sh 600 gpurun_out/prof_imdb.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_imdb -o run -- python bench.py --workload imdb --steps 20 --warmup 3 --no-cpu-baseline
