cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 900 gpurun_out/pytest_gpu.log python -m pytest tests -m gpu -q -x -p no:cacheprovider &&
tail -2 gpurun_out/pytest_gpu.log &&
for w in acm imdb dblp; do tools/gpu_step.sh 600 gpurun_out/bench_$w.log python bench.py --workload $w --no-cpu-baseline || exit 1; tail -1 gpurun_out/bench_$w.log | grep -o '"ms_per_step": [0-9.]*\|"kernels_ms.*'; done &&
tools/gpu_step.sh 600 gpurun_out/prof_acm.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_acm -o run -- python bench.py --workload acm --steps 20 --warmup 3 --no-cpu-baseline
