cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/bench_dblp.log python bench.py --workload dblp --steps 100 --warmup 5 --no-cpu-baseline &&
tools/gpu_step.sh 600 gpurun_out/bench_acm.log python bench.py --workload acm --steps 100 --warmup 5 --no-cpu-baseline &&
tools/gpu_step.sh 600 gpurun_out/bench_imdb.log python bench.py --workload imdb --steps 100 --warmup 5 --no-cpu-baseline &&
for f in dblp acm imdb; do tail -2 gpurun_out/bench_$f.log | cut -c1-300; done
