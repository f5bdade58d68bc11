cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 900 gpurun_out/pytest_gpu.log python -m pytest tests -m gpu -q -p no:cacheprovider &&
tail -4 gpurun_out/pytest_gpu.log &&
tools/gpu_step.sh 900 gpurun_out/bench_mag.log python bench.py &&
tools/gpu_step.sh 600 gpurun_out/bench_dblp.log python bench.py --workload dblp --steps 50 --warmup 5 --no-cpu-baseline &&
tools/gpu_step.sh 600 gpurun_out/bench_acm.log python bench.py --workload acm --steps 50 --warmup 5 --no-cpu-baseline &&
tools/gpu_step.sh 600 gpurun_out/bench_imdb.log python bench.py --workload imdb --steps 50 --warmup 5 --no-cpu-baseline &&
tools/gpu_step.sh 900 gpurun_out/bench_ns.log python bench.py --workload ns --steps 30 --warmup 5 --no-cpu-baseline &&
for f in mag dblp acm imdb ns; do tail -1 gpurun_out/bench_$f.log | cut -c1-400; done
