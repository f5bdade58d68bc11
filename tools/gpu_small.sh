# the non-default bench workloads (small BASELINE configs and the NS paths), one line each
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
for w in dblp acm imdb; do tools/gpu_step.sh 600 gpurun_out/bench_$w.log python bench.py --workload $w --no-cpu-baseline || exit 1; done &&
tools/gpu_step.sh 600 gpurun_out/bench_dblp_bf16.log python bench.py --workload dblp --dtype bf16 --no-cpu-baseline &&
tools/gpu_step.sh 600 gpurun_out/bench_ns.log python bench.py --workload ns --steps 50 --warmup 5 --no-cpu-baseline &&
tools/gpu_step.sh 600 gpurun_out/bench_ns_infer.log python bench.py --workload ns_infer --steps 5 --warmup 1 --no-cpu-baseline &&
for w in dblp acm imdb dblp_bf16 ns ns_infer; do echo "$w $(tail -n 2 gpurun_out/bench_$w.log | head -n 1 | grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')"; done
