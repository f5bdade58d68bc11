# GAT-family layer step on mag_like(1), Zipf(1.1) hubs against uniform destinations: bench lines
# and kernel stats.   tools/gpu_gat_zipf.sh [gat|gatv2]
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out || exit 1
wl=${1:-gat}
for z in 1.1 0; do
  tools/gpu_step.sh 400 gpurun_out/b_${wl}_z$z.log python bench.py --workload $wl --scale 1 --zipf $z --steps 10 --warmup 2 --no-cpu-baseline || exit 1
  grep '^{' gpurun_out/b_${wl}_z$z.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$wl' zipf '$z'", round(d["ms_per_step"],3), "ms", d.get("roofline",{}).get("frac"))'
  tools/gpu_step.sh 400 gpurun_out/prof_${wl}_z$z.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${wl}_z$z -o run -- python bench.py --workload $wl --scale 1 --zipf $z --steps 10 --warmup 2 --no-cpu-baseline || exit 1
done
