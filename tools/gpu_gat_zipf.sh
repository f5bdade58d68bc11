cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
for z in 1.1 0; do
  tools/gpu_step.sh 400 gpurun_out/b_gat_z$z.log python bench.py --workload gat --scale 1 --zipf $z --steps 10 --warmup 2 --no-cpu-baseline || exit 1
  tools/gpu_step.sh 400 gpurun_out/prof_gat_z$z.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gat_z$z -o run -- python bench.py --workload gat --scale 1 --zipf $z --steps 10 --warmup 2 --no-cpu-baseline || exit 1
done
