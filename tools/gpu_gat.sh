# Fused GAT: parity tests, the gat bench at mag_like(1) (+ kernel stats), and the NS epoch
# context line (mag_like(1), hidden 512).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 400 gpurun_out/t_gat.log python -u -m pytest tests/test_gpu_gat_fused.py tests/test_gpu_layers.py tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider &&
tail -3 gpurun_out/t_gat.log && grep -q " passed" gpurun_out/t_gat.log && ! grep -q " failed" gpurun_out/t_gat.log &&
tools/gpu_step.sh 400 gpurun_out/b_gat.log python bench.py --workload gat --scale 1 --steps 10 --warmup 2 --no-cpu-baseline &&
tail -1 gpurun_out/b_gat.log &&
tools/gpu_step.sh 400 gpurun_out/prof_gat.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gat -o run -- python bench.py --workload gat --scale 1 --steps 10 --warmup 2 --no-cpu-baseline &&
tools/gpu_step.sh 600 gpurun_out/b_epoch.log python bench.py --workload ns_epoch --scale 1 --hidden 512 --no-cpu-baseline &&
tail -1 gpurun_out/b_epoch.log
