# DP tests (captured all-reduce), h512 benches, A/B of bwd0 / gather block counts
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/t_dp.log python -u -m pytest tests/test_gpu_ns_dp.py -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
grep -E "passed|failed|FAILED|Error" gpurun_out/t_dp.log | tail -8 &&
tools/gpu_step.sh 300 gpurun_out/b_ns512.log python bench.py --workload ns --hidden 512 --no-full-batch --no-cpu-baseline &&
grep '^{' gpurun_out/b_ns512.log | cut -c1-300 &&
tools/gpu_step.sh 300 gpurun_out/b_epoch512.log python bench.py --workload ns_epoch --scale 1 --hidden 512 --no-cpu-baseline &&
grep '^{' gpurun_out/b_epoch512.log | cut -c1-400 &&
bash tools/ab_env.sh 2 REGNN_NSM_BWD_BLOCKS 128 64 256 &&
bash tools/ab_env.sh 2 REGNN_NSM_GATH_BLOCKS 512 1024 256
