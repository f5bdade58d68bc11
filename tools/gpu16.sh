cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -2 gpurun_out/pytest_gpu.log &&
tools/gpu_step.sh 600 gpurun_out/bench.log python bench.py --no-cpu-baseline &&
REGNN_DIST_BACKEND=gloo tools/gpu_step.sh 600 gpurun_out/bench_dp2.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 1 --scale 2 &&
tail -n 2 gpurun_out/bench.log gpurun_out/bench_dp2.log
