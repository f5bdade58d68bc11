cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 300 gpurun_out/pytest_head.log python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_dropout.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -2 gpurun_out/pytest_head.log &&
tools/gpu_step.sh 300 gpurun_out/ab_head_bwd.log python tools/ab_head_bwd.py &&
tools/gpu_step.sh 600 gpurun_out/bench.log python bench.py --no-cpu-baseline &&
tail -n 2 gpurun_out/ab_head_bwd.log && tail -n 2 gpurun_out/bench.log | grep -o '"ms_per_step": [0-9.]*\|"kernels_ms.*'
