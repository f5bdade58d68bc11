cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 300 gpurun_out/pytest_head.log python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_infer.py tests/test_gpu_layers.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -3 gpurun_out/pytest_head.log &&
HEAD_VARIANTS=16,0 tools/gpu_step.sh 300 gpurun_out/ab_head.log python tools/ab_head.py &&
tail -n 2 gpurun_out/ab_head.log &&
tools/gpu_step.sh 600 gpurun_out/bench.log python bench.py --no-cpu-baseline &&
tail -n 2 gpurun_out/bench.log | grep -o '"ms_per_step": [0-9.]*\|"kernels_ms.*'
