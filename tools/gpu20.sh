cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 300 gpurun_out/pytest_head.log python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q -k head --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -2 gpurun_out/pytest_head.log &&
HEAD_VARIANTS=0,16,17,18,19,1,4 tools/gpu_step.sh 300 gpurun_out/ab_head.log python tools/ab_head.py &&
tail -n 3 gpurun_out/ab_head.log
