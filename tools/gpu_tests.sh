# GPU parity: the named test files first (fast feedback), then the whole -m gpu suite.
# usage: tools/gpu_tests.sh [pytest file args...]
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
if [ $# -gt 0 ]; then
  tools/gpu_step.sh 600 gpurun_out/t_first.log python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
  tail -4 gpurun_out/t_first.log; grep -q " passed" gpurun_out/t_first.log && ! grep -q "failed\|error" gpurun_out/t_first.log || exit 1
fi &&
tools/gpu_step.sh 900 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
tail -3 gpurun_out/pytest_gpu.log
