cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 300 gpurun_out/pytest_drop.log python -u -m pytest tests/test_gpu_dropout.py -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider &&
tail -15 gpurun_out/pytest_drop.log &&
tools/gpu_step.sh 900 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider &&
tail -3 gpurun_out/pytest_gpu.log &&
tools/gpu_step.sh 600 gpurun_out/bench.log python bench.py --no-cpu-baseline &&
tail -1 gpurun_out/bench.log
