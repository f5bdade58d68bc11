cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/pytest_head.log python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_ns.py -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "head or feats" &&
tail -20 gpurun_out/pytest_head.log &&
tools/gpu_step.sh 600 gpurun_out/bench.log python bench.py --no-cpu-baseline &&
tail -1 gpurun_out/bench.log | cut -c1-100
