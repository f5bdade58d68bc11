# Full GPU verification: every -m gpu test, smoke(), the default bench line (NS + full-batch
# roofline leg + CPU baseline) and a kernel-trace profile of the default bench.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 900 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
tail -3 gpurun_out/pytest_gpu.log && grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q " failed" gpurun_out/pytest_gpu.log &&
tools/gpu_step.sh 300 gpurun_out/smoke.log python -c "import __graft_entry__ as g; g.smoke()" &&
tail -2 gpurun_out/smoke.log &&
tools/gpu_step.sh 900 gpurun_out/bench.log python bench.py &&
tail -1 gpurun_out/bench.log
