# round-end parity: the whole -m gpu suite, then smoke()
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 900 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
tail -3 gpurun_out/pytest_gpu.log && grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head; 
tools/gpu_step.sh 200 gpurun_out/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" && tail -2 gpurun_out/smoke.log
