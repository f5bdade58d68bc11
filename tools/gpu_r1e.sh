cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/pytest_gat.log python -u -m pytest tests/test_gpu_mag.py tests/test_gpu_layers.py -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "regat or regatv2" &&
tail -30 gpurun_out/pytest_gat.log &&
tools/gpu_step.sh 600 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider &&
tail -5 gpurun_out/pytest_gpu.log
