# head z mode, cheaper p re-formation: head tests + bench fp32 / bf16
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 300 gpurun_out/pytest_head.log python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_next.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "head" &&
tools/gpu_step.sh 300 gpurun_out/bench_z.log python bench.py --no-cpu-baseline &&
tools/gpu_step.sh 300 gpurun_out/bench_z_bf16.log python bench.py --dtype bf16 --no-cpu-baseline &&
tail -2 gpurun_out/pytest_head.log && for f in z z_bf16; do grep -o '"ms_per_step": [0-9.]*\|"kernels_ms": {[^}]*}' gpurun_out/bench_$f.log; done
