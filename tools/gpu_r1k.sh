# CSC prefix under the head's zero gradient rows: GPU suite, bench fp32 / bf16, prefix-off A/B
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread &&
tools/gpu_step.sh 300 gpurun_out/bench_pre.log python bench.py --no-cpu-baseline &&
tools/gpu_step.sh 300 gpurun_out/bench_pre_bf16.log python bench.py --dtype bf16 --no-cpu-baseline &&
tail -3 gpurun_out/pytest_gpu.log && for f in pre pre_bf16; do grep -o '"ms_per_step": [0-9.]*\|"roofline": {[^}]*}\|"kernels_ms": {[^}]*}' gpurun_out/bench_$f.log; done
