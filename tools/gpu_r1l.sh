# bf16 head hand-off (regnn_head_bwd_z dtype 1): GPU suite, bench bf16 / fp32
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread &&
tools/gpu_step.sh 300 gpurun_out/bench_l_bf16.log python bench.py --dtype bf16 --no-cpu-baseline &&
tools/gpu_step.sh 300 gpurun_out/bench_l.log python bench.py --no-cpu-baseline &&
tail -3 gpurun_out/pytest_gpu.log && for f in l_bf16 l; do grep -o '"ms_per_step": [0-9.]*\|"roofline": {[^}]*}\|"kernels_ms": {[^}]*}' gpurun_out/bench_$f.log; done
