# head p-from-logits (regnn_head_fwd_lse / regnn_head_bwd_z): GPU suite, A/B bench of both modes
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread &&
tools/gpu_step.sh 300 gpurun_out/bench_z.log python bench.py --no-cpu-baseline &&
tools/gpu_step.sh 300 gpurun_out/bench_p.log env REGNN_HEAD_P=p python bench.py --no-cpu-baseline &&
tools/gpu_step.sh 300 gpurun_out/bench_z_bf16.log python bench.py --dtype bf16 --no-cpu-baseline &&
tail -3 gpurun_out/pytest_gpu.log && for f in z p z_bf16; do grep -o '"ms_per_step": [0-9.]*\|"kernels_ms": {[^}]*}' gpurun_out/bench_$f.log; done
