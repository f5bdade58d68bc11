# head tests with the fused backward, full GPU suite, full-batch bench A/B (fused vs split head bwd)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/t_head.log python -u -m pytest tests/test_gpu_next.py tests/test_gpu_ops.py tests/test_gpu_infer.py tests/test_gpu_configs.py -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
grep -E "passed|failed|FAILED" gpurun_out/t_head.log | tail -8 &&
tools/gpu_step.sh 900 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
grep -E "passed|failed|FAILED" gpurun_out/pytest_gpu.log | tail -8 &&
for v in fused split fused; do
  REGNN_HEAD_BWD_PY=$v timeout -k 10 300 python bench.py --workload mag --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b_mag_$v.log 2>&1 || exit 1
  echo "$v $(grep '^{' gpurun_out/b_mag_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],2), "ms", {k: v for k, v in d.get("kernels_ms", {}).items() if "head" in k})')"
done
