# x6 GEMM edge tiles: GEMM tests, then interleaved h512 A/B (cur vs noedge = every wave runs 4 x 4 tiles)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 300 gpurun_out/t_gemm.log python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_ns_typed.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider && tail -1 gpurun_out/t_gemm.log &&
for r in 1 2; do
  for lib in cur noedge; do
    if [ "$lib" = cur ]; then unset REGNN_LIB; else export REGNN_LIB=$PWD/ab/libregnn_$lib.so; fi
    timeout -k 10 300 python bench.py --hidden 512 --no-full-batch --no-cpu-baseline --steps 100 > gpurun_out/h512_$lib.log 2>&1 || { tail -5 gpurun_out/h512_$lib.log; exit 1; }
    echo "$lib $(grep '^{' gpurun_out/h512_$lib.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4))')"
  done
done
