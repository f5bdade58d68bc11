# h512 split-K target A/B: REGNN_GEMM_SPLIT_TARGET 512 (default) / 256 / 1024
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
for r in 1 2; do
  for gb in 512 256 1024; do
    REGNN_GEMM_SPLIT_TARGET=$gb timeout -k 10 300 python bench.py --hidden 512 --no-full-batch --no-cpu-baseline --steps 100 > gpurun_out/gb_$gb.log 2>&1 || { tail -5 gpurun_out/gb_$gb.log; exit 1; }
    echo "split_target=$gb $(grep '^{' gpurun_out/gb_$gb.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000,1))') us"
  done
done
