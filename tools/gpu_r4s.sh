# gather grid A/B: REGNN_NSM_GATH_BLOCKS 256 (default) / 128 / 384, interleaved 300-step runs
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
for r in 1 2; do
  for gb in 256 128 384; do
    REGNN_NSM_GATH_BLOCKS=$gb timeout -k 10 300 python bench.py --no-full-batch --no-cpu-baseline --steps 300 > gpurun_out/gb_$gb.log 2>&1 || { tail -5 gpurun_out/gb_$gb.log; exit 1; }
    echo "gath_blocks=$gb $(grep '^{' gpurun_out/gb_$gb.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000,1))') us"
  done
done
