# bwd0 grid A/B: REGNN_NSM_BWD_BLOCKS per type 128 (default) / 112 / 144
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
for r in 1 2; do
  for gb in 128 112 144; do
    REGNN_NSM_BWD_BLOCKS=$gb timeout -k 10 300 python bench.py --no-full-batch --no-cpu-baseline --steps 300 > gpurun_out/gb_$gb.log 2>&1 || { tail -5 gpurun_out/gb_$gb.log; exit 1; }
    echo "bwd_blocks=$gb $(grep '^{' gpurun_out/gb_$gb.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000,1))') us"
  done
done
