# hidden-512 module path: sampler pipelined on a second stream (REGNN_NS_MODULE_PIPELINE) vs not, interleaved
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
for r in 1 2; do
  for m in off on; do
    REGNN_NS_MODULE_PIPELINE=$m timeout -k 10 300 python bench.py --hidden 512 --no-full-batch --no-cpu-baseline --steps 100 > gpurun_out/h512_$m.log 2>&1 || { tail -5 gpurun_out/h512_$m.log; exit 1; }
    echo "$m $(grep '^{' gpurun_out/h512_$m.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4))')"
  done
done
