#!/bin/bash
# A/B of library builds on the fused GAT forward (gat bench, mag_like(1), uniform destinations):
# tools/ab_gat.sh REPS lib1 lib2 ... ("cur" = the in-tree library)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
reps=$1; shift 1
for r in $(seq $reps); do
  for lib in "$@"; do
    if [ "$lib" = cur ]; then unset REGNN_LIB; else export REGNN_LIB=$PWD/ab/libregnn_$lib.so; fi
    timeout -k 10 200 python bench.py --workload gat --scale 1 --zipf 0 --steps 6 --warmup 2 --no-cpu-baseline ${AB_ARGS} > gpurun_out/ab_gat.log 2>&1 || { tail -5 gpurun_out/ab_gat.log; exit 1; }
    echo "$lib $(grep '^{' gpurun_out/ab_gat.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels_ms"]; print(round(d["ms_per_step"],2), "ms/step fused_fwd", k.get("gat_fused_fwd"), "heads_bwd", k.get("spmm_heads_bwd"))')"
  done
done
unset REGNN_LIB
