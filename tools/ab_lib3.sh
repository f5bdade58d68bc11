#!/bin/bash
# A/B of library builds in abx/ (tools/build_variant.py with AB_DIR=abx) on the NS bench:
#   tools/ab_lib3.sh REPS lib1 lib2 ...   ("cur" = the in-tree library), interleaved, 300 steps
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
reps=$1; shift 1
for r in $(seq $reps); do
  for lib in "$@"; do
    if [ "$lib" = cur ]; then unset REGNN_LIB; else export REGNN_LIB=$PWD/abx/libregnn_$lib.so; fi
    timeout -k 10 200 python bench.py --workload ns --no-full-batch --no-cpu-baseline --steps ${STEPS:-300} --warmup ${WARM:-3} ${AB_ARGS} > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    echo "[$lib K=${STEPS:-300}] $(grep '^{' gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000,1), "us", round(d["value"]/1e6,1), "M", d["ns_kernels_ms"])')"
  done
done
unset REGNN_LIB
