#!/bin/bash
# A/B of library builds on the NS bench: tools/ab_lib.sh REPS lib1.so lib2.so ... (same ABI);
# prints us/step per build per repetition, interleaved.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
reps=$1; shift
for r in $(seq $reps); do
  for lib in "$@"; do
    REGNN_LIB=$PWD/$lib timeout -k 10 200 python bench.py --workload ns --no-full-batch --no-cpu-baseline --steps 300 ${AB_ARGS} > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    echo "$lib $(grep '^{' gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000,1), "us", round(d["value"]/1e6,1), "M")')"
  done
done
