#!/bin/bash
# A/B of an environment switch on the NS bench: tools/ab_env.sh REPS VAR v1 v2 ...
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
reps=$1; var=$2; shift 2
for r in $(seq $reps); do
  for val in "$@"; do
    env $var=$val timeout -k 10 200 python bench.py --workload ns --no-full-batch --no-cpu-baseline --steps 300 ${AB_ARGS} > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    echo "$var=$val $(grep '^{' gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000,1), "us", round(d["value"]/1e6,1), "M")')"
  done
done
