#!/bin/bash
# A/B of environment settings on the NS bench, interleaved, 300 timed steps each:
#   tools/ab_env.sh REPS "ENV1" "ENV2" ...   (each ENV a space-separated VAR=value list, "-" = none)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
reps=$1; shift 1
for r in $(seq $reps); do
  for e in "$@"; do
    envs=""; [ "$e" != "-" ] && envs="$e"
    env $envs timeout -k 10 200 python bench.py --workload ns --no-full-batch --no-cpu-baseline --steps 300 ${AB_ARGS} > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    echo "[$e] $(grep '^{' gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000,1), "us", round(d["value"]/1e6,1), "M", d["ns_kernels_ms"])')"
  done
done
