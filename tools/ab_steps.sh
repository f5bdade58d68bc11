#!/bin/bash
# A/B of environment settings on the NS bench at the driver's own step count, interleaved:
#   tools/ab_steps.sh REPS STEPS WARMUP "ENV1" "ENV2" ...   (ENV a VAR=value list, "-" = none)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
reps=$1; steps=$2; warm=$3; shift 3
for r in $(seq $reps); do
  for e in "$@"; do
    envs=""; [ "$e" != "-" ] && envs="$e"
    env $envs timeout -k 10 200 python bench.py --workload ns --no-full-batch --no-cpu-baseline --steps $steps --warmup $warm ${AB_ARGS} > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    echo "[$e K=$steps W=$warm] $(grep '^{' gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000,1), "us", round(d["value"]/1e6,1), "M", d["ns_kernels_ms"])')"
  done
done
