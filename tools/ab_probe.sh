#!/bin/bash
# tools/ns_k_probe.py under several environments: tools/ab_probe.sh "PROBE ARGS" "ENV1" "ENV2" ..
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
pargs=$1; shift 1
for e in "$@"; do
  envs=""; [ "$e" != "-" ] && envs="$e"
  echo "== [$e]"
  env $envs timeout -k 10 200 python tools/ns_k_probe.py $pargs > gpurun_out/probe.log 2>&1 || { tail -5 gpurun_out/probe.log; exit 1; }
  grep -E '^(m=|pre=)' gpurun_out/probe.log
done
