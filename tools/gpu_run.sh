#!/bin/bash
# Generic GPU call: the named test files (fast feedback), then the default NS bench, then a
# rocprofv3 kernel trace of 50 graphed NS steps with the per-step window.
#   tools/gpu_run.sh [pytest file args...]      (no args: skip the tests)
# env: BENCH_ARGS (extra bench.py args), NO_PROF=1 (skip the trace)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out || exit 1
if [ $# -gt 0 ]; then
  tools/gpu_step.sh 600 gpurun_out/t_run.log python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
  tail -4 gpurun_out/t_run.log
  grep -q " passed" gpurun_out/t_run.log && ! grep -q "failed\|error" gpurun_out/t_run.log || exit 1
fi
tools/gpu_step.sh 300 gpurun_out/b_ns.log python bench.py --workload ns --no-full-batch --no-cpu-baseline $BENCH_ARGS || exit 1
grep '^{' gpurun_out/b_ns.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("BENCH", round(d["ms_per_step"]*1000,1), "us", round(d["value"]/1e6,1), "M edges/s", d["ns_kernels_ms"], "frac", round(d.get("roofline",{}).get("frac",0),4))'
[ "$NO_PROF" = 1 ] && exit 0
tools/gpu_step.sh 300 gpurun_out/prof_ns.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ns -o run -- python bench.py --workload ns --no-full-batch --no-cpu-baseline --steps 192 $BENCH_ARGS || exit 1
python tools/trace_window.py gpurun_out/prof_ns/run_kernel_trace.csv agg0w_kernel 128 timeline > gpurun_out/ns_window.txt; head -20 gpurun_out/ns_window.txt
