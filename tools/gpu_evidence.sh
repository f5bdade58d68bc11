# Round-end evidence for the NS step: PMC HBM traffic (tools/gpu_pmc_ns.sh) copied where bench.py
# reads it, the driver's own bench command (20 steps, 5 warm-ups) and the default 160-step run,
# a kernel trace + stats of 192 graphed NS steps with the per-step window, and the hidden-512
# module path (bench line + trace window). Outputs under gpurun_out/ev_*.
#   tools/gpu_evidence.sh            (NO_H512=1: skip the hidden-512 leg; NO_PMC=1: skip PMC)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out || exit 1
if [ "$NO_PMC" != 1 ]; then
  bash tools/gpu_pmc_ns.sh && cp gpurun_out/pmc_ns_fp32.json profiles/pmc_ns_fp32.json || exit 1
fi
tools/gpu_step.sh 600 gpurun_out/ev_bench_driver.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
grep '^{' gpurun_out/ev_bench_driver.log > gpurun_out/ev_bench_driver.json; cut -c1-300 gpurun_out/ev_bench_driver.json
tools/gpu_step.sh 300 gpurun_out/ev_bench_160.log python bench.py --workload ns --no-full-batch --no-cpu-baseline --steps 160 --warmup 5 || exit 1
grep '^{' gpurun_out/ev_bench_160.log > gpurun_out/ev_bench_160.json; cut -c1-200 gpurun_out/ev_bench_160.json
tools/gpu_step.sh 300 gpurun_out/ev_prof_ns.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ev_prof_ns -o run -- python bench.py --workload ns --no-full-batch --no-cpu-baseline --steps 192 --warmup 5 || exit 1
python tools/trace_window.py gpurun_out/ev_prof_ns/run_kernel_trace.csv agg0w_kernel 128 timeline > gpurun_out/ev_ns_window.txt; head -14 gpurun_out/ev_ns_window.txt
[ "$NO_H512" = 1 ] && exit 0
tools/gpu_step.sh 400 gpurun_out/ev_b_h512.log python bench.py --workload ns --hidden 512 --no-full-batch --no-cpu-baseline || exit 1
grep '^{' gpurun_out/ev_b_h512.log > gpurun_out/ev_b_h512.json; cut -c1-200 gpurun_out/ev_b_h512.json
tools/gpu_step.sh 400 gpurun_out/ev_prof_h512.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ev_prof_h512 -o run -- python bench.py --workload ns --hidden 512 --no-full-batch --no-cpu-baseline --steps 30 || exit 1
python tools/trace_window.py gpurun_out/ev_prof_h512/run_kernel_trace.csv nsagg::slot_agg_kernel 24 --between > gpurun_out/ev_h512_window.txt; head -3 gpurun_out/ev_h512_window.txt
