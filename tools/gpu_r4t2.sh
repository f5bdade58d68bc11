# final: full suite, smoke, half-wave sampler A/B, NS kernel trace window, default bench
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider && tail -1 gpurun_out/pytest_gpu.log &&
tools/gpu_step.sh 300 gpurun_out/smoke.log python -c "import __graft_entry__ as g; g.smoke()" &&
for r in 1 2; do
  for hw in 0 1; do
    REGNN_NS_HALF_WAVES=$hw timeout -k 10 300 python bench.py --no-full-batch --no-cpu-baseline --steps 300 > gpurun_out/hw_$hw.log 2>&1 || { tail -5 gpurun_out/hw_$hw.log; exit 1; }
    echo "half_waves=$hw $(grep '^{' gpurun_out/hw_$hw.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000,1))') us"
  done
done &&
tools/gpu_step.sh 300 gpurun_out/prof_ns.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ns -o run -- python bench.py --workload ns --no-full-batch --no-cpu-baseline --steps 50 &&
python tools/trace_window.py gpurun_out/prof_ns/run_kernel_trace.csv ns_batch_kernel 50 > gpurun_out/ns_window.txt; head -14 gpurun_out/ns_window.txt; cp gpurun_out/prof_ns/run_kernel_stats.csv gpurun_out/ns_kernel_stats.csv; rm -f gpurun_out/prof_ns/run_kernel_trace.csv;
tools/gpu_step.sh 600 gpurun_out/bench.log python bench.py && grep '^{' gpurun_out/bench.log | tail -1 > gpurun_out/bench_default.json && python -c "import json;d=json.load(open('gpurun_out/bench_default.json'));r=d['roofline'];print('default', d['ms_per_step'], d['value']/1e6, r['frac'], r.get('frac_hbm'), r.get('pmc'))"
