# round-4 profiles: default bench (fresh PMC), phases, h512 kernel trace
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/bench.log python bench.py && grep '^{' gpurun_out/bench.log | tail -1 > gpurun_out/bench_default.json && python -c "import json;d=json.load(open('gpurun_out/bench_default.json'));r=d['roofline'];print('default', d['ms_per_step'], d['value']/1e6, r['frac'], r.get('frac_hbm'), r.get('pmc'))" &&
REGNN_LIB=$PWD/ab/libregnn_phases.so timeout -k 10 200 python tools/nsm2_phases.py > gpurun_out/phases_nopipe.txt 2>&1; tail -29 gpurun_out/phases_nopipe.txt | head -6;
tools/gpu_step.sh 300 gpurun_out/prof_ns512.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ns512 -o run -- python bench.py --workload ns --hidden 512 --no-full-batch --no-cpu-baseline --steps 30 &&
python tools/trace_window.py gpurun_out/prof_ns512/run_kernel_trace.csv ns_batch_kernel 30 > gpurun_out/ns512_window.txt; head -16 gpurun_out/ns512_window.txt | cut -c1-120
