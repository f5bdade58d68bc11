# round-4 verification: every -m gpu test, smoke, the default bench, NS kernel trace, NS PMC
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider; tail -2 gpurun_out/pytest_gpu.log; grep -E "FAILED" gpurun_out/pytest_gpu.log | head;
tools/gpu_step.sh 300 gpurun_out/smoke.log python -c "import __graft_entry__ as g; g.smoke()" && tail -1 gpurun_out/smoke.log &&
tools/gpu_step.sh 600 gpurun_out/bench.log python bench.py && grep '^{' gpurun_out/bench.log | tail -1 > gpurun_out/bench_default.json &&
tools/gpu_step.sh 300 gpurun_out/prof_ns.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ns -o run -- python bench.py --workload ns --no-full-batch --no-cpu-baseline --steps 50 &&
python tools/trace_window.py gpurun_out/prof_ns/run_kernel_trace.csv ns_batch_kernel 50 > gpurun_out/ns_window.txt && head -12 gpurun_out/ns_window.txt &&
tools/gpu_step.sh 300 gpurun_out/b_h512.log python bench.py --hidden 512 --no-full-batch --no-cpu-baseline --steps 50 && grep '^{' gpurun_out/b_h512.log | tail -1 > gpurun_out/bench_h512.json && python -c "import json;d=json.load(open('gpurun_out/bench_h512.json'));print('h512', d['ms_per_step'], d['config']['hidden'])" &&
bash tools/gpu_pmc_ns.sh && python -c "import json;d=json.load(open('gpurun_out/pmc_ns_fp32.json'));print(json.dumps(d['nsm_step'])[:600])"
