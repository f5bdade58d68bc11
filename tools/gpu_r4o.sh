# full -m gpu suite, NS PMC (fresh code hash), then the default bench with it
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider; tail -2 gpurun_out/pytest_gpu.log; grep -E "FAILED" gpurun_out/pytest_gpu.log | head;
bash tools/gpu_pmc_ns.sh && cp gpurun_out/pmc_ns_fp32.json profiles/pmc_ns_fp32.json && python -c "import json;d=json.load(open('gpurun_out/pmc_ns_fp32.json'));print(json.dumps(d['nsm_step'])[:700])" &&
tools/gpu_step.sh 600 gpurun_out/bench.log python bench.py && grep '^{' gpurun_out/bench.log | tail -1 > gpurun_out/bench_default.json && python -c "import json;d=json.load(open('gpurun_out/bench_default.json'));r=d['roofline'];print('default', d['ms_per_step'], d['value']/1e6, r['frac'], r.get('frac_hbm'), r.get('pmc'))"
