# full -m gpu suite + smoke + default bench after the GAT ABI-40 change
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider; tail -1 gpurun_out/pytest_gpu.log; grep -E "FAILED" gpurun_out/pytest_gpu.log | head;
tools/gpu_step.sh 300 gpurun_out/smoke.log python -c "import __graft_entry__ as g; g.smoke()" && tail -1 gpurun_out/smoke.log &&
tools/gpu_step.sh 600 gpurun_out/bench.log python bench.py && grep '^{' gpurun_out/bench.log | tail -1 > gpurun_out/bench_default.json && python -c "import json;d=json.load(open('gpurun_out/bench_default.json'));r=d['roofline'];print('default', d['ms_per_step'], d['value']/1e6, r['frac'], r.get('frac_hbm'), r.get('pmc'))"
