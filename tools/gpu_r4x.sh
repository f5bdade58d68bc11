# final: full -m gpu suite, smoke, fresh NS PMC, default bench, phases, h512 bench, exchange rehearsal
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider; tail -1 gpurun_out/pytest_gpu.log; grep -E "FAILED" gpurun_out/pytest_gpu.log | head;
tools/gpu_step.sh 300 gpurun_out/smoke.log python -c "import __graft_entry__ as g; g.smoke()" && tail -1 gpurun_out/smoke.log &&
bash tools/gpu_pmc_ns.sh > gpurun_out/pmc.log 2>&1; tail -2 gpurun_out/pmc.log; cp gpurun_out/pmc_ns_fp32.json profiles/pmc_ns_fp32.json &&
tools/gpu_step.sh 600 gpurun_out/bench.log python bench.py && grep '^{' gpurun_out/bench.log | tail -1 > gpurun_out/bench_default.json && python -c "import json;d=json.load(open('gpurun_out/bench_default.json'));r=d['roofline'];print('default', d['ms_per_step'], d['value']/1e6, r['frac'], r.get('frac_hbm'), r.get('pmc'))" &&
REGNN_LIB=$PWD/ab/libregnn_phases.so timeout -k 10 200 python tools/nsm2_phases.py > gpurun_out/phases_nopipe.txt 2>&1; tail -29 gpurun_out/phases_nopipe.txt | head -6;
tools/gpu_step.sh 300 gpurun_out/b_h512.log python bench.py --hidden 512 --no-full-batch --no-cpu-baseline --steps 50 && grep '^{' gpurun_out/b_h512.log | tail -1 > gpurun_out/bench_h512.json && python -c "import json;d=json.load(open('gpurun_out/bench_h512.json'));print('h512', d['ms_per_step'])";
REGNN_NS_FORCE_EXCHANGE=1 tools/gpu_step.sh 300 gpurun_out/b_reh.log python bench.py --no-full-batch --no-cpu-baseline --steps 300 && grep '^{' gpurun_out/b_reh.log | tail -1 > gpurun_out/bench_rehearse.json && python -c "import json;d=json.load(open('gpurun_out/bench_rehearse.json'));print('rehearse', d['ms_per_step'])"
