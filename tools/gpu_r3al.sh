# final: NS PMC (re_nsm.hip changed: hash), the whole -m gpu suite, smoke, the driver's bench
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
bash tools/gpu_pmc_ns.sh > gpurun_out/pmc_ns.out 2>&1 && tail -4 gpurun_out/pmc_ns.out &&
cp gpurun_out/pmc_ns_fp32.json profiles/pmc_ns_fp32.json &&
tools/gpu_step.sh 900 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
tail -2 gpurun_out/pytest_gpu.log && grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head;
tools/gpu_step.sh 200 gpurun_out/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" && tail -2 gpurun_out/smoke.log &&
tools/gpu_step.sh 600 gpurun_out/b_default.log python bench.py &&
grep '^{' gpurun_out/b_default.log | cut -c1-200
