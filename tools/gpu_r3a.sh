# round 3, first pass: NS engine + reference-pinned NS tests, the default bench line, NS PMC
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 500 gpurun_out/t_ns.log python -u -m pytest tests/test_gpu_ns_engine.py tests/test_gpu_regnn_golden.py tests/test_gpu_ns_dp.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
tail -5 gpurun_out/t_ns.log &&
tools/gpu_step.sh 400 gpurun_out/bench.log python bench.py &&
tail -1 gpurun_out/bench.log &&
bash tools/gpu_pmc_ns.sh
