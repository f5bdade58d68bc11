# gather: the next row's entry range prefetched. NS parity tests, A/B against the old build
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/t_ns.log python -u -m pytest tests/test_gpu_ns_engine.py tests/test_gpu_ns_typed.py tests/test_gpu_regnn_golden.py -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
grep -E "passed|failed|FAILED" gpurun_out/t_ns.log | tail -8 &&
bash tools/ab_lib.sh 3 ab/libregnn_old.so re-gnn_amd/regnn_hip/libregnn_hip.so
