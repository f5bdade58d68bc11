# regnn_adam_flat with float4 and a quarter of the blocks: Adam / engine tests, then the one-rank
# rehearsal of the several-rank step (all-reduce + separate Adam in the graph), A/B old vs new
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/t_ns.log python -u -m pytest tests/test_gpu_ns_engine.py tests/test_gpu_ns_dp.py -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
grep -E "passed|failed|FAILED" gpurun_out/t_ns.log | tail -8 &&
export REGNN_NS_FORCE_EXCHANGE=1 &&
bash tools/ab_lib.sh 3 ab/libregnn_old.so re-gnn_amd/regnn_hip/libregnn_hip.so
