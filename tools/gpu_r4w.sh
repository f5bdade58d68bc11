cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
REGNN_LIB=$PWD/ab/libregnn_r12.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ns_engine.py -x -q -k "fused_step_matches_module or bitwise" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t.log 2>&1; tail -1 gpurun_out/t.log &&
bash tools/ab_lib2.sh 2 cur r12 r14
