cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_ns_engine.py tests/test_gpu_ns.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t.log 2>&1; tail -1 gpurun_out/t.log &&
REGNN_LIB=$PWD/ab/libregnn_phases.so timeout -k 10 200 python tools/nsm2_phases.py > gpurun_out/phases_nopipe.txt 2>&1; sed -n 3,12p gpurun_out/phases_nopipe.txt; tail -29 gpurun_out/phases_nopipe.txt | head -6;
bash tools/ab_lib2.sh 1 base cur
