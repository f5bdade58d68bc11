cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 500 gpurun_out/t_ns.log python -u -m pytest tests/test_gpu_ns_engine.py tests/test_gpu_regnn_golden.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && tail -3 gpurun_out/t_ns.log &&
REGNN_LIB=$PWD/ab/libregnn_phases.so timeout -k 10 200 python tools/nsm2_phases.py > gpurun_out/phases_nopipe.txt 2>&1; grep -v "mark" gpurun_out/phases_nopipe.txt | head -30; grep "head" gpurun_out/phases_nopipe.txt;
bash tools/ab_lib2.sh 2 base cur
