cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/t_ns.log python -u -m pytest tests/test_gpu_ns_typed.py tests/test_gpu_ns_engine.py tests/test_gpu_ns.py tests/test_gpu_regnn_golden.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && tail -5 gpurun_out/t_ns.log &&
bash tools/ab_lib2.sh 2 base cur &&
REGNN_LIB=$PWD/ab/libregnn_phases.so timeout -k 10 200 python tools/nsm2_phases.py > gpurun_out/phases_nopipe.txt 2>&1; tail -32 gpurun_out/phases_nopipe.txt
