cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
REGNN_LIB=$PWD/ab/libregnn_phases.so timeout -k 10 200 python tools/nsm2_phases.py > gpurun_out/phases_nopipe.txt 2>&1; cat gpurun_out/phases_nopipe.txt | tail -40 &&
REGNN_LIB=$PWD/ab/libregnn_phases.so timeout -k 10 200 python tools/nsm2_phases.py --pipeline > gpurun_out/phases_pipe.txt 2>&1; tail -40 gpurun_out/phases_pipe.txt
