cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
REGNN_LIB=$PWD/ab/libregnn_phases.so timeout -k 10 200 python tools/nsm2_phases.py > gpurun_out/phases_nopipe.txt 2>&1; head -8 gpurun_out/phases_nopipe.txt; grep "head\|agg0 " gpurun_out/phases_nopipe.txt;
REGNN_LIB=$PWD/ab/libregnn_phases.so timeout -k 10 200 python tools/nsm2_phases.py --pipeline > gpurun_out/phases_pipe.txt 2>&1; head -8 gpurun_out/phases_pipe.txt;
bash tools/ab_lib2.sh 2 base cur
