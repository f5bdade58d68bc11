cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
REGNN_LIB=$PWD/ab/libregnn_ntaph.so timeout -k 10 200 python tools/nsm2_phases.py > gpurun_out/phases_nta.txt 2>&1; tail -29 gpurun_out/phases_nta.txt | head -6;
bash tools/ab_lib2.sh 2 cur nta
