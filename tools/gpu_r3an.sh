# agg0 grid capped at 512 blocks (grid-stride over the 832 tiles) against 832 (A/B builds)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
bash tools/ab_lib.sh 2 re-gnn_amd/regnn_hip/libregnn_hip.so ab/libregnn_g512.so
