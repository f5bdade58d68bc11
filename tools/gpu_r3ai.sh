# agg0 stage-1 prefetch depth 3 (A/B build), then bwd0 / gather block counts after finalize's change
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
bash tools/ab_lib.sh 3 re-gnn_amd/regnn_hip/libregnn_hip.so ab/libregnn_pd3.so &&
bash tools/ab_env.sh 2 REGNN_NSM_BWD_BLOCKS 128 192 256 &&
bash tools/ab_env.sh 2 REGNN_NSM_GATH_BLOCKS 512 256 1024
