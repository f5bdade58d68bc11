# two targets per wave in the strided sampler, with the sampler off the critical path (lookahead 8)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
bash tools/ab_env.sh 3 REGNN_NS_HALF_WAVES 0 1
