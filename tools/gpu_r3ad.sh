# one-rank rehearsal of the several-rank NS step: eager exchange between graphs vs captured in the
# step graph (REGNN_NS_GRAPH_ALLREDUCE), against the one-rank step
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
bash tools/ab_env.sh 1 REGNN_NS_AHEAD 8 &&
export REGNN_NS_FORCE_EXCHANGE=1 &&
bash tools/ab_env.sh 2 REGNN_NS_GRAPH_ALLREDUCE 0 1
