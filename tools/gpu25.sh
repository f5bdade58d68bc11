cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
HEAD_C=349 HEAD_VARIANTS=16,0,2,4 tools/gpu_step.sh 300 gpurun_out/ab_head349.log python tools/ab_head.py &&
HEAD_C=352 HEAD_VARIANTS=16,0,2,4 tools/gpu_step.sh 300 gpurun_out/ab_head352.log python tools/ab_head.py &&
tail -n 2 gpurun_out/ab_head349.log gpurun_out/ab_head352.log
