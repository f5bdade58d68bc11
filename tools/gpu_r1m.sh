# round-end measurement set at the current code: smoke, both bench lines, PMC + kernel stats
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 300 gpurun_out/smoke.log python __graft_entry__.py smoke &&
bash tools/gpu_final.sh
