# GAT el re-form: fused tests, then A/B of the fused forward
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 300 gpurun_out/t_gat.log python -u -m pytest tests/test_gpu_gat_fused.py tests/test_gpu_layers.py tests/test_gpu_ops.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider && tail -2 gpurun_out/t_gat.log &&
bash tools/ab_gat.sh 2 cur noelx un4 noelx4
