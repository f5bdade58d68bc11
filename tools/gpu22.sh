cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 300 gpurun_out/pytest_head.log python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_dropout.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -2 gpurun_out/pytest_head.log &&
tools/gpu_step.sh 300 gpurun_out/ab_head_bwd.log python tools/ab_head_bwd.py &&
tools/gpu_step.sh 600 gpurun_out/ab_rs.log python tools/ab_spmm.py --scale 10 --rounds 3 --dropout 0.5 --variants res:256:256:0:on:1,res:256:256:0:on:2,res:256:256:0:on:4 &&
tools/gpu_step.sh 600 gpurun_out/ab_rs_bf16.log python tools/ab_spmm.py --scale 10 --rounds 3 --dtype bf16 --dropout 0.5 --variants res:256:256:0:on:1,res:256:256:0:on:2,res:256:256:0:on:4 &&
tail -n 2 gpurun_out/ab_head_bwd.log && grep -A3 '"res' gpurun_out/ab_rs.log gpurun_out/ab_rs_bf16.log
