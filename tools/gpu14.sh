cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 300 gpurun_out/pytest_drop.log python -u -m pytest tests/test_gpu_dropout.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -2 gpurun_out/pytest_drop.log &&
tools/gpu_step.sh 600 gpurun_out/ab_bf16.log python tools/ab_spmm.py --scale 10 --rounds 3 --dtype bf16 --variants res:256:256:0:off,res:256:256:0:on &&
tools/gpu_step.sh 600 gpurun_out/ab_bf16_drop.log python tools/ab_spmm.py --scale 10 --rounds 3 --dtype bf16 --dropout 0.5 --variants res:256:256:0:off,res:256:256:0:on &&
tools/gpu_step.sh 600 gpurun_out/ab_f32.log python tools/ab_spmm.py --scale 10 --rounds 3 --variants res:256:256:0:off,res:256:256:0:on &&
tools/gpu_step.sh 600 gpurun_out/ab_f32_drop.log python tools/ab_spmm.py --scale 10 --rounds 3 --dropout 0.5 --variants res:256:256:0:off,res:256:256:0:on &&
grep -A3 '"res' gpurun_out/ab_bf16.log gpurun_out/ab_bf16_drop.log gpurun_out/ab_f32.log gpurun_out/ab_f32_drop.log
