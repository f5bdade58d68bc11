cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/ab_bf16.log python tools/ab_spmm.py --scale 10 --rounds 3 --dtype bf16 --variants res:256:256:4,res:256:256:8,res:256:256:16 &&
tools/gpu_step.sh 600 gpurun_out/ab_bf16_drop.log python tools/ab_spmm.py --scale 10 --rounds 3 --dtype bf16 --dropout 0.5 --variants res:256:256 &&
tools/gpu_step.sh 600 gpurun_out/ab_f32_drop.log python tools/ab_spmm.py --scale 10 --rounds 3 --dropout 0.5 --variants res:256:256 &&
tools/gpu_step.sh 600 gpurun_out/prof_bf16.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bf16 -o run -- python bench.py --dtype bf16 --steps 5 --warmup 2 --no-cpu-baseline &&
grep -A3 '"res' gpurun_out/ab_bf16.log gpurun_out/ab_bf16_drop.log gpurun_out/ab_f32_drop.log
