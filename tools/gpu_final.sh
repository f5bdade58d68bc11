# round-end measurement set: full bench lines (fp32 default with cpu_baseline, bf16), kernel
# stats and PMC HBM traffic of the mag-10x step
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 900 gpurun_out/bench_full.log python bench.py &&
tools/gpu_step.sh 600 gpurun_out/bench_bf16.log python bench.py --dtype bf16 --no-cpu-baseline &&
tools/gpu_pmc2.sh
