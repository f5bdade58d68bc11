# kernel-trace stats of the default bench and the ns_infer workload
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 900 gpurun_out/prof_mag.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mag -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline &&
tools/gpu_step.sh 900 gpurun_out/prof_infer.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_infer -o run -- python bench.py --workload ns_infer --steps 5 --warmup 1 --no-cpu-baseline
