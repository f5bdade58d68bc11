# default bench (driver's command), GAT layer stats + PMC per kernel (mag_like(1), uniform dst)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/b_default.log python bench.py &&
tail -1 gpurun_out/b_default.log | cut -c1-400 &&
G="python bench.py --workload gat --scale 1 --zipf 0 --steps 3 --warmup 1 --no-cpu-baseline" &&
tools/gpu_step.sh 300 gpurun_out/gat_stats.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gat -o run -- $G &&
tools/gpu_step.sh 300 gpurun_out/pmc_cal_f.log rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_cal_f -o run -- python tools/pmc_calib.py &&
tools/gpu_step.sh 300 gpurun_out/pmc_cal_w.log rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_cal_w -o run -- python tools/pmc_calib.py &&
tools/gpu_step.sh 300 gpurun_out/pmc_gat_f.log rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_gat_f -o run -- $G &&
tools/gpu_step.sh 300 gpurun_out/pmc_gat_w.log rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_gat_w -o run -- $G &&
python tools/pmc_kernels.py gpurun_out/pmc_gat_f gpurun_out/pmc_gat_w gpurun_out/pmc_cal_f gpurun_out/pmc_cal_w gpurun_out/prof_gat/run_kernel_stats.csv gpurun_out/pmc_gat_fp32.json regnn::
