# GAT el re-form (UN 4): GAT-related GPU tests, A/B against the el-reading kernel, GAT stats + PMC
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 400 gpurun_out/t_gat.log python -u -m pytest tests/test_gpu_gat_fused.py tests/test_gpu_layers.py tests/test_gpu_ops.py tests/test_gpu_regnn_golden.py tests/test_gpu_mag.py tests/test_gpu_configs.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider && tail -1 gpurun_out/t_gat.log &&
bash tools/ab_gat.sh 2 cur noelx hun4 hun6 &&
G="python bench.py --workload gat --scale 1 --zipf 0 --steps 3 --warmup 1 --no-cpu-baseline" &&
tools/gpu_step.sh 300 gpurun_out/gat_stats.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gat -o run -- $G &&
tools/gpu_step.sh 300 gpurun_out/pmc_cal_f.log rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_cal_f -o run -- python tools/pmc_calib.py &&
tools/gpu_step.sh 300 gpurun_out/pmc_cal_w.log rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_cal_w -o run -- python tools/pmc_calib.py &&
tools/gpu_step.sh 300 gpurun_out/pmc_gat_f.log rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_gat_f -o run -- $G &&
tools/gpu_step.sh 300 gpurun_out/pmc_gat_w.log rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_gat_w -o run -- $G &&
python tools/pmc_kernels.py gpurun_out/pmc_gat_f gpurun_out/pmc_gat_w gpurun_out/pmc_cal_f gpurun_out/pmc_cal_w gpurun_out/prof_gat/run_kernel_stats.csv gpurun_out/pmc_gat_fp32.json regnn:: &&
grep '^{' gpurun_out/gat_stats.log | tail -1 > gpurun_out/bench_gat.json; rm -rf gpurun_out/pmc_gat_f gpurun_out/pmc_gat_w gpurun_out/pmc_cal_f gpurun_out/pmc_cal_w
