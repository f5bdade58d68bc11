# PMC HBM traffic of the fused NS model step (FETCH_SIZE / WRITE_SIZE in separate passes,
# copy-calibrated) -> gpurun_out/pmc_ns_fp32.json (copy to profiles/ to commit)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
B="python bench.py --workload ns --no-full-batch --no-cpu-baseline --graph off --steps 4 --warmup 2" &&
tools/gpu_step.sh 300 gpurun_out/pmc_cal_f.log rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_cal_f -o run -- python tools/pmc_calib.py &&
tools/gpu_step.sh 300 gpurun_out/pmc_cal_w.log rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_cal_w -o run -- python tools/pmc_calib.py &&
tools/gpu_step.sh 300 gpurun_out/pmc_ns_fetch.log rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_ns_fetch -o run -- $B &&
tools/gpu_step.sh 300 gpurun_out/pmc_ns_write.log rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_ns_write -o run -- $B &&
python tools/pmc_ns_summary.py gpurun_out/pmc_ns_fetch gpurun_out/pmc_ns_write gpurun_out/pmc_cal_f gpurun_out/pmc_cal_w gpurun_out/pmc_ns_fp32.json 10.0 512 0.5
