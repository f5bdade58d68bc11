cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
B="python bench.py --steps 2 --warmup 0 --no-cpu-baseline" &&
tools/gpu_step.sh 900 gpurun_out/pmc_fetch.log rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o run -- $B &&
tools/gpu_step.sh 900 gpurun_out/pmc_write.log rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o run -- $B &&
tools/gpu_step.sh 300 gpurun_out/pmc_cal_f.log rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_cal_f -o run -- python tools/pmc_calib.py &&
tools/gpu_step.sh 300 gpurun_out/pmc_cal_w.log rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_cal_w -o run -- python tools/pmc_calib.py &&
ls gpurun_out/pmc_fetch
