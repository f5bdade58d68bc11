# PMC HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes, copy-calibrated) + kernel stats for
# the mag-10x bench at fp32 and bf16. Summaries -> gpurun_out/pmc_mag_<dtype>.json
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 300 gpurun_out/pmc_cal_f.log rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_cal_f -o run -- python tools/pmc_calib.py &&
tools/gpu_step.sh 300 gpurun_out/pmc_cal_w.log rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_cal_w -o run -- python tools/pmc_calib.py &&
for dt in fp32 bf16; do
  B="python bench.py --workload mag --dtype $dt --steps 2 --warmup 0 --no-cpu-baseline"
  tools/gpu_step.sh 600 gpurun_out/pmc_fetch_$dt.log rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_$dt -o run -- $B || exit 1
  tools/gpu_step.sh 600 gpurun_out/pmc_write_$dt.log rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_$dt -o run -- $B || exit 1
  python tools/pmc_summary.py gpurun_out/pmc_fetch_$dt gpurun_out/pmc_write_$dt gpurun_out/pmc_cal_f gpurun_out/pmc_cal_w gpurun_out/pmc_mag_$dt.json 19397430 441617570 $dt || exit 1
  tools/gpu_step.sh 600 gpurun_out/prof_$dt.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$dt -o run -- python bench.py --workload mag --dtype $dt --steps 20 --warmup 3 --no-cpu-baseline || exit 1
done &&
for d in gpurun_out/pmc_fetch_* gpurun_out/pmc_write_* gpurun_out/pmc_cal_*; do
  f=$(find $d -name '*counter_collection.csv' | head -n 1); [ -n "$f" ] && (head -n 1 $f; grep 'regnn::\|__amd_rocclr_copyBuffer\|elementwise' $f || true) > $d.regnn_rows.csv
done; ls gpurun_out
