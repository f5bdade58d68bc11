# the driver's default bench with the refreshed NS PMC summary (traffic / frac_hbm), twice
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/b_default.log python bench.py &&
grep '^{' gpurun_out/b_default.log | cut -c1-200 &&
tools/gpu_step.sh 600 gpurun_out/b_default2.log python bench.py --no-full-batch --no-cpu-baseline &&
grep '^{' gpurun_out/b_default2.log | cut -c1-200
