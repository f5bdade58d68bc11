# gather determinism probe, the whole -m gpu suite, then the NS step at the reference's hidden 512
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 300 python tools/debug_gather.py > gpurun_out/dbg_g.txt 2>&1; tail -30 gpurun_out/dbg_g.txt;
tools/gpu_step.sh 900 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
grep -E "passed|failed|FAILED" gpurun_out/pytest_gpu.log | tail -12 &&
tools/gpu_step.sh 300 gpurun_out/b_ns512.log python bench.py --workload ns --hidden 512 --no-full-batch --no-cpu-baseline &&
tail -2 gpurun_out/b_ns512.log | head -1 | cut -c1-300 && grep -o '"ns_kernels_ms.*' gpurun_out/b_ns512.log | cut -c1-1500
