cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 300 gpurun_out/t_gemm.log python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider && tail -3 gpurun_out/t_gemm.log &&
timeout -k 10 120 python tools/ab_gemm.py > gpurun_out/ab_gemm.txt 2>&1; cat gpurun_out/ab_gemm.txt;
bash tools/gpu_r4c.sh
