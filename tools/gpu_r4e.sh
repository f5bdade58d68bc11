cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/t_wide.log python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_ns_typed.py tests/test_gpu_regnn_golden.py tests/test_gpu_ns_engine.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && tail -15 gpurun_out/t_wide.log &&
timeout -k 10 120 python tools/ab_gemm.py > gpurun_out/ab_gemm.txt 2>&1; cat gpurun_out/ab_gemm.txt;
timeout -k 10 300 python bench.py --hidden 512 --no-full-batch --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/b_h512.json 2> gpurun_out/b_h512.err; python -c "import json;d=json.load(open('gpurun_out/b_h512.json'));print('h512', d['ms_per_step'], d['config']['engine'])";
REGNN_GEMM_X6=off REGNN_WIDE_EPI=off timeout -k 10 300 python bench.py --hidden 512 --no-full-batch --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/b_h512_off.json 2>&1; grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_h512_off.json;
bash tools/ab_lib2.sh 2 base cur
