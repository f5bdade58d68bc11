# GEMM/linear/copy tests, NS/module/DP tests, h512 bench + shapes
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 900 gpurun_out/t_ns.log python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_ns_typed.py tests/test_gpu_ns_engine.py tests/test_gpu_ns.py tests/test_gpu_regnn_golden.py tests/test_gpu_ns_dp.py -q --timeout 300 --timeout-method thread -p no:cacheprovider; tail -3 gpurun_out/t_ns.log; grep -E "^FAILED|Error" gpurun_out/t_ns.log | head;
timeout -k 10 300 python bench.py --hidden 512 --no-full-batch --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/b_h512.json 2> gpurun_out/b_h512.err; python -c "import json;d=json.load(open('gpurun_out/b_h512.json'));print('h512', d['ms_per_step'], d['config']['engine'])";
timeout -k 10 300 python tools/h512_shapes.py > gpurun_out/h512_shapes.txt 2>&1; tail -30 gpurun_out/h512_shapes.txt | cut -c1-150
