cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/t_wide.log python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_ns_typed.py tests/test_gpu_ns_engine.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && tail -5 gpurun_out/t_wide.log &&
timeout -k 10 120 python tools/ab_gemm.py > gpurun_out/ab_gemm.txt 2>&1; cat gpurun_out/ab_gemm.txt;
timeout -k 10 300 python bench.py --hidden 512 --no-full-batch --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/b_h512.json 2> gpurun_out/b_h512.err; python -c "import json;d=json.load(open('gpurun_out/b_h512.json'));print('h512', d['ms_per_step'], d['config']['engine'])";
bash tools/ab_lib2.sh 2 base cur;
REGNN_NSM_AGG0_OLD=1 bash tools/ab_lib2.sh 1 cur;
REGNN_LIB=$PWD/ab/libregnn_phases.so timeout -k 10 200 python tools/nsm2_phases.py > gpurun_out/phases_nopipe.txt 2>&1; tail -40 gpurun_out/phases_nopipe.txt
