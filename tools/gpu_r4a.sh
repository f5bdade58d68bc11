cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 500 gpurun_out/t_ns.log python -u -m pytest tests/test_gpu_ns_engine.py tests/test_gpu_regnn_golden.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && tail -3 gpurun_out/t_ns.log &&
REGNN_LIB=$PWD/ab/libregnn_phases.so timeout -k 10 200 python tools/nsm2_phases.py > gpurun_out/phases_nopipe.txt 2>&1; head -8 gpurun_out/phases_nopipe.txt &&
timeout -k 10 300 python bench.py --no-full-batch --no-cpu-baseline --steps 300 --warmup 20 > gpurun_out/b_ns.json 2> gpurun_out/b_ns.err; python -c "import json;d=json.load(open('gpurun_out/b_ns.json'));print(d['ms_per_step'], d['value']/1e9, d['ns_kernels_ms'])"
