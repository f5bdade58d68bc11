# full -m gpu suite with the module path pipelined by default, then the h512 bench line
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider && tail -1 gpurun_out/pytest_gpu.log &&
tools/gpu_step.sh 300 gpurun_out/b_h512.log python bench.py --hidden 512 --no-full-batch --no-cpu-baseline --steps 50 && grep '^{' gpurun_out/b_h512.log | tail -1 > gpurun_out/bench_h512.json && python -c "import json;d=json.load(open('gpurun_out/bench_h512.json'));print('h512', d['ms_per_step'], d['config'].get('hidden'))"
