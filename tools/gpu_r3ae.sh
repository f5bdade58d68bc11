# in-graph all-reduce by default (RCCL groups): DP tests, the one-rank rehearsal, the gloo 2-rank bench
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
tools/gpu_step.sh 600 gpurun_out/t_ns.log python -u -m pytest tests/test_gpu_ns_dp.py tests/test_gpu_ns_engine.py -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
grep -E "passed|failed|FAILED" gpurun_out/t_ns.log | tail -8 &&
REGNN_NS_FORCE_EXCHANGE=1 tools/gpu_step.sh 300 gpurun_out/b_rehearse.log python bench.py --workload ns --no-full-batch --no-cpu-baseline --steps 300 &&
grep '^{' gpurun_out/b_rehearse.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["config"]["grad_exchange"], d["config"]["lookahead"])' &&
REGNN_DIST_BACKEND=gloo tools/gpu_step.sh 400 gpurun_out/b_dp2.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --scale 1 --steps 20 --warmup 3 &&
grep '^{' gpurun_out/b_dp2.log | cut -c1-200
