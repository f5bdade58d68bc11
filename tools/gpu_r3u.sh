# the multi-rank bench path rehearsed on one GPU (two ranks, gloo), then with the captured exchange
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
REGNN_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --scale 1 --steps 20 --warmup 3 > gpurun_out/b_dp2.log 2>&1; echo "rc=$?"; grep '^{' gpurun_out/b_dp2.log | cut -c1-400; tail -3 gpurun_out/b_dp2.log | cut -c1-300
