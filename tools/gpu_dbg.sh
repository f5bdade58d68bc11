cd $GRAFT_REPO_ROOT && timeout -k 10 300 python tools/debug_gather.py > gpurun_out/dbg_g.txt 2>&1; tail -60 gpurun_out/dbg_g.txt
