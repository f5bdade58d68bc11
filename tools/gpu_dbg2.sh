cd $GRAFT_REPO_ROOT && timeout -k 10 300 python tools/debug_gather2.py > gpurun_out/dbg_g2.txt 2>&1; tail -30 gpurun_out/dbg_g2.txt
