cd $GRAFT_REPO_ROOT && timeout -k 10 300 python tools/debug_det.py > gpurun_out/det.txt 2>&1; tail -60 gpurun_out/det.txt
