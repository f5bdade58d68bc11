# In-kernel phase marks of the two-layer NS step (an instrumented build: python
# tools/build_variant.py phases -DREGNN_NSM2_PHASES with AB_DIR=abx, shipped for this call only)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
REGNN_LIB=$PWD/abx/libregnn_phases.so timeout -k 10 200 python tools/nsm2_phases.py > gpurun_out/phases_nopipe.txt 2>&1; tail -45 gpurun_out/phases_nopipe.txt
