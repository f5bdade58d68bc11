# In-kernel phase marks of the two-layer NS step (instrumented builds: python
# tools/build_variant.py NAME -DREGNN_NSM2_PHASES [...] with AB_DIR=abx, shipped for this call only)
#   tools/gpu_phases.sh [NAME ...]     (default: phases)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out || exit 1
for v in ${@:-phases}; do
  REGNN_LIB=$PWD/abx/libregnn_$v.so timeout -k 10 200 python tools/nsm2_phases.py > gpurun_out/phases_$v.txt 2>&1 || { tail -5 gpurun_out/phases_$v.txt; exit 1; }
  echo "== $v"; grep -E "^(agg0|head|gather|bwd0|finalize) +blocks|mark  [0-2]:" gpurun_out/phases_$v.txt
done
