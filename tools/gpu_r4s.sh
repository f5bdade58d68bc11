cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
echo "== cur" && timeout -k 10 120 python tools/ab_gemm.py 2>&1 | grep -v amdgpu.ids | head -3 &&
echo "== bk64" && REGNN_LIB=$PWD/ab/libregnn_bk64.so timeout -k 10 120 python tools/ab_gemm.py 2>&1 | grep -v amdgpu.ids | head -3 &&
REGNN_GEMM_BK64_TEST=1 REGNN_LIB=$PWD/ab/libregnn_bk64.so timeout -k 10 200 python -u -m pytest tests/test_gpu_gemm.py -q -x --timeout 120 -p no:cacheprovider 2>&1 | tail -1
