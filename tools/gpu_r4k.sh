cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 200 python -u -m pytest tests/test_gpu_gemm.py -q -x --timeout 120 -p no:cacheprovider 2>&1 | tail -2 &&
echo "== cur (2-ahead, interleave)" && timeout -k 10 120 python tools/ab_gemm.py 2>&1 | grep -v amdgpu.ids | head -6
echo "== committed (waves 2)" && REGNN_LIB=$PWD/ab/libregnn_g2.so timeout -k 10 120 python tools/ab_gemm.py 2>&1 | grep -v amdgpu.ids | head -6
