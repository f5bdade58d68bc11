// Dense helpers of the training step on gfx950: a deterministic column sum of a tall row-major
// matrix (bias gradients of the per-node Linear heads, N up to ~2e7 rows). Each block owns a
// contiguous row range and keeps one partial per column per thread; block partials leave through
// a fixed-order slab (regnn_rel_reduce) — no atomics, rows read coalesced.
#include "regnn_common.h"

namespace regnn {

__global__ void __launch_bounds__(kBlock)
col_sum_kernel(const float* __restrict__ x, int64_t rows, int cols, int64_t rows_per_block,
               float* __restrict__ slab) {
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = min(rows, r0 + rows_per_block);
    for (int c = threadIdx.x; c < cols; c += kBlock) {
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
        int64_t r = r0;
        for (; r + 4 <= r1; r += 4) {
            s0 += x[r * cols + c];
            s1 += x[(r + 1) * cols + c];
            s2 += x[(r + 2) * cols + c];
            s3 += x[(r + 3) * cols + c];
        }
        for (; r < r1; ++r) s0 += x[r * cols + c];
        slab[(int64_t)blockIdx.x * cols + c] = (s0 + s1) + (s2 + s3);
    }
}

}  // namespace regnn

using namespace regnn;

extern "C" {

int regnn_col_sum(const float* x, int64_t rows, int32_t cols, float* slab, hipStream_t stream) {
    if (!x || !slab || rows < 0 || cols <= 0) return REGNN_EINVAL;
    const int grid = grid_for(rows, 1);      // <= kMaxGrid slab rows
    const int64_t rpb = (rows + grid - 1) / grid;
    hipLaunchKernelGGL(col_sum_kernel, dim3(grid), dim3(kBlock), 0, stream, x, rows, cols,
                       rpb > 0 ? rpb : 1, slab);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

}  // extern "C"
