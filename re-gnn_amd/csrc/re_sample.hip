// Neighbour sampler for the ogbn-mag neighbour-sampled path (replaces torch_sparse sample_adj
// behind PyG NeighborSampler, mag/regnn_ns.py:206-214). Spec in include/regnn_hip.h.
// One wave per target: lane i owns slot i of the sample set, Floyd's algorithm runs with a
// ballot membership test, and the chosen positions are ranked in-register to ascending order.
#include "regnn_common.h"

namespace regnn {

__device__ __forceinline__ uint32_t sample_hash(uint64_t seed, uint64_t t, uint64_t j) {
    uint64_t x = seed + 0x9E3779B97F4A7C15ull * (t + 1) + 0xD1B54A32D192ED03ull * (j + 1);
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return uint32_t(x >> 32);
}

__global__ void __launch_bounds__(kBlock)
sample_count_kernel(const int32_t* __restrict__ ptr, const int32_t* __restrict__ targets,
                    int64_t n, int k, int32_t* __restrict__ counts) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kBlock) {
        const int t = targets[i];
        const int d = ptr[t + 1] - ptr[t];
        counts[i] = (k < 0 || d <= k) ? d : k;
    }
}

__global__ void __launch_bounds__(kBlock)
sample_fill_kernel(const int32_t* __restrict__ ptr, const int32_t* __restrict__ idx,
                   const int32_t* __restrict__ targets, int64_t n, int k, uint64_t seed,
                   const int32_t* __restrict__ offs, int32_t* __restrict__ out_src,
                   int32_t* __restrict__ out_eid) {
    const int lane = threadIdx.x & 63;
    const int64_t wpb = kBlock / 64;
    for (int64_t i = (int64_t)blockIdx.x * wpb + threadIdx.x / 64; i < n;
         i += (int64_t)gridDim.x * wpb) {
        const int t = targets[i];
        const int b = ptr[t], d = ptr[t + 1] - b;
        const int o = offs[i];
        if (k < 0 || d <= k) {
            for (int q = lane; q < d; q += 64) {
                out_src[o + q] = idx[b + q];
                out_eid[o + q] = b + q;
            }
            continue;
        }
        int slot = -1;   // position held by this lane (lane < k)
        int filled = 0;
        for (int j = d - k; j < d; ++j) {
            const uint32_t r = sample_hash(seed, uint64_t(t), uint64_t(j));
            const int pos = int((uint64_t(r) * uint64_t(j + 1)) >> 32);
            const bool seen = __any(slot == pos);
            const int pick = seen ? j : pos;
            if (lane == filled) slot = pick;
            ++filled;
        }
        int rank = 0;
        for (int m = 0; m < k; ++m) {
            const int other = __shfl(slot, m, 64);
            rank += (lane < k && other < slot) ? 1 : 0;
        }
        if (lane < k) {
            out_src[o + rank] = idx[b + slot];
            out_eid[o + rank] = b + slot;
        }
    }
}

}  // namespace regnn

using namespace regnn;

extern "C" {

int regnn_sample_count(const int32_t* ptr, const int32_t* targets, int64_t n_targets, int32_t k,
                       int32_t* counts, hipStream_t stream) {
    if (!ptr || !targets || !counts || n_targets < 0) return REGNN_EINVAL;
    if (n_targets == 0) return REGNN_OK;
    hipLaunchKernelGGL(sample_count_kernel, dim3(grid_for(n_targets, kBlock)), dim3(kBlock), 0,
                       stream, ptr, targets, n_targets, k, counts);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

int regnn_sample_fill(const int32_t* ptr, const int32_t* idx, const int32_t* targets,
                      int64_t n_targets, int32_t k, uint64_t seed, const int32_t* offs,
                      int32_t* out_src, int32_t* out_eid, hipStream_t stream) {
    if (!ptr || !idx || !targets || !offs || !out_src || !out_eid || n_targets < 0)
        return REGNN_EINVAL;
    if (k > 64) return REGNN_EUNSUPPORTED;
    if (n_targets == 0) return REGNN_OK;
    hipLaunchKernelGGL(sample_fill_kernel, dim3(grid_for(n_targets, kBlock / 64)), dim3(kBlock), 0,
                       stream, ptr, idx, targets, n_targets, k, seed, offs, out_src, out_eid);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

}  // extern "C"
