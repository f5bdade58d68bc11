// Long-segment plans (regnn_seg_plan, include/regnn_hip.h) shared by the attention kernels
// (re_gat.hip, re_gatv2.hip): a segment with more than `split` edges is cut into `chunk`-edge
// chunks whose fp32 partial rows a fixed-order tree combines.
#pragma once
#include "regnn_common.h"

namespace regnn {

template <typename T>
__device__ __forceinline__ T from_f32(float v) {
    if constexpr (sizeof(T) == 2) return f2bf(v);
    else return v;
}

// ---- long segments (regnn_seg_plan) ---------------------------------------------------------
// A segment with more than `split` edges is skipped by the per-segment kernels and cut into
// `chunk`-edge chunks, each run by its own group into an fp32 partial row; a fixed-order tree
// (SegPlan's levels) combines a segment's partials and an emit kernel writes the result.
struct LongPlan {
    int split, chunk;                      // split = INT_MAX: every segment whole
    const int32_t* long_ids; const int32_t* chunk_long; const int32_t* chunk_off;
    int n_long, n_chunk;
    float* part;
};

inline LongPlan long_plan(const regnn_seg_plan* pl) {
    LongPlan P{};
    P.split = 0x7fffffff;
    if (pl && pl->n_long > 0 && pl->n_chunk > 0) {
        P.split = pl->split; P.chunk = pl->chunk;
        P.long_ids = pl->long_ids; P.chunk_long = pl->chunk_long; P.chunk_off = pl->chunk_off;
        P.n_long = pl->n_long; P.n_chunk = pl->n_chunk; P.part = pl->partial;
    }
    return P;
}

inline int check_plan(const regnn_seg_plan* pl, int64_t width) {
    if (!pl || pl->n_long <= 0 || pl->n_chunk <= 0) return REGNN_OK;
    if (pl->split < 1 || pl->chunk < 1 || !pl->long_ids || !pl->chunk_long || !pl->chunk_off ||
        pl->n_levels < 0 || (pl->n_levels > 0 && (!pl->level_sb || !pl->level_desc)))
        return REGNN_EINVAL;
    if (width > 0 && (!pl->partial || pl->partial_floats < pl->partial_rows * width ||
                      pl->partial_rows < pl->n_chunk))
        return REGNN_EINVAL;
    return REGNN_OK;
}

// chunk c -> (segment, edge range[, its long-segment index])
__device__ __forceinline__ void chunk_range(const LongPlan& P, const int32_t* __restrict__ ptr,
                                            int64_t c, int64_t& seg, int& beg, int& end, int& l) {
    l = P.chunk_long[c];
    seg = P.long_ids[l];
    const int rb = ptr[seg], re = ptr[seg + 1];
    beg = rb + int(c - P.chunk_off[l]) * P.chunk;
    end = min(beg + P.chunk, re);
}

__device__ __forceinline__ void chunk_range(const LongPlan& P, const int32_t* __restrict__ ptr,
                                            int64_t c, int64_t& seg, int& beg, int& end) {
    int l;
    chunk_range(P, ptr, c, seg, beg, end, l);
}

// the unit loop of the group kernels: unit -> (segment, first edge, edge count); false for a
// long segment in the per-segment pass
template <bool CH>
__device__ __forceinline__ bool group_unit(const LongPlan& P, const int32_t* __restrict__ ptr,
                                           int64_t unit, int64_t& seg, int& beg, int& n, int& l) {
    if (CH) {
        int end;
        chunk_range(P, ptr, unit, seg, beg, end, l);
        n = end - beg;
        return true;
    }
    seg = unit;
    l = -1;
    beg = ptr[seg];
    n = ptr[seg + 1] - beg;
    return n <= P.split;
}

// one tree level: partial row base_out + p = combine(rows base_in + [sb[p], sb[p+1])) in order
// (sb is relative to the level's inputs: the chunk rows, then the previous level's outputs).
// MODE 0: plain sums of W floats. MODE 1: online-softmax rows [acc F | max H | sum H] (head of
// acc column f: f / D), rescaled to the larger max.
template <int MODE>
__global__ void __launch_bounds__(kBlock)
seg_tree_level(float* __restrict__ part, const int32_t* __restrict__ sb, int64_t n_out, int W,
               int F, int H, int D, int64_t base_in, int64_t base_out) {
    for (int64_t p = blockIdx.x; p < n_out; p += gridDim.x) {
        const int64_t r0 = base_in + sb[p], r1 = base_in + sb[p + 1];
        float* __restrict__ o = part + (base_out + p) * W;
        for (int w = threadIdx.x; w < W; w += kBlock) {
            if (MODE == 0) {
                float acc = 0.f;
                for (int64_t r = r0; r < r1; ++r) acc += part[r * W + w];
                o[w] = acc;
            } else {
                const int h = w < F ? w / D : (w < F + H ? w - F : w - F - H);
                float M = -INFINITY, S = 0.f, A = 0.f;
                for (int64_t r = r0; r < r1; ++r) {
                    const float* pr = part + r * W;
                    const float m = pr[F + h], sv = pr[F + H + h], a = w < F ? pr[w] : 0.f;
                    const float mn = fmaxf(M, m);
                    if (mn == -INFINITY) continue;
                    const float f0 = M == -INFINITY ? 0.f : __expf(M - mn);
                    const float f1 = m == -INFINITY ? 0.f : __expf(m - mn);
                    A = A * f0 + a * f1;
                    S = S * f0 + sv * f1;
                    M = mn;
                }
                o[w] = w < F ? A : (w < F + H ? M : S);
            }
        }
    }
}

// row of the combined partial of long segment l
__device__ __forceinline__ int64_t final_row(const int32_t* __restrict__ chunk_off, int64_t base,
                                             int n_levels, int l) {
    return n_levels > 0 ? base + l : int64_t(chunk_off[l]);
}

// dst[long_ids[l]][w] = combined partial (plain sums), l < n_long
template <typename T>
__global__ void __launch_bounds__(kBlock)
seg_emit_sum(const float* __restrict__ part, const int32_t* __restrict__ chunk_off, int64_t base,
             int n_levels, const int32_t* __restrict__ long_ids, int n_long, int W,
             T* __restrict__ dst) {
    for (int l = blockIdx.x; l < n_long; l += gridDim.x) {
        const float* __restrict__ pr = part + final_row(chunk_off, base, n_levels, l) * W;
        const int64_t row = long_ids[l];
        for (int w = threadIdx.x; w < W; w += kBlock) dst[row * W + w] = from_f32<T>(pr[w]);
    }
}

// out[row] = acc / sum, lse[row] = max + log sum from a combined online-softmax row
template <typename T>
__global__ void __launch_bounds__(kBlock)
seg_emit_softmax(const float* __restrict__ part, const int32_t* __restrict__ chunk_off,
                 int64_t base, int n_levels, const int32_t* __restrict__ long_ids, int n_long,
                 int F, int H, int D, T* __restrict__ out, float* __restrict__ lse) {
    const int W = F + 2 * H;
    for (int l = blockIdx.x; l < n_long; l += gridDim.x) {
        const float* __restrict__ pr = part + final_row(chunk_off, base, n_levels, l) * W;
        const int64_t row = long_ids[l];
        for (int f = threadIdx.x; f < F; f += kBlock) {
            const float sv = pr[F + H + f / D];
            out[row * F + f] = from_f32<T>(sv > 0.f ? pr[f] / sv : 0.f);
        }
        for (int h = threadIdx.x; h < H; h += kBlock) {
            const float sv = pr[F + H + h];
            lse[row * H + h] = sv > 0.f ? pr[F + h] + __logf(sv) : -INFINITY;
        }
    }
}

// launch the tree levels of a plan; returns the row base of the last level
inline int64_t run_tree(const regnn_seg_plan* pl, int mode, int W, int F, int H, int D,
                        hipStream_t stream) {
    int64_t base = 0, base_in = 0;
    for (int k = 0; k < pl->n_levels; ++k) {
        const int64_t sb_off = pl->level_desc[3 * k], n_out = pl->level_desc[3 * k + 1];
        base = pl->level_desc[3 * k + 2];
        const int grid = int(n_out < kMaxGrid ? n_out : kMaxGrid);
        if (mode == 0)
            hipLaunchKernelGGL(seg_tree_level<0>, dim3(grid), dim3(kBlock), 0, stream,
                               pl->partial, pl->level_sb + sb_off, n_out, W, F, H, D, base_in,
                               base);
        else
            hipLaunchKernelGGL(seg_tree_level<1>, dim3(grid), dim3(kBlock), 0, stream,
                               pl->partial, pl->level_sb + sb_off, n_out, W, F, H, D, base_in,
                               base);
        base_in = base;
    }
    return base;
}

inline int long_grid(int n) { return n < kMaxGrid ? (n > 0 ? n : 1) : kMaxGrid; }

}  // namespace regnn
