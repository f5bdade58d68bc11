// GAT relation-embedding attention for gfx950 (layer/REGATConv.py:64-100):
//  * edge softmax over the in-edges of each destination with the u_add_v SDDMM, the relation
//    bias table and the LeakyReLU fused (one thread per (destination, head));
//  * per-head weighted SpMM (a group of lanes per destination, 16-byte row vectors; the lane's
//    head is fixed by its feature offset), and its fused transposed backward that also forms the
//    per-(edge, head) dot <g[v,h,:], x[u,h,:]> with an in-register head reduction;
//  * the softmax / LeakyReLU / u_add_v backward with deterministic relation-bias slabs.
#include "regnn_common.h"

namespace regnn {

__device__ __forceinline__ float lrelu(float x, float slope) { return x > 0.f ? x : x * slope; }

__global__ void __launch_bounds__(kBlock)
gat_softmax_fwd_kernel(const int32_t* __restrict__ ptr, const int32_t* __restrict__ idx,
                       const uint8_t* __restrict__ rel, const float* __restrict__ ee,
                       const float* __restrict__ el, const float* __restrict__ er, int64_t n_seg,
                       int H, float slope, float* __restrict__ a) {
    const int64_t total = n_seg * H;
    for (int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * kBlock) {
        const int64_t v = t / H;
        const int h = int(t - v * H);
        const int b = ptr[v], e = ptr[v + 1];
        const float erv = er[t];
        float m = -INFINITY;
        for (int k = b; k < e; ++k) {
            float s = el[(int64_t)idx[k] * H + h] + erv;
            if (ee) s += ee[rel[k] * H + h];
            m = fmaxf(m, lrelu(s, slope));
        }
        float sum = 0.f;
        for (int k = b; k < e; ++k) {
            float s = el[(int64_t)idx[k] * H + h] + erv;
            if (ee) s += ee[rel[k] * H + h];
            sum += __expf(lrelu(s, slope) - m);
        }
        const float inv = 1.f / sum;
        for (int k = b; k < e; ++k) {
            float s = el[(int64_t)idx[k] * H + h] + erv;
            if (ee) s += ee[rel[k] * H + h];
            a[(int64_t)k * H + h] = __expf(lrelu(s, slope) - m) * inv;
        }
    }
}

__global__ void __launch_bounds__(kBlock)
gat_softmax_bwd_kernel(const int32_t* __restrict__ ptr, const int32_t* __restrict__ idx,
                       const uint8_t* __restrict__ rel, const float* __restrict__ ee,
                       const float* __restrict__ el, const float* __restrict__ er,
                       const float* __restrict__ a, const float* __restrict__ ga, int64_t n_seg,
                       int H, float slope, float* __restrict__ gs_out, float* __restrict__ ger,
                       float* __restrict__ slab, int n_rel) {
    extern __shared__ float bins[];   // [n_rel][kBlock]; a thread only touches its own column
    const int tid = threadIdx.x;
    if (slab) for (int r = 0; r < n_rel; ++r) bins[r * kBlock + tid] = 0.f;
    const int64_t total = n_seg * H;
    for (int64_t t = (int64_t)blockIdx.x * kBlock + tid; t < total;
         t += (int64_t)gridDim.x * kBlock) {
        const int64_t v = t / H;
        const int h = int(t - v * H);
        const int b = ptr[v], e = ptr[v + 1];
        float dot = 0.f;
        for (int k = b; k < e; ++k) dot += a[(int64_t)k * H + h] * ga[(int64_t)k * H + h];
        const float erv = er[t];
        float gsum = 0.f;
        for (int k = b; k < e; ++k) {
            const int64_t kh = (int64_t)k * H + h;
            float s = el[(int64_t)idx[k] * H + h] + erv;
            if (ee) s += ee[rel[k] * H + h];
            const float gz = a[kh] * (ga[kh] - dot);
            const float gs = s > 0.f ? gz : gz * slope;
            gs_out[kh] = gs;
            gsum += gs;
            if (slab) bins[rel[k] * kBlock + tid] += gs;
        }
        ger[t] = gsum;
    }
    if (slab) {
        // kBlock % H == 0, so thread tid always works on head tid % H
        __syncthreads();
        for (int c = tid; c < n_rel * H; c += kBlock) {
            const int r = c / H, h = c - r * H;
            float s = 0.f;
            for (int t2 = h; t2 < kBlock; t2 += H) s += bins[r * kBlock + t2];
            slab[(int64_t)blockIdx.x * n_rel * H + c] = s;
        }
    }
}

// ---- per-head weighted SpMM ----------------------------------------------------------------
struct HeadArgs {
    const int32_t* ptr;
    const int32_t* idx;
    const int32_t* perm;
    const float* a;
    const void* src;    // x (fwd) or g (bwd)
    const void* self;   // bwd: x rows of the segment node
    void* out;
    float* ga;
    int64_t n_seg;
    int H, D;
};

template <typename T, int LPR, int NV, bool BWD>
__global__ void __launch_bounds__(kBlock) spmm_heads_kernel(HeadArgs p) {
    constexpr int EV = Vec<T>::N;
    constexpr int GPB = kBlock / LPR;
    const int tid = threadIdx.x, lane = tid & (LPR - 1);
    const int F = p.H * p.D;
    const int vph = p.D / EV;   // vectors per head (power of two, <= LPR)
    const T* __restrict__ src = static_cast<const T*>(p.src);
    for (int64_t seg = (int64_t)blockIdx.x * GPB + tid / LPR; seg < p.n_seg;
         seg += (int64_t)gridDim.x * GPB) {
        const int beg = p.ptr[seg], end = p.ptr[seg + 1];
        float acc[NV][EV] = {};
        float sx[NV][EV] = {};
        int head[NV];
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            const int o = (q * LPR + lane) * EV;
            head[q] = o < F ? o / p.D : 0;
            if (BWD && o < F) Vec<T>::load(static_cast<const T*>(p.self) + seg * F + o, sx[q]);
        }
        for (int e0 = beg; e0 < end; e0 += LPR) {
            const int e = e0 + lane;
            int j = 0, eid = 0;
            if (e < end) {
                j = p.idx[e];
                eid = p.perm ? p.perm[e] : e;
            }
            const int cnt = min(LPR, end - e0);
            for (int k = 0; k < cnt; ++k) {
                const int jj = __shfl(j, k, LPR);
                const int ek = __shfl(eid, k, LPR);
                float v[NV][EV];
#pragma unroll
                for (int q = 0; q < NV; ++q) {
                    const int o = (q * LPR + lane) * EV;
                    if (o < F) Vec<T>::load(src + (int64_t)jj * F + o, v[q]);
                    else
#pragma unroll
                        for (int t = 0; t < EV; ++t) v[q][t] = 0.f;
                }
#pragma unroll
                for (int q = 0; q < NV; ++q) {
                    const int o = (q * LPR + lane) * EV;
                    const float w = o < F ? p.a[(int64_t)ek * p.H + head[q]] : 0.f;
#pragma unroll
                    for (int t = 0; t < EV; ++t) acc[q][t] = fmaf(w, v[q][t], acc[q][t]);
                    if constexpr (BWD) {
                        float d = 0.f;
#pragma unroll
                        for (int t = 0; t < EV; ++t) d = fmaf(v[q][t], sx[q][t], d);
                        for (int m = vph >> 1; m > 0; m >>= 1) d += __shfl_xor(d, m, 64);
                        if (o < F && (lane & (vph - 1)) == 0) p.ga[(int64_t)ek * p.H + head[q]] = d;
                    }
                }
            }
        }
        T* __restrict__ out = static_cast<T*>(p.out) + seg * F;
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            const int o = (q * LPR + lane) * EV;
            if (o < F) Vec<T>::store(out + o, acc[q]);
        }
    }
}

template <typename T, bool BWD>
int dispatch_heads(HeadArgs p, hipStream_t stream) {
    constexpr int EV = Vec<T>::N;
    const int F = p.H * p.D;
    if (p.D <= 0 || p.D % EV || p.H <= 0) return REGNN_EUNSUPPORTED;
    const int vph = p.D / EV;
    if (vph & (vph - 1)) return REGNN_EUNSUPPORTED;
    const int nvec = F / EV;
#define REGNN_HEADS(LPR, NV)                                                                    \
    if (nvec <= (LPR) * (NV) && vph <= (LPR)) {                                                 \
        hipLaunchKernelGGL((spmm_heads_kernel<T, LPR, NV, BWD>),                                \
                           dim3(grid_for(p.n_seg, kBlock / (LPR))), dim3(kBlock), 0, stream, p); \
        REGNN_LAUNCH_CHECK();                                                                   \
        return REGNN_OK;                                                                        \
    }
    REGNN_HEADS(16, 1)
    REGNN_HEADS(16, 2)
    REGNN_HEADS(16, 4)
    REGNN_HEADS(64, 2)
    REGNN_HEADS(64, 4)
    REGNN_HEADS(64, 8)
#undef REGNN_HEADS
    return REGNN_EUNSUPPORTED;
}

__global__ void __launch_bounds__(kBlock)
segment_sum_kernel(const int32_t* __restrict__ ptr, const int32_t* __restrict__ perm,
                   const float* __restrict__ vals, int64_t n_seg, int H, float* __restrict__ out) {
    const int64_t total = n_seg * H;
    for (int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * kBlock) {
        const int64_t s = t / H;
        const int h = int(t - s * H);
        float acc = 0.f;
        for (int k = ptr[s]; k < ptr[s + 1]; ++k)
            acc += vals[(int64_t)(perm ? perm[k] : k) * H + h];
        out[t] = acc;
    }
}

}  // namespace regnn

using namespace regnn;

extern "C" {

int regnn_gat_softmax_fwd(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                          const float* ee_table, const float* el, const float* er, int64_t n_seg,
                          int32_t H, float slope, float* a, hipStream_t stream) {
    if (!ptr || !idx || !el || !er || !a || H <= 0 || n_seg < 0 || (ee_table && !rel))
        return REGNN_EINVAL;
    if (n_seg == 0) return REGNN_OK;
    hipLaunchKernelGGL(gat_softmax_fwd_kernel, dim3(grid_for(n_seg * H, kBlock)), dim3(kBlock), 0,
                       stream, ptr, idx, rel, ee_table, el, er, n_seg, H, slope, a);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

int regnn_gat_softmax_bwd(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                          const float* ee_table, const float* el, const float* er, const float* a,
                          const float* ga, int64_t n_seg, int32_t H, float slope, float* gs_out,
                          float* ger, float* slab, int32_t n_rel, hipStream_t stream) {
    if (!ptr || !idx || !el || !er || !a || !ga || !gs_out || !ger || H <= 0 || n_seg < 0)
        return REGNN_EINVAL;
    if ((ee_table || slab) && !rel) return REGNN_EINVAL;
    if (slab && (n_rel <= 0 || n_rel > 64 || kBlock % H)) return REGNN_EUNSUPPORTED;
    if (n_seg == 0) return REGNN_OK;
    const size_t lds = slab ? size_t(n_rel) * kBlock * sizeof(float) : 0;
    hipLaunchKernelGGL(gat_softmax_bwd_kernel, dim3(grid_for(n_seg * H, kBlock)), dim3(kBlock),
                       lds, stream, ptr, idx, rel, ee_table, el, er, a, ga, n_seg, H, slope,
                       gs_out, ger, slab, n_rel);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

int regnn_spmm_heads_fwd(const int32_t* ptr, const int32_t* idx, const int32_t* perm,
                         const float* a, const void* x, void* y, int64_t n_seg, int32_t H,
                         int32_t D, int32_t dtype, hipStream_t stream) {
    if (!ptr || !idx || !a || !x || !y || n_seg < 0) return REGNN_EINVAL;
    if (n_seg == 0) return REGNN_OK;
    HeadArgs p{ptr, idx, perm, a, x, nullptr, y, nullptr, n_seg, H, D};
    if (dtype == REGNN_F32) return dispatch_heads<float, false>(p, stream);
    if (dtype == REGNN_BF16) return dispatch_heads<bf16_t, false>(p, stream);
    return REGNN_EUNSUPPORTED;
}

int regnn_spmm_heads_bwd(const int32_t* ptr, const int32_t* idx, const int32_t* perm,
                         const float* a, const void* g, const void* x, void* gx, float* ga,
                         int64_t n_seg, int32_t H, int32_t D, int32_t dtype, hipStream_t stream) {
    if (!ptr || !idx || !a || !g || !x || !gx || !ga || n_seg < 0) return REGNN_EINVAL;
    if (n_seg == 0) return REGNN_OK;
    HeadArgs p{ptr, idx, perm, a, g, x, gx, ga, n_seg, H, D};
    if (dtype == REGNN_F32) return dispatch_heads<float, true>(p, stream);
    if (dtype == REGNN_BF16) return dispatch_heads<bf16_t, true>(p, stream);
    return REGNN_EUNSUPPORTED;
}

int regnn_segment_sum(const int32_t* ptr, const int32_t* perm, const float* vals, int64_t n_seg,
                      int32_t H, float* out, hipStream_t stream) {
    if (!ptr || !vals || !out || H <= 0 || n_seg < 0) return REGNN_EINVAL;
    if (n_seg == 0) return REGNN_OK;
    hipLaunchKernelGGL(segment_sum_kernel, dim3(grid_for(n_seg * H, kBlock)), dim3(kBlock), 0,
                       stream, ptr, perm, vals, n_seg, H, out);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

}  // extern "C"
