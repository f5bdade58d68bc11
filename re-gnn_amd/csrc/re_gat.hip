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
gat_softmax_fwd_generic(const int32_t* __restrict__ ptr, const int32_t* __restrict__ idx,
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
gat_softmax_bwd_generic(const int32_t* __restrict__ ptr, const int32_t* __restrict__ idx,
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
    constexpr int UN = NV <= 2 ? 8 : (NV <= 4 ? 4 : 2);   // edge rows in flight per step
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
            // UN edge rows in flight: every row load (and its weight) is issued before use
            for (int k0 = 0; k0 < cnt; k0 += UN) {
                float v[UN][NV][EV];
                float w[UN][NV];
                int ekk[UN];
#pragma unroll
                for (int u = 0; u < UN; ++u) {
                    const int kk = min(k0 + u, cnt - 1);
                    const int jj = __shfl(j, kk, LPR);
                    ekk[u] = __shfl(eid, kk, LPR);
#pragma unroll
                    for (int q = 0; q < NV; ++q) {
                        const int o = (q * LPR + lane) * EV;
                        if (o < F) {
                            Vec<T>::load(src + (int64_t)jj * F + o, v[u][q]);
                            w[u][q] = k0 + u < cnt ? p.a[(int64_t)ekk[u] * p.H + head[q]] : 0.f;
                        } else {
#pragma unroll
                            for (int t = 0; t < EV; ++t) v[u][q][t] = 0.f;
                            w[u][q] = 0.f;
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < UN; ++u) {
#pragma unroll
                    for (int q = 0; q < NV; ++q) {
#pragma unroll
                        for (int t = 0; t < EV; ++t) acc[q][t] = fmaf(w[u][q], v[u][q][t], acc[q][t]);
                        if constexpr (BWD) {
                            const int o = (q * LPR + lane) * EV;
                            float d = 0.f;
#pragma unroll
                            for (int t = 0; t < EV; ++t) d = fmaf(v[u][q][t], sx[q][t], d);
                            for (int m = vph >> 1; m > 0; m >>= 1) d += __shfl_xor(d, m, 64);
                            if (k0 + u < cnt && o < F && (lane & (vph - 1)) == 0)
                                p.ga[(int64_t)ekk[u] * p.H + head[q]] = d;
                        }
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
segment_sum_generic(const int32_t* __restrict__ ptr, const int32_t* __restrict__ perm,
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

// ---- group-per-segment forms (H a power of two <= kGatGroup) --------------------------------
// A group of kGatGroup lanes owns one segment and strides over its (edge, head) pairs flattened
// as p = (k - beg) * H + h, so per-edge H-vectors (a, ga, gs, el rows) are read and written
// coalesced and every lane keeps one head (lane % H). Per-head reductions combine the lanes of
// equal head with xor-shuffles over the bits above log2(H); kGatUn pairs per lane are issued
// before they are used, so a skewed segment costs deg*H / (group * kGatUn) memory round trips
// instead of 3 * deg dependent ones.
constexpr int kGatGroup = 32;
constexpr int kGatUn = 4;

__device__ __forceinline__ void softmax_merge(float& m, float& s, float mo, float so) {
    const float mn = fmaxf(m, mo);
    if (mn == -INFINITY) return;                 // both empty
    s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + (mo == -INFINITY ? 0.f : so * __expf(mo - mn));
    m = mn;
}

__device__ __forceinline__ float gat_score(const int32_t* __restrict__ idx,
                                           const uint8_t* __restrict__ rel,
                                           const float* __restrict__ ee,
                                           const float* __restrict__ el, float erv, int k, int H,
                                           int h, float slope) {
    float s = el[(int64_t)idx[k] * H + h] + erv;
    if (ee) s += ee[rel[k] * H + h];
    return lrelu(s, slope);
}

__global__ void __launch_bounds__(kBlock)
gat_softmax_fwd_group(const int32_t* __restrict__ ptr, const int32_t* __restrict__ idx,
                      const uint8_t* __restrict__ rel, const float* __restrict__ ee,
                      const float* __restrict__ el, const float* __restrict__ er, int64_t n_seg,
                      int H, int lgH, float slope, float* __restrict__ a) {
    constexpr int G = kGatGroup, U = kGatUn;
    const int lane = threadIdx.x & (G - 1), h = lane & (H - 1);
    for (int64_t seg = (int64_t)blockIdx.x * (kBlock / G) + threadIdx.x / G; seg < n_seg;
         seg += (int64_t)gridDim.x * (kBlock / G)) {
        const int beg = ptr[seg], np = (ptr[seg + 1] - beg) << lgH;
        const float erv = er[seg * H + h];
        float m = -INFINITY, sum = 0.f;
        for (int p0 = lane; p0 < np; p0 += G * U) {
            float sc[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int p = p0 + u * G;
                sc[u] = p < np ? gat_score(idx, rel, ee, el, erv, beg + (p >> lgH), H, h, slope)
                               : -INFINITY;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) softmax_merge(m, sum, sc[u], 1.f);
        }
        for (int o = H; o < G; o <<= 1)
            softmax_merge(m, sum, __shfl_xor(m, o, G), __shfl_xor(sum, o, G));
        const float inv = 1.f / sum;
        for (int p0 = lane; p0 < np; p0 += G * U) {
            float sc[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int p = p0 + u * G;
                sc[u] = p < np ? gat_score(idx, rel, ee, el, erv, beg + (p >> lgH), H, h, slope)
                               : 0.f;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int p = p0 + u * G;
                if (p < np) a[(int64_t)beg * H + p] = __expf(sc[u] - m) * inv;
            }
        }
    }
}

__global__ void __launch_bounds__(kBlock)
gat_softmax_bwd_group(const int32_t* __restrict__ ptr, const int32_t* __restrict__ idx,
                      const uint8_t* __restrict__ rel, const float* __restrict__ ee,
                      const float* __restrict__ el, const float* __restrict__ er,
                      const float* __restrict__ a, const float* __restrict__ ga, int64_t n_seg,
                      int H, int lgH, float slope, float* __restrict__ gs_out,
                      float* __restrict__ ger, float* __restrict__ slab, int n_rel) {
    constexpr int G = kGatGroup, U = kGatUn;
    extern __shared__ float bins[];   // [n_rel][kBlock]; a thread only touches its own column
    const int tid = threadIdx.x, lane = tid & (G - 1), h = lane & (H - 1);
    if (slab) for (int r = 0; r < n_rel; ++r) bins[r * kBlock + tid] = 0.f;
    for (int64_t seg = (int64_t)blockIdx.x * (kBlock / G) + tid / G; seg < n_seg;
         seg += (int64_t)gridDim.x * (kBlock / G)) {
        const int beg = ptr[seg], np = (ptr[seg + 1] - beg) << lgH;
        const float* __restrict__ as = a + (int64_t)beg * H;
        const float* __restrict__ gas = ga + (int64_t)beg * H;
        float dot = 0.f;
        for (int p0 = lane; p0 < np; p0 += G * U) {
            float d[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int p = p0 + u * G;
                d[u] = p < np ? as[p] * gas[p] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) dot += d[u];
        }
        for (int o = H; o < G; o <<= 1) dot += __shfl_xor(dot, o, G);
        const float erv = er[seg * H + h];
        float gsum = 0.f;
        for (int p0 = lane; p0 < np; p0 += G * U) {
            float sc[U], av[U], gv[U];
            int r[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int p = p0 + u * G;
                const int pc = p < np ? p : 0;
                const int k = beg + (pc >> lgH);
                float sv = el[(int64_t)idx[k] * H + h] + erv;
                r[u] = rel ? rel[k] : 0;
                if (ee) sv += ee[r[u] * H + h];
                sc[u] = sv;
                av[u] = as[pc];
                gv[u] = gas[pc];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int p = p0 + u * G;
                if (p < np) {
                    const float gz = av[u] * (gv[u] - dot);
                    const float gs = sc[u] > 0.f ? gz : gz * slope;
                    gs_out[(int64_t)beg * H + p] = gs;
                    gsum += gs;
                    if (slab) bins[r[u] * kBlock + tid] += gs;
                }
            }
        }
        for (int o = H; o < G; o <<= 1) gsum += __shfl_xor(gsum, o, G);
        if (lane < H) ger[seg * H + h] = gsum;
    }
    if (slab) {
        // G % H == 0 and kBlock % G == 0, so thread tid always works on head tid % H
        __syncthreads();
        for (int c = tid; c < n_rel * H; c += kBlock) {
            const int r = c / H, hh = c - r * H;
            float s = 0.f;
            for (int t2 = hh; t2 < kBlock; t2 += H) s += bins[r * kBlock + t2];
            slab[(int64_t)blockIdx.x * n_rel * H + c] = s;
        }
    }
}

__global__ void __launch_bounds__(kBlock)
segment_sum_group(const int32_t* __restrict__ ptr, const int32_t* __restrict__ perm,
                  const float* __restrict__ vals, int64_t n_seg, int H, int lgH,
                  float* __restrict__ out) {
    constexpr int G = kGatGroup, U = kGatUn;
    const int lane = threadIdx.x & (G - 1), h = lane & (H - 1);
    for (int64_t seg = (int64_t)blockIdx.x * (kBlock / G) + threadIdx.x / G; seg < n_seg;
         seg += (int64_t)gridDim.x * (kBlock / G)) {
        const int beg = ptr[seg], np = (ptr[seg + 1] - beg) << lgH;
        float acc = 0.f;
        for (int p0 = lane; p0 < np; p0 += G * U) {
            float v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int p = p0 + u * G;
                const int k = beg + ((p < np ? p : 0) >> lgH);
                v[u] = p < np ? vals[(int64_t)(perm ? perm[k] : k) * H + h] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) acc += v[u];
        }
        for (int o = H; o < G; o <<= 1) acc += __shfl_xor(acc, o, G);
        if (lane < H) out[seg * H + h] = acc;
    }
}

inline int gat_log2(int H) {    // log2(H) if H is a power of two <= kGatGroup, else -1
    for (int l = 0; (1 << l) <= kGatGroup; ++l)
        if ((1 << l) == H) return l;
    return -1;
}

// ---- fused score + edge softmax + weighted SpMM (layer/REGATConv.py:80-92) ---------------
// One pass per destination v: for each in-edge u -> v and head h the score
// e = LeakyReLU(el[u,h] + er[v,h] + ee[rel,h]) enters an online softmax (running max m, sum s,
// accumulator rescaled when the max grows) while the same lanes gather x[u,h,:]:
//   out[v,h,:] = sum_e exp(e - m) x[u,h,:] / s,   lse[v,h] = m + log s.
// Every lane of a head carries its own copy of (m, s) (identical: the same scores), so no
// cross-lane reduction is needed; a[e,h] is never written (the backward re-forms it from lse).
// Lanes / vectors as spmm_heads_kernel; edge ids loaded cooperatively, UN rows in flight.
struct GatFusedArgs {
    const int32_t* ptr;
    const int32_t* idx;
    const uint8_t* rel;
    const float* ee;
    const float* el;
    const float* er;
    const void* x;
    void* out;
    float* lse;
    int64_t n_seg;
    int H, D;
    float slope;
};

template <typename T, int LPR, int NV>
__global__ void __launch_bounds__(kBlock) gat_fused_fwd_kernel(GatFusedArgs p) {
    constexpr int EV = Vec<T>::N;
    constexpr int UN = NV <= 2 ? 8 : (NV <= 4 ? 4 : 2);
    constexpr int GPB = kBlock / LPR;
    const int tid = threadIdx.x, lane = tid & (LPR - 1);
    const int F = p.H * p.D;
    const T* __restrict__ src = static_cast<const T*>(p.x);
    for (int64_t seg = (int64_t)blockIdx.x * GPB + tid / LPR; seg < p.n_seg;
         seg += (int64_t)gridDim.x * GPB) {
        const int beg = p.ptr[seg], end = p.ptr[seg + 1];
        float acc[NV][EV] = {};
        float m[NV], s[NV], erv[NV];
        int head[NV];
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            const int o = (q * LPR + lane) * EV;
            head[q] = o < F ? o / p.D : 0;
            erv[q] = p.er[seg * p.H + head[q]];
            m[q] = -INFINITY;
            s[q] = 0.f;
        }
        for (int e0 = beg; e0 < end; e0 += LPR) {
            const int e = e0 + lane;
            int j = 0, r = 0;
            if (e < end) {
                j = p.idx[e];
                r = p.ee ? int(p.rel[e]) : 0;
            }
            const int cnt = min(LPR, end - e0);
            for (int k0 = 0; k0 < cnt; k0 += UN) {
                float v[UN][NV][EV];
                float sc[UN][NV];
#pragma unroll
                for (int u = 0; u < UN; ++u) {
                    const int kk = min(k0 + u, cnt - 1);
                    const int jj = __shfl(j, kk, LPR);
                    const int rr = __shfl(r, kk, LPR);
#pragma unroll
                    for (int q = 0; q < NV; ++q) {
                        const int o = (q * LPR + lane) * EV;
                        if (o < F) {
                            Vec<T>::load(src + (int64_t)jj * F + o, v[u][q]);
                            float z = p.el[(int64_t)jj * p.H + head[q]] + erv[q];
                            if (p.ee) z += p.ee[rr * p.H + head[q]];
                            sc[u][q] = lrelu(z, p.slope);
                        } else {
#pragma unroll
                            for (int t = 0; t < EV; ++t) v[u][q][t] = 0.f;
                            sc[u][q] = 0.f;
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < UN; ++u) {
                    if (k0 + u >= cnt) break;
#pragma unroll
                    for (int q = 0; q < NV; ++q) {
                        const float d = sc[u][q] - m[q];
                        const bool grow = d > 0.f;                   // new running max
                        const float ex = __expf(grow ? -d : d);
                        const float sa = grow ? ex : 1.f, sv = grow ? 1.f : ex;
#pragma unroll
                        for (int t = 0; t < EV; ++t) acc[q][t] = fmaf(acc[q][t], sa, sv * v[u][q][t]);
                        s[q] = fmaf(s[q], sa, sv);
                        m[q] = grow ? sc[u][q] : m[q];
                    }
                }
            }
        }
        T* __restrict__ out = static_cast<T*>(p.out) + seg * F;
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            const int o = (q * LPR + lane) * EV;
            if (o < F) {
                const float inv = s[q] > 0.f ? 1.f / s[q] : 0.f;
                float w[EV];
#pragma unroll
                for (int t = 0; t < EV; ++t) w[t] = acc[q][t] * inv;
                Vec<T>::store(out + o, w);
                if (o % p.D == 0)
                    p.lse[seg * p.H + head[q]] = s[q] > 0.f ? m[q] + __logf(s[q]) : -INFINITY;
            }
        }
    }
}

// a[e,h] = exp(LeakyReLU(el[u,h] + er[v,h] + ee[rel,h]) - lse[v,h]) in CSR edge order (the
// attention the fused forward did not store; its backward needs it). Group layout of
// gat_softmax_fwd_group: (edge, head) pairs flattened per segment, coalesced H-vectors.
__global__ void __launch_bounds__(kBlock)
gat_attn_lse_group(const int32_t* __restrict__ ptr, const int32_t* __restrict__ idx,
                   const uint8_t* __restrict__ rel, const float* __restrict__ ee,
                   const float* __restrict__ el, const float* __restrict__ er,
                   const float* __restrict__ lse, int64_t n_seg, int H, int lgH, float slope,
                   float* __restrict__ a) {
    constexpr int G = kGatGroup, U = kGatUn;
    const int lane = threadIdx.x & (G - 1), h = lane & (H - 1);
    for (int64_t seg = (int64_t)blockIdx.x * (kBlock / G) + threadIdx.x / G; seg < n_seg;
         seg += (int64_t)gridDim.x * (kBlock / G)) {
        const int beg = ptr[seg], np = (ptr[seg + 1] - beg) << lgH;
        const float erv = er[seg * H + h], l = lse[seg * H + h];
        for (int p0 = lane; p0 < np; p0 += G * U) {
            float sc[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int q = p0 + u * G;
                sc[u] = q < np ? gat_score(idx, rel, ee, el, erv, beg + (q >> lgH), H, h, slope)
                               : 0.f;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int q = p0 + u * G;
                if (q < np) a[(int64_t)beg * H + q] = __expf(sc[u] - l);
            }
        }
    }
}

template <typename T>
int dispatch_gat_fused(GatFusedArgs p, hipStream_t stream) {
    constexpr int EV = Vec<T>::N;
    const int F = p.H * p.D;
    if (p.D <= 0 || p.D % EV || p.H <= 0) return REGNN_EUNSUPPORTED;
    const int nvec = F / EV;
#define REGNN_GATF(LPR, NV)                                                                   \
    if (nvec <= (LPR) * (NV)) {                                                               \
        hipLaunchKernelGGL((gat_fused_fwd_kernel<T, LPR, NV>),                                \
                           dim3(grid_for(p.n_seg, kBlock / (LPR))), dim3(kBlock), 0, stream, p); \
        REGNN_LAUNCH_CHECK();                                                                 \
        return REGNN_OK;                                                                      \
    }
    REGNN_GATF(16, 1)
    REGNN_GATF(16, 2)
    REGNN_GATF(16, 4)
    REGNN_GATF(64, 2)
    REGNN_GATF(64, 4)
    REGNN_GATF(64, 8)
#undef REGNN_GATF
    return REGNN_EUNSUPPORTED;
}

// ---- attention logits el / er (layer/REGATConv.py:68-69) ------------------------------------
// el[n,h] = <ft[n,h,:], attn_l[h,:]>, er likewise: a group of 16 lanes per (node, head) reads the
// D-vector coalesced and reduces with xor-shuffles; both dots share the one read of ft.
constexpr int kDotGroup = 16;

__global__ void __launch_bounds__(kBlock)
attn_dots_fwd_kernel(const float* __restrict__ ft, const float* __restrict__ al,
                     const float* __restrict__ ar, int64_t N, int H, int D,
                     float* __restrict__ el, float* __restrict__ er) {
    constexpr int G = kDotGroup;
    const int lane = threadIdx.x & (G - 1);
    const int64_t total = N * H;
    for (int64_t t = (int64_t)blockIdx.x * (kBlock / G) + threadIdx.x / G; t < total;
         t += (int64_t)gridDim.x * (kBlock / G)) {
        const int h = int(t % H);
        const float* __restrict__ x = ft + t * D;
        float sl = 0.f, sr = 0.f;
        for (int d = lane; d < D; d += G) {
            const float v = x[d];
            sl = fmaf(v, al[h * D + d], sl);
            sr = fmaf(v, ar[h * D + d], sr);
        }
#pragma unroll
        for (int o = G / 2; o > 0; o >>= 1) {
            sl += __shfl_xor(sl, o, G);
            sr += __shfl_xor(sr, o, G);
        }
        if (lane == 0) {
            el[t] = sl;
            er[t] = sr;
        }
    }
}

// d ft[n,c] = gel[n,h] al[c] + ger[n,h] ar[c]  (c = h*D + d), and per-block partials of
// d al[c] = sum_n gel[n,h] ft[n,c] (d ar likewise) into slab row blockIdx.x: [F | F] floats.
// Block b owns rows [b*rpb, (b+1)*rpb); every launched block writes its slab row.
__global__ void __launch_bounds__(kBlock)
attn_dots_bwd_kernel(const float* __restrict__ ft, const float* __restrict__ al,
                     const float* __restrict__ ar, const float* __restrict__ gel,
                     const float* __restrict__ ger, int64_t N, int H, int D, int64_t rpb,
                     float* __restrict__ gft, float* __restrict__ slab) {
    const int F = H * D;
    const int64_t r0 = (int64_t)blockIdx.x * rpb;
    const int64_t r1 = min(N, r0 + rpb);
    for (int c = threadIdx.x; c < F; c += kBlock) {
        const int h = c / D;
        const float a_l = al[c], a_r = ar[c];
        float sl = 0.f, sr = 0.f;
        for (int64_t n = r0; n < r1; ++n) {
            const float gl = gel[n * H + h], gr = ger[n * H + h];
            const float x = ft[n * F + c];
            gft[n * F + c] = fmaf(gl, a_l, gr * a_r);
            sl = fmaf(gl, x, sl);
            sr = fmaf(gr, x, sr);
        }
        slab[(int64_t)blockIdx.x * 2 * F + c] = sl;
        slab[(int64_t)blockIdx.x * 2 * F + F + c] = sr;
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
    const int lg = gat_log2(H);
    if (lg >= 0)
        hipLaunchKernelGGL(gat_softmax_fwd_group, dim3(grid_for(n_seg, kBlock / kGatGroup)),
                           dim3(kBlock), 0, stream, ptr, idx, rel, ee_table, el, er, n_seg, H, lg,
                           slope, a);
    else
        hipLaunchKernelGGL(gat_softmax_fwd_generic, dim3(grid_for(n_seg * H, kBlock)),
                           dim3(kBlock), 0, stream, ptr, idx, rel, ee_table, el, er, n_seg, H,
                           slope, a);
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
    const int lg = gat_log2(H);
    if (lg >= 0)
        hipLaunchKernelGGL(gat_softmax_bwd_group, dim3(grid_for(n_seg, kBlock / kGatGroup)),
                           dim3(kBlock), lds, stream, ptr, idx, rel, ee_table, el, er, a, ga,
                           n_seg, H, lg, slope, gs_out, ger, slab, n_rel);
    else
        hipLaunchKernelGGL(gat_softmax_bwd_generic, dim3(grid_for(n_seg * H, kBlock)),
                           dim3(kBlock), lds, stream, ptr, idx, rel, ee_table, el, er, a, ga,
                           n_seg, H, slope, gs_out, ger, slab, n_rel);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

int regnn_gat_fused_fwd(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                        const float* ee_table, const float* el, const float* er, const void* x,
                        void* out, float* lse, int64_t n_seg, int32_t H, int32_t D, float slope,
                        int32_t dtype, hipStream_t stream) {
    if (!ptr || !idx || !el || !er || !x || !out || !lse || n_seg < 0 || (ee_table && !rel))
        return REGNN_EINVAL;
    if (n_seg == 0) return REGNN_OK;
    GatFusedArgs p{ptr, idx, rel, ee_table, el, er, x, out, lse, n_seg, H, D, slope};
    if (dtype == REGNN_F32) return dispatch_gat_fused<float>(p, stream);
    if (dtype == REGNN_BF16) return dispatch_gat_fused<bf16_t>(p, stream);
    return REGNN_EUNSUPPORTED;
}

int regnn_gat_attn_lse(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                       const float* ee_table, const float* el, const float* er, const float* lse,
                       int64_t n_seg, int32_t H, float slope, float* a, hipStream_t stream) {
    if (!ptr || !idx || !el || !er || !lse || !a || H <= 0 || n_seg < 0 || (ee_table && !rel))
        return REGNN_EINVAL;
    if (n_seg == 0) return REGNN_OK;
    const int lg = gat_log2(H);
    if (lg < 0) return REGNN_EUNSUPPORTED;
    hipLaunchKernelGGL(gat_attn_lse_group, dim3(grid_for(n_seg, kBlock / kGatGroup)), dim3(kBlock),
                       0, stream, ptr, idx, rel, ee_table, el, er, lse, n_seg, H, lg, slope, a);
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
    const int lg = gat_log2(H);
    if (lg >= 0)
        hipLaunchKernelGGL(segment_sum_group, dim3(grid_for(n_seg, kBlock / kGatGroup)),
                           dim3(kBlock), 0, stream, ptr, perm, vals, n_seg, H, lg, out);
    else
        hipLaunchKernelGGL(segment_sum_generic, dim3(grid_for(n_seg * H, kBlock)), dim3(kBlock),
                           0, stream, ptr, perm, vals, n_seg, H, out);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

int regnn_attn_dots_fwd(const float* ft, const float* attn_l, const float* attn_r, int64_t N,
                        int32_t H, int32_t D, float* el, float* er, hipStream_t stream) {
    if (!ft || !attn_l || !attn_r || !el || !er || N < 0 || H <= 0 || D <= 0) return REGNN_EINVAL;
    if (N == 0) return REGNN_OK;
    hipLaunchKernelGGL(attn_dots_fwd_kernel, dim3(grid_for(N * H, kBlock / kDotGroup)),
                       dim3(kBlock), 0, stream, ft, attn_l, attn_r, N, H, D, el, er);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

int regnn_attn_dots_bwd(const float* ft, const float* attn_l, const float* attn_r,
                        const float* gel, const float* ger, int64_t N, int32_t H, int32_t D,
                        float* gft, float* slab, int32_t slab_rows, hipStream_t stream) {
    if (!ft || !attn_l || !attn_r || !gel || !ger || !gft || !slab || N < 0 || H <= 0 ||
        D <= 0 || slab_rows <= 0)
        return REGNN_EINVAL;
    const int64_t rpb = N > 0 ? (N + slab_rows - 1) / slab_rows : 1;
    hipLaunchKernelGGL(attn_dots_bwd_kernel, dim3(slab_rows), dim3(kBlock), 0, stream, ft,
                       attn_l, attn_r, gel, ger, N, H, D, rpb, gft, slab);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

}  // extern "C"
