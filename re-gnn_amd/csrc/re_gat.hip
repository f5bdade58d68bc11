// GAT relation-embedding attention for gfx950 (layer/REGATConv.py:64-100):
//  * edge softmax over the in-edges of each destination with the u_add_v SDDMM, the relation
//    bias table and the LeakyReLU fused (one thread per (destination, head));
//  * per-head weighted SpMM (a group of lanes per destination, 16-byte row vectors; the lane's
//    head is fixed by its feature offset), and its fused transposed backward that also forms the
//    per-(edge, head) dot <g[v,h,:], x[u,h,:]> with an in-register head reduction;
//  * the softmax / LeakyReLU / u_add_v backward with deterministic relation-bias slabs.
#include "regnn_common.h"
#include "re_segplan.h"

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

// CH: the units are the chunks of long segments (fp32 partial rows of the sums); otherwise the
// segments, long ones skipped. The per-edge ga of the backward is written either way.
template <typename T, int LPR, int NV, bool BWD, bool CH>
__global__ void __launch_bounds__(kBlock) spmm_heads_kernel(HeadArgs p, LongPlan P) {
    constexpr int EV = Vec<T>::N;
#ifdef REGNN_HEADS_UN
    constexpr int UN = NV <= 2 ? REGNN_HEADS_UN : (NV <= 4 ? 4 : 2);
#else
    constexpr int UN = NV <= 2 ? 8 : (NV <= 4 ? 4 : 2);   // edge rows in flight per step
#endif
    constexpr int GPB = kBlock / LPR;
    const int tid = threadIdx.x, lane = tid & (LPR - 1);
    const int F = p.H * p.D;
    const int vph = p.D / EV;   // vectors per head (power of two, <= LPR)
    const T* __restrict__ src = static_cast<const T*>(p.src);
    const int64_t n_units = CH ? P.n_chunk : p.n_seg;
    for (int64_t unit = (int64_t)blockIdx.x * GPB + tid / LPR; unit < n_units;
         unit += (int64_t)gridDim.x * GPB) {
        int64_t seg;
        int beg, end;
        if (CH) {
            chunk_range(P, p.ptr, unit, seg, beg, end);
        } else {
            seg = unit;
            beg = p.ptr[seg];
            end = p.ptr[seg + 1];
            if (end - beg > P.split) continue;
        }
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
        if (CH) {
            float* __restrict__ pr = P.part + unit * F;
#pragma unroll
            for (int q = 0; q < NV; ++q) {
                const int o = (q * LPR + lane) * EV;
                if (o < F)
#pragma unroll
                    for (int t = 0; t < EV; ++t) pr[o + t] = acc[q][t];
            }
            continue;
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
int dispatch_heads(HeadArgs p, const regnn_seg_plan* pl, hipStream_t stream) {
    constexpr int EV = Vec<T>::N;
    const int F = p.H * p.D;
    if (p.D <= 0 || p.D % EV || p.H <= 0) return REGNN_EUNSUPPORTED;
    const int vph = p.D / EV;
    if (vph & (vph - 1)) return REGNN_EUNSUPPORTED;
    const int nvec = F / EV;
    const LongPlan P = long_plan(pl);
#define REGNN_HEADS(LPR, NV)                                                                    \
    if (nvec <= (LPR) * (NV) && vph <= (LPR)) {                                                 \
        hipLaunchKernelGGL((spmm_heads_kernel<T, LPR, NV, BWD, false>),                         \
                           dim3(grid_for(p.n_seg, kBlock / (LPR))), dim3(kBlock), 0, stream, p, P); \
        REGNN_LAUNCH_CHECK();                                                                   \
        if (P.n_chunk > 0) {                                                                    \
            hipLaunchKernelGGL((spmm_heads_kernel<T, LPR, NV, BWD, true>),                      \
                               dim3(grid_for(P.n_chunk, kBlock / (LPR))), dim3(kBlock), 0, stream, \
                               p, P);                                                           \
            const int64_t base = run_tree(pl, 0, F, F, p.H, p.D, stream);                       \
            hipLaunchKernelGGL(seg_emit_sum<T>, dim3(long_grid(P.n_long)), dim3(kBlock), 0,     \
                               stream, P.part, P.chunk_off, base, pl->n_levels, P.long_ids,     \
                               P.n_long, F, static_cast<T*>(p.out));                            \
            REGNN_LAUNCH_CHECK();                                                               \
        }                                                                                       \
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

// MODE 0: segments (long ones skipped); MODE 1: chunks -> partial rows [max H | sum H];
// MODE 2: chunks, attention from the combined (max, sum) of their segment (rows fin + 2H l)
template <int MODE>
__global__ void __launch_bounds__(kBlock)
gat_softmax_fwd_group(const int32_t* __restrict__ ptr, const int32_t* __restrict__ idx,
                      const uint8_t* __restrict__ rel, const float* __restrict__ ee,
                      const float* __restrict__ el, const float* __restrict__ er, int64_t n_seg,
                      int H, int lgH, float slope, float* __restrict__ a, LongPlan P,
                      const float* __restrict__ fin) {
    constexpr int G = kGatGroup, U = kGatUn;
    constexpr bool CH = MODE > 0;
    const int lane = threadIdx.x & (G - 1), h = lane & (H - 1);
    const int64_t n_units = CH ? P.n_chunk : n_seg;
    for (int64_t unit = (int64_t)blockIdx.x * (kBlock / G) + threadIdx.x / G; unit < n_units;
         unit += (int64_t)gridDim.x * (kBlock / G)) {
        int64_t seg;
        int beg, ne, l;
        if (!group_unit<CH>(P, ptr, unit, seg, beg, ne, l)) continue;
        const int np = ne << lgH;
        const float erv = er[seg * H + h];
        float m = -INFINITY, sum = 0.f;
        if (MODE != 2) {
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
            if (MODE == 1) {
                if (lane < H) {
                    P.part[unit * 2 * H + h] = m;
                    P.part[unit * 2 * H + H + h] = sum;
                }
                continue;
            }
        } else {
            m = fin[int64_t(l) * 2 * H + h];
            sum = fin[int64_t(l) * 2 * H + H + h];
        }
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

// MODE 0: segments (long ones skipped); MODE 1: chunks -> partial dots sum a*ga [H];
// MODE 2: chunks with their segment's combined dot (rows fin + H l) -> gs, partial gsum [H]
template <int MODE>
__global__ void __launch_bounds__(kBlock)
gat_softmax_bwd_group(const int32_t* __restrict__ ptr, const int32_t* __restrict__ idx,
                      const uint8_t* __restrict__ rel, const float* __restrict__ ee,
                      const float* __restrict__ el, const float* __restrict__ er,
                      const float* __restrict__ a, const float* __restrict__ ga, int64_t n_seg,
                      int H, int lgH, float slope, float* __restrict__ gs_out,
                      float* __restrict__ ger, float* __restrict__ slab, int n_rel, LongPlan P,
                      const float* __restrict__ fin) {
    constexpr int G = kGatGroup, U = kGatUn;
    constexpr bool CH = MODE > 0;
    extern __shared__ float bins[];   // [n_rel][kBlock]; a thread only touches its own column
    const int tid = threadIdx.x, lane = tid & (G - 1), h = lane & (H - 1);
    const bool do_bins = slab && MODE != 1;
    if (do_bins) for (int r = 0; r < n_rel; ++r) bins[r * kBlock + tid] = 0.f;
    const int64_t n_units = CH ? P.n_chunk : n_seg;
    for (int64_t unit = (int64_t)blockIdx.x * (kBlock / G) + tid / G; unit < n_units;
         unit += (int64_t)gridDim.x * (kBlock / G)) {
        int64_t seg;
        int beg, ne, l;
        if (!group_unit<CH>(P, ptr, unit, seg, beg, ne, l)) continue;
        const int np = ne << lgH;
        const float* __restrict__ as = a + (int64_t)beg * H;
        const float* __restrict__ gas = ga + (int64_t)beg * H;
        float dot = 0.f;
        if (MODE != 2) {
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
            if (MODE == 1) {
                if (lane < H) P.part[unit * H + h] = dot;
                continue;
            }
        } else {
            dot = fin[int64_t(l) * H + h];
        }
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
                    if (do_bins) bins[r[u] * kBlock + tid] += gs;
                }
            }
        }
        for (int o = H; o < G; o <<= 1) gsum += __shfl_xor(gsum, o, G);
        if (lane < H) {
            if (CH) P.part[unit * H + h] = gsum;
            else ger[seg * H + h] = gsum;
        }
    }
    if (do_bins) {
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

template <bool CH>
__global__ void __launch_bounds__(kBlock)
segment_sum_group(const int32_t* __restrict__ ptr, const int32_t* __restrict__ perm,
                  const float* __restrict__ vals, int64_t n_seg, int H, int lgH,
                  float* __restrict__ out, LongPlan P) {
    constexpr int G = kGatGroup, U = kGatUn;
    const int lane = threadIdx.x & (G - 1), h = lane & (H - 1);
    const int64_t n_units = CH ? P.n_chunk : n_seg;
    for (int64_t unit = (int64_t)blockIdx.x * (kBlock / G) + threadIdx.x / G; unit < n_units;
         unit += (int64_t)gridDim.x * (kBlock / G)) {
        int64_t seg;
        int beg, ne, l;
        if (!group_unit<CH>(P, ptr, unit, seg, beg, ne, l)) continue;
        const int np = ne << lgH;
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
        if (lane < H) {
            if (CH) P.part[unit * H + h] = acc;
            else out[seg * H + h] = acc;
        }
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
    const float* al;    // attn_l [H, D] (ELX kernels: el re-formed from the gathered row)
    int64_t n_seg;
    int H, D;
    float slope;
};

// el[u,h] as attn_dots_fwd_vec forms it: lane l of the head's D/4 lanes takes x[u,h,4l..4l+3]
// (an fmaf chain from 0), then an xor butterfly over the D/4 lanes (every lane ends with the same
// sum). The ELX forward forms it from the row it already holds, so each edge makes one random
// access (the row) instead of two (the row and el[u], 32 B of another array): bitwise the el the
// backward re-forms the attention from.
__device__ __forceinline__ float head_dot4(const float (&v)[4], const float (&a)[4], int dl) {
    float d = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) d = fmaf(v[t], a[t], d);
    for (int o = dl >> 1; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
    return d;
}

// attn_dots_fwd in the order head_dot4 uses: D % 4 == 0 and D / 4 a power of two <= 64
inline bool attn_dots_vec_ok(int D) {
    const int dl = D / 4;
    return D > 0 && D % 4 == 0 && dl <= 64 && (dl & (dl - 1)) == 0;
}

// CH: the units are the chunks of long segments (partial rows [acc | max | sum], unnormalised);
// otherwise the segments, long ones skipped.
template <typename T, int LPR, int NV, bool CH, bool ELX>
__global__ void __launch_bounds__(kBlock) gat_fused_fwd_kernel(GatFusedArgs p, LongPlan P) {
    constexpr int EV = Vec<T>::N;
    static_assert(!ELX || EV == 4, "ELX: fp32 rows");
#ifdef REGNN_GATF_UN
    constexpr int UN = NV <= 2 ? REGNN_GATF_UN : (NV <= 4 ? 4 : 2);
#else
    constexpr int UN = NV <= 4 ? 4 : 2;    // 8 rows for NV <= 2: 25.5 / 18.2 ms against 24.7 / 17.2
#endif
    constexpr int GPB = kBlock / LPR;
    const int tid = threadIdx.x, lane = tid & (LPR - 1);
    const int F = p.H * p.D;
    const T* __restrict__ src = static_cast<const T*>(p.x);
    const int64_t n_units = CH ? P.n_chunk : p.n_seg;
    for (int64_t unit = (int64_t)blockIdx.x * GPB + tid / LPR; unit < n_units;
         unit += (int64_t)gridDim.x * GPB) {
        int64_t seg;
        int beg, end;
        if (CH) {
            chunk_range(P, p.ptr, unit, seg, beg, end);
        } else {
            seg = unit;
            beg = p.ptr[seg];
            end = p.ptr[seg + 1];
            if (end - beg > P.split) continue;         // a long segment: its chunks
        }
        float acc[NV][EV] = {};
        float m[NV], s[NV], erv[NV];
        float alv[ELX ? NV : 1][4];
        int head[NV];
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            const int o = (q * LPR + lane) * EV;
            head[q] = o < F ? o / p.D : 0;
            erv[q] = p.er[seg * p.H + head[q]];
            m[q] = -INFINITY;
            s[q] = 0.f;
            if constexpr (ELX) {
#pragma unroll
                for (int t = 0; t < 4; ++t) alv[q][t] = o < F ? p.al[o + t] : 0.f;
            }
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
                            if constexpr (ELX) {       // the relation bias; el once the row is in
                                sc[u][q] = p.ee ? p.ee[rr * p.H + head[q]] : 0.f;
                            } else {
                                float z = p.el[(int64_t)jj * p.H + head[q]] + erv[q];
                                if (p.ee) z += p.ee[rr * p.H + head[q]];
                                sc[u][q] = lrelu(z, p.slope);
                            }
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
                    if constexpr (ELX) {
#pragma unroll
                        for (int q = 0; q < NV; ++q) {
                            float z = head_dot4(v[u][q], alv[q], p.D >> 2) + erv[q];
                            if (p.ee) z += sc[u][q];
                            sc[u][q] = lrelu(z, p.slope);
                        }
                    }
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
        if (CH) {
            float* __restrict__ pr = P.part + unit * (F + 2 * p.H);
#pragma unroll
            for (int q = 0; q < NV; ++q) {
                const int o = (q * LPR + lane) * EV;
                if (o < F) {
#pragma unroll
                    for (int t = 0; t < EV; ++t) pr[o + t] = acc[q][t];
                    if (o % p.D == 0) {
                        pr[F + head[q]] = m[q];
                        pr[F + p.H + head[q]] = s[q];
                    }
                }
            }
            continue;
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
template <bool CH>
__global__ void __launch_bounds__(kBlock)
gat_attn_lse_group(const int32_t* __restrict__ ptr, const int32_t* __restrict__ idx,
                   const uint8_t* __restrict__ rel, const float* __restrict__ ee,
                   const float* __restrict__ el, const float* __restrict__ er,
                   const float* __restrict__ lse, int64_t n_seg, int H, int lgH, float slope,
                   float* __restrict__ a, LongPlan P) {
    constexpr int G = kGatGroup, U = kGatUn;
    const int lane = threadIdx.x & (G - 1), h = lane & (H - 1);
    const int64_t n_units = CH ? P.n_chunk : n_seg;
    for (int64_t unit = (int64_t)blockIdx.x * (kBlock / G) + threadIdx.x / G; unit < n_units;
         unit += (int64_t)gridDim.x * (kBlock / G)) {
        int64_t seg;
        int beg, ne, lg_;
        if (!group_unit<CH>(P, ptr, unit, seg, beg, ne, lg_)) continue;
        const int np = ne << lgH;
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
int dispatch_gat_fused(GatFusedArgs p, const regnn_seg_plan* pl, hipStream_t stream) {
    constexpr int EV = Vec<T>::N;
    const int F = p.H * p.D;
    if (p.D <= 0 || p.D % EV || p.H <= 0) return REGNN_EUNSUPPORTED;
    const int nvec = F / EV;
    const LongPlan P = long_plan(pl);
#ifdef REGNN_GATF_NO_ELX
    p.al = nullptr;
#endif
#define REGNN_GATF(LPR, NV)                                                                   \
    if (nvec <= (LPR) * (NV)) {                                                               \
        const bool elx = std::is_same<T, float>::value && p.al && attn_dots_vec_ok(p.D) &&    \
                         p.D / 4 <= (LPR);                                                    \
        if (elx)                                                                              \
            hipLaunchKernelGGL((gat_fused_fwd_kernel<T, LPR, NV, false, EV == 4>),            \
                               dim3(grid_for(p.n_seg, kBlock / (LPR))), dim3(kBlock), 0, stream, \
                               p, P);                                                         \
        else                                                                                  \
            hipLaunchKernelGGL((gat_fused_fwd_kernel<T, LPR, NV, false, false>),              \
                               dim3(grid_for(p.n_seg, kBlock / (LPR))), dim3(kBlock), 0, stream, \
                               p, P);                                                         \
        REGNN_LAUNCH_CHECK();                                                                 \
        if (P.n_chunk > 0) {                                                                  \
            if (elx)                                                                          \
                hipLaunchKernelGGL((gat_fused_fwd_kernel<T, LPR, NV, true, EV == 4>),         \
                                   dim3(grid_for(P.n_chunk, kBlock / (LPR))), dim3(kBlock), 0, \
                                   stream, p, P);                                             \
            else                                                                              \
                hipLaunchKernelGGL((gat_fused_fwd_kernel<T, LPR, NV, true, false>),           \
                                   dim3(grid_for(P.n_chunk, kBlock / (LPR))), dim3(kBlock), 0, \
                                   stream, p, P);                                             \
            const int64_t base = run_tree(pl, 1, F + 2 * p.H, F, p.H, p.D, stream);           \
            hipLaunchKernelGGL(seg_emit_softmax<T>, dim3(long_grid(P.n_long)), dim3(kBlock),  \
                               0, stream, P.part, P.chunk_off, base, pl->n_levels, P.long_ids, \
                               P.n_long, F, p.H, p.D, static_cast<T*>(p.out), p.lse);         \
            REGNN_LAUNCH_CHECK();                                                             \
        }                                                                                     \
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

// The same dots in head_dot4's order (D % 4 == 0, D / 4 a power of two <= 64): D / 4 lanes per
// (node, head), lane l the fmaf chain over d = 4l..4l+3, then the xor butterfly. The fused GAT
// forward re-forms el from its gathered rows in exactly this order.
__global__ void __launch_bounds__(kBlock)
attn_dots_fwd_vec_kernel(const float* __restrict__ ft, const float* __restrict__ al,
                         const float* __restrict__ ar, int64_t N, int H, int D,
                         float* __restrict__ el, float* __restrict__ er) {
    const int dl = D >> 2;
    const int lane = threadIdx.x & (dl - 1);
    const int64_t total = N * H, per_block = kBlock / dl;
    for (int64_t t = (int64_t)blockIdx.x * per_block + threadIdx.x / dl; t < total;
         t += (int64_t)gridDim.x * per_block) {
        const int h = int(t % H);
        const float* __restrict__ x = ft + t * D + 4 * lane;
        float v[4], a[4], b[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            v[i] = x[i];
            a[i] = al[h * D + 4 * lane + i];
            b[i] = ar[h * D + 4 * lane + i];
        }
        const float sl = head_dot4(v, a, dl), sr = head_dot4(v, b, dl);
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

// The same backward for rows whose F / 4 float4 columns divide the block (D % 4 == 0, so a float4
// lies inside one head): thread = (row group g, float4 column cv); the block's RG = 256 / CPL row
// groups stride over its rows, each thread keeping UN rows' ft loads in flight; gel / ger are read
// once per (row, head) by the lanes of that head (broadcast within the wave). The row-group partial
// sums are combined in LDS in a fixed order, one slab row per block.
template <int UN>
__global__ void __launch_bounds__(kBlock)
attn_dots_bwd_vec_kernel(const float4* __restrict__ ft, const float4* __restrict__ al,
                         const float4* __restrict__ ar, const float* __restrict__ gel,
                         const float* __restrict__ ger, int64_t N, int H, int D, int CPL,
                         int64_t rpb, float4* __restrict__ gft, float* __restrict__ slab) {
    extern __shared__ float4 part[];       // [RG][2 CPL]
    const int RG = kBlock / CPL;
    const int g = threadIdx.x / CPL, cv = threadIdx.x - g * CPL;
    const int h = (4 * cv) / D;
    const int64_t r0 = (int64_t)blockIdx.x * rpb;
    const int64_t r1 = min(N, r0 + rpb);
    const float4 a_l = al[cv], a_r = ar[cv];
    float4 sl = make_float4(0.f, 0.f, 0.f, 0.f), sr = sl;
    int64_t n = r0 + g;
    for (; n + (UN - 1) * RG < r1; n += UN * RG) {
        float4 x[UN];
        float gl[UN], gr[UN];
#pragma unroll
        for (int u = 0; u < UN; ++u) {
            const int64_t m = n + (int64_t)u * RG;
            x[u] = ft[m * CPL + cv];
            gl[u] = gel[m * H + h];
            gr[u] = ger[m * H + h];
        }
#pragma unroll
        for (int u = 0; u < UN; ++u) {
            const int64_t m = n + (int64_t)u * RG;
            float4 o;
            o.x = fmaf(gl[u], a_l.x, gr[u] * a_r.x);
            o.y = fmaf(gl[u], a_l.y, gr[u] * a_r.y);
            o.z = fmaf(gl[u], a_l.z, gr[u] * a_r.z);
            o.w = fmaf(gl[u], a_l.w, gr[u] * a_r.w);
            gft[m * CPL + cv] = o;
            sl.x = fmaf(gl[u], x[u].x, sl.x); sl.y = fmaf(gl[u], x[u].y, sl.y);
            sl.z = fmaf(gl[u], x[u].z, sl.z); sl.w = fmaf(gl[u], x[u].w, sl.w);
            sr.x = fmaf(gr[u], x[u].x, sr.x); sr.y = fmaf(gr[u], x[u].y, sr.y);
            sr.z = fmaf(gr[u], x[u].z, sr.z); sr.w = fmaf(gr[u], x[u].w, sr.w);
        }
    }
    for (; n < r1; n += RG) {
        const float4 x = ft[n * CPL + cv];
        const float gl = gel[n * H + h], gr = ger[n * H + h];
        float4 o;
        o.x = fmaf(gl, a_l.x, gr * a_r.x);
        o.y = fmaf(gl, a_l.y, gr * a_r.y);
        o.z = fmaf(gl, a_l.z, gr * a_r.z);
        o.w = fmaf(gl, a_l.w, gr * a_r.w);
        gft[n * CPL + cv] = o;
        sl.x = fmaf(gl, x.x, sl.x); sl.y = fmaf(gl, x.y, sl.y);
        sl.z = fmaf(gl, x.z, sl.z); sl.w = fmaf(gl, x.w, sl.w);
        sr.x = fmaf(gr, x.x, sr.x); sr.y = fmaf(gr, x.y, sr.y);
        sr.z = fmaf(gr, x.z, sr.z); sr.w = fmaf(gr, x.w, sr.w);
    }
    part[g * 2 * CPL + cv] = sl;
    part[g * 2 * CPL + CPL + cv] = sr;
    __syncthreads();
    for (int i = threadIdx.x; i < 2 * CPL; i += kBlock) {
        float4 s = part[i];
        for (int k = 1; k < RG; ++k) {
            const float4 p = part[k * 2 * CPL + i];
            s.x += p.x; s.y += p.y; s.z += p.z; s.w += p.w;
        }
        reinterpret_cast<float4*>(slab + (int64_t)blockIdx.x * 8 * CPL)[i] = s;
    }
}

}  // namespace regnn

using namespace regnn;

extern "C" {

int regnn_gat_softmax_fwd(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                          const float* ee_table, const float* el, const float* er, int64_t n_seg,
                          int32_t H, float slope, float* a, const regnn_seg_plan* plan,
                          hipStream_t stream) {
    if (!ptr || !idx || !el || !er || !a || H <= 0 || n_seg < 0 || (ee_table && !rel))
        return REGNN_EINVAL;
    if (n_seg == 0) return REGNN_OK;
    const int lg = gat_log2(H);
    if (lg < 0) {
        hipLaunchKernelGGL(gat_softmax_fwd_generic, dim3(grid_for(n_seg * H, kBlock)),
                           dim3(kBlock), 0, stream, ptr, idx, rel, ee_table, el, er, n_seg, H,
                           slope, a);
        REGNN_LAUNCH_CHECK();
        return REGNN_OK;
    }
    if (const int rc = check_plan(plan, 2 * H)) return rc;
    const LongPlan P = long_plan(plan);
    hipLaunchKernelGGL(gat_softmax_fwd_group<0>, dim3(grid_for(n_seg, kBlock / kGatGroup)),
                       dim3(kBlock), 0, stream, ptr, idx, rel, ee_table, el, er, n_seg, H, lg,
                       slope, a, P, nullptr);
    REGNN_LAUNCH_CHECK();
    if (P.n_chunk > 0) {
        const dim3 grid(grid_for(P.n_chunk, kBlock / kGatGroup));
        hipLaunchKernelGGL(gat_softmax_fwd_group<1>, grid, dim3(kBlock), 0, stream, ptr, idx, rel,
                           ee_table, el, er, n_seg, H, lg, slope, a, P, nullptr);
        const int64_t base = run_tree(plan, 1, 2 * H, 0, H, 1, stream);
        const float* fin = P.part + base * 2 * H;
        hipLaunchKernelGGL(gat_softmax_fwd_group<2>, grid, dim3(kBlock), 0, stream, ptr, idx, rel,
                           ee_table, el, er, n_seg, H, lg, slope, a, P, fin);
        REGNN_LAUNCH_CHECK();
    }
    return REGNN_OK;
}

int regnn_gat_softmax_bwd(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                          const float* ee_table, const float* el, const float* er, const float* a,
                          const float* ga, int64_t n_seg, int32_t H, float slope, float* gs_out,
                          float* ger, float* slab, int32_t n_rel, const regnn_seg_plan* plan,
                          hipStream_t stream) {
    if (!ptr || !idx || !el || !er || !a || !ga || !gs_out || !ger || H <= 0 || n_seg < 0)
        return REGNN_EINVAL;
    if ((ee_table || slab) && !rel) return REGNN_EINVAL;
    if (slab && (n_rel <= 0 || n_rel > 64 || kBlock % H)) return REGNN_EUNSUPPORTED;
    if (n_seg == 0) return REGNN_OK;
    const size_t lds = slab ? size_t(n_rel) * kBlock * sizeof(float) : 0;
    const int lg = gat_log2(H);
    if (lg < 0) {
        hipLaunchKernelGGL(gat_softmax_bwd_generic, dim3(grid_for(n_seg * H, kBlock)),
                           dim3(kBlock), lds, stream, ptr, idx, rel, ee_table, el, er, a, ga,
                           n_seg, H, slope, gs_out, ger, slab, n_rel);
        REGNN_LAUNCH_CHECK();
        return REGNN_OK;
    }
    if (const int rc = check_plan(plan, H)) return rc;
    const LongPlan P = long_plan(plan);
    const int g0 = grid_for(n_seg, kBlock / kGatGroup);
    hipLaunchKernelGGL(gat_softmax_bwd_group<0>, dim3(g0), dim3(kBlock), lds, stream, ptr, idx,
                       rel, ee_table, el, er, a, ga, n_seg, H, lg, slope, gs_out, ger, slab,
                       n_rel, P, nullptr);
    REGNN_LAUNCH_CHECK();
    if (P.n_chunk > 0) {
        // the slab's rows past the per-segment pass hold the chunk pass's relation bins
        // (regnn_slab_rows() = 2 kMaxGrid >= both grids)
        const dim3 grid(grid_for(P.n_chunk, kBlock / kGatGroup));
        hipLaunchKernelGGL(gat_softmax_bwd_group<1>, grid, dim3(kBlock), 0, stream, ptr, idx, rel,
                           ee_table, el, er, a, ga, n_seg, H, lg, slope, gs_out, ger, nullptr,
                           n_rel, P, nullptr);
        int64_t base = run_tree(plan, 0, H, H, H, 1, stream);
        hipLaunchKernelGGL(gat_softmax_bwd_group<2>, grid, dim3(kBlock), lds, stream, ptr, idx,
                           rel, ee_table, el, er, a, ga, n_seg, H, lg, slope, gs_out, ger,
                           slab ? slab + int64_t(g0) * n_rel * H : nullptr, n_rel, P,
                           P.part + base * H);
        base = run_tree(plan, 0, H, H, H, 1, stream);
        hipLaunchKernelGGL(seg_emit_sum<float>, dim3(long_grid(P.n_long)), dim3(kBlock), 0,
                           stream, P.part, P.chunk_off, base, plan->n_levels, P.long_ids,
                           P.n_long, H, ger);
        REGNN_LAUNCH_CHECK();
    }
    return REGNN_OK;
}

int regnn_gat_fused_fwd(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                        const float* ee_table, const float* el, const float* er, const void* x,
                        void* out, float* lse, int64_t n_seg, int32_t H, int32_t D, float slope,
                        int32_t dtype, const float* attn_l, const regnn_seg_plan* plan,
                        hipStream_t stream) {
    if (!ptr || !idx || !el || !er || !x || !out || !lse || n_seg < 0 || (ee_table && !rel))
        return REGNN_EINVAL;
    if (n_seg == 0) return REGNN_OK;
    if (const int rc = check_plan(plan, int64_t(H) * D + 2 * H)) return rc;
    GatFusedArgs p{ptr, idx, rel, ee_table, el, er, x, out, lse, attn_l, n_seg, H, D, slope};
    if (dtype == REGNN_F32) return dispatch_gat_fused<float>(p, plan, stream);
    if (dtype == REGNN_BF16) return dispatch_gat_fused<bf16_t>(p, plan, stream);
    return REGNN_EUNSUPPORTED;
}

int regnn_gat_attn_lse(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                       const float* ee_table, const float* el, const float* er, const float* lse,
                       int64_t n_seg, int32_t H, float slope, float* a, const regnn_seg_plan* plan,
                       hipStream_t stream) {
    if (!ptr || !idx || !el || !er || !lse || !a || H <= 0 || n_seg < 0 || (ee_table && !rel))
        return REGNN_EINVAL;
    if (n_seg == 0) return REGNN_OK;
    const int lg = gat_log2(H);
    if (lg < 0) return REGNN_EUNSUPPORTED;
    if (const int rc = check_plan(plan, 0)) return rc;
    const LongPlan P = long_plan(plan);
    hipLaunchKernelGGL(gat_attn_lse_group<false>, dim3(grid_for(n_seg, kBlock / kGatGroup)),
                       dim3(kBlock), 0, stream, ptr, idx, rel, ee_table, el, er, lse, n_seg, H, lg,
                       slope, a, P);
    REGNN_LAUNCH_CHECK();
    if (P.n_chunk > 0) {
        hipLaunchKernelGGL(gat_attn_lse_group<true>, dim3(grid_for(P.n_chunk, kBlock / kGatGroup)),
                           dim3(kBlock), 0, stream, ptr, idx, rel, ee_table, el, er, lse, n_seg,
                           H, lg, slope, a, P);
        REGNN_LAUNCH_CHECK();
    }
    return REGNN_OK;
}

int regnn_spmm_heads_fwd(const int32_t* ptr, const int32_t* idx, const int32_t* perm,
                         const float* a, const void* x, void* y, int64_t n_seg, int32_t H,
                         int32_t D, int32_t dtype, const regnn_seg_plan* plan, hipStream_t stream) {
    if (!ptr || !idx || !a || !x || !y || n_seg < 0) return REGNN_EINVAL;
    if (n_seg == 0) return REGNN_OK;
    if (const int rc = check_plan(plan, int64_t(H) * D)) return rc;
    HeadArgs p{ptr, idx, perm, a, x, nullptr, y, nullptr, n_seg, H, D};
    if (dtype == REGNN_F32) return dispatch_heads<float, false>(p, plan, stream);
    if (dtype == REGNN_BF16) return dispatch_heads<bf16_t, false>(p, plan, stream);
    return REGNN_EUNSUPPORTED;
}

int regnn_spmm_heads_bwd(const int32_t* ptr, const int32_t* idx, const int32_t* perm,
                         const float* a, const void* g, const void* x, void* gx, float* ga,
                         int64_t n_seg, int32_t H, int32_t D, int32_t dtype,
                         const regnn_seg_plan* plan, hipStream_t stream) {
    if (!ptr || !idx || !a || !g || !x || !gx || !ga || n_seg < 0) return REGNN_EINVAL;
    if (n_seg == 0) return REGNN_OK;
    if (const int rc = check_plan(plan, int64_t(H) * D)) return rc;
    HeadArgs p{ptr, idx, perm, a, g, x, gx, ga, n_seg, H, D};
    if (dtype == REGNN_F32) return dispatch_heads<float, true>(p, plan, stream);
    if (dtype == REGNN_BF16) return dispatch_heads<bf16_t, true>(p, plan, stream);
    return REGNN_EUNSUPPORTED;
}

int regnn_segment_sum(const int32_t* ptr, const int32_t* perm, const float* vals, int64_t n_seg,
                      int32_t H, float* out, const regnn_seg_plan* plan, hipStream_t stream) {
    if (!ptr || !vals || !out || H <= 0 || n_seg < 0) return REGNN_EINVAL;
    if (n_seg == 0) return REGNN_OK;
    const int lg = gat_log2(H);
    if (lg < 0) {
        hipLaunchKernelGGL(segment_sum_generic, dim3(grid_for(n_seg * H, kBlock)), dim3(kBlock),
                           0, stream, ptr, perm, vals, n_seg, H, out);
        REGNN_LAUNCH_CHECK();
        return REGNN_OK;
    }
    if (const int rc = check_plan(plan, H)) return rc;
    const LongPlan P = long_plan(plan);
    hipLaunchKernelGGL(segment_sum_group<false>, dim3(grid_for(n_seg, kBlock / kGatGroup)),
                       dim3(kBlock), 0, stream, ptr, perm, vals, n_seg, H, lg, out, P);
    REGNN_LAUNCH_CHECK();
    if (P.n_chunk > 0) {
        hipLaunchKernelGGL(segment_sum_group<true>, dim3(grid_for(P.n_chunk, kBlock / kGatGroup)),
                           dim3(kBlock), 0, stream, ptr, perm, vals, n_seg, H, lg, out, P);
        const int64_t base = run_tree(plan, 0, H, H, H, 1, stream);
        hipLaunchKernelGGL(seg_emit_sum<float>, dim3(long_grid(P.n_long)), dim3(kBlock), 0,
                           stream, P.part, P.chunk_off, base, plan->n_levels, P.long_ids,
                           P.n_long, H, out);
        REGNN_LAUNCH_CHECK();
    }
    return REGNN_OK;
}

int regnn_attn_dots_fwd(const float* ft, const float* attn_l, const float* attn_r, int64_t N,
                        int32_t H, int32_t D, float* el, float* er, hipStream_t stream) {
    if (!ft || !attn_l || !attn_r || !el || !er || N < 0 || H <= 0 || D <= 0) return REGNN_EINVAL;
    if (N == 0) return REGNN_OK;
    if (attn_dots_vec_ok(D))
        hipLaunchKernelGGL(attn_dots_fwd_vec_kernel, dim3(grid_for(N * H, kBlock / (D / 4))),
                           dim3(kBlock), 0, stream, ft, attn_l, attn_r, N, H, D, el, er);
    else
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
    const int F = H * D, CPL = F / 4;
    const bool vec = D % 4 == 0 && CPL <= kBlock && kBlock % CPL == 0 &&
                     (reinterpret_cast<uintptr_t>(ft) | reinterpret_cast<uintptr_t>(gft) |
                      reinterpret_cast<uintptr_t>(attn_l) | reinterpret_cast<uintptr_t>(attn_r) |
                      reinterpret_cast<uintptr_t>(slab)) % 16 == 0;
    if (vec) {
        hipLaunchKernelGGL(attn_dots_bwd_vec_kernel<4>, dim3(slab_rows), dim3(kBlock),
                           size_t(kBlock / CPL) * 2 * CPL * sizeof(float4), stream,
                           reinterpret_cast<const float4*>(ft),
                           reinterpret_cast<const float4*>(attn_l),
                           reinterpret_cast<const float4*>(attn_r), gel, ger, N, H, D, CPL, rpb,
                           reinterpret_cast<float4*>(gft), slab);
    } else {
        hipLaunchKernelGGL(attn_dots_bwd_kernel, dim3(slab_rows), dim3(kBlock), 0, stream, ft,
                           attn_l, attn_r, gel, ger, N, H, D, rpb, gft, slab);
    }
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

}  // extern "C"
