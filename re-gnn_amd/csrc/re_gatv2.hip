// Attention variants on gfx950 beyond REGATConv's fused el/er softmax (re_gat.hip):
//  * per-edge logits scores for GATv2 (layer/REGATv2Conv.py:139-141, mag/regnn_layers.py:399-403):
//    s[e,h] = <att[h,:], LeakyReLU(fs[u,h,:] + fd[v,h,:])> — an SDDMM with the activation inside
//    the dot, a group of LPR lanes per destination gathering source rows (16-byte vectors, a
//    lane's head fixed by its feature offset, D/4-lane xor-shuffle reduction per head), and its
//    backward split into a CSR pass (d fd, d att partials) and a CSC pass (d fs);
//  * the edge softmax over precomputed per-edge logits (+ optional relation bias table), either
//    DGL's per-destination max-subtracted form or the ogbn-mag form with ONE global max and a
//    1e-16 guard in the denominator (mag/utils.py:45-57), and its backward with relation-bias
//    slabs (deterministic, no atomics);
//  * the u_add_v + relation-bias + LeakyReLU scores of GAT v1 written per edge (for the global
//    max of the ogbn-mag softmax).
#include "regnn_common.h"

namespace regnn {

__device__ __forceinline__ float lrelu2(float x, float slope) { return x > 0.f ? x : x * slope; }

constexpr int kSmG = 32;     // lanes per destination in the softmax kernels
constexpr int kSmU = 4;      // (edge, head) pairs in flight per lane

// ---- GATv2 scores ---------------------------------------------------------------------------
struct V2Args {
    const int32_t* ptr;    // CSR (fwd, bwd_dst) or CSC (bwd_src)
    const int32_t* idx;
    const int32_t* perm;   // CSC -> CSR edge position (bwd_src)
    const float* fs;       // [n_src, H*D]
    const float* fd;       // [n_dst, H*D]
    const float* att;      // [H*D]
    const float* gs;       // [E, H] d loss / d s (CSR order)
    float* out;            // fwd: s [E, H]; bwd_dst: g fd; bwd_src: g fs
    float* slab;           // bwd_dst: per-block d att partials [grid][H*D]
    int64_t n_seg;
    int H, D;
    float slope;
};

// MODE 0: forward scores over the CSR; 1: backward over the CSR (d fd, d att);
// 2: backward over the CSC (d fs). The segment node's own row is `self` (fd in 0/1, fs in 2)
// and the gathered row is the other side.
template <int LPR, int NV, int MODE>
__global__ void __launch_bounds__(kBlock) gatv2_kernel(V2Args p) {
    constexpr int GPB = kBlock / LPR;
    constexpr int UN = NV <= 2 ? 4 : 2;
    extern __shared__ float sat[];           // MODE 1: [GPB][F] d att partials
    const int tid = threadIdx.x, lane = tid & (LPR - 1), grp = tid / LPR;
    const int F = p.H * p.D;
    const int vph = p.D / 4;
    const float* __restrict__ self_rows = MODE == 2 ? p.fs : p.fd;
    const float* __restrict__ gath_rows = MODE == 2 ? p.fd : p.fs;
    float at[NV][4], gatt[NV][4] = {};
    int head[NV];
#pragma unroll
    for (int q = 0; q < NV; ++q) {
        const int o = (q * LPR + lane) * 4;
        head[q] = o < F ? o / p.D : 0;
        if (o < F) Vec<float>::load(p.att + o, at[q]);
        else for (int t = 0; t < 4; ++t) at[q][t] = 0.f;
    }
    for (int64_t seg = (int64_t)blockIdx.x * GPB + grp; seg < p.n_seg;
         seg += (int64_t)gridDim.x * GPB) {
        const int beg = p.ptr[seg], end = p.ptr[seg + 1];
        float sx[NV][4], acc[NV][4] = {};
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            const int o = (q * LPR + lane) * 4;
            if (o < F) Vec<float>::load(self_rows + seg * F + o, sx[q]);
            else for (int t = 0; t < 4; ++t) sx[q][t] = 0.f;
        }
        for (int e0 = beg; e0 < end; e0 += LPR) {
            const int e = e0 + lane;
            int j = 0, eid = 0;
            if (e < end) {
                j = p.idx[e];
                eid = MODE == 2 ? p.perm[e] : e;
            }
            const int cnt = min(LPR, end - e0);
            for (int k0 = 0; k0 < cnt; k0 += UN) {
                float v[UN][NV][4];
                float g[UN][NV];
                int ekk[UN];
#pragma unroll
                for (int u = 0; u < UN; ++u) {
                    const int kk = min(k0 + u, cnt - 1);
                    const int jj = __shfl(j, kk, LPR);
                    ekk[u] = __shfl(eid, kk, LPR);
#pragma unroll
                    for (int q = 0; q < NV; ++q) {
                        const int o = (q * LPR + lane) * 4;
                        if (o < F) {
                            Vec<float>::load(gath_rows + (int64_t)jj * F + o, v[u][q]);
                            g[u][q] = (MODE != 0 && k0 + u < cnt)
                                          ? p.gs[(int64_t)ekk[u] * p.H + head[q]] : 0.f;
                        } else {
#pragma unroll
                            for (int t = 0; t < 4; ++t) v[u][q][t] = 0.f;
                            g[u][q] = 0.f;
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < UN; ++u) {
#pragma unroll
                    for (int q = 0; q < NV; ++q) {
                        if constexpr (MODE == 0) {
                            float d = 0.f;
#pragma unroll
                            for (int t = 0; t < 4; ++t)
                                d = fmaf(at[q][t], lrelu2(v[u][q][t] + sx[q][t], p.slope), d);
                            for (int m = vph >> 1; m > 0; m >>= 1) d += __shfl_xor(d, m, 64);
                            const int o = (q * LPR + lane) * 4;
                            if (k0 + u < cnt && o < F && (lane & (vph - 1)) == 0)
                                p.out[(int64_t)ekk[u] * p.H + head[q]] = d;
                        } else {
#pragma unroll
                            for (int t = 0; t < 4; ++t) {
                                const float pre = v[u][q][t] + sx[q][t];
                                acc[q][t] = fmaf(g[u][q] * at[q][t], pre > 0.f ? 1.f : p.slope,
                                                 acc[q][t]);
                                if constexpr (MODE == 1)
                                    gatt[q][t] = fmaf(g[u][q], lrelu2(pre, p.slope), gatt[q][t]);
                            }
                        }
                    }
                }
            }
        }
        if constexpr (MODE != 0) {
            float* __restrict__ out = p.out + seg * F;
#pragma unroll
            for (int q = 0; q < NV; ++q) {
                const int o = (q * LPR + lane) * 4;
                if (o < F) Vec<float>::store(out + o, acc[q]);
            }
        }
    }
    if constexpr (MODE == 1) {
        // fixed-order block reduction of the groups' d att partials into slab row blockIdx.x
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            const int o = (q * LPR + lane) * 4;
            if (o < F)
                for (int t = 0; t < 4; ++t) sat[grp * F + o + t] = gatt[q][t];
        }
        __syncthreads();
        for (int c = tid; c < F; c += kBlock) {
            float s = 0.f;
            for (int gi = 0; gi < GPB; ++gi) s += sat[gi * F + c];
            p.slab[(int64_t)blockIdx.x * F + c] = s;
        }
    }
}

template <int MODE>
int launch_gatv2(V2Args p, int grid, hipStream_t stream) {
    const int F = p.H * p.D;
    if (p.D <= 0 || p.D % 4 || p.H <= 0) return REGNN_EUNSUPPORTED;
    const int vph = p.D / 4;
    if (vph & (vph - 1)) return REGNN_EUNSUPPORTED;
    const int nvec = F / 4;
#define REGNN_V2(LPR, NV)                                                                        \
    if (nvec <= (LPR) * (NV) && vph <= (LPR)) {                                                  \
        const size_t lds = MODE == 1 ? size_t(kBlock / (LPR)) * F * sizeof(float) : 0;           \
        hipLaunchKernelGGL((gatv2_kernel<LPR, NV, MODE>), dim3(grid), dim3(kBlock), lds, stream, \
                           p);                                                                   \
        REGNN_LAUNCH_CHECK();                                                                    \
        return REGNN_OK;                                                                         \
    }
    REGNN_V2(16, 1)
    REGNN_V2(16, 2)
    REGNN_V2(16, 4)
    REGNN_V2(64, 2)
    REGNN_V2(64, 4)
#undef REGNN_V2
    return REGNN_EUNSUPPORTED;
}

int v2_lpr(int H, int D) { return H * D / 4 <= 64 ? 16 : 64; }

// ---- edge softmax over per-edge logits ------------------------------------------------------
__device__ __forceinline__ void sm_merge(float& m, float& s, float mo, float so) {
    const float mn = fmaxf(m, mo);
    if (mn == -INFINITY) return;
    s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + (mo == -INFINITY ? 0.f : so * __expf(mo - mn));
    m = mn;
}

__device__ __forceinline__ float edge_logit(const float* __restrict__ s,
                                            const uint8_t* __restrict__ rel,
                                            const float* __restrict__ ee, int64_t k, int H, int h) {
    float v = s[k * H + h];
    if (ee) v += ee[rel[k] * H + h];
    return v;
}

// a = exp(z - m_v) / sum_v (gmax == NULL: m_v = per-destination max)
//   = exp(z - gmax) / (sum_v exp(z - gmax) + eps) (global max form)
__global__ void __launch_bounds__(kBlock)
edge_softmax_fwd_kernel(const int32_t* __restrict__ ptr, const float* __restrict__ s,
                        const uint8_t* __restrict__ rel, const float* __restrict__ ee,
                        const float* __restrict__ gmax, float eps, int64_t n_seg, int H, int lgH,
                        float* __restrict__ a) {
    constexpr int G = kSmG, U = kSmU;
    const int lane = threadIdx.x & (G - 1), h = lane & (H - 1);
    const float gm = gmax ? *gmax : 0.f;
    for (int64_t seg = (int64_t)blockIdx.x * (kBlock / G) + threadIdx.x / G; seg < n_seg;
         seg += (int64_t)gridDim.x * (kBlock / G)) {
        const int64_t beg = ptr[seg];
        const int np = (ptr[seg + 1] - ptr[seg]) << lgH;
        float m = gmax ? gm : -INFINITY, sum = 0.f;
        for (int p0 = lane; p0 < np; p0 += G * U) {
            float sc[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int pp = p0 + u * G;
                sc[u] = pp < np ? edge_logit(s, rel, ee, beg + (pp >> lgH), H, h) : -INFINITY;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (gmax) sum += sc[u] == -INFINITY ? 0.f : __expf(sc[u] - gm);
                else sm_merge(m, sum, sc[u], 1.f);
            }
        }
        if (gmax) {
            for (int o = H; o < G; o <<= 1) sum += __shfl_xor(sum, o, G);
        } else {
            for (int o = H; o < G; o <<= 1)
                sm_merge(m, sum, __shfl_xor(m, o, G), __shfl_xor(sum, o, G));
        }
        const float inv = 1.f / (sum + eps);
        for (int p0 = lane; p0 < np; p0 += G * U) {
            float sc[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int pp = p0 + u * G;
                sc[u] = pp < np ? edge_logit(s, rel, ee, beg + (pp >> lgH), H, h) : 0.f;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int pp = p0 + u * G;
                if (pp < np) a[beg * H + pp] = __expf(sc[u] - m) * inv;
            }
        }
    }
}

// gz = a * (ga - sum_v a*ga); slab: per (rel, head) sums of gz (d loss / d relation table)
__global__ void __launch_bounds__(kBlock)
edge_softmax_bwd_kernel(const int32_t* __restrict__ ptr, const uint8_t* __restrict__ rel,
                        const float* __restrict__ a, const float* __restrict__ ga, int64_t n_seg,
                        int H, int lgH, float* __restrict__ gz_out, float* __restrict__ slab,
                        int n_rel) {
    constexpr int G = kSmG, U = kSmU;
    extern __shared__ float bins[];   // [n_rel][kBlock]; a thread only touches its own column
    const int tid = threadIdx.x, lane = tid & (G - 1), h = lane & (H - 1);
    if (slab) for (int r = 0; r < n_rel; ++r) bins[r * kBlock + tid] = 0.f;
    for (int64_t seg = (int64_t)blockIdx.x * (kBlock / G) + tid / G; seg < n_seg;
         seg += (int64_t)gridDim.x * (kBlock / G)) {
        const int64_t beg = ptr[seg];
        const int np = (ptr[seg + 1] - ptr[seg]) << lgH;
        const float* __restrict__ as = a + beg * H;
        const float* __restrict__ gas = ga + beg * H;
        float dot = 0.f;
        for (int p0 = lane; p0 < np; p0 += G * U) {
            float d[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int pp = p0 + u * G;
                d[u] = pp < np ? as[pp] * gas[pp] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) dot += d[u];
        }
        for (int o = H; o < G; o <<= 1) dot += __shfl_xor(dot, o, G);
        for (int p0 = lane; p0 < np; p0 += G * U) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int pp = p0 + u * G;
                if (pp < np) {
                    const float gz = as[pp] * (gas[pp] - dot);
                    gz_out[beg * H + pp] = gz;
                    if (slab) bins[rel[beg + (pp >> lgH)] * kBlock + tid] += gz;
                }
            }
        }
    }
    if (slab) {
        __syncthreads();            // G % H == 0: thread tid always works on head tid % H
        for (int c = tid; c < n_rel * H; c += kBlock) {
            const int r = c / H, hh = c - r * H;
            float sm = 0.f;
            for (int t2 = hh; t2 < kBlock; t2 += H) sm += bins[r * kBlock + t2];
            slab[(int64_t)blockIdx.x * n_rel * H + c] = sm;
        }
    }
}

// s[k,h] = LeakyReLU(el[idx[k],h] + er[v,h] + ee[rel[k],h], slope) in CSR order
__global__ void __launch_bounds__(kBlock)
gat_scores_kernel(const int32_t* __restrict__ ptr, const int32_t* __restrict__ idx,
                  const uint8_t* __restrict__ rel, const float* __restrict__ ee,
                  const float* __restrict__ el, const float* __restrict__ er, int64_t n_seg,
                  int H, int lgH, float slope, float* __restrict__ s) {
    constexpr int G = kSmG;
    const int lane = threadIdx.x & (G - 1), h = lane & (H - 1);
    for (int64_t seg = (int64_t)blockIdx.x * (kBlock / G) + threadIdx.x / G; seg < n_seg;
         seg += (int64_t)gridDim.x * (kBlock / G)) {
        const int64_t beg = ptr[seg];
        const int np = (ptr[seg + 1] - ptr[seg]) << lgH;
        const float erv = er[seg * H + h];
        for (int pp = lane; pp < np; pp += G) {
            const int64_t k = beg + (pp >> lgH);
            float v = el[(int64_t)idx[k] * H + h] + erv;
            if (ee) v += ee[rel[k] * H + h];
            s[beg * H + pp] = lrelu2(v, slope);
        }
    }
}

int sm_log2(int H) {
    for (int l = 0; (1 << l) <= kSmG; ++l)
        if ((1 << l) == H) return l;
    return -1;
}

}  // namespace regnn

using namespace regnn;

extern "C" {

int regnn_gatv2_score_fwd(const int32_t* ptr, const int32_t* idx, const float* fs, const float* fd,
                          const float* att, int64_t n_seg, int32_t H, int32_t D, float slope,
                          float* s, hipStream_t stream) {
    if (!ptr || !idx || !fs || !fd || !att || !s || n_seg < 0 || H <= 0 || D <= 0)
        return REGNN_EINVAL;
    if (n_seg == 0) return REGNN_OK;
    V2Args p{ptr, idx, nullptr, fs, fd, att, nullptr, s, nullptr, n_seg, H, D, slope};
    return launch_gatv2<0>(p, grid_for(n_seg, kBlock / v2_lpr(H, D)), stream);
}

int regnn_gatv2_score_bwd_dst(const int32_t* ptr, const int32_t* idx, const float* fs,
                              const float* fd, const float* att, const float* gs, int64_t n_seg,
                              int32_t H, int32_t D, float slope, float* gfd, float* att_slab,
                              int32_t slab_rows, hipStream_t stream) {
    if (!ptr || !idx || !fs || !fd || !att || !gs || !gfd || !att_slab || n_seg < 0 || H <= 0 ||
        D <= 0 || slab_rows <= 0)
        return REGNN_EINVAL;
    if (n_seg == 0) return REGNN_OK;
    V2Args p{ptr, idx, nullptr, fs, fd, att, gs, gfd, att_slab, n_seg, H, D, slope};
    int grid = grid_for(n_seg, kBlock / v2_lpr(H, D));
    if (grid > slab_rows) grid = slab_rows;
    return launch_gatv2<1>(p, grid, stream);
}

int regnn_gatv2_score_bwd_src(const int32_t* csc_ptr, const int32_t* csc_idx,
                              const int32_t* csc2csr, const float* fs, const float* fd,
                              const float* att, const float* gs, int64_t n_src, int32_t H,
                              int32_t D, float slope, float* gfs, hipStream_t stream) {
    if (!csc_ptr || !csc_idx || !csc2csr || !fs || !fd || !att || !gs || !gfs || n_src < 0 ||
        H <= 0 || D <= 0)
        return REGNN_EINVAL;
    if (n_src == 0) return REGNN_OK;
    V2Args p{csc_ptr, csc_idx, csc2csr, fs, fd, att, gs, gfs, nullptr, n_src, H, D, slope};
    return launch_gatv2<2>(p, grid_for(n_src, kBlock / v2_lpr(H, D)), stream);
}

int regnn_edge_softmax_fwd(const int32_t* ptr, const float* s, const uint8_t* rel,
                           const float* ee_table, const float* gmax, float eps, int64_t n_seg,
                           int32_t H, float* a, hipStream_t stream) {
    if (!ptr || !s || !a || n_seg < 0 || (ee_table && !rel)) return REGNN_EINVAL;
    const int lg = sm_log2(H);
    if (lg < 0) return REGNN_EUNSUPPORTED;
    if (n_seg == 0) return REGNN_OK;
    hipLaunchKernelGGL(edge_softmax_fwd_kernel, dim3(grid_for(n_seg, kBlock / kSmG)),
                       dim3(kBlock), 0, stream, ptr, s, rel, ee_table, gmax, eps, n_seg, H, lg, a);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

int regnn_edge_softmax_bwd(const int32_t* ptr, const uint8_t* rel, const float* a,
                           const float* ga, int64_t n_seg, int32_t H, float* gz, float* slab,
                           int32_t n_rel, hipStream_t stream) {
    if (!ptr || !a || !ga || !gz || n_seg < 0 || (slab && (!rel || n_rel <= 0 || n_rel > 64)))
        return REGNN_EINVAL;
    const int lg = sm_log2(H);
    if (lg < 0) return REGNN_EUNSUPPORTED;
    if (n_seg == 0) return REGNN_OK;
    const size_t lds = slab ? size_t(n_rel) * kBlock * sizeof(float) : 0;
    hipLaunchKernelGGL(edge_softmax_bwd_kernel, dim3(grid_for(n_seg, kBlock / kSmG)),
                       dim3(kBlock), lds, stream, ptr, rel, a, ga, n_seg, H, lg, gz, slab, n_rel);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

int regnn_gat_scores(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                     const float* ee_table, const float* el, const float* er, int64_t n_seg,
                     int32_t H, float slope, float* s, hipStream_t stream) {
    if (!ptr || !idx || !el || !er || !s || n_seg < 0 || (ee_table && !rel)) return REGNN_EINVAL;
    const int lg = sm_log2(H);
    if (lg < 0) return REGNN_EUNSUPPORTED;
    if (n_seg == 0) return REGNN_OK;
    hipLaunchKernelGGL(gat_scores_kernel, dim3(grid_for(n_seg, kBlock / kSmG)), dim3(kBlock), 0,
                       stream, ptr, idx, rel, ee_table, el, er, n_seg, H, lg, slope, s);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

}  // extern "C"
