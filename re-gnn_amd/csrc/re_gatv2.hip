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
// Hub rows take the long-segment plan (regnn_seg_plan, re_segplan.h) as REGATConv's kernels do:
// the per-segment passes skip segments past the plan's split, chunk passes run their
// `chunk`-edge pieces on groups of their own (scores: independent per edge; the segment sums of
// the backward and the softmax's max / sum / dot: fp32 partial rows combined by the plan's
// fixed-order tree, then written by an emit pass).
#include "regnn_common.h"
#include "re_segplan.h"

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
// and the gathered row is the other side. CH: the units are the plan's chunks of long segments
// (MODE 1 / 2: the segment sum as an fp32 partial row per chunk); otherwise the segments, long
// ones skipped.
template <int LPR, int NV, int MODE, bool CH>
__global__ void __launch_bounds__(kBlock) gatv2_kernel(V2Args p, LongPlan P) {
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
    const int64_t n_units = CH ? P.n_chunk : p.n_seg;
    for (int64_t unit = (int64_t)blockIdx.x * GPB + grp; unit < n_units;
         unit += (int64_t)gridDim.x * GPB) {
        int64_t seg;
        int beg, end;
        if (CH) {
            chunk_range(P, p.ptr, unit, seg, beg, end);
        } else {
            seg = unit;
            beg = p.ptr[seg];
            end = p.ptr[seg + 1];
            if (end - beg > P.split) continue;     // a long segment: the chunk pass
        }
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
            float* __restrict__ out = CH ? P.part + unit * F : p.out + seg * F;
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

// grid: the per-segment pass; MODE 1 with a plan: its chunk pass writes the d att partials of its
// blocks to the slab rows after the first pass's (`grid2` rows), so the slab needs grid + grid2
template <int MODE>
int launch_gatv2(V2Args p, int grid, const regnn_seg_plan* pl, int grid2, hipStream_t stream) {
    const int F = p.H * p.D;
    if (p.D <= 0 || p.D % 4 || p.H <= 0) return REGNN_EUNSUPPORTED;
    const int vph = p.D / 4;
    if (vph & (vph - 1)) return REGNN_EUNSUPPORTED;
    const int nvec = F / 4;
    if (const int rc = check_plan(pl, MODE == 0 ? 0 : F)) return rc;
    const LongPlan P = long_plan(pl);
#define REGNN_V2(LPR, NV)                                                                        \
    if (nvec <= (LPR) * (NV) && vph <= (LPR)) {                                                  \
        const size_t lds = MODE == 1 ? size_t(kBlock / (LPR)) * F * sizeof(float) : 0;           \
        hipLaunchKernelGGL((gatv2_kernel<LPR, NV, MODE, false>), dim3(grid), dim3(kBlock), lds,  \
                           stream, p, P);                                                        \
        REGNN_LAUNCH_CHECK();                                                                    \
        if (P.n_chunk > 0) {                                                                     \
            V2Args q = p;                                                                        \
            if (MODE == 1) q.slab = p.slab + int64_t(grid) * F;                                  \
            int g2 = grid_for(P.n_chunk, kBlock / (LPR));                                        \
            if (MODE == 1 && g2 > grid2) g2 = grid2;                                             \
            hipLaunchKernelGGL((gatv2_kernel<LPR, NV, MODE, true>), dim3(g2), dim3(kBlock), lds, \
                               stream, q, P);                                                    \
            REGNN_LAUNCH_CHECK();                                                                \
            if (MODE != 0) {                                                                     \
                const int64_t base = run_tree(pl, 0, F, F, p.H, p.D, stream);                    \
                hipLaunchKernelGGL(seg_emit_sum<float>, dim3(long_grid(P.n_long)), dim3(kBlock), \
                                   0, stream, P.part, P.chunk_off, base, pl->n_levels,           \
                                   P.long_ids, P.n_long, F, p.out);                              \
                REGNN_LAUNCH_CHECK();                                                            \
            }                                                                                    \
        }                                                                                        \
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
// PASS 0: the segments (long ones skipped); 1: the plan's chunks -> partial rows [max H | sum H]
// (the tree's online-softmax rows with F = 0); 2: the chunks again, a from their segment's
// combined row (fin = the tree's last level)
__device__ __forceinline__ bool sm_unit(int PASS, const LongPlan& P, const int32_t* __restrict__ ptr,
                                        int64_t unit, int64_t& beg, int& n, int& l) {
    if (PASS) {
        int64_t seg;
        int b, e;
        chunk_range(P, ptr, unit, seg, b, e, l);
        beg = b;
        n = e - b;
        return true;
    }
    l = -1;
    beg = ptr[unit];
    n = ptr[unit + 1] - int(beg);
    return n <= P.split;
}

template <int PASS>
__global__ void __launch_bounds__(kBlock)
edge_softmax_fwd_kernel(const int32_t* __restrict__ ptr, const float* __restrict__ s,
                        const uint8_t* __restrict__ rel, const float* __restrict__ ee,
                        const float* __restrict__ gmax, float eps, int64_t n_seg, int H, int lgH,
                        float* __restrict__ a, LongPlan P, const float* __restrict__ fin,
                        int64_t fin_base, int n_levels) {
    constexpr int G = kSmG, U = kSmU;
    const int lane = threadIdx.x & (G - 1), h = lane & (H - 1);
    const float gm = gmax ? *gmax : 0.f;
    const int64_t n_units = PASS ? P.n_chunk : n_seg;
    for (int64_t unit = (int64_t)blockIdx.x * (kBlock / G) + threadIdx.x / G; unit < n_units;
         unit += (int64_t)gridDim.x * (kBlock / G)) {
        int64_t beg;
        int n, l;
        if (!sm_unit(PASS, P, ptr, unit, beg, n, l)) continue;
        const int np = n << lgH;
        float m = gmax ? gm : -INFINITY, sum = 0.f;
        if (PASS == 2) {                   // the segment's combined max / sum
            const float* fr = fin + final_row(P.chunk_off, fin_base, n_levels, l) * 2 * H;
            m = fr[h];
            sum = fr[H + h];
        } else {
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
        if (PASS == 1) {                   // the chunk's partial row
            if (lane < H) {
                P.part[unit * 2 * H + h] = m;
                P.part[unit * 2 * H + H + h] = sum;
            }
            continue;
        }
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

// gz = a * (ga - sum_v a*ga); slab: per (rel, head) sums of gz (d loss / d relation table).
// PASS 0: the segments (long ones skipped); 1: the plan's chunks -> partial dot rows [H];
// 2: the chunks again with their segment's combined dot (fin)
template <int PASS>
__global__ void __launch_bounds__(kBlock)
edge_softmax_bwd_kernel(const int32_t* __restrict__ ptr, const uint8_t* __restrict__ rel,
                        const float* __restrict__ a, const float* __restrict__ ga, int64_t n_seg,
                        int H, int lgH, float* __restrict__ gz_out, float* __restrict__ slab,
                        int n_rel, LongPlan P, const float* __restrict__ fin, int64_t fin_base,
                        int n_levels) {
    constexpr int G = kSmG, U = kSmU;
    extern __shared__ float bins[];   // [n_rel][kBlock]; a thread only touches its own column
    const int tid = threadIdx.x, lane = tid & (G - 1), h = lane & (H - 1);
    if (slab) for (int r = 0; r < n_rel; ++r) bins[r * kBlock + tid] = 0.f;
    const int64_t n_units = PASS ? P.n_chunk : n_seg;
    for (int64_t unit = (int64_t)blockIdx.x * (kBlock / G) + tid / G; unit < n_units;
         unit += (int64_t)gridDim.x * (kBlock / G)) {
        int64_t beg;
        int n, l;
        if (!sm_unit(PASS, P, ptr, unit, beg, n, l)) continue;
        const int np = n << lgH;
        const float* __restrict__ as = a + beg * H;
        const float* __restrict__ gas = ga + beg * H;
        float dot = 0.f;
        if (PASS == 2) {
            dot = fin[final_row(P.chunk_off, fin_base, n_levels, l) * H + h];
        } else {
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
        if (PASS == 1) {
            if (lane < H) P.part[unit * H + h] = dot;
            continue;
        }
        }
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
                          float* s, const regnn_seg_plan* plan, hipStream_t stream) {
    if (!ptr || !idx || !fs || !fd || !att || !s || n_seg < 0 || H <= 0 || D <= 0)
        return REGNN_EINVAL;
    if (n_seg == 0) return REGNN_OK;
    V2Args p{ptr, idx, nullptr, fs, fd, att, nullptr, s, nullptr, n_seg, H, D, slope};
    return launch_gatv2<0>(p, grid_for(n_seg, kBlock / v2_lpr(H, D)), plan, 0, stream);
}

int regnn_gatv2_score_bwd_dst(const int32_t* ptr, const int32_t* idx, const float* fs,
                              const float* fd, const float* att, const float* gs, int64_t n_seg,
                              int32_t H, int32_t D, float slope, float* gfd, float* att_slab,
                              int32_t slab_rows, const regnn_seg_plan* plan, hipStream_t stream) {
    if (!ptr || !idx || !fs || !fd || !att || !gs || !gfd || !att_slab || n_seg < 0 || H <= 0 ||
        D <= 0 || slab_rows <= 0)
        return REGNN_EINVAL;
    if (n_seg == 0) return REGNN_OK;
    V2Args p{ptr, idx, nullptr, fs, fd, att, gs, gfd, att_slab, n_seg, H, D, slope};
    const bool chunks = plan && plan->n_long > 0 && plan->n_chunk > 0;
    if (chunks && slab_rows < 2) return REGNN_EINVAL;
    int grid = grid_for(n_seg, kBlock / v2_lpr(H, D));
    const int cap = chunks ? slab_rows / 2 : slab_rows;   // with chunks: half the rows each pass
    if (grid > cap) grid = cap;
    return launch_gatv2<1>(p, grid, plan, slab_rows - grid, stream);
}

int regnn_gatv2_score_bwd_src(const int32_t* csc_ptr, const int32_t* csc_idx,
                              const int32_t* csc2csr, const float* fs, const float* fd,
                              const float* att, const float* gs, int64_t n_src, int32_t H,
                              int32_t D, float slope, float* gfs, const regnn_seg_plan* plan,
                              hipStream_t stream) {
    if (!csc_ptr || !csc_idx || !csc2csr || !fs || !fd || !att || !gs || !gfs || n_src < 0 ||
        H <= 0 || D <= 0)
        return REGNN_EINVAL;
    if (n_src == 0) return REGNN_OK;
    V2Args p{csc_ptr, csc_idx, csc2csr, fs, fd, att, gs, gfs, nullptr, n_src, H, D, slope};
    return launch_gatv2<2>(p, grid_for(n_src, kBlock / v2_lpr(H, D)), plan, 0, stream);
}

int regnn_edge_softmax_fwd(const int32_t* ptr, const float* s, const uint8_t* rel,
                           const float* ee_table, const float* gmax, float eps, int64_t n_seg,
                           int32_t H, float* a, const regnn_seg_plan* plan, hipStream_t stream) {
    if (!ptr || !s || !a || n_seg < 0 || (ee_table && !rel)) return REGNN_EINVAL;
    const int lg = sm_log2(H);
    if (lg < 0) return REGNN_EUNSUPPORTED;
    if (n_seg == 0) return REGNN_OK;
    if (const int rc = check_plan(plan, 2 * H)) return rc;
    const LongPlan P = long_plan(plan);
    hipLaunchKernelGGL(edge_softmax_fwd_kernel<0>, dim3(grid_for(n_seg, kBlock / kSmG)),
                       dim3(kBlock), 0, stream, ptr, s, rel, ee_table, gmax, eps, n_seg, H, lg, a,
                       P, nullptr, 0, 0);
    REGNN_LAUNCH_CHECK();
    if (P.n_chunk > 0) {
        const dim3 grid(grid_for(P.n_chunk, kBlock / kSmG));
        hipLaunchKernelGGL(edge_softmax_fwd_kernel<1>, grid, dim3(kBlock), 0, stream, ptr, s, rel,
                           ee_table, gmax, eps, n_seg, H, lg, a, P, nullptr, 0, 0);
        const int64_t base = run_tree(plan, 1, 2 * H, 0, H, 1, stream);
        hipLaunchKernelGGL(edge_softmax_fwd_kernel<2>, grid, dim3(kBlock), 0, stream, ptr, s, rel,
                           ee_table, gmax, eps, n_seg, H, lg, a, P, P.part, base,
                           plan->n_levels);
        REGNN_LAUNCH_CHECK();
    }
    return REGNN_OK;
}

int regnn_edge_softmax_bwd(const int32_t* ptr, const uint8_t* rel, const float* a,
                           const float* ga, int64_t n_seg, int32_t H, float* gz, float* slab,
                           int32_t n_rel, const regnn_seg_plan* plan, hipStream_t stream) {
    if (!ptr || !a || !ga || !gz || n_seg < 0 || (slab && (!rel || n_rel <= 0 || n_rel > 64)))
        return REGNN_EINVAL;
    const int lg = sm_log2(H);
    if (lg < 0) return REGNN_EUNSUPPORTED;
    if (n_seg == 0) return REGNN_OK;
    if (const int rc = check_plan(plan, H)) return rc;
    const LongPlan P = long_plan(plan);
    const size_t lds = slab ? size_t(n_rel) * kBlock * sizeof(float) : 0;
    // the slab's rows: the per-segment pass's blocks, then the chunk pass's (regnn_slab_rows()
    // = 2 kMaxGrid holds both grids)
    const int g0 = grid_for(n_seg, kBlock / kSmG);
    hipLaunchKernelGGL(edge_softmax_bwd_kernel<0>, dim3(g0), dim3(kBlock), lds, stream, ptr, rel,
                       a, ga, n_seg, H, lg, gz, slab, n_rel, P, nullptr, 0, 0);
    REGNN_LAUNCH_CHECK();
    if (P.n_chunk > 0) {
        const dim3 grid(grid_for(P.n_chunk, kBlock / kSmG));
        hipLaunchKernelGGL(edge_softmax_bwd_kernel<1>, grid, dim3(kBlock), 0, stream, ptr, rel, a,
                           ga, n_seg, H, lg, gz, nullptr, n_rel, P, nullptr, 0, 0);
        const int64_t base = run_tree(plan, 0, H, H, H, 1, stream);
        hipLaunchKernelGGL(edge_softmax_bwd_kernel<2>, grid, dim3(kBlock), lds, stream, ptr, rel,
                           a, ga, n_seg, H, lg, gz,
                           slab ? slab + int64_t(g0) * n_rel * H : nullptr, n_rel, P, P.part,
                           base, plan->n_levels);
        REGNN_LAUNCH_CHECK();
    }
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
