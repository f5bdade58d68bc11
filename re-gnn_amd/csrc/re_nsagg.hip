// Typed block aggregation of raw input rows: layer 0 of the neighbour-sampled REGNN at any hidden
// width (mag/regnn_ns.py:300-346 with the reference default hidden 512, mag/regnn_ns.py:43).
//
// The reference projects every sampled node's raw row through its type's Linear (group_input,
// mag/regnn_ns.py:300-326: ~280 k rows x 128 -> hidden per step at fan-out [25, 20]) and then
// through the first conv's weight (mag/regnn_layers.py:102) before the mean aggregation. Both
// maps are linear, so for target row v of layer 0's block
//     a_v = inv_v sum_e tab[r_e] (x_e W_t(e)^T + b_t(e)) W_0 + bias
//         = inv_v sum_t (S_vt W_t^T + w_vt b_t) W_0 + bias,
//     S_vt = sum_{e in v, type(src_e) = t} tab[r_e] x_src_e,   w_vt = sum_{same e} tab[r_e],
// and the projections run over the ~13 k target rows only. This file forms S and w from the raw
// input tables (the gather: each sampled edge reads its source's raw K-float row once) and, in
// the backward, the relation-table gradient
//     d tab[r] = sum_{e: r_e = r} (<x_src_e, gS_v,t(e)> + gw_v,t(e)).
// The GEMMs (S W_c, its two backward products) stay on hipBLASLt.
#include "regnn_common.h"

namespace regnn {
namespace nsagg {

constexpr int kMT = 8;                     // node types (REGNN_NSM_MAX_TYPES)

struct Tabs {
    const float* p[kMT];
};

template <int N>
__device__ __forceinline__ const float* pick_tab(const Tabs& t, int i) {
    const float* r = t.p[0];
#pragma unroll
    for (int k = 1; k < N; ++k)
        if (i == k) r = t.p[k];
    return r;
}

// one edge's metadata, formed by one lane of the row's group (its four dependent loads run in
// parallel over the row's edges) and broadcast to the group: source type, source row in its
// type's table, tab[r_e] (tab may be null), relation id
// (e_type / e_off: the sampler's per-edge source type and table row of a meta-only hop, read
// directly instead of through the local id, n_id, node type and local row)
struct EdgeSrc {
    const int32_t* idx; const int32_t* n_id; const int32_t* ntype; const int64_t* local;
    const int32_t* e_type; const int64_t* e_off;
};

template <int LPR>
__device__ __forceinline__ void edge_meta(const EdgeSrc& E, const uint8_t* rel, const float* tab,
                                          int e, int e1, int& t, int64_t& row, float& w, int& r) {
    t = 0; row = 0; w = 0.f; r = 0;
    if (e < e1) {
        r = rel[e];
        if (E.e_type) {
            t = E.e_type[e];
            row = E.e_off[e];
        } else {
            const int g = E.n_id[E.idx[e]];
            t = E.ntype[g];
            row = E.local[g];
        }
        w = tab ? tab[r] : 0.f;
    }
}

// S [n_rows][T][K] (row stride lds floats), w [n_rows][T] (row stride ldw). LPR = K / 4 lanes
// per row, 64 / LPR rows per wave.
template <int K, int NT>
__global__ void __launch_bounds__(kBlock)
typed_agg_kernel(const int32_t* __restrict__ ptr, EdgeSrc E, const uint8_t* __restrict__ rel,
                 const float* __restrict__ tab, Tabs xt, int T, int64_t n_rows,
                 float* __restrict__ S, float* __restrict__ wsum, int64_t lds, int64_t ldw) {
    constexpr int LPR = K / 4;
    constexpr int RPW = 64 / LPR;
    constexpr int UN = 4;
    const int lane = threadIdx.x & 63, l = lane % LPR, gl = lane - l;
    const int64_t rows_per_block = int64_t(kBlock / 64) * RPW;
    for (int64_t v0 = int64_t(blockIdx.x) * rows_per_block; v0 < n_rows;
         v0 += int64_t(gridDim.x) * rows_per_block) {
        const int64_t v = v0 + (threadIdx.x >> 6) * RPW + lane / LPR;
        if (v >= n_rows) continue;
        float4 acc[NT];
        float ws[NT];
#pragma unroll
        for (int k = 0; k < NT; ++k) {
            acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
            ws[k] = 0.f;
        }
        const int e0 = ptr[v], e1 = ptr[v + 1];
        for (int c = e0; c < e1; c += LPR) {
            int mt, mr;
            int64_t mrow;
            float mw;
            edge_meta<LPR>(E, rel, tab, c + l, e1, mt, mrow, mw, mr);
            const int m = min(LPR, e1 - c);
            for (int j = 0; j < m; j += UN) {
                float4 x[UN];
                int tt[UN];
                float ww[UN];
#pragma unroll
                for (int u = 0; u < UN; ++u) {
                    const int src = gl + min(j + u, m - 1);
                    tt[u] = __shfl(mt, src, 64);
                    const int64_t rw = __shfl(mrow, src, 64);
                    ww[u] = j + u < m ? __shfl(mw, src, 64) : 0.f;
                    x[u] = reinterpret_cast<const float4*>(pick_tab<NT>(xt, tt[u]))[rw * LPR + l];
                }
#pragma unroll
                for (int u = 0; u < UN; ++u) {
#pragma unroll
                    for (int k = 0; k < NT; ++k) {
                        if (tt[u] == k) {
                            acc[k].x = fmaf(ww[u], x[u].x, acc[k].x);
                            acc[k].y = fmaf(ww[u], x[u].y, acc[k].y);
                            acc[k].z = fmaf(ww[u], x[u].z, acc[k].z);
                            acc[k].w = fmaf(ww[u], x[u].w, acc[k].w);
                            ws[k] += ww[u];
                        }
                    }
                }
            }
        }
        float4* srow = reinterpret_cast<float4*>(S + v * lds);
#pragma unroll
        for (int k = 0; k < NT; ++k)
            if (k < T) srow[k * LPR + l] = acc[k];
        if (l < T) {
            float s = ws[0];
#pragma unroll
            for (int k = 1; k < NT; ++k)
                if (l == k) s = ws[k];
            wsum[v * ldw + l] = s;
        }
    }
}

// d tab[r] = sum_e <x_src_e, gS[v, t_e]> + gw[v, t_e]: relation bins per row group in LDS (lane 0
// of the group adds its entries in order; the group rows summed in group order), one slab row
// [n_rel] per block (the caller reduces the slab in a fixed order): bitwise reproducible
template <int K, int NT>
__global__ void __launch_bounds__(kBlock)
typed_agg_bwd_kernel(const int32_t* __restrict__ ptr, EdgeSrc E, const uint8_t* __restrict__ rel,
                     Tabs xt, int T, int64_t n_rows, const float* __restrict__ gS,
                     const float* __restrict__ gw, float* __restrict__ slab, int n_rel,
                     int64_t lds, int64_t ldw) {
    constexpr int LPR = K / 4;
    constexpr int RPW = 64 / LPR;
    constexpr int UN = 4;
    constexpr int NG = kBlock / LPR;
    __shared__ float gbins[NG][256];
    for (int i = threadIdx.x; i < NG * 256; i += kBlock) gbins[i >> 8][i & 255] = 0.f;
    __syncthreads();
    const int lane = threadIdx.x & 63, l = lane % LPR, gl = lane - l;
    float* bins = gbins[threadIdx.x / LPR];
    const int64_t rows_per_block = int64_t(kBlock / 64) * RPW;
    for (int64_t v0 = int64_t(blockIdx.x) * rows_per_block; v0 < n_rows;
         v0 += int64_t(gridDim.x) * rows_per_block) {
        const int64_t v = v0 + (threadIdx.x >> 6) * RPW + lane / LPR;
        if (v >= n_rows) continue;
        const int e0 = ptr[v], e1 = ptr[v + 1];
        if (e0 == e1) continue;
        float4 g[NT];
        const float4* grow = reinterpret_cast<const float4*>(gS + v * lds);
#pragma unroll
        for (int k = 0; k < NT; ++k) g[k] = k < T ? grow[k * LPR + l] : make_float4(0.f, 0.f, 0.f, 0.f);
        const float gwl = l < T ? gw[v * ldw + l] : 0.f;
        for (int c = e0; c < e1; c += LPR) {
            int mt, mr;
            int64_t mrow;
            float mw;
            edge_meta<LPR>(E, rel, nullptr, c + l, e1, mt, mrow, mw, mr);
            (void)mw;
            const int m = min(LPR, e1 - c);
            for (int j = 0; j < m; j += UN) {
                float4 x[UN];
                int tt[UN], rr[UN];
#pragma unroll
                for (int u = 0; u < UN; ++u) {
                    const int src = gl + min(j + u, m - 1);
                    tt[u] = __shfl(mt, src, 64);
                    rr[u] = __shfl(mr, src, 64);
                    const int64_t rw = __shfl(mrow, src, 64);
                    x[u] = reinterpret_cast<const float4*>(pick_tab<NT>(xt, tt[u]))[rw * LPR + l];
                }
#pragma unroll
                for (int u = 0; u < UN; ++u) {
                    float4 gg = g[0];
#pragma unroll
                    for (int k = 1; k < NT; ++k)
                        if (tt[u] == k) gg = g[k];
                    float d = x[u].x * gg.x + x[u].y * gg.y + x[u].z * gg.z + x[u].w * gg.w;
                    d = group_sum<LPR>(d);
                    const float b = __shfl(gwl, gl + tt[u], 64);
                    if (l == 0 && j + u < m) bins[rr[u]] += d + b;
                }
            }
        }
    }
    __syncthreads();
    for (int r = threadIdx.x; r < n_rel; r += kBlock) {
        float sr = 0.f;
        for (int k = 0; k < NG; ++k) sr += gbins[k][r];
        slab[int64_t(blockIdx.x) * n_rel + r] = sr;
    }
}

// ---- layer 0 from the sampler's per-type input sums (relation slots) -------------------------
// With one relation per (target type, source type) pair (ogbn-mag's schema), the outer hop's
// sampler (regnn_ns_hop_typed_sums, on its own stream ahead of the model) forms the parameter-free
// parts: U[v][t] = the unweighted sum of row v's sampled input rows of source type t, cnt[v][t]
// their count, x_self[v] the self loop's row and the slots' relations u_rel[v][t] (-1: none),
// u_rel[v][T] = the self loop's. Layer 0's operand [S | w | 0] is then
//     S_vt = tab[r_vt] U_vt + [t = t_self(v)] tab[r_self] x_self(v),
//     w_vt = tab[r_vt] cnt_vt + [t = t_self(v)] tab[r_self]
// (agg0's formula, re_nsm2.hip) -- one read of contiguous sums per row instead of a gather of
// every sampled row on the model's critical path. 32 lanes per row (K = 128: a float4 each), two
// rows per wave. Rows in [n, the next multiple of 128) are written as zeros (the GEMMs' live-row
// tiles read them), rows past that are left alone (nothing reads them).
constexpr int kSlotK = 128;

template <int NT>
__global__ void __launch_bounds__(kBlock)
slot_agg_kernel(const int32_t* __restrict__ sizes, int hop, const float* __restrict__ U,
                const float* __restrict__ cnt, const float* __restrict__ xself,
                const int32_t* __restrict__ urel, const float* __restrict__ tab, int n_et, int T,
                int Tp, int64_t cap, float* __restrict__ out, int64_t ld) {
    const int n = sizes[hop];
    const int64_t lim = min(cap, (int64_t(n) + 127) / 128 * 128);
    const int l = threadIdx.x & 31;
    for (int64_t v = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / 32; v < lim;
         v += int64_t(gridDim.x) * (kBlock / 32)) {
        float* o = out + v * ld;
        if (v >= n) {
#pragma unroll
            for (int t = 0; t < NT; ++t)
                if (t < T) *reinterpret_cast<float4*>(o + t * kSlotK + 4 * l) = make_float4(0.f, 0.f, 0.f, 0.f);
            if (l < Tp) o[T * kSlotK + l] = 0.f;
            continue;
        }
        const int32_t* ur = urel + v * (T + 1);
        const int rs = ur[T], ts = rs >= 0 ? rs - n_et : -1;
        const float ws = rs >= 0 ? tab[rs] : 0.f;
        const float4 xs = *reinterpret_cast<const float4*>(xself + v * kSlotK + 4 * l);
        float wl = 0.f;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            if (t >= T) continue;
            const int r = ur[t];
            const float wr = r >= 0 ? tab[r] : 0.f, wst = t == ts ? ws : 0.f;
            const float4 u = *reinterpret_cast<const float4*>(U + (v * T + t) * kSlotK + 4 * l);
            *reinterpret_cast<float4*>(o + t * kSlotK + 4 * l) =
                make_float4(fmaf(wst, xs.x, wr * u.x), fmaf(wst, xs.y, wr * u.y),
                            fmaf(wst, xs.z, wr * u.z), fmaf(wst, xs.w, wr * u.w));
            if (l == t) wl = fmaf(wr, cnt[v * T + t], wst);
        }
        if (l < Tp) o[T * kSlotK + l] = l < T ? wl : 0.f;
    }
}

// its relation-table gradient: d tab[r] = sum over (v, t) with r_vt = r of <U_vt, gS_vt> +
// cnt_vt gw_vt, and over v with r_self(v) = r of <x_self, gS_v,t_self> + gw_v,t_self. One slab
// row [n_rel] per block (launched with slab_rows blocks, 8 row groups each): each group adds its
// rows' terms into its own LDS bins in (t, then self) order, the groups summed in group order --
// bitwise reproducible; reduce the slab with regnn_rel_reduce.
template <int NT>
__global__ void __launch_bounds__(kBlock)
slot_agg_bwd_kernel(const int32_t* __restrict__ sizes, int hop, const float* __restrict__ U,
                    const float* __restrict__ cnt, const float* __restrict__ xself,
                    const int32_t* __restrict__ urel, const float* __restrict__ g, int64_t ld,
                    int n_et, int T, float* __restrict__ slab, int n_rel) {
    constexpr int NG = kBlock / 32;
    __shared__ float gbins[NG][256];
    for (int i = threadIdx.x; i < NG * 256; i += kBlock) gbins[i >> 8][i & 255] = 0.f;
    __syncthreads();
    const int n = sizes[hop];
    const int l = threadIdx.x & 31, grp = threadIdx.x / 32;
    float* bins = gbins[grp];
    for (int64_t v = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / 32; v < n;
         v += int64_t(gridDim.x) * NG) {
        const int32_t* ur = urel + v * (T + 1);
        const int rs = ur[T], ts = rs >= 0 ? rs - n_et : -1;
        const float* gr = g + v * ld;
        const float4 xs = *reinterpret_cast<const float4*>(xself + v * kSlotK + 4 * l);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            if (t >= T) continue;
            const int r = ur[t];
            const float4 gs = *reinterpret_cast<const float4*>(gr + t * kSlotK + 4 * l);
            const float4 u = *reinterpret_cast<const float4*>(U + (v * T + t) * kSlotK + 4 * l);
            const float gw = gr[T * kSlotK + t];
            if (r >= 0) {
                const float d = group_sum<32>(u.x * gs.x + u.y * gs.y + u.z * gs.z + u.w * gs.w);
                if (l == 0) bins[r] += fmaf(cnt[v * T + t], gw, d);
            }
            if (t == ts) {
                const float d = group_sum<32>(xs.x * gs.x + xs.y * gs.y + xs.z * gs.z + xs.w * gs.w);
                if (l == 0) bins[rs] += d + gw;
            }
        }
    }
    __syncthreads();
    for (int r = threadIdx.x; r < n_rel; r += kBlock) {
        float sr = 0.f;
        for (int k = 0; k < NG; ++k) sr += gbins[k][r];
        slab[int64_t(blockIdx.x) * n_rel + r] = sr;
    }
}

// ---- the mean aggregation of a block in the strided layout (regnn_ns_hop strided = 1) --------
// row i's edges at slots [i S, i S + cnt[i]] (sampled ones in CSR order, the self loop last), the
// slot order the CSR layout keeps: y[i] = inv[i] sum_e tab[rel_e] x[idx_e] + bias for live rows
// i < sizes[0], bias for the others. One wave per row, LPR lanes x VPL float4 per lane, the
// row's entries loaded lane-parallel and its source rows UN at a time in flight.
template <int VPL>
__global__ void __launch_bounds__(kBlock)
strided_spmm_kernel(const int32_t* __restrict__ live, const int32_t* __restrict__ cnt, int S,
                    const int32_t* __restrict__ idx, const uint8_t* __restrict__ rel,
                    const float* __restrict__ tab, const float* __restrict__ inv,
                    const float* __restrict__ bias, const float* __restrict__ x,
                    float* __restrict__ y, int64_t n_rows, int F) {
    constexpr int UN = 8;
    const int lane = threadIdx.x & 63;
    const int n = live[0];
    const int nv = F / 4;
    for (int64_t i = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / 64; i < n_rows;
         i += int64_t(gridDim.x) * (kBlock / 64)) {
        float4 acc[VPL];
#pragma unroll
        for (int q = 0; q < VPL; ++q) acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        const int m = i < n ? cnt[i] + 1 : 0;
        const int64_t base = i * S;
        const int my_u = lane < m ? idx[base + lane] : 0;
        const float my_w = lane < m ? (tab ? tab[rel[base + lane]] : 1.f) : 0.f;
        for (int j = 0; j < m; j += UN) {
            float4 xv[UN][VPL];
#pragma unroll
            for (int u = 0; u < UN; ++u) {
                const int uu = __shfl(my_u, min(j + u, m - 1), 64);
#pragma unroll
                for (int q = 0; q < VPL; ++q) {
                    const int c = lane + 64 * q;
                    xv[u][q] = c < nv ? reinterpret_cast<const float4*>(x + int64_t(uu) * F)[c]
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
#pragma unroll
            for (int u = 0; u < UN; ++u) {
                if (j + u >= m) continue;
                const float w = __shfl(my_w, j + u, 64);
#pragma unroll
                for (int q = 0; q < VPL; ++q) {
                    acc[q].x = fmaf(w, xv[u][q].x, acc[q].x);
                    acc[q].y = fmaf(w, xv[u][q].y, acc[q].y);
                    acc[q].z = fmaf(w, xv[u][q].z, acc[q].z);
                    acc[q].w = fmaf(w, xv[u][q].w, acc[q].w);
                }
            }
        }
        const float iv = i < n ? inv[i] : 0.f;
#pragma unroll
        for (int q = 0; q < VPL; ++q) {
            const int c = lane + 64 * q;
            if (c >= nv) continue;
            float4 b = bias ? reinterpret_cast<const float4*>(bias)[c] : make_float4(0.f, 0.f, 0.f, 0.f);
            b.x = fmaf(iv, acc[q].x, b.x);
            b.y = fmaf(iv, acc[q].y, b.y);
            b.z = fmaf(iv, acc[q].z, b.z);
            b.w = fmaf(iv, acc[q].w, b.w);
            reinterpret_cast<float4*>(y + i * F)[c] = b;
        }
    }
}

}  // namespace nsagg
}  // namespace regnn

using namespace regnn;
using namespace regnn::nsagg;

extern "C" {

static bool edge_src(const int32_t* idx, const int32_t* n_id, const int32_t* ntype,
                     const int64_t* local, const int32_t* e_type, const int64_t* e_off,
                     EdgeSrc& E) {
    E = EdgeSrc{idx, n_id, ntype, local, e_type, e_off};
    if (e_type || e_off) return e_type && e_off;
    return idx && n_id && ntype && local;
}

int regnn_ns_typed_agg(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                       const float* rel_table, const int32_t* n_id, const int32_t* ntype,
                       const int64_t* local, const int32_t* e_type, const int64_t* e_off,
                       const float* const* tables, int32_t n_types, int32_t K, int64_t n_rows,
                       float* S, float* wsum, int64_t ld_s, int64_t ld_w, hipStream_t stream) {
    EdgeSrc E;
    if (!ptr || !rel || !rel_table || !tables || !S || !wsum || n_types <= 0 || n_types > kMT ||
        n_rows < 0 || !edge_src(idx, n_id, ntype, local, e_type, e_off, E))
        return REGNN_EINVAL;
    if (ld_s < int64_t(n_types) * K || ld_s % 4 || reinterpret_cast<uintptr_t>(S) % 16 ||
        ld_w < n_types)
        return REGNN_EINVAL;
    Tabs xt{};
    for (int t = 0; t < n_types; ++t) {
        if (!tables[t]) return REGNN_EINVAL;
        xt.p[t] = tables[t];
    }
    if (n_rows == 0) return REGNN_OK;
    const int lpr = K / 4;
    const int64_t rpb = int64_t(kBlock / 64) * (64 / lpr);
    int64_t grid = (n_rows + rpb - 1) / rpb;
    if (grid > kMaxGrid) grid = kMaxGrid;
#define AGG_CASE(KK, N)                                                                        \
    if (K == KK && n_types <= N) {                                                             \
        hipLaunchKernelGGL((typed_agg_kernel<KK, N>), dim3((unsigned)grid), dim3(kBlock), 0,   \
                           stream, ptr, E, rel, rel_table, xt, n_types, n_rows, S, wsum, ld_s, \
                           ld_w);                                                              \
        REGNN_LAUNCH_CHECK();                                                                  \
        return REGNN_OK;                                                                       \
    }
    AGG_CASE(64, 4) AGG_CASE(64, 8) AGG_CASE(128, 4) AGG_CASE(128, 8)
#undef AGG_CASE
    return REGNN_EUNSUPPORTED;
}

int regnn_ns_typed_agg_bwd(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                           const int32_t* n_id, const int32_t* ntype, const int64_t* local,
                           const int32_t* e_type, const int64_t* e_off,
                           const float* const* tables, int32_t n_types, int32_t K, int64_t n_rows,
                           const float* gS, const float* gw, int64_t ld_s, int64_t ld_w,
                           float* slab, int32_t n_rel, int32_t slab_rows, hipStream_t stream) {
    EdgeSrc E;
    if (!ptr || !rel || !tables || !gS || !gw || !slab || n_types <= 0 || n_types > kMT ||
        n_rows < 0 || n_rel <= 0 || n_rel > 256 || slab_rows <= 0 ||
        !edge_src(idx, n_id, ntype, local, e_type, e_off, E))
        return REGNN_EINVAL;
    if (ld_s < int64_t(n_types) * K || ld_s % 4 || reinterpret_cast<uintptr_t>(gS) % 16 ||
        ld_w < n_types)
        return REGNN_EINVAL;
    Tabs xt{};
    for (int t = 0; t < n_types; ++t) {
        if (!tables[t]) return REGNN_EINVAL;
        xt.p[t] = tables[t];
    }
#define BWD_CASE(KK, N)                                                                        \
    if (K == KK && n_types <= N) {                                                             \
        hipLaunchKernelGGL((typed_agg_bwd_kernel<KK, N>), dim3((unsigned)slab_rows),           \
                           dim3(kBlock), 0, stream, ptr, E, rel, xt, n_types, n_rows, gS, gw,  \
                           slab, n_rel, ld_s, ld_w);                                           \
        REGNN_LAUNCH_CHECK();                                                                  \
        return REGNN_OK;                                                                       \
    }
    BWD_CASE(64, 4) BWD_CASE(64, 8) BWD_CASE(128, 4) BWD_CASE(128, 8)
#undef BWD_CASE
    return REGNN_EUNSUPPORTED;
}

int regnn_ns_spmm_strided_fwd(const int32_t* live, const int32_t* cnt, int32_t stride,
                              const int32_t* idx, const uint8_t* rel, const float* rel_table,
                              const float* inv, const float* bias, const float* x, float* y,
                              int64_t n_rows, int32_t F, hipStream_t stream) {
    if (!live || !cnt || !idx || !inv || !x || !y || (rel_table && !rel) || n_rows < 0 ||
        stride < 1 || stride > 64 || F <= 0 || F % 4)
        return REGNN_EINVAL;
    if (reinterpret_cast<uintptr_t>(x) % 16 || reinterpret_cast<uintptr_t>(y) % 16 ||
        (bias && reinterpret_cast<uintptr_t>(bias) % 16))
        return REGNN_EINVAL;
    if (n_rows == 0) return REGNN_OK;
    int64_t grid = (n_rows + kBlock / 64 - 1) / (kBlock / 64);
    if (grid > kMaxGrid) grid = kMaxGrid;
    const int vpl = (F / 4 + 63) / 64;
#define SSP_CASE(V)                                                                             \
    if (vpl <= V) {                                                                             \
        hipLaunchKernelGGL((strided_spmm_kernel<V>), dim3(unsigned(grid)), dim3(kBlock), 0,     \
                           stream, live, cnt, stride, idx, rel, rel_table, inv, bias, x, y,     \
                           n_rows, F);                                                          \
        REGNN_LAUNCH_CHECK();                                                                   \
        return REGNN_OK;                                                                        \
    }
    SSP_CASE(1) SSP_CASE(2) SSP_CASE(4)
#undef SSP_CASE
    return REGNN_EUNSUPPORTED;
}

int regnn_ns_slot_agg(const int32_t* sizes, int32_t hop, const float* U, const float* cnt,
                      const float* x_self, const int32_t* u_rel, const float* rel_table,
                      int32_t n_et, int32_t n_types, int32_t K, int64_t cap, float* out,
                      int64_t ld, hipStream_t stream) {
    if (!sizes || !U || !cnt || !x_self || !u_rel || !rel_table || !out || hop < 0 || hop > 7 ||
        n_et < 0 || n_types < 1 || cap < 0)
        return REGNN_EINVAL;
    if (K != kSlotK || n_types > 4) return REGNN_EUNSUPPORTED;
    const int Tp = (n_types + 3) & ~3;
    if (ld < int64_t(n_types) * K + Tp || ld % 4 || reinterpret_cast<uintptr_t>(out) % 16 ||
        reinterpret_cast<uintptr_t>(U) % 16 || reinterpret_cast<uintptr_t>(x_self) % 16)
        return REGNN_EINVAL;
    if (cap == 0) return REGNN_OK;
    int64_t grid = (cap + kBlock / 32 - 1) / (kBlock / 32);
    if (grid > kMaxGrid) grid = kMaxGrid;
    hipLaunchKernelGGL((slot_agg_kernel<4>), dim3(unsigned(grid)), dim3(kBlock), 0, stream, sizes,
                       hop, U, cnt, x_self, u_rel, rel_table, n_et, n_types, Tp, cap, out, ld);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

int regnn_ns_slot_agg_bwd(const int32_t* sizes, int32_t hop, const float* U, const float* cnt,
                          const float* x_self, const int32_t* u_rel, const float* g, int64_t ld,
                          int32_t n_et, int32_t n_types, int32_t K, float* slab, int32_t n_rel,
                          int32_t slab_rows, hipStream_t stream) {
    if (!sizes || !U || !cnt || !x_self || !u_rel || !g || !slab || hop < 0 || hop > 7 ||
        n_et < 0 || n_types < 1 || n_rel <= 0 || n_rel > 256 || slab_rows <= 0)
        return REGNN_EINVAL;
    if (K != kSlotK || n_types > 4) return REGNN_EUNSUPPORTED;
    if (ld < int64_t(n_types) * K + n_types || ld % 4 || reinterpret_cast<uintptr_t>(g) % 16 ||
        reinterpret_cast<uintptr_t>(U) % 16 || reinterpret_cast<uintptr_t>(x_self) % 16)
        return REGNN_EINVAL;
    hipLaunchKernelGGL((slot_agg_bwd_kernel<4>), dim3(unsigned(slab_rows)), dim3(kBlock), 0,
                       stream, sizes, hop, U, cnt, x_self, u_rel, g, ld, n_et, n_types, slab,
                       n_rel);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

}  // extern "C"
