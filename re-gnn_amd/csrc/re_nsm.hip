// Fused neighbour-sampled (NS) model step of the ogbn-mag path (regnn_nsm_step, regnn_hip.h):
// the REGNN of mag/regnn_ns.py:216-346 ('regcn', self_loop_type 2, LayerNorm, hidden 64) with
// its loss and backward over the blocks regnn_ns_hop wrote, as eight launches for two layers.
// Every kernel reads the batch's counts from `sizes` (device) and leaves rows past them alone,
// so the whole step is one HIP-graph replay with no host synchronisation.
//
//   prep        W_c[t] = lins[t].weight^T convs[0].weight, b_c[t] = lins[t].bias convs[0].weight,
//               relation tables LeakyReLU(alpha * rw_l)                (mag/regnn_layers.py:110)
//   agg0        layer 0 = group_input's per-type Linear + the first conv (mag/regnn_ns.py:300-326,
//               regnn_layers.py:80-150): the input rows aggregated per source type, then
//               projected per target row and type with the composed map; LayerNorm, relu,
//               dropout, then x @ W_1 of the next layer
//   agg         layers 1 .. L-2: mean aggregation with the relation table + bias, LayerNorm,
//               relu, dropout, x @ W_{l+1}                   (regnn_layers.py:129-148, :341-343)
//   head        layer L-1 as above, then out_lin, log_softmax, nll_loss (mean) and their
//               backward down to the pre-LayerNorm rows                   (regnn_ns.py:345, 404)
//   agg_bwd     layer l >= 1: transposed block aggregation (float atomics: a sampled block has
//               no CSC) and the relation-table dots
//   post_bwd    x @ W_{l+1} backward (its weight gradient per block), dropout / relu / LayerNorm
//               backward of layer l
//   bwd0, rel0  layer 0: the composed map's gradient per target row and type, and the
//               relation-table dots edge by edge (no source-row gradient, no atomics)
//   finalize    fixed-order reductions of every per-row / per-block partial into the gradients
//   chain       chain rule of the composed map onto lins[t] and convs[0].weight
#include "re_nsm_common.h"

namespace regnn {
namespace nsm {

// ---------------------------------------------------------------------------------------------
// prep: composed first map and the relation tables (deterministic fixed-order dots)
__global__ void __launch_bounds__(64)
prep_kernel(int T, int K, Ptrs lin_w, Ptrs lin_b, const float* __restrict__ w0, Ptrs rw,
            int L, Ints n_rel, float alpha, float* __restrict__ wc,
            float* __restrict__ tabs) {
    const int j = threadIdx.x;
    const int b = blockIdx.x;
    if (b < T * (K + 1)) {
        const int t = b / (K + 1), k = b - t * (K + 1);
        float s = 0.f;
        if (k < K) {
            const float* W = pick(lin_w.p, t);
#pragma unroll 32                                     // operand loads in flight, not one by one
            for (int o = 0; o < F; ++o) s = fmaf(W[int64_t(o) * K + k], w0[o * F + j], s);
        } else {
            const float* bb = pick(lin_b.p, t);
#pragma unroll 32
            for (int o = 0; o < F; ++o) s = fmaf(bb[o], w0[o * F + j], s);
        }
        // wcT[t]: W_c[t]^T row-major [64][K], then b_c[t] [64]
        float* o = wc + int64_t(t) * (K + 1) * F;
        if (k < K) o[int64_t(j) * K + k] = s;
        else o[int64_t(K) * F + j] = s;
        return;
    }
    const int l = b - T * (K + 1);
    if (l >= L) return;
    const int nr = pick(n_rel.v, l);
    float v = 0.f;
    if (j < nr) {
        const float x = pick(rw.p, l)[j] * alpha;
        v = x > 0.f ? x : 0.01f * x;                      // F.leaky_relu default slope
    }
    tabs[l * F + j] = v;
}

// ---------------------------------------------------------------------------------------------
// agg0 (layer 0, L >= 2): aggregate first, then project. With xs0[u] = x_u W_c[t_u] + b_c[t_u]
// (the composed first map of node type t_u), layer 0's mean aggregation regroups by source type:
//   a_v = inv_v (sum_t S_vt W_c[t] + w_vt b_c[t]) + bias,  S_vt = sum_{e in v, t_u = t} tab[r_e] x_u,
//   w_vt = sum_{e in v, t_u = t} tab[r_e],
// so the input rows are gathered once per edge (K wide) and the projection runs per target row
// and type (fp32 MFMA) instead of per source row. 16 target rows per block:
//   gather  16 lanes per row (K/64 float4 each): every edge's (type, table row) as the sampler
//           wrote them, loaded by the row's lanes together; the weighted row added to its
//           type's slot of the row in LDS; S, w to HBM for the backward;
//   project wave w -> output features 16w .. +15, D[v][j] += S_vt[k] W_c[t][k][j] over t and k
//           (lane (c, q): A = S[c][16b + 4q + i] from LDS, B = W_c^T[16w + c][16b + 4q + i] from
//           L2, the next type's columns loaded during this type's products);
//   epilogue as agg: LayerNorm, relu, dropout, then x @ W_1 of the next layer.

struct Agg0Args {
    const int32_t* sizes; int hop;
    const int32_t* ptr; const uint8_t* rel; const float* inv;
    const int32_t* edge_type; const int64_t* edge_off; Ptrs xt; int T;
    const float* wc;                       // prep's W_c[t]^T [64][K] | b_c[t] [64] per type
    const float* tab; const float* bias; const float* ln_w; const float* ln_b;
    const int64_t* state; Drop drop;
    const float* w_next;
    const int32_t* n_id; const int64_t* labels; float* nvalid;
    float* s_agg; float* s_w;
    float* a; float* stats; float* xs_next; float* gxs_next;
    // relation-slot mode (RS): s_agg / s_w hold the unweighted sums / counts of the non-self
    // edges per source type, u_self the self loop's input row, u_rel [n][T + 1] the relation of
    // each slot (-1: none; slot T: the self loop)
    int n_et; float* u_self; int32_t* u_rel;
};

// LDS: S tile [16][T*K + 4] (after the projection: W_1 [64][64] and the h rows [16][64]) |
// s_w [16][MT] | pre-LN rows [16][64] | relation table [64]
inline size_t agg0_lds(int T, int K) {
    const size_t st = size_t(16) * (T * K + 4);
    return ((st > size_t(F * F + 16 * F) ? st : size_t(F * F + 16 * F)) + 16 * MT + 16 * F + F) *
           sizeof(float);
}

// RS (relation slots, when every (target type, source type) pair has at most one relation
// besides the self loop): the input rows are summed per source type WITHOUT the relation weight
// (U_vt; the self loop's row x_v kept apart), so that S_vt = tab[r_vt] U_vt + [t = type(v)]
// tab[r_self] x_v and the relation-table gradient needs no second gather of the edges' rows:
// d tab[r_vt] = <U_vt, Z_vt> + cnt_vt beta_vt, d tab[r_self] = <x_v, Z_v,type(v)> + beta (bwd0).
template <int K, int NT, bool RS>          // NT: per-type register accumulators (T <= NT <= MT)
__global__ void __launch_bounds__(kBlock) agg0_kernel(Agg0Args A) {
    constexpr int VPL = K / 64;            // float4 per lane of a K-wide row (16 lanes per row)
    constexpr int KB = K / 16;             // float4 steps of the projection per type
    extern __shared__ float sm[];
    const int T = A.T;
    const int SR = T * K + 4;              // S tile row stride: rows 4 banks apart
    float* St = sm;                        // [16][SR]
    float* Wn = sm;                        // after the projection: [F][F]
    float* hrow = sm + F * F;              //                        [16][F]
    const int st_floats = max(16 * SR, F * F + 16 * F);
    float* sw = sm + st_floats;            // [16][MT]
    float* at = sw + 16 * MT;              // [16][F] pre-LN rows
    float* tab = at + 16 * F;              // [F]
    if (threadIdx.x < F) tab[threadIdx.x] = A.tab[threadIdx.x];
    const int n = A.sizes[A.hop];
    __syncthreads();
    const int l = threadIdx.x & 15, sub = threadIdx.x >> 4, gl = threadIdx.x & 48;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4;
    const uint32_t key = A.drop.on ? layer_key(A.state, 0) : 0u;
    const float4 gw = reinterpret_cast<const float4*>(A.ln_w)[l];
    const float4 gb = reinterpret_cast<const float4*>(A.ln_b)[l];
    for (int base = blockIdx.x * 16; base < n; base += gridDim.x * 16) {
        // ---- gather: S_vt and w_vt accumulated per type in registers (each lane its own
        // 4 * VPL features), then the row's S tile written to LDS
        const int v = base + sub;
        // (per-type sums in registers: measured faster than a read-modify-write of the LDS
        // tile per edge)
        float wsum[NT];
        float4 racc[NT][VPL];
        int rel_t[NT];                             // RS: each slot's relation (-1: none)
        float4 xself[VPL];                         // RS: the self loop's input row
        int r_self = -1;
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) {
            wsum[tt] = 0.f;
            rel_t[tt] = -1;
#pragma unroll
            for (int p = 0; p < VPL; ++p) racc[tt][p] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int p = 0; p < VPL; ++p) xself[p] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (v < n) {
            const int e0 = A.ptr[v], e1 = A.ptr[v + 1];
            for (int c0 = e0; c0 < e1; c0 += 16) {
                const int m = min(16, e1 - c0);
                int my_t = 0, my_lo = 0;           // table rows < 2^31 (checked by the host)
                float my_w = 0.f;
                int my_r = 0;
                if (l < m) {
                    my_t = A.edge_type[c0 + l];
                    my_lo = int(A.edge_off[c0 + l]);
                    my_r = A.rel[c0 + l];
                    my_w = tab[my_r];
                }
                // UN edges' rows in flight per lane, then their accumulation in edge order
                constexpr int UN = 8;
                for (int j = 0; j < m; j += UN) {
                    int t[UN], ru[UN];
                    float wt[UN];
                    float4 x[UN][VPL];
#pragma unroll
                    for (int u = 0; u < UN; ++u) {
                        const int jj = min(j + u, m - 1);
                        t[u] = __shfl(my_t, gl + jj, 64);
                        if constexpr (RS) ru[u] = __shfl(my_r, gl + jj, 64);
                        else wt[u] = __shfl(my_w, gl + jj, 64);
                        const int64_t lo = __shfl(my_lo, gl + jj, 64);
                        const float* xr = pick(A.xt.p, t[u]) + lo * K + 4 * l;
#pragma unroll
                        for (int p = 0; p < VPL; ++p) x[u][p] = *reinterpret_cast<const float4*>(xr + 64 * p);
                        if (j + u >= m) t[u] = -1;     // padding: loaded (a valid row), not added
                    }
#pragma unroll
                    for (int u = 0; u < UN; ++u) {
                        if (t[u] < 0) continue;
                        if constexpr (RS) {
                            if (ru[u] >= A.n_et) {         // the self loop (one per row)
                                r_self = ru[u];
#pragma unroll
                                for (int p = 0; p < VPL; ++p) xself[p] = x[u][p];
                                continue;
                            }
                        }
#pragma unroll
                        for (int tt = 0; tt < NT; ++tt) {
                            if (tt != t[u]) continue;
                            if constexpr (RS) {
                                wsum[tt] += 1.f;
                                rel_t[tt] = ru[u];
#pragma unroll
                                for (int p = 0; p < VPL; ++p) {
                                    racc[tt][p].x += x[u][p].x;
                                    racc[tt][p].y += x[u][p].y;
                                    racc[tt][p].z += x[u][p].z;
                                    racc[tt][p].w += x[u][p].w;
                                }
                            } else {
                                wsum[tt] += wt[u];
#pragma unroll
                                for (int p = 0; p < VPL; ++p) {
                                    racc[tt][p].x = fmaf(wt[u], x[u][p].x, racc[tt][p].x);
                                    racc[tt][p].y = fmaf(wt[u], x[u][p].y, racc[tt][p].y);
                                    racc[tt][p].z = fmaf(wt[u], x[u][p].z, racc[tt][p].z);
                                    racc[tt][p].w = fmaf(wt[u], x[u][p].w, racc[tt][p].w);
                                }
                            }
                        }
                    }
                }
            }
        }
        // the projection's first W_c fragment and W_1 (both independent of the gather) are
        // requested before the S tile's stores and barrier, so their L2 latency overlaps them
        constexpr int HB = KB / 2;             // float4 steps per half type
        float4 bcur[HB], bnext[HB];
        auto bload = [&](int step, float4 (&dst)[HB]) {
            const int tt = step >> 1, h0 = (step & 1) * HB;
            const float* wt = A.wc + int64_t(tt) * (K + 1) * F + (16 * w + c) * K + 4 * q + 16 * h0;
#pragma unroll
            for (int b = 0; b < HB; ++b) dst[b] = *reinterpret_cast<const float4*>(wt + 16 * b);
        };
        bload(0, bcur);
        float4 wn[F * F / 4 / kBlock];         // W_1, staged into the S tile once it is read
#pragma unroll
        for (int i = 0; i < F * F / 4 / kBlock; ++i)
            wn[i] = reinterpret_cast<const float4*>(A.w_next)[threadIdx.x + kBlock * i];
        const int tau = r_self - A.n_et;           // RS: the row's node type
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) {
            if (tt < T) {
                float wr = 1.f, ws = 0.f;              // RS: S = wr U + ws x_self
                if constexpr (RS) {
                    wr = rel_t[tt] >= 0 ? tab[rel_t[tt]] : 0.f;
                    ws = (tt == tau) ? tab[r_self] : 0.f;
                }
#pragma unroll
                for (int p = 0; p < VPL; ++p) {
                    float4 sv = racc[tt][p];
                    if constexpr (RS)
                        sv = make_float4(fmaf(ws, xself[p].x, wr * sv.x), fmaf(ws, xself[p].y, wr * sv.y),
                                         fmaf(ws, xself[p].z, wr * sv.z), fmaf(ws, xself[p].w, wr * sv.w));
                    *reinterpret_cast<float4*>(St + sub * SR + tt * K + 4 * l + 64 * p) = sv;
                    if (v < n)
                        *reinterpret_cast<float4*>(A.s_agg + (int64_t(v) * T + tt) * K + 4 * l + 64 * p) =
                            racc[tt][p];
                }
                if (l == 0) {
                    sw[sub * MT + tt] = RS ? fmaf(wr, wsum[tt], ws) : wsum[tt];
                    if (v < n) {
                        A.s_w[int64_t(v) * T + tt] = wsum[tt];
                        if constexpr (RS) A.u_rel[int64_t(v) * (T + 1) + tt] = rel_t[tt];
                    }
                }
            }
        }
        if constexpr (RS) {
            if (v < n) {
#pragma unroll
                for (int p = 0; p < VPL; ++p)
                    *reinterpret_cast<float4*>(A.u_self + int64_t(v) * K + 4 * l + 64 * p) = xself[p];
                if (l == 0) A.u_rel[int64_t(v) * (T + 1) + T] = r_self;
            }
        }
        __syncthreads();
        // ---- project: D[v][j] = sum_t S_vt W_c[t]  (v = 4q + r, j = 16w + c); type t + 1's
        // W_c columns are loaded while type t's products run
        f32x4 d = {0.f, 0.f, 0.f, 0.f};
        for (int step = 0; step < 2 * T; ++step) {
            if (step + 1 < 2 * T) bload(step + 1, bnext);
            const float* sa = St + c * SR + (step >> 1) * K + 16 * (step & 1) * HB + 4 * q;
#pragma unroll
            for (int b = 0; b < HB; ++b) {
                const float4 av = *reinterpret_cast<const float4*>(sa + 16 * b);
                d = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bcur[b].x, d, 0, 0, 0);
                d = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, bcur[b].y, d, 0, 0, 0);
                d = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, bcur[b].z, d, 0, 0, 0);
                d = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, bcur[b].w, d, 0, 0, 0);
            }
#pragma unroll
            for (int b = 0; b < HB; ++b) bcur[b] = bnext[b];
        }
        {
            const int j = 16 * w + c;
            const float bj = A.bias[j];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int vr = 4 * q + r;
                float bsum = 0.f;
                for (int tt = 0; tt < T; ++tt)
                    bsum = fmaf(sw[vr * MT + tt], A.wc[int64_t(tt) * (K + 1) * F + K * F + j], bsum);
                const int vv = base + vr;
                const float iv = vv < n ? A.inv[vv] : 0.f;
                at[vr * F + j] = fmaf(iv, d[r] + bsum, bj);
            }
        }
        __syncthreads();                       // S tile free: W_1 and the h rows go there
#pragma unroll
        for (int i = 0; i < F * F / 4 / kBlock; ++i)
            reinterpret_cast<float4*>(Wn)[threadIdx.x + kBlock * i] = wn[i];
        // ---- epilogue (agg_kernel's): LayerNorm, relu, dropout, x @ W_1
        const bool act = v < n;
        if (act) {
            const float4 a4 = *reinterpret_cast<const float4*>(at + sub * F + 4 * l);
            const float a[4] = {a4.x, a4.y, a4.z, a4.w};
            *reinterpret_cast<float4*>(A.a + int64_t(v) * F + 4 * l) = a4;
            const float mean = group_sum<16>(a[0] + a[1] + a[2] + a[3]) * (1.f / F);
            const float dd[4] = {a[0] - mean, a[1] - mean, a[2] - mean, a[3] - mean};
            const float var = group_sum<16>(dd[0] * dd[0] + dd[1] * dd[1] + dd[2] * dd[2] + dd[3] * dd[3]) * (1.f / F);
            const float rstd = rsqrtf(var + kLnEps);
            if (l == 0) reinterpret_cast<float2*>(A.stats)[v] = make_float2(mean, rstd);
            const float gws[4] = {gw.x, gw.y, gw.z, gw.w}, gbs[4] = {gb.x, gb.y, gb.z, gb.w};
            float mk[4];
            drop_factors(key, A.drop, v, l, mk);
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) {
                const float y = fmaf(dd[cc] * rstd, gws[cc], gbs[cc]);
                hrow[sub * F + 4 * l + cc] = fmaxf(y, 0.f) * mk[cc];
            }
        }
        __syncthreads();
        if (act) {
            float o0 = 0.f, o1 = 0.f, o2 = 0.f, o3 = 0.f;
#pragma unroll 8
            for (int k = 0; k < F; ++k) {
                const float hk = hrow[sub * F + k];
                const float4 wv = *reinterpret_cast<const float4*>(Wn + k * F + 4 * l);
                o0 = fmaf(hk, wv.x, o0); o1 = fmaf(hk, wv.y, o1);
                o2 = fmaf(hk, wv.z, o2); o3 = fmaf(hk, wv.w, o3);
            }
            *reinterpret_cast<float4*>(A.xs_next + int64_t(v) * F + 4 * l) = make_float4(o0, o1, o2, o3);
            *reinterpret_cast<float4*>(A.gxs_next + int64_t(v) * F + 4 * l) = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// agg (layer l < L-1): 16 lanes per row (4 features each), 16 rows per block. a = inv * sum_e
// tab[rel] xs[idx] + bias; LayerNorm; relu; dropout -> h; xs_next = h W_next (W_next in LDS).
struct AggArgs {
    const int32_t* sizes; int hop;
    const int32_t* ptr; const int32_t* idx; const uint8_t* rel; const float* inv;
    const float* tab; const float* xs; const float* bias; const float* ln_w; const float* ln_b;
    const int64_t* state; int layer; Drop drop;
    const float* w_next;
    float* a; float* stats; float* xs_next; float* gxs_next;
};

__global__ void __launch_bounds__(kBlock) agg_kernel(AggArgs A) {
    __shared__ float Wn[F * F];            // [k][j], read as float4 along j (broadcast per k)
    __shared__ float hrow[16][F];
    __shared__ float tab[F];
    for (int i = threadIdx.x; i < F * F / 4; i += kBlock)
        reinterpret_cast<float4*>(Wn)[i] = reinterpret_cast<const float4*>(A.w_next)[i];
    if (threadIdx.x < F) tab[threadIdx.x] = A.tab[threadIdx.x];
    __syncthreads();
    const int n = A.sizes[A.hop];
    const int l = threadIdx.x & 15, sub = threadIdx.x >> 4;
    const uint32_t key = A.drop.on ? layer_key(A.state, A.layer) : 0u;
    const float4 bias = reinterpret_cast<const float4*>(A.bias)[l];
    const float4 gw = reinterpret_cast<const float4*>(A.ln_w)[l];
    const float4 gb = reinterpret_cast<const float4*>(A.ln_b)[l];
    for (int base = blockIdx.x * 16; base < n; base += gridDim.x * 16) {
        const int v = base + sub;
        const bool act = v < n;
        if (act) {
            float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
            const int e0 = A.ptr[v], e1 = A.ptr[v + 1];
            const int gl = threadIdx.x & 48;          // first lane of this row's 16-lane group
            for (int c0 = e0; c0 < e1; c0 += 16) {   // the group loads 16 edges' ids at once
                const int m = min(16, e1 - c0);
                const int my_u = l < m ? A.idx[c0 + l] : 0;
                const int my_r = l < m ? int(A.rel[c0 + l]) : 0;
                int j = 0;
                for (; j + 2 <= m; j += 2) {
                    const int u0 = __shfl(my_u, gl + j, 64), u1 = __shfl(my_u, gl + j + 1, 64);
                    const float w0 = tab[__shfl(my_r, gl + j, 64)];
                    const float w1 = tab[__shfl(my_r, gl + j + 1, 64)];
                    const float4 x0 = *reinterpret_cast<const float4*>(A.xs + int64_t(u0) * F + 4 * l);
                    const float4 x1 = *reinterpret_cast<const float4*>(A.xs + int64_t(u1) * F + 4 * l);
                    s0 = fmaf(w0, x0.x, s0); s1 = fmaf(w0, x0.y, s1);
                    s2 = fmaf(w0, x0.z, s2); s3 = fmaf(w0, x0.w, s3);
                    s0 = fmaf(w1, x1.x, s0); s1 = fmaf(w1, x1.y, s1);
                    s2 = fmaf(w1, x1.z, s2); s3 = fmaf(w1, x1.w, s3);
                }
                if (j < m) {
                    const int u0 = __shfl(my_u, gl + j, 64);
                    const float w0 = tab[__shfl(my_r, gl + j, 64)];
                    const float4 x0 = *reinterpret_cast<const float4*>(A.xs + int64_t(u0) * F + 4 * l);
                    s0 = fmaf(w0, x0.x, s0); s1 = fmaf(w0, x0.y, s1);
                    s2 = fmaf(w0, x0.z, s2); s3 = fmaf(w0, x0.w, s3);
                }
            }
            const float iv = A.inv[v];
            const float a[4] = {fmaf(iv, s0, bias.x), fmaf(iv, s1, bias.y), fmaf(iv, s2, bias.z),
                                fmaf(iv, s3, bias.w)};
            *reinterpret_cast<float4*>(A.a + int64_t(v) * F + 4 * l) = make_float4(a[0], a[1], a[2], a[3]);
            const float mean = group_sum<16>(a[0] + a[1] + a[2] + a[3]) * (1.f / F);
            const float d[4] = {a[0] - mean, a[1] - mean, a[2] - mean, a[3] - mean};
            const float var = group_sum<16>(d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3]) * (1.f / F);
            const float rstd = rsqrtf(var + kLnEps);
            if (l == 0) reinterpret_cast<float2*>(A.stats)[v] = make_float2(mean, rstd);
            const float gws[4] = {gw.x, gw.y, gw.z, gw.w}, gbs[4] = {gb.x, gb.y, gb.z, gb.w};
            float m[4];
            drop_factors(key, A.drop, v, l, m);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const float y = fmaf(d[c] * rstd, gws[c], gbs[c]);
                hrow[sub][4 * l + c] = fmaxf(y, 0.f) * m[c];
            }
        }
        __syncthreads();
        if (act) {
            float o0 = 0.f, o1 = 0.f, o2 = 0.f, o3 = 0.f;
#pragma unroll 8
            for (int k = 0; k < F; ++k) {
                const float hk = hrow[sub][k];
                const float4 w = *reinterpret_cast<const float4*>(Wn + k * F + 4 * l);
                o0 = fmaf(hk, w.x, o0); o1 = fmaf(hk, w.y, o1);
                o2 = fmaf(hk, w.z, o2); o3 = fmaf(hk, w.w, o3);
            }
            *reinterpret_cast<float4*>(A.xs_next + int64_t(v) * F + 4 * l) = make_float4(o0, o1, o2, o3);
            *reinterpret_cast<float4*>(A.gxs_next + int64_t(v) * F + 4 * l) = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// LayerNorm / relu / dropout backward of one row held one feature per lane (wave per row):
// g = d loss / d (dropped relu output); writes ga (d / d pre-LN row), gy, gy * xhat.
__device__ __forceinline__ void ln_relu_drop_bwd(float g, float xhat, float rstd, float gw,
                                                 float gb, float mfac, float* ga, float* gy,
                                                 float* gyx) {
    const float y = fmaf(xhat, gw, gb);
    const float g_y = y > 0.f ? g * mfac : 0.f;
    const float gx = g_y * gw;
    const float m1 = wave_sum(gx) * (1.f / F);
    const float m2 = wave_sum(gx * xhat) * (1.f / F);
    *ga = rstd * (gx - m1 - xhat * m2);
    *gy = g_y;
    *gyx = g_y * xhat;
}

// keep factor of feature f (lane) of row `row`
__device__ __forceinline__ float lane_drop(uint32_t key, const Drop& d, int64_t row, int f) {
    float m[4];
    drop_factors(key, d, row, f >> 2, m);
    return (f & 3) == 0 ? m[0] : (f & 3) == 1 ? m[1] : (f & 3) == 2 ? m[2] : m[3];
}

// ---------------------------------------------------------------------------------------------
// head: the last layer + out_lin + log_softmax + nll + backward down to the pre-LN rows (ga),
// 16 target rows per block, the three products with out_lin.weight on fp32 MFMA:
//   1. aggregation + LayerNorm + relu + dropout: 16 lanes per row (agg's layout) -> h [16][64];
//   2. z = h W^T + b: class tiles of 16 split over the waves, D[v][c] (A = h[c'][16b + 4q + i],
//      B = W[16 ct + c'][16b + 4q + i]);
//   3. log_softmax, nll, g = (softmax - onehot) / n_valid per row (16 lanes per row);
//   4. gh = g W: wave w -> features 16w .. +15, 4 classes per instruction;
//   5. LayerNorm / relu / dropout backward -> ga; row sums of ga, gy, gy * xhat;
//   6. out_lin.weight partial g^T h: D[c][k], class tiles split over the waves.
// out_lin.weight staged in LDS once per block as [CT*16][64] with the float4 index XOR-swizzled
// by the row (conflict-free ds_read_b128 along k and ds_read_b32 along c). The block's
// parameter-gradient partials go to one slab row (finalize sums them):
//   [C*64: sum_v g[v][c] h[v][k] | C: sum_v g[v][c] | 64: sum_v ga | 64: sum_v gy |
//    64: sum_v gy*xhat | 1: sum_v loss_v]
struct HeadArgs {
    const int32_t* sizes; const int32_t* n_id; const int64_t* labels;
    const int32_t* ptr; const int32_t* idx; const uint8_t* rel; const float* inv;
    const float* tab; const float* xs; const float* bias; const float* ln_w; const float* ln_b;
    const int64_t* state; int layer; Drop drop;
    const float* w_out; const float* b_out; int C;
    float* ga; float* nvalid; float* part; int64_t part_w;
};

constexpr int kHeadRows = 16;          // target rows per block (one MFMA row tile)
constexpr int kMaxCT = 28;             // class tiles of 16: C <= 448

inline int64_t head_part_width(int C) { return ((int64_t(C) * (F + 1) + 3 * F + 1) + 3) & ~3ll; }
__host__ __device__ inline int head_cp(int C) { return ((C + 63) / 64) * 64 + 4; }   // z / g row stride: 4 banks apart
inline size_t head_lds(int C) {
    const int CT = (C + 15) / 16;
    const size_t wl = size_t(CT) * 16 * F;                 // also the row-sum scratch (3*16*64)
    return ((wl > size_t(3 * 16 * F) ? wl : size_t(3 * 16 * F)) + size_t(16) * head_cp(C) + 16 * 68 + 16 * 80 +
            16 * 68) * sizeof(float);
}

__device__ __forceinline__ int head_sw(int c, int k) { return c * F + (k ^ ((c & 15) << 2)); }

__global__ void __launch_bounds__(kBlock) head_kernel(HeadArgs A) {
    extern __shared__ float hl[];
    const int C = A.C, CT = (C + 15) / 16, CP = head_cp(C);
    float* Wl = hl;                                        // [CT*16][64] swizzled; later red
    float* zs = Wl + max(CT * 16 * F, 3 * 16 * F);         // [16][CP]: z, then g
    float* hs = zs + 16 * CP;                              // [16][68]: h (row reads)
    float* hs2 = hs + 16 * 68;                             // [16][80]: h (column reads)
    float* ghs = hs2 + 16 * 80;                            // [16][68]: gh
    __shared__ float tab[F];
    __shared__ float lrow[kHeadRows];
    const int l = threadIdx.x & 15, sub = threadIdx.x >> 4, gl = threadIdx.x & 48;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, cc = lane & 15, q = lane >> 4;
    const int n = A.sizes[0];
    const int v = blockIdx.x * kHeadRows + sub;
    const bool act = v < n;
    const int64_t y = act ? A.labels[A.n_id[v]] : -1;     // in flight during the staging
    {   // out_lin.weight -> LDS by LDS-DMA (global_load_lds_dwordx4: no VGPRs, in flight while
        // the aggregation's first loads go out). One wave instruction fills 4 rows (1 KiB) of
        // the image linearly; the XOR swizzle is applied to the per-lane SOURCE: lane L writes
        // slot L%16 of row c, which holds W[c][4 ((L%16) ^ (c & 15)) ..] (head_sw). Pad rows
        // c >= C read row C-1 (finite values; their classes are masked everywhere).
        const int L64 = threadIdx.x & 63;
        for (int i = threadIdx.x >> 6; i < CT * 4; i += kBlock / 64) {
            const int c = 4 * i + (L64 >> 4);
            const int cs = c < C ? c : C - 1;
            const float* src = A.w_out + int64_t(cs) * F + 4 * ((L64 & 15) ^ (c & 15));
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)src,
                (__attribute__((address_space(3))) void*)(Wl + 4 * i * F), 16, 0, 0);
        }
    }
    // the labelled-target count nll_loss divides by: every block counts the batch's targets
    // itself while the weight DMA lands (per-wave integer sums); block 0 hands it to finalize
    __shared__ int wcnt[kBlock / 64];
    {
        int cnt_valid = 0;
        for (int i = threadIdx.x; i < n; i += kBlock) cnt_valid += A.labels[A.n_id[i]] >= 0 ? 1 : 0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) cnt_valid += __shfl_xor(cnt_valid, o, 64);
        if ((threadIdx.x & 63) == 0) wcnt[threadIdx.x >> 6] = cnt_valid;
    }
    if (threadIdx.x < F) tab[threadIdx.x] = A.tab[threadIdx.x];
    __syncthreads();
    // ---- 1. aggregation, LayerNorm, relu, dropout
    const float4 gw4 = reinterpret_cast<const float4*>(A.ln_w)[l];
    const float4 gb4 = reinterpret_cast<const float4*>(A.ln_b)[l];
    const float gwf[4] = {gw4.x, gw4.y, gw4.z, gw4.w}, gbf[4] = {gb4.x, gb4.y, gb4.z, gb4.w};
    float xhat[4] = {0.f, 0.f, 0.f, 0.f}, mfac[4] = {0.f, 0.f, 0.f, 0.f}, rstd = 0.f;
    float hv[4] = {0.f, 0.f, 0.f, 0.f};
    if (act) {
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
        const int e0 = A.ptr[v], e1 = A.ptr[v + 1];
        for (int c0 = e0; c0 < e1; c0 += 16) {
            const int m = min(16, e1 - c0);
            const int my_u = l < m ? A.idx[c0 + l] : 0;
            const int my_r = l < m ? int(A.rel[c0 + l]) : 0;
            constexpr int UN = 8;
            for (int j = 0; j < m; j += UN) {
                float4 x[UN];
                float wt[UN];
#pragma unroll
                for (int u = 0; u < UN; ++u) {
                    const int jj = min(j + u, m - 1);
                    const int uu = __shfl(my_u, gl + jj, 64);
                    wt[u] = j + u < m ? tab[__shfl(my_r, gl + jj, 64)] : 0.f;
                    x[u] = *reinterpret_cast<const float4*>(A.xs + int64_t(uu) * F + 4 * l);
                }
#pragma unroll
                for (int u = 0; u < UN; ++u) {
                    if (j + u >= m) break;
                    s0 = fmaf(wt[u], x[u].x, s0); s1 = fmaf(wt[u], x[u].y, s1);
                    s2 = fmaf(wt[u], x[u].z, s2); s3 = fmaf(wt[u], x[u].w, s3);
                }
            }
        }
        const float iv = A.inv[v];
        const float4 b4 = reinterpret_cast<const float4*>(A.bias)[l];
        const float a[4] = {fmaf(iv, s0, b4.x), fmaf(iv, s1, b4.y), fmaf(iv, s2, b4.z),
                            fmaf(iv, s3, b4.w)};
        const float mean = group_sum<16>(a[0] + a[1] + a[2] + a[3]) * (1.f / F);
        const float d[4] = {a[0] - mean, a[1] - mean, a[2] - mean, a[3] - mean};
        rstd = rsqrtf(group_sum<16>(d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3]) *
                          (1.f / F) + kLnEps);
        const uint32_t key = A.drop.on ? layer_key(A.state, A.layer) : 0u;
        drop_factors(key, A.drop, v, l, mfac);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            xhat[i] = d[i] * rstd;
            hv[i] = fmaxf(fmaf(xhat[i], gwf[i], gbf[i]), 0.f) * mfac[i];
        }
    }
    *reinterpret_cast<float4*>(hs + sub * 68 + 4 * l) = make_float4(hv[0], hv[1], hv[2], hv[3]);
    *reinterpret_cast<float4*>(hs2 + sub * 80 + 4 * l) = make_float4(hv[0], hv[1], hv[2], hv[3]);
    __syncthreads();
    const int n_valid = (wcnt[0] + wcnt[1]) + (wcnt[2] + wcnt[3]);
    if (blockIdx.x == 0 && threadIdx.x == 0) *A.nvalid = float(n_valid);
    // ---- 2. z = h W^T + b -> zs (classes >= C: -inf)
    for (int ct = w; ct < CT; ct += kBlock / 64) {
        const int c = 16 * ct + cc;
        f32x4 dz = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int b = 0; b < F / 16; ++b) {
            const float4 av = *reinterpret_cast<const float4*>(hs + cc * 68 + 16 * b + 4 * q);
            const float4 bv = *reinterpret_cast<const float4*>(Wl + head_sw(c, 16 * b + 4 * q));
            dz = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bv.x, dz, 0, 0, 0);
            dz = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, bv.y, dz, 0, 0, 0);
            dz = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, bv.z, dz, 0, 0, 0);
            dz = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, bv.w, dz, 0, 0, 0);
        }
        const float bo = c < C ? A.b_out[c] : 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) zs[(4 * q + r) * CP + c] = c < C ? dz[r] + bo : -INFINITY;
    }
    __syncthreads();
    // ---- 3. log_softmax, nll, g
    {                                      // lane l holds classes l + 16i of row sub
        float zr[kMaxCT];
        float zmax = -INFINITY;
#pragma unroll
        for (int i = 0; i < kMaxCT; ++i) {
            zr[i] = i < CT ? zs[sub * CP + l + 16 * i] : -INFINITY;
            zmax = fmaxf(zmax, zr[i]);
        }
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) zmax = fmaxf(zmax, __shfl_xor(zmax, o, 64));
        float se = 0.f;
#pragma unroll
        for (int i = 0; i < kMaxCT; ++i) {
            zr[i] = expf(zr[i] - zmax);        // classes >= C: exp(-inf) = 0
            se += zr[i];
        }
        se = group_sum<16>(se);
        const float lse = zmax + logf(se), rse = 1.f / se;
        const float zy = y >= 0 ? zs[sub * CP + y] : 0.f;
        if (l == 0) lrow[sub] = y >= 0 ? lse - zy : 0.f;
        const float inv_n = y >= 0 && n_valid > 0 ? 1.f / float(n_valid) : 0.f;
#pragma unroll
        for (int i = 0; i < kMaxCT; ++i) {
            const int c = l + 16 * i;
            if (i < CT)
                zs[sub * CP + c] = act && c < C ? (zr[i] * rse - (int64_t(c) == y ? 1.f : 0.f)) * inv_n : 0.f;
        }
    }
    __syncthreads();
    // ---- 4. gh = g W: wave w -> features 16w + cc, rows 4q + r
    {
        const int k = 16 * w + cc;
        // classes 16b + 4q + i (i = instruction); two class tiles per iteration on two
        // independent accumulators, every LDS read of the pair issued before its products
        auto step = [&](int b, f32x4 d) {
            const float4 av = *reinterpret_cast<const float4*>(zs + cc * CP + 16 * b + 4 * q);
            const int c0 = 16 * b + 4 * q;
            const float w0 = Wl[head_sw(c0 + 0, k)], w1 = Wl[head_sw(c0 + 1, k)];
            const float w2 = Wl[head_sw(c0 + 2, k)], w3 = Wl[head_sw(c0 + 3, k)];
            d = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, w0, d, 0, 0, 0);
            d = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, w1, d, 0, 0, 0);
            d = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, w2, d, 0, 0, 0);
            return __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, w3, d, 0, 0, 0);
        };
        f32x4 dg0 = {0.f, 0.f, 0.f, 0.f}, dg1 = {0.f, 0.f, 0.f, 0.f};
        int b = 0;
        for (; b + 1 < CT; b += 2) {
            dg0 = step(b, dg0);
            dg1 = step(b + 1, dg1);
        }
        if (b < CT) dg0 = step(b, dg0);
#pragma unroll
        for (int r = 0; r < 4; ++r) ghs[(4 * q + r) * 68 + k] = dg0[r] + dg1[r];
    }
    __syncthreads();
    // ---- 5. LayerNorm / relu / dropout backward -> ga; per-feature row terms to red
    float* red = Wl;                       // [3][16][64]: ga, gy, gy*xhat (W no longer needed)
    {
        const float4 g4 = *reinterpret_cast<const float4*>(ghs + sub * 68 + 4 * l);
        const float g[4] = {g4.x, g4.y, g4.z, g4.w};
        float gy[4], gx[4];
        float p1 = 0.f, p2 = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float y = fmaf(xhat[i], gwf[i], gbf[i]);
            gy[i] = act && y > 0.f ? g[i] * mfac[i] : 0.f;
            gx[i] = gy[i] * gwf[i];
            p1 += gx[i];
            p2 += gx[i] * xhat[i];
        }
        const float m1 = group_sum<16>(p1) * (1.f / F), m2 = group_sum<16>(p2) * (1.f / F);
        float ga[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) ga[i] = act ? rstd * (gx[i] - m1 - xhat[i] * m2) : 0.f;
        if (act)
            *reinterpret_cast<float4*>(A.ga + int64_t(v) * F + 4 * l) = make_float4(ga[0], ga[1], ga[2], ga[3]);
        *reinterpret_cast<float4*>(red + (0 * 16 + sub) * F + 4 * l) = make_float4(ga[0], ga[1], ga[2], ga[3]);
        *reinterpret_cast<float4*>(red + (1 * 16 + sub) * F + 4 * l) = make_float4(gy[0], gy[1], gy[2], gy[3]);
        *reinterpret_cast<float4*>(red + (2 * 16 + sub) * F + 4 * l) =
            make_float4(gy[0] * xhat[0], gy[1] * xhat[1], gy[2] * xhat[2], gy[3] * xhat[3]);
    }
    __syncthreads();
    float* o = A.part + int64_t(blockIdx.x) * A.part_w;
    // ---- 6. out_lin.weight partial: D[c][k] = sum_v g[v][c] h[v][k]
    for (int ct = w; ct < CT; ct += kBlock / 64) {
        f32x4 dw[4];
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) dw[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            const int r = 4 * st + q;
            const float av = zs[r * CP + 16 * ct + cc];
#pragma unroll
            for (int kb = 0; kb < 4; ++kb)
                dw[kb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, hs2[r * 80 + 16 * kb + cc], dw[kb], 0, 0, 0);
        }
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int c = 16 * ct + 4 * q + r;
                if (c < C) o[int64_t(c) * F + 16 * kb + cc] = dw[kb][r];
            }
    }
    for (int c = threadIdx.x; c < C; c += kBlock) {           // out_lin.bias partial
        float acc = 0.f;
#pragma unroll
        for (int r = 0; r < kHeadRows; ++r) acc += zs[r * CP + c];
        o[int64_t(C) * F + c] = acc;
    }
    if (threadIdx.x < 3 * F) {                                 // conv bias, LN beta, LN gamma
        const int which = threadIdx.x >> 6, f = threadIdx.x & 63;
        float acc = 0.f;
#pragma unroll
        for (int r = 0; r < kHeadRows; ++r) acc += red[(which * 16 + r) * F + f];
        o[int64_t(C) * (F + 1) + threadIdx.x] = acc;
    }
    if (threadIdx.x == 0) {
        float acc = 0.f;
#pragma unroll
        for (int r = 0; r < kHeadRows; ++r) acc += lrow[r];
        o[int64_t(C) * (F + 1) + 3 * F] = acc;
    }
}

// ---------------------------------------------------------------------------------------------
// agg_bwd: gxs[idx_e] += tab[rel_e] inv[v] ga[v] (atomics) and per-relation dots
// inv[v] <ga[v], xs[idx_e]> in lane-private LDS bins -> slab[block][64].
struct AggBwdArgs {
    const int32_t* sizes; int hop;
    const int32_t* ptr; const int32_t* idx; const uint8_t* rel; const float* inv;
    const float* tab; const float* xs; const float* ga; float* gxs; float* slab; int n_rel;
};

__global__ void __launch_bounds__(kBlock) agg_bwd_kernel(AggBwdArgs A) {
    extern __shared__ float bins[];        // [n_rel][kBlock]: a thread owns its column
    __shared__ float tab[F];
    for (int i = threadIdx.x; i < A.n_rel * kBlock; i += kBlock) bins[i] = 0.f;
    if (threadIdx.x < F) tab[threadIdx.x] = A.tab[threadIdx.x];
    __syncthreads();
    const int n = A.sizes[A.hop];
    const int f = threadIdx.x & 63;
    for (int v = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); v < n;
         v += gridDim.x * (kBlock / 64)) {
        const float g = A.inv[v] * A.ga[int64_t(v) * F + f];
        const int e0 = A.ptr[v], e1 = A.ptr[v + 1];
        for (int c0 = e0; c0 < e1; c0 += 64) {
            // the wave loads up to 64 edges' (source, relation) at once; lane-uniform reads
            // below, so the per-edge row loads do not wait on an index load each
            const int m = min(64, e1 - c0);
            const int my_u = f < m ? A.idx[c0 + f] : 0;
            const int my_r = f < m ? int(A.rel[c0 + f]) : 0;
            int j = 0;
            for (; j + 4 <= m; j += 4) {
                int u[4], r[4];
                float x[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    u[q] = __builtin_amdgcn_readlane(my_u, j + q);
                    r[q] = __builtin_amdgcn_readlane(my_r, j + q);
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) x[q] = A.xs[int64_t(u[q]) * F + f];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    unsafeAtomicAdd(A.gxs + int64_t(u[q]) * F + f, tab[r[q]] * g);
                    bins[r[q] * kBlock + threadIdx.x] += g * x[q];
                }
            }
            for (; j < m; ++j) {
                const int u = __builtin_amdgcn_readlane(my_u, j);
                const int r = __builtin_amdgcn_readlane(my_r, j);
                unsafeAtomicAdd(A.gxs + int64_t(u) * F + f, tab[r] * g);
                bins[r * kBlock + threadIdx.x] += g * A.xs[int64_t(u) * F + f];
            }
        }
    }
    __syncthreads();
    // block sum per relation: 4 waves x 64 lanes, fixed order
    for (int r = threadIdx.x >> 6; r < A.n_rel; r += kBlock / 64) {
        float s = bins[r * kBlock + f] + bins[r * kBlock + 64 + f] + bins[r * kBlock + 128 + f] +
                  bins[r * kBlock + 192 + f];
        s = wave_sum(s);
        if (f == 0) A.slab[int64_t(blockIdx.x) * F + r] = s;
    }
    for (int r = A.n_rel + threadIdx.x; r < F; r += kBlock) A.slab[int64_t(blockIdx.x) * F + r] = 0.f;
}

// ---------------------------------------------------------------------------------------------
// post_bwd (layer l < L-1): gs = gxs_{l+1}[v]; gh = gs W_{l+1}^T; dropout / relu / LayerNorm
// backward -> ga of layer l. Wave per row. The block's partials go to one slab row:
//   [64*64: sum_v h[v]^T gs[v] (convs[l+1].weight) | 64: sum ga | 64: sum gy | 64: sum gy*xhat]
constexpr int kPostW = F * F + 3 * F;

struct PostArgs {
    const int32_t* sizes; int hop;
    const float* a; const float* stats; const float* ln_w; const float* ln_b;
    const int64_t* state; int layer; Drop drop;
    const float* w_next; const float* gxs_next;
    float* ga; float* slab;
};

__global__ void __launch_bounds__(kBlock) post_bwd_kernel(PostArgs A) {
    __shared__ float Wt[F * kWPad];        // W[k][j] at k*65 + j
    __shared__ float hs[4][F], gsr[4][F];
    __shared__ float cs[3][4][F];
    for (int i = threadIdx.x; i < F * F; i += kBlock) Wt[(i / F) * kWPad + (i % F)] = A.w_next[i];
    __syncthreads();
    const int n = A.sizes[A.hop];
    const int w = threadIdx.x >> 6, f = threadIdx.x & 63;
    const uint32_t key = A.drop.on ? layer_key(A.state, A.layer) : 0u;
    const float gwf = A.ln_w[f], gbf = A.ln_b[f];
    // this thread's 16 entries of the block's W_{l+1} gradient partial: k = tid / 4,
    // j = (tid % 4) * 16 .. +15
    const int kk = threadIdx.x >> 2, j0 = (threadIdx.x & 3) * 16;
    float acc[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) acc[c] = 0.f;
    float sga = 0.f, sgy = 0.f, sgyx = 0.f;
    for (int base = blockIdx.x * 4; base < n; base += gridDim.x * 4) {
        const int v = base + w;
        const bool act = v < n;
        float xhat = 0.f, rstd = 0.f, mfac = 0.f, gsv = 0.f;
        if (act) {
            const float2 st = reinterpret_cast<const float2*>(A.stats)[v];
            rstd = st.y;
            xhat = (A.a[int64_t(v) * F + f] - st.x) * rstd;
            mfac = lane_drop(key, A.drop, v, f);
            gsv = A.gxs_next[int64_t(v) * F + f];
        }
        hs[w][f] = act ? fmaxf(fmaf(xhat, gwf, gbf), 0.f) * mfac : 0.f;
        gsr[w][f] = gsv;
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float hk = hs[r][kk];
#pragma unroll
            for (int c = 0; c < 16; c += 4) {
                const float4 g4 = *reinterpret_cast<const float4*>(&gsr[r][j0 + c]);
                acc[c] = fmaf(hk, g4.x, acc[c]);
                acc[c + 1] = fmaf(hk, g4.y, acc[c + 1]);
                acc[c + 2] = fmaf(hk, g4.z, acc[c + 2]);
                acc[c + 3] = fmaf(hk, g4.w, acc[c + 3]);
            }
        }
        if (act) {
            float gh = 0.f;                // d loss / d h[f] = sum_j gs[j] W[f][j]
#pragma unroll 8
            for (int j = 0; j < F; ++j) gh = fmaf(gsr[w][j], Wt[f * kWPad + j], gh);
            float ga, gyv, gyx;
            ln_relu_drop_bwd(gh, xhat, rstd, gwf, gbf, mfac, &ga, &gyv, &gyx);
            A.ga[int64_t(v) * F + f] = ga;
            sga += ga; sgy += gyv; sgyx += gyx;
        }
        __syncthreads();
    }
    float* o = A.slab + int64_t(blockIdx.x) * kPostW;
#pragma unroll
    for (int c = 0; c < 16; c += 4)
        *reinterpret_cast<float4*>(o + kk * F + j0 + c) =
            make_float4(acc[c], acc[c + 1], acc[c + 2], acc[c + 3]);
    cs[0][w][f] = sga; cs[1][w][f] = sgy; cs[2][w][f] = sgyx;
    __syncthreads();
    if (threadIdx.x < 3 * F) {
        const int which = threadIdx.x >> 6;
        o[F * F + threadIdx.x] =
            ((cs[which][0][f] + cs[which][1][f]) + cs[which][2][f]) + cs[which][3][f];
    }
}

// ---------------------------------------------------------------------------------------------
// bwd0 (layer 0 backward, the GEMM half): with G_v = inv_v ga_v (ga = d loss / d a_0),
//   gW_c[t] = sum_v S_vt^T G_v,   gb_c[t] = sum_v w_vt G_v,
//   Z_vt = W_c[t] G_v (K wide),   beta_vt = <b_c[t], G_v>
// where Z and beta turn the relation-table gradient into a per-edge dot (rel0). Block (b, t)
// takes 16-row tiles (grid-stride), S and G staged in LDS with the next tile prefetched into
// registers; W_c[t] in LDS k-major (row stride 68: conflict-free ds_read_b128).
//   gW: D[k][j] (lane (c, q): k = 16 kb + c, 4 rows q per instruction), wave w owns k blocks
//       KB*w .. +KB-1 and all 4 j blocks, as a per-block partial [K*64 | 64] in the slab;
//   Z:  D[v][k] = sum_j G[v][j] W_c[t][k][j] (lane (c, q): A = G[c][16b + 4q + i] from a second
//       copy of the tile at row stride 68, B = W_c[t][16 kb + c][16b + 4q + i]).
struct Bwd0Args {
    const int32_t* sizes; int hop; int T;
    const float* inv; const float* ga; const float* s_agg; const float* s_w; const float* wc;
    float* z; float* beta; float* slab;
    // relation-slot mode (bwd0_rs_kernel): layer 0's relation table, agg0's self rows and slot
    // relations; relation dots -> rslab[t * gridDim.x + block][F]
    const float* tab; const float* u_self; const int32_t* u_rel; int n_rel, n_et; float* rslab;
};

template <int K>
__global__ void __launch_bounds__(kBlock) bwd0_kernel(Bwd0Args A) {
    constexpr int XS = K + 16, GS = F + 16, G2 = F + 4, WS = F + 4;
    constexpr int KB = K / 64;                // k blocks per wave
    constexpr int XV = K / 4 * 16 / kBlock;   // S float4 per thread per tile (K=128: 2, 64: 1)
    __shared__ float Wk[K * WS];
    __shared__ float bc[F];
    __shared__ float xsh[16 * XS];
    __shared__ float gsh[16 * GS];
    __shared__ float gs2[16 * G2];
    __shared__ float sws[16];
    const int t = blockIdx.y, T = A.T;
    const float* wct = A.wc + int64_t(t) * (K + 1) * F;
    for (int e = threadIdx.x; e < K * F; e += kBlock) {      // wcT[j][k] -> Wk[k][j]
        const int j = e / K, k = e - j * K;
        Wk[k * WS + j] = wct[e];
    }
    if (threadIdx.x < F) bc[threadIdx.x] = wct[K * F + threadIdx.x];
    const int n = A.sizes[A.hop];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4;
    const int gr = threadIdx.x >> 4, gj = threadIdx.x & 15;
    f32x4 acc[KB][4];
#pragma unroll
    for (int a = 0; a < KB; ++a)
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) acc[a][jb] = f32x4{0.f, 0.f, 0.f, 0.f};
    float bsum = 0.f;
    float4 sr[XV], gv;
    float swv = 0.f;
    auto load = [&](int v0) {
#pragma unroll
        for (int u = 0; u < XV; ++u) {
            const int e = threadIdx.x + kBlock * u;
            const int r = e / (K / 4), k4 = e - r * (K / 4);
            sr[u] = v0 + r < n ? *reinterpret_cast<const float4*>(
                                     A.s_agg + (int64_t(v0 + r) * T + t) * K + 4 * k4)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        const int v = v0 + gr;
        if (v < n) {
            const float iv = A.inv[v];
            const float4 g4 = *reinterpret_cast<const float4*>(A.ga + int64_t(v) * F + 4 * gj);
            gv = make_float4(iv * g4.x, iv * g4.y, iv * g4.z, iv * g4.w);
        } else {
            gv = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        if (threadIdx.x < 16) swv = v0 + threadIdx.x < n ? A.s_w[int64_t(v0 + threadIdx.x) * T + t] : 0.f;
    };
    int tile = blockIdx.x;
    if (tile * 16 < n) load(tile * 16);
    for (; tile * 16 < n; tile += gridDim.x) {
        const int v0 = tile * 16;
#pragma unroll
        for (int u = 0; u < XV; ++u) {
            const int e = threadIdx.x + kBlock * u;
            const int r = e / (K / 4), k4 = e - r * (K / 4);
            *reinterpret_cast<float4*>(xsh + r * XS + 4 * k4) = sr[u];
        }
        *reinterpret_cast<float4*>(gsh + gr * GS + 4 * gj) = gv;
        *reinterpret_cast<float4*>(gs2 + gr * G2 + 4 * gj) = gv;
        if (threadIdx.x < 16) sws[threadIdx.x] = swv;
        __syncthreads();
        if ((tile + gridDim.x) * 16 < n) load((tile + gridDim.x) * 16);
        if (threadIdx.x < F) {
#pragma unroll
            for (int r = 0; r < 16; ++r) bsum = fmaf(sws[r], gsh[r * GS + threadIdx.x], bsum);
        }
        // gW partial
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            const int r = 4 * st + q;
            float bv[4];
#pragma unroll
            for (int jb = 0; jb < 4; ++jb) bv[jb] = gsh[r * GS + 16 * jb + c];
#pragma unroll
            for (int a = 0; a < KB; ++a) {
                const float av = xsh[r * XS + 16 * (KB * w + a) + c];
#pragma unroll
                for (int jb = 0; jb < 4; ++jb)
                    acc[a][jb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[jb], acc[a][jb], 0, 0, 0);
            }
        }
        // Z rows of this tile: wave w -> k blocks KB*w .. +KB-1
#pragma unroll
        for (int a = 0; a < KB; ++a) {
            const int kb = KB * w + a;
            f32x4 zc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int b = 0; b < F / 16; ++b) {
                const float4 av = *reinterpret_cast<const float4*>(gs2 + c * G2 + 16 * b + 4 * q);
                const float4 bw = *reinterpret_cast<const float4*>(Wk + (16 * kb + c) * WS + 16 * b + 4 * q);
                zc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bw.x, zc, 0, 0, 0);
                zc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, bw.y, zc, 0, 0, 0);
                zc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, bw.z, zc, 0, 0, 0);
                zc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, bw.w, zc, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int v = v0 + 4 * q + r;
                if (v < n) A.z[(int64_t(v) * T + t) * K + 16 * kb + c] = zc[r];
            }
        }
        {                                      // beta_vt = <b_c[t], G_v>
            const float4 g4 = *reinterpret_cast<const float4*>(gs2 + gr * G2 + 4 * gj);
            float bt = bc[4 * gj] * g4.x + bc[4 * gj + 1] * g4.y + bc[4 * gj + 2] * g4.z +
                       bc[4 * gj + 3] * g4.w;
            bt = group_sum<16>(bt);
            if (gj == 0 && v0 + gr < n) A.beta[int64_t(v0 + gr) * T + t] = bt;
        }
        __syncthreads();
    }
    float* o = A.slab + (int64_t(t) * gridDim.x + blockIdx.x) * int64_t((K + 1) * F);
#pragma unroll
    for (int a = 0; a < KB; ++a)
#pragma unroll
        for (int jb = 0; jb < 4; ++jb)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                o[(16 * (KB * w + a) + 4 * q + i) * F + 16 * jb + c] = acc[a][jb][i];
    if (threadIdx.x < F) o[K * F + threadIdx.x] = bsum;
}

// bwd0 in relation-slot mode (agg0<.., RS = true>): the S tile is re-formed per row as
// wr U_vt + ws x_v (wr = tab[r_vt], ws = tab[r_self] when the row's type is t), the gradient
// products as bwd0_kernel's, and the relation-table dots come from the same Z fragments:
//   d tab[r_vt] += <U_vt, Z_vt> + cnt_vt beta_vt,   d tab[r_self] += <x_v, Z_vt> + beta_vt
// (no Z / beta to HBM, no second pass over the edges). Row r of the tile keeps its own column
// of the relation bins in LDS (fixed summation order: deterministic), one slab row per block.
inline size_t bwd0_rs_lds(int K, int n_rel) {
    return sizeof(float) * (size_t(K) * (F + 4) + F + 2 * 16 * (K + 4) + 16 * (F + 16) +
                            16 * (F + 4) + F + 16 * 4 + 16 * 2 + 4 * 16 * 2 + size_t(n_rel) * 16);
}

template <int K>
__global__ void __launch_bounds__(kBlock) bwd0_rs_kernel(Bwd0Args A) {
    constexpr int XS = K + 4, GS = F + 16, G2 = F + 4, WS = F + 4;
    constexpr int KB = K / 64;                // k blocks per wave
    constexpr int XV = K / 4 * 16 / kBlock;   // float4 per thread per 16-row tile
    extern __shared__ float sm[];
    float* Wk = sm;                           // [K][WS]
    float* bc = Wk + K * WS;                  // [F]
    float* ush = bc + F;                      // [16][XS] U_vt
    float* xsh = ush + 16 * XS;               // [16][XS] x_v (self loop rows)
    float* gsh = xsh + 16 * XS;               // [16][GS]
    float* gs2 = gsh + 16 * GS;               // [16][G2]
    float* tabl = gs2 + 16 * G2;              // [F]
    float* rm = tabl + F;                     // [16][4]: wr, ws, cnt, beta
    int* rr = reinterpret_cast<int*>(rm + 64);  // [16][2]: r_vt (or -1), r_self (or -1)
    float* dred = reinterpret_cast<float*>(rr + 32);   // [4 waves][16][2]
    float* bins = dred + 128;                 // [n_rel][16]
    const int t = blockIdx.y, T = A.T;
    const float* wct = A.wc + int64_t(t) * (K + 1) * F;
    for (int e = threadIdx.x; e < K * F; e += kBlock) {      // wcT[j][k] -> Wk[k][j]
        const int j = e / K, k = e - j * K;
        Wk[k * WS + j] = wct[e];
    }
    if (threadIdx.x < F) {
        bc[threadIdx.x] = wct[K * F + threadIdx.x];
        tabl[threadIdx.x] = A.tab[threadIdx.x];
    }
    for (int i = threadIdx.x; i < A.n_rel * 16; i += kBlock) bins[i] = 0.f;
    const int n = A.sizes[A.hop];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4;
    const int gr = threadIdx.x >> 4, gj = threadIdx.x & 15;
    f32x4 acc[KB][4];
#pragma unroll
    for (int a = 0; a < KB; ++a)
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) acc[a][jb] = f32x4{0.f, 0.f, 0.f, 0.f};
    float bsum = 0.f;
    float4 ur[XV], xr[XV], gv;
    float cntv = 0.f;
    int relv = -1, rsv = -1;
    auto load = [&](int v0) {
#pragma unroll
        for (int u = 0; u < XV; ++u) {
            const int e = threadIdx.x + kBlock * u;
            const int r = e / (K / 4), k4 = e - r * (K / 4);
            const bool ok = v0 + r < n;
            ur[u] = ok ? *reinterpret_cast<const float4*>(A.s_agg + (int64_t(v0 + r) * T + t) * K + 4 * k4)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
            xr[u] = ok ? *reinterpret_cast<const float4*>(A.u_self + int64_t(v0 + r) * K + 4 * k4)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        const int v = v0 + gr;
        if (v < n) {
            const float iv = A.inv[v];
            const float4 g4 = *reinterpret_cast<const float4*>(A.ga + int64_t(v) * F + 4 * gj);
            gv = make_float4(iv * g4.x, iv * g4.y, iv * g4.z, iv * g4.w);
        } else {
            gv = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        if (threadIdx.x < 16) {
            const int vv = v0 + threadIdx.x;
            const bool ok = vv < n;
            cntv = ok ? A.s_w[int64_t(vv) * T + t] : 0.f;
            relv = ok ? A.u_rel[int64_t(vv) * (T + 1) + t] : -1;
            rsv = ok ? A.u_rel[int64_t(vv) * (T + 1) + T] : -1;
        }
    };
    int tile = blockIdx.x;
    if (tile * 16 < n) load(tile * 16);
    for (; tile * 16 < n; tile += gridDim.x) {
        const int v0 = tile * 16;
        if (threadIdx.x < 16) {                // row meta: S = wr U + ws x_self
            const bool self = rsv >= 0 && rsv - A.n_et == t;
            const float wr = relv >= 0 ? tabl[relv] : 0.f;
            const float ws = self ? tabl[rsv] : 0.f;
            rm[4 * threadIdx.x] = wr;
            rm[4 * threadIdx.x + 1] = ws;
            rm[4 * threadIdx.x + 2] = cntv;
            rr[2 * threadIdx.x] = (relv >= 0 && cntv > 0.f) ? relv : -1;
            rr[2 * threadIdx.x + 1] = self ? rsv : -1;
        }
#pragma unroll
        for (int u = 0; u < XV; ++u) {
            const int e = threadIdx.x + kBlock * u;
            const int r = e / (K / 4), k4 = e - r * (K / 4);
            *reinterpret_cast<float4*>(ush + r * XS + 4 * k4) = ur[u];
            *reinterpret_cast<float4*>(xsh + r * XS + 4 * k4) = xr[u];
        }
        *reinterpret_cast<float4*>(gsh + gr * GS + 4 * gj) = gv;
        *reinterpret_cast<float4*>(gs2 + gr * G2 + 4 * gj) = gv;
        __syncthreads();
        if ((tile + gridDim.x) * 16 < n) load((tile + gridDim.x) * 16);
        if (threadIdx.x < F) {
#pragma unroll
            for (int r = 0; r < 16; ++r)
                bsum = fmaf(fmaf(rm[4 * r], rm[4 * r + 2], rm[4 * r + 1]), gsh[r * GS + threadIdx.x], bsum);
        }
        // gW partial over the re-formed S rows
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            const int r = 4 * st + q;
            const float wr = rm[4 * r], ws = rm[4 * r + 1];
            float bv[4];
#pragma unroll
            for (int jb = 0; jb < 4; ++jb) bv[jb] = gsh[r * GS + 16 * jb + c];
#pragma unroll
            for (int a = 0; a < KB; ++a) {
                const int k = 16 * (KB * w + a) + c;
                const float av = fmaf(ws, xsh[r * XS + k], wr * ush[r * XS + k]);
#pragma unroll
                for (int jb = 0; jb < 4; ++jb)
                    acc[a][jb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[jb], acc[a][jb], 0, 0, 0);
            }
        }
        // Z fragments (wave w -> k blocks KB*w .. +KB-1) dotted with U and x_self
        float pu[4] = {0.f, 0.f, 0.f, 0.f}, ps[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int a = 0; a < KB; ++a) {
            const int kb = KB * w + a;
            f32x4 zc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int b = 0; b < F / 16; ++b) {
                const float4 av = *reinterpret_cast<const float4*>(gs2 + c * G2 + 16 * b + 4 * q);
                const float4 bw = *reinterpret_cast<const float4*>(Wk + (16 * kb + c) * WS + 16 * b + 4 * q);
                zc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bw.x, zc, 0, 0, 0);
                zc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, bw.y, zc, 0, 0, 0);
                zc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, bw.z, zc, 0, 0, 0);
                zc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, bw.w, zc, 0, 0, 0);
            }
            // zc[r] = Z[row 4 q + r][k = 16 kb + c]
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                pu[r] = fmaf(zc[r], ush[(4 * q + r) * XS + 16 * kb + c], pu[r]);
                ps[r] = fmaf(zc[r], xsh[(4 * q + r) * XS + 16 * kb + c], ps[r]);
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            pu[r] = group_sum<16>(pu[r]);
            ps[r] = group_sum<16>(ps[r]);
        }
        if (c == 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                dred[(w * 16 + 4 * q + r) * 2] = pu[r];
                dred[(w * 16 + 4 * q + r) * 2 + 1] = ps[r];
            }
        }
        {                                      // beta_vt = <b_c[t], G_v>
            const float4 g4 = *reinterpret_cast<const float4*>(gs2 + gr * G2 + 4 * gj);
            float bt = bc[4 * gj] * g4.x + bc[4 * gj + 1] * g4.y + bc[4 * gj + 2] * g4.z +
                       bc[4 * gj + 3] * g4.w;
            bt = group_sum<16>(bt);
            if (gj == 0) rm[4 * gr + 3] = bt;
        }
        __syncthreads();
        if (threadIdx.x < 16) {                // row r's relation dots into its bin column
            const int r = threadIdx.x;
            const float du = ((dred[(0 * 16 + r) * 2] + dred[(1 * 16 + r) * 2]) +
                              dred[(2 * 16 + r) * 2]) + dred[(3 * 16 + r) * 2];
            const float ds = ((dred[(0 * 16 + r) * 2 + 1] + dred[(1 * 16 + r) * 2 + 1]) +
                              dred[(2 * 16 + r) * 2 + 1]) + dred[(3 * 16 + r) * 2 + 1];
            const float bt = rm[4 * r + 3];
            if (rr[2 * r] >= 0) bins[rr[2 * r] * 16 + r] += fmaf(rm[4 * r + 2], bt, du);
            if (rr[2 * r + 1] >= 0) bins[rr[2 * r + 1] * 16 + r] += ds + bt;
        }
        __syncthreads();
    }
    float* o = A.slab + (int64_t(t) * gridDim.x + blockIdx.x) * int64_t((K + 1) * F);
#pragma unroll
    for (int a = 0; a < KB; ++a)
#pragma unroll
        for (int jb = 0; jb < 4; ++jb)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                o[(16 * (KB * w + a) + 4 * q + i) * F + 16 * jb + c] = acc[a][jb][i];
    if (threadIdx.x < F) o[K * F + threadIdx.x] = bsum;
    __syncthreads();
    if (threadIdx.x < F) {
        float sr = 0.f;
        if (threadIdx.x < A.n_rel)
#pragma unroll
            for (int r = 0; r < 16; ++r) sr += bins[threadIdx.x * 16 + r];
        A.rslab[(int64_t(t) * gridDim.x + blockIdx.x) * F + threadIdx.x] = sr;
    }
}

// rel0 (layer 0 backward, the edge half): d tab[r] = sum_{e: rel_e = r} inv_v <ga_v, xs0[u_e]>
// = sum_e (<x_u, Z_{v,t_u}> + beta_{v,t_u}), the input row gathered again (agg0's per-edge type
// and table row). 16 lanes per target row, lane-private relation bins -> one slab row per block.
struct Rel0Args {
    const int32_t* sizes; int hop; int T;
    const int32_t* ptr; const int32_t* cnt; int stride;
    const uint8_t* rel; const int32_t* edge_type; const int64_t* edge_off;
    Ptrs xt; const float* z; const float* beta; float* slab; int n_rel;
};

template <int K>
__global__ void __launch_bounds__(kBlock) rel0_kernel(Rel0Args A) {
    constexpr int VPL = K / 64;
    extern __shared__ float bins[];        // [n_rel][kBlock]: a thread owns its column
    for (int i = threadIdx.x; i < A.n_rel * kBlock; i += kBlock) bins[i] = 0.f;
    __syncthreads();
    const int n = A.sizes[A.hop];
    const int T = A.T;
    const int l = threadIdx.x & 15, sub = threadIdx.x >> 4, gl = threadIdx.x & 48;
    for (int base = blockIdx.x * 16; base < n; base += gridDim.x * 16) {
        const int v = base + sub;
        if (v >= n) continue;
        int e0, e1;
        row_range(A.ptr, A.cnt, A.stride, v, e0, e1);
        for (int c0 = e0; c0 < e1; c0 += 16) {
            const int m = min(16, e1 - c0);
            int my_t = 0, my_r = 0;
            int64_t my_lo = 0;
            if (l < m) {
                my_t = A.edge_type[c0 + l];
                my_lo = A.edge_off[c0 + l];
                my_r = int(A.rel[c0 + l]);
            }
            const int lo_lo = int(uint32_t(uint64_t(my_lo))), lo_hi = int(uint64_t(my_lo) >> 32);
            constexpr int UN = 8;                  // edges in flight per lane
            for (int j = 0; j < m; j += UN) {
                int r[UN];
                float dsum[UN];
                float4 x[UN][VPL], zz[UN][VPL];
#pragma unroll
                for (int u = 0; u < UN; ++u) {
                    const int jj = min(j + u, m - 1);
                    const int t = __shfl(my_t, gl + jj, 64);
                    r[u] = __shfl(my_r, gl + jj, 64);
                    const int64_t lo = int64_t((uint64_t(uint32_t(__shfl(lo_hi, gl + jj, 64))) << 32) |
                                               uint32_t(__shfl(lo_lo, gl + jj, 64)));
                    const float* xr = pick(A.xt.p, t) + lo * K + 4 * l;
                    const float* zr = A.z + (int64_t(v) * T + t) * K + 4 * l;
                    dsum[u] = l == 0 ? A.beta[int64_t(v) * T + t] : 0.f;
#pragma unroll
                    for (int p = 0; p < VPL; ++p) {
                        x[u][p] = *reinterpret_cast<const float4*>(xr + 64 * p);
                        zz[u][p] = *reinterpret_cast<const float4*>(zr + 64 * p);
                    }
                }
#pragma unroll
                for (int u = 0; u < UN; ++u) {
                    if (j + u >= m) break;
#pragma unroll
                    for (int p = 0; p < VPL; ++p)
                        dsum[u] += x[u][p].x * zz[u][p].x + x[u][p].y * zz[u][p].y +
                                   x[u][p].z * zz[u][p].z + x[u][p].w * zz[u][p].w;
                    bins[r[u] * kBlock + threadIdx.x] += dsum[u];
                }
            }
        }
    }
    __syncthreads();
    const int w = threadIdx.x >> 6, f = threadIdx.x & 63;
    for (int r = w; r < A.n_rel; r += kBlock / 64) {
        float s = bins[r * kBlock + f] + bins[r * kBlock + 64 + f] + bins[r * kBlock + 128 + f] +
                  bins[r * kBlock + 192 + f];
        s = wave_sum(s);
        if (f == 0) A.slab[int64_t(blockIdx.x) * F + r] = s;
    }
    for (int r = A.n_rel + threadIdx.x; r < F; r += kBlock) A.slab[int64_t(blockIdx.x) * F + r] = 0.f;
}

// ---------------------------------------------------------------------------------------------
// finalize: every gradient is a fixed-order sum of per-block partials. A job sums `nparts` rows
// (stride pstride) of a slab segment of `width` floats into dst; 32 entries per block, 8
// thread groups over the partials, combined in a fixed order.
enum { kOpCopy = 0, kOpRel = 1, kOpLoss = 2 };

struct Job {
    const float* src;
    int64_t pstride;
    int nparts, width, op, blocks;
    float* dst;
    const float* aux;        // kOpRel: relation_weight; kOpLoss: the labelled-target count
};

constexpr int kMaxJobs = 32;

struct FinArgs {
    int n_jobs;
    float alpha;
    int start[kMaxJobs];     // first block of each job: the block -> job search reads 2 lines of
                             // kernel arguments at once instead of walking the 48-byte Jobs
    Job job[kMaxJobs];
};

__global__ void __launch_bounds__(kBlock) finalize_kernel(FinArgs A) {
    __shared__ float red[8][33];
    int ji = 0;
#pragma unroll
    for (int i = 1; i < kMaxJobs; ++i) ji += (i < A.n_jobs && int(blockIdx.x) >= A.start[i]);
    const int b = blockIdx.x - A.start[ji];
    const Job J = A.job[ji];
    const int el = threadIdx.x & 31, grp = threadIdx.x >> 5;
    const int e = b * 32 + el;
    float s = 0.f;
    if (e < J.width) {
        const float* src = J.src + e;
        int p = grp;
        for (; p + 56 < J.nparts; p += 64) {           // 8 partial rows in flight per thread
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = src[int64_t(p + 8 * u) * J.pstride];
#pragma unroll
            for (int u = 0; u < 8; ++u) s += v[u];
        }
        for (; p < J.nparts; p += 8) s += src[int64_t(p) * J.pstride];
    }
    red[grp][el] = s;
    __syncthreads();
    if (threadIdx.x < 32 && e < J.width) {
        const float tot = ((red[0][el] + red[1][el]) + (red[2][el] + red[3][el])) +
                          ((red[4][el] + red[5][el]) + (red[6][el] + red[7][el]));
        float out = tot;
        if (J.op == kOpRel) {
            const float x = J.aux[e] * A.alpha;                // d tab / d rw (LeakyReLU)
            out = tot * A.alpha * (x > 0.f ? 1.f : 0.01f);
        } else if (J.op == kOpLoss) {
            const float nv = *J.aux;
            out = nv > 0.f ? tot / nv : 0.f;
        }
        J.dst[e] = out;
    }
}

// chain rule of the composed map W_c[t] = W_t^T W_0, b_c[t] = b_t W_0:
//   blocks [0, 64): g W_0[o][:] = sum_t (sum_k W_t[o][k] gW_c[t][k][:] + b_t[o] gb_c[t][:]),
//     4 thread groups over (t, k), combined in a fixed order;
//   blocks [64, 64 + 64 T): g W_t[o][k] = sum_j W_0[o][j] gW_c[t][k][j] (thread k), and
//     g b_t[o] (thread K)
struct ChainArgs {
    int T; int K; Ptrs lin_w; Ptrs lin_b; const float* w0; const float* gwc;
    float* g_lin_w[MT]; float* g_lin_b[MT]; float* g_w0;
};

template <int K>
__global__ void __launch_bounds__(kBlock) chain_kernel(ChainArgs A) {
    __shared__ float red[4][F];
    __shared__ float w0r[F];
    if (blockIdx.x < F) {
        const int o = blockIdx.x, j = threadIdx.x & 63, g = threadIdx.x >> 6;
        float s = 0.f;
        for (int t = 0; t < A.T; ++t) {
            const float* W = pick(A.lin_w.p, t) + int64_t(o) * K;
            const float* gw = A.gwc + int64_t(t) * (K + 1) * F;
#pragma unroll 8
            for (int k = g; k < K; k += 4) s = fmaf(W[k], gw[int64_t(k) * F + j], s);
            if (g == 0) s = fmaf(pick(A.lin_b.p, t)[o], gw[int64_t(K) * F + j], s);
        }
        red[g][j] = s;
        __syncthreads();
        if (threadIdx.x < F)
            A.g_w0[o * F + j] = ((red[0][j] + red[1][j]) + red[2][j]) + red[3][j];
        return;
    }
    const int b = blockIdx.x - F;
    const int t = b / F, o = b - t * F;
    if (threadIdx.x < F) w0r[threadIdx.x] = A.w0[o * F + threadIdx.x];
    __syncthreads();
    const int k = threadIdx.x;
    if (k > K) return;
    const float* gw = A.gwc + (int64_t(t) * (K + 1) + k) * F;
    float s = 0.f;
#pragma unroll 4
    for (int j = 0; j < F; j += 4) {
        const float4 g4 = *reinterpret_cast<const float4*>(gw + j);
        s = fmaf(w0r[j], g4.x, s);
        s = fmaf(w0r[j + 1], g4.y, s);
        s = fmaf(w0r[j + 2], g4.z, s);
        s = fmaf(w0r[j + 3], g4.w, s);
    }
    if (k < K) pick(A.g_lin_w, t)[int64_t(o) * K + k] = s;
    else pick(A.g_lin_b, t)[o] = s;
}

// ---------------------------------------------------------------------------------------------
// Adam over flat parameter / gradient / moment buffers (torch.optim.Adam's arithmetic, L2 weight
// decay added to the gradient). The step count lives on the device: every block uses
// t = step[0] + 1 and the last block to finish stores it (ticket), so a captured graph advances
// it on every replay.
// one element of torch.optim.Adam (L2 weight decay added to the gradient)
__device__ __forceinline__ void adam_one(float gi, float& pi, float& mi, float& vi, float b1,
                                         float b2, float eps, float wd, float gscale,
                                         float step_size, float bc2_sqrt) {
    gi *= gscale;                              // gscale: 1 / ranks after a SUM all-reduce
    if (wd != 0.f) gi = gi + wd * pi;
    mi = mi + (1.f - b1) * (gi - mi);                                  // exp_avg.lerp_(grad, 1-b1)
    vi = vi * b2 + (1.f - b2) * gi * gi;                               // mul_(b2).addcmul_
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    pi = pi - step_size * (mi / denom);
}

// V = 4: four elements per thread through float4 (n % 4 == 0, 16-byte aligned buffers): a
// quarter of the blocks, so a quarter of the completion tickets on the one counter (each block's
// returning atomic on it serialises at the end of the launch)
template <int V>
__global__ void __launch_bounds__(kBlock)
adam_flat_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                 float* __restrict__ v, int64_t n, float lr, float b1, float b2, float eps,
                 float wd, float gscale, int64_t* __restrict__ step, unsigned* __restrict__ ticket) {
    using VT = typename std::conditional<V == 4, float4, float>::type;
    __shared__ bool last;
    // the first operands are requested together with the step count (independent loads: one
    // memory latency, not two, before the first update)
    const int64_t nv = n / V;
    const int64_t i0 = int64_t(blockIdx.x) * kBlock + threadIdx.x, stride = int64_t(gridDim.x) * kBlock;
    VT g0{}, p0{}, m0{}, v0{};
    if (i0 < nv) {
        g0 = reinterpret_cast<const VT*>(g)[i0]; p0 = reinterpret_cast<const VT*>(p)[i0];
        m0 = reinterpret_cast<const VT*>(m)[i0]; v0 = reinterpret_cast<const VT*>(v)[i0];
    }
    // ticket null: the step count was advanced before this launch (read only, no ticket)
    const int64_t t = ticket ? step[0] + 1 : step[0];
    const double bc1 = 1.0 - pow(double(b1), double(t));
    const double bc2 = 1.0 - pow(double(b2), double(t));
    const float step_size = float(double(lr) / bc1);
    const float bc2_sqrt = float(sqrt(bc2));
    for (int64_t i = i0; i < nv; i += stride) {
        VT gi, pi, mi, vi;
        if (i == i0) {
            gi = g0; pi = p0; mi = m0; vi = v0;
        } else {
            gi = reinterpret_cast<const VT*>(g)[i]; pi = reinterpret_cast<const VT*>(p)[i];
            mi = reinterpret_cast<const VT*>(m)[i]; vi = reinterpret_cast<const VT*>(v)[i];
        }
        if constexpr (V == 4) {
            adam_one(gi.x, pi.x, mi.x, vi.x, b1, b2, eps, wd, gscale, step_size, bc2_sqrt);
            adam_one(gi.y, pi.y, mi.y, vi.y, b1, b2, eps, wd, gscale, step_size, bc2_sqrt);
            adam_one(gi.z, pi.z, mi.z, vi.z, b1, b2, eps, wd, gscale, step_size, bc2_sqrt);
            adam_one(gi.w, pi.w, mi.w, vi.w, b1, b2, eps, wd, gscale, step_size, bc2_sqrt);
        } else {
            adam_one(gi, pi, mi, vi, b1, b2, eps, wd, gscale, step_size, bc2_sqrt);
        }
        reinterpret_cast<VT*>(m)[i] = mi;
        reinterpret_cast<VT*>(v)[i] = vi;
        reinterpret_cast<VT*>(p)[i] = pi;
    }
    // the ticket only orders every block's read of step[0] (its value is consumed above) before
    // the last block's store of it; the parameter stores need no fence before it
    if (!ticket) return;                   // (block-uniform)
    __syncthreads();
    if (threadIdx.x == 0) last = atomicAdd(ticket, 1u) == gridDim.x - 1;
    __syncthreads();
    if (last && threadIdx.x == 0) {
        step[0] = t;
        ticket[0] = 0u;
    }
}

// ---------------------------------------------------------------------------------------------
struct SlabLayout {
    int64_t rel[ML], post[ML], head, proj, total;
    int head_blocks;
};

inline SlabLayout slab_layout(const regnn_nsm_params* p, int cap0) {
    SlabLayout s{};
    int64_t o = 0;
    for (int l = 0; l < ML; ++l) {        // relation dots of layer l: rel0 (l = 0), agg_bwd
        s.rel[l] = o;                     // layer 0: rel0's or bwd0_rs's (T x kProjBlocks) rows
        if (l < p->n_layers)
            o += int64_t(l == 0 && kProjBlocks * MT > kAggBlocks ? kProjBlocks * MT : kAggBlocks) * F;
    }
    for (int l = 0; l < ML; ++l) {        // post_bwd of layer l < L-1
        s.post[l] = o;
        if (l + 1 < p->n_layers) o += int64_t(kPostBlocks) * kPostW;
    }
    s.head_blocks = (cap0 + kHeadRows - 1) / kHeadRows;
    s.head = o;
    o += int64_t(s.head_blocks) * head_part_width(p->n_classes);
    s.proj = o;
    o += int64_t(p->n_types) * kProjBlocks * (p->k_in + 1) * F;
    s.total = o;
    return s;
}

struct JobList {
    FinArgs A{};
    int blocks = 0;
    void add(const float* src, int64_t pstride, int nparts, int width, float* dst, int op = kOpCopy,
             const float* aux = nullptr) {
        A.start[A.n_jobs] = blocks;
        Job& j = A.job[A.n_jobs++];
        j.src = src; j.pstride = pstride; j.nparts = nparts; j.width = width; j.dst = dst;
        j.op = op; j.aux = aux; j.blocks = (width + 31) / 32;
        blocks += j.blocks;
    }
};

}  // namespace nsm
}  // namespace regnn

using namespace regnn;
using namespace regnn::nsm;

int regnn_nsm_rel0(const regnn_nsm_params* p, const regnn_nsm_work* w, float* slab,
                   hipStream_t stream) {
    const int T = p->n_types, K = p->k_in, L = p->n_layers, h = L - 1;
    Ptrs xt{};
    for (int t = 0; t < T; ++t) xt.p[t] = p->x_tab[t];
    Rel0Args R{};
    R.sizes = w->sizes; R.hop = h; R.T = T;
    R.ptr = w->blk_ptr[h]; R.cnt = w->blk_cnt[h]; R.stride = w->stride[h];
    R.rel = w->blk_rel[h]; R.edge_type = w->edge_type;
    R.edge_off = w->edge_off; R.xt = xt; R.z = w->z; R.beta = w->beta;
    R.slab = slab; R.n_rel = p->n_rel[0];
    const size_t lds = size_t(p->n_rel[0]) * kBlock * sizeof(float);
    if (K == 128)
        hipLaunchKernelGGL(rel0_kernel<128>, dim3(kAggBlocks), dim3(kBlock), lds, stream, R);
    else
        hipLaunchKernelGGL(rel0_kernel<64>, dim3(kAggBlocks), dim3(kBlock), lds, stream, R);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

extern "C" {

int64_t regnn_nsm_slab_floats(const regnn_nsm_params* p, int32_t cap0) {
    if (!p || cap0 <= 0) return -1;
    if (regnn_nsm2_covers(p)) return regnn_nsm2_slab_floats(p, cap0);
    return slab_layout(p, cap0).total;
}

int regnn_nsm_step(const regnn_nsm_params* p, const regnn_nsm_work* w, hipStream_t stream) {
    if (!p || !w) return REGNN_EINVAL;
    const int T = p->n_types, K = p->k_in, L = p->n_layers, C = p->n_classes;
    if (T < 1 || T > MT || L < 2 || L > ML || C < 1 || C > 448 || (K != 64 && K != 128) ||
        T * (K + 1) > 600 || !(p->p_drop >= 0.f && p->p_drop < 1.f))
        return REGNN_EUNSUPPORTED;
    for (int l = 0; l < L; ++l)
        if (p->n_rel[l] < 1 || p->n_rel[l] > F) return REGNN_EUNSUPPORTED;
    if (!w->state || !w->sizes || !w->n_id || !w->ntype || !w->local || !w->labels || !w->wc ||
        !w->gwc || !w->tabs || !w->nvalid || !w->edge_type || !w->edge_off || !w->s_agg ||
        !w->s_w || !w->z || !w->beta || !w->slab ||
        !p->loss || !p->out_w || !p->out_b || !p->g_out_w || !p->g_out_b || w->cap[0] <= 0)
        return REGNN_EINVAL;
    for (int t = 0; t < T; ++t)
        if (!p->x_tab[t] || !p->lin_w[t] || !p->lin_b[t] || !p->g_lin_w[t] || !p->g_lin_b[t])
            return REGNN_EINVAL;
    for (int l = 0; l < L; ++l) {
        const int h = L - 1 - l;
        if (!p->conv_w[l] || !p->conv_b[l] || !p->conv_rw[l] || !p->ln_w[l] || !p->ln_b[l] ||
            !p->g_conv_w[l] || !p->g_conv_b[l] || !p->g_conv_rw[l] || !p->g_ln_w[l] ||
            !p->g_ln_b[l] || (l > 0 && (!w->xs[l] || !w->gxs[l])) || !w->ga[l] || !w->blk_ptr[h] ||
            !w->blk_idx[h] || !w->blk_rel[h] || !w->blk_inv[h] || w->cap[h] <= 0 ||
            w->cap[h + 1] <= 0)
            return REGNN_EINVAL;
        if (l < L - 1 && (!w->a[l] || !w->stats[l])) return REGNN_EINVAL;
    }
    // relation-slot mode: the caller vouches that every (target type, source type) pair has at
    // most one relation besides the self loops (relation ids >= n_edge_types)
    const bool rs = p->rel_slots != 0;
    if (rs && (!w->u_self || !w->u_rel || p->n_edge_types < 0 || p->n_edge_types + T > p->n_rel[0]))
        return REGNN_EINVAL;
    if (w->part < 0 || w->part > 2) return REGNN_EINVAL;
    if (regnn_nsm2_covers(p)) return regnn_nsm2_step(p, w, stream);
    // the fused optimizer, the strided blocks and the split into parts: two-layer step only
    if (w->part) return REGNN_EUNSUPPORTED;
    if (w->adam) return REGNN_EUNSUPPORTED;
    for (int h = 0; h < L; ++h)
        if (w->stride[h]) return REGNN_EUNSUPPORTED;
    const SlabLayout S = slab_layout(p, w->cap[0]);
    const Drop drop = make_drop(p->p_drop);
    Ptrs lin_w{}, lin_b{}, xt{}, rw{};
    for (int t = 0; t < T; ++t) {
        lin_w.p[t] = p->lin_w[t];
        lin_b.p[t] = p->lin_b[t];
        xt.p[t] = p->x_tab[t];
    }
    for (int l = 0; l < L; ++l) rw.p[l] = p->conv_rw[l];

    // 1. composed first map + relation tables
    Ints nrel{};
    for (int l = 0; l < L; ++l) nrel.v[l] = p->n_rel[l];
    hipLaunchKernelGGL(prep_kernel, dim3(T * (K + 1) + L), dim3(64), 0, stream, T, K, lin_w,
                       lin_b, p->conv_w[0], rw, L, nrel, p->alpha, w->wc, w->tabs);
    REGNN_LAUNCH_CHECK();
    // 2. layer 0: gather per source type, project per target row, LayerNorm ... x @ W_1
    {
        const int h = L - 1;
        Agg0Args A{};
        A.sizes = w->sizes; A.hop = h;
        A.ptr = w->blk_ptr[h]; A.rel = w->blk_rel[h]; A.inv = w->blk_inv[h];
        A.edge_type = w->edge_type; A.edge_off = w->edge_off; A.xt = xt; A.T = T; A.wc = w->wc;
        A.n_id = w->n_id; A.labels = w->labels; A.nvalid = w->nvalid;
        A.tab = w->tabs; A.bias = p->conv_b[0]; A.ln_w = p->ln_w[0]; A.ln_b = p->ln_b[0];
        A.state = w->state; A.drop = drop; A.w_next = p->conv_w[1];
        A.s_agg = w->s_agg; A.s_w = w->s_w;
        A.a = w->a[0]; A.stats = w->stats[0]; A.xs_next = w->xs[1]; A.gxs_next = w->gxs[1];
        A.n_et = p->n_edge_types; A.u_self = w->u_self; A.u_rel = w->u_rel;
        int grid = (w->cap[h] + 15) / 16;
        if (grid > 2048) grid = 2048;
        const size_t lds = agg0_lds(T, K);
#define AGG0_CASE(KK, NN, RS)                                                                  \
        if (K == KK && (NN == MT || T <= NN) && rs == RS) {                                    \
            static size_t done = 0;                                                            \
            if (!set_lds(reinterpret_cast<const void*>(&agg0_kernel<KK, NN, RS>), lds, &done)) \
                return REGNN_EUNSUPPORTED;                                                     \
            hipLaunchKernelGGL((agg0_kernel<KK, NN, RS>), dim3(grid), dim3(kBlock), lds, stream, A); \
            REGNN_LAUNCH_CHECK();                                                              \
        } else
        AGG0_CASE(128, 4, true) AGG0_CASE(128, MT, true) AGG0_CASE(64, 4, true)
        AGG0_CASE(64, MT, true) AGG0_CASE(128, 4, false) AGG0_CASE(128, MT, false)
        AGG0_CASE(64, 4, false) AGG0_CASE(64, MT, false)
            return REGNN_EUNSUPPORTED;
#undef AGG0_CASE
    }
    // 3. layers 1 .. L-2
    for (int l = 1; l < L - 1; ++l) {
        const int h = L - 1 - l;
        AggArgs A{};
        A.sizes = w->sizes; A.hop = h;
        A.ptr = w->blk_ptr[h]; A.idx = w->blk_idx[h]; A.rel = w->blk_rel[h]; A.inv = w->blk_inv[h];
        A.tab = w->tabs + l * F; A.xs = w->xs[l]; A.bias = p->conv_b[l];
        A.ln_w = p->ln_w[l]; A.ln_b = p->ln_b[l]; A.state = w->state; A.layer = l; A.drop = drop;
        A.w_next = p->conv_w[l + 1];
        A.a = w->a[l]; A.stats = w->stats[l]; A.xs_next = w->xs[l + 1]; A.gxs_next = w->gxs[l + 1];
        int grid = (w->cap[h] + 15) / 16;
        if (grid > 1024) grid = 1024;
        hipLaunchKernelGGL(agg_kernel, dim3(grid), dim3(kBlock), 0, stream, A);
        REGNN_LAUNCH_CHECK();
    }
    // 4. last layer + head + loss + backward to its pre-LN rows
    const int64_t hw = head_part_width(C);
    {
        const int l = L - 1;
        HeadArgs H{};
        H.sizes = w->sizes; H.n_id = w->n_id; H.labels = w->labels;
        H.ptr = w->blk_ptr[0]; H.idx = w->blk_idx[0]; H.rel = w->blk_rel[0]; H.inv = w->blk_inv[0];
        H.tab = w->tabs + l * F; H.xs = w->xs[l]; H.bias = p->conv_b[l];
        H.ln_w = p->ln_w[l]; H.ln_b = p->ln_b[l]; H.state = w->state; H.layer = l; H.drop = drop;
        H.w_out = p->out_w; H.b_out = p->out_b; H.C = C;
        H.ga = w->ga[l]; H.nvalid = w->nvalid; H.part = w->slab + S.head; H.part_w = hw;
        const size_t lds = head_lds(C);
        static size_t done = 0;
        if (lds > 156 * 1024 || !set_lds(reinterpret_cast<const void*>(&head_kernel), lds, &done))
            return REGNN_EUNSUPPORTED;
        hipLaunchKernelGGL(head_kernel, dim3(S.head_blocks), dim3(kBlock), lds, stream, H);
        REGNN_LAUNCH_CHECK();
    }
    // 5. backward, last layer first, down to layer 0's pre-LN rows
    for (int l = L - 1; l >= 1; --l) {
        const int h = L - 1 - l;
        AggBwdArgs B{};
        B.sizes = w->sizes; B.hop = h;
        B.ptr = w->blk_ptr[h]; B.idx = w->blk_idx[h]; B.rel = w->blk_rel[h]; B.inv = w->blk_inv[h];
        B.tab = w->tabs + l * F; B.xs = w->xs[l]; B.ga = w->ga[l]; B.gxs = w->gxs[l];
        B.slab = w->slab + S.rel[l]; B.n_rel = p->n_rel[l];
        hipLaunchKernelGGL(agg_bwd_kernel, dim3(kAggBlocks), dim3(kBlock),
                           size_t(p->n_rel[l]) * kBlock * sizeof(float), stream, B);
        REGNN_LAUNCH_CHECK();
        PostArgs Q{};
        const int lp = l - 1, hp = L - 1 - lp;
        Q.sizes = w->sizes; Q.hop = hp;
        Q.a = w->a[lp]; Q.stats = w->stats[lp]; Q.ln_w = p->ln_w[lp]; Q.ln_b = p->ln_b[lp];
        Q.state = w->state; Q.layer = lp; Q.drop = drop;
        Q.w_next = p->conv_w[l]; Q.gxs_next = w->gxs[l];
        Q.ga = w->ga[lp]; Q.slab = w->slab + S.post[lp];
        hipLaunchKernelGGL(post_bwd_kernel, dim3(kPostBlocks), dim3(kBlock), 0, stream, Q);
        REGNN_LAUNCH_CHECK();
    }
    // 6. layer 0: the composed map's gradient and Z / beta per target row and type, then the
    //    relation-table dots edge by edge
    {
        const int h = L - 1;
        Bwd0Args B{};
        B.sizes = w->sizes; B.hop = h; B.T = T;
        B.inv = w->blk_inv[h]; B.ga = w->ga[0]; B.s_agg = w->s_agg; B.s_w = w->s_w; B.wc = w->wc;
        B.z = w->z; B.beta = w->beta; B.slab = w->slab + S.proj;
        const dim3 grid(kProjBlocks, T);
        if (rs) {
            B.tab = w->tabs; B.u_self = w->u_self; B.u_rel = w->u_rel;
            B.n_rel = p->n_rel[0]; B.n_et = p->n_edge_types; B.rslab = w->slab + S.rel[0];
            const size_t lds = bwd0_rs_lds(K, p->n_rel[0]);
            static size_t done128 = 0, done64 = 0;
            const void* kfn = K == 128 ? reinterpret_cast<const void*>(&bwd0_rs_kernel<128>)
                                       : reinterpret_cast<const void*>(&bwd0_rs_kernel<64>);
            if (!set_lds(kfn, lds, K == 128 ? &done128 : &done64)) return REGNN_EUNSUPPORTED;
            if (K == 128)
                hipLaunchKernelGGL(bwd0_rs_kernel<128>, grid, dim3(kBlock), lds, stream, B);
            else
                hipLaunchKernelGGL(bwd0_rs_kernel<64>, grid, dim3(kBlock), lds, stream, B);
            REGNN_LAUNCH_CHECK();
        } else if (K == 128) {
            hipLaunchKernelGGL(bwd0_kernel<128>, grid, dim3(kBlock), 0, stream, B);
        } else {
            hipLaunchKernelGGL(bwd0_kernel<64>, grid, dim3(kBlock), 0, stream, B);
        }
        REGNN_LAUNCH_CHECK();
    }
    if (!rs) {
        const int rc = regnn_nsm_rel0(p, w, w->slab + S.rel[0], stream);
        if (rc != REGNN_OK) return rc;
    }
    // 7. reductions of every partial into the gradients (and the composed map's gradient)
    {
        JobList J;
        J.A.alpha = p->alpha;
        const float* hp = w->slab + S.head;
        const int nh = S.head_blocks;
        J.add(hp, hw, nh, C * F, p->g_out_w);
        J.add(hp + int64_t(C) * F, hw, nh, C, p->g_out_b);
        J.add(hp + int64_t(C) * (F + 1), hw, nh, F, p->g_conv_b[L - 1]);
        J.add(hp + int64_t(C) * (F + 1) + F, hw, nh, F, p->g_ln_b[L - 1]);
        J.add(hp + int64_t(C) * (F + 1) + 2 * F, hw, nh, F, p->g_ln_w[L - 1]);
        J.add(hp + int64_t(C) * (F + 1) + 3 * F, hw, nh, 1, p->loss, kOpLoss, w->nvalid);
        for (int l = 0; l < L; ++l)
            J.add(w->slab + S.rel[l], F, (l == 0 && rs) ? kProjBlocks * T : kAggBlocks,
                  p->n_rel[l], p->g_conv_rw[l], kOpRel, p->conv_rw[l]);
        for (int l = 0; l + 1 < L; ++l) {
            const float* pp = w->slab + S.post[l];
            J.add(pp, kPostW, kPostBlocks, F * F, p->g_conv_w[l + 1]);
            J.add(pp + F * F, kPostW, kPostBlocks, F, p->g_conv_b[l]);
            J.add(pp + F * F + F, kPostW, kPostBlocks, F, p->g_ln_b[l]);
            J.add(pp + F * F + 2 * F, kPostW, kPostBlocks, F, p->g_ln_w[l]);
        }
        const int64_t pw = int64_t(K + 1) * F;
        for (int t = 0; t < T; ++t)
            J.add(w->slab + S.proj + int64_t(t) * kProjBlocks * pw, pw, kProjBlocks, int(pw),
                  w->gwc + t * pw);
        hipLaunchKernelGGL(finalize_kernel, dim3(J.blocks), dim3(kBlock), 0, stream, J.A);
        REGNN_LAUNCH_CHECK();
    }
    // 8. chain rule onto lins[t] and convs[0].weight
    {
        ChainArgs A{};
        A.T = T; A.K = K; A.lin_w = lin_w; A.lin_b = lin_b; A.w0 = p->conv_w[0]; A.gwc = w->gwc;
        for (int t = 0; t < T; ++t) {
            A.g_lin_w[t] = p->g_lin_w[t];
            A.g_lin_b[t] = p->g_lin_b[t];
        }
        A.g_w0 = p->g_conv_w[0];
        if (K == 128)
            hipLaunchKernelGGL(chain_kernel<128>, dim3(F + T * F), dim3(kBlock), 0, stream, A);
        else
            hipLaunchKernelGGL(chain_kernel<64>, dim3(F + T * F), dim3(kBlock), 0, stream, A);
        REGNN_LAUNCH_CHECK();
    }
    return REGNN_OK;
}

int regnn_adam_flat(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                    float lr, float beta1, float beta2, float eps, float weight_decay,
                    float grad_scale, int64_t* step, uint32_t* ticket, hipStream_t stream) {
    if (!param || !grad || !exp_avg || !exp_avg_sq || !step || n < 0) return REGNN_EINVAL;
    if (n == 0) return REGNN_OK;
    auto al = [](const void* q) { return reinterpret_cast<uintptr_t>(q) % 16 == 0; };
    const bool vec = n % 4 == 0 && al(param) && al(grad) && al(exp_avg) && al(exp_avg_sq);
    int64_t grid = (n / (vec ? 4 : 1) + kBlock - 1) / kBlock;
    if (grid > 1024) grid = 1024;
    if (vec)
        hipLaunchKernelGGL(adam_flat_kernel<4>, dim3(unsigned(grid)), dim3(kBlock), 0, stream, param,
                           grad, exp_avg, exp_avg_sq, n, lr, beta1, beta2, eps, weight_decay,
                           grad_scale, step, ticket);
    else
        hipLaunchKernelGGL(adam_flat_kernel<1>, dim3(unsigned(grid)), dim3(kBlock), 0, stream, param,
                           grad, exp_avg, exp_avg_sq, n, lr, beta1, beta2, eps, weight_decay,
                           grad_scale, step, ticket);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

}  // extern "C"
