// Two-layer fused NS model step (regnn_nsm_step with L = 2, the reference's num_layers default):
// the REGNN of mag/regnn_ns.py:216-346 ('regcn', self_loop_type 2, LayerNorm, hidden 64) forward
// + nll_loss + backward over the blocks regnn_ns_hop wrote, in five launches (six without
// relation slots), every reduction in a fixed order or exact: two runs of a step give bitwise
// equal gradients. Optionally the Adam update of every parameter ends the last launch.
//
//   agg0      layer 0 (group_input mag/regnn_ns.py:300-326 + REGCNConv mag/regnn_layers.py:
//             80-150): the sampled input rows summed per target row and source type, projected
//             in two fp32-MFMA stages -- P = sum_t (S_t W_t^T + w_t b_t) (group_input's Linear,
//             moved after the mean aggregation by linearity) and a = inv (P W_0) + bias (the
//             conv's x @ W) -- then LayerNorm, relu, dropout -> h0. Keeps P, a and the LN stats
//             for the backward.
//   head      layer 1 aggregated first and projected second (a = inv (sum_e tab[r_e] h0[u_e]) W_1
//             + bias, the same linearity), LayerNorm, relu, dropout, out_lin, log_softmax,
//             nll_loss (mean over the labelled targets) and the backward to GH = inv ga W_1^T.
//   gather    layer 1's transposed aggregation as a gather over the sampler's transposed index
//             of hop 0's block (a 16-lane group per layer-0 row, every CU): gh0[u] = sum over u's
//             edges of tab[r] GH[v] and the relation-table dots <h0[u], GH[v]>, both as exact
//             2^-40 fixed-point integer sums (the segment order does not matter), then the
//             LayerNorm / relu / dropout backward -> G0 = inv ga0 rows and their row terms.
//   bwd0      layer 0's backward per target row: gP = G0 W_0^T, the W_0 gradient P^T G0; per
//             source type t the
//             weight gradient gP^T S_t, the bias term, and the relation-table dots from
//             Z_t = gP W_t (relation slots: <U_t, Z_t> in registers; else Z and beta for rel0).
//   rel0      (no relation slots) layer 0's relation-table dots edge by edge (re_nsm.hip).
//   finalize  every gradient as a fixed-order sum of per-block partials; with an optimizer
//             attached, Adam (regnn_adam_flat's arithmetic) on each element right after its sum.
#include "re_nsm_common.h"

#include <cstdlib>

namespace regnn {
namespace nsm2 {
using namespace regnn::nsm;

constexpr int kRows = 16;                  // target rows per block (one MFMA row tile)
// bwd0 blocks per node type and gather blocks (the slab layout follows them). The defaults are
// the measured choice; REGNN_NSM_BWD_BLOCKS / REGNN_NSM_GATH_BLOCKS override them for A/B runs
// (read once per process, so regnn_nsm_slab_floats and regnn_nsm_step agree).
inline int env_blocks(const char* name, int dflt) {
    const char* e = getenv(name);
    const int v = e ? atoi(e) : 0;
    return v >= 16 && v <= 4096 ? v : dflt;
}
static const int kBwdBlocks = env_blocks("REGNN_NSM_BWD_BLOCKS", 128);   // wave groups per type
// bwd0's wave groups per block (REGNN_NSM_BWD_GROUPS, 1 or 2): two groups in half the blocks
// (one 512-thread block per CU) share the W_t image and sum their partials in LDS
static const int kBwdGroups = [] {
    const char* e = getenv("REGNN_NSM_BWD_GROUPS");
    return e && e[0] == '1' ? 1 : 2;
}();
constexpr int kMaxCT = 27;                 // class tiles of 16 (the head's LDS holds C <= 384)
constexpr float kFixScale = 1099511627776.0f;      // 2^40: fixed point of layer 1's scatter
constexpr float kFixInv = 9.094947017729282e-13f;  // 2^-40

// terms are rounded to 2^-40; an int64 sum holds |total| < 2^23. Every term is checked against
// kFixTermMax = 2^8, so sums of up to 2^15 terms (a hub row's 32768 entries, a block's relation
// bins) cannot wrap: gradient rows of a mean loss are many orders of magnitude inside that
// range, and the rounding (<= 4.6e-13 per term) is far below fp32 resolution of the sums it
// feeds. A term outside it (or NaN) sets the step's overflow flag and the step's loss reads NaN.
constexpr float kFixTermMax = 256.f;
// rn(x 2^40) as an int64 for |x 2^40| < 2^51 (= __float2ll_rn(x * 2^40), ties to even): x 2^40
// is exact in fp64, the fma adds 1.5 2^52 so the rounding lands on the integer in the low
// mantissa bits; subtracting the constant's bit pattern leaves the two's complement value (two
// fp64 / two integer instructions instead of the generic f32 -> i64 conversion sequence)
__device__ __forceinline__ unsigned long long to_fix(float x) {
    const double d = __builtin_fma(double(x), 1099511627776.0, 6755399441055744.0);
    return (unsigned long long)(__double_as_longlong(d) - 0x4338000000000000ll);
}
__device__ __forceinline__ unsigned long long to_fix_chk(float x, bool& bad) {
    bad |= !(fabsf(x) < kFixTermMax);
    return to_fix(fminf(fmaxf(x, -kFixTermMax), kFixTermMax));
}

__device__ __forceinline__ float from_fix(unsigned long long q) {
    return float((long long)q) * kFixInv;
}

// relation table entry j of LeakyReLU(alpha * relation_weight) (mag/regnn_layers.py:109-111)
__device__ __forceinline__ float rel_tab(const float* rw, int nr, float alpha, int j) {
    if (j >= nr) return 0.f;
    const float x = rw[j] * alpha;
    return x > 0.f ? x : 0.01f * x;
}

// phase timestamps of an instrumented build (-DREGNN_NSM2_PHASES, tools/nsm2_phases.py only):
// thread 0 of blocks < 32 records wall_clock64() at marked points of each kernel
#ifdef REGNN_NSM2_PHASES
__device__ unsigned long long g_nsm2_phase[4][32][16];
#define PH(kern, k)                                                                            \
    do {                                                                                       \
        if (threadIdx.x == 0 && blockIdx.x < 32 && blockIdx.y == 0)                             \
            g_nsm2_phase[kern][blockIdx.x][k] = wall_clock64();                                \
    } while (0)
// entry / exit of every block (kern 0 agg0, 1 head, 2 gather, 3 bwd0, 4 finalize)
__device__ unsigned long long g_nsm2_edge[5][2][4096];
// the gather's hub pieces (j < 64): marks along the piece path
__device__ unsigned long long g_nsm2_gp[64][8];
#define PG(j, k)                                                                               \
    do {                                                                                       \
        if (threadIdx.x == 0 && (j) < 64) g_nsm2_gp[j][k] = wall_clock64();                    \
    } while (0)
#define PE(kern, k)                                                                            \
    do {                                                                                       \
        const unsigned b_ = blockIdx.x + blockIdx.y * gridDim.x;                               \
        if (threadIdx.x == 0 && b_ < 4096) g_nsm2_edge[kern][k][b_] = wall_clock64();          \
    } while (0)
#else
#define PH(kern, k) do {} while (0)
#define PE(kern, k) do {} while (0)
#define PG(j, k) do {} while (0)
#endif

#define MFMA4(av, b0, b1, b2, b3, d)                                 \
    d = __builtin_amdgcn_mfma_f32_16x16x4f32((av).x, (b0), d, 0, 0, 0); \
    d = __builtin_amdgcn_mfma_f32_16x16x4f32((av).y, (b1), d, 0, 0, 0); \
    d = __builtin_amdgcn_mfma_f32_16x16x4f32((av).z, (b2), d, 0, 0, 0); \
    d = __builtin_amdgcn_mfma_f32_16x16x4f32((av).w, (b3), d, 0, 0, 0)

// ---------------------------------------------------------------------------------------------
// agg0. MFMA lane (c, q) of wave w: A = tile row c, k = 16 b + 4 q + i (i: the 4 instructions of
// a float4), B = column 16 w + c; D row 4 q + r, column 16 w + c.
struct Agg0Args {
    const int32_t* sizes; int hop;
    const int32_t* ptr; const int32_t* cnt; int stride; const uint8_t* rel; const float* inv;
    const int32_t* edge_type; const int64_t* edge_off; Ptrs xt; int T;
    Ptrs lin_w; Ptrs lin_b;                // lins[t].weight [64][K] (row j, column k), bias [64]
    const float* rw; int n_rel; float alpha;
    const float* w0; const float* bias; const float* ln_w; const float* ln_b;
    const int64_t* state; Drop drop;
    float* s_agg; float* s_w;
    float* a; float* stats; float* h; float* p;
    // the labelled-target count nll_loss divides by (the last block; the head reads it)
    const int32_t* n_id; const int64_t* labels; float* nvalid;
    // relation slots (RS): s_agg / s_w hold the unweighted sums / counts of the non-self edges
    // per source type, u_self the self loop's input row, u_rel [n][T + 1] each slot's relation
    int n_et; float* u_self; int32_t* u_rel;
};

// LDS: S tile [16][T K + 4] | s_w [16][MT] | P [16][68] | pre-LN rows [16][64] | table [64] |
// W_0 [64][64]
inline size_t agg0_lds(int T, int K) {
    return (size_t(16) * (T * K + 4) + 16 * MT + 16 * 68 + 16 * F + F + F * F) * sizeof(float);
}

template <int K, int NT, bool RS>
__global__ void __launch_bounds__(kBlock, 2) agg0_kernel(Agg0Args A) {
    constexpr int VPL = K / 64;            // float4 per lane of a K-wide row (16 lanes per row)
    constexpr int KB = K / 16;
    constexpr int HB = KB / 2;             // float4 steps per half type
    extern __shared__ float sm[];
    PH(0, 12);
    PE(0, 0);
    const int T = A.T;
    const int SR = T * K + 4;
    float* St = sm;                        // [16][SR]
    float* sw = St + 16 * SR;              // [16][MT]
    float* Pt = sw + 16 * MT;              // [16][68]
    float* at = Pt + 16 * 68;              // [16][F]
    float* tab = at + 16 * F;              // [F]
    float* w0s = tab + F;                  // [F][F]: W_0 (the second stage's B operand)
    if (threadIdx.x < F) tab[threadIdx.x] = rel_tab(A.rw, A.n_rel, A.alpha, threadIdx.x);
    for (int i = threadIdx.x; i < F * F / 4; i += kBlock)
        reinterpret_cast<float4*>(w0s)[i] = reinterpret_cast<const float4*>(A.w0)[i];
    const int n = A.sizes[A.hop];
    const int l = threadIdx.x & 15, sub = threadIdx.x >> 4, gl = threadIdx.x & 48;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4;
    const uint32_t key = A.drop.on ? layer_key(A.state, 0) : 0u;
    const float4 gw = reinterpret_cast<const float4*>(A.ln_w)[l];
    const float4 gb = reinterpret_cast<const float4*>(A.ln_b)[l];
    const float bj = A.bias[16 * w + c];
    float lbj[NT];                         // lins[t].bias[16 w + c]: stage 1's bias terms
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) lbj[tt] = tt < T ? pick(A.lin_b.p, tt)[16 * w + c] : 0.f;
    PH(0, 0);
    if (blockIdx.x == gridDim.x - 1) {         // block-uniform
        __shared__ int cntw[kBlock / 64];
        int cv = 0;
        const int nb = A.sizes[0];
        for (int i = threadIdx.x; i < nb; i += kBlock) cv += A.labels[A.n_id[i]] >= 0 ? 1 : 0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) cv += __shfl_xor(cv, o, 64);
        if ((threadIdx.x & 63) == 0) cntw[threadIdx.x >> 6] = cv;
        __syncthreads();
        if (threadIdx.x == 0) *A.nvalid = float((cntw[0] + cntw[1]) + (cntw[2] + cntw[3]));
    }
    __syncthreads();
    for (int base = blockIdx.x * 16; base < n; base += gridDim.x * 16) {
        // stage 1's first two W_t fragments are requested before the gather (their L2 latency
        // under it); stage 1 then keeps two fragments in flight
        constexpr int PD = NT <= 4 ? 2 : 1;      // fragments in flight (8 node types: 1, VGPRs)
        float4 bq[PD + 1][HB];
        auto bload = [&](int step, float4 (&dst)[HB]) {
            const int tt = step >> 1, h0 = (step & 1) * HB;
            const float* wt = pick(A.lin_w.p, tt) + (16 * w + c) * K + 4 * q + 16 * h0;
#pragma unroll
            for (int b = 0; b < HB; ++b) dst[b] = *reinterpret_cast<const float4*>(wt + 16 * b);
        };
        if constexpr (PD == 2) {                     // 2 T >= 2: a type has two halves
            bload(0, bq[0]);
            bload(1, bq[1]);
        }
        // ---- gather: per-type register sums of this lane's 4 * VPL features
        const int v = base + sub;
        float iv4[4];                      // stage 2's row scales, requested before the gather
#pragma unroll
        for (int r = 0; r < 4; ++r) iv4[r] = base + 4 * q + r < n ? A.inv[base + 4 * q + r] : 0.f;
        float wsum[NT];
        float4 racc[NT][VPL];
        int rel_t[NT];
        float4 xself[VPL];
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
            int e0, e1;
            row_range(A.ptr, A.cnt, A.stride, v, e0, e1);
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
                constexpr int UN = 8;              // edges' rows in flight per lane
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
        PH(0, 1);
        if constexpr (PD == 1) bload(0, bq[0]);      // (8 node types: after the gather)
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
        PH(0, 2);
        // ---- stage 1: P[v][j] = sum_t S_vt W_t[j][:] + w_vt b_t[j]; type t + 1's rows of W_t
        // are loaded while type t's products run
        f32x4 d = {0.f, 0.f, 0.f, 0.f};
        if constexpr (PD == 2) {
#pragma unroll
            for (int step = 0; step < 2 * NT; ++step) {
                if (step < 2 * T) {
                    if (step + 2 < 2 * T) bload(step + 2, bq[(step + 2) % 3]);
                    const float* sa = St + c * SR + (step >> 1) * K + 16 * (step & 1) * HB + 4 * q;
#pragma unroll
                    for (int b = 0; b < HB; ++b) {
                        const float4 av = *reinterpret_cast<const float4*>(sa + 16 * b);
                        const float4 bv = bq[step % 3][b];
                        MFMA4(av, bv.x, bv.y, bv.z, bv.w, d);
                    }
                }
            }
        } else {
            for (int step = 0; step < 2 * T; ++step) {
                if (step + 1 < 2 * T) bload(step + 1, bq[1]);
                const float* sa = St + c * SR + (step >> 1) * K + 16 * (step & 1) * HB + 4 * q;
#pragma unroll
                for (int b = 0; b < HB; ++b) {
                    const float4 av = *reinterpret_cast<const float4*>(sa + 16 * b);
                    MFMA4(av, bq[0][b].x, bq[0][b].y, bq[0][b].z, bq[0][b].w, d);
                }
#pragma unroll
                for (int b = 0; b < HB; ++b) bq[0][b] = bq[1][b];
            }
        }
        {
            const int j = 16 * w + c;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int vr = 4 * q + r;
                float bsum = 0.f;
#pragma unroll
                for (int tt = 0; tt < NT; ++tt)
                    if (tt < T) bsum = fmaf(sw[vr * MT + tt], lbj[tt], bsum);
                Pt[vr * 68 + j] = d[r] + bsum;
            }
        }
        __syncthreads();
        PH(0, 3);
        // ---- stage 2: a = inv (P W_0) + bias
        {
            f32x4 d2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const float4 av = *reinterpret_cast<const float4*>(Pt + c * 68 + 16 * b + 4 * q);
                const float* wb = w0s + (16 * b + 4 * q) * F + 16 * w + c;     // W_0[k][16 w + c]
                MFMA4(av, wb[0], wb[F], wb[2 * F], wb[3 * F], d2);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) at[(4 * q + r) * F + 16 * w + c] = fmaf(iv4[r], d2[r], bj);
        }
        __syncthreads();
        // ---- epilogue: P and a kept, LayerNorm, relu, dropout -> h0
        if (v < n) {
            *reinterpret_cast<float4*>(A.p + int64_t(v) * F + 4 * l) =
                *reinterpret_cast<const float4*>(Pt + sub * 68 + 4 * l);
            const float4 a4 = *reinterpret_cast<const float4*>(at + sub * F + 4 * l);
            const float av[4] = {a4.x, a4.y, a4.z, a4.w};
            *reinterpret_cast<float4*>(A.a + int64_t(v) * F + 4 * l) = a4;
            const float mean = group_sum<16>(av[0] + av[1] + av[2] + av[3]) * (1.f / F);
            const float dd[4] = {av[0] - mean, av[1] - mean, av[2] - mean, av[3] - mean};
            const float var = group_sum<16>(dd[0] * dd[0] + dd[1] * dd[1] + dd[2] * dd[2] + dd[3] * dd[3]) * (1.f / F);
            const float rstd = rsqrtf(var + kLnEps);
            if (l == 0) reinterpret_cast<float2*>(A.stats)[v] = make_float2(mean, rstd);
            const float gws[4] = {gw.x, gw.y, gw.z, gw.w}, gbs[4] = {gb.x, gb.y, gb.z, gb.w};
            float mk[4];
            drop_factors(key, A.drop, v, l, mk);
            float hv[4];
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) hv[cc] = fmaxf(fmaf(dd[cc] * rstd, gws[cc], gbs[cc]), 0.f) * mk[cc];
            *reinterpret_cast<float4*>(A.h + int64_t(v) * F + 4 * l) = make_float4(hv[0], hv[1], hv[2], hv[3]);
        }
        __syncthreads();                       // the tiles are reused by the next rows
        PH(0, 4);
    }
    PE(0, 1);
}

// agg0 for 128-wide input rows: 16 rows x 32 lanes (one float4 of the row per lane), 512 threads,
// <= 128 VGPRs and ~46 KB of LDS so two blocks share a CU and every tile of a batch (~350 of the
// capacity's 832) is resident at once; stage 1's eight waves split the node types in two halves
// whose partial products meet in LDS in a fixed order. Same outputs as agg0_kernel<128, ..>.
constexpr int kAggW = 512;
// rows of a tile (<= 16: the MFMA tiles stay 16 rows, the rest are padding). 12 / 14 rows (more,
// lighter tiles for the CUs that hold two) measured 109.1-109.8 / 107.4-108.4 against 107.9 us
#ifndef REGNN_AGG_ROWS
#define REGNN_AGG_ROWS 16
#endif
constexpr int kAggRows = REGNN_AGG_ROWS;
// with the sampler's sums (PRE), stage 1's W_t fragments are all requested at the kernel's start
#ifndef REGNN_AGG0_EARLY_W
#define REGNN_AGG0_EARLY_W 1
#endif

inline size_t agg0w_lds(int T) {          // St [16][T K + 4] | sw [16][MT] | Pt [16][68] |
    return (size_t(16) * (T * 128 + 4) + 16 * MT + 16 * 68 + 16 * F + 16 * F) * sizeof(float);
}                                         // at [16][64] | red [16][64]

// PRE (relation slots): the row's per-type input sums, counts, self row and slot relations were
// formed by the sampler (regnn_ns_hop_typed_sums into s_agg / s_w / u_self / u_rel): the gather
// phase is one round of contiguous loads, and nothing of them is written here
template <int NT, bool RS, bool PRE = false>
__global__ void __launch_bounds__(kAggW, 4) agg0w_kernel(Agg0Args A) {
    static_assert(!PRE || RS, "the sampler's sums need relation slots");
    constexpr int K = 128, HB = K / 32;    // float4 steps per half type (stage 1)
    extern __shared__ float sm[];
    PH(0, 12);
    PE(0, 0);
    const int T = A.T;
    const int SR = T * K + 4;
    float* St = sm;                        // [16][SR]
    float* sw = St + 16 * SR;              // [16][MT]
    float* Pt = sw + 16 * MT;              // [16][68]
    float* at = Pt + 16 * 68;              // [16][F]
    float* red = at + 16 * F;              // [16][F]: stage 1's second half
    const int n = A.sizes[A.hop];
    const int l = threadIdx.x & 31, sub = threadIdx.x >> 5, gl = threadIdx.x & 32;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4;
    const int ct = w & 3, kh = w >> 2;     // stage 1: column tile, type half
    if (blockIdx.x == gridDim.x - 1) {     // block-uniform: the labelled-target count
        __shared__ int cntw[kAggW / 64];
        int cv = 0;
        const int nb = A.sizes[0];
        for (int i = threadIdx.x; i < nb; i += kAggW) cv += A.labels[A.n_id[i]] >= 0 ? 1 : 0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) cv += __shfl_xor(cv, o, 64);
        if (lane == 0) cntw[w] = cv;
        __syncthreads();
        if (threadIdx.x == 0) {
            int t = 0;
            for (int k = 0; k < kAggW / 64; ++k) t += cntw[k];
            *A.nvalid = float(t);
        }
    }
    const int base = blockIdx.x * kAggRows;
    if (base >= n) return;                 // block-uniform (the grid is capacity-sized)
    // PRE: every W_t fragment stage 1 reads (this wave's types, both halves) requested first,
    // under the input loads: nothing they depend on is produced in this kernel
    const int nst = 2 * ((T - kh + 1) / 2);                 // stage-1 steps of this wave's types
    constexpr bool EW = PRE && REGNN_AGG0_EARLY_W;
    float4 bq_all[EW ? NT : 1][K / 32];
    if constexpr (EW) {
#pragma unroll
        for (int step = 0; step < NT; ++step) {
            if (step < nst) {
                const int tt = kh + 2 * (step >> 1), h0 = (step & 1) * (K / 32);
                const float* wt = pick(A.lin_w.p, tt) + (16 * ct + c) * K + 4 * q + 16 * h0;
#pragma unroll
                for (int b = 0; b < K / 32; ++b)
                    bq_all[step][b] = *reinterpret_cast<const float4*>(wt + 16 * b);
            }
        }
    }
    // the relation table in registers of every lane (n_rel <= 64), read by shuffles
    const float tabw = rel_tab(A.rw, A.n_rel, A.alpha, lane);
    // ---- gather: per-type register sums of this lane's 4 features of row v
    const int v = base + sub;
    const bool rv = sub < kAggRows && v < n;   // a row of this tile and of the batch
    float wsum[NT];
    float4 racc[NT];
    int rel_t[NT];
    float4 xself = make_float4(0.f, 0.f, 0.f, 0.f);
    int r_self = -1;
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
        wsum[tt] = 0.f;
        rel_t[tt] = -1;
        racc[tt] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    int e0 = 0, e1 = 0;
    if constexpr (PRE) {
        if (rv) {
#pragma unroll
            for (int tt = 0; tt < NT; ++tt) {
                if (tt < T) {
                    racc[tt] = *reinterpret_cast<const float4*>(A.s_agg + (int64_t(v) * T + tt) * K + 4 * l);
                    wsum[tt] = A.s_w[int64_t(v) * T + tt];
                    rel_t[tt] = A.u_rel[int64_t(v) * (T + 1) + tt];
                }
            }
            xself = *reinterpret_cast<const float4*>(A.u_self + int64_t(v) * K + 4 * l);
            r_self = A.u_rel[int64_t(v) * (T + 1) + T];
        }
    } else if (rv) {
        row_range(A.ptr, A.cnt, A.stride, v, e0, e1);
    }
    for (int c0 = e0; c0 < e1; c0 += 32) {
        const int m = min(32, e1 - c0);
        int my_t = 0, my_lo = 0, my_r = 0;  // table rows < 2^31 (checked by the host)
        if (l < m) {
            my_t = A.edge_type[c0 + l];
            my_lo = int(A.edge_off[c0 + l]);
            my_r = A.rel[c0 + l];
        }
        constexpr int UN = 12;             // edges' rows in flight per lane
        // (the weighted path's relation weight straight from relation_weight, branch-free: a
        // shuffle from the table lanes could read lanes of a row already done)
        float my_w = 0.f;
        if constexpr (!RS) {
            const float tr = A.rw[min(my_r, A.n_rel - 1)] * A.alpha;
            my_w = my_r < A.n_rel ? (tr > 0.f ? tr : 0.01f * tr) : 0.f;
        }
        for (int j = 0; j < m; j += UN) {
            int t[UN], ru[UN];
            float4 x[UN];
#pragma unroll
            for (int u = 0; u < UN; ++u) {
                const int jj = min(j + u, m - 1);
                t[u] = __shfl(my_t, gl + jj, 64);
                if constexpr (RS) ru[u] = __shfl(my_r, gl + jj, 64);
                else ru[u] = __float_as_int(__shfl(my_w, gl + jj, 64));
                const int64_t lo = __shfl(my_lo, gl + jj, 64);
                x[u] = *reinterpret_cast<const float4*>(pick(A.xt.p, t[u]) + lo * K + 4 * l);
                if (j + u >= m) t[u] = -1;     // padding: loaded (a valid row), not added
            }
#pragma unroll
            for (int u = 0; u < UN; ++u) {
                if (t[u] < 0) continue;
                if constexpr (RS) {
                    if (ru[u] >= A.n_et) {         // the self loop (one per row)
                        r_self = ru[u];
                        xself = x[u];
                        continue;
                    }
                }
#pragma unroll
                for (int tt = 0; tt < NT; ++tt) {
                    if (tt != t[u]) continue;
                    if constexpr (RS) {
                        wsum[tt] += 1.f;
                        rel_t[tt] = ru[u];
                        racc[tt].x += x[u].x; racc[tt].y += x[u].y;
                        racc[tt].z += x[u].z; racc[tt].w += x[u].w;
                    } else {
                        const float wt = __int_as_float(ru[u]);
                        wsum[tt] += wt;
                        racc[tt].x = fmaf(wt, x[u].x, racc[tt].x);
                        racc[tt].y = fmaf(wt, x[u].y, racc[tt].y);
                        racc[tt].z = fmaf(wt, x[u].z, racc[tt].z);
                        racc[tt].w = fmaf(wt, x[u].w, racc[tt].w);
                    }
                }
            }
        }
    }
    PH(0, 1);
    const int tau = r_self - A.n_et;           // RS: the row's node type
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
        if (tt < T) {
            float wr = 1.f, ws = 0.f;              // RS: S = wr U + ws x_self
            if constexpr (RS) {
                const float tr = __shfl(tabw, max(rel_t[tt], 0), 64);
                const float tsf = __shfl(tabw, max(r_self, 0), 64);
                wr = rel_t[tt] >= 0 ? tr : 0.f;
                ws = (tt == tau) ? tsf : 0.f;
            }
            float4 sv = racc[tt];
            if constexpr (RS)
                sv = make_float4(fmaf(ws, xself.x, wr * sv.x), fmaf(ws, xself.y, wr * sv.y),
                                 fmaf(ws, xself.z, wr * sv.z), fmaf(ws, xself.w, wr * sv.w));
            *reinterpret_cast<float4*>(St + sub * SR + tt * K + 4 * l) = sv;
            if (rv && !PRE)
                *reinterpret_cast<float4*>(A.s_agg + (int64_t(v) * T + tt) * K + 4 * l) = racc[tt];
            if (l == 0) {
                sw[sub * MT + tt] = RS ? fmaf(wr, wsum[tt], ws) : wsum[tt];
                if (rv && !PRE) {
                    A.s_w[int64_t(v) * T + tt] = wsum[tt];
                    if constexpr (RS) A.u_rel[int64_t(v) * (T + 1) + tt] = rel_t[tt];
                }
            }
        }
    }
    if constexpr (RS && !PRE) {
        if (rv) {
            *reinterpret_cast<float4*>(A.u_self + int64_t(v) * K + 4 * l) = xself;
            if (l == 0) A.u_rel[int64_t(v) * (T + 1) + T] = r_self;
        }
    }
    // stage 2's operands (waves 0..3), requested before stage 1 (their latency under it)
    float w0c[16], iv4[4];
    float bj = 0.f;
    if (w < 4) {
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int i = 0; i < 4; ++i) w0c[4 * b + i] = A.w0[(16 * b + 4 * q + i) * F + 16 * w + c];
#pragma unroll
        for (int r = 0; r < 4; ++r)
            iv4[r] = 4 * q + r < kAggRows && base + 4 * q + r < n ? A.inv[base + 4 * q + r] : 0.f;
        bj = A.bias[16 * w + c];
    }
    __syncthreads();
    PH(0, 2);
    // ---- stage 1: wave (ct, kh) forms sum over its half's types of S_t W_t^T for columns
    // 16 ct + c; W_t fragments from L2, two in flight
    f32x4 d = {0.f, 0.f, 0.f, 0.f};
    if constexpr (EW) {
#pragma unroll
        for (int step = 0; step < NT; ++step) {
            if (step < nst) {
                const int tt = kh + 2 * (step >> 1);
                const float* sa = St + c * SR + tt * K + 16 * (step & 1) * HB + 4 * q;
#pragma unroll
                for (int b = 0; b < HB; ++b) {
                    const float4 av = *reinterpret_cast<const float4*>(sa + 16 * b);
                    const float4 bv = bq_all[step][b];
                    MFMA4(av, bv.x, bv.y, bv.z, bv.w, d);
                }
            }
        }
    } else {
        float4 bq[3][HB];
        auto bload = [&](int step, float4 (&dst)[HB]) {     // step: (type tt = kh + 2 (step >> 1), half)
            const int tt = kh + 2 * (step >> 1), h0 = (step & 1) * HB;
            const float* wt = pick(A.lin_w.p, tt) + (16 * ct + c) * K + 4 * q + 16 * h0;
#pragma unroll
            for (int b = 0; b < HB; ++b) dst[b] = *reinterpret_cast<const float4*>(wt + 16 * b);
        };
        if (nst > 0) bload(0, bq[0]);
        if (nst > 1) bload(1, bq[1]);
#pragma unroll
        for (int step = 0; step < NT; ++step) {             // NT >= 2 * ceil(NT / 2) steps bound
            if (step < nst) {
                if (step + 2 < nst) bload(step + 2, bq[(step + 2) % 3]);
                const int tt = kh + 2 * (step >> 1);
                const float* sa = St + c * SR + tt * K + 16 * (step & 1) * HB + 4 * q;
#pragma unroll
                for (int b = 0; b < HB; ++b) {
                    const float4 av = *reinterpret_cast<const float4*>(sa + 16 * b);
                    const float4 bv = bq[step % 3][b];
                    MFMA4(av, bv.x, bv.y, bv.z, bv.w, d);
                }
            }
        }
    }
    if (kh == 1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) red[(4 * q + r) * F + 16 * ct + c] = d[r];
    }
    __syncthreads();
    if (kh == 0) {                         // P = half 0 + half 1 + sum_t w_vt b_t
        const int j = 16 * ct + c;
        float lbj[NT];
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) lbj[tt] = tt < T ? pick(A.lin_b.p, tt)[j] : 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int vr = 4 * q + r;
            float bsum = 0.f;
#pragma unroll
            for (int tt = 0; tt < NT; ++tt)
                if (tt < T) bsum = fmaf(sw[vr * MT + tt], lbj[tt], bsum);
            Pt[vr * 68 + j] = (d[r] + red[vr * F + j]) + bsum;
        }
    }
    __syncthreads();
    PH(0, 3);
    // ---- stage 2: a = inv (P W_0) + bias
    if (w < 4) {
        f32x4 d2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const float4 av = *reinterpret_cast<const float4*>(Pt + c * 68 + 16 * b + 4 * q);
            MFMA4(av, w0c[4 * b], w0c[4 * b + 1], w0c[4 * b + 2], w0c[4 * b + 3], d2);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) at[(4 * q + r) * F + 16 * w + c] = fmaf(iv4[r], d2[r], bj);
    }
    __syncthreads();
    // ---- epilogue (threads 0..255: 16 rows x 16 lanes): P and a kept, LayerNorm, relu,
    // dropout -> h0
    if (threadIdx.x < kBlock) {
        const int l16 = threadIdx.x & 15, s16 = threadIdx.x >> 4;
        const int vv = base + s16;
        if (s16 < kAggRows && vv < n) {
            const float4 gw = reinterpret_cast<const float4*>(A.ln_w)[l16];
            const float4 gb = reinterpret_cast<const float4*>(A.ln_b)[l16];
            *reinterpret_cast<float4*>(A.p + int64_t(vv) * F + 4 * l16) =
                *reinterpret_cast<const float4*>(Pt + s16 * 68 + 4 * l16);
            const float4 a4 = *reinterpret_cast<const float4*>(at + s16 * F + 4 * l16);
            const float av[4] = {a4.x, a4.y, a4.z, a4.w};
            *reinterpret_cast<float4*>(A.a + int64_t(vv) * F + 4 * l16) = a4;
            const float mean = group_sum<16>(av[0] + av[1] + av[2] + av[3]) * (1.f / F);
            const float dd[4] = {av[0] - mean, av[1] - mean, av[2] - mean, av[3] - mean};
            const float var = group_sum<16>(dd[0] * dd[0] + dd[1] * dd[1] + dd[2] * dd[2] + dd[3] * dd[3]) * (1.f / F);
            const float rstd = rsqrtf(var + kLnEps);
            if (l16 == 0) reinterpret_cast<float2*>(A.stats)[vv] = make_float2(mean, rstd);
            const float gws[4] = {gw.x, gw.y, gw.z, gw.w}, gbs[4] = {gb.x, gb.y, gb.z, gb.w};
            const uint32_t key = A.drop.on ? layer_key(A.state, 0) : 0u;
            float mk[4];
            drop_factors(key, A.drop, vv, l16, mk);
            float hv[4];
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) hv[cc] = fmaxf(fmaf(dd[cc] * rstd, gws[cc], gbs[cc]), 0.f) * mk[cc];
            *reinterpret_cast<float4*>(A.h + int64_t(vv) * F + 4 * l16) = make_float4(hv[0], hv[1], hv[2], hv[3]);
        }
    }
    PH(0, 4);
    PE(0, 1);
}

// ---------------------------------------------------------------------------------------------
// head: 16 target rows per block.
//   1. Hagg[v] = sum_e tab[r_e] h0[u_e] (16 lanes per row) -> LDS;
//   2. a = inv (Hagg W_1) + bias (MFMA, W_1 fragments from L2 in registers);
//   3. LayerNorm, relu, dropout -> h (16 lanes per row);
//   4. z = h W_out^T + b_out (class tiles over the waves), log_softmax, nll, g = (softmax -
//      onehot) / n_valid, gh = g W_out, LayerNorm / relu / dropout backward -> ga, G = inv ga;
//   5. g and h rows -> HBM (finalize forms out_lin's weight gradient g^T h from them over every
//      row, MFMA tiles on otherwise idle CUs); partials: out_lin bias, conv bias / LN terms, loss;
//   6. GH = G W_1^T -> HBM (the scatter's rows) and the W_1 partial Hagg^T G (MFMA).
// out_lin.weight staged by LDS-DMA into an XOR-swizzled image (head_sw), as re_nsm.hip's head.
// Slab row per block: [C g out_b | 64 conv bias | 64 LN beta | 64 LN gamma | 1 loss | 64*64 g W_1]
struct HeadArgs {
    const int32_t* sizes; const int32_t* n_id; const int64_t* labels;
    const int32_t* ptr; const int32_t* cnt; int stride;
    const int32_t* idx; const uint8_t* rel; const float* inv;
    const float* rw; int n_rel; float alpha;
    const float* h; const float* w1; const float* bias; const float* ln_w; const float* ln_b;
    const int64_t* state; Drop drop;
    const float* w_out; const float* b_out; int C;
    float* gh; float* nvalid; float* part; int64_t part_w;
    float* g_rows; float* h_rows;          // [blocks * 16][C] softmax gradient, [blocks * 16][64] h
};

// o_w1 (the W_1 partial) starts on a 16-byte boundary: finalize sums it with float4 loads
__host__ __device__ inline int64_t head_o_w1(int C) {
    return (int64_t(C) + 3 * F + 1 + 3) & ~3ll;
}
inline int64_t head_part_width(int C) { return head_o_w1(C) + F * F; }
__host__ __device__ inline int head_cp(int C) { return ((C + 63) / 64) * 64 + 4; }
__host__ __device__ inline int head_wl(int C) {
    const int wl = ((C + 15) / 16) * 16 * F, red = 3 * 16 * F + 16 * 68;
    return wl > red ? wl : red;
}
inline size_t head_lds(int C) {
    return (size_t(head_wl(C)) + 16 * head_cp(C) + 16 * 68 + 16 * 80 + 16 * 68 + 16 * 68 +
            3 * 16 * 68) * sizeof(float);
}

__device__ __forceinline__ int head_sw(int c, int k) { return c * F + (k ^ ((c & 15) << 2)); }

// 16 waves: the row phases (16 rows x 16 lanes) run on threads 0..255, the class-tile loops
// (logits, gh) and the softmax (64 lanes per row) on all 16 waves; out_lin.weight's LDS-DMA
// staging on waves 4..15 under the aggregation
constexpr int kHeadThreads = 1024;
constexpr int kHeadW = kHeadThreads / 64;  // waves
constexpr int kHeadSL = kHeadThreads / 16; // softmax lanes per row
constexpr int kHeadNQ = kHeadW / 4;        // gh: class parts (4 feature tiles x kHeadNQ)
static_assert(kHeadNQ == 4 && kHeadSL == 64, "step 4c / 4d sum four class parts; 4b a wave per row");

__global__ void __launch_bounds__(kHeadThreads, 1) head_kernel(HeadArgs A) {
    extern __shared__ float hl[];
    const int C = A.C, CT = (C + 15) / 16, CP = head_cp(C);
    float* Wl = hl;                        // W_out image; after step 4: red [3][16][64]
    float* zs = Wl + head_wl(C);           // [16][CP]: z, then g
    float* hs = zs + 16 * CP;              // [16][68]: h (row reads), then G
    float* hs2 = hs + 16 * 68;             // [16][80]: h (column reads)
    float* ghs = hs2 + 16 * 80;            // [16][68]: a, then gh
    float* hg = ghs + 16 * 68;             // [16][68]: Hagg
    float* ghp = hg + 16 * 68;             // [16][68] x 3: gh over class parts 1 .. 3
    float* red = Wl;
    __shared__ float lrow[kRows];
    __shared__ float bo_s[16 * kMaxCT];    // out_lin.bias (classes >= C: 0)
    const bool rowt = threadIdx.x < kBlock;    // the row phases' threads
    const int l = threadIdx.x & 15, sub = (threadIdx.x >> 4) & 15, gl = threadIdx.x & 48;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, cc = lane & 15, q = lane >> 4;
    const int wq = w & 3, wh = w >> 2;        // feature tile, class part (step 4c)
    PH(1, 12);
    PE(1, 0);
    const int n = A.sizes[0];
    const int v = blockIdx.x * kRows + sub;
    const bool act = rowt && v < n;
    // Order of the global requests: the aggregation's chain first (nothing waits behind the
    // staging), then step 2 / 3's operands, then out_lin's LDS-DMA; the barriers up to step 4a
    // order LDS only (lds_sync), so the DMA lands under steps 1-3.
    const int r32 = threadIdx.x / kHeadSL, l32 = threadIdx.x % kHeadSL;   // step 4b: a row's lanes
    const int v32 = blockIdx.x * kRows + r32;
    const int nid32 = v32 < n ? A.n_id[v32] : -1;
    PH(1, 0);
    PH(1, 1);
    // ---- 1. Hagg on waves 0..3 (16 lanes per row, up to 32 entries' rows in flight: one round
    // of loads for the sampled rows <= 32), while waves 4..7 stage out_lin.weight into its LDS
    // image (their loads overlap the aggregation's)
    if (rowt) {
        const int vr = blockIdx.x * kRows + sub;
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
        if (vr < n) {
            int e0, e1;
            row_range(A.ptr, A.cnt, A.stride, vr, e0, e1);
            for (int c0 = e0; c0 < e1; c0 += 32) {
                const int m = min(32, e1 - c0);
                const int my_u0 = l < m ? A.idx[c0 + l] : 0;
                const int my_r0 = l < m ? int(A.rel[c0 + l]) : 0;
                const int my_u1 = l + 16 < m ? A.idx[c0 + 16 + l] : 0;
                const int my_r1 = l + 16 < m ? int(A.rel[c0 + 16 + l]) : 0;
                constexpr int UN = 32;
                float4 x[UN];
#pragma unroll
                for (int u = 0; u < UN; ++u) {
                    const int jj = min(u, m - 1);
                    const int uu = __shfl(jj < 16 ? my_u0 : my_u1, gl + (jj & 15), 64);
                    x[u] = *reinterpret_cast<const float4*>(A.h + int64_t(uu) * F + 4 * l);
                }
                // each lane's own entries' relation weights (unconditional loads after the
                // rows are requested), broadcast by shuffles
                const float tr0 = A.rw[min(my_r0, A.n_rel - 1)] * A.alpha;
                const float tr1 = A.rw[min(my_r1, A.n_rel - 1)] * A.alpha;
                const float w0 = my_r0 < A.n_rel ? (tr0 > 0.f ? tr0 : 0.01f * tr0) : 0.f;
                const float w1 = my_r1 < A.n_rel ? (tr1 > 0.f ? tr1 : 0.01f * tr1) : 0.f;
#pragma unroll
                for (int u = 0; u < UN; ++u) {     // branch-free: a padding entry (a clamped
                    // valid row) gets weight 0, which adds exact zeros
                    const float ws = __shfl(u < 16 ? w0 : w1, gl + (u & 15), 64);
                    const float wt = u < m ? ws : 0.f;
                    s0 = fmaf(wt, x[u].x, s0); s1 = fmaf(wt, x[u].y, s1);
                    s2 = fmaf(wt, x[u].z, s2); s3 = fmaf(wt, x[u].w, s3);
                }
            }
        }
        *reinterpret_cast<float4*>(hg + sub * 68 + 4 * l) = make_float4(s0, s1, s2, s3);
    } else {
        // out_lin.weight -> LDS: image row i (4 classes) slot L%16 of class c = 4 i + L / 16 holds
        // W[c][4 ((L%16) ^ (c & 15)) ..] (head_sw); pad rows c >= C read row C-1
        // by LDS-DMA: vmcnt is per wave, so only these four waves wait for it (at the barrier)
        const int L64 = threadIdx.x & 63;
        for (int i = w - 4; i < CT * 4; i += kHeadW - 4) {
            const int c = 4 * i + (L64 >> 4);
            const int cs = c < C ? c : C - 1;
            const float* src = A.w_out + int64_t(cs) * F + 4 * ((L64 & 15) ^ (c & 15));
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)src,
                (__attribute__((address_space(3))) void*)(Wl + 4 * i * F), 16, 0, 0);
        }
    }
    // steps 2 - 4's operands: the labels and the labelled-target count (agg0 counted it), W_1
    // fragments, biases, row scales, LayerNorm weights, out_lin.bias
    const int64_t y = nid32 >= 0 ? A.labels[nid32] : -1;
    const float nvalid = *A.nvalid;
    const float bj2 = A.bias[16 * wq + cc];
    float iv2[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int vv = blockIdx.x * kRows + 4 * q + r;
        iv2[r] = vv < n ? A.inv[vv] : 0.f;
    }
    float w1c[16];                         // W_1[16 b + 4 q + i][16 w + cc]: step 2's B operand
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i) w1c[4 * b + i] = A.w1[(16 * b + 4 * q + i) * F + 16 * wq + cc];
    const float4 gw4 = reinterpret_cast<const float4*>(A.ln_w)[l];
    const float4 gb4 = reinterpret_cast<const float4*>(A.ln_b)[l];
    const float ivv = act ? A.inv[v] : 0.f;
    for (int c = threadIdx.x; c < 16 * kMaxCT; c += kHeadThreads) bo_s[c] = c < A.C ? A.b_out[c] : 0.f;
    __syncthreads();
    PH(1, 2);
    // ---- 2. a = inv (Hagg W_1) + bias -> ghs
    if (w < 4) {
        f32x4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const float4 av = *reinterpret_cast<const float4*>(hg + cc * 68 + 16 * b + 4 * q);
            MFMA4(av, w1c[4 * b], w1c[4 * b + 1], w1c[4 * b + 2], w1c[4 * b + 3], d);
        }
        const int j = 16 * w + cc;
#pragma unroll
        for (int r = 0; r < 4; ++r) ghs[(4 * q + r) * 68 + j] = fmaf(iv2[r], d[r], bj2);
    }
    lds_sync();
    // ---- 3. LayerNorm, relu, dropout
    const float gwf[4] = {gw4.x, gw4.y, gw4.z, gw4.w}, gbf[4] = {gb4.x, gb4.y, gb4.z, gb4.w};
    float xhat[4] = {0.f, 0.f, 0.f, 0.f}, mfac[4] = {0.f, 0.f, 0.f, 0.f}, rstd = 0.f;
    float hv[4] = {0.f, 0.f, 0.f, 0.f};
    if (act) {
        const float4 a4 = *reinterpret_cast<const float4*>(ghs + sub * 68 + 4 * l);
        const float a[4] = {a4.x, a4.y, a4.z, a4.w};
        const float mean = group_sum<16>(a[0] + a[1] + a[2] + a[3]) * (1.f / F);
        const float d[4] = {a[0] - mean, a[1] - mean, a[2] - mean, a[3] - mean};
        rstd = rsqrtf(group_sum<16>(d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3]) *
                          (1.f / F) + kLnEps);
        const uint32_t key = A.drop.on ? layer_key(A.state, 1) : 0u;
        drop_factors(key, A.drop, v, l, mfac);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            xhat[i] = d[i] * rstd;
            hv[i] = fmaxf(fmaf(xhat[i], gwf[i], gbf[i]), 0.f) * mfac[i];
        }
    }
    if (rowt) {
        *reinterpret_cast<float4*>(hs + sub * 68 + 4 * l) = make_float4(hv[0], hv[1], hv[2], hv[3]);
        *reinterpret_cast<float4*>(hs2 + sub * 80 + 4 * l) = make_float4(hv[0], hv[1], hv[2], hv[3]);
    }
    __syncthreads();
    PH(1, 3);
    // ---- 4a. z = h W^T + b -> zs (classes >= C: -inf)
    for (int ct = w; ct < CT; ct += kHeadThreads / 64) {
        const int c = 16 * ct + cc;
        f32x4 dz = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int b = 0; b < F / 16; ++b) {
            const float4 av = *reinterpret_cast<const float4*>(hs + cc * 68 + 16 * b + 4 * q);
            const float4 bv = *reinterpret_cast<const float4*>(Wl + head_sw(c, 16 * b + 4 * q));
            MFMA4(av, bv.x, bv.y, bv.z, bv.w, dz);
        }
        const float bo = bo_s[c];
#pragma unroll
        for (int r = 0; r < 4; ++r) zs[(4 * q + r) * CP + c] = c < C ? dz[r] + bo : -INFINITY;
    }
    __syncthreads();
    PH(1, 8);
    // ---- 4b. log_softmax, nll, g: lane l32 of row r32 holds classes l32 + SL i (all waves)
    {
        constexpr int NI = (16 * kMaxCT + kHeadSL - 1) / kHeadSL;
        const int CW = 16 * CT;                // classes >= C hold -inf
        float zr[NI];
        float zmax = -INFINITY;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int c = l32 + kHeadSL * i;
            zr[i] = c < CW ? zs[r32 * CP + c] : -INFINITY;
            zmax = fmaxf(zmax, zr[i]);
        }
#pragma unroll
        for (int o = kHeadSL / 2; o > 0; o >>= 1) zmax = fmaxf(zmax, __shfl_xor(zmax, o, 64));
        float se = 0.f;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            zr[i] = expf(zr[i] - zmax);        // classes >= C: exp(-inf) = 0
            se += zr[i];
        }
        se = group_sum<kHeadSL>(se);
        const float lse = zmax + logf(se), rse = 1.f / se;
        const bool ok = v32 < n;
        const float zy = y >= 0 ? zs[r32 * CP + y] : 0.f;
        if (l32 == 0) lrow[r32] = y >= 0 ? lse - zy : 0.f;
        const float inv_n = y >= 0 && nvalid > 0.f ? 1.f / nvalid : 0.f;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int c = l32 + kHeadSL * i;
            if (c < CW)
                zs[r32 * CP + c] = ok && c < C ? (zr[i] * rse - (int64_t(c) == y ? 1.f : 0.f)) * inv_n : 0.f;
        }
    }
    __syncthreads();
    PH(1, 9);
    // ---- 4c. gh = g W: wave w -> features 16 wq + cc, rows 4 q + r, class tiles of part wh
    {
        const int k = 16 * wq + cc;
        const int ctp = (CT + kHeadNQ - 1) / kHeadNQ, b0 = min(CT, wh * ctp), b1 = min(CT, b0 + ctp);
        auto step = [&](int b, f32x4 d) {
            const float4 av = *reinterpret_cast<const float4*>(zs + cc * CP + 16 * b + 4 * q);
            const int c0 = 16 * b + 4 * q;
            const float w0 = Wl[head_sw(c0 + 0, k)], w1 = Wl[head_sw(c0 + 1, k)];
            const float w2 = Wl[head_sw(c0 + 2, k)], w3 = Wl[head_sw(c0 + 3, k)];
            MFMA4(av, w0, w1, w2, w3, d);
            return d;
        };
        f32x4 dg0 = {0.f, 0.f, 0.f, 0.f}, dg1 = {0.f, 0.f, 0.f, 0.f};
        int b = b0;
        for (; b + 1 < b1; b += 2) {
            dg0 = step(b, dg0);
            dg1 = step(b + 1, dg1);
        }
        if (b < b1) dg0 = step(b, dg0);
        float* gd = wh ? ghp + (wh - 1) * 16 * 68 : ghs;
#pragma unroll
        for (int r = 0; r < 4; ++r) gd[(4 * q + r) * 68 + k] = dg0[r] + dg1[r];
    }
    __syncthreads();
    PH(1, 4);
    // ---- 4d. LayerNorm / relu / dropout backward -> ga; G = inv ga -> hs; row terms -> red
    float4 w1r[4];                         // W_1[16 w + cc][16 b + 4 q ..]: step 6's B operand
#pragma unroll
    for (int b = 0; b < 4; ++b)
        w1r[b] = *reinterpret_cast<const float4*>(A.w1 + (16 * wq + cc) * F + 16 * b + 4 * q);
    if (rowt) {
        // the class parts' gh in a fixed order: (0 + 1) + (2 + 3)
        const float4 ga4 = *reinterpret_cast<const float4*>(ghs + sub * 68 + 4 * l);
        const float4 gb4 = *reinterpret_cast<const float4*>(ghp + sub * 68 + 4 * l);
        const float4 gc4 = *reinterpret_cast<const float4*>(ghp + 16 * 68 + sub * 68 + 4 * l);
        const float4 gd4 = *reinterpret_cast<const float4*>(ghp + 2 * 16 * 68 + sub * 68 + 4 * l);
        const float g[4] = {(ga4.x + gb4.x) + (gc4.x + gd4.x), (ga4.y + gb4.y) + (gc4.y + gd4.y),
                            (ga4.z + gb4.z) + (gc4.z + gd4.z), (ga4.w + gb4.w) + (gc4.w + gd4.w)};
        float gy[4], gx[4];
        float p1 = 0.f, p2 = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float yv = fmaf(xhat[i], gwf[i], gbf[i]);
            gy[i] = act && yv > 0.f ? g[i] * mfac[i] : 0.f;
            gx[i] = gy[i] * gwf[i];
            p1 += gx[i];
            p2 += gx[i] * xhat[i];
        }
        const float m1 = group_sum<16>(p1) * (1.f / F), m2 = group_sum<16>(p2) * (1.f / F);
        float ga[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) ga[i] = act ? rstd * (gx[i] - m1 - xhat[i] * m2) : 0.f;
        *reinterpret_cast<float4*>(hs + sub * 68 + 4 * l) =
            make_float4(ivv * ga[0], ivv * ga[1], ivv * ga[2], ivv * ga[3]);
        *reinterpret_cast<float4*>(red + (0 * 16 + sub) * F + 4 * l) = make_float4(ga[0], ga[1], ga[2], ga[3]);
        *reinterpret_cast<float4*>(red + (1 * 16 + sub) * F + 4 * l) = make_float4(gy[0], gy[1], gy[2], gy[3]);
        *reinterpret_cast<float4*>(red + (2 * 16 + sub) * F + 4 * l) =
            make_float4(gy[0] * xhat[0], gy[1] * xhat[1], gy[2] * xhat[2], gy[3] * xhat[3]);
    }
    __syncthreads();
    PH(1, 10);
    float* o = A.part + int64_t(blockIdx.x) * A.part_w;
    const int64_t o_ob = 0, o_cb = C, o_loss = o_cb + 3 * F;
    const int64_t o_w1 = head_o_w1(C);
    // ---- 5. g rows (classes < C) and h rows -> HBM for finalize's out_lin weight tiles
    {                                      // (the out_lin bias partial from the same reads)
        float* gr = A.g_rows + int64_t(blockIdx.x) * kRows * C;
        for (int c = threadIdx.x; c < C; c += kHeadThreads) {
            float acc = 0.f;
#pragma unroll
            for (int r = 0; r < kRows; ++r) {
                const float gv = zs[r * CP + c];
                gr[r * C + c] = gv;
                acc += gv;
            }
            o[o_ob + c] = acc;
        }
        float* hr = A.h_rows + int64_t(blockIdx.x) * kRows * F;
        for (int i = threadIdx.x; i < kRows * F; i += kHeadThreads)
            hr[i] = hs2[(i >> 6) * 80 + (i & 63)];
    }
    if (threadIdx.x < 3 * F) {                                 // conv bias, LN beta, LN gamma
        const int which = threadIdx.x >> 6, f = threadIdx.x & 63;
        float acc = 0.f;
#pragma unroll
        for (int r = 0; r < kRows; ++r) acc += red[(which * 16 + r) * F + f];
        o[o_cb + threadIdx.x] = acc;
    }
    if (threadIdx.x == 0) {
        float acc = 0.f;
#pragma unroll
        for (int r = 0; r < kRows; ++r) acc += lrow[r];
        o[o_loss] = acc;
    }
    PH(1, 5);
    // ---- 6. GH = G W_1^T -> HBM; W_1 partial D[k][j] = sum_v Hagg[v][k] G[v][j]
    if (w < 4) {
        f32x4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const float4 av = *reinterpret_cast<const float4*>(hs + cc * 68 + 16 * b + 4 * q);
            MFMA4(av, w1r[b].x, w1r[b].y, w1r[b].z, w1r[b].w, d);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int vv = blockIdx.x * kRows + 4 * q + r;
            if (vv < n) A.gh[int64_t(vv) * F + 16 * w + cc] = d[r];
        }
        f32x4 dw[4];
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) dw[jb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            const int r = 4 * st + q;
            const float av = hg[r * 68 + 16 * w + cc];
#pragma unroll
            for (int jb = 0; jb < 4; ++jb)
                dw[jb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, hs[r * 68 + 16 * jb + cc], dw[jb], 0, 0, 0);
        }
#pragma unroll
        for (int jb = 0; jb < 4; ++jb)
#pragma unroll
            for (int i = 0; i < 4; ++i) o[o_w1 + (16 * w + 4 * q + i) * F + 16 * jb + cc] = dw[jb][i];
    }
    PH(1, 7);
    PE(1, 1);
}

// ---------------------------------------------------------------------------------------------
// gather: layer 0's rows u (hop 0's sources), 4 features per lane of a 16-lane group:
//   gh0[u] = sum over u's edges e of hop 0's block (the sampler's transposed index) of
//            tab[r_e] GH[v_e], and the relation dots <h0[u], GH[v_e]>: exact 2^-40 fixed-point
//            integer sums (registers / LDS), so neither the segment order nor the split of a
//            segment over groups changes a bit;
//   h0 re-formed from a0, the LN stats and the dropout mask; the LayerNorm / relu / dropout
//   backward -> G0[u] = inv0[u] ga0[u] (HBM, bwd0's rows) and the rows' sums of ga0, gy and
//   gy xhat (conv bias, LN beta / gamma).
// Rows with <= kShort edges: one group each (grid-stride), the entries loaded lane-parallel and
// their GH rows 8 in flight. Longer rows (the hubs: the sampler's ascending csc_long list): a
// whole workgroup each, the segment's 16-entry chunks over its groups, the partial sums added in
// LDS. Row terms per group in a fixed row order, summed over the groups in order.
// Slab row per block: [64 relation dots | 64 sum ga0 | 64 sum gy | 64 sum gy xhat]
struct GathArgs {
    const int32_t* sizes; int hop;
    const int32_t* cptr; const int32_t* cent; const int32_t* clong; const float* gh;
    const float* a; const float* stats; const float* inv;
    const float* ln_w; const float* ln_b; const int64_t* state; Drop drop;
    const float* rw; int n_rel; float alpha;
    float* g0; float* slab;
    // hub rows (> kShort entries): their 16-entry chunks spread over every group of the grid;
    // exact sums in hub_acc [kLongCap][64], the last chunk's group (hub_ticket) runs the row's
    // backward and adds its row terms to hub_terms [3][64] (all exact 2^-40 integers; hub_acc /
    // hub_ticket zeroed by that group, hub_terms by finalize); hub_terms[192]: the overflow flag
    unsigned long long* hub_acc; int32_t* hub_ticket; unsigned long long* hub_terms;
};

// 512 threads (32 row groups) per block: a hub piece's entries over 32 groups (a 439-entry row:
// 14 per group instead of 28); 256 blocks keep the 8192 groups of the short rows
constexpr int kGathT = 512, kGathG = kGathT / 16;
// 192 blocks: 104.3-104.9 us per step against 105.7-106.2 at 256, 106.0-106.7 at 160, 106.6-107.0
// at 128 (round 5, lookahead 32: fewer gather blocks beside the sampler's launches)
static const int kGathBlocks = env_blocks("REGNN_NSM_GATH_BLOCKS", 192);

constexpr int kGathW = 4 * F;
constexpr int kShort = 16;                 // = re_ns.hip kCscShort

struct RowIn {                             // one lane's 4 features of layer 0's row u
    float xh[4], yv[4], mk[4], h0[4], rstd, iv;
};

__device__ __forceinline__ RowIn row_in(const GathArgs& A, uint32_t key, int u, int l,
                                         const float (&lw)[4], const float (&lb)[4]) {
    RowIn R;
    const float4 a4 = *reinterpret_cast<const float4*>(A.a + int64_t(u) * F + 4 * l);
    const float2 st = reinterpret_cast<const float2*>(A.stats)[u];
    R.iv = A.inv[u];
    R.rstd = st.y;
    const float av[4] = {a4.x, a4.y, a4.z, a4.w};
    drop_factors(key, A.drop, u, l, R.mk);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        R.xh[i] = (av[i] - st.x) * st.y;
        R.yv[i] = fmaf(R.xh[i], lw[i], lb[i]);
        R.h0[i] = fmaxf(R.yv[i], 0.f) * R.mk[i];
    }
    return R;
}

// `m` entries of a segment starting at c (m <= 16, uniform over the group): fixed-point sums of
// tab[r] GH[v] into acc and the relation dots into the block's bins
// `my`: lane l's entry word of the chunk (l < m), loaded by the caller
template <int UN>
__device__ __forceinline__ void gather_chunk_my(const GathArgs& A, const float* tab,
                                                unsigned long long (&rb)[4], int my, int m, int l,
                                                int gl, const RowIn& R,
                                                unsigned long long (&acc)[4], bool& bad) {
    for (int j = 0; j < m; j += UN) {
        int pk[UN];
        float4 g[UN];
#pragma unroll
        for (int u = 0; u < UN; ++u) {
            pk[u] = __shfl(my, gl + min(j + u, m - 1), 64);
            g[u] = *reinterpret_cast<const float4*>(A.gh + int64_t(pk[u] >> 8) * F + 4 * l);
        }
#pragma unroll
        for (int u = 0; u < UN; ++u) {
            if (j + u >= m) continue;          // uniform over the group (continue: the loop
                                               // unrolls, a break leaves g[] in scratch; a
                                               // branch-free form computed the short rows'
                                               // padding too: the gather 4.0 -> 6.2 us p50)
            const float t = tab[pk[u] & 255];
            acc[0] += to_fix_chk(t * g[u].x, bad);
            acc[1] += to_fix_chk(t * g[u].y, bad);
            acc[2] += to_fix_chk(t * g[u].z, bad);
            acc[3] += to_fix_chk(t * g[u].w, bad);
            // an explicit fma chain: the entry's slot u in the (atomically ordered) segment must
            // not change how its dot is contracted, or the exact sums see different terms
            const float d = group_sum<16>(fmaf(R.h0[3], g[u].w, fmaf(R.h0[2], g[u].z,
                                               fmaf(R.h0[1], g[u].y, R.h0[0] * g[u].x))));
            // the dot into its relation's bin: lane r % 16, slot r / 16 (registers, exact; LDS
            // atomics per entry would serialize the groups on the few relations' bins)
            const unsigned long long dq = to_fix_chk(d, bad);
            const int r = pk[u] & 255;
            const bool mine = (r & 15) == l;
#pragma unroll
            for (int k = 0; k < 4; ++k) rb[k] += mine && (r >> 4) == k ? dq : 0ull;
        }
    }
}

template <int UN>
__device__ __forceinline__ void gather_chunk(const GathArgs& A, const float* tab,
                                             unsigned long long (&rb)[4], int c, int m, int l,
                                             int gl, const RowIn& R,
                                             unsigned long long (&acc)[4], bool& bad) {
    const int my = l < m ? A.cent[c + l] : 0;
    gather_chunk_my<UN>(A, tab, rb, my, m, l, gl, R, acc, bad);
}

// the LayerNorm / relu / dropout backward of row u from its sums; G0 row to HBM, row terms
__device__ __forceinline__ void row_bwd(const GathArgs& A, int u, int l, const RowIn& R,
                                        const float (&lw)[4], const unsigned long long (&acc)[4],
                                        float (&sga)[4], float (&sgy)[4], float (&sgyx)[4]) {
    float gy[4], gx[4], p1 = 0.f, p2 = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        gy[i] = R.yv[i] > 0.f ? from_fix(acc[i]) * R.mk[i] : 0.f;
        gx[i] = gy[i] * lw[i];
        p1 += gx[i];
        p2 += gx[i] * R.xh[i];
    }
    const float m1 = group_sum<16>(p1) * (1.f / F), m2 = group_sum<16>(p2) * (1.f / F);
    float ga[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        ga[i] = R.rstd * (gx[i] - m1 - R.xh[i] * m2);
        sga[i] += ga[i];
        sgy[i] += gy[i];
        sgyx[i] += gy[i] * R.xh[i];
    }
    *reinterpret_cast<float4*>(A.g0 + int64_t(u) * F + 4 * l) =
        make_float4(R.iv * ga[0], R.iv * ga[1], R.iv * ga[2], R.iv * ga[3]);
}

// the row's backward for a hub row from its exact totals; its row terms go to hub_terms exactly
// (which workgroup runs it depends on the atomics' order: integer sums keep the result
// independent of it)
__device__ __forceinline__ void hub_row_bwd(const GathArgs& A, int u, int l, const RowIn& R,
                                            const float (&lw)[4],
                                            const unsigned long long (&tot)[4], bool& bad) {
    float sga[4] = {0.f, 0.f, 0.f, 0.f}, sgy[4] = {0.f, 0.f, 0.f, 0.f}, sgyx[4] = {0.f, 0.f, 0.f, 0.f};
    row_bwd(A, u, l, R, lw, tot, sga, sgy, sgyx);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        atomicAdd(A.hub_terms + 0 * F + 4 * l + i, to_fix_chk(sga[i], bad));
        atomicAdd(A.hub_terms + 1 * F + 4 * l + i, to_fix_chk(sgy[i], bad));
        atomicAdd(A.hub_terms + 2 * F + 4 * l + i, to_fix_chk(sgyx[i], bad));
    }
}

// Hub rows: the sampler's piece table (REGNN_CSC_LONG_TAB) cuts each into pieces of <= 1024
// entries; piece j runs on workgroup grid - 1 - j (the blocks past the short rows' range), its
// 16 groups taking even shares of the entries with up to 16 rows in flight, the partial sums added exactly
// in LDS. A row of one piece finishes there; a longer row's pieces store their sums to
// hub_acc[j] and the piece that completes the row's ticket sums them (exact) and runs the row's
// backward (device-scope fences: only for rows past 1024 entries).
__global__ void __launch_bounds__(kGathT) gather_kernel(GathArgs A) {
    __shared__ unsigned long long bins[F];
    __shared__ unsigned long long lgh[F];
    __shared__ float tab[F];
    __shared__ float rt[3][kGathG][F];
    __shared__ int s_last;
    PH(2, 8);
    PE(2, 0);
    const int nblk = int(gridDim.x);
    const int n_piece = A.clong[REGNN_CSC_LONG_NPIECE];
    if (threadIdx.x < F) {
        bins[threadIdx.x] = 0ull;
        lgh[threadIdx.x] = 0ull;
        tab[threadIdx.x] = rel_tab(A.rw, A.n_rel, A.alpha, threadIdx.x);
    }
    __syncthreads();
    const int n = A.sizes[A.hop];
    const int l = threadIdx.x & 15, grp = threadIdx.x >> 4, gl = threadIdx.x & 48;
    const uint32_t key = A.drop.on ? layer_key(A.state, 0) : 0u;
    const float4 lw4 = reinterpret_cast<const float4*>(A.ln_w)[l];
    const float4 lb4 = reinterpret_cast<const float4*>(A.ln_b)[l];
    const float lw[4] = {lw4.x, lw4.y, lw4.z, lw4.w}, lb[4] = {lb4.x, lb4.y, lb4.z, lb4.w};
    float sga[4] = {0.f, 0.f, 0.f, 0.f}, sgy[4] = {0.f, 0.f, 0.f, 0.f}, sgyx[4] = {0.f, 0.f, 0.f, 0.f};
    bool bad = false;                          // a fixed-point term out of range (to_fix_chk)
    unsigned long long rb[4] = {0ull, 0ull, 0ull, 0ull};   // relation bins l + 16 k (exact)
    // hub pieces j = grid - 1 - block, + grid, ... (block-uniform; usually one per block)
    for (int j = nblk - 1 - int(blockIdx.x); j < n_piece; j += nblk) {
        const int4 pc = reinterpret_cast<const int4*>(A.clong + REGNN_CSC_LONG_TAB)[j];
        const int u = pc.x, e0 = pc.y, cnt = pc.z;
        const int li = pc.w >> 16, k = (pc.w >> 8) & 255, npc = pc.w & 255;
        PG(j, 0);
        const RowIn R = row_in(A, key, u, l, lw, lb);
        unsigned long long acc[4] = {0ull, 0ull, 0ull, 0ull};
        // the piece's entries in even shares over the 32 groups (a 64-entry row: 2 per group,
        // not 16 on each of four); chunk width by the share (block-uniform)
        const int per = (cnt + kGathG - 1) / kGathG, g0 = min(cnt, per * grp), g1 = min(cnt, g0 + per);
        if (per <= 4) {
            if (g1 > g0) gather_chunk<4>(A, tab, rb, e0 + g0, g1 - g0, l, gl, R, acc, bad);
        } else if (per <= 8) {
            if (g1 > g0) gather_chunk<8>(A, tab, rb, e0 + g0, g1 - g0, l, gl, R, acc, bad);
        } else {                               // <= 64 entries: up to 4 chunks, whose entry
            int myk[4];                        // words are all requested first
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int ck = g0 + kShort * k, mk = min(kShort, g1 - ck);
                myk[k] = mk > 0 && l < mk ? A.cent[e0 + ck + l] : 0;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int ck = g0 + kShort * k, mk = min(kShort, g1 - ck);
                if (mk > 0) gather_chunk_my<kShort>(A, tab, rb, myk[k], mk, l, gl, R, acc, bad);
            }
        }
        PG(j, 1);
#pragma unroll
        for (int i = 0; i < 4; ++i) atomicAdd(lgh + 4 * l + i, acc[i]);   // LDS, exact
        __syncthreads();
        PG(j, 2);
        if (npc == 1) {                        // the whole row in this block (a fixed one):
            if (grp == 0) {                    // its row terms join the block's own sums
                const unsigned long long tot[4] = {lgh[4 * l], lgh[4 * l + 1], lgh[4 * l + 2],
                                                   lgh[4 * l + 3]};
                row_bwd(A, u, l, R, lw, tot, sga, sgy, sgyx);
            }
            PG(j, 3);
        } else {
            unsigned long long* ha = A.hub_acc + int64_t(j) * F;
            if (threadIdx.x < F)
                __hip_atomic_store(ha + threadIdx.x, lgh[threadIdx.x], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            __threadfence();
            __syncthreads();
            if (threadIdx.x == 0) s_last = atomicAdd(A.hub_ticket + li, 1) == npc - 1;
            __syncthreads();
            if (s_last) {                      // every piece of row u is in hub_acc
                __threadfence();
                if (grp == 0) {
                    const unsigned long long* h0 = A.hub_acc + int64_t(j - k) * F + 4 * l;
                    unsigned long long tot[4] = {0ull, 0ull, 0ull, 0ull};
                    for (int q = 0; q < npc; ++q)
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                            tot[i] += __hip_atomic_load(h0 + int64_t(q) * F + i, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
                    if (l == 0)
                        __hip_atomic_store(A.hub_ticket + li, 0, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    hub_row_bwd(A, u, l, R, lw, tot, bad);
                }
            }
        }
        __syncthreads();                       // lgh read; cleared for this block's next piece
        if (threadIdx.x < F) lgh[threadIdx.x] = 0ull;
        __syncthreads();
    }
    // ---- rows with <= kShort edges: one group each, on the blocks without a hub piece (piece j
    // runs on block grid - 1 - j): a hub block's short row would wait behind its piece (the
    // kernel's tail), so the short rows go to the other blocks while they can hold them all
    const int hub_blocks = min(n_piece, nblk);
    int sblocks = nblk - hub_blocks;
    if (sblocks * kGathG < n) sblocks = nblk;  // too few: every block takes short rows
    if (int(blockIdx.x) >= sblocks) sblocks = 0;        // (block-uniform) a hub block: none
    for (int u = blockIdx.x * kGathG + grp; sblocks && u < n; u += sblocks * kGathG) {
        const int c0 = A.cptr[u], m = A.cptr[u + 1] - c0;
        if (m > kShort) continue;              // a hub: its pieces above
        const RowIn R = row_in(A, key, u, l, lw, lb);
        unsigned long long acc[4] = {0ull, 0ull, 0ull, 0ull};
        gather_chunk<8>(A, tab, rb, c0, m, l, gl, R, acc, bad);
        row_bwd(A, u, l, R, lw, acc, sga, sgy, sgyx);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        rt[0][grp][4 * l + i] = sga[i];
        rt[1][grp][4 * l + i] = sgy[i];
        rt[2][grp][4 * l + i] = sgyx[i];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (rb[k]) atomicAdd(bins + l + 16 * k, rb[k]);      // LDS, exact: order-free
    __syncthreads();
    if (bad) A.hub_terms[3 * F] = 1ull;       // the overflow flag (finalize: NaN loss, reset)
    float* o = A.slab + int64_t(blockIdx.x) * kGathW;
    if (threadIdx.x < F) o[threadIdx.x] = float((long long)bins[threadIdx.x]) * kFixInv;
    if (threadIdx.x < 3 * F) {
        const int which = threadIdx.x >> 6, f = threadIdx.x & 63;
        float sum = 0.f;
#pragma unroll
        for (int g = 0; g < kGathG; ++g) sum += rt[which][g][f];
        o[F + threadIdx.x] = sum;
    }
    PH(2, 9);
    PE(2, 1);
}

// ---------------------------------------------------------------------------------------------
// bwd0: block (b, t) takes 16-row tiles b, b + gridDim.x, ... of layer 0's targets; the next
// tile's rows are prefetched into registers while this one is processed. Per tile:
//   gP     = G0 W_0^T (MFMA; G0 = the gather's rows, W_0 rows from L2 in registers); t = 0: the
//          W_0 partial P^T G0;
//   type t gW_t partial gP^T S_t (stored [64][K], lins[t].weight's layout), gb_t = sum w_t gP,
//          Z_t = gP W_t (MFMA, W_t staged in LDS k-major): relation slots: the relation dots
//          <U_t, Z_t> + cnt beta and <x_self, Z_t> + beta in per-row bin columns (no Z to HBM);
//          else Z, beta -> HBM for rel0.
struct Bwd0Args {
    const int32_t* sizes; int hop; int T;
    const float* g0;
    const float* p; const float* w0;
    const float* s_agg; const float* s_w; Ptrs lin_w; Ptrs lin_b;
    const float* rw; int n_rel; float alpha; int n_et;
    const float* u_self; const int32_t* u_rel;
    float* z; float* beta;
    float* slab;     // [t][block][(K + 1) * 64]: g W_t ([64][K]) | g b_t
    float* rslab;    // relation slots: [t][block][64] relation dots
    float* slab0;    // [block][64 * 64]: g W_0
    int64_t* adam_step;  // the fused Adam's step count (advanced here, read by finalize) or null
};

constexpr int kPost0W = F * F;

// a wave group's LDS (tile buffers, row meta, relation bins)
template <int K, bool RS>
constexpr size_t bwd0_group_floats(int n_rel) {
    return size_t(16) * (K + 4) * (RS ? 2 : 1) + 16 * (F + 16) + 16 * (F + 4) + 2 * 16 * 68 +
           16 * 4 + 16 * 2 + 4 * 16 * 2 + size_t(n_rel) * 16;
}
template <int K, bool RS, int NG>
constexpr size_t bwd0_lds_floats(int n_rel) {
    return size_t(K) * (F + 4) + 2 * F + NG * bwd0_group_floats<K, RS>(n_rel);
}

// NG wave groups of 4 waves per block: group g takes tiles NG b + g, NG (b + grid) + g, ..; the
// groups' W_t image is shared and their partials meet in LDS (group 0 + group 1, fixed order)
// before one slab row per block: NG = 2 with half the blocks keeps the waves per CU and halves
// the split-K slab finalize reads.
template <int K, bool RS, int NG>
__global__ void __launch_bounds__(kBlock * NG) bwd0_kernel(Bwd0Args A) {
    static_assert(NG == 1 || NG == 2, "one or two wave groups");
    constexpr int XS = K + 4, GS = F + 16, G2 = F + 4, WS = F + 4;
    constexpr int KB = K / 64;                // k blocks per wave
    constexpr int XV = K / 4 * 16 / kBlock;   // float4 per thread per 16-row tile of a K-wide row
    extern __shared__ float sm[];
    PH(2, 12);
    PE(3, 0);
    float* Wk = sm;                           // [K][WS]: W_t k-major; after the loop: group 1's
                                              // W_t partial on its way to group 0
    // the fused Adam's step count advances here, the launch before finalize, which reads it:
    // no completion ticket among finalize's blocks (their contended atomic was its tail)
    if (A.adam_step && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) A.adam_step[0] += 1;
    float* bc = Wk + K * WS;                  // [F] b_t
    float* tabl = bc + F;                     // [F]
    const int grp = NG == 1 ? 0 : int(threadIdx.x) / kBlock;
    const int tid = int(threadIdx.x) - grp * kBlock;
    float* gbase = tabl + F + grp * bwd0_group_floats<K, RS>(A.n_rel);
    float* ush = gbase;                       // [16][XS] U_t (RS) or S_t
    float* xsh = ush + 16 * XS;               // [16][XS] x_self (RS only)
    float* gsh = xsh + (RS ? 16 * XS : 0);    // [16][GS] gP
    float* gs2 = gsh + 16 * GS;               // [16][G2] gP
    float* g0s = gs2 + 16 * G2;               // [16][68] G0
    float* psh = g0s + 16 * 68;               // [16][68] P (t = 0)
    float* rm = psh + 16 * 68;                // [16][4]: wr, ws, cnt, beta
    int* rr = reinterpret_cast<int*>(rm + 64);  // [16][2]: r_vt (or -1), r_self (or -1)
    float* dred = reinterpret_cast<float*>(rr + 32);   // [4 waves][16][2]
    float* bins = dred + 128;                 // [n_rel][16]
    const int t = blockIdx.y, T = A.T;
    const bool t0 = t == 0;
    const float* wt = pick(A.lin_w.p, t);
    // W_t[j][k] -> Wk[k][j]: lane-consecutive j (conflict-free LDS writes), a float4 of row j
    // per element group, every load of the thread in flight at once
#pragma unroll
    for (int e = threadIdx.x; e < K / 4 * F; e += kBlock * NG) {
        const int j = e & (F - 1), k4 = e >> 6;
        const float4 v = *reinterpret_cast<const float4*>(wt + j * K + 4 * k4);
        Wk[(4 * k4 + 0) * WS + j] = v.x;
        Wk[(4 * k4 + 1) * WS + j] = v.y;
        Wk[(4 * k4 + 2) * WS + j] = v.z;
        Wk[(4 * k4 + 3) * WS + j] = v.w;
    }
    if (threadIdx.x < F) {
        bc[threadIdx.x] = pick(A.lin_b.p, t)[threadIdx.x];
        tabl[threadIdx.x] = rel_tab(A.rw, A.n_rel, A.alpha, threadIdx.x);
    }
    if constexpr (RS)
        for (int i = tid; i < A.n_rel * 16; i += kBlock) bins[i] = 0.f;
    const int n = A.sizes[A.hop];
    const int w = tid >> 6, lane = tid & 63, c = lane & 15, q = lane >> 4;
    const int gr = tid >> 4, gj = tid & 15;
    float4 w0r[4];                            // W_0[16 w + c][16 b + 4 q ..]: gP's B operand
#pragma unroll
    for (int b = 0; b < 4; ++b)
        w0r[b] = *reinterpret_cast<const float4*>(A.w0 + (16 * w + c) * F + 16 * b + 4 * q);
    f32x4 acc[KB][4], acc0[4];
#pragma unroll
    for (int a = 0; a < KB; ++a)
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) acc[a][jb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) acc0[jb] = f32x4{0.f, 0.f, 0.f, 0.f};
    float bsum = 0.f;
    // prefetched rows of the next tile
    float4 ur[XV], xr[XV];
    float4 g4 = make_float4(0.f, 0.f, 0.f, 0.f), p4 = make_float4(0.f, 0.f, 0.f, 0.f);
    float cntv = 0.f;
    int relv = -1, rsv = -1;
    auto load = [&](int v0) {
#pragma unroll
        for (int u = 0; u < XV; ++u) {
            const int e = tid + kBlock * u;
            const int r = e / (K / 4), k4 = e - r * (K / 4);
            const bool ok = v0 + r < n;
            ur[u] = ok ? *reinterpret_cast<const float4*>(A.s_agg + (int64_t(v0 + r) * T + t) * K + 4 * k4)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
            if constexpr (RS)
                xr[u] = ok ? *reinterpret_cast<const float4*>(A.u_self + int64_t(v0 + r) * K + 4 * k4)
                           : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        const int v = v0 + gr;
        const bool okv = v < n;
        g4 = okv ? *reinterpret_cast<const float4*>(A.g0 + int64_t(v) * F + 4 * gj)
                 : make_float4(0.f, 0.f, 0.f, 0.f);
        if (t0)
            p4 = okv ? *reinterpret_cast<const float4*>(A.p + int64_t(v) * F + 4 * gj)
                     : make_float4(0.f, 0.f, 0.f, 0.f);
        if (tid < 16) {
            const int vv = v0 + tid;
            const bool ok = vv < n;
            cntv = ok ? A.s_w[int64_t(vv) * T + t] : 0.f;
            if constexpr (RS) {
                relv = ok ? A.u_rel[int64_t(vv) * (T + 1) + t] : -1;
                rsv = ok ? A.u_rel[int64_t(vv) * (T + 1) + T] : -1;
            }
        }
    };
    const int stride = int(gridDim.x) * NG;   // tiles per round of the grid
    PH(2, 0);
    if ((int(blockIdx.x) * NG + grp) * 16 < n) load((int(blockIdx.x) * NG + grp) * 16);
    __syncthreads();
    PH(2, 1);
    // rounds: block-uniform (every group reaches every barrier); a group past the rows idles
    for (int base = int(blockIdx.x) * NG; base * 16 < n; base += stride) {
        const int tile = base + grp;
        const bool has = tile * 16 < n;       // group-uniform
        const int v0 = tile * 16;
        if (has) {
            *reinterpret_cast<float4*>(g0s + gr * 68 + 4 * gj) = g4;
            if (t0) *reinterpret_cast<float4*>(psh + gr * 68 + 4 * gj) = p4;
            if (tid < 16) {                    // row meta: S = wr U + ws x_self (RS)
                if constexpr (RS) {
                    const bool self = rsv >= 0 && rsv - A.n_et == t;
                    rm[4 * tid] = relv >= 0 ? tabl[relv] : 0.f;
                    rm[4 * tid + 1] = self ? tabl[rsv] : 0.f;
                    rr[2 * tid] = (relv >= 0 && cntv > 0.f) ? relv : -1;
                    rr[2 * tid + 1] = self ? rsv : -1;
                } else {
                    rm[4 * tid] = 1.f;
                    rm[4 * tid + 1] = 0.f;
                }
                rm[4 * tid + 2] = cntv;
            }
#pragma unroll
            for (int u = 0; u < XV; ++u) {
                const int e = tid + kBlock * u;
                const int r = e / (K / 4), k4 = e - r * (K / 4);
                *reinterpret_cast<float4*>(ush + r * XS + 4 * k4) = ur[u];
                if constexpr (RS) *reinterpret_cast<float4*>(xsh + r * XS + 4 * k4) = xr[u];
            }
        }
        __syncthreads();
        if ((tile + stride) * 16 < n) load((tile + stride) * 16);
        // ---- gP = G0 W_0^T -> gsh / gs2; t = 0: W_0 partial D[k][j] = sum_v P[v][k] G0[v][j]
        if (has) {
            f32x4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const float4 av = *reinterpret_cast<const float4*>(g0s + c * 68 + 16 * b + 4 * q);
                MFMA4(av, w0r[b].x, w0r[b].y, w0r[b].z, w0r[b].w, d);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                gsh[(4 * q + r) * GS + 16 * w + c] = d[r];
                gs2[(4 * q + r) * G2 + 16 * w + c] = d[r];
            }
            if (t0) {
#pragma unroll
                for (int st = 0; st < 4; ++st) {
                    const int r = 4 * st + q;
                    const float av = psh[r * 68 + 16 * w + c];
#pragma unroll
                    for (int jb = 0; jb < 4; ++jb)
                        acc0[jb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, g0s[r * 68 + 16 * jb + c], acc0[jb], 0, 0, 0);
                }
            }
        }
        __syncthreads();
        if (has) {
            if (tid < F) {                     // g b_t = sum_v w_vt gP_v
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float wv = RS ? fmaf(rm[4 * r], rm[4 * r + 2], rm[4 * r + 1]) : rm[4 * r + 2];
                    bsum = fmaf(wv, gsh[r * GS + tid], bsum);
                }
            }
            // g W_t partial D[k][j] = sum_v S_vt[k] gP_v[j] over the tile's (re-formed) S rows
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
                    const float av = RS ? fmaf(ws, xsh[r * XS + k], wr * ush[r * XS + k]) : ush[r * XS + k];
#pragma unroll
                    for (int jb = 0; jb < 4; ++jb)
                        acc[a][jb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[jb], acc[a][jb], 0, 0, 0);
                }
            }
            // Z_t = gP W_t (wave w -> k blocks KB w ..): relation dots (RS) or Z to HBM
            float pu[4] = {0.f, 0.f, 0.f, 0.f}, ps[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int a = 0; a < KB; ++a) {
                const int kb = KB * w + a;
                f32x4 zc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int b = 0; b < F / 16; ++b) {
                    const float4 av = *reinterpret_cast<const float4*>(gs2 + c * G2 + 16 * b + 4 * q);
                    const float4 bw = *reinterpret_cast<const float4*>(Wk + (16 * kb + c) * WS + 16 * b + 4 * q);
                    MFMA4(av, bw.x, bw.y, bw.z, bw.w, zc);
                }
                // zc[r] = Z[row 4 q + r][k = 16 kb + c]
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if constexpr (RS) {
                        pu[r] = fmaf(zc[r], ush[(4 * q + r) * XS + 16 * kb + c], pu[r]);
                        ps[r] = fmaf(zc[r], xsh[(4 * q + r) * XS + 16 * kb + c], ps[r]);
                    } else {
                        const int v = v0 + 4 * q + r;
                        if (v < n) A.z[(int64_t(v) * T + t) * K + 16 * kb + c] = zc[r];
                    }
                }
            }
            if constexpr (RS) {
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
            }
            {                                  // beta_vt = <b_t, gP_v>
                const float4 g4v = *reinterpret_cast<const float4*>(gs2 + gr * G2 + 4 * gj);
                float bt = bc[4 * gj] * g4v.x + bc[4 * gj + 1] * g4v.y + bc[4 * gj + 2] * g4v.z +
                           bc[4 * gj + 3] * g4v.w;
                bt = group_sum<16>(bt);
                if (gj == 0) {
                    if constexpr (RS) rm[4 * gr + 3] = bt;
                    else if (v0 + gr < n) A.beta[int64_t(v0 + gr) * T + t] = bt;
                }
            }
        }
        __syncthreads();
        if constexpr (RS) {
            if (has && tid < 16) {             // row r's relation dots into its bin column
                const int r = tid;
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
    }
    PH(2, 2);
    if constexpr (NG == 2) {
        // group 1's partials into LDS (W_t partial over Wk, the rest over its tile buffers),
        // group 0 adds them to its own: one slab row per block
        float* xg = tabl + F + bwd0_group_floats<K, RS>(A.n_rel);   // group 1's region
        float* x0 = xg + 4 * 64 * 16;          // after its W_0 partial: the bias partial
        __syncthreads();                       // every group done with Wk
        if (grp == 1) {
#pragma unroll
            for (int a = 0; a < KB; ++a)
#pragma unroll
                for (int jb = 0; jb < 4; ++jb)
                    *reinterpret_cast<f32x4*>(Wk + ((w * KB + a) * 4 + jb) * 256 + 4 * lane) = acc[a][jb];
            if (t0) {
#pragma unroll
                for (int jb = 0; jb < 4; ++jb)
                    *reinterpret_cast<f32x4*>(xg + (w * 4 + jb) * 256 + 4 * lane) = acc0[jb];
            }
            if (tid < F) x0[tid] = bsum;
        }
        __syncthreads();
        if (grp == 1) return;                  // (no barrier follows)
#pragma unroll
        for (int a = 0; a < KB; ++a)
#pragma unroll
            for (int jb = 0; jb < 4; ++jb)
                acc[a][jb] += *reinterpret_cast<const f32x4*>(Wk + ((w * KB + a) * 4 + jb) * 256 + 4 * lane);
        if (t0) {
#pragma unroll
            for (int jb = 0; jb < 4; ++jb)
                acc0[jb] += *reinterpret_cast<const f32x4*>(xg + (w * 4 + jb) * 256 + 4 * lane);
        }
        if (tid < F) bsum += x0[tid];
    }
    // ---- partials: g W_t as [64][K] (lins[t].weight's layout), g b_t
    float* o = A.slab + (int64_t(t) * gridDim.x + blockIdx.x) * int64_t((K + 1) * F);
#pragma unroll
    for (int a = 0; a < KB; ++a)
#pragma unroll
        for (int jb = 0; jb < 4; ++jb)
        {
            const f32x4 v4 = acc[a][jb];
            // non-temporal: the launch boundary after bwd0 measured 3.3 us instead of 4.6 (the
            // same for agg0's per-type sums measured nothing)
            __builtin_nontemporal_store(v4, reinterpret_cast<f32x4*>(o + int64_t(16 * jb + c) * K + 16 * (KB * w + a) + 4 * q));
        }
    if (tid < F) o[K * F + tid] = bsum;
    if constexpr (RS) {
        if (tid < F) {
            float sr = 0.f;
            if (tid < A.n_rel) {
#pragma unroll
                for (int r = 0; r < 16; ++r) sr += bins[tid * 16 + r];
                if constexpr (NG == 2) {       // group 1's bins, added after group 0's
                    const float* bins1 = bins + bwd0_group_floats<K, RS>(A.n_rel);
                    float s1 = 0.f;
#pragma unroll
                    for (int r = 0; r < 16; ++r) s1 += bins1[tid * 16 + r];
                    sr += s1;
                }
            }
            A.rslab[(int64_t(t) * gridDim.x + blockIdx.x) * F + tid] = sr;
        }
    }
    if (t0) {
        float* o0 = A.slab0 + int64_t(blockIdx.x) * kPost0W;
#pragma unroll
        for (int jb = 0; jb < 4; ++jb)
#pragma unroll
            for (int i = 0; i < 4; ++i) o0[(16 * w + 4 * q + i) * F + 16 * jb + c] = acc0[jb][i];
    }
    PE(3, 1);
}

// ---------------------------------------------------------------------------------------------
// finalize: every gradient a fixed-order sum of per-block partials (re_nsm.hip's job table);
// with the optimizer attached, element e of a job's destination (a view into the flat gradient
// bucket) is followed by Adam on parameter (dst + e - grad_base) of the flat buffers.
enum { kOpCopy = 0, kOpRel = 1, kOpLoss = 2, kOpFix = 3, kOpOutW = 4 };

struct Job {
    const float* src;
    int64_t pstride;
    int nparts, width, op, adam, vec;    // vec: 4 elements per thread (float4 partial rows)
    int cb;                  // columns (elements, or float4 columns if vec) per block: 32, 16, 8
    float* dst;
    const float* aux;        // kOpRel: relation_weight; kOpLoss: the labelled-target count;
                             // kOpOutW: the head's h rows (src: its g rows, nparts rows, width C)
    unsigned long long* fix; // kOpFix: 2^-40 fixed-point terms added to the sum, then zeroed
};

struct AdamArgs {
    float* p; float* m; float* v; const float* gbase; int64_t n;
    float lr, b1, b2, eps, wd, gscale;
    const int64_t* step; int on;           // step: this step's t (bwd0 advanced it)
};

constexpr int kMaxJobs = 32;

struct FinArgs {
    int n_jobs;
    float alpha;
    int start[kMaxJobs];
    Job job[kMaxJobs];
    AdamArgs adam;
};

// the bias corrections of this step, once per block (thread 64)
__device__ __forceinline__ void adam_consts(const AdamArgs& O, int64_t& s_t, float& s_step,
                                            float& s_bc2) {
    if (O.on && threadIdx.x == 64) {
        const int64_t t = O.step[0];
        const double bc1 = 1.0 - pow(double(O.b1), double(t));
        const double bc2 = 1.0 - pow(double(O.b2), double(t));
        s_t = t;
        s_step = float(double(O.lr) / bc1);
        s_bc2 = float(sqrt(bc2));
    }
}

// torch.optim.Adam on one element (regnn_adam_flat's arithmetic)
__device__ __forceinline__ void adam_elem(const AdamArgs& O, int64_t i, float g, float pi,
                                          float mi, float vi, float s_step, float s_bc2) {
    float gi = g * O.gscale;
    if (O.wd != 0.f) gi = gi + O.wd * pi;
    const float mn = mi + (1.f - O.b1) * (gi - mi);
    const float vn = vi * O.b2 + (1.f - O.b2) * gi * gi;
    O.m[i] = mn;
    O.v[i] = vn;
    O.p[i] = pi - s_step * (mn / (sqrtf(vn) / s_bc2 + O.eps));
}

// the G = 256 / cb group sums of one column, combined in a fixed tree (8-wide trees, then
// pairwise over the 8-group chunks)
template <typename V, typename Add>
__device__ __forceinline__ V group_tree(const V* red, int cb, int el, Add add) {
    const int G = kBlock / cb;
    V c[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (8 * k < G) {
            const V* r = red + 8 * k * cb + el;
            c[k] = add(add(add(r[0], r[cb]), add(r[2 * cb], r[3 * cb])),
                       add(add(r[4 * cb], r[5 * cb]), add(r[6 * cb], r[7 * cb])));
        }
    }
    if (G == 8) return c[0];
    if (G == 16) return add(c[0], c[1]);
    return add(add(c[0], c[1]), add(c[2], c[3]));
}

__device__ __forceinline__ float4 add4(float4 a, float4 b) {
    return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

// 4 consecutive elements per thread: cb float4 columns x 256 / cb partial groups per block
// (narrow jobs get more groups: fewer dependent load rounds over their partial rows); partials
// grp, grp + G, ... summed in order, the groups in a fixed tree
__device__ __forceinline__ void finalize_vec(const FinArgs& A, const Job& J, const AdamArgs& O,
                                             int b, int el, int grp, int64_t& s_t, float& s_step,
                                             float& s_bc2) {
    __shared__ float4 red4[kBlock];
    const int cb = J.cb, G = kBlock / cb;
    const int e = (b * cb + el) * 4;
    const int64_t i = (J.dst + e) - O.gbase;
    const bool stepped = O.on && J.adam && grp == 0 && e < J.width && i >= 0 && i < O.n;
    float pi[4] = {0.f, 0.f, 0.f, 0.f}, mi[4] = {0.f, 0.f, 0.f, 0.f}, vi[4] = {0.f, 0.f, 0.f, 0.f};
    if (stepped) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            pi[k] = O.p[i + k]; mi[k] = O.m[i + k]; vi[k] = O.v[i + k];
        }
    }
    adam_consts(O, s_t, s_step, s_bc2);
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (e < J.width) {
        const float4* src = reinterpret_cast<const float4*>(J.src + e);
        const int64_t ps = J.pstride / 4;
        int p = grp;
        for (; p + 7 * G < J.nparts; p += 8 * G) {
            float4 vv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) vv[u] = src[int64_t(p + G * u) * ps];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                s.x += vv[u].x; s.y += vv[u].y; s.z += vv[u].z; s.w += vv[u].w;
            }
        }
        for (; p < J.nparts; p += G) {
            const float4 v = src[int64_t(p) * ps];
            s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
    }
    red4[grp * cb + el] = s;
    __syncthreads();
    if (grp == 0 && e < J.width) {
        const float4 tot = group_tree(red4, cb, el, add4);
        *reinterpret_cast<float4*>(J.dst + e) = tot;
        if (stepped) {
            const float t4[4] = {tot.x, tot.y, tot.z, tot.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) adam_elem(O, i + k, t4[k], pi[k], mi[k], vi[k], s_step, s_bc2);
        }
    }
}

__device__ __forceinline__ void finalize_scalar(const FinArgs& A, const Job& J, const AdamArgs& O,
                                                int b, int el, int grp, int64_t& s_t,
                                                float& s_step, float& s_bc2) {
    __shared__ float red[kBlock];
    const int cb = J.cb, G = kBlock / cb;
    const int e = b * cb + el;
    // the optimizer's operands of this thread's element, requested before the partial sums
    const int64_t i = (J.dst + e) - O.gbase;
    const bool stepped = O.on && J.adam && grp == 0 && e < J.width && i >= 0 && i < O.n;
    float pi = 0.f, mi = 0.f, vi = 0.f;
    if (stepped) {
        pi = O.p[i]; mi = O.m[i]; vi = O.v[i];
    }
    adam_consts(O, s_t, s_step, s_bc2);
    float s = 0.f;
    if (e < J.width) {
        const float* src = J.src + e;
        int p = grp;
        for (; p + 7 * G < J.nparts; p += 8 * G) {     // 8 partial rows in flight per thread
            float vv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) vv[u] = src[int64_t(p + G * u) * J.pstride];
#pragma unroll
            for (int u = 0; u < 8; ++u) s += vv[u];
        }
        for (; p < J.nparts; p += G) s += src[int64_t(p) * J.pstride];
    }
    red[grp * cb + el] = s;
    __syncthreads();
    PH(3, 1);
    if (grp == 0 && e < J.width) {
        const float tot = group_tree(red, cb, el, [](float a, float b) { return a + b; });
        float out = tot;
        if (J.op == kOpRel) {
            const float x = J.aux[e] * A.alpha;                // d tab / d rw (LeakyReLU)
            out = tot * A.alpha * (x > 0.f ? 1.f : 0.01f);
        } else if (J.op == kOpLoss) {
            const float nv = *J.aux;
            out = nv > 0.f ? tot / nv : 0.f;
            if (J.fix && J.fix[0]) {           // the gather's fixed-point range was exceeded
                out = __builtin_nanf("");
                J.fix[0] = 0ull;
            }
        } else if (J.op == kOpFix) {           // the gather's hub rows (exact), then reset
            out = tot + float((long long)J.fix[e]) * kFixInv;
            J.fix[e] = 0ull;
        }
        J.dst[e] = out;
        // torch.optim.Adam (regnn_adam_flat's arithmetic); a gradient outside the bucket (a
        // frozen parameter's scratch buffer) is not stepped
        if (stepped) adam_elem(O, i, out, pi, mi, vi, s_step, s_bc2);
    }
}

// out_lin.weight's gradient tile (16 classes x 16 features) of block b = 4 class-tile + feature
// tile: D[c][k] = sum_v g[v][c] h[v][k] over the head's rows (rows past the batch hold zeros);
// wave w takes rows w R/4 .., the four row quarters added in a fixed order (MFMA lane (c, q):
// A = g[v0 + q][c0 + c], B = h[v0 + q][k0 + c]; D row 4 q + r = class, column c = feature)
__device__ __forceinline__ void finalize_outw(const Job& J, const AdamArgs& O, int b,
                                              int64_t& s_t, float& s_step, float& s_bc2) {
    __shared__ float red[4][256];
    const int C = J.width, R = J.nparts;
    const int c0 = 16 * (b >> 2), k0 = 16 * (b & 3);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, cc = lane & 15, q = lane >> 4;
    // this thread's element after the reduction: class c0 + t / 16, feature k0 + t % 16
    const int ec = c0 + (threadIdx.x >> 4), ek = k0 + (threadIdx.x & 15);
    const int64_t e = int64_t(ec) * F + ek;
    const int64_t i = (J.dst + e) - O.gbase;
    const bool stepped = O.on && J.adam && ec < C && i >= 0 && i < O.n;
    float pi = 0.f, mi = 0.f, vi = 0.f;
    if (stepped) {
        pi = O.p[i]; mi = O.m[i]; vi = O.v[i];
    }
    adam_consts(O, s_t, s_step, s_bc2);
    const int rq = ((R + 15) / 16) * 4;        // rows per wave (a multiple of 4)
    const int v0 = w * rq, v1 = min(R, v0 + rq);
    const int cl = min(c0 + cc, C - 1);
    const bool cok = c0 + cc < C;
    const float* g = J.src + cl;
    const float* h = J.aux + k0 + cc;
    f32x4 d = {0.f, 0.f, 0.f, 0.f};
    constexpr int UN = 32;                     // every row of a 512-row batch in one load round
    for (int v = v0; v < v1; v += 4 * UN) {
        float av[UN], bv[UN];
#pragma unroll
        for (int u = 0; u < UN; ++u) {          // clamped rows (zeroed past the range below)
            const int vv = v + 4 * u + q;
            const int vc = vv < v1 ? vv : v0;
            av[u] = g[int64_t(vc) * C];
            bv[u] = h[int64_t(vc) * F];
        }
        __builtin_amdgcn_sched_barrier(0);      // every load issued before the first MFMA
#pragma unroll
        for (int u = 0; u < UN; ++u) {
            const bool ok = v + 4 * u + q < v1;
            d = __builtin_amdgcn_mfma_f32_16x16x4f32(ok && cok ? av[u] : 0.f, ok ? bv[u] : 0.f, d, 0, 0, 0);
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) red[w][(4 * q + r) * 16 + cc] = d[r];
    __syncthreads();
    if (ec < C) {
        const int t = threadIdx.x;
        const float tot = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
        J.dst[e] = tot;
        if (stepped) adam_elem(O, i, tot, pi, mi, vi, s_step, s_bc2);
    }
}

__global__ void __launch_bounds__(kBlock) finalize_kernel(FinArgs A) {
    __shared__ int64_t s_t;
    __shared__ float s_step, s_bc2;
    int ji = 0;
#pragma unroll
    for (int i = 1; i < kMaxJobs; ++i) ji += (i < A.n_jobs && int(blockIdx.x) >= A.start[i]);
    const int b = blockIdx.x - A.start[ji];
    const Job J = A.job[ji];
    const AdamArgs& O = A.adam;
    PH(3, 0);
    PE(4, 0);
    const int el = threadIdx.x % J.cb, grp = threadIdx.x / J.cb;
    if (J.op == kOpOutW) {                     // block-uniform
        finalize_outw(J, O, b, s_t, s_step, s_bc2);
    } else if (J.vec) {
        finalize_vec(A, J, O, b, el, grp, s_t, s_step, s_bc2);
    } else {
        finalize_scalar(A, J, O, b, el, grp, s_t, s_step, s_bc2);
    }
    PH(3, 2);
    PE(4, 1);
}

struct JobList {
    FinArgs A{};
    int blocks = 0;
    void add(const float* src, int64_t pstride, int nparts, int width, float* dst, int op = kOpCopy,
             const float* aux = nullptr, unsigned long long* fix = nullptr) {
        A.start[A.n_jobs] = blocks;
        Job& j = A.job[A.n_jobs++];
        j.src = src; j.pstride = pstride; j.nparts = nparts; j.width = width; j.dst = dst;
        j.op = op; j.aux = aux; j.fix = fix; j.adam = op != kOpLoss;
        j.vec = op == kOpCopy && width % 4 == 0 && pstride % 4 == 0 &&
                reinterpret_cast<uintptr_t>(src) % 16 == 0 &&
                reinterpret_cast<uintptr_t>(dst) % 16 == 0;
        const int cols = j.vec ? width / 4 : width;
        // wide jobs over many partial rows (bwd0's 128 per type): 16 columns x 16 groups per
        // block, twice the blocks and half the partial rows per thread (107.7-108.7 against
        // 108.5-108.7 us per step with 32 columns)
        j.cb = cols <= 8 ? 8 : (cols <= 16 || (j.vec && nparts >= 64)) ? 16 : 32;
        blocks += (cols + j.cb - 1) / j.cb;
    }
    // out_lin.weight [C][64] = g^T h: g rows [rows][C], h rows [rows][64]; 4 blocks per 16 classes
    void add_outw(const float* g, const float* h, int rows, int C, float* dst) {
        A.start[A.n_jobs] = blocks;
        Job& j = A.job[A.n_jobs++];
        j.src = g; j.aux = h; j.pstride = 0; j.nparts = rows; j.width = C; j.dst = dst;
        j.op = kOpOutW; j.fix = nullptr; j.adam = 1; j.vec = 0; j.cb = 16;
        blocks += 4 * ((C + 15) / 16);
    }
};

struct Slab2 {
    int64_t head, hg, hh, gath, rel0, proj, post0, total;
    int head_blocks, rel0_rows;
};

inline Slab2 slab2(const regnn_nsm_params* p, int cap0) {
    Slab2 s{};
    s.head_blocks = (cap0 + kRows - 1) / kRows;
    int64_t o = 0;
    s.head = o;
    o += int64_t(s.head_blocks) * head_part_width(p->n_classes);
    s.hg = o;                                  // the head's g rows [rows][C] and h rows [rows][64]
    o += int64_t(s.head_blocks) * kRows * p->n_classes;
    s.hh = o;
    o += int64_t(s.head_blocks) * kRows * F;
    s.gath = o;                                // the gather's relation dots and row terms
    o += int64_t(kGathBlocks) * kGathW;
    s.rel0 = o;                                // bwd0's (RS) or rel0's relation rows
    s.rel0_rows = p->rel_slots ? p->n_types * kBwdBlocks : kAggBlocks;
    o += int64_t(p->n_types * kBwdBlocks > kAggBlocks ? p->n_types * kBwdBlocks : kAggBlocks) * F;
    s.proj = o;
    o += int64_t(p->n_types) * kBwdBlocks * (p->k_in + 1) * F;
    s.post0 = o;
    o += int64_t(kBwdBlocks) * kPost0W;
    s.total = o;
    return s;
}

}  // namespace nsm2
}  // namespace regnn

using namespace regnn;
using namespace regnn::nsm2;

#ifdef REGNN_NSM2_PHASES
extern "C" int regnn_nsm2_phases(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_nsm2_phase), sizeof(g_nsm2_phase)) == hipSuccess ? 0 : 3;
}
extern "C" int regnn_nsm2_edges(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_nsm2_edge), sizeof(g_nsm2_edge)) == hipSuccess ? 0 : 3;
}
extern "C" int regnn_nsm2_gpieces(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_nsm2_gp), sizeof(g_nsm2_gp)) == hipSuccess ? 0 : 3;
}
extern "C" int regnn_nsm2_edges_reset(void) {
    static unsigned long long zero[5][2][4096];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_nsm2_edge), zero, sizeof(zero)) == hipSuccess ? 0 : 3;
}
#endif

// entry points used by re_nsm.hip's regnn_nsm_step / regnn_nsm_slab_floats for L = 2
int64_t regnn_nsm2_slab_floats(const regnn_nsm_params* p, int32_t cap0) {
    return slab2(p, cap0).total;
}

// the caller's two_layer flag decides (it allocated the two-layer buffers: hop 0's edge capacity
// fits the transposed index), so the slab size and the step always agree
bool regnn_nsm2_covers(const regnn_nsm_params* p) {
    return p->two_layer == 1 && p->n_layers == 2 && p->n_classes <= 16 * kMaxCT &&
           head_lds(p->n_classes) <= size_t(160 * 1024 - 2560);
}

// the jobs whose partials are complete after the gather: out_lin, the head's layer-1 terms, the
// loss, W_1, layer 1's relation table, layer 0's conv bias / LayerNorm (the gather's row terms)
static void add_early_jobs(JobList& J, const regnn_nsm_params* p, const regnn_nsm_work* w,
                           const Slab2& S) {
    const int C = p->n_classes;
    J.A.alpha = p->alpha;
    const int64_t hw = head_part_width(C);
    const float* hp = w->slab + S.head;
    const int nh = S.head_blocks;
    const int64_t o_cb = C, o_w1 = head_o_w1(C);
    J.add_outw(w->slab + S.hg, w->slab + S.hh, nh * kRows, C, p->g_out_w);
    J.add(hp, hw, nh, C, p->g_out_b);
    J.add(hp + o_cb, hw, nh, F, p->g_conv_b[1]);
    J.add(hp + o_cb + F, hw, nh, F, p->g_ln_b[1]);
    J.add(hp + o_cb + 2 * F, hw, nh, F, p->g_ln_w[1]);
    J.add(hp + o_cb + 3 * F, hw, nh, 1, p->loss, kOpLoss, w->nvalid, w->hub_terms + 3 * F);
    J.add(hp + o_w1, hw, nh, F * F, p->g_conv_w[1]);
    const float* gs = w->slab + S.gath;
    J.add(gs, kGathW, kGathBlocks, p->n_rel[1], p->g_conv_rw[1], kOpRel, p->conv_rw[1]);
    J.add(gs + F, kGathW, kGathBlocks, F, p->g_conv_b[0], kOpFix, nullptr, w->hub_terms);
    J.add(gs + 2 * F, kGathW, kGathBlocks, F, p->g_ln_b[0], kOpFix, nullptr, w->hub_terms + F);
    J.add(gs + 3 * F, kGathW, kGathBlocks, F, p->g_ln_w[0], kOpFix, nullptr, w->hub_terms + 2 * F);
}

static void launch_finalize(JobList& J, const regnn_nsm_params* p, const regnn_nsm_adam* ad,
                            hipStream_t stream) {
    J.A.alpha = p->alpha;
    if (ad) {
        AdamArgs& O = J.A.adam;
        O.p = ad->param; O.m = ad->exp_avg; O.v = ad->exp_avg_sq; O.gbase = ad->grad_base;
        O.n = ad->n;
        O.lr = ad->lr; O.b1 = ad->beta1; O.b2 = ad->beta2; O.eps = ad->eps;
        O.wd = ad->weight_decay; O.gscale = ad->grad_scale; O.step = ad->step; O.on = 1;
    }
    hipLaunchKernelGGL(finalize_kernel, dim3(J.blocks), dim3(kBlock), 0, stream, J.A);
}

int regnn_nsm2_step(const regnn_nsm_params* p, const regnn_nsm_work* w, hipStream_t stream) {
    const int T = p->n_types, K = p->k_in, C = p->n_classes;
    const bool rs = p->rel_slots != 0;
    if (!w->p0 || !w->gh1 || !w->csc_ptr0 || !w->csc_ent0 || !w->csc_long0 || !w->xs[1] || !w->a[0] ||
        !w->stats[0] || !w->ga[0] || !w->hub_acc || !w->hub_ticket || !w->hub_terms)
        return REGNN_EINVAL;
    for (int h = 0; h < 2; ++h)
        if (w->stride[h] < 0 || (w->stride[h] && !w->blk_cnt[h])) return REGNN_EINVAL;
    const regnn_nsm_adam* ad = w->adam;
    if (ad && (!ad->param || !ad->exp_avg || !ad->exp_avg_sq || !ad->grad_base || !ad->step))
        return REGNN_EINVAL;
    // split_finalize: the gradients final after the gather (head, layer 1, layer 0's LayerNorm and
    // conv bias) are reduced by a finalize launch at the end of part 1, so a caller can exchange
    // them while part 2 runs; the fused Adam (its step count advances in bwd0) excludes it
    const bool split = w->split_finalize != 0;
    if (split && ad) return REGNN_EINVAL;
    const Slab2 S = slab2(p, w->cap[0]);
    const Drop drop = make_drop(p->p_drop);
    Ptrs lin_w{}, lin_b{}, xt{};
    for (int t = 0; t < T; ++t) {
        lin_w.p[t] = p->lin_w[t];
        lin_b.p[t] = p->lin_b[t];
        xt.p[t] = p->x_tab[t];
    }
    const bool first = w->part != 2, second = w->part != 1;
    // layer 0's input sums formed by the sampler (regnn_ns_hop_typed_sums)
    const bool pre = w->pre_sums != 0;
    // 1. layer 0
    if (first) {
        const int h = 1;
        Agg0Args A{};
        A.sizes = w->sizes; A.hop = h;
        A.ptr = w->blk_ptr[h]; A.cnt = w->blk_cnt[h]; A.stride = w->stride[h];
        A.rel = w->blk_rel[h]; A.inv = w->blk_inv[h];
        A.edge_type = w->edge_type; A.edge_off = w->edge_off; A.xt = xt; A.T = T;
        A.lin_w = lin_w; A.lin_b = lin_b;
        A.rw = p->conv_rw[0]; A.n_rel = p->n_rel[0]; A.alpha = p->alpha;
        A.w0 = p->conv_w[0]; A.bias = p->conv_b[0]; A.ln_w = p->ln_w[0]; A.ln_b = p->ln_b[0];
        A.state = w->state; A.drop = drop;
        A.s_agg = w->s_agg; A.s_w = w->s_w;
        A.a = w->a[0]; A.stats = w->stats[0]; A.h = w->xs[1]; A.p = w->p0;
        A.n_et = p->n_edge_types; A.u_self = w->u_self; A.u_rel = w->u_rel;
        A.n_id = w->n_id; A.labels = w->labels; A.nvalid = w->nvalid;
        int grid = (w->cap[h] + 15) / 16;
        if (pre && (K != 128 || T > 4 || !rs)) return REGNN_EINVAL;
        if (K == 128 && T <= 4 && (pre || !getenv("REGNN_NSM_AGG0_OLD"))) {  // every tile its own block
            grid = (w->cap[h] + kAggRows - 1) / kAggRows;
            const size_t lds = agg0w_lds(T);
#define AGG0W_CASE(NN, RS, PRE)                                                                \
            if (rs == RS && pre == PRE) {                                                      \
                static size_t done = 0;                                                        \
                if (!set_lds(reinterpret_cast<const void*>(&agg0w_kernel<NN, RS, PRE>), lds, &done)) \
                    return REGNN_EUNSUPPORTED;                                                 \
                hipLaunchKernelGGL((agg0w_kernel<NN, RS, PRE>), dim3(grid), dim3(kAggW), lds, stream, A); \
                REGNN_LAUNCH_CHECK();                                                          \
            } else
            AGG0W_CASE(4, true, true) AGG0W_CASE(4, true, false) AGG0W_CASE(4, false, false)
                return REGNN_EUNSUPPORTED;
#undef AGG0W_CASE
        } else {
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
    }
    // 2. layer 1 + head + loss + backward to GH, transposed aggregation into layer 0's rows
    const int64_t hw = head_part_width(C);
    if (first) {
        HeadArgs H{};
        H.sizes = w->sizes; H.n_id = w->n_id; H.labels = w->labels;
        H.ptr = w->blk_ptr[0]; H.cnt = w->blk_cnt[0]; H.stride = w->stride[0];
        H.idx = w->blk_idx[0]; H.rel = w->blk_rel[0]; H.inv = w->blk_inv[0];
        H.rw = p->conv_rw[1]; H.n_rel = p->n_rel[1]; H.alpha = p->alpha;
        H.h = w->xs[1]; H.w1 = p->conv_w[1]; H.bias = p->conv_b[1];
        H.ln_w = p->ln_w[1]; H.ln_b = p->ln_b[1]; H.state = w->state; H.drop = drop;
        H.w_out = p->out_w; H.b_out = p->out_b; H.C = C;
        H.gh = w->gh1; H.nvalid = w->nvalid; H.part = w->slab + S.head; H.part_w = hw;
        H.g_rows = w->slab + S.hg; H.h_rows = w->slab + S.hh;
        const size_t lds = head_lds(C);
        static size_t done = 0;
        if (!set_lds(reinterpret_cast<const void*>(&head_kernel), lds, &done))
            return REGNN_EUNSUPPORTED;
        hipLaunchKernelGGL(head_kernel, dim3(S.head_blocks), dim3(kHeadThreads), lds, stream, H);
        REGNN_LAUNCH_CHECK();
    }
    // 3. layer 1's transposed aggregation (a gather), layer 0's LayerNorm backward
    if (first) {
        GathArgs G{};
        G.sizes = w->sizes; G.hop = 1; G.cptr = w->csc_ptr0; G.cent = w->csc_ent0;
        G.clong = w->csc_long0; G.gh = w->gh1;
        G.a = w->a[0]; G.stats = w->stats[0]; G.inv = w->blk_inv[1];
        G.ln_w = p->ln_w[0]; G.ln_b = p->ln_b[0]; G.state = w->state; G.drop = drop;
        G.rw = p->conv_rw[1]; G.n_rel = p->n_rel[1]; G.alpha = p->alpha;
        G.g0 = w->ga[0]; G.slab = w->slab + S.gath;
        G.hub_acc = w->hub_acc; G.hub_ticket = w->hub_ticket; G.hub_terms = w->hub_terms;
        hipLaunchKernelGGL(gather_kernel, dim3(kGathBlocks), dim3(kGathT), 0, stream, G);
        REGNN_LAUNCH_CHECK();
        if (split) {
            JobList J;
            add_early_jobs(J, p, w, S);
            launch_finalize(J, p, nullptr, stream);
            REGNN_LAUNCH_CHECK();
        }
    }
    if (!second) return REGNN_OK;
    // 4. layer 0's backward (nb0 blocks per type: one slab row each)
    const int nb0 = kBwdBlocks / kBwdGroups;
    {
        Bwd0Args B{};
        B.sizes = w->sizes; B.hop = 1; B.T = T;
        B.g0 = w->ga[0]; B.p = w->p0; B.w0 = p->conv_w[0];
        B.s_agg = w->s_agg; B.s_w = w->s_w; B.lin_w = lin_w; B.lin_b = lin_b;
        B.rw = p->conv_rw[0]; B.n_rel = p->n_rel[0]; B.alpha = p->alpha; B.n_et = p->n_edge_types;
        B.u_self = w->u_self; B.u_rel = w->u_rel; B.z = w->z; B.beta = w->beta;
        B.slab = w->slab + S.proj; B.rslab = w->slab + S.rel0; B.slab0 = w->slab + S.post0;
        B.adam_step = ad ? ad->step : nullptr;
        const dim3 grid(nb0, T);
#define BWD0_CASE(KK, RS, NG)                                                                  \
        if (K == KK && rs == RS && kBwdGroups == NG) {                                         \
            static size_t done = 0;                                                            \
            const size_t lds = bwd0_lds_floats<KK, RS, NG>(p->n_rel[0]) * sizeof(float);       \
            if (!set_lds(reinterpret_cast<const void*>(&bwd0_kernel<KK, RS, NG>), lds, &done)) \
                return REGNN_EUNSUPPORTED;                                                     \
            hipLaunchKernelGGL((bwd0_kernel<KK, RS, NG>), grid, dim3(kBlock * NG), lds, stream, B); \
            REGNN_LAUNCH_CHECK();                                                              \
        } else
        BWD0_CASE(128, true, 2) BWD0_CASE(64, true, 2) BWD0_CASE(128, false, 2) BWD0_CASE(64, false, 2)
        BWD0_CASE(128, true, 1) BWD0_CASE(64, true, 1) BWD0_CASE(128, false, 1) BWD0_CASE(64, false, 1)
            return REGNN_EUNSUPPORTED;
#undef BWD0_CASE
    }
    // 5. no relation slots: layer 0's relation dots edge by edge (re_nsm.hip's rel0)
    if (!rs) {
        const int rc = regnn_nsm_rel0(p, w, w->slab + S.rel0, stream);
        if (rc != REGNN_OK) return rc;
    }
    // 6. fixed-order reductions (+ Adam): the late jobs (bwd0's and rel0's partials), and the early
    // ones here too unless part 1 reduced them (split_finalize)
    {
        JobList J;
        if (!split) add_early_jobs(J, p, w, S);
        const int64_t pw = int64_t(K + 1) * F;
        J.add(w->slab + S.rel0, F, rs ? T * nb0 : S.rel0_rows, p->n_rel[0], p->g_conv_rw[0], kOpRel,
              p->conv_rw[0]);
        for (int t = 0; t < T; ++t) {
            const float* src = w->slab + S.proj + int64_t(t) * nb0 * pw;
            J.add(src, pw, nb0, K * F, p->g_lin_w[t]);
            J.add(src + int64_t(K) * F, pw, nb0, F, p->g_lin_b[t]);
        }
        J.add(w->slab + S.post0, kPost0W, nb0, F * F, p->g_conv_w[0]);
        launch_finalize(J, p, ad, stream);
        REGNN_LAUNCH_CHECK();
    }
    return REGNN_OK;
}
