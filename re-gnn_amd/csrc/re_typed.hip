// Per-node-type input rows of the ogbn-mag path (mag/regnn_ns.py:300-326, REGNN.group_input):
// every sampled node's feature row comes from its own type's table (raw paper features, random
// or learned embeddings of the other types), and for feats_type != 2 goes through its own
// type's Linear. The reference does this with one boolean mask per type (a host sync each) and
// a Linear over each masked subset.
//
//   typed_gather    out[i] = tab[type(i)][local(i)]        (feats_type 2: a shared Linear follows,
//                                                          a plain GEMM, left to hipBLASLt)
//   typed_scatter   gtab[type(i)][local(i)] += g[i]       (its backward into learned tables)
//   typed_linear    Y[order[i]] = tab[t][src[i]] W[t]^T + b[t] over the rows sorted by type:
//                   the gather fused into an fp32-MFMA GEMM per type run (no gathered copy, no
//                   Linear per masked subset, no all-types GEMM)
//   typed_wgrad     gW[t] = sum_i gY[order[i]]^T tab[t][src[i]], gb[t] = sum_i gY[order[i]]:
//                   per-chunk partials (one 1024-row chunk of one type run, 64 output columns)
//                   reduced in fixed chunk order (deterministic; no atomics)
#include "regnn_common.h"

namespace regnn {
namespace typed {

constexpr int MT = 8;                  // node types
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct Tabs {
    const float* p[MT];
};

// ---------------------------------------------------------------------------------------------
// gather / scatter: KV = K / 4 float4 vectors per row, one thread per vector
__global__ void __launch_bounds__(kBlock)
gather_kernel(const int64_t* __restrict__ n_id, int64_t n, const int64_t* __restrict__ ntype,
              const int64_t* __restrict__ local, int T, Tabs tab, int KV, float* __restrict__ out) {
    const int64_t total = n * KV;
    for (int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * kBlock) {
        const int64_t i = e / KV;
        const int v = int(e - i * KV);
        const int64_t g = n_id ? n_id[i] : i;
        const int64_t t = ntype[g];
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (t >= 0 && t < T && tab.p[t])
            x = reinterpret_cast<const float4*>(tab.p[t] + local[g] * (int64_t)(4 * KV))[v];
        reinterpret_cast<float4*>(out)[e] = x;
    }
}

__global__ void __launch_bounds__(kBlock)
scatter_kernel(const int64_t* __restrict__ n_id, int64_t n, const int64_t* __restrict__ ntype,
               const int64_t* __restrict__ local, int T, Tabs gtab, int K,
               const float* __restrict__ g) {
    const int64_t total = n * K;
    for (int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * kBlock) {
        const int64_t i = e / K;
        const int k = int(e - i * K);
        const int64_t gi = n_id ? n_id[i] : i;
        const int64_t t = ntype[gi];
        if (t >= 0 && t < T && gtab.p[t])
            atomicAdd(const_cast<float*>(gtab.p[t]) + local[gi] * (int64_t)K + k, g[e]);
    }
}

// ---------------------------------------------------------------------------------------------
// run chunks: type t's sorted run [off[t], off[t+1]) is cut into chunks of CH rows; chunk c of
// the launch maps to (t, first row, rows) by a walk over the T runs (T <= 8, read per block).
__device__ __forceinline__ bool chunk_of(const int32_t* __restrict__ off, int T, int CH,
                                         int64_t c, int& t, int64_t& p0, int& cnt) {
    int64_t base = 0;
    for (int u = 0; u < T; ++u) {
        const int64_t a = off[u], b = off[u + 1];
        const int64_t nc = (b - a + CH - 1) / CH;
        if (c < base + nc) {
            t = u;
            p0 = a + (c - base) * CH;
            cnt = int(min<int64_t>(CH, b - p0));
            return true;
        }
        base += nc;
    }
    return false;
}

struct FwdArgs {
    const int64_t* order;      // [n] output row of sorted entry i
    const int64_t* src;        // [n] row of entry i in its type's table
    const int32_t* off;        // [T+1] type runs (device)
    int T, O;
    Tabs tab;                  // [t] tables, [*, K]
    Tabs W;                    // [t] weights [O, K]  (per type; may alias)
    Tabs b;                    // [t] biases [O] or NULL
    float* Y;                  // [n, O]
};

// One block = one chunk of RB rows of one type; the chunk's input rows gathered into LDS once;
// wave w takes output column tiles w, w+4, ... and, per tile, holds its 16 rows of W[t] in
// registers over all RB/16 row tiles. Transposed MFMA (C = W X^T): lane (j, q) ends with row j
// and output columns 16 ct + 4 q .. +3 (one 16-byte store). k-step s, quarter q supplies
// k = KQ q + s (A and B alike), so each lane reads its KQ contiguous floats.
template <int KQ, int RB>
__global__ void __launch_bounds__(kBlock) fwd_kernel(FwdArgs A) {
    constexpr int K = 4 * KQ, LD = K + 4;
    extern __shared__ float Xl[];                        // [RB][LD]
    int t, cnt;
    int64_t p0;
    if (!chunk_of(A.off, A.T, RB, blockIdx.x, t, p0, cnt)) return;   // block-uniform
    const float* tab = A.tab.p[t];
    for (int e = threadIdx.x; e < RB * KQ; e += kBlock) {
        const int r = e / KQ, v = e - r * KQ;
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (r < cnt && tab) x = reinterpret_cast<const float4*>(tab + A.src[p0 + r] * K)[v];
        *reinterpret_cast<float4*>(Xl + r * LD + 4 * v) = x;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4;
    const int w = threadIdx.x >> 6;
    const float* W = A.W.p[t];
    const float* bias = A.b.p[t];
    const int n_rt = (cnt + 15) / 16;
    int64_t orow[RB / 16];
#pragma unroll
    for (int rt = 0; rt < RB / 16; ++rt)
        orow[rt] = (rt < n_rt && 16 * rt + j < cnt) ? A.order[p0 + 16 * rt + j] : -1;
    for (int ct = w; ct < A.O / 16; ct += 4) {
        float a[KQ];
        const float4* wp = reinterpret_cast<const float4*>(W + (int64_t)(16 * ct + j) * K + KQ * q);
#pragma unroll
        for (int u = 0; u < KQ / 4; ++u) {
            const float4 x = wp[u];
            a[4 * u] = x.x; a[4 * u + 1] = x.y; a[4 * u + 2] = x.z; a[4 * u + 3] = x.w;
        }
        f32x4 b0 = {0.f, 0.f, 0.f, 0.f};
        if (bias) b0 = *reinterpret_cast<const f32x4*>(bias + 16 * ct + 4 * q);
        for (int rt = 0; rt < n_rt; ++rt) {
            f32x4 acc = b0;
            const float* xr = Xl + (16 * rt + j) * LD + KQ * q;
#pragma unroll
            for (int u = 0; u < KQ / 4; ++u) {
                const float4 x = *reinterpret_cast<const float4*>(xr + 4 * u);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[4 * u], x.x, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[4 * u + 1], x.y, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[4 * u + 2], x.z, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[4 * u + 3], x.w, acc, 0, 0, 0);
            }
            int64_t orr = orow[0];
#pragma unroll
            for (int r2 = 1; r2 < RB / 16; ++r2) if (r2 == rt) orr = orow[r2];
            if (orr >= 0)
                *reinterpret_cast<f32x4*>(A.Y + orr * A.O + 16 * ct + 4 * q) = acc;
        }
    }
}

struct WgradArgs {
    const int64_t* order;
    const int64_t* src;
    const int32_t* off;
    int T, O;
    Tabs tab;
    const float* gY;           // [n, O]
    float* slab;               // [chunks][O * (K + 1)]: [O][K] weight partial | [O] bias partial
};

constexpr int kWRows = 1024;           // rows of one wgrad chunk
constexpr int kWSub = 32;              // rows staged per step

// Block (chunk c, output group og of 64 columns): wave w owns output columns 64 og + 16 w .. +15
// and every k tile of 16: D[o][k] += gY[row][o] X[row][k] over 4 rows per MFMA (lane (i, q):
// A = gY[row 4 s + q][o 16 w + i], B = X[row 4 s + q][16 kt + i]). 32-row steps staged in LDS.
template <int KQ>
__global__ void __launch_bounds__(kBlock) wgrad_kernel(WgradArgs A) {
    constexpr int K = 4 * KQ, KT = K / 16, LX = K + 4, LG = 64 + 4;
    __shared__ float Xl[kWSub * LX];
    __shared__ float Gl[kWSub * LG];
    int t, cnt;
    int64_t p0;
    if (!chunk_of(A.off, A.T, kWRows, blockIdx.x, t, p0, cnt)) return;
    const int og = blockIdx.y;
    const float* tab = A.tab.p[t];
    const int lane = threadIdx.x & 63, i = lane & 15, q = lane >> 4;
    const int w = threadIdx.x >> 6;
    f32x4 acc[KT];
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) acc[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
    float gsum = 0.f;
    for (int r0 = 0; r0 < cnt; r0 += kWSub) {
        for (int e = threadIdx.x; e < kWSub * KQ; e += kBlock) {
            const int r = e / KQ, v = e - r * KQ;
            float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
            if (r0 + r < cnt && tab)
                x = reinterpret_cast<const float4*>(tab + A.src[p0 + r0 + r] * K)[v];
            *reinterpret_cast<float4*>(Xl + r * LX + 4 * v) = x;
        }
        for (int e = threadIdx.x; e < kWSub * 16; e += kBlock) {
            const int r = e >> 4, v = e & 15;
            float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
            if (r0 + r < cnt)
                g = reinterpret_cast<const float4*>(A.gY + A.order[p0 + r0 + r] * A.O +
                                                    64 * og)[v];
            *reinterpret_cast<float4*>(Gl + r * LG + 4 * v) = g;
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < kWSub / 4; ++s) {
            const float a = Gl[(4 * s + q) * LG + 16 * w + i];
            gsum += a;
#pragma unroll
            for (int kt = 0; kt < KT; ++kt)
                acc[kt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, Xl[(4 * s + q) * LX + 16 * kt + i],
                                                               acc[kt], 0, 0, 0);
        }
        __syncthreads();
    }
    float* out = A.slab + (int64_t)blockIdx.x * A.O * (K + 1);
    // D layout: lane (i, q) holds D[4 q + r][i] -> output column 16 w + 4 q + r, k = 16 kt + i
#pragma unroll
    for (int kt = 0; kt < KT; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
            out[(int64_t)(64 * og + 16 * w + 4 * q + r) * K + 16 * kt + i] = acc[kt][r];
    gsum += __shfl_xor(gsum, 16, 64);
    gsum += __shfl_xor(gsum, 32, 64);
    if (q == 0) out[(int64_t)A.O * K + 64 * og + 16 * w + i] = gsum;
}

struct ReduceArgs {
    const int32_t* off;
    int T, O, K, G;
    int wg[MT];                // type -> weight group
    const float* slab;
    Tabs gW;                   // [g] [O, K]
    Tabs gb;                   // [g] [O] or NULL
};

// one thread per (group, element of [O*K | O]): the sum over the group's chunks in chunk order
__global__ void __launch_bounds__(kBlock) reduce_kernel(ReduceArgs A) {
    const int64_t per = (int64_t)A.O * (A.K + 1);
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= per * A.G) return;
    const int g = int(e / per);
    const int64_t x = e - g * per;
    float s = 0.f;
    int64_t c0 = 0;
    for (int u = 0; u < A.T; ++u) {
        const int64_t nc = (int64_t(A.off[u + 1]) - A.off[u] + kWRows - 1) / kWRows;
        if (A.wg[u] == g)
            for (int64_t c = c0; c < c0 + nc; ++c) s += A.slab[c * per + x];
        c0 += nc;
    }
    if (x < (int64_t)A.O * A.K) const_cast<float*>(A.gW.p[g])[x] = s;
    else if (A.gb.p[g]) const_cast<float*>(A.gb.p[g])[x - (int64_t)A.O * A.K] = s;
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace typed
}  // namespace regnn

using namespace regnn;
using namespace regnn::typed;

extern "C" {

int regnn_typed_gather(const int64_t* n_id, int64_t n, const int64_t* node_type,
                       const int64_t* local_idx, int32_t T, const float* const* tab, int32_t K,
                       float* out, hipStream_t stream) {
    if (n < 0 || T <= 0 || T > MT || K <= 0 || (K & 3) || !node_type || !local_idx || !tab ||
        (n > 0 && !out) || !aligned16(out))
        return REGNN_EINVAL;
    Tabs tb{};
    for (int t = 0; t < T; ++t) {
        if (!aligned16(tab[t])) return REGNN_EINVAL;
        tb.p[t] = tab[t];
    }
    if (n == 0) return REGNN_OK;
    hipLaunchKernelGGL(gather_kernel, dim3(grid_for(n * (K / 4), kBlock)), dim3(kBlock), 0, stream,
                       n_id, n, node_type, local_idx, T, tb, K / 4, out);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

int regnn_typed_scatter(const int64_t* n_id, int64_t n, const int64_t* node_type,
                        const int64_t* local_idx, int32_t T, float* const* gtab, int32_t K,
                        const float* g, hipStream_t stream) {
    if (n < 0 || T <= 0 || T > MT || K <= 0 || !node_type || !local_idx || !gtab ||
        (n > 0 && !g))
        return REGNN_EINVAL;
    Tabs tb{};
    for (int t = 0; t < T; ++t) tb.p[t] = gtab[t];
    if (n == 0) return REGNN_OK;
    hipLaunchKernelGGL(scatter_kernel, dim3(grid_for(n * K, kBlock)), dim3(kBlock), 0, stream,
                       n_id, n, node_type, local_idx, T, tb, K, g);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

int64_t regnn_typed_chunks(int64_t n, int32_t T, int32_t rows) {
    if (n < 0 || T <= 0 || rows <= 0) return -1;
    return (n + rows - 1) / rows + T;                 // upper bound over any split into T runs
}

int64_t regnn_typed_slab_floats(int64_t n, int32_t T, int32_t K, int32_t O) {
    const int64_t c = regnn_typed_chunks(n, T, kWRows);
    return c < 0 ? -1 : c * (int64_t)O * (K + 1);
}

int regnn_typed_linear_fwd(const int64_t* order, const int64_t* src, const int32_t* type_off,
                           int64_t n, int32_t T, const float* const* tab, const float* const* W,
                           const float* const* b, int32_t K, int32_t O, float* Y,
                           hipStream_t stream) {
    if (n < 0 || T <= 0 || T > MT || !tab || !W || !b || !type_off || O <= 0 ||
        (n > 0 && (!order || !src || !Y)) || !aligned16(Y))
        return REGNN_EINVAL;
    if ((K != 64 && K != 128 && K != 256) || (O & 15)) return REGNN_EUNSUPPORTED;
    FwdArgs A{order, src, type_off, T, O, {}, {}, {}, Y};
    for (int t = 0; t < T; ++t) {
        if (!W[t] || !aligned16(tab[t]) || !aligned16(W[t]) || !aligned16(b[t]))
            return REGNN_EINVAL;
        A.tab.p[t] = tab[t];
        A.W.p[t] = W[t];
        A.b.p[t] = b[t];
    }
    if (n == 0) return REGNN_OK;
#define TL_FWD(KQ, RB)                                                                          \
    {                                                                                           \
        const int64_t grid = regnn_typed_chunks(n, T, RB);                                      \
        const size_t lds = sizeof(float) * RB * (4 * KQ + 4);                                   \
        hipLaunchKernelGGL((fwd_kernel<KQ, RB>), dim3(grid), dim3(kBlock), lds, stream, A);     \
    }
    if (K == 64) TL_FWD(16, 128)
    else if (K == 128) TL_FWD(32, 128)
    else TL_FWD(64, 64)
#undef TL_FWD
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

int regnn_typed_linear_wgrad(const int64_t* order, const int64_t* src, const int32_t* type_off,
                             int64_t n, int32_t T, const float* const* tab, const int32_t* wgroup,
                             int32_t G, int32_t K, int32_t O, const float* gY, float* slab,
                             float* const* gW, float* const* gb, hipStream_t stream) {
    if (n < 0 || T <= 0 || T > MT || G <= 0 || G > T || !tab || !wgroup || !type_off ||
        !gW || !gb || !slab || (n > 0 && (!order || !src || !gY)) || !aligned16(gY))
        return REGNN_EINVAL;
    if ((K != 64 && K != 128 && K != 256) || (O & 63)) return REGNN_EUNSUPPORTED;
    WgradArgs A{order, src, type_off, T, O, {}, gY, slab};
    ReduceArgs R{type_off, T, O, K, G, {}, slab, {}, {}};
    for (int t = 0; t < T; ++t) {
        if (!aligned16(tab[t]) || wgroup[t] < 0 || wgroup[t] >= G) return REGNN_EINVAL;
        A.tab.p[t] = tab[t];
        R.wg[t] = wgroup[t];
    }
    for (int g = 0; g < G; ++g) {
        if (!gW[g]) return REGNN_EINVAL;
        R.gW.p[g] = gW[g];
        R.gb.p[g] = gb[g];
    }
    if (n > 0) {
        const dim3 grid(unsigned(regnn_typed_chunks(n, T, kWRows)), unsigned(O / 64));
        if (K == 64) hipLaunchKernelGGL(wgrad_kernel<16>, grid, dim3(kBlock), 0, stream, A);
        else if (K == 128) hipLaunchKernelGGL(wgrad_kernel<32>, grid, dim3(kBlock), 0, stream, A);
        else hipLaunchKernelGGL(wgrad_kernel<64>, grid, dim3(kBlock), 0, stream, A);
        REGNN_LAUNCH_CHECK();
    }
    // with n == 0 every group's chunk list is empty: the reduce writes zeros
    const int64_t total = (int64_t)G * O * (K + 1);
    hipLaunchKernelGGL(reduce_kernel, dim3(unsigned((total + kBlock - 1) / kBlock)), dim3(kBlock),
                       0, stream, R);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

}  // extern "C"
