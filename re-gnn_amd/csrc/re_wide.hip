// The wide NS model's per-layer epilogue (mag/regnn_ns.py:341-343 after mag/regnn_layers.py:
// 131-135 at hidden 128 .. 1024, the reference's default width 512): one launch forward, one
// backward, instead of torch's addcmul / bias / residual add / LayerNorm / relu / dropout kernels
// and their backward (~150 us per step at hidden 512, mag-10x, before).
//
//   a = rs[v] x[v] + bias (+ res[v])      (the mean's 1 / in-count, the conv bias, the residual)
//   y = dropout(relu(LayerNorm(a)))       (the dropout mask: the fused step's hash spec keyed on
//                                          the sampler's batch state, regnn_hip.h, so a batch
//                                          draws the same masks on either engine)
// backward: from gy, a and the row statistics: ga (d a), gx = rs ga, and per-block partials of
// sum ga (bias), sum gy' xhat (LN weight), sum gy' (LN bias) -> fixed-order reduce.
//
// Rows of H fp32: LPR = min(64, H / 4) lanes per row, VPL = H / (4 LPR) 16-byte vectors per lane
// (vector j of lane l = column block l + LPR j: coalesced), 256-thread blocks of 256 / LPR rows.
#include "re_nsm_common.h"

namespace regnn {
namespace wide {
using namespace regnn::nsm;

struct LnArgs {
    int64_t n; int H;
    const float* x; const float* rs; const float* bias; const float* res;
    const float* gamma; const float* beta;
    const int64_t* state; int layer; Drop drop;
    float* a; float* stats; float* y;                  // forward outputs
    const float* a_in; const float* stats_in;          // backward inputs
    const float* gy; float* gx; float* gres; float* slab;   // backward
    const int32_t* live;                               // rows >= *live skipped (may be null)
};

// the rows a launch covers: n, or the device count of live rows (a capacity-sized block whose
// rows past it nothing reads; a skipped row would only add exact zeros to the backward partials)
__device__ __forceinline__ int64_t ln_rows(const LnArgs& A) {
    return A.live ? min(A.n, int64_t(*A.live)) : A.n;
}

template <int LPR>
__device__ __forceinline__ float row_sum(float v) {
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ void drop4(uint32_t key, const Drop& d, int64_t row, int nvec, int vec,
                                      float (&m)[4]) {
    m[0] = m[1] = m[2] = m[3] = 1.f;
    if (!d.on) return;
    if (d.b8) drop_apply<4, 8>(key, d.thresh, d.scale, row, nvec, vec, m);
    else drop_apply<4, 16>(key, d.thresh, d.scale, row, nvec, vec, m);
}

template <int LPR, int VPL>
__global__ void __launch_bounds__(kBlock) ln_fwd_kernel(LnArgs A) {
    constexpr int RPB = kBlock / LPR;                  // rows per block
    const int l = threadIdx.x % LPR, g = threadIdx.x / LPR;
    const int H = A.H, nvec = H / 4;
    const uint32_t key = A.drop.on ? layer_key(A.state, A.layer) : 0u;
    float4 gw[VPL], gb[VPL], bs[VPL];
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
        const int c = 4 * (l + LPR * j);
        gw[j] = *reinterpret_cast<const float4*>(A.gamma + c);
        gb[j] = *reinterpret_cast<const float4*>(A.beta + c);
        bs[j] = A.bias ? *reinterpret_cast<const float4*>(A.bias + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const int64_t n = ln_rows(A);
    for (int64_t v = int64_t(blockIdx.x) * RPB + g; v < n; v += int64_t(gridDim.x) * RPB) {
        const float s = A.rs ? A.rs[v] : 1.f;
        float a[VPL][4];
        float sum = 0.f;
#pragma unroll
        for (int j = 0; j < VPL; ++j) {
            const int c = 4 * (l + LPR * j);
            const float4 x = *reinterpret_cast<const float4*>(A.x + v * H + c);
            float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
            if (A.res) r = *reinterpret_cast<const float4*>(A.res + v * H + c);
            a[j][0] = fmaf(s, x.x, bs[j].x) + r.x; a[j][1] = fmaf(s, x.y, bs[j].y) + r.y;
            a[j][2] = fmaf(s, x.z, bs[j].z) + r.z; a[j][3] = fmaf(s, x.w, bs[j].w) + r.w;
            *reinterpret_cast<float4*>(A.a + v * H + c) = make_float4(a[j][0], a[j][1], a[j][2], a[j][3]);
            sum += (a[j][0] + a[j][1]) + (a[j][2] + a[j][3]);
        }
        const float mean = row_sum<LPR>(sum) / float(H);
        float sq = 0.f;
#pragma unroll
        for (int j = 0; j < VPL; ++j)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float d = a[j][k] - mean;
                sq = fmaf(d, d, sq);
            }
        const float rstd = rsqrtf(row_sum<LPR>(sq) / float(H) + kLnEps);
        if (l == 0) reinterpret_cast<float2*>(A.stats)[v] = make_float2(mean, rstd);
#pragma unroll
        for (int j = 0; j < VPL; ++j) {
            const int vec = l + LPR * j;
            float m[4];
            drop4(key, A.drop, v, nvec, vec, m);
            const float gwf[4] = {gw[j].x, gw[j].y, gw[j].z, gw[j].w};
            const float gbf[4] = {gb[j].x, gb[j].y, gb[j].z, gb[j].w};
            float o[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) o[k] = fmaxf(fmaf((a[j][k] - mean) * rstd, gwf[k], gbf[k]), 0.f) * m[k];
            *reinterpret_cast<float4*>(A.y + v * H + 4 * vec) = make_float4(o[0], o[1], o[2], o[3]);
        }
    }
}

// backward; slab row per block: [H sum ga | H sum gy' xhat | H sum gy'] (reduced in block order)
template <int LPR, int VPL>
__global__ void __launch_bounds__(kBlock) ln_bwd_kernel(LnArgs A) {
    constexpr int RPB = kBlock / LPR;
    extern __shared__ float red[];                    // [RPB][3 H] row-group partials
    const int l = threadIdx.x % LPR, g = threadIdx.x / LPR;
    const int H = A.H, nvec = H / 4;
    const uint32_t key = A.drop.on ? layer_key(A.state, A.layer) : 0u;
    float4 gw[VPL], gb[VPL];
    float pa[VPL][4], pw[VPL][4], pb[VPL][4];
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
        const int c = 4 * (l + LPR * j);
        gw[j] = *reinterpret_cast<const float4*>(A.gamma + c);
        gb[j] = *reinterpret_cast<const float4*>(A.beta + c);
#pragma unroll
        for (int k = 0; k < 4; ++k) pa[j][k] = pw[j][k] = pb[j][k] = 0.f;
    }
    const int64_t n = ln_rows(A);
    for (int64_t v = int64_t(blockIdx.x) * RPB + g; v < n; v += int64_t(gridDim.x) * RPB) {
        const float2 st = reinterpret_cast<const float2*>(A.stats_in)[v];
        const float s = A.rs ? A.rs[v] : 1.f;
        float xh[VPL][4], gx[VPL][4];
        float p1 = 0.f, p2 = 0.f;
#pragma unroll
        for (int j = 0; j < VPL; ++j) {
            const int vec = l + LPR * j, c = 4 * vec;
            const float4 a4 = *reinterpret_cast<const float4*>(A.a_in + v * H + c);
            const float4 g4 = *reinterpret_cast<const float4*>(A.gy + v * H + c);
            float m[4];
            drop4(key, A.drop, v, nvec, vec, m);
            const float av[4] = {a4.x, a4.y, a4.z, a4.w}, gv[4] = {g4.x, g4.y, g4.z, g4.w};
            const float gwf[4] = {gw[j].x, gw[j].y, gw[j].z, gw[j].w};
            const float gbf[4] = {gb[j].x, gb[j].y, gb[j].z, gb[j].w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                xh[j][k] = (av[k] - st.x) * st.y;
                const float yv = fmaf(xh[j][k], gwf[k], gbf[k]);
                const float gyv = yv > 0.f ? gv[k] * m[k] : 0.f;          // relu, dropout
                pw[j][k] = fmaf(gyv, xh[j][k], pw[j][k]);
                pb[j][k] += gyv;
                gx[j][k] = gyv * gwf[k];
                p1 += gx[j][k];
                p2 = fmaf(gx[j][k], xh[j][k], p2);
            }
        }
        const float m1 = row_sum<LPR>(p1) / float(H), m2 = row_sum<LPR>(p2) / float(H);
#pragma unroll
        for (int j = 0; j < VPL; ++j) {
            const int c = 4 * (l + LPR * j);
            float ga[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                ga[k] = st.y * (gx[j][k] - m1 - xh[j][k] * m2);
                pa[j][k] += ga[k];
            }
            *reinterpret_cast<float4*>(A.gx + v * H + c) = make_float4(s * ga[0], s * ga[1], s * ga[2], s * ga[3]);
            if (A.gres) *reinterpret_cast<float4*>(A.gres + v * H + c) = make_float4(ga[0], ga[1], ga[2], ga[3]);
        }
    }
    // rows past the live count: zero gradients (the x6 GEMM that reads gx takes rows past its
    // m_live / k_live as zeros: its last k-step spans a few of them)
    for (int64_t v = n + int64_t(blockIdx.x) * RPB + g; v < A.n; v += int64_t(gridDim.x) * RPB) {
#pragma unroll
        for (int j = 0; j < VPL; ++j) {
            const int c = 4 * (l + LPR * j);
            *reinterpret_cast<float4*>(A.gx + v * H + c) = make_float4(0.f, 0.f, 0.f, 0.f);
            if (A.gres) *reinterpret_cast<float4*>(A.gres + v * H + c) = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    // the row groups' partials in LDS, summed in group order
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
        const int c = 4 * (l + LPR * j);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            red[g * 3 * H + c + k] = pa[j][k];
            red[g * 3 * H + H + c + k] = pw[j][k];
            red[g * 3 * H + 2 * H + c + k] = pb[j][k];
        }
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 3 * H; e += kBlock) {
        float t = 0.f;
        for (int r = 0; r < RPB; ++r) t += red[r * 3 * H + e];
        A.slab[int64_t(blockIdx.x) * 3 * H + e] = t;
    }
}


// Several relation tables at once (every conv layer's leaky_relu(alpha rw), mag/regnn_layers.py:
// 110-111), or their backward d rw = g alpha (alpha rw > 0 ? 1 : slope): one launch for all
constexpr int kTabsMax = 4;
struct TabsArgs {
    const float* rw[kTabsMax]; const float* g[kTabsMax]; float* out[kTabsMax];
    int start[kTabsMax + 1]; int count; float alpha, slope;
};

__global__ void __launch_bounds__(kBlock) rel_tabs_kernel(TabsArgs A) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= A.start[A.count]) return;
    int t = 0;
#pragma unroll
    for (int q = 1; q < kTabsMax; ++q) t += (q < A.count && i >= A.start[q]) ? 1 : 0;
    const int e = i - A.start[t];
    const float x = A.alpha * A.rw[t][e];
    A.out[t][e] = A.g[t] ? A.g[t][e] * (x > 0.f ? A.alpha : A.slope * A.alpha)
                         : (x > 0.f ? x : A.slope * x);
}

}  // namespace wide
}  // namespace regnn

using namespace regnn;
using namespace regnn::wide;

namespace {

int ln_launch(LnArgs& A, bool bwd, int blocks, hipStream_t stream) {
    const int H = A.H;
#define LN_CASE(LPR_, VPL_)                                                                    \
    if (H == 4 * LPR_ * VPL_ && (LPR_ == 64 || H == 4 * LPR_)) {                               \
        if (bwd) {                                                                             \
            const size_t lds = size_t(kBlock / LPR_) * 3 * H * sizeof(float);                  \
            static size_t done = 0;                                                            \
            if (!set_lds(reinterpret_cast<const void*>(&ln_bwd_kernel<LPR_, VPL_>), lds, &done)) \
                return REGNN_EUNSUPPORTED;                                                     \
            hipLaunchKernelGGL((ln_bwd_kernel<LPR_, VPL_>), dim3(blocks), dim3(kBlock), lds, stream, A); \
        } else {                                                                               \
            hipLaunchKernelGGL((ln_fwd_kernel<LPR_, VPL_>), dim3(blocks), dim3(kBlock), 0, stream, A); \
        }                                                                                      \
        REGNN_LAUNCH_CHECK();                                                                  \
        return REGNN_OK;                                                                       \
    }
    LN_CASE(16, 1) LN_CASE(32, 1) LN_CASE(64, 1) LN_CASE(64, 2) LN_CASE(64, 4)
#undef LN_CASE
    return REGNN_EUNSUPPORTED;
}

bool aligned(const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; }

}  // namespace

extern "C" {

int regnn_rel_tabs(const float* const* rw, const float* const* gtab, float* const* out,
                   const int32_t* n, int32_t count, float alpha, float slope, hipStream_t stream) {
    using namespace regnn::wide;
    if (!rw || !out || !n || count < 1 || count > kTabsMax) return REGNN_EINVAL;
    TabsArgs A{};
    A.count = count;
    A.alpha = alpha;
    A.slope = slope;
    A.start[0] = 0;
    for (int t = 0; t < count; ++t) {
        if (!rw[t] || !out[t] || n[t] < 0) return REGNN_EINVAL;
        A.rw[t] = rw[t];
        A.g[t] = gtab ? gtab[t] : nullptr;
        if (gtab && !gtab[t]) return REGNN_EINVAL;
        A.out[t] = out[t];
        A.start[t + 1] = A.start[t] + n[t];
    }
    const int total = A.start[count];
    if (total == 0) return REGNN_OK;
    hipLaunchKernelGGL(rel_tabs_kernel, dim3(unsigned((total + kBlock - 1) / kBlock)), dim3(kBlock),
                       0, stream, A);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

int regnn_wide_ln_fwd(int64_t n, int32_t H, const float* x, const float* rs, const float* bias,
                      const float* res, const float* gamma, const float* beta,
                      const int64_t* state, int32_t layer, float p_drop, float* a, float* stats,
                      float* y, const int32_t* live, hipStream_t stream) {
    if (n < 0 || !x || !gamma || !beta || !a || !stats || !y || !(p_drop >= 0.f && p_drop < 1.f) ||
        (p_drop > 0.f && !state))
        return REGNN_EINVAL;
    if (n == 0) return REGNN_OK;
    if (!aligned(x) || !aligned(a) || !aligned(y) || (res && !aligned(res)) || (bias && !aligned(bias)) ||
        !aligned(gamma) || !aligned(beta))
        return REGNN_EUNSUPPORTED;
    LnArgs A{};
    A.n = n; A.H = H; A.x = x; A.rs = rs; A.bias = bias; A.res = res; A.gamma = gamma; A.beta = beta;
    A.state = state; A.layer = layer; A.drop = make_drop(p_drop);
    A.a = a; A.stats = stats; A.y = y; A.live = live;
    const int rpb = kBlock / (H >= 256 ? 64 : H / 4);
    int64_t blocks = (n + rpb - 1) / rpb;
    if (blocks > kMaxGrid) blocks = kMaxGrid;
    return ln_launch(A, false, int(blocks), stream);
}

int64_t regnn_wide_ln_slab_rows(int64_t n, int32_t H) {
    const int rpb = kBlock / (H >= 256 ? 64 : H / 4);
    int64_t blocks = (n + rpb - 1) / rpb;
    if (blocks > 512) blocks = 512;
    return blocks < 1 ? 1 : blocks;
}

int regnn_wide_ln_bwd(int64_t n, int32_t H, const float* gy, const float* a, const float* stats,
                      const float* rs, const float* gamma, const float* beta,
                      const int64_t* state, int32_t layer, float p_drop, float* gx, float* gres,
                      float* slab, const int32_t* live, hipStream_t stream) {
    if (n < 0 || !gy || !a || !stats || !gamma || !beta || !gx || !slab ||
        !(p_drop >= 0.f && p_drop < 1.f) || (p_drop > 0.f && !state))
        return REGNN_EINVAL;
    if (!aligned(gy) || !aligned(a) || !aligned(gx) || (gres && !aligned(gres)) || !aligned(gamma) ||
        !aligned(beta))
        return REGNN_EUNSUPPORTED;
    LnArgs A{};
    A.n = n; A.H = H; A.gy = gy; A.a_in = a; A.stats_in = stats; A.rs = rs; A.gamma = gamma; A.beta = beta;
    A.state = state; A.layer = layer; A.drop = make_drop(p_drop);
    A.gx = gx; A.gres = gres; A.slab = slab; A.live = live;
    return ln_launch(A, true, int(regnn_wide_ln_slab_rows(n, H)), stream);
}

}  // extern "C"
