// Dense helpers of the training step on gfx950: the fused output head (MFMA logits + softmax
// cross-entropy), a row-wise softmax-xent for other widths, and a deterministic column sum of a
// tall row-major matrix (bias gradients of the per-node Linear heads, N up to ~2e7 rows). Each block owns a
// contiguous row range and keeps one partial per column per thread; block partials leave through
// a fixed-order slab (regnn_rel_reduce) — no atomics, rows read coalesced.
#include "regnn_common.h"

namespace regnn {

__global__ void __launch_bounds__(kBlock)
col_sum_kernel(const float* __restrict__ x, int64_t rows, int cols, int64_t rows_per_block,
               float* __restrict__ slab) {
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = min(rows, r0 + rows_per_block);
    for (int c = threadIdx.x; c < cols; c += kBlock) {
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
        int64_t r = r0;
        for (; r + 4 <= r1; r += 4) {
            s0 += x[r * cols + c];
            s1 += x[(r + 1) * cols + c];
            s2 += x[(r + 2) * cols + c];
            s3 += x[(r + 3) * cols + c];
        }
        for (; r < r1; ++r) s0 += x[r * cols + c];
        slab[(int64_t)blockIdx.x * cols + c] = (s0 + s1) + (s2 + s3);
    }
}

// One wave per row of a [rows, cols] logits matrix (row stride ld): log-sum-exp, the row's
// cross-entropy term and the scaled softmax gradient p = scale * (softmax(z) - onehot(label)),
// written once. Replaces torch's logsumexp / exp / sub / index_put chain, which splits >2^31-
// element tensors into 32-bit chunks and re-reads the logits ~6 times.
__global__ void __launch_bounds__(kBlock)
softmax_xent_kernel(const float* __restrict__ z, int64_t rows, int cols, int64_t ld,
                    const int64_t* __restrict__ labels, float scale, float* __restrict__ p,
                    float* __restrict__ loss_rows) {
    const int lane = threadIdx.x & 63;
    const int64_t wpb = kBlock / 64;
    for (int64_t r = (int64_t)blockIdx.x * wpb + threadIdx.x / 64; r < rows;
         r += (int64_t)gridDim.x * wpb) {
        const float* zr = z + r * ld;
        float m = -INFINITY;
        for (int c = lane; c < cols; c += 64) m = fmaxf(m, zr[c]);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
        float s = 0.f;
        for (int c = lane; c < cols; c += 64) s += __expf(zr[c] - m);
        s = group_sum<64>(s);
        const float lse = m + __logf(s);
        const int64_t y = labels[r];
        float* pr = p + r * (int64_t)cols;
        for (int c = lane; c < cols; c += 64) {
            const float v = __expf(zr[c] - lse);
            pr[c] = scale * (c == y ? v - 1.f : v);
        }
        if (lane == 0) loss_rows[r] = lse - zr[y];
    }
}

// ---------------------------------------------------------------------------------------------
// Fused output head: logits = h W^T + b over every row, and for the first n_loss rows the CE
// term lse - z[y] and the scaled softmax gradient p = scale * (softmax(z) - onehot(y)), from the
// accumulators (run_regnn.py:146-148 out_lin + log_softmax + nll over the train rows).
//
// fp32 MFMA v_mfma_f32_16x16x4_f32 (exact f32 fma chain, 64 FLOP/clk/SIMD) computing the tile
// TRANSPOSED, logits^T = W h^T: A = W (class on lane & 15), B = h^T (node on lane & 15). The
// C/D layout (col = lane & 15, row = 4 * (lane >> 4) + reg) then gives lane (q, c) node c and the
// 4 consecutive classes 16 t + 4 q + 0..3 of every 16-class tile t: one 16-byte store per tile
// and lane, and a node's softmax reductions are in-lane over 4 NT values plus 2 xor-shuffles
// across the quarters. One wave owns 16 nodes and all NT x 16 classes (NT accumulators of
// 4 regs: 88 for 349 classes; 2 waves per SIMD without spills); W^T lives in LDS for the whole
// persistent block (8 waves share one copy). The K = 64 reduction is split by lane quarter:
// quarter q supplies k = 16 q + s at k-step s, so each lane reads 16 contiguous floats of its row.
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4_u __attribute__((ext_vector_type(4), aligned(4)));   // dword-aligned rows
constexpr int kHeadK = 64;
constexpr int kHeadBlock = 512;
constexpr int kHeadMaxC = 24 * 16;
constexpr int kX6MaxNT = 23;      // bf16x6 head: three bf16 copies of W^T fit the 160 KiB LDS

// FL: diagnostic variant bits for A/B timing only (regnn_tune key 3): 1 = no prefetch,
// 2 = no logits stores, 4 = no loss-row epilogue. Shipped variant: FL = 0.
// AMAX: inference variant (mag/regnn_ns.py:367 out_lin + the caller's argmax): no logits
// stores and no loss rows; amax[node] = first class of maximal logit (torch.argmax ties).
// Tail of the fused head for one 16-node tile, shared by the fp32-MFMA and the bf16x6 kernels:
// argmax (AMAX), logits stores, and for loss rows log-sum-exp, CE term and the scaled softmax
// gradient. zy_part(y) returns this lane's share of the label logit z_y (its k-slice of h against
// W[y], plus the bias in one quarter); the four quarters are summed with 2 shuffles.
template <int NT, int FL, bool AMAX, typename ZY>
__device__ __forceinline__ void head_tail(f32x4 (&acc)[NT], int64_t node, int64_t tile, int q,
                                          int C, int64_t ld, int64_t rows, int64_t n_loss,
                                          float scale,
                                          const int64_t* __restrict__ labels,
                                          float* __restrict__ logits, float* __restrict__ p,
                                          float* __restrict__ loss_rows,
                                          int64_t* __restrict__ amax, ZY zy_part) {
    const bool valid = node < rows;
    if constexpr (AMAX) {
        float bv = -INFINITY;
        int bi = 0x7fffffff;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int cls = 16 * t + 4 * q + i;
                if (cls < C && (acc[t][i] > bv || (acc[t][i] == bv && cls < bi))) {
                    bv = acc[t][i];
                    bi = cls;
                }
            }
#pragma unroll
        for (int o = 16; o <= 32; o <<= 1) {
            const float ov = __shfl_xor(bv, o, 64);
            const int oi = __shfl_xor(bi, o, 64);
            if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
        }
        if (valid && q == 0) amax[node] = bi;
        return;
    }
    // ---- logits of every valid node: one 16-byte store per class tile (plain stores: the L2
    // merges the half-line pieces; non-temporal stores bypass that and ran 2x slower). With rows
    // padded to 16 classes the last tile is stored whole too (its pad classes hold 0) ----
    const bool padded = ld >= 16 * NT;
    if (!(FL & 2) && valid) {
        float* lr = logits + node * ld + 4 * q;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            if ((t + 1 < NT || padded || 16 * t + 16 <= C)) {
                *reinterpret_cast<f32x4_u*>(lr + 16 * t) = acc[t];
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (16 * t + 4 * q + i < C) lr[16 * t + i] = acc[t][i];
            }
        }
    }
    if ((FL & 4) || tile * 16 >= n_loss) return;        // wave-uniform
    // ---- loss rows: log-sum-exp, CE term, scaled softmax gradient ----
    float m = -INFINITY;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if ((t + 1 < NT || 16 * t + 16 <= C) || 16 * t + 4 * q + i < C) m = fmaxf(m, acc[t][i]);
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    // The label's logit z_y comes from its own 64-term dot (zy_part + 2 shuffles), not from
    // a per-class compare: 88 compares per lane would hold 88 VCC masks and spill the SGPR
    // file. acc becomes exp(z - m) in place (one exp per class, reused for the gradient); the
    // label's entry of p is fixed up afterwards.
    const int y = node < n_loss ? (int)labels[node] : 0;
    float zy = zy_part(y);
    zy += __shfl_xor(zy, 16, 64);
    zy += __shfl_xor(zy, 32, 64);
    float se = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int cls = 16 * t + 4 * q + i;
            const float e = ((t + 1 < NT || 16 * t + 16 <= C) || cls < C) ? __expf(acc[t][i] - m) : 0.f;
            acc[t][i] = e;
            se += e;
        }
    se += __shfl_xor(se, 16, 64);
    se += __shfl_xor(se, 32, 64);
    const float lse = m + __logf(se);
    if (node < n_loss) {
        float* pr = p + node * ld + 4 * q;
        const float r = scale / se;
        if (p) {                               // kernel-uniform (null: regnn_head_fwd_lse)
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const f32x4 v = acc[t] * r;
                if ((t + 1 < NT || padded || 16 * t + 16 <= C)) {
                    *reinterpret_cast<f32x4_u*>(pr + 16 * t) = v;
                } else {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if (16 * t + 4 * q + i < C) pr[16 * t + i] = v[i];
                }
            }
        }
        const int yq = y - 4 * q;              // the label's slot in this lane's tiles
        if (yq >= 0 && (yq & 15) < 4) {        // same lane, same address: ordered after
            loss_rows[node] = lse - zy;
            if (p) p[node * ld + y] = __expf(zy - m) * r - scale;
            else loss_rows[n_loss + node] = lse;   // regnn_head_fwd_lse: [2, n] loss | lse
        }
    }
}

template <int NT, int FL, bool AMAX = false, int BLK = kHeadBlock>
__global__ void __launch_bounds__(BLK)
head_fwd_kernel(const float* __restrict__ h, int64_t rows, const float* __restrict__ W,
                const float* __restrict__ bias, int C, int64_t ld, const int64_t* __restrict__ labels,
                int64_t n_loss, float scale, float* __restrict__ logits, float* __restrict__ p,
                float* __restrict__ loss_rows, int64_t* __restrict__ amax) {
    constexpr bool PIPE = !(FL & 1);
    constexpr int K = kHeadK, CP = NT * 16, LDW = CP + 1;   // +1: the four lane quarters read
    static_assert((K * LDW) % 4 == 0, "bias slot must be 16-byte aligned");
    extern __shared__ float Wl[];                           // rows 16 apart -> other banks
    for (int idx = threadIdx.x; idx < CP * K; idx += blockDim.x) {
        const int j = idx / K, k = idx - j * K;
        Wl[k * LDW + j] = j < C ? W[(int64_t)j * K + k] : 0.f;
    }
    float* bl = Wl + K * LDW;                               // bias after W^T (16-B aligned)
    for (int j = threadIdx.x; j < CP; j += blockDim.x) bl[j] = (bias && j < C) ? bias[j] : 0.f;
    __syncthreads();
    const int lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4;
    const int wpb = blockDim.x >> 6;
    const int64_t n_tiles = (rows + 15) / 16;
    const float* wq = Wl + (16 * q) * LDW + c;
    const f32x4* bl4 = reinterpret_cast<const f32x4*>(Wl + K * LDW) + q;   // bias[16 t + 4 q]
    auto load_a = [&](int64_t tile, float* a) {
        const int64_t arow = min(tile * 16 + c, rows - 1);
        const float4* hp = reinterpret_cast<const float4*>(h + arow * K + 16 * q);
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const float4 x = hp[v];
            a[4 * v] = x.x; a[4 * v + 1] = x.y; a[4 * v + 2] = x.z; a[4 * v + 3] = x.w;
        }
    };
    const int64_t tstride = (int64_t)gridDim.x * wpb;
    int64_t tile = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6);
    float a[16], an[16];
    if (PIPE && tile < n_tiles) load_a(tile, an);
    for (; tile < n_tiles; tile += tstride) {
        const int64_t node = tile * 16 + c;
        if (PIPE) {
#pragma unroll
            for (int k = 0; k < 16; ++k) a[k] = an[k];
            if (tile + tstride < n_tiles) load_a(tile + tstride, an);   // next tile in flight
        } else {
            load_a(tile, a);
        }
        f32x4 acc[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = bl4[4 * t];
        {
            float bw[NT], bn[NT];
#pragma unroll
            for (int t = 0; t < NT; ++t) bw[t] = wq[t * 16];
#pragma unroll
            for (int s = 0; s < 16; ++s) {
                if (s + 1 < 16) {
#pragma unroll
                    for (int t = 0; t < NT; ++t) bn[t] = wq[(s + 1) * LDW + t * 16];
                }
#pragma unroll
                for (int t = 0; t < NT; ++t)
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(bw[t], a[s], acc[t], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);  // step s+1's B reads overlap step s's MFMAs
#pragma unroll
                for (int t = 0; t < NT; ++t) bw[t] = bn[t];
            }
        }
        head_tail<NT, FL, AMAX>(acc, node, tile, q, C, ld, rows, n_loss, scale, labels, logits, p,
                                loss_rows, amax, [&](int y) {
            float z = 0.f;
#pragma unroll
            for (int s = 0; s < 16; ++s) z = fmaf(a[s], Wl[(16 * q + s) * LDW + y], z);
            return z + (q == 0 ? Wl[K * LDW + y] : 0.f);       // + bias[y] once over the quarters
        });
    }
}

// ---------------------------------------------------------------------------------------------
// The same head on bf16 MFMA with fp32 accuracy ("bf16x6"): every fp32 operand x is split into
// three bf16 parts x = x0 + x1 + x2 (round-to-nearest each, |x - x0 - x1 - x2| <= 2^-24 |x|), and
// the six products x_i y_j with i + j <= 2 are accumulated in fp32 by v_mfma_f32_16x16x32_bf16
// (exact bf16 x bf16 products): the dropped terms are below fp32 resolution. Six 16-cycle MFMAs
// per 16x16x32 step replace eight 32-cycle fp32 16x16x4 MFMAs: 2.7x the MFMA rate.
//
// Same transposed tile as head_fwd_kernel (A = W rows, class on lane & 15; B = h^T, node on
// lane & 15; C/D: lane (q, c) holds node c, classes 16 t + 4 q + 0..3), so the tail is shared.
// For 16x16x32 lane (q, c) supplies A[c][k = 8q + j] / B[k = 8q + j][c] (j = 0..7) of each
// 32-wide k chunk: features 32 kc + 8q .. +7 of its node. The three splits of W live in LDS as
// bf16 rows of 72 (64 + 8 pad: 144-byte rows put the 16 class rows of a b128 read on disjoint
// banks), bias after them: 3 * CP * 144 + 4 * CP bytes (<= 153.5 KiB for NT <= 23).
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
constexpr int kX6Row = 72;

__device__ __forceinline__ void split3(float x, uint16_t& a, uint16_t& b, uint16_t& c) {
    a = f2bf(x);
    const float r = x - bf2f(a);
    b = f2bf(r);
    c = f2bf(r - bf2f(b));
}

__device__ __forceinline__ bf16x8_t pack8(const uint16_t (&v)[8]) {
    uint4 u;
    u.x = uint32_t(v[0]) | (uint32_t(v[1]) << 16);
    u.y = uint32_t(v[2]) | (uint32_t(v[3]) << 16);
    u.z = uint32_t(v[4]) | (uint32_t(v[5]) << 16);
    u.w = uint32_t(v[6]) | (uint32_t(v[7]) << 16);
    return __builtin_bit_cast(bf16x8_t, u);
}

template <int NT, bool AMAX, typename TH = float>
__global__ void __launch_bounds__(kHeadBlock)
head_fwd_x6_kernel(const TH* __restrict__ h, int64_t rows, const float* __restrict__ W,
                   const float* __restrict__ bias, int C, int64_t ld,
                   const int64_t* __restrict__ labels,
                   int64_t n_loss, float scale, float* __restrict__ logits, float* __restrict__ p,
                   float* __restrict__ loss_rows, int64_t* __restrict__ amax) {
    constexpr int K = kHeadK, CP = NT * 16, LDB = kX6Row;
    extern __shared__ uint16_t Wb[];                       // [3][CP][LDB] bf16, then fp32 bias
    for (int idx = threadIdx.x; idx < CP * K; idx += blockDim.x) {
        const int j = idx / K, k = idx - j * K;
        uint16_t s0, s1, s2;
        split3(j < C ? W[(int64_t)j * K + k] : 0.f, s0, s1, s2);
        Wb[j * LDB + k] = s0;
        Wb[(CP + j) * LDB + k] = s1;
        Wb[(2 * CP + j) * LDB + k] = s2;
    }
    float* bl = reinterpret_cast<float*>(Wb + 3 * CP * LDB);    // 16-byte aligned (LDB % 8 == 0)
    for (int j = threadIdx.x; j < CP; j += blockDim.x) bl[j] = (bias && j < C) ? bias[j] : 0.f;
    __syncthreads();
    const int lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4;
    const int wpb = blockDim.x >> 6;
    const int64_t n_tiles = (rows + 15) / 16;
    const f32x4* bl4 = reinterpret_cast<const f32x4*>(bl) + q;  // bias[16 t + 4 q]
    // lane's A rows: class 16 t + c of split s, k offset 32 kc + 8 q
    const uint16_t* wa = Wb + c * LDB + 8 * q;
    const int64_t tstride = (int64_t)gridDim.x * wpb;
    // features 32 kc + 8 q + j of the lane's node; the next tile's rows are loaded one tile ahead
    auto load_a = [&](int64_t tile, float (&a)[2][8]) {
        const int64_t arow = min(tile * 16 + c, rows - 1);
#pragma unroll
        for (int kc = 0; kc < 2; ++kc) {
            if constexpr (sizeof(TH) == 2) {                 // bf16 rows: one 16-byte load
                Vec<bf16_t>::load(h + arow * K + 32 * kc + 8 * q, a[kc]);
            } else {
                const float4* hp = reinterpret_cast<const float4*>(h + arow * K + 32 * kc + 8 * q);
                const float4 x0 = hp[0], x1 = hp[1];
                a[kc][0] = x0.x; a[kc][1] = x0.y; a[kc][2] = x0.z; a[kc][3] = x0.w;
                a[kc][4] = x1.x; a[kc][5] = x1.y; a[kc][6] = x1.z; a[kc][7] = x1.w;
            }
        }
    };
    int64_t tile = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6);
    float a[2][8], an[2][8];
    if (tile < n_tiles) load_a(tile, an);
    for (; tile < n_tiles; tile += tstride) {
        const int64_t node = tile * 16 + c;
#pragma unroll
        for (int kc = 0; kc < 2; ++kc)
#pragma unroll
            for (int j = 0; j < 8; ++j) a[kc][j] = an[kc][j];
        if (tile + tstride < n_tiles) load_a(tile + tstride, an);
        // bf16 rows are exact in their first split: the three products with its zero
        // remainders are skipped (3 MFMAs per step instead of 6)
        constexpr bool EXH = sizeof(TH) == 2;
        bf16x8_t hb[2][3];
#pragma unroll
        for (int kc = 0; kc < 2; ++kc) {
            uint16_t s0[8], s1[8], s2[8];
            if constexpr (EXH) {
#pragma unroll
                for (int j = 0; j < 8; ++j) s0[j] = f2bf(a[kc][j]);
                hb[kc][0] = pack8(s0);
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) split3(a[kc][j], s0[j], s1[j], s2[j]);
                hb[kc][0] = pack8(s0);
                hb[kc][1] = pack8(s1);
                hb[kc][2] = pack8(s2);
            }
        }
        f32x4 acc[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            acc[t] = bl4[4 * t];
#pragma unroll
            for (int kc = 0; kc < 2; ++kc) {
                const uint16_t* w = wa + (16 * t) * LDB + 32 * kc;
                const bf16x8_t w0 = *reinterpret_cast<const bf16x8_t*>(w);
                const bf16x8_t w1 = *reinterpret_cast<const bf16x8_t*>(w + CP * LDB);
                const bf16x8_t w2 = *reinterpret_cast<const bf16x8_t*>(w + 2 * CP * LDB);
                // small products first
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2, hb[kc][0], acc[t], 0, 0, 0);
                if constexpr (!EXH) {
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, hb[kc][1], acc[t], 0, 0, 0);
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0, hb[kc][2], acc[t], 0, 0, 0);
                }
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, hb[kc][0], acc[t], 0, 0, 0);
                if constexpr (!EXH)
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0, hb[kc][1], acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0, hb[kc][0], acc[t], 0, 0, 0);
            }
        }
        head_tail<NT, 0, AMAX>(acc, node, tile, q, C, ld, rows, n_loss, scale, labels, logits, p,
                               loss_rows, amax, [&](int y) {
            const float* wy = W + (int64_t)y * K + 8 * q;         // fp32 W row (L2-resident)
            float z = 0.f;
#pragma unroll
            for (int kc = 0; kc < 2; ++kc)
#pragma unroll
                for (int j = 0; j < 8; ++j) z = fmaf(a[kc][j], wy[32 * kc + j], z);
            return z + (q == 0 ? bl[y] : 0.f);
        });
    }
}

template <int NT, bool AMAX, typename TH = float>
int launch_head_x6(const TH* h, int64_t rows, const float* W, const float* b, int C, int64_t ld,
                   const int64_t* labels, int64_t n_loss, float scale, float* logits, float* p,
                   float* loss_rows, hipStream_t stream, int64_t* amax = nullptr) {
    const size_t lds = (size_t)3 * NT * 16 * kX6Row * sizeof(uint16_t) + NT * 16 * sizeof(float);
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(&head_fwd_x6_kernel<NT, AMAX, TH>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return REGNN_ELAUNCH;
        attr = true;
    }
    const int64_t tiles = (rows + 15) / 16;
    int64_t grid = (tiles + kHeadBlock / 64 - 1) / (kHeadBlock / 64);
    const int cap = resident_blocks(reinterpret_cast<const void*>(&head_fwd_x6_kernel<NT, AMAX, TH>),
                                    lds, kHeadBlock);
    if (grid > cap) grid = cap;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL((head_fwd_x6_kernel<NT, AMAX, TH>), dim3((unsigned)grid), dim3(kHeadBlock), lds,
                       stream, h, rows, W, b, C, ld, labels, n_loss, scale, logits, p, loss_rows,
                       amax);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

template <int NT, int FL, bool AMAX = false, int BLK = kHeadBlock>
int launch_head_v(const float* h, int64_t rows, const float* W, const float* b, int C, int64_t ld,
                const int64_t* labels, int64_t n_loss, float scale, float* logits, float* p,
                float* loss_rows, hipStream_t stream, int64_t* amax = nullptr) {
    const size_t lds = ((size_t)kHeadK * (NT * 16 + 1) + NT * 16) * sizeof(float);
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(&head_fwd_kernel<NT, FL, AMAX, BLK>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return REGNN_ELAUNCH;
        attr = true;
    }
    const int64_t tiles = (rows + 15) / 16;
    int64_t grid = (tiles + BLK / 64 - 1) / (BLK / 64);
    const int cap = resident_blocks(
        reinterpret_cast<const void*>(&head_fwd_kernel<NT, FL, AMAX, BLK>), lds, BLK);
    if (grid > cap) grid = cap;
    if (grid < 1) grid = 1;
    auto kern = &head_fwd_kernel<NT, FL, AMAX, BLK>;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(BLK), lds, stream, h, rows, W, b,
                       C, ld, labels, n_loss, scale, logits, p, loss_rows, amax);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

template <int NT>
int launch_head(const float* h, int64_t rows, const float* W, const float* b, int C, int64_t ld,
                const int64_t* labels, int64_t n_loss, float scale, float* logits, float* p,
                float* loss_rows, hipStream_t stream) {
#define HEAD_V(fl) launch_head_v<NT, fl>(h, rows, W, b, C, ld, labels, n_loss, scale, logits, \
                                            p, loss_rows, stream)
    if (NT == 22 && g_tune_head != 0) {
        switch (g_tune_head) {
            case 1: return HEAD_V(1);
            case 2: return HEAD_V(2);
            case 4: return HEAD_V(4);
            case 16: return HEAD_V(0);                     // the fp32-MFMA kernel
            default: break;
        }
    }
    if constexpr (NT <= kX6MaxNT)
        return launch_head_x6<NT, false>(h, rows, W, b, C, ld, labels, n_loss, scale, logits, p,
                                         loss_rows, stream);
    return HEAD_V(0);
#undef HEAD_V
}

// ---------------------------------------------------------------------------------------------
// Output-head backward (run_regnn.py:146-148 through out_lin), from the scaled softmax gradient
// p [n, C] of regnn_head_fwd, each kernel reading p once:
//   head_gh_kernel    gh = gscale * p W          [n, 64]  (d loss / d h of the loss rows)
//   head_wgrad_kernel gW = p^T h, gb = colsum(p)  per-block partial slab rows (fixed-order reduce)
// fp32 MFMA v_mfma_f32_16x16x4_f32 (exact f32 products, fp32 accumulation).
//
// gh is computed transposed (gh^T = W^T p^T) with the same operand trick as head_fwd: k-step
// (t, i) takes class 16 t + 4 q + i from lane quarter q, so the B operand is component i of the
// lane's 16-byte load p[row][16 t + 4 q ..] and W^T comes from LDS; each lane ends with 4
// consecutive k of its row per 16-k tile (16-byte stores). 16 waves per block share one W^T copy
// (4 per SIMD); a wave streams its rows' p in batches of kGhBatch class tiles (16 accumulator
// registers, no register-resident p row), so the kernel runs near the p read rate. Rows
// [n, n_out) of gh (nodes without a loss term) are written as zeros in the same launch.
constexpr int kGhBlock = 1024;
constexpr int kGhBatch = 4;

template <int NT>
__global__ void __launch_bounds__(kGhBlock)
head_gh_kernel(const float* __restrict__ p, int64_t n, int C, int64_t ld, const float* __restrict__ W,
               const float* __restrict__ gscale, float* __restrict__ gh, int64_t n_out) {
    constexpr int K = kHeadK, CP = NT * 16, LDW = CP + 1;
    extern __shared__ float Wl[];
    for (int idx = threadIdx.x; idx < CP * K; idx += blockDim.x) {
        const int j = idx / K, k = idx - j * K;
        Wl[k * LDW + j] = j < C ? W[(int64_t)j * K + k] : 0.f;
    }
    __syncthreads();
    const float sc = gscale ? *gscale : 1.f;
    const int lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4;
    const int wpb = blockDim.x >> 6;
    const int64_t n_tiles = (n + 15) / 16;
    for (int64_t tile = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6); tile < n_tiles;
         tile += (int64_t)gridDim.x * wpb) {
        const int64_t row = tile * 16 + c;
        const bool valid = row < n;
        const float* pr = p + (valid ? row : n - 1) * ld + 4 * q;
        f32x4 acc[4];
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) acc[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
        for (int t0 = 0; t0 < NT; t0 += kGhBatch) {
            f32x4 pv[kGhBatch];
#pragma unroll
            for (int j = 0; j < kGhBatch; ++j) {
                const int t = t0 + j;
                if (t + 1 < NT || (t < NT && 16 * t + 16 <= C)) {
                    pv[j] = *reinterpret_cast<const f32x4_u*>(pr + 16 * t);
                } else {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        pv[j][i] = (t < NT && 16 * t + 4 * q + i < C) ? pr[16 * t + i] : 0.f;
                }
            }
#pragma unroll
            for (int j = 0; j < kGhBatch; ++j) {
                if (t0 + j >= NT) break;             // wave-uniform; LDS past CP is not W^T
                const float* wr = Wl + c * LDW + 16 * (t0 + j) + 4 * q;   // + (16 kt) LDW + i
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int kt = 0; kt < 4; ++kt)
                        acc[kt] = __builtin_amdgcn_mfma_f32_16x16x4f32(wr[16 * kt * LDW + i],
                                                                       pv[j][i], acc[kt], 0, 0, 0);
            }
        }
        if (valid) {
            float* gr = gh + row * K + 4 * q;
#pragma unroll
            for (int kt = 0; kt < 4; ++kt)
                *reinterpret_cast<f32x4*>(gr + 16 * kt) = acc[kt] * sc;
        }
    }
    // rows without a loss term: d loss / d h = 0
    const int64_t z0 = n * K / 4, z1 = n_out * K / 4;
    for (int64_t v = z0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < z1;
         v += (int64_t)gridDim.x * blockDim.x)
        reinterpret_cast<f32x4*>(gh)[v] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// gh with fp32 accuracy on bf16 MFMA (the bf16x6 split of head_fwd_x6_kernel): gh^T = W^T p^T
// over 32-class chunks, A = W^T rows (feature 16 kt + c; three bf16 splits in LDS, rows of
// CP32 + 8 bf16: 16-byte aligned, the 16 feature rows of a b128 read on disjoint banks), B = the
// lane's p row (classes 32 ch + 8 q .. +7, split on the fly). 4 waves per SIMD (~70 VGPRs).
// ZP ("p from z", regnn_head_bwd_z): the operand pointer holds the logits rows z instead of p,
// and p = scale (exp(z - lse) - [class == label]) is formed on the fly from the per-row lse of
// regnn_head_fwd_lse, so the forward never writes p (the n x C fp32 rows it would store and these
// kernels read back are the logits rows the caller gets anyway).
// four consecutive features of a row in fp32 / bf16 storage (16 / 8 bytes)
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
__device__ __forceinline__ void st4(bf16_t* p, f32x4 v) {
    *reinterpret_cast<uint2*>(p) = make_uint2(uint32_t(f2bf(v[0])) | (uint32_t(f2bf(v[1])) << 16),
                                              uint32_t(f2bf(v[2])) | (uint32_t(f2bf(v[3])) << 16));
}
__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ f32x4 ld4(const bf16_t* p) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    return f32x4{bf2f(u.x & 0xffffu), bf2f(u.x >> 16), bf2f(u.y & 0xffffu), bf2f(u.y >> 16)};
}

struct PSrc {
    const float* lse;
    const int64_t* labels;
    float scale;
};
constexpr float kLog2e = 1.4426950408889634f;

// p = scale (exp(z - lse) - [label]) with zl2 = lse log2(e): one FMA into v_exp_f32, one FMA out
__device__ __forceinline__ float zp_val(float z, float zl2, bool is_label, float scale) {
    const float e = __builtin_amdgcn_exp2f(fmaf(z, kLog2e, -zl2));
    return fmaf(e, scale, is_label ? -scale : 0.f);
}

// TO: storage type of gh, hx and nx_out (float, or bf16_t for a bf16 feature pipeline: gh and
// nx_out are rounded as the stored-gradient path would round them, g first, then post * g)
template <int NT, bool ZP = false, typename TO = float>
__global__ void __launch_bounds__(kGhBlock)
head_gh_x6_kernel(const float* __restrict__ p, int64_t n, int C, int64_t ld,
                  const float* __restrict__ W,
                  const float* __restrict__ gscale, TO* __restrict__ gh, int64_t n_out,
                  const float* __restrict__ nx_scale, const TO* __restrict__ hx,
                  TO* __restrict__ nx_out, float* __restrict__ nx_dot, PSrc ps) {
    constexpr int K = kHeadK, NCH = (NT + 1) / 2, CP32 = 32 * NCH, LDR = CP32 + 8;
    extern __shared__ uint16_t Wt[];                       // [3][K][LDR] bf16
    for (int idx = threadIdx.x; idx < CP32 * K; idx += blockDim.x) {
        const int j = idx / K, k = idx - j * K;             // class j, feature k (W read rowwise)
        uint16_t s0, s1, s2;
        split3(j < C ? W[(int64_t)j * K + k] : 0.f, s0, s1, s2);
        Wt[k * LDR + j] = s0;
        Wt[(K + k) * LDR + j] = s1;
        Wt[(2 * K + k) * LDR + j] = s2;
    }
    __syncthreads();
    const float sc = gscale ? *gscale : 1.f;
    const int lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4;
    const int wpb = blockDim.x >> 6;
    const int64_t n_tiles = (n + 15) / 16;
    const uint16_t* wa = Wt + c * LDR + 8 * q;             // + (s K + 16 kt) LDR + 32 ch
    float zl = 0.f;                                        // ZP: the lane row's lse, label
    int zy = -1;
    auto load_p = [&](const float* pr, int ch, float (&v)[8]) {
        const int cls0 = 32 * ch + 8 * q;
        if (cls0 + 8 <= C) {
            const f32x4 x0 = *reinterpret_cast<const f32x4_u*>(pr + cls0);
            const f32x4 x1 = *reinterpret_cast<const f32x4_u*>(pr + cls0 + 4);
#pragma unroll
            for (int i = 0; i < 4; ++i) { v[i] = x0[i]; v[4 + i] = x1[i]; }
            if constexpr (ZP) {
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] = zp_val(v[i], zl, cls0 + i == zy, ps.scale);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                float x = cls0 + i < C ? pr[cls0 + i] : 0.f;
                if constexpr (ZP) x = cls0 + i < C ? zp_val(x, zl, cls0 + i == zy, ps.scale) : 0.f;
                v[i] = x;
            }
        }
    };
    for (int64_t tile = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6); tile < n_tiles;
         tile += (int64_t)gridDim.x * wpb) {
        const int64_t row = tile * 16 + c;
        const bool valid = row < n;
        const float* pr = p + (valid ? row : n - 1) * ld;
        if constexpr (ZP) {
            zl = ps.lse[valid ? row : n - 1] * kLog2e;
            zy = (int)ps.labels[valid ? row : n - 1];
        }
        f32x4 acc[4];
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) acc[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
        float v[8], vn[8];
        load_p(pr, 0, vn);
#pragma unroll 1
        for (int ch = 0; ch < NCH; ++ch) {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = vn[i];
            if (ch + 1 < NCH) load_p(pr, ch + 1, vn);        // next chunk in flight
            uint16_t s0[8], s1[8], s2[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) split3(v[i], s0[i], s1[i], s2[i]);
            const bf16x8_t b0 = pack8(s0), b1 = pack8(s1), b2 = pack8(s2);
#pragma unroll
            for (int kt = 0; kt < 4; ++kt) {
                const uint16_t* w = wa + (16 * kt) * LDR + 32 * ch;
                const bf16x8_t w0 = *reinterpret_cast<const bf16x8_t*>(w);
                const bf16x8_t w1 = *reinterpret_cast<const bf16x8_t*>(w + K * LDR);
                const bf16x8_t w2 = *reinterpret_cast<const bf16x8_t*>(w + 2 * K * LDR);
                acc[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2, b0, acc[kt], 0, 0, 0);
                acc[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, b1, acc[kt], 0, 0, 0);
                acc[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0, b2, acc[kt], 0, 0, 0);
                acc[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, b0, acc[kt], 0, 0, 0);
                acc[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0, b1, acc[kt], 0, 0, 0);
                acc[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0, b0, acc[kt], 0, 0, 0);
            }
        }
        float d = 0.f, ns = 1.f;
        if (valid) {
            TO* gr = gh + row * K + 4 * q;
            f32x4 g[4];
#pragma unroll
            for (int kt = 0; kt < 4; ++kt) {
                g[kt] = acc[kt] * sc;
                st4(gr + 16 * kt, g[kt]);
                if constexpr (sizeof(TO) == 2)
#pragma unroll
                    for (int i = 0; i < 4; ++i) g[kt][i] = round_to<TO>(g[kt][i]);
            }
            if (nx_scale) {                                  // kernel-uniform
                // the consumer-side row pass of h's producer (regnn_head_gh_next)
                ns = nx_scale[row];
                const TO* hr = hx + row * K + 4 * q;
                TO* orow = nx_out + row * K + 4 * q;
#pragma unroll
                for (int kt = 0; kt < 4; ++kt) {
                    const f32x4 hv = ld4(hr + 16 * kt);
#pragma unroll
                    for (int i = 0; i < 4; ++i) d = fmaf(g[kt][i], hv[i], d);
                    st4(orow + 16 * kt, g[kt] * ns);
                }
            }
        }
        if (nx_scale) {                                      // a row's 64 features: lanes c + 16 q
            d += __shfl_xor(d, 16);
            d += __shfl_xor(d, 32);
            if (valid && q == 0) nx_dot[row] = d / ns;
        }
    }
    const int64_t z0 = n * K / 4, z1 = n_out * K / 4;      // rows without a loss term: zero
    for (int64_t v = z0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < z1;
         v += (int64_t)gridDim.x * blockDim.x) {
        st4(gh + 4 * v, f32x4{0.f, 0.f, 0.f, 0.f});     // nx_out rows >= n: not written
    }
    if (nx_scale)
        for (int64_t r = n + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n_out;
             r += (int64_t)gridDim.x * blockDim.x)
            nx_dot[r] = 0.f;
}

// gW^T partial of this block's row range: wave w owns class tiles w, w + 8, w + 16; per 4-row
// k-step lane (q, c) feeds A = p[row0 + q][16 t + c] and B = h[row0 + q][16 j + c], so D[cls][k]
// accumulates over the rows; gb rides along in VALU adds of the same A values. 8 k-steps
// (32 rows) of loads are issued before their MFMAs.
template <int NT>
__global__ void __launch_bounds__(kHeadBlock)
head_wgrad_kernel(const float* __restrict__ p, int64_t n, int C, int64_t ld, const float* __restrict__ h,
                  int64_t rows_per_block, float* __restrict__ slab) {
    constexpr int K = kHeadK, CP = NT * 16, MT = (NT + 7) / 8, KS = 8;
    const int lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4, w = threadIdx.x >> 6;
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = min(n, r0 + rows_per_block);
    f32x4 acc[MT][4];
    float gb[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
        gb[m] = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[m][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    for (int64_t row0 = r0; row0 < r1; row0 += 4 * KS) {
        float a[KS][MT], b[KS][4];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int64_t rr = row0 + 4 * s + q;
            const bool ok = rr < r1;
            const int64_t rc = ok ? rr : r0;
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                const int cls = 16 * (w + 8 * m) + c;
                const bool in = ok && (w + 8 * m) < NT && cls < C;
                const float v = p[rc * ld + (cls < C ? cls : 0)];
                a[s][m] = in ? v : 0.f;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float v = h[rc * K + 16 * j + c];
                b[s][j] = ok ? v : 0.f;
            }
        }
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                gb[m] += a[s][m];
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s][m], b[s][j], acc[m][j],
                                                                     0, 0, 0);
            }
    }
    float* out = slab + (int64_t)blockIdx.x * (CP * K + CP);
#pragma unroll
    for (int m = 0; m < MT; ++m) {
        const int t = w + 8 * m;
        if (t >= NT) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) out[(16 * t + 4 * q + r) * K + 16 * j + c] = acc[m][j][r];
        float g = gb[m];
        g += __shfl_xor(g, 16, 64);
        g += __shfl_xor(g, 32, 64);
        if (q == 0) out[CP * K + 16 * t + c] = g;
    }
}

// gW = p^T h / gb = colsum(p) partials with fp32 accuracy on bf16 MFMA (bf16x6 split, as
// head_fwd_x6_kernel): D[cls][feature] tiles over this block's row range, one 16x16x32 k-step per
// 32 rows: lane (q, c) supplies rows r0 + 8 q + j (j = 0..7) of A = p[., 16 t + c] and
// B = h[., 64 fb + 16 kt + c], loaded 4 (fp32) / 2 (bf16) bytes per lane (16 lanes read one
// contiguous row segment) and split into three bf16 fragments in registers. Work units
// (class tile t, 64-feature block fb) go to waves round-robin (u = w + 8 m): the output head
// (C = 349, K = 64) gives a wave class tiles w, w + 8, w + 16; an input projection's d weight
// (C = 64 outputs, K = 128 inputs) one (tile, block) pair per wave.
template <typename TP, typename TH, int NT, int KH, bool ZP = false>
__global__ void __launch_bounds__(kHeadBlock)
wgrad_x6_kernel(const TP* __restrict__ p, int64_t n, int C, int64_t ld,
                const TH* __restrict__ h, int64_t rows_per_block, float* __restrict__ slab,
                PSrc ps) {
    constexpr int KB = KH / 64, NU = NT * KB, MU = (NU + 7) / 8, CP = NT * 16;
    constexpr bool EXACT = sizeof(TP) == 2 && sizeof(TH) == 2;   // bf16 x bf16: one product
    constexpr bool EXACT_H = sizeof(TH) == 2;                    // bf16 h: three products
    const int lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4, w = threadIdx.x >> 6;
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = min(n, r0 + rows_per_block);
    auto ld_p = [&](int64_t i) -> float {
        if constexpr (sizeof(TP) == 4) return p[i]; else return bf2f(p[i]);
    };
    auto ld_h = [&](int64_t i) -> float {
        if constexpr (sizeof(TH) == 4) return h[i]; else return bf2f(h[i]);
    };
    f32x4 acc[MU][4];
    float gb[MU];
#pragma unroll
    for (int m = 0; m < MU; ++m) {
        gb[m] = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[m][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if constexpr (KB == 1) {
        // The h operand is the same for every wave of the block: per 32-row k-step, lanes
        // 0..255 of the block split one (kt, q, c) column piece each (8 rows) and publish its
        // three bf16 fragments in LDS (double-buffered, one barrier per step); every wave then
        // reads its B fragments with ds_read_b128 instead of splitting 32 values per lane.
        __shared__ bf16x8_t hs[2][3][4][4][16];             // [buf][split][kt][q][c]: 24 KiB
        const int gid = threadIdx.x;
        const int wkt = (gid >> 6) & 3, wq = (gid >> 4) & 3, wc = gid & 15;
        int buf = 0;
        for (int64_t row0 = r0; row0 < r1; row0 += 32, buf ^= 1) {
            if (gid < 256) {
                uint16_t s0[8], s1[8], s2[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int64_t rr = row0 + 8 * wq + j;
                    const float hv = ld_h((rr < r1 ? rr : r0) * KH + 16 * wkt + wc);
                    split3(rr < r1 ? hv : 0.f, s0[j], s1[j], s2[j]);
                }
                hs[buf][0][wkt][wq][wc] = pack8(s0);
                hs[buf][1][wkt][wq][wc] = pack8(s1);
                hs[buf][2][wkt][wq][wc] = pack8(s2);
            }
            float a[MU][8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int64_t rr = row0 + 8 * q + j;
                const bool ok = rr < r1;
                const int64_t rc = ok ? rr : r0;
                float zl = 0.f;
                int zy = -1;
                if constexpr (ZP) {
                    zl = ps.lse[rc] * kLog2e;
                    zy = (int)ps.labels[rc];
                }
#pragma unroll
                for (int m = 0; m < MU; ++m) {
                    const int u = w + 8 * m, t = u % NT;
                    const int cls = 16 * t + c;
                    const bool in = ok && u < NU && cls < C;
                    float v = ld_p(rc * ld + (cls < C ? cls : 0));
                    if constexpr (ZP) v = zp_val(v, zl, cls == zy, ps.scale);
                    a[m][j] = in ? v : 0.f;
                }
            }
            __syncthreads();                                 // block-uniform: r0, r1, row0
            bf16x8_t bf[4][3];
#pragma unroll
            for (int kt = 0; kt < 4; ++kt)
#pragma unroll
                for (int sp = 0; sp < 3; ++sp) bf[kt][sp] = hs[buf][sp][kt][q][c];
#pragma unroll
            for (int m = 0; m < MU; ++m) {
                if (w + 8 * m >= NU) continue;               // wave-uniform
                uint16_t s0[8], s1[8], s2[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    gb[m] += a[m][j];
                    split3(a[m][j], s0[j], s1[j], s2[j]);
                }
                const bf16x8_t a0 = pack8(s0), a1 = pack8(s1), a2 = pack8(s2);
#pragma unroll
                for (int kt = 0; kt < 4; ++kt) {
                    if constexpr (!EXACT) {
                        acc[m][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2, bf[kt][0], acc[m][kt], 0, 0, 0);
                        if constexpr (!EXACT_H) {
                            acc[m][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bf[kt][1], acc[m][kt], 0, 0, 0);
                            acc[m][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bf[kt][2], acc[m][kt], 0, 0, 0);
                        }
                        acc[m][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bf[kt][0], acc[m][kt], 0, 0, 0);
                        if constexpr (!EXACT_H)
                            acc[m][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bf[kt][1], acc[m][kt], 0, 0, 0);
                    }
                    acc[m][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bf[kt][0], acc[m][kt], 0, 0, 0);
                }
            }
        }
    } else {
        for (int64_t row0 = r0; row0 < r1; row0 += 32) {
            float a[MU][8], b[MU][4][8];
    #pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int64_t rr = row0 + 8 * q + j;
                const bool ok = rr < r1;
                const int64_t rc = ok ? rr : r0;
                float zl = 0.f;
                int zy = -1;
                if constexpr (ZP) {
                    zl = ps.lse[rc] * kLog2e;
                    zy = (int)ps.labels[rc];
                }
    #pragma unroll
                for (int m = 0; m < MU; ++m) {
                    const int u = w + 8 * m, t = u % NT, fb = u / NT;
                    const int cls = 16 * t + c;
                    const bool in = ok && u < NU && cls < C;
                    float v = ld_p(rc * ld + (cls < C ? cls : 0));
                    if constexpr (ZP) v = zp_val(v, zl, cls == zy, ps.scale);
                    a[m][j] = in ? v : 0.f;
                    if (KB > 1 || m == 0) {
    #pragma unroll
                        for (int kt = 0; kt < 4; ++kt) {
                            const float hv = ld_h(rc * KH + 64 * (KB > 1 ? fb : 0) + 16 * kt + c);
                            b[m][kt][j] = ok ? hv : 0.f;
                        }
                    }
                }
            }
    #pragma unroll
            for (int m = 0; m < MU; ++m) {
                if (w + 8 * m >= NU) continue;                   // wave-uniform
                const int mb = KB > 1 ? m : 0;                   // KB == 1: units share h
                bf16x8_t bf[4][3];
    #pragma unroll
                for (int kt = 0; kt < 4; ++kt) {
                    uint16_t s0[8], s1[8], s2[8];
                    if constexpr (EXACT_H) {             // bf16 h: exact in its first split
    #pragma unroll
                        for (int j = 0; j < 8; ++j) s0[j] = f2bf(b[mb][kt][j]);
                        bf[kt][0] = pack8(s0);
                    } else {
    #pragma unroll
                        for (int j = 0; j < 8; ++j) split3(b[mb][kt][j], s0[j], s1[j], s2[j]);
                        bf[kt][0] = pack8(s0); bf[kt][1] = pack8(s1); bf[kt][2] = pack8(s2);
                    }
                }
                uint16_t s0[8], s1[8], s2[8];
    #pragma unroll
                for (int j = 0; j < 8; ++j) {
                    gb[m] += a[m][j];
                    split3(a[m][j], s0[j], s1[j], s2[j]);
                }
                const bf16x8_t a0 = pack8(s0), a1 = pack8(s1), a2 = pack8(s2);
    #pragma unroll
                for (int kt = 0; kt < 4; ++kt) {
                    if constexpr (!EXACT) {
                        acc[m][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2, bf[kt][0], acc[m][kt], 0, 0, 0);
                        if constexpr (!EXACT_H) {
                            acc[m][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bf[kt][1], acc[m][kt], 0, 0, 0);
                            acc[m][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bf[kt][2], acc[m][kt], 0, 0, 0);
                        }
                        acc[m][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bf[kt][0], acc[m][kt], 0, 0, 0);
                        if constexpr (!EXACT_H)
                            acc[m][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bf[kt][1], acc[m][kt], 0, 0, 0);
                    }
                    acc[m][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bf[kt][0], acc[m][kt], 0, 0, 0);
                }
            }
        }
    }
    float* out = slab + (int64_t)blockIdx.x * (CP * KH + CP);
#pragma unroll
    for (int m = 0; m < MU; ++m) {
        const int u = w + 8 * m, t = u % NT, fb = u / NT;
        if (u >= NU) continue;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                out[(16 * t + 4 * q + r) * KH + 64 * fb + 16 * kt + c] = acc[m][kt][r];
        float g = gb[m];
        g += __shfl_xor(g, 16, 64);
        g += __shfl_xor(g, 32, 64);
        if (fb == 0 && q == 0) out[CP * KH + 16 * t + c] = g;
    }
}

// slab rows for n rows of p: grid blocks of >= 256 rows, one slab row each (<= slab_rows)
template <typename TP, typename TH, int NT, int KH, bool ZP = false>
int launch_wgrad_x6(const TP* p, int64_t n, int C, int64_t ld, const TH* h, float* slab,
                    int slab_rows, hipStream_t stream, PSrc ps = PSrc{nullptr, nullptr, 0.f}) {
    int64_t grid = slab_rows;
    const int64_t rpb_min = 256;
    if (grid * rpb_min > n) grid = (n + rpb_min - 1) / rpb_min;
    if (grid < 1) grid = 1;
    int64_t rpb = (n + grid - 1) / grid;
    rpb = (rpb + 31) / 32 * 32;
    grid = (n + rpb - 1) / rpb;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL((wgrad_x6_kernel<TP, TH, NT, KH, ZP>), dim3((unsigned)grid),
                       dim3(kHeadBlock), 0, stream, p, n, C, ld, h, rpb, slab, ps);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

// gh of regnn_head_bwd_z (p re-formed from the logits rows), storage type TO for gh / hx / nx_out
template <int NT, typename TO>
int launch_gh_z(const float* z, int64_t n, int C, int64_t ld, const float* W,
                const float* gscale, void* gh, int64_t n_out, const float* nx_scale,
                const void* hx, void* nx_out, float* nx_dot, PSrc ps, hipStream_t stream) {
    constexpr int K = kHeadK;
    constexpr size_t lds = (size_t)3 * K * (32 * ((NT + 1) / 2) + 8) * sizeof(uint16_t);
    auto kern = &head_gh_x6_kernel<NT, true, TO>;
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return REGNN_ELAUNCH;
        attr = true;
    }
    const int64_t tiles = (n + 15) / 16;
    int64_t grid = (tiles + kGhBlock / 64 - 1) / (kGhBlock / 64);
    const int cap = resident_blocks(reinterpret_cast<const void*>(kern), lds, kGhBlock);
    if (grid > cap) grid = cap;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kGhBlock), lds, stream, z, n, C, ld, W,
                       gscale, static_cast<TO*>(gh), n_out, nx_scale,
                       static_cast<const TO*>(hx), static_cast<TO*>(nx_out), nx_dot, ps);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

template <int NT>
int launch_head_bwd(const float* p, int64_t n, int C, int64_t ld, const float* W, const float* h,
                    const float* gscale, float* gh, int64_t n_out, float* slab, int slab_rows,
                    hipStream_t stream, const float* nx_scale = nullptr,
                    const float* hx = nullptr, float* nx_out = nullptr,
                    float* nx_dot = nullptr, PSrc ps = PSrc{nullptr, nullptr, 0.f},
                    int dtype = 0) {
    constexpr int K = kHeadK;
    if (nx_scale && !gh) return REGNN_EINVAL;
    if (ps.lse) {                                  // p from the logits rows: bf16x6 kernels only
        if (gh) {
            const int rc = dtype == 1
                ? launch_gh_z<NT, bf16_t>(p, n, C, ld, W, gscale, gh, n_out, nx_scale, hx, nx_out,
                                          nx_dot, ps, stream)
                : launch_gh_z<NT, float>(p, n, C, ld, W, gscale, gh, n_out, nx_scale, hx, nx_out,
                                         nx_dot, ps, stream);
            if (rc != REGNN_OK) return rc;
        }
        if (slab && dtype == 1)                    // h rows in bf16 (exact in their first split)
            return launch_wgrad_x6<float, bf16_t, NT, kHeadK, true>(
                p, n, C, ld, reinterpret_cast<const bf16_t*>(h), slab, slab_rows, stream, ps);
        if (slab)
            return launch_wgrad_x6<float, float, NT, kHeadK, true>(p, n, C, ld, h, slab,
                                                                  slab_rows, stream, ps);
        return REGNN_OK;
    }
    if (gh && (g_tune_head != 16 || nx_scale)) {   // bf16x6 gh (default)
        constexpr size_t lds = (size_t)3 * K * (32 * ((NT + 1) / 2) + 8) * sizeof(uint16_t);
        static bool attr6 = false;
        if (!attr6) {
            if (hipFuncSetAttribute(reinterpret_cast<const void*>(&head_gh_x6_kernel<NT>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds) != hipSuccess)
                return REGNN_ELAUNCH;
            attr6 = true;
        }
        const int64_t tiles = (n + 15) / 16;
        int64_t grid = (tiles + kGhBlock / 64 - 1) / (kGhBlock / 64);
        const int cap = resident_blocks(reinterpret_cast<const void*>(&head_gh_x6_kernel<NT>),
                                        lds, kGhBlock);
        if (grid > cap) grid = cap;
        if (grid < 1) grid = 1;
        hipLaunchKernelGGL((head_gh_x6_kernel<NT>), dim3((unsigned)grid), dim3(kGhBlock), lds,
                           stream, p, n, C, ld, W, gscale, gh, n_out, nx_scale, hx, nx_out,
                           nx_dot, ps);
        REGNN_LAUNCH_CHECK();
    } else if (gh) {
        const size_t lds = (size_t)K * (NT * 16 + 1) * sizeof(float);
        static bool attr = false;
        if (!attr) {
            if (hipFuncSetAttribute(reinterpret_cast<const void*>(&head_gh_kernel<NT>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds) != hipSuccess)
                return REGNN_ELAUNCH;
            attr = true;
        }
        const int64_t tiles = (n + 15) / 16;
        int64_t grid = (tiles + kGhBlock / 64 - 1) / (kGhBlock / 64);
        const int cap = resident_blocks(reinterpret_cast<const void*>(&head_gh_kernel<NT>), lds,
                                        kGhBlock);
        if (grid > cap) grid = cap;
        if (grid < 1) grid = 1;
        hipLaunchKernelGGL((head_gh_kernel<NT>), dim3((unsigned)grid), dim3(kGhBlock), lds,
                           stream, p, n, C, ld, W, gscale, gh, n_out);
        REGNN_LAUNCH_CHECK();
    }
    if (slab) {
        int64_t grid = slab_rows;
        const int64_t rpb_min = 256;
        if (grid * rpb_min > n) grid = (n + rpb_min - 1) / rpb_min;
        if (grid < 1) grid = 1;
        int64_t rpb = (n + grid - 1) / grid;
        rpb = (rpb + 31) / 32 * 32;
        grid = (n + rpb - 1) / rpb;
        if (grid < 1) grid = 1;
        if (g_tune_head != 16)
            return launch_wgrad_x6<float, float, NT, kHeadK>(p, n, C, ld, h, slab, slab_rows,
                                                            stream);
        else
            hipLaunchKernelGGL((head_wgrad_kernel<NT>), dim3((unsigned)grid), dim3(kHeadBlock), 0,
                               stream, p, n, C, ld, h, rpb, slab);
        REGNN_LAUNCH_CHECK();
    }
    return REGNN_OK;
}

// ---------------------------------------------------------------------------------------------
// Per-type input projection fused with the first aggregation's pre-scale (model/REGCN.py:31-35
// fc_list + layer/REGraphConv.py:56,73-76): for rows r of one node type
//   h[row0 + r]  = x[r] W^T + b                        (the layer input, kept for the backward)
//   xs[row0 + r] = scale[row0 + r] * drop(h[row0 + r])  (what the aggregation gathers)
// with drop the regnn_spmm_fwd_dropout mask of (global row, 16-byte vector), applied to h as
// stored (rounded to the storage type), so xs equals regnn_row_scale(h). This removes the
// separate row pass over h (2 N F s bytes) and replaces the hipBLASLt GEMM.
// fp32-accurate bf16 MFMA (bf16x6 split as head_fwd_x6_kernel; bf16 inputs are exact in their
// first split, so 3 products suffice), transposed tile: A = W rows (feature 16 kt + c), B = x^T
// (node on lane & 15), lane (q, c) ends with features 16 kt + 4 q .. +3 of node c.
constexpr int kProjF = 64;

template <typename T> struct XLoad;
template <> struct XLoad<float> {
    // 8 consecutive features k0 .. k0+7 (zero past K)
    __device__ __forceinline__ static void load(const float* row, int k0, int K, float (&v)[8]) {
        if (k0 + 8 <= K && (K & 3) == 0) {
            const float4 a = *reinterpret_cast<const float4*>(row + k0);
            const float4 b = *reinterpret_cast<const float4*>(row + k0 + 4);
            v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
            v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = k0 + j < K ? row[k0 + j] : 0.f;
        }
    }
};
template <> struct XLoad<bf16_t> {
    __device__ __forceinline__ static void load(const bf16_t* row, int k0, int K, float (&v)[8]) {
        if (k0 + 8 <= K && (K & 7) == 0) {
            Vec<bf16_t>::load(row + k0, v);
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = k0 + j < K ? bf2f(row[k0 + j]) : 0.f;
        }
    }
};

__device__ __forceinline__ float to_storage(float v, float*) { return v; }
__device__ __forceinline__ float to_storage(float v, bf16_t*) { return bf2f(f2bf(v)); }

template <typename T, int NCH>
__global__ void __launch_bounds__(kHeadBlock)
type_project_kernel(const T* __restrict__ x, int64_t rows, int K, const float* __restrict__ W,
                    const float* __restrict__ bias, const float* __restrict__ scale,
                    const uint64_t* __restrict__ drop_seed, uint32_t drop_thresh,
                    float drop_scale, int64_t row0, T* __restrict__ h, T* __restrict__ xs) {
    constexpr int F = kProjF, KP = 32 * NCH, LDR = KP + 8, EV = Vec<T>::N;
    constexpr bool EXACT_X = sizeof(T) == 2;            // bf16 x: its first split is exact
    extern __shared__ uint16_t Wp[];                   // [3][F][LDR] bf16 splits of W
    for (int idx = threadIdx.x; idx < F * KP; idx += blockDim.x) {
        const int f = idx / KP, k = idx - f * KP;
        uint16_t s0, s1, s2;
        split3(k < K ? W[(int64_t)f * K + k] : 0.f, s0, s1, s2);
        Wp[f * LDR + k] = s0;
        Wp[(F + f) * LDR + k] = s1;
        Wp[(2 * F + f) * LDR + k] = s2;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4;
    const int wpb = blockDim.x >> 6;
    const int64_t n_tiles = (rows + 15) / 16;
    const uint16_t* wa = Wp + c * LDR + 8 * q;
    uint32_t key = 0;
    if (drop_seed) key = drop_key(drop_seed);
    for (int64_t tile = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6); tile < n_tiles;
         tile += (int64_t)gridDim.x * wpb) {
        const int64_t r = tile * 16 + c;
        const bool valid = r < rows;
        const T* xr = x + (valid ? r : rows - 1) * K;
        f32x4 acc[4];
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) acc[kt] = *reinterpret_cast<const f32x4*>(bias + 16 * kt + 4 * q);
#pragma unroll 1
        for (int ch = 0; ch < NCH; ++ch) {
            float v[8];
            XLoad<T>::load(xr, 32 * ch + 8 * q, K, v);
            uint16_t s0[8], s1[8], s2[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) split3(v[j], s0[j], s1[j], s2[j]);
            const bf16x8_t b0 = pack8(s0), b1 = pack8(s1), b2 = pack8(s2);
#pragma unroll
            for (int kt = 0; kt < 4; ++kt) {
                const uint16_t* w = wa + (16 * kt) * LDR + 32 * ch;
                const bf16x8_t w0 = *reinterpret_cast<const bf16x8_t*>(w);
                const bf16x8_t w1 = *reinterpret_cast<const bf16x8_t*>(w + F * LDR);
                const bf16x8_t w2 = *reinterpret_cast<const bf16x8_t*>(w + 2 * F * LDR);
                acc[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2, b0, acc[kt], 0, 0, 0);
                if constexpr (!EXACT_X) {
                    acc[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, b1, acc[kt], 0, 0, 0);
                    acc[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0, b2, acc[kt], 0, 0, 0);
                }
                acc[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, b0, acc[kt], 0, 0, 0);
                if constexpr (!EXACT_X)
                    acc[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0, b1, acc[kt], 0, 0, 0);
                acc[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0, b0, acc[kt], 0, 0, 0);
            }
        }
        if (!valid) continue;
        const int64_t g = row0 + r;                     // global row: scale index, mask counter
        const float sc = scale ? scale[g] : 1.f;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
            const int f0 = 16 * kt + 4 * q;              // this lane's 4 features
            float hv[4], xv[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                hv[i] = to_storage(acc[kt][i], static_cast<T*>(nullptr));
                xv[i] = hv[i] * sc;
            }
            if (drop_seed) {
                // the mask of the 16-byte vector holding f0 (fp32: exactly these 4 features;
                // bf16: 8 features, this lane's half)
                float m[EV];
#pragma unroll
                for (int i = 0; i < EV; ++i) m[i] = 1.f;
                const int vec = f0 / EV, off = f0 - vec * EV;
                if ((drop_thresh & 0xFFu) == 0)
                    drop_apply<EV, 8>(key, drop_thresh, drop_scale, g, F / EV, vec, m);
                else
                    drop_apply<EV, 16>(key, drop_thresh, drop_scale, g, F / EV, vec, m);
#pragma unroll
                for (int i = 0; i < 4; ++i) xv[i] = m[off + i] != 0.f ? xv[i] * drop_scale : 0.f;
            }
            if constexpr (sizeof(T) == 4) {
                if (h)                                   // kernel-uniform (NULL: xs only)
                    *reinterpret_cast<float4*>(h + g * F + f0) = make_float4(hv[0], hv[1], hv[2], hv[3]);
                *reinterpret_cast<float4*>(xs + g * F + f0) = make_float4(xv[0], xv[1], xv[2], xv[3]);
            } else {
                uint2 hb, xb;
                hb.x = uint32_t(f2bf(hv[0])) | (uint32_t(f2bf(hv[1])) << 16);
                hb.y = uint32_t(f2bf(hv[2])) | (uint32_t(f2bf(hv[3])) << 16);
                xb.x = uint32_t(f2bf(xv[0])) | (uint32_t(f2bf(xv[1])) << 16);
                xb.y = uint32_t(f2bf(xv[2])) | (uint32_t(f2bf(xv[3])) << 16);
                if (h) *reinterpret_cast<uint2*>(h + g * F + f0) = hb;
                *reinterpret_cast<uint2*>(xs + g * F + f0) = xb;
            }
        }
    }
}

template <typename T, int NCH>
int launch_type_project(const void* x, int64_t rows, int K, const float* W, const float* b,
                        const float* scale, const uint64_t* seed, uint32_t keep16, float dscale,
                        int64_t row0, void* h, void* xs, hipStream_t stream) {
    constexpr size_t lds = (size_t)3 * kProjF * (32 * NCH + 8) * sizeof(uint16_t);
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(&type_project_kernel<T, NCH>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return REGNN_ELAUNCH;
        attr = true;
    }
    const int64_t tiles = (rows + 15) / 16;
    int64_t grid = (tiles + kHeadBlock / 64 - 1) / (kHeadBlock / 64);
    const int cap = resident_blocks(reinterpret_cast<const void*>(&type_project_kernel<T, NCH>),
                                    lds, kHeadBlock);
    if (grid > cap) grid = cap;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL((type_project_kernel<T, NCH>), dim3((unsigned)grid), dim3(kHeadBlock), lds,
                       stream, static_cast<const T*>(x), rows, K, W, b, scale, seed, keep16, dscale,
                       row0, static_cast<T*>(h), static_cast<T*>(xs));
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

template <typename T>
int dispatch_type_project(const void* x, int64_t rows, int K, const float* W, const float* b,
                          const float* scale, const uint64_t* seed, uint32_t keep16, float dscale,
                          int64_t row0, void* h, void* xs, hipStream_t stream) {
    switch ((K + 31) / 32) {
#define TP_CASE(nch) \
        case nch: return launch_type_project<T, nch>(x, rows, K, W, b, scale, seed, keep16, \
                                                     dscale, row0, h, xs, stream);
        TP_CASE(1) TP_CASE(2) TP_CASE(3) TP_CASE(4) TP_CASE(5) TP_CASE(6) TP_CASE(7) TP_CASE(8)
#undef TP_CASE
        default: return REGNN_EUNSUPPORTED;
    }
}

// ---------------------------------------------------------------------------------------------
// Linear(K -> C <= 64) weight / bias gradient for tall inputs (model/REGCN.py:31-35 fc_list
// backward): gW = g^T x, gb = colsum(g), fp32-accurate on bf16 MFMA (bf16x6). Each wave streams
// rows, 32 per 16x16x32 k-step, and keeps every output tile of its 64-feature block: lane (q, c)
// loads 16 bytes of each of its 8 rows 8 q + j from g (classes 4c .. 4c+3) and from x (features
// 64 fb + 4c .. +3), and component i of those loads feeds the MFMA pair (class 4m + ip, feature
// 64 fb + 4n + ix) -- 16 tiles, 64 accumulator registers, every byte of g and x read once per
// feature block. KB = K / 64 waves share a row stream (one per feature block); 8 / KB streams per
// block, each writing its own slab row.
template <typename T>
__device__ __forceinline__ f32x4 load4f(const T* p) {
    if constexpr (sizeof(T) == 4) {
        return *reinterpret_cast<const f32x4_u*>(p);
    } else {
        const uint2 u = *reinterpret_cast<const uint2*>(p);
        return f32x4{bf2f(u.x & 0xffffu), bf2f(u.x >> 16), bf2f(u.y & 0xffffu), bf2f(u.y >> 16)};
    }
}

template <typename T, int KB>
__global__ void __launch_bounds__(kHeadBlock)
linear_wgrad_kernel(const T* __restrict__ g, int64_t n, int C, int64_t ldg,
                    const T* __restrict__ x, int64_t rows_per_block, float* __restrict__ slab) {
    constexpr int K = 64 * KB, NS = 8 / KB;
    constexpr bool EXACT = sizeof(T) == 2;             // bf16 operands: one product
    const int lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4, w = threadIdx.x >> 6;
    const int fb = w % KB, st = w / KB;
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = min(n, r0 + rows_per_block);
    const bool cfull = 4 * c + 4 <= C;
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 gb = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int64_t row0 = r0 + 32 * st; row0 < r1; row0 += 32 * NS) {
        f32x4 P[8], X[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int64_t rr = row0 + 8 * q + j;
            const bool ok = rr < r1;
            const int64_t rc = ok ? rr : r0;
            f32x4 pv;
            if (cfull) {
                pv = load4f(g + rc * ldg + 4 * c);
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float v = sizeof(T) == 4 ? float(g[rc * ldg + min(4 * c + i, C - 1)])
                                                   : bf2f(uint32_t(g[rc * ldg + min(4 * c + i, C - 1)]));
                    pv[i] = 4 * c + i < C ? v : 0.f;
                }
            }
            const f32x4 xv = load4f(x + rc * K + 64 * fb + 4 * c);
            P[j] = ok ? pv : f32x4{0.f, 0.f, 0.f, 0.f};
            X[j] = ok ? xv : f32x4{0.f, 0.f, 0.f, 0.f};
            gb += P[j];
        }
        bf16x8_t A[4][3];
#pragma unroll
        for (int ip = 0; ip < 4; ++ip) {
            uint16_t s0[8], s1[8], s2[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) split3(P[j][ip], s0[j], s1[j], s2[j]);
            A[ip][0] = pack8(s0); A[ip][1] = pack8(s1); A[ip][2] = pack8(s2);
        }
#pragma unroll
        for (int ix = 0; ix < 4; ++ix) {
            uint16_t s0[8], s1[8], s2[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) split3(X[j][ix], s0[j], s1[j], s2[j]);
            const bf16x8_t b0 = pack8(s0), b1 = pack8(s1), b2 = pack8(s2);
#pragma unroll
            for (int ip = 0; ip < 4; ++ip) {
                f32x4& d = acc[ip][ix];
                if constexpr (!EXACT) {
                    d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[ip][2], b0, d, 0, 0, 0);
                    d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[ip][1], b1, d, 0, 0, 0);
                    d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[ip][0], b2, d, 0, 0, 0);
                    d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[ip][1], b0, d, 0, 0, 0);
                    d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[ip][0], b1, d, 0, 0, 0);
                }
                d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[ip][0], b0, d, 0, 0, 0);
            }
        }
    }
    // D[m][n] of tile (ip, ix) in lane (q, c = n), register r: m = 4 q + r -> class 4 m + ip,
    // feature 64 fb + 4 n + ix; slab row (block, stream): [64 * K + 64], class-major
    float* out = slab + ((int64_t)blockIdx.x * NS + st) * (64 * K + 64);
#pragma unroll
    for (int ip = 0; ip < 4; ++ip)
#pragma unroll
        for (int ix = 0; ix < 4; ++ix)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                out[(4 * (4 * q + r) + ip) * K + 64 * fb + 4 * c + ix] = acc[ip][ix][r];
    if (fb == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float v = gb[i];
            v += __shfl_xor(v, 16, 64);
            v += __shfl_xor(v, 32, 64);
            if (q == 0) out[64 * K + 4 * c + i] = v;
        }
    }
}

template <typename T, int KB>
int launch_linear_wgrad(const T* g, int64_t n, int C, int64_t ldg, const T* x, float* slab,
                        int slab_rows, hipStream_t stream) {
    constexpr int NS = 8 / KB;
    int64_t grid = slab_rows / NS;
    const int64_t rpb_min = 32 * NS * 4;
    if (grid * rpb_min > n) grid = (n + rpb_min - 1) / rpb_min;
    if (grid < 1) grid = 1;
    int64_t rpb = (n + grid - 1) / grid;
    rpb = (rpb + 32 * NS - 1) / (32 * NS) * (32 * NS);
    grid = (n + rpb - 1) / rpb;
    if (grid < 1) grid = 1;
    if (grid * NS > slab_rows) return REGNN_EINVAL;
    hipLaunchKernelGGL((linear_wgrad_kernel<T, KB>), dim3((unsigned)grid), dim3(kHeadBlock), 0,
                       stream, g, n, C, ldg, x, rpb, slab);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

}  // namespace regnn

using namespace regnn;

extern "C" {

int regnn_type_project(const void* x, int64_t rows, int32_t K, int32_t F, int32_t dtype,
                       const float* W, const float* b, const float* scale,
                       const uint64_t* drop_seed, uint32_t drop_keep16, float drop_scale,
                       int64_t row0, void* h, void* xs, hipStream_t stream) {
    if (rows < 0 || K <= 0 || F != kProjF || !W || !b || row0 < 0 ||
        (rows > 0 && (!x || !xs)) || (drop_seed && drop_keep16 > 65536u) ||
        (reinterpret_cast<uintptr_t>(b) & 15) || (reinterpret_cast<uintptr_t>(h) & 7) ||
        (reinterpret_cast<uintptr_t>(xs) & 7))
        return REGNN_EINVAL;
    if (K > 256) return REGNN_EUNSUPPORTED;
    if (rows == 0) return REGNN_OK;
    if (dtype == REGNN_F32)
        return dispatch_type_project<float>(x, rows, K, W, b, scale, drop_seed, drop_keep16,
                                            drop_scale, row0, h, xs, stream);
    if (dtype == REGNN_BF16)
        return dispatch_type_project<bf16_t>(x, rows, K, W, b, scale, drop_seed, drop_keep16,
                                             drop_scale, row0, h, xs, stream);
    return REGNN_EUNSUPPORTED;
}

int regnn_linear_wgrad(const void* g, int64_t n, int32_t C, int64_t ldg, const void* x,
                       int32_t K, int32_t dtype, float* slab, int32_t slab_rows,
                       hipStream_t stream) {
    if (!g || !x || !slab || n < 0 || C <= 0 || C > 64 || ldg < C || slab_rows <= 0)
        return REGNN_EINVAL;
    if (K != 64 && K != 128 && K != 256) return REGNN_EUNSUPPORTED;
    if (n == 0) return REGNN_OK;
    // 16-byte x rows; bf16 g rows are read 8 bytes at a time (fp32: 4-byte aligned loads)
    if (slab_rows < 8 || (reinterpret_cast<uintptr_t>(x) & 15) ||
        (dtype == REGNN_BF16 && ((reinterpret_cast<uintptr_t>(g) & 7) || (ldg & 3))))
        return REGNN_EINVAL;
#define LW_CASE(T, KB)                                                                          \
    if (K == 64 * KB)                                                                           \
        return launch_linear_wgrad<T, KB>(static_cast<const T*>(g), n, C, ldg,                  \
                                          static_cast<const T*>(x), slab, slab_rows, stream);
    if (dtype == REGNN_F32) { LW_CASE(float, 1) LW_CASE(float, 2) LW_CASE(float, 4) }
    if (dtype == REGNN_BF16) { LW_CASE(bf16_t, 1) LW_CASE(bf16_t, 2) LW_CASE(bf16_t, 4) }
#undef LW_CASE
    return REGNN_EUNSUPPORTED;
}

int regnn_col_sum(const float* x, int64_t rows, int32_t cols, float* slab, hipStream_t stream) {
    if (!x || !slab || rows < 0 || cols <= 0) return REGNN_EINVAL;
    const int grid = grid_for(rows, 1);      // <= kMaxGrid slab rows
    const int64_t rpb = (rows + grid - 1) / grid;
    hipLaunchKernelGGL(col_sum_kernel, dim3(grid), dim3(kBlock), 0, stream, x, rows, cols,
                       rpb > 0 ? rpb : 1, slab);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

int regnn_softmax_xent(const float* logits, int64_t rows, int32_t cols, int64_t ld,
                       const int64_t* labels, float scale, float* p, float* loss_rows,
                       hipStream_t stream) {
    if (!logits || !labels || !p || !loss_rows || rows < 0 || cols <= 0 || ld < cols)
        return REGNN_EINVAL;
    if (rows == 0) return REGNN_OK;
    hipLaunchKernelGGL(softmax_xent_kernel, dim3(grid_for(rows, kBlock / 64)), dim3(kBlock), 0,
                       stream, logits, rows, cols, ld, labels, scale, p, loss_rows);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

int regnn_head_fwd(const float* h, int64_t rows, int32_t K, const float* W, const float* b,
                   int32_t C, int64_t ld, const int64_t* labels, int64_t n_loss, float scale,
                   float* logits, float* p, float* loss_rows, hipStream_t stream) {
    if (!h || !W || !logits || rows < 0 || K != kHeadK || C <= 0 || C > kHeadMaxC || ld < C ||
        n_loss < 0 || n_loss > rows || (n_loss > 0 && (!labels || !p || !loss_rows)) ||
        (reinterpret_cast<uintptr_t>(h) & 15))
        return REGNN_EINVAL;
    if (rows == 0) return REGNN_OK;
    switch ((C + 15) / 16) {
#define HEAD_CASE(nt) \
        case nt: return launch_head<nt>(h, rows, W, b, C, ld, labels, n_loss, scale, logits, p, \
                                        loss_rows, stream);
        HEAD_CASE(1) HEAD_CASE(2) HEAD_CASE(3) HEAD_CASE(4) HEAD_CASE(5) HEAD_CASE(6)
        HEAD_CASE(7) HEAD_CASE(8) HEAD_CASE(9) HEAD_CASE(10) HEAD_CASE(11) HEAD_CASE(12)
        HEAD_CASE(13) HEAD_CASE(14) HEAD_CASE(15) HEAD_CASE(16) HEAD_CASE(17) HEAD_CASE(18)
        HEAD_CASE(19) HEAD_CASE(20) HEAD_CASE(21) HEAD_CASE(22) HEAD_CASE(23) HEAD_CASE(24)
#undef HEAD_CASE
        default: return REGNN_EINVAL;
    }
}

int regnn_head_argmax(const float* h, int64_t rows, int32_t K, const float* W, const float* b,
                      int32_t C, int64_t* out, hipStream_t stream) {
    if (!h || !W || !out || rows < 0 || K != kHeadK || C <= 0 || C > kHeadMaxC ||
        (reinterpret_cast<uintptr_t>(h) & 15))
        return REGNN_EINVAL;
    if (rows == 0) return REGNN_OK;
    switch ((C + 15) / 16) {
#define AMAX_CASE(nt) \
        case nt: return launch_head_v<nt, 0, true>(h, rows, W, b, C, C, nullptr, 0, 1.f,      \
                                                   nullptr, nullptr, nullptr, stream, out);
        AMAX_CASE(1) AMAX_CASE(2) AMAX_CASE(3) AMAX_CASE(4) AMAX_CASE(5) AMAX_CASE(6)
        AMAX_CASE(7) AMAX_CASE(8) AMAX_CASE(9) AMAX_CASE(10) AMAX_CASE(11) AMAX_CASE(12)
        AMAX_CASE(13) AMAX_CASE(14) AMAX_CASE(15) AMAX_CASE(16) AMAX_CASE(17) AMAX_CASE(18)
        AMAX_CASE(19) AMAX_CASE(20) AMAX_CASE(21) AMAX_CASE(22) AMAX_CASE(23) AMAX_CASE(24)
#undef AMAX_CASE
        default: return REGNN_EINVAL;
    }
}

int regnn_head_bwd(const float* p, int64_t n, int32_t C, int64_t ld, int32_t K, const float* W,
                   const float* h, const float* gscale, float* gh, int64_t n_out, float* slab,
                   int32_t slab_rows, hipStream_t stream) {
    if (!p || n < 0 || K != kHeadK || C <= 0 || C > kHeadMaxC || ld < C || (gh && !W) ||
        (gh && n_out < n) || (slab && (!h || slab_rows <= 0)) ||
        (gh && (reinterpret_cast<uintptr_t>(gh) & 15)))
        return REGNN_EINVAL;
    if (n == 0 && !(gh && n_out > 0)) return REGNN_OK;
    switch ((C + 15) / 16) {
#define HB_CASE(nt) \
        case nt: return launch_head_bwd<nt>(p, n, C, ld, W, h, gscale, gh, n_out, slab,       \
                                            slab_rows, stream);
        HB_CASE(1) HB_CASE(2) HB_CASE(3) HB_CASE(4) HB_CASE(5) HB_CASE(6)
        HB_CASE(7) HB_CASE(8) HB_CASE(9) HB_CASE(10) HB_CASE(11) HB_CASE(12)
        HB_CASE(13) HB_CASE(14) HB_CASE(15) HB_CASE(16) HB_CASE(17) HB_CASE(18)
        HB_CASE(19) HB_CASE(20) HB_CASE(21) HB_CASE(22) HB_CASE(23) HB_CASE(24)
#undef HB_CASE
        default: return REGNN_EINVAL;
    }
}

}  // extern "C"

template <int NT>
int head_fwd_lse_nt(const void* h, int64_t rows, const float* W, const float* b, int C,
                    int64_t ld, const int64_t* labels, int64_t n_loss, float* logits,
                    float* loss_lse, int dtype, hipStream_t stream) {
    if (dtype == 0)
        return launch_head<NT>(static_cast<const float*>(h), rows, W, b, C, ld, labels, n_loss,
                               1.f, logits, nullptr, loss_lse, stream);
    if constexpr (NT <= kX6MaxNT)
        return launch_head_x6<NT, false, bf16_t>(static_cast<const bf16_t*>(h), rows, W, b, C,
                                                 ld, labels, n_loss, 1.f, logits, nullptr,
                                                 loss_lse, stream);
    return REGNN_EUNSUPPORTED;
}

extern "C" {

int regnn_head_fwd_lse(const void* h, int64_t rows, int32_t K, const float* W, const float* b,
                       int32_t C, int64_t ld, const int64_t* labels, int64_t n_loss,
                       float* logits, float* loss_lse, int32_t dtype, hipStream_t stream) {
    if (!h || !W || !logits || rows < 0 || K != kHeadK || C <= 0 || C > kHeadMaxC || ld < C ||
        n_loss < 0 || n_loss > rows || (n_loss > 0 && (!labels || !loss_lse)) ||
        (dtype != 0 && dtype != 1) || (reinterpret_cast<uintptr_t>(h) & 15))
        return REGNN_EINVAL;
    if (rows == 0) return REGNN_OK;
    switch ((C + 15) / 16) {
#define HEAD_CASE(nt) \
        case nt: return head_fwd_lse_nt<nt>(h, rows, W, b, C, ld, labels, n_loss, logits,       \
                                            loss_lse, dtype, stream);
        HEAD_CASE(1) HEAD_CASE(2) HEAD_CASE(3) HEAD_CASE(4) HEAD_CASE(5) HEAD_CASE(6)
        HEAD_CASE(7) HEAD_CASE(8) HEAD_CASE(9) HEAD_CASE(10) HEAD_CASE(11) HEAD_CASE(12)
        HEAD_CASE(13) HEAD_CASE(14) HEAD_CASE(15) HEAD_CASE(16) HEAD_CASE(17) HEAD_CASE(18)
        HEAD_CASE(19) HEAD_CASE(20) HEAD_CASE(21) HEAD_CASE(22) HEAD_CASE(23) HEAD_CASE(24)
#undef HEAD_CASE
        default: return REGNN_EINVAL;
    }
}
int regnn_head_bwd_z(const float* z, int64_t n, int32_t C, int64_t ld, int32_t K,
                     const float* W, const void* h, const float* gscale, void* gh,
                     int64_t n_out, float* slab, int32_t slab_rows, const float* lse,
                     const int64_t* labels, float scale, const void* hx, const float* nx_scale,
                     void* nx_out, float* nx_dot, int32_t dtype, hipStream_t stream) {
    if (!z || n < 0 || K != kHeadK || C <= 0 || C > kHeadMaxC || ld < C || (gh && !W) ||
        (dtype != 0 && dtype != 1) || (nx_scale && !hx) ||
        (gh && n_out < n) || (slab && (!h || slab_rows <= 0)) || (n > 0 && (!lse || !labels)) ||
        (nx_scale && (!gh || !nx_out || !nx_dot)) ||
        ((reinterpret_cast<uintptr_t>(gh) | reinterpret_cast<uintptr_t>(nx_out) |
          (nx_scale ? reinterpret_cast<uintptr_t>(hx) : 0)) & (dtype == 1 ? 7 : 15)))
        return REGNN_EINVAL;
    if (n == 0 && !(gh && n_out > 0)) return REGNN_OK;
    const PSrc ps{lse, labels, scale};
    switch ((C + 15) / 16) {
#define HB_CASE(nt) \
        case nt: return launch_head_bwd<nt>(z, n, C, ld, W, static_cast<const float*>(h),      \
                                            gscale,                                           \
                                            static_cast<float*>(gh), n_out, slab, slab_rows,  \
                                            stream, nx_scale, static_cast<const float*>(hx),  \
                                            static_cast<float*>(nx_out), nx_dot, ps, dtype);
        HB_CASE(1) HB_CASE(2) HB_CASE(3) HB_CASE(4) HB_CASE(5) HB_CASE(6)
        HB_CASE(7) HB_CASE(8) HB_CASE(9) HB_CASE(10) HB_CASE(11) HB_CASE(12)
        HB_CASE(13) HB_CASE(14) HB_CASE(15) HB_CASE(16) HB_CASE(17) HB_CASE(18)
        HB_CASE(19) HB_CASE(20) HB_CASE(21) HB_CASE(22) HB_CASE(23) HB_CASE(24)
#undef HB_CASE
        default: return REGNN_EINVAL;
    }
}
int regnn_head_gh_next(const float* p, int64_t n, int32_t C, int64_t ld, int32_t K,
                       const float* W, const float* gscale, float* gh, int64_t n_out,
                       const float* nx_scale, const float* h, float* nx_out, float* nx_dot,
                       hipStream_t stream) {
    if (!p || n < 0 || K != kHeadK || C <= 0 || C > kHeadMaxC || ld < C || !W || !gh ||
        n_out < n || !nx_scale || !h || !nx_out || !nx_dot ||
        ((reinterpret_cast<uintptr_t>(gh) | reinterpret_cast<uintptr_t>(h) |
          reinterpret_cast<uintptr_t>(nx_out)) & 15))
        return REGNN_EINVAL;
    if (n_out == 0) return REGNN_OK;
    switch ((C + 15) / 16) {
#define HB_CASE(nt) \
        case nt: return launch_head_bwd<nt>(p, n, C, ld, W, nullptr, gscale, gh, n_out, nullptr, \
                                            0, stream, nx_scale, h, nx_out, nx_dot);
        HB_CASE(1) HB_CASE(2) HB_CASE(3) HB_CASE(4) HB_CASE(5) HB_CASE(6)
        HB_CASE(7) HB_CASE(8) HB_CASE(9) HB_CASE(10) HB_CASE(11) HB_CASE(12)
        HB_CASE(13) HB_CASE(14) HB_CASE(15) HB_CASE(16) HB_CASE(17) HB_CASE(18)
        HB_CASE(19) HB_CASE(20) HB_CASE(21) HB_CASE(22) HB_CASE(23) HB_CASE(24)
#undef HB_CASE
        default: return REGNN_EINVAL;
    }
}

}  // extern "C"
