// fp32-accurate dense GEMM on bf16 MFMA ("bf16x6", the split of re_dense.hip's head kernels):
// C = op(A) op(B) (+ beta C) with every fp32 operand x = x0 + x1 + x2 in bf16 and the six
// products x_i y_j (i + j <= 2) accumulated in fp32 by v_mfma_f32_16x16x32_bf16. The wide NS
// model (mag/regnn_ns.py:216-346 at hidden 128 .. 512, the reference's default width) runs its
// projections on it: group_input + the first conv's x @ W composed over the block's targets
// (mag/regnn_layers.py:101-107 by linearity), the other convs' x @ W, out_lin, and their
// backward products.
//
// Block tile 128 x 128 (or 64 x 128 for a live-row-bounded product: gemm_x6_kernel's TBM), k-step
// 32, 256 threads: wave w computes rows 64 (w >> 1) .., columns 64 (w & 1) .. as 4 x 4 MFMA tiles
// (96 MFMAs per k-step; 2 x 4 at 64 rows). The next k-step's operands are
// requested before this step's MFMAs (registers) and split into the three bf16 parts on their
// way into LDS. LDS rows of 32 bf16 padded to 40 (80 bytes: the 16 rows of an 8-element
// fragment read fall on distinct banks).
//
// Split-K (splits > 1): block z of the grid's third dimension sums k-steps z, z + splits, ...
// into its own partial C (work [splits][M][N]); regnn_gemm_x6 then adds the partials in split
// order (fixed: bitwise reproducible).
#include "regnn_common.h"

namespace regnn {
namespace gemm {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

// (BK 64 measured: 256 VGPRs and 3x slower; one LDS stage of BK 32 it is)
#ifndef GEMM_BK
#define GEMM_BK 32
#endif
// row tiles of A: BM = 128, or 64 (gemm_x6_kernel's TBM) where a capacity-sized operand leaves
// fewer live 128-row tiles than CUs; column tiles BN = 128
constexpr int BM = 128, BN = 128, BK = GEMM_BK, RS = BK + 8;
constexpr int kThreads = 256;
// quads (row, 4 k) per thread of an R-row operand tile
template <int R> constexpr int nq() { return R * BK / 4 / kThreads; }
// bf16 of the LDS stage: A (TBM rows) then B (BN rows), 3 splits each
template <int TBM> constexpr int stage() { return 3 * (TBM + BN) * RS; }

__device__ __forceinline__ void split3(float x, uint16_t& a, uint16_t& b, uint16_t& c) {
    a = f2bf(x);
    const float r = x - bf2f(a);
    b = f2bf(r);
    c = f2bf(r - bf2f(b));
}

// one operand tile (R rows r = m or n, 32 k) as R / 32 quads (row r, k .. k + 3) per thread:
//   KC (k contiguous): element (r, k) at p[r * ld + k]; quad i of thread t: i' = t + 256 i,
//      r = i' / 8, k = 4 (i' % 8): one float4 load
//   !KC (r contiguous): element (r, k) at p[k * ld + r]; i' = t + 256 i, r = i' % R,
//      k = 4 (i' / R): four loads, each coalesced over the wave (consecutive r)
template <bool KC, int R>
__device__ __forceinline__ void quad_rk(int i, int& r, int& k) {
    const int q = threadIdx.x + kThreads * i;
    if constexpr (KC) { r = q / (BK / 4); k = 4 * (q % (BK / 4)); }
    else { r = q % R; k = 4 * (q / R); }
}

template <bool KC, bool VEC, int R>
__device__ __forceinline__ void load_tile(const float* __restrict__ p, int64_t ld, int64_t r0,
                                          int64_t nr, int64_t k0, int64_t K,
                                          float4 (&v)[nq<R>()]) {
#pragma unroll
    for (int i = 0; i < nq<R>(); ++i) {
        int r, k;
        quad_rk<KC, R>(i, r, k);
        const int64_t rr = r0 + r, kk = k0 + k;
        // clamped addresses, then a select: unconditional loads (a load under a branch is
        // waited on at once)
        const bool rok = rr < nr;
        const int64_t rc = rok ? rr : 0;
        if constexpr (KC && VEC) {
            const bool ok = rok && kk < K;         // (K a multiple of 4)
            const float4 x = *reinterpret_cast<const float4*>(p + rc * ld + (ok ? kk : 0));
            v[i] = ok ? x : make_float4(0.f, 0.f, 0.f, 0.f);
        } else if constexpr (KC) {                 // rows without 16-byte alignment: 4 loads
            float e[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const bool ok = rok && kk + j < K;
                const float x = p[rc * ld + (ok ? kk + j : 0)];
                e[j] = ok ? x : 0.f;
            }
            v[i] = make_float4(e[0], e[1], e[2], e[3]);
        } else {
            float e[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const bool ok = rok && kk + j < K;
                const float x = p[(ok ? kk + j : 0) * ld + rc];
                e[j] = ok ? x : 0.f;
            }
            v[i] = make_float4(e[0], e[1], e[2], e[3]);
        }
    }
}

// the tile's three bf16 splits into LDS [3][R][RS] (row = m or n, column = k): 8-byte writes
template <bool KC, int R>
__device__ __forceinline__ void store_tile(uint16_t* __restrict__ s, const float4 (&v)[nq<R>()]) {
#pragma unroll
    for (int i = 0; i < nq<R>(); ++i) {
        int r, k;
        quad_rk<KC, R>(i, r, k);
        const float x[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
        uint16_t a[4], b[4], c[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) split3(x[j], a[j], b[j], c[j]);
        uint16_t* d = s + r * RS + k;
        *reinterpret_cast<uint2*>(d) = make_uint2(a[0] | (uint32_t(a[1]) << 16), a[2] | (uint32_t(a[3]) << 16));
        *reinterpret_cast<uint2*>(d + R * RS) = make_uint2(b[0] | (uint32_t(b[1]) << 16), b[2] | (uint32_t(b[3]) << 16));
        *reinterpret_cast<uint2*>(d + 2 * R * RS) = make_uint2(c[0] | (uint32_t(c[1]) << 16), c[2] | (uint32_t(c[3]) << 16));
    }
}

// C[m][n] = sum_k opA[m][k] opB[k][n]; TA: A stored [K][M] (lda >= M), else [M][K]; TB: B
// stored [N][K], else [K][N]. Wave w: rows TBM / 2 (w >> 1) .., columns 64 (w & 1) .. of the
// TBM x 128 tile as (TBM / 32) x 4 MFMA tiles (96 MFMAs per k-step at TBM = 128 against 24
// fragment reads from LDS). One k-step of wave (wr, wc)'s MFMA tiles: NI x NJ of them (the rest
// lie past M / N: an edge tile's waves skip the products nothing reads, e.g. the 4 extra columns
// of a 516-wide operand cost 1 / 8 of a tile's MFMAs instead of a whole tile's).
template <int NI, int NJ, int TBM>
__device__ __forceinline__ void mma_step(const uint16_t* sa, const uint16_t* sb, int wr, int wc,
                                         int c, int q, f32x4 (&acc)[4][4]) {
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
        bf16x8_t b[NJ][3];
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int s = 0; s < 3; ++s)
                b[j][s] = *reinterpret_cast<const bf16x8_t*>(sb + (s * BN + 64 * wc + 16 * j + c) * RS + 32 * ks + 8 * q);
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            bf16x8_t a[3];
#pragma unroll
            for (int s = 0; s < 3; ++s)
                a[s] = *reinterpret_cast<const bf16x8_t*>(sa + (s * TBM + (TBM / 2) * wr + 16 * i + c) * RS + 32 * ks + 8 * q);
#pragma unroll
            for (int j = 0; j < NJ; ++j) {             // small products first
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[j][0], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[j][1], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[j][2], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[j][0], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[j][1], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[j][0], acc[i][j], 0, 0, 0);
            }
        }
    }
}

// valid 16-wide MFMA tiles of a wave's `span` rows or columns from b of ext: 0, 1 or span / 16
// (2 / 3 of 4 run as 4)
__device__ __forceinline__ int wave_tiles(int64_t b, int64_t ext, int span) {
    const int64_t v = ext - b;
    return v <= 0 ? 0 : (v <= 16 ? 1 : span / 16);
}

// m_live / k_live (device counts, may be null): the operands' rows past them are zeros (a
// capacity-sized sampled block's unused rows), so a row tile m0 >= *m_live computes nothing (its
// C rows get beta C) and the k-steps past *k_live are skipped: the same result, the GEMM's work
// scaled to the batch's live rows. Every C element sums its k-steps in order and each k-step's
// six products in a fixed order whatever TBM is: the two row tilings give the same bits.
template <bool TA, bool TB, bool VEC, int TBM>
__global__ void __launch_bounds__(kThreads, 2)
gemm_x6_kernel(int64_t M, int64_t N, int64_t K, const float* __restrict__ A, int64_t lda,
               const float* __restrict__ B, int64_t ldb, float* __restrict__ C, int64_t ldc,
               float beta, float* __restrict__ work, const int32_t* __restrict__ m_live,
               const int32_t* __restrict__ k_live) {
    static_assert(TBM == 128 || TBM == 64, "row tile 128 or 64");
    constexpr int WRS = TBM / 2;                      // a wave's rows
    extern __shared__ uint16_t lds[];                 // [stage<TBM>()]
    constexpr bool AKC = !TA, BKC = TB;               // k contiguous in A / B
    const int64_t m0 = int64_t(blockIdx.y) * TBM, n0 = int64_t(blockIdx.x) * BN;
    const int z = blockIdx.z, S = gridDim.z;
    const int64_t Ke = k_live ? min(K, int64_t(*k_live)) : K;
    const bool dead = m_live && m0 >= int64_t(*m_live);
    // split-K: a dead row tile writes no partial (gemm_reduce_kernel skips the rows past m_live)
    if (dead && gridDim.z > 1) return;
    const int64_t nk = dead ? 0 : (Ke + BK - 1) / BK;
    const int lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4, w = threadIdx.x >> 6;
    const int wr = w >> 1, wc = w & 1;
    const int NI = wave_tiles(m0 + WRS * wr, M, WRS), NJ = wave_tiles(n0 + 64 * wc, N, 64);
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float4 va[nq<TBM>()], vb[nq<BN>()];
    int64_t kt = z;
    if (kt < nk) {
        load_tile<AKC, VEC, TBM>(A, lda, m0, M, kt * BK, K, va);
        load_tile<BKC, VEC, BN>(B, ldb, n0, N, kt * BK, K, vb);
    }
    const uint16_t* sa = lds;
    const uint16_t* sb = lds + 3 * TBM * RS;
    for (; kt < nk; kt += S) {
        __syncthreads();                              // (the previous step's reads are done)
        store_tile<AKC, TBM>(lds, va);
        store_tile<BKC, BN>(lds + 3 * TBM * RS, vb);
        __syncthreads();
        if (kt + S < nk) {                            // the next k-step's operands, in flight
            load_tile<AKC, VEC, TBM>(A, lda, m0, M, (kt + S) * BK, K, va);
            load_tile<BKC, VEC, BN>(B, ldb, n0, N, (kt + S) * BK, K, vb);
        }
#ifdef REGNN_GEMM_NO_EDGE
        mma_step<WRS / 16, 4, TBM>(sa, sb, wr, wc, c, q, acc);
#else
        if (NI == WRS / 16 && NJ == 4) mma_step<WRS / 16, 4, TBM>(sa, sb, wr, wc, c, q, acc);
        else if (NI == 1 && NJ == 4) mma_step<1, 4, TBM>(sa, sb, wr, wc, c, q, acc);
        else if (NI == WRS / 16 && NJ == 1) mma_step<WRS / 16, 1, TBM>(sa, sb, wr, wc, c, q, acc);
        else if (NI == 1 && NJ == 1) mma_step<1, 1, TBM>(sa, sb, wr, wc, c, q, acc);
#endif
    }
    // D lane (q, c): rows 4 q + r of the 16-row tile, column c
#pragma unroll
    for (int i = 0; i < WRS / 16; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t n = n0 + 64 * wc + 16 * j + c;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t m = m0 + WRS * wr + 16 * i + 4 * q + r;
                if (m < M && n < N) {
                    if (S == 1) {
                        float* o = C + m * ldc + n;
                        *o = beta != 0.f ? acc[i][j][r] + beta * *o : acc[i][j][r];
                    } else {
                        work[(int64_t(z) * M + m) * N + n] = acc[i][j][r];
                    }
                }
            }
        }
}

// C = sum_z work[z] (in split order) + beta C; rows past m_live (may be null) are beta C (the
// partials hold nothing there)
__global__ void __launch_bounds__(kThreads)
gemm_reduce_kernel(int64_t M, int64_t N, const float* __restrict__ work, int S, float* __restrict__ C,
                   int64_t ldc, float beta, const int32_t* __restrict__ m_live) {
    const int64_t total = M * N;
    const int64_t live = m_live ? min(M, int64_t(*m_live)) * N : total;
    for (int64_t e = int64_t(blockIdx.x) * kThreads + threadIdx.x; e < total;
         e += int64_t(gridDim.x) * kThreads) {
        if (e >= live) {
            const int64_t m = e / N, n = e - m * N;
            float* o = C + m * ldc + n;
            *o = beta != 0.f ? beta * *o : 0.f;
            continue;
        }
        // the splits' loads 8 at a time in flight (clamped addresses, unconditional), added in
        // split order (the same bits as one load and add per split)
        float s = work[e];
        for (int z = 1; z < S; z += 8) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = work[int64_t(z + j < S ? z + j : 0) * total + e];
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (z + j < S) s += v[j];
        }
        const int64_t m = e / N, n = e - m * N;
        float* o = C + m * ldc + n;
        *o = beta != 0.f ? s + beta * *o : s;
    }
}

// ---- several strided 2-D fp32 copies in one launch (the module path's parameter gradients into
// the flat bucket): descriptors by value in the kernel arguments
constexpr int kCopyMax = 32;
struct CopyArgs {
    regnn_copy2d d[kCopyMax];
    int64_t start[kCopyMax + 1];           // element prefix over the descriptors
    int n;
};

__global__ void __launch_bounds__(kThreads) copy2d_kernel(CopyArgs A) {
    const int64_t total = A.start[A.n];
    for (int64_t e = int64_t(blockIdx.x) * kThreads + threadIdx.x; e < total;
         e += int64_t(gridDim.x) * kThreads) {
        int k = 0;
        while (k + 1 < A.n && e >= A.start[k + 1]) ++k;
        const regnn_copy2d& d = A.d[k];
        const int64_t i = e - A.start[k], r = i / d.cols, c = i - r * d.cols;
        d.dst[i] = d.src[r * d.s0 + c * d.s1];
    }
}

}  // namespace gemm
}  // namespace regnn

using namespace regnn;
using namespace regnn::gemm;

static bool gemm_bm64() {                     // read per launch: tests switch it
    const char* v = getenv("REGNN_GEMM_BM64");
    return !(v && (v[0] == '0' || v[0] == 'o'));
}

extern "C" {

int64_t regnn_gemm_x6_work_floats(int64_t M, int64_t N, int32_t splits) {
    return splits > 1 ? int64_t(splits) * M * N : 0;
}

int regnn_gemm_x6(int32_t trans_a, int32_t trans_b, int64_t M, int64_t N, int64_t K,
                  const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                  float beta, float* work, int32_t splits, const int32_t* m_live,
                  const int32_t* k_live, hipStream_t stream) {
    if (M < 0 || N < 0 || K < 0 || splits < 1 || splits > 64) return REGNN_EINVAL;
    if (M == 0 || N == 0) return REGNN_OK;
    if (!A || !B || !C || (splits > 1 && !work)) return REGNN_EINVAL;
    // 16-byte operand vectors along each operand's contiguous dimension where the shapes and
    // addresses allow (else per-element loads: e.g. out_lin's 349 classes)
    const int64_t ca = trans_a ? M : K, cb = trans_b ? K : N;
    const bool vec = !(ca % 4 || cb % 4 || lda % 4 || ldb % 4 ||
                       reinterpret_cast<uintptr_t>(A) % 16 || reinterpret_cast<uintptr_t>(B) % 16);
    if (lda < (trans_a ? M : K) || ldb < (trans_b ? K : N) || ldc < N) return REGNN_EINVAL;
    // 64-row tiles for a capacity-sized operand without split-K (m_live: its live rows are
    // usually far fewer than its capacity, e.g. ~4.9 k of 13 312 at mag-10x, whose ~39 live
    // 128-row tiles x N / 128 leave CUs idle); REGNN_GEMM_BM64=off: 128 everywhere (A/B)
    const bool bm64 = m_live && splits == 1 && gemm_bm64();
    const int tbm = bm64 ? 64 : BM;
    const int64_t gy = (M + tbm - 1) / tbm, gx = (N + BN - 1) / BN;
    if (gy > 65535 || gx > 65535) return REGNN_EUNSUPPORTED;
    const dim3 grid{unsigned(gx), unsigned(gy), unsigned(splits)};
    const size_t lds = size_t(bm64 ? stage<64>() : stage<BM>()) * sizeof(uint16_t);
#define GEMM_CASE(TA_, TB_, V_)                                                                \
    if (bool(trans_a) == TA_ && bool(trans_b) == TB_ && vec == V_) {                           \
        if (bm64)                                                                              \
            hipLaunchKernelGGL((gemm_x6_kernel<TA_, TB_, V_, 64>), grid, dim3(kThreads), lds,   \
                               stream, M, N, K, A, lda, B, ldb, C, ldc, beta, work, m_live,    \
                               k_live);                                                        \
        else                                                                                   \
            hipLaunchKernelGGL((gemm_x6_kernel<TA_, TB_, V_, BM>), grid, dim3(kThreads), lds,   \
                               stream, M, N, K, A, lda, B, ldb, C, ldc, beta, work, m_live,    \
                               k_live);                                                        \
    }
    GEMM_CASE(false, false, true) GEMM_CASE(false, true, true) GEMM_CASE(true, false, true)
    GEMM_CASE(true, true, true) GEMM_CASE(false, false, false) GEMM_CASE(false, true, false)
    GEMM_CASE(true, false, false) GEMM_CASE(true, true, false)
#undef GEMM_CASE
    REGNN_LAUNCH_CHECK();
    if (splits > 1) {
        int64_t blocks = (M * N + kThreads - 1) / kThreads;
        if (blocks > 4096) blocks = 4096;
        hipLaunchKernelGGL(gemm_reduce_kernel, dim3(unsigned(blocks)), dim3(kThreads), 0, stream, M,
                           N, work, splits, C, ldc, beta, m_live);
        REGNN_LAUNCH_CHECK();
    }
    return REGNN_OK;
}

int regnn_copy2d_many(const regnn_copy2d* d, int32_t n, hipStream_t stream) {
    if (n < 0 || (n && !d)) return REGNN_EINVAL;
    for (int32_t b = 0; b < n; b += kCopyMax) {
        CopyArgs A{};
        A.n = n - b < kCopyMax ? n - b : kCopyMax;
        for (int k = 0; k < A.n; ++k) {
            const regnn_copy2d& x = d[b + k];
            if (x.rows < 0 || x.cols < 0 || (x.rows * x.cols && (!x.src || !x.dst)))
                return REGNN_EINVAL;
            A.d[k] = x;
            A.start[k + 1] = A.start[k] + x.rows * x.cols;
        }
        const int64_t total = A.start[A.n];
        if (!total) continue;
        int64_t blocks = (total + kThreads - 1) / kThreads;
        if (blocks > 2048) blocks = 2048;
        hipLaunchKernelGGL(copy2d_kernel, dim3(unsigned(blocks)), dim3(kThreads), 0, stream, A);
        REGNN_LAUNCH_CHECK();
    }
    return REGNN_OK;
}

}  // extern "C"
