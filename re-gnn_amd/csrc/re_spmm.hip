// Relation-embedding SpMM for gfx950: forward aggregation, fused transposed backward
// (SpMM + SDDMM 'dot' + relation-bin and node-norm gradients), weighted degree / norm and its
// backward, long-segment split path and deterministic slab reduction.
//
// Mapping (wave64): a segment (CSR row / CSC column) is owned by a group of LPR lanes; each lane
// holds NV 16-byte vectors of the F-wide feature row, so one group gathers a whole neighbour row
// per step (F=64 fp32: 16 lanes x 16 B = 256 B, four rows per wave-instruction). Neighbour ids,
// relation weights and scales are loaded coalesced, one edge per lane, and broadcast inside the
// group with width-LPR shuffles; UN rows are issued before any is consumed so each lane keeps
// UN*NV 16-byte loads in flight. Relation gradients go to lane-private LDS bins
// [n_rel][256 threads] (no cross-lane traffic per edge, no atomics) and leave the block through a
// fixed-order slab: bitwise reproducible.
#include <mutex>

#include "regnn_common.h"

namespace regnn {

struct SpmmArgs {
    const int32_t* ptr;
    const int32_t* idx;
    const uint8_t* rel;
    const float* tab;
    const float* edge_w;
    const float* in_scale;
    const float* out_scale;
    const float* bias;
    const void* src;       // gathered rows (x in forward, g in backward)
    void* out;             // y in forward, gx in backward
    const void* self;      // backward: forward input x of the segment's own node
    const void* ng_a;      // backward node grad: g rows
    const void* ng_b;      // backward node grad: y rows
    float* slab;
    int32_t n_rel;
    float* edge_grad;
    float* node_grad;
    int64_t n_seg;
    int32_t F;
    int32_t split;
    const int32_t* chunk_sched;  // processing slot -> chunk (NULL: identity); see make_args
    int32_t chunk;
    const int32_t* long_ids;
    int32_t n_long;
    const int32_t* chunk_long;
    const int32_t* chunk_off;
    int32_t n_chunk;
    float* chunk_partial;
    const int32_t* level_sb;     // tree reduction of chunk partials (see regnn_spmm_fwd)
    int32_t n_levels;
    const int64_t* level_desc;   // HOST [n_levels][3]: sb offset, n_out, partial row base
    int32_t slab_row0;     // first slab row this launch writes
    const uint64_t* drop_seed;   // fused dropout of the gathered rows (DROP kernels only)
    uint32_t drop_thresh;
    float drop_scale;
    const void* residual;  // forward epilogue: + residual row (dtype as out)
    const float* ln_w;     // forward epilogue: LayerNorm over the row (epi & kEpiLN)
    const float* ln_b;
    float ln_eps;
    int32_t epi;           // kEpiLN | kEpiReLU
    const float* nx_scale; // backward: the producer's post-scale of this op's input x (see
    void* nx_out;          //   regnn_spmm_bwd_next): nx_out = nx_scale * gx,
    float* nx_dot;         //   nx_dot = <gx, x> / nx_scale
                           // forward (regnn_spmm_fwd_next): the consumer's pre-scale of y,
                           //   nx_out = drop'(nx_scale * y) with drop' = (nx_seed, nx_thresh,
    const uint64_t* nx_seed;  //   nx_dscale), the row_scale_kernel spec
    uint32_t nx_thresh;
    float nx_dscale;
    int32_t self_pre;      // backward: `self` holds out_scale * drop(x) (the gathered rows of the
                           //   forward), not x: no mask on load, per-edge dots without out_scale,
                           //   node grad divided by out_scale (REGNN_SELF_PRESCALED)
};

enum { kEpiLN = 1, kEpiReLU = 2 };

// Backward per-edge dot products (SDDMM 'dot'), compile-time so the gather loop has no
// run-time branches: MODE 0 forward; 1 backward without per-edge dots; 2 relation bins (slab);
// 3 per-edge gradient; 4 both.
enum { kFwd = 0, kBwd = 1, kBwdSlab = 2, kBwdEdge = 3, kBwdBoth = 4 };

__device__ const float kOneF[1] = {1.f};
__device__ const uint8_t kZeroU8[4] = {0, 0, 0, 0};

// DROP: fused dropout of the forward input rows, 0 = none, 16 / 8 = bits per feature draw
template <typename T, int LPR, int NV, int MODE, int UNT = 0, bool FULL = false, int DROP = 0>
struct Seg {
    static constexpr int EV = Vec<T>::N;
    static constexpr bool BWD = MODE != kFwd;
    static constexpr bool SLAB = MODE == kBwdSlab || MODE == kBwdBoth;
    static constexpr bool EDGE = MODE == kBwdEdge || MODE == kBwdBoth;
    // rows gathered per step: 8 x 16-byte loads in flight per lane (NV vectors per row)
    static constexpr int UN0 = UNT > 0 ? UNT : (NV >= 8 ? 1 : (8 / NV));
    static constexpr int UN = UN0 < LPR ? UN0 : LPR;
    static constexpr int NVEC = LPR * NV;    // 16-byte vectors per row (FULL rows)

    __device__ __forceinline__ static int off(int q, int lane) { return (q * LPR + lane) * EV; }

    // Branch-free: the address is clamped into the row and out-of-row lanes are zeroed with a
    // select afterwards. A guarded load makes hipcc branch around it and wait vmcnt(0) right
    // after, serialising every gather of the unrolled batch (seen in the ISA).
    __device__ __forceinline__ static void load_raw(const T* row, int F, int lane, uint4 (&v)[NV]) {
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            const int o = off(q, lane);
            if constexpr (FULL) {           // F == LPR * NV * EV: every lane is inside the row
                v[q] = load16(row + o);
            } else {
                const bool in = o < F;
                const uint4 r = load16(row + (in ? o : 0));
                v[q] = make_uint4(in ? r.x : 0u, in ? r.y : 0u, in ? r.z : 0u, in ? r.w : 0u);
            }
        }
    }

    __device__ __forceinline__ static void load_row(const T* row, int F, int lane,
                                                    float (&v)[NV][EV]) {
        uint4 r[NV];
        load_raw(row, F, lane, r);
#pragma unroll
        for (int q = 0; q < NV; ++q) unpack<T>(r[q], v[q]);
    }

    // the forward input row of the segment's own node (backward): raw = x[seg], v = drop(x[seg])
    __device__ __forceinline__ static void load_self(const SpmmArgs& a, int64_t seg, int lane,
                                                     float (&v)[NV][EV], float (&raw)[NV][EV]) {
        load_row(static_cast<const T*>(a.self) + seg * a.F, a.F, lane, raw);
#pragma unroll
        for (int q = 0; q < NV; ++q)
#pragma unroll
            for (int t = 0; t < EV; ++t) v[q][t] = raw[q][t];
        if constexpr (DROP) {
            if (!a.self_pre) {                                     // kernel-uniform
                const uint32_t key = drop_key(a.drop_seed);
#pragma unroll
                for (int q = 0; q < NV; ++q)
                    drop_apply<EV, DROP>(key, a.drop_thresh, a.drop_scale, seg, NVEC, q * LPR + lane,
                                         v[q]);
            }
        }
    }

    __device__ __forceinline__ static float dot(const float (&a)[NV][EV], const float (&b)[NV][EV]) {
        float s = 0.f;
#pragma unroll
        for (int q = 0; q < NV; ++q)
#pragma unroll
            for (int t = 0; t < EV; ++t) s = fmaf(a[q][t], b[q][t], s);
        return s;
    }

    // Accumulate edges [beg, end) (beg < end) of one segment into acc. The backward modes also
    // form the per-edge dot <src[j], self> * in_scale[j] * os (relation bins / edge_grad).
    //
    // Per-edge metadata is software-pipelined over batches of LPR edges (one edge per lane): while
    // batch b is gathered, the in_scale / relation-table lookups of batch b+1 (ids loaded one
    // iteration earlier) and the id / relation loads of batch b+2 are in flight. Every load is
    // unconditional: edge indices are clamped to the segment, absent optional arrays read one
    // constant (kOneF / kZeroU8), and a batch tail is processed as a full step with weight 0 and
    // the dot scale 0, so no run-time branch forces a vmcnt(0) inside the loop.
    __device__ __forceinline__ static void accumulate(const SpmmArgs& a, int beg, int end, int lane,
                                                      float os, const float (&sx)[NV][EV],
                                                      float (&acc)[NV][EV], float* bins, int tid) {
        const T* __restrict__ src = static_cast<const T*>(a.src);
        const int F = a.F;
        const int last = end - 1;
        const float* tabp = a.tab ? a.tab : kOneF;
        const float* scp = a.in_scale ? a.in_scale : kOneF;
        const float* ewp = a.edge_w ? a.edge_w : kOneF;
        const uint8_t* relp = a.rel ? a.rel : kZeroU8;
        const int tm = a.tab ? 0xff : 0, sm = a.in_scale ? -1 : 0;
        const int em = a.edge_w ? -1 : 0, rm = a.rel ? -1 : 0;
        uint32_t dkey = 0;
        if constexpr (DROP && !BWD) dkey = drop_key(a.drop_seed);

        int ec = min(beg + lane, last);
        int j0 = a.idx[ec], r0 = relp[ec & rm];
        float ew0 = ewp[ec & em];
        float s0 = scp[j0 & sm], t0 = tabp[r0 & tm];
        ec = min(beg + LPR + lane, last);
        int j1 = a.idx[ec], r1 = relp[ec & rm];
        float ew1 = ewp[ec & em];
        for (int e0 = beg; e0 < end; e0 += LPR) {
            const float s1 = scp[j1 & sm], t1 = tabp[r1 & tm];        // lookups, batch b+1
            const int e2 = min(e0 + 2 * LPR + lane, last);            // ids, batch b+2
            const int j2 = a.idx[e2], r2 = relp[e2 & rm];
            const float ew2 = ewp[e2 & em];
            const bool live = e0 + lane < end;
            const float w0 = live ? t0 * ew0 * s0 : 0.f;
            const float d0 = live ? s0 * os : 0.f;                   // dot scale (backward)
            const int cnt = min(LPR, end - e0);
            for (int k = 0; k < cnt; k += UN) {
                int jj[UN];
                float wk[UN];
                uint4 raw[UN][NV];
#pragma unroll
                for (int u = 0; u < UN; ++u) jj[u] = __shfl(j0, k + u, LPR);
#pragma unroll
                for (int u = 0; u < UN; ++u) load_raw(src + (int64_t)jj[u] * F, F, lane, raw[u]);
#pragma unroll
                for (int u = 0; u < UN; ++u) wk[u] = __shfl(w0, k + u, LPR);
#pragma unroll
                for (int u = 0; u < UN; ++u) {
                    float v[NV][EV];
#pragma unroll
                    for (int q = 0; q < NV; ++q) unpack<T>(raw[u][q], v[q]);
                    if constexpr (DROP && !BWD) {
#pragma unroll
                        for (int q = 0; q < NV; ++q)
                            drop_apply<EV, DROP>(dkey, a.drop_thresh, a.drop_scale, jj[u], NVEC,
                                           q * LPR + lane, v[q]);
                    }
#pragma unroll
                    for (int q = 0; q < NV; ++q)
#pragma unroll
                        for (int t = 0; t < EV; ++t) acc[q][t] = fmaf(wk[u], v[q][t], acc[q][t]);
                    if constexpr (SLAB || EDGE) {
                        const float p = dot(v, sx) * __shfl(d0, k + u, LPR);
                        if constexpr (SLAB) bins[__shfl(r0, k + u, LPR) * kBlock + tid] += p;
                        if constexpr (EDGE) {
                            const float sum = group_sum<LPR>(p);
                            if (lane == 0 && k + u < cnt) a.edge_grad[e0 + k + u] = sum;
                        }
                    }
                }
            }
            j0 = j1; r0 = r1; ew0 = ew1; s0 = s1; t0 = t1;
            j1 = j2; r1 = r2; ew1 = ew2;
        }
    }

    // y = act(LN(os * acc + bias + residual)) (mag/regnn_layers.py:146-150 update() + residual
    // + self.norm, then the caller's F.relu, mag/regnn_ns.py:361-362): the row's mean and
    // variance are LPR-lane group sums, two passes like torch's LayerNorm (biased variance).
    __device__ __forceinline__ static void epilogue_fused(const SpmmArgs& a, int64_t seg, int lane,
                                                          float os, const float (&acc)[NV][EV],
                                                          T* __restrict__ out) {
        const int F = a.F;
        float r[NV][EV], res[NV][EV];
        if (a.residual) load_row(static_cast<const T*>(a.residual) + seg * F, F, lane, res);
        float s = 0.f;
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            const int o = off(q, lane);
            const bool in = o < F;
#pragma unroll
            for (int t = 0; t < EV; ++t) {
                float v = acc[q][t] * os;
                if (a.bias && in) v += a.bias[o + t];
                if (a.residual) v += res[q][t];
                r[q][t] = in ? v : 0.f;
                s += r[q][t];
            }
        }
        if (a.epi & kEpiLN) {
            const float mean = group_sum<LPR>(s) / float(F);
            float s2 = 0.f;
#pragma unroll
            for (int q = 0; q < NV; ++q) {
                const bool in = off(q, lane) < F;
#pragma unroll
                for (int t = 0; t < EV; ++t) {
                    const float d = r[q][t] - mean;
                    s2 += in ? d * d : 0.f;
                }
            }
            const float rstd = rsqrtf(group_sum<LPR>(s2) / float(F) + a.ln_eps);
#pragma unroll
            for (int q = 0; q < NV; ++q) {
                const int o = off(q, lane);
                if (o < F) {
#pragma unroll
                    for (int t = 0; t < EV; ++t) {
                        float v = (r[q][t] - mean) * rstd;
                        if (a.ln_w) v *= a.ln_w[o + t];
                        if (a.ln_b) v += a.ln_b[o + t];
                        r[q][t] = v;
                    }
                }
            }
        }
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            const int o = off(q, lane);
            if (o < F) {
                if (a.epi & kEpiReLU) {
#pragma unroll
                    for (int t = 0; t < EV; ++t) r[q][t] = fmaxf(r[q][t], 0.f);
                }
                Vec<T>::store(out + o, r[q]);
            }
        }
    }

    // y = os * acc + bias; backward node grad = <self, acc> + <g_i, y_i> / in_scale[i].
    __device__ __forceinline__ static void epilogue(const SpmmArgs& a, int64_t seg, int lane,
                                                    float os, const float (&sx)[NV][EV],
                                                    float (&acc)[NV][EV],
                                                    const float (&sraw)[NV][EV]) {
        const int F = a.F;
        if constexpr (BWD) {
            if (a.node_grad) {
                float ng = dot(sx, acc);
                if (a.self_pre) ng /= os;                          // <drop(x), acc> = <self, acc>/os
                if (a.ng_a && a.ng_b) {
                    float ga[NV][EV], yb[NV][EV];
                    load_row(static_cast<const T*>(a.ng_a) + seg * F, F, lane, ga);
                    load_row(static_cast<const T*>(a.ng_b) + seg * F, F, lane, yb);
                    const float is = a.in_scale ? a.in_scale[seg] : 1.f;
                    ng += dot(ga, yb) / is;
                }
                ng = group_sum<LPR>(ng);
                if (lane == 0) a.node_grad[seg] = ng;
            }
        }
        T* __restrict__ out = static_cast<T*>(a.out) + seg * F;
        if constexpr (!BWD) {
            if (a.residual || a.epi) {          // wave-uniform: fused forward epilogue
                epilogue_fused(a, seg, lane, os, acc, out);
                return;
            }
        }
        uint32_t dkey = 0;
        if constexpr (DROP && BWD) dkey = drop_key(a.drop_seed);
        // backward with the producer's pre-scale folded in (regnn_spmm_bwd_next): gx also leaves
        // as nx_scale * gx, and <gx, x> / nx_scale, for the producing aggregation's backward;
        // forward (regnn_spmm_fwd_next): y also leaves as the consumer's drop'(nx_scale * y)
        const bool nx = a.nx_scale != nullptr;                   // wave-uniform
        const float ns = nx ? a.nx_scale[seg] : 1.f;
        float nd = 0.f;
        uint32_t nkey = 0;
        if (!BWD && nx && a.nx_seed) nkey = drop_key(a.nx_seed);
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            const int o = off(q, lane);
            if (o < F) {
                float r[EV];
#pragma unroll
                for (int t = 0; t < EV; ++t) {
                    r[t] = acc[q][t] * os;
                    if (!BWD && a.bias) r[t] += a.bias[o + t];
                }
                // backward through the fused dropout of the forward input rows
                if constexpr (DROP && BWD)
                    drop_apply<EV, DROP>(dkey, a.drop_thresh, a.drop_scale, seg, NVEC, q * LPR + lane, r);
                Vec<T>::store(out + o, r);
                if (nx) {
                    // from the stored (dtype-rounded) values, as a row pass over `out` would see
                    float rs[EV];
#pragma unroll
                    for (int t = 0; t < EV; ++t) {
                        const float rv = round_to<T>(r[t]);
                        if constexpr (BWD) nd = fmaf(rv, sraw[q][t], nd);
                        rs[t] = rv * ns;
                    }
                    if constexpr (!BWD) {
                        if (a.nx_seed) {
                            if ((a.nx_thresh & 0xFFu) == 0)
                                drop_apply<EV, 8>(nkey, a.nx_thresh, a.nx_dscale, seg, NVEC, q * LPR + lane, rs);
                            else
                                drop_apply<EV, 16>(nkey, a.nx_thresh, a.nx_dscale, seg, NVEC, q * LPR + lane, rs);
                        }
                    }
                    Vec<T>::store(static_cast<T*>(a.nx_out) + seg * F + o, rs);
                }
            }
        }
        if constexpr (BWD) {
            if (nx) {
                nd = group_sum<LPR>(nd);
                if (lane == 0) a.nx_dot[seg] = nd / ns;
            }
        }
    }
};

__device__ __forceinline__ void bins_zero(float* bins, int n_rel, int tid) {
    for (int r = 0; r < n_rel; ++r) bins[r * kBlock + tid] = 0.f;
}

// fixed-order block reduction of the lane-private bins into slab row `row`
__device__ __forceinline__ void bins_flush(float* bins, int n_rel, int tid, float* slab, int row) {
    __syncthreads();
    for (int r = tid; r < n_rel; r += kBlock) {
        float s = 0.f;
        for (int t = 0; t < kBlock; ++t) s += bins[r * kBlock + t];
        slab[(int64_t)row * n_rel + r] = s;
    }
}

template <typename T, int LPR, int NV, int MODE, int UNT, bool FULL, int DROP>
__global__ void __launch_bounds__(kBlock) spmm_main(SpmmArgs a) {
    extern __shared__ float bins[];
    using S = Seg<T, LPR, NV, MODE, UNT, FULL, DROP>;
    constexpr int GPB = kBlock / LPR;
    const int tid = threadIdx.x, lane = tid & (LPR - 1);
    if constexpr (S::SLAB) bins_zero(bins, a.n_rel, tid);
    const bool need_self = S::SLAB || S::EDGE || (S::BWD && (a.node_grad || a.nx_scale));
    for (int64_t seg = (int64_t)blockIdx.x * GPB + tid / LPR; seg < a.n_seg;
         seg += (int64_t)gridDim.x * GPB) {
        const int beg = a.ptr[seg], end = a.ptr[seg + 1];
        if (a.split > 0 && end - beg > a.split) continue;   // long-segment path
        float acc[NV][S::EV] = {};
        float sx[NV][S::EV] = {}, sraw[NV][S::EV] = {};
        if (need_self) S::load_self(a, seg, lane, sx, sraw);
        const float os = a.out_scale ? a.out_scale[seg] : 1.f;
        if (beg < end) S::accumulate(a, beg, end, lane, a.self_pre ? 1.f : os, sx, acc, bins, tid);
        S::epilogue(a, seg, lane, os, sx, acc, sraw);
    }
    if constexpr (S::SLAB) bins_flush(bins, a.n_rel, tid, a.slab, a.slab_row0 + blockIdx.x);
}

// one group per chunk of a long segment: raw partial sums (fp32) -> chunk_partial
template <typename T, int LPR, int NV, int MODE, int UNT, bool FULL, int DROP>
__global__ void __launch_bounds__(kBlock) spmm_chunks(SpmmArgs a) {
    extern __shared__ float bins[];
    using S = Seg<T, LPR, NV, MODE, UNT, FULL, DROP>;
    constexpr int GPB = kBlock / LPR;
    const int tid = threadIdx.x, lane = tid & (LPR - 1);
    if constexpr (S::SLAB) bins_zero(bins, a.n_rel, tid);
    for (int64_t i = (int64_t)blockIdx.x * GPB + tid / LPR; i < a.n_chunk;
         i += (int64_t)gridDim.x * GPB) {
        const int64_t c = a.chunk_sched ? a.chunk_sched[i] : i;     // group-uniform
        const int l = a.chunk_long[c];
        const int64_t seg = a.long_ids[l];
        const int k = int(c) - a.chunk_off[l];
        const int s0 = a.ptr[seg], s1 = a.ptr[seg + 1];
        const int beg = s0 + k * a.chunk;
        const int end = min(s1, beg + a.chunk);
        float acc[NV][S::EV] = {};
        float sx[NV][S::EV] = {}, sraw[NV][S::EV] = {};
        if constexpr (S::SLAB || S::EDGE) S::load_self(a, seg, lane, sx, sraw);
        const float os = a.out_scale ? a.out_scale[seg] : 1.f;
        if (beg < end) S::accumulate(a, beg, end, lane, a.self_pre ? 1.f : os, sx, acc, bins, tid);
        float* part = a.chunk_partial + c * a.F;
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            const int o = S::off(q, lane);
            if (o < a.F) {
#pragma unroll
                for (int t = 0; t < S::EV; ++t) part[o + t] = acc[q][t];
            }
        }
    }
    if constexpr (S::SLAB) bins_flush(bins, a.n_rel, tid, a.slab, a.slab_row0 + blockIdx.x);
}

// one level of the fixed-order tree over chunk partials: output row p = sum of input rows
// [sb[p], sb[p+1]) in order (consecutive rows of one long segment), one group per output row
template <int LPR>
__global__ void __launch_bounds__(kBlock)
partial_reduce(const float* __restrict__ in, const int32_t* __restrict__ sb, int64_t n_out, int F,
               float* __restrict__ out) {
    constexpr int GPB = kBlock / LPR;
    const int tid = threadIdx.x, lane = tid & (LPR - 1);
    const int nv = F / 4;
    for (int64_t p = (int64_t)blockIdx.x * GPB + tid / LPR; p < n_out;
         p += (int64_t)gridDim.x * GPB) {
        const int b = sb[p], e = sb[p + 1];
        for (int v = lane; v < nv; v += LPR) {
            float acc[4] = {0.f, 0.f, 0.f, 0.f};
            int r = b;
            for (; r + 4 <= e; r += 4) {
                float x[4][4];
#pragma unroll
                for (int u = 0; u < 4; ++u) Vec<float>::load(in + (int64_t)(r + u) * F + 4 * v, x[u]);
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int t = 0; t < 4; ++t) acc[t] += x[u][t];
            }
            for (; r < e; ++r) {
                float x[4];
                Vec<float>::load(in + (int64_t)r * F + 4 * v, x);
#pragma unroll
                for (int t = 0; t < 4; ++t) acc[t] += x[t];
            }
            Vec<float>::store(out + p * F + 4 * v, acc);
        }
    }
}

// one group per long segment: its fully reduced partial row, then the epilogue
template <typename T, int LPR, int NV, int MODE, int UNT, bool FULL, int DROP>
__global__ void __launch_bounds__(kBlock) spmm_fixup(SpmmArgs a, int64_t final_base) {
    using S = Seg<T, LPR, NV, MODE, UNT, FULL, DROP>;
    constexpr int GPB = kBlock / LPR;
    const int tid = threadIdx.x, lane = tid & (LPR - 1);
    const bool need_self = S::BWD && (a.node_grad || a.nx_scale);
    for (int64_t l = (int64_t)blockIdx.x * GPB + tid / LPR; l < a.n_long;
         l += (int64_t)gridDim.x * GPB) {
        const int64_t seg = a.long_ids[l];
        float acc[NV][S::EV] = {};
        float sx[NV][S::EV] = {}, sraw[NV][S::EV] = {};
        if (need_self) S::load_self(a, seg, lane, sx, sraw);
        const int64_t row = final_base >= 0 ? final_base + l : a.chunk_off[l];
        const float* part = a.chunk_partial + row * a.F;
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            const int o = S::off(q, lane);
            if (o < a.F) {
#pragma unroll
                for (int t = 0; t < S::EV; ++t) acc[q][t] = part[o + t];
            }
        }
        const float os = a.out_scale ? a.out_scale[seg] : 1.f;
        S::epilogue(a, seg, lane, os, sx, acc, sraw);
    }
}

template <typename T, int LPR, int NV, int MODE, int UNT = 0, bool FULL = false, int DROP = 0>
int launch_spmm(SpmmArgs a, hipStream_t stream) {
    using S = Seg<T, LPR, NV, MODE, UNT, FULL, DROP>;
    constexpr int GPB = kBlock / LPR;
    const size_t lds = S::SLAB ? size_t(a.n_rel) * kBlock * sizeof(float) : 0;
    const int g1 = grid_resident(spmm_main<T, LPR, NV, MODE, UNT, FULL, DROP>, a.n_seg, GPB, lds);
    a.slab_row0 = 0;
    hipLaunchKernelGGL((spmm_main<T, LPR, NV, MODE, UNT, FULL, DROP>), dim3(g1), dim3(kBlock), lds,
                       stream, a);
    REGNN_LAUNCH_CHECK();
    if (a.split > 0 && a.n_chunk > 0) {
        a.slab_row0 = kMaxGrid;
        const int g2 =
            grid_resident(spmm_chunks<T, LPR, NV, MODE, UNT, FULL, DROP>, a.n_chunk, GPB, lds);
        hipLaunchKernelGGL((spmm_chunks<T, LPR, NV, MODE, UNT, FULL, DROP>), dim3(g2), dim3(kBlock),
                           lds, stream, a);
        REGNN_LAUNCH_CHECK();
        int64_t base_in = 0, final_base = -1;
        for (int k = 0; k < a.n_levels; ++k) {
            const int64_t sb_off = a.level_desc[3 * k], n_out = a.level_desc[3 * k + 1];
            const int64_t base_out = a.level_desc[3 * k + 2];
            hipLaunchKernelGGL((partial_reduce<16>), dim3(grid_for(n_out, kBlock / 16)),
                               dim3(kBlock), 0, stream, a.chunk_partial + base_in * a.F,
                               a.level_sb + sb_off, n_out, a.F, a.chunk_partial + base_out * a.F);
            REGNN_LAUNCH_CHECK();
            base_in = base_out;
            final_base = base_out;
        }
        const int g3 = grid_for(a.n_long, GPB);
        hipLaunchKernelGGL((spmm_fixup<T, LPR, NV, MODE, UNT, FULL, DROP>), dim3(g3), dim3(kBlock),
                           0, stream, a, final_base);
        REGNN_LAUNCH_CHECK();
    }
    return REGNN_OK;
}

template <typename T, int LPR, int NV, int UNT = 0, bool FULL = false, int DROP = 0>
int launch_mode(SpmmArgs a, int mode, hipStream_t stream) {
    switch (mode) {
        case kFwd: return launch_spmm<T, LPR, NV, kFwd, UNT, FULL, DROP>(a, stream);
        case kBwd: return launch_spmm<T, LPR, NV, kBwd, UNT, FULL, DROP>(a, stream);
        case kBwdSlab: return launch_spmm<T, LPR, NV, kBwdSlab, UNT, FULL, DROP>(a, stream);
        case kBwdEdge: return launch_spmm<T, LPR, NV, kBwdEdge, UNT, FULL, DROP>(a, stream);
        default: return launch_spmm<T, LPR, NV, kBwdBoth, UNT, FULL, DROP>(a, stream);
    }
}

// F = 16 vectors (F=64 fp32 / F=128 bf16), the BASELINE hidden size: exact fit (no lane masking)
// and a tunable number of rows in flight per lane (regnn_tune key 2: 0 = 8, or 4 / 16)
template <typename T>
int launch_f16v(SpmmArgs a, int mode, hipStream_t stream) {
    if (a.drop_seed) {
        if ((a.drop_thresh & 0xFFu) == 0) return launch_mode<T, 16, 1, 8, true, 8>(a, mode, stream);
        return launch_mode<T, 16, 1, 8, true, 16>(a, mode, stream);
    }
    if (g_tune_un == 4) return launch_mode<T, 16, 1, 4, true>(a, mode, stream);
    if (g_tune_un == 16) return launch_mode<T, 16, 1, 16, true>(a, mode, stream);
    return launch_mode<T, 16, 1, 8, true>(a, mode, stream);
}

// (lanes per segment, vectors per lane) for a row of nvec 16-byte vectors
template <typename T>
int dispatch(SpmmArgs a, int mode, hipStream_t stream) {
    constexpr int EV = Vec<T>::N;
    if (a.F <= 0 || a.F % EV) return REGNN_EUNSUPPORTED;
    const int nvec = a.F / EV;
    if (a.drop_seed && nvec != 16 && nvec != 8) return REGNN_EUNSUPPORTED;   // fused dropout
    if (nvec <= 4) return launch_mode<T, 4, 1>(a, mode, stream);
    if (nvec == 8 && a.drop_seed) {          // F = 64 bf16: fused dropout on 128-byte rows
        if ((a.drop_thresh & 0xFFu) == 0) return launch_mode<T, 8, 1, 0, true, 8>(a, mode, stream);
        return launch_mode<T, 8, 1, 0, true, 16>(a, mode, stream);
    }
    if (nvec <= 8) return launch_mode<T, 8, 1>(a, mode, stream);
    if (nvec == 16) return launch_f16v<T>(a, mode, stream);
    if (nvec <= 16) return launch_mode<T, 16, 1>(a, mode, stream);
    if (nvec <= 32) return launch_mode<T, 16, 2>(a, mode, stream);
    if (nvec <= 48) return launch_mode<T, 16, 3>(a, mode, stream);
    if (nvec <= 64) return launch_mode<T, 16, 4>(a, mode, stream);
    if (nvec <= 128) return launch_mode<T, 64, 2>(a, mode, stream);
    if (nvec <= 256) return launch_mode<T, 64, 4>(a, mode, stream);
    return REGNN_EUNSUPPORTED;
}

// ---------------------------------------------------------------------------------------------
// degree / norm
// ---------------------------------------------------------------------------------------------
// Weighted degree, one thread per row (consecutive rows per wave, so a wave's relation-id reads
// walk one contiguous stretch of the CSR). The relation ids are read as aligned 32-bit words
// (4 edges per load, bytes outside [b, e) masked) and the table lives in LDS, so a row costs
// ~deg/4 independent loads instead of deg dependent (id -> table) global load pairs.
__device__ __forceinline__ void rel_words(int b, int e, int& w0, int& w1) {
    w0 = b >> 2;
    w1 = (e + 3) >> 2;
}

__device__ __forceinline__ uint32_t word_mask(int w, int b, int e) {
    // bit k of the result set iff byte k of word w is an edge of [b, e)
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int pos = 4 * w + k;
        m |= (pos >= b && pos < e) ? (1u << k) : 0u;
    }
    return m;
}

__global__ void __launch_bounds__(kBlock)
degree_kernel(const int32_t* __restrict__ ptr, const uint8_t* __restrict__ rel,
              const float* __restrict__ tab, int32_t n_rel, int64_t n_seg, float power,
              int32_t split, float* __restrict__ deg, float* __restrict__ norm) {
    __shared__ float stab[256];
    for (int r = threadIdx.x; r < 256; r += kBlock) stab[r] = (tab && r < n_rel) ? tab[r] : 0.f;
    __syncthreads();
    const uint32_t* __restrict__ rel32 = reinterpret_cast<const uint32_t*>(rel);
    for (int64_t v = (int64_t)blockIdx.x * kBlock + threadIdx.x; v < n_seg;
         v += (int64_t)gridDim.x * kBlock) {
        const int b = ptr[v], e = ptr[v + 1];
        if (split > 0 && e - b > split) continue;
        float d;
        if (tab) {
            d = 0.f;
            int w0, w1;
            rel_words(b, e, w0, w1);
            for (int w = w0; w < w1; ++w) {
                const uint32_t x = rel32[w];
                const uint32_t m = word_mask(w, b, e);
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (m & (1u << k)) d += stab[(x >> (8 * k)) & 0xFFu];
            }
        } else {
            d = float(e - b);
        }
        deg[v] = d;
        if (norm) norm[v] = powf(fmaxf(d, 1.f), power);
    }
}

__global__ void __launch_bounds__(kBlock)
degree_long_kernel(const int32_t* __restrict__ ptr, const float* __restrict__ tab,
                   const int32_t* __restrict__ long_ids, int32_t n_long,
                   const int32_t* __restrict__ long_cnt, int32_t n_rel, float power,
                   float* __restrict__ deg, float* __restrict__ norm) {
    for (int l = blockIdx.x * kBlock + threadIdx.x; l < n_long; l += gridDim.x * kBlock) {
        const int64_t v = long_ids[l];
        float d;
        if (tab) {
            d = 0.f;
            for (int r = 0; r < n_rel; ++r) d += tab[r] * float(long_cnt[(int64_t)l * n_rel + r]);
        } else {
            d = float(ptr[v + 1] - ptr[v]);
        }
        deg[v] = d;
        if (norm) norm[v] = powf(fmaxf(d, 1.f), power);
    }
}

constexpr int kDegCntMaxRel = 16;   // regnn_degree_cnt / _bwd: relation tables up to 16 entries

__device__ __forceinline__ float dnorm_ddeg(float d, float g, float power) {
    // d/d deg of max(deg,1)^power with torch clamp semantics (gradient passes where deg >= 1)
    return d >= 1.f ? g * power * powf(d, power - 1.f) : 0.f;
}

__global__ void __launch_bounds__(kBlock)
degree_bwd_kernel(const int32_t* __restrict__ ptr, const uint8_t* __restrict__ rel,
                  const float* __restrict__ deg, const float* __restrict__ g_norm, int64_t n_seg,
                  float power, int32_t n_rel, int32_t split, const int32_t* __restrict__ long_ids,
                  int32_t n_long, const int32_t* __restrict__ long_cnt, float* __restrict__ slab) {
    // one thread per row, relation ids read as 32-bit words (as degree_kernel); the row's degree
    // gradient goes into the thread's own LDS relation bins (no atomics, fixed order)
    extern __shared__ float bins[];
    const int tid = threadIdx.x;
    bins_zero(bins, n_rel, tid);
    const uint32_t* __restrict__ rel32 = reinterpret_cast<const uint32_t*>(rel);
    for (int64_t v = (int64_t)blockIdx.x * kBlock + tid; v < n_seg;
         v += (int64_t)gridDim.x * kBlock) {
        const int b = ptr[v], e = ptr[v + 1];
        if (split > 0 && e - b > split) continue;
        const float gd = dnorm_ddeg(deg[v], g_norm[v], power);
        int w0, w1;
        rel_words(b, e, w0, w1);
        for (int w = w0; w < w1; ++w) {
            const uint32_t x = rel32[w];
            const uint32_t m = word_mask(w, b, e);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (m & (1u << k)) bins[((x >> (8 * k)) & 0xFFu) * kBlock + tid] += gd;
        }
    }
    for (int l = blockIdx.x * kBlock + tid; l < n_long; l += gridDim.x * kBlock) {
        const int64_t v = long_ids[l];
        const float gd = dnorm_ddeg(deg[v], g_norm[v], power);
        for (int r = 0; r < n_rel; ++r)
            bins[r * kBlock + tid] += gd * float(long_cnt[(int64_t)l * n_rel + r]);
    }
    bins_flush(bins, n_rel, tid, slab, blockIdx.x);
}

// Weighted degree and its backward from the graph's per-row relation histogram cnt [n_seg, n_rel]
// (uint16, RelPack.row_cnt: static per graph and relation-id tensor, long rows zero): a row
// costs n_rel coalesced 2-byte reads instead of a walk over its relation ids, and the backward
// is a reduction of gd[v] * cnt[v, r] over rows in registers (no LDS bins). The long rows are
// then overwritten by degree_long_kernel (forward) / added from long_cnt (backward).
__global__ void __launch_bounds__(kBlock)
degree_cnt_kernel(const uint16_t* __restrict__ cnt, const float* __restrict__ tab,
                  int32_t n_rel, int64_t n_seg, float power, float* __restrict__ deg,
                  float* __restrict__ norm) {
    __shared__ float stab[kDegCntMaxRel];
    for (int r = threadIdx.x; r < kDegCntMaxRel; r += kBlock) stab[r] = r < n_rel ? tab[r] : 0.f;
    __syncthreads();
    for (int64_t v = (int64_t)blockIdx.x * kBlock + threadIdx.x; v < n_seg;
         v += (int64_t)gridDim.x * kBlock) {
        const uint16_t* c = cnt + v * n_rel;
        float d = 0.f;
        for (int r = 0; r < n_rel; ++r) d = fmaf(stab[r], float(c[r]), d);
        deg[v] = d;
        if (norm) norm[v] = powf(fmaxf(d, 1.f), power);
    }
}

__global__ void __launch_bounds__(kBlock)
degree_cnt_bwd_kernel(const uint16_t* __restrict__ cnt, const float* __restrict__ deg,
                      const float* __restrict__ g_norm, int64_t n_seg, float power, int32_t n_rel,
                      const int32_t* __restrict__ long_ids, int32_t n_long,
                      const int32_t* __restrict__ long_cnt, float* __restrict__ slab) {
    float acc[kDegCntMaxRel];
#pragma unroll
    for (int r = 0; r < kDegCntMaxRel; ++r) acc[r] = 0.f;
    const int tid = threadIdx.x;
    for (int64_t v = (int64_t)blockIdx.x * kBlock + tid; v < n_seg;
         v += (int64_t)gridDim.x * kBlock) {
        const float gd = dnorm_ddeg(deg[v], g_norm[v], power);
        const uint16_t* c = cnt + v * n_rel;
#pragma unroll
        for (int r = 0; r < kDegCntMaxRel; ++r)
            if (r < n_rel) acc[r] = fmaf(gd, float(c[r]), acc[r]);
    }
    for (int l = blockIdx.x * kBlock + tid; l < n_long; l += gridDim.x * kBlock) {
        const int64_t v = long_ids[l];
        const float gd = dnorm_ddeg(deg[v], g_norm[v], power);
#pragma unroll
        for (int r = 0; r < kDegCntMaxRel; ++r)
            if (r < n_rel) acc[r] = fmaf(gd, float(long_cnt[(int64_t)l * n_rel + r]), acc[r]);
    }
    __shared__ float red[kBlock / 64][kDegCntMaxRel];
#pragma unroll
    for (int r = 0; r < kDegCntMaxRel; ++r) {
        const float t = group_sum<64>(acc[r]);
        if ((tid & 63) == 0) red[tid >> 6][r] = t;
    }
    __syncthreads();
    if (tid < n_rel) {
        float t = 0.f;
        for (int w = 0; w < kBlock / 64; ++w) t += red[w][tid];       // fixed order
        slab[(int64_t)blockIdx.x * n_rel + tid] = t;
    }
}

// one block per output column k: fixed-order sum over slab rows
__global__ void __launch_bounds__(kBlock)
rel_reduce_kernel(const float* __restrict__ slab, int64_t n_rows, int32_t width,
                  float* __restrict__ out, int32_t accumulate) {
    // one block per column; thread t sums rows t, t + kBlock, ... (4 independent partials in
    // flight), then the waves combine in a fixed order: deterministic
    __shared__ float part[kBlock / 64];
    const int k = blockIdx.x, tid = threadIdx.x;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int64_t r = tid;
    for (; r + 3 * kBlock < n_rows; r += 4 * kBlock) {
        s0 += slab[r * width + k];
        s1 += slab[(r + kBlock) * width + k];
        s2 += slab[(r + 2 * kBlock) * width + k];
        s3 += slab[(r + 3 * kBlock) * width + k];
    }
    for (; r < n_rows; r += kBlock) s0 += slab[r * width + k];
    float s = group_sum<64>((s0 + s1) + (s2 + s3));
    if ((tid & 63) == 0) part[tid >> 6] = s;
    __syncthreads();
    if (tid == 0) {
        float t = 0.f;
        for (int w = 0; w < kBlock / 64; ++w) t += part[w];
        out[k] = accumulate ? out[k] + t : t;
    }
}

// wide slabs (per-block partials of a whole weight matrix): one thread per column walks the
// rows in order, so a warp reads consecutive columns of one row (coalesced), fixed order
// (rows r * stride, r < n_rows; the second stage of the split reduce below reads stride rps)
__global__ void __launch_bounds__(kBlock)
rel_reduce_wide_kernel(const float* __restrict__ slab, int64_t n_rows, int32_t width,
                       float* __restrict__ out, int32_t accumulate, int64_t stride = 1) {
    const int k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= width) return;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    const int64_t ws = stride * width;
    int64_t r = 0;
    for (; r + 4 <= n_rows; r += 4) {
        s0 += slab[r * ws + k];
        s1 += slab[(r + 1) * ws + k];
        s2 += slab[(r + 2) * ws + k];
        s3 += slab[(r + 3) * ws + k];
    }
    for (; r < n_rows; ++r) s0 += slab[r * ws + k];
    const float t = (s0 + s1) + (s2 + s3);
    out[k] = accumulate ? out[k] + t : t;
}

// first stage of a tall wide slab's reduce: (column k, split s) sums rows [s rps, (s+1) rps) in
// order and leaves the sum in row s rps, which no other thread reads (in place, no scratch);
// blockIdx.y = s fills the chip where one thread per column gives only width / 256 blocks
__global__ void __launch_bounds__(kBlock)
rel_reduce_split_kernel(float* __restrict__ slab, int64_t n_rows, int32_t width, int64_t rps) {
    const int k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= width) return;
    const int64_t r0 = (int64_t)blockIdx.y * rps, r1 = min(n_rows, r0 + rps);
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int64_t r = r0;
    for (; r + 4 <= r1; r += 4) {
        s0 += slab[r * width + k];
        s1 += slab[(r + 1) * width + k];
        s2 += slab[(r + 2) * width + k];
        s3 += slab[(r + 3) * width + k];
    }
    for (; r < r1; ++r) s0 += slab[r * width + k];
    slab[r0 * width + k] = (s0 + s1) + (s2 + s3);
}

// out[u] = scale[u] * drop(x[u]) and optionally dot[u] = <x[u], z[u]> / scale[u]; LPR lanes per
// row, 16 bytes per lane per step (streaming, coalesced). The aggregation then gathers finished
// rows: the dropout mask is hashed N*F times instead of E*F (once per gathered edge) and the
// per-edge scale lookup leaves the gather's dependent load chain. The mask is the
// regnn_spmm_fwd_dropout spec (row, vector index of the row), so regnn_spmm_bwd_dropout with the
// same seed differentiates it. The dot is the output-side norm gradient <g, y_raw> = <g, y>/post
// of the backward, formed here while g streams by.
template <typename T, int LPR, int DROP, int U>
__global__ void __launch_bounds__(kBlock)
row_scale_kernel(const T* __restrict__ x, const float* __restrict__ scale, T* __restrict__ out,
                 int64_t n_rows, int32_t nvec, const uint64_t* __restrict__ drop_seed,
                 uint32_t drop_thresh, float drop_scale, const T* __restrict__ z,
                 float* __restrict__ dot) {
    constexpr int EV = Vec<T>::N;
    constexpr int GPB = kBlock / LPR;
    const int lane = threadIdx.x & (LPR - 1);
    // U rows per group per step (U x 16 B loads in flight per lane; regnn_tune key 4)
    uint32_t key = 0;
    if constexpr (DROP) key = drop_key(drop_seed);
    const int64_t G = (int64_t)gridDim.x * GPB;
    for (int64_t r0 = (int64_t)blockIdx.x * GPB + threadIdx.x / LPR; r0 < n_rows; r0 += G * U) {
        int64_t rr[U];
        bool ok[U];
        float s[U], d[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            ok[u] = r0 + u * G < n_rows;             // group-uniform
            rr[u] = ok[u] ? r0 + u * G : r0;
            s[u] = scale ? scale[rr[u]] : 1.f;
            d[u] = 0.f;
        }
        for (int vec = lane; vec < nvec; vec += LPR) {
            float v[U][EV], w[U][EV];
#pragma unroll
            for (int u = 0; u < U; ++u) Vec<T>::load(x + (rr[u] * nvec + vec) * EV, v[u]);
            if (dot) {
#pragma unroll
                for (int u = 0; u < U; ++u) Vec<T>::load(z + (rr[u] * nvec + vec) * EV, w[u]);
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int t = 0; t < EV; ++t) d[u] = fmaf(v[u][t], w[u][t], d[u]);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
#pragma unroll
                for (int t = 0; t < EV; ++t) v[u][t] *= s[u];
                if constexpr (DROP)
                    drop_apply<EV, DROP>(key, drop_thresh, drop_scale, rr[u], nvec, vec, v[u]);
                if (ok[u]) Vec<T>::store(out + (rr[u] * nvec + vec) * EV, v[u]);
            }
        }
        if (dot) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const float t = group_sum<LPR>(d[u]);
                if (lane == 0 && ok[u]) dot[rr[u]] = t / s[u];
            }
        }
    }
}

template <typename T, int LPR>
int launch_row_scale_lpr(const T* x, const float* scale, T* out, int64_t n_rows, int nvec,
                         const uint64_t* seed, uint32_t keep16, float dscale, const T* z,
                         float* dot, hipStream_t stream) {
    constexpr int GPB = kBlock / LPR;
#define REGNN_ROW_SCALE(D, U)                                                                    \
    hipLaunchKernelGGL((row_scale_kernel<T, LPR, D, U>),                                         \
                       dim3(grid_resident(row_scale_kernel<T, LPR, D, U>, n_rows, GPB, 0)),      \
                       dim3(kBlock), 0, stream, x, scale, out, n_rows, nvec, seed, keep16, dscale, \
                       z, dot)
    if (g_tune_rowscale == 0 || g_tune_rowscale == 1) {
        if (!seed) REGNN_ROW_SCALE(0, 1);
        else if ((keep16 & 0xFFu) == 0) REGNN_ROW_SCALE(8, 1);
        else REGNN_ROW_SCALE(16, 1);
    } else if (g_tune_rowscale == 2) {
        if (!seed) REGNN_ROW_SCALE(0, 2);
        else if ((keep16 & 0xFFu) == 0) REGNN_ROW_SCALE(8, 2);
        else REGNN_ROW_SCALE(16, 2);
    } else {
        if (!seed) REGNN_ROW_SCALE(0, 4);
        else if ((keep16 & 0xFFu) == 0) REGNN_ROW_SCALE(8, 4);
        else REGNN_ROW_SCALE(16, 4);
    }
#undef REGNN_ROW_SCALE
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

template <typename T>
int launch_row_scale(const void* x, const float* scale, void* out, int64_t n_rows, int32_t F,
                     const uint64_t* seed, uint32_t keep16, float dscale, const void* z,
                     float* dot, hipStream_t stream) {
    constexpr int EV = Vec<T>::N;
    if (F % EV) return REGNN_EUNSUPPORTED;
    const int nvec = F / EV;
    const T* xs = static_cast<const T*>(x);
    const T* zs = static_cast<const T*>(z);
    T* o = static_cast<T*>(out);
    if (nvec <= 4)
        return launch_row_scale_lpr<T, 4>(xs, scale, o, n_rows, nvec, seed, keep16, dscale, zs, dot,
                                          stream);
    if (nvec <= 8)
        return launch_row_scale_lpr<T, 8>(xs, scale, o, n_rows, nvec, seed, keep16, dscale, zs, dot,
                                          stream);
    return launch_row_scale_lpr<T, 16>(xs, scale, o, n_rows, nvec, seed, keep16, dscale, zs, dot,
                                       stream);
}

int64_t g_tune_grid_cap = 0;
int64_t g_tune_un = 0;
int64_t g_tune_head = 0;
int64_t g_tune_rowscale = 0;

int resident_blocks(const void* kernel, size_t lds, int block) {
    struct Entry { const void* k; size_t lds; int block; int blocks; };
    static std::mutex mu;
    static Entry cache[64];
    static int n_cache = 0;
    static int n_cu = 0;
    std::lock_guard<std::mutex> lock(mu);
    for (int i = 0; i < n_cache; ++i)
        if (cache[i].k == kernel && cache[i].lds == lds && cache[i].block == block)
            return cache[i].blocks;
    if (n_cu == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            n_cu = 256;
    }
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, lds) != hipSuccess ||
        per_cu <= 0)
        per_cu = 4;
    const int blocks = per_cu * n_cu;
    if (n_cache < 64) cache[n_cache++] = {kernel, lds, block, blocks};
    return blocks;
}

}  // namespace regnn

using namespace regnn;

extern "C" {

int64_t regnn_tune(int32_t key, int64_t value) {
    if (key == 1) {
        const int64_t old = g_tune_grid_cap;
        g_tune_grid_cap = value < 0 ? 0 : value;
        return old;
    }
    if (key == 2) {
        const int64_t old = g_tune_un;
        g_tune_un = value;
        return old;
    }
    if (key == 3) {
        const int64_t old = g_tune_head;
        g_tune_head = value;
        return old;
    }
    if (key == 4) {
        const int64_t old = g_tune_rowscale;
        g_tune_rowscale = value;
        return old;
    }
    return -1;
}

int64_t regnn_slab_rows(int64_t, int32_t) { return 2 * int64_t(kMaxGrid); }

static SpmmArgs make_args(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                          const float* tab, const float* edge_w, const float* in_scale,
                          const float* out_scale, int64_t n_seg, int32_t F, int32_t split,
                          int32_t chunk, const int32_t* long_ids, int32_t n_long,
                          const int32_t* chunk_long, const int32_t* chunk_off, int32_t n_chunk,
                          float* chunk_partial, const int32_t* level_sb, int32_t n_levels,
                          const int64_t* level_desc) {
    SpmmArgs a{};
    a.ptr = ptr; a.idx = idx; a.rel = rel; a.tab = tab; a.edge_w = edge_w;
    a.in_scale = in_scale; a.out_scale = out_scale; a.n_seg = n_seg; a.F = F;
    // split < 0: the scheduled plan form, chunk_long[n_chunk, 2 n_chunk) = the chunk handled
    // in processing slot i (regnn_hip.h, long-segment plans)
    a.split = split < 0 ? -split : split;
    a.chunk_sched = split < 0 ? chunk_long + n_chunk : nullptr;
    a.chunk = chunk; a.long_ids = long_ids; a.n_long = n_long;
    a.chunk_long = chunk_long; a.chunk_off = chunk_off; a.n_chunk = n_chunk;
    a.chunk_partial = chunk_partial;
    a.level_sb = level_sb; a.n_levels = n_levels; a.level_desc = level_desc;
    return a;
}

static int check_common(const int32_t* ptr, const int32_t* idx, const void* src, const void* out,
                        int64_t n_seg, int32_t split, int32_t chunk, const int32_t* long_ids,
                        int32_t n_long, const int32_t* chunk_long, const int32_t* chunk_off,
                        int32_t n_chunk, const float* chunk_partial, const uint8_t* rel,
                        const float* tab) {
    if (n_seg < 0 || !ptr || (n_seg > 0 && (!idx || !src || !out))) return REGNN_EINVAL;
    if (tab && !rel) return REGNN_EINVAL;
    if (split != 0 && n_long > 0 &&
        (chunk <= 0 || !long_ids || !chunk_long || !chunk_off || !chunk_partial || n_chunk <= 0))
        return REGNN_EINVAL;
    return REGNN_OK;
}

static int spmm_fwd_impl(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                         const float* rel_table, const float* edge_w, const float* in_scale,
                         const float* out_scale, const float* bias, const void* x, void* y,
                         int64_t n_seg, int32_t F, int32_t dtype, int32_t split, int32_t chunk,
                         const int32_t* long_ids, int32_t n_long, const int32_t* chunk_long,
                         const int32_t* chunk_off, int32_t n_chunk, float* chunk_partial,
                         const int32_t* level_sb, int32_t n_levels, const int64_t* level_desc,
                         const uint64_t* drop_seed, uint32_t drop_keep16, float drop_scale,
                         const void* residual, const float* ln_w, const float* ln_b,
                         float ln_eps, int32_t epi, hipStream_t stream) {
    int st = check_common(ptr, idx, x, y, n_seg, split, chunk, long_ids, n_long, chunk_long,
                          chunk_off, n_chunk, chunk_partial, rel, rel_table);
    if (st) return st;
    if (n_seg == 0) return REGNN_OK;
    if (n_levels < 0 || (n_levels > 0 && (!level_sb || !level_desc))) return REGNN_EINVAL;
    if (n_long == 0) { split = 0; n_chunk = 0; n_levels = 0; }
    SpmmArgs a = make_args(ptr, idx, rel, rel_table, edge_w, in_scale, out_scale, n_seg, F, split,
                           chunk, long_ids, n_long, chunk_long, chunk_off, n_chunk, chunk_partial,
                           level_sb, n_levels, level_desc);
    a.bias = bias; a.src = x; a.out = y;
    a.drop_seed = drop_seed; a.drop_thresh = drop_keep16; a.drop_scale = drop_scale;
    a.residual = residual; a.ln_w = ln_w; a.ln_b = ln_b; a.ln_eps = ln_eps; a.epi = epi;
    if (dtype == REGNN_F32) return dispatch<float>(a, kFwd, stream);
    if (dtype == REGNN_BF16) return dispatch<bf16_t>(a, kFwd, stream);
    return REGNN_EUNSUPPORTED;
}

static int spmm_fwd_next_impl(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                              const float* rel_table, const float* edge_w, const float* in_scale,
                              const float* out_scale, const float* bias, const void* x, void* y,
                              int64_t n_seg, int32_t F, int32_t dtype, int32_t split,
                              int32_t chunk, const int32_t* long_ids, int32_t n_long,
                              const int32_t* chunk_long, const int32_t* chunk_off,
                              int32_t n_chunk, float* chunk_partial, const int32_t* level_sb,
                              int32_t n_levels, const int64_t* level_desc,
                              const uint64_t* drop_seed, uint32_t drop_keep16, float drop_scale,
                              const float* nx_scale, const uint64_t* nx_seed, uint32_t nx_keep16,
                              float nx_dscale, void* nx_out, hipStream_t stream) {
    int st = check_common(ptr, idx, x, y, n_seg, split, chunk, long_ids, n_long, chunk_long,
                          chunk_off, n_chunk, chunk_partial, rel, rel_table);
    if (st) return st;
    if (!nx_scale || !nx_out || (nx_seed && nx_keep16 > 65536u)) return REGNN_EINVAL;
    if (drop_seed && drop_keep16 > 65536u) return REGNN_EINVAL;
    if (n_seg == 0) return REGNN_OK;
    if (n_levels < 0 || (n_levels > 0 && (!level_sb || !level_desc))) return REGNN_EINVAL;
    if (n_long == 0) { split = 0; n_chunk = 0; n_levels = 0; }
    SpmmArgs a = make_args(ptr, idx, rel, rel_table, edge_w, in_scale, out_scale, n_seg, F, split,
                           chunk, long_ids, n_long, chunk_long, chunk_off, n_chunk, chunk_partial,
                           level_sb, n_levels, level_desc);
    a.bias = bias; a.src = x; a.out = y;
    a.drop_seed = drop_seed; a.drop_thresh = drop_keep16; a.drop_scale = drop_scale;
    a.nx_scale = nx_scale; a.nx_out = nx_out;
    a.nx_seed = nx_seed; a.nx_thresh = nx_keep16; a.nx_dscale = nx_dscale;
    if (dtype == REGNN_F32) return dispatch<float>(a, kFwd, stream);
    if (dtype == REGNN_BF16) return dispatch<bf16_t>(a, kFwd, stream);
    return REGNN_EUNSUPPORTED;
}

static int spmm_bwd_impl(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                         const float* rel_table, const float* edge_w, const float* in_scale,
                         const float* out_scale, const void* g, const void* x, const void* y,
                         void* gx, float* slab, int32_t n_rel, float* edge_grad,
                         float* node_grad, int64_t n_seg, int32_t F, int32_t dtype, int32_t split,
                         int32_t chunk, const int32_t* long_ids, int32_t n_long,
                         const int32_t* chunk_long, const int32_t* chunk_off, int32_t n_chunk,
                         float* chunk_partial, const int32_t* level_sb, int32_t n_levels,
                         const int64_t* level_desc, const uint64_t* drop_seed,
                         uint32_t drop_keep16, float drop_scale, hipStream_t stream,
                         const float* nx_scale = nullptr, void* nx_out = nullptr,
                         float* nx_dot = nullptr) {
    int st = check_common(ptr, idx, g, gx, n_seg, split, chunk, long_ids, n_long, chunk_long,
                          chunk_off, n_chunk, chunk_partial, rel, rel_table);
    if (st) return st;
    if (slab && (!rel || n_rel <= 0 || n_rel > 64)) return REGNN_EINVAL;
    if (nx_scale && (!nx_out || !nx_dot || !x)) return REGNN_EINVAL;
    if ((slab || edge_grad || node_grad) && !x) return REGNN_EINVAL;
    if (n_seg == 0) return REGNN_OK;
    if (n_levels < 0 || (n_levels > 0 && (!level_sb || !level_desc))) return REGNN_EINVAL;
    if (n_long == 0) { split = 0; n_chunk = 0; n_levels = 0; }
    SpmmArgs a = make_args(ptr, idx, rel, rel_table, edge_w, in_scale, out_scale, n_seg, F, split,
                           chunk, long_ids, n_long, chunk_long, chunk_off, n_chunk, chunk_partial,
                           level_sb, n_levels, level_desc);
    a.src = g; a.out = gx; a.self = x; a.ng_a = y ? g : nullptr; a.ng_b = y;
    a.slab = slab; a.n_rel = n_rel; a.edge_grad = edge_grad; a.node_grad = node_grad;
    a.drop_seed = drop_seed; a.drop_thresh = drop_keep16; a.drop_scale = drop_scale;
    a.nx_scale = nx_scale; a.nx_out = nx_out; a.nx_dot = nx_dot;
    if (drop_seed && (slab || edge_grad || node_grad) && !x) return REGNN_EINVAL;
    a.self_pre = (dtype & REGNN_SELF_PRESCALED) ? 1 : 0;
    dtype &= ~REGNN_SELF_PRESCALED;
    if (a.self_pre && (nx_scale || edge_grad)) return REGNN_EINVAL;
    const int mode = slab ? (edge_grad ? kBwdBoth : kBwdSlab) : (edge_grad ? kBwdEdge : kBwd);
    if (dtype == REGNN_F32) return dispatch<float>(a, mode, stream);
    if (dtype == REGNN_BF16) return dispatch<bf16_t>(a, mode, stream);
    return REGNN_EUNSUPPORTED;
}

int regnn_spmm_fwd(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                   const float* rel_table, const float* edge_w, const float* in_scale,
                   const float* out_scale, const float* bias, const void* x, void* y,
                   int64_t n_seg, int32_t F, int32_t dtype, int32_t split, int32_t chunk,
                   const int32_t* long_ids, int32_t n_long, const int32_t* chunk_long,
                   const int32_t* chunk_off, int32_t n_chunk, float* chunk_partial,
                   const int32_t* level_sb, int32_t n_levels, const int64_t* level_desc,
                   hipStream_t stream) {
    return spmm_fwd_impl(ptr, idx, rel, rel_table, edge_w, in_scale, out_scale, bias, x, y, n_seg,
                         F, dtype, split, chunk, long_ids, n_long, chunk_long, chunk_off, n_chunk,
                         chunk_partial, level_sb, n_levels, level_desc, nullptr, 0, 1.f, nullptr,
                         nullptr, nullptr, 0.f, 0, stream);
}

int regnn_spmm_fwd_fused(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                         const float* rel_table, const float* edge_w, const float* in_scale,
                         const float* out_scale, const float* bias, const void* x, void* y,
                         int64_t n_seg, int32_t F, int32_t dtype, int32_t split, int32_t chunk,
                         const int32_t* long_ids, int32_t n_long, const int32_t* chunk_long,
                         const int32_t* chunk_off, int32_t n_chunk, float* chunk_partial,
                         const int32_t* level_sb, int32_t n_levels, const int64_t* level_desc,
                         const void* residual, const float* ln_w, const float* ln_b,
                         float ln_eps, int32_t epi, hipStream_t stream) {
    if (epi & ~(kEpiLN | kEpiReLU)) return REGNN_EINVAL;
    if ((epi & kEpiLN) && !(ln_eps > 0.f)) return REGNN_EINVAL;
    return spmm_fwd_impl(ptr, idx, rel, rel_table, edge_w, in_scale, out_scale, bias, x, y, n_seg,
                         F, dtype, split, chunk, long_ids, n_long, chunk_long, chunk_off, n_chunk,
                         chunk_partial, level_sb, n_levels, level_desc, nullptr, 0, 1.f, residual,
                         ln_w, ln_b, ln_eps, epi, stream);
}

int regnn_spmm_fwd_dropout(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                           const float* rel_table, const float* edge_w, const float* in_scale,
                           const float* out_scale, const float* bias, const void* x, void* y,
                           int64_t n_seg, int32_t F, int32_t dtype, int32_t split, int32_t chunk,
                           const int32_t* long_ids, int32_t n_long, const int32_t* chunk_long,
                           const int32_t* chunk_off, int32_t n_chunk, float* chunk_partial,
                           const int32_t* level_sb, int32_t n_levels, const int64_t* level_desc,
                           const uint64_t* drop_seed, uint32_t drop_keep16, float drop_scale,
                           hipStream_t stream) {
    if (!drop_seed || drop_keep16 > 65536u) return REGNN_EINVAL;
    return spmm_fwd_impl(ptr, idx, rel, rel_table, edge_w, in_scale, out_scale, bias, x, y, n_seg,
                         F, dtype, split, chunk, long_ids, n_long, chunk_long, chunk_off, n_chunk,
                         chunk_partial, level_sb, n_levels, level_desc, drop_seed, drop_keep16,
                         drop_scale, nullptr, nullptr, nullptr, 0.f, 0, stream);
}

int regnn_spmm_fwd_next(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                        const float* rel_table, const float* edge_w, const float* in_scale,
                        const float* out_scale, const float* bias, const void* x, void* y,
                        int64_t n_seg, int32_t F, int32_t dtype, int32_t split, int32_t chunk,
                        const int32_t* long_ids, int32_t n_long, const int32_t* chunk_long,
                        const int32_t* chunk_off, int32_t n_chunk, float* chunk_partial,
                        const int32_t* level_sb, int32_t n_levels, const int64_t* level_desc,
                        const uint64_t* drop_seed, uint32_t drop_keep16, float drop_scale,
                        const float* nx_scale, const uint64_t* nx_seed, uint32_t nx_keep16,
                        float nx_dscale, void* nx_out, hipStream_t stream) {
    return spmm_fwd_next_impl(ptr, idx, rel, rel_table, edge_w, in_scale, out_scale, bias, x, y,
                              n_seg, F, dtype, split, chunk, long_ids, n_long, chunk_long,
                              chunk_off, n_chunk, chunk_partial, level_sb, n_levels, level_desc,
                              drop_seed, drop_keep16, drop_scale, nx_scale, nx_seed, nx_keep16,
                              nx_dscale, nx_out, stream);
}

int regnn_spmm_bwd(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                   const float* rel_table, const float* edge_w, const float* in_scale,
                   const float* out_scale, const void* g, const void* x, const void* y, void* gx,
                   float* slab, int32_t n_rel, float* edge_grad, float* node_grad,
                   int64_t n_seg, int32_t F, int32_t dtype, int32_t split, int32_t chunk,
                   const int32_t* long_ids, int32_t n_long, const int32_t* chunk_long,
                   const int32_t* chunk_off, int32_t n_chunk, float* chunk_partial,
                   const int32_t* level_sb, int32_t n_levels, const int64_t* level_desc,
                   hipStream_t stream) {
    return spmm_bwd_impl(ptr, idx, rel, rel_table, edge_w, in_scale, out_scale, g, x, y, gx, slab,
                         n_rel, edge_grad, node_grad, n_seg, F, dtype, split, chunk, long_ids,
                         n_long, chunk_long, chunk_off, n_chunk, chunk_partial, level_sb,
                         n_levels, level_desc, nullptr, 0, 1.f, stream);
}

int regnn_spmm_bwd_dropout(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                           const float* rel_table, const float* edge_w, const float* in_scale,
                           const float* out_scale, const void* g, const void* x, const void* y,
                           void* gx, float* slab, int32_t n_rel, float* edge_grad,
                           float* node_grad, int64_t n_seg, int32_t F, int32_t dtype,
                           int32_t split, int32_t chunk, const int32_t* long_ids, int32_t n_long,
                           const int32_t* chunk_long, const int32_t* chunk_off, int32_t n_chunk,
                           float* chunk_partial, const int32_t* level_sb, int32_t n_levels,
                           const int64_t* level_desc, const uint64_t* drop_seed,
                           uint32_t drop_keep16, float drop_scale, hipStream_t stream) {
    if (!drop_seed || drop_keep16 > 65536u) return REGNN_EINVAL;
    return spmm_bwd_impl(ptr, idx, rel, rel_table, edge_w, in_scale, out_scale, g, x, y, gx, slab,
                         n_rel, edge_grad, node_grad, n_seg, F, dtype, split, chunk, long_ids,
                         n_long, chunk_long, chunk_off, n_chunk, chunk_partial, level_sb,
                         n_levels, level_desc, drop_seed, drop_keep16, drop_scale, stream);
}

int regnn_spmm_bwd_next(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                        const float* rel_table, const float* edge_w, const float* in_scale,
                        const float* out_scale, const void* g, const void* x, const void* y,
                        void* gx, float* slab, int32_t n_rel, float* edge_grad, float* node_grad,
                        int64_t n_seg, int32_t F, int32_t dtype, int32_t split, int32_t chunk,
                        const int32_t* long_ids, int32_t n_long, const int32_t* chunk_long,
                        const int32_t* chunk_off, int32_t n_chunk, float* chunk_partial,
                        const int32_t* level_sb, int32_t n_levels, const int64_t* level_desc,
                        const uint64_t* drop_seed, uint32_t drop_keep16, float drop_scale,
                        const float* nx_scale, void* nx_out, float* nx_dot, hipStream_t stream) {
    if (!nx_scale || (drop_seed && drop_keep16 > 65536u)) return REGNN_EINVAL;
    return spmm_bwd_impl(ptr, idx, rel, rel_table, edge_w, in_scale, out_scale, g, x, y, gx, slab,
                         n_rel, edge_grad, node_grad, n_seg, F, dtype, split, chunk, long_ids,
                         n_long, chunk_long, chunk_off, n_chunk, chunk_partial, level_sb,
                         n_levels, level_desc, drop_seed, drop_keep16, drop_scale, stream,
                         nx_scale, nx_out, nx_dot);
}

int regnn_row_scale(const void* x, const float* scale, void* out, int64_t n_rows, int32_t F,
                    int32_t dtype, const uint64_t* drop_seed, uint32_t drop_keep16,
                    float drop_scale, const void* z, float* dot, hipStream_t stream) {
    if (n_rows < 0 || F <= 0 || (n_rows > 0 && (!x || !out))) return REGNN_EINVAL;
    if (drop_seed && drop_keep16 > 65536u) return REGNN_EINVAL;
    if ((dot != nullptr) != (z != nullptr)) return REGNN_EINVAL;
    if (n_rows == 0) return REGNN_OK;
    if (dtype == REGNN_F32)
        return launch_row_scale<float>(x, scale, out, n_rows, F, drop_seed, drop_keep16,
                                       drop_scale, z, dot, stream);
    if (dtype == REGNN_BF16)
        return launch_row_scale<bf16_t>(x, scale, out, n_rows, F, drop_seed, drop_keep16,
                                        drop_scale, z, dot, stream);
    return REGNN_EUNSUPPORTED;
}

int regnn_degree(const int32_t* ptr, const uint8_t* rel, const float* rel_table, int64_t n_seg,
                 float power, int32_t split, const int32_t* long_ids, int32_t n_long,
                 const int32_t* long_cnt, int32_t n_rel, float* deg, float* norm,
                 hipStream_t stream) {
    if (!ptr || !deg || n_seg < 0 || (rel_table && !rel)) return REGNN_EINVAL;
    if (split > 0 && n_long > 0 && (!long_ids || (rel_table && !long_cnt))) return REGNN_EINVAL;
    if (n_seg == 0) return REGNN_OK;
    if (n_long == 0) split = 0;
    if (rel_table && (n_rel <= 0 || n_rel > 256)) return REGNN_EINVAL;
    hipLaunchKernelGGL(degree_kernel, dim3(grid_resident(degree_kernel, n_seg, kBlock, 0)),
                       dim3(kBlock), 0, stream, ptr, rel, rel_table, n_rel, n_seg, power, split,
                       deg, norm);
    REGNN_LAUNCH_CHECK();
    if (split > 0) {
        hipLaunchKernelGGL(degree_long_kernel, dim3(grid_for(n_long, kBlock)), dim3(kBlock), 0,
                           stream, ptr, rel_table, long_ids, n_long, long_cnt, n_rel, power, deg,
                           norm);
        REGNN_LAUNCH_CHECK();
    }
    return REGNN_OK;
}

int regnn_degree_bwd(const int32_t* ptr, const uint8_t* rel, const float* deg, const float* g_norm,
                     int64_t n_seg, float power, int32_t n_rel, int32_t split,
                     const int32_t* long_ids, int32_t n_long, const int32_t* long_cnt,
                     float* slab, hipStream_t stream) {
    if (!ptr || !rel || !deg || !g_norm || !slab || n_rel <= 0 || n_rel > 64) return REGNN_EINVAL;
    if (split > 0 && n_long > 0 && (!long_ids || !long_cnt)) return REGNN_EINVAL;
    if (n_seg == 0) return REGNN_OK;
    if (n_long == 0) split = 0;
    const size_t lds = size_t(n_rel) * kBlock * sizeof(float);
    hipLaunchKernelGGL(degree_bwd_kernel,
                       dim3(grid_resident(degree_bwd_kernel, n_seg, kBlock, lds)),
                       dim3(kBlock), lds, stream,
                       ptr, rel, deg, g_norm, n_seg, power, n_rel, split, long_ids,
                       split > 0 ? n_long : 0, long_cnt, slab);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

int regnn_degree_cnt(const uint16_t* cnt, const float* rel_table, int32_t n_rel, int64_t n_seg,
                     float power, const int32_t* ptr, const int32_t* long_ids, int32_t n_long,
                     const int32_t* long_cnt, float* deg, float* norm, hipStream_t stream) {
    if (!cnt || !rel_table || !deg || n_seg < 0 || n_rel <= 0 || n_rel > kDegCntMaxRel ||
        (n_long > 0 && (!ptr || !long_ids || !long_cnt)))
        return REGNN_EINVAL;
    if (n_seg == 0) return REGNN_OK;
    hipLaunchKernelGGL(degree_cnt_kernel, dim3(grid_resident(degree_cnt_kernel, n_seg, kBlock, 0)),
                       dim3(kBlock), 0, stream, cnt, rel_table, n_rel, n_seg, power, deg, norm);
    REGNN_LAUNCH_CHECK();
    if (n_long > 0) {
        hipLaunchKernelGGL(degree_long_kernel, dim3(grid_for(n_long, kBlock)), dim3(kBlock), 0,
                           stream, ptr, rel_table, long_ids, n_long, long_cnt, n_rel, power, deg,
                           norm);
        REGNN_LAUNCH_CHECK();
    }
    return REGNN_OK;
}

int regnn_degree_cnt_bwd(const uint16_t* cnt, const float* deg, const float* g_norm,
                         int64_t n_seg, float power, int32_t n_rel, const int32_t* long_ids,
                         int32_t n_long, const int32_t* long_cnt, float* slab,
                         hipStream_t stream) {
    if (!cnt || !deg || !g_norm || !slab || n_seg < 0 || n_rel <= 0 || n_rel > kDegCntMaxRel ||
        (n_long > 0 && (!long_ids || !long_cnt)))
        return REGNN_EINVAL;
    if (n_seg == 0 && n_long == 0) return REGNN_OK;
    hipLaunchKernelGGL(degree_cnt_bwd_kernel,
                       dim3(grid_resident(degree_cnt_bwd_kernel, n_seg, kBlock, 0)),
                       dim3(kBlock), 0, stream, cnt, deg, g_norm, n_seg, power, n_rel, long_ids,
                       n_long, long_cnt, slab);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

int regnn_rel_reduce(float* slab, int64_t n_rows, int32_t width, float* out,
                     int32_t accumulate, hipStream_t stream) {
    if (!slab || !out || width <= 0 || n_rows < 0) return REGNN_EINVAL;
    const int64_t cols = (width + kBlock - 1) / kBlock;
    if (width >= 4096 && n_rows >= 256) {
        // split rows so that ~2048 blocks run, >= 32 rows per split
        int64_t splits = (2048 + cols - 1) / cols;
        if (splits > n_rows / 32) splits = n_rows / 32;
        const int64_t rps = (n_rows + splits - 1) / splits;
        splits = (n_rows + rps - 1) / rps;
        hipLaunchKernelGGL(rel_reduce_split_kernel, dim3((unsigned)cols, (unsigned)splits),
                           dim3(kBlock), 0, stream, slab, n_rows, width, rps);
        REGNN_LAUNCH_CHECK();
        hipLaunchKernelGGL(rel_reduce_wide_kernel, dim3((unsigned)cols), dim3(kBlock), 0, stream,
                           slab, splits, width, out, accumulate, rps);
    } else if (width >= 4096)
        hipLaunchKernelGGL(rel_reduce_wide_kernel, dim3((unsigned)cols), dim3(kBlock), 0, stream,
                           slab, n_rows, width, out, accumulate, (int64_t)1);
    else
        hipLaunchKernelGGL(rel_reduce_kernel, dim3(width), dim3(kBlock), 0, stream, slab, n_rows,
                           width, out, accumulate);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

}  // extern "C"
