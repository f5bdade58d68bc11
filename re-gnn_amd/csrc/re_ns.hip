// Device-resident neighbour-sampled (NS) pipeline for the ogbn-mag path (mag/regnn_ns.py):
// the per-batch sampler that replaces torch_sparse sample_adj behind PyG NeighborSampler
// (mag/regnn_ns.py:206-214, consumed at :399-401), built so that a whole NS training step runs
// with no host synchronisation and can be captured in a HIP graph:
//
//  * every buffer is sized by its capacity (batch B, fan-outs k_h): targets of hop h fill
//    n_id[0, n_h), the hop appends its new nodes at n_id[n_h, n_{h+1}); the counts live in a
//    device int32 array `sizes` ([h] = n_h, [8 + h] = edges of hop h's block incl. self loops);
//  * the sampled block of a hop is written straight in the layout its aggregation reads: CSR by
//    target (local ids), the target's self loop last in its row (mag/regnn_layers.py:90-96),
//    0-based relation ids (edge type, or num_edge_types + node type for the loop), 1/in-count;
//  * first-seen de-duplication without sorting: a direct-mapped table over the global node ids
//    (g2l: stamp << 32 | local id; first: (~stamp) << 32 | block position, 64-bit atomicMin).
//    Entries carry the hop's stamp, so nothing is reset between hops or steps;
//  * the flag scan runs tile-parallel with the tile offsets scanned by the last tile to finish.
//
// Sampler spec (bit-identical to oracle/sampler_oracle.py and to regnn_sample_fill): Floyd
// sampling of k distinct in-edge positions per target with hash(seed, t, j), ascending order;
// n_id = targets, then new sources in first-seen order over the target-major edge list.
#include "regnn_common.h"

#include <cstdlib>

namespace regnn {

constexpr int kNsTile = 1024;        // block positions per flag tile (256 threads x 4)

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}

// per-(epoch, global batch, hop) seed: sampler_oracle.hop_seed
__device__ __forceinline__ uint64_t ns_hop_seed(const int64_t* state, int hop) {
    const uint64_t base = uint64_t(state[0]), epoch = uint64_t(state[1]),
                   batch = uint64_t(state[3]);
    return mix64(base ^ mix64((epoch << 40) ^ (batch << 8) ^ uint64_t(hop)));
}

__device__ __forceinline__ uint32_t ns_stamp(const int64_t* state, int hop) {
    return uint32_t(uint64_t(state[4]) * 8u + uint64_t(hop) + 1u);
}

__device__ __forceinline__ uint32_t ns_hash(uint64_t seed, uint64_t t, uint64_t j) {
    return uint32_t(mix64(seed + 0x9E3779B97F4A7C15ull * (t + 1) + 0xD1B54A32D192ED03ull * (j + 1))
                    >> 32);
}

// exclusive block scan of one int per thread; *total = block sum. lds: NT / 64 + 1 ints.
template <int NT>
__device__ __forceinline__ int block_exscan(int v, int* lds, int* total) {
    constexpr int NW = NT / 64;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) lds[w] = x;
    __syncthreads();
    if (w == 0) {
        const int s = lane < NW ? lds[lane] : 0;
        int t = s;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(t, o, 64);
            if (lane >= o) t += y;
        }
        if (lane < NW) lds[lane] = t - s;
        if (lane == NW - 1) lds[NW] = t;
    }
    __syncthreads();
    const int r = x - v + lds[w];
    *total = lds[NW];
    __syncthreads();
    return r;
}

// step prologue: the targets of this rank's next batch (rank r of W takes global batches r,
// r+W, ... of the epoch permutation; a rank past the last batch wraps, so every rank runs the
// same number of steps), the batch id the hop seeds use, a new dedup stamp.
__global__ void __launch_bounds__(kBlock)
ns_batch_kernel(const int64_t* __restrict__ perm, int64_t n_perm, int B, int rank, int world,
                int64_t* __restrict__ state, int32_t* __restrict__ n_id,
                int32_t* __restrict__ sizes, int64_t* __restrict__ stamp_src) {
    __shared__ int64_t s_start, s_cnt;
    if (threadIdx.x == 0) {
        const int64_t nb = (n_perm + B - 1) / B;
        const int64_t j = state[2];
        int64_t g = int64_t(rank) + j * int64_t(world);
        if (nb > 0) g %= nb;
        const int64_t start = g * B;
        int64_t cnt = n_perm - start;
        if (cnt > B) cnt = B;
        if (cnt < 0) cnt = 0;
        s_start = start;
        s_cnt = cnt;
        state[3] = g;
        state[2] = j + 1;
        if (stamp_src) {                   // a counter shared by several samplers of one table
            const int64_t st = stamp_src[0] + 1;
            stamp_src[0] = st;
            state[4] = st;
        } else {
            state[4] = state[4] + 1;
        }
        sizes[0] = int32_t(cnt);
    }
    if (threadIdx.x < 8) sizes[8 + threadIdx.x] = 0;   // strided hops add their edges per block
    __syncthreads();
    for (int i = threadIdx.x; i < s_cnt; i += blockDim.x) n_id[i] = int32_t(perm[s_start + i]);
}

// one wave per target: Floyd sampling (regnn_sample_fill's spec) into fixed-stride slots
__global__ void __launch_bounds__(kBlock)
ns_sample_kernel(const int32_t* __restrict__ ptr, const int32_t* __restrict__ idx,
                 const int32_t* __restrict__ n_id, const int32_t* __restrict__ sizes, int hop,
                 int cap, int k, const int64_t* __restrict__ state, uint64_t* __restrict__ g2l,
                 int32_t* __restrict__ samp, int32_t* __restrict__ spos,
                 int32_t* __restrict__ scnt) {
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    if (i >= cap) return;
    const int n = sizes[hop];
    if (i >= n) {
        if (lane == 0) scnt[i] = 0;
        return;
    }
    const uint32_t stamp = ns_stamp(state, hop);
    const uint64_t seed = ns_hop_seed(state, hop);
    const int t = n_id[i];
    if (lane == 0) g2l[t] = (uint64_t(stamp) << 32) | uint32_t(i);
    const int b = ptr[t], d = ptr[t + 1] - b;
    const int64_t o = int64_t(i) * k;
    if (d <= k) {
        for (int q = lane; q < d; q += 64) {
            samp[o + q] = idx[b + q];
            spos[o + q] = b + q;
        }
        if (lane == 0) scnt[i] = d;
        return;
    }
    int slot = -1;
    // lane i < k forms draw i's position up front (one hash per lane instead of k); the Floyd
    // resolution then walks the draws in order
    const int jl = d - k + lane;
    const int my_pos = lane < k ? int((uint64_t(ns_hash(seed, uint64_t(t), uint64_t(jl))) *
                                       uint64_t(jl + 1)) >> 32) : 0;
    for (int i = 0; i < k; ++i) {
        const int pos = __shfl(my_pos, i, 64);
        const bool seen = __any(slot == pos);
        if (lane == i) slot = seen ? d - k + i : pos;
    }
    int rank = 0;
    for (int m = 0; m < k; ++m) {
        const int other = __shfl(slot, m, 64);
        rank += (lane < k && other < slot) ? 1 : 0;
    }
    if (lane < k) {
        samp[o + rank] = idx[b + slot];
        spos[o + rank] = b + slot;
    }
    if (lane == 0) scnt[i] = k;
}

// Strided layout (the fused engine's blocks): row i owns slots [i S, i S + S), S = k + 1 -- its
// sampled edges in ascending position order, then its self loop at i S + cnt_i, the rest empty
// (gsrc -2, blk_idx -1). A slot's position is known at sampling time, so the sampling wave also
// writes what ns_rows_kernel + ns_place_kernel write in the CSR layout (no prefix scan): relation,
// CSR position, target row, the dedup candidate (first-seen order over the slots = the CSR order
// restricted to the edges); meta-only (lean): the source's type / table row instead. Edge counts
// are added per block into sizes[8 + hop] (zeroed by ns_batch_kernel / set_targets) and state[5].
// G lanes per target: 64, or 32 (two targets per wave) when the row's k + 1 slots fit in 32 lanes
// (fan-outs <= 31: half the waves and half the sampling instructions of a hop)
constexpr int kNsStrWaves = 16;            // waves per block

template <int G>
__global__ void __launch_bounds__(64 * kNsStrWaves)
ns_sample_strided_kernel(const int32_t* __restrict__ ptr, const int32_t* __restrict__ idx,
                         const uint8_t* __restrict__ etype, const int32_t* __restrict__ ntype,
                         int num_edge_types, const int32_t* __restrict__ n_id,
                         int32_t* __restrict__ sizes, int hop, int cap, int k,
                         int64_t* __restrict__ state, uint64_t* __restrict__ g2l,
                         uint64_t* __restrict__ first, int32_t* __restrict__ scnt,
                         int32_t* __restrict__ gsrc, int32_t* __restrict__ blk_idx,
                         uint8_t* __restrict__ blk_rel, int32_t* __restrict__ blk_pos,
                         int32_t* __restrict__ blk_row, float* __restrict__ inv,
                         const int64_t* __restrict__ local, int32_t* __restrict__ e_type,
                         int64_t* __restrict__ e_off, int lean, int32_t* __restrict__ csc_cnt) {
    constexpr int TPW = 64 / G;                // targets per wave
    __shared__ int wsum[kNsStrWaves * TPW];
    const int wl = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int lane = wl % G, tl = wv * TPW + wl / G;   // lane within the target's group
    const uint64_t gmask = G == 64 ? ~0ull : (0xFFFFFFFFull << (wl & 32));
    const int i = blockIdx.x * (kNsStrWaves * TPW) + tl;
    const int n = sizes[hop];
    const int S = k + 1;
    const int64_t base = int64_t(i) * S;
    if (csc_cnt && i < cap)                    // the transposed index's counters (resolve adds)
        for (int q = lane; q < S; q += G) csc_cnt[base + q] = 0;
    int cnt = -1;                              // -1: no row (past the batch)
    if (i < cap && i >= n) {
        if (!lean)
            for (int q = lane; q < S; q += G) {
                gsrc[base + q] = -2;
                blk_idx[base + q] = -1;
            }
        if (lane == 0) {
            scnt[i] = 0;
            inv[i] = 1.f;
        }
    } else if (i < n) {
        const uint32_t stamp = ns_stamp(state, hop);
        const uint64_t seed = ns_hop_seed(state, hop);
        const int t = n_id[i];
        if (!lean && lane == 0) g2l[t] = (uint64_t(stamp) << 32) | uint32_t(i);
        const int b = ptr[t], d = ptr[t + 1] - b;
        cnt = d < k ? d : k;
        int slot = lane < d ? lane : -1, rank = lane;  // deg <= k: every position, in order
        if (d > k) {                               // Floyd (regnn_sample_fill's spec)
            slot = -1;
            const int jl = d - k + lane;         // draw i's position formed by lane i up front
            const int my_pos = lane < k ? int((uint64_t(ns_hash(seed, uint64_t(t), uint64_t(jl))) *
                                               uint64_t(jl + 1)) >> 32) : 0;
            for (int i = 0; i < k; ++i) {
                const int pos = __shfl(my_pos, i, G);
                const bool seen = (__ballot(slot == pos) & gmask) != 0;
                if (lane == i) slot = seen ? d - k + i : pos;
            }
            rank = 0;
            for (int m = 0; m < k; ++m) {
                const int other = __shfl(slot, m, G);
                rank += (lane < k && other < slot) ? 1 : 0;
            }
        }
        if (lane < cnt) {
            const int p = b + slot;
            const int u = idx[p];
            const int64_t bp = base + rank;
            blk_rel[bp] = etype[p];
            if (lean) {
                e_type[bp] = ntype[u];
                e_off[bp] = local[u];
            } else {
                gsrc[bp] = u;
                blk_pos[bp] = p;
                blk_row[bp] = i;
                if (uint32_t(g2l[u] >> 32) != stamp)      // not (yet) known as a target: a
                    atomicMin(reinterpret_cast<unsigned long long*>(first + u),   // candidate
                              (unsigned long long)((uint64_t(~stamp) << 32) | uint32_t(bp)));
            }
        } else if (lane == cnt) {                  // the self loop closes the row
            const int64_t bp = base + cnt;
            const int tt = ntype[t];
            blk_rel[bp] = uint8_t(num_edge_types + tt);
            if (lean || e_type) {
                e_type[bp] = tt;
                e_off[bp] = local[t];
            }
            if (!lean) {
                gsrc[bp] = -1;
                blk_idx[bp] = i;
                blk_pos[bp] = -1;
                blk_row[bp] = i;
            }
        } else if (!lean && lane < S) {
            gsrc[base + lane] = -2;
            blk_idx[base + lane] = -1;
        }
        if (lane == 0) {
            scnt[i] = cnt;
            inv[i] = 1.f / float(cnt + 1);
        }
    }
    if (lane == 0) wsum[tl] = cnt + 1;          // edges of the row, self loop included
    __syncthreads();
    if (threadIdx.x == 0) {
        int e = 0;
#pragma unroll
        for (int q = 0; q < kNsStrWaves * TPW; ++q) e += wsum[q];
        if (e) {
            atomicAdd(sizes + 8 + hop, e);
            atomicAdd(reinterpret_cast<unsigned long long*>(state + 5), (unsigned long long)e);
        }
        if (lean && blockIdx.x == 0) sizes[hop + 1] = n;
    }
}

// row offsets (sampled count + the self loop), 1/in-count and the self-loop entries: one tile of
// kNsRowsTile rows per block, the tiles' exclusive prefix by decoupled look-back (integer sums:
// exact in any order). status[tile] = stamp << 32 | kind << 30 | value, kind 1 = the tile's own
// count, 2 = inclusive prefix; entries of another stamp are stale (nothing is reset between
// steps). A block only waits on lower tiles, which were dispatched before it.
constexpr int kNsRowsIT = 4;
constexpr int kNsRowsTile = kBlock * kNsRowsIT;

__device__ __forceinline__ uint64_t lb_pack(uint32_t stamp, uint32_t kind, uint32_t v) {
    return (uint64_t(stamp) << 32) | (uint64_t(kind) << 30) | uint64_t(v);
}

__global__ void __launch_bounds__(kBlock)
ns_rows_kernel(const int32_t* __restrict__ scnt, const int32_t* __restrict__ n_id,
               const int32_t* __restrict__ ntype, int num_edge_types, int32_t* __restrict__ sizes,
               int hop, int cap, int64_t* __restrict__ state, int32_t* __restrict__ blk_ptr,
               int32_t* __restrict__ blk_idx, uint8_t* __restrict__ blk_rel,
               int32_t* __restrict__ blk_pos, int32_t* __restrict__ blk_row,
               int32_t* __restrict__ gsrc, float* __restrict__ inv,
               uint64_t* __restrict__ status, const int64_t* __restrict__ local,
               int32_t* __restrict__ e_type, int64_t* __restrict__ e_off, int lean,
               int32_t* __restrict__ csc_cnt, int cap_e) {
    __shared__ int lds[kBlock / 64 + 1];
    __shared__ int s_prefix;
    if (csc_cnt)                       // the transposed index's per-source counters (resolve adds)
        for (int i = blockIdx.x * kBlock + threadIdx.x; i < cap_e; i += gridDim.x * kBlock)
            csc_cnt[i] = 0;
    const int n = sizes[hop];
    const uint32_t stamp = ns_stamp(state, hop);
    const int tile = blockIdx.x;
    const int i0 = tile * kNsRowsTile + threadIdx.x * kNsRowsIT;
    int vals[kNsRowsIT], rels[kNsRowsIT], gids[kNsRowsIT];
    int64_t offs[kNsRowsIT];
    int s = 0;
#pragma unroll
    for (int j = 0; j < kNsRowsIT; ++j) {
        const int i = i0 + j;
        const bool live = i < cap && i < n;
        vals[j] = live ? scnt[i] + 1 : 0;
        gids[j] = live ? n_id[i] : 0;
        s += vals[j];
    }
#pragma unroll
    for (int j = 0; j < kNsRowsIT; ++j) {
        rels[j] = vals[j] ? ntype[gids[j]] : 0;
        offs[j] = vals[j] && local ? local[gids[j]] : 0;
    }
    int total;
    const int ex = block_exscan<kBlock>(s, lds, &total);
    if (threadIdx.x == 0) {
        int prefix = 0;
        if (tile == 0) {
            __hip_atomic_store(status, lb_pack(stamp, 2u, uint32_t(total)), __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __hip_atomic_store(status + tile, lb_pack(stamp, 1u, uint32_t(total)),
                               __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            for (int p = tile - 1; p >= 0;) {
                const uint64_t st =
                    __hip_atomic_load(status + p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                if (uint32_t(st >> 32) != stamp) continue;            // not yet published
                prefix += int(st & 0x3FFFFFFFu);
                if (((st >> 30) & 3u) == 2u) break;
                --p;
            }
            __hip_atomic_store(status + tile, lb_pack(stamp, 2u, uint32_t(prefix + total)),
                               __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
        s_prefix = prefix;
    }
    __syncthreads();
    int off = s_prefix + ex;
#pragma unroll
    for (int j = 0; j < kNsRowsIT; ++j) {
        const int i = i0 + j;
        if (i < cap) {
            blk_ptr[i] = off;
            if (i < n) {
                const int lp = off + vals[j] - 1;      // the self loop closes the row
                blk_idx[lp] = i;
                blk_rel[lp] = uint8_t(rels[j] + num_edge_types);
                blk_pos[lp] = -1;
                blk_row[lp] = i;
                gsrc[lp] = -1;
                inv[i] = 1.f / float(vals[j]);
                if (e_type) {
                    e_type[lp] = rels[j];
                    e_off[lp] = offs[j];
                }
            } else {
                inv[i] = 1.f;
            }
        }
        off += vals[j];
    }
    if (tile == int(gridDim.x) - 1 && threadIdx.x == 0) {
        const int E = s_prefix + total;
        blk_ptr[cap] = E;
        sizes[8 + hop] = E;
        state[5] += E;
        if (lean) sizes[hop + 1] = n;  // meta-only hop: no new nodes are recorded
    }
}

__device__ __forceinline__ uint64_t first_key(uint32_t stamp, int bp) {
    return (uint64_t(~stamp) << 32) | uint32_t(bp);
}

// sampled slots -> block positions; candidate first occurrences of non-target sources
__global__ void __launch_bounds__(kBlock)
ns_place_kernel(const int32_t* __restrict__ samp, const int32_t* __restrict__ spos,
                const int32_t* __restrict__ scnt, const int32_t* __restrict__ sizes, int hop,
                int cap, int k, const int64_t* __restrict__ state, const uint8_t* __restrict__ etype,
                const uint64_t* __restrict__ g2l, uint64_t* __restrict__ first,
                const int32_t* __restrict__ blk_ptr, uint8_t* __restrict__ blk_rel,
                int32_t* __restrict__ blk_pos, int32_t* __restrict__ blk_row,
                int32_t* __restrict__ gsrc,
                const int32_t* __restrict__ ntype, const int64_t* __restrict__ local,
                int32_t* __restrict__ e_type, int64_t* __restrict__ e_off, int lean) {
    const int64_t s = int64_t(blockIdx.x) * kBlock + threadIdx.x;
    if (s >= int64_t(cap) * k) return;
    const int i = int(s / k), r = int(s - int64_t(i) * k);
    if (i >= sizes[hop] || r >= scnt[i]) return;
    const int bp = blk_ptr[i] + r;
    const int u = samp[s], p = spos[s];
    gsrc[bp] = u;
    blk_rel[bp] = etype[p];
    blk_pos[bp] = p;
    blk_row[bp] = i;
    if (lean) {                        // meta-only hop: the source's type and table row, no dedup
        e_type[bp] = ntype[u];
        e_off[bp] = local[u];
        return;
    }
    const uint32_t stamp = ns_stamp(state, hop);
    if (uint32_t(g2l[u] >> 32) != stamp)
        atomicMin(reinterpret_cast<unsigned long long*>(first + u),
                  (unsigned long long)first_key(stamp, bp));
}

// first-occurrence flags per tile, tile counts; the last tile scans the tile counts and writes
// n_{h+1}
__global__ void __launch_bounds__(kBlock)
ns_flags_kernel(const int32_t* __restrict__ gsrc, int32_t* __restrict__ sizes, int hop,
                const int64_t* __restrict__ state, const uint64_t* __restrict__ g2l,
                const uint64_t* __restrict__ first, uint8_t* __restrict__ flag,
                int32_t* __restrict__ tiles, int n_tiles, int cap_strided) {
    __shared__ int lds[kBlock / 64 + 1];
    __shared__ bool last;
    const int E = cap_strided ? cap_strided : sizes[8 + hop];
    const uint32_t stamp = ns_stamp(state, hop);
    const int base = blockIdx.x * kNsTile + threadIdx.x * 4;
    int c = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int bp = base + j;
        if (bp < E) {
            const int u = gsrc[bp];
            const bool f = u >= 0 && uint32_t(g2l[u] >> 32) != stamp &&
                           first[u] == first_key(stamp, bp);
            flag[bp] = f ? 1 : 0;
            c += f ? 1 : 0;
        }
    }
    int total;
    block_exscan<kBlock>(c, lds, &total);
    if (threadIdx.x == 0) {
        tiles[blockIdx.x] = total;
        __threadfence();
        const int ticket = atomicAdd(tiles + n_tiles, 1);
        last = ticket == int(gridDim.x) - 1;
    }
    __syncthreads();
    if (!last) return;
    __threadfence();
    int carry = 0;
    for (int b0 = 0; b0 < int(gridDim.x); b0 += kBlock) {
        const int b = b0 + threadIdx.x;
        const int v = b < int(gridDim.x) ? reinterpret_cast<volatile int32_t*>(tiles)[b] : 0;
        int tot;
        const int ex = block_exscan<kBlock>(v, lds, &tot);
        if (b < int(gridDim.x)) tiles[b] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) {
        sizes[hop + 1] = sizes[hop] + carry;
        tiles[n_tiles] = 0;
    }
}

// new nodes: n_id append and their local id in g2l
__global__ void __launch_bounds__(kBlock)
ns_finish_kernel(const int32_t* __restrict__ gsrc, const int32_t* __restrict__ sizes, int hop,
                 const int64_t* __restrict__ state, const uint8_t* __restrict__ flag,
                 const int32_t* __restrict__ tiles, uint64_t* __restrict__ g2l,
                 int32_t* __restrict__ n_id, int cap_strided) {
    __shared__ int lds[kBlock / 64 + 1];
    const int E = cap_strided ? cap_strided : sizes[8 + hop];
    const int n = sizes[hop];
    const uint32_t stamp = ns_stamp(state, hop);
    const int base = blockIdx.x * kNsTile + threadIdx.x * 4;
    int f[4], c = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        f[j] = base + j < E ? flag[base + j] : 0;
        c += f[j];
    }
    int total;
    int off = tiles[blockIdx.x] + block_exscan<kBlock>(c, lds, &total);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (f[j]) {
            const int u = gsrc[base + j];
            const int loc = n + off;
            n_id[loc] = u;
            g2l[u] = (uint64_t(stamp) << 32) | uint32_t(loc);
            ++off;
        }
    }
}

// The strided layout's de-duplication in one pass (ns_flags_kernel + ns_finish_kernel): tile t's
// first-occurrence flags over its kNsTile slots, their count published in status[t] (stamp <<
// 32 | kind << 30 | value, kind 1 = the tile's count, 2 = inclusive prefix, as ns_rows_kernel),
// the exclusive prefix by decoupled look-back over the lower tiles (dispatched before this one),
// then the tile's new nodes appended to n_id in slot order and their local ids written to g2l.
// The last tile sets sizes[hop + 1]. A new node's flag is decided by its owning slot before any
// block writes its g2l entry (only that slot writes it), so the one-pass order is safe.
__global__ void __launch_bounds__(kBlock)
ns_flags_finish_kernel(const int32_t* __restrict__ gsrc, int32_t* __restrict__ sizes, int hop,
                       const int64_t* __restrict__ state, uint64_t* __restrict__ g2l,
                       const uint64_t* __restrict__ first, uint64_t* __restrict__ status,
                       int32_t* __restrict__ n_id, int cap_e) {
    __shared__ int lds[kBlock / 64 + 1];
    __shared__ int s_prefix;
    const uint32_t stamp = ns_stamp(state, hop);
    const int n = sizes[hop];
    const int tile = blockIdx.x;
    const int base = tile * kNsTile + threadIdx.x * 4;
    int u[4], c = 0;
    bool f[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int bp = base + j;
        u[j] = bp < cap_e ? gsrc[bp] : -2;
        f[j] = u[j] >= 0 && uint32_t(g2l[u[j]] >> 32) != stamp &&
               first[u[j]] == first_key(stamp, bp);
        c += f[j] ? 1 : 0;
    }
    int total;
    const int ex = block_exscan<kBlock>(c, lds, &total);
    // every tile publishes its count, then the first wave reads all lower tiles' counts at once
    // (one lane per tile, 64 per round) until each carries this hop's stamp: a few round trips
    // whatever the tile's position (a serial walk cost one round trip per lower tile)
    if (threadIdx.x == 0)
        __hip_atomic_store(status + tile, lb_pack(stamp, 1u, uint32_t(total)), __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x < 64) {
        int prefix = 0;
        for (int p0 = 0; p0 < tile; p0 += 64) {
            const int p = p0 + int(threadIdx.x);
            int v = 0;
            if (p < tile) {
                uint64_t st;
                do {
                    st = __hip_atomic_load(status + p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                } while (uint32_t(st >> 32) != stamp);                // not yet published
                v = int(st & 0x3FFFFFFFu);
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
            prefix += v;
        }
        if (threadIdx.x == 0) {
            s_prefix = prefix;
            if (tile == int(gridDim.x) - 1) sizes[hop + 1] = n + prefix + total;
        }
    }
    __syncthreads();
    int off = s_prefix + ex;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (f[j]) {
            const int loc = n + off;
            n_id[loc] = u[j];
            g2l[u[j]] = (uint64_t(stamp) << 32) | uint32_t(loc);
            ++off;
        }
    }
}

// every sampled edge's local source id (and, when asked, its source's node type and row in
// that type's table, read beside the dedup table)
__global__ void __launch_bounds__(kBlock)
ns_resolve_kernel(const int32_t* __restrict__ gsrc, const int32_t* __restrict__ sizes, int hop,
                  const uint64_t* __restrict__ g2l, int32_t* __restrict__ blk_idx, int cap_e,
                  const int32_t* __restrict__ ntype, const int64_t* __restrict__ local,
                  int32_t* __restrict__ e_type, int64_t* __restrict__ e_off,
                  int32_t* __restrict__ csc_cnt, int strided) {
    const int bp = blockIdx.x * kBlock + threadIdx.x;
    if (bp >= cap_e || (!strided && bp >= sizes[8 + hop])) return;
    const int u = gsrc[bp];
    if (u == -2) return;               // an empty slot of the strided layout
    int lid;
    if (u < 0) {                       // the self loop (written by ns_rows_kernel)
        lid = blk_idx[bp];
    } else {
        lid = int32_t(uint32_t(g2l[u]));
        blk_idx[bp] = lid;
        if (e_type) {
            e_type[bp] = ntype[u];
            e_off[bp] = local[u];
        }
    }
    if (csc_cnt) atomicAdd(csc_cnt + lid, 1);        // integer: exact in any order
}

// The block's transposed index (one workgroup): csc_ptr = exclusive scan of the per-source edge
// counts over the n_{hop+1} sources, then every edge's entry (target row << 8 | relation) placed
// in its source's segment. The order inside a segment follows the LDS cursor atomics (not
// deterministic); the consumer's sums over a segment are exact fixed-point integer sums, so its
// results do not depend on it. Also the sources with more than kCscShort edges, ascending
// (csc_long[0] = their number, csc_long[1 ..] = the ids): the consumer gives each a whole
// workgroup. Cursors in LDS: n_{hop+1} <= kCscMax.
constexpr int kCscThreads = 1024;
constexpr int kCscMax = 32768;
constexpr int kCscShort = 16;
// the hub rows' work table after the ids (include/regnn_hip.h REGNN_CSC_LONG_*): every hub row
// cut into pieces of <= kCscPiece entries, one int4 (source row, first entry, entries, li << 16 |
// piece index << 8 | pieces of the row) per piece, pieces of a row consecutive
constexpr int kCscPiece = REGNN_CSC_PIECE;
constexpr int kCscLongCap = REGNN_CSC_LONG_CAP;

__global__ void __launch_bounds__(kCscThreads)
ns_csc_kernel(const int32_t* __restrict__ sizes, int hop, const int32_t* __restrict__ blk_idx,
              const int32_t* __restrict__ blk_row, const uint8_t* __restrict__ blk_rel,
              const int32_t* __restrict__ csc_cnt, int32_t* __restrict__ csc_ptr,
              int32_t* __restrict__ csc_ent, int32_t* __restrict__ csc_long, int cap_strided) {
    __shared__ int cur[kCscMax];
    __shared__ int lds[kCscThreads / 64 + 1];
    const int n = sizes[hop + 1], E = cap_strided ? cap_strided : sizes[8 + hop];
    constexpr int IT = 8;
    int carry = 0, lcarry = 0, pcarry = 0;
    int4* pieces = reinterpret_cast<int4*>(csc_long + REGNN_CSC_LONG_TAB);
    for (int base = 0; base < n; base += kCscThreads * IT) {
        const int i0 = base + threadIdx.x * IT;
        int v[IT], s = 0, nl = 0, np = 0;
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            v[j] = i0 + j < n ? csc_cnt[i0 + j] : 0;
            s += v[j];
            nl += v[j] > kCscShort ? 1 : 0;
            np += v[j] > kCscShort ? (v[j] + kCscPiece - 1) / kCscPiece : 0;
        }
        int total, ltotal, ptotal;
        int off = carry + block_exscan<kCscThreads>(s, lds, &total);
        int loff = lcarry + block_exscan<kCscThreads>(nl, lds, &ltotal);
        int poff = pcarry + block_exscan<kCscThreads>(np, lds, &ptotal);
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            if (i0 + j < n) {
                csc_ptr[i0 + j] = off;
                cur[i0 + j] = off;
                if (v[j] > kCscShort) {
                    const int li = loff++;
                    csc_long[1 + li] = i0 + j;
                    const int npc = (v[j] + kCscPiece - 1) / kCscPiece;
                    for (int k = 0; k < npc; ++k, ++poff)
                        pieces[poff] = make_int4(i0 + j, off + k * kCscPiece,
                                                 min(kCscPiece, v[j] - k * kCscPiece),
                                                 (li << 16) | (k << 8) | npc);
                }
            }
            off += v[j];
        }
        carry += total;
        lcarry += ltotal;
        pcarry += ptotal;
    }
    if (threadIdx.x == 0) {
        csc_ptr[n] = carry;
        csc_long[0] = lcarry;
        csc_long[REGNN_CSC_LONG_NPIECE] = pcarry;
    }
    __syncthreads();
    for (int bp = threadIdx.x; bp < E; bp += kCscThreads) {
        const int u = blk_idx[bp];
        if (u < 0) continue;           // an empty slot of the strided layout
        const int slot = atomicAdd(cur + u, 1);
        csc_ent[slot] = (blk_row[bp] << 8) | int(blk_rel[bp]);
    }
}

// The transposed index built by many blocks in one launch (replaces the one-workgroup
// ns_csc_kernel on the strided path). Every block resolves its slots' local source ids (as
// ns_resolve_kernel) and takes each entry's rank in its source's segment from the counter's
// returned atomic; the last block to arrive (a ticket) scans the counts into csc_ptr, the hub list
// and the piece table and publishes them (agent release, a stamped flag); every block then places
// its own entries at csc_ptr[source] + rank (the others wait on the flag: the last block is
// running, it took the last ticket). The order inside a segment follows the counters' atomics
// (unspecified: the consumer's sums are exact fixed-point).
constexpr int kCscScanT = 256;             // 256-thread blocks: they fit beside the model's kernels
// counts per lane per pass (lane-contiguous): 16 in the index's own launch, 4 beside the sums
// (whose launch would otherwise hold the larger LDS in every block)
template <int Q>
constexpr int csc_scan_pad() { return 64 * Q + 64; }   // LDS words per wave (padded)

// The scan of the per-source counts by one 256-thread block: per pass each wave loads 64 Q
// counts coalesced, transposes them through LDS (index e at e + e / Q) so each lane holds Q
// consecutive counts, scans lane-serially and across the wave (shuffles),
// combines the four waves through LDS, and writes csc_ptr back coalesced through the same LDS.
// Hub rows (more than kCscShort entries) are listed ascending with their pieces.
template <int Q>
__device__ void csc_scan_block(const int32_t* __restrict__ csc_cnt, int n,
                               int32_t* __restrict__ csc_ptr, int32_t* __restrict__ csc_long,
                               int* __restrict__ sbuf, int* __restrict__ swave) {
    constexpr int NW = kCscScanT / 64, WE = 64 * Q;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int* buf = sbuf + w * csc_scan_pad<Q>();
    int carry = 0, lcarry = 0, pcarry = 0;
    int4* pieces = reinterpret_cast<int4*>(csc_long + REGNN_CSC_LONG_TAB);
    for (int base = 0; base < n; base += NW * WE) {
        const int wb = base + w * WE;
        int v[Q];
#pragma unroll
        for (int j = 0; j < Q; ++j) {
            const int e = j * 64 + lane;
            v[j] = wb + e < n ? csc_cnt[wb + e] : 0;   // (behind the ticket's acquire)
        }
#pragma unroll
        for (int j = 0; j < Q; ++j) {
            const int e = j * 64 + lane;
            buf[e + e / Q] = v[j];
        }
        __syncthreads();
        int s = 0, nl = 0, np = 0;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            v[q] = buf[lane * (Q + 1) + q];
            s += v[q];
            nl += v[q] > kCscShort ? 1 : 0;
            np += v[q] > kCscShort ? (v[q] + kCscPiece - 1) / kCscPiece : 0;
        }
        int xs = s, xl = nl, xp = np;             // inclusive wave scans
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int ys = __shfl_up(xs, o, 64), yl = __shfl_up(xl, o, 64),
                      yp = __shfl_up(xp, o, 64);
            if (lane >= o) {
                xs += ys;
                xl += yl;
                xp += yp;
            }
        }
        if (lane == 63) {
            swave[w] = xs;
            swave[NW + w] = xl;
            swave[2 * NW + w] = xp;
        }
        __syncthreads();
        int ws = carry, wl = lcarry, wp = pcarry, ts = 0, tl = 0, tp = 0;
#pragma unroll
        for (int u = 0; u < NW; ++u) {
            const int a = swave[u], b = swave[NW + u], c = swave[2 * NW + u];
            if (u < w) {
                ws += a;
                wl += b;
                wp += c;
            }
            ts += a;
            tl += b;
            tp += c;
        }
        int off = ws + xs - s, loff = wl + xl - nl, poff = wp + xp - np;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int i = wb + lane * Q + q;
            buf[lane * (Q + 1) + q] = off;
            if (v[q] > kCscShort && i < n) {
                const int li = loff++;
                csc_long[1 + li] = i;
                const int npc = (v[q] + kCscPiece - 1) / kCscPiece;
                for (int k = 0; k < npc; ++k, ++poff)
                    pieces[poff] = make_int4(i, off + k * kCscPiece,
                                             min(kCscPiece, v[q] - k * kCscPiece),
                                             (li << 16) | (k << 8) | npc);
            }
            off += v[q];
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < Q; ++j) {
            const int e = j * 64 + lane;
            if (wb + e < n) csc_ptr[wb + e] = buf[e + e / Q];
        }
        carry += ts;
        lcarry += tl;
        pcarry += tp;
        __syncthreads();                          // buf / swave reused by the next pass
    }
    if (threadIdx.x == 0) {
        csc_ptr[n] = carry;
        csc_long[0] = lcarry;
        csc_long[REGNN_CSC_LONG_NPIECE] = pcarry;
    }
}

struct NsCscJob {
    int hop, cap_e;
    const int32_t* gsrc; const uint64_t* g2l;
    int32_t* blk_idx; const int32_t* blk_row; const uint8_t* blk_rel;
    int32_t* csc_cnt; int32_t* tiles; int32_t* csc_ptr; int32_t* csc_ent; int32_t* csc_long;
};

// The strided transposed index's control words, past everything the CSR path's flag tiles use
// (tiles[0 .. n_tiles]: the tile counts / prefixes and their ticket): ctl[0] the arrival ticket
// (reset by the last block), ctl[1] the published stamp (no other kernel writes it, so a leftover
// value never equals this hop's stamp), ctl[2] a sticky error word (1: a waiting block's bounded
// spin ran out before the publish; its entries were not placed). tiles >= n_tiles + 4 ints.
__device__ __forceinline__ int32_t* csc_ctl(const NsCscJob& J) {
    return J.tiles + (J.cap_e + kNsTile - 1) / kNsTile + 1;
}

// One workgroup (block `bid` of `nb`) of the transposed index's launch (control words: csc_ctl)
template <int Q>
__device__ void csc_resolve_place(const NsCscJob& J, const int32_t* __restrict__ sizes,
                                  const int64_t* __restrict__ state, int bid, int nb) {
    __shared__ int sbuf[(kCscScanT / 64) * csc_scan_pad<Q>()];
    __shared__ int swave[3 * (kCscScanT / 64)];
    __shared__ int last, ok;
    int32_t* ctl = csc_ctl(J);
    const int bp = bid * kCscScanT + threadIdx.x;
    int lid = -1, rank = 0, ent = 0;
    if (bp < J.cap_e) {
        const int u = J.gsrc[bp];
        if (u != -2) {                     // -2: an empty slot of the strided layout
            ent = (J.blk_row[bp] << 8) | int(J.blk_rel[bp]);
            if (u < 0) {                   // the self loop
                lid = J.blk_idx[bp];
            } else {
                lid = int32_t(uint32_t(J.g2l[u]));
                J.blk_idx[bp] = lid;
            }
            rank = atomicAdd(J.csc_cnt + lid, 1);        // integer: exact in any order
        }
    }
    const uint32_t stamp = ns_stamp(state, J.hop);
    __syncthreads();                       // every count of this block added (values returned)
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last = __hip_atomic_fetch_add(ctl, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
               nb - 1;
        ok = 1;
    }
    __syncthreads();
    if (last) {
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        csc_scan_block<Q>(J.csc_cnt, sizes[J.hop + 1], J.csc_ptr, J.csc_long, sbuf, swave);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(ctl, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(ctl + 1, int(stamp), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    } else if (threadIdx.x == 0) {
        // one lane polls the published stamp (relaxed), then one acquire; bounded (a watchdog:
        // the last block holds a CU and runs to the publish). A spin that runs out places
        // nothing (csc_ptr may be stale) and raises the sticky error word the host checks
        // (DeviceSampler.check_index)
        int seen = 0;
        for (uint32_t spins = 0; spins < (1u << 26) && !seen; ++spins) {
            seen = uint32_t(__hip_atomic_load(ctl + 1, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT)) == stamp;
            if (!seen) __builtin_amdgcn_s_sleep(1);
        }
        if (!seen) {
            __hip_atomic_store(ctl + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok = 0;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (lid >= 0 && ok) J.csc_ent[J.csc_ptr[lid] + rank] = ent;
}

inline int csc_blocks(int64_t cap_e) { return int((cap_e + kCscScanT - 1) / kCscScanT); }

__global__ void __launch_bounds__(kCscScanT)
ns_resolve_csc_kernel(NsCscJob J, const int32_t* __restrict__ sizes,
                      const int64_t* __restrict__ state) {
    csc_resolve_place<16>(J, sizes, state, blockIdx.x, gridDim.x);
}

// The fused step's outer hop with layer 0's parameter-free input sums (relation slots): the
// meta-only strided hop of ns_sample_strided_kernel (same sampling, same slots, edge meta and
// counts), and then the row's G lanes gather its sampled raw input rows (K = 128 floats: G = 32
// lanes x float4 per row, two rows per wave; G = 64: each half of the wave a float4 of alternate
// rows) and sum them per source node type (mag/regnn_ns.py:300-326 + mag/regnn_layers.py:110-144:
// with one relation per (target type, source type) pair, sum_{e: type t} tab[r_e] x_e =
// tab[r_t] sum_{e: type t} x_e, so the sums do not depend on the parameters and run G steps ahead
// on the sampler's stream). Writes per row i: s_agg[i][t][:] (unweighted sums), s_w[i][t]
// (counts), u_self[i][:] (the self loop's row), u_rel[i][t] (the slot's relation or -1),
// u_rel[i][T] (the self loop's relation) -- what agg0's gather phase formed (regnn_nsm_work), in
// agg0's order: the entries in slot order (ascending CSR position), so G = 32 gives agg0's bits.
struct NsSumArgs {
    const int32_t* ptr; const int32_t* idx; const uint8_t* etype; const int32_t* ntype;
    const int64_t* local; int n_et;
    const int32_t* n_id; int32_t* sizes; int hop; int cap; int k;
    int64_t* state;
    int32_t* scnt; uint8_t* blk_rel; float* inv; int32_t* e_type; int64_t* e_off;
    const float* xt[8]; int T;
    float* s_agg; float* s_w; float* u_self; int32_t* u_rel;
    NsCscJob csc; int csc_blocks;          // an earlier hop's transposed index (csc_blocks > 0)
};

template <int NT>
__device__ __forceinline__ const float* pick_tab(const NsSumArgs& A, int t) {
    const float* r = A.xt[0];
#pragma unroll
    for (int q = 1; q < NT; ++q)
        if (t == q) r = A.xt[q];
    return r;
}

constexpr int kNsSumK = 128;               // input row width of the sums kernel
// entries' rows in flight per lane (32 lanes per row: two rounds of 11 for a fan-out of 20). All
// 21 in one round (REGNN_NS_SUM_UN32=21: 168 VGPRs, 3 waves per SIMD) measured 118.3 against
// 106.7 us per step: the sampler's kernel then holds more of the GPU beside the model
#ifndef REGNN_NS_SUM_UN32
#define REGNN_NS_SUM_UN32 11
#endif
template <int G>
constexpr int ns_sum_un() { return G == 32 ? REGNN_NS_SUM_UN32 : 11; }
constexpr int kNsSumOcc = REGNN_NS_SUM_UN32 > 11 ? 3 : 4;   // waves per SIMD the registers allow
constexpr int kNsSumWaves = 4;             // waves per block (256 threads: they fit beside the
                                           // model's kernels on a shared CU)

template <int G, int NT>
__global__ void __launch_bounds__(64 * kNsSumWaves, kNsSumOcc)
ns_sample_sums_kernel(NsSumArgs A) {
    // the first csc_blocks workgroups build the earlier hop's transposed index (latency-bound:
    // dispatched first, they run beside the sums instead of ahead of them)
    if (int(blockIdx.x) < A.csc_blocks) {
        csc_resolve_place<4>(A.csc, A.sizes, A.state, blockIdx.x, A.csc_blocks);
        return;
    }
    const int bid = blockIdx.x - A.csc_blocks, nbk = gridDim.x - A.csc_blocks;
    constexpr int K = kNsSumK;
    constexpr int kNsSumUN = ns_sum_un<G>();
    constexpr int TPW = 64 / G;                // rows per wave
    constexpr int H = G == 64 ? 2 : 1;         // lane groups of 32 per row (each a float4 column)
    __shared__ int wsum[kNsSumWaves * TPW];
    const int wl = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int lane = wl % G, tl = wv * TPW + wl / G;
    const uint64_t gmask = G == 64 ? ~0ull : (0xFFFFFFFFull << (wl & 32));
    const int n = A.sizes[A.hop];
    const int k = A.k, S = k + 1;
    int etot = 0;                              // this lane's rows' edges (lane 0 of a row)
    // grid-stride over row groups (uniform per block): a grid smaller than the rows (the launch's
    // REGNN_NS_SUM_BLOCKS) keeps the kernel on fewer CUs beside the model's kernels
    for (int ib = bid * (kNsSumWaves * TPW); ib < A.cap; ib += nbk * (kNsSumWaves * TPW)) {
    const int i = ib + tl;
    const int64_t base = int64_t(i) * S;
    int cnt = -1;                              // -1: no row (past the batch)
    if (i < A.cap && i >= n) {
        if (lane == 0) {
            A.scnt[i] = 0;
            A.inv[i] = 1.f;
        }
    } else if (i < n) {
        const uint64_t seed = ns_hop_seed(A.state, A.hop);
        const int t = A.n_id[i];
        const int b = A.ptr[t], d = A.ptr[t + 1] - b;
        cnt = d < k ? d : k;
        int slot = lane < d ? lane : -1, rank = lane;  // deg <= k: every position, in order
        int src = lane;                        // the lane holding slot `lane`'s draw
        if (d > k) {                               // Floyd (regnn_sample_fill's spec)
            slot = -1;
            const int jl = d - k + lane;
            const int my_pos = lane < k ? int((uint64_t(ns_hash(seed, uint64_t(t), uint64_t(jl))) *
                                               uint64_t(jl + 1)) >> 32) : 0;
            for (int q = 0; q < k; ++q) {
                const int pos = __shfl(my_pos, q, G);
                const bool seen = (__ballot(slot == pos) & gmask) != 0;
                if (lane == q) slot = seen ? d - k + q : pos;
            }
            rank = 0;
            for (int m = 0; m < k; ++m) {
                const int other = __shfl(slot, m, G);
                rank += (lane < k && other < slot) ? 1 : 0;
            }
            for (int m = 0; m < k; ++m)            // inverse: slot j's draw
                if (__shfl(rank, m, G) == lane) src = m;
        }
        // this lane's draw: a sampled edge (lane < cnt)
        int my_t = 0, my_lo = 0, my_r = 0;     // table rows < 2^31 (checked by the host)
        if (lane < cnt) {
            const int p = b + slot;
            const int u = A.idx[p];
            const int64_t bp = base + rank;
            my_r = A.etype[p];
            my_t = A.ntype[u];
            const int64_t lo = A.local[u];
            my_lo = int(lo);
            A.blk_rel[bp] = uint8_t(my_r);
            A.e_type[bp] = my_t;
            A.e_off[bp] = lo;
        }
        // slot order: lane j < cnt takes slot j's entry, lane cnt the self loop
        int st = __shfl(my_t, src, G), sr = __shfl(my_r, src, G), slo = __shfl(my_lo, src, G);
        if (lane == cnt) {
            const int64_t bp = base + cnt;
            st = A.ntype[t];
            sr = A.n_et + st;
            const int64_t lo = A.local[t];
            slo = int(lo);
            A.blk_rel[bp] = uint8_t(sr);
            A.e_type[bp] = st;
            A.e_off[bp] = lo;
        }
        if (lane == 0) {
            A.scnt[i] = cnt;
            A.inv[i] = 1.f / float(cnt + 1);
        }
        // ---- the row's input sums over its entries j = h, h + H, ..; lane l a float4 column
        const int h = lane >> 5, l = lane & 31;
        const int ne = cnt + 1;
        float4 racc[NT];
        float ws[NT];
        int rt[NT];
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) {
            racc[tt] = make_float4(0.f, 0.f, 0.f, 0.f);
            ws[tt] = 0.f;
            rt[tt] = -1;
        }
        float4 xs = make_float4(0.f, 0.f, 0.f, 0.f);
        int rs = -1;
        for (int j0 = 0; j0 < ne; j0 += H * kNsSumUN) {
            float4 x[kNsSumUN];
#pragma unroll
            for (int u = 0; u < kNsSumUN; ++u) {
                const int j = j0 + H * u + h;
                const int jj = j < ne ? j : ne - 1;  // padding: a valid row, loaded, not added
                const int tj = __shfl(st, jj, G);
                const int64_t lo = __shfl(slo, jj, G);
                x[u] = *reinterpret_cast<const float4*>(pick_tab<NT>(A, tj) + lo * K + 4 * l);
            }
            // (each entry's type / relation shuffled again here: arrays of them held across the
            // loads cost the registers that keep every row in flight)
#pragma unroll
            for (int u = 0; u < kNsSumUN; ++u) {
                const int j = j0 + H * u + h;
                const int jj = j < ne ? j : ne - 1;
                const int tj = __shfl(st, jj, G), rj = __shfl(sr, jj, G);
                if (j >= ne) continue;
                if (rj >= A.n_et) {                // the self loop (one per row)
                    xs = x[u];
                    rs = rj;
                    continue;
                }
#pragma unroll
                for (int tt = 0; tt < NT; ++tt) {
                    if (tt != tj) continue;
                    ws[tt] += 1.f;
                    rt[tt] = rj;
                    racc[tt].x += x[u].x; racc[tt].y += x[u].y;
                    racc[tt].z += x[u].z; racc[tt].w += x[u].w;
                }
            }
        }
        if constexpr (H == 2) {
            // the two halves' sums (even / odd slots): half 0's first, the same bits in both
            auto both = [&](float v) {
                const float o = __shfl_xor(v, 32, 64);
                return h == 0 ? v + o : o + v;
            };
#pragma unroll
            for (int tt = 0; tt < NT; ++tt) {
                racc[tt] = make_float4(both(racc[tt].x), both(racc[tt].y), both(racc[tt].z),
                                       both(racc[tt].w));
                ws[tt] = both(ws[tt]);
                rt[tt] = max(rt[tt], __shfl_xor(rt[tt], 32, 64));
            }
            const int rso = __shfl_xor(rs, 32, 64);
            const float4 xo = make_float4(__shfl_xor(xs.x, 32, 64), __shfl_xor(xs.y, 32, 64),
                                          __shfl_xor(xs.z, 32, 64), __shfl_xor(xs.w, 32, 64));
            if (rs < 0) {
                xs = xo;
                rs = rso;
            }
        }
        const int T = A.T;
#pragma unroll
        for (int tt = 0; tt < NT; ++tt)
            if (tt < T && (H == 1 || (tt & 1) == h))
                *reinterpret_cast<float4*>(A.s_agg + (int64_t(i) * T + tt) * K + 4 * l) = racc[tt];
        if (H == 1 || h == 1) *reinterpret_cast<float4*>(A.u_self + int64_t(i) * K + 4 * l) = xs;
        if (lane < T) {
            float wv_ = 0.f;
            int rv_ = -1;
#pragma unroll
            for (int tt = 0; tt < NT; ++tt)
                if (tt == lane) {
                    wv_ = ws[tt];
                    rv_ = rt[tt];
                }
            A.s_w[int64_t(i) * T + lane] = wv_;
            A.u_rel[int64_t(i) * (T + 1) + lane] = rv_;
        } else if (lane == T) {
            A.u_rel[int64_t(i) * (T + 1) + T] = rs;
        }
    }
    etot += cnt + 1;                           // edges of the row, self loop included
    }
    if (lane == 0) wsum[tl] = etot;
    __syncthreads();
    if (threadIdx.x == 0) {
        int e = 0;
#pragma unroll
        for (int q = 0; q < kNsSumWaves * TPW; ++q) e += wsum[q];
        if (e) {
            atomicAdd(A.sizes + 8 + A.hop, e);
            atomicAdd(reinterpret_cast<unsigned long long*>(A.state + 5), (unsigned long long)e);
        }
        if (bid == 0) A.sizes[A.hop + 1] = n;
    }
}

// Backward of the sampled block's mean aggregation y[v] = s[v] sum_e tab[rel_e] x[idx_e] + b
// (mag/regnn_layers.py:129,142-148 through torch_scatter's mean): per target row v the scaled
// gradient s[v] g[v] is scattered to the gathered rows with hardware float atomics (the block's
// sources have no CSC: a sampled hub is gathered by many targets of this batch), and the
// relation dots <s[v] g[v], x[u]> go into per-block LDS bins -> one slab row per block.
template <int LPR>
__global__ void __launch_bounds__(kBlock)
ns_spmm_bwd_kernel(const int32_t* __restrict__ ptr, const int32_t* __restrict__ idx,
                   const uint8_t* __restrict__ rel, const float* __restrict__ tab,
                   const float* __restrict__ out_scale, const float* __restrict__ g,
                   const float* __restrict__ x, float* __restrict__ gx, float* __restrict__ slab,
                   int n_rel, int64_t n_rows, int F) {
    __shared__ float bins[256];
    for (int r = threadIdx.x; r < n_rel; r += blockDim.x) bins[r] = 0.f;
    __syncthreads();
    constexpr int RPW = 64 / LPR;
    const int lane = threadIdx.x & 63, l = lane % LPR, sub = lane / LPR;
    const int64_t rows_per_block = int64_t(kBlock / 64) * RPW;
    for (int64_t v0 = int64_t(blockIdx.x) * rows_per_block; v0 < n_rows;
         v0 += int64_t(gridDim.x) * rows_per_block) {
        const int64_t v = v0 + (threadIdx.x >> 6) * RPW + sub;
        if (v >= n_rows) continue;
        const int e0 = ptr[v], e1 = ptr[v + 1];
        if (e0 == e1) continue;
        const float sc = out_scale ? out_scale[v] : 1.f;
        for (int f0 = 4 * l; f0 < F; f0 += 4 * LPR) {
            const float4 gv4 = *reinterpret_cast<const float4*>(g + v * F + f0);
            const float gv[4] = {gv4.x * sc, gv4.y * sc, gv4.z * sc, gv4.w * sc};
            for (int e = e0; e < e1; ++e) {
                const int u = idx[e];
                const int r = rel ? rel[e] : 0;
                const float w = tab ? tab[r] : 1.f;
                float* dst = gx + int64_t(u) * F + f0;
#pragma unroll
                for (int i = 0; i < 4; ++i) unsafeAtomicAdd(dst + i, w * gv[i]);
                if (slab) {
                    const float4 xv = *reinterpret_cast<const float4*>(x + int64_t(u) * F + f0);
                    float d = gv[0] * xv.x + gv[1] * xv.y + gv[2] * xv.z + gv[3] * xv.w;
                    d = group_sum<LPR>(d);
                    if (l == 0) atomicAdd(bins + r, d);
                }
            }
        }
    }
    if (!slab) return;
    __syncthreads();
    for (int r = threadIdx.x; r < n_rel; r += blockDim.x) slab[int64_t(blockIdx.x) * n_rel + r] = bins[r];
}

// The same backward as a gather over the block's transposed index (regnn_ns_hop csc_*: per local
// source u its entries (target row v << 8 | relation r)): gx[u] = sum tab[r] s[v] g[v], every row
// written once (no zero fill, no atomics to HBM); the relation dots s[v] <g[v], x[u]> from the
// source row held in registers, per-block LDS bins -> one slab row per block. F = 4 LPR VPL.
// Rows with <= kCscShort entries: one LPR-lane group each, UN entries' rows in flight; the hub
// rows (the sampler's csc_long list): a workgroup each, its groups taking interleaved entries,
// the group partials added in LDS in group order.
template <int LPR, int VPL>
__device__ __forceinline__ void csc_entries(const int32_t* __restrict__ cent,
                                            const float* __restrict__ tab,
                                            const float* __restrict__ out_scale,
                                            const float* __restrict__ g, float* bins, bool dots,
                                            int c0, int c1, int step, int l, int gl,
                                            const float4 (&xr)[VPL], float4 (&acc)[VPL]) {
    constexpr int F = 4 * LPR * VPL;
    constexpr int UN = 8;
    for (int c = c0; c < c1; c += UN * step) {
        int vv[UN], rr[UN];
        float ww[UN], ss[UN];
        float4 gv[UN][VPL];
#pragma unroll
        for (int u = 0; u < UN; ++u) {
            const int cc = c + u * step;
            const int en = cc < c1 ? cent[cc] : 0;
            vv[u] = en >> 8;
            rr[u] = en & 255;
        }
#pragma unroll
        for (int u = 0; u < UN; ++u) {
            ss[u] = out_scale ? out_scale[vv[u]] : 1.f;
            ww[u] = (c + u * step < c1) ? (tab ? tab[rr[u]] : 1.f) * ss[u] : 0.f;
#pragma unroll
            for (int p = 0; p < VPL; ++p)
                gv[u][p] = *reinterpret_cast<const float4*>(g + int64_t(vv[u]) * F + 4 * (l + LPR * p));
        }
#pragma unroll
        for (int u = 0; u < UN; ++u) {
            float d = 0.f;
#pragma unroll
            for (int p = 0; p < VPL; ++p) {
                acc[p].x = fmaf(ww[u], gv[u][p].x, acc[p].x);
                acc[p].y = fmaf(ww[u], gv[u][p].y, acc[p].y);
                acc[p].z = fmaf(ww[u], gv[u][p].z, acc[p].z);
                acc[p].w = fmaf(ww[u], gv[u][p].w, acc[p].w);
                d = fmaf(gv[u][p].w, xr[p].w, fmaf(gv[u][p].z, xr[p].z,
                         fmaf(gv[u][p].y, xr[p].y, fmaf(gv[u][p].x, xr[p].x, d))));
            }
            if (dots) {                        // the group's own bin row, in entry order
                d = group_sum<LPR>(d);
                if (l == 0 && c + u * step < c1) bins[rr[u]] += ss[u] * d;
            }
        }
    }
    (void)gl;
}

// The hub rows' chunks (hub_work mode): every piece of the sampler's hub table
// (REGNN_CSC_LONG_TAB) cut into chunks of kCscChunk entries, one workgroup each; cpre = the
// exclusive chunk prefix over the pieces (in LDS), returns the chunk count.
constexpr int kCscUN = 8;                  // csc_entries' rows in flight per lane
__device__ __forceinline__ int csc_chunk_scan(const int32_t* __restrict__ clong, int chunk,
                                              int* cpre, int* wsum) {
    const int n_piece = clong[REGNN_CSC_LONG_NPIECE];
    const int4* pt = reinterpret_cast<const int4*>(clong + REGNN_CSC_LONG_TAB);
    int cnt[8], run = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int p = 8 * threadIdx.x + j;
        cnt[j] = p < n_piece ? (pt[p].z + chunk - 1) / chunk : 0;
        run += cnt[j];
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int xv = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(xv, o, 64);
        if (lane >= o) xv += y;
    }
    if (lane == 63) wsum[w] = xv;
    __syncthreads();
    int e = xv - run;
    for (int k = 0; k < w; ++k) e += wsum[k];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int p = 8 * threadIdx.x + j;
        if (p <= n_piece) cpre[p] = e;
        if (p < n_piece) e += cnt[j];
    }
    __syncthreads();
    return cpre[n_piece];
}

template <int LPR, int VPL>
__global__ void __launch_bounds__(kBlock)
ns_spmm_bwd_csc_kernel(const int32_t* __restrict__ cptr, const int32_t* __restrict__ cent,
                       const int32_t* __restrict__ clong, const float* __restrict__ tab,
                       const float* __restrict__ out_scale, const float* __restrict__ g,
                       const float* __restrict__ x, float* __restrict__ gx,
                       float* __restrict__ slab, int n_rel, const int32_t* __restrict__ sizes,
                       int size_idx, int64_t cap_rows, float* __restrict__ hub_work) {
    constexpr int F = 4 * LPR * VPL;
    constexpr int NG = kBlock / LPR;       // row groups per block
    constexpr int CH = NG * kCscUN;        // hub chunk: one round of every group's rows
    // relation bins per row group (lane 0 of a group adds its entries in order; the groups'
    // rows are summed in group order at the end: no order-dependent float atomics)
    __shared__ float gbins[NG][256];
    __shared__ float4 part[NG * LPR * VPL];
    for (int i = threadIdx.x; i < NG * 256; i += kBlock) gbins[i >> 8][i & 255] = 0.f;
    __syncthreads();
    const bool dots = slab != nullptr;
    const int l = threadIdx.x % LPR, grp = threadIdx.x / LPR, gl = (threadIdx.x & 63) - l;
    float* bins = gbins[grp];
    const int64_t n_rows = sizes ? min(cap_rows, int64_t(sizes[size_idx])) : cap_rows;
    // ---- hub chunks (block-uniform): chunk j runs on block grid - 1 - j (+ grid, ..); at most
    // 32768 / CH + MAXPIECE chunks (the hub_work bound), so the blocks below that range skip the
    // piece table's scan
    if (hub_work && int(gridDim.x) - 1 - int(blockIdx.x) < 32768 / CH + REGNN_CSC_LONG_MAXPIECE) {
        __shared__ int cpre[REGNN_CSC_LONG_MAXPIECE + 1];
        __shared__ int wsum[kBlock / 64];
        const int total = csc_chunk_scan(clong, CH, cpre, wsum);
        for (int j = int(gridDim.x) - 1 - int(blockIdx.x); j < total; j += gridDim.x) {
            const int n_piece = clong[REGNN_CSC_LONG_NPIECE];
            int lo = 0, hi = n_piece - 1;      // the piece p with cpre[p] <= j < cpre[p + 1]
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (cpre[mid] <= j) lo = mid; else hi = mid - 1;
            }
            const int4 pc = reinterpret_cast<const int4*>(clong + REGNN_CSC_LONG_TAB)[lo];
            const int64_t u = pc.x;
            const int e0 = pc.y + CH * (j - cpre[lo]);
            const int e1 = min(e0 + CH, pc.y + pc.z);
            float4 acc[VPL], xr[VPL];
#pragma unroll
            for (int p = 0; p < VPL; ++p) {
                acc[p] = make_float4(0.f, 0.f, 0.f, 0.f);
                xr[p] = dots ? *reinterpret_cast<const float4*>(x + u * F + 4 * (l + LPR * p))
                             : make_float4(0.f, 0.f, 0.f, 0.f);
            }
            const int c0 = e0 + kCscUN * grp;
            csc_entries<LPR, VPL>(cent, tab, out_scale, g, bins, dots, c0, min(c0 + kCscUN, e1),
                                  1, l, gl, xr, acc);
#pragma unroll
            for (int p = 0; p < VPL; ++p) part[(grp * VPL + p) * LPR + l] = acc[p];
            __syncthreads();
            for (int i = threadIdx.x; i < LPR * VPL; i += kBlock) {
                float4 s4 = part[i];
                for (int k = 1; k < NG; ++k) {
                    const float4 q = part[k * LPR * VPL + i];
                    s4.x += q.x; s4.y += q.y; s4.z += q.z; s4.w += q.w;
                }
                const int p = i / LPR, ll = i % LPR;
                *reinterpret_cast<float4*>(hub_work + int64_t(j) * F + 4 * (ll + LPR * p)) = s4;
            }
            __syncthreads();
        }
    }
    // ---- rows with <= kCscShort entries (and the rows past the batch: zeros)
    for (int64_t u = int64_t(blockIdx.x) * NG + grp; u < cap_rows; u += int64_t(gridDim.x) * NG) {
        const bool live = u < n_rows;
        const int c0 = live ? cptr[u] : 0, c1 = live ? cptr[u + 1] : 0;
        if (c1 - c0 > kCscShort) continue;     // a hub: the workgroup pass below
        float4 acc[VPL], xr[VPL];
#pragma unroll
        for (int p = 0; p < VPL; ++p) {
            acc[p] = make_float4(0.f, 0.f, 0.f, 0.f);
            xr[p] = dots && live ? *reinterpret_cast<const float4*>(x + u * F + 4 * (l + LPR * p))
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        csc_entries<LPR, VPL>(cent, tab, out_scale, g, bins, dots, c0, c1, 1, l, gl, xr, acc);
#pragma unroll
        for (int p = 0; p < VPL; ++p)
            *reinterpret_cast<float4*>(gx + u * F + 4 * (l + LPR * p)) = acc[p];
    }
    // ---- hub rows: a workgroup each (without hub_work)
    const int n_long = clong && !hub_work ? clong[0] : 0;
    for (int li = blockIdx.x; li < n_long; li += gridDim.x) {
        const int64_t u = clong[1 + li];
        const int c0 = cptr[u], c1 = cptr[u + 1];
        float4 acc[VPL], xr[VPL];
#pragma unroll
        for (int p = 0; p < VPL; ++p) {
            acc[p] = make_float4(0.f, 0.f, 0.f, 0.f);
            xr[p] = dots ? *reinterpret_cast<const float4*>(x + u * F + 4 * (l + LPR * p))
                         : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        csc_entries<LPR, VPL>(cent, tab, out_scale, g, bins, dots, c0 + grp, c1, NG, l, gl, xr, acc);
#pragma unroll
        for (int p = 0; p < VPL; ++p) part[(grp * VPL + p) * LPR + l] = acc[p];
        __syncthreads();
        for (int i = threadIdx.x; i < LPR * VPL; i += kBlock) {
            float4 s4 = part[i];
            for (int k = 1; k < NG; ++k) {
                const float4 q = part[k * LPR * VPL + i];
                s4.x += q.x; s4.y += q.y; s4.z += q.z; s4.w += q.w;
            }
            const int p = i / LPR, ll = i % LPR;
            *reinterpret_cast<float4*>(gx + u * F + 4 * (ll + LPR * p)) = s4;
        }
        __syncthreads();
    }
    if (!dots) return;
    __syncthreads();
    for (int r = threadIdx.x; r < n_rel; r += kBlock) {
        float sr = 0.f;
        for (int k = 0; k < NG; ++k) sr += gbins[k][r];
        slab[int64_t(blockIdx.x) * n_rel + r] = sr;
    }
}

// hub_work mode's second launch: each hub row's chunk sums added in chunk order -> gx[u]
template <int F>
__global__ void __launch_bounds__(kBlock)
ns_csc_hub_sum_kernel(const int32_t* __restrict__ clong, int chunk,
                      const float* __restrict__ hub_work, float* __restrict__ gx) {
    __shared__ int cpre[REGNN_CSC_LONG_MAXPIECE + 1];
    __shared__ int wsum[kBlock / 64];
    csc_chunk_scan(clong, chunk, cpre, wsum);
    const int n_piece = clong[REGNN_CSC_LONG_NPIECE];
    const int4* pt = reinterpret_cast<const int4*>(clong + REGNN_CSC_LONG_TAB);
    for (int p = blockIdx.x; p < n_piece; p += gridDim.x) {
        const int4 pc = pt[p];
        if ((pc.w >> 8) & 255) continue;       // not the row's first piece
        const int npc = pc.w & 255;
        const int c0 = cpre[p], c1 = cpre[p + npc];
        for (int f = threadIdx.x; f < F; f += kBlock) {
            // the chunk partials in chunk order; 8 loads in flight per round (the adds in the
            // same order: one dependent load per chunk measured ~10 us per launch at F = 512)
            float sacc = 0.f;
            int c = c0;
            for (; c + 8 <= c1; c += 8) {
                float v[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = hub_work[int64_t(c + k) * F + f];
#pragma unroll
                for (int k = 0; k < 8; ++k) sacc += v[k];
            }
            for (; c < c1; ++c) sacc += hub_work[int64_t(c) * F + f];
            gx[int64_t(pc.x) * F + f] = sacc;
        }
    }
}


// ---- module-path helpers (the wide NS model's small per-step ops in one launch each)
// y[i] = labels[n_id[i]] for the batch's live targets i < sizes[0], else `ignore`
// (mag/regnn_ns.py:404: y = data.y[n_id[:batch_size]], nll_loss over the targets)
__global__ void __launch_bounds__(kBlock)
ns_labels_kernel(const int32_t* __restrict__ n_id, const int32_t* __restrict__ sizes,
                 const int64_t* __restrict__ labels, int B, int64_t ignore, int64_t* __restrict__ y) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i < B) y[i] = i < sizes[0] ? labels[n_id[i]] : ignore;
}

// the relation table tab = leaky_relu(alpha rw) (mag/regnn_layers.py:110-111) and its backward
// grw = gtab * alpha * (alpha rw > 0 ? 1 : slope)
__global__ void __launch_bounds__(kBlock)
rel_tab_kernel(const float* __restrict__ rw, const float* __restrict__ gtab, int n, float alpha,
               float slope, float* __restrict__ out) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float x = alpha * rw[i];
    out[i] = gtab ? gtab[i] * (x > 0.f ? alpha : slope * alpha) : (x > 0.f ? x : slope * x);
}


// log_softmax + nll_loss (mean over rows whose label != ignore; mag/regnn_ns.py:404-405 over the
// model's out_lin logits): a wave per row writes lse[r] and the row's loss (0 on an ignored row)
// and validity; one workgroup then sums them in a fixed order (deterministic) into out = {mean
// loss, valid count}; backward: gz[r][c] = g / count * (exp(z[r][c] - lse[r]) - [c == y_r]), 0 on
// ignored rows (a wave per row)
__global__ void __launch_bounds__(kBlock)
xent_rows_kernel(const float* __restrict__ z, const int64_t* __restrict__ y, int B, int C,
                 int64_t ignore, float* __restrict__ lse, float* __restrict__ rowloss) {
    const int r = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (r >= B) return;
    const float* zr = z + int64_t(r) * C;
    const int64_t yr = y[r];
    float m = -INFINITY;
    for (int c = lane; c < C; c += 64) m = fmaxf(m, zr[c]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    float se = 0.f;
    for (int c = lane; c < C; c += 64) se += expf(zr[c] - m);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) se += __shfl_xor(se, o, 64);
    const float l = m + logf(se);
    if (lane == 0) {
        lse[r] = l;
        rowloss[r] = yr != ignore ? l - zr[yr] : 0.f;
        rowloss[B + r] = yr != ignore ? 1.f : 0.f;
    }
}

constexpr int kXentT = 1024;
__global__ void __launch_bounds__(kXentT)
xent_sum_kernel(const float* __restrict__ rowloss, int B, float* __restrict__ out) {
    __shared__ float ls[kXentT], lc[kXentT];
    float s = 0.f, n = 0.f;                  // thread t: rows t, t + 1024, .. in order
    for (int r = threadIdx.x; r < B; r += kXentT) {
        s += rowloss[r];
        n += rowloss[B + r];
    }
    ls[threadIdx.x] = s;
    lc[threadIdx.x] = n;
    __syncthreads();
    for (int h = kXentT / 2; h > 0; h >>= 1) {   // a fixed-shape tree
        if (int(threadIdx.x) < h) {
            ls[threadIdx.x] += ls[threadIdx.x + h];
            lc[threadIdx.x] += lc[threadIdx.x + h];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out[0] = ls[0] / lc[0];              // (0 / 0 = nan with no valid row, as nll_loss)
        out[1] = lc[0];
    }
}

__global__ void __launch_bounds__(kBlock)
xent_bwd_kernel(const float* __restrict__ z, const int64_t* __restrict__ y,
                const float* __restrict__ lse, const float* __restrict__ stat,
                const float* __restrict__ g, int B, int C, int64_t ignore, float* __restrict__ gz) {
    const int r = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (r >= B) return;
    const int64_t yr = y[r];
    const float scale = yr != ignore ? g[0] / stat[1] : 0.f;
    const float l = lse[r];
    const float* zr = z + int64_t(r) * C;
    float* gr = gz + int64_t(r) * C;
    for (int c = lane; c < C; c += 64)
        gr[c] = scale * (expf(zr[c] - l) - (int64_t(c) == yr ? 1.f : 0.f));
}

// The module path's loss in one launch: the labels of a capacity-sized batch (regnn_ns_labels),
// log_softmax + nll per row (xent_rows_kernel) and, in the last workgroup to finish (an agent-scope
// ticket, reset by that workgroup), the fixed-order mean (thread t sums rows t, t + 256, .. in
// order, then a fixed-shape tree): mag/regnn_ns.py:404-405 over out_lin's logits.
__global__ void __launch_bounds__(kBlock)
ns_xent_fwd_kernel(const float* __restrict__ z, const int32_t* __restrict__ n_id,
                   const int32_t* __restrict__ sizes, const int64_t* __restrict__ labels, int B,
                   int C, int64_t ignore, int64_t* __restrict__ y, float* __restrict__ lse,
                   float* __restrict__ rowloss, float* __restrict__ out, int32_t* ticket) {
    __shared__ float ls[kBlock], lc[kBlock];
    __shared__ int last;
    const int r = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (r < B) {
        const int64_t yr = r < sizes[0] ? labels[n_id[r]] : ignore;
        const float* zr = z + int64_t(r) * C;
        float m = -INFINITY;
        for (int c = lane; c < C; c += 64) m = fmaxf(m, zr[c]);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
        float se = 0.f;
        for (int c = lane; c < C; c += 64) se += expf(zr[c] - m);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) se += __shfl_xor(se, o, 64);
        const float l = m + logf(se);
        if (lane == 0) {
            y[r] = yr;
            lse[r] = l;
            rowloss[r] = yr != ignore ? l - zr[yr] : 0.f;
            rowloss[B + r] = yr != ignore ? 1.f : 0.f;
        }
    }
    // every wave releases its own rows' stores at agent scope (the barrier is workgroup scope),
    // then one ticket per workgroup
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        last = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
               int(gridDim.x) - 1;
    }
    __syncthreads();
    if (!last) return;
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    float s = 0.f, n = 0.f;
    for (int i = threadIdx.x; i < B; i += kBlock) {
        s += rowloss[i];
        n += rowloss[B + i];
    }
    ls[threadIdx.x] = s;
    lc[threadIdx.x] = n;
    __syncthreads();
    for (int h = kBlock / 2; h > 0; h >>= 1) {
        if (int(threadIdx.x) < h) {
            ls[threadIdx.x] += ls[threadIdx.x + h];
            lc[threadIdx.x] += lc[threadIdx.x + h];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out[0] = ls[0] / lc[0];                // (0 / 0 = nan with no valid row, as nll_loss)
        out[1] = lc[0];
        __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Its backward with out_lin's bias gradient: a workgroup per 16 classes over every row (16 row
// lanes x 16 classes), gz = g[0] / out[1] (softmax(z) - onehot(y)) (xent_bwd_kernel's value) and
// gb[c] = sum_r gz[r][c]: row lane j sums rows j, j + 16, .. in order, the 16 lanes in order.
__global__ void __launch_bounds__(kBlock)
xent_bwd_colsum_kernel(const float* __restrict__ z, const int64_t* __restrict__ y,
                       const float* __restrict__ lse, const float* __restrict__ stat,
                       const float* __restrict__ g, int B, int C, int64_t ignore,
                       float* __restrict__ gz, float* __restrict__ gb) {
    __shared__ float part[16][17];
    const int cl = threadIdx.x & 15, rl = threadIdx.x >> 4;
    const int c = blockIdx.x * 16 + cl;
    const float gs = g[0] / stat[1];
    float acc = 0.f;
    if (c < C) {
#pragma unroll 4
        for (int r = rl; r < B; r += 16) {
            const int64_t yr = y[r];
            const float scale = yr != ignore ? gs : 0.f;
            const float v = scale * (expf(z[int64_t(r) * C + c] - lse[r]) - (int64_t(c) == yr ? 1.f : 0.f));
            gz[int64_t(r) * C + c] = v;
            acc += v;
        }
    }
    part[rl][cl] = acc;
    __syncthreads();
    if (threadIdx.x < 16 && c < C) {
        float t = 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j) t += part[j][threadIdx.x];
        gb[c] = t;
    }
}

}  // namespace regnn

using namespace regnn;

// two targets per wave in the strided sampler: REGNN_NS_HALF_WAVES=1 (off by default — measured
// 136.6 vs 135.0 us per fused step at hidden 64: the sampler runs beside the model, and its
// instruction count is not what the step waits on)
static bool ns_half_waves() {
    const char* v = getenv("REGNN_NS_HALF_WAVES");   // read per launch: tests switch it
    return v && v[0] == '1';
}


extern "C" {

int64_t regnn_ns_csc_hub_work_floats(int32_t F) {
    // chunks of (256 / LPR) * 8 entries over <= 32768 hub entries, + one partial chunk per piece
    const int lpr = F >= 256 ? 64 : F / 4;
    const int ch = (kBlock / lpr) * kCscUN;
    return int64_t(32768 / ch + REGNN_CSC_LONG_MAXPIECE) * F;
}

int regnn_ns_spmm_bwd_csc(const int32_t* csc_ptr, const int32_t* csc_ent, const int32_t* csc_long,
                          const float* rel_table, const float* out_scale, const float* g,
                          const float* x, float* gx, float* slab, int32_t n_rel,
                          const int32_t* sizes, int32_t size_idx, int64_t cap_rows, int32_t F,
                          int32_t slab_rows, float* hub_work, hipStream_t stream) {
    if (!csc_ptr || !csc_ent || !g || !gx || cap_rows < 0 || F <= 0 || n_rel < 0 || n_rel > 256 ||
        (slab && (!x || n_rel == 0 || slab_rows <= 0)) || (sizes && size_idx < 0))
        return REGNN_EINVAL;
    if (cap_rows == 0) return REGNN_OK;
    if (hub_work && !csc_long) return REGNN_EINVAL;
    const int grid = slab ? slab_rows : kMaxGrid;
#define NSC_CASE(L, V)                                                                         \
    if (F == 4 * L * V) {                                                                      \
        hipLaunchKernelGGL((ns_spmm_bwd_csc_kernel<L, V>), dim3(grid), dim3(kBlock), 0,        \
                           stream, csc_ptr, csc_ent, csc_long, rel_table, out_scale, g, x, gx, \
                           slab, n_rel, sizes, size_idx, cap_rows, hub_work);                  \
        REGNN_LAUNCH_CHECK();                                                                  \
        if (hub_work) {                                                                        \
            hipLaunchKernelGGL((ns_csc_hub_sum_kernel<4 * L * V>), dim3(256), dim3(kBlock), 0, \
                               stream, csc_long, (kBlock / L) * kCscUN, hub_work, gx);         \
            REGNN_LAUNCH_CHECK();                                                              \
        }                                                                                      \
        return REGNN_OK;                                                                       \
    }
    NSC_CASE(16, 1) NSC_CASE(32, 1) NSC_CASE(64, 1) NSC_CASE(64, 2) NSC_CASE(64, 4)
    NSC_CASE(64, 8)
#undef NSC_CASE
    return REGNN_EUNSUPPORTED;
}

int regnn_ns_xent_fwd(const float* z, const int32_t* n_id, const int32_t* sizes,
                      const int64_t* labels, int32_t B, int32_t C, int64_t ignore, int64_t* y,
                      float* lse, float* rowloss, float* out, int32_t* ticket, hipStream_t stream) {
    if (!z || !n_id || !sizes || !labels || !y || !lse || !rowloss || !out || !ticket || B <= 0 ||
        C <= 0)
        return REGNN_EINVAL;
    hipLaunchKernelGGL(ns_xent_fwd_kernel, dim3(unsigned((B + 3) / 4)), dim3(kBlock), 0, stream, z,
                       n_id, sizes, labels, B, C, ignore, y, lse, rowloss, out, ticket);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

int regnn_xent_bwd_colsum(const float* z, const int64_t* y, const float* lse, const float* stat,
                          const float* g, int32_t B, int32_t C, int64_t ignore, float* gz,
                          float* gb, hipStream_t stream) {
    if (!z || !y || !lse || !stat || !g || !gz || !gb || B < 0 || C <= 0) return REGNN_EINVAL;
    hipLaunchKernelGGL(xent_bwd_colsum_kernel, dim3(unsigned((C + 15) / 16)), dim3(kBlock), 0,
                       stream, z, y, lse, stat, g, B, C, ignore, gz, gb);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

int regnn_softmax_xent_fwd(const float* z, const int64_t* y, int32_t B, int32_t C, int64_t ignore,
                           float* lse, float* rowloss, float* out, hipStream_t stream) {
    if (!z || !y || !lse || !rowloss || !out || B < 0 || C <= 0) return REGNN_EINVAL;
    if (B > 0) {
        hipLaunchKernelGGL(xent_rows_kernel, dim3(unsigned((B + 3) / 4)), dim3(kBlock), 0, stream,
                           z, y, B, C, ignore, lse, rowloss);
        REGNN_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(xent_sum_kernel, dim3(1), dim3(kXentT), 0, stream, rowloss, B, out);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

int regnn_softmax_xent_bwd(const float* z, const int64_t* y, const float* lse, const float* stat,
                           const float* g, int32_t B, int32_t C, int64_t ignore, float* gz,
                           hipStream_t stream) {
    if (!z || !y || !lse || !stat || !g || !gz || B < 0 || C <= 0) return REGNN_EINVAL;
    if (B == 0) return REGNN_OK;
    hipLaunchKernelGGL(xent_bwd_kernel, dim3(unsigned((B + 3) / 4)), dim3(kBlock), 0, stream, z, y,
                       lse, stat, g, B, C, ignore, gz);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

int regnn_ns_labels(const int32_t* n_id, const int32_t* sizes, const int64_t* labels, int32_t B,
                    int64_t ignore, int64_t* y, hipStream_t stream) {
    if (!n_id || !sizes || !labels || !y || B < 0) return REGNN_EINVAL;
    if (B == 0) return REGNN_OK;
    hipLaunchKernelGGL(ns_labels_kernel, dim3(unsigned((B + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       stream, n_id, sizes, labels, B, ignore, y);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

int regnn_rel_tab(const float* rw, const float* gtab, int32_t n, float alpha, float slope,
                  float* out, hipStream_t stream) {
    if (!rw || !out || n < 0) return REGNN_EINVAL;
    if (n == 0) return REGNN_OK;
    hipLaunchKernelGGL(rel_tab_kernel, dim3(unsigned((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       stream, rw, gtab, n, alpha, slope, out);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

int regnn_ns_batch(const int64_t* perm, int64_t n_perm, int32_t batch, int32_t rank,
                   int32_t world, int64_t* state, int32_t* n_id, int32_t* sizes,
                   int64_t* stamp_src, hipStream_t stream) {
    if (!perm || !state || !n_id || !sizes || n_perm < 0 || batch <= 0 || world <= 0 ||
        rank < 0 || rank >= world)
        return REGNN_EINVAL;
    hipLaunchKernelGGL(ns_batch_kernel, dim3(1), dim3(kBlock), 0, stream, perm, n_perm, batch,
                       rank, world, state, n_id, sizes, stamp_src);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

int regnn_ns_hop(const int32_t* ptr, const int32_t* idx, const uint8_t* etype,
                 const int32_t* ntype, int32_t num_edge_types, int32_t k, int32_t hop,
                 int64_t* state, int32_t* sizes, int32_t* n_id, int32_t cap_dst,
                 uint64_t* g2l, uint64_t* first, int32_t* samp, int32_t* spos, int32_t* scnt,
                 int32_t* gsrc, uint8_t* flag, int32_t* tiles, uint64_t* status,
                 int32_t* blk_ptr, int32_t* blk_idx, uint8_t* blk_rel, int32_t* blk_pos,
                 int32_t* blk_row, float* inv, const int64_t* local, int32_t* edge_type,
                 int64_t* edge_off, int32_t meta_only, int32_t* csc_cnt, int32_t* csc_ptr,
                 int32_t* csc_ent, int32_t* csc_long, int32_t strided, hipStream_t stream) {
    if (!ptr || !idx || !etype || !ntype || !state || !sizes || !n_id || !g2l || !first ||
        !samp || !spos || !scnt || !gsrc || !flag || !tiles || !status || !blk_ptr || !blk_idx ||
        !blk_rel || !blk_pos || !blk_row || !inv || cap_dst <= 0 || hop < 0 || hop > 6 || num_edge_types < 0)
        return REGNN_EINVAL;
    if (!!local != !!edge_type || !!local != !!edge_off || (meta_only && !local))
        return REGNN_EINVAL;
    const bool csc = csc_cnt != nullptr;
    if (csc != (csc_ptr != nullptr) || csc != (csc_ent != nullptr) ||
        csc != (csc_long != nullptr) || (csc && meta_only))
        return REGNN_EINVAL;
    const int lean = meta_only ? 1 : 0;
    if (k < 1 || k > 64) return REGNN_EUNSUPPORTED;
    const int64_t cap_e = int64_t(cap_dst) * (k + 1);
    if (cap_e >= (int64_t(1) << 31)) return REGNN_EUNSUPPORTED;
    const int n_tiles = int((cap_e + kNsTile - 1) / kNsTile);
    if (csc && cap_e > kCscMax) return REGNN_EUNSUPPORTED;
    if (strided == 3) {
        // the transposed index only (the part a strided = 2 call left out), on whatever stream
        // the caller runs it: resolve + counts + ranks, scan, placement
        if (!csc || edge_type || lean) return REGNN_EINVAL;
        const int ce = int(cap_e);
        const NsCscJob J{hop, ce, gsrc, g2l, blk_idx, blk_row, blk_rel, csc_cnt, tiles, csc_ptr,
                         csc_ent, csc_long};
        hipLaunchKernelGGL(ns_resolve_csc_kernel, dim3(unsigned(csc_blocks(cap_e))),
                           dim3(kCscScanT), 0, stream, J, sizes, state);
        REGNN_LAUNCH_CHECK();
        return REGNN_OK;
    }
    if (strided) {
        // sampling + placement in one launch, no row-offset scan (the layout above)
        if (k + 1 <= 32 && ns_half_waves())
            hipLaunchKernelGGL(ns_sample_strided_kernel<32>,
                               dim3(unsigned((cap_dst + 2 * kNsStrWaves - 1) / (2 * kNsStrWaves))),
                               dim3(64 * kNsStrWaves), 0, stream, ptr, idx, etype, ntype,
                               num_edge_types, n_id, sizes, hop, cap_dst, k, state, g2l, first,
                               scnt, gsrc, blk_idx, blk_rel, blk_pos, blk_row, inv, local,
                               edge_type, edge_off, lean, csc_cnt);
        else
            hipLaunchKernelGGL(ns_sample_strided_kernel<64>,
                               dim3(unsigned((cap_dst + kNsStrWaves - 1) / kNsStrWaves)),
                               dim3(64 * kNsStrWaves), 0, stream, ptr, idx, etype, ntype,
                               num_edge_types, n_id, sizes, hop, cap_dst, k, state, g2l, first,
                               scnt, gsrc, blk_idx, blk_rel, blk_pos, blk_row, inv, local,
                               edge_type, edge_off, lean, csc_cnt);
        REGNN_LAUNCH_CHECK();
        if (lean) return REGNN_OK;
        const int ce = int(cap_e);
        // de-duplication in one pass (status: >= n_tiles entries on this path)
        hipLaunchKernelGGL(ns_flags_finish_kernel, dim3(n_tiles), dim3(kBlock), 0, stream, gsrc,
                           sizes, hop, state, g2l, first, status, n_id, ce);
        REGNN_LAUNCH_CHECK();
        if (csc && !edge_type && strided == 2) return REGNN_OK;   // the index: a strided = 3 call
        if (csc && !edge_type) {
            // the transposed index by many blocks in one launch: resolve + counts + ranks, the
            // last block's scan, every block's placement
            const NsCscJob J{hop, ce, gsrc, g2l, blk_idx, blk_row, blk_rel, csc_cnt, tiles,
                             csc_ptr, csc_ent, csc_long};
            hipLaunchKernelGGL(ns_resolve_csc_kernel, dim3(unsigned(csc_blocks(cap_e))),
                               dim3(kCscScanT), 0, stream, J, sizes, state);
            REGNN_LAUNCH_CHECK();
            return REGNN_OK;
        }
        hipLaunchKernelGGL(ns_resolve_kernel, dim3(unsigned((cap_e + kBlock - 1) / kBlock)),
                           dim3(kBlock), 0, stream, gsrc, sizes, hop, g2l, blk_idx, ce, ntype,
                           local, edge_type, edge_off, csc_cnt, 1);
        REGNN_LAUNCH_CHECK();
        if (csc) {
            hipLaunchKernelGGL(ns_csc_kernel, dim3(1), dim3(kCscThreads), 0, stream, sizes, hop,
                               blk_idx, blk_row, blk_rel, csc_cnt, csc_ptr, csc_ent, csc_long, ce);
            REGNN_LAUNCH_CHECK();
        }
        return REGNN_OK;
    }
    hipLaunchKernelGGL(ns_sample_kernel, dim3((cap_dst + 3) / 4), dim3(kBlock), 0, stream, ptr,
                       idx, n_id, sizes, hop, cap_dst, k, state, g2l, samp, spos, scnt);
    REGNN_LAUNCH_CHECK();
    hipLaunchKernelGGL(ns_rows_kernel, dim3((cap_dst + kNsRowsTile - 1) / kNsRowsTile),
                       dim3(kBlock), 0, stream, scnt, n_id, ntype, num_edge_types, sizes, hop,
                       cap_dst, state, blk_ptr, blk_idx, blk_rel, blk_pos, blk_row, gsrc, inv, status, local,
                       edge_type, edge_off, lean, csc_cnt, int(cap_e));
    REGNN_LAUNCH_CHECK();
    const int64_t slots = int64_t(cap_dst) * k;
    hipLaunchKernelGGL(ns_place_kernel, dim3(unsigned((slots + kBlock - 1) / kBlock)),
                       dim3(kBlock), 0, stream, samp, spos, scnt, sizes, hop, cap_dst, k, state,
                       etype, g2l, first, blk_ptr, blk_rel, blk_pos, blk_row, gsrc, ntype, local, edge_type,
                       edge_off, lean);
    REGNN_LAUNCH_CHECK();
    if (lean) return REGNN_OK;         // no dedup, no n_id append, no local source ids
    hipLaunchKernelGGL(ns_flags_kernel, dim3(n_tiles), dim3(kBlock), 0, stream, gsrc, sizes, hop,
                       state, g2l, first, flag, tiles, n_tiles, 0);
    REGNN_LAUNCH_CHECK();
    hipLaunchKernelGGL(ns_finish_kernel, dim3(n_tiles), dim3(kBlock), 0, stream, gsrc, sizes, hop,
                       state, flag, tiles, g2l, n_id, 0);
    REGNN_LAUNCH_CHECK();
    hipLaunchKernelGGL(ns_resolve_kernel, dim3(unsigned((cap_e + kBlock - 1) / kBlock)),
                       dim3(kBlock), 0, stream, gsrc, sizes, hop, g2l, blk_idx, int(cap_e), ntype, local,
                       edge_type, edge_off, csc_cnt, 0);
    REGNN_LAUNCH_CHECK();
    if (csc) {
        hipLaunchKernelGGL(ns_csc_kernel, dim3(1), dim3(kCscThreads), 0, stream, sizes, hop, blk_idx,
                           blk_row, blk_rel, csc_cnt, csc_ptr, csc_ent, csc_long, 0);
        REGNN_LAUNCH_CHECK();
    }
    return REGNN_OK;
}

int regnn_ns_hop_typed_sums(const int32_t* ptr, const int32_t* idx, const uint8_t* etype,
                            const int32_t* ntype, int32_t num_edge_types, int32_t k, int32_t hop,
                            int64_t* state, int32_t* sizes, const int32_t* n_id, int32_t cap_dst,
                            int32_t* scnt, uint8_t* blk_rel, float* inv, const int64_t* local,
                            int32_t* edge_type, int64_t* edge_off, const float* const* tables,
                            int32_t n_types, int32_t K, float* s_agg, float* s_w, float* u_self,
                            int32_t* u_rel, const regnn_ns_csc_job* csc, hipStream_t stream) {
    if (!ptr || !idx || !etype || !ntype || !state || !sizes || !n_id || !scnt || !blk_rel ||
        !inv || !local || !edge_type || !edge_off || !tables || !s_agg || !s_w || !u_self ||
        !u_rel || cap_dst <= 0 || hop < 0 || hop > 6 || num_edge_types < 0)
        return REGNN_EINVAL;
    if (K != kNsSumK || n_types < 1 || n_types > 4 || k < 1 || k > 63) return REGNN_EUNSUPPORTED;
    if (int64_t(cap_dst) * (k + 1) >= (int64_t(1) << 31)) return REGNN_EUNSUPPORTED;
    NsSumArgs A{};
    A.ptr = ptr; A.idx = idx; A.etype = etype; A.ntype = ntype; A.local = local;
    A.n_et = num_edge_types; A.n_id = n_id; A.sizes = sizes; A.hop = hop; A.cap = cap_dst;
    A.k = k; A.state = state; A.scnt = scnt; A.blk_rel = blk_rel; A.inv = inv;
    A.e_type = edge_type; A.e_off = edge_off; A.T = n_types;
    for (int t = 0; t < n_types; ++t) {
        if (!tables[t] || reinterpret_cast<uintptr_t>(tables[t]) % 16) return REGNN_EINVAL;
        A.xt[t] = tables[t];
    }
    for (int t = n_types; t < 8; ++t) A.xt[t] = tables[0];
    if (reinterpret_cast<uintptr_t>(s_agg) % 16 || reinterpret_cast<uintptr_t>(u_self) % 16)
        return REGNN_EINVAL;
    A.s_agg = s_agg; A.s_w = s_w; A.u_self = u_self; A.u_rel = u_rel;
    if (csc) {
        if (!csc->gsrc || !csc->g2l || !csc->blk_idx || !csc->blk_row || !csc->blk_rel ||
            !csc->csc_cnt || !csc->tiles || !csc->csc_ptr || !csc->csc_ent || !csc->csc_long ||
            csc->hop < 0 || csc->hop >= hop || csc->cap_e <= 0)
            return REGNN_EINVAL;
        if (csc->cap_e > kCscMax) return REGNN_EUNSUPPORTED;
        A.csc = NsCscJob{csc->hop, csc->cap_e, csc->gsrc, csc->g2l, csc->blk_idx, csc->blk_row,
                         csc->blk_rel, csc->csc_cnt, csc->tiles, csc->csc_ptr, csc->csc_ent,
                         csc->csc_long};
        A.csc_blocks = csc_blocks(csc->cap_e);
    }
    static const int sum_blocks = [] {     // REGNN_NS_SUM_BLOCKS: cap the grid (0: a row per lane group)
        const char* v = getenv("REGNN_NS_SUM_BLOCKS");
        return v ? atoi(v) : 0;
    }();
    auto grid = [&](int rows_per_block) {
        const int g = (cap_dst + rows_per_block - 1) / rows_per_block;
        return dim3(unsigned(A.csc_blocks + (sum_blocks > 0 && sum_blocks < g ? sum_blocks : g)));
    };
    if (k + 1 <= 32)                   // two rows per wave (32 lanes each): sums in slot order
        hipLaunchKernelGGL((ns_sample_sums_kernel<32, 4>), grid(2 * kNsSumWaves),
                           dim3(64 * kNsSumWaves), 0, stream, A);
    else
        hipLaunchKernelGGL((ns_sample_sums_kernel<64, 4>), grid(kNsSumWaves),
                           dim3(64 * kNsSumWaves), 0, stream, A);
    REGNN_LAUNCH_CHECK();
    return REGNN_OK;
}

int regnn_ns_spmm_bwd(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                      const float* rel_table, const float* out_scale, const float* g,
                      const float* x, float* gx, float* slab, int32_t n_rel, int64_t n_rows,
                      int32_t F, hipStream_t stream) {
    if (!ptr || !idx || !g || !gx || n_rows < 0 || F <= 0 || (F & 3) || n_rel < 0 ||
        n_rel > 256 || (slab && (!x || !rel || !rel_table || n_rel == 0)))
        return REGNN_EINVAL;
    if (n_rows == 0) return REGNN_OK;
    const int nvec = F / 4;
    int lpr = 16;                      // lanes per row: the largest power of two <= 16 dividing F/4
    while (nvec % lpr) lpr >>= 1;
    const int64_t rpb = int64_t(kBlock / 64) * (64 / lpr);
    int64_t grid = (n_rows + rpb - 1) / rpb;
    if (grid > kMaxGrid) grid = kMaxGrid;
    if (grid < 1) grid = 1;
#define NSB_CASE(L)                                                                            \
    if (lpr == L) {                                                                            \
        hipLaunchKernelGGL((ns_spmm_bwd_kernel<L>), dim3((unsigned)grid), dim3(kBlock), 0,     \
                           stream, ptr, idx, rel, rel_table, out_scale, g, x, gx, slab, n_rel, \
                           n_rows, F);                                                         \
        REGNN_LAUNCH_CHECK();                                                                  \
        return REGNN_OK;                                                                       \
    }
    NSB_CASE(16) NSB_CASE(8) NSB_CASE(4) NSB_CASE(2) NSB_CASE(1)
#undef NSB_CASE
    return REGNN_EUNSUPPORTED;
}

}  // extern "C"
