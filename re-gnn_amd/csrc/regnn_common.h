// Shared device helpers for the gfx950 RE-GNN kernels (wave64, 16-byte row vectors).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include "../../include/regnn_hip.h"

namespace regnn {

constexpr int kBlock = 256;       // 4 waves of 64
constexpr int kMaxGrid = 2048;    // grid-stride cap (8 blocks per CU); bounds the slab rows

using bf16_t = uint16_t;          // storage type for REGNN_BF16 rows

// fp32 <-> bf16 (round to nearest even via the gfx950 conversion instruction)
__device__ __forceinline__ float bf2f(uint32_t bits16) { return __uint_as_float(bits16 << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
    __hip_bfloat16 h = __float2bfloat16(f);
    return *reinterpret_cast<uint16_t*>(&h);
}

// One 16-byte vector of a feature row, widened to fp32.
template <typename T> struct Vec;

template <> struct Vec<float> {
    static constexpr int N = 4;
    __device__ __forceinline__ static void load(const float* p, float (&v)[4]) {
        const float4 t = *reinterpret_cast<const float4*>(p);
        v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    }
    __device__ __forceinline__ static void store(float* p, const float (&v)[4]) {
        *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    }
};

template <> struct Vec<bf16_t> {
    static constexpr int N = 8;
    __device__ __forceinline__ static void load(const bf16_t* p, float (&v)[8]) {
        const uint4 t = *reinterpret_cast<const uint4*>(p);
        const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            v[2 * i] = __uint_as_float(w[i] << 16);
            v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
        }
    }
    __device__ __forceinline__ static void store(bf16_t* p, const float (&v)[8]) {
        uint32_t w[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
            w[i] = uint32_t(f2bf(v[2 * i])) | (uint32_t(f2bf(v[2 * i + 1])) << 16);
        *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
    }
};

// a value as it reads back after a store in T (fp32: itself; bf16: round to nearest even)
template <typename T>
__device__ __forceinline__ float round_to(float v) {
    if constexpr (sizeof(T) == 2) return __uint_as_float(uint32_t(f2bf(v)) << 16);
    else return v;
}

// raw 16-byte vector load (kept packed in 4 VGPRs until use) and its widening to fp32
__device__ __forceinline__ uint4 load16(const void* p) { return *reinterpret_cast<const uint4*>(p); }

template <typename T>
__device__ __forceinline__ void unpack(const uint4& r, float (&v)[Vec<T>::N]);

template <>
__device__ __forceinline__ void unpack<float>(const uint4& r, float (&v)[4]) {
    v[0] = __uint_as_float(r.x); v[1] = __uint_as_float(r.y);
    v[2] = __uint_as_float(r.z); v[3] = __uint_as_float(r.w);
}

template <>
__device__ __forceinline__ void unpack<bf16_t>(const uint4& r, float (&v)[8]) {
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        v[2 * i] = __uint_as_float(w[i] << 16);
        v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
}

// Fused dropout keep mask (spec in regnn_hip.h, regnn_spmm_fwd_dropout): the murmur3 finaliser
// over a per-call key and the element's 16-byte-vector counter, 16 bits per feature.
__host__ __device__ __forceinline__ uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h;
}

__device__ __forceinline__ uint32_t drop_key(const uint64_t* seed) {
    const uint64_t s = *seed;
    return fmix32(uint32_t(s) ^ fmix32(uint32_t(s >> 32) ^ 0x5BD1E995u));
}

// v[t] *= keep(t) ? scale : 0 for feature vector `vec` (of nvec per row) of row `row`.
// BITS = 16: two features per 32-bit draw; BITS = 8 (keep16 a multiple of 256): four.
template <int EV, int BITS>
__device__ __forceinline__ void drop_apply(uint32_t key, uint32_t thresh, float scale, int64_t row,
                                           int nvec, int vec, float (&v)[EV]) {
    const uint64_t c = uint64_t(row) * uint64_t(nvec) + uint64_t(vec);
    const uint32_t hi = uint32_t(c >> 32);
    uint32_t h = fmix32(uint32_t(c) ^ key ^ ((hi << 16) | (hi >> 16)));
    if constexpr (BITS == 16) {
#pragma unroll
        for (int k = 0; k < EV / 2; ++k) {
            if (k) h = fmix32(h + 0x9E3779B9u);
            v[2 * k] = (h & 0xFFFFu) < thresh ? v[2 * k] * scale : 0.f;
            v[2 * k + 1] = (h >> 16) < thresh ? v[2 * k + 1] * scale : 0.f;
        }
    } else {
        const uint32_t t8 = thresh >> 8;
#pragma unroll
        for (int k = 0; k < EV / 4; ++k) {
            if (k) h = fmix32(h + 0x9E3779B9u);
#pragma unroll
            for (int b = 0; b < 4; ++b)
                v[4 * k + b] = ((h >> (8 * b)) & 0xFFu) < t8 ? v[4 * k + b] * scale : 0.f;
        }
    }
}

template <int W>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
    for (int o = W / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, W);
    return v;
}

inline int grid_for(int64_t units, int per_block) {
    int64_t g = (units + per_block - 1) / per_block;
    if (g < 1) g = 1;
    return int(g < kMaxGrid ? g : kMaxGrid);
}

// Tuning knobs (regnn_tune): grid cap of the grid-stride gather kernels. 0 = the kernel's
// resident capacity (occupancy API x CUs: every block in the first dispatch round, so the
// grid-stride loop has no partial last round), > 0 = a fixed cap.
extern int64_t g_tune_grid_cap;
extern int64_t g_tune_un;        // rows in flight per lane for F = 16 vectors (0 = 8)
extern int64_t g_tune_head;      // fused head variant: 0 = pipelined, 1 = plain
extern int64_t g_tune_rowscale;  // rows in flight per lane group of regnn_row_scale (0 = 1)

int resident_blocks(const void* kernel, size_t lds, int block = kBlock);  // per CU x CUs, cached

// grid for a grid-stride gather kernel: one round of resident blocks (<= kMaxGrid)
template <typename K>
inline int grid_resident(K kernel, int64_t units, int per_block, size_t lds) {
    int64_t g = (units + per_block - 1) / per_block;
    if (g < 1) g = 1;
    int64_t cap = g_tune_grid_cap > 0 ? g_tune_grid_cap
                                      : resident_blocks(reinterpret_cast<const void*>(kernel), lds);
    if (cap > kMaxGrid) cap = kMaxGrid;
    if (cap < 1) cap = kMaxGrid;
    return int(g < cap ? g : cap);
}

}  // namespace regnn

#define REGNN_LAUNCH_CHECK()                                        \
    do {                                                            \
        if (hipGetLastError() != hipSuccess) return REGNN_ELAUNCH;  \
    } while (0)
