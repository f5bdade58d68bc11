// Shared pieces of the fused NS model step (re_nsm.hip: the general L-layer path, re_nsm2.hip:
// the two-layer path): widths, per-type pointer tables, the dropout key / mask of the step
// (spec in regnn_hip.h), wave reductions.
#pragma once
#include "regnn_common.h"

#include <type_traits>

namespace regnn {
namespace nsm {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int F = 64;                  // hidden width
constexpr int MT = REGNN_NSM_MAX_TYPES;
constexpr int ML = REGNN_NSM_MAX_LAYERS;
constexpr int kAggBlocks = 512;        // persistent grids: fixed, so the slab layout is static
constexpr int kPostBlocks = 256;
constexpr int kProjBlocks = 128;       // per node type
constexpr int kWPad = 65;              // padded row stride of 64-wide matrices in LDS
constexpr float kLnEps = 1e-5f;

struct Ptrs {                          // per-type / per-layer pointer tables passed by value
    const float* p[MT];
};

struct Ints {
    int v[ML];
};

template <typename T, int N>
__device__ __forceinline__ T pick(const T (&a)[N], int i) {
    T r = a[0];
#pragma unroll
    for (int k = 1; k < N; ++k)
        if (i == k) r = a[k];
    return r;
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}

// dropout key of layer `layer` for the current batch (spec in regnn_hip.h): the seed, the epoch
// and the global batch, so a batch draws the same masks whichever sampler slot produced it
__device__ __forceinline__ uint32_t layer_key(const int64_t* state, int layer) {
    const uint64_t s = mix64(uint64_t(state[0]) ^
                             mix64((uint64_t(state[1]) << 40) ^ (uint64_t(state[3]) << 8) ^
                                   (uint64_t(layer) + 0x51ED27ull)));
    return fmix32(uint32_t(s) ^ fmix32(uint32_t(s >> 32) ^ 0x5BD1E995u));
}

struct Drop {
    uint32_t thresh;    // keep16
    float scale;        // 1 / keep
    bool on, b8;        // b8: 8-bit draws (keep16 a multiple of 256), as the host picks for the
                        // other fused-dropout kernels
};

// keep factors (0 or scale) of the 4 features of 16-byte vector `vec` of row `row`
__device__ __forceinline__ void drop_factors(uint32_t key, const Drop& d, int64_t row, int vec,
                                             float (&m)[4]) {
    m[0] = m[1] = m[2] = m[3] = 1.f;
    if (!d.on) return;
    if (d.b8) drop_apply<4, 8>(key, d.thresh, d.scale, row, F / 4, vec, m);
    else drop_apply<4, 16>(key, d.thresh, d.scale, row, F / 4, vec, m);
}

__device__ __forceinline__ float wave_sum(float v) { return group_sum<64>(v); }

// f(std::integral_constant<int, I>) for I = B .. E - 1: register arrays indexed by it keep
// constant indices (a #pragma unroll loop unrolled after SROA leaves its array in scratch)
template <int B, int E, typename Fn>
__device__ __forceinline__ void static_for(Fn&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// a workgroup barrier ordering LDS only: this wave's LDS traffic completes (lgkmcnt), global
// loads stay in flight across it (a __syncthreads() waits for every outstanding global access)
__device__ __forceinline__ void lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// the edge range of a block's row v: CSR (stride 0) or the fixed-stride layout of regnn_ns_hop
// strided (row v at v * stride, its cnt[v] sampled edges then its self loop)
__device__ __forceinline__ void row_range(const int32_t* ptr, const int32_t* cnt, int stride,
                                          int v, int& e0, int& e1) {
    if (stride) {
        e0 = v * stride;
        e1 = e0 + cnt[v] + 1;
    } else {
        e0 = ptr[v];
        e1 = ptr[v + 1];
    }
}

inline Drop make_drop(float p) {
    Drop d{};
    d.on = p > 0.f;
    const float keep = 1.f - p;
    int k16 = int(keep * 65536.f + 0.5f);
    if (k16 > 65536) k16 = 65536;
    d.thresh = uint32_t(k16);
    d.scale = d.on ? 1.f / keep : 1.f;
    d.b8 = (k16 % 256) == 0;
    return d;
}

// raise a kernel's dynamic-LDS limit to `bytes` once (the largest size asked so far is kept)
inline bool set_lds(const void* k, size_t bytes, size_t* done) {
    if (bytes <= 64 * 1024 || bytes <= *done) return true;
    if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, int(bytes)) !=
        hipSuccess)
        return false;
    *done = bytes;
    return true;
}

}  // namespace nsm
}  // namespace regnn

// the two-layer step (re_nsm2.hip), dispatched by regnn_nsm_step / regnn_nsm_slab_floats
bool regnn_nsm2_covers(const regnn_nsm_params* p);
int64_t regnn_nsm2_slab_floats(const regnn_nsm_params* p, int32_t cap0);
int regnn_nsm2_step(const regnn_nsm_params* p, const regnn_nsm_work* w, hipStream_t stream);
// re_nsm.hip's edge pass of layer 0's relation-table dots (rel0), into `slab` (kAggBlocks rows)
int regnn_nsm_rel0(const regnn_nsm_params* p, const regnn_nsm_work* w, float* slab,
                   hipStream_t stream);
