// Store ceiling of the fused output head's logits on one MI355X: 19.4 M rows x 352 fp32 (27 GB,
// run_regnn.py:146's all-node logits at mag-10x) written with different per-instruction shapes.
// Test infrastructure, not product code.
//
//   coalesced  a wave stores 1 KiB contiguous per instruction (grid-stride over the buffer)
//   tile16     the head kernel's shape: a wave owns 16 rows; per instruction lane (row c, quarter
//              q) stores 16 B at column 16 t + 4 q -> 16 rows x 64 B
//   line128    8 lanes per row, 8 rows per instruction: 128 B of one row per 8 lanes
//   rowstage   a wave owns 16 rows and stores them one row at a time, 1 KiB + 384 B per row
//              (what an LDS-staged tile store would issue)
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/store_probe tools/store_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); std::exit(1); } } while (0)

constexpr int64_t kRows = 19397430;
constexpr int kLd = 352;                 // floats per row (349 classes padded to 16)

__global__ void __launch_bounds__(256) coalesced(float4* __restrict__ out, int64_t n4) {
  const float4 v = make_float4(1.f, 2.f, 3.f, 4.f);
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n4; i += int64_t(gridDim.x) * 256)
    out[i] = v;
}

__global__ void __launch_bounds__(512) tile16(float* __restrict__ out, int64_t rows) {
  const int lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4;
  const int64_t tiles = (rows + 15) / 16;
  const float4 v = make_float4(1.f, 2.f, 3.f, 4.f);
  for (int64_t tile = int64_t(blockIdx.x) * 8 + (threadIdx.x >> 6); tile < tiles;
       tile += int64_t(gridDim.x) * 8) {
    const int64_t row = tile * 16 + c;
    if (row >= rows) continue;
    float* r = out + row * kLd + 4 * q;
#pragma unroll
    for (int t = 0; t < kLd / 16; ++t) *reinterpret_cast<float4*>(r + 16 * t) = v;
  }
}

__global__ void __launch_bounds__(512) line128(float* __restrict__ out, int64_t rows) {
  const int lane = threadIdx.x & 63, c = lane >> 3, j = lane & 7;   // 8 rows x 8 lanes
  const int64_t tiles = (rows + 15) / 16;
  const float4 v = make_float4(1.f, 2.f, 3.f, 4.f);
  for (int64_t tile = int64_t(blockIdx.x) * 8 + (threadIdx.x >> 6); tile < tiles;
       tile += int64_t(gridDim.x) * 8) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t row = tile * 16 + 8 * h + c;
      if (row >= rows) continue;
      float* r = out + row * kLd + 4 * j;
#pragma unroll
      for (int t = 0; t < kLd / 32; ++t) *reinterpret_cast<float4*>(r + 32 * t) = v;
    }
  }
}

__global__ void __launch_bounds__(512) rowstage(float* __restrict__ out, int64_t rows) {
  const int lane = threadIdx.x & 63;
  const int64_t tiles = (rows + 15) / 16;
  const float4 v = make_float4(1.f, 2.f, 3.f, 4.f);
  for (int64_t tile = int64_t(blockIdx.x) * 8 + (threadIdx.x >> 6); tile < tiles;
       tile += int64_t(gridDim.x) * 8) {
    for (int c = 0; c < 16; ++c) {
      const int64_t row = tile * 16 + c;
      if (row >= rows) break;
      float4* r = reinterpret_cast<float4*>(out + row * kLd);
      r[lane] = v;                                   // 1 KiB
      if (lane < kLd / 4 - 64) r[64 + lane] = v;     // the remaining 384 B
    }
  }
}

template <typename F>
static void timeit(const char* name, F launch, double bytes) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  launch();
  CK(hipEventRecord(a));
  const int reps = 5;
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  std::printf("%-10s %8.3f ms  %6.2f TB/s\n", name, ms, bytes / (ms * 1e-3) / 1e12);
}

int main() {
  const int64_t n = kRows * kLd;
  float* out;
  CK(hipMalloc(&out, n * sizeof(float)));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const double bytes = double(n) * 4;
  timeit("coalesced", [&] { hipLaunchKernelGGL(coalesced, dim3(cus * 8), dim3(256), 0, 0,
                                               reinterpret_cast<float4*>(out), n / 4); }, bytes);
  for (int occ : {2, 4}) {
    std::printf("-- %d blocks of 512 per CU\n", occ);
    timeit("tile16", [&] { hipLaunchKernelGGL(tile16, dim3(cus * occ), dim3(512), 0, 0, out, kRows); }, bytes);
    timeit("line128", [&] { hipLaunchKernelGGL(line128, dim3(cus * occ), dim3(512), 0, 0, out, kRows); }, bytes);
    timeit("rowstage", [&] { hipLaunchKernelGGL(rowstage, dim3(cus * occ), dim3(512), 0, 0, out, kRows); }, bytes);
  }
  CK(hipFree(out));
  return 0;
}
