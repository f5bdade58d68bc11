// Random row-gather ceiling on one MI355X: how fast can a kernel fetch B-byte rows at random
// indices out of a table far larger than L2 + Infinity Cache? This is the roofline the SpMM
// gathers actually face (an fp32 F=64 row is 256 B, a bf16 row 128 B). Test infrastructure, not
// product code.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/gather_probe tools/gather_probe.hip
// Run:   tools/gather_probe            (prints one line per row size / index order)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <random>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); std::exit(1); } } while (0)

// LPR lanes x 16 B per row; each lane group keeps UN rows in flight.
template <int LPR, int UN>
__global__ void __launch_bounds__(256) gather_kernel(const uint4* __restrict__ tab,
                                                     const int* __restrict__ idx, int64_t m,
                                                     float* __restrict__ out) {
  const int lane = threadIdx.x % LPR;
  const int64_t group = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) / LPR;
  const int64_t groups = int64_t(gridDim.x) * blockDim.x / LPR;
  float acc = 0.f;
  for (int64_t base = group * UN; base < m; base += groups * UN) {
    uint4 v[UN];
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      const int64_t e = base + u;
      const int r = e < m ? __builtin_nontemporal_load(idx + e) : 0;
      v[u] = tab[int64_t(r) * LPR + lane];
    }
#pragma unroll
    for (int u = 0; u < UN; ++u)
      if (base + u < m)
        acc += __uint_as_float(v[u].x) + __uint_as_float(v[u].y) + __uint_as_float(v[u].z) +
               __uint_as_float(v[u].w);
  }
  out[int64_t(blockIdx.x) * blockDim.x + threadIdx.x] = acc;
}

template <int LPR, int UN>
static float run(const uint4* tab, const int* idx, int64_t m, float* out, int blocks) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL((gather_kernel<LPR, UN>), dim3(blocks), dim3(256), 0, 0, tab, idx, m, out);
  CK(hipEventRecord(a));
  const int reps = 5;
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((gather_kernel<LPR, UN>), dim3(blocks), dim3(256), 0, 0, tab, idx, m, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms / reps;
}

template <int LPR, int UN>
static void probe(const uint4* tab, int64_t tab_bytes, int* d_idx, int64_t m, float* out,
                  int blocks, const char* order, std::vector<int>& h_idx) {
  const int64_t rows = tab_bytes / (16 * LPR);
  std::mt19937_64 rng(LPR * 1000 + UN);
  std::uniform_int_distribution<int> dist(0, int(rows - 1));
  for (auto& x : h_idx) x = dist(rng);
  if (order[0] == 's') std::sort(h_idx.begin(), h_idx.end());
  CK(hipMemcpy(d_idx, h_idx.data(), m * sizeof(int), hipMemcpyHostToDevice));
  const float ms = run<LPR, UN>(tab, d_idx, m, out, blocks);
  const double row_b = 16.0 * LPR, gathered = row_b * m, with_idx = gathered + 4.0 * m;
  std::printf("row %4d B  UN %2d  %-6s  %8.3f ms  %6.2f G rows/s  %6.3f TB/s rows  %6.3f TB/s rows+idx\n",
              int(row_b), UN, order, ms, m / ms / 1e6, gathered / ms / 1e9, with_idx / ms / 1e9);
}

int main() {
  const int64_t tab_bytes = int64_t(8) << 30;  // 8 GiB: 32x L2 + Infinity Cache
  const int64_t m = int64_t(1) << 26;          // 67 M gathers per launch
  uint4* tab;
  int* idx;
  float* out;
  CK(hipMalloc(&tab, tab_bytes));
  CK(hipMemset(tab, 0, tab_bytes));
  CK(hipMalloc(&idx, m * sizeof(int)));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int blocks = cus * 8;
  CK(hipMalloc(&out, int64_t(blocks) * 256 * sizeof(float)));
  std::vector<int> h(m);
  for (const char* order : {"random", "sorted"}) {
    probe<4, 8>(tab, tab_bytes, idx, m, out, blocks, order, h);     // 64 B rows
    probe<8, 8>(tab, tab_bytes, idx, m, out, blocks, order, h);     // 128 B rows (bf16 F=64)
    probe<8, 16>(tab, tab_bytes, idx, m, out, blocks, order, h);
    probe<16, 8>(tab, tab_bytes, idx, m, out, blocks, order, h);    // 256 B rows (fp32 F=64)
    probe<32, 4>(tab, tab_bytes, idx, m, out, blocks, order, h);    // 512 B rows
  }
  CK(hipFree(tab));
  CK(hipFree(idx));
  CK(hipFree(out));
  return 0;
}
