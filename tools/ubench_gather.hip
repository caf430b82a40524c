// Row-gather bandwidth on the projection's access pattern: N rows of 64 fp32 (256 B) read in a
// random slot order (the canonical order of a late iteration) vs in slot order, one lane per row.
// Prints GB/s of row bytes; the practical ceiling the projection kernel is measured against.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_gather.hip -o tools/ubench_gather
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

__global__ __launch_bounds__(256) void k_gather(const float4* __restrict__ X,
                                                const uint32_t* __restrict__ slots, uint32_t n,
                                                uint32_t* __restrict__ out) {
  const uint32_t p = blockIdx.x * 256u + threadIdx.x;
  if (p >= n) return;
  const float4* r = X + (size_t)slots[p] * 16;
  float s = 0.0f;
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const float4 v = r[m];
    s += v.x + v.y + v.z + v.w;
  }
  out[p] = s >= 0.0f ? 1u : 0u;
}

int main() {
  const uint32_t n = 10000000;
  std::vector<uint32_t> perm(n);
  std::iota(perm.begin(), perm.end(), 0u);
  float4* X;
  uint32_t *slots, *out;
  hipMalloc(&X, sizeof(float4) * 16 * (size_t)n);
  hipMalloc(&slots, 4ull * n);
  hipMalloc(&out, 4ull * n);
  hipMemset(X, 0, sizeof(float4) * 16 * (size_t)n);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int shuffled = 0; shuffled < 2; ++shuffled) {
    if (shuffled) std::shuffle(perm.begin(), perm.end(), std::mt19937(7));
    hipMemcpy(slots, perm.data(), 4ull * n, hipMemcpyHostToDevice);
    for (int w = 0; w < 3; ++w) k_gather<<<(n + 255) / 256, 256>>>(X, slots, n, out);
    hipEventRecord(a);
    const int reps = 20;
    for (int w = 0; w < reps; ++w) k_gather<<<(n + 255) / 256, 256>>>(X, slots, n, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double bytes = (double)n * (256 + 8);
    printf("%s: %.1f us per pass, %.0f GB/s (row + slot + key bytes)\n",
           shuffled ? "random slot order" : "slot order", ms * 1e3 / reps, bytes / (ms / reps * 1e-3) / 1e9);
  }
  return 0;
}
