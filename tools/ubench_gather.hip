// Row-gather bandwidth on the projection's access pattern: N rows of W fp32 read in a random slot
// order (the canonical order of a late iteration) vs in slot order, one lane per row.
// Prints GB/s of row bytes; the practical ceiling the projection kernel is measured against.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_gather.hip -o tools/ubench_gather
//   tools/ubench_gather [N = 10000000] [W = 64 (C2) | 32 (C4: N = 100000000)] [contig = 0 | 1]
// contig = 1 allocates the rows with hipDeviceMallocContiguous (physically contiguous)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

template <int Q>  // float4s per row
__global__ __launch_bounds__(256) void k_gather(const float4* __restrict__ X,
                                                const uint32_t* __restrict__ slots, uint32_t n,
                                                uint32_t* __restrict__ out) {
  const uint32_t p = blockIdx.x * 256u + threadIdx.x;
  if (p >= n) return;
  const float4* r = X + (size_t)slots[p] * Q;
  float s = 0.0f;
#pragma unroll
  for (int m = 0; m < Q; ++m) {
    const float4 v = r[m];
    s += v.x + v.y + v.z + v.w;
  }
  out[p] = s >= 0.0f ? 1u : 0u;
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atol(argv[1]) : 10000000u;
  const int wf = argc > 2 ? atoi(argv[2]) : 64;
  if (wf != 32 && wf != 64) return 1;
  const int q = wf / 4;
  auto launch = [&](const float4* X, const uint32_t* slots, uint32_t* out) {
    if (q == 16) k_gather<16><<<(n + 255) / 256, 256>>>(X, slots, n, out);
    else k_gather<8><<<(n + 255) / 256, 256>>>(X, slots, n, out);
  };
  std::vector<uint32_t> perm(n);
  std::iota(perm.begin(), perm.end(), 0u);
  float4* X;
  uint32_t *slots, *out;
  const bool contig = argc > 3 && atoi(argv[3]) != 0;
  if (contig) {
    if (hipExtMallocWithFlags(reinterpret_cast<void**>(&X), sizeof(float4) * q * (size_t)n,
                              hipDeviceMallocContiguous) != hipSuccess) {
      printf("contiguous allocation failed\n");
      return 2;
    }
  } else {
    (void)hipMalloc(&X, sizeof(float4) * q * (size_t)n);
  }
  hipMalloc(&slots, 4ull * n);
  hipMalloc(&out, 4ull * n);
  hipMemset(X, 0, sizeof(float4) * q * (size_t)n);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int shuffled = 0; shuffled < 2; ++shuffled) {
    if (shuffled) std::shuffle(perm.begin(), perm.end(), std::mt19937(7));
    hipMemcpy(slots, perm.data(), 4ull * n, hipMemcpyHostToDevice);
    for (int w = 0; w < 3; ++w) launch(X, slots, out);
    hipEventRecord(a);
    const int reps = 20;
    for (int w = 0; w < reps; ++w) launch(X, slots, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double bytes = (double)n * (4.0 * wf + 8);
    printf("N %u, %d-B rows%s, %s: %.1f us per pass, %.0f GB/s (row + slot + key bytes)\n",
           n, 4 * wf, contig ? " (contiguous)" : "", shuffled ? "random slot order" : "slot order", ms * 1e3 / reps, bytes / (ms / reps * 1e-3) / 1e9);
  }
  return 0;
}
