// Microbenchmark: same-address device-scope atomics from many workgroups (the list counters of
// k_tail_local / k_small_screen's flushes).  G workgroups x 256 threads; thread t < L of each
// workgroup adds 1 to counter t (each on its own 128-B line) and (mode 1) uses the returned value,
// mode 0 does no atomics, mode 2 uses one counter line per workgroup % 16 ("striped").
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_atomics.hip -o tools/ubench_atomics
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void k(unsigned* ctr, unsigned* out, int lists, int mode) {
  const unsigned t = threadIdx.x;
  unsigned v = 0;
  if (t < (unsigned)lists) {
    if (mode == 1) v = atomicAdd(&ctr[t * 32], 1u);
    else if (mode == 2) v = atomicAdd(&ctr[(t * 16 + (blockIdx.x & 15)) * 32], 1u);
    else v = t;
  }
  __syncthreads();
  if (t < (unsigned)lists) out[blockIdx.x * 64 + t] = v;
}

int main(int argc, char** argv) {
  const int lists = argc > 1 ? atoi(argv[1]) : 19;
  unsigned *ctr, *out;
  hipMalloc(&ctr, 64 * 16 * 32 * 4);
  hipMalloc(&out, 8192 * 64 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int mode = 0; mode < 3; ++mode)
    for (int g : {128, 256, 512, 1024, 2048, 4096}) {
      float best = 1e9f;
      for (int rep = 0; rep < 20; ++rep) {
        hipMemset(ctr, 0, 64 * 16 * 32 * 4);
        hipEventRecord(a);
        k<<<g, 256>>>(ctr, out, lists, mode);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
      }
      printf("mode %d (%s) workgroups %5d lists %2d: %8.2f us\n", mode,
             mode == 0 ? "none" : mode == 1 ? "same address" : "16-way striped", g, lists, best * 1e3);
    }
  return 0;
}
