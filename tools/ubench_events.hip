// Do stream-ordered HIP event pairs time only their own stream's kernel?  
// Stream A runs a long spin kernel; stream B (forked from A by an event, like the merge streams)
// records e0, runs a short spin kernel, records e1.  Printed: elapsed(e0, e1) against the short
// kernel's own in-kernel duration (s_memrealtime, 100 MHz), for several layouts.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void spin(uint64_t ticks, uint64_t* out) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {}
  if (out && threadIdx.x == 0 && blockIdx.x == 0) *out = __builtin_amdgcn_s_memrealtime() - t0;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
  hipStream_t a, b, c;
  int lo, hi;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  CK(hipStreamCreateWithPriority(&a, hipStreamNonBlocking, hi));
  CK(hipStreamCreateWithPriority(&b, hipStreamNonBlocking, lo));
  CK(hipStreamCreateWithPriority(&c, hipStreamNonBlocking, lo));
  hipEvent_t e0, e1, ea0, ea1, fork;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&ea0)); CK(hipEventCreate(&ea1));
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  uint64_t* d; CK(hipMalloc(&d, 64));
  for (int layout = 0; layout < 4; ++layout) {
    for (int rep = 0; rep < 3; ++rep) {
      // 0: B alone; 1: long kernel on A concurrently (A small grid); 2: long kernel on A filling the
      // chip; 3: like 2 plus a third stream with its own event pair
      CK(hipEventRecord(fork, a));
      CK(hipStreamWaitEvent(b, fork, 0));
      CK(hipStreamWaitEvent(c, fork, 0));
      if (layout >= 1) {
        CK(hipEventRecord(ea0, a));
        spin<<<layout >= 2 ? 2048 : 8, 256, 0, a>>>(50000, nullptr);  // 500 us
        CK(hipEventRecord(ea1, a));
      }
      CK(hipEventRecord(e0, b));
      spin<<<8, 64, 0, b>>>(5000, d);  // 50 us
      CK(hipEventRecord(e1, b));
      if (layout == 3) spin<<<8, 64, 0, c>>>(5000, nullptr);
      CK(hipDeviceSynchronize());
      float ms = 0, msa = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (layout >= 1) CK(hipEventElapsedTime(&msa, ea0, ea1));
      uint64_t k = 0; CK(hipMemcpy(&k, d, 8, hipMemcpyDeviceToHost));
      printf("layout %d rep %d: B events %.1f us, B kernel %.1f us, A events %.1f us\n", layout, rep,
             ms * 1e3, k * 0.01, msa * 1e3);
    }
  }
  return 0;
}
