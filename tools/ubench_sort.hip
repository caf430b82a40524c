// Microbenchmark of the bucket sort (klsh_sort.hip) and the device scan.  Build: make -C kmerlsh_amd/csrc ubench; run: tools/ubench_sort N BITS REPS.
#include <hip/hip_runtime.h>
#include <hipcub/device/device_radix_sort.hpp>  // reference point only: the library's stable radix sort

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <vector>

#include "klsh_device.h"

namespace klsh {
struct DstCopyExcl {  // out[i] = exclusive prefix (src read-only)
  uint32_t* out;
  const uint32_t* unused;
  __device__ void operator()(uint32_t i, uint32_t prefix, uint32_t) const { out[i] = prefix; }
};
}  // namespace klsh

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atol(argv[1]) : 9469536u;
  const int bits = argc > 2 ? atoi(argv[2]) : 23;
  const int reps = argc > 3 ? atoi(argv[3]) : 20;
  std::vector<uint32_t> keys(n);
  uint64_t x = 88172645463325252ull;
  for (auto& k : keys) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    k = (uint32_t)(x >> 20) & ((bits >= 32) ? 0xFFFFFFFFu : ((1u << bits) - 1u));
  }
  uint32_t *k0, *v0, *k1, *v1, *ws, *ts, *kk, *vv;
  klsh::Counters* ctr;
  const size_t wsw = klsh::sort_ws_words(n), tsw = klsh::scan_ws_words(n);
  CK(hipMalloc(&k0, 4ull * n)); CK(hipMalloc(&v0, 4ull * n));
  CK(hipMalloc(&k1, 4ull * n)); CK(hipMalloc(&v1, 4ull * n));
  CK(hipMalloc(&kk, 4ull * n)); CK(hipMalloc(&vv, 4ull * n));
  CK(hipMalloc(&ws, 4 * wsw)); CK(hipMalloc(&ts, 4 * tsw)); CK(hipMalloc(&ctr, sizeof(klsh::Counters)));
  CK(hipMemset(ws, 0, 4 * wsw)); CK(hipMemset(ts, 0, 4 * tsw)); CK(hipMemset(ctr, 0, sizeof(klsh::Counters)));
  std::vector<uint32_t> iota(n);
  std::iota(iota.begin(), iota.end(), 0u);
  CK(hipMemcpy(kk, keys.data(), 4ull * n, hipMemcpyHostToDevice));
  CK(hipMemcpy(vv, iota.data(), 4ull * n, hipMemcpyHostToDevice));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  uint32_t *ok = nullptr, *ov = nullptr;
  float sort_ms = 0, scan_ms = 0;
  for (int r = 0; r < reps + 2; ++r) {
    CK(hipMemcpyAsync(k0, kk, 4ull * n, hipMemcpyDeviceToDevice, s));
    CK(hipMemcpyAsync(v0, vv, 4ull * n, hipMemcpyDeviceToDevice, s));
    CK(hipEventRecord(a, s));
    klsh::radix_sort(k0, v0, k1, v1, n, bits, ws, &ok, &ov, s);
    CK(hipEventRecord(b, s));
    CK(hipStreamSynchronize(s));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r >= 2) sort_ms += ms;
  }
  // the same sort through hipCUB / rocPRIM (onesweep), timed the same way, checked below
  float lib_ms = 0;
  {
    size_t tb = 0;
    CK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k0, k1, v0, v1, n, 0, bits, s));
    void* tmp;
    CK(hipMalloc(&tmp, tb));
    for (int r = 0; r < reps + 2; ++r) {
      CK(hipMemcpyAsync(k0, kk, 4ull * n, hipMemcpyDeviceToDevice, s));
      CK(hipMemcpyAsync(v0, vv, 4ull * n, hipMemcpyDeviceToDevice, s));
      CK(hipEventRecord(a, s));
      CK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, k0, k1, v0, v1, n, 0, bits, s));
      CK(hipEventRecord(b, s));
      CK(hipStreamSynchronize(s));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (r >= 2) lib_ms += ms;
    }
    CK(hipFree(tmp));
  }
  std::vector<uint32_t> lp(n);
  CK(hipMemcpy(lp.data(), v1, 4ull * n, hipMemcpyDeviceToHost));
  // verify (our sort ran again so ok/ov hold its output)
  for (int r = 0; r < 1; ++r) {
    CK(hipMemcpyAsync(k0, kk, 4ull * n, hipMemcpyDeviceToDevice, s));
    CK(hipMemcpyAsync(v0, vv, 4ull * n, hipMemcpyDeviceToDevice, s));
    klsh::radix_sort(k0, v0, k1, v1, n, bits, ws, &ok, &ov, s);
    CK(hipStreamSynchronize(s));
  }
  std::vector<uint32_t> gp(n), gk(n);
  CK(hipMemcpy(gp.data(), ov, 4ull * n, hipMemcpyDeviceToHost));
  CK(hipMemcpy(gk.data(), ok, 4ull * n, hipMemcpyDeviceToHost));
  std::vector<uint32_t> want(iota);
  std::stable_sort(want.begin(), want.end(), [&](uint32_t i, uint32_t j) { return keys[i] < keys[j]; });
  const bool sort_ok = gp == want;
  printf("hipcub SortPairs %s %.1f us\n", lp == want ? "ok" : "BAD", 1e3 * lib_ms / reps);
  // scan: exclusive prefix of the (unsorted) keys into a buffer of its own
  for (int r = 0; r < reps + 2; ++r) {
    CK(hipEventRecord(a, s));
    klsh::device_scan(klsh::SrcArray{kk}, klsh::DstCopyExcl{vv == ov ? v1 : (ov == v1 ? v0 : v1), kk}, n, ts, &ctr->total, &ctr->err, s);
    CK(hipEventRecord(b, s));
    CK(hipStreamSynchronize(s));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r >= 2) scan_ms += ms;
  }
  std::vector<uint32_t> sc(n);
  CK(hipMemcpy(sc.data(), ov == v1 ? v0 : v1, 4ull * n, hipMemcpyDeviceToHost));
  uint32_t run = 0;
  bool scan_ok = true;
  for (uint32_t i = 0; i < n; ++i) {
    scan_ok = scan_ok && sc[i] == run;
    run += keys[i];
  }
  klsh::Counters hc;
  CK(hipMemcpy(&hc, ctr, sizeof(hc), hipMemcpyDeviceToHost));
  printf("n=%u bits=%d sort=%s %.1f us  scan=%s %.1f us  total=%u (want %u) err=%u\n",
         n, bits, sort_ok ? "ok" : "BAD", 1e3 * sort_ms / reps, scan_ok ? "ok" : "BAD",
         1e3 * scan_ms / reps, hc.total, run, hc.err);
  return sort_ok && scan_ok && hc.err == 0 ? 0 : 1;
}
