// Probe: do v_mfma_f32_32x32x16_f16, v_dot2_f32_f16 and v_cvt_f16_f32 keep fp16 subnormals on
// gfx950 under the default HIP float mode?  (The certified screens' bounds assume they do; the
// printout decides whether the bound needs the flush-safe 2^-14 absolute term.)
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f16v __attribute__((ext_vector_type(16)));
__global__ void probe(float* out, float tiny) {
  const int lane = threadIdx.x;
  h8 a, b;
  for (int e = 0; e < 8; ++e) { a[e] = (_Float16)(lane == 0 && e == 0 ? tiny : 0.0f); b[e] = (_Float16)1.0f; }
  f16v acc;
  for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
  const h2 x = {(_Float16)tiny, (_Float16)0.0f}, y = {(_Float16)1.0f, (_Float16)0.0f};
  const float d2 = __builtin_amdgcn_fdot2(x, y, 0.0f, false);
  if (lane == 0) {
    out[0] = acc[0];                       // A[0][0..7] . B[0..7][0] = tiny (row 0, col 0)
    out[1] = d2;                           // tiny * 1
    out[2] = (float)(_Float16)tiny;        // the conversion itself
  }
}
int main() {
  float* d;
  (void)hipMalloc(&d, 16);
  const float tiny = 3.0e-6f;  // fp16 subnormal (min normal 6.1e-5)
  probe<<<1, 64>>>(d, tiny);
  float h[3];
  (void)hipMemcpy(h, d, 12, hipMemcpyDeviceToHost);
  printf("input %.9g (fp16 subnormal)\nmfma_f16: %.9g\nfdot2: %.9g\ncvt_f16: %.9g\n", tiny, h[0], h[1], h[2]);
  printf("%s\n", (h[0] != 0.0f && h[1] != 0.0f && h[2] != 0.0f) ? "subnormals kept" : "FLUSHED somewhere");
  return 0;
}
