// gfx950 (CDNA4) kernels for the kmerLSH cluster loop.
//
// Numerics contract: the reference is scalar SSE fp32 with no FMA, so every dot
// product here is a strictly sequential chain of separately rounded multiplies and adds
// (this file is compiled with -ffp-contract=off; tests/test_isa.py checks the code object has no
// v_fma/v_fmac/v_pk_fma in these kernels), sqrt and division are the correctly rounded IEEE
// operations (hipcc default; never -fno-hip-fp32-correctly-rounded-divide-sqrt).  Parallelism
// comes from rows, pairs and buckets — never from splitting one dot product.
//
// Kernels (per LSH iteration):
//   k_project       sign-hash every live row   (reference hash/lshash.cc:44-59, cluster.cc:232-237)
//   k_radix_*       stable bucketing by key    (reference cluster.cc:15-30 merge_hashtable)
//   k_merge_small   greedy merge, lane/bucket  (reference cluster.cc:56-87 p_cluster,
//   k_merge_large   greedy merge, wave/bucket   distance.cc:27-38, funcAB.cc:49-71)
//   k_scan_*        survivor compaction        (reference cluster.cc:39-45 merge_abundance)
#include <hip/hip_runtime.h>

#include <stdlib.h>

#include <string>
#include <type_traits>

#include "klsh_device.h"

namespace klsh {

// ========================================================================= projection ==========
// Packed-f32 projection.  The same sequential chains as k_project, two per instruction:
// v_pk_mul_f32 / v_pk_add_f32 round each half exactly like v_mul_f32 / v_add_f32 (no fusion,
// -ffp-contract=off), so the keys are bit-identical, at twice the f32 VALU issue rate — the
// unpacked kernel sits at the non-packed VALU ceiling (2·h·d single-rate ops per row), not at HBM.
// Hyperplanes sit in LDS as [h/4][D] float4 quads (w_4q[k], w_4q+1[k], w_4q+2[k], w_4q+3[k]), so
// one broadcast ds_read_b128 feeds 4 chains at column k; h is padded to a multiple of 4 with
// zero hyperplanes whose bits are dropped.  CH quads (4·CH chains) run at once for ILP.
typedef float f32x2 __attribute__((ext_vector_type(2)));


// acc + w * (x, x), x one half of a register pair (op_sel picks the half; no register copies).
// Multiply and add stay one asm block so the scheduler cannot hoist the products of every
// column ahead of the chain (that spilled); both are separately rounded, never fused.
__device__ __forceinline__ void pk_mac_lo(f32x2& acc, f32x2 w, f32x2 x) {
  f32x2 t;
  asm("v_pk_mul_f32 %1, %2, %3 op_sel_hi:[1,0]\n\tv_pk_add_f32 %0, %0, %1"
      : "+v"(acc), "=&v"(t) : "v"(w), "v"(x));
}
__device__ __forceinline__ void pk_mac_hi(f32x2& acc, f32x2 w, f32x2 x) {
  f32x2 t;
  asm("v_pk_mul_f32 %1, %2, %3 op_sel:[0,1] op_sel_hi:[1,1]\n\tv_pk_add_f32 %0, %0, %1"
      : "+v"(acc), "=&v"(t) : "v"(w), "v"(x));
}

// RPL rows per lane (rows p and p + 256 of the workgroup's 256 * RPL): every hyperplane read
// from LDS feeds RPL rows — the single-row kernel is bound by the LDS broadcast reads about as
// much as by the VALU.
// n_dev (may be null): the row count lives on the device (an iteration queued before the
// previous one's survivors were counted); then h = floor(log2 n) (cluster.cc:194) is derived here.
template <int D, int CH, int RPL>
__global__ __launch_bounds__(256) void k_project_pk(const float* __restrict__ X, int dp,
                                                    const uint32_t* __restrict__ slots,
                                                    uint32_t* __restrict__ keys, uint32_t n,
                                                    const float* __restrict__ W, int h,
                                                    uint32_t key_or,
                                                    const uint32_t* __restrict__ n_dev = nullptr,
                                                    KTime kt = kNoTime,
                                                    const uint32_t* __restrict__ woff_dev = nullptr) {
  constexpr int QMAX = kMaxHyperplanes / 4;
  __shared__ __attribute__((aligned(16))) float4 sw[QMAX * D];
  kt_fold(kt);
  kt_begin(kt, KC_PROJECT);
  if (n_dev) {
    n = *n_dev;
    if (n == 0) return;
    h = 31 - __builtin_clz(n);
    if (woff_dev) W += (size_t)*woff_dev * dp;
  }
  const int nq = (h + 3) >> 2;
  for (int i = threadIdx.x; i < nq * D; i += 256) {
    const int q = i / D, k = i % D;
    float4 v;
    v.x = 4 * q + 0 < h ? W[(4 * q + 0) * dp + k] : 0.0f;
    v.y = 4 * q + 1 < h ? W[(4 * q + 1) * dp + k] : 0.0f;
    v.z = 4 * q + 2 < h ? W[(4 * q + 2) * dp + k] : 0.0f;
    v.w = 4 * q + 3 < h ? W[(4 * q + 3) * dp + k] : 0.0f;
    sw[i] = v;
  }
  const uint32_t p0 = blockIdx.x * (256u * RPL) + threadIdx.x;
  __syncthreads();
  if (p0 >= n) return;
  f32x2 x[RPL][D / 2];  // (x[2m], x[2m+1]) of each row
#pragma unroll
  for (int r = 0; r < RPL; ++r) {
    const uint32_t pr = p0 + 256u * r;
    const float4* src = reinterpret_cast<const float4*>(X + (size_t)slots[pr < n ? pr : p0] * dp);
#pragma unroll
    for (int m = 0; m < D / 4; ++m) {
      const float4 v = src[m];
      x[r][2 * m] = (f32x2){v.x, v.y};
      x[r][2 * m + 1] = (f32x2){v.z, v.w};
    }
  }
  uint32_t key[RPL];
#pragma unroll
  for (int r = 0; r < RPL; ++r) key[r] = 0;
  auto quads = [&](int q, auto ch) {
    constexpr int C = decltype(ch)::value;
    f32x2 a[RPL][C][2];
#pragma unroll
    for (int r = 0; r < RPL; ++r)
#pragma unroll
      for (int c = 0; c < C; ++c) a[r][c][0] = a[r][c][1] = (f32x2){0.0f, 0.0f};
#pragma unroll
    for (int k = 0; k < D; ++k) {
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const float4 w = sw[(q + c) * D + k];
        const f32x2 w01 = (f32x2){w.x, w.y}, w23 = (f32x2){w.z, w.w};
#pragma unroll
        for (int r = 0; r < RPL; ++r) {
          if (k & 1) {
            pk_mac_hi(a[r][c][0], w01, x[r][k / 2]);
            pk_mac_hi(a[r][c][1], w23, x[r][k / 2]);
          } else {
            pk_mac_lo(a[r][c][0], w01, x[r][k / 2]);
            pk_mac_lo(a[r][c][1], w23, x[r][k / 2]);
          }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < RPL; ++r)
#pragma unroll
      for (int c = 0; c < C; ++c)
        key[r] = key[r] * 16u + (a[r][c][0].x >= 0.0f ? 8u : 0u) +
                 (a[r][c][0].y >= 0.0f ? 4u : 0u) + (a[r][c][1].x >= 0.0f ? 2u : 0u) +
                 (a[r][c][1].y >= 0.0f ? 1u : 0u);
  };
  int q = 0;
  for (; q + CH <= nq; q += CH) quads(q, std::integral_constant<int, CH>{});
  for (; q < nq; ++q) quads(q, std::integral_constant<int, 1>{});
#pragma unroll
  for (int r = 0; r < RPL; ++r) {
    const uint32_t pr = p0 + 256u * r;
    if (pr < n) keys[pr] = (key[r] >> (uint32_t)(4 * nq - h)) | key_or;  // drop padding bits
  }
  kt_end(kt, KC_PROJECT);
}

// Wide rows (d > 64 or any width without a register kernel), packed f32: every lane keeps the
// chains of all h hyperplanes (up to 8 quads = 16 register pairs) and streams its row through
// in 16-B pieces, in k order, so each chain is still the reference's sequential sum.  The
// hyperplanes sit in LDS as [k][quad] float4 (one broadcast ds_read_b128 feeds 4 chains).
template <int RPL>
__global__ __launch_bounds__(256) void k_project_wide_pk(const float* __restrict__ X, int d,
                                                         int dp, const uint32_t* __restrict__ slots,
                                                         uint32_t* __restrict__ keys, uint32_t n,
                                                         const float* __restrict__ W, int h,
                                                         uint32_t key_or, KTime kt) {
  extern __shared__ __attribute__((aligned(16))) float4 swq[];  // [dp][nq]
  constexpr int QMAX = kMaxHyperplanes / 4;
  kt_fold(kt);
  kt_begin(kt, KC_PROJECT);
  const int nq = (h + 3) >> 2;
  for (int i = threadIdx.x; i < dp * nq; i += 256) {
    const int k = i / nq, q = i % nq;
    float4 v;
    v.x = 4 * q + 0 < h ? W[(4 * q + 0) * dp + k] : 0.0f;
    v.y = 4 * q + 1 < h ? W[(4 * q + 1) * dp + k] : 0.0f;
    v.z = 4 * q + 2 < h ? W[(4 * q + 2) * dp + k] : 0.0f;
    v.w = 4 * q + 3 < h ? W[(4 * q + 3) * dp + k] : 0.0f;
    swq[i] = v;
  }
  const uint32_t p0 = blockIdx.x * (256u * RPL) + threadIdx.x;
  __syncthreads();
  if (p0 >= n) return;
  const float* x[RPL];
#pragma unroll
  for (int r = 0; r < RPL; ++r) {
    const uint32_t pr = p0 + 256u * r;
    x[r] = X + (size_t)slots[pr < n ? pr : p0] * dp;
  }
  f32x2 a[RPL][QMAX][2];
#pragma unroll
  for (int r = 0; r < RPL; ++r)
#pragma unroll
    for (int q = 0; q < QMAX; ++q) a[r][q][0] = a[r][q][1] = (f32x2){0.0f, 0.0f};
  auto column = [&](const float4* wk, const f32x2 (&xx)[RPL], bool hi) {
#pragma unroll
    for (int q = 0; q < QMAX; ++q) {
      if (q < nq) {  // wave-uniform
        const float4 w = wk[q];
        const f32x2 w01 = (f32x2){w.x, w.y}, w23 = (f32x2){w.z, w.w};
#pragma unroll
        for (int r = 0; r < RPL; ++r) {
          if (hi) {
            pk_mac_hi(a[r][q][0], w01, xx[r]);
            pk_mac_hi(a[r][q][1], w23, xx[r]);
          } else {
            pk_mac_lo(a[r][q][0], w01, xx[r]);
            pk_mac_lo(a[r][q][1], w23, xx[r]);
          }
        }
      }
    }
  };
  const int d4 = d & ~3;
  for (int k = 0; k < d4; k += 4) {
    f32x2 x01[RPL], x23[RPL];
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
      const float4 v = *reinterpret_cast<const float4*>(x[r] + k);
      x01[r] = (f32x2){v.x, v.y};
      x23[r] = (f32x2){v.z, v.w};
    }
    column(swq + (size_t)k * nq, x01, false);
    column(swq + (size_t)(k + 1) * nq, x01, true);
    column(swq + (size_t)(k + 2) * nq, x23, false);
    column(swq + (size_t)(k + 3) * nq, x23, true);
  }
  for (int k = d4; k < d; ++k) {
    f32x2 xk[RPL];
#pragma unroll
    for (int r = 0; r < RPL; ++r) xk[r] = (f32x2){x[r][k], x[r][k]};
    column(swq + (size_t)k * nq, xk, false);
  }
#pragma unroll
  for (int r = 0; r < RPL; ++r) {
    uint32_t key = 0;
#pragma unroll
    for (int q = 0; q < QMAX; ++q)
      if (q < nq)
        key = key * 16u + (a[r][q][0].x >= 0.0f ? 8u : 0u) + (a[r][q][0].y >= 0.0f ? 4u : 0u) +
              (a[r][q][1].x >= 0.0f ? 2u : 0u) + (a[r][q][1].y >= 0.0f ? 1u : 0u);
    const uint32_t pr = p0 + 256u * r;
    if (pr < n) keys[pr] = (key >> (uint32_t)(4 * nq - h)) | key_or;
  }
  kt_end(kt, KC_PROJECT);
}

// Any d: 32 running sums in registers (unrolled, predicated on the wave-uniform h), the row
// streamed in 4-float chunks; per-hyperplane summation order is unchanged by the chunking.
__global__ __launch_bounds__(256) void k_project_generic(const float* __restrict__ X, int d,
                                                         int dp, const uint32_t* __restrict__ slots,
                                                         uint32_t* __restrict__ keys, uint32_t n,
                                                         const float* __restrict__ W, int h,
                                                         uint32_t key_or, KTime kt) {
  kt_fold(kt);
  kt_begin(kt, KC_PROJECT);
  const uint32_t p = blockIdx.x * 256u + threadIdx.x;
  if (p >= n) return;
  const float* x = X + (size_t)slots[p] * dp;
  float s[kMaxHyperplanes];
#pragma unroll
  for (int j = 0; j < kMaxHyperplanes; ++j) s[j] = 0.0f;
  const int d4 = d & ~3;
  for (int k = 0; k < d4; k += 4) {
    const float4 v = *reinterpret_cast<const float4*>(x + k);
#pragma unroll
    for (int j = 0; j < kMaxHyperplanes; ++j) {
      if (j < h) {
        const float* w = W + (size_t)j * dp + k;
        s[j] = s[j] + w[0] * v.x;
        s[j] = s[j] + w[1] * v.y;
        s[j] = s[j] + w[2] * v.z;
        s[j] = s[j] + w[3] * v.w;
      }
    }
  }
  for (int k = d4; k < d; ++k) {
    const float v = x[k];
#pragma unroll
    for (int j = 0; j < kMaxHyperplanes; ++j)
      if (j < h) s[j] = s[j] + W[(size_t)j * dp + k] * v;
  }
  uint32_t key = 0;
#pragma unroll
  for (int j = 0; j < kMaxHyperplanes; ++j)
    if (j < h) key = key * 2u + (s[j] >= 0.0f ? 1u : 0u);
  keys[p] = key | key_or;
  kt_end(kt, KC_PROJECT);
}

typedef float pf32x16 __attribute__((ext_vector_type(16)));

// The projection from the fp16 row image (Rows::xh), certified.  x~ = fp16(x) is read (2d bytes a
// row, half the f32 row gather) and S = x~ . w is taken on v_mfma_f32_32x32x16_f16 with w split
// into fp16 hi + lo (two MFMAs per 16 columns; x~ needs no split).  Against the reference's
// sequential f32 sum s of the f32 row (hash/lshash.cc:44-51):
//   |S - s| <= |S - x~.w|        w split residual 2^-22 |w_k| (+ 2^-25 absolute where w_lo is
//                                 subnormal) and the MFMA's f32 sums, (17 + 2 ceil(d/16)) 2^-23
//            + |x~.w - x.w|      fp16 rounding of x: 2^-11 |x_k| (+ 2^-25 absolute, subnormals)
//            + |x.w - s|         the reference's own (d + 1) 2^-24
// summed over k with Cauchy-Schwarz: <= eps |w||x| + abs_c (|w| + |x~|) (h16_eps / h16_abs, with
// 1.5x headroom; |x| <= 1.001 |x~| covers the 2^-11).  Signs with |S| above the bound are the
// reference's bits; the rest (fp16 overflow, NaN, |S| within the bound: ~0.5 % of the
// row-hyperplane pairs at d = 64) go to the fix-up list (k_project_fix: the exact chains on the
// f32 row).  32 rows x 32 hyperplanes per MFMA tile; the next group's rows are loaded during the
// current group.
typedef _Float16 ph16x8 __attribute__((ext_vector_type(8)));

float h16_eps(int d) {
  const float ks = (float)((d + 15) / 16);
  return 1.5f * (0x1p-11f + 0x1p-22f + (17.0f + 2.0f * ks) * 0x1p-23f + (float)(d + 1) * 0x1p-24f);
}
float h16_abs(int d) { return 1.5f * 2.0f * 0x1p-25f * std::sqrt((float)d); }

// Lane-owned rows: every lane loads one whole fp16 row (2d bytes), then one v_permlane32_swap per
// dword turns the chunk pair (cols 16s..16s+7, 16s+8..16s+15) of lanes L and L + 32 into the
// B operands of two 32-row tiles (lanes 0-31 keep their low chunk and take lane L + 32's, lanes
// 32-63 keep their high chunk and take lane L - 32's).  The product is S^T = W X^T, so lane L
// holds, for row L & 31 of a tile, the 16 hyperplanes (i&3) + 8(i>>2) + 4(L>>5): the key bits
// of a row are lane-local (two lanes, one swap to combine), no ballots.  Close calls go to this
// workgroup's segment and are settled at the end of the kernel by the same workgroup, one lane
// per listed row: the f32 row loaded once, the reference's sequential chain (hash/lshash.cc:44-51,
// mul then add, never fused) per flagged hyperplane from the f32 hyperplanes in LDS.
typedef _Float16 ph16x2 __attribute__((ext_vector_type(2)));

template <int D>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_project_h16(const uint16_t* __restrict__ XH,
                                                     const float* __restrict__ X, int dp,
                                                     const uint32_t* __restrict__ slots,
                                                     uint32_t* __restrict__ keys, uint32_t n,
                                                     const float* __restrict__ W, int h,
                                                     uint32_t key_or, float eps, float abs_c,
                                                     ProjectWork pw, uint32_t segcap, KTime kt,
                                                     const uint32_t* __restrict__ n_dev,
                                                     const uint32_t* __restrict__ woff_dev) {
  constexpr int KS = D / 16;  // k-steps of 16 columns
  __shared__ ph16x8 sa[2][KS][64];  // A fragments (w_hi, w_lo) of every lane, per k-step
  __shared__ __attribute__((aligned(16))) float swf[32 * D];  // f32 hyperplanes (exact chains)
  __shared__ float swn[32];         // |w_j| (bounds)
  __shared__ uint32_t s_cnt;        // entries of this workgroup's fix-up segment
  __shared__ uint32_t s_close;      // close calls (statistics)
  kt_fold(kt);
  kt_begin(kt, KC_PROJECT);
  if (n_dev) {
    n = *n_dev;
    h = n ? 31 - __builtin_clz(n) : 0;
    if (woff_dev) W += (size_t)*woff_dev * dp;
  }
  const uint32_t t = threadIdx.x, lane = t & 63u, hh = lane >> 5;
  const uint32_t wv = t >> 6;
  const uint32_t step = gridDim.x * 256u;
  uint32_t g0 = (blockIdx.x * 4u + wv) * 64u;
  // the wave's first rows are requested before the hyperplanes are staged, so their latency
  // overlaps the staging (a launch of a few hundred thousand rows is one or two groups a wave);
  // loads are unconditional (a lane past n reads slots[0]'s row, unused)
  auto load_rows = [&](ph16x8 (&xr)[2 * KS], uint32_t sl) __attribute__((always_inline)) {
    const uint16_t* src = XH + (size_t)sl * dp;
#pragma unroll
    for (int c = 0; c < 2 * KS; ++c) xr[c] = *reinterpret_cast<const ph16x8*>(src + 8 * c);
  };
  // the hyperplane loads and the slot load are issued together (one round trip, not one per
  // element), then the rows, whose latency the LDS staging below overlaps
  constexpr int NWL = 32 * D / 256;
  float wl[NWL];
#pragma unroll
  for (int i = 0; i < NWL; ++i) {
    const int e = (int)t + 256 * i, j = e / D, k = e % D;
    wl[i] = W[(size_t)(j < h ? j : 0) * dp + k];
  }
  const uint32_t sl0 = slots[g0 + lane < n ? g0 + lane : 0u];
  __builtin_amdgcn_sched_barrier(0);  // (keeps every hyperplane load ahead of the row loads)
  ph16x8 xr[2 * KS];  // the lane's row, 8 columns per chunk
  load_rows(xr, sl0);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < NWL; ++i) {
    const int e = (int)t + 256 * i;
    swf[e] = e / D < h ? wl[i] : 0.0f;
  }
  if (t == 0) s_cnt = s_close = 0u;
  __syncthreads();
  {  // |w_j|: 8 lanes per hyperplane (a bound: any summation order, the hardware sqrt, x 1.001)
    const int j = (int)(t >> 3), p = (int)(t & 7u);
    float a = 0.0f;
#pragma unroll
    for (int k = p; k < D; k += 8) a += swf[j * D + k] * swf[j * D + k];
    a += __shfl_xor(a, 1, 64);
    a += __shfl_xor(a, 2, 64);
    a += __shfl_xor(a, 4, 64);
    if (p == 0) swn[j] = __builtin_amdgcn_sqrtf(a) * 1.001f;
  }
  // A fragment of lane L at k-step s: hyperplane L & 31, columns 16s + 8(L >> 5) + 0..7, split
  for (int e = (int)t; e < KS * 64; e += 256) {
    const int sk = e >> 6, L = e & 63, j = L & 31, k0 = 16 * sk + 8 * (L >> 5);
    ph16x8 hi8, lo8;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float w = swf[j * D + k0 + q];
      const _Float16 hi = (_Float16)w;
      hi8[q] = hi;
      lo8[q] = (_Float16)(w - (float)hi);  // w - hi is exact in f32
    }
    sa[0][sk][L] = hi8;
    sa[1][sk][L] = lo8;
  }
  __syncthreads();
  uint4* seg = reinterpret_cast<uint4*>(pw.fix) + (size_t)blockIdx.x * segcap;
  auto group = [&](const ph16x8 (&xr)[2 * KS], uint32_t g0) __attribute__((always_inline)) {
    float ss = 0.0f;  // |x~|^2 of the lane's row (a bound only)
#pragma unroll
    for (int c = 0; c < 2 * KS; ++c)
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        const ph16x2 v = {xr[c][e], xr[c][e + 1]};
        ss = __builtin_amdgcn_fdot2(v, v, ss, false);
      }
    const float xn = __builtin_amdgcn_sqrtf(ss) * 1.001f;  // >= |x| (or inf / NaN)
    pf32x16 accA, accB;
#pragma unroll
    for (int i = 0; i < 16; ++i) accA[i] = accB[i] = 0.0f;
#pragma unroll
    for (int sk = 0; sk < KS; ++sk) {
      uint4 a = *reinterpret_cast<const uint4*>(&xr[2 * sk]);
      uint4 b = *reinterpret_cast<const uint4*>(&xr[2 * sk + 1]);
      auto p0 = __builtin_amdgcn_permlane32_swap(a.x, b.x, false, false);
      auto p1 = __builtin_amdgcn_permlane32_swap(a.y, b.y, false, false);
      auto p2 = __builtin_amdgcn_permlane32_swap(a.z, b.z, false, false);
      auto p3 = __builtin_amdgcn_permlane32_swap(a.w, b.w, false, false);
      a = make_uint4(p0[0], p1[0], p2[0], p3[0]);  // tile A (rows of lanes 0-31)
      b = make_uint4(p0[1], p1[1], p2[1], p3[1]);  // tile B (rows of lanes 32-63)
      const ph16x8 fa = *reinterpret_cast<const ph16x8*>(&a);
      const ph16x8 fb = *reinterpret_cast<const ph16x8*>(&b);
      const ph16x8 wh = sa[0][sk][lane], wl = sa[1][sk][lane];
      accA = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, fa, accA, 0, 0, 0);
      accB = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, fb, accB, 0, 0, 0);
      accA = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl, fa, accA, 0, 0, 0);
      accB = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl, fb, accB, 0, 0, 0);
    }
    // acc[i] = S[hyperplane (i&3) + 8(i>>2) + 4hh][tile row lane & 31]; tile A's row R is lane
    // R's own, tile B's lane 32 + R's
    const float xo = __shfl_xor(xn, 32, 64);
    uint32_t bits[2], amb[2];
#pragma unroll
    for (int tb = 0; tb < 2; ++tb) {
      const float xr_n = (tb == 0) == (hh == 0) ? xn : xo;  // |x~| of the tile row
      const float c1 = eps * xr_n + abs_c, c2 = abs_c * xr_n;
      const bool huge = !(xr_n <= 0x1p100f);  // NaN, inf (fp16 overflow): exact chains
      uint32_t bt = 0u, am = 0u;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int j = (i & 3) + 8 * (i >> 2) + 4 * (int)hh;
        if (j < h) {
          const float sv = tb ? accB[i] : accA[i];
          const float bound = swn[j] * c1 + c2;
          bt |= (sv >= 0.0f ? 1u : 0u) << j;
          am |= ((!(__builtin_fabsf(sv) > bound) || huge) ? 1u : 0u) << j;
        }
      }
      bits[tb] = bt | (uint32_t)__shfl_xor((int)bt, 32, 64);
      amb[tb] = am | (uint32_t)__shfl_xor((int)am, 32, 64);
    }
    const uint32_t row = g0 + lane;  // lane L writes tile A row L (L < 32) / tile B row L - 32
    const uint32_t mb = hh ? bits[1] : bits[0], ma = hh ? amb[1] : amb[0];
    if (row < n) {
      uint32_t key_bits = mb & ~ma;  // close calls start at 0: the fix-up sets the ones >= 0
      bool done = true;
      if (ma) {  // to this workgroup's fix-up segment (settled below; in place if it is full)
        atomicAdd(&s_close, (uint32_t)__popc(ma));
        const uint32_t at = atomicAdd(&s_cnt, 1u);
        if (at < segcap) {
          seg[at] = make_uint4(row, ma, key_bits, 0u);
          done = false;
        } else {
          const float* x = X + (size_t)slots[row] * dp;
          uint32_t a = ma;
          while (a) {
            const int j = __builtin_ctz(a);
            a &= a - 1u;
            float sd = 0.0f;  // -ffp-contract=off: the reference's mul, add order
            for (int k = 0; k < D; ++k) sd = sd + swf[j * D + k] * x[k];
            if (sd >= 0.0f) key_bits |= 1u << j;
          }
        }
      }
      // hyperplane 0 is the key's most significant bit
      if (done) keys[row] = (h > 0 ? (__builtin_bitreverse32(key_bits) >> (32 - h)) : 0u) | key_or;
    }
  };
  while (g0 < n) {
    const uint32_t sl = slots[g0 + step + lane < n ? g0 + step + lane : 0u];  // the next group's
    group(xr, g0);
    g0 += step;
    if (g0 >= n) break;
    load_rows(xr, sl);
  }
  __syncthreads();
  // the close calls of this workgroup's rows
  const uint32_t cnt = min(s_cnt, segcap);
  for (uint32_t e = t; e < cnt; e += 256) {
    const uint4 f = seg[e];
    const float* x = X + (size_t)slots[f.x] * dp;
    float4 u[D / 4];
#pragma unroll
    for (int q = 0; q < D / 4; ++q) u[q] = *reinterpret_cast<const float4*>(x + 4 * q);
    uint32_t key_bits = f.z, a = f.y;
    while (a) {
      const int j = __builtin_ctz(a);
      a &= a - 1u;
      const float* w = swf + j * D;
      float sd = 0.0f;
#pragma unroll
      for (int q = 0; q < D / 4; ++q) {
        const float4 v = *reinterpret_cast<const float4*>(w + 4 * q);
        sd = sd + v.x * u[q].x;
        sd = sd + v.y * u[q].y;
        sd = sd + v.z * u[q].z;
        sd = sd + v.w * u[q].w;
      }
      if (sd >= 0.0f) key_bits |= 1u << j;
    }
    keys[f.x] = (h > 0 ? (__builtin_bitreverse32(key_bits) >> (32 - h)) : 0u) | key_or;
  }
  if (t == 0 && s_close)  // the call's running total (16 spread 64-bit counters at ws[32..64))
    atomicAdd(reinterpret_cast<unsigned long long*>(pw.ws + 32 + 2 * (blockIdx.x & 15u)),
              (unsigned long long)s_close);
  kt_end(kt, KC_PROJECT);
}

// Wide rows (d > 64, any d): a certified matrix-core screen with an fp16x3 split — x = xh + xl,
// w = wh + wl (xh = fp16(x), xl = fp16(x - xh): 22 bits of the f32 value), S = xh.wh + xh.wl +
// xl.wh on v_mfma_f32_32x32x16_f16 — and a bound that scales with T = sum_k |x_k||w_k| (a fourth
// MFMA, |xh|.|wh|), not with |x||w|.  Against the reference's sequential f32 sum s
// (hash/lshash.cc:44-51):
//   |S - s| <= eps_w T + abs_w (|w| + |x|)
//     eps_w: split residuals and the dropped xl.wl (3 * 2^-22), the MFMA's f32 sums ((17 + 3 ceil(d/16))
//            * 2^-23 of the summed magnitudes), the reference's own ((d + 1) * 2^-24), x 1.5
//     abs_w: fp16 subnormals (2^-25 per element, both operands, Cauchy-Schwarz: sqrt(d) 2^-25), x 3
// with T taken as the computed |xh|.|wh| MFMA x (1 + 2^-9) (>= sum |x_k||w_k|: fp16 rounding of
// both operands, the MFMA's own sums of positive terms).  Against round 3's bf16x3 split and
// eps |w||x| bound this leaves a few times fewer close calls at d = 512 (both the 2^-16 split term
// and the Cauchy-Schwarz slack are gone).  An element past fp16's range (|x| >= 65520: inf in xh),
// NaN or inf makes S or T non-finite, and the pair goes to the exact chain.  The hyperplane
// fragments are pre-split in LDS ([k-step][lane] hi, lo: 64 KB at d = 512) and the row streamed 64
// columns per round (8 loads in flight per lane).  The pairs the screen cannot call go to a list
// that k_project_fix settles with the exact sequential chains afterwards, one lane per pair —
// in-wave they would stall 31 other rows.  Six waves per workgroup: the 64-KB fragment table is
// shared by 6 waves instead of 4, so two workgroups per CU keep 12 waves (3 per SIMD) of row loads
// in flight, not 8.
typedef _Float16 wh16x8 __attribute__((ext_vector_type(8)));
constexpr int kWideNT = 384;

float wide_eps(int d) {
  const float ks = (float)((d + 15) / 16);
  return 1.5f * (3.0f * 0x1p-22f + (17.0f + 3.0f * ks) * 0x1p-23f + (float)(d + 1) * 0x1p-24f);
}
float wide_abs(int d) { return 3.0f * 0x1p-25f * std::sqrt((float)d); }

__device__ __forceinline__ void hsplit8(float4 u, float4 v, wh16x8& hi, wh16x8& lo, wh16x8& ah) {
  const float x[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const _Float16 hb = (_Float16)x[j];
    hi[j] = hb;
    lo[j] = (_Float16)(x[j] - (float)hb);  // x - hi is exact in f32 (finite hi)
    ah[j] = __builtin_fabsf16(hb);
  }
}

// DT > 0: d == DT (a multiple of 64), every row load unconditional and the round loop unrolled,
// so each round waits only for its own loads (vmcnt counts, not vmcnt(0)) and the next round's
// stay in flight behind the math; one round is kept ahead (two measured 2030-2035 vs 1995-2003
// ms per C5 step).
constexpr int kWidePF = 1;
template <int DT>
__global__ __launch_bounds__(kWideNT, 2) void k_project_mfma_wide(const float* __restrict__ X, int d, int dp,
                                                           const uint32_t* __restrict__ slots,
                                                           uint32_t* __restrict__ keys, uint32_t n,
                                                           const float* __restrict__ W, int h,
                                                           uint32_t key_or, float eps, float abs_c,
                                                           ProjectWork pw, KTime kt) {
  extern __shared__ __attribute__((aligned(16))) unsigned char psm[];
  kt_fold(kt);
  kt_begin(kt, KC_PROJECT);
  const int KS = (d + 15) / 16;
  wh16x8* bfr = reinterpret_cast<wh16x8*>(psm);  // [KS][64 lanes][hi, lo]
  float* swn = reinterpret_cast<float*>(psm + (size_t)KS * 64 * 2 * sizeof(wh16x8));  // [32]
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6, r = lane & 31u, hh = lane >> 5;
  // hyperplane fragments: entry (s, L) = W[j = L&31][16s + 8(L>>5) + 0..7], split
  if constexpr (DT > 0) {
    // d = DT: thread t owns entries e = t + 384u, i.e. hyperplane j = t & 31, column half t >> 5
    // & 1 and k-steps wv + 6u — every load issued before the first is waited for (a loop of
    // loads under a bounds check waited for each: ~100 us of the launch at C5's late iterations),
    // and |w_j| summed from the same registers (12 partial sums per hyperplane, added in a fixed
    // order: a bound, any order will do)
    constexpr int KSC = DT / 16, NE = (KSC * 64 + kWideNT - 1) / kWideNT;
    __shared__ float wpart[32][kWideNT / 32];
    const int j = (int)(t & 31u), half = (int)((t >> 5) & 1u), jc = j < h ? j : 0;
    float4 wl[NE][2];
#pragma unroll
    for (int u = 0; u < NE; ++u) {
      const int sk = min((int)wv + (int)(kWideNT / 64) * u, KSC - 1);
      const float* src = W + (size_t)jc * dp + 16 * sk + 8 * half;
      wl[u][0] = *reinterpret_cast<const float4*>(src);
      wl[u][1] = *reinterpret_cast<const float4*>(src + 4);
    }
    float sq = 0.0f;
#pragma unroll
    for (int u = 0; u < NE; ++u) {
      const int sk = (int)wv + (int)(kWideNT / 64) * u;
      if (sk < KSC) {
        float x[8] = {wl[u][0].x, wl[u][0].y, wl[u][0].z, wl[u][0].w,
                      wl[u][1].x, wl[u][1].y, wl[u][1].z, wl[u][1].w};
        wh16x8 hi, lo;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          if (j >= h) x[q] = 0.0f;
          const _Float16 hb = (_Float16)x[q];
          hi[q] = hb;
          lo[q] = (_Float16)(x[q] - (float)hb);
          sq += x[q] * x[q];
        }
        const int e = sk * 64 + (int)lane;
        bfr[2 * e] = hi;
        bfr[2 * e + 1] = lo;
      }
    }
    wpart[j][t >> 5] = sq;
    __syncthreads();
    if (t < 32) {
      float a = 0.0f;
#pragma unroll
      for (int q = 0; q < (int)(kWideNT / 32); ++q) a += wpart[t][q];
      swn[t] = __builtin_amdgcn_sqrtf(a) * 1.001f;
    }
  } else {
    for (int e = (int)t; e < KS * 64; e += kWideNT) {
      const int sk = e >> 6, L = e & 63, j = L & 31, k0 = 16 * sk + 8 * (L >> 5);
      float x[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) x[q] = (j < h && k0 + q < d) ? W[(size_t)j * dp + k0 + q] : 0.0f;
      wh16x8 hi, lo;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const _Float16 hb = (_Float16)x[q];
        hi[q] = hb;
        lo[q] = (_Float16)(x[q] - (float)hb);
      }
      bfr[2 * e] = hi;
      bfr[2 * e + 1] = lo;
    }
    if (t < 32) {
      float a = 0.0f;
      for (int k = 0; k < d; ++k) {
        const float v = (int)t < h ? W[(size_t)t * dp + k] : 0.0f;
        a += v * v;
      }
      swn[t] = __builtin_amdgcn_sqrtf(a) * 1.001f;
    }
  }
  __syncthreads();
  const float wn = swn[r];
  const bool col_ok = (int)r < h;
  constexpr uint32_t NWV = kWideNT / 64;
  const uint32_t step = gridDim.x * NWV * 32u;
  for (uint32_t g0 = (blockIdx.x * NWV + wv) * 32u; g0 < n; g0 += step) {
    const uint32_t row = g0 + r;
    const bool valid = row < n;
    const float* xr = X + (size_t)slots[valid ? row : g0] * dp;
    pf32x16 acc, aab;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = aab[i] = 0.0f;
    float ss = 0.0f;
    // 4 k-steps (64 columns) per round; the next round's loads are issued before this round's math
    float4 xa[4][2], xn4[4][2];
    auto load_round = [&](int s0, float4 (&dst)[4][2]) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int k0 = 16 * (s0 + q) + 8 * (int)hh;
        dst[q][0] = k0 + 4 <= dp ? *reinterpret_cast<const float4*>(xr + k0) : make_float4(0.f, 0.f, 0.f, 0.f);
        dst[q][1] = k0 + 8 <= dp ? *reinterpret_cast<const float4*>(xr + k0 + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    };
    if constexpr (DT > 0) {
      constexpr int R = DT / 64, PF = kWidePF, NB = PF + 1;
      float4 xb[NB][4][2];
      auto load_full = [&](int rd, float4 (&dst)[4][2]) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int k0 = 64 * rd + 16 * q + 8 * (int)hh;
          dst[q][0] = *reinterpret_cast<const float4*>(xr + k0);
          dst[q][1] = *reinterpret_cast<const float4*>(xr + k0 + 4);
        }
      };
#pragma unroll
      for (int rd = 0; rd < PF && rd < R; ++rd) load_full(rd, xb[rd % NB]);
#pragma unroll
      for (int rd = 0; rd < R; ++rd) {
        if (rd + PF < R) load_full(rd + PF, xb[(rd + PF) % NB]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 u = xb[rd % NB][q][0], v = xb[rd % NB][q][1];
          wh16x8 ah, al, aa;
          hsplit8(u, v, ah, al, aa);
          ss += u.x * u.x + u.y * u.y + u.z * u.z + u.w * u.w + v.x * v.x + v.y * v.y + v.z * v.z +
                v.w * v.w;
          const int sk = 4 * rd + q;
          const wh16x8 bh = bfr[2 * (sk * 64 + lane)], bl = bfr[2 * (sk * 64 + lane) + 1];
          wh16x8 ba;
#pragma unroll
          for (int e = 0; e < 8; ++e) ba[e] = __builtin_fabsf16(bh[e]);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc, 0, 0, 0);
          aab = __builtin_amdgcn_mfma_f32_32x32x16_f16(aa, ba, aab, 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);  // keeps the loads PF rounds ahead, not all hoisted
      }
    } else {
    load_round(0, xa);
    for (int s0 = 0; s0 < KS; s0 += 4) {
      if (s0 + 4 < KS) load_round(s0 + 4, xn4);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (s0 + q < KS) {  // wave-uniform
          wh16x8 ah, al, aa;
          hsplit8(xa[q][0], xa[q][1], ah, al, aa);
          ss += xa[q][0].x * xa[q][0].x + xa[q][0].y * xa[q][0].y + xa[q][0].z * xa[q][0].z +
                xa[q][0].w * xa[q][0].w + xa[q][1].x * xa[q][1].x + xa[q][1].y * xa[q][1].y +
                xa[q][1].z * xa[q][1].z + xa[q][1].w * xa[q][1].w;
          const wh16x8 bh = bfr[2 * ((s0 + q) * 64 + lane)], bl = bfr[2 * ((s0 + q) * 64 + lane) + 1];
          wh16x8 ba;
#pragma unroll
          for (int e = 0; e < 8; ++e) ba[e] = __builtin_fabsf16(bh[e]);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc, 0, 0, 0);
          aab = __builtin_amdgcn_mfma_f32_32x32x16_f16(aa, ba, aab, 0, 0, 0);
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        xa[q][0] = xn4[q][0];
        xa[q][1] = xn4[q][1];
      }
    }
    }
    ss += __shfl_xor(ss, 32, 64);
    const float xn = __builtin_amdgcn_sqrtf(ss) * 1.001f;
    uint32_t bits = 0u, amb = 0u;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t ri = (i & 3) + 8u * (i >> 2) + 4u * hh;
      const float xni = __shfl(xn, (int)ri, 64);
      const float sv = acc[i];
      const float bound = eps * (aab[i] * (1.0f + 0x1p-9f)) + abs_c * (wn + xni) + 0x1p-120f;
      const bool pos = col_ok && sv >= 0.0f;
      // NaN / inf anywhere (S, T or the norms), or |S| within the bound: the exact chain decides
      const bool am = col_ok && (!(__builtin_fabsf(sv) > bound) || !(xni <= 0x1p60f));
      const uint64_t bp = __ballot(pos), ba = __ballot(am);
      const uint32_t r0 = (i & 3) + 8u * (i >> 2);
      if (lane == r0) {
        bits = (uint32_t)bp;
        amb = (uint32_t)ba;
      }
      if (lane == r0 + 4u) {
        bits = (uint32_t)(bp >> 32);
        amb = (uint32_t)(ba >> 32);
      }
    }
    if (lane < 32 && valid) {
      keys[row] = (h > 0 ? (__builtin_bitreverse32(bits) >> (32 - h)) : 0u) | key_or;
      if (amb) {  // to the fix-up list (the exact chains; in place if the list is full)
        const uint32_t c = (uint32_t)__popc(amb);
        const uint32_t at = atomicAdd(&pw.ws[0], c);
        uint32_t a = amb, k = 0;
        while (a) {
          const int j = __builtin_ctz(a);
          a &= a - 1u;
          if (at + k < pw.cap) {
            pw.fix[at + k] = make_uint2(row, (uint32_t)j);
          } else {
            const float* x = X + (size_t)slots[row] * dp;
            const float* w = W + (size_t)j * dp;
            float sd = 0.0f;
            for (int q = 0; q < d; ++q) sd = sd + w[q] * x[q];
            const uint32_t bit = 1u << (h - 1 - j);
            keys[row] = sd >= 0.0f ? (keys[row] | bit) : (keys[row] & ~bit);
          }
          ++k;
        }
      }
    }
  }
}

// The exact sequential chain (hash/lshash.cc:44-51) of each listed (row, hyperplane) pair; the
// key bit is set or cleared atomically (several pairs may share a row).  Persistent grid; the last
// workgroup returns the list counters to zero.
__global__ __launch_bounds__(256) void k_project_fix(const float* __restrict__ X, int d, int dp,
                                                     const uint32_t* __restrict__ slots,
                                                     uint32_t* __restrict__ keys,
                                                     const float* __restrict__ W, int h,
                                                     ProjectWork pw, KTime kt,
                                                     const uint32_t* __restrict__ n_dev = nullptr,
                                                     const uint32_t* __restrict__ woff_dev = nullptr) {
  extern __shared__ __attribute__((aligned(16))) float fw[];  // the h hyperplanes, stride dp
  __shared__ uint32_t s_last;
  if (n_dev) {  // a queued iteration: h and the hyperplane offset from the device
    const uint32_t n = *n_dev;
    h = n ? 31 - __builtin_clz(n) : 0;
    if (woff_dev) W += (size_t)*woff_dev * dp;
  }
  const uint32_t count = min(pw.ws[0], pw.cap);
  if (blockIdx.x * 256u < count) {
    // the h hyperplanes into LDS, 16 float4 loads in flight per lane (dp is a multiple of 4):
    // a loop of one load per round trip was ~80 us of every launch, whatever its pair count.  The
    // stores are unconditional at the clamped index (past nv - 1 they rewrite element nv - 1 with
    // its own value): a store under `< nv` let the compiler sink each load into its branch, which
    // made the 16 loads 16 round trips again
    const int nv = h * dp / 4;
    const float4* W4 = reinterpret_cast<const float4*>(W);
    float4* fw4 = reinterpret_cast<float4*>(fw);
    constexpr int U = 16;
    for (int i0 = (int)threadIdx.x; i0 < nv; i0 += 256 * U) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = W4[min(i0 + 256 * u, nv - 1)];
#pragma unroll
      for (int u = 0; u < U; ++u) fw4[min(i0 + 256 * u, nv - 1)] = v[u];  // (see below)
    }
  }
  __syncthreads();
  for (uint32_t e = blockIdx.x * 256u + threadIdx.x; e < count; e += gridDim.x * 256u) {
    const uint2 f = pw.fix[e];
    const float* x = X + (size_t)slots[f.x] * dp;
    const float* w = fw + (size_t)f.y * dp;
    float sd = 0.0f;
    int k = 0;
    for (; k + 64 <= d; k += 64) {  // 64 columns per round, the row's loads issued first
      float4 u[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) u[q] = *reinterpret_cast<const float4*>(x + k + 4 * q);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const float4 v = *reinterpret_cast<const float4*>(w + k + 4 * q);
        sd = sd + v.x * u[q].x;
        sd = sd + v.y * u[q].y;
        sd = sd + v.z * u[q].z;
        sd = sd + v.w * u[q].w;
      }
    }
    for (; k < d; ++k) sd = sd + w[k] * x[k];
    const uint32_t bit = 1u << (h - 1 - (int)f.y);
    if (sd >= 0.0f) atomicOr(&keys[f.x], bit);
    else atomicAnd(&keys[f.x], ~bit);
  }
  if (threadIdx.x == 0) s_last = atomicAdd(&pw.ws[1], 1u) == gridDim.x - 1 ? 1u : 0u;
  __syncthreads();
  if (s_last && threadIdx.x == 0) {
    // the call's running total of settled pairs (ws[4..5], read by the engine's statistics)
    atomicAdd(reinterpret_cast<unsigned long long*>(pw.ws + 4), (unsigned long long)pw.ws[0]);
    atomicExch(&pw.ws[0], 0u);
    atomicExch(&pw.ws[1], 0u);
  }
  kt_end(kt, KC_PROJECT);  // the screen + fix-up span (k_project_mfma_wide stamps the start)
}

// The fp16-image screen (its close calls settled in the wave).  h: the iteration's h, or (n_dev
// given) ignored: the kernel derives it from the device count.
static void launch_h16(const Rows& r, const uint32_t* slots, uint32_t* keys, uint32_t n,
                       const float* W, int h, uint32_t key_or, hipStream_t s,
                       const ProjectWork& pw, KTime kt, const uint32_t* n_dev,
                       const uint32_t* woff_dev) {
  const uint32_t gmax = pw.h16_grid ? std::max(256u, pw.h16_grid) : kH16Grid;  // "h16_grid"
  const uint32_t grid = std::min<uint32_t>((n + 255) / 256, gmax);
  uint32_t segcap = (pw.cap / 2) / grid;  // 16-B fix-up entries per workgroup
  if (pw.segcap) segcap = std::min(segcap, pw.segcap);  // "h16_segcap" (tests: the in-place path)
  const float eps = h16_eps(r.d), abs_c = h16_abs(r.d);
  auto go = [&](auto screen) {
    screen<<<grid, 256, 0, s>>>(r.xh, r.x, r.dp, slots, keys, n, W, h, key_or, eps, abs_c, pw,
                                segcap, kt, n_dev, woff_dev);
  };
  if (r.d == 64) go(k_project_h16<64>);
  else if (r.d == 32) go(k_project_h16<32>);
  else go(k_project_h16<16>);
}

static bool h16_ok(const Rows& r, const ProjectWork* pw) {
  return pw && pw->variant != kProjPacked && r.xh && (r.d == 16 || r.d == 32 || r.d == 64);
}

bool project_device_n_ok(int d) {
  return d == 8 || d == 16 || d == 32 || d == 64;  // and the default variant (below)
}

void launch_project_device_n(const Rows& r, const uint32_t* slots, uint32_t* keys, uint32_t n_max,
                             const float* W, const uint32_t* n_dev, hipStream_t s, KTime kt,
                             const uint32_t* woff_dev, const ProjectWork* pw) {
  if (n_max == 0) return;
  if (h16_ok(r, pw)) {
    const int hmax = 31 - __builtin_clz(n_max);  // h of the device count is <= this
    launch_h16(r, slots, keys, n_max, W, hmax, 0u, s, *pw, kt, n_dev, woff_dev);
    return;
  }
  const dim3 grid((n_max + 255) / 256), block(256);
  auto go = [&](auto kern) {
    kern<<<grid, block, 0, s>>>(r.x, r.dp, slots, keys, n_max, W, 0, 0u, n_dev, kt, woff_dev);
  };
  switch (r.d) {
    case 8: go(k_project_pk<8, 2, 1>); break;
    case 16: go(k_project_pk<16, 2, 1>); break;
    case 32: go(k_project_pk<32, 2, 1>); break;
    default: go(k_project_pk<64, 2, 1>); break;
  }
}

// The projection of a call: the certified matrix-core screens where they exist (the fp16 row
// image at d = 16, 32, 64; the bf16x3 screen + exact fix-up pass above 64), else the packed exact
// VALU chains (d = 8 and any d without a screen, or option "projection" = kProjPacked): the
// wide-row packed kernel with the hyperplanes in LDS, else the generic kernel.
int launch_project(const Rows& r, const uint32_t* slots, uint32_t* keys, uint32_t n,
                    const float* W, int h, uint32_t key_or, hipStream_t s, const ProjectWork* pw,
                    KTime kt) {
  if (n == 0) return kPkNone;
  const dim3 grid((n + 255) / 256), block(256);
  if (pw && pw->variant != kProjPacked && r.d > 64 && h > 0) {
    const size_t lds = (size_t)((r.d + 15) / 16) * 64 * 2 * 16 + 32 * sizeof(float);
    const size_t flds = sizeof(float) * (size_t)h * r.dp;  // the fix-up kernel's hyperplanes
    if (lds <= 96 * 1024 && flds <= 128 * 1024) {
      static const bool lds_ok =
          hipFuncSetAttribute(reinterpret_cast<const void*>(&k_project_mfma_wide<0>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024) == hipSuccess &&
          hipFuncSetAttribute(reinterpret_cast<const void*>(&k_project_mfma_wide<512>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024) == hipSuccess &&
          hipFuncSetAttribute(reinterpret_cast<const void*>(&k_project_fix),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024) == hipSuccess;
      (void)lds_ok;
      const uint32_t groups = (n + kWideNT / 2 - 1) / (kWideNT / 2);  // 32 rows per wave
      // option "wide_grid": one resident round (2 workgroups of 6 waves per CU): C5 projection
      // 1203 -> 1076 ms per step (256..8192 swept on one box: 256 -> 1073, 512 -> 1076, 1024 ->
      // 1112, 2048 -> 1203, 4096 -> 1318, 8192 -> 1533)
      const uint32_t wcap = pw->wide_grid ? std::max(64u, pw->wide_grid) : 512u;
      const dim3 gm(std::min<uint32_t>(groups, wcap));
      // stamped as one span: the screen (start) and the fix-up of its close calls (end)
      KTime k1 = kt;
      k1.fold = -1;
      if (r.d == 512 && !pw->wide_rolled)  // option "wide_unrolled" (default 1)
        k_project_mfma_wide<512><<<gm, dim3(kWideNT), lds, s>>>(r.x, r.d, r.dp, slots, keys, n, W,
                                                                h, key_or, wide_eps(r.d),
                                                                wide_abs(r.d), *pw, kt);
      else
        k_project_mfma_wide<0><<<gm, dim3(kWideNT), lds, s>>>(r.x, r.d, r.dp, slots, keys, n, W, h,
                                                              key_or, wide_eps(r.d), wide_abs(r.d),
                                                              *pw, kt);
      const uint32_t fcap = pw->fix_grid ? std::max(16u, pw->fix_grid) : 1024u;  // "fix_grid"
      k_project_fix<<<fcap, block, flds, s>>>(r.x, r.d, r.dp, slots, keys, W, h, *pw, k1);
      return kPkWide;
    }
  }
  if (h16_ok(r, pw) && h > 0) {
    launch_h16(r, slots, keys, n, W, h, key_or, s, *pw, kt, nullptr, nullptr);
    return kPkH16;
  }
  auto go_pk = [&](auto kern) {
    kern<<<grid, block, 0, s>>>(r.x, r.dp, slots, keys, n, W, h, key_or, nullptr, kt, nullptr);
  };
  switch (r.d) {
    case 8: go_pk(k_project_pk<8, 2, 1>); break;
    case 16: go_pk(k_project_pk<16, 2, 1>); break;
    case 32: go_pk(k_project_pk<32, 2, 1>); break;
    case 64: go_pk(k_project_pk<64, 2, 1>); break;
    default: {
      const size_t lds = sizeof(float4) * (size_t)r.dp * (size_t)((h + 3) / 4);
      if (lds <= 64 * 1024) {
        static const bool lds_ok =
            hipFuncSetAttribute(reinterpret_cast<const void*>(&k_project_wide_pk<1>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024) == hipSuccess;
        (void)lds_ok;
        k_project_wide_pk<1><<<grid, block, lds, s>>>(r.x, r.d, r.dp, slots, keys, n, W, h, key_or,
                                                      kt);
      } else {
        k_project_generic<<<grid, block, 0, s>>>(r.x, r.d, r.dp, slots, keys, n, W, h, key_or, kt);
      }
    }
  }
  return kPkPacked;
}

// Stable compaction of the live slots (merge_abundance's concatenation, cluster.cc:39-45) in two
// coalesced passes: per-tile live counts (wave ballots), then every tile sums the counts before
// it itself and writes its survivors in order — position k*256 + t is read by thread t, the
// output offset of each wave's survivors comes from the ballots, so reads and writes stay
// contiguous per wave (the generic scan reads and writes 16 consecutive items per lane).
constexpr int kCompactTile = 4096;
__global__ __launch_bounds__(256) void k_compact_count(const uint32_t* __restrict__ slots,
                                                       uint32_t n, uint32_t* __restrict__ counts,
                                                       KTime kt) {
  __shared__ uint32_t wsum[4];
  kt_begin(kt, KC_COMPACT);
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint32_t T0 = blockIdx.x * (uint32_t)kCompactTile;
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < kCompactTile / 256; ++k) {
    const uint32_t i = T0 + k * 256u + t;
    const uint32_t v = slots[i < n ? i : 0u];  // unconditional: the tile's loads all in flight
    c += (uint32_t)__popcll(__ballot(i < n && v != kInvalid));
  }
  if (lane == 0) wsum[wv] = c;
  __syncthreads();
  if (t == 0) counts[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

// The iteration's run counts (k_runs, k_merge_huge's list) into *ctr, and rc back to zero.
__device__ __forceinline__ void collect_run_counts(Counters* ctr, RunCounters* rc) {
  if (!rc) return;
  ctr->n_seg = rc->n_seg.v;
  rc->n_seg.v = 0u;
#pragma unroll
  for (int c = 0; c < kGroupClasses; ++c) {
    ctr->n_cls[c] = rc->n_cls[c].v;
    rc->n_cls[c].v = 0u;
  }
#pragma unroll
  for (int c = 0; c < kBigClasses; ++c) {
    ctr->n_big[c] = rc->n_big[c].v;
    rc->n_big[c].v = 0u;
  }
  ctr->n_huge = rc->n_huge.v;
  rc->n_huge.v = 0u;
  ctr->n_over = rc->n_over.v;
  rc->n_over.v = 0u;
  ctr->n_small_rows = rc->n_small_rows.v;
  rc->n_small_rows.v = 0u;
#pragma unroll
  for (int c = 0; c < kBigClasses; ++c) {
    ctr->n_big_rows[c] = rc->n_big_rows[c].v;
    rc->n_big_rows[c].v = 0u;
  }
  ctr->n_huge_rows = rc->n_huge_rows.v;
  rc->n_huge_rows.v = 0u;
#pragma unroll
  for (int c = 0; c < kGroupClasses; ++c) rc->n_act[c].v = 0u;
  ctr->n_act_rows = rc->n_act_rows.v;
  rc->n_act_rows.v = 0u;
  ctr->screened = rc->screened.v;
  rc->screened.v = 0u;
}

// Publish the iteration's counters to the host (see Publish), `total` filled in.
__device__ __forceinline__ void publish_counters(Counters* ctr, uint32_t total, const Publish& pub,
                                                 uint32_t n_in) {
  Counters c = *ctr;
  c.total = total;
  if (pub.n_next) *pub.n_next = total;  // for an iteration already queued (device-side n)
  if (pub.woff && n_in) *pub.woff += 31u - (uint32_t)__builtin_clz(n_in);  // h of this iteration
  const uint32_t* src = reinterpret_cast<const uint32_t*>(&c);
  uint32_t* dst = reinterpret_cast<uint32_t*>(pub.host);
  for (int i = 0; i < (int)(sizeof(Counters) / 4); ++i) {
    __hip_atomic_store(dst + i, src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    reinterpret_cast<uint32_t*>(ctr)[i] = 0u;  // the next iteration starts from zero
  }
  __threadfence_system();
  __hip_atomic_store(pub.seq_host, pub.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_publish(Counters* ctr, Publish pub, RunCounters* rc) {
  collect_run_counts(ctr, rc);
  if (pub.host) publish_counters(ctr, ctr->total, pub, 0u);
}

__global__ __launch_bounds__(256) void k_compact_apply(const uint32_t* __restrict__ slots,
                                                       uint32_t n,
                                                       const uint32_t* __restrict__ counts,
                                                       uint32_t* __restrict__ out,
                                                       uint32_t* __restrict__ total,
                                                       Counters* ctr, Publish pub,
                                                       RunCounters* rc, KTime kt) {
  constexpr int K = kCompactTile / 256;
  __shared__ uint32_t cnt[K * 4], pre[K * 4 + 1], wsum[4];
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint32_t T0 = blockIdx.x * (uint32_t)kCompactTile;
  // survivors of the tiles before this one
  uint32_t before = 0;
  for (uint32_t j = t; j < blockIdx.x; j += 256) before += counts[j];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) before += __shfl_xor(before, o, 64);
  if (lane == 0) wsum[wv] = before;
  uint32_t v[K];
  uint64_t m[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {  // every load issued first (unconditional: one wait, not K)
    const uint32_t i = T0 + k * 256u + t;
    v[k] = slots[i < n ? i : 0u];
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if (T0 + k * 256u + t >= n) v[k] = kInvalid;
    m[k] = __ballot(v[k] != kInvalid);
    if (lane == 0) cnt[k * 4 + wv] = (uint32_t)__popcll(m[k]);
  }
  __syncthreads();
  if (t == 0) {  // offsets of the (row k, wave w) groups in position order
    uint32_t a = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    for (int q = 0; q < K * 4; ++q) {
      pre[q] = a;
      a += cnt[q];
    }
    pre[K * 4] = a;
  }
  __syncthreads();
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (v[k] != kInvalid) out[pre[k * 4 + wv] + (uint32_t)__popcll(m[k] & below)] = v[k];
  if (blockIdx.x == gridDim.x - 1 && t == 0) {
    *total = pre[K * 4];
    collect_run_counts(ctr, rc);
    if (pub.host) publish_counters(ctr, pre[K * 4], pub, n);
  }
  kt_end(kt, KC_COMPACT);
}

// Small iterations (<= 256 tiles, every tile resident at once): the same compaction in ONE launch
// with a look-back — a tile publishes its survivor count (tagged with the launch's epoch) right
// after counting, then sums the counts of the tiles before it (thread j waits for tile j's word;
// a predecessor publishes before it waits for anyone, so the waits cannot cycle).  One dependent
// launch less per iteration.  A wait that exceeds its bound sets ctr->err (reported, not hung).
__global__ __launch_bounds__(256) void k_compact_lb(const uint32_t* __restrict__ slots, uint32_t n,
                                                    uint32_t* __restrict__ out,
                                                    unsigned long long* __restrict__ status,
                                                    uint32_t epoch, uint32_t* __restrict__ total,
                                                    Counters* ctr, Publish pub, RunCounters* rc,
                                                    KTime kt, const uint32_t* n_dev) {
  constexpr int K = kCompactTile / 256;
  __shared__ uint32_t cnt[K * 4], pre[K * 4 + 1], wsum[4];
  kt_begin(kt, KC_COMPACT);
  // device-side n: every workgroup reads it before it publishes its status, and the last one
  // (which rewrites the word through pub.n_next) only after every status is in
  if (n_dev) n = *n_dev;
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint32_t T0 = blockIdx.x * (uint32_t)kCompactTile;
  uint32_t v[K];
  uint64_t m[K];
  uint32_t mine = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) {  // every load issued first (unconditional: one wait, not K)
    const uint32_t i = T0 + k * 256u + t;
    v[k] = slots[i < n ? i : 0u];
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if (T0 + k * 256u + t >= n) v[k] = kInvalid;
    m[k] = __ballot(v[k] != kInvalid);
    mine += (uint32_t)__popcll(m[k]);
    if (lane == 0) cnt[k * 4 + wv] = (uint32_t)__popcll(m[k]);
  }
  if (lane == 0) wsum[wv] = mine;
  __syncthreads();
  if (t == 0)
    __hip_atomic_store(&status[blockIdx.x],
                       ((unsigned long long)epoch << 32) | (wsum[0] + wsum[1] + wsum[2] + wsum[3]),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint32_t before = 0;
  if (t < blockIdx.x) {
    unsigned long long w = 0;
    for (uint32_t spin = 0;; ++spin) {
      w = __hip_atomic_load(&status[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((uint32_t)(w >> 32) == epoch) break;
      if (spin > (1u << 24)) {  // a protocol failure: report it instead of hanging
        atomicOr(&ctr->err, 4u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    before = (uint32_t)w;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) before += __shfl_xor(before, o, 64);
  __syncthreads();  // wsum is rewritten below
  if (lane == 0) wsum[wv] = before;
  __syncthreads();
  if (t == 0) {  // offsets of the (row k, wave w) groups in position order
    uint32_t a = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    for (int q = 0; q < K * 4; ++q) {
      pre[q] = a;
      a += cnt[q];
    }
    pre[K * 4] = a;
  }
  __syncthreads();
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (v[k] != kInvalid) out[pre[k * 4 + wv] + (uint32_t)__popcll(m[k] & below)] = v[k];
  if (blockIdx.x == gridDim.x - 1 && t == 0) {
    *total = pre[K * 4];
    collect_run_counts(ctr, rc);
    if (pub.host) publish_counters(ctr, pre[K * 4], pub, n);
  }
  kt_end(kt, KC_COMPACT);
}

void launch_compact(const uint32_t* slots, uint32_t n, uint32_t* out, uint32_t* tile_sums,
                    Counters* ctr, hipStream_t s, const Publish* pub, RunCounters* rc, KTime kt,
                    const LookBack* lb, const uint32_t* n_dev) {
  const Publish none{nullptr, nullptr, 0u, nullptr};
  if (n_dev) {  // a queued iteration: the one-launch look-back compaction over <= 256 tiles
    const uint32_t ntiles = (n + kCompactTile - 1) / kCompactTile;
    if (!lb || !lb->status || ntiles == 0 || ntiles > 256u) return;  // (the caller checks)
    const uint32_t epoch = ++lb->epoch;
    k_compact_lb<<<ntiles, 256, 0, s>>>(slots, n, out, lb->status, epoch, &ctr->total, ctr,
                                        pub ? *pub : none, rc, kt, n_dev);
    return;
  }
  if (n == 0) {
    (void)hipMemsetAsync(&ctr->total, 0, sizeof(uint32_t), s);
    k_publish<<<1, 1, 0, s>>>(ctr, pub ? *pub : none, rc);
    return;
  }
  const uint32_t ntiles = (n + kCompactTile - 1) / kCompactTile;
  if (lb && lb->status && ntiles <= 256u) {
    const uint32_t epoch = ++lb->epoch;
    k_compact_lb<<<ntiles, 256, 0, s>>>(slots, n, out, lb->status, epoch, &ctr->total, ctr,
                                        pub ? *pub : none, rc, kt, nullptr);
    return;
  }
  uint32_t* counts = tile_sums + kScanSumsWord;
  k_compact_count<<<ntiles, 256, 0, s>>>(slots, n, counts, kt);
  k_compact_apply<<<ntiles, 256, 0, s>>>(slots, n, counts, out, &ctr->total, ctr, pub ? *pub : none,
                                         rc, kt);
}

// ============================================================================= mode C =========
// convertHTMat (io/ioMatrix.cc:372-386): value = float(log(cnt + 1.0)) - v_kmers[j] (the double
// log comes from a host-built 65536-entry table, exact), keep iff sum(cnt) > 0.1 * d.
__global__ __launch_bounds__(256) void k_convert(Rows r, const uint16_t* __restrict__ counts,
                                                 uint32_t bs, const float* __restrict__ lut,
                                                 const float* __restrict__ v_kmers,
                                                 uint32_t* __restrict__ keep) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= bs) return;
  const int d = r.d;
  float* x = r.x + (size_t)i * r.dp;
  uint64_t total = 0;
  float nn = 0.0f;
  for (int j = 0; j < d; ++j) {
    const uint32_t c = counts[(size_t)j * bs + i];
    total += c;
    const float v = lut[c] - v_kmers[j];
    x[j] = v;
    nn = nn + v * v;
  }
  for (int j = d; j < r.dp; ++j) x[j] = 0.0f;
  r.nrm[i] = nn;
  r.cnt[i] = 1;
  r.head[i] = i;
  r.tail[i] = i;
  r.nxt[i] = kNil;
  keep[i] = ((double)total > 0.1 * (double)d) ? 1u : 0u;
}

void launch_convert(const Rows& r, const uint16_t* counts, uint32_t bs, const float* lut,
                    const float* v_kmers, uint32_t* keep, uint32_t* order, uint32_t* tile_sums,
                    Counters* ctr, hipStream_t s) {
  if (bs == 0) {
    (void)hipMemsetAsync(&ctr->total, 0, sizeof(uint32_t), s);
    return;
  }
  k_convert<<<(bs + 255) / 256, 256, 0, s>>>(r, counts, bs, lut, v_kmers, keep);
  device_scan(SrcArray{keep}, DstCompactIndex{order}, bs, tile_sums, &ctr->total, &ctr->err, s);
}

__global__ void k_stamp_fold(KStampBlock* blk, int set) { kt_fold_set(blk, set, threadIdx.x); }

void launch_stamp_fold(KStampBlock* blk, int set, hipStream_t s) {
  if (blk) k_stamp_fold<<<1, 64, 0, s>>>(blk, set);
}

// ============================================================================== misc ==========
__global__ __launch_bounds__(256) void k_norms(Rows r, uint32_t n) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  r.nrm[i] = norm_mem(r.x + (size_t)i * r.dp, r.d);
}

void launch_norms(const Rows& r, uint32_t n, hipStream_t s) {
  if (n) k_norms<<<(n + 255) / 256, 256, 0, s>>>(r, n);
}

// fp16 image of the rows (round to nearest even; |x| >= 65520 becomes inf, which the screen
// sends to the exact chains)
__global__ __launch_bounds__(256) void k_shadow_build(Rows r, uint64_t words) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < words; i += (uint64_t)gridDim.x * 256ull) {
    const float4 v = reinterpret_cast<const float4*>(r.x)[i];
    const _Float16 h4[4] = {(_Float16)v.x, (_Float16)v.y, (_Float16)v.z, (_Float16)v.w};
    reinterpret_cast<uint2*>(r.xh)[i] = *reinterpret_cast<const uint2*>(h4);
  }
}

void launch_shadow_build(const Rows& r, uint64_t n, hipStream_t s) {
  const uint64_t words = n * (uint64_t)r.dp / 4;  // float4 groups (dp is a multiple of 4)
  if (!r.xh || !words) return;
  k_shadow_build<<<(uint32_t)std::min<uint64_t>(16384, (words + 255) / 256), 256, 0, s>>>(r, words);
}


// One row per wave-pass, grid-strided: a launch's work-items must stay below 2^32 (C5's result,
// 9.98M rows x 512, is 5.1e9 floats — a thread per float wrapped and dropped 2^32 of them).
__global__ __launch_bounds__(256) void k_gather_rows(Rows r, const uint32_t* __restrict__ order,
                                                     uint32_t n, float* __restrict__ out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = blockIdx.x * 4u + (threadIdx.x >> 6), nwaves = gridDim.x * 4u;
  for (uint32_t i = wave; i < n; i += nwaves) {
    const float* src = r.x + (size_t)order[i] * r.dp;
    float* dst = out + (size_t)i * r.d;
    for (int k = (int)lane; k < r.d; k += 64) dst[k] = src[k];
  }
}

void launch_gather_rows(const Rows& r, const uint32_t* order, uint32_t n, float* out,
                        hipStream_t s) {
  if (n) k_gather_rows<<<std::min<uint32_t>((n + 3) / 4, 65536u), 256, 0, s>>>(r, order, n, out);
}

__global__ void k_fp_selftest(const float* a, const float* b, uint32_t n, float* so, float* dv) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  so[i] = __builtin_sqrtf(a[i]);
  dv[i] = a[i] / b[i];
}

void launch_fp_selftest(const float* a, const float* b, uint32_t n, float* sqrt_out,
                        float* div_out, hipStream_t s) {
  if (n) k_fp_selftest<<<(n + 255) / 256, 256, 0, s>>>(a, b, n, sqrt_out, div_out);
}

}  // namespace klsh
