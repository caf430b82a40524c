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

#include "klsh_internal.h"

namespace klsh {

// ============================================================================ helpers ==========
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// The merge test of cluster.cc:68-69 given the exact sequential dot product and the cached
// sequential norms: sim = dot / (sqrtf(|a|^2) * sqrtf(|b|^2)); dist = 1 - sim; 1 - dist >= thr.
__device__ __forceinline__ bool cos_decide(float dot, float ni, float nj, float thr) {
  const float den = __builtin_sqrtf(ni) * __builtin_sqrtf(nj);
  const float sim = dot / den;
  const float dist = 1.0f - sim;
  return (1.0f - dist) >= thr;
}

// Consensus element (funcAB.cc:65): v1*c1/n + v2*c2/n, each op rounded, current row first.
__device__ __forceinline__ float consensus(float cur, float fa, float cand, float fb, float fn) {
  const float a = (cur * fa) / fn;
  const float b = (cand * fb) / fn;
  return a + b;
}

template <int D>
__device__ __forceinline__ void load_row(const float* __restrict__ p, float (&x)[D]) {
#pragma unroll
  for (int k = 0; k < D; k += 4) {
    const float4 v = *reinterpret_cast<const float4*>(p + k);
    x[k] = v.x;
    x[k + 1] = v.y;
    x[k + 2] = v.z;
    x[k + 3] = v.w;
  }
}

template <int D>
__device__ __forceinline__ float dot_reg_mem(const float (&a)[D], const float* __restrict__ b) {
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < D; k += 4) {
    const float4 v = *reinterpret_cast<const float4*>(b + k);
    s = s + a[k] * v.x;
    s = s + a[k + 1] * v.y;
    s = s + a[k + 2] * v.z;
    s = s + a[k + 3] * v.w;
  }
  return s;
}

__device__ __forceinline__ float dot_mem_mem(const float* a, const float* b, int d) {
  float s = 0.0f;
  for (int k = 0; k < d; ++k) s = s + a[k] * b[k];
  return s;
}

__device__ __forceinline__ float norm_mem(const float* a, int d) {
  float s = 0.0f;
  for (int k = 0; k < d; ++k) s = s + a[k] * a[k];
  return s;
}

// Member list of `cur` goes in front of `cand`'s (funcAB.cc:51-55: ids = ids_cur ++ ids_cand).
__device__ __forceinline__ void link_members(const Rows& r, uint32_t cur, uint32_t cand) {
  const uint32_t ca = r.cnt[cur], cb = r.cnt[cand];
  r.nxt[r.tail[cur]] = r.head[cand];
  r.head[cand] = r.head[cur];
  r.cnt[cand] = ca + cb;
  r.cnt[cur] = 0;
}

// ========================================================================= projection ==========
// One lane per live row; the row sits in registers, the h hyperplanes in LDS (broadcast reads).
// Loop order per hyperplane is the reference's: s = ((0 + w0 x0) + w1 x1) + ...
template <int D>
__global__ __launch_bounds__(256) void k_project(const float* __restrict__ X, int dp,
                                                 const uint32_t* __restrict__ slots,
                                                 uint32_t* __restrict__ keys, uint32_t n,
                                                 const float* __restrict__ W, int h,
                                                 uint32_t key_or) {
  __shared__ __attribute__((aligned(16))) float sw[kMaxHyperplanes * D];
  for (int i = threadIdx.x; i < h * D; i += 256) sw[i] = W[(i / D) * dp + (i % D)];
  __syncthreads();
  const uint32_t p = blockIdx.x * 256u + threadIdx.x;
  if (p >= n) return;
  float x[D];
  load_row<D>(X + (size_t)slots[p] * dp, x);
  uint32_t key = 0;
  for (int j = 0; j < h; ++j) {
    const float* w = sw + j * D;
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < D; ++k) s = s + w[k] * x[k];
    key = key * 2u + (s >= 0.0f ? 1u : 0u);
  }
  keys[p] = key | key_or;
}

// Any d: 32 running sums in registers (unrolled, predicated on the wave-uniform h), the row
// streamed in 4-float chunks; per-hyperplane summation order is unchanged by the chunking.
__global__ __launch_bounds__(256) void k_project_generic(const float* __restrict__ X, int d,
                                                         int dp, const uint32_t* __restrict__ slots,
                                                         uint32_t* __restrict__ keys, uint32_t n,
                                                         const float* __restrict__ W, int h,
                                                         uint32_t key_or) {
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
}

void launch_project(const Rows& r, const uint32_t* slots, uint32_t* keys, uint32_t n,
                    const float* W, int h, uint32_t key_or, hipStream_t s) {
  if (n == 0) return;
  const dim3 grid((n + 255) / 256), block(256);
  switch (r.d) {
    case 8: k_project<8><<<grid, block, 0, s>>>(r.x, r.dp, slots, keys, n, W, h, key_or); break;
    case 16: k_project<16><<<grid, block, 0, s>>>(r.x, r.dp, slots, keys, n, W, h, key_or); break;
    case 32: k_project<32><<<grid, block, 0, s>>>(r.x, r.dp, slots, keys, n, W, h, key_or); break;
    case 64: k_project<64><<<grid, block, 0, s>>>(r.x, r.dp, slots, keys, n, W, h, key_or); break;
    default:
      k_project_generic<<<grid, block, 0, s>>>(r.x, r.d, r.dp, slots, keys, n, W, h, key_or);
  }
}

// =============================================================================== scans ==========
// 256-lane exclusive scan; returns the lane's exclusive prefix, *total = block sum.
__device__ __forceinline__ uint32_t block_excl_scan_256(uint32_t v, uint32_t* total) {
  __shared__ uint32_t wsum[5];
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t a = 0;
    for (int i = 0; i < 4; ++i) {
      const uint32_t t = wsum[i];
      wsum[i] = a;
      a += t;
    }
    wsum[4] = a;
  }
  __syncthreads();
  const uint32_t r = x - v + wsum[w];
  *total = wsum[4];
  __syncthreads();
  return r;
}

struct SrcArray {
  const uint32_t* a;
  __device__ uint32_t operator()(uint32_t i) const { return a[i]; }
};
struct DstExclusive {  // in-place exclusive prefix
  uint32_t* a;
  __device__ void operator()(uint32_t i, uint32_t prefix, uint32_t) const { a[i] = prefix; }
};
struct SrcLive {
  const uint32_t* s;
  __device__ uint32_t operator()(uint32_t i) const { return s[i] != kInvalid ? 1u : 0u; }
};
struct DstCompact {
  const uint32_t* s;
  uint32_t* out;
  __device__ void operator()(uint32_t i, uint32_t prefix, uint32_t v) const {
    if (v) out[prefix] = s[i];
  }
};
struct DstCompactIndex {  // out[prefix] = i for kept i
  uint32_t* out;
  __device__ void operator()(uint32_t i, uint32_t prefix, uint32_t v) const {
    if (v) out[prefix] = i;
  }
};

template <class Src>
__global__ __launch_bounds__(256) void k_scan_tile_sum(Src src, uint32_t n, uint32_t* tile_sums) {
  const uint32_t base = blockIdx.x * (uint32_t)kScanTile + threadIdx.x * 16u;
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k)
    if (base + k < n) acc += src(base + k);
  uint32_t total;
  block_excl_scan_256(acc, &total);
  if (threadIdx.x == 0) tile_sums[blockIdx.x] = total;
}

// One workgroup of 1024 lanes scans the tile sums in place (exclusive); *total = grand total.
__global__ __launch_bounds__(1024) void k_scan_tiles(uint32_t* tile_sums, uint32_t ntiles,
                                                     uint32_t* total) {
  __shared__ uint32_t wsum[17];
  __shared__ uint32_t carry;
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t c = 0; c < ntiles; c += 1024) {
    const uint32_t i = c + threadIdx.x;
    const uint32_t v = i < ntiles ? tile_sums[i] : 0u;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t a = 0;
      for (int k = 0; k < 16; ++k) {
        const uint32_t t = wsum[k];
        wsum[k] = a;
        a += t;
      }
      wsum[16] = a;
    }
    __syncthreads();
    if (i < ntiles) tile_sums[i] = carry + wsum[w] + x - v;
    __syncthreads();
    if (threadIdx.x == 0) carry += wsum[16];
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}

template <class Src, class Dst>
__global__ __launch_bounds__(256) void k_scan_apply(Src src, Dst dst, uint32_t n,
                                                    const uint32_t* __restrict__ tile_sums) {
  const uint32_t base = blockIdx.x * (uint32_t)kScanTile + threadIdx.x * 16u;
  uint32_t v[16];
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    v[k] = (base + k < n) ? src(base + k) : 0u;
    acc += v[k];
  }
  uint32_t total;
  uint32_t run = block_excl_scan_256(acc, &total) + tile_sums[blockIdx.x];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if (base + k < n) dst(base + k, run, v[k]);
    run += v[k];
  }
}

template <class Src, class Dst>
static void device_scan(Src src, Dst dst, uint32_t n, uint32_t* tile_sums, uint32_t* total,
                        hipStream_t s) {
  const uint32_t ntiles = (n + kScanTile - 1) / kScanTile;
  if (ntiles == 0) {
    (void)hipMemsetAsync(total, 0, sizeof(uint32_t), s);
    return;
  }
  k_scan_tile_sum<Src><<<ntiles, 256, 0, s>>>(src, n, tile_sums);
  k_scan_tiles<<<1, 1024, 0, s>>>(tile_sums, ntiles, total);
  k_scan_apply<Src, Dst><<<ntiles, 256, 0, s>>>(src, dst, n, tile_sums);
}

void launch_compact(const uint32_t* slots, uint32_t n, uint32_t* out, uint32_t* tile_sums,
                    Counters* ctr, hipStream_t s) {
  device_scan(SrcLive{slots}, DstCompact{slots, out}, n, tile_sums, &ctr->total, s);
}

// ========================================================================== radix sort ==========
// Stable LSD radix sort, 8-bit digits.  hist layout [digit][tile] so that one exclusive scan of
// the flattened array gives every (digit, tile) its global output offset.
__global__ __launch_bounds__(256) void k_radix_hist(const uint32_t* __restrict__ keys, uint32_t n,
                                                    int shift, uint32_t ntiles,
                                                    uint32_t* __restrict__ hist) {
  __shared__ uint32_t c[256];
  c[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t base = blockIdx.x * (uint32_t)kRadixTile;
  for (int r = 0; r < kRadixTile / 256; ++r) {
    const uint32_t i = base + r * 256u + threadIdx.x;
    if (i < n) atomicAdd(&c[(keys[i] >> shift) & 255u], 1u);
  }
  __syncthreads();
  hist[threadIdx.x * ntiles + blockIdx.x] = c[threadIdx.x];
}

// Each tile is processed in 8 rounds of 256 keys in input order; inside a round the rank of a
// key among equal digits is (earlier waves' counts) + (lower lanes' count from a 64-lane match
// mask built with 8 ballots), so the scatter is stable.
__global__ __launch_bounds__(256) void k_radix_scatter(const uint32_t* __restrict__ kin,
                                                       const uint32_t* __restrict__ vin,
                                                       uint32_t* __restrict__ kout,
                                                       uint32_t* __restrict__ vout, uint32_t n,
                                                       int shift, uint32_t ntiles,
                                                       const uint32_t* __restrict__ hist) {
  __shared__ uint32_t base[256];
  __shared__ uint32_t wcnt[4][256];
  const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
  base[t] = hist[t * ntiles + blockIdx.x];
  wcnt[0][t] = wcnt[1][t] = wcnt[2][t] = wcnt[3][t] = 0;
  __syncthreads();
  const uint32_t tile0 = blockIdx.x * (uint32_t)kRadixTile;
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int r = 0; r < kRadixTile / 256; ++r) {
    const uint32_t i = tile0 + r * 256u + t;
    const bool valid = i < n;
    const uint32_t k = valid ? kin[i] : 0u;
    const uint32_t v = valid ? vin[i] : 0u;
    const uint32_t dig = (k >> shift) & 255u;
    uint64_t match = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const bool bit = (dig >> b) & 1u;
      const uint64_t m = __ballot(bit);
      match &= bit ? m : ~m;
    }
    const uint32_t rank = __popcll(match & lt_mask);
    if (valid && rank == 0) wcnt[w][dig] = __popcll(match);
    __syncthreads();
    if (valid) {
      uint32_t pos = base[dig] + rank;
      for (uint32_t q = 0; q < w; ++q) pos += wcnt[q][dig];
      kout[pos] = k;
      vout[pos] = v;
    }
    __syncthreads();
    base[t] += wcnt[0][t] + wcnt[1][t] + wcnt[2][t] + wcnt[3][t];
    wcnt[0][t] = wcnt[1][t] = wcnt[2][t] = wcnt[3][t] = 0;
    __syncthreads();
  }
}

void radix_sort(uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, uint32_t n, int bits,
                uint32_t* hist, uint32_t* tile_sums, Counters* ctr, uint32_t** out_k,
                uint32_t** out_v, hipStream_t s) {
  uint32_t *ki = k0, *vi = v0, *ko = k1, *vo = v1;
  const uint32_t ntiles = (n + kRadixTile - 1) / kRadixTile;
  for (int shift = 0; shift < bits && n > 1; shift += 8) {
    k_radix_hist<<<ntiles, 256, 0, s>>>(ki, n, shift, ntiles, hist);
    device_scan(SrcArray{hist}, DstExclusive{hist}, 256u * ntiles, tile_sums, &ctr->total, s);
    k_radix_scatter<<<ntiles, 256, 0, s>>>(ki, vi, ko, vo, n, shift, ntiles, hist);
    uint32_t* t;
    t = ki; ki = ko; ko = t;
    t = vi; vi = vo; vo = t;
  }
  *out_k = ki;
  *out_v = vi;
}

// ============================================================================ greedy merge ======
// p_cluster (cluster.cc:56-87) over the slot run s[0..b): row i merges into the FIRST j < i that
// passes the cosine test; the consensus replaces j, i is overwritten by the last live entry and
// re-tested (i not advanced).  Returns the survivor count; survivors are s[0..size).

// One lane owns a whole bucket (b <= kSmallBucket).  D > 0: rows of exactly D floats.
template <int D>
__device__ uint32_t greedy_lane(uint32_t* s, uint32_t b, float thr, const Rows& r) {
  uint32_t size = b, i = 1;
  while (i < size) {
    const uint32_t si = s[i];
    float xi[D];
    load_row<D>(r.x + (size_t)si * r.dp, xi);
    const float ni = r.nrm[si];
    uint32_t j = 0;
    for (; j < i; ++j) {
      const uint32_t sj = s[j];
      const float dot = dot_reg_mem<D>(xi, r.x + (size_t)sj * r.dp);
      if (cos_decide(dot, ni, r.nrm[sj], thr)) break;
    }
    if (j < i) {
      const uint32_t sj = s[j];
      float* xj = r.x + (size_t)sj * r.dp;
      const float fa = (float)(int)r.cnt[si], fb = (float)(int)r.cnt[sj];
      const float fn = (float)(int)(r.cnt[si] + r.cnt[sj]);
      float nn = 0.0f;
#pragma unroll
      for (int k = 0; k < D; k += 4) {
        float4 v = *reinterpret_cast<const float4*>(xj + k);
        v.x = consensus(xi[k], fa, v.x, fb, fn);
        v.y = consensus(xi[k + 1], fa, v.y, fb, fn);
        v.z = consensus(xi[k + 2], fa, v.z, fb, fn);
        v.w = consensus(xi[k + 3], fa, v.w, fb, fn);
        nn = nn + v.x * v.x;
        nn = nn + v.y * v.y;
        nn = nn + v.z * v.z;
        nn = nn + v.w * v.w;
        *reinterpret_cast<float4*>(xj + k) = v;
      }
      r.nrm[sj] = nn;
      link_members(r, si, sj);
      s[i] = s[size - 1];
      --size;
    } else {
      ++i;
    }
  }
  return size;
}

__device__ uint32_t greedy_lane_generic(uint32_t* s, uint32_t b, float thr, const Rows& r) {
  uint32_t size = b, i = 1;
  const int d = r.d;
  while (i < size) {
    const uint32_t si = s[i];
    const float* xi = r.x + (size_t)si * r.dp;
    const float ni = r.nrm[si];
    uint32_t j = 0;
    for (; j < i; ++j) {
      const uint32_t sj = s[j];
      if (cos_decide(dot_mem_mem(xi, r.x + (size_t)sj * r.dp, d), ni, r.nrm[sj], thr)) break;
    }
    if (j < i) {
      const uint32_t sj = s[j];
      float* xj = r.x + (size_t)sj * r.dp;
      const float fa = (float)(int)r.cnt[si], fb = (float)(int)r.cnt[sj];
      const float fn = (float)(int)(r.cnt[si] + r.cnt[sj]);
      float nn = 0.0f;
      for (int k = 0; k < d; ++k) {
        const float v = consensus(xi[k], fa, xj[k], fb, fn);
        xj[k] = v;
        nn = nn + v * v;
      }
      r.nrm[sj] = nn;
      link_members(r, si, sj);
      s[i] = s[size - 1];
      --size;
    } else {
      ++i;
    }
  }
  return size;
}

// One lane per position; the lane at the head of a run (first position of a key) owns the run.
template <int D>
__global__ __launch_bounds__(256) void k_merge_small(const uint32_t* __restrict__ key,
                                                     uint32_t* __restrict__ slots, uint32_t lo,
                                                     uint32_t hi, float thr, int bucket_thr,
                                                     Rows r, uint32_t* __restrict__ large_list,
                                                     uint2* __restrict__ over_list,
                                                     Counters* ctr) {
  const uint32_t p = lo + blockIdx.x * 256u + threadIdx.x;
  if (p >= hi) return;
  const uint32_t k = key[p];
  if (p > lo && key[p - 1] == k) return;
  uint32_t q = p + 1;
  while (q < hi && q - p <= (uint32_t)kSmallBucket && key[q] == k) ++q;
  if (q - p > (uint32_t)kSmallBucket) {
    large_list[atomicAdd(&ctr->n_large, 1u)] = p;
    return;
  }
  const uint32_t b = q - p;
  if (bucket_thr >= 0 && b > (uint32_t)bucket_thr) {  // cluster.cc:286 -> nestedCluster
    over_list[atomicAdd(&ctr->n_over, 1u)] = make_uint2(p, b);
    return;
  }
  if (b < 2) return;
  uint32_t size;
  if constexpr (D > 0) size = greedy_lane<D>(slots + p, b, thr, r);
  else size = greedy_lane_generic(slots + p, b, thr, r);
  for (uint32_t t = size; t < b; ++t) slots[p + t] = kInvalid;
  if (b > size) atomicAdd(&ctr->merges, b - size);
}

// One wave (64 lanes) per long bucket: for the current i, lanes test candidates j = c*64+lane in
// order; the lowest lane of the first chunk with a hit is the reference's first match.
template <int D>
__global__ __launch_bounds__(64) void k_merge_large(const uint32_t* __restrict__ key,
                                                    uint32_t* __restrict__ slots, uint32_t hi,
                                                    float thr, int bucket_thr, Rows r,
                                                    const uint32_t* __restrict__ large_list,
                                                    uint2* __restrict__ over_list, Counters* ctr) {
  extern __shared__ __attribute__((aligned(16))) float sx[];  // consensus row for the norm
  const uint32_t lane = threadIdx.x;
  const uint32_t nlarge = __hip_atomic_load(&ctr->n_large, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int d = r.d;
  for (uint32_t li = blockIdx.x; li < nlarge; li += gridDim.x) {
    const uint32_t p = large_list[li];
    const uint32_t k = key[p];
    uint32_t e = hi;
    for (uint32_t c = p + 1; c < hi; c += 64) {
      const uint32_t q = c + lane;
      const bool stop = q >= hi || key[q] != k;
      const uint64_t m = __ballot(stop);
      if (m) {
        e = c + (uint32_t)(__ffsll((unsigned long long)m) - 1);
        break;
      }
    }
    const uint32_t b = e - p;
    if (bucket_thr >= 0 && b > (uint32_t)bucket_thr) {
      if (lane == 0) over_list[atomicAdd(&ctr->n_over, 1u)] = make_uint2(p, b);
      continue;
    }
    uint32_t* s = slots + p;
    uint32_t size = b, i = 1;
    while (i < size) {
      const uint32_t si = s[i];
      const float* xip = r.x + (size_t)si * r.dp;
      const float ni = r.nrm[si];
      int found = -1;
      if constexpr (D > 0) {
        float xi[D > 0 ? D : 4];
        load_row<(D > 0 ? D : 4)>(xip, xi);
        for (uint32_t c = 0; c < i; c += 64) {
          const uint32_t j = c + lane;
          bool ok = false;
          if (j < i) {
            const uint32_t sj = s[j];
            ok = cos_decide(dot_reg_mem<(D > 0 ? D : 4)>(xi, r.x + (size_t)sj * r.dp), ni,
                            r.nrm[sj], thr);
          }
          const uint64_t m = __ballot(ok);
          if (m) {
            found = (int)(c + (uint32_t)(__ffsll((unsigned long long)m) - 1));
            break;
          }
        }
      } else {
        for (uint32_t c = 0; c < i; c += 64) {
          const uint32_t j = c + lane;
          bool ok = false;
          if (j < i) {
            const uint32_t sj = s[j];
            ok = cos_decide(dot_mem_mem(xip, r.x + (size_t)sj * r.dp, d), ni, r.nrm[sj], thr);
          }
          const uint64_t m = __ballot(ok);
          if (m) {
            found = (int)(c + (uint32_t)(__ffsll((unsigned long long)m) - 1));
            break;
          }
        }
      }
      if (found >= 0) {
        const uint32_t sj = s[found];
        float* xj = r.x + (size_t)sj * r.dp;
        const uint32_t ca = r.cnt[si], cb = r.cnt[sj];
        const float fa = (float)(int)ca, fb = (float)(int)cb, fn = (float)(int)(ca + cb);
        for (int kk = lane; kk < d; kk += 64) {
          const float v = consensus(xip[kk], fa, xj[kk], fb, fn);
          sx[kk] = v;
          xj[kk] = v;
        }
        __syncthreads();
        if (lane == 0) {
          float nn = 0.0f;
          for (int kk = 0; kk < d; ++kk) nn = nn + sx[kk] * sx[kk];
          r.nrm[sj] = nn;
          link_members(r, si, sj);
          s[i] = s[size - 1];
        }
        __syncthreads();
        --size;
      } else {
        ++i;
      }
    }
    for (uint32_t t = size + lane; t < b; t += 64) s[t] = kInvalid;
    if (lane == 0 && b > size) atomicAdd(&ctr->merges, b - size);
    __syncthreads();
  }
}

void launch_merge(const Rows& r, const uint32_t* key, uint32_t* slots, uint32_t lo, uint32_t hi,
                  float thr, int bucket_thr, uint32_t* large_list, uint2* over_list, Counters* ctr,
                  hipStream_t s) {
  if (hi <= lo) return;
  const uint32_t n = hi - lo;
  const dim3 g1((n + 255) / 256), b1(256);
  // The wave kernel reads the queue length from device memory; its grid is a fixed
  // over-subscription of the 256 CUs, each workgroup striding over the queue.
  const dim3 g2(2048), b2(64);
  const size_t lds = sizeof(float) * (size_t)r.dp;
  switch (r.d) {
#define KLSH_MERGE_CASE(DD)                                                                     \
  case DD:                                                                                      \
    k_merge_small<DD><<<g1, b1, 0, s>>>(key, slots, lo, hi, thr, bucket_thr, r, large_list,   \
                                        over_list, ctr);                                               \
    k_merge_large<DD><<<g2, b2, lds, s>>>(key, slots, hi, thr, bucket_thr, r, large_list,       \
                                          over_list, ctr);                                      \
    break;
    KLSH_MERGE_CASE(8)
    KLSH_MERGE_CASE(16)
    KLSH_MERGE_CASE(32)
    KLSH_MERGE_CASE(64)
#undef KLSH_MERGE_CASE
    default:
      k_merge_small<0><<<g1, b1, 0, s>>>(key, slots, lo, hi, thr, bucket_thr, r, large_list,
                                         over_list, ctr);
      k_merge_large<0><<<g2, b2, lds, s>>>(key, slots, hi, thr, bucket_thr, r, large_list,
                                           over_list, ctr);
  }
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
  device_scan(SrcArray{keep}, DstCompactIndex{order}, bs, tile_sums, &ctr->total, s);
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

__global__ __launch_bounds__(256) void k_gather_rows(Rows r, const uint32_t* __restrict__ order,
                                                     uint32_t n, float* __restrict__ out) {
  const uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  const uint64_t total = (uint64_t)n * (uint64_t)r.d;
  if (t >= total) return;
  const uint32_t i = (uint32_t)(t / (uint64_t)r.d);
  const uint32_t k = (uint32_t)(t % (uint64_t)r.d);
  out[t] = r.x[(size_t)order[i] * r.dp + k];
}

void launch_gather_rows(const Rows& r, const uint32_t* order, uint32_t n, float* out,
                        hipStream_t s) {
  const uint64_t total = (uint64_t)n * (uint64_t)r.d;
  if (total) k_gather_rows<<<(unsigned)((total + 255) / 256), 256, 0, s>>>(r, order, n, out);
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
