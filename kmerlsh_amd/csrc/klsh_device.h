// Device helpers shared by the gfx950 kernels (klsh_kernels.hip, klsh_merge.hip).
// Numerics contract: see klsh_kernels.hip (sequential fp32, no FMA, IEEE sqrt/div).
#pragma once
#include <hip/hip_runtime.h>

#include "klsh_internal.h"

namespace klsh {
// ---- per-kernel-class stamps (KStampBlock, klsh_internal.h) ----------------------------------
__device__ __forceinline__ unsigned long long stamp_now() { return __builtin_amdgcn_s_memrealtime(); }
// the workgroup's start / end (thread 0; its waves end within a few microseconds of each other)
__device__ __forceinline__ void kt_begin(const KTime& kt, int c) {
  if (kt.blk && threadIdx.x == 0) {
    const unsigned long long now = stamp_now();
    atomicMin(&kt.blk->set[kt.set].t0[c][blockIdx.x % kStampSlots].v, now);
    if (kt.phase >= 0) atomicMin(&kt.blk->set[kt.set].t0[kt.phase][blockIdx.x % kStampSlots].v, now);
  }
}
__device__ __forceinline__ void kt_end(const KTime& kt, int c) {
  if (kt.blk && threadIdx.x == 0) {
    const unsigned long long now = stamp_now();
    atomicMax(&kt.blk->set[kt.set].t1[c][blockIdx.x % kStampSlots].v, now);
    if (kt.phase >= 0) atomicMax(&kt.blk->set[kt.set].t1[kt.phase][blockIdx.x % kStampSlots].v, now);
  }
}
// set `f`'s spans into the totals, then cleared; threads [0, KC_COUNT) of one workgroup
__device__ __forceinline__ void kt_fold_set(KStampBlock* blk, int f, uint32_t t) {
  if (t >= (uint32_t)KC_COUNT) return;
  KStampSet& st = blk->set[f];
  unsigned long long lo = ~0ull, hi = 0ull;
  for (int q = 0; q < kStampSlots; ++q) {
    lo = min(lo, __hip_atomic_load(&st.t0[t][q].v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    hi = max(hi, __hip_atomic_load(&st.t1[t][q].v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    __hip_atomic_store(&st.t0[t][q].v, ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&st.t1[t][q].v, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (hi != 0ull && lo != ~0ull && hi >= lo) {
    blk->ticks[t] += hi - lo;
    blk->launches[t] += 1ull;
  }
}
// the projection's first workgroup folds the previous iteration's set
__device__ __forceinline__ void kt_fold(const KTime& kt) {
  if (kt.blk && kt.fold >= 0 && blockIdx.x == 0) kt_fold_set(kt.blk, kt.fold, threadIdx.x);
}
}  // namespace klsh


namespace klsh {

// ============================================================================ helpers ==========
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// The merge test of cluster.cc:68-69 given the exact sequential dot product and
// den = sqrtf(|a|^2) * sqrtf(|b|^2) (each sqrt correctly rounded, cached per row): see Decider.
__device__ __forceinline__ bool decide(const Decider& dc, float dot, float den) {
  if (dc.fast) {
    const bool den_ok = den >= 0x1p-100f && den <= 0x1p100f;  // rcp(den) normal, no flush
    const float q = dot * __builtin_amdgcn_rcpf(den);
    if (den_ok && q >= dc.s_hi) return true;
    if (den_ok && q <= dc.s_lo) return false;
  }
  return dot / den >= dc.s_star;  // correctly rounded quotient; NaN never merges
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

// Coalesced gather of the 64 rows owned by the lanes of a wave (lane l's row is slot `slot`,
// present if `valid`) into an LDS tile with padded row stride D + 4 floats.  Each wave
// instruction moves 64/(D/4) whole rows (D/4 lanes per row, 16 B per lane) instead of 64
// scattered 16-B pieces; afterwards lane l reads its row from tile + l * (D + 4) (the padding
// keeps those row-per-lane reads free of bank conflicts).
template <int D>
__device__ __forceinline__ void stage_rows(const float* __restrict__ X, int dp, uint32_t slot,
                                           bool valid, float* tile) {
  constexpr int CPR = D / 4;     // 16-B chunks per row
  constexpr int RPI = 64 / CPR;  // rows per wave instruction
  const uint32_t lane = __lane_id();
  const uint32_t q = lane % CPR, rsub = lane / CPR;
  float4 v[CPR];
#pragma unroll
  for (int it = 0; it < CPR; ++it) {
    const uint32_t row = it * RPI + rsub;
    const uint32_t s = (uint32_t)__shfl((int)slot, (int)row, 64);
    const int ok = __shfl(valid ? 1 : 0, (int)row, 64);
    v[it] = ok ? *reinterpret_cast<const float4*>(X + (size_t)s * dp + 4 * q)
               : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  }
#pragma unroll
  for (int it = 0; it < CPR; ++it)
    *reinterpret_cast<float4*>(tile + (it * RPI + rsub) * (D + 4) + 4 * q) = v[it];
}

// stage_rows split in two, so a wave can issue the next batch's row loads early (software
// pipelining) and store them to LDS later: gather_rows loads this wave's 64 rows into v[],
// store_rows writes v[] to the tile (the same layout as stage_rows).
template <int D>
__device__ __forceinline__ void gather_rows(const float* __restrict__ X, int dp, uint32_t slot,
                                            bool valid, float4 (&v)[D / 4]) {
  constexpr int CPR = D / 4, RPI = 64 / CPR;
  const uint32_t lane = __lane_id();
  const uint32_t q = lane % CPR, rsub = lane / CPR;
#pragma unroll
  for (int it = 0; it < CPR; ++it) {
    const uint32_t row = it * RPI + rsub;
    const uint32_t s = (uint32_t)__shfl((int)slot, (int)row, 64);
    const int ok = __shfl(valid ? 1 : 0, (int)row, 64);
    v[it] = ok ? *reinterpret_cast<const float4*>(X + (size_t)s * dp + 4 * q)
               : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  }
}
template <int D>
__device__ __forceinline__ void store_rows(const float4 (&v)[D / 4], float* tile) {
  constexpr int CPR = D / 4, RPI = 64 / CPR;
  const uint32_t lane = __lane_id();
  const uint32_t q = lane % CPR, rsub = lane / CPR;
#pragma unroll
  for (int it = 0; it < CPR; ++it)
    *reinterpret_cast<float4*>(tile + (it * RPI + rsub) * (D + 4) + 4 * q) = v[it];
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
// Row stores of the merge kernels: x and, when kept, its fp16 image (Rows::xh) — every write of
// a row goes through these, so the projection's screen always reads fp16(x).  `at`: float index
// (slot * dp + column), a multiple of 4 for store_row4.
__device__ __forceinline__ void store_row4(const Rows& r, size_t at, float4 v) {
  *reinterpret_cast<float4*>(r.x + at) = v;
  if (r.xh) {
    const _Float16 h4[4] = {(_Float16)v.x, (_Float16)v.y, (_Float16)v.z, (_Float16)v.w};
    *reinterpret_cast<uint2*>(r.xh + at) = *reinterpret_cast<const uint2*>(h4);
  }
}
__device__ __forceinline__ void store_row1(const Rows& r, size_t at, float v) {
  r.x[at] = v;
  if (r.xh) {
    const _Float16 hv = (_Float16)v;
    r.xh[at] = *reinterpret_cast<const uint16_t*>(&hv);
  }
}

__device__ __forceinline__ void link_members(const Rows& r, uint32_t cur, uint32_t cand) {
  const uint32_t ca = r.cnt[cur], cb = r.cnt[cand];
  r.nxt[r.tail[cur]] = r.head[cand];
  r.head[cand] = r.head[cur];
  r.cnt[cand] = ca + cb;
  r.cnt[cur] = 0;
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

// ------------------------------------------------------------ single-pass scan (look-back) ----
// Tiles are taken in ticket order (atomic counter), so a tile only ever waits on tiles that are
// already running.  Each tile publishes its aggregate at once, then its inclusive prefix once the
// look-back (one wave, 64 predecessors per step) has found one.  Status words carry an epoch
// (one per scan launch, kept on the device), so stale words of earlier scans read as "not yet" and
// the status array never needs clearing; the last workgroup to finish resets the ticket and
// advances the epoch.  A wait that exceeds kSpinLimit polls (a broken invariant, never expected)
// sets *err and gives up instead of hanging the GPU.
constexpr uint32_t kStatusAgg = 1u, kStatusPrefix = 2u;
constexpr uint32_t kEpochMask = 0x3FFFFFFFu;
constexpr uint32_t kSpinLimit = 1u << 22;
// Scan workspace (the engine's tile_sums buffer): words [0] ticket, [1] done, [2] epoch, then the
// 64-bit tile status array from word kScanStatusWord (klsh_internal.h: scan_ws_words).

__device__ __forceinline__ uint64_t status_pack(uint32_t epoch, uint32_t flag, uint32_t value) {
  return ((uint64_t)((epoch << 2) | flag) << 32) | value;
}
__device__ __forceinline__ void status_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t status_load(const uint64_t* p) {
  return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// flag of a status word if it belongs to `epoch`, else 0 (not published yet)
__device__ __forceinline__ uint32_t status_flag(uint64_t v, uint32_t epoch) {
  const uint32_t hi = (uint32_t)(v >> 32);
  return (hi >> 2) == epoch ? (hi & 3u) : 0u;
}

// Exclusive prefix of tile `tile` (> 0) from the status words of tiles [0, tile): called by all
// 64 lanes of one wave; every lane returns the same value.
__device__ __forceinline__ uint32_t lookback_wave(const uint64_t* status, uint32_t tile,
                                                  uint32_t epoch, uint32_t* err) {
  const uint32_t lane = __lane_id();
  uint32_t excl = 0;
  int64_t j = (int64_t)tile - 1;  // lane l looks at tile j - l
  uint32_t spins = 0;
  while (true) {
    const int64_t idx = j - (int64_t)lane;
    uint64_t v = 0;
    uint32_t f = kStatusPrefix;  // before tile 0: an empty prefix
    if (idx >= 0) {
      v = status_load(status + idx);
      f = status_flag(v, epoch);
    }
    while (__ballot(f == 0u)) {  // some predecessor has published nothing yet
      if (++spins > kSpinLimit) {
        if (lane == 0) atomicOr(err, 1u);
        return excl;
      }
      __builtin_amdgcn_s_sleep(1);
      if (f == 0u) {
        v = status_load(status + idx);
        f = status_flag(v, epoch);
      }
    }
    const uint64_t pm = __ballot(f == kStatusPrefix);
    const uint32_t stop = pm ? (uint32_t)__builtin_ctzll(pm) : 63u;  // nearest prefix (or all 64)
    uint32_t c = (lane <= stop && idx >= 0) ? (uint32_t)v : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    excl += c;
    if (pm) return excl;
    j -= 64;
  }
}

template <class Src, class Dst>
__global__ __launch_bounds__(256) void k_scan_lb(Src src, Dst dst, uint32_t n, uint32_t* ws,
                                                 uint32_t* total, uint32_t* err) {
  __shared__ uint32_t s_tile, s_epoch, s_excl;
  const uint32_t t = threadIdx.x;
  uint64_t* status = reinterpret_cast<uint64_t*>(ws + kScanStatusWord);
  if (t == 0) {
    s_tile = atomicAdd(&ws[0], 1u);
    s_epoch = (ws[2] + 1u) & kEpochMask;
  }
  __syncthreads();
  const uint32_t tile = s_tile, epoch = s_epoch;
  const uint32_t ntiles = (n + kScanTile - 1) / kScanTile;
  if (tile < ntiles) {
    const uint32_t base = tile * (uint32_t)kScanTile + t * 16u;
    uint32_t v[16];
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      v[k] = (base + k < n) ? src(base + k) : 0u;
      acc += v[k];
    }
    uint32_t tsum;
    const uint32_t in_tile = block_excl_scan_256(acc, &tsum);
    if (t == 0) status_store(status + tile, status_pack(epoch, tile == 0 ? kStatusPrefix : kStatusAgg, tsum));
    if (t < 64) {
      const uint32_t excl = tile == 0 ? 0u : lookback_wave(status, tile, epoch, err);
      if (t == 0) {
        if (tile > 0) status_store(status + tile, status_pack(epoch, kStatusPrefix, excl + tsum));
        s_excl = excl;
        if (tile == ntiles - 1) *total = excl + tsum;
      }
    }
    __syncthreads();
    uint32_t run = s_excl + in_tile;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (base + k < n) dst(base + k, run, v[k]);
      run += v[k];
    }
  } else if (tile == 0) {  // n == 0
    if (t == 0) *total = 0;
  }
  // the last workgroup out resets the ticket and moves the epoch on
  if (t == 0) {
    if (atomicAdd(&ws[1], 1u) == gridDim.x - 1) {
      atomicExch(&ws[0], 0u);
      atomicExch(&ws[1], 0u);
      atomicExch(&ws[2], epoch);
    }
  }
}

// Two-kernel variant: tile sums, then every tile sums the tile sums before it itself (ntiles^2/2
// L2-resident reads in all: no single-workgroup scan, no waiting between workgroups).
template <class Src, class Dst>
__global__ __launch_bounds__(256) void k_scan_apply_redundant(Src src, Dst dst, uint32_t n,
                                                              const uint32_t* __restrict__ tile_sums,
                                                              uint32_t* total) {
  __shared__ uint32_t wsum[4];
  const uint32_t t = threadIdx.x, tile = blockIdx.x;
  uint32_t before = 0;
  for (uint32_t i = t; i < tile; i += 256) before += tile_sums[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) before += __shfl_xor(before, o, 64);
  if ((t & 63u) == 0) wsum[t >> 6] = before;
  __syncthreads();
  before = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  const uint32_t base = tile * (uint32_t)kScanTile + t * 16u;
  uint32_t v[16];
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    v[k] = (base + k < n) ? src(base + k) : 0u;
    acc += v[k];
  }
  uint32_t tsum;
  uint32_t run = block_excl_scan_256(acc, &tsum) + before;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if (base + k < n) dst(base + k, run, v[k]);
    run += v[k];
  }
  if (tile == gridDim.x - 1 && t == 0) *total = before + tsum;
}

template <class Src, class Dst>
inline void device_scan_2k(Src src, Dst dst, uint32_t n, uint32_t* tile_sums, uint32_t* total,
                           hipStream_t s) {
  const uint32_t ntiles = (n + kScanTile - 1) / kScanTile;
  if (ntiles == 0) {
    (void)hipMemsetAsync(total, 0, sizeof(uint32_t), s);
    return;
  }
  uint32_t* ts = tile_sums + kScanSumsWord;
  k_scan_tile_sum<Src><<<ntiles, 256, 0, s>>>(src, n, ts);
  k_scan_apply_redundant<Src, Dst><<<ntiles, 256, 0, s>>>(src, dst, n, ts, total);
}

// Exclusive scan of src over [0, n) feeding dst(i, prefix, value); *total = sum.  `ws` is the
// scan workspace (zeroed once at allocation, scan_ws_words(n) words).
template <class Src, class Dst>
inline void device_scan(Src src, Dst dst, uint32_t n, uint32_t* ws, uint32_t* total,
                        uint32_t* err, hipStream_t s) {
  // auto: the look-back kernel below 2^20 items (one launch; as fast as the others there), the
  // two-kernel scan above (tools/ubench_sort on MI355X: 18.5 vs 15.9 us at 1M, 201 vs 87 us at
  // 9.47M — look-back chains across ~2000 co-resident tiles)
  if (n >= (1u << 20)) return device_scan_2k(src, dst, n, ws, total, s);
  const uint32_t ntiles = (n + kScanTile - 1) / kScanTile;
  k_scan_lb<Src, Dst><<<ntiles ? ntiles : 1u, 256, 0, s>>>(src, dst, n, ws, total, err);
}

}  // namespace klsh
