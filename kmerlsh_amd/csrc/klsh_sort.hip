// Stable bucketing of one LSH iteration: merge_hashtable (reference function/cluster.cc:15-30)
// walks the rows in canonical order and appends each to the bucket of its key; buckets are then
// visited in ascending key order.  That is exactly a stable sort of (key, slot) by key, done here
// as an LSD radix sort with B-bit digits (B = 8..10, so 23-bit keys take three passes and
// 17..20-bit keys two).  Per pass, three launches:
//
//   k_sort_hist     per-tile digit counts, [digit][tile] (4096-key tiles)
//   k_sort_dscan    one workgroup per digit: exclusive scan of its row over the tiles + the digit's
//                   total (no look-back: every row is independent, digit bases come from the
//                   totals, which each scatter workgroup scans itself)
//   k_sort_scatter  ranks of the tile's keys among equal digits (wave ballots, in position order),
//                   the tile ordered by digit in LDS, then written out in per-digit runs
//
// Tile layout: wave w of a workgroup owns the 1024 consecutive positions [w*1024, w*1024 + 1024)
// of its tile, item j of lane l being position w*1024 + j*64 + l — every load and store
// instruction is one contiguous 256-B segment, and a wave's running per-digit counts taken in item
// order are ranks in position order (stability).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "klsh_device.h"

namespace klsh {

constexpr uint32_t kSortTile = 4096;  // keys per workgroup (4 waves x 16 items x 64 lanes)
constexpr int kSortItems = 16;

// The tile of workgroup b among n: consecutive tiles on one XCD.  Workgroups are dealt round-robin
// over the 8 XCDs (MI355X_MICROARCH.md, dispatch placement: b and b + 8 share one — for speed
// only, the mapping is a bijection whatever the placement), and a scatter pass writes each digit
// of a tile as a ~64-B segment right after the previous tile's segment of that digit: with the
// neighbouring tiles on one XCD those partial lines meet in one L2 instead of eight.
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t n) {
#ifdef KLSH_SORT_NO_XCD
  (void)n;
  return b;
#else
  const uint32_t q = n >> 3, r = n & 7u, x = b & 7u;
  return x * q + min(x, r) + (b >> 3);
#endif
}

template <int B>
__global__ __launch_bounds__(256) void k_sort_hist(const uint32_t* __restrict__ keys, uint32_t n,
                                                   int shift, uint32_t ntiles,
                                                   uint32_t* __restrict__ hist, KTime kt,
                                                   const uint32_t* __restrict__ n_dev) {
  constexpr uint32_t RAD = 1u << B, MASK = RAD - 1u;
  __shared__ uint32_t c[RAD];
  kt_begin(kt, KC_SORT);  // (only the first pass's launch carries kt)
  if (n_dev) n = *n_dev;  // tiles past it count nothing
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint32_t tile = xcd_tile(blockIdx.x, ntiles);
  for (uint32_t d = t; d < RAD; d += 256) c[d] = 0u;
  const uint32_t base = tile * kSortTile + wv * 1024u + lane;
  uint32_t k[kSortItems];
#pragma unroll
  for (int j = 0; j < kSortItems; ++j) {
    const uint32_t p = base + (uint32_t)j * 64u;
    k[j] = p < n ? keys[p] : 0u;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kSortItems; ++j)
    if (base + (uint32_t)j * 64u < n) atomicAdd(&c[(k[j] >> shift) & MASK], 1u);
  __syncthreads();
  for (uint32_t d = t; d < RAD; d += 256) hist[(size_t)d * ntiles + tile] = c[d];
}

// Workgroup d: hist[d][0..ntiles) -> its exclusive prefix over the tiles; dtot[d] = digit total.
__global__ __launch_bounds__(256) void k_sort_dscan(uint32_t* __restrict__ hist, uint32_t ntiles,
                                                    uint32_t* __restrict__ dtot) {
  uint32_t* row = hist + (size_t)blockIdx.x * ntiles;
  const uint32_t t = threadIdx.x;
  const uint32_t per = (ntiles + 255u) / 256u;
  const uint32_t lo = min(ntiles, t * per), hi = min(ntiles, lo + per);
  uint32_t acc = 0;
  for (uint32_t i = lo; i < hi; ++i) acc += row[i];
  uint32_t total;
  uint32_t run = block_excl_scan_256(acc, &total);
  for (uint32_t i = lo; i < hi; ++i) {
    const uint32_t v = row[i];
    row[i] = run;
    run += v;
  }
  if (t == 0) dtot[blockIdx.x] = total;
}

template <int B>
__global__ __launch_bounds__(256) void k_sort_scatter(const uint32_t* __restrict__ kin,
                                                      const uint32_t* __restrict__ vin,
                                                      uint32_t* __restrict__ kout,
                                                      uint32_t* __restrict__ vout, uint32_t n,
                                                      int shift, uint32_t ntiles,
                                                      const uint32_t* __restrict__ hist,
                                                      const uint32_t* __restrict__ dtot, KTime kt,
                                                      const uint32_t* __restrict__ n_dev) {
  constexpr uint32_t RAD = 1u << B, MASK = RAD - 1u, PER = RAD / 256u;
  if (n_dev) n = *n_dev;
  __shared__ uint32_t lk[kSortTile], lv[kSortTile];
  __shared__ uint32_t wc[4][RAD];  // per-wave running digit counts, then their wave prefixes
  __shared__ uint32_t ls[RAD];     // tile-local start of each digit
  __shared__ uint32_t gb[RAD];     // output position of tile-local entry 0 of each digit
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint32_t tile = xcd_tile(blockIdx.x, ntiles);
  const uint32_t T0 = tile * kSortTile;
  const uint32_t base = T0 + wv * 1024u + lane;
  for (uint32_t i = t; i < 4u * RAD; i += 256) (&wc[0][0])[i] = 0u;
  uint32_t k[kSortItems], v[kSortItems];
#pragma unroll
  for (int j = 0; j < kSortItems; ++j) {
    const uint32_t p = base + (uint32_t)j * 64u;
    k[j] = p < n ? kin[p] : 0u;
    v[j] = p < n ? vin[p] : 0u;
  }
  __syncthreads();
  // rank of each item among the wave's earlier items with the same digit
  const uint64_t lt = lane ? (~0ull >> (64u - lane)) : 0ull;
  uint32_t lr[kSortItems];
#pragma unroll
  for (int j = 0; j < kSortItems; ++j) {
    const bool valid = base + (uint32_t)j * 64u < n;
    const uint32_t dig = (k[j] >> shift) & MASK;
    uint64_t match = __ballot(valid);
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const bool bit = (dig >> b) & 1u;
      const uint64_t mb = __ballot(bit);
      match &= bit ? mb : ~mb;
    }
    const uint32_t old = wc[wv][dig];  // every lane reads before the group's leader writes
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (valid && (match & lt) == 0ull) wc[wv][dig] = old + (uint32_t)__popcll(match);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    lr[j] = old + (uint32_t)__popcll(match & lt);
  }
  __syncthreads();
  // per digit: wave prefixes, tile totals -> local starts; digit totals -> global bases
  uint32_t tot[PER], dt[PER];
  uint32_t acc = 0, dacc = 0;
#pragma unroll
  for (uint32_t q = 0; q < PER; ++q) {
    const uint32_t d = t * PER + q;
    const uint32_t c0 = wc[0][d], c1 = wc[1][d], c2 = wc[2][d], c3 = wc[3][d];
    wc[0][d] = 0u;
    wc[1][d] = c0;
    wc[2][d] = c0 + c1;
    wc[3][d] = c0 + c1 + c2;
    tot[q] = c0 + c1 + c2 + c3;
    acc += tot[q];
    dt[q] = dtot[d];
    dacc += dt[q];
  }
  uint32_t total;
  uint32_t lpre = block_excl_scan_256(acc, &total);
  uint32_t dpre = block_excl_scan_256(dacc, &total);
#pragma unroll
  for (uint32_t q = 0; q < PER; ++q) {
    const uint32_t d = t * PER + q;
    ls[d] = lpre;
    gb[d] = dpre + hist[(size_t)d * ntiles + tile] - lpre;
    lpre += tot[q];
    dpre += dt[q];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kSortItems; ++j) {
    if (base + (uint32_t)j * 64u < n) {
      const uint32_t dig = (k[j] >> shift) & MASK;
      const uint32_t pos = ls[dig] + wc[wv][dig] + lr[j];
      lk[pos] = k[j];
      lv[pos] = v[j];
    }
  }
  __syncthreads();
  const uint32_t m = T0 < n ? min(kSortTile, n - T0) : 0u;
  for (uint32_t e = t; e < m; e += 256) {
    const uint32_t kk = lk[e];
    const uint32_t o = gb[(kk >> shift) & MASK] + e;
    kout[o] = kk;
    vout[o] = lv[e];
  }
  kt_end(kt, KC_SORT);  // (only the last pass's launch carries kt)
}

uint64_t sort_ws_words(uint64_t slots) {
  // [digit][tile] counts for up to 2^10 digits, then the digit totals
  return 1024ull * ((slots + kSortTile - 1) / kSortTile) + 1024 + 64;
}

// first / last: the pass opens / closes the sort's timed span (kt may be null)
template <int B>
static void sort_pass(const uint32_t* ki, const uint32_t* vi, uint32_t* ko, uint32_t* vo,
                      uint32_t n, int shift, uint32_t* ws, hipStream_t s, KTime kt,
                      bool first, bool last, const uint32_t* n_dev) {
  const uint32_t ntiles = (n + kSortTile - 1) / kSortTile;
  uint32_t* hist = ws;
  uint32_t* dtot = ws + (size_t)(1u << B) * ntiles;
  k_sort_hist<B><<<ntiles, 256, 0, s>>>(ki, n, shift, ntiles, hist, first ? kt : kNoTime, n_dev);
  k_sort_dscan<<<1u << B, 256, 0, s>>>(hist, ntiles, dtot);
  k_sort_scatter<B><<<ntiles, 256, 0, s>>>(ki, vi, ko, vo, n, shift, ntiles, hist, dtot,
                                           last ? kt : kNoTime, n_dev);
}

const uint32_t* radix_sort_top(const uint32_t* k0, const uint32_t* v0, uint32_t* k1, uint32_t* v1,
                               uint32_t n, int bits, uint32_t* ws, hipStream_t s, KTime kt,
                               const uint32_t* n_dev) {
  const uint32_t ntiles = (n + kSortTile - 1) / kSortTile;
  sort_pass<kTailTopBits>(k0, v0, k1, v1, n, bits - kTailTopBits, ws, s, kt, true, true, n_dev);
  return ws + ((size_t)1 << kTailTopBits) * ntiles;
}

// With n_dev the passes are those of `bits` whatever the device count turns out to be: a queued
// iteration's keys have h <= bits significant bits, and a pass over digits that are all zero is a
// stable identity, so the order is the same as a sort on h bits.
void radix_sort(uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, uint32_t n, int bits,
                uint32_t* ws, uint32_t** out_k, uint32_t** out_v, hipStream_t s, KTime kt,
                const uint32_t* n_dev) {
  uint32_t *ki = k0, *vi = v0, *ko = k1, *vo = v1;
  if (n > 1 && bits > 0) {
    // P passes of B-bit digits: 1..10 bits one pass, 11..20 two, 21..30 three, 31..32 four
    // (two passes of 11-bit digits for 21..22-bit keys measured 228-232 vs 210-214 ms on C2:
    // a 2048-digit scatter's 80 KB of LDS and 11 ballots per key cost more than the pass saved)
    const int P = (bits + 9) / 10;
    const int B = std::max(8, (bits + P - 1) / P);
    for (int p = 0; p < P; ++p) {
      const int shift = p * B;
      const bool first = p == 0, last = p == P - 1;
      if (B == 8) sort_pass<8>(ki, vi, ko, vo, n, shift, ws, s, kt, first, last, n_dev);
      else if (B == 9) sort_pass<9>(ki, vi, ko, vo, n, shift, ws, s, kt, first, last, n_dev);
      else sort_pass<10>(ki, vi, ko, vo, n, shift, ws, s, kt, first, last, n_dev);
      std::swap(ki, ko);
      std::swap(vi, vo);
    }
  }
  *out_k = ki;
  *out_v = vi;
}

}  // namespace klsh
