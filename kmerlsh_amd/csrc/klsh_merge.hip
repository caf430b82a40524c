// Greedy in-bucket merge for gfx950: p_cluster (reference function/cluster.cc:56-87) with the
// cosine test (function/distance.cc:27-38) and the consensus (function/funcAB.cc:49-71), run
// over every bucket of one LSH iteration.
//
// The reference walks a bucket sequentially: row i merges into the FIRST j < i with
// 1 - cosine(i, j) >= thr; the consensus replaces j, row i is overwritten by the last row and
// re-tested.  A decision only changes when one of its two rows changes, and only the candidate j
// of a merge changes, so the GPU version evaluates decisions in bulk and replays the walk:
//
//   segment scan    bucket runs = positions where the sorted key changes (parallel scan)
//   k_classify      runs of 2..64 rows to size-class lists; longer runs to big / huge /
//                   nestedCluster lists
//   k_merge_group   runs of 2..64 rows, in place, by G-lane groups (G = 2,4,...,64; 64/G runs
//                   per wave, one kernel per class): lane g holds row g in
//                   registers and in LDS, the group evaluates every pairwise decision of the run
//                   at once (each an exact sequential fp32 dot product; decisions are
//                   symmetric), then replays the walk on the decision bits; after a merge only
//                   the decisions of rows still to be visited against the new row are redone.
//   k_merge_big     one workgroup per run of 65..896 rows: the same scheme with the run's
//                   decision matrix (and rows, up to 384) in LDS, kept in POSITION space so
//                   every step of the walk is a few bit operations.
//   k_merge_huge    longer runs: one workgroup per run, the reference order directly.
//
// Results are positional (survivors in place, kInvalid after), so they do not depend on which
// wave handled which run or in what order.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <limits>

#include "klsh_device.h"

namespace klsh {

// ------------------------------------------------------------------------------- helpers -----
__device__ __forceinline__ void lds_fence() {
  // orders this workgroup's LDS and global stores before later loads from other lanes of the same
  // wave (waits for outstanding global stores: use only where a global store must be seen)
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
}
__device__ __forceinline__ void wave_lds_fence() {
  // LDS executes one wave's instructions in order: within a wave only the compiler must be kept
  // from moving LDS accesses across this point (no wait for outstanding global stores)
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}
// The all-pairs decisions of 65..896-row runs go through the certified MFMA Gram screen when the
// decider has a fast path and d is a multiple of 16 (else the exact VALU tiles).
constexpr bool kGramTiles = true;

// Merge profiling (diagnostics build only: -DKLSH_MERGE_PROF, make prof): per size class, the
// runs, rows, merges and wall-clock ticks (100 MHz) of each phase, summed over the call.
#ifdef KLSH_MERGE_PROF
__device__ unsigned long long g_mprof[8][12];  // [k] 8: loads, 9: norms, 10: walk loop
#define MPROF_T() wall_clock64()
#define MPROF_ADD(c, k, v) atomicAdd(&g_mprof[c][k], (unsigned long long)(v))
#define MPROF_MAX(c, k, v) atomicMax(&g_mprof[c][k], (unsigned long long)(v))
__device__ unsigned long long g_sprof[8][8];  // small-run batches per G class: batches, clocks in
                                              // stage, pairwise, walk, write-back
__device__ unsigned long long g_wprof[8][8];  // walk phases in shader clocks: find, select+
                                              // consensus, dots, bits, steps, find rounds
#define WPROF_CLK() __builtin_amdgcn_s_memtime()
__device__ unsigned long long g_gprof[8];  // Gram tiles: tiles, ambiguous pairs, sum of the wave's
                                           // longest lane list, clocks: acc, screen, exact, bits
#define GPROF_ADD(k, v) atomicAdd(&g_gprof[k], (unsigned long long)(v))
__device__ unsigned long long g_tprof[8];  // k_tail_local phases (10-ns ticks summed over
                                           // workgroups): base, counts, lists, scatter; workgroups;
                                           // max total
#define TPROF_ADD(k, v) atomicAdd(&g_tprof[k], (unsigned long long)(v))
#else
#define TPROF_ADD(k, v) (void)0
#define GPROF_ADD(k, v) (void)0
#define MPROF_T() 0ull
#define MPROF_ADD(c, k, v) (void)0
#define MPROF_MAX(c, k, v) (void)0
#define WPROF_CLK() 0ull
#endif

__device__ __forceinline__ void lds_barrier() {
  // workgroup barrier for LDS data only: this wave's LDS stores have landed (lgkmcnt(0)), then
  // s_barrier — without the vmcnt(0) wait of __syncthreads for outstanding global stores
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t shfl32(uint32_t v, uint32_t src) {
  return (uint32_t)__shfl((int)v, (int)src, 64);
}
__device__ __forceinline__ float shflf(float v, uint32_t src) { return __shfl(v, (int)src, 64); }
__device__ __forceinline__ uint64_t shfl64(uint64_t v, uint32_t src) {
  const uint32_t lo = shfl32((uint32_t)v, src), hi = shfl32((uint32_t)(v >> 32), src);
  return ((uint64_t)hi << 32) | lo;
}
// v_writelane_b32: lane `l` (a constant after unrolling) of v becomes the wave-uniform value s
__device__ __forceinline__ uint32_t writelane(uint32_t v, uint32_t s, int l) {
#ifdef __OPTIMIZE__
  asm volatile("v_writelane_b32 %0, %1, %2"
               : "=v"(v)
               : "s"(__builtin_amdgcn_readfirstlane(s)), "i"(l), "0"(v));
  return v;
#else  // (the host-sanitizer build compiles device code at -O0: no constant lane to encode)
  return (int)__lane_id() == l ? s : v;
#endif
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}
__device__ __forceinline__ uint64_t lanes_below(uint32_t lane) {
  return lane ? (~0ull >> (64 - lane)) : 0ull;
}

// Wave-aggregated append of `slot` for the lanes with `pred` (all lanes of the wave must call).
__device__ __forceinline__ void append_slot(bool pred, uint32_t slot, uint32_t* list,
                                            uint32_t* counter) {
  const uint64_t m = __ballot(pred);
  if (m == 0ull) return;
  const uint32_t lane = __lane_id();
  const uint32_t leader = (uint32_t)(__ffsll((unsigned long long)m) - 1);
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
  base = shfl32(base, leader);
  if (pred) list[base + (uint32_t)__popcll(m & lanes_below(lane))] = slot;
}

// In-place kernels: record `slot` as rewritten once per iteration.
__device__ __forceinline__ void mark_dirty(uint32_t slot, const MergeWork& w, Counters* ctr) {
  if (w.dlist && w.mark[slot] != w.stamp) {
    w.mark[slot] = w.stamp;
    w.dlist[atomicAdd(&ctr->n_delta, 1u)] = slot;
  }
}

template <int D>
__device__ __forceinline__ float dot_reg_lds(const float (&a)[D], const float* b) {
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

template <int D>
__device__ __forceinline__ void dot2_reg_lds(const float (&a)[D], const float* b0, const float* b1,
                                             float& s0, float& s1) {
  s0 = 0.0f;
  s1 = 0.0f;
#pragma unroll
  for (int k = 0; k < D; k += 4) {
    const float4 u = *reinterpret_cast<const float4*>(b0 + k);
    const float4 v = *reinterpret_cast<const float4*>(b1 + k);
    s0 = s0 + a[k] * u.x;
    s1 = s1 + a[k] * v.x;
    s0 = s0 + a[k + 1] * u.y;
    s1 = s1 + a[k + 1] * v.y;
    s0 = s0 + a[k + 2] * u.z;
    s1 = s1 + a[k + 2] * v.z;
    s0 = s0 + a[k + 3] * u.w;
    s1 = s1 + a[k + 3] * v.w;
  }
}

template <int D>
__device__ __forceinline__ float dot_lds_lds(const float* a, const float* b) {
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < D; k += 4) {
    const float4 u = *reinterpret_cast<const float4*>(a + k);
    const float4 v = *reinterpret_cast<const float4*>(b + k);
    s = s + u.x * v.x;
    s = s + u.y * v.y;
    s = s + u.z * v.z;
    s = s + u.w * v.w;
  }
  return s;
}

__device__ __forceinline__ int size_class(uint32_t b) {  // G = 2 << class lanes per run
  return b <= 2 ? 0 : b <= 4 ? 1 : b <= 8 ? 2 : b <= 16 ? 3 : b <= 32 ? 4 : 5;
}

// Pre-screen of one pair from an approximate dot product g (a Gram tile, or short chains) within
// kGramMargin * |a||b| of the reference's sequential one: 1 = merge, 0 = no merge, 2 = too close
// to call (or den outside the fast range): the exact sequential dot decides.
__device__ __forceinline__ uint32_t prescreen(const Decider& dc, float g, float den) {
  if (den >= 0x1p-60f && den <= 0x1p60f) {
    const float q = g * __builtin_amdgcn_rcpf(den);
    if (q >= dc.g_hi) return 1u;
    if (q <= dc.g_lo) return 0u;
  }
  return 2u;
}

// --------------------------------------------------------------------- G-lane groups -----
// One batch: 64/G runs of one size class, G lanes per run; lane g of a group is position g of its
// run and holds that position's row (registers, and LDS row `lane` for its partners).  The lane's
// slot is already loaded (the caller pipelines it one batch ahead).
//
// 1. Every pairwise decision of the run, each unordered pair once (lane g pairs with the rows
//    k = 1 .. b/2 positions after it, cyclically; decide(a, c) == decide(c, a): the same products
//    in the same order and the same sqrt product, so the partner receives the bit).  The result is
//    the symmetric decision matrix, one row of position bits per lane.
// 2. The walk, kept in POSITION space: lane q holds the bits of the row at position q against the
//    rows at every position (P), that row's id, slot, metadata and data.  The next merge is the
//    first lane q >= i whose P has a bit below q (one ballot); its first match j is the lowest lane
//    p < i whose bit i is set (the matrix is symmetric: one more ballot).  A merge rewrites the row
//    at j (consensus, split over the group's lanes, in LDS), moves the last position's row and
//    state to lane i (swap-remove), remaps bit `last` to bit i everywhere, and re-decides bit j
//    for the positions still to be visited — through the certified short-chain screen, exact
//    chains only for close calls — whose ballot is the new row's P.
// GT: the group width at compile time, or 0: g_rt at run time (one code path for every class:
// the persistent small-run loop then needs the registers of one instance, not of five).
template <int GT, int D>
__device__ __forceinline__ void merge_batch(uint32_t p, uint32_t b, uint32_t slot,
                                            uint32_t* slots, const Decider& dc, const Rows& r,
                                            float* lds, uint32_t* dlist, Counters* ctr,
                                            uint32_t g_rt = 0) {
  const uint32_t G = GT ? (uint32_t)GT : g_rt;
  constexpr int ST = D + 4;  // padded row stride: 16 lanes of a ds_read_b128 hit distinct banks
  const uint32_t lane = __lane_id();
  const uint32_t g = lane & (G - 1);
  const uint32_t gbase = lane - g;
  const uint64_t gmask = (G == 64) ? ~0ull : (((1ull << (G & 63)) - 1ull) << gbase);
  float* myrow = lds + lane * ST;
  [[maybe_unused]] const uint64_t sp0 = WPROF_CLK();
  [[maybe_unused]] uint64_t sp1 = 0, sp2 = 0, sp3 = 0;
  const bool valid = g < b;
  // the lane's own row straight from memory (no cross-lane address shuffles), then to LDS for its
  // partners
  float x[D];
  if (valid) {
    load_row<D>(r.x + (size_t)slot * r.dp, x);
  } else {
#pragma unroll
    for (int k = 0; k < D; ++k) x[k] = 0.0f;
  }
#pragma unroll
  for (int k = 0; k < D; k += 4)
    *reinterpret_cast<float4*>(myrow + k) = make_float4(x[k], x[k + 1], x[k + 2], x[k + 3]);
  wave_lds_fence();
  // the row's norm: recomputed from the row (the same sequential chain that made the cached
  // value, distance.cc:33-34, so the same bits) instead of a random 4-B read of r.nrm
  float nrm = 0.0f;
#pragma unroll
  for (int k = 0; k < D; ++k) nrm = nrm + x[k] * x[k];
  float sq = __builtin_sqrtf(nrm);  // this row's sqrtf(|x|^2), distance.cc:37
  const uint32_t bmax = wave_max(b);
#ifdef KLSH_MERGE_PROF
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  sp1 = WPROF_CLK();
#endif

  // 1. the pairwise decisions
  uint64_t P = 0ull;  // group-local position bits
  {
    const uint32_t half = b / 2;
    auto partner = [&](uint32_t k) {  // (g + k) mod b, for k <= b
      const uint32_t j = g + k;
      return j >= b ? j - b : j;
    };
    auto share = [&](uint32_t k, bool bit) {  // bit = decide(g, g + k); give it to g + k
      const uint32_t src = g >= k ? g - k : g + b - k;  // lane holding decide(src, g)
      const uint32_t in = (uint32_t)__shfl((int)bit, (int)(gbase + (src & (G - 1))), 64);
      if (valid && k <= half) {
        P |= (uint64_t)bit << partner(k);
        P |= (uint64_t)in << src;
      }
    };
    for (uint32_t k = 1; k <= bmax / 2; k += 2) {  // two partners per step: independent chains
      const uint32_t j0 = partner(min(k, b)), j1 = partner(min(k + 1, b));
      const float s0 = shflf(sq, gbase + (j0 & (G - 1))), s1 = shflf(sq, gbase + (j1 & (G - 1)));
      bool h0 = false, h1 = false;
      if (valid && k <= half) {
        float d0, d1;
        dot2_reg_lds<D>(x, lds + (gbase + j0) * ST, lds + (gbase + j1) * ST, d0, d1);
        h0 = decide(dc, d0, sq * s0);
        h1 = k + 1 <= half && decide(dc, d1, sq * s1);
      }
      share(k, h0);
      share(k + 1, h1);
    }
  }
#ifdef KLSH_MERGE_PROF
  sp2 = WPROF_CLK();
#endif

  // 2. the walk.  Per position lane: row id, slot, member count / list ends (loaded only by waves
  //    with a matching pair: three random 4-B reads per row, as much traffic as the row itself),
  //    the row's sqrt-norm, the row (x), dirty = rewritten by a merge.
  uint32_t size = b;
  uint32_t nmerged = 0;
  bool dirty = false;
  const uint64_t matched = __ballot(valid && P != 0ull);
  if (matched) {
    uint32_t rid = g, cnt = 0u, hd = 0u, tl = 0u;
    // metadata only for the runs with a matching pair: ~1 % of the rows merge per iteration, and
    // three random 4-B reads cost a line each (as much traffic as the row itself)
    if (valid && (matched & gmask) != 0ull) {
      cnt = r.cnt[slot];
      hd = r.head[slot];
      tl = r.tail[slot];
    }
    uint32_t i = 1;  // group-uniform
    while (true) {
      const uint64_t below = g ? (~0ull >> (64u - g)) : 0ull;
      const bool hit = g >= i && g < size && (P & below) != 0ull;
      const uint64_t m = __ballot(hit) & gmask;
      if (__ballot(m != 0ull) == 0ull) break;  // every group of the wave is done
      const bool active = m != 0ull;
      uint32_t j = 0, last = 0;
      if (active) {
        i = (uint32_t)__builtin_ctzll(m >> gbase);
        j = (uint32_t)__builtin_ctzll((__ballot(g < i && ((P >> i) & 1ull)) & gmask) >> gbase);
        last = size - 1;
      }
      // the rows at positions i (current), j (candidate), last (moves to i)
      const uint32_t li = gbase + (i & (G - 1)), lj = gbase + (j & (G - 1));
      const uint32_t ll = gbase + (last & (G - 1));
      const uint32_t ri = shfl32(rid, li), rj = shfl32(rid, lj);
      const uint32_t ci = shfl32(cnt, li), cj = shfl32(cnt, lj);
      const uint32_t hi_ = shfl32(hd, li), ti = shfl32(tl, li), hj = shfl32(hd, lj);
      const uint32_t m_rid = shfl32(rid, ll), m_slot = shfl32(slot, ll), m_cnt = shfl32(cnt, ll);
      const uint32_t m_hd = shfl32(hd, ll), m_tl = shfl32(tl, ll);
      const float m_sq = shflf(sq, ll);
      const uint64_t m_P = shfl64(P, ll);
      if (active) {
        // consensus (funcAB.cc:65), current row first, split over the group's lanes, in place
        const float fa = (float)(int)ci, fb = (float)(int)cj, fn = (float)(int)(ci + cj);
        const float* rowr = lds + (gbase + ri) * ST;
        float* rowc = lds + (gbase + rj) * ST;
        for (int k = (int)g; k < D; k += G) rowc[k] = consensus(rowr[k], fa, rowc[k], fb, fn);
        if (g == j) {
          r.nxt[ti] = hj;  // ids_current ++ ids_candidate (funcAB.cc:51-55)
          cnt = ci + cj;
          hd = hi_;
          dirty = true;
        }
        if (g == i) r.cnt[slot] = 0u;  // the current row is gone
        // swap-remove: the last position's row and state move to position i
        if (g == i && i != last) {
          rid = m_rid;
          slot = m_slot;
          cnt = m_cnt;
          hd = m_hd;
          tl = m_tl;
          sq = m_sq;
          P = m_P;
        }
        if (i != last) {
          const uint64_t bl = (P >> last) & 1ull;
          P = (P & ~((1ull << i) | (1ull << last))) | (bl << i);
        }
        --size;
        ++nmerged;
      }
      wave_lds_fence();
      const bool need = active && g >= i && g < size;
      // decisions of the positions still to be visited against the new row at j; both rows are
      // read from LDS 16 B at a time (the lane's own row is its row id's: no registers held
      // across the walk)
      const float* cr = lds + (gbase + rj) * ST;
      const float* xr = lds + (gbase + rid) * ST;
      float n4[4] = {0.0f, 0.0f, 0.0f, 0.0f}, d4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int k = 0; k < D; k += 4) {
        const float4 v = *reinterpret_cast<const float4*>(cr + k);
        const float4 u = *reinterpret_cast<const float4*>(xr + k);
        n4[0] = n4[0] + v.x * v.x;
        n4[1] = n4[1] + v.y * v.y;
        n4[2] = n4[2] + v.z * v.z;
        n4[3] = n4[3] + v.w * v.w;
        d4[0] = d4[0] + u.x * v.x;
        d4[1] = d4[1] + u.y * v.y;
        d4[2] = d4[2] + u.z * v.z;
        d4[3] = d4[3] + u.w * v.w;
      }
      uint32_t dn = 0u;
      if (need) {
        const float sc_a = __builtin_sqrtf((n4[0] + n4[1]) + (n4[2] + n4[3]));
        dn = dc.fast ? prescreen(dc, (d4[0] + d4[1]) + (d4[2] + d4[3]), sq * sc_a) : 2u;
      }
      if (__ballot(dn == 2u)) {  // rare: the reference's sequential chains settle the close calls
        float nn = 0.0f, dot = 0.0f;
#pragma unroll
        for (int k = 0; k < D; k += 4) {
          const float4 v = *reinterpret_cast<const float4*>(cr + k);
          const float4 u = *reinterpret_cast<const float4*>(xr + k);
          nn = nn + v.x * v.x;
          nn = nn + v.y * v.y;
          nn = nn + v.z * v.z;
          nn = nn + v.w * v.w;
          dot = dot + u.x * v.x;
          dot = dot + u.y * v.y;
          dot = dot + u.z * v.z;
          dot = dot + u.w * v.w;
        }
        if (dn == 2u) dn = decide(dc, dot, sq * __builtin_sqrtf(nn)) ? 1u : 0u;
      }
      const uint64_t dm = (__ballot(need && dn == 1u) & gmask) >> gbase;
      if (need) P = dn ? (P | (1ull << j)) : (P & ~(1ull << j));
      if (active && g == j) P = dm;  // the new row against the positions still to be visited
    }
    // write back: survivors in position order, kInvalid after; rewritten rows and metadata
    if (valid && size < b) slots[p + g] = g < size ? slot : kInvalid;
    if (valid && dirty) {  // a rewritten row sits at a position below every merge after it
      const float* src = lds + (gbase + rid) * ST;
      const size_t xo = (size_t)slot * r.dp;
      float nv = 0.0f;  // its exact sequential norm (distance.cc:33-34)
#pragma unroll
      for (int k = 0; k < D; k += 4) {
        const float4 v = *reinterpret_cast<const float4*>(src + k);
        nv = nv + v.x * v.x;
        nv = nv + v.y * v.y;
        nv = nv + v.z * v.z;
        nv = nv + v.w * v.w;
        store_row4(r, xo + k, v);
      }
      r.nrm[slot] = nv;
      r.cnt[slot] = cnt;
      r.head[slot] = hd;
    }
  }
#ifdef KLSH_MERGE_PROF
  sp3 = WPROF_CLK();
#endif
  if (dlist) append_slot(valid && dirty, slot, dlist, &ctr->n_delta);
  wave_lds_fence();
#ifdef KLSH_MERGE_PROF
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  if (lane == 0) {
    const int c = (int)__builtin_ctz(G) - 1;
    const uint64_t sp4 = WPROF_CLK();
    atomicAdd(&g_sprof[c][0], 1ull);
    atomicAdd(&g_sprof[c][1], sp1 - sp0);
    atomicAdd(&g_sprof[c][2], sp2 - sp1);
    atomicAdd(&g_sprof[c][3], sp3 - sp2);
    atomicAdd(&g_sprof[c][4], sp4 - sp3);
  }
#endif
  (void)nmerged;
}

// ------------------------------------------------- the fp16 screen of one batch -----
typedef _Float16 sh16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 sh16x2 __attribute__((ext_vector_type(2)));
typedef float pf16acc __attribute__((ext_vector_type(16)));
typedef float pf4acc __attribute__((ext_vector_type(4)));

// The fp16 screen of one batch: 64/G runs of class c (G = 2 << c lanes each, lane g = position g
// of its run, b = its run's length, x = its fp16 row).  True on the lanes of a run that some pair
// of which the screen cannot rule out (or that holds a row without a usable norm); false: the run
// cannot merge.  LDS (this wave's): lrow [64][D + 8] halves, linv / lsrow / lflag [64].
template <int D>
__device__ __forceinline__ bool screen_batch(int c, uint32_t b, const sh16x8 (&x)[D / 8],
                                             _Float16* lrow, float* linv, float* lsrow,
                                             uint32_t* lflag, float s_star, float m0, float a2) {
  constexpr int STH = D + 8;  // LDS row stride in halves (16-B pad)
  const uint32_t lane = __lane_id();
  const uint32_t G = 2u << c;
  const uint32_t g = lane & (G - 1);
  const bool valid = g < b;
  float ss = 0.0f;
#pragma unroll
  for (int q = 0; q < D / 8; ++q) {
    *reinterpret_cast<sh16x8*>(lrow + lane * STH + 8 * q) = valid ? x[q] : sh16x8{};
#pragma unroll
    for (int hi2 = 0; hi2 < 8; hi2 += 2) {
      const sh16x2 v = {x[q][hi2], x[q][hi2 + 1]};
      ss = __builtin_amdgcn_fdot2(v, v, ss, false);
    }
  }
  // a row without a usable norm (zero, tiny, fp16 overflow, NaN) cannot be screened: its run
  // goes to the exact merge
  const bool bad = valid && !(ss >= 0x1p-100f && ss <= 0x1p100f);
  const uint32_t lg = (uint32_t)__builtin_ctz(G);  // log2 G
  const float il = valid && !bad ? 1.0f / __builtin_sqrtf(ss) : 0.0f;
  linv[lane] = il;
  lsrow[lane] = s_star - (m0 + a2 * il);
  lflag[lane] = 0u;
  wave_lds_fence();
  if (bad) lflag[lane >> lg] = 1u;
  const uint64_t vmask = __ballot(valid && !bad);  // rows the Gram test reads
  // The Gram blocks of the batch's runs on the matrix cores (x~ . x~ exact products, f32 sums):
  // 32 x 32 tiles for runs of 17..64 rows (the upper-triangular tiles of each run), 16 x 16
  // diagonal tiles for shorter runs (4 per batch, runs never cross a 16-row block).  A pair
  // (R < C) of one run that the screen cannot rule out flags the run in LDS.  The tests are
  // branch-free over per-row terms loaded up front (a load inside each test's branch was a wait
  // on LDS per entry): a pair is ruled out when G/(|x~a||x~b|) < s* - (m0 + a2 (1/|x~a| +
  // 1/|x~b|)), evaluated as (G ir) ic < lsrow[R] - a2 ic — the margin's terms summed in another
  // order, a few ulps of s* against the margin's 1.5x headroom; pair validity is one per-lane
  // mask per tile, applied once to the tile's failures.
  auto test = [&](float sv, float ir, float sr, float ic, float kc) -> bool {
    return !(sv * ir * ic < sr - kc);  // NaN / inf: not ruled out
  };
  // bits (q & 3) + 8 (q >> 2) of w -> bit q (the tile rows of a lane, 32 x 32 layout)
  auto rows16 = [](uint32_t w) -> uint32_t {
    return (w & 0xFu) | ((w >> 4) & 0xF0u) | ((w >> 8) & 0xF00u) | ((w >> 12) & 0xF000u);
  };
  if constexpr (D < 32) {  // (not launched: screen_ok needs d >= 32) rule nothing out
    lflag[lane] = 1u;
  } else if (G >= 32u) {
    const uint32_t r32 = lane & 31u, k8 = 8u * (lane >> 5);
#pragma unroll 1
    for (int tt = 0; tt < 3; ++tt) {
      const uint32_t tr = tt == 2 ? 1u : 0u, tc = tt == 0 ? 0u : 1u;
      if (G == 32u && tt == 1) continue;  // two runs: their diagonal tiles only
      pf16acc acc;
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[q] = 0.0f;
#pragma unroll
      for (int ks = 0; ks < D / 16; ++ks) {
        const sh16x8 fa = *reinterpret_cast<const sh16x8*>(lrow + (tr * 32u + r32) * STH + 16 * ks + k8);
        const sh16x8 fb = *reinterpret_cast<const sh16x8*>(lrow + (tc * 32u + r32) * STH + 16 * ks + k8);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa, fb, acc, 0, 0, 0);
      }
      const uint32_t C = tc * 32u + r32, hb = 4u * (lane >> 5);
      const float ic = linv[C], kc = a2 * ic;
      float4 irv[4], srv[4];  // rows tr*32 + 8j + hb + (0..3)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        irv[j] = *reinterpret_cast<const float4*>(linv + tr * 32u + 8u * (uint32_t)j + hb);
        srv[j] = *reinterpret_cast<const float4*>(lsrow + tr * 32u + 8u * (uint32_t)j + hb);
      }
      // the lane's pairs (one run per tested tile): rows the image carries, column too, and
      // R < C on a diagonal tile (local row (q&3) + 8(q>>2) + hb below r32)
      uint32_t pm = rows16((uint32_t)(vmask >> (tr * 32u + hb)));
      if (tr == tc) {
        const uint32_t lim = r32 > hb ? r32 - hb : 0u;
        pm &= rows16(lim >= 32u ? 0xFFFFFFFFu : ((1u << lim) - 1u));
      }
      if (!((vmask >> C) & 1ull)) pm = 0u;
      uint32_t fm = 0u;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const float4 v = irv[q >> 2], u = srv[q >> 2];
        const float ir = (q & 3) == 0 ? v.x : (q & 3) == 1 ? v.y : (q & 3) == 2 ? v.z : v.w;
        const float sr = (q & 3) == 0 ? u.x : (q & 3) == 1 ? u.y : (q & 3) == 2 ? u.z : u.w;
        fm |= test(acc[q], ir, sr, ic, kc) ? (1u << q) : 0u;
      }
      if (fm & pm) lflag[C >> lg] = 1u;
    }
  } else {
    const uint32_t r16 = lane & 15u, k8 = 8u * (lane >> 4);
#pragma unroll 1
    for (int tb = 0; tb < 4; ++tb) {
      pf4acc acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int ks = 0; ks < D / 32; ++ks) {
        const sh16x8 f = *reinterpret_cast<const sh16x8*>(lrow + (16u * tb + r16) * STH + 32 * ks + k8);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(f, f, acc, 0, 0, 0);
      }
      const uint32_t C = 16u * tb + r16, rb = 16u * tb + 4u * (lane >> 4);
      const float ic = linv[C], kc = a2 * ic;
      const float4 v = *reinterpret_cast<const float4*>(linv + rb);
      const float4 u = *reinterpret_cast<const float4*>(lsrow + rb);
      const float irq[4] = {v.x, v.y, v.z, v.w}, srq[4] = {u.x, u.y, u.z, u.w};
      bool fail = false;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t R = rb + (uint32_t)q;
        const bool pair = (R < C) & ((R >> lg) == (C >> lg)) & (((vmask >> R) & (vmask >> C) & 1ull) != 0ull);
        fail |= pair & test(acc[q], irq[q], srq[q], ic, kc);
      }
      if (fail) lflag[C >> lg] = 1u;
    }
  }
  wave_lds_fence();
  return lflag[lane >> lg] != 0u;
}

// ------------------------------------------------- all small-run classes in one launch -----
// Runs of 2..64 rows of every size class in ONE persistent launch: the batches of all classes
// (a batch = one wave's 64/G runs of class G; 64 runs of 2 for the pair class) are numbered in
// one space, most expensive class first, and wave w takes batches w, w + grid, ...  Compared
// with one kernel per class on three streams this removes the per-class launch chains and the
// idle tails of the small classes.  The next batch's list entry and slot are loaded while the
// current batch is merged.
template <int G>
__device__ __forceinline__ uint32_t batches_of(uint32_t n) {
  return (n + (64u / G) - 1) / (64u / G);
}

template <int D>
__device__ __forceinline__ void pair_batch(const uint2* __restrict__ list, uint32_t n, uint32_t bi,
                                           uint32_t* __restrict__ slots, const Decider& dc,
                                           const Rows& r, Counters* ctr, uint32_t* dlist) {
  const uint32_t k = bi * 64u + __lane_id();
  bool merged = false;
  uint32_t s0 = 0;
  if (k < n) {
    const uint2 e = list[k];
    s0 = slots[e.x];
    const uint32_t s1 = slots[e.x + 1];
    float x0[D], x1[D];
    load_row<D>(r.x + (size_t)s0 * r.dp, x0);
    load_row<D>(r.x + (size_t)s1 * r.dp, x1);
    float dot = 0.0f;
#pragma unroll
    for (int q = 0; q < D; ++q) dot = dot + x1[q] * x0[q];  // cosine(c[1], c[0]), in order
    // the norms, recomputed from the rows in registers (the cached chain, distance.cc:33-34)
    float n0 = 0.0f, n1 = 0.0f;
#pragma unroll
    for (int q = 0; q < D; ++q) {
      n0 = n0 + x0[q] * x0[q];
      n1 = n1 + x1[q] * x1[q];
    }
    if (decide(dc, dot, __builtin_sqrtf(n1) * __builtin_sqrtf(n0))) {
      merged = true;
      const uint32_t ca = r.cnt[s1], cb = r.cnt[s0];  // current = row 1, candidate = row 0
      const float fa = (float)(int)ca, fb = (float)(int)cb, fn = (float)(int)(ca + cb);
      float nn = 0.0f;
      const size_t xo = (size_t)s0 * r.dp;
#pragma unroll
      for (int q = 0; q < D; q += 4) {
        float4 v;
        v.x = consensus(x1[q], fa, x0[q], fb, fn);
        v.y = consensus(x1[q + 1], fa, x0[q + 1], fb, fn);
        v.z = consensus(x1[q + 2], fa, x0[q + 2], fb, fn);
        v.w = consensus(x1[q + 3], fa, x0[q + 3], fb, fn);
        nn = nn + v.x * v.x;
        nn = nn + v.y * v.y;
        nn = nn + v.z * v.z;
        nn = nn + v.w * v.w;
        store_row4(r, xo + q, v);
      }
      r.nrm[s0] = nn;
      link_members(r, s1, s0);  // ids_current ++ ids_candidate; cnt[s1] = 0
      slots[e.x + 1] = kInvalid;
    }
  }
  if (dlist) append_slot(merged, s0, dlist, &ctr->n_delta);
}

// One wave's share of the small-run batches: waves `wave`, `wave + nwaves`, ... of the batch
// space; lds = this wave's 64 * (D + 4) floats.
template <int D>
__device__ __forceinline__ void small_loop(const MergeWork& w, uint32_t* __restrict__ slots,
                                           const Decider& dc, const Rows& r, Counters* ctr,
                                           float* lds, uint32_t wave, uint32_t nwaves) {
  constexpr int NC = kGroupClasses;
  uint32_t n[NC], nb[NC], start[NC + 1];
  // after the fp16 screen: only the runs it could not rule out (the others merge nothing)
  const CountLine* counts = w.screened ? w.rc->n_act : w.rc->n_cls;
  const uint2* const* lists = w.screened ? w.act : w.cls;
#pragma unroll
  for (int c = 0; c < NC; ++c)
    n[c] = __hip_atomic_load(&counts[c].v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  nb[0] = (n[0] + 63u) / 64u;
  nb[1] = batches_of<4>(n[1]);
  nb[2] = batches_of<8>(n[2]);
  nb[3] = batches_of<16>(n[3]);
  nb[4] = batches_of<32>(n[4]);
  nb[5] = batches_of<64>(n[5]);
  // batch space: class 5 (64-row runs) first ... class 0 (pairs) last
  start[NC] = 0;
  {
    uint32_t a = 0;
#pragma unroll
    for (int c = NC - 1; c >= 0; --c) {
      start[c] = a;
      a += nb[c];
    }
    start[NC] = a;  // total
  }
  const uint32_t total = start[NC];
  const uint32_t lane = __lane_id();
  auto locate = [&](uint32_t t, int& c, uint32_t& bi) {
    c = 0;
#pragma unroll
    for (int q = NC - 1; q >= 0; --q)
      if (t >= start[q] && t < start[q] + nb[q]) c = q;
    bi = t - start[c];
  };
  // the lane's (run, position) in batch bi of class c: entry and slot
  auto fetch = [&](uint32_t t, uint2& e, uint32_t& slot) {
    e = make_uint2(0u, 0u);
    slot = 0u;
    if (t >= total) return;
    int c;
    uint32_t bi;
    locate(t, c, bi);
    if (c == 0) return;  // pairs load their own
    const uint32_t G = 2u << c, NG = 64u / G;
    const uint32_t k = bi * NG + lane / G, g = lane & (G - 1);
    if (k < n[c]) {
      e = lists[c][k];
      if (g < e.y) slot = slots[e.x + g];
    }
  };
  uint2 e;
  uint32_t slot;
  fetch(wave, e, slot);
  for (uint32_t t = wave; t < total; t += nwaves) {
    uint2 e_next;
    uint32_t slot_next;
    fetch(t + nwaves, e_next, slot_next);
    int c;
    uint32_t bi;
    locate(t, c, bi);
    switch (c) {  // wave-uniform
      case 0: pair_batch<D>(lists[0], n[0], bi, slots, dc, r, ctr, w.dlist); break;
      case 1: merge_batch<4, D>(e.x, e.y, slot, slots, dc, r, lds, w.dlist, ctr); break;
      case 2: merge_batch<8, D>(e.x, e.y, slot, slots, dc, r, lds, w.dlist, ctr); break;
      case 3: merge_batch<16, D>(e.x, e.y, slot, slots, dc, r, lds, w.dlist, ctr); break;
      case 4: merge_batch<32, D>(e.x, e.y, slot, slots, dc, r, lds, w.dlist, ctr); break;
      default: merge_batch<64, D>(e.x, e.y, slot, slots, dc, r, lds, w.dlist, ctr); break;
    }
    e = e_next;
    slot = slot_next;
  }
}


// ------------------------------------------------- the fp16 screen of the small runs -----
// Every run of 2..64 rows is first tested on the fp16 row image (Rows::xh, half the bytes of the
// f32 rows): a run can merge only if some pair (a, b) passes cosine >= s* (cluster.cc:66-69), and
//   |x~a.x~b / (|x~a| |x~b|) - fl(dot_ref / fl(sqrtf(nrm_a) sqrtf(nrm_b)))| <= m
// with m = m0 + a2 (1/|x~a| + 1/|x~b|): the fp16 rounding of both rows (2^-11 each, relative, plus
// 2^-25 absolute per element for subnormals), the screen's f32 sums, the reference's own sequential
// sums and the quotient's roundings, 1.5x headroom (screen_margins).  A run none of whose pairs
// reaches s* - m cannot merge: it is left as it is — the walk's result for it is "no change" — and
// only the others go on to k_merge_small (lists MergeWork::act), which decides them exactly on the
// f32 rows.  A row whose image has no usable norm (zero, tiny, fp16 overflow, NaN) keeps its run.
//
// The screen is a gather of 64 fp16 rows per batch followed by little arithmetic (the Gram blocks
// on the matrix cores), so what bounds it is the bytes in flight: each wave keeps the rows of the
// next kAhead batches loading in registers while it screens one (and the slots and list entries
// of the batches after those), so a wave has up to kAhead * 8 KB of row loads outstanding instead
// of waiting for one batch at a time.  One wave per workgroup; the batches of every class (64/G
// runs of G lanes, lane g = position g) in one persistent space, most expensive class first;
// passed runs collect in LDS per class and go out 32+ at a time (one atomic per flush).
// (lookahead 1 / 3 and 3 waves per EU measured the same as 2 / 2)
constexpr int kScreenAhead = 2;  // batches whose rows are in flight while one is screened

template <int D>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void k_small_screen(MergeWork w, const uint32_t* __restrict__ slots,
                                                     Rows r, float s_star, float m0, float a2,
                                                     KTime kt) {
  constexpr int NC = kGroupClasses, STH = D + 8;  // LDS row stride in halves (16-B pad)
  constexpr int NR = kScreenAhead + 1;            // row buffers: the screened batch + the ones ahead
  constexpr uint32_t kBuf = 256;                  // passed runs kept in LDS before a flush
  __shared__ __attribute__((aligned(16))) _Float16 lrow[64 * STH];
  __shared__ __attribute__((aligned(16))) float linv[64];
  __shared__ __attribute__((aligned(16))) float lsrow[64];  // s* - (m0 + a2 / |x~|): the row's part
  __shared__ uint32_t lflag[64];  // per run of the batch: some pair not ruled out
  __shared__ uint2 buf[kBuf];     // passed runs (start, length | class << 16)
  __shared__ uint32_t fcnt[NC], fbase[NC];
  kt_begin(kt, KC_SCREEN);
  const uint32_t lane = __lane_id();
  if (blockIdx.x == 0 && lane == 0) w.rc->screened.v = 1u;
  uint32_t n[NC], nb[NC], start[NC + 1];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    // (scalar: every batch index and class below is wave-uniform, so list pointers stay in SGPRs
    // and no vector load of a pointer makes the wave wait for its outstanding row loads)
    n[c] = __builtin_amdgcn_readfirstlane(
        __hip_atomic_load(&w.rc->n_cls[c].v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const uint32_t per = 32u >> c;  // runs per batch: 64 / G, G = 2 << c
    nb[c] = (n[c] + per - 1u) / per;
  }
  {
    uint32_t a = 0;
#pragma unroll
    for (int c = NC - 1; c >= 0; --c) {
      start[c] = a;
      a += nb[c];
    }
    start[NC] = a;
  }
  const uint32_t total = start[NC], stride = gridDim.x;
  uint32_t nbuf = 0, brows = 0;  // (wave-uniform)
  // this wave's passed runs to the global lists: per class, one add and the entries
  auto flush = [&]() {
    if (lane < (uint32_t)NC) fcnt[lane] = 0u;
    wave_lds_fence();
    for (uint32_t i = lane; i < nbuf; i += 64) atomicAdd(&fcnt[buf[i].y >> 16], 1u);
    wave_lds_fence();
    if (lane < (uint32_t)NC) {
      const uint32_t c = fcnt[lane];
      fbase[lane] = c ? atomicAdd(&w.rc->n_act[lane].v, c) : 0u;
      fcnt[lane] = 0u;
    }
    if (lane == 0 && brows) atomicAdd(&w.rc->n_act_rows.v, brows);
    wave_lds_fence();
    for (uint32_t i = lane; i < nbuf; i += 64) {
      const uint2 e = buf[i];
      const uint32_t c = e.y >> 16;
      const uint32_t at = fbase[c] + atomicAdd(&fcnt[c], 1u);
      w.act[c][at] = make_uint2(e.x, e.y & 0xFFFFu);
    }
    wave_lds_fence();
    nbuf = brows = 0u;
  };
  const uint64_t below = lanes_below(lane);
  auto class_of = [&](uint32_t t) -> int {  // (wave-uniform: t is)
    int c = 0;
#pragma unroll
    for (int q = NC - 1; q >= 0; --q)
      if (t >= start[q] && t < start[q] + nb[q]) c = q;
    return __builtin_amdgcn_readfirstlane(c);
  };
  auto list_of = [&](int c) -> const uint2* {
    return c == 0 ? w.cls[0] : c == 1 ? w.cls[1] : c == 2 ? w.cls[2] : c == 3 ? w.cls[3]
         : c == 4 ? w.cls[4] : w.cls[5];
  };
  // Every load below is unconditional (a lane with nothing to load reads a valid dummy address),
  // so the loads of the batches ahead are never waited for early: the compiler counts them.
  // the lane's run entry in batch t ((0, 0) past the end)
  auto entry_of = [&](uint32_t t) -> uint2 {
    const int c = class_of(t);
    const uint32_t G = 2u << c, NG = 64u / G;
    const uint32_t k = (t - start[c]) * NG + lane / G;
    const bool ok = t < total && k < n[c];
    const uint2 e = list_of(c)[ok ? k : 0u];  // (every list holds >= 64 entries)
    return ok ? e : make_uint2(0u, 0u);
  };
  auto slot_of = [&](uint32_t t, const uint2& e) -> uint32_t {
    const uint32_t g = lane & ((2u << class_of(t)) - 1u);
    return slots[g < e.y ? e.x + g : e.x];
  };
  auto load_rows = [&](uint32_t slot, sh16x8 (&x)[D / 8]) {
    const uint16_t* src = r.xh + (size_t)slot * r.dp;
#pragma unroll
    for (int q = 0; q < D / 8; ++q) x[q] = *reinterpret_cast<const sh16x8*>(src + 8 * q);
  };
  // one batch: rows x (arrived), entry e
  auto screen = [&](uint32_t t, const uint2& e, const sh16x8 (&x)[D / 8]) {
    const int c = class_of(t);
    const uint32_t G = 2u << c;
    const uint32_t g = lane & (G - 1);
    const uint32_t b = e.y;
    const bool grp = screen_batch<D>(c, b, x, lrow, linv, lsrow, lflag, s_star, m0, a2);
    const bool leader = g == 0u && b >= 2u && grp;
    const uint64_t lead = __ballot(leader);
    if (lead) {
      if (nbuf + 64u > kBuf) flush();  // (rare: the buffer holds a wave's passed runs)
      if (leader)
        buf[nbuf + (uint32_t)__popcll(lead & below)] = make_uint2(e.x, b | ((uint32_t)c << 16));
      uint32_t rsum = leader ? b : 0u;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) rsum += (uint32_t)__shfl_xor((int)rsum, o, 64);
      nbuf += (uint32_t)__popcll(lead);
      brows += rsum;
    }
    wave_lds_fence();  // the rows of this batch are read before the next batch overwrites them
  };
  // The pipeline (batches t0, t0 + stride, ...): batch j is screened while the rows of j+1 ..
  // j+kAhead, the slot of j+kAhead+1 and the entries of j+kAhead+1, j+kAhead+2 are in flight.
  // Row buffers rotate through NR register arrays (the loop is unrolled NR times so every index
  // is static).
  sh16x8 xb[NR][D / 8];
  uint2 eb[NR];  // entries of the batches whose rows are (to be) in xb (same index)
  const uint32_t t0 = blockIdx.x;
  {
    uint2 e0[NR];
#pragma unroll
    for (int k = 0; k < NR; ++k) e0[k] = entry_of(t0 + (uint32_t)k * stride);
#pragma unroll
    for (int k = 0; k < NR - 1; ++k) {
      eb[k] = e0[k];
      load_rows(slot_of(t0 + (uint32_t)k * stride, e0[k]), xb[k]);
    }
    eb[NR - 1] = e0[NR - 1];
  }
  uint32_t s_next = slot_of(t0 + (uint32_t)(NR - 1) * stride, eb[NR - 1]);
  uint2 e_next = entry_of(t0 + (uint32_t)NR * stride);
  // Issue order matters: the slot and entry loads go out BEFORE the row loads, so that waiting
  // for them next step (vmcnt counts in issue order) leaves the rows in flight.
  auto step = [&](uint32_t t, int cur) {  // cur: the buffer of batch t
    const int nxt = (cur + NR - 1) % NR;  // the buffer of batch t + kAhead * stride
    const uint32_t ta = t + (uint32_t)NR * stride;
    const uint32_t s_rows = s_next;       // slot of batch t + kAhead (arrived a step ago)
    s_next = slot_of(ta, e_next);
    const uint2 e_after = entry_of(ta + stride);
    load_rows(s_rows, xb[nxt]);
    const uint2 e_cur = eb[cur];
    eb[cur] = e_next;  // batch t + NR * stride's rows go to this buffer next time round
    e_next = e_after;
    screen(t, e_cur, xb[cur]);
  };
  // (whole rounds of NR steps: a batch past the end screens nothing, and a branch-free body
  // keeps the compiler's count of the loads in flight exact across the loop)
  for (uint32_t t = t0; t < total; t += (uint32_t)NR * stride) {
#pragma unroll
    for (int k = 0; k < NR; ++k) step(__builtin_amdgcn_readfirstlane(t + (uint32_t)k * stride), k);
  }
  if (nbuf) flush();
  kt_end(kt, KC_SCREEN);
}

template <int D>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void k_merge_small(
    MergeWork w, uint32_t* __restrict__ slots,
                                                    Decider dc, Rows r, Counters* ctr) {
  __shared__ __attribute__((aligned(16))) float lds[64 * (D + 4)];
  kt_begin(w.kt, KC_SMALL);
  small_loop<D>(w, slots, dc, r, ctr, lds, blockIdx.x, gridDim.x);
  kt_end(w.kt, KC_SMALL);
}

// Runs of equal keys, listed by size class, in three launches and no contended atomics:
//   k_runs_count  a tile of 4096 positions is read coalesced (position k*256 + t by thread t), its
//                 head flags become a 4096-bit bitmap (wave ballots, kept in global memory with the
//                 first head past the tile end), each head finds its run's end as the next set bit
//                 and its list (size class, big class, huge, oversize); per-list counts per tile
//   k_runs_scan   one workgroup per list: exclusive scan of its counts over the tiles, the total
//                 into the list's counter
//   k_runs_write  every head again from the stored bitmap, its entry at the tile's base + a rank
// (one global add per list per tile — the single-kernel version — serialised ~2300 adds per counter
// at C2 size, 80-100 us).  Entries within a list are in no particular order; every merge result is
// positional.
constexpr uint32_t kRunTile = 4096;
constexpr int kRunLists = kGroupClasses + kBigClasses + 2;  // small classes, big classes, huge, over
// + the head count (n_seg), rows in small runs, rows in each big class and in huge runs
constexpr int kRunRows = kRunLists + 2 + kBigClasses + 1;

__device__ __forceinline__ uint32_t* run_counter(RunCounters* rc, int l) {
  return l < kGroupClasses ? &rc->n_cls[l].v
         : l < kGroupClasses + kBigClasses ? &rc->n_big[l - kGroupClasses].v
         : l == kRunLists - 2 ? &rc->n_huge.v
         : l == kRunLists - 1 ? &rc->n_over.v
         : l == kRunLists ? &rc->n_seg.v
         : l == kRunLists + 1 ? &rc->n_small_rows.v
         : l < kRunLists + 2 + kBigClasses ? &rc->n_big_rows[l - kRunLists - 2].v
                                           : &rc->n_huge_rows.v;
}

// The list of a run of b rows (-1: one row).
__device__ __forceinline__ int run_class(uint32_t b, int bucket_thr) {
  if (bucket_thr >= 0 && b > (uint32_t)bucket_thr) return kRunLists - 1;  // cluster.cc:286
  if (b > 64u) {
    if (b > (uint32_t)kBigRows[kBigClasses - 1]) return kRunLists - 2;
    int c = 0;
    while (b > (uint32_t)kBigRows[c]) ++c;
    return kGroupClasses + c;
  }
  return b >= 2 ? size_class(b) : -1;
}

// The entries of list l (0 <= l < kRunLists).  With a per-lane l this is a vector load from the
// kernel-argument block, and a store through it waits for that load: the run-listing kernels read
// the pointers once into an LDS table (run_list_table) instead of once per entry.
__device__ __forceinline__ uint2* run_list_ptr(const MergeWork& w, int l) {
  uint2* p = l == kRunLists - 2 ? w.huge : w.over;
#pragma unroll
  for (int c = 0; c < kBigClasses; ++c) p = l == kGroupClasses + c ? w.big[c] : p;
#pragma unroll
  for (int c = 0; c < kGroupClasses; ++c) p = l == c ? w.cls[c] : p;
  return p;
}

// Threads 0 .. kRunLists-1 fill tab with the list pointers (visible after the next barrier),
// typed as global memory: a generic pointer read back from LDS would make every entry store a
// flat store, which the LDS waits that follow it also wait for.
using RunListPtr = __attribute__((address_space(1))) uint64_t*;
__device__ __forceinline__ void run_list_table(const MergeWork& w, RunListPtr* tab) {
  const uint32_t t = threadIdx.x;
  RunListPtr p = (RunListPtr)(uint64_t*)run_list_ptr(w, (int)min(t, (uint32_t)kRunLists - 1u));
  if (t < (uint32_t)kRunLists) tab[t] = p;
}
// A (start, length) entry as one 64-bit store (uint2 layout: x in the low word).
__device__ __forceinline__ uint64_t run_entry(uint32_t start, uint32_t len) {
  return (uint64_t)len << 32 | start;
}

// What run counter `l` (kRunRows of them) receives for a run of b rows in list lr.
__device__ __forceinline__ uint32_t run_contrib(int l, int lr, uint32_t b) {
  if (l < kRunLists) return l == lr ? 1u : 0u;
  if (l == kRunLists) return 0u;  // heads: counted where the head is found
  if (l == kRunLists + 1) return (lr >= 0 && lr < kGroupClasses) ? b : 0u;
  if (l < kRunLists + 2 + kBigClasses) return lr == kGroupClasses + (l - kRunLists - 2) ? b : 0u;
  return lr == kRunLists - 2 ? b : 0u;
}

// Exclusive suffix minimum over the 256 threads of a workgroup: min of v over threads > t (~0u if
// none).  Every thread must call it.
__device__ __forceinline__ uint32_t block_excl_suffix_min_256(uint32_t v) {
  __shared__ uint32_t sm[256];
  const uint32_t t = threadIdx.x;
  sm[t] = v;
  __syncthreads();
  for (uint32_t o = 1; o < 256; o <<= 1) {  // inclusive suffix min, Hillis-Steele
    const uint32_t u = t + o < 256 ? sm[t + o] : ~0u;
    __syncthreads();
    sm[t] = min(sm[t], u);
    __syncthreads();
  }
  const uint32_t r = t + 1 < 256 ? sm[t + 1] : ~0u;
  __syncthreads();
  return r;
}

// The run starting at tile-local position q (a head of bitmap hb): its length and list (-1: one row).
__device__ __forceinline__ int run_list(const uint64_t* hb, uint32_t T0, uint32_t tail_end,
                                        uint32_t q, int bucket_thr, uint32_t& b) {
  uint32_t wi = q >> 6;
  uint64_t m = hb[wi] & ~((2ull << (q & 63u)) - 1ull);  // heads after q in its word
  while (!m && ++wi < kRunTile / 64) m = hb[wi];
  const uint32_t next = m ? T0 + wi * 64u + (uint32_t)__builtin_ctzll(m) : tail_end;
  b = next - (T0 + q);
  return run_class(b, bucket_thr);
}

// Per tile: the head bitmap, the first head (global position, ~0u = none) and the last head
// (tile-local, ~0u = none), and per-list counts of every run that starts in the tile EXCEPT its
// last one: that run's end is the first head of a later tile (tail_end), found by a suffix minimum
// over the tiles' first heads in the scan / write kernel — so no tile walks forward past its end
// (linear in n at any run length).
__global__ __launch_bounds__(256) void k_runs_count(const uint32_t* __restrict__ key, uint32_t lo,
                                                    uint32_t n, int bucket_thr, uint32_t ntiles,
                                                    uint64_t* __restrict__ hbits,
                                                    uint2* __restrict__ heads_fl,
                                                    uint32_t* __restrict__ counts, KTime kt,
                                                    const uint32_t* __restrict__ n_dev) {
  kt_begin(kt, KC_RUNS);
  if (n_dev) n = *n_dev;  // tiles past it find no heads and count nothing
  __shared__ uint64_t hb[kRunTile / 64];
  __shared__ uint32_t lcnt[kRunRows];
  __shared__ uint32_t s_last;
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint32_t T0 = blockIdx.x * kRunTile;
  if (t < (uint32_t)kRunRows) lcnt[t] = 0u;
  const uint32_t* kp = key + lo;
  uint32_t a[16], pv[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t i = T0 + (uint32_t)k * 256u + t;
    a[k] = i < n ? kp[i] : 0u;
    pv[k] = (i < n && i > 0) ? kp[i - 1] : 0u;
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t i = T0 + (uint32_t)k * 256u + t;
    const uint64_t m = __ballot(i < n && (i == 0 || a[k] != pv[k]));
    if (lane == 0) {
      hb[k * 4 + wv] = m;
      hbits[(size_t)blockIdx.x * (kRunTile / 64) + k * 4 + wv] = m;
    }
  }
  __syncthreads();
  if (wv == 0) {  // the tile's first and last heads (bitmap word `lane`)
    const uint64_t m = hb[lane];
    const uint64_t nz = __ballot(m != 0ull);
    uint32_t first = ~0u, last = ~0u;
    if (nz) {
      const uint32_t wf = (uint32_t)__builtin_ctzll(nz), wl = 63u - (uint32_t)__builtin_clzll(nz);
      first = T0 + wf * 64u + (uint32_t)__builtin_ctzll(hb[wf]);
      last = wl * 64u + 63u - (uint32_t)__builtin_clzll(hb[wl]);
    }
    if (lane == 0) {
      s_last = last;
      heads_fl[blockIdx.x] = make_uint2(first, last);
    }
  }
  __syncthreads();
  const uint32_t lastq = s_last;
  const uint64_t lt = lane ? (~0ull >> (64u - lane)) : 0ull;
  uint32_t heads = 0, small_rows = 0;
  uint32_t lrows[kBigClasses + 1] = {};  // rows per big class, then huge
#pragma unroll 4
  for (int k = 0; k < 16; ++k) {
    const uint32_t q = (uint32_t)k * 256u + t;
    int l = -1;
    if ((hb[q >> 6] >> (q & 63u)) & 1ull) {
      ++heads;
      if (q != lastq) {  // (the last run's list: the scan / write kernel)
        uint32_t b;
        l = run_list(hb, T0, 0u, q, bucket_thr, b);
        if (l >= 0 && l < kGroupClasses) small_rows += b;
#pragma unroll
        for (int c = 0; c <= kBigClasses; ++c)
          if (l == kGroupClasses + c) lrows[c] += b;
      }
    }
    // lanes with the same list: one LDS add by the lowest of them
    const uint32_t id = (uint32_t)(l + 1);  // 0 = no entry
    uint64_t match = ~0ull;
#pragma unroll
    for (int bit = 0; bit < 4; ++bit) {
      const uint64_t mb = __ballot((id >> bit) & 1u);
      match &= ((id >> bit) & 1u) ? mb : ~mb;
    }
    if (l >= 0 && (match & lt) == 0ull) atomicAdd(&lcnt[l], (uint32_t)__popcll(match));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    heads += __shfl_xor(heads, o, 64);
    small_rows += __shfl_xor(small_rows, o, 64);
#pragma unroll
    for (int c = 0; c <= kBigClasses; ++c) lrows[c] += __shfl_xor(lrows[c], o, 64);
  }
  if (lane == 0 && heads) atomicAdd(&lcnt[kRunLists], heads);
  if (lane == 0 && small_rows) atomicAdd(&lcnt[kRunLists + 1], small_rows);
#pragma unroll
  for (int c = 0; c <= kBigClasses; ++c)
    if (lane == 0 && lrows[c]) atomicAdd(&lcnt[kRunLists + 2 + c], lrows[c]);
  __syncthreads();
  if (t < (uint32_t)kRunRows) counts[(size_t)t * ntiles + blockIdx.x] = lcnt[t];
}

// The last run of tile j (tile-local head `last`, ~0u = none) ends at tail_end: its length.
__device__ __forceinline__ uint32_t last_run_len(uint32_t j, uint32_t last, uint32_t tail_end) {
  return last == ~0u ? 0u : tail_end - (j * kRunTile + last);
}

// Workgroup l: the tiles' last runs (their ends from a suffix minimum over the first heads; list
// 0's workgroup writes the tail ends) into counts[l], then counts[l][0..ntiles) -> exclusive prefix
// over the tiles; the total -> list l's counter.
__global__ __launch_bounds__(256) void k_runs_scan(uint32_t* __restrict__ counts, uint32_t ntiles,
                                                   uint32_t n, int bucket_thr,
                                                   const uint2* __restrict__ heads_fl,
                                                   uint32_t* __restrict__ tail_ends,
                                                   RunCounters* rc) {
  const int l = (int)blockIdx.x;
  uint32_t* row = counts + (size_t)l * ntiles;
  const uint32_t t = threadIdx.x;
  const uint32_t per = (ntiles + 255u) / 256u;
  const uint32_t a = min(ntiles, t * per), e = min(ntiles, a + per);
  // A thread's tiles are read CH at a time, every load of a chunk issued before any use (index
  // clamped into the chunk, no branch around a load): one round trip per chunk, not per tile —
  // this one-workgroup-per-list launch is a latency chain.
  constexpr uint32_t CH = 8;
  uint32_t fmin = ~0u;  // first head of this thread's tiles
  for (uint32_t i0 = a; i0 < e; i0 += CH) {
    uint32_t hx[CH];
#pragma unroll
    for (uint32_t c = 0; c < CH; ++c) hx[c] = heads_fl[min(i0 + c, e - 1u)].x;
#pragma unroll
    for (uint32_t c = 0; c < CH; ++c) fmin = min(fmin, hx[c]);  // (clamped repeats: harmless)
  }
  uint32_t after = block_excl_suffix_min_256(fmin);  // first head after this thread's tiles
  uint32_t acc = 0;
  for (uint32_t i1 = e; i1 > a;) {  // reverse: `after` is the first head after tile i
    const uint32_t i0 = i1 - a > CH ? i1 - CH : a;
    uint2 hf[CH];
    uint32_t rv[CH];
#pragma unroll
    for (uint32_t c = 0; c < CH; ++c) {
      const uint32_t j = min(i0 + c, i1 - 1u);
      hf[c] = heads_fl[j];
      rv[c] = row[j];
    }
#pragma unroll
    for (int c = (int)CH - 1; c >= 0; --c) {
      const uint32_t i = i0 + (uint32_t)c;
      if (i < i1) {
        const uint32_t te = min(after, n);
        if (l == 0) tail_ends[i] = te;
        const uint32_t b = last_run_len(i, hf[c].y, te);
        uint32_t v = rv[c];
        if (b) v += run_contrib(l, run_class(b, bucket_thr), b);
        row[i] = v;
        acc += v;
        after = min(after, hf[c].x);
      }
    }
    i1 = i0;
  }
  uint32_t total;
  uint32_t run = block_excl_scan_256(acc, &total);
  for (uint32_t i0 = a; i0 < e; i0 += CH) {
    uint32_t rv[CH];
#pragma unroll
    for (uint32_t c = 0; c < CH; ++c) rv[c] = row[min(i0 + c, e - 1u)];
#pragma unroll
    for (uint32_t c = 0; c < CH; ++c)
      if (i0 + c < e) {
        row[i0 + c] = run;
        run += rv[c];
      }
  }
  if (t == 0) *run_counter(rc, l) = total;
}

// SCAN (ntiles <= 256, every iteration below 2^20 positions): `counts` are the raw per-tile counts
// and each workgroup sums its own list bases (the tiles before it; thread t holds tile t, and adds
// tile t's last run once the suffix minimum of the first heads gives its end) — and workgroup 0
// the list totals — so k_runs_scan is not launched: one dependent launch less.
template <bool SCAN>
__global__ __launch_bounds__(256) void k_runs_write(uint32_t lo, uint32_t n, int bucket_thr,
                                                    uint32_t ntiles,
                                                    const uint64_t* __restrict__ hbits,
                                                    const uint2* __restrict__ heads_fl,
                                                    const uint32_t* __restrict__ tail_ends,
                                                    const uint32_t* __restrict__ counts,
                                                    MergeWork w, const uint32_t* __restrict__ n_dev) {
  __shared__ uint64_t hb[kRunTile / 64];
  __shared__ uint32_t lbase[kRunLists], lfill[kRunLists];
  __shared__ uint32_t s_tail_end;
  __shared__ RunListPtr lptr[kRunLists];
  const uint32_t t = threadIdx.x;
  const uint32_t T0 = blockIdx.x * kRunTile;
  // (the header loads unconditional, index clamped: issued together, one round trip)
  uint32_t cb = 0u, te = 0u;
  if constexpr (!SCAN) {
    cb = counts[(size_t)min(t, (uint32_t)kRunLists - 1u) * ntiles + blockIdx.x];
    te = tail_ends[blockIdx.x];
  }
  const uint64_t hv = hbits[(size_t)blockIdx.x * (kRunTile / 64) + (t & (kRunTile / 64 - 1u))];
  run_list_table(w, lptr);
  if (t < kRunTile / 64) hb[t] = hv;
  if constexpr (SCAN) {
    if (n_dev) n = *n_dev;
    __shared__ uint32_t red[2][4][kRunRows];
    const uint32_t lane = t & 63u, wv = t >> 6;
    uint32_t cv[kRunRows];  // every load in flight before the reductions
#pragma unroll
    for (int l = 0; l < kRunRows; ++l) cv[l] = t < ntiles ? counts[(size_t)l * ntiles + t] : 0u;
    const uint2 hf = t < ntiles ? heads_fl[t] : make_uint2(~0u, ~0u);
    const uint32_t te = min(block_excl_suffix_min_256(hf.x), n);  // the end of tile t's last run
    if (t == blockIdx.x) s_tail_end = te;
    const uint32_t lb = t < ntiles ? last_run_len(t, hf.y, te) : 0u;
    const int lr = lb ? run_class(lb, bucket_thr) : -1;
#pragma unroll
    for (int l = 0; l < kRunRows; ++l) cv[l] += lb ? run_contrib(l, lr, lb) : 0u;
#pragma unroll
    for (int l = 0; l < kRunRows; ++l) {
      const uint32_t v = cv[l];
      uint32_t before = t < blockIdx.x ? v : 0u, all = v;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        before += __shfl_xor(before, o, 64);
        all += __shfl_xor(all, o, 64);
      }
      if (lane == 0) {
        red[0][wv][l] = before;
        red[1][wv][l] = all;
      }
    }
    __syncthreads();
    if (t < (uint32_t)kRunLists) {
      lbase[t] = red[0][0][t] + red[0][1][t] + red[0][2][t] + red[0][3][t];
      lfill[t] = 0u;
    }
    if (blockIdx.x == 0 && t < (uint32_t)kRunRows)
      *run_counter(w.rc, (int)t) = red[1][0][t] + red[1][1][t] + red[1][2][t] + red[1][3][t];
  } else {
    if (t < (uint32_t)kRunLists) {
      lbase[t] = cb;
      lfill[t] = 0u;
    }
    if (t == 0) s_tail_end = te;
  }
  __syncthreads();
  const uint32_t tail_end = s_tail_end;
#pragma unroll 4
  for (int k = 0; k < 16; ++k) {
    const uint32_t q = (uint32_t)k * 256u + t;
    if ((hb[q >> 6] >> (q & 63u)) & 1ull) {
      uint32_t b;
      const int l = run_list(hb, T0, tail_end, q, bucket_thr, b);
      if (l < 0) continue;
      const uint32_t at = lbase[l] + atomicAdd(&lfill[l], 1u);
      lptr[l][at] = run_entry(lo + T0 + q, b);
    }
  }
  kt_end(w.kt, KC_RUNS);
}

// ------------------------------------------- small iterations: local bucket sort + runs -----
// Below 2^20 positions the stable bucket order (merge_hashtable, cluster.cc:15-30) is built in two
// steps: a stable partition by the top kTailTopBits = 9 key bits (radix_sort_top: one hist / dscan / scatter
// pass), then this kernel — workgroup d takes top bucket d, a contiguous range of the partition in
// canonical order, and sorts it stably by the remaining `lb` low bits (a counting sort in LDS:
// digit counts, their exclusive scan, then ranks among equal digits in position order from wave
// ballots, 4096 keys per round).  Equal keys of one top bucket have equal low bits, so the runs
// of the iteration are exactly the low digits with a count >= 2: their (start, length) entries
// come straight from the digit counts, classified as k_runs_write does (run_class), with one
// list-counter add per list per bucket — the whole run finding of these iterations without the
// tile kernels (k_runs_count / k_runs_write) or the second radix pass (3 launches).
__global__ __launch_bounds__(256) void k_tail_local(const uint32_t* __restrict__ kin,
                                                    const uint32_t* __restrict__ vin,
                                                    uint32_t* __restrict__ kout,
                                                    uint32_t* __restrict__ vout,
                                                    const uint32_t* __restrict__ dtot, int lb,
                                                    int bucket_thr, MergeWork w) {
  // (4 or 8 keys per lane per round measured the same as 16; J adaptive vs always 16: C2 run
  // listing 18.2 vs 18.4 ms per step, one box, three rounds)
  constexpr uint32_t kItems = 16;  // keys per lane per round at most
  constexpr uint32_t kRad = 1u << kTailLowBits, kPer = kRad / 256u;  // digits per thread
  __shared__ uint32_t cnt[kRad];      // low-digit counts, then their exclusive starts
  __shared__ uint32_t run_[kRad];     // running count of each digit over the rounds
  __shared__ uint32_t wc[4][kRad];    // per-wave digit counts of a round, then wave prefixes
  __shared__ uint32_t lcnt[kRunRows];  // this bucket's list counts, rows, heads
  __shared__ uint32_t lbase[kRunLists];
  __shared__ RunListPtr lptr[kRunLists];
  __shared__ uint32_t red[4];
  kt_begin(w.kt, KC_RUNS);
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint32_t d = blockIdx.x;
  const uint32_t RAD = 1u << lb, MASK = RAD - 1u;
  [[maybe_unused]] uint64_t tp0 = MPROF_T(), tp1 = 0;
  // the bucket: [base, base + m) of the partition
  // (every global load of this kernel is unconditional, index clamped into range: a load under a
  // branch is waited for at once, and these few-hundred-key buckets are a chain of round trips)
  uint32_t part = 0;
  const uint32_t m = dtot[d];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t i = t * 4u + (uint32_t)q;
    const uint32_t x = dtot[i < d ? i : 0u];
    part += i < d ? x : 0u;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
  if (lane == 0) red[wv] = part;
  for (uint32_t i = t; i < kRad; i += 256) {
    cnt[i] = 0u;
    run_[i] = 0u;
    wc[0][i] = wc[1][i] = wc[2][i] = wc[3][i] = 0u;
  }
  if (t < (uint32_t)kRunRows) lcnt[t] = 0u;
  __syncthreads();
  const uint32_t base = red[0] + red[1] + red[2] + red[3];
  if (m == 0u) {
    kt_end(w.kt, KC_RUNS);
    return;
  }
#ifdef KLSH_MERGE_PROF
  if (t == 0) { tp1 = MPROF_T(); TPROF_ADD(0, tp1 - tp0); TPROF_ADD(4, 1); }
#endif
  // 1. low-digit counts, in the scatter's layout: a round covers J * 256 positions, wave wv the J*64
  //    consecutive ones from wv*J*64 (item j of lane l: + j*64 + l), J = ceil(m / 256) up to 16 —
  //    so a bucket of a few hundred keys is spread over all four waves instead of being wave 0's
  //    chain of ranks.  The keys and slots of the first round are loaded together: a bucket of one
  //    round (almost all of them) is read once, the scatter below reuses the registers
  const uint32_t J = min(kItems, (m + 255u) / 256u), kChunk = J * 256u, kWave = J * 64u;
  uint32_t k[kItems], v[kItems];
#pragma unroll
  for (int j = 0; j < (int)kItems; ++j) {
    const uint32_t p = wv * kWave + (uint32_t)j * 64u + lane;
    const bool ok = (uint32_t)j < J && p < m;
    k[j] = kin[base + (ok ? p : 0u)];
    v[j] = vin[base + (ok ? p : 0u)];
  }
#pragma unroll
  for (int j = 0; j < (int)kItems; ++j)
    if ((uint32_t)j < J && wv * kWave + (uint32_t)j * 64u + lane < m) atomicAdd(&cnt[k[j] & MASK], 1u);
  for (uint32_t r0 = kChunk; r0 < m; r0 += kChunk) {  // (rare) further rounds: keys only
    uint32_t kk[kItems];
#pragma unroll
    for (int j = 0; j < (int)kItems; ++j) {
      const uint32_t p = r0 + wv * kWave + (uint32_t)j * 64u + lane;
      kk[j] = kin[base + (p < m ? p : 0u)];
    }
#pragma unroll
    for (int j = 0; j < (int)kItems; ++j)
      if (r0 + wv * kWave + (uint32_t)j * 64u + lane < m) atomicAdd(&cnt[kk[j] & MASK], 1u);
  }
  __syncthreads();
#ifdef KLSH_MERGE_PROF
  if (t == 0) { const uint64_t x = MPROF_T(); TPROF_ADD(1, x - tp1); tp1 = x; }
#endif
  // 2. the runs (digits with a count >= 2) per list, and the digit starts
  uint32_t c4[kPer], acc = 0, heads = 0, small_rows = 0;
  uint32_t lrows[kBigClasses + 1] = {};
  int l4[kPer];
#pragma unroll
  for (int q = 0; q < (int)kPer; ++q) {
    const uint32_t dg = t * kPer + (uint32_t)q;
    c4[q] = dg < RAD ? cnt[dg] : 0u;
    acc += c4[q];
    heads += c4[q] ? 1u : 0u;
    l4[q] = c4[q] >= 2u ? run_class(c4[q], bucket_thr) : -1;
    if (l4[q] >= 0) {
      atomicAdd(&lcnt[l4[q]], 1u);
      if (l4[q] < kGroupClasses) small_rows += c4[q];
#pragma unroll
      for (int c = 0; c <= kBigClasses; ++c)
        if (l4[q] == kGroupClasses + c) lrows[c] += c4[q];
    }
  }
  uint32_t total;
  uint32_t pre = block_excl_scan_256(acc, &total);  // (syncs: every lcnt add is in)
#pragma unroll
  for (int q = 0; q < (int)kPer; ++q) {
    const uint32_t dg = t * kPer + (uint32_t)q;
    if (dg < RAD) cnt[dg] = pre;
    pre += c4[q];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    heads += __shfl_xor(heads, o, 64);
    small_rows += __shfl_xor(small_rows, o, 64);
#pragma unroll
    for (int c = 0; c <= kBigClasses; ++c) lrows[c] += __shfl_xor(lrows[c], o, 64);
  }
  if (lane == 0) {
    if (heads) atomicAdd(&lcnt[kRunLists], heads);
    if (small_rows) atomicAdd(&lcnt[kRunLists + 1], small_rows);
#pragma unroll
    for (int c = 0; c <= kBigClasses; ++c)
      if (lrows[c]) atomicAdd(&lcnt[kRunLists + 2 + c], lrows[c]);
  }
  __syncthreads();
  if (t < (uint32_t)kRunRows && lcnt[t]) {  // one add per list (and counter) per bucket
    const uint32_t v = atomicAdd(run_counter(w.rc, (int)t), lcnt[t]);
    if (t < (uint32_t)kRunLists) lbase[t] = v;
  }
  if (t < (uint32_t)kRunLists) lcnt[t] = 0u;  // (reused as the list cursors)
  run_list_table(w, lptr);
  __syncthreads();
#pragma unroll
  for (int q = 0; q < (int)kPer; ++q) {
    const int l = l4[q];
    if (l >= 0) {
      const uint32_t dg = t * kPer + (uint32_t)q;
      const uint32_t at = lbase[l] + atomicAdd(&lcnt[l], 1u);
      lptr[l][at] = run_entry(base + cnt[dg], c4[q]);
    }
  }
  // 3. the stable scatter, J * 256 keys per round (wave wv: positions wv*J*64 + j*64 + lane)
#ifdef KLSH_MERGE_PROF
  __syncthreads();
  if (t == 0) { const uint64_t x = MPROF_T(); TPROF_ADD(2, x - tp1); tp1 = x; }
#endif
  const uint64_t lt = lane ? (~0ull >> (64u - lane)) : 0ull;
  for (uint32_t r0 = 0; r0 < m; r0 += kChunk) {
    uint32_t lr[kItems];
    if (m > kChunk) {  // (block-uniform) a bucket of several rounds reloads each round
#pragma unroll
      for (int j = 0; j < (int)kItems; ++j) {
        const uint32_t p = r0 + wv * kWave + (uint32_t)j * 64u + lane;
        k[j] = kin[base + (p < m ? p : 0u)];
        v[j] = vin[base + (p < m ? p : 0u)];
      }
    }
#pragma unroll
    for (int j = 0; j < (int)kItems; ++j) {
      lr[j] = 0u;
      if ((uint32_t)j < J) {  // (uniform)
        const bool valid = r0 + wv * kWave + (uint32_t)j * 64u + lane < m;
        const uint32_t dig = k[j] & MASK;
        uint64_t match = __ballot(valid);
        for (int b = 0; b < lb; ++b) {
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
    }
    __syncthreads();
    for (uint32_t dg = t; dg < RAD; dg += 256) {  // wave prefixes of this round
      const uint32_t c0 = wc[0][dg], c1 = wc[1][dg], c2 = wc[2][dg], c3 = wc[3][dg];
      const uint32_t at = cnt[dg] + run_[dg];
      wc[0][dg] = at;
      wc[1][dg] = at + c0;
      wc[2][dg] = at + c0 + c1;
      wc[3][dg] = at + c0 + c1 + c2;
      run_[dg] += c0 + c1 + c2 + c3;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < (int)kItems; ++j) {
      if ((uint32_t)j < J && r0 + wv * kWave + (uint32_t)j * 64u + lane < m) {
        const uint32_t o = base + wc[wv][k[j] & MASK] + lr[j];
        kout[o] = k[j];
        vout[o] = v[j];
      }
    }
    __syncthreads();
    for (uint32_t dg = t; dg < RAD; dg += 256) wc[0][dg] = wc[1][dg] = wc[2][dg] = wc[3][dg] = 0u;
    __syncthreads();
  }
#ifdef KLSH_MERGE_PROF
  if (t == 0) {
    const uint64_t x = MPROF_T();
    TPROF_ADD(3, x - tp1);
    atomicMax(&g_tprof[5], (unsigned long long)(x - tp0));
  }
#endif
  kt_end(w.kt, KC_RUNS);
}

// ------------------------------------------------------------------- runs of 65..896 rows -----
// One workgroup per run.  The run's metadata and its decision matrix live in LDS, the rows too
// when they fit (ROWS_LDS; otherwise they are read from memory, L2-resident, and staged one
// 64-row column block at a time for the decision phase).  The matrix is kept in POSITION space:
// P[y] bit q = decide(row y, row at position q), so the walk's "first j < i" is a
// find-first-set over W words, and positions that find nothing are skipped in bulk.
// ---------------------------------------------------------------- MFMA pre-screen -----
// The all-pairs decisions of a run are a Gram matrix X X^T (b x b x d).  The matrix cores compute
// it with a bf16x3 split (x = hi + lo, hi = bf16(x), lo = bf16(x - hi); G = hi.hi + hi.lo + lo.hi
// accumulated in f32), within kGramMargin * |a||b| of the reference's sequential f32 dot — so
// G / den settles every pair whose quotient is not within the margin of s*; the few that are
// take the exact sequential dot (the reference's order), so every decision is still bit-exact.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void split8(const float* p, bool ok, bf16x8& hi, bf16x8& lo) {
  float x[8];
  if (ok) {
    const float4 u = *reinterpret_cast<const float4*>(p);
    const float4 v = *reinterpret_cast<const float4*>(p + 4);
    x[0] = u.x; x[1] = u.y; x[2] = u.z; x[3] = u.w;
    x[4] = v.x; x[5] = v.y; x[6] = v.z; x[7] = v.w;
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = 0.0f;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 h = (__bf16)x[j];
    hi[j] = h;
    lo[j] = (__bf16)(x[j] - (float)h);  // x - hi is exact in f32
  }
}

// One wave: the decisions of rows [R*64, R*64+64) against rows [C*64, C*64+64) (C <= R; pairs
// c < a only), ORed into the position-space matrix P (W words per row, both P[a] bit c and
// P[c] bit a).  rowA(a) / rowB(c) give the rows (LDS or memory); D = d, a multiple of 16.
// The bf16x3 products of rows [a0, a0+64) x [c0, c0+64) over KD columns, accumulated into acc:
// rowA(a) / rowB(c) point at the columns to take (LDS or memory), KD a multiple of 16.
template <int KD, class RowA, class RowB>
__device__ __forceinline__ void gram_acc(uint32_t a0, uint32_t c0, uint32_t b, RowA rowA,
                                         RowB rowB, f32x16 (&acc)[2][2]) {
  const uint32_t lane = __lane_id(), r = lane & 31u, h = lane >> 5;
#pragma unroll
  for (int s = 0; s < KD / 16; ++s) {
    bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const uint32_t a = a0 + m * 32u + r, c = c0 + m * 32u + r;
      split8(a < b ? rowA(a) + 16 * s + 8 * h : nullptr, a < b, ah[m], al[m]);
      split8(c < b ? rowB(c) + 16 * s + 8 * h : nullptr, c < b, bh[m], bl[m]);
    }
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[m], bh[n], acc[m][n], 0, 0, 0);
        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[m], bl[n], acc[m][n], 0, 0, 0);
        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[m], bh[n], acc[m][n], 0, 0, 0);
      }
  }
}

template <int D, class RowA, class RowB>
__device__ __forceinline__ void gram_decide(uint32_t R, uint32_t C, uint32_t b,
                                            const f32x16 (&acc)[2][2], RowA rowA, RowB rowB,
                                            const float* sq, const Decider& dc, uint64_t* P,
                                            int W, uint32_t* fb);

template <int D, class RowA, class RowB>
__device__ __forceinline__ void gram_decide_slow(uint32_t R, uint32_t C, uint32_t b,
                                                 const f32x16 (&acc)[2][2], RowA rowA, RowB rowB,
                                                 const float* sq, const Decider& dc, uint64_t* P,
                                                 int W, uint32_t* fb);

// The decisions from accumulated Gram values (gram_acc) as wave masks: every compare of the
// 64 x 64 tile is one v_cmp whose lane mask IS the ballot the matrix words are assembled from, so
// the screen has no branches, no per-pair LDS reads and no per-lane bit packing.  A pair is a hit
// when G >= g_hi * den and a miss when G <= g_lo * den (den = sqrt|a|^2 * sqrt|b|^2, the
// reference's, distance.cc:37; the products' rounding is ~1e-7 of a margin of 1e-4 -- a pair it
// moves across g_hi or g_lo only changes between "settled" and "close call").  Rows past b enter
// with sq = 1 and a zero Gram row/column (gram_acc's zero fill), so they are misses; the diagonal
// tile masks c >= a.  A tile with any close call (or NaN, or a norm outside [2^-30, 2^30], where
// den may leave the screen's range) goes to gram_decide_slow, which decides it exactly as before.
// A tile without a hit writes nothing: P and fb start empty.
template <int D, class RowA, class RowB>
__device__ __forceinline__ void gram_decide(uint32_t R, uint32_t C, uint32_t b,
                                            const f32x16 (&acc)[2][2], RowA rowA, RowB rowB,
                                            const float* sq, const Decider& dc, uint64_t* P,
                                            int W, uint32_t* fb) {
  // d <= 32 (C4's 32-sample rows): tiles with a close call are common enough there that the mask
  // pass is mostly paid twice -- the lane-by-lane path alone measured C4 992-996 -> 925 ms (one box,
  // interleaved); at d = 64 the masks win (C2 214 -> 203 ms)
  if constexpr (D <= 32) {
    gram_decide_slow<D>(R, C, b, acc, rowA, rowB, sq, dc, P, W, fb);
    return;
  }
  const uint32_t lane = __lane_id(), r = lane & 31u, h = lane >> 5;
  const uint32_t a0 = R * 64u, c0 = C * 64u;
  // the norms of my two columns and of my 32 rows (loaded together: one LDS wait)
  float sc[2], sa[2][16];
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    const uint32_t c = c0 + 32u * n + r;
    sc[n] = sq[min(c, b - 1u)];
    sc[n] = c < b ? sc[n] : 1.0f;
  }
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t a = a0 + 32u * m + (i & 3) + 8u * (i >> 2) + 4u * h;
      sa[m][i] = sq[min(a, b - 1u)];
      sa[m][i] = a < b ? sa[m][i] : 1.0f;
    }
  bool bad = false;
  auto out = [](float v) { return !(v >= 0x1p-30f && v <= 0x1p30f); };
#pragma unroll
  for (int n = 0; n < 2; ++n) bad = bad || out(sc[n]);
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int i = 0; i < 16; ++i) bad = bad || out(sa[m][i]);
  const bool diag = R == C;
  uint64_t anyhit = 0ull, close = __ballot(bad);
  uint64_t own = 0ull;                       // lane L: the word of row a0 + L over the block's columns
  uint32_t tm[2][2] = {{0u, 0u}, {0u, 0u}};  // column c0 + 32n + r: bits over rows 32m + .. (h = 0)
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float thi = dc.g_hi * sa[m][i], tlo = dc.g_lo * sa[m][i];
      const uint32_t ar = (uint32_t)((i & 3) + 8 * (i >> 2));  // row within the half block (h = 0)
      uint64_t bal[2];
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const float g = acc[m][n][i];
        uint64_t H = __ballot(g >= thi * sc[n]);
        uint64_t L = __ballot(g <= tlo * sc[n]);
        if (diag) {  // pairs c < a only (uniform branch)
          const uint64_t lt = m < n ? 0ull : m > n ? ~0ull : __ballot(r < ar + 4u * h);
          H &= lt;
          L |= ~lt;
        }
        close |= ~(H | L);
        anyhit |= H;
        bal[n] = H;
        tm[n][m] |= ((H >> lane) & 1ull) ? (1u << ar) : 0u;
      }
      // rows 32m + ar (lanes h = 0) and 32m + ar + 4 (h = 1): their words over the block's columns
      const uint64_t w0 = (bal[0] & 0xFFFFFFFFull) | (bal[1] << 32);
      const uint64_t w1 = (bal[0] >> 32) | (bal[1] & 0xFFFFFFFF00000000ull);
      const int r0 = 32 * m + (int)ar;
      uint32_t olo = (uint32_t)own, ohi = (uint32_t)(own >> 32);
      olo = writelane(olo, (uint32_t)w0, r0);
      ohi = writelane(ohi, (uint32_t)(w0 >> 32), r0);
      olo = writelane(olo, (uint32_t)w1, r0 + 4);
      ohi = writelane(ohi, (uint32_t)(w1 >> 32), r0 + 4);
      own = ((uint64_t)ohi << 32) | olo;
    }
  if (close) {  // (wave-uniform) rare: the lane-by-lane path with the exact chains
    gram_decide_slow<D>(R, C, b, acc, rowA, rowB, sq, dc, P, W, fb);
    return;
  }
  if (!anyhit) return;
  if (own && a0 + lane < b) {
    atomicOr((unsigned long long*)&P[(a0 + lane) * W + C], (unsigned long long)own);
    // fb (k_merge_long): row a's first match below it, over every column block
    if (fb) atomicMin(&fb[a0 + lane], C * 64u + (uint32_t)__builtin_ctzll(own));
  }
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    // my column's bits: rows 32m + ar + 4h of the block
    const uint64_t mine = ((uint64_t)tm[n][1] << 32 | tm[n][0]) << (4u * h);
    const uint64_t full = mine | shfl64(mine, lane ^ 32u);
    const uint32_t c = c0 + 32u * n + r;
    if (h == 0 && full && c < b) atomicOr((unsigned long long*)&P[c * W + R], (unsigned long long)full);
  }
}

// One wave: the decisions of rows [R*64, R*64+64) against rows [C*64, C*64+64) (C <= R; pairs
// c < a only), ORed into the position-space matrix P (W words per row, both P[a] bit c and
// P[c] bit a).  rowA(a) / rowB(c) give the rows (LDS or memory); D = d, a multiple of 16.
template <int D, class RowA, class RowB>
__device__ __forceinline__ void gram_tile(uint32_t R, uint32_t C, uint32_t b, RowA rowA, RowB rowB,
                                          const float* sq, const Decider& dc, uint64_t* P, int W,
                                          uint32_t* fb = nullptr) {
  f32x16 acc[2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[m][n][i] = 0.0f;
  [[maybe_unused]] const uint64_t gc0 = WPROF_CLK();
  gram_acc<D>(R * 64u, C * 64u, b, rowA, rowB, acc);
#ifdef KLSH_MERGE_PROF
  asm volatile("s_nop 0" ::"v"(acc[1][1][15]) : "memory");
  if (__lane_id() == 0) GPROF_ADD(3, WPROF_CLK() - gc0);
#endif
  [[maybe_unused]] const uint64_t gc1 = WPROF_CLK();
  gram_decide<D>(R, C, b, acc, rowA, rowB, sq, dc, P, W, fb);
#ifdef KLSH_MERGE_PROF
  if (__lane_id() == 0) {
    GPROF_ADD(7, 1);
    GPROF_ADD(4, WPROF_CLK() - gc1);
  }
#endif
}

// The decisions from accumulated Gram values (gram_acc), lane by lane: pre-screen against dc's
// margin, the reference's sequential dot over D columns (rowA / rowB: whole rows) for the close
// calls.  gram_decide's path for a tile with a close call or a row of extreme norm.
template <int D, class RowA, class RowB>
__device__ __forceinline__ void gram_decide_slow(uint32_t R, uint32_t C, uint32_t b,
                                                 const f32x16 (&acc)[2][2], RowA rowA, RowB rowB,
                                                 const float* sq, const Decider& dc, uint64_t* P,
                                                 int W, uint32_t* fb) {
  const uint32_t lane = __lane_id(), r = lane & 31u, h = lane >> 5;
  const uint32_t a0 = R * 64u, c0 = C * 64u;
  [[maybe_unused]] const uint64_t gcd = WPROF_CLK();
  // decisions: acc[m][n][i] is G[a][c] with a = a0 + 32m + (i&3) + 8(i>>2) + 4h, c = c0 + 32n + r;
  // bit e = 32m + 16n + i of hitm / ambm
  uint64_t hitm = 0ull, ambm = 0ull;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const uint32_t a = a0 + 32u * m + (i & 3) + 8u * (i >> 2) + 4u * h;
        const uint32_t c = c0 + 32u * n + r;
        if (a < b && c < a) {
          const uint32_t v = prescreen(dc, acc[m][n][i], sq[a] * sq[c]);
          const int e = 32 * m + 16 * n + i;
          hitm |= (uint64_t)(v & 1u) << e;
          ambm |= (uint64_t)(v >> 1) << e;
        }
      }
#ifdef KLSH_MERGE_PROF
  asm volatile("s_nop 0" ::"v"((uint32_t)ambm) : "memory");
  [[maybe_unused]] uint64_t gc1 = WPROF_CLK();
  {
    const uint32_t na = (uint32_t)__builtin_popcountll(ambm);
    uint32_t mx = na;
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
    uint32_t sm = na;
    for (int o = 32; o > 0; o >>= 1) sm += (uint32_t)__shfl_xor((int)sm, o, 64);
    if (lane == 0) {
      GPROF_ADD(0, 1);
      GPROF_ADD(1, sm);
      GPROF_ADD(2, mx);
    }
  }
#endif
  while (ambm) {  // rare: the exact sequential dot (the reference's order) decides
    const int e = __builtin_ctzll(ambm);
    ambm &= ambm - 1ull;
    const int m = e >> 5, n = (e >> 4) & 1, i = e & 15;
    const uint32_t a = a0 + 32u * m + (i & 3) + 8u * (i >> 2) + 4u * h;
    const uint32_t c = c0 + 32u * n + r;
    const float* pa = rowA(a);
    const float* pc = rowB(c);
    float sdot = 0.0f;
    for (int k = 0; k < D; k += 4) {
      const float4 u = *reinterpret_cast<const float4*>(pa + k);
      const float4 v = *reinterpret_cast<const float4*>(pc + k);
      sdot = sdot + u.x * v.x;
      sdot = sdot + u.y * v.y;
      sdot = sdot + u.z * v.z;
      sdot = sdot + u.w * v.w;
    }
    if (decide(dc, sdot, sq[a] * sq[c])) hitm |= 1ull << e;
  }
#ifdef KLSH_MERGE_PROF
  {
    asm volatile("s_nop 0" ::"v"((uint32_t)hitm) : "memory");
    const uint64_t gc2 = WPROF_CLK();
    if (lane == 0) GPROF_ADD(5, gc2 - gc1);
    gc1 = gc2;
  }
#endif
  uint64_t tmask[2] = {0ull, 0ull};  // column c0+32n+r: bits over the 64 rows of block R
  uint64_t own = 0ull;                // lane L ends up with the word of row a0 + L
#pragma unroll
  for (int m = 0; m < 2; ++m) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t ar = 32u * m + (i & 3) + 8u * (i >> 2) + 4u * h;  // row within the block
      uint64_t bal[2];
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const bool hit = (hitm >> (32 * m + 16 * n + i)) & 1ull;
        tmask[n] |= (hit ? 1ull : 0ull) << ar;
        bal[n] = __ballot(hit);
      }
      // rows r0 (lanes with h = 0) and r0 + 4 (h = 1): their 64-bit words over the block's columns
      const uint32_t r0 = 32u * m + (i & 3) + 8u * (i >> 2);
      const uint64_t w0 = (bal[0] & 0xFFFFFFFFull) | (bal[1] << 32);
      const uint64_t w1 = (bal[0] >> 32) | (bal[1] & 0xFFFFFFFF00000000ull);
      if (lane == r0) own = w0;
      if (lane == r0 + 4u) own = w1;
    }
  }
  if (own && a0 + lane < b) {
    atomicOr((unsigned long long*)&P[(a0 + lane) * W + C], (unsigned long long)own);
    // fb (k_merge_long): row a's first match below it, over every column block
    if (fb) atomicMin(&fb[a0 + lane], C * 64u + (uint32_t)__builtin_ctzll(own));
  }
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    const uint64_t full = tmask[n] | shfl64(tmask[n], lane ^ 32u);
    const uint32_t c = c0 + 32u * n + r;
    if (h == 0 && full && c < b) atomicOr((unsigned long long*)&P[c * W + R], (unsigned long long)full);
  }
}

// s + sequential sum of a[e] * b[e], e < n, a and b in memory (16-B aligned rows)
__device__ __forceinline__ float dot_acc_mem(float s, const float* a, const float* b, int n) {
  int k = 0;
  for (; k + 4 <= n; k += 4) {
    const float4 u = *reinterpret_cast<const float4*>(a + k);
    const float4 v = *reinterpret_cast<const float4*>(b + k);
    s = s + u.x * v.x;
    s = s + u.y * v.y;
    s = s + u.z * v.z;
    s = s + u.w * v.w;
  }
  for (; k < n; ++k) s = s + a[k] * b[k];
  return s;
}

// The same sequential sum for a compile-time width D (a multiple of 4; D == 0: runtime d): every
// load is issued before the chain starts, so the chain does not wait on a load every 4 terms.
template <int D>
__device__ __forceinline__ float dot_seq(const float* a, const float* b, int d) {
  if constexpr (D == 0) {
    return dot_acc_mem(0.0f, a, b, d);
  } else {
    float4 u[D / 4], v[D / 4];
#pragma unroll
    for (int k = 0; k < D / 4; ++k) {
      u[k] = *reinterpret_cast<const float4*>(a + 4 * k);
      v[k] = *reinterpret_cast<const float4*>(b + 4 * k);
    }
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < D / 4; ++k) {
      s = s + u[k].x * v[k].x;
      s = s + u[k].y * v[k].y;
      s = s + u[k].z * v[k].z;
      s = s + u[k].w * v[k].w;
    }
    return s;
  }
}

// The walk of one 65..896-row run over its position-space decision matrix P (k_merge_big*),
// shared by the whole workgroup: every step finds the first position q >= i whose row matches a
// position below q (positions that find nothing change nothing), does the reference's merge
// there, and recomputes the decisions of the rows still to be visited against the new row —
// spread over all NT lanes (the new row's norm on one lane meanwhile).  Rows are read from
// rowsL (LDS, stride ST) if given, else from memory; the new row is kept in LDS (cbuf).
template <int RB, int NT, bool ROWS_LDS, int D = 0>
__device__ __forceinline__ void big_walk(uint32_t p, uint32_t b, uint64_t* P, uint32_t* slot,
                                         float* nrm, uint32_t* cnt, uint32_t* hd, uint32_t* tl,
                                         uint32_t* pos2row, float* sq, float* rowsL, int ST,
                                         float* cbuf, uint32_t* wbuf, const Rows& r,
                                         const Decider& dc, uint32_t* slots, uint32_t* dlist,
                                         Counters* ctr) {
  constexpr int W = RB / 64, NW = NT / 64, KP = (RB + NT - 1) / NT;
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const int d = r.d, dp = r.dp;
  auto rowp = [&](uint32_t a) -> const float* {
    return ROWS_LDS ? rowsL + a * ST : r.x + (size_t)slot[a] * dp;
  };
  uint32_t i = 1, size = b, par = 0;
  [[maybe_unused]] uint64_t wp[6] = {0, 0, 0, 0, 0, 0}, c0 = 0, c1 = 0;
  while (true) {
    // 1. the next position that merges
    c0 = WPROF_CLK();
    uint32_t q = size;
    for (uint32_t q0 = i; q0 < size; q0 += NT) {
      ++wp[5];
      const uint32_t qq = q0 + t;
      bool hit = false;
      if (qq < size) {
        const uint64_t* Py = P + pos2row[qq] * W;
#pragma unroll
        for (int k = 0; k < W; ++k) {
          const uint32_t lo = (uint32_t)k * 64u;
          if (lo < qq) {
            const uint64_t wk = Py[k];
            hit |= (qq - lo >= 64u ? wk : (wk & ((1ull << (qq - lo)) - 1ull))) != 0ull;
          }
        }
      }
      const uint64_t m = __ballot(hit);
      if (lane == 0)
        wbuf[par * NW + wv] = m ? q0 + wv * 64u + (uint32_t)(__ffsll((unsigned long long)m) - 1)
                                : 0xFFFFFFFFu;
      lds_barrier();
      uint32_t best = 0xFFFFFFFFu;
#pragma unroll
      for (int w = 0; w < NW; ++w) best = min(best, wbuf[par * NW + w]);
      par ^= 1u;
      if (best != 0xFFFFFFFFu) {  // block-uniform
        q = best;
        break;
      }
    }
    c1 = WPROF_CLK();
    wp[0] += c1 - c0;
    c0 = c1;
    if (q >= size) break;
    ++wp[4];
    i = q;
    // 2. its first matching position j < i (every wave computes it)
    const uint32_t rr = pos2row[i];
    uint64_t word = 0ull;
    if (lane < (uint32_t)W) {
      word = P[rr * W + lane];
      const uint32_t lo = lane * 64u;
      if (lo >= i) word = 0ull;
      else if (i - lo < 64u) word &= (1ull << (i - lo)) - 1ull;
    }
    const uint64_t nz = __ballot(word != 0ull);
    const uint32_t wd = (uint32_t)(__ffsll((unsigned long long)nz) - 1);
    const uint64_t wbits = shfl64(word, wd);
    const uint32_t j = wd * 64u + (uint32_t)(__ffsll((unsigned long long)wbits) - 1);
    const uint32_t c = pos2row[j];
    const uint32_t ca = cnt[rr], cb = cnt[c];
    const uint32_t hr = hd[rr], tr = tl[rr], hc = hd[c];
    const uint32_t moved_row = pos2row[size - 1];
    lds_barrier();  // all reads of the old state are done
    // 3. consensus (funcAB.cc:65), current row first; member links and the swap-remove
    const float fa = (float)(int)ca, fb = (float)(int)cb, fn = (float)(int)(ca + cb);
    float* xc = r.x + (size_t)slot[c] * dp;
    const float* xr = rowp(rr);
    float* lc = ROWS_LDS ? rowsL + c * ST : cbuf;  // the new row c, in LDS
    for (int k = (int)t; k < d; k += NT) {
      const float v = consensus(xr[k], fa, ROWS_LDS ? lc[k] : xc[k], fb, fn);
      lc[k] = v;
      if (!ROWS_LDS) store_row1(r, (size_t)slot[c] * dp + k, v);  // LDS rows go out at the end
    }
    if (t == 0) {
      r.nxt[tr] = hc;  // ids_current ++ ids_candidate (funcAB.cc:51-55)
      hd[c] = hr;
      cnt[c] = ca + cb;
      cnt[rr] = 0u;
      pos2row[i] = moved_row;
    }
    if (ROWS_LDS) lds_barrier();
    else __syncthreads();  // the new row in memory is visible to the workgroup
    --size;
    const uint32_t moved = size;  // old position of the row now at i
    c1 = WPROF_CLK();
    wp[1] += c1 - c0;
    c0 = c1;
    // 4. dot products of the rows still to be visited with row c; row c's norm
    float dots[KP];
#pragma unroll
    for (int kp = 0; kp < KP; ++kp) {
      const uint32_t qq = i + t + (uint32_t)kp * NT;
      dots[kp] = qq < size ? dot_seq<D>(rowp(pos2row[qq]), lc, d) : 0.0f;
    }
    if (t == NT - 1) {
      const float nn = dot_seq<D>(lc, lc, d);  // distance.cc:33-34
      nrm[c] = nn;
      sq[c] = __builtin_sqrtf(nn);
    }
    lds_barrier();
    c1 = WPROF_CLK();
    wp[2] += c1 - c0;
    c0 = c1;
    // 5. position-space bits: the moved row's bit goes to position i, bit j is re-decided
    const float sc = sq[c];
#pragma unroll
    for (int kp = 0; kp < KP; ++kp) {
      const uint32_t qq = i + t + (uint32_t)kp * NT;
      if (qq < size) {
        const uint32_t y = pos2row[qq];
        uint64_t* Py = P + y * W;
        const bool bm = (Py[moved / 64] >> (moved & 63u)) & 1ull;
        Py[moved / 64] &= ~(1ull << (moved & 63u));
        Py[i / 64] = bm ? (Py[i / 64] | (1ull << (i & 63u))) : (Py[i / 64] & ~(1ull << (i & 63u)));
        const bool dn = decide(dc, dots[kp], sq[y] * sc);
        Py[j / 64] = dn ? (Py[j / 64] | (1ull << (j & 63u))) : (Py[j / 64] & ~(1ull << (j & 63u)));
      }
    }
    lds_barrier();
    c1 = WPROF_CLK();
    wp[3] += c1 - c0;
  }
#ifdef KLSH_MERGE_PROF
  if (t == 0) {
    const int cls = RB <= 128 ? 0 : RB <= 384 ? 1 : 2;
    for (int k = 0; k < 6; ++k) atomicAdd(&g_wprof[cls][k], (unsigned long long)wp[k]);
  }
#endif
  // write back: survivors in position order, kInvalid after; rewritten rows; metadata
  for (uint32_t q = t; q < b; q += NT) slots[p + q] = q < size ? slot[pos2row[q]] : kInvalid;
  if (ROWS_LDS) {  // a survivor was rewritten iff its count rose (the global count is still old)
    const uint32_t c4 = (uint32_t)dp / 4;
    for (uint32_t idx = t; idx < size * c4; idx += NT) {
      const uint32_t q = idx / c4, k = (idx % c4) * 4;
      const uint32_t y = pos2row[q];
      if (r.cnt[slot[y]] != cnt[y])
        store_row4(r, (size_t)slot[y] * dp + k, *reinterpret_cast<const float4*>(rowsL + y * ST + k));
    }
    __syncthreads();
  }
  for (uint32_t q0 = 0; q0 < size; q0 += NT) {  // uniform trip count (ballot inside)
    const uint32_t q = q0 + t;
    bool rewritten = false;
    if (q < size) {
      const uint32_t y = pos2row[q];
      rewritten = r.cnt[slot[y]] != cnt[y];  // every merge into a row raises its count
      r.nrm[slot[y]] = nrm[y];
      r.cnt[slot[y]] = cnt[y];
      r.head[slot[y]] = hd[y];
    }
    if (dlist) append_slot(rewritten, q < size ? slot[pos2row[q]] : 0u, dlist, &ctr->n_delta);
  }
}

// The same walk for runs whose rows sit in LDS at a register width (D = 8..64), built around ONE
// workgroup barrier per merge step (big_walk needs four):
//  * positions are owned statically — lane t holds positions t, t + NT, ... — with their rows in
//    registers (a row at a position >= i never changes; only the row moved into position i by the
//    swap-remove is reloaded, by its one owner);
//  * the owner of a position updates its P row after a merge and tests it at once, so the next
//    merge (its position, first matching position j, and both row ids) is a wave ballot + one
//    64-bit word per wave in LDS, read by every wave after the barrier;
//  * every wave computes the merge itself (consensus into a wave-private copy of the new row, the
//    member links by one lane) and applies the step's writes to the shared state (pos2row, counts,
//    list heads, the new row) at the START of the next step: every wave writes the same values,
//    each before its own reads, so no wave can see a half-written step and no second barrier is
//    needed;
//  * the decisions against the new row come from short chains (four interleaved partial sums of
//    its norm and of each dot product, |error| <= 2 * 64 * 2^-24 |a||b| each — far inside
//    kGramMargin), settled by the same certified pre-screen as the Gram tiles; only pairs within
//    the margin of the threshold run the reference's sequential chains.  The new row's exact norm
//    (distance.cc:33-34) is needed by nobody during the walk — rows at positions below i are never
//    tested again — so it is computed once per rewritten row at the write-back.
template <int RB, int NT, int D>
__device__ __forceinline__ void big_walk_reg(uint32_t p, uint32_t b, uint64_t* P, uint32_t* slot,
                                             float* nrm, uint32_t* cnt, const uint32_t* cnt0,
                                             uint32_t* hd, uint32_t* tl,
                                             uint32_t* pos2row, float* sq, float* rowsL,
                                             float* cwall, uint64_t* wbuf, const Rows& r,
                                             const Decider& dc, uint32_t* slots, uint32_t* dlist,
                                             Counters* ctr) {
  constexpr int W = RB / 64, NW = NT / 64, KP = (RB + NT - 1) / NT, ST = D + 4;
  constexpr uint32_t kNone = 0xFFFFFFFFu;
  constexpr uint64_t kNone64 = ~0ull;
  static_assert(RB <= 1024, "positions are packed in 10 bits");
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  float* cw = cwall + wv * 64;  // this wave's copy of the newest row
  float xr[KP][D];              // the rows at my positions t + kp * NT
  uint32_t yr[KP];              // their row ids
  float sqy[KP];                // their sqrtf(norm)
#pragma unroll
  for (int kp = 0; kp < KP; ++kp) {
    const uint32_t q = t + (uint32_t)kp * NT;
    yr[kp] = q;
    sqy[kp] = 0.0f;
    if (q < b) {
      load_row<D>(rowsL + q * ST, xr[kp]);
      sqy[kp] = sq[q];
    }
  }
  // the first position below q that row y (words w) matches, or kNone
  auto first_below = [&](const uint64_t (&w)[W], uint32_t q) -> uint32_t {
#pragma unroll
    for (int k = 0; k < W; ++k) {
      const uint32_t lo = (uint32_t)k * 64u;
      if (lo < q) {
        uint64_t m = w[k];
        if (q - lo < 64u) m &= (1ull << (q - lo)) - 1ull;
        if (m) return lo + (uint32_t)__builtin_ctzll(m);
      }
    }
    return kNone;
  };
  // a hit: (position << 20 | its first match << 10 | its row) << 32 | the matching row
  auto pack = [](uint32_t q, uint32_t j, uint32_t y, uint32_t c) -> uint64_t {
    return ((uint64_t)((q << 20) | (j << 10) | y) << 32) | c;
  };
  // the wave's first hit (lowest position: kp-major, then lane order) -> wbuf[par][wv]
  auto publish = [&](uint32_t par, const uint64_t (&hit)[KP]) {
    uint64_t best = kNone64;
#pragma unroll
    for (int kp = 0; kp < KP; ++kp) {
      const uint64_t m = __ballot(hit[kp] != kNone64);
      if (m && best == kNone64) best = shfl64(hit[kp], (uint32_t)__builtin_ctzll(m));
    }
    if (lane == 0) wbuf[par * NW + wv] = best;
  };
  uint32_t size = b, par = 0;
  [[maybe_unused]] const uint64_t wt0 = MPROF_T();
  {
    uint64_t hit[KP];
#pragma unroll
    for (int kp = 0; kp < KP; ++kp) {
      const uint32_t q = t + (uint32_t)kp * NT;
      hit[kp] = kNone64;
      if (q >= 1 && q < b) {
        uint64_t w[W];
#pragma unroll
        for (int k = 0; k < W; ++k) w[k] = P[q * W + k];
        const uint32_t j = first_below(w, q);
        if (j != kNone) hit[kp] = pack(q, j, q, j);  // positions are the rows before any merge
      }
    }
    publish(par, hit);
  }
  lds_barrier();
  // the previous step's writes, applied by every wave at the start of the next step
  bool have = false;
  uint32_t ip = 0, mp = 0, cp = 0, rp = 0, cntp = 0, hdp = 0;
  float cvp = 0.0f;
  [[maybe_unused]] uint64_t steps = 0, wp[6] = {0, 0, 0, 0, 0, 0}, ck = WPROF_CLK(), ck1 = 0;
  while (true) {
    uint64_t best = kNone64;
#pragma unroll
    for (int w = 0; w < NW; ++w) best = min(best, wbuf[par * NW + w]);
    par ^= 1u;
    if (have) {
      if (lane == 0) {
        pos2row[ip] = mp;
        cnt[cp] = cntp;
        cnt[rp] = 0u;
        hd[cp] = hdp;
      }
      if (lane < (uint32_t)D) rowsL[cp * ST + lane] = cvp;
      wave_lds_fence();
    }
    if (best == kNone64) break;
    ++steps;
    const uint32_t hi = (uint32_t)(best >> 32);
    const uint32_t i = hi >> 20, j = (hi >> 10) & 1023u, rr = hi & 1023u, c = (uint32_t)best;
    const uint32_t moved = pos2row[size - 1];
    const uint32_t ca = cnt[rr], cb = cnt[c], hr = hd[rr], tr = tl[rr], hc = hd[c];
#ifdef KLSH_MERGE_PROF
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    ck1 = WPROF_CLK(); wp[0] += ck1 - ck; ck = ck1;
#endif
    // consensus (funcAB.cc:65), current row first, into this wave's copy of the new row c
    const float fa = (float)(int)ca, fb = (float)(int)cb, fn = (float)(int)(ca + cb);
    float cv = 0.0f;
    if (lane < (uint32_t)D) {
      cv = consensus(rowsL[rr * ST + lane], fa, rowsL[c * ST + lane], fb, fn);
      cw[lane] = cv;
    }
    if (t == 0) r.nxt[tr] = hc;  // ids_current ++ ids_candidate (funcAB.cc:51-55)
    wave_lds_fence();
    --size;  // swap-remove: the row at the old last position (size) moves to position i
#pragma unroll
    for (int kp = 0; kp < KP; ++kp) {
      if (t + (uint32_t)kp * NT == i && i < size) {
        yr[kp] = moved;
        load_row<D>(rowsL + moved * ST, xr[kp]);
        sqy[kp] = sq[moved];
      }
    }
    float cvec[D];
    load_row<D>(cw, cvec);
#ifdef KLSH_MERGE_PROF
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    ck1 = WPROF_CLK(); wp[1] += ck1 - ck; ck = ck1;
#endif
    // short chains: four interleaved partial sums (a screen, not the reference's order)
    float n4[4] = {0.0f, 0.0f, 0.0f, 0.0f}, d4[KP][4];
#pragma unroll
    for (int kp = 0; kp < KP; ++kp) d4[kp][0] = d4[kp][1] = d4[kp][2] = d4[kp][3] = 0.0f;
#pragma unroll
    for (int k = 0; k < D; ++k) {
      n4[k & 3] = n4[k & 3] + cvec[k] * cvec[k];
#pragma unroll
      for (int kp = 0; kp < KP; ++kp) d4[kp][k & 3] = d4[kp][k & 3] + xr[kp][k] * cvec[k];
    }
    const float sc_a = __builtin_sqrtf((n4[0] + n4[1]) + (n4[2] + n4[3]));
    uint32_t dn[KP];
    bool amb = false;
#pragma unroll
    for (int kp = 0; kp < KP; ++kp) {
      const uint32_t q = t + (uint32_t)kp * NT;
      dn[kp] = 0u;
      if (q >= i && q < size) {
        const float dot_a = (d4[kp][0] + d4[kp][1]) + (d4[kp][2] + d4[kp][3]);
        dn[kp] = dc.fast ? prescreen(dc, dot_a, sqy[kp] * sc_a) : 2u;
        amb = amb || dn[kp] == 2u;
      }
    }
    if (__ballot(amb)) {  // rare: the reference's sequential chains settle the close calls
      float nn = 0.0f;
#pragma unroll
      for (int k = 0; k < D; ++k) nn = nn + cvec[k] * cvec[k];
      const float sc = __builtin_sqrtf(nn);
#pragma unroll
      for (int kp = 0; kp < KP; ++kp) {
        if (dn[kp] == 2u) {
          float dot = 0.0f;
#pragma unroll
          for (int k = 0; k < D; ++k) dot = dot + xr[kp][k] * cvec[k];
          dn[kp] = decide(dc, dot, sqy[kp] * sc) ? 1u : 0u;
        }
      }
    }
#ifdef KLSH_MERGE_PROF
    asm volatile("s_nop 0" ::"v"(dn[0]) : "memory");
    ck1 = WPROF_CLK(); wp[2] += ck1 - ck; ck = ck1;
#endif
    uint64_t hit[KP];
#pragma unroll
    for (int kp = 0; kp < KP; ++kp) {
      const uint32_t q = t + (uint32_t)kp * NT;
      hit[kp] = kNone64;
      if (q >= i && q < size) {
        const uint32_t y = yr[kp];
        uint64_t w[W];
#pragma unroll
        for (int k = 0; k < W; ++k) w[k] = P[y * W + k];
        // position-space bits: the moved row's bit goes to position i, bit j is re-decided
        const bool bm = (w[size >> 6] >> (size & 63u)) & 1ull;
#pragma unroll
        for (int k = 0; k < W; ++k) {
          uint64_t v = w[k];
          if ((uint32_t)k == (size >> 6)) v &= ~(1ull << (size & 63u));
          if ((uint32_t)k == (i >> 6)) v = bm ? (v | (1ull << (i & 63u))) : (v & ~(1ull << (i & 63u)));
          if ((uint32_t)k == (j >> 6))
            v = dn[kp] ? (v | (1ull << (j & 63u))) : (v & ~(1ull << (j & 63u)));
          if (v != w[k]) P[y * W + k] = v;
          w[k] = v;
        }
        const uint32_t jj = first_below(w, q);
        // the row at position jj as of this step (position i now holds the moved row)
        if (jj != kNone) hit[kp] = pack(q, jj, y, jj == i ? moved : pos2row[jj]);
      }
    }
    publish(par, hit);
    have = true;
    ip = i;
    mp = moved;
    cp = c;
    rp = rr;
    cntp = ca + cb;
    hdp = hr;
    cvp = cv;
#ifdef KLSH_MERGE_PROF
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    ck1 = WPROF_CLK(); wp[3] += ck1 - ck; ck = ck1;
#endif
    lds_barrier();
#ifdef KLSH_MERGE_PROF
    ck1 = WPROF_CLK(); wp[5] += ck1 - ck; ck = ck1;
#endif
  }
#ifdef KLSH_MERGE_PROF
  if (t == 0) {
    const int cls = RB <= 128 ? 0 : RB <= 192 ? 1 : 2;
    atomicAdd(&g_wprof[cls][4], (unsigned long long)steps);
    for (int k = 0; k < 4; ++k) atomicAdd(&g_wprof[cls][k], (unsigned long long)wp[k]);
    atomicAdd(&g_wprof[cls][5], (unsigned long long)wp[5]);
    MPROF_ADD(RB <= 128 ? 0 : RB <= 192 ? 1 : RB <= 384 ? 2 : 3, 10, MPROF_T() - wt0);
  }
#endif
  __syncthreads();
  if (size == b) return;  // (block-uniform) no merge: the run, its rows and metadata are as loaded
  // write back: survivors in position order, kInvalid after; rewritten rows; metadata
  for (uint32_t q = t; q < b; q += NT) slots[p + q] = q < size ? slot[pos2row[q]] : kInvalid;
  {  // a survivor was rewritten iff its count rose
    constexpr uint32_t c4 = (uint32_t)D / 4;
    for (uint32_t idx = t; idx < size * c4; idx += NT) {
      const uint32_t q = idx / c4, k = (idx % c4) * 4;
      const uint32_t y = pos2row[q];
      if (cnt0[y] != cnt[y])
        store_row4(r, (size_t)slot[y] * r.dp + k, *reinterpret_cast<const float4*>(rowsL + y * ST + k));
    }
  }
  for (uint32_t q0 = 0; q0 < size; q0 += NT) {  // uniform trip count (ballot inside)
    const uint32_t q = q0 + t;
    bool rewritten = false;
    if (q < size) {
      const uint32_t y = pos2row[q];
      // every merge into a row raises its count, and a row's head changes only through a merge
      // into it (SetConsensus, funcAB.cc:49-71: ids = ids_cur ++ ids_cand, so the candidate's
      // slot takes the merged-away row's head and the sum of both counts); swap-remove moves a
      // row's position, never its slot's data.  So "count unchanged" implies "head, norm and row
      // unchanged" and those slots need no write-back.
      rewritten = cnt0[y] != cnt[y];
      if (rewritten) {  // the exact sequential norm of the new row (distance.cc:33-34)
        float nv = 0.0f;
#pragma unroll
        for (int k = 0; k < D; ++k) nv = nv + rowsL[y * ST + k] * rowsL[y * ST + k];
        r.nrm[slot[y]] = nv;
        r.cnt[slot[y]] = cnt[y];
        r.head[slot[y]] = hd[y];
      }
    }
    if (dlist) append_slot(rewritten, q < size ? slot[pos2row[q]] : 0u, dlist, &ctr->n_delta);
  }
}

template <int D, int RB, bool ROWS_LDS>
struct BigLayout {
  static constexpr int ST = D + 4;
  static constexpr int W = RB / 64;
  static constexpr size_t rows = 0;
  static constexpr size_t P = rows + sizeof(float) * ST * (ROWS_LDS ? RB : 64);
  static constexpr size_t meta = P + sizeof(uint64_t) * RB * W;
  static constexpr size_t bytes = meta + sizeof(uint32_t) * RB * 8;
};

// The fp16 screen of one big run (k_merge_tail, option tail_big_screen): k_small_screen's certified
// test (screen_margins) over every pair of the run's image rows, 32 x 32 blocks on
// v_mfma_f32_32x32x16_f16.  Returns whether the run can merge at all (some pair not ruled out, or a
// row whose image has no usable norm); false: the walk would change nothing — no f32 row is read.
// slot[0, b): the run's slots (LDS); hrows: room for b x (D + 8) halves; linv: b floats.
template <int D, int NT>
__device__ __forceinline__ bool big_screen_pass(uint32_t b, const uint32_t* slot, const Rows& r,
                                                float s_star, float m0, float a2,
                                                _Float16* hrows, float* linv, uint32_t* flag) {
  constexpr int STH = D + 8, LPR = D / 8, NW = NT / 64;  // a lane loads 16 B = 8 halves
  constexpr uint32_t RPR = NT / LPR;                      // rows per round
  constexpr int KB = 4;
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  if (t == 0) *flag = 0u;
  {
    const uint32_t sub = (t % LPR) * 8u, rr = t / LPR;
    const uint32_t rounds = (b + RPR - 1u) / RPR;
    for (uint32_t g0 = 0; g0 < rounds; g0 += KB) {  // block-uniform
      sh16x8 v[KB];
#pragma unroll
      for (int k = 0; k < KB; ++k) {
        const uint32_t a = min((g0 + (uint32_t)k) * RPR + rr, b - 1u);
        v[k] = *reinterpret_cast<const sh16x8*>(r.xh + (size_t)slot[a] * r.dp + sub);
      }
#pragma unroll
      for (int k = 0; k < KB; ++k) {  // (unconditional at the clamped index, as in big_runs)
        const uint32_t a = min((g0 + (uint32_t)k) * RPR + rr, b - 1u);
        *reinterpret_cast<sh16x8*>(hrows + a * STH + sub) = v[k];
      }
    }
  }
  lds_barrier();
  bool bad = false;
  for (uint32_t a = t; a < b; a += NT) {  // |x~|, as k_small_screen computes it
    float ss = 0.0f;
#pragma unroll
    for (int q = 0; q < D / 8; ++q) {
      const sh16x8 x = *reinterpret_cast<const sh16x8*>(hrows + a * STH + 8 * q);
#pragma unroll
      for (int h2 = 0; h2 < 8; h2 += 2) {
        const sh16x2 v = {x[h2], x[h2 + 1]};
        ss = __builtin_amdgcn_fdot2(v, v, ss, false);
      }
    }
    const bool bd = !(ss >= 0x1p-100f && ss <= 0x1p100f);
    bad = bad || bd;
    linv[a] = bd ? 0.0f : 1.0f / __builtin_sqrtf(ss);
  }
  if (bad) *flag = 1u;
  lds_barrier();
  if (*flag) return true;  // (block-uniform) a row the image cannot carry: the exact merge
  const uint32_t nb = (b + 31u) / 32u, r32 = lane & 31u, k8 = 8u * (lane >> 5);
  const uint32_t ntiles = nb * (nb + 1u) / 2u;
  bool fail = false;
  for (uint32_t ti = wv; ti < ntiles; ti += NW) {  // wave-uniform: blocks tr <= tc
    uint32_t tc = (uint32_t)((__builtin_sqrtf(8.0f * (float)ti + 1.0f) - 1.0f) * 0.5f);
    while (tc * (tc + 1u) / 2u > ti) --tc;
    while ((tc + 1u) * (tc + 2u) / 2u <= ti) ++tc;
    const uint32_t tr = ti - tc * (tc + 1u) / 2u;
    pf16acc acc;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.0f;
    const uint32_t ra = min(tr * 32u + r32, b - 1u), ca = min(tc * 32u + r32, b - 1u);
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) {
      const sh16x8 fa = *reinterpret_cast<const sh16x8*>(hrows + ra * STH + 16 * ks + k8);
      const sh16x8 fb = *reinterpret_cast<const sh16x8*>(hrows + ca * STH + 16 * ks + k8);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa, fb, acc, 0, 0, 0);
    }
    const uint32_t C = tc * 32u + r32;
    const float ic = linv[ca];
    float4 irv[4];  // rows tr*32 + 8j + 4h + (0..3)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      irv[j] = *reinterpret_cast<const float4*>(linv + min(tr * 32u + 8u * (uint32_t)j + 4u * (lane >> 5), (b - 1u) & ~3u));
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const uint32_t R = tr * 32u + (uint32_t)(q & 3) + 8u * (uint32_t)(q >> 2) + 4u * (lane >> 5);
      const float4 v = irv[q >> 2];
      const float ir = (q & 3) == 0 ? v.x : (q & 3) == 1 ? v.y : (q & 3) == 2 ? v.z : v.w;
      const float qv = acc[q] * ir * ic;
      const float m = m0 + a2 * (ir + ic);
      fail = fail | ((R < C) & (C < b) & !(qv < s_star - m));  // NaN / inf: not ruled out
    }
  }
  if (fail) *flag = 1u;
  lds_barrier();
  return *flag != 0u;
}

struct BigScreen {
  uint32_t on;
  float s_star, m0, a2;
};

// The runs li = first, first + stride, ... (< count) of list `list` (size class cls), one
// workgroup of NT lanes per run, with smem = BigLayout<D, RB, ROWS_LDS>::bytes of LDS.
// bs.on (k_merge_tail, d = 32 / 64 with the fp16 image): each run is screened first
// (big_screen_pass) and left alone when no pair of it can merge.
template <int D, int RB, int NT, bool ROWS_LDS>
__device__ __forceinline__ void big_runs(const uint2* __restrict__ list, int cls, uint32_t count,
                                         uint32_t first, uint32_t stride,
                                         uint32_t* __restrict__ slots, const Decider& dc,
                                         const Rows& r, Counters* ctr, uint32_t* dlist,
                                         unsigned char* smem, BigScreen bs = BigScreen{0u, 0.0f, 0.0f, 0.0f}) {
  using L = BigLayout<D, RB, ROWS_LDS>;
  constexpr int ST = L::ST, W = L::W, NW = NT / 64;
  float* rows = reinterpret_cast<float*>(smem + L::rows);  // rows, or one staged column block
  uint64_t* P = reinterpret_cast<uint64_t*>(smem + L::P);  // [row][W] position-space masks
  uint32_t* slot = reinterpret_cast<uint32_t*>(smem + L::meta);
  float* nrm = reinterpret_cast<float*>(slot + RB);
  uint32_t* cnt = slot + 2 * RB;
  uint32_t* hd = slot + 3 * RB;
  uint32_t* tl = slot + 4 * RB;
  uint32_t* pos2row = slot + 5 * RB;
  float* sq = reinterpret_cast<float*>(slot + 6 * RB);  // sqrtf(nrm), distance.cc:37
  uint32_t* cnt0 = slot + 7 * RB;                       // the counts as loaded (rewritten rows)
  __shared__ uint32_t wbuf[2 * NW];
  __shared__ __attribute__((aligned(16))) float cwall[NW * 64];  // big_walk_reg's new-row copies
  __shared__ uint64_t wbuf64[2 * NW];                              // big_walk_reg's published hits
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  auto row_ptr = [&](uint32_t a) -> const float* {
    return ROWS_LDS ? rows + a * ST : r.x + (size_t)slot[a] * r.dp;
  };

  for (uint32_t li = first; li < count; li += stride) {
    const uint2 e = list[li];
    const uint32_t p = e.x, b = e.y;
    const uint32_t nblk = (b + 63) / 64;
    [[maybe_unused]] const uint64_t pt0 = MPROF_T();
    if constexpr (!ROWS_LDS) {
      for (uint32_t a = t; a < b; a += NT) {
        const uint32_t s = slots[p + a];
        slot[a] = s;
        nrm[a] = r.nrm[s];
        sq[a] = __builtin_sqrtf(nrm[a]);
        cnt[a] = cnt0[a] = r.cnt[s];
        hd[a] = r.head[s];
        tl[a] = r.tail[s];
        pos2row[a] = a;
      }
    }
    for (uint32_t a = t; a < b * (uint32_t)W; a += NT) P[a] = 0ull;
    if constexpr (ROWS_LDS) {
      // Three memory latencies, every load of a round in flight at once (loads under a bounds
      // branch would each be waited for on the spot): the run's slots; then the metadata and
      // the rows by slot, d/4 lanes per row, a float4 each, KB rows per lane per round.
      constexpr int KA = (RB + NT - 1) / NT;
      uint32_t sl[KA], mc[KA], mh[KA], mt[KA];
#pragma unroll
      for (int ka = 0; ka < KA; ++ka) sl[ka] = slots[p + min(t + (uint32_t)ka * NT, b - 1u)];
      if constexpr (D == 32 || D == 64) {
        if (bs.on) {  // (uniform) the fp16 screen first: a run that cannot merge is left as it is
          __shared__ uint32_t sflag;
#pragma unroll
          for (int ka = 0; ka < KA; ++ka) {
            const uint32_t a = t + (uint32_t)ka * NT;
            if (a < b) slot[a] = sl[ka];
          }
          lds_barrier();
          if (!big_screen_pass<D, NT>(b, slot, r, bs.s_star, bs.m0, bs.a2,
                                      reinterpret_cast<_Float16*>(rows), sq, &sflag)) {
            __syncthreads();
            continue;
          }
        }
      }
#pragma unroll
      for (int ka = 0; ka < KA; ++ka) {
        mc[ka] = r.cnt[sl[ka]];
        mh[ka] = r.head[sl[ka]];
        mt[ka] = r.tail[sl[ka]];
      }
#pragma unroll
      for (int ka = 0; ka < KA; ++ka) {
        const uint32_t a = t + (uint32_t)ka * NT;
        if (a < b) {
          slot[a] = sl[ka];
          pos2row[a] = a;
        }
      }
      lds_barrier();  // slot[] (the metadata loads stay in flight)
      constexpr uint32_t LPR = (uint32_t)D / 4;  // lanes per row: a float4 each
      constexpr uint32_t RPR = NT / LPR;         // rows per workgroup round
      constexpr int KB = D >= 64 ? 8 : D >= 32 ? 4 : 2;
      static_assert(D % 4 == 0 && NT % LPR == 0, "whole rows per round");
      const uint32_t sub = (t % LPR) * 4u, rr = t / LPR;
      const uint32_t rounds = (b + RPR - 1u) / RPR;
      for (uint32_t g0 = 0; g0 < rounds; g0 += KB) {  // block-uniform
        float4 v[KB];
#pragma unroll
        for (int k = 0; k < KB; ++k) {
          const uint32_t a = min((g0 + (uint32_t)k) * RPR + rr, b - 1u);
          v[k] = *reinterpret_cast<const float4*>(r.x + (size_t)slot[a] * r.dp + sub);
        }
        // (stores unconditional at the clamped index — a row past b rewrites row b - 1 with its own
        // value: a store under `a < b` lets the compiler sink its load into the branch, and the KB
        // loads become KB round trips.  A scheduling barrier between the two loops, to keep
        // k_merge_tail's register-tight schedule from pairing the rest, spilled: not used)
#pragma unroll
        for (int k = 0; k < KB; ++k) {
          const uint32_t a = min((g0 + (uint32_t)k) * RPR + rr, b - 1u);
          *reinterpret_cast<float4*>(rows + a * ST + sub) = v[k];
        }
      }
#pragma unroll
      for (int ka = 0; ka < KA; ++ka) {
        const uint32_t a = t + (uint32_t)ka * NT;
        if (a < b) {
          cnt[a] = cnt0[a] = mc[ka];
          hd[a] = mh[ka];
          tl[a] = mt[ka];
        }
      }
      lds_barrier();
#ifdef KLSH_MERGE_PROF
      if (t == 0) MPROF_ADD(cls, 8, MPROF_T() - pt0);
#endif
      // norms recomputed from the rows in LDS (the cached chain, distance.cc:33-34: same bits)
      // instead of a random 4-B read each
      for (uint32_t a = t; a < b; a += NT) {
        float n = 0.0f;
#pragma unroll
        for (int k = 0; k < D; k += 4) {
          const float4 v = *reinterpret_cast<const float4*>(rows + a * ST + k);
          n = n + v.x * v.x;
          n = n + v.y * v.y;
          n = n + v.z * v.z;
          n = n + v.w * v.w;
        }
        nrm[a] = n;
        sq[a] = __builtin_sqrtf(n);
      }
    }
    __syncthreads();
#ifdef KLSH_MERGE_PROF
    if (t == 0) MPROF_ADD(cls, 9, MPROF_T() - pt0);
#endif

    // decisions in 64x64 tiles (row block R, column block C <= R): lanes = rows of R with the
    // row in registers, columns walked in order (LDS broadcast); the wave's ballot at column c
    // is P[c]'s word R, the lane's own bits form P[a]'s word C.
    auto tile = [&](uint32_t R, uint32_t C, const float* colrows) {
      const uint32_t a = R * 64u + lane;
      float xa[D];
      if (a < b) {
        load_row<D>(row_ptr(a), xa);
      } else {
#pragma unroll
        for (int k = 0; k < D; ++k) xa[k] = 0.0f;
      }
      const float sa = a < b ? sq[a] : 0.0f;
      uint64_t own = 0ull;
      const uint32_t c0 = C * 64u, c1 = min(b, c0 + 64u);
      for (uint32_t c = c0; c < c1; c += 2) {
        const uint32_t cb = (c + 1 < c1) ? c + 1 : c;
        float d0, d1;
        dot2_reg_lds<D>(xa, colrows + (c - c0) * ST, colrows + (cb - c0) * ST, d0, d1);
        const bool h0 = a < b && c < a && decide(dc, d0, sa * sq[c]);
        const bool h1 = a < b && c + 1 < c1 && c + 1 < a && decide(dc, d1, sa * sq[cb]);
        const uint64_t m0 = __ballot(h0), m1 = __ballot(h1);
        if (lane == 0) {
          if (m0) atomicOr((unsigned long long*)&P[c * W + R], (unsigned long long)m0);
          if (m1) atomicOr((unsigned long long*)&P[cb * W + R], (unsigned long long)m1);
        }
        own |= (h0 ? 1ull : 0ull) << (c - c0);
        if (c + 1 < c1) own |= (h1 ? 1ull : 0ull) << (c + 1 - c0);
      }
      if (a < b && own) atomicOr((unsigned long long*)&P[a * W + C], (unsigned long long)own);
    };
    const bool gram = kGramTiles && D % 16 == 0 && dc.fast;  // uniform
    if constexpr (ROWS_LDS) {
      const uint32_t ntiles = nblk * (nblk + 1) / 2;
      for (uint32_t ti = wv; ti < ntiles; ti += NW) {
        uint32_t R = 0;
        while ((R + 1) * (R + 2) / 2 <= ti) ++R;
        const uint32_t C = ti - R * (R + 1) / 2;
        if constexpr (D % 16 == 0) {
          if (gram) {
            auto rl = [&](uint32_t a) -> const float* { return rows + a * ST; };
            gram_tile<D>(R, C, b, rl, rl, sq, dc, P, W);
            continue;
          }
        }
        tile(R, C, rows + C * 64u * ST);
      }
    } else if (gram) {
      if constexpr (D % 16 == 0) {
        auto rm = [&](uint32_t a) -> const float* { return r.x + (size_t)slot[a] * r.dp; };
        const uint32_t ntiles = nblk * (nblk + 1) / 2;
        for (uint32_t ti = wv; ti < ntiles; ti += NW) {
          uint32_t R = 0;
          while ((R + 1) * (R + 2) / 2 <= ti) ++R;
          const uint32_t C = ti - R * (R + 1) / 2;
          gram_tile<D>(R, C, b, rm, rm, sq, dc, P, W);
        }
      }
    } else {
      for (uint32_t C = 0; C < nblk; ++C) {
        for (uint32_t q = t; q < 64u * (uint32_t)(D / 4); q += NT) {
          const uint32_t a = C * 64u + q / (D / 4), k = (q % (D / 4)) * 4;
          if (a < b)
            *reinterpret_cast<float4*>(rows + (a - C * 64u) * ST + k) =
                *reinterpret_cast<const float4*>(r.x + (size_t)slot[a] * r.dp + k);
        }
        __syncthreads();
        for (uint32_t R = C + wv; R < nblk; R += NW) tile(R, C, rows);
        __syncthreads();
      }
    }
    __syncthreads();
    [[maybe_unused]] const uint64_t pt1 = MPROF_T();
    if constexpr (ROWS_LDS && D > 0 && D <= 64) {
      big_walk_reg<RB, NT, D>(p, b, P, slot, nrm, cnt, cnt0, hd, tl, pos2row, sq, rows, cwall,
                              wbuf64, r, dc, slots, dlist, ctr);
    } else {
      big_walk<RB, NT, ROWS_LDS, D>(p, b, P, slot, nrm, cnt, hd, tl, pos2row, sq,
                                 ROWS_LDS ? rows : nullptr, ST, rows, wbuf, r, dc, slots, dlist,
                                 ctr);
    }
    __syncthreads();
#ifdef KLSH_MERGE_PROF
    if (t == 0) {
      const uint64_t pt2 = MPROF_T();
      uint32_t live = 0;
      for (uint32_t q = 0; q < b; ++q) live += slots[p + q] != kInvalid ? 1u : 0u;
      MPROF_ADD(cls, 0, 1);
      MPROF_ADD(cls, 1, b);
      MPROF_ADD(cls, 2, b - live);
      MPROF_ADD(cls, 3, pt1 - pt0);
      MPROF_ADD(cls, 4, pt2 - pt1);
      MPROF_MAX(cls, 5, pt2 - pt0);
      MPROF_MAX(cls, 6, b);
    }
#endif
  }
}

constexpr uint32_t kHugeLdsRows = 8192;  // a huge run's slots and norms in LDS up to this length
template <int D, int NT>
__device__ __forceinline__ void huge_runs(const uint2* __restrict__ list, uint32_t count,
                                          uint32_t first, uint32_t stride,
                                          uint32_t* __restrict__ slots, const Decider& dc,
                                          const Rows& r, const MergeWork& w, Counters* ctr,
                                          unsigned char* smem);

// One size class of 65..896-row runs (w.big[cls]).  w.huge_fold (385..896 class only): the
// workgroups also walk the >896-row runs afterwards (huge_runs with NT lanes), so no k_merge_huge
// is launched — the engine sets it after iterations without such runs, where a launch of its own
// would have been empty.
template <int D, int RB, int NT, bool ROWS_LDS>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(RB <= 192 ? 2 : 1))) void k_merge_big(
    MergeWork w, int cls, uint32_t* __restrict__ slots, Decider dc, Rows r, Counters* ctr) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  kt_begin(w.kt, KC_BIG128 + cls);
  const uint32_t count =
      __hip_atomic_load(&w.rc->n_big[cls].v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  big_runs<D, RB, NT, ROWS_LDS>(w.big[cls], cls, count, blockIdx.x, gridDim.x, slots, dc, r, ctr,
                                w.dlist, smem);
  if constexpr (RB == kBigRows[kBigClasses - 1]) {
    if (w.huge_fold) {
      __syncthreads();  // (the LDS layouts overlap)
      const uint32_t nh =
          __hip_atomic_load(&w.rc->n_huge.v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      huge_runs<D, NT>(w.huge, nh, blockIdx.x, gridDim.x, slots, dc, r, w, ctr, smem);
    }
  }
  kt_end(w.kt, KC_BIG128 + cls);
}

// Small iterations: every merge class in ONE launch on the main stream (no fork/join across
// streams, ≈35 us per iteration there): workgroups [0, nbig) take the 65..896-row runs (the
// longest class first), the others run four small-run waves each.
template <int D>
__global__ __launch_bounds__(256) void k_merge_tail(MergeWork w, uint32_t* __restrict__ slots,
                                                    Decider dc, Rows r, Counters* ctr,
                                                    uint32_t nbig) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  kt_begin(w.kt, KC_TAIL);
  if (blockIdx.x < nbig) {
    uint32_t cnt[kBigClasses];
#pragma unroll
    for (int c = 0; c < kBigClasses; ++c)
      cnt[c] = __hip_atomic_load(&w.rc->n_big[c].v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t nh = __hip_atomic_load(&w.rc->n_huge.v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // one index space, longest runs first: > 896 (no k_merge_huge launch in these iterations),
    // 385..896, 193..384, 129..192, 65..128
    const uint32_t a4 = nh, a3 = a4 + cnt[3], a2 = a3 + cnt[2], a1 = a2 + cnt[1],
                   total = a1 + cnt[0];
    const BigScreen bs{w.big_screen, w.bs_s_star, w.bs_m0, w.bs_a2};
    for (uint32_t li = blockIdx.x; li < total; li += nbig) {  // block-uniform
      if (li < a4)
        huge_runs<D, 256>(w.huge, li + 1, li, 1u << 30, slots, dc, r, w, ctr, smem);
      else if (li < a3)
        big_runs<D, 896, 256, false>(w.big[3], 3, li - a4 + 1, li - a4, 1u << 30, slots, dc, r,
                                     ctr, w.dlist, smem);
      else if (li < a2)
        big_runs<D, 384, 256, true>(w.big[2], 2, li - a3 + 1, li - a3, 1u << 30, slots, dc, r, ctr,
                                    w.dlist, smem, bs);
      else if (li < a1)
        big_runs<D, 192, 256, true>(w.big[1], 1, li - a2 + 1, li - a2, 1u << 30, slots, dc, r, ctr,
                                    w.dlist, smem, bs);
      else
        big_runs<D, 128, 256, true>(w.big[0], 0, li - a1 + 1, li - a1, 1u << 30, slots, dc, r, ctr,
                                    w.dlist, smem, bs);
      __syncthreads();
    }
  } else {
    const uint32_t wv = threadIdx.x >> 6;
    float* lds = reinterpret_cast<float*>(smem) + wv * 64 * (D + 4);
    small_loop<D>(w, slots, dc, r, ctr, lds, (blockIdx.x - nbig) * 4u + wv, (gridDim.x - nbig) * 4u);
  }
  kt_end(w.kt, KC_TAIL);
}

// ------------------------------------------------------ runs longer than 896 rows: workgroups -----
// The reference walk directly (no decision matrix: it would not fit), one workgroup of NT lanes
// per run: the visited row i sits in LDS, every lane tests one candidate j < i per chunk (rows
// from memory, one exact sequential dot product each), and the first hit of the chunk is found
// by a ballot + cross-wave min.  The run's slots and sqrtf(norms) live in LDS when they fit.
constexpr int kHugeNT = 512;
constexpr int kHugeKB = 8;  // visited rows tested per pass (half at d = 64); 16 measured the same

// The runs li = first, first + stride, ... (< count) of the huge list, one workgroup of NT lanes
// per run (k_merge_huge: 512 lanes; k_merge_tail's big-run workgroups: 256), smem = huge_lds().
template <int D, int NT>  // D: d at compile time (unrolled dots), 0 = any d
__device__ __forceinline__ void huge_runs(const uint2* __restrict__ list, uint32_t count,
                                          uint32_t first, uint32_t stride,
                                          uint32_t* __restrict__ slots, const Decider& dc,
                                          const Rows& r, const MergeWork& w, Counters* ctr,
                                          unsigned char* smem) {
  constexpr int NW = NT / 64;
  constexpr int kHugeNT = NT;  // (the body below is written for any NT)
  uint32_t* ls = reinterpret_cast<uint32_t*>(smem);             // [kHugeLdsRows] slots
  float* lq = reinterpret_cast<float*>(ls + kHugeLdsRows);       // [kHugeLdsRows] sqrtf(nrm)
  float* xi = lq + kHugeLdsRows;                                 // [dp] the visited row
  __shared__ uint32_t wmin[2][NW];
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const int d = r.d, dp = r.dp;
  uint32_t par = 0;
  for (uint32_t li = first; li < count; li += stride) {
    const uint2 e = list[li];
    const uint32_t p = e.x, b = e.y;
    const bool in_lds = b <= kHugeLdsRows;
    [[maybe_unused]] const uint64_t pt0 = MPROF_T();
    uint32_t* S = in_lds ? ls : slots + p;
    if (in_lds)
      for (uint32_t a = t; a < b; a += kHugeNT) {
        const uint32_t sa = slots[p + a];
        ls[a] = sa;
        lq[a] = __builtin_sqrtf(r.nrm[sa]);
      }
    __syncthreads();
    auto sqrt_at = [&](uint32_t a) { return in_lds ? lq[a] : __builtin_sqrtf(r.nrm[S[a]]); };
    uint32_t size = b, i = 1;
    if constexpr (D > 0) {
      // KB visited rows at once: positions i .. i+kc-1 are tested against every position below
      // them in one pass over the run (each candidate row j loaded once for KB dot products).
      // Until some candidate matches, the walk would visit exactly these rows in this order with
      // nothing changed, so the first candidate a* with a match (smallest j) is the reference's
      // next merge and the candidates before it simply advance i; the ones after it are
      // re-tested next pass.  A hit of candidate 0 ends the pass at its chunk (as the one-row walk
      // did), so merge-dense runs pay no extra chunks.
      constexpr int KB = D <= 32 ? kHugeKB : kHugeKB / 2;
      float* xk = xi;                          // [KB][dp] candidate rows
      float* sqk = xk + KB * dp;               // [KB] their sqrtf(norms)
      uint32_t* wk = reinterpret_cast<uint32_t*>(sqk + KB);  // [KB][NW] per-wave first hits
      while (i < size) {  // block-uniform
        const uint32_t kc = min((uint32_t)KB, size - i);
        for (uint32_t q = t; q < kc * (uint32_t)(D / 4); q += kHugeNT) {
          const uint32_t a = q / (D / 4), k4 = q % (D / 4);
          *reinterpret_cast<float4*>(xk + a * dp + 4 * k4) =
              *reinterpret_cast<const float4*>(r.x + (size_t)S[i + a] * dp + 4 * k4);
        }
        if (t < kc) sqk[t] = sqrt_at(i + t);
        __syncthreads();
        uint32_t first[KB];  // this wave's first hit per candidate (wave-uniform)
#pragma unroll
        for (int a = 0; a < KB; ++a) first[a] = 0xFFFFFFFFu;
        const uint32_t jend = i + kc - 1;  // candidate a tests positions j < i + a
        for (uint32_t c0 = 0; c0 < jend; c0 += kHugeNT) {
          const uint32_t j = c0 + t;
          bool ok[KB];
#pragma unroll
          for (int a = 0; a < KB; ++a) ok[a] = false;
          if (j < jend) {
            float xj[D];
            load_row<D>(r.x + (size_t)S[j] * dp, xj);
            const float sqj = sqrt_at(j);
#pragma unroll
            for (int a = 0; a < KB; ++a)
              if ((uint32_t)a < kc && j < i + (uint32_t)a)
                ok[a] = decide(dc, dot_reg_lds<D>(xj, xk + a * dp), sqk[a] * sqj);
          }
#pragma unroll
          for (int a = 0; a < KB; ++a) {
            const uint64_t m = __ballot(ok[a]);
            if (m && first[a] == 0xFFFFFFFFu)
              first[a] = c0 + wv * 64u + (uint32_t)(__ffsll((unsigned long long)m) - 1);
          }
          if (lane == 0) wmin[par][wv] = first[0];
          __syncthreads();
          bool hit0 = false;
#pragma unroll
          for (int q = 0; q < NW; ++q) hit0 = hit0 || wmin[par][q] != 0xFFFFFFFFu;
          par ^= 1u;
          if (hit0) break;  // block-uniform
        }
        if (lane < (uint32_t)KB) {
          uint32_t v = 0xFFFFFFFFu;
#pragma unroll
          for (int a = 0; a < KB; ++a)
            if (lane == (uint32_t)a) v = first[a];
          wk[lane * NW + wv] = v;
        }
        __syncthreads();
        uint32_t astar = 0xFFFFFFFFu, found = 0xFFFFFFFFu;
        for (uint32_t a = 0; a < kc && astar == 0xFFFFFFFFu; ++a) {
          uint32_t best = 0xFFFFFFFFu;
#pragma unroll
          for (int q = 0; q < NW; ++q) best = min(best, wk[a * NW + q]);
          if (best != 0xFFFFFFFFu) {
            astar = a;
            found = best;
          }
        }
        __syncthreads();  // wk and xk are rewritten by the next pass
        if (astar == 0xFFFFFFFFu) {
          i += kc;
          continue;
        }
        i += astar;
        float* xa = xk + astar * dp;
        const uint32_t si = S[i];
        // c[j] = SetConsensus(c[i], c[j]); c[i] = c[--size]  (cluster.cc:70-75)
        const uint32_t sj = S[found];
        const uint32_t ca = r.cnt[si], cb = r.cnt[sj];
        const float fa = (float)(int)ca, fb = (float)(int)cb, fn = (float)(int)(ca + cb);
        float* xj = r.x + (size_t)sj * dp;
        for (int k = (int)t; k < d; k += kHugeNT) {
          const float v = consensus(xa[k], fa, xj[k], fb, fn);
          xa[k] = v;  // the new row, for its norm
          store_row1(r, (size_t)sj * dp + k, v);
        }
        __syncthreads();  // the new row is in memory and in LDS
        if (t == 0) {
          const float nn = dot_seq<D>(xa, xa, d);  // distance.cc:33-34
          r.nrm[sj] = nn;
          if (in_lds) lq[found] = __builtin_sqrtf(nn);
          link_members(r, si, sj);
          mark_dirty(sj, w, ctr);
          S[i] = S[size - 1];
          if (in_lds) lq[i] = lq[size - 1];
        }
        __syncthreads();
        --size;
      }
    } else {
      while (i < size) {  // block-uniform
        const uint32_t si = S[i];
        const float sqi = sqrt_at(i);
        for (int k = (int)t * 4; k < dp; k += kHugeNT * 4)
          *reinterpret_cast<float4*>(xi + k) =
              *reinterpret_cast<const float4*>(r.x + (size_t)si * dp + k);
        __syncthreads();
        uint32_t found = 0xFFFFFFFFu;
        for (uint32_t c0 = 0; c0 < i; c0 += kHugeNT) {  // the first j < i that matches
          const uint32_t j = c0 + t;
          bool ok = false;
          if (j < i) {
            const uint32_t sj = S[j];
            ok = decide(dc, dot_seq<D>(xi, r.x + (size_t)sj * dp, d), sqi * sqrt_at(j));
          }
          const uint64_t m = __ballot(ok);
          if (lane == 0)
            wmin[par][wv] = m ? c0 + wv * 64u + (uint32_t)(__ffsll((unsigned long long)m) - 1)
                              : 0xFFFFFFFFu;
          __syncthreads();
          uint32_t best = 0xFFFFFFFFu;
#pragma unroll
          for (int q = 0; q < NW; ++q) best = min(best, wmin[par][q]);
          par ^= 1u;
          if (best != 0xFFFFFFFFu) {  // block-uniform
            found = best;
            break;
          }
        }
        if (found == 0xFFFFFFFFu) {
          ++i;
          continue;
        }
        // c[j] = SetConsensus(c[i], c[j]); c[i] = c[--size]  (cluster.cc:70-75)
        const uint32_t sj = S[found];
        const uint32_t ca = r.cnt[si], cb = r.cnt[sj];
        const float fa = (float)(int)ca, fb = (float)(int)cb, fn = (float)(int)(ca + cb);
        float* xj = r.x + (size_t)sj * dp;
        for (int k = (int)t; k < d; k += kHugeNT) {
          const float v = consensus(xi[k], fa, xj[k], fb, fn);
          xi[k] = v;  // the new row, for its norm
          store_row1(r, (size_t)sj * dp + k, v);
        }
        __syncthreads();  // the new row is in memory and in LDS
        if (t == 0) {
          const float nn = dot_seq<D>(xi, xi, d);  // distance.cc:33-34
          r.nrm[sj] = nn;
          if (in_lds) lq[found] = __builtin_sqrtf(nn);
          link_members(r, si, sj);
          mark_dirty(sj, w, ctr);
          S[i] = S[size - 1];
          if (in_lds) lq[i] = lq[size - 1];
        }
        __syncthreads();
        --size;
      }
    }
    if (in_lds)
      for (uint32_t a = t; a < size; a += kHugeNT) slots[p + a] = ls[a];
    for (uint32_t a = size + t; a < b; a += kHugeNT) slots[p + a] = kInvalid;
    __syncthreads();
    if (t == 0) {
      MPROF_ADD(kBigClasses, 0, 1);
      MPROF_ADD(kBigClasses, 1, b);
      MPROF_ADD(kBigClasses, 2, b - size);
      MPROF_ADD(kBigClasses, 4, MPROF_T() - pt0);
      MPROF_MAX(kBigClasses, 5, MPROF_T() - pt0);
      MPROF_MAX(kBigClasses, 6, b);
    }
  }
}

template <int D>
__global__ __launch_bounds__(kHugeNT) void k_merge_huge(const uint2* __restrict__ list,
                                                       const uint32_t* count_ptr,
                                                       uint32_t* __restrict__ slots, Decider dc,
                                                       Rows r, MergeWork w, Counters* ctr) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  kt_begin(w.kt, KC_HUGE);
  const uint32_t count = __hip_atomic_load(count_ptr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  huge_runs<D, kHugeNT>(list, count, blockIdx.x, gridDim.x, slots, dc, r, w, ctr, smem);
  kt_end(w.kt, KC_HUGE);
}

// LDS of huge_runs: slots + sqrt norms, then the candidate rows + their norms + per-wave first
// hits (register widths), or the visited row
static size_t huge_lds(int d, int dp, int nt) {
  const bool batched = d == 8 || d == 16 || d == 32 || d == 64;
  return sizeof(uint32_t) * kHugeLdsRows * 2 +
         (batched ? sizeof(float) * (size_t)dp * kHugeKB + sizeof(float) * kHugeKB +
                        sizeof(uint32_t) * kHugeKB * (nt / 64)
                  : sizeof(float) * (size_t)dp);
}

// ------------------------------------- runs over 896 rows: Gram bit matrix + one step per merge -----
// k_merge_long<D> (d = 16 or 32, a decider with a fast path): one 512-lane workgroup per run of up
// to kLongRows rows (longer runs keep huge_runs, in the same launch).  huge_runs pays a pass over
// the run for every 4-8 visited rows whether they merge or not (C4: 1.2K-row runs with ~12 % of
// their rows merging, 4.6 ms of walk each); here
//  1. every decision of the run comes from the certified MFMA Gram tiles (gram_tile; exact chains
//     for the close calls) into a position-space bit matrix in global memory (w.long_P, b words
//     of ceil(b/64) per row, up to 2 MB per workgroup; P[y] bit q = decide(row y, row at q)), and
//     fb[q], the first position below q that q matches, from the same tiles;
//  2. the walk then costs one step per MERGE: the lowest position q >= i with a match (one 64-bit
//     word per wave in LDS and one barrier), the consensus into its first match j, the last
//     position's row moved into i, and every position still to be visited re-decides its bit j
//     against the new row (short chains + the certified pre-screen, exact chains for the close
//     calls), takes its bit i from the moved row's matrix row (symmetric; untouched above i),
//     stores both bits (atomics) and updates its fb from them — rescanning its row of the matrix
//     only when its first match was one of the two and is gone.
// Lane t owns positions t + 512k: the rows of the first LongRegs<D>::KP of them stay in registers
// (a row at a position >= i never changes; the row moved into i comes from an LDS copy that the
// owner of the last position keeps), the rest are read from memory per step.
constexpr int kLongNT = 512;
constexpr uint32_t kLongWords = kLongRows / 64;  // matrix words per row at the longest run
template <int D>
struct LongRegs {
  static constexpr int KP = 0;
};
template <>
struct LongRegs<16> {
  static constexpr int KP = 8;
};
template <>
struct LongRegs<32> {
  static constexpr int KP = 3;
};
static size_t long_lds() { return sizeof(uint32_t) * kLongRows * 7; }

// k_merge_long's global-memory hand-offs between waves: the matrix words are updated by atomics
// (performed in L2) and read back by other waves, and rewritten rows are read by every wave, so
// reads bypass the CU's L1 (agent-scope loads) and every barrier that publishes such writes first
// waits for them (__syncthreads alone does not wait for outstanding vector-memory writes).
__device__ __forceinline__ uint64_t ld_l2(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_l2(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void vm_barrier() {
  __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0)
  __syncthreads();
}

// First set bit of the matrix row Py in [lo, hi), with bit j taken as dn and bit i (kNone: none)
// as bm — this step's two stores may not have landed yet.  Rare (a first match that is gone).
__device__ __noinline__ uint32_t long_rescan(const uint64_t* Py, uint32_t lo, uint32_t hi, uint32_t j,
                                             bool dn, uint32_t i, bool bm) {
  const uint64_t bj = 1ull << (j & 63u), bi = 1ull << (i & 63u);
  for (uint32_t k = lo >> 6; k * 64u < hi; ++k) {
    uint64_t wd = ld_l2(Py + k);
    if (k == (j >> 6)) wd = dn ? (wd | bj) : (wd & ~bj);
    if (i != 0xFFFFFFFFu && k == (i >> 6)) wd = bm ? (wd | bi) : (wd & ~bi);
    if (k == (lo >> 6)) wd &= ~0ull << (lo & 63u);
    if (hi - k * 64u < 64u) wd &= (1ull << (hi - k * 64u)) - 1ull;
    if (wd) return k * 64u + (uint32_t)__builtin_ctzll(wd);
  }
  return 0xFFFFFFFFu;
}

// Typed views of a global row and an LDS row as 16-B vectors (builtin vectors: assignable in an
// address space).  Through generic pointers every access is a flat one (both wait counters, and
// a flat load-store pair per element where the compiler cannot rule out overlap).
typedef float klsh_f4 __attribute__((ext_vector_type(4)));
using GRow4 = const __attribute__((address_space(1))) klsh_f4*;
using LRow4 = __attribute__((address_space(3))) klsh_f4*;

// dst[0, D) = src[0, D) for a global row src and an LDS row dst: every load before the stores.
template <int D>
__device__ __forceinline__ void copy_row_to_lds(float* dst, const float* src) {
  const GRow4 g = (GRow4)(const klsh_f4*)src;
  const LRow4 l = (LRow4)(klsh_f4*)dst;
  klsh_f4 v[D / 4];
#pragma unroll
  for (int k = 0; k < D / 4; ++k) v[k] = g[k];
#pragma unroll
  for (int k = 0; k < D / 4; ++k) l[k] = v[k];
}

// One position of k_merge_long past the register ones: its row from memory against the new row
// (short chains + pre-screen, the sequential chains for a close call); the row copied to `last`
// if given.  Out of line: the register positions' rows stay live around the call.  xp: a global
// row; cw, last: LDS rows (typed below).
template <int D>
__device__ __noinline__ uint32_t long_mem_decide(const float* xp, const float* cw, float sy,
                                                 float sc_a, Decider dc, float* last) {
  const GRow4 xg = (GRow4)(const klsh_f4*)xp;
  const LRow4 cl = (LRow4)(klsh_f4*)const_cast<float*>(cw);
  float d4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int k = 0; k < D; k += 4) {
    const klsh_f4 u = cl[k / 4];
    const klsh_f4 xv = xg[k / 4];
    d4[0] = d4[0] + xv.x * u.x;
    d4[1] = d4[1] + xv.y * u.y;
    d4[2] = d4[2] + xv.z * u.z;
    d4[3] = d4[3] + xv.w * u.w;
  }
  uint32_t v = prescreen(dc, (d4[0] + d4[1]) + (d4[2] + d4[3]), sy * sc_a);
  if (v == 2u) {
    float nn = 0.0f, dot = 0.0f;
    for (int k = 0; k < D; ++k) nn = nn + cw[k] * cw[k];
    for (int k = 0; k < D; ++k) dot = dot + xp[k] * cw[k];
    v = decide(dc, dot, sy * __builtin_sqrtf(nn)) ? 1u : 0u;
  }
  // (the row kept in registers from the loop above for this copy measured slower: C4 892 ->
  // 907 ms, the extra registers of this out-of-line call saved and restored around it; an
  // element loop here was one round trip per element — the pointers may alias)
  if (last) copy_row_to_lds<D>(last, xp);  // (last: the caller's LDS row)
  return v;
}

template <int D>
__device__ __forceinline__ void long_run(uint32_t p, uint32_t b, uint64_t* __restrict__ P,
                                         uint32_t* __restrict__ slots, const Decider& dc,
                                         const Rows& r, const MergeWork& w, Counters* ctr,
                                         unsigned char* smem) {
  constexpr int NT = kLongNT, NW = NT / 64;
  constexpr int KR = LongRegs<D>::KP;               // positions per lane with the row in registers
  constexpr int KT = (int)(kLongRows / (uint32_t)NT);  // positions per lane
  constexpr uint32_t CT = kLongRows;
  constexpr uint32_t kNone = 0xFFFFFFFFu;
  constexpr uint64_t kNone64 = ~0ull;
  static_assert(KR > 0 && KR <= KT && CT <= 4096, "positions are packed in 12 bits");
  uint32_t* slot = reinterpret_cast<uint32_t*>(smem);  // by row id
  uint32_t* cnt = slot + CT;
  uint32_t* hd = slot + 2 * CT;
  uint32_t* tl = slot + 3 * CT;
  uint32_t* pos2row = slot + 4 * CT;
  float* sq = reinterpret_cast<float*>(slot + 5 * CT);  // sqrtf(nrm), distance.cc:37
  uint32_t* fb = slot + 6 * CT;                          // by POSITION
  __shared__ __attribute__((aligned(16))) float cwall[NW][D];  // each wave's copy of the new row
  __shared__ __attribute__((aligned(16))) float lrow[2][D];    // the row at the last position
  __shared__ uint64_t wbuf[2][NW];
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint32_t W = (b + 63u) >> 6;
  const int dp = r.dp;
  [[maybe_unused]] const uint64_t pt0 = MPROF_T();
  // 1. metadata in LDS, the matrix zeroed
  for (uint32_t a = t; a < b; a += NT) {
    const uint32_t s = slots[p + a];
    slot[a] = s;
    cnt[a] = r.cnt[s];
    hd[a] = r.head[s];
    tl[a] = r.tail[s];
    pos2row[a] = a;
    sq[a] = __builtin_sqrtf(r.nrm[s]);
    fb[a] = kNone;
  }
  {
    uint4* P4 = reinterpret_cast<uint4*>(P);
    const uint32_t n4 = (b * W + 1u) / 2u;  // (one word past b * W at most: inside the block)
    for (uint32_t q = t; q < n4; q += NT) P4[q] = make_uint4(0u, 0u, 0u, 0u);
  }
  vm_barrier();  // (the zeros are in L2 before any tile's atomics)
  // 2. every decision of the run, and each position's first match below it
  {
    auto rm = [&](uint32_t a) -> const float* { return r.x + (size_t)slot[a] * dp; };
    const uint32_t ntiles = W * (W + 1u) / 2u;
    for (uint32_t ti = wv; ti < ntiles; ti += NW) {
      uint32_t R = (uint32_t)((__builtin_sqrtf(8.0f * (float)ti + 1.0f) - 1.0f) * 0.5f);
      while (R * (R + 1u) / 2u > ti) --R;
      while ((R + 1u) * (R + 2u) / 2u <= ti) ++R;
      gram_tile<D>(R, ti - R * (R + 1u) / 2u, b, rm, rm, sq, dc, P, (int)W, fb);
    }
  }
  vm_barrier();
  [[maybe_unused]] const uint64_t pt1 = MPROF_T();
  // 3. the walk
  float xr[KR][D];  // rows of my register positions t + kp * NT
#pragma unroll
  for (int kp = 0; kp < KR; ++kp) {
    const uint32_t q = t + (uint32_t)kp * NT;
    if (q < b) {
      load_row<D>(r.x + (size_t)slot[q] * dp, xr[kp]);
    } else {
#pragma unroll
      for (int k = 0; k < D; ++k) xr[kp][k] = 0.0f;
    }
  }
  // a hit: position (12 bits) | its first match | its row | the row at the first match
  auto pack = [](uint32_t q, uint32_t j, uint32_t y, uint32_t c) -> uint64_t {
    return ((uint64_t)q << 36) | ((uint64_t)j << 24) | ((uint64_t)y << 12) | (uint64_t)c;
  };
  auto publish = [&](uint32_t par, uint64_t mine) {  // the wave's lowest hit -> wbuf[par][wv]
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mine = min(mine, shfl64(mine, lane ^ (uint32_t)o));
    if (lane == 0) wbuf[par][wv] = mine;
  };
  auto put_last = [&](uint32_t buf, const float (&x)[D]) {
#pragma unroll
    for (int k = 0; k < D; k += 4)
      *reinterpret_cast<float4*>(&lrow[buf][k]) = make_float4(x[k], x[k + 1], x[k + 2], x[k + 3]);
  };
  uint32_t size = b, par = 0, lp = 0;
  {
    uint64_t mine = kNone64;
    for (uint32_t q = t; q < b; q += NT) {
      const uint32_t f = fb[q];
      if (q >= 1u && f != kNone) mine = min(mine, pack(q, f, q, f));
    }
    publish(0, mine);
    const uint32_t ql = b - 1u;  // the last position's row
    if (t == ql % NT) {
      float xl[D];
      load_row<D>(r.x + (size_t)slot[ql] * dp, xl);
      put_last(0, xl);
    }
  }
  __syncthreads();
  bool have = false;
  uint32_t ip = 0, mp = 0, cp = 0, rp = 0, cntp = 0, hdp = 0;
  [[maybe_unused]] uint64_t steps = 0;
  while (true) {
    uint64_t best = kNone64;
#pragma unroll
    for (int q = 0; q < NW; ++q) best = min(best, wbuf[par][q]);
    par ^= 1u;
    if (have) {  // the previous step's writes to the shared state, by every wave before its reads
      if (lane == 0) {
        pos2row[ip] = mp;
        cnt[cp] = cntp;
        cnt[rp] = 0u;
        hd[cp] = hdp;
      }
      // the previous step's new row to memory (wave 0's copy): not during that step, when other
      // waves were still reading the old row for their own consensus
      if (wv == 0 && lane < (uint32_t)D) store_row1(r, (size_t)slot[cp] * dp + lane, cwall[0][lane]);
      wave_lds_fence();
    }
    if (best == kNone64) break;
    ++steps;
    // (wave-uniform values: scalar registers)
    const uint32_t hi32 = __builtin_amdgcn_readfirstlane((uint32_t)(best >> 32));
    const uint32_t lo32 = __builtin_amdgcn_readfirstlane((uint32_t)best);
    const uint32_t i = hi32 >> 4, j = ((hi32 & 15u) << 8) | (lo32 >> 24),
                   rr = (lo32 >> 12) & 0xFFFu, c = lo32 & 0xFFFu;
    const uint32_t last = size - 1u;
    const uint32_t moved = __builtin_amdgcn_readfirstlane(pos2row[last]);  // (rr if i is last)
    const uint32_t ca = __builtin_amdgcn_readfirstlane(cnt[rr]),
                   cb = __builtin_amdgcn_readfirstlane(cnt[c]),
                   hr = __builtin_amdgcn_readfirstlane(hd[rr]),
                   tr = __builtin_amdgcn_readfirstlane(tl[rr]),
                   hc = __builtin_amdgcn_readfirstlane(hd[c]);
    const uint32_t s_r = __builtin_amdgcn_readfirstlane(slot[rr]),
                   s_c = __builtin_amdgcn_readfirstlane(slot[c]);
    const uint32_t f_last = __builtin_amdgcn_readfirstlane(fb[last]);
    // the moved row's matrix row: its bits at the positions above i are the Gram tiles' own
    const uint64_t pm = lane < W ? ld_l2(P + (size_t)moved * W + lane) : 0ull;
    // consensus (funcAB.cc:65), current row first, into this wave's copy of the new row c
    const float fa = (float)(int)ca, fbc = (float)(int)cb, fn = (float)(int)(ca + cb);
    if (lane < (uint32_t)D) {
      // row c as of now: the previous step's new row if it is that row again (its store above may
      // not have landed), else memory (every earlier store landed at its step's barrier)
      const float xc = have && c == cp ? cwall[wv][lane] : ld_l2(r.x + (size_t)s_c * dp + lane);
      const float v = consensus(ld_l2(r.x + (size_t)s_r * dp + lane), fa, xc, fbc, fn);
      cwall[wv][lane] = v;
    }
    if (t == 0) r.nxt[tr] = hc;  // ids_current ++ ids_candidate (funcAB.cc:51-55)
    wave_lds_fence();
    size = last;  // swap-remove: the row at the old last position moves to i
    const float* cw = &cwall[wv][0];
    float n4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int k = 0; k < D; k += 4) {
      const float4 u = *reinterpret_cast<const float4*>(cw + k);
      n4[0] = n4[0] + u.x * u.x;
      n4[1] = n4[1] + u.y * u.y;
      n4[2] = n4[2] + u.z * u.z;
      n4[3] = n4[3] + u.w * u.w;
    }
    const float sc_a = __builtin_sqrtf((n4[0] + n4[1]) + (n4[2] + n4[3]));
    uint64_t mine = kNone64;
    // position q >= i (row y) with bit j re-decided (dn) and bit i taken (bm): store both bits,
    // update fb[q], offer a hit
    auto settle = [&](uint32_t q, uint32_t y, bool dn, bool bm) {
      uint64_t* Py = P + (size_t)y * W;
      const uint64_t bj = 1ull << (j & 63u), bi = 1ull << (i & 63u);
      if (dn) atomicOr((unsigned long long*)&Py[j >> 6], (unsigned long long)bj);
      else atomicAnd((unsigned long long*)&Py[j >> 6], (unsigned long long)~bj);
      uint32_t f;
      bool lost;
      uint32_t lower;
      if (q == i) {  // the moved row: below i only bit j changed
        f = f_last < i ? f_last : kNone;
        lost = f == j && !dn;
        lower = dn ? j : kNone;
      } else {
        if (bm) atomicOr((unsigned long long*)&Py[i >> 6], (unsigned long long)bi);
        else atomicAnd((unsigned long long*)&Py[i >> 6], (unsigned long long)~bi);
        f = fb[q];
        lost = (f == j && !dn) || (f == i && !bm);
        lower = dn ? j : (bm ? i : kNone);
      }
      if (!lost) {
        f = min(f, lower);
      } else if (lower < f) {
        f = lower;
      } else {  // the first match is gone: the unchanged bits between it and `lower`
        const uint32_t g = long_rescan(Py, f + 1u, min(lower, q), j, dn, q != i ? i : kNone, bm);
        f = g != kNone ? g : lower;
      }
      fb[q] = f;
      if (f != kNone) mine = min(mine, pack(q, f, y, f == i ? moved : pos2row[f]));
    };
    // the register positions: decisions first (rows live), then the bookkeeping (rows dead)
    uint32_t dmask = 0u;
#pragma unroll
    for (int kp = 0; kp < KR; ++kp) {
      const uint32_t q = t + (uint32_t)kp * NT;
      if (q >= i && q < size) {
        const uint32_t y = q == i ? moved : pos2row[q];
        const float sy = sq[y];
        if (q == i) {
#pragma unroll
          for (int k = 0; k < D; ++k) xr[kp][k] = lrow[lp][k];
        }
        float d4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int k = 0; k < D; k += 4) {
          const float4 u = *reinterpret_cast<const float4*>(cw + k);
          d4[0] = d4[0] + xr[kp][k] * u.x;
          d4[1] = d4[1] + xr[kp][k + 1] * u.y;
          d4[2] = d4[2] + xr[kp][k + 2] * u.z;
          d4[3] = d4[3] + xr[kp][k + 3] * u.w;
        }
        uint32_t v = prescreen(dc, (d4[0] + d4[1]) + (d4[2] + d4[3]), sy * sc_a);
        if (v == 2u) {  // rare: the reference's sequential chains (distance.cc:27-38)
          float nn = 0.0f, dot = 0.0f;
#pragma unroll
          for (int k = 0; k < D; ++k) nn = nn + cw[k] * cw[k];
#pragma unroll
          for (int k = 0; k < D; ++k) dot = dot + xr[kp][k] * cw[k];
          v = decide(dc, dot, sy * __builtin_sqrtf(nn)) ? 1u : 0u;
        }
        dmask |= v << kp;
        if (q == size - 1u) put_last(lp ^ 1u, xr[kp]);  // the next swap-remove's row
      }
      asm volatile("" ::: "memory");  // (the new row is re-read from LDS per position)
    }
#pragma unroll
    for (int kp = 0; kp < KR; ++kp) {
      const uint32_t q = t + (uint32_t)kp * NT;
      // bit i of row q := decide(q, moved) = the moved row's bit q (wave-uniform shuffle)
      const uint64_t wm = shfl64(pm, (q >> 6) & 63u);
      const bool bm = (wm >> (q & 63u)) & 1ull;
      if (q >= i && q < size) settle(q, q == i ? moved : pos2row[q], (dmask >> kp) & 1u, bm);
    }
#pragma unroll 1
    for (int kp = KR; kp < KT; ++kp) {  // positions past them (runs over KR * 512 rows): memory
      const uint32_t q = t + (uint32_t)kp * NT;
      const uint64_t wm = shfl64(pm, (q >> 6) & 63u);
      const bool bm = (wm >> (q & 63u)) & 1ull;
      if (q >= i && q < size) {
        const uint32_t y = q == i ? moved : pos2row[q];
        const float* xp = r.x + (size_t)slot[y] * dp;
        const uint32_t v = long_mem_decide<D>(xp, cw, sq[y], sc_a, dc, q == size - 1u ? &lrow[lp ^ 1u][0] : nullptr);
        settle(q, y, v != 0u, bm);
      }
    }
    publish(par, mine);
    have = true;
    ip = i;
    mp = moved;
    cp = c;
    rp = rr;
    cntp = ca + cb;
    hdp = hr;
    lp ^= 1u;
    vm_barrier();  // this step's matrix bits and the new row are in L2
  }
  vm_barrier();
  // write back: survivors in position order, kInvalid after; rewritten rows' norms and metadata
  for (uint32_t q = t; q < b; q += NT) slots[p + q] = q < size ? slot[pos2row[q]] : kInvalid;
  for (uint32_t q0 = 0; q0 < size; q0 += NT) {  // uniform trip count (ballot inside)
    const uint32_t q = q0 + t;
    bool rewritten = false;
    uint32_t s = 0;
    if (q < size) {
      const uint32_t y = pos2row[q];
      s = slot[y];
      rewritten = r.cnt[s] != cnt[y];  // every merge into a row raises its count
      if (rewritten) {  // the exact sequential norm of the new row (distance.cc:33-34)
        float xv[D];
#pragma unroll
        for (int k = 0; k < D; ++k) xv[k] = ld_l2(r.x + (size_t)s * dp + k);
        float nv = 0.0f;
#pragma unroll
        for (int k = 0; k < D; ++k) nv = nv + xv[k] * xv[k];
        r.nrm[s] = nv;
        r.cnt[s] = cnt[y];
        r.head[s] = hd[y];
      }
    }
    if (w.dlist) append_slot(rewritten, s, w.dlist, &ctr->n_delta);
  }
  __syncthreads();
#ifdef KLSH_MERGE_PROF
  if (t == 0) {
    const uint64_t pt2 = MPROF_T();
    MPROF_ADD(kBigClasses, 0, 1);
    MPROF_ADD(kBigClasses, 1, b);
    MPROF_ADD(kBigClasses, 2, b - size);
    MPROF_ADD(kBigClasses, 3, pt1 - pt0);
    MPROF_ADD(kBigClasses, 4, pt2 - pt1);
    MPROF_MAX(kBigClasses, 5, pt2 - pt0);
    MPROF_MAX(kBigClasses, 6, b);
  }
#endif
}

// One index space over the >896-row list and (list2, option long_runs = 4) the 385..896-row
// list after it: the longest walks first.
template <int D>
__global__ __launch_bounds__(kLongNT) void k_merge_long(const uint2* __restrict__ list,
                                                        const uint32_t* count_ptr,
                                                        const uint2* __restrict__ list2,
                                                        const uint32_t* count2_ptr,
                                                        uint32_t* __restrict__ slots, Decider dc,
                                                        Rows r, MergeWork w, Counters* ctr) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  kt_begin(w.kt, KC_HUGE);
  const uint32_t count = __hip_atomic_load(count_ptr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t count2 =
      list2 ? __hip_atomic_load(count2_ptr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
  uint64_t* P = w.long_P + (size_t)blockIdx.x * kLongRows * kLongWords;
  for (uint32_t li = blockIdx.x; li < count + count2; li += gridDim.x) {  // block-uniform
    const uint2* l = li < count ? list : list2;
    const uint32_t k = li < count ? li : li - count;
    const uint2 e = l[k];
    if (e.y <= kLongRows) long_run<D>(e.x, e.y, P, slots, dc, r, w, ctr, smem);
    else huge_runs<D, kLongNT>(l, k + 1u, k, 1u << 30, slots, dc, r, w, ctr, smem);
    __syncthreads();
  }
  kt_end(w.kt, KC_HUGE);
}

// k_merge_long takes the >896-row runs (and with option long_runs = 4 the 385..896-row ones)
static bool long_ok_for(const MergeWork& w, const Decider& dc, const Rows& r) {
  return w.long_P && w.long_groups && w.long_off != 1u && dc.fast && (r.d == 16 || r.d == 32);
}
static bool long896(const MergeWork& w, const Decider& dc, const Rows& r) {
  return w.long_off == 4u && long_ok_for(w, dc, r);
}

static void launch_huge(const MergeWork& w, uint32_t* slots, const Decider& dc, const Rows& r,
                        Counters* ctr, uint32_t n, hipStream_t s) {
  const bool with896 = long896(w, dc, r);
  if (w.huge_fold && !with896) return;  // the 385..896-row kernel walks them (k_merge_big)
  uint32_t g = (uint32_t)std::min<uint64_t>(512, n / (kBigRows[kBigClasses - 1] + 1) + 1);
  if (w.huge_cap && !with896) g = std::min(g, w.huge_cap);  // (the kernel strides over its list)
  if (with896) g = (uint32_t)std::min<uint64_t>(1024, n / (kBigRows[kBigClasses - 2] + 1) + 1);
  if (long_ok_for(w, dc, r)) {
    const size_t lds = std::max(long_lds(), huge_lds(r.d, r.dp, kLongNT));
    static const bool lds_ok = [lds] {
      bool ok = true;
      for (const void* f : {reinterpret_cast<const void*>(&k_merge_long<16>),
                            reinterpret_cast<const void*>(&k_merge_long<32>)})
        ok = ok && hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) ==
                       hipSuccess;
      return ok;
    }();
    (void)lds_ok;
    g = std::min(g, w.long_groups);
    const uint2* l2 = with896 ? w.big[kBigClasses - 1] : nullptr;
    const uint32_t* c2 = &w.rc->n_big[kBigClasses - 1].v;
    if (r.d == 16)
      k_merge_long<16><<<g, kLongNT, lds, s>>>(w.huge, &w.rc->n_huge.v, l2, c2, slots, dc, r, w, ctr);
    else
      k_merge_long<32><<<g, kLongNT, lds, s>>>(w.huge, &w.rc->n_huge.v, l2, c2, slots, dc, r, w, ctr);
    return;
  }
  const size_t lds = huge_lds(r.d, r.dp, kHugeNT);
  static const bool lds_ok = [] {
    bool ok = true;
    for (const void* f : {reinterpret_cast<const void*>(&k_merge_huge<0>),
                          reinterpret_cast<const void*>(&k_merge_huge<8>),
                          reinterpret_cast<const void*>(&k_merge_huge<16>),
                          reinterpret_cast<const void*>(&k_merge_huge<32>),
                          reinterpret_cast<const void*>(&k_merge_huge<64>)})
      ok = ok && hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024) ==
                     hipSuccess;
    return ok;
  }();
  (void)lds_ok;
  switch (r.d) {
    case 8: k_merge_huge<8><<<g, kHugeNT, lds, s>>>(w.huge, &w.rc->n_huge.v, slots, dc, r, w, ctr); break;
    case 16: k_merge_huge<16><<<g, kHugeNT, lds, s>>>(w.huge, &w.rc->n_huge.v, slots, dc, r, w, ctr); break;
    case 32: k_merge_huge<32><<<g, kHugeNT, lds, s>>>(w.huge, &w.rc->n_huge.v, slots, dc, r, w, ctr); break;
    case 64: k_merge_huge<64><<<g, kHugeNT, lds, s>>>(w.huge, &w.rc->n_huge.v, slots, dc, r, w, ctr); break;
    default: k_merge_huge<0><<<g, kHugeNT, lds, s>>>(w.huge, &w.rc->n_huge.v, slots, dc, r, w, ctr);
  }
}

// ------------------------------------------------------------------ wide rows (any d) -----
// Rows that do not fit in registers (d > 64, or a width without a register kernel): the same
// G-lane group scheme, but the pairwise decisions are accumulated over 64-column chunks staged
// through LDS (each lane's chains continue across chunks, so every dot product keeps the
// reference's k order), and the walk's recomputations read the two rows from memory.
constexpr int kWideKC = 64;

// The exact group merges' chunk width (C5: 32 columns halve the staged tile to 9 KB per wave, so
// LDS no longer caps the waves per CU below what the registers allow)
constexpr int kWideXKC = 32;

// Columns [c0, c0 + kcp) of the 64 lanes' rows -> LDS rows (stride KC + 4), coalesced:
// KC/4 lanes per row, 256/KC rows per wave instruction.  kcp is a multiple of 4.
template <int KC = kWideKC>
__device__ __forceinline__ void stage_chunk(const float* __restrict__ X, int dp, uint32_t slot,
                                            bool valid, int c0, int kcp, float* tile) {
  constexpr int ST = KC + 4, LPR = KC / 4, RPI = 64 / LPR;
  const uint32_t lane = __lane_id();
  const uint32_t q = lane & (LPR - 1u), rsub = lane / LPR;
  const bool col_ok = (int)(4 * q) < kcp;
  // Loads and stores unconditional (a lane past its run reads its slot's row, valid memory — the
  // callers pass slot 0 there — and the column clamped to c0; both zeroed after the load): a
  // load under `ok && col_ok` was a branch per row with its shuffles waited in front of it, and
  // a store under `col_ok` lets the compiler sink the load into it.  Columns kcp .. KC of the
  // tile (a partial last chunk) get zeros; the readers use n <= kcp of them.
  uint32_t s[LPR];
  bool ok[LPR];
#pragma unroll
  for (int it = 0; it < LPR; ++it) {
    const uint32_t row = it * RPI + rsub;
    s[it] = shfl32(slot, row);
    const int vr = __shfl(valid ? 1 : 0, (int)row, 64);  // (every lane: a shuffle under col_ok
    ok[it] = col_ok && vr != 0;                           // reads inactive lanes as 0)
  }
  float4 v[LPR];
#pragma unroll
  for (int it = 0; it < LPR; ++it)
    v[it] = *reinterpret_cast<const float4*>(X + (size_t)s[it] * dp + c0 + (col_ok ? 4 * q : 0u));
#pragma unroll
  for (int it = 0; it < LPR; ++it) {
    if (!ok[it]) v[it] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    *reinterpret_cast<float4*>(tile + (it * RPI + rsub) * ST + 4 * q) = v[it];
  }
}

template <int N>
__device__ __forceinline__ float dot_acc_reg(float s, const float (&a)[N], const float* b) {
#pragma unroll
  for (int k = 0; k < N; k += 4) {
    const float4 v = *reinterpret_cast<const float4*>(b + k);
    s = s + a[k] * v.x;
    s = s + a[k + 1] * v.y;
    s = s + a[k + 2] * v.z;
    s = s + a[k + 3] * v.w;
  }
  return s;
}

// DG: d at compile time for the runs of G >= 8 rows (their pairwise decisions from one 64x64
// MFMA Gram tile, certified with the wide margin the caller's decider carries, exact chains only
// for the close calls), 0 = every pair by its exact chain.
template <int G, int DG = 0>
__device__ __forceinline__ void merge_batch_wide(uint32_t p, uint32_t b, uint32_t slot,
                                                 uint32_t* slots, const Decider& dc,
                                                 const Rows& r, float* tile, uint32_t* dlist,
                                                 Counters* ctr) {
  constexpr int ST = kWideKC + 4;
  constexpr int NK = G / 2;  // partners per lane: k = 1 .. b/2 <= G/2
  const uint32_t lane = threadIdx.x;
  const uint32_t g = lane & (G - 1);
  const uint32_t gbase = lane - g;
  const uint64_t gmask = (G == 64) ? ~0ull : (((1ull << (G & 63)) - 1ull) << gbase);
  const int d = r.d, dp = r.dp;
  const bool valid = g < b;
  float nrm = valid ? r.nrm[slot] : 0.0f;
  float sq = __builtin_sqrtf(nrm);  // distance.cc:37
  const float* myx = r.x + (size_t)slot * dp;
  const uint32_t bmax = wave_max(b);
  const uint32_t half = b / 2, kmax = bmax / 2;
  auto partner = [&](uint32_t k) {  // (g + k) mod b, for k <= b
    const uint32_t j = g + k;
    return j >= b ? j - b : j;
  };

  uint64_t full = 0ull;
  if constexpr (DG > 0 && G >= 8) {
    // 1'. the batch's decisions from one Gram tile on the matrix cores (bf16x3): the 64 lanes'
    //     rows against each other, accumulated over the same LDS-staged 64-column chunks, pairs
    //     across runs masked off afterwards; close calls by the exact chain (gram_decide)
    __shared__ uint64_t Pw[64];  // position masks
    __shared__ uint32_t sl[64];
    __shared__ float sqs[64];
    f32x16 acc[2][2];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[m][n][i] = 0.0f;
    for (int c0 = 0; c0 < DG; c0 += kWideKC) {
      wave_lds_fence();  // the previous chunk's reads are done
      stage_chunk(r.x, dp, slot, valid, c0, kWideKC, tile);
      wave_lds_fence();
      auto rl = [&](uint32_t a) -> const float* { return tile + a * ST; };
      gram_acc<kWideKC>(0u, 0u, 64u, rl, rl, acc);
    }
    wave_lds_fence();
    Pw[lane] = 0ull;
    sl[lane] = slot;  // (a lane past its run holds a valid row: slot 0)
    sqs[lane] = valid ? sq : 1.0f;
    wave_lds_fence();
    auto rm = [&](uint32_t a) -> const float* { return r.x + (size_t)sl[a] * dp; };
    gram_decide<DG>(0u, 0u, 64u, acc, rm, rm, sqs, dc, Pw, 1, nullptr);
    __builtin_amdgcn_s_waitcnt(0x0070);  // (its atomics into LDS) vmcnt(0) lgkmcnt(0)
    wave_lds_fence();
    const uint64_t runbits = b >= 64u ? ~0ull : ((1ull << b) - 1ull);
    full = valid ? ((Pw[lane] >> gbase) & runbits & ~(1ull << g)) : 0ull;
    wave_lds_fence();
  } else {
  // 1. every pairwise dot product of the run, chunk by chunk (lane g vs positions g + k)
  constexpr int XKC = kWideXKC, XST = XKC + 4;
  float acc[NK];
#pragma unroll
  for (int k = 0; k < NK; ++k) acc[k] = 0.0f;
  for (int c0 = 0; c0 < d; c0 += XKC) {
    const int n = min(XKC, d - c0), kcp = min(XKC, dp - c0);
    wave_lds_fence();  // the previous chunk's reads are done
    stage_chunk<XKC>(r.x, dp, slot, valid, c0, kcp, tile);
    wave_lds_fence();
    const float* mine = tile + lane * XST;
    if (n == XKC) {
      float x[XKC];
      load_row<XKC>(mine, x);
#pragma unroll
      for (int k = 1; k <= NK; ++k)
        if ((uint32_t)k <= kmax && valid && (uint32_t)k <= half)
          acc[k - 1] = dot_acc_reg<XKC>(acc[k - 1], x, tile + (gbase + partner(k)) * XST);
    } else {
#pragma unroll
      for (int k = 1; k <= NK; ++k)
        if ((uint32_t)k <= kmax && valid && (uint32_t)k <= half)
          acc[k - 1] = dot_acc_mem(acc[k - 1], mine, tile + (gbase + partner(k)) * XST, n);
    }
  }
#pragma unroll
  for (int k = 1; k <= NK; ++k) {
    if ((uint32_t)k <= kmax) {  // wave-uniform
      const uint32_t j = partner(min((uint32_t)k, b));
      const float sj = shflf(sq, gbase + (j & (G - 1)));
      const bool bit = valid && (uint32_t)k <= half && decide(dc, acc[k - 1], sq * sj);
      const uint32_t src = g >= (uint32_t)k ? g - k : g + b - k;  // lane holding decide(src, g)
      const uint32_t in = (uint32_t)__shfl((int)bit, (int)(gbase + (src & (G - 1))), 64);
      if (valid && (uint32_t)k <= half) {
        full |= (uint64_t)bit << j;
        full |= (uint64_t)in << src;
      }
    }
  }
  }

  // member counts and list ends only for the runs with a matching pair (as merge_batch)
  const bool grp = (__ballot(valid && full != 0ull) & gmask) != 0ull;
  uint32_t cnt = 0u, hd = 0u, tl = 0u;
  if (valid && grp) {
    cnt = r.cnt[slot];
    hd = r.head[slot];
    tl = r.tail[slot];
  }

  // 2. the walk, replayed on the bits (as merge_batch); rows live in memory
  uint32_t rowid = g, mypos = g;
  bool alive = valid, dirty = false;
  uint32_t i = 1, size = b;
  while (true) {
    const uint64_t mybit = g < size ? (1ull << rowid) : 0ull;
    uint64_t incl = mybit;
#pragma unroll
    for (uint32_t o = 1; o < (uint32_t)G; o <<= 1) {
      const uint64_t y = shfl64(incl, lane >= o ? lane - o : lane);
      if (g >= o) incl |= y;
    }
    const uint64_t frow = shfl64(full, gbase + rowid);
    const bool hit = g >= i && g < size && (frow & (incl & ~mybit)) != 0ull;
    const uint64_t m = __ballot(hit) & gmask;
    if (__ballot(m != 0ull) == 0ull) break;
    if (m != 0ull) {
      i = (uint32_t)(__ffsll((unsigned long long)m) - 1) - gbase;
      const uint32_t rr = shfl32(rowid, gbase + i);
      const uint64_t fr = shfl64(frow, gbase + i);
      const uint64_t mj = __ballot(g < i && ((fr >> rowid) & 1ull)) & gmask;
      const uint32_t jpos = (uint32_t)(__ffsll((unsigned long long)mj) - 1) - gbase;
      const uint32_t c = shfl32(rowid, gbase + jpos);
      const uint32_t ca = shfl32(cnt, gbase + rr), cb = shfl32(cnt, gbase + c);
      const uint32_t hr = shfl32(hd, gbase + rr), tr = shfl32(tl, gbase + rr);
      const uint32_t hc = shfl32(hd, gbase + c);
      const uint32_t slot_r = shfl32(slot, gbase + rr), slot_c = shfl32(slot, gbase + c);
      const float fa = (float)(int)ca, fb = (float)(int)cb, fn = (float)(int)(ca + cb);
      const float* xr = r.x + (size_t)slot_r * dp;
      float* xc = r.x + (size_t)slot_c * dp;
      for (int k = (int)g; k < d; k += G)
        store_row1(r, (size_t)slot_c * dp + k, consensus(xr[k], fa, xc[k], fb, fn));
      lds_fence();  // the new row c is visible to the group's lanes
      if (g == rr) alive = false;
      if (g == 0) r.nxt[tr] = hc;  // ids_current ++ ids_candidate (funcAB.cc:51-55)
      const uint32_t last = shfl32(rowid, gbase + size - 1);  // swap-remove
      if (g == i) rowid = last;
      if (g == last) mypos = i;
      --size;
      // lane c: its exact sequential norm; rows still to be visited: their dot with row c
      const bool todo = alive && mypos >= i && mypos < size;
      float dot = 0.0f;
      if (g == c || todo) dot = dot_acc_mem(0.0f, myx, xc, d);
      if (g == c) {
        nrm = dot;
        sq = __builtin_sqrtf(dot);
        cnt = ca + cb;
        hd = hr;
        dirty = true;
      }
      const float sc = shflf(sq, gbase + c);
      if (todo) full = decide(dc, dot, sq * sc) ? (full | (1ull << c)) : (full & ~(1ull << c));
    }
  }

  // 3. write back
  const uint32_t pos_slot = shfl32(slot, gbase + rowid);
  if (valid && size < b) slots[p + g] = g < size ? pos_slot : kInvalid;
  if (valid && alive && dirty) {
    r.nrm[slot] = nrm;
    r.cnt[slot] = cnt;
    r.head[slot] = hd;
  }
  if (dlist) append_slot(valid && alive && dirty, slot, dlist, &ctr->n_delta);
  if (valid && !alive) r.cnt[slot] = 0u;
  lds_fence();
}

template <int G, int DG = 0>
__global__ __launch_bounds__(64) void k_merge_group_wide(const uint2* __restrict__ list,
                                                         const uint32_t* count_ptr,
                                                         uint32_t* __restrict__ slots, Decider dc,
                                                         Rows r, Counters* ctr, uint32_t* dlist,
                                                         KTime kt) {
  __shared__ __attribute__((aligned(16))) float tile[64 * ((DG > 0 && G >= 8 ? kWideKC : kWideXKC) + 4)];
  constexpr uint32_t NG = 64 / G;
  kt_begin(kt, KC_SMALL);
  const uint32_t n = __hip_atomic_load(count_ptr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t nb = (n + NG - 1) / NG;
  const uint32_t g = threadIdx.x & (G - 1), grp = threadIdx.x / G;
  for (uint32_t bi = blockIdx.x; bi < nb; bi += gridDim.x) {
    const uint32_t k = bi * NG + grp;
    const uint2 e = k < n ? list[k] : make_uint2(0u, 0u);
    const uint32_t slot = g < e.y ? slots[e.x + g] : 0u;
    merge_batch_wide<G, DG>(e.x, e.y, slot, slots, dc, r, tile, dlist, ctr);
  }
  kt_end(kt, KC_SMALL);
}

// Runs of 65..896 rows with wide rows: one workgroup per run, the decision matrix in LDS in
// position space (as k_merge_big).  A 64x64 decision tile is one wave's job: its 64 rows'
// chains (one per lane, 64 columns each) run over KC-column chunks, the column block's chunk
// staged in the wave's own LDS region and read by broadcast.
template <int RB, int NT, int KC>
struct BigWideLayout {
  static constexpr int W = RB / 64;
  static constexpr int NW = NT / 64;
  static constexpr int STB = KC;  // unpadded: the tile is filled lane-linearly (and read by broadcast)
  static constexpr size_t tiles = 0;
  static constexpr size_t P = tiles + sizeof(float) * NW * 64 * STB;
  static constexpr size_t meta = P + sizeof(uint64_t) * RB * W;
  static constexpr size_t bytes = meta + sizeof(uint32_t) * RB * 8;
};

template <int RB, int NT, int KC>
__global__ __launch_bounds__(NT) void k_merge_big_wide(MergeWork w, int cls,
                                                       uint32_t* __restrict__ slots, Decider dc,
                                                       Rows r, Counters* ctr) {
  using L = BigWideLayout<RB, NT, KC>;
  const uint2* __restrict__ list = w.big[cls];
  uint32_t* const dlist = w.dlist;
  RunCounters* const rc = w.rc;
  const KTime kt = w.kt;
  kt_begin(kt, KC_BIG128 + cls);
  constexpr int W = L::W, NW = L::NW, STB = L::STB;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint64_t* P = reinterpret_cast<uint64_t*>(smem + L::P);
  uint32_t* slot = reinterpret_cast<uint32_t*>(smem + L::meta);
  float* nrm = reinterpret_cast<float*>(slot + RB);
  uint32_t* cnt = slot + 2 * RB;
  uint32_t* hd = slot + 3 * RB;
  uint32_t* tl = slot + 4 * RB;
  uint32_t* pos2row = slot + 5 * RB;
  float* sq = reinterpret_cast<float*>(slot + 6 * RB);
  __shared__ uint32_t wbuf[2 * NW];
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  float* ctile = reinterpret_cast<float*>(smem + L::tiles) + wv * 64 * STB;  // this wave's
  const int d = r.d, dp = r.dp;
  const uint32_t count =
      __hip_atomic_load(&rc->n_big[cls].v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  auto row_ptr = [&](uint32_t a) -> const float* { return r.x + (size_t)slot[a] * dp; };

  for (uint32_t li = blockIdx.x; li < count; li += gridDim.x) {
    const uint2 e = list[li];
    const uint32_t p = e.x, b = e.y;
    const uint32_t nblk = (b + 63) / 64;
    [[maybe_unused]] const uint64_t pt0 = MPROF_T();
    for (uint32_t a = t; a < b; a += NT) {
      const uint32_t s = slots[p + a];
      slot[a] = s;
      nrm[a] = r.nrm[s];
      sq[a] = __builtin_sqrtf(nrm[a]);
      cnt[a] = r.cnt[s];
      hd[a] = r.head[s];
      tl[a] = r.tail[s];
      pos2row[a] = a;
    }
    for (uint32_t a = t; a < b * (uint32_t)W; a += NT) P[a] = 0ull;
    __syncthreads();

    // decision tiles (R, C <= R), one per wave at a time
    const uint32_t ntiles = nblk * (nblk + 1) / 2;
    for (uint32_t ti = wv; ti < ntiles; ti += NW) {
      uint32_t R = 0;
      while ((R + 1) * (R + 2) / 2 <= ti) ++R;
      const uint32_t C = ti - R * (R + 1) / 2;
      const uint32_t a = R * 64u + lane;
      const bool va = a < b;
      const float* xa = row_ptr(va ? a : 0u);  // (a lane past the run reads row 0, unused)
      const uint32_t c0 = C * 64u, c1 = min(b, c0 + 64u);
      float acc[64];
#pragma unroll
      for (int c = 0; c < 64; ++c) acc[c] = 0.0f;
      for (int k0 = 0; k0 < d; k0 += KC) {
        const int n = min(KC, d - k0), kcp = min(KC, dp - k0);
        lds_fence();
        if (kcp == KC) {
          // a full chunk straight into LDS (global_load_lds, 16 B a lane: the tile is unpadded, so
          // instruction i fills floats [256 i, 256 i + 256) lane-linearly) — no registers, every
          // load in flight at once; rows past the run read row c0 (never read back)
          constexpr uint32_t PER = KC / 4;
#pragma unroll
          for (uint32_t i = 0; i < PER; ++i) {
            const uint32_t q = lane + 64u * i, row = q / PER, e4 = q % PER;
            const uint32_t sr = slot[c0 + row < c1 ? c0 + row : c0];
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)(r.x + (size_t)sr * dp + k0 + 4 * e4),
                (__attribute__((address_space(3))) void*)(ctile + 256u * i), 16, 0, 0);
          }
          __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the tile has landed
        } else {
          for (uint32_t q = lane; q < 64u * (uint32_t)(kcp / 4); q += 64) {
            const uint32_t row = q / (uint32_t)(kcp / 4), e4 = q % (uint32_t)(kcp / 4);
            if (c0 + row < c1)
              *reinterpret_cast<float4*>(ctile + row * STB + 4 * e4) =
                  *reinterpret_cast<const float4*>(r.x + (size_t)slot[c0 + row] * dp + k0 + 4 * e4);
          }
        }
        lds_fence();
        if (n == KC) {
          float x[KC];
#pragma unroll
          for (int k = 0; k < KC; k += 4) {
            float4 v = *reinterpret_cast<const float4*>(xa + k0 + k);
            if (!va) v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            x[k] = v.x; x[k + 1] = v.y; x[k + 2] = v.z; x[k + 3] = v.w;
          }
#pragma unroll
          for (int c = 0; c < 64; ++c)
            if (c0 + c < c1) acc[c] = dot_acc_reg<KC>(acc[c], x, ctile + c * STB);
        } else {
#pragma unroll
          for (int c = 0; c < 64; ++c)
            if (c0 + c < c1 && va) {
              float s = acc[c];
              for (int k = 0; k < n; ++k) s = s + xa[k0 + k] * ctile[c * STB + k];
              acc[c] = s;
            }
        }
      }
      const float sa = va ? sq[a] : 0.0f;
      uint64_t own = 0ull;
#pragma unroll
      for (int c = 0; c < 64; ++c) {
        const uint32_t cc = c0 + c;
        if (cc < c1) {  // wave-uniform
          const bool h = va && cc < a && decide(dc, acc[c], sa * sq[cc]);
          const uint64_t m = __ballot(h);
          if (lane == 0 && m) atomicOr((unsigned long long*)&P[cc * W + R], (unsigned long long)m);
          own |= (h ? 1ull : 0ull) << c;
        }
      }
      if (va && own) atomicOr((unsigned long long*)&P[a * W + C], (unsigned long long)own);
    }
    __syncthreads();

    big_walk<RB, NT, false>(p, b, P, slot, nrm, cnt, hd, tl, pos2row, sq, nullptr, 0,
                     reinterpret_cast<float*>(smem + L::tiles), wbuf, r, dc, slots, dlist, ctr);
    __syncthreads();
  }
  if constexpr (RB == kBigRows[kBigClasses - 1]) {
    if (w.huge_fold) {  // the >896-row runs too (see k_merge_big)
      const uint32_t nh =
          __hip_atomic_load(&w.rc->n_huge.v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      huge_runs<0, NT>(w.huge, nh, blockIdx.x, gridDim.x, slots, dc, r, w, ctr, smem);
    }
  }
  kt_end(kt, KC_BIG128 + cls);
}

// ----------------------------------------------------------------------------- launch -----
// The smallest float s with fl(1 - fl(1 - s)) >= thr (cluster.cc:68-69), by bisection over the
// ordered floats; see Decider.
static float sim_roundtrip(float s) {
  volatile float dist = 1.0f - s;
  volatile float sim = 1.0f - dist;
  return sim;
}
static uint32_t ordered(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
static float from_ordered(uint32_t o) {
  const uint32_t u = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

Decider make_decider(float thr) {
  Decider dc{std::numeric_limits<float>::quiet_NaN(), 0.0f, 0.0f, 0u, 0.0f, 0.0f};
  uint32_t lo = ordered(-std::numeric_limits<float>::infinity());
  uint32_t hi = ordered(std::numeric_limits<float>::infinity());
  if (!(sim_roundtrip(from_ordered(hi)) >= thr)) return dc;  // nothing passes (thr NaN)
  while (lo < hi) {  // invariant: hi passes
    const uint32_t mid = lo + (hi - lo) / 2;
    if (sim_roundtrip(from_ordered(mid)) >= thr) hi = mid;
    else lo = mid + 1;
  }
  dc.s_star = from_ordered(hi);
  if (dc.s_star >= 0x1p-60f && dc.s_star <= 0x1p60f) {
    dc.s_lo = from_ordered(hi - 8);
    dc.s_hi = from_ordered(hi + 8);
    dc.fast = 1u;
    dc.g_lo = dc.s_star - kGramMargin;
    dc.g_hi = dc.s_star + kGramMargin;
  }
  return dc;
}

template <int D, int RB, int NT, bool ROWS_LDS>
static void launch_big(const MergeWork& w, int c, uint32_t* slots, const Decider& dc, const Rows& r,
                       Counters* ctr, uint32_t n, hipStream_t s) {
  using L = BigLayout<D, RB, ROWS_LDS>;
  const bool fold = RB == kBigRows[kBigClasses - 1] && w.huge_fold;
  const size_t lds = fold ? std::max(L::bytes, huge_lds(D, r.dp, NT)) : L::bytes;
  static const bool lds_ok = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&k_merge_big<D, RB, NT, ROWS_LDS>),
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)std::max<size_t>(L::bytes, 96 * 1024)) == hipSuccess;
  }();
  (void)lds_ok;
  const uint32_t lo = c == 0 ? 65u : (uint32_t)kBigRows[c - 1] + 1u;
  const uint32_t g = (uint32_t)std::min<uint64_t>(1024, n / lo + 1);
  k_merge_big<D, RB, NT, ROWS_LDS><<<g, NT, lds, s>>>(w, c, slots, dc, r, ctr);
}

// Fork the size-class kernels onto the auxiliary streams (after k_runs on s) and join them back
// into s.  Every class writes disjoint runs, so the order between classes is free.
struct Fork {
  const MergeWork& w;
  hipStream_t s;
  bool on;
  Fork(const MergeWork& w_, hipStream_t s_) : w(w_), s(s_) {
#ifdef KLSH_SERIAL_MERGE  // diagnostics build only: every class in order on the main stream
    on = false;
#else
    on = w.aux[0] != nullptr;
#endif
    if (!on) return;
    (void)hipEventRecord(w.fork, s);
    for (int i = 0; i < kMergeStreams; ++i) (void)hipStreamWaitEvent(w.aux[i], w.fork, 0);
  }
  hipStream_t lane(int i) const { return on ? w.aux[i] : s; }
  ~Fork() {
    if (!on) return;
    for (int i = 0; i < kMergeStreams; ++i) {
      (void)hipEventRecord(w.join[i], w.aux[i]);
      (void)hipStreamWaitEvent(s, w.join[i], 0);
    }
  }
};

// The small-run screen's margin (k_small_screen): |q~ - q_ref| <= m0 + a2 (1/|x~a| + 1/|x~b|) for
// the screen's quotient q~ = x~a.x~b / (|x~a| |x~b|) against the reference's fl(dot / den):
//   m0: fp16 rounding of both rows in the dot (2 * 2^-11) and in the two norms (2 * 2^-11),
//       2^-20 for the products of the rounding errors, (4d + 16) 2^-24 for the f32 sums of the
//       screen and of the reference (dot, |a|^2, |b|^2) and the sqrt / product / quotient roundings
//   a2: 2^-25 per element absolute (fp16 subnormals, which gfx950 keeps in the conversion, the
//       MFMA and v_dot2_f32_f16 under the default float mode: tools/denorm_probe.hip), summed with
//       Cauchy-Schwarz: sqrt(d) 2^-25 (|a| + |b|) / (|a||b|), doubled (the norms' own share)
// all times 1.5 for headroom.  Only with a fast decider (a normal s*) and the fp16 image.
static void screen_margins(int d, float* m0, float* a2) {
  *m0 = 1.5f * (0x1p-9f + 0x1p-20f + (4.0f * (float)d + 16.0f) * 0x1p-24f);
  *a2 = 1.5f * 2.0f * 0x1p-25f * std::sqrt((float)d);
}
static bool screen_ok(const Rows& r, const Decider& dc, const MergeWork& w) {
  return w.small_screen && r.xh && dc.fast && (r.d == 32 || r.d == 64);  // (tiles: d >= 32)
}

// The small-run merge's persistent launch (option "small_grid"; default 12288).
static uint32_t small_grid(const MergeWork& w) {
  return w.small_grid ? std::max(256u, w.small_grid) : 12288u;
}

// Iterations below this many positions run every merge class in ONE launch (k_merge_tail) on the
// main stream: there the cross-stream fork/join (~35 us) costs more than the overlap buys.

template <int D>
static void launch_groups(const Rows& r, uint32_t* slots, const Decider& dc, const MergeWork& w,
                          Counters* ctr, uint32_t n, hipStream_t s) {
  if (n < tail_merge_max(w)) {
    using L896 = BigLayout<D, 896, false>;
    using L384 = BigLayout<D, 384, true>;
    using L192 = BigLayout<D, 192, true>;
    using L128 = BigLayout<D, 128, true>;
    constexpr size_t small_lds = 4 * 64 * (D + 4) * sizeof(float);
    const size_t lds = std::max({L896::bytes, L384::bytes, L192::bytes, L128::bytes, small_lds,
                                 huge_lds(D, r.dp, 256)});
    static const bool lds_ok =
        hipFuncSetAttribute(reinterpret_cast<const void*>(&k_merge_tail<D>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess;
    (void)lds_ok;
    // options "tail_big_groups" / "tail_small_groups": 32 / 64 / 128 / 256 and 128 / 256 / 512 /
    // 1024 swept (round 3)
    const uint32_t nbig = w.tail_nbig ? w.tail_nbig : 128u;
    const uint32_t nsmall = w.tail_nsmall ? w.tail_nsmall : 512u;
    MergeWork wt = w;
    wt.big_screen = 0u;
    if (w.tail_big_screen && screen_ok(r, dc, w)) {
      screen_margins(r.d, &wt.bs_m0, &wt.bs_a2);
      wt.bs_s_star = dc.s_star;
      wt.big_screen = 1u;
    }
    if (w.tail_screen && screen_ok(r, dc, w)) {
      // the fp16 screen of the small runs first (few of them merge this late in the loop), on
      // the same stream: k_merge_tail's small-run waves then take only the runs it passed
      float m0, a2;
      screen_margins(r.d, &m0, &a2);
      // (option tail_screen_grid; one box, interleaved C2: 512 → 214.9, 1024 → 210.0, 2048 →
      // 208.1 ms per step; tail_screen = 0: 213.3 ms)
      const uint32_t sgrid = w.tail_screen_grid ? std::max(64u, w.tail_screen_grid) : 2048u;
      k_small_screen<D><<<sgrid, 64, 0, s>>>(w, slots, r, dc.s_star, m0, a2, w.kt);
      wt.screened = 1u;
    }
    k_merge_tail<D><<<nbig + nsmall, 256, lds, s>>>(wt, slots, dc, r, ctr, nbig);
    return;
  }
  const Fork f(w, s);
  // The small-run chain (screen + merge: the merge phase's critical path in 146 of C2's 218
  // multi-launch iterations, rocprofv3 trace) on the main stream: it starts without the fork's
  // cross-stream wait, and at the join only the aux streams are waited for; the >384-row classes
  // on aux 2 (C2, one box, interleaved: 203.9 -> 200.8 ms per step).  Not when the previous
  // iteration had many 385..896-row runs (w.big896_aux, C4): the long walks are the critical
  // path there and keep the main stream (C4 989 -> 1120 ms with the small chain on it).
  const bool long_heavy = w.big896_aux != 0u;
  const hipStream_t s_small = long_heavy ? f.lane(2) : s, s_long = long_heavy ? s : f.lane(2);
  // longest walks first on each stream; the longest runs (few, long walks) on the main stream,
  // concurrent with the auxiliary ones (it waits for them at the join)
  launch_big<D, 384, 256, true>(w, 2, slots, dc, r, ctr, n, f.lane(0));
  // many 385..896-row runs (w.big896_aux): they go on aux 2, ahead of the small runs, instead of
  // in front of the >896-row runs on the main stream — serialised, the two long-walk classes
  // make the main stream the critical path (C4 1794 -> 1432 ms); with a handful of them (C2)
  // the main stream is the better place (measured 281-285 vs 284-294 ms)
  if (!long896(w, dc, r))
    launch_big<D, 896, 256, false>(w, 3, slots, dc, r, ctr, n, w.big896_aux ? f.lane(2) : s_long);
  launch_huge(w, slots, dc, r, ctr, n, s_long);
  // 129..192 rows: two workgroups per CU (62 KB of LDS at d = 64, VGPRs capped at 256 like the
  // 65..128 class), ahead of 65..128 on aux 1
  launch_big<D, 192, 256, true>(w, 1, slots, dc, r, ctr, n, f.lane(1));
  launch_big<D, 128, 128, true>(w, 0, slots, dc, r, ctr, n, f.lane(1));
  // every small-run class in one persistent launch (the kernel strides over its batches)
  // HIP events on its own stream too (bench.py's headline cross-check: this launch is alone on
  // aux 2, so the event pair measures it, unlike the big-run classes that wait for CU resources)
  // 12288 one-wave workgroups, 6 per resident slot (2048 at 2 waves per SIMD): the batch stride
  // of a persistent wave is long enough that its rows come from all over the lists, and waves
  // retire and re-enter as the big-run workgroups come and go (C2, same box, interleaved:
  // 4608 -> 255.9 / 258.0 ms, 8192 -> 255.4 / 252.3, 12288 -> 250.8 / 251.7, 16384 -> 256.0 /
  // 253.9; small-run merge 79.4 -> 70.5 ms per step)
  // the fp16 screen first (option small_screen, where the row image exists): the merge then
  // takes only the runs it could not rule out
  if (screen_ok(r, dc, w)) {
    float m0, a2;
    screen_margins(r.d, &m0, &a2);
    // (option small_screen_grid; one-wave workgroups: 2048 → 207.9 / 207.8 vs 3072 → 211.2 /
    // 211.1 ms per C2 step on one box, 1024 → 227–228, 1536 / 2560 within noise of 2048)
    const uint32_t sgrid = w.screen_grid ? std::max(64u, w.screen_grid) : 2048u;
    k_small_screen<D><<<sgrid, 64, 0, s_small>>>(w, slots, r, dc.s_star, m0, a2, w.kt);
    MergeWork ws = w;
    ws.screened = 1u;
    if (w.small_ev[0]) (void)hipEventRecord(w.small_ev[0], s_small);
    k_merge_small<D><<<small_grid(w), 64, 0, s_small>>>(ws, slots, dc, r, ctr);
  } else {
    if (w.small_ev[0]) (void)hipEventRecord(w.small_ev[0], s_small);
    k_merge_small<D><<<small_grid(w), 64, 0, s_small>>>(w, slots, dc, r, ctr);
  }
  if (w.small_ev[0]) (void)hipEventRecord(w.small_ev[1], s_small);
}

template <int RB, int NT, int KC>
static void launch_big_wide(const MergeWork& w, int c, uint32_t* slots, const Decider& dc,
                            const Rows& r, Counters* ctr, uint32_t n, hipStream_t s) {
  using L = BigWideLayout<RB, NT, KC>;
  const bool fold = RB == kBigRows[kBigClasses - 1] && w.huge_fold;
  const size_t lds = fold ? std::max(L::bytes, huge_lds(r.d, r.dp, NT)) : L::bytes;
  static const bool lds_ok = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&k_merge_big_wide<RB, NT, KC>),
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)std::max<size_t>(L::bytes, 96 * 1024)) == hipSuccess;
  }();
  (void)lds_ok;
  const uint32_t lo = c == 0 ? 65u : (uint32_t)kBigRows[c - 1] + 1u;
  const uint32_t g = (uint32_t)std::min<uint64_t>(1024, n / lo + 1);
  k_merge_big_wide<RB, NT, KC><<<g, NT, lds, s>>>(w, c, slots, dc, r, ctr);
}

// |G - dot_ref| / (|a||b|) for the bf16x3 Gram value at width d against the reference's sequential
// f32 dot: split residuals 3.03 * 2^-16, the MFMA's f32 sums (16 internal adds + one per chained
// MFMA, three per k-step, at 2u), the reference's own (d + 1) * 2^-24 and the approximate quotient
// (4 * 2^-24), with 1.5x headroom (kGramMargin, 1e-4, covers d <= 64; at d = 512 this is 1.37e-4).
static float wide_gram_margin(int d) {
  const float ks = (float)((d + 15) / 16);
  return 1.5f * (3.03f * 0x1p-16f + (17.0f + 3.0f * ks) * 0x1p-23f + (float)(d + 1) * 0x1p-24f +
                 4.0f * 0x1p-24f);
}

static void launch_groups_wide(const Rows& r, uint32_t* slots, const Decider& dc,
                               const MergeWork& w, Counters* ctr, uint32_t n, hipStream_t s) {
  auto grid = [&](int c, uint32_t per_wave) {
    // up to 8192 one-wave workgroups per class (was 2048: C5 2.58 / 2.55 -> 2.36 / 2.33 s per
    // step, interleaved on one box), as for the register-row small-run launch
    // option "wide_group_grid": 4096 -> 1221, 8192 -> 1141, 16384 -> 1103, 32768 -> 1102 ms
    // per C5 step (one box)
    const uint64_t cap = w.wide_group_grid ? std::max(64u, w.wide_group_grid) : 16384u;
    return (uint32_t)std::min<uint64_t>(cap, group_class_capacity(c, n) / per_wave + 1);
  };
  const Fork f(w, s);
  launch_big_wide<384, 256, 32>(w, 2, slots, dc, r, ctr, n, f.lane(0));
  launch_big_wide<384, 256, 32>(w, 1, slots, dc, r, ctr, n, f.lane(0));  // 129..192 rows
  launch_big_wide<896, 256, 16>(w, 3, slots, dc, r, ctr, n, f.on ? s : f.lane(0));
  launch_huge(w, slots, dc, r, ctr, n, f.on ? s : f.lane(0));
  launch_big_wide<128, 128, 32>(w, 0, slots, dc, r, ctr, n, f.lane(1));
  // the small-run classes (runs of 2..64 rows), each a persistent launch of up to 16384
  // one-wave workgroups
  RunCounters* rc = w.rc;
  const hipStream_t sl = f.lane(2);
  // (an fp16-image screen of these runs, k_small_screen_wide, ruled out 96 % of C5's small-run
  // rows and still cost more than it saved — 2.25 -> 2.78 s per step — and was removed in round 5)
  // runs of 8..64 rows at d = 512 (C5): pairwise decisions on the matrix cores (option
  // wide_gram) with the margin of the bf16x3 Gram value at this width (wide_gram_margin)
  const bool gram = w.wide_gram && dc.fast && r.d == 512;
  const uint32_t gmin = w.wide_gram;  // the smallest group width that decides on the matrix cores
  Decider dg = dc;
  if (gram) {
    const float m = wide_gram_margin(r.d);
    dg.g_lo = dc.s_star - m;
    dg.g_hi = dc.s_star + m;
  }
  // The six classes on four streams, not one chain (each class's launch ends with a tail of
  // latency-bound walks that leaves the chip idle, and the classes' register budgets differ, so
  // two of them share a SIMD's register file): the main stream takes 64 (behind the short
  // 385..896-row class), aux 0 32 (behind the 129..384-row classes), aux 1 8 and 4 (behind the
  // 65..128-row class), aux 2 16 and 2.  C5, interleaved on one box: one chain 1896 / 1898 ms,
  // this 1733 / 1736 (1691 / 1716 on a second box, where two other assignments measured
  // 1679–1713 ms).  Index: 5 - class (64, 32, 16, 8, 4, 2).
  const hipStream_t gs[6] = {s, f.lane(0), sl, f.lane(1), f.lane(1), sl};
  auto group = [&](auto kern, int c, uint32_t per_wave, const Decider& dd) {
    kern<<<grid(c, per_wave), 64, 0, gs[5 - c]>>>(w.cls[c], &rc->n_cls[c].v, slots, dd, r, ctr,
                                                   w.dlist, w.kt);
  };
  if (gram && gmin <= 64) group(k_merge_group_wide<64, 512>, 5, 1, dg);
  else group(k_merge_group_wide<64>, 5, 1, dc);
  if (gram && gmin <= 32) group(k_merge_group_wide<32, 512>, 4, 2, dg);
  else group(k_merge_group_wide<32>, 4, 2, dc);
  if (gram && gmin <= 16) group(k_merge_group_wide<16, 512>, 3, 4, dg);
  else group(k_merge_group_wide<16>, 3, 4, dc);
  if (gram && gmin <= 8) group(k_merge_group_wide<8, 512>, 2, 8, dg);
  else group(k_merge_group_wide<8>, 2, 8, dc);
  group(k_merge_group_wide<4>, 1, 16, dc);
  group(k_merge_group_wide<2>, 0, 32, dc);
}

void launch_runs(const uint32_t* key, uint32_t lo, uint32_t n, int bucket_thr, const MergeWork& w,
                 hipStream_t s, const uint32_t* n_dev) {
  const uint32_t ntiles = (n + kRunTile - 1) / kRunTile;
  // run_ws: counts [kRunRows][ntiles], tail ends [ntiles], then 8-byte aligned: first / last
  // heads (uint2) [ntiles], head bitmaps [ntiles][64]
  uint32_t* counts = w.run_ws;
  uint32_t* tail_ends = counts + (size_t)kRunRows * ntiles;
  uint2* heads_fl = reinterpret_cast<uint2*>(counts + (((kRunRows + 1u) * ntiles + 1u) & ~1u));
  uint64_t* hbits = reinterpret_cast<uint64_t*>(heads_fl + ntiles);
  k_runs_count<<<ntiles, 256, 0, s>>>(key, lo, n, bucket_thr, ntiles, hbits, heads_fl, counts,
                                      w.kt, n_dev);
  const bool fused = ntiles <= 256u;  // the write kernel scans the counts itself
  if (fused) {
    k_runs_write<true><<<ntiles, 256, 0, s>>>(lo, n, bucket_thr, ntiles, hbits, heads_fl,
                                              tail_ends, counts, w, n_dev);
  } else {
    k_runs_scan<<<kRunRows, 256, 0, s>>>(counts, ntiles, n, bucket_thr, heads_fl, tail_ends, w.rc);
    k_runs_write<false><<<ntiles, 256, 0, s>>>(lo, n, bucket_thr, ntiles, hbits, heads_fl,
                                               tail_ends, counts, w, nullptr);
  }
}

void launch_tail_local(const uint32_t* kin, const uint32_t* vin, uint32_t* kout, uint32_t* vout,
                       const uint32_t* dtot, int bits, int bucket_thr, const MergeWork& w,
                       hipStream_t s) {
  k_tail_local<<<1u << kTailTopBits, 256, 0, s>>>(kin, vin, kout, vout, dtot, bits - kTailTopBits,
                                                   bucket_thr, w);
}

void launch_merge(const Rows& r, const uint32_t* key, uint32_t* slots, uint32_t lo, uint32_t hi,
                  float thr, int bucket_thr, const MergeWork& w, Counters* ctr, hipStream_t s,
                  const uint32_t* n_dev, bool runs_ready) {
  if (hi <= lo) return;
  const uint32_t n = hi - lo;
  if (n_dev && (lo != 0 || n >= tail_merge_max(w))) return;  // (the caller checks)
  const Decider dc = make_decider(thr);
  if (!runs_ready) launch_runs(key, lo, n, bucket_thr, w, s, n_dev);
  // the merge phase of a multi-launch iteration is stamped as a whole too (KC_MERGE: the wall of
  // its concurrent classes, bench.py's roofline phases)
  MergeWork wm = w;
  if (w.kt.blk && (n >= tail_merge_max(w) || !project_device_n_ok(r.d))) wm.kt.phase = KC_MERGE;
  switch (r.d) {
    case 8: launch_groups<8>(r, slots, dc, wm, ctr, n, s); break;
    case 16: launch_groups<16>(r, slots, dc, wm, ctr, n, s); break;
    case 32: launch_groups<32>(r, slots, dc, wm, ctr, n, s); break;
    case 64: launch_groups<64>(r, slots, dc, wm, ctr, n, s); break;
    default: launch_groups_wide(r, slots, dc, wm, ctr, n, s);
  }
}


// Prints and clears the merge profile (diagnostics build only; a no-op otherwise).
void merge_prof_dump(FILE* f) {
#ifdef KLSH_MERGE_PROF
  unsigned long long h[8][12];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_mprof), sizeof(h)) != hipSuccess) return;
  const char* names[kBigClasses + 1] = {"big128", "big192", "big384", "big896", "huge"};
  for (int c = 0; c <= kBigClasses; ++c)
    if (h[c][0])
      fprintf(f, "[mprof] %-7s runs %8llu rows %10llu merges %9llu  load+tiles %9.3f ms  walk %9.3f ms"
                 "  (per run %7.2f + %7.2f us)  max run %8.2f us  max b %llu\n",
              names[c], h[c][0], h[c][1], h[c][2], h[c][3] * 1e-5, h[c][4] * 1e-5,
              h[c][3] * 1e-2 / h[c][0], h[c][4] * 1e-2 / h[c][0], h[c][5] * 1e-2, h[c][6]);
  for (int c = 0; c <= kBigClasses; ++c)
    if (h[c][0])
      fprintf(f, "[mprof] %-7s per run: loads %7.2f  +norms %7.2f  (cum) us;  walk loop %7.2f us\n",
              names[c], h[c][8] * 1e-2 / h[c][0], h[c][9] * 1e-2 / h[c][0], h[c][10] * 1e-2 / h[c][0]);
  unsigned long long wpf[8][8];
  if (hipMemcpyFromSymbol(wpf, HIP_SYMBOL(g_wprof), sizeof(wpf)) == hipSuccess)
    for (int c = 0; c < kBigClasses; ++c)
      if (wpf[c][4])
        fprintf(f, "[wprof] %-7s steps %9llu  clocks/step: find|select %7.0f  select+consensus|consensus %7.0f"
                   "  dots %7.0f  bits %7.0f   find rounds/step|barrier clocks %.2f\n",
                names[c], wpf[c][4], (double)wpf[c][0] / wpf[c][4], (double)wpf[c][1] / wpf[c][4],
                (double)wpf[c][2] / wpf[c][4], (double)wpf[c][3] / wpf[c][4],
                (double)wpf[c][5] / wpf[c][4]);
  unsigned long long spf[8][8];
  if (hipMemcpyFromSymbol(spf, HIP_SYMBOL(g_sprof), sizeof(spf)) == hipSuccess)
    for (int c = 1; c < 6; ++c)
      if (spf[c][0])
        fprintf(f, "[sprof] G=%-2d batches %9llu  clocks/batch: stage %7.0f  pairwise %7.0f  walk %7.0f"
                   "  write %7.0f\n", 2 << c, spf[c][0], (double)spf[c][1] / spf[c][0],
                (double)spf[c][2] / spf[c][0], (double)spf[c][3] / spf[c][0], (double)spf[c][4] / spf[c][0]);
  unsigned long long g[8];
  if (hipMemcpyFromSymbol(g, HIP_SYMBOL(g_gprof), sizeof(g)) == hipSuccess && g[7])
    fprintf(f, "[gprof] tiles %llu (gram_tile)  clocks/tile: acc %.0f  decide %.0f;  slow-path tiles %llu:"
               " close pairs %llu (longest lane %.2f per slow tile), exact loop clocks/slow tile %.0f\n",
            g[7], (double)g[3] / g[7], (double)g[4] / g[7], g[0], g[1], (double)g[2] / g[0],
            (double)g[5] / g[0]);
  unsigned long long tq[8];
  if (hipMemcpyFromSymbol(tq, HIP_SYMBOL(g_tprof), sizeof(tq)) == hipSuccess && tq[4])
    fprintf(f, "[tprof] k_tail_local workgroups %llu  per workgroup us: base %.2f  counts %.2f  lists %.2f"
               "  scatter %.2f  (max total %.2f)\n", tq[4], tq[0] * 1e-2 / tq[4], tq[1] * 1e-2 / tq[4],
            tq[2] * 1e-2 / tq[4], tq[3] * 1e-2 / tq[4], tq[5] * 1e-2);
  unsigned long long z[8][12] = {};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_tprof), z, sizeof(tq));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_gprof), z, sizeof(g));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_mprof), z, sizeof(z));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_wprof), z, sizeof(unsigned long long) * 64);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_sprof), z, sizeof(unsigned long long) * 64);
#else
  (void)f;
#endif
}

}  // namespace klsh
