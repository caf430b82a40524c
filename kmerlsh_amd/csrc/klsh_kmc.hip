// Mode B on gfx950: the k-mer table of a set of KMC databases (reference buildKHtable with
// kmc = false, io/ioHT.cc:83-199, over KmcRead / KmcCount, kmer/kmc_reader.cc:26-169).
//
//   k_kmc_decode  one lane per KMC record of a chunk of the .kmc_suf stream: its prefix is the
//                 last LUT entry <= its record index (binary search; the LUT walk of
//                 CKMCFile::ReadNextKmer, kmer/kmc_api/kmc_file.cpp:438-532), its suffix the
//                 record's big-endian bytes, its counter the little-endian ones; records outside
//                 [min_count, max_count] are dropped (rep = all ones).  The k-mer becomes the
//                 reference Kmer's 8-byte image (base i at bits 2i) and its canonical form
//                 rep = (km < twin) ? km : twin in memcmp order (kmer/Kmer.cc:76-187).
//   k_kmc_union   rep -> table slot (open addressing, 64-bit CAS), first[slot] = the smallest
//                 (sample, record) ordinal that listed it
//   k_kmc_count   count[slot] += the record's counter (clamped at 65535 when written out: the
//                 reference's per-step clamp, kmc_reader.cc:105-108, gives the same total)
//   k_kmc_collect occupied slots -> (ordinal low / high words, slot) for the first-appearance order
//   k_kmc_emit    one sample's uint16 column in output order (WriteHT, io/ioHT.cc:30-55)
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "klsh_internal.h"

namespace klsh {

constexpr uint64_t kKmcEmpty = ~0ull;

__device__ __forceinline__ uint64_t kmc_hash(uint64_t k) {  // murmur3 finalizer
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

__device__ __forceinline__ uint64_t reverse_bases(uint64_t v, int k) {
  uint64_t x = v;
  x = ((x >> 2) & 0x3333333333333333ull) | ((x & 0x3333333333333333ull) << 2);
  x = ((x >> 4) & 0x0F0F0F0F0F0F0F0Full) | ((x & 0x0F0F0F0F0F0F0F0Full) << 4);
  x = __builtin_bswap64(x);
  return x >> (64 - 2 * k);
}

__global__ __launch_bounds__(256) void k_kmc_decode(const uint8_t* __restrict__ recs, uint64_t n,
                                                    uint64_t rec0, KmcParams kp,
                                                    const uint64_t* __restrict__ lut,
                                                    uint64_t lut_n, uint64_t* __restrict__ rep,
                                                    uint32_t* __restrict__ cnt,
                                                    uint32_t* __restrict__ n_valid) {
  uint32_t valid = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256ull) {
    const uint64_t r = rec0 + i;
    // largest index with lut[idx] <= r (entries of empty prefixes repeat their successor's value)
    uint64_t lo = 0, hi = lut_n;  // lut[0] = 0 <= r; lut[lut_n - 1] = total + 1 > r
    while (hi - lo > 1) {
      const uint64_t mid = (lo + hi) >> 1;
      if (lut[mid] <= r) lo = mid;
      else hi = mid;
    }
    const uint8_t* p = recs + i * (uint64_t)kp.rec_size;
    uint64_t suf = 0;
    for (uint32_t b = 0; b < kp.sufix_size; ++b) suf = (suf << 8) | p[b];
    uint32_t c = 0;
    for (uint32_t b = 0; b < kp.counter_size; ++b) c |= (uint32_t)p[kp.sufix_size + b] << (8 * b);
    uint64_t key = kKmcEmpty;
    if (c >= kp.min_count && (uint64_t)c <= kp.max_count) {
      const uint64_t pre = lo & kp.prefix_mask;
      const uint64_t v = kp.p == 0 ? suf : (pre << (2 * (kp.k - kp.p))) | suf;  // s[0] on top
      const uint64_t img = reverse_bases(v, kp.k);  // base i at bits 2i
      // the twin's base i is the complement of base k-1-i: exactly the complemented KMC value
      const uint64_t tw = ~v & (kp.k == 32 ? ~0ull : ((1ull << (2 * kp.k)) - 1ull));
      key = __builtin_bswap64(img) < __builtin_bswap64(tw) ? img : tw;
      ++valid;
    }
    rep[i] = key;
    cnt[i] = c;
  }
  // one add per wave
  for (int o = 32; o > 0; o >>= 1) valid += __shfl_xor(valid, o, 64);
  if ((threadIdx.x & 63u) == 0 && valid) atomicAdd(n_valid, valid);
}

__device__ __forceinline__ uint64_t kmc_slot_insert(unsigned long long* tab, uint64_t mask,
                                                    uint64_t key) {
  uint64_t h = kmc_hash(key) & mask;
  while (true) {
    const unsigned long long prev = atomicCAS(&tab[h], (unsigned long long)kKmcEmpty,
                                              (unsigned long long)key);
    if (prev == kKmcEmpty || prev == key) return h;
    h = (h + 1) & mask;
  }
}

__device__ __forceinline__ uint64_t kmc_slot_find(const uint64_t* tab, uint64_t mask, uint64_t key) {
  uint64_t h = kmc_hash(key) & mask;
  while (true) {
    const uint64_t t = tab[h];
    if (t == key) return h;
    if (t == kKmcEmpty) return ~0ull;
    h = (h + 1) & mask;
  }
}

__global__ __launch_bounds__(256) void k_kmc_union(const uint64_t* __restrict__ rep, uint64_t n,
                                                   uint64_t ord0, unsigned long long* tab,
                                                   unsigned long long* first, uint64_t mask) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256ull) {
    const uint64_t key = rep[i];
    if (key == kKmcEmpty) continue;
    const uint64_t h = kmc_slot_insert(tab, mask, key);
    atomicMin(&first[h], (unsigned long long)(ord0 + i));
  }
}

__global__ __launch_bounds__(256) void k_kmc_count(const uint64_t* __restrict__ rep,
                                                   const uint32_t* __restrict__ cnt, uint64_t n,
                                                   const uint64_t* __restrict__ tab, uint64_t mask,
                                                   uint32_t* __restrict__ acc) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256ull) {
    const uint64_t key = rep[i];
    if (key == kKmcEmpty) continue;
    const uint64_t h = kmc_slot_find(tab, mask, key);
    if (h != ~0ull) atomicAdd(&acc[h], min(cnt[i], 65535u));  // a sum past 65535 is clamped later
  }
}

__global__ __launch_bounds__(256) void k_kmc_collect(const uint64_t* __restrict__ tab,
                                                     const uint64_t* __restrict__ first,
                                                     uint64_t cap, uint32_t* __restrict__ lo,
                                                     uint32_t* __restrict__ slot,
                                                     uint32_t* __restrict__ n_out) {
  // cap is a power of two >= 1024: every wave's 64 lanes are in or out of range together
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t below = lane ? (~0ull >> (64u - lane)) : 0ull;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < cap; i += (uint64_t)gridDim.x * 256ull) {
    const bool occ = tab[i] != kKmcEmpty;
    const uint64_t m = __ballot(occ);
    if (!m) continue;
    uint32_t base = 0;  // one add per wave, not per entry (a single counter)
    if (lane == (uint32_t)__builtin_ctzll(m)) base = atomicAdd(n_out, (uint32_t)__popcll(m));
    base = __shfl(base, (int)__builtin_ctzll(m), 64);
    if (occ) {
      const uint32_t o = base + (uint32_t)__popcll(m & below);
      lo[o] = (uint32_t)first[i];
      slot[o] = (uint32_t)i;
    }
  }
}

// hi[i] = high word of the first-appearance ordinal of slot slots[i]
__global__ __launch_bounds__(256) void k_kmc_hi(const uint64_t* __restrict__ first,
                                                const uint32_t* __restrict__ slots, uint64_t n,
                                                uint32_t* __restrict__ hi) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256ull)
    hi[i] = (uint32_t)(first[slots[i]] >> 32);
}

__global__ __launch_bounds__(256) void k_kmc_emit_keys(const uint64_t* __restrict__ tab,
                                                       const uint32_t* __restrict__ order,
                                                       uint64_t n, uint64_t* __restrict__ out) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256ull)
    out[i] = tab[order[i]];
}

__global__ __launch_bounds__(256) void k_kmc_emit(const uint32_t* __restrict__ acc,
                                                  const uint32_t* __restrict__ order, uint64_t n,
                                                  uint16_t* __restrict__ out) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256ull)
    out[i] = (uint16_t)min(acc[order[i]], 65535u);
}

static uint32_t grid_for(uint64_t n) {
  const uint64_t g = (n + 255) / 256;
  return (uint32_t)(g < 16384 ? (g ? g : 1) : 16384);
}

void launch_kmc_decode(const uint8_t* recs, uint64_t n, uint64_t rec0, const KmcParams& kp,
                       const uint64_t* lut, uint64_t lut_n, uint64_t* rep, uint32_t* cnt,
                       uint32_t* n_valid, hipStream_t s) {
  if (n) k_kmc_decode<<<grid_for(n), 256, 0, s>>>(recs, n, rec0, kp, lut, lut_n, rep, cnt, n_valid);
}
void launch_kmc_union(const uint64_t* rep, uint64_t n, uint64_t ord0, uint64_t* tab,
                      uint64_t* first, uint64_t mask, hipStream_t s) {
  if (n)
    k_kmc_union<<<grid_for(n), 256, 0, s>>>(rep, n, ord0, reinterpret_cast<unsigned long long*>(tab),
                                            reinterpret_cast<unsigned long long*>(first), mask);
}
void launch_kmc_count(const uint64_t* rep, const uint32_t* cnt, uint64_t n, const uint64_t* tab,
                      uint64_t mask, uint32_t* acc, hipStream_t s) {
  if (n) k_kmc_count<<<grid_for(n), 256, 0, s>>>(rep, cnt, n, tab, mask, acc);
}
void launch_kmc_collect(const uint64_t* tab, const uint64_t* first, uint64_t cap, uint32_t* lo,
                        uint32_t* slot, uint32_t* n_out, hipStream_t s) {
  k_kmc_collect<<<grid_for(cap), 256, 0, s>>>(tab, first, cap, lo, slot, n_out);
}
void launch_kmc_hi(const uint64_t* first, const uint32_t* slots, uint64_t n, uint32_t* hi,
                   hipStream_t s) {
  if (n) k_kmc_hi<<<grid_for(n), 256, 0, s>>>(first, slots, n, hi);
}
void launch_kmc_emit_keys(const uint64_t* tab, const uint32_t* order, uint64_t n, uint64_t* out,
                          hipStream_t s) {
  if (n) k_kmc_emit_keys<<<grid_for(n), 256, 0, s>>>(tab, order, n, out);
}
void launch_kmc_emit(const uint32_t* acc, const uint32_t* order, uint64_t n, uint16_t* out,
                     hipStream_t s) {
  if (n) k_kmc_emit<<<grid_for(n), 256, 0, s>>>(acc, order, n, out);
}

}  // namespace klsh
