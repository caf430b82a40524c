// Mode E on gfx950: the differential k-mer sets and the per-read k-mer vote of read extraction.
//
// Reference: IOFQ::CheckRead (io/ioFastQ.cc:5-76) walks every read k-mer by k-mer
// (Kmer::forwardBase, kmer/Kmer.cc:210-237), takes the canonical form
// rep = (km < km.twin()) ? km : km.twin() (operator< = memcmp of the 8 bytes, kmer/Kmer.cc:76-78;
// twin = reverse complement, :150-187), looks it up in an unordered_set<Kmer> and keeps the read
// when hits / (len - k + 1) > kmer_vote (float arithmetic), for reads of at least k + 10 bases.
//
// Here a k-mer is the 64-bit little-endian image of the reference's 8 bytes: base i at bits
// [2i, 2i+2), A/C/G/T = 0/1/2/3 and every other character 0 (Kmer::set_kmer's switch, :115-135).
// memcmp order of the bytes is the order of the byte-swapped word.
//
//   k_kset_insert  open-addressing table (linear probing, 64-bit CAS), the set's k-mers as read
//                  from kmer_set.hex; the all-ones word is the empty marker (never a canonical
//                  rep: the all-T k-mer's twin is 0)
//   k_check_reads  one wave per read: the read's bases staged as 2-bit codes in LDS (one byte
//                  each), one lane per k-mer position building its word from LDS, reverse
//                  complement with bit operations, one probe sequence per lane, a wave sum of the
//                  hits; reads longer than the LDS window are walked in windows
//
// Bound: the probes.  One random 8-B table read (64-B line) per k-mer position; the sequence is
// read once (1 B per base).  A set of a few million k-mers (2x capacity, 8 B per slot) is tens of
// MB and stays in L2 / MALL, so the kernel is latency- not HBM-bound at realistic sizes.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "klsh_internal.h"

namespace klsh {

constexpr uint64_t kKsetEmpty = ~0ull;
constexpr int kCheckWaves = 4;        // waves per workgroup, each on its own reads
constexpr uint32_t kCheckWindow = 2048;  // k-mer positions per LDS window (per wave)

__device__ __forceinline__ uint64_t fmix64(uint64_t k) {  // murmur3 finalizer
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

__global__ __launch_bounds__(256) void k_kset_insert(const uint64_t* __restrict__ kmers, uint64_t n,
                                                     unsigned long long* __restrict__ tab,
                                                     uint64_t mask) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256ull) {
    const unsigned long long key = kmers[i];
    if (key == kKsetEmpty) continue;  // cannot be a canonical rep: never looked up
    uint64_t h = fmix64(key) & mask;
    while (true) {
      const unsigned long long prev = atomicCAS(&tab[h], (unsigned long long)kKsetEmpty, key);
      if (prev == kKsetEmpty || prev == key) break;
      h = (h + 1) & mask;
    }
  }
}

// reverse complement of the k-base word v (bases in bits [0, 2k))
__device__ __forceinline__ uint64_t revcomp(uint64_t v, int k) {
  uint64_t x = ~v;
  x = ((x >> 2) & 0x3333333333333333ull) | ((x & 0x3333333333333333ull) << 2);
  x = ((x >> 4) & 0x0F0F0F0F0F0F0F0Full) | ((x & 0x0F0F0F0F0F0F0F0Full) << 4);
  x = __builtin_bswap64(x);
  return x >> (64 - 2 * k);
}

__device__ __forceinline__ uint32_t base_code(uint32_t c) {  // set_kmer / forwardBase switch
  return c == 'C' ? 1u : c == 'G' ? 2u : c == 'T' ? 3u : 0u;
}

__device__ __forceinline__ bool kset_has(const uint64_t* __restrict__ tab, uint64_t mask,
                                         uint64_t key) {
  uint64_t h = fmix64(key) & mask;
  while (true) {
    const uint64_t t = tab[h];
    if (t == key) return true;
    if (t == kKsetEmpty) return false;
    h = (h + 1) & mask;
  }
}

__global__ __launch_bounds__(256) void k_check_reads(const uint8_t* __restrict__ seq,
                                                     const uint64_t* __restrict__ off, uint64_t n,
                                                     int k, float vote,
                                                     const uint64_t* __restrict__ tab, uint64_t mask,
                                                     uint32_t* __restrict__ hits,
                                                     uint8_t* __restrict__ flags) {
  __shared__ uint8_t codes[kCheckWaves][kCheckWindow + 64];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  uint8_t* cw = codes[wv];
  const uint64_t kmask = k == 32 ? ~0ull : ((1ull << (2 * k)) - 1ull);
  const uint64_t waves = (uint64_t)gridDim.x * kCheckWaves;
  for (uint64_t r = (uint64_t)blockIdx.x * kCheckWaves + wv; r < n; r += waves) {  // wave-uniform
    const uint64_t a = off[r];
    const uint64_t len = off[r + 1] - a;
    if (len < (uint64_t)k + 10u) {  // io/ioFastQ.cc:19-25 (an empty read included)
      if (lane == 0) {
        hits[r] = 0u;
        flags[r] = 0u;
      }
      continue;
    }
    const uint64_t npos = len - (uint64_t)k + 1u;
    uint32_t cnt = 0;
    for (uint64_t w0 = 0; w0 < npos; w0 += kCheckWindow) {
      const uint32_t np = (uint32_t)(npos - w0 < kCheckWindow ? npos - w0 : kCheckWindow);
      const uint32_t nb = np + (uint32_t)k - 1u;  // bases of the window
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      for (uint32_t q = lane; q < nb; q += 64u) cw[q] = (uint8_t)base_code(seq[a + w0 + q]);
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      for (uint32_t p = lane; p < np; p += 64u) {
        uint64_t v = 0;
        for (int i = 0; i < k; ++i) v |= (uint64_t)cw[p + (uint32_t)i] << (2 * i);
        v &= kmask;
        const uint64_t t = revcomp(v, k);
        const uint64_t key = __builtin_bswap64(v) < __builtin_bswap64(t) ? v : t;
        cnt += kset_has(tab, mask, key) ? 1u : 0u;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    if (lane == 0) {
      hits[r] = cnt;
      // kmer_count / (len - k + 1) in float, correctly rounded (ioFastQ.cc:61)
      flags[r] = ((float)cnt / (float)npos > vote) ? 1u : 0u;
    }
  }
}

void launch_kset_insert(const uint64_t* kmers, uint64_t n, uint64_t* tab, uint64_t mask,
                        hipStream_t s) {
  if (n == 0) return;
  const uint64_t g = (n + 255) / 256 < 8192 ? (n + 255) / 256 : 8192;
  k_kset_insert<<<(uint32_t)g, 256, 0, s>>>(kmers, n, reinterpret_cast<unsigned long long*>(tab),
                                            mask);
}

void launch_check_reads(const uint8_t* seq, const uint64_t* off, uint64_t n, int k, float vote,
                        const uint64_t* tab, uint64_t mask, uint32_t* hits, uint8_t* flags,
                        hipStream_t s) {
  if (n == 0) return;
  const uint64_t w = (n + kCheckWaves - 1) / kCheckWaves, g = w < 16384 ? w : 16384;
  k_check_reads<<<(uint32_t)g, 64 * kCheckWaves, 0, s>>>(seq, off, n, k, vote, tab, mask, hits,
                                                         flags);
}

}  // namespace klsh
