// gfx950 kernels of the sharded Cluster() loop: key-range ownership, the
// (key, slot) exchange buffers, and the merge deltas that keep every rank's replica of the rows
// identical.  No arithmetic of the reference lives here — only integer bookkeeping and copies.
#include <hip/hip_runtime.h>

#include "klsh_device.h"

namespace klsh {

// ------------------------------------------------------------------------- key-range bins -----
__global__ __launch_bounds__(256) void k_bin_hist(const uint32_t* __restrict__ keys, uint32_t n,
                                                  int shift, uint32_t nbins,
                                                  uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[1u << kMaxBinBits];
  for (uint32_t b = threadIdx.x; b < nbins; b += 256) h[b] = 0;
  __syncthreads();
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u)
    atomicAdd(&h[keys[i] >> shift], 1u);
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nbins; b += 256)
    if (h[b]) atomicAdd(&hist[b], h[b]);
}

void launch_bin_hist(const uint32_t* keys, uint32_t n, int shift, uint32_t nbins, uint32_t* hist,
                     hipStream_t s) {
  (void)hipMemsetAsync(hist, 0, sizeof(uint32_t) * nbins, s);
  if (n == 0) return;
  const uint32_t g = (uint32_t)std::min<uint64_t>(1024, (n + 255) / 256);
  k_bin_hist<<<g, 256, 0, s>>>(keys, n, shift, nbins, hist);
}

// One workgroup of 256 lanes, 16 bins each.  A bin's owner is decided by the midpoint of its row
// range in the global bin order, so ranges are contiguous and balanced to within one bin; every
// rank computes the same.  A lane reads its 16 counts of a rank as four 16-B loads (nbins is a
// power of two: at 16 bins or more a lane's bins are all in range and aligned) and adds a rank's
// counts to the matrix once per owner run of its bins — no load waits on a branch over the value
// of the one before (one lane-serial round trip per bin and rank: ≈ 16·W of them per iteration).
__global__ __launch_bounds__(256) void k_bin_split(const uint32_t* __restrict__ hist_all,
                                                   int world, uint32_t nbins, uint64_t total,
                                                   uint32_t* __restrict__ owner,
                                                   uint32_t* __restrict__ cntmat) {
  constexpr uint32_t PER = (1u << kMaxBinBits) / 256;
  static_assert(PER % 4 == 0, "whole 16-B loads");
  __shared__ uint32_t mat[kMaxRanks * kMaxRanks];
  for (uint32_t k = threadIdx.x; k < (uint32_t)(world * world); k += 256) mat[k] = 0;
  const uint32_t b0 = threadIdx.x * PER;
  const uint32_t nb = b0 < nbins ? min(PER, nbins - b0) : 0u;  // this lane's bins
  // rank r's counts of this lane's bins (0 past nb)
  auto load = [&](int r, uint32_t (&c)[PER]) {
    const uint32_t* src = hist_all + (size_t)r * nbins + b0;
    if (nb == PER) {
#pragma unroll
      for (uint32_t q = 0; q < PER / 4; ++q) {
        const uint4 v = reinterpret_cast<const uint4*>(src)[q];
        c[4 * q] = v.x;
        c[4 * q + 1] = v.y;
        c[4 * q + 2] = v.z;
        c[4 * q + 3] = v.w;
      }
    } else {  // fewer than 16 bins in all: lane 0 holds them
#pragma unroll
      for (uint32_t j = 0; j < PER; ++j) c[j] = j < nb ? src[j] : 0u;
    }
  };
  uint32_t tot[PER] = {};
#pragma unroll 2
  for (int r = 0; r < world; ++r) {
    uint32_t c[PER];
    load(r, c);
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) tot[j] += c[j];
  }
  uint32_t acc = 0;
#pragma unroll
  for (uint32_t j = 0; j < PER; ++j) acc += tot[j];
  uint32_t block_total;
  uint64_t run = block_excl_scan_256(acc, &block_total);  // rows in bins before b0
  uint32_t ow[PER];
#pragma unroll
  for (uint32_t j = 0; j < PER; ++j) {
    const uint64_t mid2 = 2 * run + tot[j];  // twice the midpoint
    const uint64_t o = total ? (mid2 * (uint64_t)world) / (2 * total) : 0;
    ow[j] = (uint32_t)(o >= (uint64_t)world ? world - 1 : o);
    if (j < nb) owner[b0 + j] = ow[j];
    run += tot[j];
  }
  __syncthreads();  // (mat zeroed)
#pragma unroll 2
  for (int g = 0; g < world; ++g) {
    uint32_t c[PER];
    load(g, c);
    uint32_t cur = ow[0], sum = 0;
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) {
      if (j < nb && ow[j] != cur) {
        if (sum) atomicAdd(&mat[g * world + cur], sum);
        cur = ow[j];
        sum = 0;
      }
      sum += c[j];
    }
    if (sum) atomicAdd(&mat[g * world + cur], sum);
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < (uint32_t)(world * world); k += 256) cntmat[k] = mat[k];
}

void launch_bin_split(const uint32_t* hist_all, int world, uint32_t nbins, uint64_t total,
                      uint32_t* owner, uint32_t* cntmat, hipStream_t s) {
  k_bin_split<<<1, 256, 0, s>>>(hist_all, world, nbins, total, owner, cntmat);
}

// --------------------------------------------------------------------- exchange buffers -----
__global__ __launch_bounds__(256) void k_dest(const uint32_t* __restrict__ keys, uint32_t n,
                                              int shift, const uint32_t* __restrict__ owner,
                                              uint32_t* __restrict__ dest,
                                              uint32_t* __restrict__ idx) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  dest[i] = owner[keys[i] >> shift];
  idx[i] = i;
}

void launch_dest(const uint32_t* keys, uint32_t n, int shift, const uint32_t* owner,
                 uint32_t* dest, uint32_t* idx, hipStream_t s) {
  if (n) k_dest<<<(n + 255) / 256, 256, 0, s>>>(keys, n, shift, owner, dest, idx);
}

__global__ __launch_bounds__(256) void k_pack_pairs(const uint32_t* __restrict__ keys,
                                                    const uint32_t* __restrict__ slots,
                                                    const uint32_t* __restrict__ idx, uint32_t n,
                                                    uint2* __restrict__ out) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const uint32_t j = idx[i];
  out[i] = make_uint2(keys[j], slots[j]);
}

void launch_pack_pairs(const uint32_t* keys, const uint32_t* slots, const uint32_t* idx,
                       uint32_t n, uint2* out, hipStream_t s) {
  if (n) k_pack_pairs<<<(n + 255) / 256, 256, 0, s>>>(keys, slots, idx, n, out);
}

__global__ __launch_bounds__(256) void k_unpack_pairs(const uint2* __restrict__ in, uint32_t n,
                                                      uint32_t* __restrict__ keys,
                                                      uint32_t* __restrict__ slots) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const uint2 v = in[i];
  keys[i] = v.x;
  slots[i] = v.y;
}

void launch_unpack_pairs(const uint2* in, uint32_t n, uint32_t* keys, uint32_t* slots,
                         hipStream_t s) {
  if (n) k_unpack_pairs<<<(n + 255) / 256, 256, 0, s>>>(in, n, keys, slots);
}

// Stable partition of (key, slot) by owning rank in one read pass + one scatter pass (replaces
// the dest -> 8-bit radix sort -> pack sequence).  Tile = 4096 positions; wave w of a tile owns
// the contiguous positions [w*1024, w*1024 + 1024), 64 at a time, so "tile-major, then wave, then
// step, then lane" is position order.  counts[o * ntiles + tile] = pairs of owner o in the tile;
// after an exclusive scan over that owner-major array they are the tile's output offsets.
constexpr uint32_t kPartTile = 4096;

// Lanes of the wave whose owner equals mine (owner < 64: six ballots).
__device__ __forceinline__ uint64_t same_owner(uint32_t o, bool valid) {
  uint64_t m = __ballot(valid);
#pragma unroll
  for (int b = 0; b < 6; ++b) {
    const uint64_t on = __ballot(valid && ((o >> b) & 1u));
    m &= ((o >> b) & 1u) ? on : ~on;
  }
  return valid ? m : 0ull;
}

__global__ __launch_bounds__(256) void k_part_count(const uint32_t* __restrict__ keys, uint32_t n,
                                                    int shift, const uint32_t* __restrict__ owner,
                                                    int world, uint32_t ntiles,
                                                    uint32_t* __restrict__ counts) {
  __shared__ uint32_t c[kMaxRanks];
  const uint32_t t = threadIdx.x, lane = t & 63u;
  if (t < (uint32_t)world) c[t] = 0u;
  __syncthreads();
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  const uint32_t T0 = blockIdx.x * kPartTile;
#pragma unroll 1
  for (uint32_t k = 0; k < kPartTile / 256; ++k) {
    const uint32_t i = T0 + k * 256u + t;
    const bool v = i < n;
    const uint32_t o = v ? owner[keys[i] >> shift] : 0u;
    const uint64_t peers = same_owner(o, v);
    if (v && (peers & below) == 0ull) atomicAdd(&c[o], (uint32_t)__popcll(peers));
  }
  __syncthreads();
  if (t < (uint32_t)world) counts[(size_t)t * ntiles + blockIdx.x] = c[t];
}

__global__ __launch_bounds__(256) void k_part_scatter(const uint32_t* __restrict__ keys,
                                                      const uint32_t* __restrict__ slots,
                                                      uint32_t n, int shift,
                                                      const uint32_t* __restrict__ owner,
                                                      int world, uint32_t ntiles,
                                                      const uint32_t* __restrict__ offs,
                                                      uint2* __restrict__ out) {
  __shared__ uint32_t run[4][kMaxRanks];  // per wave: its next output position per owner
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint32_t base = blockIdx.x * kPartTile + wv * (kPartTile / 4);
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  constexpr uint32_t K = kPartTile / 256;
  if (lane < (uint32_t)world) run[wv][lane] = 0u;
  __builtin_amdgcn_wave_barrier();
  // pass 1: this wave's pairs per owner
#pragma unroll 1
  for (uint32_t k = 0; k < K; ++k) {
    const uint32_t i = base + k * 64u + lane;
    const bool v = i < n;
    const uint32_t o = v ? owner[keys[i] >> shift] : 0u;
    const uint64_t peers = same_owner(o, v);
    if (v && (peers & below) == 0ull) run[wv][o] += (uint32_t)__popcll(peers);
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  // the tile's offset per owner + the pairs of the waves before this one
  uint32_t pre = 0u;
  if (lane < (uint32_t)world) {
    pre = offs[(size_t)lane * ntiles + blockIdx.x];
    for (uint32_t w = 0; w < wv; ++w) pre += run[w][lane];
  }
  __syncthreads();
  if (lane < (uint32_t)world) run[wv][lane] = pre;
  __builtin_amdgcn_wave_barrier();
  // pass 2: scatter in position order (the keys are re-read, from L2)
#pragma unroll 1
  for (uint32_t k = 0; k < K; ++k) {
    const uint32_t i = base + k * 64u + lane;
    const bool v = i < n;
    const uint32_t key = v ? keys[i] : 0u;
    const uint32_t slot = v ? slots[i] : 0u;
    const uint32_t o = v ? owner[key >> shift] : 0u;
    const uint64_t peers = same_owner(o, v);
    const uint32_t at = v ? run[wv][o] : 0u;
    __builtin_amdgcn_wave_barrier();
    if (v) {
      out[at + (uint32_t)__popcll(peers & below)] = make_uint2(key, slot);
      if ((peers & below) == 0ull) run[wv][o] = at + (uint32_t)__popcll(peers);
    }
    __builtin_amdgcn_wave_barrier();
  }
}

int launch_partition(const uint32_t* keys, const uint32_t* slots, uint32_t n, int shift,
                     const uint32_t* owner, int world, uint32_t* counts, uint32_t* tile_sums,
                     Counters* ctr, uint2* out, hipStream_t s) {
  if (n == 0) return 0;
  if (world < 1 || world > 64) return -1;
  const uint32_t ntiles = (n + kPartTile - 1) / kPartTile;
  k_part_count<<<ntiles, 256, 0, s>>>(keys, n, shift, owner, world, ntiles, counts);
  device_scan(SrcArray{counts}, DstExclusive{counts}, (uint32_t)world * ntiles, tile_sums,
              &ctr->total, &ctr->err, s);
  k_part_scatter<<<ntiles, 256, 0, s>>>(keys, slots, n, shift, owner, world, ntiles, counts, out);
  return 0;
}

// ------------------------------------------------------------------------------- deltas -----
// One thread per record word, grid-strided (a launch stays below 2^32 work-items): consecutive
// lanes write consecutive words (and read one row).
constexpr uint32_t kDeltaGrid = 65536;
__global__ __launch_bounds__(256) void k_delta_pack(Rows r, const uint32_t* __restrict__ ds,
                                                    uint32_t n, uint32_t* __restrict__ rec) {
  const uint32_t R = (uint32_t)delta_words(r.dp);
  for (uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x; t < (uint64_t)n * R;
       t += (uint64_t)gridDim.x * 256u) {
  const uint32_t i = (uint32_t)(t / R), w = (uint32_t)(t % R);
  const uint32_t s = ds[i];
  uint32_t v;
  switch (w) {
    case 0: v = s; break;
    case 1: v = r.cnt[s]; break;
    case 2: v = r.head[s]; break;
    case 3: v = r.tail[s]; break;
    case 4: v = __float_as_uint(r.nrm[s]); break;
    default: v = __float_as_uint(r.x[(size_t)s * r.dp + (w - 5)]);
  }
  rec[t] = v;
  }
}

void launch_delta_pack(const Rows& r, const uint32_t* delta_slots, uint32_t n, uint32_t* rec,
                       hipStream_t s) {
  const uint64_t total = (uint64_t)n * (uint64_t)delta_words(r.dp);
  if (total)
    k_delta_pack<<<(unsigned)std::min<uint64_t>((total + 255) / 256, kDeltaGrid), 256, 0, s>>>(
        r, delta_slots, n, rec);
}

__global__ __launch_bounds__(256) void k_delta_apply(Rows r, const uint32_t* __restrict__ rec,
                                                     uint32_t n) {
  const uint32_t R = (uint32_t)delta_words(r.dp);
  for (uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x; t < (uint64_t)n * R;
       t += (uint64_t)gridDim.x * 256u) {
  const uint32_t i = (uint32_t)(t / R), w = (uint32_t)(t % R);
  const uint32_t s = rec[(uint64_t)i * R];
  const uint32_t v = rec[t];
  switch (w) {
    case 0: break;
    case 1: r.cnt[s] = v; break;
    case 2: r.head[s] = v; break;
    case 3: r.tail[s] = v; break;
    case 4: r.nrm[s] = __uint_as_float(v); break;
    default:
      r.x[(size_t)s * r.dp + (w - 5)] = __uint_as_float(v);
      if (r.xh) {  // the fp16 image of the replica's row follows it
        const _Float16 hv = (_Float16)__uint_as_float(v);
        r.xh[(size_t)s * r.dp + (w - 5)] = *reinterpret_cast<const uint16_t*>(&hv);
      }
  }
  }
}

// The words the host needs from an exchange (send-count matrix; every rank's counters and this
// rank's Counters) into mapped host memory, then the sequence word with a system-scope release:
// the host polls it instead of a device-to-host copy plus an event or stream sync (two packets
// and a wait each, ~10-20 us per exchange).  One workgroup.
__global__ __launch_bounds__(256) void k_publish_words(const uint32_t* __restrict__ a, uint32_t na,
                                                       const uint32_t* __restrict__ b, uint32_t nb,
                                                       uint32_t* dst, uint32_t* seq_host,
                                                       uint32_t seq) {
  for (uint32_t i = threadIdx.x; i < na + nb; i += 256)
    __hip_atomic_store(dst + i, i < na ? a[i] : b[i - na], __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(seq_host, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

void launch_publish_words(const uint32_t* a, uint32_t na, const uint32_t* b, uint32_t nb,
                          uint32_t* dst, uint32_t* seq_host, uint32_t seq, hipStream_t s) {
  k_publish_words<<<1, 256, 0, s>>>(a, na, b, nb, dst, seq_host, seq);
}

void launch_delta_apply(const Rows& r, const uint32_t* rec, uint32_t n, hipStream_t s) {
  const uint64_t total = (uint64_t)n * (uint64_t)delta_words(r.dp);
  if (total)
    k_delta_apply<<<(unsigned)std::min<uint64_t>((total + 255) / 256, kDeltaGrid), 256, 0, s>>>(
        r, rec, n);
}

__global__ __launch_bounds__(256) void k_min_u32(uint32_t* __restrict__ a,
                                                 const uint32_t* __restrict__ b, size_t n) {
  const size_t i = (size_t)blockIdx.x * 256u + threadIdx.x;
  if (i < n) a[i] = min(a[i], b[i]);
}

void launch_min_u32(uint32_t* a, const uint32_t* b, size_t n, hipStream_t s) {
  if (n) k_min_u32<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(a, b, n);
}

}  // namespace klsh
