// klsh-synth v1: deterministic synthetic k-mer count matrices.
//
// The survey measured the reference on numpy-generated data that cannot be regenerated
// bit-for-bit elsewhere; this generator fixes the workload definition instead: a counter-based
// hash (splitmix64 finalizer) keyed by (seed, row, sample) feeds every draw, so any machine with
// this glibc produces the same kmer_count.bin, and rows can be generated in parallel.
//
//   genome(i)      = H(seed, i, 0x100) mod G                   G = n/50 by default
//   m(i)           = 1 + (H(seed, i, 0x101) & 1)               multiplicity
//   z(g, s)        = Box-Muller of two uniforms keyed (g, s)   profile exponent ~ N(0,1)
//   lambda(i, s)   = exp(2 + z(genome(i), s)) * m(i)
//   count(i, s)    = min(Poisson(lambda), 65535)  (inversion below 30, rounded normal above)
//   coverage(s)    = sum_i [count > 0] ln(count), double, ascending i (kmer_count.log)
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <thread>
#include <vector>

#include <cstdlib>

namespace {

// Host worker threads: OMP_NUM_THREADS if set (the GPU boxes set it to their CPU share), else
// min(16, hardware threads).
static int klsh_default_threads() {
  if (const char* e = std::getenv("OMP_NUM_THREADS")) {
    const int v = std::atoi(e);
    if (v > 0) return v;
  }
  return (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
}

inline uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
inline uint64_t H(uint64_t seed, uint64_t a, uint64_t b) { return mix64(mix64(seed ^ mix64(a)) + b); }
inline double U(uint64_t u) { return ((double)(u >> 11) + 0.5) * (1.0 / 9007199254740992.0); }
inline double gauss(uint64_t a, uint64_t b) {
  const double u1 = U(a), u2 = U(b);
  return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
}

template <class F>
void parallel_for(uint64_t n, int threads, F f) {
  if (threads <= 0) threads = klsh_default_threads();
  threads = (int)std::min<uint64_t>((uint64_t)threads, std::max<uint64_t>(1, n));
  std::vector<std::thread> pool;
  const uint64_t chunk = (n + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    const uint64_t a = t * chunk, b = std::min(n, a + chunk);
    if (a >= b) break;
    pool.emplace_back([=] { f(a, b); });
  }
  for (auto& th : pool) th.join();
}

}  // namespace

extern "C" int klsh_synth_counts(uint64_t n, int d, uint64_t seed, uint64_t genomes, int threads,
                                 uint16_t* counts, double* coverage) {
  if (d <= 0 || !counts) return -1;
  const uint64_t G = genomes ? genomes : std::max<uint64_t>(1, n / 50);
  std::vector<double> lam_g((size_t)G * d);
  parallel_for(G, threads, [&](uint64_t a, uint64_t b) {
    for (uint64_t g = a; g < b; ++g)
      for (int s = 0; s < d; ++s)
        lam_g[g * d + s] = std::exp(2.0 + gauss(H(seed ^ 0xA5A5A5A5ull, g, 2 * (uint64_t)s),
                                                H(seed ^ 0xA5A5A5A5ull, g, 2 * (uint64_t)s + 1)));
  });
  parallel_for(n, threads, [&](uint64_t a, uint64_t b) {
    for (uint64_t i = a; i < b; ++i) {
      const uint64_t g = H(seed, i, 0x100) % G;
      const double m = 1.0 + (double)(H(seed, i, 0x101) & 1u);
      for (int s = 0; s < d; ++s) {
        const double lam = lam_g[g * d + s] * m;
        const uint64_t r1 = H(seed ^ 0x5A5A5A5Aull, i, (uint64_t)s);
        uint64_t c;
        if (lam < 30.0) {
          const double u = U(r1);
          double p = std::exp(-lam), F = p;
          c = 0;
          while (u > F && c < 1000) {
            ++c;
            p *= lam / (double)c;
            F += p;
          }
        } else {
          const double z = gauss(r1, H(seed ^ 0x3C3C3C3Cull, i, (uint64_t)s));
          const double v = std::floor(lam + std::sqrt(lam) * z + 0.5);
          c = v < 0.0 ? 0 : (uint64_t)v;
        }
        counts[(size_t)s * n + i] = (uint16_t)std::min<uint64_t>(c, 65535);
      }
    }
  });
  if (coverage) {
    parallel_for((uint64_t)d, threads, [&](uint64_t a, uint64_t b) {
      for (uint64_t s = a; s < b; ++s) {
        double acc = 0.0;
        const uint16_t* col = counts + s * n;
        for (uint64_t i = 0; i < n; ++i)
          if (col[i] > 0) acc += std::log((double)col[i]);
        coverage[s] = acc;
      }
    });
  }
  return 0;
}
