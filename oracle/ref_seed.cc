// TEST INFRASTRUCTURE ONLY — linked into oracle/_ref builds of the reference, never into the product.
//
// Deterministic seeding for the reference kmerLSH objects.  The reference draws every hyperplane
// from `std::mt19937 gen(rd())` with a fresh `std::random_device rd` (reference
// hash/lshash.cc:6-7), so two runs never agree.  libstdc++ exports
// `std::random_device::_M_getval()` (GLIBCXX_3.4.18); defining it in the executable makes every
// `rd()` call return
//
//     seed_k = KLSH_SEED + k * 2654435761   (mod 2^32),  k = 0, 1, 2, ... (process-wide call count)
//
// which is the seeding convention the product exposes as `--seed`.  One `rd()`
// call happens per hyperplane, in process order: init pass, then main loop; nested-bucket tables
// in ascending bucket order when run with OMP_THREAD_LIMIT=1 / -T 1.
#include <atomic>
#include <cstdlib>
#include <random>

static std::atomic<unsigned long> g_klsh_seed_counter{0};

unsigned int std::random_device::_M_getval() {
  static const unsigned int base =
      std::getenv("KLSH_SEED") ? (unsigned int)std::strtoul(std::getenv("KLSH_SEED"), nullptr, 10)
                               : 12345u;
  const unsigned long k = g_klsh_seed_counter.fetch_add(1);
  return base + (unsigned int)k * 2654435761u;
}
