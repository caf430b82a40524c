// Hyperplane draws, host side.  The reference draws each hyperplane from a fresh
// std::mt19937 and std::normal_distribution<double>(0,1), casting each draw to float
// (reference hash/lshash.cc:3-17).  Those are libstdc++ header templates; instantiating them
// here (g++, no -march, -ffp-contract=off: libstdc++'s polar method must not be FMA-contracted)
// gives the same bits as the reference binary.  Seeding convention: SURVEY.md §8(c).
//
// This is control, not the hot path: <= 32 hyperplanes of d floats per LSH iteration.
#include <stdint.h>

#include <algorithm>
#include <random>
#include <thread>
#include <vector>

#include <cstdlib>


// Host worker threads: OMP_NUM_THREADS if set (the GPU boxes set it to their CPU share), else
// min(16, hardware threads).
static int klsh_default_threads() {
  if (const char* e = std::getenv("OMP_NUM_THREADS")) {
    const int v = std::atoi(e);
    if (v > 0) return v;
  }
  return (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
}

extern "C" {

uint32_t klsh_host_seed(uint32_t base, uint64_t k) { return base + (uint32_t)k * 2654435761u; }

void klsh_host_hyperplane(uint32_t seed, int d, float* out) {
  std::mt19937 engine(seed);
  std::normal_distribution<double> gauss(0.0, 1.0);
  for (int i = 0; i < d; ++i) out[i] = static_cast<float>(gauss(engine));
}

// Hyperplanes k0 .. k0+count-1, row j at out + j*stride (padding floats left untouched).
void klsh_host_hyperplanes(uint32_t base, uint64_t k0, uint64_t count, int d, int stride,
                           float* out, int threads) {
  if (count == 0) return;
  if (threads <= 0) threads = klsh_default_threads();
  const uint64_t per = 8;  // hyperplanes per work item
  const uint64_t items = (count + per - 1) / per;
  const int nt = (int)std::min<uint64_t>((uint64_t)threads, items);
  auto work = [&](int t) {
    for (uint64_t it = (uint64_t)t; it < items; it += (uint64_t)nt)
      for (uint64_t j = it * per; j < std::min(count, (it + 1) * per); ++j)
        klsh_host_hyperplane(klsh_host_seed(base, k0 + j), d, out + j * (uint64_t)stride);
  };
  if (nt <= 1 || count < 16) {
    work(0);
    if (nt > 1)
      for (int t = 1; t < nt; ++t) work(t);
    return;
  }
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
}

}  // extern "C"
