// klsh_cluster.hpp — drop-in replacement for the reference's Cluster() call (header-only).
//
// Reference seam (wthanone/kmerLSH): function/cluster.h:42
//     void Cluster(vector<Abundance*>* unknown_abundance_ptr, float min_similarity,
//                  int cluster_iteration, unsigned int threads_to_use, int dim,
//                  int bucket_size_threshold, bool verbose);
// called at app/kmerLSH.cc:323 (init pass), :377 (re-cluster passes) and :490 (main loop).
//
// klsh::Cluster has the same signature and in-place semantics for any row type with the
// reference Abundance's public members `std::vector<float> _values` and
// `std::vector<uint64_t> _ids` (common/abundance.h:18-36): merged inputs are deleted, surviving
// rows are re-created in the reference's output order, and the id lists are the reference's
// concatenations.  The arithmetic runs on the gfx950 engine (libklsh.so, include/klsh.h); there
// is no CPU fallback — if no device is available the call throws std::runtime_error.
//
// Determinism: the reference seeds every hyperplane from std::random_device; here hyperplane k of
// the process is drawn from std::mt19937(seed + k*2654435761), with `seed` from
// $KLSH_SEED (default 12345) and k counted across calls, so results equal the reference run with
// the oracle/ref_seed.cc interposer at -T 1.
#ifndef KLSH_CLUSTER_HPP
#define KLSH_CLUSTER_HPP

#include <stdint.h>
#include <stdlib.h>

#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

#include "klsh.h"

namespace klsh {

struct Process {  // one device context and RNG stream per process (the reference's rd() stream)
  klsh_ctx* ctx = nullptr;
  uint32_t seed = 12345u;
  uint64_t counter = 0;
  static Process& get() {
    static Process p;
    if (!p.ctx) {
      int err = 0;
      const char* dev = getenv("KLSH_DEVICE");
      p.ctx = klsh_create(dev ? atoi(dev) : 0, &err);
      if (!p.ctx) throw std::runtime_error(std::string("klsh_create: ") + klsh_last_error());
      if (const char* s = getenv("KLSH_SEED")) p.seed = (uint32_t)strtoul(s, nullptr, 10);
    }
    return p;
  }
  ~Process() {
    if (ctx) klsh_destroy(ctx);
  }
};

inline void check(int rc, const char* what) {
  if (rc != KLSH_OK) throw std::runtime_error(std::string(what) + ": " + klsh_last_error());
}

template <class Abundance>
void Cluster(std::vector<Abundance*>* rows, float min_similarity, int cluster_iteration,
             unsigned int threads_to_use, int dim, int bucket_size_threshold, bool verbose) {
  (void)threads_to_use;  // results never depend on a thread count
  Process& P = Process::get();
  const uint64_t n = rows->size();
  std::vector<float> x(n * (uint64_t)dim);
  std::vector<uint64_t> off(n + 1, 0), ids;
  for (uint64_t i = 0; i < n; ++i) {
    const Abundance* a = (*rows)[i];
    std::copy(a->_values.begin(), a->_values.begin() + dim, x.begin() + i * dim);
    off[i + 1] = off[i] + a->_ids.size();
    ids.insert(ids.end(), a->_ids.begin(), a->_ids.end());
  }
  check(klsh_load_rows(P.ctx, x.data(), n, dim, off.data(), ids.data()), "klsh_load_rows");
  std::vector<uint64_t> trace(cluster_iteration > 0 ? cluster_iteration : 1);
  klsh_stats st{};
  st.struct_size = sizeof(st);
  check(klsh_cluster(P.ctx, min_similarity, cluster_iteration, bucket_size_threshold, P.seed,
                     &P.counter, trace.data(), &st),
        "klsh_cluster");
  if (verbose) {
    for (uint64_t t = 0; t < st.iterations; ++t)
      printf("Size of profilings : %llu\n", (unsigned long long)trace[t]);
    printf("kmerLSH algorithm hash+cluster takes (secs): %g\n", st.wall_ms / 1000.0);
  }
  uint64_t m = 0, nout = 0;
  check(klsh_count(P.ctx, &nout, &m), "klsh_count");
  x.resize(nout * (uint64_t)dim);
  off.assign(nout + 1, 0);
  ids.resize(m);
  check(klsh_result(P.ctx, x.data(), off.data(), ids.data()), "klsh_result");
  // only now are the input rows released: a failure above leaves *rows as it was (still owned by
  // the caller), never holding freed pointers
  for (Abundance* a : *rows) delete a;
  rows->clear();
  rows->reserve(nout);
  for (uint64_t i = 0; i < nout; ++i) {
    Abundance* a = new Abundance();
    a->_values.assign(x.begin() + i * dim, x.begin() + (i + 1) * dim);
    a->_ids.assign(ids.begin() + off[i], ids.begin() + off[i + 1]);
    rows->push_back(a);
  }
}

}  // namespace klsh

#endif
