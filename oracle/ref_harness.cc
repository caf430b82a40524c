// TEST INFRASTRUCTURE ONLY — a driver that links the UNMODIFIED reference objects built from
// /root/reference by oracle/Makefile (into oracle/_ref/) and calls the reference's own functions,
// so the golden vectors under tests/golden/ are produced by the reference itself.
//
// Reference entry points called (file:line in /root/reference):
//   Hash::LSH::generateHashTable        hash/lshash.cc:36
//   Hash::LSH::random_projection        hash/lshash.cc:53
//   p_lsh / merge_hashtable             function/cluster.cc:4 / :15
//   p_cluster / nestedCluster           function/cluster.cc:56 / :89
//   merge_abundance                     function/cluster.cc:39
//   Cluster                             function/cluster.cc:181
//   Core::Distance::cosine              function/distance.cc:27
//   Core::AB::SetConsensus              function/funcAB.cc:49
//   Utility::IOMat::ReadClusterAll      io/ioMatrix.cc:48
//   Utility::IOMat::SaveResult / SaveBinary   io/ioMatrix.cc:265 / :322
//   Utility::IOMat::convertHTMat        io/ioMatrix.cc:353
//   alglib::studentttest2               utils/alglib-3.15.0/src/statistics.cpp:12502 (AB::WRS's test,
//                                       function/funcAB.cc:100)
//
// Run with OMP_THREAD_LIMIT=1 (T=1 semantics) and KLSH_SEED=<seed> (ref_seed.cc).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "function/cluster.h"
#include "io/ioMatrix.h"
#include "utils/alglib-3.15.0/src/statistics.h"

using namespace std;

// function/cluster.cc:15 defines merge_hashtable with a size_t hash_func_num while cluster.h:31
// declares it with an int (two different symbols): the definition's signature, to link to it.
void merge_hashtable(vector<vector<Abundance*>>* final_table, size_t hash_func_num,
                     const vector<vector<Abundance*>*>& part_hash_values,
                     const vector<vector<int>*>& part_hash_keys);

static vector<float> read_f32(const char* path, size_t count) {
  vector<float> v(count);
  FILE* f = fopen(path, "rb");
  if (!f) { perror(path); exit(2); }
  if (count && fread(v.data(), 4, count, f) != count) { fprintf(stderr, "short read %s\n", path); exit(2); }
  fclose(f);
  return v;
}

static void write_bytes(const char* path, const void* p, size_t n) {
  FILE* f = fopen(path, "wb");
  if (!f) { perror(path); exit(2); }
  if (n) fwrite(p, 1, n, f);
  fclose(f);
}

static vector<Abundance*> rows_to_abundance(const vector<float>& x, size_t n, int d) {
  vector<Abundance*> v;
  v.reserve(n);
  for (size_t i = 0; i < n; ++i) {
    Abundance* a = new Abundance();
    a->_values.assign(x.begin() + i * d, x.begin() + (i + 1) * d);
    a->_ids.push_back(i);
    v.push_back(a);
  }
  return v;
}

static void save(vector<Abundance*>* v, const string& prefix) {
  // The reference's own writers, ignore_small = 0 (every cluster).
  IOMat::SaveResult(v, prefix + ".clust", true, 0, false);
  IOMat::SaveBinary(v, prefix, true, 0, false);
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr,
            "usage:\n"
            "  ref_harness rng H D                          (hex floats of generateHashTable(H,D))\n"
            "  ref_harness keys ROWS N D H OUT              (uint32 keys via random_projection)\n"
            "  ref_harness pcluster ROWS N D THR OUTPREFIX  (one bucket through p_cluster)\n"
            "  ref_harness cosine ROWS N D OUT              (float cosine distance for pairs (i, i+1))\n"
            "  ref_harness consensus ROWS D CA CB OUT       (SetConsensus of row0 (CA ids) and row1 (CB ids))\n"
            "  ref_harness cluster ROWS N D MINSIM I BTHR OUTPREFIX\n"
            "  ref_harness cluster_from BINPREFIX D MINSIM I BTHR OUTPREFIX   (input via ReadClusterAll)\n"
            "  ref_harness cluster_w ROWS OFF IDS N D MINSIM I BTHR OUTPREFIX (binary member lists)\n"
            "  ref_harness iter_w ROWS OFF IDS N D THR BTHR [K STEP]  (K (default 1) iterations of\n"
            "                                               Cluster's body from threshold THR, each timed)\n"
            "  ref_harness convert COUNTS N D VKMERS OUTPREFIX  (uint16 sample-major counts -> convertHTMat)\n"
            "  ref_harness ttest VALUES N M COUNT OUT       (f32 cases of N+M values -> studentttest2,\n"
            "                                               f64 bothtails/lefttail/righttail per case)\n");
    return 1;
  }
  const string cmd = argv[1];
  if (cmd == "rng") {
    const int h = atoi(argv[2]), d = atoi(argv[3]);
    hashTable t = LSH::generateHashTable(h, d);
    for (int j = 0; j < h; ++j) {
      for (int i = 0; i < d; ++i) {
        uint32_t b;
        memcpy(&b, &t[j][i], 4);
        printf("%s%08x", i ? " " : "", b);
      }
      printf("\n");
    }
    return 0;
  }
  if (cmd == "keys") {
    const size_t n = strtoull(argv[3], nullptr, 10);
    const int d = atoi(argv[4]), h = atoi(argv[5]);
    vector<float> x = read_f32(argv[2], n * d);
    hashTable t = LSH::generateHashTable(h, d);
    vector<uint32_t> keys(n);
    for (size_t i = 0; i < n; ++i) {
      vector<float> row(x.begin() + i * d, x.begin() + (i + 1) * d);
      keys[i] = (uint32_t)LSH::random_projection(row, t);
    }
    write_bytes(argv[6], keys.data(), n * 4);
    return 0;
  }
  if (cmd == "pcluster") {
    const size_t n = strtoull(argv[3], nullptr, 10);
    const int d = atoi(argv[4]);
    const float thr = (float)atof(argv[5]);
    vector<float> x = read_f32(argv[2], n * d);
    vector<Abundance*> bucket = rows_to_abundance(x, n, d);
    vector<Abundance*> out;
    p_cluster(&out, &bucket, thr);
    save(&out, argv[6]);
    return 0;
  }
  if (cmd == "cosine") {
    const size_t n = strtoull(argv[3], nullptr, 10);
    const int d = atoi(argv[4]);
    vector<float> x = read_f32(argv[2], n * d);
    vector<float> out;
    for (size_t i = 0; i + 1 < n; ++i) {
      vector<float> a(x.begin() + i * d, x.begin() + (i + 1) * d);
      vector<float> b(x.begin() + (i + 1) * d, x.begin() + (i + 2) * d);
      out.push_back(Distance::cosine(a, b));
    }
    write_bytes(argv[5], out.data(), out.size() * 4);
    return 0;
  }
  if (cmd == "consensus") {
    const int d = atoi(argv[3]);
    const int ca = atoi(argv[4]), cb = atoi(argv[5]);
    vector<float> x = read_f32(argv[2], 2 * (size_t)d);
    Abundance a, b, c;
    a._values.assign(x.begin(), x.begin() + d);
    b._values.assign(x.begin() + d, x.begin() + 2 * d);
    for (int i = 0; i < ca; ++i) a._ids.push_back(i);
    for (int i = 0; i < cb; ++i) b._ids.push_back(1000000 + i);
    AB::SetConsensus(&c, a, b);
    write_bytes(argv[6], c._values.data(), (size_t)d * 4);
    return 0;
  }
  if (cmd == "cluster" || cmd == "cluster_from" || cmd == "cluster_w" || cmd == "iter_w") {
    vector<Abundance*> v;
    int argi;
    int d;
    if (cmd == "cluster_w" || cmd == "iter_w") {  // ROWS.f32 OFF.u64 IDS.u64 N D ...: rows with member-id lists
      const size_t n = strtoull(argv[5], nullptr, 10);
      d = atoi(argv[6]);
      vector<float> x = read_f32(argv[2], n * d);
      vector<uint64_t> off(n + 1);
      FILE* f = fopen(argv[3], "rb");
      if (!f || fread(off.data(), 8, n + 1, f) != n + 1) { fprintf(stderr, "read off\n"); return 2; }
      fclose(f);
      vector<uint64_t> ids(off[n]);
      f = fopen(argv[4], "rb");
      if (!f || (off[n] && fread(ids.data(), 8, off[n], f) != off[n])) { fprintf(stderr, "read ids\n"); return 2; }
      fclose(f);
      v.reserve(n);
      for (size_t i = 0; i < n; ++i) {
        Abundance* a = new Abundance();
        a->_values.assign(x.begin() + i * d, x.begin() + (i + 1) * d);
        a->_ids.assign(ids.begin() + off[i], ids.begin() + off[i + 1]);
        v.push_back(a);
      }
      argi = 7;
    } else if (cmd == "cluster") {
      const size_t n = strtoull(argv[3], nullptr, 10);
      d = atoi(argv[4]);
      vector<float> x = read_f32(argv[2], n * d);
      v = rows_to_abundance(x, n, d);
      argi = 5;
    } else {
      d = atoi(argv[3]);
      IOMat::ReadClusterAll(&v, d, argv[2], false);
      argi = 4;
    }
    // threads_to_use: 1 (T=1 semantics, deterministic) unless KLSH_REF_THREADS asks for more
    // (timing only: at T>1 the reference's bucket order depends on scheduling, cluster.cc:281)
    const char* te = getenv("KLSH_REF_THREADS");
    const unsigned threads = te ? std::max(1, atoi(te)) : 1u;
    if (cmd == "iter_w") {
      // One pass of Cluster()'s loop body (function/cluster.cc:199-331) at the caller's threshold
      // — Cluster() itself always starts its schedule at 0.95 (:190) — through the reference's
      // own p_lsh, merge_hashtable, p_cluster / nestedCluster and merge_abundance, with the same
      // OpenMP structure, so bench.py can time an iteration of the loop at its scheduled value.
      // optional K STEP: K consecutive iterations at THR, THR - STEP, ... (the schedule's own
      // decrement, cluster.cc:330), each timed: the later ones run on the state the loop itself
      // left (its allocations and member lists), not on one freshly built from arrays
      const float thr0 = (float)atof(argv[argi]);
      const int bthr = atoi(argv[argi + 1]);
      const int k_iters = argc > argi + 2 ? std::max(1, atoi(argv[argi + 2])) : 1;
      const float step = argc > argi + 3 ? (float)atof(argv[argi + 3]) : 0.0f;
      float thr = thr0;
      for (int it = 0; it < k_iters; ++it) {
      const size_t n0 = v.size();
      const auto t0 = chrono::high_resolution_clock::now();
      const size_t h = floor(log2(v.size()));
      const size_t buckets = size_t(pow(2, h));
      vector<vector<Abundance*>> table(buckets, vector<Abundance*>());
      hashTable ht = LSH::generateHashTable(h, d);
      vector<vector<Abundance*>*> pv;
      vector<vector<int>*> pk;
      for (unsigned i = 0; i < threads; ++i) {
        pv.push_back(new vector<Abundance*>());
        pk.push_back(new vector<int>());
      }
      const int na = (int)v.size();
#pragma omp parallel for num_threads(threads)
      for (int i = 0; i < na; ++i) p_lsh(pv[omp_get_thread_num()], pk[omp_get_thread_num()], ht, v[i]);
      merge_hashtable(&table, h, pv, pk);
      for (unsigned i = 0; i < threads; ++i) {
        delete pv[i];
        delete pk[i];
      }
      vector<vector<Abundance*>*> part;
      for (unsigned i = 0; i < threads; ++i) part.push_back(new vector<Abundance*>());
      omp_set_nested(1);
      omp_set_max_active_levels(2);
#pragma omp parallel for num_threads(threads) schedule(dynamic)
      for (size_t s = 0; s < buckets; ++s) {
        auto& cand = table[s];
        const int tid = omp_get_thread_num();
        if (cand.size() > (size_t)bthr) {
          nestedCluster(&cand, thr, d, 3, false);
          part[tid]->insert(part[tid]->end(), cand.begin(), cand.end());
        } else {
          p_cluster(part[tid], &cand, thr);
        }
      }
      omp_set_nested(0);
      merge_abundance(&v, part);
      for (unsigned i = 0; i < threads; ++i) delete part[i];
      const double secs =
          chrono::duration<double>(chrono::high_resolution_clock::now() - t0).count();
      printf("iteration: %zu -> %zu rows at threshold %.9g, %u threads\n", n0, v.size(), thr, threads);
      printf("one iteration takes (secs): %.6f\n", secs);
      fflush(stdout);
      thr -= step;
      }
      return 0;
    }
    const float min_sim = (float)atof(argv[argi]);
    const int iters = atoi(argv[argi + 1]);
    const int bthr = atoi(argv[argi + 2]);
    Cluster(&v, min_sim, iters, threads ? threads : 1u, d, bthr, true);
    save(&v, argv[argi + 3]);
    return 0;
  }
  if (cmd == "convert") {
    const size_t n = strtoull(argv[3], nullptr, 10);
    const int d = atoi(argv[4]);
    vector<uint16_t> counts((size_t)n * d);
    FILE* f = fopen(argv[2], "rb");
    if (!f || fread(counts.data(), 2, counts.size(), f) != counts.size()) { fprintf(stderr, "read\n"); return 2; }
    fclose(f);
    vector<float> vk = read_f32(argv[5], d);
    vector<float_t> v_kmers(vk.begin(), vk.end());
    vector<uint16_t*> ary(d);
    for (int j = 0; j < d; ++j) ary[j] = counts.data() + (size_t)j * n;
    vector<Abundance*> v;
    IOMat::convertHTMat(ary.data(), v_kmers, d, false, n, 0, &v);
    save(&v, argv[6]);
    return 0;
  }
  if (cmd == "ttest") {  // the values as AB::WRS passes them: float -> double (funcAB.cc:88-93)
    const int n = atoi(argv[3]), m = atoi(argv[4]);
    const size_t count = strtoull(argv[5], nullptr, 10);
    vector<float> v = read_f32(argv[2], count * (size_t)(n + m));
    vector<double> out(3 * count);
    for (size_t c = 0; c < count; ++c) {
      vector<double> x(n > 0 ? n : 1), y(m > 0 ? m : 1);
      for (int i = 0; i < n; ++i) x[i] = (double)v[c * (n + m) + i];
      for (int j = 0; j < m; ++j) y[j] = (double)v[c * (n + m) + n + j];
      alglib::real_1d_array ax, ay;
      ax.setcontent(n, x.data());
      ay.setcontent(m, y.data());
      double both = 0, left = 0, right = 0;
      alglib::studentttest2(ax, n, ay, m, both, left, right);
      out[3 * c] = both;
      out[3 * c + 1] = left;
      out[3 * c + 2] = right;
    }
    write_bytes(argv[6], out.data(), out.size() * 8);
    return 0;
  }
  fprintf(stderr, "unknown command %s\n", cmd.c_str());
  return 1;
}
