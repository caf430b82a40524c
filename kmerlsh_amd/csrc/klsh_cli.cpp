// kmerLSH-compatible command line (mode C) over the gfx950 engine.
//
// Same flags and files as the reference (app/kmerLSH.cc:147-276, :432-520): run in the directory
// holding kmer_count.bin / kmer_count.log, with -a/-b sample lists; writes
// <F>.clust ("<n>\t<id>\t...\n" per cluster with more than 5 members, io/ioMatrix.cc:265-294)
// and <F> (raw fp32 centroids of the same clusters, io/ioMatrix.cc:322-351).
//   kmerLSH -a A.txt -b B.txt [-I iters] [-N min_sim] [-F file] [-M C --only] [--verbose]
//           [--seed S] [--device D]
// Additions: --seed (the reference seeds from std::random_device; SURVEY.md §8(c) convention)
// and --device.  -T is accepted and ignored (results never depend on a thread count).
// The init pass keeps the reference's 1e8-row batching and re-cluster passes
// (app/kmerLSH.cc:278-430); its tmp-file round trip is lossless and stays in memory.
#include <getopt.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <string>
#include <vector>

#include "klsh.h"

namespace {

int count_lines(const char* path) {  // std::getline count (io/ioHT.cc:3-19)
  FILE* f = fopen(path, "rb");
  if (!f) {
    fprintf(stderr, "Unable to open info file");
    return 0;
  }
  int n = 0, c, last = '\n', any = 0;
  while ((c = fgetc(f)) != EOF) {
    any = 1;
    if (c == '\n') n++;
    last = c;
  }
  fclose(f);
  if (any && last != '\n') n++;
  return n;
}

struct RowSet {  // flat vector<Abundance*>
  int d = 0;
  std::vector<float> rows;
  std::vector<uint64_t> off{0};
  std::vector<uint64_t> ids;
  uint64_t n() const { return off.size() - 1; }
};

int check(int rc, const char* what) {
  if (rc != KLSH_OK) {
    fprintf(stderr, "kmerLSH: %s failed (%d): %s\n", what, rc, klsh_last_error());
    exit(2);
  }
  return rc;
}

void fetch(klsh_ctx* ctx, int d, RowSet* out) {
  uint64_t n = 0, m = 0;
  check(klsh_count(ctx, &n, &m), "klsh_count");
  std::vector<float> rows(n * (uint64_t)d);
  std::vector<uint64_t> off(n + 1), ids(m);
  check(klsh_result(ctx, rows.data(), off.data(), ids.data()), "klsh_result");
  const uint64_t base = out->ids.size();
  out->rows.insert(out->rows.end(), rows.begin(), rows.end());
  for (uint64_t i = 1; i <= n; ++i) out->off.push_back(base + off[i]);
  out->ids.insert(out->ids.end(), ids.begin(), ids.end());
}

void run_cluster(klsh_ctx* ctx, float min_sim, int iters, int bthr, uint32_t seed,
                 uint64_t* counter, bool verbose) {
  std::vector<uint64_t> trace(iters > 0 ? iters : 1);
  klsh_stats st;
  check(klsh_cluster(ctx, min_sim, iters, bthr, seed, counter, trace.data(), &st), "klsh_cluster");
  if (verbose) {
    for (uint64_t t = 0; t < st.iterations; ++t)
      printf("Size of profilings : %llu\n", (unsigned long long)trace[t]);
    printf("kmerLSH algorithm hash+cluster takes (secs): %g\n", st.wall_ms / 1000.0);
  }
}

void load_slice(klsh_ctx* ctx, const RowSet& rs, uint64_t a, uint64_t n) {
  std::vector<uint64_t> off(n + 1);
  for (uint64_t i = 0; i <= n; ++i) off[i] = rs.off[a + i] - rs.off[a];
  check(klsh_load_rows(ctx, rs.rows.data() + a * rs.d, n, rs.d, off.data(), rs.ids.data() + rs.off[a]),
        "klsh_load_rows");
}

char* put_u64(char* p, uint64_t v) {
  char tmp[24];
  int k = 0;
  do {
    tmp[k++] = (char)('0' + v % 10);
    v /= 10;
  } while (v);
  while (k) *p++ = tmp[--k];
  return p;
}

}  // namespace

int main(int argc, char** argv) {
  const char *in1 = nullptr, *in2 = nullptr;
  std::string out = "clustering_result.txt", mode;
  int iters = 100, verbose = 0, only = 0, device = 0;
  float min_sim = 0.80f;
  uint32_t seed = 12345u;
  static struct option lo[] = {{"verbose", no_argument, 0, 1},
                               {"only", no_argument, 0, 2},
                               {"seed", required_argument, 0, 3},
                               {"device", required_argument, 0, 4},
                               {"input1", required_argument, 0, 'a'},
                               {"input2", required_argument, 0, 'b'},
                               {"cluster_iteration", required_argument, 0, 'I'},
                               {"min_similarity", required_argument, 0, 'N'},
                               {"clust_file_name", required_argument, 0, 'F'},
                               {"mode", required_argument, 0, 'M'},
                               {"tmp_dir", required_argument, 0, 5},
                               {0, 0, 0, 0}};
  int c;
  while ((c = getopt_long(argc, argv, "o:p:a:b:H:I:N:X:C:T:K:S:P:V:F:M:", lo, nullptr)) != -1) {
    switch (c) {
      case 1: verbose = 1; break;
      case 2: only = 1; break;
      case 3: seed = (uint32_t)strtoul(optarg, nullptr, 10); break;
      case 4: device = atoi(optarg); break;
      case 'a': in1 = optarg; break;
      case 'b': in2 = optarg; break;
      case 'I': iters = atoi(optarg); break;
      case 'N': min_sim = (float)atof(optarg); break;
      case 'F': out = optarg; break;
      case 'M': mode = optarg; break;
      default: break;
    }
  }
  if (argc < 2 || !in1 || !in2) {
    fprintf(stderr, "usage: kmerLSH -a A.txt -b B.txt [-I iters] [-N min_sim] [-F out] [-M C --only]\n");
    return 1;
  }
  if (!mode.empty() && mode != "C") {
    fprintf(stderr, "kmerLSH (gfx950): only mode C (clustering) is implemented\n");
    return 1;
  }
  (void)only;
  const auto t0 = std::chrono::steady_clock::now();
  const int d = count_lines(in1) + count_lines(in2);

  FILE* lf = fopen("kmer_count.log", "r");
  if (!lf) {
    perror("kmer_count.log");
    return 1;
  }
  unsigned long long kmap = 0;
  if (fscanf(lf, "%llu", &kmap) != 1) return 1;
  std::vector<float> v_kmers(d);
  for (int j = 0; j < d; ++j) {  // ss >> float_t, then coverage / kmap_size (float)
    char buf[128];
    if (fscanf(lf, "%127s", buf) != 1) return 1;
    v_kmers[j] = strtof(buf, nullptr) / (float)kmap;
  }
  fclose(lf);
  std::vector<uint16_t> counts((size_t)kmap * d);
  FILE* bf = fopen("kmer_count.bin", "rb");
  if (!bf || fread(counts.data(), 2, counts.size(), bf) != counts.size()) {
    fprintf(stderr, "kmer_count.bin: short read\n");
    return 1;
  }
  fclose(bf);

  int err = 0;
  klsh_ctx* ctx = klsh_create(device, &err);
  if (!ctx) {
    fprintf(stderr, "kmerLSH: %s\n", klsh_last_error());
    return 2;
  }
  uint64_t counter = 0;
  const uint64_t batch_thresh = 100000000ull;
  float similarity = min_sim;
  RowSet cur;
  cur.d = d;
  bool resident = false;  // single batch: the init-pass state stays on the device
  {
    const uint64_t nbatch = kmap / batch_thresh;
    uint64_t offset = 0;
    for (uint64_t i = 0; i < nbatch + 1; ++i) {
      const uint64_t bs = (i == nbatch) ? kmap - offset : batch_thresh;
      check(klsh_load_counts(ctx, counts.data(), kmap, offset, bs, d, v_kmers.data()), "klsh_load_counts");
      run_cluster(ctx, similarity, 1, (int)(batch_thresh / 1000), seed, &counter, verbose);
      if (nbatch == 0) resident = true;
      else fetch(ctx, d, &cur);
      offset += bs;
    }
  }
  std::vector<uint16_t>().swap(counts);
  if (!resident) {
    while (cur.n() > batch_thresh) {  // app/kmerLSH.cc:354-411
      similarity = (float)((double)similarity - 0.001);
      const uint64_t nbatch = cur.n() / batch_thresh;
      RowSet next;
      next.d = d;
      uint64_t offset = 0;
      for (uint64_t i = 0; i < nbatch + 1; ++i) {
        const uint64_t bs = (i == nbatch) ? cur.n() - offset : batch_thresh;
        load_slice(ctx, cur, offset, bs);
        run_cluster(ctx, similarity, 1 + 4, (int)(batch_thresh / 1000), seed, &counter, verbose);
        fetch(ctx, d, &next);
        offset += bs;
      }
      cur = std::move(next);
    }
    load_slice(ctx, cur, 0, cur.n());
  }
  run_cluster(ctx, min_sim, iters, 1000000, seed, &counter, verbose);  // app/kmerLSH.cc:490

  RowSet fin;
  fin.d = d;
  fetch(ctx, d, &fin);
  klsh_destroy(ctx);

  // SaveResult / SaveBinary, ignore_small = 5 (app/kmerLSH.cc:498-499)
  const std::string clust = out + ".clust";
  FILE* fc = fopen(clust.c_str(), "wb");
  FILE* fb = fopen(out.c_str(), "wb");
  if (!fc || !fb) {
    perror("output");
    return 1;
  }
  std::vector<char> buf(1 << 22);
  char* p = buf.data();
  for (uint64_t i = 0; i < fin.n(); ++i) {
    const uint64_t a = fin.off[i], e = fin.off[i + 1];
    if (e - a <= 5) continue;
    fwrite(fin.rows.data() + i * d, sizeof(float), d, fb);
    for (uint64_t k = (uint64_t)-1; k == (uint64_t)-1 || k < e; k = (k == (uint64_t)-1) ? a : k + 1) {
      if ((size_t)(p - buf.data()) > buf.size() - 64) {
        fwrite(buf.data(), 1, p - buf.data(), fc);
        p = buf.data();
      }
      if (k == (uint64_t)-1) p = put_u64(p, e - a);
      else {
        *p++ = '\t';
        p = put_u64(p, fin.ids[k]);
      }
    }
    *p++ = '\n';
  }
  fwrite(buf.data(), 1, p - buf.data(), fc);
  fclose(fc);
  fclose(fb);
  const double secs =
      std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  printf("kmerLSH (gfx950) in total takes (secs): %g, clusters: %llu\n", secs,
         (unsigned long long)fin.n());
  return 0;
}
