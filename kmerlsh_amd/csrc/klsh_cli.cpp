// kmerLSH-compatible command line (modes C and E) over the gfx950 engine.
//
// Same flags and files as the reference (app/kmerLSH.cc:147-276, :432-580), run in the directory
// holding kmer_count.bin / kmer_count.log, with -a/-b sample lists ("<fastq> <kmc name>" lines):
//   mode C  writes <F>.clust ("<n>\t<id>\t...\n" per cluster with more than 5 members,
//           io/ioMatrix.cc:265-294) and <F> (raw fp32 centroids of the same clusters, :322-351);
//   mode E  reads <F> / <F>.clust back (io/ioMatrix.cc:48-119), tests every cluster with more than
//           -S members (AB::WRS, function/funcAB.cc:73-109), builds the two differential k-mer
//           sets from kmer_set.hex on the GPU and writes <o>_<sample> / <p>_<sample>: the reads
//           whose k-mer vote passes -V (IOFQ::Extracting, io/ioFastQ.cc:161-195).
//   mode B  reads the KMC databases named in the lists' second column and writes kmer_set.hex,
//           kmer_count.bin, kmer_count.log (io/ioHT.cc:83-199 with existing databases).
// Mode selection as the reference's (app/kmerLSH.cc:234-275): -M E [--only] extracts only,
// -M C --only clusters only, -M C clusters and then extracts, -M B --only builds the table only,
// -M B builds, clusters and extracts; mode K (running the KMC counter itself) is not part of
// this engine.
//   kmerLSH -a A.txt -b B.txt [-o A -p B] [-I iters] [-N min_sim] [-K k] [-S size] [-P pval]
//           [-V vote] [-F file] [-M C|E] [--only] [--verbose] [--seed S] [--device D]
// Additions: --seed (the reference seeds from std::random_device; SURVEY.md §8(c) convention)
// and --device.  -T is accepted and ignored (results never depend on a thread count).
// The init pass keeps the reference's 1e8-row batching and re-cluster passes
// (app/kmerLSH.cc:278-430); its tmp-file round trip is lossless and stays in memory.
#include <getopt.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <ctype.h>

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
  klsh_stats st{};
  st.struct_size = sizeof(st);
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

// GetInput (io/ioHT.cc:3-19): token `col` (0: the sample, 1: its KMC database name) of every line
// (std::getline) of a sample list
std::vector<std::string> sample_paths(const char* path, int col = 0) {
  std::vector<std::string> out;
  FILE* f = fopen(path, "rb");
  if (!f) {
    fprintf(stderr, "Unable to open info file");
    return out;
  }
  std::string line;
  int c;
  bool any = false;
  auto flush = [&]() {
    size_t a = 0, b = 0;
    for (int t = 0; t <= col; ++t) {
      a = b;
      while (a < line.size() && isspace((unsigned char)line[a])) ++a;
      b = a;
      while (b < line.size() && !isspace((unsigned char)line[b])) ++b;
    }
    out.push_back(line.substr(a, b - a));
    line.clear();
  };
  while ((c = fgetc(f)) != EOF) {
    any = true;
    if (c == '\n') flush();
    else line.push_back((char)c);
  }
  if (any && !line.empty()) flush();
  fclose(f);
  return out;
}

// Mode B (buildKHtable with kmc = false, io/ioHT.cc:83-199): the KMC databases named in the sample
// lists' second column -> kmer_set.hex / kmer_count.bin / kmer_count.log in the current directory.
int run_build(klsh_ctx* ctx, const char* in1, const char* in2, int k, bool verbose) {
  std::vector<std::string> names = sample_paths(in1, 1), n2 = sample_paths(in2, 1);
  names.insert(names.end(), n2.begin(), n2.end());
  std::vector<const char*> ptrs;
  for (const auto& n : names) ptrs.push_back(n.c_str());
  klsh_khtable_stats st{};
  st.struct_size = sizeof(st);
  check(klsh_build_khtable(ctx, ptrs.data(), (int)ptrs.size(), k, "", &st), "klsh_build_khtable");
  if (verbose)
    printf("k-mer table: %llu k-mers from %llu records of %zu databases (%.1f ms, %.1f ms reading)\n",
           (unsigned long long)st.kmap_size, (unsigned long long)st.records, names.size(),
           st.total_ms, st.io_ms);
  return 0;
}

// Mode E (app/kmerLSH.cc:521-580).
int run_extract(klsh_ctx* ctx, const std::vector<std::string>& s1,
                const std::vector<std::string>& s2, const std::string& clust_file,
                const std::string& out1, const std::string& out2, int k, int size_thresh,
                float pval, float vote, bool verbose) {
  const int n1 = (int)s1.size(), n2 = (int)s2.size(), d = n1 + n2;
  if (verbose) printf("Start to extract the differential reads from raw data\n");
  // IOMat::ReadClusterAll: centroid rows of <F>, member lists of <F>.clust, paired line by line
  FILE* fb = fopen(clust_file.c_str(), "rb");
  if (!fb) {
    printf("Error! file ( %s ) not open!\n", clust_file.c_str());
    return 1;
  }
  fseek(fb, 0, SEEK_END);
  const uint64_t line_cnt = d > 0 ? (uint64_t)ftell(fb) / (sizeof(float) * d) : 0;
  fseek(fb, 0, SEEK_SET);
  std::vector<float> values(line_cnt * (uint64_t)d);
  if (line_cnt && fread(values.data(), sizeof(float) * d, line_cnt, fb) != line_cnt) {
    fprintf(stderr, "kmerLSH: short read of %s\n", clust_file.c_str());
    return 1;
  }
  fclose(fb);
  const std::string cf = clust_file + ".clust";
  FILE* fc = fopen(cf.c_str(), "rb");
  if (!fc) {
    printf("Error! file ( %s ) not open!\n", cf.c_str());
    return 1;
  }
  std::vector<uint64_t> counts, ids, off{0};
  {
    std::string line;
    int c;
    auto parse = [&]() {  // strtol chain: n, then up to n ids, missing ones stay 0
      const char* p = line.c_str();
      char* e = nullptr;
      const uint64_t n = (uint64_t)strtol(p, &e, 10);
      uint64_t got = 0;
      std::vector<uint64_t> v(n, 0);
      while (p != e && got < n) {
        p = e;
        v[got++] = (uint64_t)strtol(p, &e, 10);
      }
      counts.push_back(n);
      ids.insert(ids.end(), v.begin(), v.end());
      off.push_back(ids.size());
      line.clear();
    };
    bool any = false;
    while ((c = fgetc(fc)) != EOF) {
      any = true;
      if (c == '\n') parse();
      else line.push_back((char)c);
    }
    if (any && !line.empty()) parse();
    fclose(fc);
  }
  if (counts.size() != line_cnt) {
    fprintf(stderr, "kmerLSH: %s has %zu clusters, %s %llu rows (the reference requires equal)\n",
            cf.c_str(), counts.size(), clust_file.c_str(), (unsigned long long)line_cnt);
    return 1;
  }
  std::vector<uint8_t> group(line_cnt);
  check(klsh_wrs(values.data(), line_cnt, n1, n2, counts.data(), pval, size_thresh, group.data()),
        "klsh_wrs");
  // kmer_count.log: kmap_size; kmer_set.hex: kmap_size k-mers of 8 bytes (Kmer::writeBytes)
  FILE* lf = fopen("kmer_count.log", "r");
  unsigned long long kmap = 0;
  if (!lf || fscanf(lf, "%llu", &kmap) != 1) {
    fprintf(stderr, "kmerLSH: kmer_count.log unreadable\n");
    return 1;
  }
  fclose(lf);
  // distinct ids per group (the reference's two unordered_sets); a k-mer goes to A if its id is in
  // A's set, else to B if in B's (app/kmerLSH.cc:565-571)
  std::vector<uint8_t> in1(kmap, 0), in2(kmap, 0);
  uint64_t na = 0, nb = 0;
  for (uint64_t c = 0; c < line_cnt; ++c)
    for (uint64_t q = off[c]; q < off[c + 1]; ++q) {
      if (ids[q] >= kmap) continue;
      if (group[c] == 1 && !in1[ids[q]]) in1[ids[q]] = 1, na += 1;
      if (group[c] == 2 && !in2[ids[q]]) in2[ids[q]] = 1, nb += 1;
    }
  if (verbose) {
    printf("# of differential kmers in group A : %llu\n", (unsigned long long)na);
    printf("# of differential kmers in group B : %llu\n", (unsigned long long)nb);
  }
  std::vector<uint64_t> kmers(kmap), k1, k2;
  FILE* kf = fopen("kmer_set.hex", "rb");
  if (!kf || fread(kmers.data(), 8, kmap, kf) != kmap) {
    fprintf(stderr, "kmerLSH: kmer_set.hex unreadable\n");
    return 1;
  }
  fclose(kf);
  for (uint64_t i = 0; i < kmap; ++i) {
    if (in1[i]) k1.push_back(kmers[i]);
    else if (in2[i]) k2.push_back(kmers[i]);
  }
  int err = 0;
  klsh_kset* set1 = klsh_kset_create(ctx, k1.data(), k1.size(), &err);
  check(err, "klsh_kset_create");
  klsh_kset* set2 = klsh_kset_create(ctx, k2.data(), k2.size(), &err);
  check(err, "klsh_kset_create");
  for (int g = 0; g < 2; ++g) {  // IOFQ::Extracting per group
    const auto& ss = g == 0 ? s1 : s2;
    const std::string& pre = g == 0 ? out1 : out2;
    if (verbose) printf("start %d threads\n", 1);
    for (const std::string& path : ss) {
      const size_t slash = path.find_last_of('/');
      const std::string base = slash == std::string::npos ? path : path.substr(slash + 1);
      const std::string out = pre + "_" + base;
      if (verbose) printf("writing to %s\n", out.c_str());
      fflush(stdout);
      klsh_extract_stats st{};
      st.struct_size = sizeof(st);
      check(klsh_extract_fastq(ctx, g == 0 ? set1 : set2, path.c_str(), out.c_str(), k, vote, &st),
            "klsh_extract_fastq");
      if (verbose)
        printf("  %llu reads, %llu extracted; k-mer vote kernel %.3f ms, parse %.3f ms\n",
               (unsigned long long)st.reads, (unsigned long long)st.reads_extracted, st.kernel_ms,
               st.parse_ms);
    }
  }
  klsh_kset_destroy(set1);
  klsh_kset_destroy(set2);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  const char *in1 = nullptr, *in2 = nullptr;
  std::string out = "clustering_result.txt", mode, out1, out2;
  int iters = 100, verbose = 0, only = 0, device = 0, kmer_k = 23, size_thresh = 500000;
  float min_sim = 0.80f, pval = 0.01f, vote = 0.5f;
  uint32_t seed = 12345u;
  static struct option lo[] = {{"verbose", no_argument, 0, 1},
                               {"only", no_argument, 0, 2},
                               {"seed", required_argument, 0, 3},
                               {"device", required_argument, 0, 4},
                               {"output1", required_argument, 0, 'o'},
                               {"output2", required_argument, 0, 'p'},
                               {"kmer_size", required_argument, 0, 'K'},
                               {"size_thresh", required_argument, 0, 'S'},
                               {"pval_thresh", required_argument, 0, 'P'},
                               {"kmer_vote", required_argument, 0, 'V'},
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
      case 'o': out1 = optarg; break;
      case 'p': out2 = optarg; break;
      case 'K': kmer_k = atoi(optarg); break;
      case 'S': size_thresh = atoi(optarg); break;
      case 'P': pval = (float)atof(optarg); break;
      case 'V': vote = (float)atof(optarg); break;
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
    fprintf(stderr, "usage: kmerLSH -a A.txt -b B.txt [-o A -p B] [-I iters] [-N min_sim] [-K k] "
                    "[-S size] [-P pval] [-V vote] [-F out] [-M C|E] [--only]\n");
    return 1;
  }
  if (mode != "B" && mode != "C" && mode != "E") {
    fprintf(stderr, "kmerLSH (gfx950): modes B (k-mer table from KMC databases), C (clustering) and "
                    "E (extraction) are implemented; K (running the KMC counter) is not: count "
                    "with KMC, then pass -M B\n");
    return 1;
  }
  // app/kmerLSH.cc:234-275: --only runs the named mode; without it the later modes follow
  const bool building = mode == "B", clustering = mode == "C" || (mode == "B" && !only);
  const bool extracting = mode == "E" || !only;
  const auto t0 = std::chrono::steady_clock::now();
  const int d = count_lines(in1) + count_lines(in2);
  if (building) {
    int err = 0;
    klsh_ctx* ctx = klsh_create(device, &err);
    if (!ctx) {
      fprintf(stderr, "kmerLSH: %s\n", klsh_last_error());
      return 2;
    }
    const int rc = run_build(ctx, in1, in2, kmer_k, verbose);
    klsh_destroy(ctx);
    if (rc || (!clustering && !extracting)) return rc;
  }
  if (!clustering) {
    int err = 0;
    klsh_ctx* ctx = klsh_create(device, &err);
    if (!ctx) {
      fprintf(stderr, "kmerLSH: %s\n", klsh_last_error());
      return 2;
    }
    const int rc = run_extract(ctx, sample_paths(in1), sample_paths(in2), out, out1, out2, kmer_k,
                               size_thresh, pval, vote, verbose);
    klsh_destroy(ctx);
    const double secs =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (verbose) printf("extracting reads takes (secs): %g\n", secs);
    return rc;
  }

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
  // app/kmerLSH.cc's 1e8-row batch size; KLSH_TEST_BATCH_THRESH overrides it for the tests that
  // pin the multi-batch init and re-cluster branch against the oracle's CLI (never set otherwise)
  uint64_t batch_thresh = 100000000ull;
  if (const char* e = getenv("KLSH_TEST_BATCH_THRESH"))
    if (strtoull(e, nullptr, 10) >= 1000) batch_thresh = strtoull(e, nullptr, 10);
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
  int rc = 0;
  if (extracting)
    rc = run_extract(ctx, sample_paths(in1), sample_paths(in2), out, out1, out2, kmer_k,
                     size_thresh, pval, vote, verbose);
  klsh_destroy(ctx);
  const double secs =
      std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  printf("kmerLSH (gfx950) in total takes (secs): %g, clusters: %llu\n", secs,
         (unsigned long long)fin.n());
  return rc;
}
