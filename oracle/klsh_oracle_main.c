/* TEST INFRASTRUCTURE ONLY — mode-C command line over the oracle restatement, used to pin the
 * restatement against the reference's end-to-end KATs.
 *
 * Mirrors reference app/kmerLSH.cc: flags (:147-276), kmerCluster mode C (:432-520),
 * init_clustering (:278-430) including its 1e8-row batching, and the writers
 * io/ioMatrix.cc:265-294 (SaveResult) / :322-351 (SaveBinary).  The tmp-file round trip of the
 * reference (SaveBinary/ReadClusterAll) is lossless, so it is done in memory here.
 *
 *   klsh_oracle -a A.txt -b B.txt [-I iters] [-N min_sim] [-F out] [-T threads] [--seed S]
 *               [--verbose] [-M C --only]        (run in the directory holding kmer_count.*)
 */
#include <getopt.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "klsh_oracle.h"

static int count_lines(const char* path) { /* std::getline loop count (io/ioHT.cc:3-19) */
  FILE* f = fopen(path, "rb");
  if (!f) { fprintf(stderr, "Unable to open info file"); return 0; }
  int n = 0, c, last = '\n', any = 0;
  while ((c = fgetc(f)) != EOF) { any = 1; if (c == '\n') n++; last = c; }
  fclose(f);
  if (any && last != '\n') n++;
  return n;
}

typedef struct rowset { /* a vector<Abundance*> in flat form */
  float* rows;
  uint64_t n, cap;
  uint64_t* off; /* n+1 */
  uint64_t* ids;
  uint64_t m, mcap;
} rowset;

static void rs_append(rowset* r, int d, const float* rows, uint64_t n, const uint64_t* off,
                      const uint64_t* ids) {
  if (r->n + n > r->cap) {
    r->cap = (r->n + n) * 2 + 16;
    r->rows = realloc(r->rows, sizeof(float) * r->cap * d);
    r->off = realloc(r->off, sizeof(uint64_t) * (r->cap + 1));
  }
  const uint64_t nm = off[n] - off[0];
  if (r->m + nm > r->mcap) {
    r->mcap = (r->m + nm) * 2 + 16;
    r->ids = realloc(r->ids, sizeof(uint64_t) * r->mcap);
  }
  memcpy(r->rows + r->n * d, rows, sizeof(float) * n * d);
  if (r->n == 0) r->off[0] = 0;
  for (uint64_t i = 0; i < n; ++i) r->off[r->n + i + 1] = r->m + (off[i + 1] - off[0]);
  memcpy(r->ids + r->m, ids + off[0], sizeof(uint64_t) * nm);
  r->n += n;
  r->m += nm;
}

/* Cluster() over rows [a, a+n) of src, appending survivors to dst. */
static void cluster_batch(const rowset* src, uint64_t a, uint64_t n, int d, float min_sim,
                          int iters, int bthr, klsh_oracle_rng* rng, int threads, int verbose,
                          rowset* dst) {
  uint64_t* off = malloc(sizeof(uint64_t) * (n + 1));
  for (uint64_t i = 0; i <= n; ++i) off[i] = src->off[a + i] - src->off[a];
  klsh_oracle_state* st =
      klsh_oracle_create(src->rows + a * d, n, d, off, src->ids + src->off[a]);
  uint64_t* trace = malloc(sizeof(uint64_t) * (iters > 0 ? iters : 1));
  const int ran = klsh_oracle_cluster(st, min_sim, iters, bthr, rng, trace, threads);
  if (verbose)
    for (int t = 0; t < ran; ++t) printf("Size of profilings : %llu\n", (unsigned long long)trace[t]);
  const uint64_t c = klsh_oracle_count(st), m = klsh_oracle_members(st);
  float* rows = malloc(sizeof(float) * (c * d + 1));
  uint64_t* o2 = malloc(sizeof(uint64_t) * (c + 1));
  uint64_t* ids = malloc(sizeof(uint64_t) * (m + 1));
  klsh_oracle_result(st, rows, o2, ids);
  rs_append(dst, d, rows, c, o2, ids);
  free(rows); free(o2); free(ids); free(trace); free(off);
  klsh_oracle_destroy(st);
}

int main(int argc, char** argv) {
  const char *in1 = NULL, *in2 = NULL, *out = "clustering_result.txt", *mode = "";
  int iters = 100, threads = 0, verbose = 0, only = 0;
  float min_sim = 0.80f;
  uint32_t seed = 12345u;
  static struct option lo[] = {{"verbose", no_argument, 0, 1},  {"only", no_argument, 0, 2},
                               {"seed", required_argument, 0, 3}, {"input1", required_argument, 0, 'a'},
                               {"input2", required_argument, 0, 'b'}, {0, 0, 0, 0}};
  int c;
  while ((c = getopt_long(argc, argv, "o:p:a:b:H:I:N:X:C:T:K:S:P:V:F:M:", lo, NULL)) != -1) {
    switch (c) {
      case 1: verbose = 1; break;
      case 2: only = 1; break;
      case 3: seed = (uint32_t)strtoul(optarg, NULL, 10); break;
      case 'a': in1 = optarg; break;
      case 'b': in2 = optarg; break;
      case 'I': iters = atoi(optarg); break;
      case 'N': min_sim = (float)atof(optarg); break;
      case 'T': threads = atoi(optarg); break;
      case 'F': out = optarg; break;
      case 'M': mode = optarg; break;
      default: break;
    }
  }
  (void)only;
  if (strcmp(mode, "C") != 0) fprintf(stderr, "klsh_oracle: only mode C is restated\n");
  if (!in1 || !in2) { fprintf(stderr, "need -a and -b\n"); return 1; }
  const int d = count_lines(in1) + count_lines(in2);

  /* kmer_count.log: kmap_size then one coverage per sample (app/kmerLSH.cc:471-482). */
  FILE* lf = fopen("kmer_count.log", "r");
  if (!lf) { perror("kmer_count.log"); return 1; }
  unsigned long long kmap = 0;
  if (fscanf(lf, "%llu", &kmap) != 1) return 1;
  float* v_kmers = malloc(sizeof(float) * d);
  for (int j = 0; j < d; ++j) {
    char buf[128];
    if (fscanf(lf, "%127s", buf) != 1) return 1;
    const float cov = strtof(buf, NULL);
    v_kmers[j] = cov / (float)kmap;
  }
  fclose(lf);

  FILE* bf = fopen("kmer_count.bin", "rb");
  if (!bf) { perror("kmer_count.bin"); return 1; }
  uint16_t* counts = malloc(sizeof(uint16_t) * ((size_t)kmap * d + 1));
  if (fread(counts, 2, (size_t)kmap * d, bf) != (size_t)kmap * d) { fprintf(stderr, "short bin\n"); return 1; }
  fclose(bf);

  klsh_oracle_rng rng = {seed, 0};
  /* app/kmerLSH.cc's 1e8-row batch size; KLSH_TEST_BATCH_THRESH (>= 1000) overrides it for the
   * tests of the multi-batch init and re-cluster branch */
  uint64_t batch_thresh = 100000000ull;
  {
    const char* e = getenv("KLSH_TEST_BATCH_THRESH");
    if (e && strtoull(e, NULL, 10) >= 1000) batch_thresh = strtoull(e, NULL, 10);
  }
  rowset cur = {0}, next = {0};
  /* init_clustering first pass (app/kmerLSH.cc:303-345): batches of 1e8 rows, I=1, bthr 1e5. */
  float similarity = min_sim;
  {
    const uint64_t nbatch = kmap / batch_thresh;
    uint64_t offset = 0;
    float* rows = malloc(sizeof(float) * ((kmap < batch_thresh ? kmap : batch_thresh) * d + 1));
    uint64_t* ids = malloc(sizeof(uint64_t) * ((kmap < batch_thresh ? kmap : batch_thresh) + 1));
    for (uint64_t i = 0; i < nbatch + 1; ++i) {
      const uint64_t bs = (i == nbatch) ? kmap - offset : batch_thresh;
      const uint64_t kept = klsh_oracle_convert(counts, kmap, offset, bs, d, v_kmers, rows, ids);
      rowset b = {0};
      uint64_t* off = malloc(sizeof(uint64_t) * (kept + 1));
      for (uint64_t k = 0; k <= kept; ++k) off[k] = k;
      rs_append(&b, d, rows, kept, off, ids);
      free(off);
      cluster_batch(&b, 0, kept, d, similarity, 1, (int)(batch_thresh / 1000), &rng, threads,
                    verbose, &cur);
      free(b.rows); free(b.off); free(b.ids);
      offset += bs;
    }
    free(rows); free(ids);
  }
  free(counts);
  /* re-cluster passes while more than 1e8 rows remain (app/kmerLSH.cc:354-411). */
  while (cur.n > batch_thresh) {
    similarity = (float)((double)similarity - 0.001);
    const uint64_t nbatch = cur.n / batch_thresh;
    uint64_t offset = 0;
    memset(&next, 0, sizeof(next));
    for (uint64_t i = 0; i < nbatch + 1; ++i) {
      const uint64_t bs = (i == nbatch) ? cur.n - offset : batch_thresh;
      cluster_batch(&cur, offset, bs, d, similarity, 1 + 4, (int)(batch_thresh / 1000), &rng,
                    threads, verbose, &next);
      offset += bs;
    }
    free(cur.rows); free(cur.off); free(cur.ids);
    cur = next;
  }
  /* main loop (app/kmerLSH.cc:490), bucket threshold 1e6 (:440). */
  rowset fin = {0};
  cluster_batch(&cur, 0, cur.n, d, min_sim, iters, 1000000, &rng, threads, verbose, &fin);

  /* SaveResult / SaveBinary with ignore_small = 5 (app/kmerLSH.cc:498-499). */
  char path[4096];
  snprintf(path, sizeof(path), "%s.clust", out);
  FILE* fc = fopen(path, "wb");
  FILE* fb = fopen(out, "wb");
  for (uint64_t i = 0; i < fin.n; ++i) {
    const uint64_t a = fin.off[i], e = fin.off[i + 1];
    if (e - a > 5) {
      fprintf(fc, "%llu", (unsigned long long)(e - a));
      for (uint64_t k = a; k < e; ++k) fprintf(fc, "\t%llu", (unsigned long long)fin.ids[k]);
      fputc('\n', fc);
      fwrite(fin.rows + i * d, sizeof(float), d, fb);
    }
  }
  fclose(fc);
  fclose(fb);
  printf("clusters: %llu\n", (unsigned long long)fin.n);
  free(v_kmers);
  free(cur.rows); free(cur.off); free(cur.ids);
  free(fin.rows); free(fin.off); free(fin.ids);
  return 0;
}
