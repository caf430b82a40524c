/* TEST INFRASTRUCTURE ONLY — plain-C CPU restatement of the reference kmerLSH hot path.
 * See klsh_oracle.h for who may use it.  Parity: PINNED against oracle/_ref outputs
 * (tests/golden/) and the SURVEY.md §8(c) KATs.
 *
 * Every function cites the reference file:line (under /root/reference) it restates.
 * Compile with -ffp-contract=off and without -ffast-math/-march: the reference is scalar SSE fp32
 * (mulss/addss/divss/sqrtss, no FMA).
 */
#include "klsh_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

/* ============================================================================ RNG ============ */
/* std::mt19937 (libstdc++ bits/random.tcc: seed(), _M_gen_rand(), operator()). */
typedef struct mt19937 {
  uint32_t x[624];
  int p;
} mt19937;

static void mt_seed(mt19937* m, uint32_t s) {
  m->x[0] = s;
  for (int i = 1; i < 624; ++i) m->x[i] = 1812433253u * (m->x[i - 1] ^ (m->x[i - 1] >> 30)) + (uint32_t)i;
  m->p = 624;
}

static void mt_twist(mt19937* m) {
  const uint32_t upper = 0x80000000u, lower = 0x7fffffffu, a = 0x9908b0dfu;
  int k;
  for (k = 0; k < 624 - 397; ++k) {
    uint32_t y = (m->x[k] & upper) | (m->x[k + 1] & lower);
    m->x[k] = m->x[k + 397] ^ (y >> 1) ^ ((y & 1u) ? a : 0u);
  }
  for (; k < 623; ++k) {
    uint32_t y = (m->x[k] & upper) | (m->x[k + 1] & lower);
    m->x[k] = m->x[k + 397 - 624] ^ (y >> 1) ^ ((y & 1u) ? a : 0u);
  }
  uint32_t y = (m->x[623] & upper) | (m->x[0] & lower);
  m->x[623] = m->x[396] ^ (y >> 1) ^ ((y & 1u) ? a : 0u);
  m->p = 0;
}

static uint32_t mt_next(mt19937* m) {
  if (m->p >= 624) mt_twist(m);
  uint32_t z = m->x[m->p++];
  z ^= (z >> 11) & 0xffffffffu;
  z ^= (z << 7) & 0x9d2c5680u;
  z ^= (z << 15) & 0xefc60000u;
  z ^= (z >> 18);
  return z;
}

/* std::generate_canonical<double, 53>(mt19937): two 32-bit draws, low word first, summed in
 * double (one rounding), scaled by 2^-64 (libstdc++ bits/random.tcc generate_canonical). */
static double mt_canonical(mt19937* m) {
  double sum = 0.0, tmp = 1.0;
  for (int k = 0; k < 2; ++k) {
    sum += (double)mt_next(m) * tmp;
    tmp *= 4294967296.0;
  }
  double ret = sum / tmp;
  if (ret >= 1.0) ret = nextafter(1.0, 0.0);
  return ret;
}

/* One hyperplane: fresh engine + fresh normal_distribution<double>(0,1) (Marsaglia polar method
 * with one saved value, libstdc++ bits/random.tcc normal_distribution::operator()), each draw
 * cast to float (reference hash/lshash.cc:3-17). */
void klsh_oracle_hyperplane(uint32_t seed, int d, float* w) {
  mt19937 m;
  mt_seed(&m, seed);
  int saved_available = 0;
  double saved = 0.0;
  for (int i = 0; i < d; ++i) {
    double ret;
    if (saved_available) {
      saved_available = 0;
      ret = saved;
    } else {
      double x, y, r2;
      do {
        x = 2.0 * mt_canonical(&m) - 1.0;
        y = 2.0 * mt_canonical(&m) - 1.0;
        r2 = x * x + y * y;
      } while (r2 > 1.0 || r2 == 0.0);
      const double mult = sqrt(-2.0 * log(r2) / r2);
      saved = x * mult;
      saved_available = 1;
      ret = y * mult;
    }
    ret = ret * 1.0 + 0.0; /* stddev 1, mean 0 */
    w[i] = (float)ret;
  }
}

/* reference hash/lshash.cc:36-42 — one rd() (here: one seed) per hyperplane, in order. */
void klsh_oracle_table(klsh_oracle_rng* rng, int h, int d, float* w) {
  for (int j = 0; j < h; ++j) {
    const uint32_t seed = rng->base + (uint32_t)rng->counter * 2654435761u;
    rng->counter++;
    klsh_oracle_hyperplane(seed, d, w + (size_t)j * d);
  }
}

/* ==================================================================== arithmetic =========== */
/* reference hash/lshash.cc:44-51 (sum >= 0 -> 1) and :53-59 (key = key*2 + bit). */
uint32_t klsh_oracle_key(const float* x, int d, const float* w, int h) {
  uint32_t key = 0;
  for (int j = 0; j < h; ++j) {
    const float* f = w + (size_t)j * d;
    float sum = 0.0f;
    for (int i = 0; i < d; ++i) sum += f[i] * x[i];
    key = key * 2u + (sum >= 0.0f ? 1u : 0u);
  }
  return key;
}

/* reference function/distance.cc:27-38. lhs = current row, rhs = candidate row. */
float klsh_oracle_cosine(const float* lhs, const float* rhs, int d) {
  float similarity = 0.0f, magnitude_lhs = 0.0f, magnitude_rhs = 0.0f;
  for (int i = 0; i < d; ++i) {
    similarity += lhs[i] * rhs[i];
    magnitude_lhs += lhs[i] * lhs[i];
    magnitude_rhs += rhs[i] * rhs[i];
  }
  similarity /= sqrtf(magnitude_lhs) * sqrtf(magnitude_rhs);
  return 1.0f - similarity;
}

/* reference function/cluster.cc:68-69: `1 - distance >= threshold`, all float. */
int klsh_oracle_decide(const float* cur, const float* cand, int d, float thr) {
  const float distance = klsh_oracle_cosine(cur, cand, d);
  return (1.0f - distance) >= thr;
}

/* reference function/funcAB.cc:49-71: new[i] = v1[i]*c1/n + v2[i]*c2/n, ab1 = current. */
void klsh_oracle_consensus(const float* cur, uint32_t ca, const float* cand, uint32_t cb, int d,
                           float* out) {
  const int c1 = (int)ca, c2 = (int)cb, all = c1 + c2;
  const float f1 = (float)c1, f2 = (float)c2, fa = (float)all;
  for (int i = 0; i < d; ++i) out[i] = cur[i] * f1 / fa + cand[i] * f2 / fa;
}

/* ===================================================================== state ================ */
struct klsh_oracle_state {
  int d;
  uint64_t n0;       /* slots */
  uint64_t members;  /* member nodes */
  float* x;          /* n0*d */
  uint32_t* cnt;     /* members per slot */
  uint64_t* head;    /* first member node of slot */
  uint64_t* tail;    /* last member node of slot */
  uint64_t* next;    /* member node -> next node (UINT64_MAX = end) */
  uint64_t* ids;     /* member node -> k-mer id */
  uint32_t* order;   /* live slots, canonical order */
  uint64_t n;        /* live count */
};

#define NIL UINT64_MAX

klsh_oracle_state* klsh_oracle_create(const float* rows, uint64_t n, int d,
                                      const uint64_t* member_offsets, const uint64_t* member_ids) {
  klsh_oracle_state* st = (klsh_oracle_state*)calloc(1, sizeof(*st));
  st->d = d;
  st->n0 = n;
  st->n = n;
  st->members = member_offsets ? member_offsets[n] : n;
  st->x = (float*)malloc(sizeof(float) * (n * (size_t)d + 1));
  if (n) memcpy(st->x, rows, sizeof(float) * n * (size_t)d);
  st->cnt = (uint32_t*)malloc(sizeof(uint32_t) * (n + 1));
  st->head = (uint64_t*)malloc(sizeof(uint64_t) * (n + 1));
  st->tail = (uint64_t*)malloc(sizeof(uint64_t) * (n + 1));
  st->order = (uint32_t*)malloc(sizeof(uint32_t) * (n + 1));
  st->next = (uint64_t*)malloc(sizeof(uint64_t) * (st->members + 1));
  st->ids = (uint64_t*)malloc(sizeof(uint64_t) * (st->members + 1));
  for (uint64_t i = 0; i < n; ++i) {
    st->order[i] = (uint32_t)i;
    if (member_offsets) {
      const uint64_t a = member_offsets[i], b = member_offsets[i + 1];
      st->cnt[i] = (uint32_t)(b - a);
      st->head[i] = (b > a) ? a : NIL;
      st->tail[i] = (b > a) ? b - 1 : NIL;
      for (uint64_t m = a; m < b; ++m) {
        st->ids[m] = member_ids[m];
        st->next[m] = (m + 1 < b) ? m + 1 : NIL;
      }
    } else {
      st->cnt[i] = 1;
      st->head[i] = st->tail[i] = i;
      st->ids[i] = member_ids ? member_ids[i] : i;
      st->next[i] = NIL;
    }
  }
  return st;
}

void klsh_oracle_destroy(klsh_oracle_state* st) {
  if (!st) return;
  free(st->x); free(st->cnt); free(st->head); free(st->tail);
  free(st->next); free(st->ids); free(st->order);
  free(st);
}

uint64_t klsh_oracle_count(const klsh_oracle_state* st) { return st->n; }
uint64_t klsh_oracle_members(const klsh_oracle_state* st) { return st->members; }

/* Merge slot `cur` (row i) into slot `cand` (row j): the new Abundance replaces candidates[j]
 * (reference function/cluster.cc:70-74); ids = ids_cur ++ ids_cand (funcAB.cc:51-55). */
static void merge_into(klsh_oracle_state* st, uint32_t cur, uint32_t cand) {
  const int d = st->d;
  float* xc = st->x + (size_t)cur * d;
  float* xj = st->x + (size_t)cand * d;
  float tmp[4096];
  float* out = d <= 4096 ? tmp : (float*)malloc(sizeof(float) * d);
  klsh_oracle_consensus(xc, st->cnt[cur], xj, st->cnt[cand], d, out);
  memcpy(xj, out, sizeof(float) * d);
  if (out != tmp) free(out);
  st->cnt[cand] = st->cnt[cur] + st->cnt[cand];
  if (st->head[cur] != NIL) {
    if (st->head[cand] != NIL) st->next[st->tail[cur]] = st->head[cand];
    else st->tail[cand] = st->tail[cur];
    st->head[cand] = st->head[cur];
  }
  st->cnt[cur] = 0;
  st->head[cur] = st->tail[cur] = NIL;
}

/* reference function/cluster.cc:56-87 (p_cluster): first-fit greedy, swap-remove.  Works in place
 * on s[0..b) and returns the survivor count; survivors are s[0..size) in final array order. */
static uint64_t p_cluster(klsh_oracle_state* st, uint32_t* s, uint64_t b, float thr) {
  const int d = st->d;
  uint64_t size = b, i = 1;
  while (i < size) {
    const float* xi = st->x + (size_t)s[i] * d;
    uint64_t j;
    for (j = 0; j < i; ++j) {
      if (klsh_oracle_decide(xi, st->x + (size_t)s[j] * d, d, thr)) {
        merge_into(st, s[i], s[j]);
        s[i] = s[--size];
        break;
      }
    }
    if (j == i) ++i;
  }
  return size;
}

/* `size > bucket_size_threshold` with size_t size and int threshold (cluster.cc:286): the int is
 * converted to size_t, so a negative threshold never triggers. */
static int oversize(uint64_t size, int thr) { return thr >= 0 && size > (uint64_t)thr; }

static int floor_log2_count(uint64_t n) { /* floor(log2(n)) in double (cluster.cc:194,203) */
  return (int)floor(log2((double)n));
}

/* Stable counting sort of s[0..n) by key into dst (reference function/cluster.cc:15-30,
 * merge_hashtable: push_back in original order).  start must hold nb+1 entries. */
static void bucket_sort(const uint32_t* s, const uint32_t* keys, uint64_t n, uint64_t nb,
                        uint32_t* dst, uint64_t* start) {
  memset(start, 0, sizeof(uint64_t) * (nb + 1));
  for (uint64_t p = 0; p < n; ++p) start[keys[p] + 1]++;
  for (uint64_t b = 0; b < nb; ++b) start[b + 1] += start[b];
  uint64_t* fill = (uint64_t*)malloc(sizeof(uint64_t) * (nb + 1));
  memcpy(fill, start, sizeof(uint64_t) * (nb + 1));
  for (uint64_t p = 0; p < n; ++p) dst[fill[keys[p]]++] = s[p];
  free(fill);
}

/* reference function/cluster.cc:89-178 (nestedCluster): one fresh LSH split of an oversize
 * bucket (table w of h rows, drawn by the caller in bucket order), then p_cluster per
 * sub-bucket; survivors concatenated in sub-bucket order into s[0..). No recursion. */
static uint64_t nested_cluster(klsh_oracle_state* st, uint32_t* s, uint64_t b, float thr,
                               const float* w, int h) {
  const int d = st->d;
  const uint64_t nb = (uint64_t)1 << h;
  uint32_t* keys = (uint32_t*)malloc(sizeof(uint32_t) * b);
  uint32_t* tmp = (uint32_t*)malloc(sizeof(uint32_t) * b);
  uint64_t* start = (uint64_t*)malloc(sizeof(uint64_t) * (nb + 1));
  for (uint64_t p = 0; p < b; ++p) keys[p] = klsh_oracle_key(st->x + (size_t)s[p] * d, d, w, h);
  bucket_sort(s, keys, b, nb, tmp, start);
  uint64_t out = 0;
  for (uint64_t k = 0; k < nb; ++k) {
    const uint64_t a = start[k], e = start[k + 1];
    if (e == a) continue;
    const uint64_t c = p_cluster(st, tmp + a, e - a, thr);
    memmove(s + out, tmp + a, sizeof(uint32_t) * c);
    out += c;
  }
  free(keys); free(tmp); free(start);
  return out;
}

/* reference function/cluster.cc:181-340 (Cluster), T=1 semantics. */
int klsh_oracle_cluster(klsh_oracle_state* st, float min_similarity, int iters,
                        int bucket_size_threshold, klsh_oracle_rng* rng, uint64_t* nt_trace,
                        int nthreads) {
  return klsh_oracle_cluster_prefix(st, min_similarity, iters, iters, bucket_size_threshold, rng,
                                    nt_trace, nthreads);
}

int klsh_oracle_cluster_prefix(klsh_oracle_state* st, float min_similarity, int iters,
                               int run_iters, int bucket_size_threshold, klsh_oracle_rng* rng,
                               uint64_t* nt_trace, int nthreads) {
  const int d = st->d;
  const float max_similarity = 0.95f;
  const float sim_step = (max_similarity - min_similarity) / (float)iters;
  float threshold = max_similarity;
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#else
  (void)nthreads;
#endif
  int it;
  if (run_iters > iters) run_iters = iters;
  for (it = 0; it < run_iters; ++it) {
    const uint64_t n = st->n;
    if (nt_trace) nt_trace[it] = n;
    if (n == 0) { /* reference aborts here (floor(log2(0)) -> size_t); we no-op */
      threshold -= sim_step;
      continue;
    }
    const int h = floor_log2_count(n);
    const uint64_t nb = (uint64_t)1 << h;
    float* w = (float*)malloc(sizeof(float) * ((size_t)h * d + 1));
    klsh_oracle_table(rng, h, d, w);

    uint32_t* keys = (uint32_t*)malloc(sizeof(uint32_t) * n);
#pragma omp parallel for schedule(static) num_threads(nthreads)
    for (int64_t p = 0; p < (int64_t)n; ++p)
      keys[p] = klsh_oracle_key(st->x + (size_t)st->order[p] * d, d, w, h);

    uint32_t* sorted = (uint32_t*)malloc(sizeof(uint32_t) * n);
    uint64_t* start = (uint64_t*)malloc(sizeof(uint64_t) * (nb + 1));
    bucket_sort(st->order, keys, n, nb, sorted, start);

    /* Oversize buckets draw their nested tables in ascending bucket order (T=1 RNG order). */
    uint64_t n_over = 0;
    for (uint64_t k = 0; k < nb; ++k)
      if (oversize(start[k + 1] - start[k], bucket_size_threshold)) n_over++;
    uint64_t* over_bucket = (uint64_t*)malloc(sizeof(uint64_t) * (n_over + 1));
    int* over_h = (int*)malloc(sizeof(int) * (n_over + 1));
    float** over_w = (float**)malloc(sizeof(float*) * (n_over + 1));
    n_over = 0;
    for (uint64_t k = 0; k < nb; ++k) {
      const uint64_t b = start[k + 1] - start[k];
      if (oversize(b, bucket_size_threshold)) {
        over_bucket[n_over] = k;
        over_h[n_over] = floor_log2_count(b);
        over_w[n_over] = (float*)malloc(sizeof(float) * ((size_t)over_h[n_over] * d + 1));
        klsh_oracle_table(rng, over_h[n_over], d, over_w[n_over]);
        n_over++;
      }
    }

    /* Buckets are independent and write their survivors in place: output is positional, so
     * any thread count gives the T=1 result. */
    uint64_t* surv = (uint64_t*)malloc(sizeof(uint64_t) * (nb + 1));
    uint64_t oi = 0;
#pragma omp parallel for schedule(dynamic, 256) num_threads(nthreads)
    for (int64_t k = 0; k < (int64_t)nb; ++k) {
      const uint64_t a = start[k], b = start[k + 1] - start[k];
      if (oversize(b, bucket_size_threshold)) continue;
      surv[k] = b ? p_cluster(st, sorted + a, b, threshold) : 0;
    }
    for (oi = 0; oi < n_over; ++oi) {
      const uint64_t k = over_bucket[oi];
      surv[k] = nested_cluster(st, sorted + start[k], start[k + 1] - start[k], threshold,
                               over_w[oi], over_h[oi]);
      free(over_w[oi]);
    }
    /* merge_abundance (cluster.cc:39-45): concatenate survivors in bucket order. */
    uint64_t out = 0;
    for (uint64_t k = 0; k < nb; ++k) {
      memmove(st->order + out, sorted + start[k], sizeof(uint32_t) * surv[k]);
      out += surv[k];
    }
    st->n = out;
    free(w); free(keys); free(sorted); free(start); free(surv);
    free(over_bucket); free(over_h); free(over_w);
    threshold -= sim_step;
  }
  return it;
}

uint64_t klsh_oracle_pcluster(klsh_oracle_state* st, float threshold) {
  st->n = p_cluster(st, st->order, st->n, threshold);
  return st->n;
}

void klsh_oracle_result(const klsh_oracle_state* st, float* rows, uint64_t* member_offsets,
                        uint64_t* member_ids) {
  const int d = st->d;
  uint64_t m = 0;
  for (uint64_t p = 0; p < st->n; ++p) {
    const uint32_t s = st->order[p];
    if (rows) memcpy(rows + p * (size_t)d, st->x + (size_t)s * d, sizeof(float) * d);
    if (member_offsets) member_offsets[p] = m;
    for (uint64_t node = st->head[s]; node != NIL; node = st->next[node]) {
      if (member_ids) member_ids[m] = st->ids[node];
      m++;
    }
  }
  if (member_offsets) member_offsets[st->n] = m;
}

/* ==================================================================== mode C ================ */
/* reference io/ioMatrix.cc:353-408 (convertHTMat), with io/ioHT.cc:59-81 (ReadHT) layout:
 * counts are sample-major, sample j's column starts at j*n_total. */
uint64_t klsh_oracle_convert(const uint16_t* counts, uint64_t n_total, uint64_t batch_offset,
                             uint64_t batch_size, int d, const float* v_kmers, float* rows_out,
                             uint64_t* ids_out) {
  uint64_t kept = 0;
  float* values = (float*)malloc(sizeof(float) * (d + 1));
  for (uint64_t i = 0; i < batch_size; ++i) {
    uint64_t total_cnt = 0;
    for (int j = 0; j < d; ++j) {
      const uint64_t cnt = counts[(size_t)j * n_total + batch_offset + i];
      total_cnt += cnt;
      values[j] = (float)log((double)cnt + 1.0) - v_kmers[j];
    }
    if ((double)total_cnt > 0.1 * d) {
      memcpy(rows_out + kept * (size_t)d, values, sizeof(float) * d);
      ids_out[kept] = batch_offset + i;
      kept++;
    }
  }
  free(values);
  return kept;
}
