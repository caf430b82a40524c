/* TEST INFRASTRUCTURE ONLY — plain-C CPU restatement of the reference kmerLSH hot path.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
 * and only as the checker (or the timed CPU baseline).  The product (kmerlsh_amd/) never links,
 * loads or calls it.
 *
 * Parity status: PINNED.  The restatement is checked bit-for-bit against outputs of the
 * unmodified reference objects (built from /root/reference by oracle/Makefile into oracle/_ref/
 * and driven by oracle/ref_harness.cc) through the fixtures in tests/golden/, and against the
 * survey's end-to-end KAT md5s (katF, katG, katN).
 *
 * Semantics are the reference at T=1 (OMP_THREAD_LIMIT=1), seeded per SURVEY.md §8(c):
 * hyperplane k of a run is drawn from std::mt19937(base + k*2654435761).
 */
#ifndef KLSH_ORACLE_H
#define KLSH_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- RNG: libstdc++ (GCC 11) mt19937 + normal_distribution<double>, restated ---------------- */
typedef struct klsh_oracle_rng {
  uint32_t base;    /* KLSH_SEED */
  uint64_t counter; /* number of hyperplanes drawn so far (= reference rd() calls) */
} klsh_oracle_rng;

/* One hyperplane of d floats drawn from a fresh mt19937(seed) (reference hash/lshash.cc:3-17). */
void klsh_oracle_hyperplane(uint32_t seed, int d, float* w);
/* h hyperplanes (reference hash/lshash.cc:36-42), consuming h seeds from rng. w is h*d floats. */
void klsh_oracle_table(klsh_oracle_rng* rng, int h, int d, float* w);

/* ---- per-row / per-pair arithmetic ---------------------------------------------------------- */
/* key = MSB-first sign bits (reference hash/lshash.cc:44-59). */
uint32_t klsh_oracle_key(const float* x, int d, const float* w, int h);
/* 1 - dot/(sqrt|a|^2 sqrt|b|^2), sequential fp32 (reference function/distance.cc:27-38). */
float klsh_oracle_cosine(const float* cur, const float* cand, int d);
/* merge decision `1 - cosine >= thr` (reference function/cluster.cc:68-69). */
int klsh_oracle_decide(const float* cur, const float* cand, int d, float thr);
/* weighted mean (reference function/funcAB.cc:49-71). */
void klsh_oracle_consensus(const float* cur, uint32_t ca, const float* cand, uint32_t cb, int d,
                           float* out);

/* ---- the clustering loop --------------------------------------------------------------------- */
typedef struct klsh_oracle_state klsh_oracle_state;

/* rows: n*d fp32 row-major.  member_offsets: n+1 offsets into member_ids (NULL => row i is the
 * singleton {ids ? ids[i] : i}). */
klsh_oracle_state* klsh_oracle_create(const float* rows, uint64_t n, int d,
                                      const uint64_t* member_offsets, const uint64_t* member_ids);
void klsh_oracle_destroy(klsh_oracle_state* st);
uint64_t klsh_oracle_count(const klsh_oracle_state* st);
uint64_t klsh_oracle_members(const klsh_oracle_state* st);

/* Cluster() (reference function/cluster.cc:181-340) at T=1 semantics.
 * nt_trace (may be NULL) receives the live count at the start of each iteration (the reference's
 * "Size of profilings" line, cluster.cc:210) — `iters` entries; the function returns the number
 * of iterations run.  nthreads: OpenMP threads (results do not depend on it). */
int klsh_oracle_cluster(klsh_oracle_state* st, float min_similarity, int iters,
                        int bucket_size_threshold, klsh_oracle_rng* rng, uint64_t* nt_trace,
                        int nthreads);

/* The first run_iters iterations of Cluster(..., iters, ...): the threshold schedule of an
 * `iters`-iteration call (sim_step = (0.95 - min_similarity) / iters), stopped early.  Pins the
 * prefixes of the long configs (C4, C5) whose full loops the oracle cannot finish quickly. */
int klsh_oracle_cluster_prefix(klsh_oracle_state* st, float min_similarity, int iters,
                               int run_iters, int bucket_size_threshold, klsh_oracle_rng* rng,
                               uint64_t* nt_trace, int nthreads);

/* p_cluster (reference function/cluster.cc:56-87) over the live rows taken as ONE bucket in
 * their current order; survivors become the live rows.  Returns the survivor count. */
uint64_t klsh_oracle_pcluster(klsh_oracle_state* st, float threshold);

/* Output in canonical order: rows (count*d), member_offsets (count+1), member_ids (members). */
void klsh_oracle_result(const klsh_oracle_state* st, float* rows, uint64_t* member_offsets,
                        uint64_t* member_ids);

/* ---- mode-C producer (reference io/ioMatrix.cc:353-408) --------------------------------------- */
/* counts: sample-major d x n uint16 (column stride n_total starting at batch_offset).  Writes the
 * kept rows (sum of counts > 0.1*d) and their ids (batch_offset + i).  Returns the kept count. */
uint64_t klsh_oracle_convert(const uint16_t* counts, uint64_t n_total, uint64_t batch_offset,
                             uint64_t batch_size, int d, const float* v_kmers, float* rows_out,
                             uint64_t* ids_out);

#ifdef __cplusplus
}
#endif
#endif
