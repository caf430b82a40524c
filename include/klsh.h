/* klsh — MI355X-native LSH k-mer clustering engine: the C-ABI drop-in boundary.
 *
 * The reference (wthanone/kmerLSH) has no plugin/FFI layer; its seam for this hot path is the C++
 * function
 *     void Cluster(vector<Abundance*>* rows, float min_similarity, int cluster_iteration,
 *                  unsigned threads_to_use, int dim, int bucket_size_threshold, bool verbose)
 * (reference function/cluster.h:42, body function/cluster.cc:181-340), called from
 * app/kmerLSH.cc:323 (init pass), :377 (re-cluster passes) and :490 (main loop).  The entry points
 * below replace that call and the functions on its path; include/klsh_cluster.hpp wraps them back
 * into the reference's exact signature.
 *
 * Conventions: every int-returning call returns 0 or a negative KLSH_E_* code; no C++ exception
 * crosses this boundary.  The library owns device memory; the caller owns every host buffer
 * (size queries first: klsh_count).  One context per host thread; not re-entrant on one context.
 * All host pointers are plain host memory; nothing here takes or returns a torch type.
 *
 * Determinism: results equal the reference at -T 1 (OMP_THREAD_LIMIT=1) with the seeding
 * convention of SURVEY.md §8(c): hyperplane k of a run is drawn from
 * std::mt19937(seed_base + k*2654435761) with std::normal_distribution<double>(0,1), cast to
 * float.  `rng_counter` carries k across calls (init pass, then main loop).
 */
#ifndef KLSH_H
#define KLSH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KLSH_OK 0
#define KLSH_E_ARG (-1)      /* bad argument (null pointer, d <= 0, sizes) */
#define KLSH_E_HIP (-2)      /* a HIP runtime call failed (message: klsh_last_error) */
#define KLSH_E_NOMEM (-3)    /* device or host allocation failed */
#define KLSH_E_STATE (-4)    /* call out of order (e.g. klsh_cluster before a load) */
#define KLSH_E_NODEVICE (-5) /* no gfx950 device visible: the engine has no CPU fallback */
#define KLSH_E_RANGE (-6)    /* a size exceeds what the engine supports (rows >= 2^32, d > 4096) */

/* ABI version of this header.  2: every statistics struct starts with `struct_size`, which the
 * caller sets to sizeof(the struct) (the library refuses a mismatch instead of writing past a
 * smaller struct); klsh_get_option.  3: klsh_stats.kern has KLSH_KCLASSES = 13 classes (the
 * merge-phase wall, KLSH_K_MERGE). */
#define KLSH_ABI_VERSION 3

typedef struct klsh_ctx klsh_ctx;

/* Per-kernel-class statistics of a call: summed span of the class's launches (first workgroup
 * start to last workgroup end, read from the GPU clock inside the kernels), launches, and the
 * rows they handled (the unit of each class's algorithmic bytes).
 * Index = KLSH_K_*. */
#define KLSH_K_PROJECT 0  /* sign-hash of every live row (k_project_*) */
#define KLSH_K_SORT 1     /* stable bucket sort, all passes (span of the first to last launch) */
#define KLSH_K_RUNS 2     /* run finding and size-class lists (span) */
#define KLSH_K_SMALL 3    /* runs of 2..64 rows (k_merge_small; d > 64: the k_merge_group_wide chain) */
#define KLSH_K_BIG128 4   /* runs of 65..128 rows (k_merge_big / k_merge_big_wide) */
#define KLSH_K_BIG192 5   /* 129..192 */
#define KLSH_K_BIG384 6   /* 193..384 */
#define KLSH_K_BIG896 7   /* 385..896 */
#define KLSH_K_HUGE 8     /* longer runs (k_merge_huge) */
#define KLSH_K_TAIL 9     /* iterations below tail_merge_rows positions (default 2^22): every merge
                             class in one k_merge_tail */
#define KLSH_K_COMPACT 10 /* survivor compaction (span) */
#define KLSH_K_SCREEN 11  /* fp16 screen of the runs of 2..64 rows (SMALL then merges the ones left) */
#define KLSH_K_MERGE 12   /* a phase, not a kernel: the merge launches of each iteration at >=
                             tail_merge_rows positions (default 2^22), and of every iteration at
                             d > 64, together — first workgroup start of any merge class to the
                             last end (their concurrent wall) */
#define KLSH_KCLASSES 13
typedef struct klsh_kstat {
  double ms;
  uint64_t launches;
  uint64_t rows;
  uint64_t runs;
} klsh_kstat;

/* Per-call statistics (all times are milliseconds). */
typedef struct klsh_stats {
  uint64_t struct_size;    /* in: sizeof(klsh_stats) (KLSH_ABI_VERSION check) */
  uint64_t iterations;     /* iterations run */
  uint64_t sum_rows;       /* sum over iterations of N_t (rows projected) */
  uint64_t sum_merges;     /* sum over iterations of M_t = N_t - N_{t+1} */
  uint64_t sum_proj_bits;  /* sum over iterations of N_t * h_t (row-hyperplane dot products) */
  uint64_t nested_calls;   /* oversize buckets sent through nestedCluster */
  uint64_t hyperplanes;    /* hyperplanes drawn by this call */
  uint64_t n_final;        /* live rows after the call */
  uint64_t project_launches;        /* projection launches (every iteration has one) */
  uint64_t project_timed_launches;  /* the ones inside project_ms (queued tail batches carry no
                                       HIP events; their time is in kern[KLSH_K_PROJECT]) */
  double wall_ms;          /* host wall clock of the whole call */
  double project_ms;       /* HIP-event time of project_timed_launches projection launches */
  double sort_ms;          /* HIP-event time of the bucket (radix) sort */
  double merge_ms;         /* HIP-event time of the greedy in-bucket merge kernels */
  double compact_ms;       /* HIP-event time of the survivor compaction */
  double host_ms;          /* host-side hyperplane generation */
  double comm_ms;          /* sharded loop: host time in inter-rank exchanges (incl. waits) */
  uint64_t world;          /* ranks the call ran on (1 = single GPU) */
  /* the small-run merge (runs of 2..64 rows) of the iterations where it is a launch of its own
   * (>= 2^20 positions): HIP-event time on its stream, launches, rows in those runs, merges of
   * the whole iteration (small-run merges are ~97% of them on C2) */
  double small_ms;
  uint64_t small_launches;
  uint64_t small_rows;
  uint64_t small_iter_merges;
  /* per kernel class (single-GPU loop; option "kernel_timing", default on) */
  klsh_kstat kern[KLSH_KCLASSES];
  /* certified projection screens (d > 64, or the fp16 row image at d = 16, 32, 64): the
   * (row, hyperplane) pairs the screen could not call and the exact chains settled */
  uint64_t proj_fix_pairs;
} klsh_stats;

/* ---- lifetime ------------------------------------------------------------------------------- */
/* Create a context on HIP device `device` (ordinal).  *err receives the status. */
klsh_ctx* klsh_create(int device, int* err);
void klsh_destroy(klsh_ctx* ctx);
const char* klsh_last_error(void);  /* thread-local text for the last failure */
const char* klsh_version(void);
int klsh_abi_version(void);         /* KLSH_ABI_VERSION of the built library */

/* ---- loading the rows (replaces building vector<Abundance*>) ---------------------------------- */
/* rows: n x d fp32 row-major (reference common/abundance.h:18-36, `_values`).
 * member_offsets (n+1) / member_ids: each row's id list (`_ids`); NULL member_offsets means row i
 * is the singleton {member_ids ? member_ids[i] : i} (reference io/ioMatrix.cc:373). */
int klsh_load_rows(klsh_ctx* ctx, const float* rows, uint64_t n, int d,
                   const uint64_t* member_offsets, const uint64_t* member_ids);

/* Mode-C producer on the GPU (reference io/ioHT.cc:59-81 ReadHT + io/ioMatrix.cc:353-408
 * convertHTMat): counts is the whole sample-major kmer_count.bin image (d columns of n_total
 * uint16), the batch is rows [batch_offset, batch_offset+batch_size); v_kmers[j] =
 * coverage_j / kmap_size as the reference computes it (app/kmerLSH.cc:471-482).  Rows with
 * sum(count) <= 0.1*d are dropped; ids are batch_offset + i. */
int klsh_load_counts(klsh_ctx* ctx, const uint16_t* counts, uint64_t n_total,
                     uint64_t batch_offset, uint64_t batch_size, int d, const float* v_kmers);

/* Keep a device-side copy of the loaded state / restore it (for repeated timing; both are
 * device-to-device copies). */
int klsh_snapshot(klsh_ctx* ctx);
int klsh_restore(klsh_ctx* ctx);

/* ---- the hot path ------------------------------------------------------------------------------ */
/* Cluster() (reference function/cluster.cc:181-340) over the loaded rows: `iterations` rounds of
 * hyperplane draw -> sign-hash every live row -> stable bucket -> greedy cosine merge per bucket
 * (nestedCluster for buckets above bucket_size_threshold), threshold falling from 0.95 toward
 * min_similarity.  nt_trace (may be NULL) receives N_t at the start of each iteration.
 * stats may be NULL. */
int klsh_cluster(klsh_ctx* ctx, float min_similarity, int iterations, int bucket_size_threshold,
                 uint32_t seed_base, uint64_t* rng_counter, uint64_t* nt_trace, klsh_stats* stats);

/* ---- multi-GPU: one rank per GPU, the loop sharded by key range -------------- */
/* Every rank loads the same rows (replicas) and calls klsh_cluster with the same arguments; the
 * result — order, rows, member lists and rng_counter — is identical to the single-GPU call on
 * every rank.  RCCL (one process per GPU): rank 0 creates the 128-byte id, the caller ships it
 * to the other ranks (any side channel), each rank calls klsh_comm_init on its context. */
int klsh_comm_unique_id(uint8_t* id /* 128 bytes */);
int klsh_comm_init(klsh_ctx* ctx, int rank, int world, const uint8_t* id /* 128 bytes */);
/* In-process group over `world` contexts (any devices, several may share one GPU); each rank's
 * klsh_cluster must then run on its own host thread, concurrently.  For tests on one GPU. */
int klsh_comm_init_local(klsh_ctx** ctxs, int world);
int klsh_comm_info(klsh_ctx* ctx, int* rank, int* world);
/* Options of a context.  Results never depend on them, except "stop_after".
 *   "shard_min_rows"   sharded loop: below this many live rows every rank runs the remaining
 *                      iterations on its own replica, without exchanges (default 2^21; 0 = always)
 *   "phase_timing"     0/1: per-phase HIP events (adds latency; default 0)
 *   "kernel_timing"    0/1: the per-class statistics of klsh_stats.kern (default 1)
 *   "tail_batch"       0/1: queue the small late iterations 32 at a time (default 1)
 *   "tail_local"       0/1: their bucket sort as a top-10-bit pass + per-bucket LDS sorts that
 *                      also list the runs (default 1; 0 = the LSD passes + run kernels)
 *   "huge_fold"        1 (tests): runs over 896 rows always walked inside the 385..896-row
 *                      kernel (default 0: only after several iterations without such runs)
 *   "projection"       0 = the certified matrix-core screens where they exist (default: the fp16
 *                      row image at d = 16, 32, 64 — kept beside the rows, 2 bytes per value —
 *                      and bf16x3 above 64), 1 = the exact packed VALU chains only (no fp16 image)
 *   "stop_after"       k > 0: klsh_cluster runs only the first k iterations of its threshold
 *                      schedule, e.g. to pin a prefix of a long loop; 0 = all (default)
 *   "hyperplane_window" hyperplane rows drawn up front per call; the rest are drawn when the loop
 *                      reaches them (0 = default: all of them while they fit in 256 MB, else 64
 *                      iterations' worth)
 *   "comm_timeout_s"   a collective still incomplete after this many seconds aborts (default 600)
 *   launch sizes, 0 = the measured default: "h16_grid", "wide_grid", "fix_grid" (projection),
 *   "small_grid", "tail_big_groups", "tail_small_groups", "wide_group_grid",
 *   "small_screen_grid" (merge);
 *   "small_screen"     1 = runs of 2..64 rows are screened on the fp16 row image first and only
 *                      the ones the screen cannot rule out are merged on the f32 rows
 *   "tail_screen"      1 (default) = the fp16 small-run screen also runs in front of the one-launch
 *                      merge (k_merge_tail), whose small-run waves then walk only the runs it passed
 *   "tail_big_screen"  1 (default) = there, 65..384-row runs are first screened on the fp16 image
 *                      in their workgroup; a run with no pair within the margin reads no f32 row
 *   "tail_screen_grid" workgroups of that screen's persistent launch (0 = 2048)
 *   "hyperplane_async" 1 (default) = a call's hyperplanes are drawn on the host by a background
 *                      thread while its first iterations run (uploaded as they are needed, no
 *                      stream sync); 0 = drawn and uploaded before the loop starts
 *   "hip_events"       1 = HIP event pairs around the projection and the small-run merge of the
 *                      host-driven iterations (klsh_stats project_ms / small_ms, cross-checks of
 *                      the in-kernel stamps); 0 (default): none — a record costs ~9 us of stream
 *                      time per iteration
 *   "tail_merge_rows"  iterations below this many rows merge every class in one launch (default
 *                      2^22, at most 2^22 — the largest size its parity is pinned at; tests
 *                      lower it to reach the per-class launches at
 *                      small sizes).  Iterations below min(this, 2^20) rows are also queued
 *                      several at a time (one host sync per batch)
 *   "h16_segcap" (tests) caps the fp16 projection's per-workgroup fix-up segment.
 *   "long_runs"        4 (default) = runs over 384 rows at d = 16 / 32 through k_merge_long
 *                      (Gram bit matrix + one walk step per merge); 1 = only runs over 896 rows;
 *                      0 = k_merge_huge for those
 *   "wide_unrolled"    1 (default) = d = 512 projected by the unrolled screen; 0 = the generic one
 *   "wide_gram"        at d = 512 the group merges of runs of at least this many rows (8, 16, 32
 *                      or 64; default 32) take their decisions from an MFMA Gram matrix with a
 *                      certified margin, the uncertain pairs from the exact chains; 0 = none
 *   "progress"         N > 0: a line on stderr every N iterations (long profiling runs) */
int klsh_set_option(klsh_ctx* ctx, const char* name, int64_t value);
/* Any option above, plus read-only diagnostics: "fp16_image" (1 = the loaded rows have the fp16
 * image), "last_hash_kernel" (klsh_hash_keys' projection kernel: 0 packed chains, 1 fp16-image
 * screen, 2 f32 fp16x3 wide-row screen, -1 none) and
 * "last_hash_close_pairs" (its (row, hyperplane) pairs settled by the exact chains). */
int klsh_get_option(klsh_ctx* ctx, const char* name, int64_t* value);

/* ---- results ---------------------------------------------------------------------------------- */
int klsh_count(klsh_ctx* ctx, uint64_t* n_rows, uint64_t* n_members);
/* Canonical order: rows (n_rows*d), member_offsets (n_rows+1), member_ids (n_members); any may
 * be NULL. */
int klsh_result(klsh_ctx* ctx, float* rows, uint64_t* member_offsets, uint64_t* member_ids);

/* ---- path functions, exposed for parity tests ------------------------------------------------- */
/* Hash::LSH::random_projection(row, table) (reference hash/lshash.cc:44-59) for n rows on the
 * GPU: keys[i] = MSB-first sign bits of the h hyperplanes (table: h x d, row-major).  The same
 * kernels and options as the loop's projection (the fp16 row image is built from `rows` where
 * the loop would keep one). */
int klsh_hash_keys(klsh_ctx* ctx, const float* rows, uint64_t n, int d, const float* table, int h,
                   uint32_t* keys);
/* merge_hashtable (reference function/cluster.cc:15-30) on the GPU: the stable bucket order of n
 * keys by their low `bits` bits (keys must be < 2^bits for a pure bucket order; higher bits are
 * carried along unsorted).  sorted_keys[i] = keys[perm[i]]; perm lists original positions, equal
 * keys in their original order. */
int klsh_bucket_sort(klsh_ctx* ctx, const uint32_t* keys, uint64_t n, int bits,
                     uint32_t* sorted_keys, uint32_t* perm);
/* The buckets of n sorted keys as the merge step takes them (the runs of equal keys; the
 * reference's lsh_table entries, function/cluster.cc:205-300): every run of 2 or more keys in start
 * order with its length and its list (0..5: 2, 3-4, 5-8, 9-16, 17-32, 33-64 rows; 6..9: 65-128,
 * 129-192, 193-384, 385-896; 10: longer; 11: longer than bucket_thr >= 0, i.e. nestedCluster).
 * *n_runs: in, the capacity of the outputs; out, the run count (KLSH_E_RANGE if it exceeds the
 * capacity).  A test hook. */
int klsh_bucket_runs(klsh_ctx* ctx, const uint32_t* sorted_keys, uint64_t n, int bucket_thr,
                     uint64_t* n_runs, uint32_t* starts, uint32_t* lengths, int32_t* lists);
/* p_cluster (reference function/cluster.cc:56-87) over the loaded rows taken as ONE bucket in
 * load order, at threshold thr.  Afterwards klsh_count/klsh_result give the survivors. */
int klsh_pcluster(klsh_ctx* ctx, float thr);
/* LSH::generateHashTable (reference hash/lshash.cc:36-42) under the seeding convention:
 * h hyperplanes of d floats starting at draw index *rng_counter (advanced by h). */
int klsh_hyperplanes(uint32_t seed_base, uint64_t* rng_counter, int h, int d, float* table);
/* The merge test's sqrt and division exactly as the kernels evaluate them (sqrt_out[i] =
 * sqrtf(a[i]), div_out[i] = a[i] / b[i]); for checking IEEE correct rounding on the device. */
int klsh_fp_selftest(klsh_ctx* ctx, const float* a, const float* b, uint64_t n, float* sqrt_out,
                     float* div_out);

/* ---- mode E: differential k-mers and read extraction (reference app/kmerLSH.cc:521-580) ------- */
/* AB::WRS (reference function/funcAB.cc:73-109) for every cluster at once: a cluster with more than
 * size_thresh members (member_counts[c]) is tested with ALGLIB's pooled two-sample Student t-test
 * (alglib::studentttest2, utils/alglib-3.15.0/src/statistics.cpp:12502) of its centroid's first n1
 * values against the next n2 (centroids: n_clusters x (n1+n2) fp32, taken as double).
 * group[c] = 2 if lefttail <= pvalue_thresh (its ids go to group B's k-mers), else 1 if
 * righttail <= pvalue_thresh (group A), else 0.  Host computation, no device needed. */
int klsh_wrs(const float* centroids, uint64_t n_clusters, int n1, int n2,
             const uint64_t* member_counts, float pvalue_thresh, int size_thresh, uint8_t* group);
/* The test itself: alglib::studentttest2(x, n, y, m) -> both / left / right tails (bit-exact). */
int klsh_ttest2(const double* x, int64_t n, const double* y, int64_t m, double* bothtails,
                double* lefttail, double* righttail);

/* FASTQ records as the reference reads them (utils/fastq.cc FastqFile + kmer/kseq.h:153-200, gzip or
 * plain): the name is the whole header line, the sequence its isgraph() characters, the quality
 * the next len characters in [33,127].  klsh_fastq_next reads up to max_reads records into
 * reader-owned buffers valid until the next call (offset arrays have count+1 entries) and returns
 * the count; 0 = end of file (a truncated record ends the file, as in the reference). */
typedef struct klsh_fastq klsh_fastq;
klsh_fastq* klsh_fastq_open(const char* path, int* err);
int64_t klsh_fastq_next(klsh_fastq* f, uint64_t max_reads, const char** seq,
                        const uint64_t** seq_offsets, const char** name,
                        const uint64_t** name_offsets, const char** qual,
                        const uint64_t** qual_offsets);
void klsh_fastq_close(klsh_fastq* f);

/* A differential k-mer set on the context's device (the reference's uset_t, hash/HashTables.h:20):
 * kmers are the 8-byte images of Kmer objects as kmer_set.hex stores them (kmer/Kmer.cc:307),
 * read as little-endian uint64 (base i at bits 2i..2i+1, A/C/G/T = 0..3). */
typedef struct klsh_kset klsh_kset;
klsh_kset* klsh_kset_create(klsh_ctx* ctx, const uint64_t* kmers, uint64_t n, int* err);
void klsh_kset_destroy(klsh_kset* set);
/* IOFQ::CheckRead (reference io/ioFastQ.cc:5-76) on the GPU: read r = seq[read_offsets[r] ..
 * read_offsets[r+1]); hits[r] (may be NULL) = k-mer positions whose canonical k-mer is in the set,
 * flags[r] = 1 iff the read has at least k+10 bases and hits / (len-k+1) > kmer_vote (float). */
int klsh_check_reads(klsh_ctx* ctx, const klsh_kset* set, const char* seq,
                     const uint64_t* read_offsets, uint64_t n_reads, int k, float kmer_vote,
                     uint32_t* hits, uint8_t* flags);
typedef struct klsh_extract_stats {
  uint64_t struct_size; /* in: sizeof(klsh_extract_stats) */
  uint64_t reads, bases, reads_tested, kmers_checked, reads_extracted, abnormal;
  double kernel_ms;  /* HIP-event time of the k-mer vote kernels */
  double parse_ms;   /* host FASTQ parsing (gzip included) */
  double total_ms;
} klsh_extract_stats;
/* IOFQ::ReadExtract (reference io/ioFastQ.cc:78-159) for one sample: every record of in_path whose
 * k-mer vote passes, written to out_path as "@name\nseq\n+\nqual\n" (plain text, byte-identical to
 * the reference's output).  stats may be NULL. */
int klsh_extract_fastq(klsh_ctx* ctx, const klsh_kset* set, const char* in_path,
                       const char* out_path, int k, float kmer_vote, klsh_extract_stats* stats);

/* ---- mode B: the k-mer table of KMC databases (reference io/ioHT.cc:83-199, kmc = false) ------- */
/* buildKHtable over KMC databases (KMC1 or KMC2/3 layout, <name>.kmc_pre / <name>.kmc_suf, listing
 * as kmer/kmc_api/kmc_file.cpp:66-532): the union of canonical k-mers over the samples, each
 * sample's summed counts clamped at 65535, written to <out_dir>/ kmer_set.hex (8 bytes per k-mer),
 * kmer_count.bin (sample-major uint16) and kmer_count.log ("%llu" rows, "\t%f" coverage = float sum
 * of log(count) per sample).  The files equal the reference's byte for byte: rows in the order of its
 * libcuckoo table after KmcRead's inserts at -T 1 (while the table never grows; a growing
 * reference table re-inserts from hardware_concurrency() threads, and that order is replayed here
 * as if those threads ran one after another).
 * out_dir NULL or "" = the current directory.  stats may be NULL. */
typedef struct klsh_khtable_stats {
  uint64_t struct_size; /* in: sizeof(klsh_khtable_stats) */
  uint64_t kmap_size, records, records_listed;
  double io_ms;     /* host reads of the .kmc_suf streams */
  double total_ms;
  double order_ms;  /* host replay of the reference's libcuckoo inserts (the row order) */
} klsh_khtable_stats;
/* The row order alone (a test hook): the libcuckoo table order (kmer/Kmer.cc:138 hash, the
 * vendored utils/libcuckoo/cuckoohash_map.hh, 8-slot buckets, 2^16 buckets to start) of n DISTINCT
 * k-mer images inserted in the given order: order[i] = index of the table's i-th element.  Returns
 * the table's final hash power (>= 16), or a negative KLSH_E_* code.  Host only. */
int klsh_cuckoo_order(const uint64_t* images, uint64_t n, int k, uint32_t* order);
/* The host parse of a KMC database's prefix file (<name>.kmc_pre: version, header, prefix LUT) as
 * klsh_build_khtable does it, every file-derived offset checked (a test hook).  Host only. */
int klsh_kmc_info(const char* name, int* k, uint64_t* total, uint64_t* lut_entries);
int klsh_build_khtable(klsh_ctx* ctx, const char* const* kmc_names, int n_samples, int k,
                       const char* out_dir, klsh_khtable_stats* stats);

/* ---- synthetic workload (klsh-synth v1) ------------------------------------ */
/* Host-side, deterministic on any machine (integer hashing + glibc exp/log/sqrt): fills counts
 * (sample-major d x n uint16, the kmer_count.bin layout) and coverage[d] = sum over i of ln(c)
 * for c > 0, summed in double in ascending i (the kmer_count.log convention).  Rows belong to
 * `genomes` groups (n/50 if 0): profile(g,s) = exp(2 + z), z ~ N(0,1); multiplicity m in {1,2};
 * count = min(Poisson(profile*m), 65535) (inversion below 30, normal approximation above).
 * threads <= 0: all host threads. */
int klsh_synth_counts(uint64_t n, int d, uint64_t seed, uint64_t genomes, int threads,
                      uint16_t* counts, double* coverage);

#ifdef __cplusplus
}
#endif
#endif
