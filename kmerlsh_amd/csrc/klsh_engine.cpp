// Host engine behind the C ABI (include/klsh.h): device state, the per-iteration launch
// sequence of Cluster() (reference function/cluster.cc:181-340), nestedCluster orchestration
// (:89-178) and result extraction.  The arithmetic of the path runs only in the gfx950 kernels
// (klsh_kernels.hip); there is no CPU fallback — without a gfx950 device klsh_create fails.
//
// Per LSH iteration t (N_t live rows, h_t = floor(log2 N_t)):
//   1. hyperplanes k_t .. k_t+h_t-1 (pre-drawn on the host, uploaded once per call)
//   2. k_project: key of every live row, in canonical order
//   3. radix sort (key, slot): the stable bucket order of merge_hashtable
//   4. k_merge_small / k_merge_large: greedy p_cluster in every bucket, in place
//   5. compaction of survivors -> canonical order of iteration t+1
//   6. one device->host copy of the counters (N_{t+1}, oversize buckets) and a stream sync
// Oversize buckets (> bucket_size_threshold) are then re-hashed with fresh hyperplanes drawn in
// ascending bucket order (the reference's T=1 RNG order), sorted, merged, and 5 is redone.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <stddef.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cstring>
#include <chrono>
#include <cmath>
#include <deque>
#include <functional>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "klsh.h"
#include "klsh_comm.h"
#include "klsh_internal.h"

extern "C" {
uint32_t klsh_host_seed(uint32_t base, uint64_t k);
void klsh_host_hyperplanes(uint32_t base, uint64_t k0, uint64_t count, int d, int stride,
                           float* out, int threads);
}

using klsh::Counters;
using klsh::Rows;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define KLSH_HIP(call)                                                                   \
  do {                                                                                   \
    hipError_t e_ = (call);                                                              \
    if (e_ != hipSuccess)                                                                \
      return fail(KLSH_E_HIP, std::string(#call) + " -> " + hipGetErrorString(e_));      \
  } while (0)

double now_ms() {
  return std::chrono::duration<double, std::milli>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int floor_log2(uint64_t n) { return (int)std::floor(std::log2((double)n)); }  // cluster.cc:194

template <class T>
int dalloc(T** p, size_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  if (hipMalloc((void**)p, sizeof(T) * count) != hipSuccess) {
    *p = nullptr;
    return fail(KLSH_E_NOMEM, "hipMalloc of " + std::to_string(sizeof(T) * count) + " bytes");
  }
  return 0;
}

template <class T>
void dfree(T*& p) {
  if (p) (void)hipFree((void*)p);
  p = nullptr;
}

struct Snapshot {
  bool valid = false;
  uint64_t n_live = 0;
  float* x = nullptr;
  float* nrm = nullptr;
  uint32_t *cnt = nullptr, *head = nullptr, *tail = nullptr, *nxt = nullptr, *order = nullptr;
};

}  // namespace

struct klsh_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev[8] = {};
  hipEvent_t sev[2] = {};  // around the small-run merge launch (HIP-event cross-check)
  // per-kernel-class stamps (klsh_stats.kern, KStampBlock in klsh_internal.h): the timed
  // iterations of a call stamp sets kt_iter & 1 in turn
  klsh::KStampBlock* kstamp = nullptr;
  uint64_t kt_iter = 0;
  klsh::LookBack lb{nullptr, 0};  // the one-launch compaction of small iterations
  bool kernel_timing = true;  // option "kernel_timing"
  bool hip_events = false;    // option "hip_events": HIP event pairs around the projection and
                              // the small-run merge (cross-checks of the stamps; cost latency)

  // sizes
  int d = 0, dp = 0;
  uint64_t slots = 0, members = 0, n_live = 0;
  uint64_t cap_slots = 0, cap_members = 0;
  int cap_dp = 0;
  bool loaded = false;

  // device state
  Rows rows{};
  uint32_t* order = nullptr;  // canonical live slots
  uint32_t* alt = nullptr;    // second slot buffer (sort / compaction ping-pong)
  uint32_t* keys = nullptr;
  uint32_t* keys2 = nullptr;
  uint32_t* nk1 = nullptr;    // nested scratch
  uint32_t* nk2 = nullptr;
  uint32_t* nv2 = nullptr;
  uint32_t* hist = nullptr;
  uint32_t* tile_sums = nullptr;
  klsh::MergeWork mw{};
  klsh::ProjectWork pw{};     // wide-row matrix-core projection: fix-up list
  Counters* ctr = nullptr;
  Counters* h_ctr = nullptr;  // pinned
  float* W = nullptr;         // hyperplane pool on the device, [k - w_k0][dp]
  uint64_t w_k0 = 0, w_count = 0, w_cap = 0, w_alloc = 0;
  uint32_t w_base = 0;
  int w_dp = 0, w_d = 0;
  // The call's window drawn in the background (predraw_hyperplanes): a host thread draws rows
  // [w_k0, w_k0 + w_target) in order into pinned memory and publishes how many are done
  // (w_drawn); ensure_hyperplanes uploads the drawn rows it needs on the stream, without a
  // stream sync — the host RNG (~3.5 ms per C2 call, ~25 ms at C5's d = 512) runs beside the
  // GPU's first iterations instead of in front of them.
  std::thread drawer;
  std::atomic<uint64_t> w_drawn{0};
  std::atomic<bool> draw_stop{false};
  uint64_t w_target = 0;
  float* w_pin = nullptr;
  size_t w_pin_floats = 0;

  // host
  std::vector<uint64_t> ids;  // member node -> k-mer id
  Snapshot snap;

  // sharded loop: this rank's exchange and its buffers (sized with the slots)
  klsh::Comm* comm = nullptr;
  uint2* sbuf = nullptr;       // (key, slot) pairs grouped by destination rank
  uint2* rbuf = nullptr;       // (key, slot) pairs received, in source-rank order
  uint32_t* mark = nullptr;    // [slots] iteration stamp of the last rewrite (in-place kernels)
  uint32_t stamp = 0;
  uint32_t* dslots = nullptr;  // survivors rewritten by a merge (this rank)
  uint32_t* bins = nullptr;    // [4096] key-bin histogram of this rank
  uint32_t* bins_all = nullptr;
  uint32_t* owner = nullptr;   // [4096] bin -> rank
  uint32_t* cntmat = nullptr;  // [W][W] pairs rank g sends rank r
  uint32_t* small = nullptr;   // [W + 1][4] per-rank counters exchange
  uint32_t* h_small = nullptr; // pinned: cntmat or the counters exchange
  // mapped: the sharded loop's per-iteration publishes (k_publish_words): [sequence word, 64 B]
  // [payload]; host and device views
  uint32_t* shp_host = nullptr;
  uint32_t* shp_dev = nullptr;
  uint32_t shp_seq = 0;
  uint32_t* drec = nullptr;    // delta records of this rank, then of all ranks
  uint32_t* drec_all = nullptr;
  size_t drec_cap = 0, drec_all_cap = 0;  // words
  uint64_t shard_cap = 0;
  double t_enqueued = 0.0;  // diagnostics (KLSH_ITER_LOG): host time when an iteration was queued
  // Counters through mapped pinned memory (klsh::Publish): the host polls pub_seq instead of a
  // copy launch + stream sync after every iteration (a copy + sync if mapped memory is refused).
  Counters* pub_host = nullptr;   // host view
  Counters* pub_dev = nullptr;    // device view of the same memory
  uint32_t* pub_seq_host = nullptr;
  uint32_t* pub_seq_dev = nullptr;
  uint32_t pub_seq = 0;
  // Queued tail batches (run_batched): every iteration publishes into its own ring slot, the host
  // waits for the last sequence number of a chunk and reads the chunk's slots.
  static constexpr int kRing = 2 * 32;
  Counters* ring_host = nullptr;
  Counters* ring_dev = nullptr;
  bool ctr_clean = false;  // *ctr is known to be zero (the publisher zeroed it)
  // Queued-ahead projection (small iterations, where no bucket can be oversize): the next
  // iteration's sign-hash is enqueued behind the compaction, reading N from n_next_dev, before
  // the host has the counters.
  uint32_t* n_next_dev = nullptr;
  bool spec_pending = false;
  uint64_t spec_k = 0;
  int spec_ev = 0;
  bool spec_swap = false;  // the queued keys went to keys2 (this iteration's sorted keys were in keys)
  bool zero_copy = true;
  klsh::RunCounters* rc = nullptr;  // run-list counters (device, one 128-B line each)
  // fp16 image of the rows for the projection's screen (Rows::xh), kept at d = 16, 32, 64 unless
  // option "projection" asks for the exact packed chains; every row store of the merge kernels
  // writes it too (store_row4 / store_row1)
  uint16_t* xh_alloc = nullptr;
  bool shadow_wanted(int d_) const {
    return pw.variant != klsh::kProjPacked && klsh::shadow_width_ok(d_);
  }
  // Queued tail batches (run_batched; option "tail_batch", default on), their bucket sort as a
  // top-bits pass + the LDS bucket sort that lists the runs (option "tail_local", default on)
  bool tail_batch = true;
  bool tail_local = true;
  // klsh_hash_keys diagnostics (klsh_get_option): the projection kernel of the last call and
  // the (row, hyperplane) pairs its screen left to the exact chains
  int last_hash_kernel = klsh::kPkNone;
  uint64_t last_hash_close = 0;

  ~klsh_ctx() { release(); }

  // Per-phase HIP events (sort / merge / compaction) cost latency in every iteration — an event
  // record on the stream is tens of microseconds in the small late iterations — so they are on
  // only with KLSH_PHASE_TIMING=1.  The projection is always bracketed (bench.py's roofline).
  bool phase_timing = false;  // option "phase_timing"

  // Sharded loop: below this many live rows the per-iteration exchanges cost more than they save
  // (the late iterations are latency-bound on one GPU already), so every rank takes the whole
  // canonical order and runs the remaining iterations on its replica — identically, with no
  // communication.  klsh_set_option(ctx, "shard_min_rows", n); 0 = always sharded.
  uint64_t shard_min_rows = 1u << 21;
  uint32_t huge_quiet = 0;  // consecutive iterations without >896-row runs (MergeWork::huge_fold)
  bool huge_fold_always = false;  // option "huge_fold" (tests): fold in every iteration
  // option "comm_timeout_s": a collective that has not completed after this long aborts the group
  double comm_timeout_s = 600.0;

  // "stop_after" (klsh_set_option): run only the first k iterations of a call's threshold
  // schedule (0 = all).  Prefix parity tests of the long configs use it; results of the
  // iterations that do run are unchanged.
  int stop_after = 0;
  hipEvent_t counts_ev = nullptr;  // sharded loop: the send counts are on the host
  int progress = 0;  // option "progress": a line on stderr every this many iterations (profiling runs)
  void tick(int it) const {
    if (progress > 0 && it % progress == 0) {
      fprintf(stderr, "[klsh] iteration %d\n", it);
      fflush(stderr);
    }
  }
  // "hyperplane_window" (klsh_set_option): rows drawn up front per call (0 = the default bound)
  uint64_t hyperplane_window = 0;
  // "hyperplane_async" (klsh_set_option): 1 (default) = the call's window drawn by a background
  // thread while the loop starts (predraw_hyperplanes); 0 = drawn and uploaded before it
  uint32_t hyperplane_async = 1;

  int world() const { return comm ? comm->world : 1; }
  int rank() const { return comm ? comm->rank : 0; }

  void release_shard() {
    dfree(sbuf); dfree(rbuf); dfree(mark); dfree(dslots); dfree(bins); dfree(bins_all);
    dfree(owner); dfree(cntmat); dfree(small); dfree(drec); dfree(drec_all);
    if (h_small) (void)hipHostFree(h_small);
    h_small = nullptr;
    if (shp_host) (void)hipHostFree(shp_host);
    shp_host = shp_dev = nullptr;
    drec_cap = drec_all_cap = 0;
    shard_cap = 0;
  }
  int reserve_shard() {
    const int W = world();
    if (shard_cap >= cap_slots && sbuf) return 0;
    release_shard();
    const uint64_t s = std::max<uint64_t>(cap_slots, 1);
    const size_t nb = (size_t)1 << klsh::kMaxBinBits;
    int e = 0;
    if ((e = dalloc(&sbuf, s)) || (e = dalloc(&rbuf, s)) || (e = dalloc(&mark, s)) ||
        (e = dalloc(&dslots, s)) || (e = dalloc(&bins, nb)) || (e = dalloc(&bins_all, nb * W)) ||
        (e = dalloc(&owner, nb)) || (e = dalloc(&cntmat, (size_t)W * W)) ||
        (e = dalloc(&small, (size_t)(W + 1) * 4))) {
      release_shard();
      return e;
    }
    if (hipHostMalloc((void**)&h_small, sizeof(uint32_t) * std::max(W * W, (W + 1) * 4),
                      hipHostMallocDefault) != hipSuccess) {
      release_shard();
      return fail(KLSH_E_NOMEM, "pinned exchange buffer");
    }
    {
      const size_t words = 16 + std::max<size_t>((size_t)W * W, 4 * (size_t)W + sizeof(Counters) / 4);
      void *hp = nullptr, *dp = nullptr;
      if (hipHostMalloc(&hp, sizeof(uint32_t) * words, hipHostMallocMapped | hipHostMallocCoherent) !=
              hipSuccess ||
          hipHostGetDevicePointer(&dp, hp, 0) != hipSuccess) {
        if (hp) (void)hipHostFree(hp);
        release_shard();
        return fail(KLSH_E_NOMEM, "mapped exchange buffer");
      }
      memset(hp, 0, sizeof(uint32_t) * words);
      shp_host = static_cast<uint32_t*>(hp);
      shp_dev = static_cast<uint32_t*>(dp);
      shp_seq = 0;
    }
    if (hipMemset(mark, 0, sizeof(uint32_t) * s) != hipSuccess) {
      release_shard();
      return fail(KLSH_E_HIP, "mark init");
    }
    stamp = 0;
    shard_cap = s;
    return 0;
  }
  int reserve_words(uint32_t** p, size_t* cap, size_t words) {
    if (words <= *cap && *p) return 0;
    dfree(*p);
    *cap = 0;
    const size_t w = std::max<size_t>(words + words / 4, 1 << 16);
    if (int e = dalloc(p, w)) return e;
    *cap = w;
    return 0;
  }

  void release_state() {
    dfree(rows.x); dfree(rows.nrm); dfree(rows.cnt); dfree(rows.head); dfree(rows.tail);
    dfree(rows.nxt); dfree(order); dfree(alt); dfree(keys); dfree(keys2); dfree(nk1);
    dfree(nk2); dfree(nv2); dfree(hist); dfree(tile_sums); dfree(mw.over); dfree(mw.run_ws);
    dfree(mw.huge);
    dfree(mw.long_P);
    mw.long_groups = 0;
    dfree(pw.fix);
    dfree(pw.ws);
    pw.cap = 0;
    for (auto& c : mw.big) dfree(c);
    for (auto& c : mw.cls) dfree(c);
    for (auto& c : mw.act) dfree(c);
    dfree(kstamp);
    dfree(lb.status);
    dfree(xh_alloc);
    rows.xh = nullptr;
    cap_slots = cap_members = 0;
    cap_dp = 0;
    drop_snapshot();
  }
  void drop_snapshot() {
    dfree(snap.x); dfree(snap.nrm); dfree(snap.cnt); dfree(snap.head); dfree(snap.tail);
    dfree(snap.nxt); dfree(snap.order);
    snap.valid = false;
  }
  void join_drawer() {
    if (drawer.joinable()) {
      draw_stop.store(true);
      drawer.join();
      draw_stop.store(false);
    }
    w_target = 0;
  }
  void release() {
    join_drawer();
    if (w_pin) (void)hipHostFree(w_pin);
    w_pin = nullptr;
    w_pin_floats = 0;
    release_shard();
    delete comm;
    comm = nullptr;
    release_state();
    dfree(W);
    dfree(ctr);
    dfree(rc);
    mw.rc = nullptr;
    if (h_ctr) (void)hipHostFree(h_ctr);
    h_ctr = nullptr;
    dfree(n_next_dev);
    if (pub_host) (void)hipHostFree(pub_host);
    pub_host = nullptr;
    pub_dev = nullptr;
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e), e = nullptr;
    for (auto& e : sev)
      if (e) (void)hipEventDestroy(e), e = nullptr;
    if (counts_ev) (void)hipEventDestroy(counts_ev);
    counts_ev = nullptr;
    for (int i = 0; i < klsh::kMergeStreams; ++i) {
      if (mw.join[i]) (void)hipEventDestroy(mw.join[i]);
      if (mw.aux[i]) (void)hipStreamDestroy(mw.aux[i]);
      mw.join[i] = nullptr;
      mw.aux[i] = nullptr;
    }
    if (mw.fork) (void)hipEventDestroy(mw.fork);
    mw.fork = nullptr;
    if (stream) (void)hipStreamDestroy(stream);
    stream = nullptr;
  }

  // k_merge_long's bit matrices (runs over 896 rows at d = 16 / 32): one per workgroup, a
  // workgroup per 897 slots up to 256 (2 MB each: up to 512 MB).  None while option long_runs
  // is 0 (k_merge_huge walks those runs; the matrices are released when it is switched off).
  int ensure_long(uint64_t s, int d_) {
    const uint32_t want = klsh::long_ok(d_) && s >= 897 && mw.long_off != 1u
                              ? (uint32_t)std::min<uint64_t>(256, s / 897 + 1)
                              : 0u;
    if (want == 0 && mw.long_groups) {
      dfree(mw.long_P);
      mw.long_groups = 0;
      return 0;
    }
    if (want <= mw.long_groups) return 0;
    dfree(mw.long_P);
    mw.long_groups = 0;
    if (int e = dalloc(&mw.long_P, (size_t)want * klsh::kLongRows * (klsh::kLongRows / 64)))
      return e;
    mw.long_groups = want;
    return 0;
  }

  // (Re)allocate device state for `ns` slots, `nm` member nodes, row width d.
  int reserve(uint64_t ns, uint64_t nm, int d_) {
    if (ns >= 0xFFFFFFF0ull || nm >= 0xFFFFFFF0ull) return fail(KLSH_E_RANGE, "rows >= 2^32");
    if (d_ <= 0 || d_ > 4096) return fail(KLSH_E_RANGE, "d must be in [1, 4096]");
    const int dp_ = (d_ + 3) & ~3;
    if (ns <= cap_slots && nm <= cap_members && dp_ <= cap_dp) {
      d = d_;
      dp = dp_;
      rows.d = d;
      rows.dp = dp;
      if (shadow_wanted(d) && !xh_alloc)  // (an earlier load at a width without the image)
        if (int e = dalloc(&xh_alloc, cap_slots * (uint64_t)cap_dp)) return e;
      rows.xh = shadow_wanted(d) ? xh_alloc : nullptr;
      drop_snapshot();
      return ensure_long(cap_slots, d_);
    }
    release_state();
    const uint64_t s = std::max<uint64_t>(ns, 1), m = std::max<uint64_t>(nm, 1);
    int e = 0;
    if ((e = dalloc(&rows.x, s * dp_)) || (e = dalloc(&rows.nrm, s)) || (e = dalloc(&rows.cnt, s)) ||
        (e = dalloc(&rows.head, s)) || (e = dalloc(&rows.tail, s)) || (e = dalloc(&rows.nxt, m)) ||
        (e = dalloc(&order, s)) || (e = dalloc(&alt, s)) || (e = dalloc(&keys, s)) ||
        (e = dalloc(&keys2, s)) || (e = dalloc(&nk1, s + 64)) || (e = dalloc(&nk2, s)) ||
        (e = dalloc(&nv2, s)) ||
        (e = dalloc(&hist, klsh::sort_ws_words(s))) ||
        (e = dalloc(&tile_sums, klsh::scan_ws_words(s))) ||
        (e = dalloc(&mw.over, s + 64)) || (e = dalloc(&mw.run_ws, klsh::run_ws_words(s))) ||
        (e = dalloc(&pw.fix, s)) || (e = dalloc(&pw.ws, 64)) ||
        (e = dalloc(&mw.big[0], s / 65 + 64)) || (e = dalloc(&mw.big[1], s / 129 + 64)) ||
        (e = dalloc(&mw.big[2], s / 193 + 64)) || (e = dalloc(&mw.big[3], s / 385 + 64)) ||
        (e = dalloc(&mw.huge, s / 897 + 64))) {
      release_state();
      return e;
    }
    if (shadow_wanted(d_)) {  // (in the large-buffer group: see below)
      if ((e = dalloc(&xh_alloc, s * dp_))) {
        release_state();
        return e;
      }
    }
    if ((e = ensure_long(s, d_))) {
      release_state();
      return e;
    }
    for (int c = 0; c < klsh::kGroupClasses; ++c) {
      if ((e = dalloc(&mw.cls[c], klsh::group_class_capacity(c, s))) ||
          (e = dalloc(&mw.act[c], klsh::group_class_capacity(c, s)))) {
        release_state();
        return e;
      }
    }
    // the look-back workspaces start zeroed (tickets, done counters, epochs, histograms) and the
    // kernels return them to zero; they are never cleared again
    pw.cap = (uint32_t)s;
    if (hipMemset(pw.ws, 0, sizeof(uint32_t) * 64) != hipSuccess ||
        hipMemset(hist, 0, sizeof(uint32_t) * klsh::sort_ws_words(s)) != hipSuccess ||
        hipMemset(tile_sums, 0, sizeof(uint32_t) * klsh::scan_ws_words(s)) != hipSuccess) {
      release_state();
      return fail(KLSH_E_HIP, "workspace init");
    }
    // The stamp block and the look-back status words: small buffers allocated AFTER the rows and
    // workspaces.  (Allocated at context creation, ahead of the multi-GB state, they cost a C2 step
    // 252 -> 330 ms on MI355X: every random-access kernel slowed, the sort scatter 2.5x — the
    // large buffers evidently lost their large-page backing; A/B in DESIGN.md §6.)
    {
      std::vector<unsigned char> init(sizeof(klsh::KStampBlock), 0);
      auto* b = reinterpret_cast<klsh::KStampBlock*>(init.data());
      for (auto& st : b->set)
        for (auto& cls : st.t0)
          for (auto& ln : cls) ln.v = ~0ull;  // every start line ~0, every end line and total 0
      if ((e = dalloc(&kstamp, 1)) || (e = dalloc(&lb.status, 256))) {
        release_state();
        return e;
      }
      if (hipMemcpy(kstamp, init.data(), init.size(), hipMemcpyHostToDevice) != hipSuccess ||
          hipMemset(lb.status, 0, sizeof(unsigned long long) * 256) != hipSuccess) {
        release_state();
        return fail(KLSH_E_HIP, "stamp / look-back init");
      }
      lb.epoch = 0;
    }
    mw.tile_sums = tile_sums;
    cap_slots = s;
    cap_members = m;
    cap_dp = dp_;
    d = d_;
    dp = dp_;
    rows.d = d;
    rows.dp = dp;
    rows.xh = shadow_wanted(d) ? xh_alloc : nullptr;
    return 0;
  }
  // Option "projection" changed: keep the fp16 image (allocated and rebuilt from x) or drop it.
  int apply_projection_variant() {
    if (!cap_slots) return 0;  // nothing reserved yet: reserve() decides
    if (shadow_wanted(d)) {
      if (!xh_alloc) {
        if (int e = dalloc(&xh_alloc, cap_slots * (uint64_t)cap_dp)) return e;
      }
      rows.xh = xh_alloc;
      klsh::launch_shadow_build(rows, slots, stream);  // merges did not keep it while it was off
      KLSH_HIP(hipGetLastError());
      KLSH_HIP(hipStreamSynchronize(stream));
    } else {
      rows.xh = nullptr;
    }
    return 0;
  }

  // Make hyperplanes [k0, k0+count) of stream `base` resident on the device (drawn on the host).
  // The resident window [w_k0, w_k0 + w_count) only grows forward; anything else restarts it.
  // Rows [k0, k0 + count) inside the background-drawn window: true when ensure_hyperplanes can
  // append them without touching rows the stream may be reading.
  bool lazy_covers(uint32_t base, uint64_t k0, uint64_t count) const {
    return w_target && W && w_base == base && w_dp == dp && w_d == d && k0 >= w_k0 &&
           k0 + count <= w_k0 + w_target;
  }
  int ensure_hyperplanes(uint32_t base, uint64_t k0, uint64_t count, double* host_ms) {
    if (count == 0) return 0;
    const bool same_stream = W && w_base == base && w_dp == dp && w_d == d;
    if (same_stream && k0 >= w_k0 && k0 + count <= w_k0 + w_count) return 0;
    const double t0 = now_ms();
    if (lazy_covers(base, k0, count)) {  // wait for the drawer, then append what it has
      const uint64_t need = k0 + count - w_k0;
      while (w_drawn.load(std::memory_order_acquire) < need) std::this_thread::yield();
      const uint64_t avail = w_drawn.load(std::memory_order_acquire);
      KLSH_HIP(hipMemcpyAsync(W + w_count * dp, w_pin + w_count * dp,
                              sizeof(float) * (avail - w_count) * dp, hipMemcpyHostToDevice,
                              stream));
      w_count = avail;
      if (host_ms) *host_ms += now_ms() - t0;
      return 0;
    }
    join_drawer();
    if (!(same_stream && k0 >= w_k0 && k0 + count <= w_k0 + w_cap)) {
      // (the window's row capacity carries over only for the same row width: w_cap rows of
      // another dp would scale the allocation by the width ratio on every change of d)
      const uint64_t cap = std::max<uint64_t>({count, 4096, same_stream ? w_cap : 0});
      if (!W || cap * (uint64_t)dp > w_alloc) {
        dfree(W);
        if (int e = dalloc(&W, cap * (uint64_t)dp)) return e;
        w_alloc = cap * (uint64_t)dp;
      }
      w_cap = w_alloc / (uint64_t)dp;
      w_k0 = k0;
      w_count = 0;
      w_base = base;
      w_dp = dp;
      w_d = d;
    }
    const uint64_t start = w_k0 + w_count, n = k0 + count - start;
    std::vector<float> host((size_t)n * dp, 0.0f);
    klsh_host_hyperplanes(base, start, n, d, dp, host.data(), 0);
    KLSH_HIP(hipMemcpyAsync(W + (start - w_k0) * dp, host.data(), sizeof(float) * host.size(),
                            hipMemcpyHostToDevice, stream));
    KLSH_HIP(hipStreamSynchronize(stream));
    w_count += n;
    if (host_ms) *host_ms += now_ms() - t0;
    return 0;
  }
  const float* hyperplane_ptr(uint64_t k) const { return W + (k - w_k0) * (uint64_t)dp; }
  // The hyperplanes of the first iterations of a call, drawn up front: every iteration's h_t
  // (<= hmax) for all of them when that fits in 64 Mi floats (256 MB: C2 draws 11.5 K rows of 64),
  // else the first 64 iterations' worth — ensure_hyperplanes extends the window when the loop
  // gets there (-I 10000 at d = 4096 would otherwise need ~3.8 GB up front, host and device).
  // The window is drawn by a background thread (see `drawer`) when it holds every iteration's rows;
  // a smaller window (option hyperplane_window, or a call too long for 64 Mi floats) is drawn here
  // and extended in place as before.
  int predraw_hyperplanes(uint32_t base, uint64_t k0, uint64_t hmax, int iterations,
                          double* host_ms) {
    join_drawer();
    const uint64_t want = hmax * (uint64_t)iterations;
    const uint64_t cap = hyperplane_window ? hyperplane_window
                                           : std::max<uint64_t>(hmax * 64, (64ull << 20) / (uint64_t)dp);
    const uint64_t count = std::min(want, cap);
    if (count == 0) return 0;
    if (hyperplane_window || count < want || !hyperplane_async)
      return ensure_hyperplanes(base, k0, count, host_ms);
    const double t0 = now_ms();
    if (!w_pin || count * (uint64_t)dp > w_pin_floats) {
      if (w_pin) (void)hipHostFree(w_pin);
      w_pin = nullptr;
      w_pin_floats = 0;
      if (hipHostMalloc((void**)&w_pin, sizeof(float) * count * (uint64_t)dp,
                        hipHostMallocDefault) != hipSuccess)
        return fail(KLSH_E_HIP, "pinned hyperplane window");
      w_pin_floats = count * (uint64_t)dp;
    }
    w_drawn.store(0);
    float* out = w_pin;
    const int dd = d, ddp = dp;
    drawer = std::thread([this, base, k0, count, out, dd, ddp] {
      // the first iterations' rows first (the loop starts on them), then larger chunks over the
      // host's worker threads
      uint64_t r = 0, chunk = 64;
      while (r < count && !draw_stop.load(std::memory_order_relaxed)) {
        const uint64_t n = std::min(chunk, count - r);
        if (ddp != dd) std::memset(out + r * ddp, 0, sizeof(float) * n * ddp);  // row padding
        klsh_host_hyperplanes(base, k0 + r, n, dd, ddp, out + r * ddp, chunk <= 64 ? 1 : 0);
        r += n;
        w_drawn.store(r, std::memory_order_release);
        chunk = 2048;
      }
    });
    // (the drawer runs meanwhile) a queued launch of an earlier call may still read the device
    // window, which is rewritten from its first row
    KLSH_HIP(hipStreamSynchronize(stream));
    const uint64_t rows = std::max<uint64_t>(count, 4096);
    if (!W || rows * (uint64_t)dp > w_alloc) {
      dfree(W);
      if (int e = dalloc(&W, rows * (uint64_t)dp)) return e;
      w_alloc = rows * (uint64_t)dp;
    }
    w_cap = w_alloc / (uint64_t)dp;
    w_k0 = k0;
    w_count = 0;
    w_base = base;
    w_dp = dp;
    w_d = d;
    w_target = count;
    if (host_ms) *host_ms += now_ms() - t0;
    return 0;
  }

  // zero the iteration counters (and the run-list counters) on the stream
  int reset_counters() {
    KLSH_HIP(hipMemsetAsync(ctr, 0, sizeof(Counters), stream));
    KLSH_HIP(hipMemsetAsync(rc, 0, sizeof(klsh::RunCounters), stream));
    return 0;
  }
  int sync_counters() {
    ctr_clean = false;
    KLSH_HIP(hipMemcpyAsync(h_ctr, ctr, sizeof(Counters), hipMemcpyDeviceToHost, stream));
    KLSH_HIP(hipStreamSynchronize(stream));
    return check_device_err();
  }
  // Wait for the counters the compaction published with sequence number `seq` (spin on the
  // mapped word; every few thousand polls the stream is queried, so a failed kernel is reported
  // instead of waited for).
  int wait_published(uint32_t seq) {
    volatile uint32_t* p = pub_seq_host;
    uint64_t spins = 0;
    while (*p != seq) {
      __builtin_ia32_pause();
      if ((++spins & 0xFFFu) == 0) {
        const hipError_t q = hipStreamQuery(stream);
        if (q == hipSuccess) {
          std::atomic_thread_fence(std::memory_order_seq_cst);
          if (*p != seq) return fail(KLSH_E_HIP, "counters not published by a finished stream");
          break;
        }
        if (q != hipErrorNotReady) return fail(KLSH_E_HIP, std::string("stream: ") + hipGetErrorString(q));
      }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    memcpy(h_ctr, (const void*)pub_host, sizeof(Counters));
    ctr_clean = true;
    return check_device_err();
  }
  // Wait until the published sequence word reaches `seq` (queued batches publish one sequence
  // number per iteration, so the word may already be past it).
  int wait_seq(uint32_t seq) {
    volatile uint32_t* p = pub_seq_host;
    uint64_t spins = 0;
    while ((int32_t)(*p - seq) < 0) {
      __builtin_ia32_pause();
      if ((++spins & 0xFFFu) == 0) {
        const hipError_t q = hipStreamQuery(stream);
        if (q == hipSuccess) {
          std::atomic_thread_fence(std::memory_order_seq_cst);
          if ((int32_t)(*p - seq) < 0)
            return fail(KLSH_E_HIP, "counters not published by a finished stream");
          break;
        }
        if (q != hipErrorNotReady) return fail(KLSH_E_HIP, std::string("stream: ") + hipGetErrorString(q));
      }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    return 0;
  }
  int check_device_err() const {
    if (h_ctr->err)
      return fail(KLSH_E_HIP, "device protocol failure (look-back wait limit), code " +
                                  std::to_string(h_ctr->err));
    return 0;
  }
};

namespace {

float elapsed(hipEvent_t a, hipEvent_t b) {
  float ms = 0.0f;
  if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return 0.0f;
  return ms;
}

}  // namespace

// Rows per kernel class of one iteration (the unit of each class's algorithmic bytes), from the
// counters that iteration published.  tail: the iteration ran every merge class in k_merge_tail.
static void count_class_rows(klsh_stats* st, const Counters& c, uint64_t n, bool tail) {
  using namespace klsh;
  uint64_t big_rows = 0, big_runs = 0, small_runs = 0;
  for (int b = 0; b < kBigClasses; ++b) big_rows += c.n_big_rows[b], big_runs += c.n_big[b];
  for (int b = 0; b < kGroupClasses; ++b) small_runs += c.n_cls[b];
  for (int k : {KC_PROJECT, KC_SORT, KC_COMPACT}) st->kern[k].rows += n;
  st->kern[KC_RUNS].rows += n;
  st->kern[KC_RUNS].runs += c.n_seg;
  st->kern[KC_HUGE].rows += c.n_huge_rows;
  st->kern[KC_HUGE].runs += c.n_huge;
  if (tail) {
    if (c.screened) {  // the screen saw every small run, k_merge_tail the ones it passed
      st->kern[KC_SCREEN].rows += c.n_small_rows;
      st->kern[KC_SCREEN].runs += small_runs;
      st->kern[KC_TAIL].rows += c.n_act_rows + big_rows;
    } else {
      st->kern[KC_TAIL].rows += c.n_small_rows + big_rows;
    }
    st->kern[KC_TAIL].runs += small_runs + big_runs;
    return;
  }
  if (c.screened) {  // the screen saw every small run, the merge only the ones it passed
    st->kern[KC_SCREEN].rows += c.n_small_rows;
    st->kern[KC_SCREEN].runs += small_runs;
    st->kern[KC_SMALL].rows += c.n_act_rows;
  } else {
    st->kern[KC_SMALL].rows += c.n_small_rows;
    st->kern[KC_SMALL].runs += small_runs;
  }
  for (int b = 0; b < kBigClasses; ++b) {
    st->kern[KC_BIG128 + b].rows += c.n_big_rows[b];
    st->kern[KC_BIG128 + b].runs += c.n_big[b];
  }
}

// The call's per-class spans: fold the last iteration's set, then read and clear the totals.
static int collect_kernel_times(klsh_ctx* ctx, int last_set, klsh_stats* st) {
  using namespace klsh;
  hipStream_t s = ctx->stream;
  if (last_set >= 0) launch_stamp_fold(ctx->kstamp, last_set, s);
  KLSH_HIP(hipGetLastError());
  unsigned long long tot[2][KC_COUNT];
  KLSH_HIP(hipMemcpyAsync(tot[0], ctx->kstamp->ticks, sizeof(tot), hipMemcpyDeviceToHost, s));
  KLSH_HIP(hipMemsetAsync(ctx->kstamp->ticks, 0, sizeof(tot), s));
  KLSH_HIP(hipStreamSynchronize(s));
  static_assert(offsetof(KStampBlock, launches) == offsetof(KStampBlock, ticks) + sizeof(unsigned long long) * KC_COUNT,
                "ticks and launches are adjacent");
  for (int k = 0; k < KC_COUNT; ++k) {
    st->kern[k].ms += (double)tot[0][k] * 1e-5;  // 100 MHz ticks
    st->kern[k].launches += tot[1][k];
  }
  return 0;
}

namespace klsh {
int ctx_device(const klsh_ctx* ctx) { return ctx->device; }
hipStream_t ctx_stream(const klsh_ctx* ctx) { return ctx->stream; }
int set_error(int code, const char* msg) { return fail(code, msg); }
}  // namespace klsh

// ===================================================================================== C ABI ===
extern "C" {

const char* klsh_last_error(void) { return g_err.c_str(); }
const char* klsh_version(void) { return "klsh-mi355x 0.2 (gfx950)"; }
int klsh_abi_version(void) { return KLSH_ABI_VERSION; }

klsh_ctx* klsh_create(int device, int* err) {
  auto set = [&](int e) {
    if (err) *err = e;
  };
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
    fail(KLSH_E_NODEVICE, "no HIP device visible (the engine has no CPU fallback)");
    set(KLSH_E_NODEVICE);
    return nullptr;
  }
  if (device < 0 || device >= count) {
    fail(KLSH_E_ARG, "device ordinal out of range");
    set(KLSH_E_ARG);
    return nullptr;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess ||
      std::string(prop.gcnArchName).find("gfx950") == std::string::npos) {
    fail(KLSH_E_NODEVICE, std::string("device is not gfx950: ") + prop.gcnArchName);
    set(KLSH_E_NODEVICE);
    return nullptr;
  }
  if (hipSetDevice(device) != hipSuccess) {
    fail(KLSH_E_HIP, "hipSetDevice");
    set(KLSH_E_HIP);
    return nullptr;
  }
  klsh_ctx* c = new klsh_ctx();
  c->device = device;
  // The big-run merge streams (aux 0 and the main stream, which carries the >384-row and
  // >896-row runs) get the highest priority: their workgroups need most of a CU's LDS and would
  // otherwise wait behind the small-run waves — on C4, where the >896-row runs are the critical
  // path, a normal-priority main stream doubled their time (KLSH_BIG_PRIORITY=0: all equal)
  int prio_lo = 0, prio_hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
  const bool big_prio = true;
  bool ok = hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking,
                                        big_prio ? prio_hi : prio_lo) == hipSuccess;
  // Every event here only times work or orders streams of this device: none makes device
  // writes visible to the host (the counters come back through the published mapped line, with
  // its own system-scope release).  A default event ends with a system-scope release — an L2
  // writeback of everything the kernel before it wrote, 6-16 us of stream time per event on C2
  // (the projection -> sort and fork / join gaps of the round-3 trace) — so timing events skip
  // the fence and the fork / join events release at device scope.
  const unsigned tflags = hipEventDisableSystemFence;
  const unsigned oflags = hipEventDisableTiming | hipEventReleaseToDevice;
  for (auto& e : c->ev) ok = ok && hipEventCreateWithFlags(&e, tflags) == hipSuccess;
  for (auto& e : c->sev) ok = ok && hipEventCreateWithFlags(&e, tflags) == hipSuccess;
  for (int i = 0; i < klsh::kMergeStreams; ++i) {
    const bool hi = i == 0;  // (the 65..192-row stream high too: measured equal)
    ok = ok && hipStreamCreateWithPriority(&c->mw.aux[i], hipStreamNonBlocking,
                                           (hi && big_prio) ? prio_hi : prio_lo) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&c->mw.join[i], oflags) == hipSuccess;
  }
  ok = ok && hipEventCreateWithFlags(&c->mw.fork, oflags) == hipSuccess;
  ok = ok && hipMalloc((void**)&c->ctr, sizeof(Counters)) == hipSuccess;
  ok = ok && hipHostMalloc((void**)&c->h_ctr, sizeof(Counters), hipHostMallocDefault) == hipSuccess;
  ok = ok && hipMemset(c->ctr, 0, sizeof(Counters)) == hipSuccess;  // err starts clear
  ok = ok && hipMalloc((void**)&c->rc, sizeof(klsh::RunCounters)) == hipSuccess &&
       hipMemset(c->rc, 0, sizeof(klsh::RunCounters)) == hipSuccess;
  c->mw.rc = c->rc;
  ok = ok && hipMalloc((void**)&c->n_next_dev, 64) == hipSuccess &&
       hipMemset(c->n_next_dev, 0, 64) == hipSuccess;
  if (ok && c->zero_copy) {
    void* hp = nullptr;
    void* dp = nullptr;
    // [published counters][sequence word, 64 B][kRing ring slots]
    const size_t ring_at = sizeof(Counters) + 64;
    const size_t bytes = ring_at + sizeof(Counters) * klsh_ctx::kRing;
    if (hipHostMalloc(&hp, bytes, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess &&
        hipHostGetDevicePointer(&dp, hp, 0) == hipSuccess) {
      memset(hp, 0, bytes);
      c->pub_host = static_cast<Counters*>(hp);
      c->pub_dev = static_cast<Counters*>(dp);
      c->pub_seq_host = reinterpret_cast<uint32_t*>(static_cast<char*>(hp) + sizeof(Counters));
      c->pub_seq_dev = reinterpret_cast<uint32_t*>(static_cast<char*>(dp) + sizeof(Counters));
      c->ring_host = reinterpret_cast<Counters*>(static_cast<char*>(hp) + ring_at);
      c->ring_dev = reinterpret_cast<Counters*>(static_cast<char*>(dp) + ring_at);
    } else {
      if (hp) (void)hipHostFree(hp);
      c->zero_copy = false;  // fall back to copy + sync
    }
  }
  if (!ok) {
    delete c;
    fail(KLSH_E_HIP, "stream/event/counter allocation failed");
    set(KLSH_E_HIP);
    return nullptr;
  }
  memset(c->h_ctr, 0, sizeof(Counters));
  set(KLSH_OK);
  return c;
}

void klsh_destroy(klsh_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  delete ctx;
}

int klsh_load_rows(klsh_ctx* ctx, const float* rows, uint64_t n, int d,
                   const uint64_t* member_offsets, const uint64_t* member_ids) {
  if (!ctx || (!rows && n)) return fail(KLSH_E_ARG, "null argument");
  KLSH_HIP(hipSetDevice(ctx->device));
  const uint64_t m = member_offsets ? member_offsets[n] : n;
  if (int e = ctx->reserve(n, m, d)) return e;
  hipStream_t s = ctx->stream;
  if (n) {
    KLSH_HIP(hipMemsetAsync(ctx->rows.x, 0, sizeof(float) * n * ctx->dp, s));
    KLSH_HIP(hipMemcpy2DAsync(ctx->rows.x, sizeof(float) * ctx->dp, rows, sizeof(float) * d,
                              sizeof(float) * d, n, hipMemcpyHostToDevice, s));
  }
  std::vector<uint32_t> cnt(n), head(n), tail(n), nxt(m), ord(n);
  ctx->ids.assign(m, 0);
  for (uint64_t i = 0; i < n; ++i) {
    ord[i] = (uint32_t)i;
    if (member_offsets) {
      const uint64_t a = member_offsets[i], b = member_offsets[i + 1];
      cnt[i] = (uint32_t)(b - a);
      head[i] = b > a ? (uint32_t)a : klsh::kNil;
      tail[i] = b > a ? (uint32_t)(b - 1) : klsh::kNil;
      for (uint64_t k = a; k < b; ++k) {
        nxt[k] = k + 1 < b ? (uint32_t)(k + 1) : klsh::kNil;
        ctx->ids[k] = member_ids ? member_ids[k] : k;
      }
    } else {
      cnt[i] = 1;
      head[i] = tail[i] = (uint32_t)i;
      nxt[i] = klsh::kNil;
      ctx->ids[i] = member_ids ? member_ids[i] : i;
    }
  }
  if (n) {
    KLSH_HIP(hipMemcpyAsync(ctx->rows.cnt, cnt.data(), 4 * n, hipMemcpyHostToDevice, s));
    KLSH_HIP(hipMemcpyAsync(ctx->rows.head, head.data(), 4 * n, hipMemcpyHostToDevice, s));
    KLSH_HIP(hipMemcpyAsync(ctx->rows.tail, tail.data(), 4 * n, hipMemcpyHostToDevice, s));
    KLSH_HIP(hipMemcpyAsync(ctx->order, ord.data(), 4 * n, hipMemcpyHostToDevice, s));
  }
  if (m) KLSH_HIP(hipMemcpyAsync(ctx->rows.nxt, nxt.data(), 4 * m, hipMemcpyHostToDevice, s));
  klsh::launch_norms(ctx->rows, (uint32_t)n, s);
  KLSH_HIP(hipGetLastError());
  KLSH_HIP(hipStreamSynchronize(s));
  ctx->slots = n;
  ctx->members = m;
  klsh::launch_shadow_build(ctx->rows, ctx->slots, s);
  KLSH_HIP(hipGetLastError());
  ctx->n_live = n;
  ctx->loaded = true;
  return 0;
}

int klsh_load_counts(klsh_ctx* ctx, const uint16_t* counts, uint64_t n_total,
                     uint64_t batch_offset, uint64_t batch_size, int d, const float* v_kmers) {
  if (!ctx || !counts || !v_kmers) return fail(KLSH_E_ARG, "null argument");
  if (batch_offset + batch_size > n_total) return fail(KLSH_E_ARG, "batch outside the matrix");
  KLSH_HIP(hipSetDevice(ctx->device));
  const uint64_t bs = batch_size;
  if (int e = ctx->reserve(bs, bs, d)) return e;
  hipStream_t s = ctx->stream;
  // float(log(c + 1.0)) for every uint16 count: glibc double log on the host, exact.
  static std::vector<float> lut;
  if (lut.empty()) {
    lut.resize(65536);
    for (int c = 0; c < 65536; ++c) lut[c] = (float)std::log((double)c + 1.0);
  }
  uint16_t* dcounts = nullptr;
  float *dlut = nullptr, *dv = nullptr;
  if (int e = dalloc(&dcounts, (size_t)bs * d)) return e;
  if (int e = dalloc(&dlut, 65536)) { dfree(dcounts); return e; }
  if (int e = dalloc(&dv, d)) { dfree(dcounts); dfree(dlut); return e; }
  int rc = 0;
  do {
    if (bs) {
      if (hipMemcpy2DAsync(dcounts, sizeof(uint16_t) * bs, counts + batch_offset,
                           sizeof(uint16_t) * n_total, sizeof(uint16_t) * bs, d,
                           hipMemcpyHostToDevice, s) != hipSuccess) {
        rc = fail(KLSH_E_HIP, "count upload");
        break;
      }
    }
    if (hipMemcpyAsync(dlut, lut.data(), sizeof(float) * 65536, hipMemcpyHostToDevice, s) !=
            hipSuccess ||
        hipMemcpyAsync(dv, v_kmers, sizeof(float) * d, hipMemcpyHostToDevice, s) != hipSuccess) {
      rc = fail(KLSH_E_HIP, "lut upload");
      break;
    }
    if (ctx->reset_counters()) {
      rc = fail(KLSH_E_HIP, "counter reset");
      break;
    }
    klsh::launch_convert(ctx->rows, dcounts, (uint32_t)bs, dlut, dv, ctx->keys, ctx->order,
                         ctx->tile_sums, ctx->ctr, s);
    if (hipGetLastError() != hipSuccess) {
      rc = fail(KLSH_E_HIP, "convert launch");
      break;
    }
    if ((rc = ctx->sync_counters())) break;
  } while (false);
  (void)hipStreamSynchronize(s);
  dfree(dcounts);
  dfree(dlut);
  dfree(dv);
  if (rc) return rc;
  ctx->ids.resize(bs);
  for (uint64_t i = 0; i < bs; ++i) ctx->ids[i] = batch_offset + i;
  ctx->slots = bs;
  ctx->members = bs;
  klsh::launch_shadow_build(ctx->rows, ctx->slots, s);
  KLSH_HIP(hipGetLastError());
  ctx->n_live = bs ? ctx->h_ctr->total : 0;
  ctx->loaded = true;
  return 0;
}

int klsh_snapshot(klsh_ctx* ctx) {
  if (!ctx || !ctx->loaded) return fail(KLSH_E_STATE, "nothing loaded");
  KLSH_HIP(hipSetDevice(ctx->device));
  Snapshot& sn = ctx->snap;
  if (!sn.valid) {
    int e = 0;
    const uint64_t s = std::max<uint64_t>(ctx->slots, 1), m = std::max<uint64_t>(ctx->members, 1);
    if ((e = dalloc(&sn.x, s * ctx->dp)) || (e = dalloc(&sn.nrm, s)) || (e = dalloc(&sn.cnt, s)) ||
        (e = dalloc(&sn.head, s)) || (e = dalloc(&sn.tail, s)) || (e = dalloc(&sn.nxt, m)) ||
        (e = dalloc(&sn.order, s))) {
      ctx->drop_snapshot();
      return e;
    }
  }
  hipStream_t st = ctx->stream;
  const uint64_t s = ctx->slots, m = ctx->members;
  KLSH_HIP(hipMemcpyAsync(sn.x, ctx->rows.x, 4 * s * ctx->dp, hipMemcpyDeviceToDevice, st));
  KLSH_HIP(hipMemcpyAsync(sn.nrm, ctx->rows.nrm, 4 * s, hipMemcpyDeviceToDevice, st));
  KLSH_HIP(hipMemcpyAsync(sn.cnt, ctx->rows.cnt, 4 * s, hipMemcpyDeviceToDevice, st));
  KLSH_HIP(hipMemcpyAsync(sn.head, ctx->rows.head, 4 * s, hipMemcpyDeviceToDevice, st));
  KLSH_HIP(hipMemcpyAsync(sn.tail, ctx->rows.tail, 4 * s, hipMemcpyDeviceToDevice, st));
  KLSH_HIP(hipMemcpyAsync(sn.nxt, ctx->rows.nxt, 4 * m, hipMemcpyDeviceToDevice, st));
  KLSH_HIP(hipMemcpyAsync(sn.order, ctx->order, 4 * ctx->n_live, hipMemcpyDeviceToDevice, st));
  KLSH_HIP(hipStreamSynchronize(st));
  sn.n_live = ctx->n_live;
  sn.valid = true;
  return 0;
}

int klsh_restore(klsh_ctx* ctx) {
  if (!ctx || !ctx->snap.valid) return fail(KLSH_E_STATE, "no snapshot");
  KLSH_HIP(hipSetDevice(ctx->device));
  Snapshot& sn = ctx->snap;
  hipStream_t st = ctx->stream;
  const uint64_t s = ctx->slots, m = ctx->members;
  KLSH_HIP(hipMemcpyAsync(ctx->rows.x, sn.x, 4 * s * ctx->dp, hipMemcpyDeviceToDevice, st));
  KLSH_HIP(hipMemcpyAsync(ctx->rows.nrm, sn.nrm, 4 * s, hipMemcpyDeviceToDevice, st));
  KLSH_HIP(hipMemcpyAsync(ctx->rows.cnt, sn.cnt, 4 * s, hipMemcpyDeviceToDevice, st));
  KLSH_HIP(hipMemcpyAsync(ctx->rows.head, sn.head, 4 * s, hipMemcpyDeviceToDevice, st));
  KLSH_HIP(hipMemcpyAsync(ctx->rows.tail, sn.tail, 4 * s, hipMemcpyDeviceToDevice, st));
  KLSH_HIP(hipMemcpyAsync(ctx->rows.nxt, sn.nxt, 4 * m, hipMemcpyDeviceToDevice, st));
  KLSH_HIP(hipMemcpyAsync(ctx->order, sn.order, 4 * sn.n_live, hipMemcpyDeviceToDevice, st));
  KLSH_HIP(hipStreamSynchronize(st));
  klsh::launch_shadow_build(ctx->rows, ctx->slots, st);  // (rebuilt, not snapshotted)
  KLSH_HIP(hipGetLastError());
  ctx->n_live = sn.n_live;
  return 0;
}

// Merge + compaction of one iteration's sorted runs (fk/fv, n positions, in place on fv) into
// `out` (with ctx->mw.dlist set, the merge kernels also list the survivors they rewrote).
// Ends with the counters on the host: total (survivors), n_over (oversize runs), n_delta.
// kt: the iteration's stamps (kNoTime: untimed).
static int merge_main(klsh_ctx* ctx, uint32_t* fk, uint32_t* fv, uint32_t n, float thr,
                      int bucket_thr, uint32_t* out, klsh_stats* st, bool timed,
                      bool sync = true, const std::function<int(uint32_t*)>* after = nullptr,
                      klsh::KTime kt = klsh::kNoTime) {
  hipStream_t s = ctx->stream;
  if (timed) KLSH_HIP(hipEventRecord(ctx->ev[2], s));
  // the small-run merge is a launch of its own at >= 2^20 positions (register widths): its HIP
  // events are the headline's cross-check
  const bool time_small = (ctx->hip_events || ctx->phase_timing) && kt.blk && st && sync &&
                          n >= klsh::tail_merge_max(ctx->mw) && klsh::project_device_n_ok(ctx->d);
  ctx->mw.small_ev[0] = time_small ? ctx->sev[0] : nullptr;
  ctx->mw.small_ev[1] = time_small ? ctx->sev[1] : nullptr;
  ctx->mw.kt = kt;
  klsh::launch_merge(ctx->rows, fk, fv, 0, n, thr, bucket_thr, ctx->mw, ctx->ctr, s);
  ctx->mw.kt = klsh::kNoTime;
  ctx->mw.small_ev[0] = ctx->mw.small_ev[1] = nullptr;
  KLSH_HIP(hipGetLastError());
  if (timed) KLSH_HIP(hipEventRecord(ctx->ev[3], s));
  const bool zc = sync && ctx->zero_copy;
  klsh::Publish pub{ctx->pub_dev, ctx->pub_seq_dev, ++ctx->pub_seq, ctx->n_next_dev};
  klsh::launch_compact(fv, n, out, ctx->tile_sums, ctx->ctr, s, zc ? &pub : nullptr, ctx->rc, kt,
                       ctx->lb.status ? &ctx->lb : nullptr);
  KLSH_HIP(hipGetLastError());
  if (timed) KLSH_HIP(hipEventRecord(ctx->ev[4], s));
  if (zc && after)  // work queued behind the compaction before the host waits for it
    if (int e = (*after)(out)) return e;
  if (!sync) return 0;  // the caller fetches the counters with its own exchange
  ctx->t_enqueued = now_ms();
  if (zc) {
    if (int e = ctx->wait_published(pub.seq)) return e;
  } else {
    ctx->ctr_clean = false;
    if (int e = ctx->sync_counters()) return e;
  }
  if (kt.blk && st) {  // this iteration's rows per kernel class
    const bool tail = n < klsh::tail_merge_max(ctx->mw) && klsh::project_device_n_ok(ctx->d);
    count_class_rows(st, *ctx->h_ctr, n, tail);
  }
  if (time_small) {  // the compaction (published) runs after the merge streams' join
    KLSH_HIP(hipEventSynchronize(ctx->sev[1]));
    st->small_ms += elapsed(ctx->sev[0], ctx->sev[1]);
    st->small_launches += 1;
    st->small_rows += ctx->h_ctr->screened ? ctx->h_ctr->n_act_rows : ctx->h_ctr->n_small_rows;
    st->small_iter_merges += n - ctx->h_ctr->total;
  }
  if (timed && zc) KLSH_HIP(hipEventSynchronize(ctx->ev[4]));
  if (timed && st) {
    st->merge_ms += elapsed(ctx->ev[2], ctx->ev[3]);
    st->compact_ms += elapsed(ctx->ev[3], ctx->ev[4]);
  }
  return 0;
}

// The oversize runs of the last merge_main, ascending (the reference's T=1 order):
// (start, length) pairs and the hyperplanes their nestedCluster calls draw (floor(log2 b) each).
static int oversize_runs(klsh_ctx* ctx, std::vector<uint2>* over, uint64_t* hyperplanes) {
  const uint32_t n_over = ctx->h_ctr->n_over;
  over->resize(n_over);
  *hyperplanes = 0;
  if (n_over == 0) return 0;
  KLSH_HIP(hipMemcpy(over->data(), ctx->mw.over, sizeof(uint2) * n_over, hipMemcpyDeviceToHost));
  std::sort(over->begin(), over->end(), [](const uint2& a, const uint2& b) { return a.x < b.x; });
  for (const uint2& o : *over) *hyperplanes += (uint64_t)floor_log2(o.y);
  return 0;
}

// nestedCluster (cluster.cc:286-288 -> :89-178) for each oversize run, ascending, drawing
// hyperplanes from *rng_counter on; then the survivors are compacted again into `out`.  Ends with
// the counters on the host.
static int merge_nested(klsh_ctx* ctx, uint32_t* fk, uint32_t* fv, uint32_t n, float thr,
                        const std::vector<uint2>& over, uint32_t seed_base, uint64_t* rng_counter,
                        uint32_t* out, klsh_stats* st) {
  hipStream_t s = ctx->stream;
  for (uint32_t oi = 0; oi < (uint32_t)over.size(); ++oi) {
    const uint32_t p = over[oi].x, b = over[oi].y;
    const int h2 = floor_log2(b);
    const uint64_t k = *rng_counter;
    *rng_counter += (uint64_t)h2;
    if (st) {
      st->hyperplanes += (uint64_t)h2;
      st->nested_calls += 1;
    }
    if (int e = ctx->ensure_hyperplanes(seed_base, k, (uint64_t)h2, st ? &st->host_ms : nullptr))
      return e;
    // Sub-keys carry bit 31 (main keys are < 2^h <= 2^31, so never have it) and a bit 30 that
    // alternates between consecutive oversize regions, so no run crosses a region boundary.
    const uint32_t key_or = 0x80000000u | ((oi & 1u) << 30);
    klsh::launch_project(ctx->rows, fv + p, ctx->nk1, b, ctx->hyperplane_ptr(k), h2, key_or, s,
                         &ctx->pw);
    uint32_t *rk = nullptr, *rv = nullptr;
    klsh::radix_sort(ctx->nk1, fv + p, ctx->nk2, ctx->nv2, b, h2, ctx->hist, &rk, &rv, s);
    KLSH_HIP(hipMemcpyAsync(fk + p, rk, 4ull * b, hipMemcpyDeviceToDevice, s));
    if (rv != fv + p) KLSH_HIP(hipMemcpyAsync(fv + p, rv, 4ull * b, hipMemcpyDeviceToDevice, s));
    // fresh run lists for the region
    KLSH_HIP(hipMemsetAsync(ctx->rc, 0, sizeof(klsh::RunCounters), s));
    klsh::launch_merge(ctx->rows, fk, fv, p, p + b, thr, -1, ctx->mw, ctx->ctr, s);
    KLSH_HIP(hipGetLastError());
  }
  klsh::launch_compact(fv, n, out, ctx->tile_sums, ctx->ctr, s, nullptr, ctx->rc);
  KLSH_HIP(hipGetLastError());
  return ctx->sync_counters();
}

// Single-GPU: merge, compaction and nested buckets of one iteration.  fk/fv: sorted keys/slots
// (fv is one of ctx->order / ctx->alt).  Returns with the new canonical order in ctx->order and
// ctx->n_live updated.
static int merge_and_compact(klsh_ctx* ctx, uint32_t* fk, uint32_t* fv, uint32_t n, float thr,
                             int bucket_thr, uint32_t seed_base, uint64_t* rng_counter,
                             klsh_stats* st, bool timed,
                             const std::function<int(uint32_t*)>* after = nullptr,
                             klsh::KTime kt = klsh::kNoTime) {
  uint32_t* out = (fv == ctx->order) ? ctx->alt : ctx->order;
  if (int e = merge_main(ctx, fk, fv, n, thr, bucket_thr, out, st, timed, true, after, kt))
    return e;
  // many 385..896-row runs this iteration: the next one runs that class on an auxiliary stream
  ctx->mw.big896_aux = ctx->h_ctr->n_big[klsh::kBigClasses - 1] >= 64u ? 1u : 0u;
  // no >896-row runs this iteration: the next one's launch for them is 64 workgroups (C4 has
  // iterations without them between ones with dozens: a cap of 4 serialised those walks,
  // k_merge_huge<32> 746 -> 1024 ms per step)
  ctx->mw.huge_cap = ctx->h_ctr->n_huge == 0 ? 64u : 0u;
  // several iterations in a row without them: the next one walks any >896-row runs inside the
  // 385..896-row kernel instead of launching k_merge_huge (an empty launch on C2 / C5)
  ctx->huge_quiet = ctx->h_ctr->n_huge == 0 ? ctx->huge_quiet + 1 : 0;
  ctx->mw.huge_fold = (ctx->huge_quiet >= 4 || ctx->huge_fold_always) ? 1u : 0u;
  if (ctx->h_ctr->n_over > 0) {
    std::vector<uint2> over;
    uint64_t hyp = 0;
    if (int e = oversize_runs(ctx, &over, &hyp)) return e;
    if (int e = merge_nested(ctx, fk, fv, n, thr, over, seed_base, rng_counter, out, st))
      return e;
  }
  if (out == ctx->alt) std::swap(ctx->order, ctx->alt);
  ctx->n_live = ctx->h_ctr->total;
  return 0;
}

// ------------------------------------------------------------------ queued tail batches -----
// Once no bucket can be oversize (N_t <= bucket_size_threshold: nestedCluster, which needs the
// host's RNG order, cannot happen) and N_t < 2^20 (the one-launch merge and compaction), the rest
// of the loop needs nothing from the host: every kernel of an iteration reads N_t from
// n_next_dev, the projection finds its hyperplanes at the offset woff (each compaction advances it
// by its own h = floor(log2 N_t), cluster.cc:194-196), the sort runs the passes of the largest h
// ahead (passes over all-zero digits are stable identities), the threshold schedule is known.
// Iterations are queued C at a time, two chunks in flight; every compaction publishes into its own
// ring slot and the host reads a chunk's slots when its last sequence number is in — the trace,
// the RNG counter and the statistics come out exactly as the per-iteration loop's.
static bool batch_eligible(const klsh_ctx* ctx, uint64_t n, int bucket_thr, int iters_left) {
  // (< 2^20 too: the queued compaction is the one-launch look-back over <= 256 tiles)
  if (!ctx->tail_batch || n < 2 || n >= std::min<uint64_t>(klsh::tail_merge_max(ctx->mw), 1u << 20) ||
      iters_left < 2)
    return false;
  if (bucket_thr >= 0 && n > (uint64_t)bucket_thr) return false;
  if (!ctx->zero_copy || !ctx->ring_dev || !ctx->lb.status || ctx->phase_timing) return false;
  if (!klsh::project_device_n_ok(ctx->d) || ctx->mw.dlist) return false;
#ifdef KLSH_DIAG
  if (getenv("KLSH_BUCKET_STATS") || getenv("KLSH_ITER_LOG")) return false;
#endif
  // every queued iteration's hyperplanes resident at once
  return (uint64_t)iters_left * (uint64_t)floor_log2(n) * (uint64_t)ctx->dp <= (64ull << 20);
}

static int run_batched(klsh_ctx* ctx, float& threshold, float sim_step, int it, int it_end,
                       int bucket_size_threshold, uint32_t seed_base, uint64_t* rng_counter,
                       uint64_t* nt_trace, klsh_stats* st,
                       const std::function<klsh::KTime(uint64_t)>& ktime) {
  hipStream_t s = ctx->stream;
#ifdef KLSH_MERGE_PROF
  if (getenv("KLSH_MERGE_PROF")) {  // diagnostics: the head's merge profile apart from the tail's
    fprintf(stderr, "[mprof] ---- head: iterations before %d\n", it);
    klsh::merge_prof_dump(stderr);
    fprintf(stderr, "[mprof] ---- tail: iterations %d..%d\n", it, it_end - 1);
  }
#endif
  constexpr int C = klsh_ctx::kRing / 2;  // iterations per chunk
  uint64_t n_known = ctx->n_live;         // N after the last iteration the host has read
  const int h0 = floor_log2(n_known);
  const uint64_t k0 = *rng_counter;
  const uint64_t need = (uint64_t)(it_end - it) * (uint64_t)h0;
  if (!(ctx->W && ctx->w_base == seed_base && ctx->w_dp == ctx->dp && ctx->w_d == ctx->d &&
        k0 >= ctx->w_k0 && k0 + need <= ctx->w_k0 + ctx->w_count)) {
    // a window restart may overwrite rows a queued projection still reads; an append may not
    if (!ctx->lazy_covers(seed_base, k0, need)) KLSH_HIP(hipStreamSynchronize(s));
    if (int e = ctx->ensure_hyperplanes(seed_base, k0, need, &st->host_ms)) return e;
  }
  uint32_t* n_dev = ctx->n_next_dev;
  uint32_t* woff_dev = ctx->n_next_dev + 1;
  KLSH_HIP(hipMemsetD32Async(n_dev, (int)(uint32_t)n_known, 1, s));
  KLSH_HIP(hipMemsetD32Async(woff_dev, (int)(uint32_t)(k0 - ctx->w_k0), 1, s));
  bool queued = ctx->spec_pending;  // the first projection is already on the stream
  ctx->spec_pending = false;
  if (queued && ctx->spec_swap) std::swap(ctx->keys, ctx->keys2);
  ctx->spec_swap = false;
  if (!queued && !ctx->ctr_clean)
    if (int e = ctx->reset_counters()) return e;
  if (queued && ctx->spec_k != k0) return fail(KLSH_E_STATE, "queued projection out of step");

  struct Chunk {
    int it0, count, slot0;
    uint32_t seq_last;
  };
  std::deque<Chunk> inflight;
  int next = it, slot = 0;
  float thr = threshold;
  uint64_t n_max = n_known;
  auto enqueue = [&](int count) -> int {
    const int hb = floor_log2(n_max);  // h of every iteration of the chunk is <= hb
    for (int c = 0; c < count; ++c, ++next) {
      const klsh::KTime kt = ktime(ctx->kt_iter++);
      if (!queued)
        klsh::launch_project_device_n(ctx->rows, ctx->order, ctx->keys, (uint32_t)n_max, ctx->W,
                                      n_dev, s, kt, woff_dev, &ctx->pw);
      queued = false;
      uint32_t *fk = nullptr, *fv = nullptr;
      const bool local = ctx->tail_local && klsh::tail_local_ok((uint32_t)n_max, hb);
      if (local) {  // top-bits partition, then the buckets sorted in LDS with their runs listed
        const uint32_t* dtot = klsh::radix_sort_top(ctx->keys, ctx->order, ctx->keys2, ctx->alt,
                                                    (uint32_t)n_max, hb, ctx->hist, s, kt, n_dev);
        ctx->mw.kt = kt;
        klsh::launch_tail_local(ctx->keys2, ctx->alt, ctx->keys, ctx->order, dtot, hb,
                                bucket_size_threshold, ctx->mw, s);
        fk = ctx->keys;
        fv = ctx->order;
      } else {
        klsh::radix_sort(ctx->keys, ctx->order, ctx->keys2, ctx->alt, (uint32_t)n_max, hb,
                         ctx->hist, &fk, &fv, s, kt, n_dev);
        ctx->mw.kt = kt;
      }
      klsh::launch_merge(ctx->rows, fk, fv, 0, (uint32_t)n_max, thr, bucket_size_threshold,
                         ctx->mw, ctx->ctr, s, n_dev, local);
      ctx->mw.kt = klsh::kNoTime;
      uint32_t* out = (fv == ctx->order) ? ctx->alt : ctx->order;
      klsh::Publish pub{ctx->ring_dev + slot, ctx->pub_seq_dev, ++ctx->pub_seq, n_dev, woff_dev};
      klsh::launch_compact(fv, (uint32_t)n_max, out, ctx->tile_sums, ctx->ctr, s, &pub, ctx->rc,
                           kt, &ctx->lb, n_dev);
      if (out == ctx->alt) std::swap(ctx->order, ctx->alt);
      thr -= sim_step;
      slot = (slot + 1) % klsh_ctx::kRing;
    }
    KLSH_HIP(hipGetLastError());
    return 0;
  };
  while (next < it_end || !inflight.empty()) {
    while (next < it_end && inflight.size() < 2) {
      const Chunk ch{next, std::min(C, it_end - next), slot, 0u};
      if (int e = enqueue(ch.count)) return e;
      inflight.push_back(ch);
      inflight.back().seq_last = ctx->pub_seq;
    }
    const Chunk ch = inflight.front();
    inflight.pop_front();
    if (int e = ctx->wait_seq(ch.seq_last)) return e;
    for (int c = 0; c < ch.count; ++c) {
      const Counters cc = ctx->ring_host[(ch.slot0 + c) % klsh_ctx::kRing];
      const uint64_t n_in = n_known;
      if (cc.err)
        return fail(KLSH_E_HIP, "device protocol failure (look-back wait limit), code " +
                                    std::to_string(cc.err));
      if (cc.n_over || n_in == 0 || cc.total == 0 || cc.total > n_in)
        return fail(KLSH_E_STATE, "queued iteration published inconsistent counters");
      const int h = floor_log2(n_in);
      if (nt_trace) nt_trace[ch.it0 + c] = n_in;
      st->iterations += 1;
      ctx->tick(ch.it0 + c);
      st->project_launches += 1;  // (no HIP events around queued launches: not in project_ms)
      *rng_counter += (uint64_t)h;
      st->hyperplanes += (uint64_t)h;
      st->sum_rows += n_in;
      st->sum_proj_bits += n_in * (uint64_t)h;
      st->sum_merges += n_in - cc.total;
      if (ctx->kernel_timing && ctx->kstamp) count_class_rows(st, cc, n_in, true);
#ifdef KLSH_DIAG
      static FILE* batch_log = [] {  // diagnostics build: the run classes of queued iterations
        const char* e = getenv("KLSH_ITER_LOG");
        return e ? fopen(e, "a") : nullptr;
      }();
      if (batch_log)
        fprintf(batch_log, "%d %llu %d batched runs %u small_rows %u big %u %u %u %u huge %u\n",
                ch.it0 + c, (unsigned long long)n_in, h, cc.n_seg, cc.n_small_rows, cc.n_big[0],
                cc.n_big[1], cc.n_big[2], cc.n_big[3], cc.n_huge);
      if (batch_log) fflush(batch_log);
#endif
      *ctx->h_ctr = cc;
      n_known = cc.total;
    }
    n_max = n_known;  // tighter grids for the chunks queued from now on
  }
  threshold = thr;
  ctx->n_live = n_known;
  ctx->ctr_clean = true;  // every publisher zeroed the counters behind it
  return 0;
}

// Iterations [it_begin, it_end) of the single-device loop over the whole canonical order
// (cluster.cc:193-334).  `threshold` is advanced by sim_step per iteration.
static int run_single(klsh_ctx* ctx, float& threshold, float sim_step, int it_begin, int it_end,
                      int bucket_size_threshold, uint32_t seed_base, uint64_t* rng_counter,
                      uint64_t* nt_trace, klsh_stats* st) {
  hipStream_t s = ctx->stream;
#ifdef KLSH_DIAG  // diagnostics build: per-iteration wall time (it, n, h, ms)
  static FILE* iter_log = [] {
    const char* e = getenv("KLSH_ITER_LOG");
    return e ? fopen(e, "a") : nullptr;
  }();
#else
  FILE* const iter_log = nullptr;
#endif
  // per-class timing: iteration `it` uses set it & 1 (its queued projection included); the
  // previous iteration's set is read once this one's work is queued
  // per-class stamps: the call's iterations stamp sets 0, 1, 0, ... in turn (ctx->kt_iter); a
  // projection first folds the set of the iteration before it
  const uint64_t kt_first = ctx->kt_iter;
  auto ktime = [&](uint64_t j) -> klsh::KTime {
    if (!ctx->kernel_timing || !st) return klsh::kNoTime;
    if (!ctx->kstamp) return klsh::kNoTime;
    return klsh::KTime{ctx->kstamp, (int)(j & 1u), j > kt_first ? (int)((j - 1) & 1u) : -1};
  };
  for (int it = it_begin; it < it_end; ++it) {
    const uint64_t n = ctx->n_live;
    if (batch_eligible(ctx, n, bucket_size_threshold, it_end - it)) {  // the rest, queued
      const std::function<klsh::KTime(uint64_t)> kt_fn = ktime;
      if (int e = run_batched(ctx, threshold, sim_step, it, it_end, bucket_size_threshold,
                              seed_base, rng_counter, nt_trace, st, kt_fn))
        return e;
      break;
    }
    const double t_it = iter_log ? now_ms() : 0.0;
    if (nt_trace) nt_trace[it] = n;
    st->iterations += 1;
    ctx->tick(it);
    if (n == 0) {  // the reference aborts here (cluster.cc:194 on an empty vector); no-op
      threshold -= sim_step;
      continue;
    }
    const int h = floor_log2(n);
    const uint64_t k = *rng_counter;
    *rng_counter += (uint64_t)h;
    st->hyperplanes += (uint64_t)h;
    if (int e = ctx->ensure_hyperplanes(seed_base, k, (uint64_t)h, &st->host_ms)) return e;

    // the projection: queued by the previous iteration (device-side N), or now
    const bool queued = ctx->spec_pending;
    ctx->spec_pending = false;
    if (queued && ctx->spec_swap) std::swap(ctx->keys, ctx->keys2);  // the queued keys' buffer
    ctx->spec_swap = false;
    const uint64_t j = ctx->kt_iter++;  // this iteration's stamp set
    if (queued && ctx->spec_k != k) return fail(KLSH_E_STATE, "queued projection out of step");
    const int e0 = queued ? ctx->spec_ev : 0;
    // the projection runs alone on the main stream: with option hip_events an event pair times it
    // (beside its stamps).  Off by default: each record is a marker packet the stream waits on,
    // ~9 us between the projection and the sort of every host-driven iteration (rocprofv3 trace,
    // round 6) — the in-kernel stamps time it without one.
    const bool rec = ctx->hip_events || ctx->phase_timing;
    if (!queued) {
      if (!ctx->ctr_clean) if (int e = ctx->reset_counters()) return e;
      if (rec) KLSH_HIP(hipEventRecord(ctx->ev[e0], s));
      klsh::launch_project(ctx->rows, ctx->order, ctx->keys, (uint32_t)n, ctx->hyperplane_ptr(k), h,
                           0u, s, &ctx->pw, ktime(j));
      KLSH_HIP(hipGetLastError());
      if (rec) KLSH_HIP(hipEventRecord(ctx->ev[e0 + 1], s));
    }
    ctx->ctr_clean = false;
    uint32_t *fk = nullptr, *fv = nullptr;
    klsh::radix_sort(ctx->keys, ctx->order, ctx->keys2, ctx->alt, (uint32_t)n, h, ctx->hist,
                     &fk, &fv, s, ktime(j));
    KLSH_HIP(hipGetLastError());
    if (ctx->phase_timing) KLSH_HIP(hipEventRecord(ctx->ev[5], s));
#ifdef KLSH_DIAG
    if (const char* path = getenv("KLSH_BUCKET_STATS")) {  // diagnostics: run-length histogram
      std::vector<uint32_t> hk(n);
      KLSH_HIP(hipMemcpyAsync(hk.data(), fk, 4 * n, hipMemcpyDeviceToHost, s));
      KLSH_HIP(hipStreamSynchronize(s));
      uint64_t hist[12] = {0}, pairs = 0, maxb = 0, rows_in[12] = {0};
      for (uint64_t a = 0; a < n;) {
        uint64_t b = a + 1;
        while (b < n && hk[b] == hk[a]) ++b;
        const uint64_t len = b - a;
        int c = 0;
        while (c < 11 && (1ull << c) < len) ++c;  // class c: len in (2^(c-1), 2^c]
        hist[c]++;
        rows_in[c] += len;
        pairs += len * (len - 1) / 2;
        maxb = std::max(maxb, len);
        a = b;
      }
      if (FILE* f = fopen(path, "a")) {
        fprintf(f, "{\"it\": %d, \"n\": %llu, \"h\": %d, \"pairs\": %llu, \"max\": %llu, \"hist\": [", it,
                (unsigned long long)n, h, (unsigned long long)pairs, (unsigned long long)maxb);
        for (int c = 0; c < 12; ++c) fprintf(f, "%s%llu", c ? ", " : "", (unsigned long long)hist[c]);
        fprintf(f, "], \"rows\": [");
        for (int c = 0; c < 12; ++c) fprintf(f, "%s%llu", c ? ", " : "", (unsigned long long)rows_in[c]);
        fprintf(f, "]}\n");
        fclose(f);
      }
    }
#endif
    // Queue the next iteration's projection behind this compaction.  If this iteration turns out
    // to have oversize buckets (nestedCluster changes rows and draws hyperplanes first), the
    // queued keys are simply recomputed; they go to the key buffer the nested work is not reading
    // (this iteration's sorted keys fk stay intact), keys2 when fk is keys — the next iteration
    // then swaps the two pointers.
#ifdef KLSH_DIAG
    const bool diag_stats = getenv("KLSH_BUCKET_STATS") != nullptr;
#else
    const bool diag_stats = false;
#endif
    const bool ahead = ctx->zero_copy && it + 1 < it_end &&
                       klsh::project_device_n_ok(ctx->d) && !diag_stats;
    uint32_t* const spec_out = fk == ctx->keys ? ctx->keys2 : ctx->keys;
    const std::function<int(uint32_t*)> queue_next = [&](uint32_t* next_order) -> int {
      const uint64_t k_next = k + (uint64_t)h;  // h_next <= h: inside the drawn window
      if (int e = ctx->ensure_hyperplanes(seed_base, k_next, (uint64_t)h, &st->host_ms)) return e;
      const int ne = e0 == 0 ? 6 : 0;
      if (rec) KLSH_HIP(hipEventRecord(ctx->ev[ne], s));
      klsh::launch_project_device_n(ctx->rows, next_order, spec_out, (uint32_t)n,
                                    ctx->hyperplane_ptr(k_next), ctx->n_next_dev, s, ktime(j + 1),
                                    nullptr, &ctx->pw);
      KLSH_HIP(hipGetLastError());
      if (rec) KLSH_HIP(hipEventRecord(ctx->ev[ne + 1], s));
      ctx->spec_pending = true;
      ctx->spec_swap = spec_out == ctx->keys2;
      ctx->spec_k = k_next;
      ctx->spec_ev = ne;
      return 0;
    };
    if (int e = merge_and_compact(ctx, fk, fv, (uint32_t)n, threshold, bucket_size_threshold,
                                  seed_base, rng_counter, st, ctx->phase_timing,
                                  ahead ? &queue_next : nullptr, ktime(j)))
      return e;
    if (ctx->spec_pending && *rng_counter != ctx->spec_k) {  // nested ran: recomputed next time
      ctx->spec_pending = false;
      ctx->spec_swap = false;
      // the discarded launch stamped the next iteration's projection lines: clear them, or the
      // recomputed projection's span would start at the discarded one (across the nested work)
      if (ctx->kernel_timing && ctx->kstamp) {
        klsh::KStampSet* set = &ctx->kstamp->set[ctx->kt_iter & 1u];
        KLSH_HIP(hipMemsetAsync(&set->t0[klsh::KC_PROJECT][0], 0xFF,
                                sizeof(set->t0[klsh::KC_PROJECT]), s));
        KLSH_HIP(hipMemsetAsync(&set->t1[klsh::KC_PROJECT][0], 0,
                                sizeof(set->t1[klsh::KC_PROJECT]), s));
      }
    }
    if (rec) {
      st->project_ms += elapsed(ctx->ev[e0], ctx->ev[e0 + 1]);
      st->project_timed_launches += 1;
    }
    if (rec && ctx->phase_timing) st->sort_ms += elapsed(ctx->ev[1], ctx->ev[5]);
    st->project_launches += 1;
    st->sum_rows += n;
    st->sum_proj_bits += n * (uint64_t)h;
    st->sum_merges += n - ctx->n_live;
    threshold -= sim_step;
    if (iter_log)  // (diagnostics build)
      fprintf(iter_log, "%d %llu %d %.4f %.4f %u %u %u %u\n", it, (unsigned long long)n, h,
              now_ms() - t_it, ctx->t_enqueued - t_it, ctx->h_ctr->n_big[0], ctx->h_ctr->n_big[1],
              ctx->h_ctr->n_big[2] + ctx->h_ctr->n_big[3], ctx->h_ctr->n_huge);
  }
  if (iter_log) fflush(iter_log);
  if (ctx->kernel_timing && ctx->kstamp && st && ctx->kt_iter > kt_first)  // per-class spans
    if (int e = collect_kernel_times(ctx, (int)((ctx->kt_iter - 1) & 1u), st)) return e;
  return 0;
}

// ============================================================ sharded loop ===
// Every rank holds a replica of the rows; the canonical order of iteration t is the concatenation
// over ranks of each rank's survivors ("mine").  Per iteration:
//   project mine -> keys; bin histogram (top <= 12 key bits) -> allgather -> every rank derives
//   the same bin -> rank ownership (contiguous key ranges balanced by rows) and send counts;
//   stable partition of (key, slot) by owner -> all-to-all-v -> received pairs are in canonical
//   order restricted to this rank's key range; stable radix sort by key = merge_hashtable's
//   bucket order for those keys; greedy merge + compaction -> the new "mine"; the survivors a
//   merge rewrote are broadcast (allgather-v of rows + metadata) so every replica stays identical.
// Oversize buckets (nestedCluster) draw hyperplanes in ascending bucket order, i.e. rank order
// then local order: a small allgather of (runs, hyperplanes) gives each rank its RNG offset.
// Member links are written only by the rank that merged them; the end of the call combines them
// with an element-wise min (an unwritten link is kNil = 0xFFFFFFFF) and gathers the global order.
static int cluster_sharded_body(klsh_ctx* ctx, float min_similarity, int iterations,
                                int run_iters, int bucket_size_threshold, uint32_t seed_base,
                                uint64_t* rng_counter, uint64_t* nt_trace, klsh_stats* st) {
  klsh::Comm* cm = ctx->comm;
  const int W = cm->world, g = cm->rank;
  hipStream_t s = ctx->stream;
  if (int e = ctx->reserve_shard()) return e;
  auto comm_fail = [&](const char* what) {
    return fail(KLSH_E_HIP, std::string(what) + ": " + cm->err);
  };
  const double t_start = now_ms();
  double t_comm = 0.0;
  auto timed_comm = [&](auto fn) {
    const double t0 = now_ms();
    const int rc = fn();
    t_comm += now_ms() - t0;
    return rc;
  };

  const float max_similarity = 0.95f;  // cluster.cc:190-192 (all float)
  const float sim_step = (max_similarity - min_similarity) / (float)iterations;
  float threshold = max_similarity;

  // my block of the global canonical order
  uint64_t N = ctx->n_live;
  uint32_t n_g = 0;
  {
    const uint64_t lo = N * (uint64_t)g / (uint64_t)W, hi = N * (uint64_t)(g + 1) / (uint64_t)W;
    n_g = (uint32_t)(hi - lo);
    if (n_g) KLSH_HIP(hipMemcpyAsync(ctx->alt, ctx->order + lo, 4ull * n_g, hipMemcpyDeviceToDevice, s));
    std::swap(ctx->order, ctx->alt);
  }
  std::vector<uint32_t> n_all(W, 0);  // survivors per rank after the last exchange
  for (int r = 0; r < W; ++r)
    n_all[r] = (uint32_t)(N * (uint64_t)(r + 1) / W - N * (uint64_t)r / W);

  ctx->w_count = 0;
  if (N > 0 && iterations > 0) {
    if (int e = ctx->predraw_hyperplanes(seed_base, *rng_counter, (uint64_t)floor_log2(N),
                                         iterations, &st->host_ms))
      return e;
  }
  const int R = klsh::delta_words(ctx->dp);
  std::vector<size_t> scnt(W), soff(W), rcnt(W), roff(W), dcnt(W), doff(W);

  bool replicated = false;
  for (int it = 0; it < run_iters; ++it) {
    if (N < ctx->shard_min_rows) {  // the replicated tail: every rank runs the rest on its own
      std::vector<size_t> cnt(W), off(W);
      size_t acc = 0;
      for (int r = 0; r < W; ++r) {
        cnt[r] = 4ull * n_all[r];
        off[r] = acc;
        acc += cnt[r];
      }
      if (timed_comm([&] { return cm->allgatherv(ctx->order, ctx->alt, cnt.data(), off.data(), s); }))
        return comm_fail("order allgather");
      std::swap(ctx->order, ctx->alt);
      ctx->n_live = N;
      replicated = true;
      if (int e = run_single(ctx, threshold, sim_step, it, run_iters, bucket_size_threshold,
                             seed_base, rng_counter, nt_trace, st))
        return e;
      N = ctx->n_live;
      break;
    }
    if (nt_trace) nt_trace[it] = N;
    st->iterations += 1;
    ctx->tick(it);
    if (N == 0) {
      threshold -= sim_step;
      continue;
    }
    const int h = floor_log2(N);
    const uint64_t k = *rng_counter;
    *rng_counter += (uint64_t)h;
    st->hyperplanes += (uint64_t)h;
    if (int e = ctx->ensure_hyperplanes(seed_base, k, (uint64_t)h, &st->host_ms)) return e;

    // 1. keys of my rows, key-range ownership, send counts
    if (!ctx->ctr_clean) if (int e = ctx->reset_counters()) return e;
    ctx->ctr_clean = false;
    // (HIP events around the projection only with hip_events / phase_timing: a record is a
    // marker packet the stream waits on, ~9 us per iteration)
    const bool rec = ctx->hip_events || ctx->phase_timing;
    if (rec) KLSH_HIP(hipEventRecord(ctx->ev[0], s));
    klsh::launch_project(ctx->rows, ctx->order, ctx->keys, n_g, ctx->hyperplane_ptr(k), h, 0u, s,
                         &ctx->pw);
    KLSH_HIP(hipGetLastError());
    if (rec) KLSH_HIP(hipEventRecord(ctx->ev[1], s));
    const int B = std::min(h, klsh::kMaxBinBits);
    const int shift = h - B;
    const uint32_t nbins = 1u << B;
    klsh::launch_bin_hist(ctx->keys, n_g, shift, nbins, ctx->bins, s);
    if (timed_comm([&] { return cm->allgather(ctx->bins, ctx->bins_all, 4ull * nbins, s); }))
      return comm_fail("bin histogram allgather");
    klsh::launch_bin_split(ctx->bins_all, W, nbins, N, ctx->owner, ctx->cntmat, s);
    // the send counts to the host through mapped memory (k_publish_words): no copy, no event
    const uint32_t seq_counts = ++ctx->shp_seq;
    klsh::launch_publish_words(ctx->cntmat, (uint32_t)(W * W), nullptr, 0u, ctx->shp_dev + 16,
                               ctx->shp_dev, seq_counts, s);
    // 2a. the stable partition by owner needs only the device's ownership map: it is queued
    //     before the host waits (for the counts only, not for it), so it runs during the round trip
    if (klsh::launch_partition(ctx->keys, ctx->order, n_g, shift, ctx->owner, W, ctx->nk1,
                               ctx->tile_sums, ctx->ctr, ctx->sbuf, s))
      return fail(KLSH_E_ARG, "partition: unsupported world size");
    KLSH_HIP(hipGetLastError());
    if (timed_comm([&] { return cm->wait_flag(ctx->shp_host, seq_counts, s); }))
      return comm_fail("send counts");
    std::atomic_thread_fence(std::memory_order_acquire);
    memcpy(ctx->h_small, ctx->shp_host + 16, 4ull * W * W);
    uint32_t m_g = 0;
    for (int r = 0; r < W; ++r) {
      scnt[r] = 8ull * ctx->h_small[g * W + r];
      rcnt[r] = 8ull * ctx->h_small[r * W + g];
      soff[r] = r ? soff[r - 1] + scnt[r - 1] : 0;
      roff[r] = r ? roff[r - 1] + rcnt[r - 1] : 0;
      m_g += ctx->h_small[r * W + g];
    }

    // 2b. exchange the partitioned (key, slot) pairs: all-to-all-v
    if (timed_comm([&] {
          return cm->alltoallv(ctx->sbuf, scnt.data(), soff.data(), ctx->rbuf, rcnt.data(),
                               roff.data(), s);
        }))
      return comm_fail("pair all-to-all");
    klsh::launch_unpack_pairs(ctx->rbuf, m_g, ctx->keys, ctx->alt, s);
    if (ctx->phase_timing) KLSH_HIP(hipEventRecord(ctx->ev[6], s));

    // 3. bucket order of my key range, merge, compaction, delta list
    uint32_t *fk = nullptr, *fv = nullptr;
    klsh::radix_sort(ctx->keys, ctx->alt, ctx->keys2, ctx->order, m_g, h, ctx->hist, &fk, &fv, s);
    KLSH_HIP(hipGetLastError());
    if (ctx->phase_timing) KLSH_HIP(hipEventRecord(ctx->ev[5], s));
    uint32_t* out = (fv == ctx->order) ? ctx->alt : ctx->order;
    ctx->mw.dlist = ctx->dslots;  // the merge kernels list the survivors they rewrite
    ctx->mw.mark = ctx->mark;
    ctx->mw.stamp = ++ctx->stamp;
    const int rc_merge = merge_main(ctx, fk, fv, m_g, threshold, bucket_size_threshold, out, st,
                                    ctx->phase_timing, /*sync=*/false);
    if (rc_merge) {
      ctx->mw.dlist = nullptr;
      return rc_merge;
    }
    // 4. counters of every rank in one exchange and one host sync: oversize runs, survivors,
    //    rewritten rows (n_over, total, n_delta are adjacent in Counters)
    KLSH_HIP(hipMemcpyAsync(ctx->small + 4 * W, &ctx->ctr->n_over, 12, hipMemcpyDeviceToDevice, s));
    if (timed_comm([&] { return cm->allgather(ctx->small + 4 * W, ctx->small, 16, s); }))
      return comm_fail("counter allgather");
    // every rank's counters and this rank's Counters to the host through mapped memory
    static_assert(sizeof(Counters) % 4 == 0, "Counters published as words");
    const uint32_t seq_ctr = ++ctx->shp_seq;
    klsh::launch_publish_words(ctx->small, (uint32_t)(4 * W), reinterpret_cast<const uint32_t*>(ctx->ctr),
                               (uint32_t)(sizeof(Counters) / 4), ctx->shp_dev + 16, ctx->shp_dev,
                               seq_ctr, s);
    if (timed_comm([&] { return cm->wait_flag(ctx->shp_host, seq_ctr, s); })) return comm_fail("counters");
    std::atomic_thread_fence(std::memory_order_acquire);
    memcpy(ctx->h_small, ctx->shp_host + 16, 16ull * W);
    memcpy(ctx->h_ctr, ctx->shp_host + 16 + 4 * W, sizeof(Counters));
    if (int e = ctx->check_device_err()) return e;
    if (ctx->phase_timing && st) {
      st->merge_ms += elapsed(ctx->ev[2], ctx->ev[3]);
      st->compact_ms += elapsed(ctx->ev[3], ctx->ev[4]);
    }
    std::vector<uint32_t> surv(W), ndel(W);
    uint64_t any_over = 0;
    for (int r = 0; r < W; ++r) {
      any_over += ctx->h_small[4 * r];
      surv[r] = ctx->h_small[4 * r + 1];
      ndel[r] = ctx->h_small[4 * r + 2];
    }
    if (any_over) {  // nestedCluster somewhere: RNG offsets need every rank's hyperplane count
      std::vector<uint2> over;
      uint64_t my_hyp = 0;
      if (int e = oversize_runs(ctx, &over, &my_hyp)) return e;
      auto exchange_counters = [&](uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3) -> int {
        uint32_t* hs = ctx->h_small;
        hs[0] = a0; hs[1] = a1; hs[2] = a2; hs[3] = a3;
        KLSH_HIP(hipMemcpyAsync(ctx->small + 4 * W, hs, 16, hipMemcpyHostToDevice, s));
        if (timed_comm([&] { return cm->allgather(ctx->small + 4 * W, ctx->small, 16, s); }))
          return comm_fail("counter allgather");
        KLSH_HIP(hipMemcpyAsync(hs, ctx->small, 16ull * W, hipMemcpyDeviceToHost, s));
        if (timed_comm([&] { return cm->wait(s); })) return comm_fail("counter exchange");
        return 0;
      };
      if (int e = exchange_counters((uint32_t)my_hyp, 0, 0, 0)) return e;
      uint64_t hyp_before = 0, hyp_all = 0;
      for (int r = 0; r < W; ++r) {
        if (r < g) hyp_before += ctx->h_small[4 * r];
        hyp_all += ctx->h_small[4 * r];
      }
      uint64_t rng = *rng_counter + hyp_before;
      if (!over.empty()) {
        const int rc_nested = merge_nested(ctx, fk, fv, m_g, threshold, over, seed_base, &rng, out, st);
        if (rc_nested) {
          ctx->mw.dlist = nullptr;
          return rc_nested;
        }
      }
      *rng_counter += hyp_all;
      if (int e = exchange_counters(ctx->h_ctr->total, ctx->h_ctr->n_delta, 0, 0)) return e;
      for (int r = 0; r < W; ++r) {
        surv[r] = ctx->h_small[4 * r];
        ndel[r] = ctx->h_small[4 * r + 1];
      }
    }
    ctx->mw.dlist = nullptr;

    // 5. merge deltas to every replica
    uint64_t nd_all = 0;
    for (int r = 0; r < W; ++r) {
      dcnt[r] = 4ull * R * ndel[r];
      doff[r] = 4ull * R * nd_all;
      nd_all += ndel[r];
    }
    if (nd_all) {
      if (int e = ctx->reserve_words(&ctx->drec, &ctx->drec_cap, (size_t)R * ndel[g] + 1)) return e;
      if (int e = ctx->reserve_words(&ctx->drec_all, &ctx->drec_all_cap, (size_t)R * nd_all)) return e;
      klsh::launch_delta_pack(ctx->rows, ctx->dslots, ndel[g], ctx->drec, s);
      if (timed_comm([&] {
            return cm->allgatherv(ctx->drec, ctx->drec_all, dcnt.data(), doff.data(), s);
          }))
        return comm_fail("delta allgather");
      klsh::launch_delta_apply(ctx->rows, ctx->drec_all, (uint32_t)nd_all, s);
      KLSH_HIP(hipGetLastError());
    }

    if (out == ctx->alt) std::swap(ctx->order, ctx->alt);
    const uint64_t N_next = std::accumulate(surv.begin(), surv.end(), (uint64_t)0);
    if (rec) {
      st->project_ms += elapsed(ctx->ev[0], ctx->ev[1]);
      st->project_timed_launches += 1;
    }
    if (ctx->phase_timing) st->sort_ms += elapsed(ctx->ev[6], ctx->ev[5]);
    st->project_launches += 1;
    st->sum_rows += N;
    st->sum_proj_bits += N * (uint64_t)h;
    st->sum_merges += N - N_next;
    N = N_next;
    n_g = surv[g];
    n_all = surv;
    threshold -= sim_step;
  }

  // global canonical order on every rank, combined member links
  if (!replicated) {
    std::vector<size_t> cnt(W), off(W);
    size_t acc = 0;
    for (int r = 0; r < W; ++r) {
      cnt[r] = 4ull * n_all[r];
      off[r] = acc;
      acc += cnt[r];
    }
    if (timed_comm([&] { return cm->allgatherv(ctx->order, ctx->alt, cnt.data(), off.data(), s); }))
      return comm_fail("order allgather");
    std::swap(ctx->order, ctx->alt);
  }
  if (timed_comm([&] { return cm->allreduce_min_u32(ctx->rows.nxt, ctx->members, s); }))
    return comm_fail("member link allreduce");
  if (timed_comm([&] { return cm->wait(s); })) return comm_fail("member link allreduce");
  ctx->n_live = N;
  st->n_final = N;
  st->comm_ms = t_comm;
  st->wall_ms = now_ms() - t_start;
  return 0;
}

// A rank that fails mid-call aborts the group, so the other ranks' pending and next collectives
// fail too instead of waiting for it forever; the context's group is unusable afterwards.
static int cluster_sharded(klsh_ctx* ctx, float min_similarity, int iterations, int run_iters,
                           int bucket_size_threshold, uint32_t seed_base, uint64_t* rng_counter,
                           uint64_t* nt_trace, klsh_stats* st) {
  if (ctx->comm->aborted) return fail(KLSH_E_STATE, "communicator aborted by an earlier failure");
  const int rc = cluster_sharded_body(ctx, min_similarity, iterations, run_iters,
                                      bucket_size_threshold, seed_base, rng_counter, nt_trace, st);
  if (rc) {
    const std::string msg = g_err;
    ctx->comm->abort();
    ctx->mw.dlist = nullptr;
    g_err = msg;
  }
  return rc;
}

int klsh_cluster(klsh_ctx* ctx, float min_similarity, int iterations, int bucket_size_threshold,
                 uint32_t seed_base, uint64_t* rng_counter, uint64_t* nt_trace, klsh_stats* stats) {
  if (!ctx || !rng_counter) return fail(KLSH_E_ARG, "null argument");
  if (!ctx->loaded) {
    if (ctx->comm) ctx->comm->abort();  // the other ranks must not wait for this one
    return fail(KLSH_E_STATE, "klsh_cluster before a load");
  }
  KLSH_HIP(hipSetDevice(ctx->device));
  if (stats && stats->struct_size != sizeof(klsh_stats))
    return fail(KLSH_E_ARG, "klsh_stats.struct_size != sizeof(klsh_stats): built against another "
                            "klsh.h (KLSH_ABI_VERSION " + std::to_string(KLSH_ABI_VERSION) + ")");
  klsh_stats local{};
  klsh_stats* st = stats ? stats : &local;
  memset(st, 0, sizeof(*st));
  st->struct_size = sizeof(*st);
  st->world = (uint64_t)ctx->world();
  ctx->mw.huge_cap = 0;  // (set per iteration from the run counts by the single-device loop)
  ctx->mw.huge_fold = ctx->huge_fold_always ? 1u : 0u;
  ctx->huge_quiet = 0;
  ctx->mw.dlist = nullptr;
  const int run_iters = ctx->stop_after > 0 ? std::min(iterations, ctx->stop_after) : iterations;
  if (ctx->comm)  // any bound group, world 1 included (measures the sharded machinery alone)
    return cluster_sharded(ctx, min_similarity, iterations, run_iters, bucket_size_threshold,
                           seed_base, rng_counter, nt_trace, st);
  const double t_start = now_ms();

  // cluster.cc:190-192 (all float)
  const float max_similarity = 0.95f;
  const float sim_step = (max_similarity - min_similarity) / (float)iterations;
  float threshold = max_similarity;

  ctx->ctr_clean = false;
  ctx->spec_pending = false;
  ctx->spec_swap = false;
  // no run counts yet: only very large inputs start with the 385..896-row class on aux 2
  ctx->mw.big896_aux = ctx->n_live >= (1u << 24) ? 1u : 0u;
  // Every call draws its hyperplanes afresh (the reference draws them inside Cluster(),
  // lshash.cc:36-42), so repeated timed calls never reuse a previous call's tables.
  ctx->w_count = 0;
  // Pre-draw the hyperplanes this call can need without nested buckets (h_t is non-increasing),
  // up to a bounded window; later ones are drawn when reached.
  if (ctx->n_live > 0 && iterations > 0) {
    if (int e = ctx->predraw_hyperplanes(seed_base, *rng_counter,
                                         (uint64_t)floor_log2(ctx->n_live), iterations,
                                         &st->host_ms))
      return e;
  }

  if (int e = run_single(ctx, threshold, sim_step, 0, run_iters, bucket_size_threshold, seed_base,
                         rng_counter, nt_trace, st))
    return e;
  // The survivor counters are published by the compaction's last workgroup, which need not be
  // the last to finish writing ctx->order: drain the stream before klsh_count/klsh_result read it.
  KLSH_HIP(hipStreamSynchronize(ctx->stream));
  if (ctx->pw.ws) {  // pairs the certified projection screens left to the exact chains
    // ws[4..6): the wide-row fix-up kernel's total; ws[32..64): the fp16 screen's 16 counters
    uint32_t w[64];
    KLSH_HIP(hipMemcpy(w, ctx->pw.ws, sizeof(w), hipMemcpyDeviceToHost));
    unsigned long long fixed = 0, part = 0;
    for (int i : {4, 32, 34, 36, 38, 40, 42, 44, 46, 48, 50, 52, 54, 56, 58, 60, 62}) {
      memcpy(&part, w + i, sizeof(part));
      fixed += part;
    }
    KLSH_HIP(hipMemset(ctx->pw.ws + 4, 0, 8));
    KLSH_HIP(hipMemset(ctx->pw.ws + 32, 0, 128));
    st->proj_fix_pairs = fixed;
  }
  st->n_final = ctx->n_live;
  st->wall_ms = now_ms() - t_start;
#ifdef KLSH_MERGE_PROF
  if (getenv("KLSH_MERGE_PROF")) klsh::merge_prof_dump(stderr);
#endif
  return 0;
}

int klsh_comm_unique_id(uint8_t* id) {
  if (!id) return fail(KLSH_E_ARG, "null argument");
  std::string err;
  if (klsh::rccl_unique_id(id, &err)) return fail(KLSH_E_HIP, err);
  return 0;
}

int klsh_comm_init(klsh_ctx* ctx, int rank, int world, const uint8_t* id) {
  if (!ctx || !id || world < 1 || rank < 0 || rank >= world || world > klsh::kMaxRanks)
    return fail(KLSH_E_ARG, "bad argument");
  KLSH_HIP(hipSetDevice(ctx->device));
  std::string err;
  klsh::Comm* c = klsh::make_rccl_comm(rank, world, id, ctx->device, &err);
  if (!c) return fail(KLSH_E_HIP, err);
  c->timeout_s = ctx->comm_timeout_s;
  ctx->release_shard();
  delete ctx->comm;
  ctx->comm = c;
  return 0;
}

int klsh_comm_init_local(klsh_ctx** ctxs, int world) {
  if (!ctxs || world < 1 || world > klsh::kMaxRanks) return fail(KLSH_E_ARG, "bad argument");
  for (int r = 0; r < world; ++r)
    if (!ctxs[r]) return fail(KLSH_E_ARG, "null context");
  std::vector<klsh::Comm*> cs(world);
  klsh::make_local_comms(world, cs.data());
  for (int r = 0; r < world; ++r) {
    ctxs[r]->release_shard();
    delete ctxs[r]->comm;
    ctxs[r]->comm = cs[r];
  }
  return 0;
}

// Options (include/klsh.h).  Results never depend on them, except that "stop_after" stops early.
int klsh_set_option(klsh_ctx* ctx, const char* name, int64_t value) {
  if (!ctx || !name) return fail(KLSH_E_ARG, "null argument");
  const std::string n(name);
  auto flag = [&](bool* f) {
    *f = value != 0;
    return 0;
  };
  // launch sizes (0 = the default): unsigned 32-bit, bounded so no grid overflows
  auto grid = [&](uint32_t* g) {
    if (value < 0 || value > (1 << 20)) return fail(KLSH_E_ARG, n + " must be in [0, 2^20]");
    *g = (uint32_t)value;
    return 0;
  };
  if (n == "shard_min_rows") {
    if (value < 0) return fail(KLSH_E_ARG, "shard_min_rows must be >= 0");
    ctx->shard_min_rows = (uint64_t)value;
    return 0;
  }
  if (n == "phase_timing") return flag(&ctx->phase_timing);
  if (n == "kernel_timing") return flag(&ctx->kernel_timing);
  if (n == "tail_batch") return flag(&ctx->tail_batch);
  if (n == "huge_fold") return flag(&ctx->huge_fold_always);
  if (n == "tail_local") return flag(&ctx->tail_local);
  if (n == "hyperplane_async") {
    if (value != 0 && value != 1) return fail(KLSH_E_ARG, "hyperplane_async must be 0 or 1");
    ctx->hyperplane_async = (uint32_t)value;
    return 0;
  }
  if (n == "hyperplane_window") {
    if (value < 0) return fail(KLSH_E_ARG, "hyperplane_window must be >= 0");
    ctx->hyperplane_window = (uint64_t)value;
    return 0;
  }
  if (n == "progress") {
    if (value < 0 || value > INT32_MAX) return fail(KLSH_E_ARG, "progress must be >= 0");
    ctx->progress = (int)value;
    return 0;
  }
  if (n == "stop_after") {
    if (value < 0 || value > INT32_MAX) return fail(KLSH_E_ARG, "stop_after must be in [0, 2^31)");
    ctx->stop_after = (int)value;
    return 0;
  }
  if (n == "projection") {
    if (value != klsh::kProjAuto && value != klsh::kProjPacked)
      return fail(KLSH_E_ARG, "projection must be 0 (default) or 1 (exact packed chains)");
    KLSH_HIP(hipSetDevice(ctx->device));
    ctx->pw.variant = (uint32_t)value;
    return ctx->apply_projection_variant();
  }
  if (n == "wide_gram") {
    if (value != 0 && value != 8 && value != 16 && value != 32 && value != 64)
      return fail(KLSH_E_ARG, "wide_gram must be 0, 8, 16, 32 or 64");
    ctx->mw.wide_gram = (uint32_t)value;
    return 0;
  }
  if (n == "wide_unrolled") {
    if (value != 0 && value != 1) return fail(KLSH_E_ARG, "wide_unrolled must be 0 or 1");
    ctx->pw.wide_rolled = value ? 0u : 1u;
    return 0;
  }
  if (n == "long_runs") {
    if (value != 0 && value != 1 && value != 4) return fail(KLSH_E_ARG, "long_runs must be 0, 1 or 4");
    ctx->mw.long_off = value == 1 ? 0u : value == 0 ? 1u : 4u;
    KLSH_HIP(hipSetDevice(ctx->device));
    return ctx->cap_slots ? ctx->ensure_long(ctx->cap_slots, ctx->d) : 0;
  }
  if (n == "comm_timeout_s") {
    if (value <= 0) return fail(KLSH_E_ARG, "comm_timeout_s must be > 0");
    ctx->comm_timeout_s = (double)value;
    if (ctx->comm) ctx->comm->timeout_s = (double)value;
    return 0;
  }
  if (n == "h16_grid") return grid(&ctx->pw.h16_grid);
  if (n == "h16_segcap") return grid(&ctx->pw.segcap);
  if (n == "wide_grid") return grid(&ctx->pw.wide_grid);
  if (n == "fix_grid") return grid(&ctx->pw.fix_grid);
  if (n == "small_grid") return grid(&ctx->mw.small_grid);
  if (n == "tail_big_groups") return grid(&ctx->mw.tail_nbig);
  if (n == "tail_small_groups") return grid(&ctx->mw.tail_nsmall);
  if (n == "wide_group_grid") return grid(&ctx->mw.wide_group_grid);
  if (n == "small_screen_grid") return grid(&ctx->mw.screen_grid);
  if (n == "tail_merge_rows") {
    // capped at the largest size the one-launch merge's parity is pinned at (2^22: C2's
    // iterations of 2^21..2^22 positions, test_mid_local_sort's 2.6M rows); above it, runs over
    // 896 rows at d = 16 / 32 would walk in huge_runs instead of k_merge_long, which no test covers
    if (value < 0 || value > (1 << 22)) return fail(KLSH_E_ARG, "tail_merge_rows must be in [0, 2^22]");
    ctx->mw.tail_max = (uint32_t)value;
    return 0;
  }
  if (n == "tail_screen") {
    if (value != 0 && value != 1) return fail(KLSH_E_ARG, "tail_screen must be 0 or 1");
    ctx->mw.tail_screen = (uint32_t)value;
    return 0;
  }
  if (n == "tail_screen_grid") return grid(&ctx->mw.tail_screen_grid);
  if (n == "tail_big_screen") {
    if (value != 0 && value != 1) return fail(KLSH_E_ARG, "tail_big_screen must be 0 or 1");
    ctx->mw.tail_big_screen = (uint32_t)value;
    return 0;
  }
  if (n == "hip_events") {
    if (value != 0 && value != 1) return fail(KLSH_E_ARG, "hip_events must be 0 or 1");
    ctx->hip_events = value != 0;
    return 0;
  }
  if (n == "small_screen") {
    if (value != 0 && value != 1) return fail(KLSH_E_ARG, "small_screen must be 0 or 1");
    ctx->mw.small_screen = (uint32_t)value;
    return 0;
  }
  return fail(KLSH_E_ARG, "unknown option " + n);
}

int klsh_get_option(klsh_ctx* ctx, const char* name, int64_t* value) {
  if (!ctx || !name || !value) return fail(KLSH_E_ARG, "null argument");
  const std::string n(name);
  if (n == "shard_min_rows") *value = (int64_t)ctx->shard_min_rows;
  else if (n == "phase_timing") *value = ctx->phase_timing;
  else if (n == "kernel_timing") *value = ctx->kernel_timing;
  else if (n == "tail_batch") *value = ctx->tail_batch;
  else if (n == "huge_fold") *value = ctx->huge_fold_always;
  else if (n == "tail_local") *value = ctx->tail_local;
  else if (n == "hyperplane_window") *value = (int64_t)ctx->hyperplane_window;
  else if (n == "hyperplane_async") *value = ctx->hyperplane_async;
  else if (n == "stop_after") *value = ctx->stop_after;
  else if (n == "progress") *value = ctx->progress;
  else if (n == "projection") *value = ctx->pw.variant;
  else if (n == "comm_timeout_s") *value = (int64_t)ctx->comm_timeout_s;
  else if (n == "h16_grid") *value = ctx->pw.h16_grid;
  else if (n == "h16_segcap") *value = ctx->pw.segcap;
  else if (n == "wide_grid") *value = ctx->pw.wide_grid;
  else if (n == "fix_grid") *value = ctx->pw.fix_grid;
  else if (n == "small_grid") *value = ctx->mw.small_grid;
  else if (n == "tail_big_groups") *value = ctx->mw.tail_nbig;
  else if (n == "tail_small_groups") *value = ctx->mw.tail_nsmall;
  else if (n == "wide_group_grid") *value = ctx->mw.wide_group_grid;
  else if (n == "small_screen_grid") *value = ctx->mw.screen_grid;
  else if (n == "tail_merge_rows") *value = klsh::tail_merge_max(ctx->mw);
  else if (n == "small_screen") *value = ctx->mw.small_screen;
  else if (n == "hip_events") *value = ctx->hip_events ? 1 : 0;
  else if (n == "tail_screen") *value = ctx->mw.tail_screen;
  else if (n == "tail_screen_grid") *value = ctx->mw.tail_screen_grid;
  else if (n == "tail_big_screen") *value = ctx->mw.tail_big_screen;
  else if (n == "long_runs") *value = ctx->mw.long_off == 1u ? 0 : ctx->mw.long_off == 0u ? 1 : ctx->mw.long_off;
  else if (n == "wide_gram") *value = ctx->mw.wide_gram;
  else if (n == "wide_unrolled") *value = ctx->pw.wide_rolled ? 0 : 1;
  else if (n == "fp16_image") *value = ctx->rows.xh != nullptr;
  else if (n == "last_hash_kernel") *value = ctx->last_hash_kernel;
  else if (n == "last_hash_close_pairs") *value = (int64_t)ctx->last_hash_close;
  else return fail(KLSH_E_ARG, "unknown option " + n);
  return 0;
}

int klsh_comm_info(klsh_ctx* ctx, int* rank, int* world) {
  if (!ctx) return fail(KLSH_E_ARG, "null ctx");
  if (rank) *rank = ctx->rank();
  if (world) *world = ctx->world();
  return 0;
}

int klsh_count(klsh_ctx* ctx, uint64_t* n_rows, uint64_t* n_members) {
  if (!ctx) return fail(KLSH_E_ARG, "null ctx");
  if (!ctx->loaded) return fail(KLSH_E_STATE, "nothing loaded");
  if (n_rows) *n_rows = ctx->n_live;
  if (n_members) {
    KLSH_HIP(hipSetDevice(ctx->device));
    // members of live rows = sum of cnt over the live slots
    std::vector<uint32_t> ord(ctx->n_live), cnt(ctx->slots);
    if (ctx->n_live)
      KLSH_HIP(hipMemcpy(ord.data(), ctx->order, 4 * ctx->n_live, hipMemcpyDeviceToHost));
    if (ctx->slots)
      KLSH_HIP(hipMemcpy(cnt.data(), ctx->rows.cnt, 4 * ctx->slots, hipMemcpyDeviceToHost));
    uint64_t m = 0;
    for (uint32_t sl : ord) m += cnt[sl];
    *n_members = m;
  }
  return 0;
}

int klsh_result(klsh_ctx* ctx, float* rows, uint64_t* member_offsets, uint64_t* member_ids) {
  if (!ctx) return fail(KLSH_E_ARG, "null ctx");
  if (!ctx->loaded) return fail(KLSH_E_STATE, "nothing loaded");
  KLSH_HIP(hipSetDevice(ctx->device));
  const uint64_t n = ctx->n_live;
  hipStream_t s = ctx->stream;
  if (rows && n) {
    float* tmp = nullptr;
    if (int e = dalloc(&tmp, n * (uint64_t)ctx->d)) return e;
    klsh::launch_gather_rows(ctx->rows, ctx->order, (uint32_t)n, tmp, s);
    hipError_t e1 = hipMemcpyAsync(rows, tmp, sizeof(float) * n * ctx->d, hipMemcpyDeviceToHost, s);
    hipError_t e2 = hipStreamSynchronize(s);
    dfree(tmp);
    if (e1 != hipSuccess || e2 != hipSuccess) return fail(KLSH_E_HIP, "result rows copy");
  }
  if (member_offsets || member_ids) {
    std::vector<uint32_t> ord(n), head(ctx->slots), nxt(ctx->members);
    if (n) KLSH_HIP(hipMemcpy(ord.data(), ctx->order, 4 * n, hipMemcpyDeviceToHost));
    if (ctx->slots)
      KLSH_HIP(hipMemcpy(head.data(), ctx->rows.head, 4 * ctx->slots, hipMemcpyDeviceToHost));
    if (ctx->members)
      KLSH_HIP(hipMemcpy(nxt.data(), ctx->rows.nxt, 4 * ctx->members, hipMemcpyDeviceToHost));
    uint64_t m = 0;
    for (uint64_t i = 0; i < n; ++i) {
      if (member_offsets) member_offsets[i] = m;
      if (ord[i] >= ctx->slots) return fail(KLSH_E_STATE, "corrupt live order");
      for (uint32_t node = head[ord[i]]; node != klsh::kNil; node = nxt[node]) {
        // every member belongs to exactly one live row: a longer walk is a broken list
        if (node >= ctx->members || m >= ctx->members)
          return fail(KLSH_E_STATE, "corrupt member list");
        if (member_ids) member_ids[m] = ctx->ids[node];
        ++m;
      }
    }
    if (member_offsets) member_offsets[n] = m;
  }
  return 0;
}

// The projection kernels the loop uses, on caller rows: the same dispatch (launch_project) with
// the context's projection options, the fp16 row image built from the rows where the loop keeps
// one (d = 16, 32, 64), so the certified screens and their exact fix-up paths are what a test of
// this entry point exercises.
int klsh_hash_keys(klsh_ctx* ctx, const float* rows, uint64_t n, int d, const float* table, int h,
                   uint32_t* keys) {
  if (!ctx || (!rows && n) || (!keys && n) || (!table && h > 0)) return fail(KLSH_E_ARG, "null argument");
  if (d <= 0 || d > 4096 || h < 0 || h > 31) return fail(KLSH_E_RANGE, "d or h out of range");
  if (n >= 0xFFFFFFF0ull) return fail(KLSH_E_RANGE, "rows >= 2^32");
  ctx->last_hash_kernel = klsh::kPkNone;
  ctx->last_hash_close = 0;
  if (n == 0) return 0;
  KLSH_HIP(hipSetDevice(ctx->device));
  const int dp = (d + 3) & ~3;
  Rows r{};
  r.d = d;
  r.dp = dp;
  uint32_t *slots = nullptr, *dkeys = nullptr;
  float* W = nullptr;
  uint16_t* xh = nullptr;
  klsh::ProjectWork pw = ctx->pw;  // the context's launch options, fresh workspaces
  pw.fix = nullptr;
  pw.ws = nullptr;
  auto release = [&] {
    dfree(r.x); dfree(slots); dfree(dkeys); dfree(W); dfree(pw.fix); dfree(pw.ws); dfree(xh);
  };
  int e = 0;
  const bool image = ctx->shadow_wanted(d);
  if ((e = dalloc(&r.x, n * dp)) || (e = dalloc(&slots, n)) || (e = dalloc(&dkeys, n)) ||
      (e = dalloc(&W, (uint64_t)std::max(h, 1) * dp)) || (e = dalloc(&pw.fix, n)) ||
      (e = dalloc(&pw.ws, 64)) || (image && (e = dalloc(&xh, n * dp)))) {
    release();
    return e;
  }
  pw.cap = (uint32_t)n;
  r.xh = xh;
  hipStream_t s = ctx->stream;
  std::vector<uint32_t> iota(n);
  for (uint64_t i = 0; i < n; ++i) iota[i] = (uint32_t)i;
  int rc = 0;
  if (hipMemsetAsync(r.x, 0, sizeof(float) * n * dp, s) != hipSuccess ||
      hipMemcpy2DAsync(r.x, 4 * dp, rows, 4 * d, 4 * d, n, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemsetAsync(W, 0, sizeof(float) * std::max(h, 1) * dp, s) != hipSuccess ||
      hipMemsetAsync(pw.ws, 0, sizeof(uint32_t) * 64, s) != hipSuccess ||
      (h > 0 && hipMemcpy2DAsync(W, 4 * dp, table, 4 * d, 4 * d, h, hipMemcpyHostToDevice, s) !=
                    hipSuccess) ||
      hipMemcpyAsync(slots, iota.data(), 4 * n, hipMemcpyHostToDevice, s) != hipSuccess) {
    rc = fail(KLSH_E_HIP, "upload");
  } else {
    if (image) klsh::launch_shadow_build(r, n, s);
    const int kern = klsh::launch_project(r, slots, dkeys, (uint32_t)n, W, h, 0u, s, &pw);
    uint32_t w[64];
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(keys, dkeys, 4 * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(w, pw.ws, sizeof(w), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
      rc = fail(KLSH_E_HIP, "projection");
    } else {
      // close calls: ws[4..6) the wide-row fix-up total, ws[32..64) the fp16 screen's counters
      unsigned long long fixed = 0, part = 0;
      for (int i : {4, 32, 34, 36, 38, 40, 42, 44, 46, 48, 50, 52, 54, 56, 58, 60, 62}) {
        memcpy(&part, w + i, sizeof(part));
        fixed += part;
      }
      ctx->last_hash_kernel = kern;
      ctx->last_hash_close = fixed;
    }
  }
  (void)hipStreamSynchronize(s);
  release();
  return rc;
}

int klsh_bucket_sort(klsh_ctx* ctx, const uint32_t* keys, uint64_t n, int bits,
                     uint32_t* sorted_keys, uint32_t* perm) {
  if (!ctx || (n && (!keys || !sorted_keys || !perm))) return fail(KLSH_E_ARG, "null argument");
  if (bits < 0 || bits > 32) return fail(KLSH_E_RANGE, "bits out of range");
  if (n >= 0xFFFFFFF0ull) return fail(KLSH_E_RANGE, "keys >= 2^32");
  if (n == 0) return 0;
  KLSH_HIP(hipSetDevice(ctx->device));
  uint32_t *k0 = nullptr, *v0 = nullptr, *k1 = nullptr, *v1 = nullptr, *ws = nullptr, *ts = nullptr;
  Counters* ctr = nullptr;
  const uint64_t ts_words = klsh::scan_ws_words(n);
  int e = 0;
  auto release = [&] {
    dfree(k0); dfree(v0); dfree(k1); dfree(v1); dfree(ws); dfree(ts); dfree(ctr);
  };
  if ((e = dalloc(&k0, n)) || (e = dalloc(&v0, n)) || (e = dalloc(&k1, n)) || (e = dalloc(&v1, n)) ||
      (e = dalloc(&ws, klsh::sort_ws_words(n))) || (e = dalloc(&ts, ts_words)) ||
      (e = dalloc(&ctr, 1))) {
    release();
    return e;
  }
  hipStream_t s = ctx->stream;
  std::vector<uint32_t> iota(n);
  for (uint64_t i = 0; i < n; ++i) iota[i] = (uint32_t)i;
  Counters hc{};
  int rc = 0;
  uint32_t *ok = nullptr, *ov = nullptr;
  if (hipMemsetAsync(ws, 0, sizeof(uint32_t) * klsh::sort_ws_words(n), s) != hipSuccess ||
      hipMemsetAsync(ts, 0, sizeof(uint32_t) * ts_words, s) != hipSuccess ||
      hipMemsetAsync(ctr, 0, sizeof(Counters), s) != hipSuccess ||
      hipMemcpyAsync(k0, keys, 4 * n, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(v0, iota.data(), 4 * n, hipMemcpyHostToDevice, s) != hipSuccess) {
    rc = fail(KLSH_E_HIP, "upload");
  } else {
    klsh::radix_sort(k0, v0, k1, v1, (uint32_t)n, bits, ws, &ok, &ov, s);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(sorted_keys, ok, 4 * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(perm, ov, 4 * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(&hc, ctr, sizeof(Counters), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      rc = fail(KLSH_E_HIP, "sort");
    else if (hc.err)
      rc = fail(KLSH_E_HIP, "device protocol failure in the sort");
  }
  (void)hipStreamSynchronize(s);
  release();
  return rc;
}

// The run finding of merge_main alone on caller keys (a test hook): every run of 2+ equal keys
// of n sorted keys with its list, in start order.
int klsh_bucket_runs(klsh_ctx* ctx, const uint32_t* sorted_keys, uint64_t n, int bucket_thr,
                     uint64_t* n_runs, uint32_t* starts, uint32_t* lengths, int32_t* lists) {
  if (!ctx || !n_runs || (n && !sorted_keys)) return fail(KLSH_E_ARG, "null argument");
  if (n >= 0xFFFFFFF0ull) return fail(KLSH_E_RANGE, "keys >= 2^32");
  const uint64_t cap = *n_runs;
  *n_runs = 0;
  if (n == 0) return 0;
  KLSH_HIP(hipSetDevice(ctx->device));
  using klsh::kBigClasses;
  using klsh::kGroupClasses;
  klsh::MergeWork w{};
  uint32_t* dk = nullptr;
  klsh::RunCounters* rc = nullptr;
  auto release = [&] {
    dfree(dk); dfree(rc); dfree(w.run_ws); dfree(w.huge); dfree(w.over);
    for (auto& c : w.cls) dfree(c);
    for (auto& c : w.big) dfree(c);
  };
  int e = 0;
  if ((e = dalloc(&dk, n)) || (e = dalloc(&rc, 1)) || (e = dalloc(&w.run_ws, klsh::run_ws_words(n))) ||
      (e = dalloc(&w.huge, n / 897 + 64)) || (e = dalloc(&w.over, n / 2 + 64))) {
    release();
    return e;
  }
  for (int c = 0; c < kGroupClasses && !e; ++c) e = dalloc(&w.cls[c], klsh::group_class_capacity(c, n));
  for (int c = 0; c < kBigClasses && !e; ++c)
    e = dalloc(&w.big[c], n / ((c ? klsh::kBigRows[c - 1] : 64) + 1) + 64);
  if (e) {
    release();
    return e;
  }
  w.rc = rc;
  w.kt = klsh::kNoTime;
  hipStream_t s = ctx->stream;
  klsh::RunCounters hc{};
  int rc_ = 0;
  if (hipMemsetAsync(rc, 0, sizeof(*rc), s) != hipSuccess ||
      hipMemcpyAsync(dk, sorted_keys, 4 * n, hipMemcpyHostToDevice, s) != hipSuccess) {
    rc_ = fail(KLSH_E_HIP, "upload");
  } else {
    klsh::launch_runs(dk, 0, (uint32_t)n, bucket_thr, w, s);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(&hc, rc, sizeof(hc), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      rc_ = fail(KLSH_E_HIP, "run finding");
  }
  std::vector<std::array<uint32_t, 3>> runs;  // (start, length, list)
  auto take = [&](const uint2* list, uint32_t count, int l) -> int {
    std::vector<uint2> h(count);
    if (count && hipMemcpy(h.data(), list, sizeof(uint2) * count, hipMemcpyDeviceToHost) != hipSuccess)
      return fail(KLSH_E_HIP, "list copy");
    for (const uint2& x : h) runs.push_back({x.x, x.y, (uint32_t)l});
    return 0;
  };
  for (int c = 0; c < kGroupClasses && !rc_; ++c) rc_ = take(w.cls[c], hc.n_cls[c].v, c);
  for (int c = 0; c < kBigClasses && !rc_; ++c) rc_ = take(w.big[c], hc.n_big[c].v, kGroupClasses + c);
  if (!rc_) rc_ = take(w.huge, hc.n_huge.v, klsh::kRunListCount - 2);
  if (!rc_) rc_ = take(w.over, hc.n_over.v, klsh::kRunListCount - 1);
  release();
  if (rc_) return rc_;
  std::sort(runs.begin(), runs.end());
  *n_runs = runs.size();
  if (runs.size() > cap) return fail(KLSH_E_RANGE, "more runs than the output holds (see *n_runs)");
  for (size_t i = 0; i < runs.size(); ++i) {
    if (starts) starts[i] = runs[i][0];
    if (lengths) lengths[i] = runs[i][1];
    if (lists) lists[i] = (int32_t)runs[i][2];
  }
  return 0;
}

int klsh_pcluster(klsh_ctx* ctx, float thr) {
  if (!ctx) return fail(KLSH_E_ARG, "null ctx");
  if (!ctx->loaded) return fail(KLSH_E_STATE, "nothing loaded");
  KLSH_HIP(hipSetDevice(ctx->device));
  const uint32_t n = (uint32_t)ctx->n_live;
  if (n == 0) return 0;
  hipStream_t s = ctx->stream;
  if (int e = ctx->reset_counters()) return e;
  ctx->mw.huge_fold = ctx->huge_fold_always ? 1u : 0u;
  ctx->mw.huge_cap = 0;
  KLSH_HIP(hipMemsetAsync(ctx->keys, 0, 4ull * n, s));  // one bucket: every key equal
  uint64_t dummy = 0;
  if (int e = merge_and_compact(ctx, ctx->keys, ctx->order, n, thr, -1, 0, &dummy, nullptr, false))
    return e;
  KLSH_HIP(hipStreamSynchronize(s));  // see klsh_cluster: the order may still be in flight
  return 0;
}

int klsh_hyperplanes(uint32_t seed_base, uint64_t* rng_counter, int h, int d, float* table) {
  if (!rng_counter || (!table && h > 0) || d <= 0 || h < 0) return fail(KLSH_E_ARG, "bad argument");
  klsh_host_hyperplanes(seed_base, *rng_counter, (uint64_t)h, d, d, table, 1);
  *rng_counter += (uint64_t)h;
  return 0;
}

int klsh_fp_selftest(klsh_ctx* ctx, const float* a, const float* b, uint64_t n, float* sqrt_out,
                     float* div_out) {
  if (!ctx || !a || !b || !sqrt_out || !div_out) return fail(KLSH_E_ARG, "null argument");
  if (n == 0) return 0;
  KLSH_HIP(hipSetDevice(ctx->device));
  float *da = nullptr, *db = nullptr, *ds = nullptr, *dd = nullptr;
  int e = 0;
  if ((e = dalloc(&da, n)) || (e = dalloc(&db, n)) || (e = dalloc(&ds, n)) || (e = dalloc(&dd, n))) {
    dfree(da); dfree(db); dfree(ds); dfree(dd);
    return e;
  }
  hipStream_t s = ctx->stream;
  int rc = 0;
  if (hipMemcpyAsync(da, a, 4 * n, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(db, b, 4 * n, hipMemcpyHostToDevice, s) != hipSuccess) {
    rc = fail(KLSH_E_HIP, "upload");
  } else {
    klsh::launch_fp_selftest(da, db, (uint32_t)n, ds, dd, s);
    if (hipMemcpyAsync(sqrt_out, ds, 4 * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(div_out, dd, 4 * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      rc = fail(KLSH_E_HIP, "selftest");
  }
  (void)hipStreamSynchronize(s);
  dfree(da); dfree(db); dfree(ds); dfree(dd);
  return rc;
}

}  // extern "C"
