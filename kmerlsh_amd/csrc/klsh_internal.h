// Internal interface between the host engine (klsh_engine.cpp) and the gfx950 kernels
// (klsh_kernels.hip).  Not part of the C ABI.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>

#include "klsh.h"

namespace klsh {

constexpr uint32_t kInvalid = 0xFFFFFFFFu;  // dead position marker in a bucket's slot run
constexpr uint32_t kNil = 0xFFFFFFFFu;      // end of a member list
constexpr int kMaxHyperplanes = 32;         // keys are uint32 (h = floor(log2 N) <= 31)
constexpr int kScanTile = 4096;             // items per scan workgroup (256 lanes x 16)
// Sort workspace (u32 words) for `slots` keys: [digit][tile] counts and digit totals
// (klsh_sort.hip).
uint64_t sort_ws_words(uint64_t slots);
// Scan workspace (u32 words): [0, 64) ticket / done / epoch of the look-back scan, then its 64-bit
// tile status words (room for 2^32 items), then the tile sums of the multi-kernel scans and of
// the compaction — apart, so a tile sum can never pass for a look-back status word.
constexpr uint32_t kScanStatusWord = 64;
constexpr uint64_t kScanSumsWord = kScanStatusWord + 2ull * (1ull << 20);
inline uint64_t scan_ws_words(uint64_t slots) {
  return kScanSumsWord + (256 * slots) / kScanTile + 1024;
}

// Bucket runs of 65..896 rows are merged by one workgroup with the run's decision matrix in LDS
// (k_merge_big; three size classes, rows in LDS up to 384); longer runs by one wave from memory
// (k_merge_huge).
// 65..128, 129..192, 193..384, 385..896 rows: the 129..192 class has its own layout (62 KB of
// LDS at d = 64) so two of its workgroups share a CU, where a 384-row layout needs 130 KB
constexpr int kBigClasses = 4;
constexpr int kBigRows[kBigClasses] = {128, 192, 384, 896};

// Runs of 2..64 rows are merged by G-lane groups, one size class per G = 2, 4, ..., 64
// (class c holds runs of 2^c < b <= 2^(c+1) rows).
constexpr int kGroupClasses = 6;
inline uint64_t group_class_capacity(int c, uint64_t cap) { return cap / ((1ull << c) + 1) + 64; }

// Run-list counters: k_runs' workgroups add to each of them once, so each sits on a 128-B line of
// its own (adds to one line serialise at ~5-10 ns each; 13 counters on one line made k_runs
// ~10x slower than its key reads).  Device only: the compaction copies them into Counters for
// the host and zeroes them for the next iteration.
struct alignas(128) CountLine {
  uint32_t v;
  uint32_t pad_[31];
};
struct RunCounters {
  CountLine n_seg, n_cls[kGroupClasses], n_big[kBigClasses], n_huge, n_over, n_small_rows;
  CountLine n_big_rows[kBigClasses], n_huge_rows;  // rows in the big / huge runs (kernel rooflines)
  // the small-run screen (k_small_screen): runs of each class it could not rule out, their rows,
  // and a flag that it ran this iteration
  CountLine n_act[kGroupClasses], n_act_rows, screened;
};

// Run-finding workspace (u32 words) for `slots` positions: 19 counts + a tail end + the first /
// last heads + a 4096-bit head bitmap per 4096-position tile.
inline uint64_t run_ws_words(uint64_t slots) { return (slots / 4096 + 2) * (19 + 1 + 2 + 128) + 64; }

// Device-side per-iteration counters (zeroed by the host before each iteration).
struct Counters {
  uint32_t n_seg;                  // bucket runs (k_runs)
  uint32_t n_cls[kGroupClasses];   // runs of 2..64 rows queued per size class
  uint32_t n_big[kBigClasses];     // runs of 65..896 rows queued for k_merge_big, per class
  uint32_t n_huge;                 // longer runs queued for k_merge_huge
  uint32_t n_over;                 // runs longer than bucket_size_threshold (nestedCluster)
  uint32_t total;                  // result of the last scan/compaction (live rows)
  uint32_t n_delta;                // sharded loop: survivors rewritten by a merge this iteration
  uint32_t err;                    // a device-side protocol failure (look-back wait limit); 0 = ok
  uint32_t n_small_rows;           // rows in the runs of 2..64 rows (the small-run merge's rows)
  uint32_t n_big_rows[kBigClasses];  // rows in the runs of each big class
  uint32_t n_huge_rows;            // rows in the runs of k_merge_huge
  uint32_t n_act_rows;             // rows in the small runs the screen passed to k_merge_small
  uint32_t screened;               // 1: the small-run screen ran this iteration
};

// Per-kernel-class timing (bench.py's roofline) from in-kernel stamps: every workgroup of a timed
// launch stamps the 100 MHz real-time counter (s_memrealtime) at its start (atomicMin) and at its
// end (atomicMax) into one of kStampSlots lines of its class, so a class's span in an iteration is
// first workgroup start -> last workgroup end — the span rocprofv3's kernel trace reports — with
// no marker packets in the streams.  (HIP event pairs measure from the moment a stream reaches a
// kernel, resource waits included: tools/ubench_events shows a 50-us kernel timed at 550 us behind
// a chip-filling kernel of another stream, and event pairs around every merge class added 13-20
// ms to a C2 step.)  Iteration t stamps set t & 1; the first workgroup of iteration t+1's
// projection folds set t into the per-class totals (iteration t is complete by then: stream
// order) and clears it; the engine folds the last set at the end of a call.
enum KClass : int {
  KC_PROJECT = 0, KC_SORT, KC_RUNS, KC_SMALL, KC_BIG128, KC_BIG192, KC_BIG384, KC_BIG896, KC_HUGE,
  KC_TAIL, KC_COMPACT, KC_SCREEN,
  KC_MERGE,  // (a phase) the merge launches of an iteration at >= tail_merge_rows positions
            // (default 2^22; every iteration at d > 64), all classes
  KC_COUNT
};
constexpr int kStampSlots = 16;
struct alignas(128) StampLine {
  unsigned long long v;
  unsigned long long pad_[15];
};
struct KStampSet {
  StampLine t0[KC_COUNT][kStampSlots];  // earliest workgroup start (~0 = none)
  StampLine t1[KC_COUNT][kStampSlots];  // latest workgroup end (0 = none)
};
struct KStampBlock {
  KStampSet set[2];
  unsigned long long ticks[KC_COUNT];  // summed spans (10 ns ticks)
  unsigned long long launches[KC_COUNT];
};
// What a launch carries (by value): blk == nullptr = untimed; set = the set it stamps; fold >= 0:
// the projection folds that set first (the previous iteration's).
struct KTime {
  KStampBlock* blk;
  int set;
  int fold;
  int phase = -1;  // >= 0: the launch also stamps this phase class (its first start, last end)
};
constexpr KTime kNoTime{nullptr, 0, -1, -1};
// Fold set `t` into the totals and clear it (one workgroup; device code, klsh_device.h).

// Merge workspace (device), sized for `cap` positions.
struct MergeWork {
  uint2* cls[kGroupClasses];       // (start, length) of runs per size class
  // the runs of each class the fp16 screen could not rule out (k_small_screen), and whether the
  // small-run merge reads these instead of cls (set per launch)
  uint2* act[kGroupClasses];
  uint32_t screened;
  uint2* big[kBigClasses];         // (start, length) of runs for k_merge_big, per class
  uint2* huge;                     // (start, length) of runs for k_merge_huge
  uint2* over;                     // (start, length) of oversize runs
  uint32_t* tile_sums;
  RunCounters* rc;                 // the run counts of this iteration (device)
  uint32_t* run_ws;                // run finding: per-tile list counts, head bitmaps (run_ws_words)
  // Sharded loop only (nullptr otherwise): every survivor a merge rewrote is appended to dlist
  // (ctr->n_delta entries, any order, each slot once); mark[slot] == stamp dedupes the kernels
  // that merge in place (stamp: unique per iteration, never reused by a context).
  uint32_t* dlist;
  uint32_t* mark;
  uint32_t stamp;
  // Size classes run concurrently on kMergeStreams auxiliary streams (fork after the run
  // classification, join before the compaction): in the late, small iterations each class kernel
  // is one long sequential walk, and serialised walks would add up.  aux[0] == nullptr: one stream.
  // 385..896-row runs on aux 2 instead of ahead of the >896-row runs on the main stream: set by
  // the engine when the previous iteration had many of them (C4: thousands; C2: < 10)
  uint32_t big896_aux;
  // >896-row runs: the launch's workgroup cap (0 = one per 897 positions, at most 512).  The
  // engine sets a cap of 64 after an iteration without such runs: an empty launch of hundreds of
  // 512-lane workgroups waits for CUs behind the other classes (C2: 25 ms per step of span)
  uint32_t huge_cap;
  // 1: no k_merge_huge launch; the 385..896-row kernel's workgroups walk the >896-row list after
  // their own (set after several iterations without such runs: C2 and C5 never have any, and an
  // empty launch still costs its dispatch; C4, where they recur, keeps the 512-lane kernel)
  uint32_t huge_fold;
  // runs over 896 rows at d = 16 / 32 (k_merge_long): each workgroup's bit matrix, kLongRows x
  // kLongRows / 64 words, and the number of workgroups it has room for (0: k_merge_huge)
  uint64_t* long_P;
  uint32_t long_groups;
  // option "long_runs": 4 (default) = k_merge_long also takes the 385..896-row runs, 1 = only
  // the longer ones, 0 = k_merge_huge for those (long_off = 1)
  uint32_t long_off = 4;
  // launch sizes (klsh_set_option; 0 = the measured default, see the launch code)
  uint32_t small_grid;       // "small_grid": the small-run merge's persistent launch
  uint32_t tail_nbig;        // "tail_big_groups": k_merge_tail's big-run workgroups
  uint32_t tail_nsmall;      // "tail_small_groups": k_merge_tail's small-run workgroups
  uint32_t wide_group_grid;  // "wide_group_grid": the wide-row group merges, per class
  uint32_t screen_grid;      // "small_screen_grid": the small-run screen's persistent launch
  // "wide_gram": at d = 512 the group merges of runs of at least this many rows (8, 16, 32, 64)
  // decide on the matrix cores; 0 = none
  uint32_t wide_gram = 32;
  uint32_t small_screen = 1;  // "small_screen": 1 = screen the small runs on the fp16 image first
  // "tail_screen": 1 = the small-run screen also runs in front of k_merge_tail (iterations below
  // tail_merge_rows), whose small-run waves then walk only the runs it passed
  uint32_t tail_screen = 1;
  // "tail_big_screen": 1 = there, k_merge_tail's 65..384-row runs are first screened on the fp16
  // image in their workgroup (the small-run screen's certified test); a run with no pair left
  // reads no f32 row.  big_screen / bs_*: set per launch (the test's threshold and margins).
  uint32_t tail_big_screen = 1;
  uint32_t big_screen = 0;
  float bs_s_star = 0.0f, bs_m0 = 0.0f, bs_a2 = 0.0f;
  uint32_t tail_screen_grid;  // "tail_screen_grid": its persistent launch there (0: 2048)
  // "tail_merge_rows": below this many positions every merge class runs in ONE launch
  // (k_merge_tail); 0 = the default 2^22 (tests lower it to reach the per-class launches)
  uint32_t tail_max;
  hipStream_t aux[3];
  KTime kt;                // per-class stamps of this iteration's merge launches
  hipEvent_t small_ev[2];  // HIP events around the small-run launch (nullptr: not recorded)
  hipEvent_t fork;
  hipEvent_t join[3];
};
constexpr int kMergeStreams = 3;
constexpr uint32_t kLongRows = 4096;  // the longest run k_merge_long walks (longer: k_merge_huge)
inline bool long_ok(int d) { return d == 16 || d == 32; }
// (2^22 since round 5: with the small-run screen and the big-run prescreen inside it, the one
// launch beat the four-stream fork/join down to 4M positions — C2, one box, interleaved: 2^20
// 200.2, 2^21 196.5, 2^22 193.1, 2^23 ~= 2^22, 2^24 +1 ms per step)
inline uint32_t tail_merge_max(const MergeWork& w) { return w.tail_max ? w.tail_max : (1u << 22); }

// Row state, structure-of-arrays, one entry per slot (a slot is a row of the loaded matrix;
// a merge writes the consensus into the candidate's slot, cluster.cc:70-74).
struct Rows {
  float* x;        // [slots][dp] fp32 rows, dp = d rounded up to 4 (16-B aligned rows)
  float* nrm;      // [slots] sequential sum of squares (distance.cc:33-34), cached exactly
  uint32_t* cnt;   // [slots] member count (|_ids|)
  uint32_t* head;  // [slots] first member node
  uint32_t* tail;  // [slots] last member node
  uint32_t* nxt;   // [members] next member node (kNil = end)
  int d;
  int dp;
  // [slots][dp] fp16 image of x (round to nearest; may be null): the projection's certified
  // screen reads it instead of x (half the bytes of the row gather).  Kept equal to fp16(x):
  // rebuilt after a load / restore, written with x by every merge store (store_row4/store_row1)
  // and by the sharded delta apply.
  uint16_t* xh = nullptr;
};
// The fp16 image is kept for these widths (the matrix-core screen takes 16 columns per step).
// (the wide-row variants that read an fp16 image of d > 64 rows were measured slower and removed)
inline bool shadow_width_ok(int d) { return d == 16 || d == 32 || d == 64; }

// The merge test of cluster.cc:68-69 as a threshold on the quotient.  The reference computes
// sim = dot / (sqrtf(|a|^2) * sqrtf(|b|^2)); dist = 1 - sim; and merges when 1 - dist >= thr.
// s -> fl(1 - fl(1 - s)) is monotone in s, so the test is exactly fl(dot / den) >= s_star for the
// smallest float s_star that passes (computed on the host by make_decider, NaN if none does).
// Fast path (`fast` != 0, s_star a positive normal float): q = dot * rcp(den) is within 2 ulp of
// dot / den, so q >= s_hi (s_star + 8 ulp) or q <= s_lo (s_star - 8 ulp) settles the test and only
// quotients within a few ulp of s_star take the correctly rounded division.
// Pre-screen (`fast` only): a Gram value G from the bf16x3 MFMA tiles (kGramMargin below) settles
// the test when G / den >= g_hi or <= g_lo; pairs in between take the exact sequential dot.
struct Decider {
  float s_star, s_lo, s_hi;
  uint32_t fast;
  float g_lo, g_hi;
};
// |G - dot| <= 5.4e-5 * |a| |b| for the bf16x3 Gram value at d <= 64 (split residuals
// 3.03 * 2^-16, the MFMA sum <= 29 chained f32 adds per term at 2u, the reference's own 65u; see
// the wide-row projection's bound) against the reference's sequential f32 dot; the margin adds headroom for den's
// rounding and the approximate quotient.
constexpr float kGramMargin = 1.0e-4f;
Decider make_decider(float thr);

// Workspace of the wide-row matrix-core projection: the (row, hyperplane) pairs its screen could
// not call (fix[0 .. cap)), a counter and a done counter (ws[0], ws[1]) that the fix-up kernel
// returns to zero.  Zeroed once at allocation.
struct ProjectWork {
  uint2* fix;
  uint32_t* ws;
  uint32_t cap;
  // launch sizes and test hooks (klsh_set_option; 0 = default)
  uint32_t h16_grid;   // "h16_grid": fp16-image projection workgroups, at most
  uint32_t wide_grid;  // "wide_grid": wide-row screen workgroups, at most
  uint32_t fix_grid;   // "fix_grid": wide-row fix-up workgroups
  uint32_t segcap;     // "h16_segcap" (tests): fix-up entries per fp16-projection workgroup
  uint32_t variant;    // "projection": kProjAuto / kProjPacked / kProjScreen (set per launch)
  uint32_t wide_rolled;  // "wide_unrolled" = 0: d = 512 through the generic wide screen
};
// Projection variants (klsh_set_option "projection"): the default picks the certified
// matrix-core screen where it exists (the fp16 row image at d = 16 / 32 / 64, bf16x3 above 64)
// and the packed exact VALU chains elsewhere; kProjPacked forces the exact chains (no fp16 image
// is kept then); kProjScreen asks for the screen (an error where none exists).  Keys are the
// same bits either way.
constexpr uint32_t kProjAuto = 0, kProjPacked = 1, kProjScreen = 2;
// workgroups of the fp16-image projection, at most (C2 per step: 2048 -> 46.1, 4096 -> 46.5,
// 8192 -> 48.5, 16384 -> 52.9, 32768 -> 55.5 ms, interleaved on one box)
constexpr uint32_t kH16Grid = 2048;

// ---- launch wrappers (all asynchronous on `s`) ------------------------------------------------
// keys[p] = sign-hash of row slots[p] against h hyperplanes W (h x dp), OR'ed with key_or.
// The packed projection of an iteration queued before its row count is known: n and h come from
// the device word n_dev (written by the previous compaction), n_max bounds the grid.  Only for
// d in {8, 16, 32, 64} (project_device_n_ok).
bool project_device_n_ok(int d);
// woff_dev (may be null): the iteration's hyperplanes start woff_dev[0] rows after W (a batch of
// iterations queued at once: each compaction advances it by its own h, see Publish::woff).
void launch_project_device_n(const Rows& r, const uint32_t* slots, uint32_t* keys, uint32_t n_max,
                             const float* W, const uint32_t* n_dev, hipStream_t s,
                             KTime kt = kNoTime, const uint32_t* woff_dev = nullptr,
                             const ProjectWork* pw = nullptr);

// pw (may be null): the workspace that enables the matrix-core screens (the fp16 row image where
// r.xh is set, bf16x3 for d > 64).  Returns the kernel it launched (ProjKernel).
enum ProjKernel : int { kPkNone = -1, kPkPacked = 0, kPkH16 = 1, kPkWide = 2 };
int launch_project(const Rows& r, const uint32_t* slots, uint32_t* keys, uint32_t n,
                   const float* W, int h, uint32_t key_or, hipStream_t s,
                   const ProjectWork* pw = nullptr, KTime kt = kNoTime);

// Stable LSD radix sort of (keys, vals)[0..n) on the low `bits` bits (klsh_sort.hip); ping-pong
// buffers, *out_k/*out_v = the pair holding the result.  ws: sort_ws_words(n) words.
// n_dev (may be null): the key count is read on the device (<= n, which sizes the grids).
void radix_sort(uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, uint32_t n, int bits,
                uint32_t* ws, uint32_t** out_k, uint32_t** out_v, hipStream_t s,
                KTime kt = kNoTime, const uint32_t* n_dev = nullptr);

// Greedy merge (p_cluster) over every bucket run of equal key in positions [lo, hi) of
// (key, slots), in place: survivors first in each run, kInvalid after.  Runs longer than
// bucket_thr (>= 0) are queued to w.over (start, length) and left untouched.
// n_dev (may be null; lo == 0 and hi < 2^20 only): the position count is read on the device
// (<= hi, which sizes the grids).
// runs_ready: the run lists of [lo, hi) are already built (launch_tail_local).
void launch_merge(const Rows& r, const uint32_t* key, uint32_t* slots, uint32_t lo, uint32_t hi,
                  float thr, int bucket_thr, const MergeWork& w, Counters* ctr, hipStream_t s,
                  const uint32_t* n_dev = nullptr, bool runs_ready = false);

// Small iterations (< 2^20 positions, keys of 10..19 bits): the stable bucket sort in two steps
// that also builds the run lists.  radix_sort_top: the stable partition of (k0, v0) by the top
// kTailTopBits of `bits` key bits into (k1, v1); returns the top buckets' sizes.
// launch_tail_local: every top bucket of (k1, v1) sorted stably by its low bits - kTailTopBits
// bits into (k0, v0), and its runs of 2+ equal keys listed into w (as launch_runs would).
const uint32_t* radix_sort_top(const uint32_t* k0, const uint32_t* v0, uint32_t* k1, uint32_t* v1,
                               uint32_t n, int bits, uint32_t* ws, hipStream_t s, KTime kt,
                               const uint32_t* n_dev);
void launch_tail_local(const uint32_t* kin, const uint32_t* vin, uint32_t* kout, uint32_t* vout,
                       const uint32_t* dtot, int bits, int bucket_thr, const MergeWork& w,
                       hipStream_t s);
// the top-bits partition's digit width: 9 (512 top buckets of ~1K keys at C2's tail; the local
// sorts then take up to 10 low bits) measured C2 188.0-188.7 -> 186.1-186.4 ms against 10 (one box,
// interleaved, three rounds: the run listing 19.8 -> 18.3 ms per step, half the workgroups and
// half the same-address list-counter adds); 8 (256 buckets, up to 11 low bits) measured slower:
// run listing 18.4 -> 20.7 ms per step
constexpr int kTailTopBits = 9;
// the local sorts' digit capacity: the low bits of a 19-bit key (the queued iterations have
// N < 2^20, so h <= 19), at least 2^10
constexpr int kTailLowBits = 19 - kTailTopBits > 10 ? 19 - kTailTopBits : 10;
inline bool tail_local_ok(uint32_t n_max, int bits) {
  return n_max <= (1u << 20) && bits > kTailTopBits && bits <= kTailTopBits + kTailLowBits;
}

// Bucket runs of positions [lo, lo + n) of sorted keys (n_dev: the count read on the device, as
// launch_merge): every run of 2+ equal keys into its list of w (size classes, big classes, huge,
// oversize), the counts into w.rc.  (launch_merge's first step; klsh_bucket_runs for tests.)
constexpr int kRunListCount = kGroupClasses + kBigClasses + 2;
void launch_runs(const uint32_t* key, uint32_t lo, uint32_t n, int bucket_thr, const MergeWork& w,
                 hipStream_t s, const uint32_t* n_dev = nullptr);

// Counters handed to the host through mapped pinned memory (no copy launch, no stream sync): the
// compaction's last workgroup writes *ctr (total filled in) to `host`, zeroes *ctr for the next
// iteration, then writes `seq` to *seq_host (system-scope release); the host polls *seq_host.
struct Publish {
  Counters* host;     // device pointer of the mapped host copy (nullptr: no publishing)
  uint32_t* seq_host;
  uint32_t seq;
  uint32_t* n_next;   // device word that also receives the survivor count (may be null)
  // device word advanced by floor(log2 n) of the compacted iteration (may be null): the next
  // iteration's hyperplane offset when a batch of iterations is queued at once (cluster.cc:194-196
  // draws h = floor(log2 N_t) hyperplanes per iteration)
  uint32_t* woff = nullptr;
};

// The look-back compaction's tile status words (>= 256, zeroed once) and the epoch of its last
// launch (status words carry the epoch, so they are never cleared).
struct LookBack {
  unsigned long long* status;
  mutable uint32_t epoch;
};

// out[0..total) = slots[p] for p with slots[p] != kInvalid, stable; ctr->total = count.  rc (may
// be null): the iteration's run counters, copied into *ctr (and zeroed) before the publish.  lb
// (may be null): one launch instead of two when n fits 256 tiles.  n_dev (may be null; needs lb
// and n <= 256 tiles): the slot count is read on the device (<= n, which sizes the grid).
void launch_compact(const uint32_t* slots, uint32_t n, uint32_t* out, uint32_t* tile_sums,
                    Counters* ctr, hipStream_t s, const Publish* pub = nullptr,
                    RunCounters* rc = nullptr, KTime kt = kNoTime,
                    const LookBack* lb = nullptr, const uint32_t* n_dev = nullptr);
// Fold set `set` of blk into its totals and clear it (the end of a timed call).
void launch_stamp_fold(KStampBlock* blk, int set, hipStream_t s);
// a[0..na) then b[0..nb) to dst (mapped host memory, device view), then *seq_host = seq (release)
void launch_publish_words(const uint32_t* a, uint32_t na, const uint32_t* b, uint32_t nb,
                          uint32_t* dst, uint32_t* seq_host, uint32_t seq, hipStream_t s);

// Mode-C producer: rows x[i] (slot i) from counts (d x bs, sample-major), LUT ln(c+1),
// v_kmers; order[] = kept rows (sum > 0.1 d) compacted; ctr->total = kept count.
void launch_convert(const Rows& r, const uint16_t* counts, uint32_t bs, const float* lut,
                    const float* v_kmers, uint32_t* keep, uint32_t* order, uint32_t* tile_sums,
                    Counters* ctr, hipStream_t s);

// Sequential norms nrm[slot] for slots [0, n) (after a load).
void launch_norms(const Rows& r, uint32_t n, hipStream_t s);
// r.xh = fp16(r.x) for slots [0, n).
void launch_shadow_build(const Rows& r, uint64_t n, hipStream_t s);


// out[i*d + k] = x[order[i]][k] (compact result rows).
void launch_gather_rows(const Rows& r, const uint32_t* order, uint32_t n, float* out,
                        hipStream_t s);

// Floating-point self test: sqrt_out[i] = sqrtf(a[i]); div_out[i] = a[i] / b[i] as the merge
// kernels evaluate them.
void launch_fp_selftest(const float* a, const float* b, uint32_t n, float* sqrt_out,
                        float* div_out, hipStream_t s);

// ---- sharded loop (klsh_shard.hip) ----------------------------------------------
constexpr int kMaxBinBits = 12;           // key ranges are unions of 2^12 top-bit bins
constexpr int kMaxRanks = 64;

// hist[bin] += 1 for every key (bin = key >> shift, < nbins); hist zeroed by the caller.
void launch_bin_hist(const uint32_t* keys, uint32_t n, int shift, uint32_t nbins, uint32_t* hist,
                     hipStream_t s);
// From every rank's histogram (hist_all[W][nbins]) and the total row count: owner[bin] = the rank
// owning the bin (contiguous, balanced by rows), cntmat[g * W + r] = rows rank g sends rank r.
void launch_bin_split(const uint32_t* hist_all, int world, uint32_t nbins, uint64_t total,
                      uint32_t* owner, uint32_t* cntmat, hipStream_t s);
// dest[i] = owner[keys[i] >> shift]; idx[i] = i.
// Stable partition of (keys[i], slots[i]), i < n, by owner[keys[i] >> shift] (world <= 64)
// into out, owner-major (out's owner blocks start at the exclusive prefix of the send counts).
// counts: world * ceil(n / 4096) words of workspace.  Returns -1 for an unsupported world.
int launch_partition(const uint32_t* keys, const uint32_t* slots, uint32_t n, int shift,
                     const uint32_t* owner, int world, uint32_t* counts, uint32_t* tile_sums,
                     Counters* ctr, uint2* out, hipStream_t s);
void launch_dest(const uint32_t* keys, uint32_t n, int shift, const uint32_t* owner,
                 uint32_t* dest, uint32_t* idx, hipStream_t s);
// out[i] = (keys[idx[i]], slots[idx[i]]).
void launch_pack_pairs(const uint32_t* keys, const uint32_t* slots, const uint32_t* idx,
                       uint32_t n, uint2* out, hipStream_t s);
// keys[i] = in[i].x, slots[i] = in[i].y.
void launch_unpack_pairs(const uint2* in, uint32_t n, uint32_t* keys, uint32_t* slots,
                         hipStream_t s);
// Delta records, stride 5 + dp words: slot, cnt, head, tail, nrm bits, row[dp].
__host__ __device__ inline int delta_words(int dp) { return 5 + dp; }
void launch_delta_pack(const Rows& r, const uint32_t* delta_slots, uint32_t n, uint32_t* rec,
                       hipStream_t s);
void launch_delta_apply(const Rows& r, const uint32_t* rec, uint32_t n, hipStream_t s);
// Merge profile of the diagnostics build (-DKLSH_MERGE_PROF): print and clear.
void merge_prof_dump(FILE* f);

// a[i] = min(a[i], b[i])
void launch_min_u32(uint32_t* a, const uint32_t* b, size_t n, hipStream_t s);

// ---- mode E (klsh_extract.hip): differential k-mer sets and the per-read k-mer vote ----------
// tab: `mask + 1` (a power of two) 64-bit slots, all ones = empty; kmers[i] == all ones skipped.
void launch_kset_insert(const uint64_t* kmers, uint64_t n, uint64_t* tab, uint64_t mask,
                        hipStream_t s);
// Read r = seq[off[r] .. off[r+1]): hits[r] = its k-mer positions whose canonical k-mer is in the
// set, flags[r] = hits / (len - k + 1) > vote (float), both 0 for reads shorter than k + 10.
void launch_check_reads(const uint8_t* seq, const uint64_t* off, uint64_t n, int k, float vote,
                        const uint64_t* tab, uint64_t mask, uint32_t* hits, uint8_t* flags,
                        hipStream_t s);

// ---- mode B (klsh_kmc.hip): the k-mer table of KMC databases ---------------------------------
struct KmcParams {
  int k, p;                   // k-mer length, LUT prefix symbols
  uint32_t sufix_size;        // (k - p) / 4 bytes per record
  uint32_t counter_size;      // bytes
  uint32_t rec_size;          // sufix_size + counter_size
  uint32_t min_count;
  uint64_t max_count;
  uint64_t prefix_mask;       // (1 << 2p) - 1
};
// records [0, n) of a .kmc_suf chunk starting at record rec0 -> canonical rep (all ones = outside
// [min_count, max_count]) and counter; *n_valid += records kept.  lut: lut_n entries, the last the
// total + 1 sentinel.
void launch_kmc_decode(const uint8_t* recs, uint64_t n, uint64_t rec0, const KmcParams& kp,
                       const uint64_t* lut, uint64_t lut_n, uint64_t* rep, uint32_t* cnt,
                       uint32_t* n_valid, hipStream_t s);
void launch_kmc_union(const uint64_t* rep, uint64_t n, uint64_t ord0, uint64_t* tab,
                      uint64_t* first, uint64_t mask, hipStream_t s);
void launch_kmc_count(const uint64_t* rep, const uint32_t* cnt, uint64_t n, const uint64_t* tab,
                      uint64_t mask, uint32_t* acc, hipStream_t s);
// occupied slots -> (low word of their first-appearance ordinal, slot), *n_out of them
void launch_kmc_collect(const uint64_t* tab, const uint64_t* first, uint64_t cap, uint32_t* lo,
                        uint32_t* slot, uint32_t* n_out, hipStream_t s);
void launch_kmc_hi(const uint64_t* first, const uint32_t* slots, uint64_t n, uint32_t* hi,
                   hipStream_t s);
void launch_kmc_emit_keys(const uint64_t* tab, const uint32_t* order, uint64_t n, uint64_t* out,
                          hipStream_t s);
void launch_kmc_emit(const uint32_t* acc, const uint32_t* order, uint64_t n, uint16_t* out,
                     hipStream_t s);

// The engine's context, for the other host translation units (klsh_extract.cpp).
int ctx_device(const klsh_ctx* ctx);
hipStream_t ctx_stream(const klsh_ctx* ctx);
int set_error(int code, const char* msg);  // sets klsh_last_error(), returns code

}  // namespace klsh
