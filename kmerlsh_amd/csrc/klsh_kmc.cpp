// Mode B behind the C ABI (include/klsh.h): kmer_set.hex / kmer_count.bin / kmer_count.log from
// a set of KMC databases (reference buildKHtable with kmc = false, io/ioHT.cc:83-199; KmcRead /
// KmcCount, kmer/kmc_reader.cc:26-169; CKMCFile listing, kmer/kmc_api/kmc_file.cpp:66-532).
//
// The host streams each .kmc_suf in chunks (the files are the I/O); the GPU decodes the records
// (klsh_kmc.hip), builds the union of canonical k-mers in a device hash table (pass 1) and, per
// sample, the summed counts (pass 2).  The coverage of a sample is a float running sum of
// log(count) in file order, exactly the reference's accumulation, so it stays on the host.
//
// Row order: the reference writes its rows in the iteration order of its libcuckoo table
// (ckhmap_t, hash/HashTables.h:22; iterated by io/ioHT.cc:140-149 and WriteHT :30-55), filled by
// KmcRead's inserts (kmer/kmc_reader.cc:5-20, 66-70: at -T 1 one insert per listed k-mer in
// sample, then listing order).  A duplicate insert changes nothing, so the table is the result of
// inserting the distinct k-mers in first-appearance order: the GPU finds them (pass 1), the host
// replays libcuckoo's sequential insert on them (CuckooOrder below), and the rows come out in
// that table's order.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <chrono>
#include <cmath>
#include <string>
#include <vector>

#include "klsh.h"
#include "klsh_internal.h"

namespace {

using klsh::set_error;

double now_ms() {
  return std::chrono::duration<double, std::milli>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// CKMCFile::OpenForListing + ReadParamsFrom_prefix_file_buf (kmc_file.cpp:66-300), restated.
struct KmcDb {
  uint32_t version = 0, k = 0, mode = 0, counter_size = 0, p = 0, sig_len = 0, min_count = 0;
  uint64_t max_count = 0, total = 0;
  std::vector<uint64_t> lut;  // cumulative record index per (bin,) prefix; last = total + 1
  std::string suf;
  std::string err;

  bool open(const std::string& name) {
    std::vector<uint8_t> pre;
    {
      FILE* f = fopen((name + ".kmc_pre").c_str(), "rb");
      if (!f) return fail("cannot open " + name + ".kmc_pre");
      fseek(f, 0, SEEK_END);
      const long sz = ftell(f);
      fseek(f, 0, SEEK_SET);
      pre.resize(sz > 0 ? (size_t)sz : 0);
      const size_t got = pre.empty() ? 0 : fread(pre.data(), 1, pre.size(), f);
      fclose(f);
      if (got != pre.size() || pre.size() < 24) return fail(name + ".kmc_pre: short file");
    }
    if (memcmp(pre.data(), "KMCP", 4) || memcmp(pre.data() + pre.size() - 4, "KMCP", 4))
      return fail(name + ".kmc_pre: bad marker");
    uint64_t size = pre.size() - 8;
    auto u32 = [&](size_t o) { uint32_t v; memcpy(&v, pre.data() + o, 4); return v; };
    auto u64 = [&](size_t o) { uint64_t v; memcpy(&v, pre.data() + o, 8); return v; };
    version = u32(pre.size() - 12);
    const uint64_t header_offset = pre[pre.size() - 8];  // fgetc: the low byte
    // (the reader trusts the file; here every offset derived from it is checked first)
    if (version == 0x200) {
      size -= 4;
      if (header_offset + 8 + 36 > pre.size()) return fail(name + ".kmc_pre: bad header offset");
      const size_t h = pre.size() - (header_offset + 8);
      k = u32(h);
      mode = u32(h + 4);
      counter_size = u32(h + 8);
      p = u32(h + 12);
      sig_len = u32(h + 16);
      min_count = u32(h + 20);
      max_count = u32(h + 24);
      total = u64(h + 28);
      if (sig_len > 16) return fail(name + ".kmc_pre: bad signature length");
      const uint64_t sig_map = (1ull << (2 * sig_len)) + 1;
      if (sig_map * 4 + header_offset + 8 > size) return fail(name + ".kmc_pre: short LUT");
      const uint64_t lut_bytes = size - (sig_map * 4 + header_offset + 8);
      if (4 + (lut_bytes + 8) / 8 * 8 > pre.size()) return fail(name + ".kmc_pre: short LUT");
      lut.resize((lut_bytes + 8) / 8);
      memcpy(lut.data(), pre.data() + 4, lut.size() * 8);
      lut[lut_bytes / 8] = total + 1;
      lut.resize(lut_bytes / 8 + 1);
    } else if (version == 0) {
      const uint64_t n = (size - 4) / 8;
      std::vector<uint64_t> buf(n);
      memcpy(buf.data(), pre.data() + 4, n * 8);
      size -= 4;
      if (header_offset > size) return fail(name + ".kmc_pre: bad header offset");
      const uint64_t hi = (size - header_offset) / 8;
      if (hi + 4 >= n) return fail(name + ".kmc_pre: bad header");
      k = (uint32_t)buf[hi];
      mode = (uint32_t)(buf[hi] >> 32);
      counter_size = (uint32_t)buf[hi + 1];
      p = (uint32_t)(buf[hi + 1] >> 32);
      min_count = (uint32_t)buf[hi + 2];
      max_count = buf[hi + 2] >> 32;
      total = buf[hi + 3];
      max_count += buf[hi + 4] & 0xFFFFFFFF00000000ull;
      buf[hi] = total + 1;
      buf.resize(hi + 1);
      lut.swap(buf);
    } else {
      return fail(name + ".kmc_pre: unsupported KMC version");
    }
    if (mode != 0) return fail(name + ": quality-aware (float) counters are not supported");
    for (size_t i = 1; i < lut.size(); ++i)  // the decode's binary search needs a sorted LUT
      if (lut[i] < lut[i - 1]) return fail(name + ".kmc_pre: LUT not ascending");
    if (k < 1 || k > 32 || p > k || (k - p) % 4 || counter_size < 1 || counter_size > 4 || p > 15)
      return fail(name + ": unsupported k / prefix / counter layout");
    suf = name + ".kmc_suf";
    return true;
  }
  bool fail(const std::string& m) {
    err = m;
    return false;
  }
  klsh::KmcParams params() const {
    klsh::KmcParams kp{};
    kp.k = (int)k;
    kp.p = (int)p;
    kp.sufix_size = (k - p) / 4;
    kp.counter_size = counter_size;
    kp.rec_size = kp.sufix_size + counter_size;
    kp.min_count = min_count;
    kp.max_count = max_count;
    kp.prefix_mask = (1ull << (2 * p)) - 1ull;
    return kp;
  }
};

// ---------------------------------------------------------------- libcuckoo table order -----
// Kmer::hash() (kmer/Kmer.cc:138-147): MurmurHash3_x64_64 of the Kmer's first k_bytes = (k+3)/4
// bytes with seed 0, i.e. the first half of hash/hash.cc's MurmurHash3_x64_128 — an early
// revision of that function (bmix64 with the per-block c1/c2 schedule, h1/h2 started from
// 0x9368e53c2f6af274 / 0x586dcd208f7cd3fd).  k_bytes <= 8, so the input is one tail block: the
// image's low k_bytes bytes (the Kmer's bytes in memory order, little-endian) as k1, k2 = 0.
inline uint64_t rotl64(uint64_t v, int r) { return (v << r) | (v >> (64 - r)); }
inline uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}
uint64_t kmer_hash(uint64_t image, int nbytes) {
  uint64_t h1 = 0x9368e53c2f6af274ull, h2 = 0x586dcd208f7cd3fdull;
  const uint64_t c1 = 0x87c37b91114253d5ull, c2 = 0x4cf5ad432745937full;
  uint64_t k1 = nbytes >= 8 ? image : (image & ((1ull << (8 * nbytes)) - 1ull));
  if (nbytes > 0) {  // one bmix64 round on the tail (k2 = 0 leaves h2's xor unchanged)
    k1 *= c1;
    k1 = rotl64(k1, 23);
    k1 *= c2;
    h1 ^= k1;
    h1 += h2;
    h2 = rotl64(h2, 41);
    h2 += h1;
    h1 = h1 * 3 + 0x52dce729ull;
    h2 = h2 * 3 + 0x38495ab5ull;
  }
  h2 ^= (uint64_t)nbytes;
  h1 += h2;
  h2 += h1;
  h1 = fmix64(h1);
  h2 = fmix64(h2);
  return h1 + h2;
}

// cuckoohash_map (utils/libcuckoo/cuckoohash_map.hh, the vendored revision) restated for one
// thread: 2^hp buckets of SLOT_PER_BUCKET = 8 slots (cuckoohash_config.h:7), hp = 16 for the
// default-constructed table (DEFAULT_SIZE = 2^16 * 8 elements, reserve_calc :382-387).  An
// element's buckets: i1 = hv & mask, i2 = (i1 ^ ((hv >> hp) + 1) * 0x5bd1e995) & mask
// (index_hash / alt_index :893-908).  insert (:513-523, cuckoo_insert :1428-1483): the first free
// slot of i1, else of i2, else a cuckoo path found by slot_search's breadth-first search (:983-
// 1022: a 501-entry queue seeded with i1 then i2, slots in order, each displaced key's other
// bucket checked for a free slot before being queued, paths of at most MAX_BFS_DEPTH = 4 moves)
// and applied from its far end (cuckoopath_move :1124-1176); no path: the table doubles
// (cuckoo_expand_simple :1627-1667, every element of old bucket 0, 1, ... re-inserted into the new
// table) and the insert is retried.  Elements are indices into the caller's arrays.
class CuckooOrder {
 public:
  static constexpr uint32_t kEmpty = 0xFFFFFFFFu;
  static constexpr int kSlots = 8, kMaxDepth = 4, kQueue = 500 + 1;
  CuckooOrder(const std::vector<uint64_t>& hv, int hp) : hv_(hv) { init(hp); }
  void insert(uint32_t e) {
    while (!try_insert(e)) expand();
  }
  // the table's elements in iteration order (buckets ascending, slots ascending)
  std::vector<uint32_t> order() const {
    std::vector<uint32_t> out;
    for (uint32_t v : tab_)
      if (v != kEmpty) out.push_back(v);
    return out;
  }
  int hashpower() const { return hp_; }

 private:
  const std::vector<uint64_t>& hv_;
  int hp_ = 0;
  uint64_t mask_ = 0;
  std::vector<uint32_t> tab_;  // [bucket][slot]

  void init(int hp) {
    hp_ = hp;
    mask_ = (1ull << hp) - 1ull;
    tab_.assign((size_t)kSlots << hp, kEmpty);
  }
  uint64_t i1(uint64_t h) const { return h & mask_; }
  uint64_t alt(uint64_t h, uint64_t b) const {
    const uint64_t tag = (h >> hp_) + 1ull;
    return (b ^ (tag * 0x5bd1e995ull)) & mask_;
  }
  uint32_t& at(uint64_t b, int s) { return tab_[(size_t)b * kSlots + s]; }
  int first_free(uint64_t b) {
    for (int s = 0; s < kSlots; ++s)
      if (at(b, s) == kEmpty) return s;
    return -1;
  }
  struct BSlot {
    uint64_t bucket, pathcode;
    int depth;
  };
  // slot_search: the breadth-first search for a bucket with a free slot
  bool search(uint64_t a, uint64_t b, BSlot* found) {
    BSlot q[kQueue];
    int first = 0, last = 0;
    auto next = [](int i) { return i == kQueue - 1 ? 0 : i + 1; };
    auto not_full = [&] { return next(last) != first; };
    q[last] = {a, 0, 0};
    last = next(last);
    q[last] = {b, 1, 0};
    last = next(last);
    while (not_full()) {
      BSlot x = q[first];
      first = next(first);
      for (int s = 0; s < kSlots && not_full(); ++s) {
        if (at(x.bucket, s) == kEmpty) {
          x.pathcode = x.pathcode * kSlots + (uint64_t)s;
          *found = x;
          return true;
        }
        BSlot y{alt(hv_[at(x.bucket, s)], x.bucket), x.pathcode * kSlots + (uint64_t)s, x.depth + 1};
        const int j = first_free(y.bucket);
        if (j >= 0) {
          y.pathcode = y.pathcode * kSlots + (uint64_t)j;
          *found = y;
          return true;
        }
        if (y.depth != kMaxDepth) {
          q[last] = y;
          last = next(last);
        }
      }
    }
    return false;
  }
  bool try_insert(uint32_t e) {
    const uint64_t h = hv_[e], a = i1(h), b = alt(h, a);
    int s = first_free(a);
    if (s >= 0) return at(a, s) = e, true;
    s = first_free(b);
    if (s >= 0) return at(b, s) = e, true;
    BSlot x;
    if (!search(a, b, &x)) return false;
    // cuckoopath_search: slots from the path code (last first), buckets from the start bucket
    // and each displaced key's other bucket
    uint64_t pb[kMaxDepth + 1];
    int ps[kMaxDepth + 1];
    uint64_t code = x.pathcode;
    for (int i = x.depth; i >= 0; --i) {
      ps[i] = (int)(code % kSlots);
      code /= kSlots;
    }
    pb[0] = code == 0 ? a : b;
    for (int i = 1; i <= x.depth; ++i) pb[i] = alt(hv_[at(pb[i - 1], ps[i - 1])], pb[i - 1]);
    // cuckoopath_move: from the free slot back to the start bucket
    for (int d = x.depth; d > 0; --d) {
      at(pb[d], ps[d]) = at(pb[d - 1], ps[d - 1]);
      at(pb[d - 1], ps[d - 1]) = kEmpty;
    }
    at(pb[0], ps[0]) = e;
    return true;
  }
  void expand() {
    std::vector<uint32_t> old;
    old.swap(tab_);
    init(hp_ + 1);
    for (uint32_t v : old)
      if (v != kEmpty) insert(v);
  }
};

}  // namespace

// Test hook (tests/test_sanitizers.py): the host parse of one KMC database's prefix file (the
// header and the prefix LUT, everything klsh_build_khtable reads before its device work).
extern "C" int klsh_kmc_info(const char* name, int* k, uint64_t* total, uint64_t* lut_entries) {
  if (!name) return set_error(KLSH_E_ARG, "null argument");
  KmcDb db;
  if (!db.open(name)) return set_error(KLSH_E_ARG, db.err.c_str());
  if (k) *k = (int)db.k;
  if (total) *total = db.total;
  if (lut_entries) *lut_entries = db.lut.size();
  return KLSH_OK;
}

// Test hook (tests/test_mode_b.py): the libcuckoo table order of `n` distinct k-mer images
// inserted in the given order; order[i] = the index of the i-th element of the table.  Returns the
// final hash power.
extern "C" int klsh_cuckoo_order(const uint64_t* images, uint64_t n, int k, uint32_t* order) {
  if ((!images || !order) && n) return set_error(KLSH_E_ARG, "null argument");
  if (k < 1 || k > 32) return set_error(KLSH_E_RANGE, "k must be in [1, 32]");
  if (n >= 0xFFFFFFFFull) return set_error(KLSH_E_RANGE, "too many k-mers");
  std::vector<uint64_t> hv(n);
  for (uint64_t i = 0; i < n; ++i) hv[i] = kmer_hash(images[i], (k + 3) / 4);
  CuckooOrder t(hv, 16);
  for (uint64_t i = 0; i < n; ++i) t.insert((uint32_t)i);
  const std::vector<uint32_t> o = t.order();
  if (!o.empty()) memcpy(order, o.data(), o.size() * 4);
  return t.hashpower();
}

#define KLSH_KHIP(call)                                                                   \
  do {                                                                                    \
    hipError_t e_ = (call);                                                               \
    if (e_ != hipSuccess) {                                                               \
      rc = set_error(KLSH_E_HIP, (std::string(#call) + " -> " + hipGetErrorString(e_)).c_str()); \
      goto done;                                                                          \
    }                                                                                     \
  } while (0)

extern "C" int klsh_build_khtable(klsh_ctx* ctx, const char* const* kmc_names, int n_samples,
                                  int k, const char* out_dir, klsh_khtable_stats* st) {
  if (!ctx || !kmc_names || n_samples <= 0) return set_error(KLSH_E_ARG, "bad argument");
  if (k < 1 || k > 32) return set_error(KLSH_E_RANGE, "k must be in [1, 32] (Kmer::MAX_K)");
  const double t_start = now_ms();
  if (st && st->struct_size != sizeof(klsh_khtable_stats))
    return set_error(KLSH_E_ARG, "klsh_khtable_stats.struct_size != sizeof: built against another klsh.h");
  klsh_khtable_stats local{};
  local.struct_size = sizeof(local);
  std::vector<KmcDb> dbs(n_samples);
  uint64_t records = 0;
  for (int j = 0; j < n_samples; ++j) {
    if (!kmc_names[j] || !dbs[j].open(kmc_names[j]))
      return set_error(KLSH_E_ARG, kmc_names[j] ? dbs[j].err.c_str() : "null database name");
    if ((int)dbs[j].k != k)
      return set_error(KLSH_E_ARG, (std::string(kmc_names[j]) + ": k-mer length differs from -K").c_str());
    records += dbs[j].total;
  }
  if (hipSetDevice(klsh::ctx_device(ctx)) != hipSuccess) return set_error(KLSH_E_HIP, "hipSetDevice");
  const hipStream_t s = klsh::ctx_stream(ctx);
  const std::string dir = (out_dir && *out_dir) ? std::string(out_dir) + "/" : std::string();

  uint64_t cap = 1024;
  while (cap < 2 * (records + (uint64_t)n_samples)) cap <<= 1;
  if (cap > (1ull << 32)) return set_error(KLSH_E_RANGE, "more than 2^31 distinct k-mers");
  const uint64_t mask = cap - 1;
  constexpr uint64_t kChunkBytes = 64ull << 20;
  int rc = KLSH_OK;
  uint64_t *tab = nullptr, *first = nullptr, *drep = nullptr, *dlut = nullptr, *keys_out = nullptr;
  uint32_t *acc = nullptr, *dcnt = nullptr, *nvalid = nullptr, *lo = nullptr, *lo2 = nullptr;
  uint32_t *slots = nullptr, *slots2 = nullptr, *ws = nullptr;
  uint16_t* col = nullptr;
  uint8_t* drec = nullptr;
  std::vector<uint8_t> hrec(kChunkBytes);
  std::vector<uint32_t> order_dbg;
  std::vector<uint64_t> base(n_samples + 1, 0);
  uint32_t kmap = 0;
  FILE *fh = nullptr, *fb = nullptr, *fl = nullptr;
  std::vector<float> coverage(n_samples, 0.0f);
  uint64_t max_lut = 0, max_chunk_recs = 0;
  for (const auto& db : dbs) {
    max_lut = std::max<uint64_t>(max_lut, db.lut.size());
    max_chunk_recs = std::max<uint64_t>(max_chunk_recs, kChunkBytes / db.params().rec_size + 1);
  }
  KLSH_KHIP(hipMalloc((void**)&tab, cap * 8));
  KLSH_KHIP(hipMalloc((void**)&first, cap * 8));
  KLSH_KHIP(hipMalloc((void**)&acc, cap * 4));
  KLSH_KHIP(hipMalloc((void**)&drec, kChunkBytes + 64));
  KLSH_KHIP(hipMalloc((void**)&drep, max_chunk_recs * 8));
  KLSH_KHIP(hipMalloc((void**)&dcnt, max_chunk_recs * 4));
  KLSH_KHIP(hipMalloc((void**)&dlut, max_lut * 8));
  KLSH_KHIP(hipMalloc((void**)&nvalid, 64));
  KLSH_KHIP(hipMemsetAsync(tab, 0xFF, cap * 8, s));
  KLSH_KHIP(hipMemsetAsync(first, 0xFF, cap * 8, s));

  // Stream sample j's records through decode + `per_chunk` (pass 1: union; pass 2: counts).
  for (int pass = 0; pass < 2; ++pass) {
    for (int j = 0; j < n_samples; ++j) {
      const KmcDb& db = dbs[j];
      const klsh::KmcParams kp = db.params();
      KLSH_KHIP(hipMemcpyAsync(dlut, db.lut.data(), db.lut.size() * 8, hipMemcpyHostToDevice, s));
      KLSH_KHIP(hipMemsetAsync(nvalid, 0, 4, s));
      if (pass == 1) KLSH_KHIP(hipMemsetAsync(acc, 0, cap * 4, s));
      FILE* f = fopen(db.suf.c_str(), "rb");
      if (!f) {
        rc = set_error(KLSH_E_ARG, ("cannot open " + db.suf).c_str());
        goto done;
      }
      char mark[4];
      if (fread(mark, 1, 4, f) != 4 || memcmp(mark, "KMCS", 4)) {
        fclose(f);
        rc = set_error(KLSH_E_ARG, (db.suf + ": bad marker").c_str());
        goto done;
      }
      const uint64_t per_chunk = kChunkBytes / kp.rec_size;
      float cov = 0.0f;
      for (uint64_t r0 = 0; r0 < db.total; r0 += per_chunk) {
        const uint64_t n = std::min<uint64_t>(per_chunk, db.total - r0);
        const double tio = now_ms();
        if (fread(hrec.data(), kp.rec_size, n, f) != n) {
          fclose(f);
          rc = set_error(KLSH_E_ARG, (db.suf + ": short file").c_str());
          goto done;
        }
        local.io_ms += now_ms() - tio;
        KLSH_KHIP(hipMemcpyAsync(drec, hrec.data(), n * kp.rec_size, hipMemcpyHostToDevice, s));
        klsh::launch_kmc_decode(drec, n, r0, kp, dlut, db.lut.size(), drep, dcnt, nvalid, s);
        if (pass == 0) klsh::launch_kmc_union(drep, n, base[j] + r0, tab, first, mask, s);
        else klsh::launch_kmc_count(drep, dcnt, n, tab, mask, acc, s);
        KLSH_KHIP(hipGetLastError());
        if (pass == 1) {  // tot_coverage += log(cnt), float, file order (kmc_reader.cc:143)
          for (uint64_t i = 0; i < n; ++i) {
            const uint8_t* q = hrec.data() + i * kp.rec_size + kp.sufix_size;
            uint32_t c = 0;
            for (uint32_t b = 0; b < kp.counter_size; ++b) c |= (uint32_t)q[b] << (8 * b);
            if (c >= db.min_count && (uint64_t)c <= db.max_count) cov += log((double)c);
          }
        }
        KLSH_KHIP(hipStreamSynchronize(s));  // hrec is reused by the next read
      }
      fclose(f);
      local.records += db.total;
      if (pass == 0) {
        uint32_t nv = 0;
        KLSH_KHIP(hipMemcpy(&nv, nvalid, 4, hipMemcpyDeviceToHost));
        local.records_listed += nv;
        // fewer listed than the total: KmcRead's vector keeps default (all-A) k-mers at the end
        if (nv < db.total) {
          const uint64_t zero = 0;
          KLSH_KHIP(hipMemcpyAsync(drep, &zero, 8, hipMemcpyHostToDevice, s));
          klsh::launch_kmc_union(drep, 1, base[j] + db.total, tab, first, mask, s);
          KLSH_KHIP(hipGetLastError());
          KLSH_KHIP(hipStreamSynchronize(s));
        }
        base[j + 1] = base[j] + db.total + 1;
      } else {
        coverage[j] = cov;
        // this sample's column in output order (WriteHT, io/ioHT.cc:30-55)
        klsh::launch_kmc_emit(acc, slots, kmap, col, s);
        KLSH_KHIP(hipGetLastError());
        std::vector<uint16_t> hcol(kmap);
        if (kmap) KLSH_KHIP(hipMemcpyAsync(hcol.data(), col, kmap * 2ull, hipMemcpyDeviceToHost, s));
        KLSH_KHIP(hipStreamSynchronize(s));
        if (kmap && fwrite(hcol.data(), 2, kmap, fb) != kmap) {
          rc = set_error(KLSH_E_ARG, "kmer_count.bin: write failed");
          goto done;
        }
      }
    }
    if (pass == 0) {
      // first-appearance order: occupied slots sorted by their 64-bit ordinal (two stable
      // 32-bit radix sorts, low word then high word)
      KLSH_KHIP(hipMalloc((void**)&lo, (cap / 2 + 64) * 4));
      KLSH_KHIP(hipMalloc((void**)&lo2, (cap / 2 + 64) * 4));
      KLSH_KHIP(hipMalloc((void**)&slots, (cap / 2 + 64) * 4));
      KLSH_KHIP(hipMalloc((void**)&slots2, (cap / 2 + 64) * 4));
      KLSH_KHIP(hipMalloc((void**)&ws, klsh::sort_ws_words(cap / 2 + 64) * 4));
      KLSH_KHIP(hipMemsetAsync(nvalid, 0, 4, s));
      klsh::launch_kmc_collect(tab, first, cap, lo, slots, nvalid, s);
      KLSH_KHIP(hipGetLastError());
      KLSH_KHIP(hipMemcpyAsync(&kmap, nvalid, 4, hipMemcpyDeviceToHost, s));
      KLSH_KHIP(hipStreamSynchronize(s));
      uint32_t *ok_ = nullptr, *ov_ = nullptr;
      klsh::radix_sort(lo, slots, lo2, slots2, kmap, 32, ws, &ok_, &ov_, s);
      const uint64_t last = base[n_samples];
      int hbits = 0;
      while (hbits < 32 && (last >> 32) >> hbits) ++hbits;
      if (hbits) {
        uint32_t* hk = ok_ == lo ? lo2 : lo;  // the free key buffer
        uint32_t* hv = ov_ == slots ? slots2 : slots;
        klsh::launch_kmc_hi(first, ov_, kmap, hk, s);
        uint32_t *ok2 = nullptr, *ov2 = nullptr;
        klsh::radix_sort(hk, ov_, ok_, hv, kmap, hbits, ws, &ok2, &ov2, s);
        ov_ = ov2;
      }
      KLSH_KHIP(hipGetLastError());
      if (ov_ != slots) KLSH_KHIP(hipMemcpyAsync(slots, ov_, kmap * 4ull, hipMemcpyDeviceToDevice, s));
      KLSH_KHIP(hipMalloc((void**)&keys_out, (uint64_t)std::max<uint32_t>(kmap, 1) * 8));
      KLSH_KHIP(hipMalloc((void**)&col, (uint64_t)std::max<uint32_t>(kmap, 1) * 2));
      klsh::launch_kmc_emit_keys(tab, slots, kmap, keys_out, s);
      KLSH_KHIP(hipGetLastError());
      std::vector<uint64_t> hkeys(kmap);
      std::vector<uint32_t> hslots(kmap);
      if (kmap) {
        KLSH_KHIP(hipMemcpyAsync(hkeys.data(), keys_out, kmap * 8ull, hipMemcpyDeviceToHost, s));
        KLSH_KHIP(hipMemcpyAsync(hslots.data(), slots, kmap * 4ull, hipMemcpyDeviceToHost, s));
      }
      KLSH_KHIP(hipStreamSynchronize(s));
      {  // the reference's row order: its libcuckoo table after the first-appearance inserts
        const double tc = now_ms();
        std::vector<uint64_t> hv(kmap);
        for (uint32_t i = 0; i < kmap; ++i) hv[i] = kmer_hash(hkeys[i], (k + 3) / 4);
        CuckooOrder table(hv, 16);
        for (uint32_t i = 0; i < kmap; ++i) table.insert(i);
        const std::vector<uint32_t> ord = table.order();
        std::vector<uint64_t> k2(kmap);
        std::vector<uint32_t> s2(kmap);
        for (uint32_t i = 0; i < kmap; ++i) {
          k2[i] = hkeys[ord[i]];
          s2[i] = hslots[ord[i]];
        }
        hkeys.swap(k2);
        if (kmap) KLSH_KHIP(hipMemcpyAsync(slots, s2.data(), kmap * 4ull, hipMemcpyHostToDevice, s));
        KLSH_KHIP(hipStreamSynchronize(s));
        local.order_ms = now_ms() - tc;
      }
      // kmer_set.hex: the k-mers' 8-byte images in row order (Kmer::writeBytes, kmer/Kmer.cc:307)
      fh = fopen((dir + "kmer_set.hex").c_str(), "wb");
      fb = fopen((dir + "kmer_count.bin").c_str(), "wb");
      fl = fopen((dir + "kmer_count.log").c_str(), "w");
      if (!fh || !fb || !fl) {
        rc = set_error(KLSH_E_ARG, "cannot write kmer_set.hex / kmer_count.bin / kmer_count.log");
        goto done;
      }
      if (kmap && fwrite(hkeys.data(), 8, kmap, fh) != kmap) {
        rc = set_error(KLSH_E_ARG, "kmer_set.hex: write failed");
        goto done;
      }
    }
  }
  // kmer_count.log: "%llu" kmap_size, then "\t%f" per sample coverage (io/ioHT.cc:170-187)
  fprintf(fl, "%llu", (unsigned long long)kmap);
  for (int j = 0; j < n_samples; ++j) fprintf(fl, "\t%f", (double)coverage[j]);
  local.kmap_size = kmap;

done:
  if (fh) fclose(fh);
  if (fb) fclose(fb);
  if (fl) fclose(fl);
  for (void* ptr : {(void*)tab, (void*)first, (void*)drep, (void*)dlut, (void*)keys_out, (void*)acc,
                    (void*)dcnt, (void*)nvalid, (void*)lo, (void*)lo2, (void*)slots, (void*)slots2,
                    (void*)ws, (void*)col, (void*)drec})
    if (ptr) (void)hipFree(ptr);
  local.total_ms = now_ms() - t_start;
  if (st) *st = local;
  return rc;
}
