// Mode B behind the C ABI (include/klsh.h): kmer_set.hex / kmer_count.bin / kmer_count.log from
// a set of KMC databases (reference buildKHtable with kmc = false, io/ioHT.cc:83-199; KmcRead /
// KmcCount, kmer/kmc_reader.cc:26-169; CKMCFile listing, kmer/kmc_api/kmc_file.cpp:66-532).
//
// The host streams each .kmc_suf in chunks (the files are the I/O); the GPU decodes the records
// (klsh_kmc.hip), builds the union of canonical k-mers in a device hash table (pass 1) and, per
// sample, the summed counts (pass 2).  The coverage of a sample is a float running sum of
// log(count) in file order, exactly the reference's accumulation, so it stays on the host.
//
// Row order: the reference writes its rows in libcuckoo's table order (and fills the table from
// several threads); here rows are in first-appearance order (sample order, then file order) —
// deterministic, and the same set of rows with the same counts and the same kmer_count.log.
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
    if (version == 0x200) {
      size -= 4;
      const size_t h = pre.size() - (header_offset + 8);
      k = u32(h);
      mode = u32(h + 4);
      counter_size = u32(h + 8);
      p = u32(h + 12);
      sig_len = u32(h + 16);
      min_count = u32(h + 20);
      max_count = u32(h + 24);
      total = u64(h + 28);
      const uint64_t sig_map = (1ull << (2 * sig_len)) + 1;
      const uint64_t lut_bytes = size - (sig_map * 4 + header_offset + 8);
      lut.resize((lut_bytes + 8) / 8);
      memcpy(lut.data(), pre.data() + 4, lut.size() * 8);
      lut[lut_bytes / 8] = total + 1;
      lut.resize(lut_bytes / 8 + 1);
    } else if (version == 0) {
      const uint64_t n = (size - 4) / 8;
      std::vector<uint64_t> buf(n);
      memcpy(buf.data(), pre.data() + 4, n * 8);
      size -= 4;
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

}  // namespace

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
  klsh_khtable_stats local{};
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
      if (kmap) KLSH_KHIP(hipMemcpyAsync(hkeys.data(), keys_out, kmap * 8ull, hipMemcpyDeviceToHost, s));
      KLSH_KHIP(hipStreamSynchronize(s));
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
