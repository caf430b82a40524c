// Host-code sanitizer driver (built by `make -C kmerlsh_amd/csrc asan`: the library's host code and
// this driver under AddressSanitizer + UndefinedBehaviorSanitizer; run by tests/test_sanitizers.py,
// CPU only).  It drives every host entry point that reads untrusted input or does host arithmetic
// the GPU path depends on, with valid inputs, edge cases and seeded random corruptions:
//   fastq DIR       every file in DIR through klsh_fastq_open/next (plain and gzip, valid files,
//                   then truncated and byte-flipped copies written here)
//   kmc NAME...     each KMC database's prefix parse (klsh_kmc_info) on the file and on 300
//                   truncated / byte-flipped copies (8 of a prefix file over 1 MB)
//   ttest           klsh_ttest2 / klsh_wrs on random groups, n or m <= 1, constants, NaN / inf
//   cuckoo          klsh_cuckoo_order on random distinct k-mers (k = 1..32), growth included
//   rng             klsh_hyperplanes and klsh_synth_counts on small shapes
// Any sanitizer report aborts the process (-fno-sanitize-recover=all): exit 0 = clean.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <limits>
#include <random>
#include <string>
#include <unordered_set>
#include <vector>

#include "klsh.h"

namespace {

std::vector<unsigned char> slurp(const std::string& path) {
  std::vector<unsigned char> b;
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return b;
  unsigned char buf[1 << 16];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) b.insert(b.end(), buf, buf + n);
  fclose(f);
  return b;
}

void spill(const std::string& path, const std::vector<unsigned char>& b) {
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) {
    perror(path.c_str());
    exit(2);
  }
  if (!b.empty()) fwrite(b.data(), 1, b.size(), f);
  fclose(f);
}

// a corrupted copy: truncated at a random point, or a few random bytes changed
std::vector<unsigned char> corrupt(const std::vector<unsigned char>& b, std::mt19937_64& rng) {
  std::vector<unsigned char> c = b;
  if (c.empty()) return c;
  if (rng() % 2) {
    c.resize(rng() % c.size());
  } else {
    const int flips = 1 + (int)(rng() % 8);
    for (int i = 0; i < flips; ++i) c[rng() % c.size()] = (unsigned char)rng();
  }
  return c;
}

uint64_t read_fastq(const std::string& path) {
  int err = 0;
  klsh_fastq* f = klsh_fastq_open(path.c_str(), &err);
  if (!f) return 0;
  uint64_t recs = 0, bytes = 0;
  while (true) {
    const char *seq, *name, *qual;
    const uint64_t *so, *no, *qo;
    const int64_t n = klsh_fastq_next(f, 1000, &seq, &so, &name, &no, &qual, &qo);
    if (n <= 0) break;
    for (int64_t r = 0; r < n; ++r) {  // touch every byte the reader hands out
      for (uint64_t i = so[r]; i < so[r + 1]; ++i) bytes += (unsigned char)seq[i];
      for (uint64_t i = no[r]; i < no[r + 1]; ++i) bytes += (unsigned char)name[i];
      for (uint64_t i = qo[r]; i < qo[r + 1]; ++i) bytes += (unsigned char)qual[i];
    }
    recs += (uint64_t)n;
  }
  klsh_fastq_close(f);
  return recs + (bytes & 1);
}

int cmd_fastq(int argc, char** argv) {
  std::mt19937_64 rng(7);
  const std::string tmp = std::string(argv[2]) + "/_corrupt";
  uint64_t total = 0;
  for (int a = 3; a < argc; ++a) {
    const std::string path = argv[a];
    total += read_fastq(path);
    const auto b = slurp(path);
    for (int rep = 0; rep < 40; ++rep) {
      spill(tmp, corrupt(b, rng));
      total += read_fastq(tmp);
    }
  }
  // synthetic streams: random bytes over the FASTQ alphabet, plain and gzip
  for (int rep = 0; rep < 60; ++rep) {
    std::string s;
    const char alpha[] = "@+ACGTNacgtn\r\n!IJ>~ \t";
    const size_t len = rng() % 20000;
    for (size_t i = 0; i < len; ++i) s += alpha[rng() % (sizeof alpha - 1)];
    spill(tmp, std::vector<unsigned char>(s.begin(), s.end()));
    total += read_fastq(tmp);
    gzFile g = gzopen(tmp.c_str(), "wb");
    gzwrite(g, s.data(), (unsigned)s.size());
    gzclose(g);
    total += read_fastq(tmp);
  }
  remove(tmp.c_str());
  printf("fastq ok (%llu records)\n", (unsigned long long)total);
  return 0;
}

int cmd_kmc(int argc, char** argv) {
  std::mt19937_64 rng(11);
  int ok = 0, refused = 0;
  for (int a = 2; a < argc; ++a) {
    const std::string name = argv[a];
    int k = 0;
    uint64_t total = 0, lut = 0;
    if (klsh_kmc_info(name.c_str(), &k, &total, &lut) != KLSH_OK) {
      fprintf(stderr, "valid database refused: %s: %s\n", name.c_str(), klsh_last_error());
      return 1;
    }
    const auto pre = slurp(name + ".kmc_pre");
    const std::string tmp = name + "_corrupt";
    const int reps = pre.size() < (1u << 20) ? 300 : 8;  // (p = 12 prefix files are 128 MB)
    for (int rep = 0; rep < reps; ++rep) {
      spill(tmp + ".kmc_pre", corrupt(pre, rng));
      if (klsh_kmc_info(tmp.c_str(), &k, &total, &lut) == KLSH_OK) ++ok;
      else ++refused;
    }
    remove((tmp + ".kmc_pre").c_str());
  }
  printf("kmc ok (%d corrupt copies parsed, %d refused)\n", ok, refused);
  return 0;
}

int cmd_ttest() {
  std::mt19937_64 rng(13);
  std::normal_distribution<double> nd(0.0, 1.0);
  const double specials[] = {0.0, -0.0, 1e-300, 1e300, std::numeric_limits<double>::infinity(),
                             std::numeric_limits<double>::quiet_NaN(), 5.0};
  for (int rep = 0; rep < 4000; ++rep) {
    const int64_t n = (int64_t)(rng() % 12), m = (int64_t)(rng() % 12);
    std::vector<double> x(std::max<int64_t>(n, 1)), y(std::max<int64_t>(m, 1));
    const int kind = (int)(rng() % 4);
    for (auto* v : {&x, &y})
      for (double& e : *v)
        e = kind == 0 ? nd(rng) : kind == 1 ? 3.0 : kind == 2 ? specials[rng() % 7] : nd(rng) * 1e-8;
    double b = 0, l = 0, r = 0;
    klsh_ttest2(x.data(), n, y.data(), m, &b, &l, &r);
  }
  // WRS over random centroid tables, including n1 or n2 = 0
  for (int rep = 0; rep < 200; ++rep) {
    const int n1 = (int)(rng() % 5), n2 = (int)(rng() % 5);
    const uint64_t nc = rng() % 50;
    std::vector<float> c(std::max<uint64_t>(nc * (n1 + n2), 1));
    for (float& v : c) v = (float)nd(rng);
    std::vector<uint64_t> cnt(std::max<uint64_t>(nc, 1));
    for (auto& v : cnt) v = rng() % 10;
    std::vector<uint8_t> g(std::max<uint64_t>(nc, 1));
    klsh_wrs(c.data(), nc, n1, n2, cnt.data(), 0.05f, 2, g.data());
  }
  printf("ttest ok\n");
  return 0;
}

int cmd_cuckoo() {
  std::mt19937_64 rng(17);
  for (int k = 1; k <= 32; k += 3) {
    const uint64_t space = k >= 32 ? ~0ull : (1ull << (2 * k));
    const uint64_t want = std::min<uint64_t>(space / 2, k == 31 ? 600000 : 20000);
    std::unordered_set<uint64_t> seen;
    std::vector<uint64_t> im;
    while (im.size() < want) {
      const uint64_t v = k >= 32 ? rng() : rng() % space;
      if (seen.insert(v).second) im.push_back(v);
    }
    std::vector<uint32_t> order(im.size());
    const int hp = klsh_cuckoo_order(im.data(), im.size(), k, order.data());
    if (hp < 16) {
      fprintf(stderr, "cuckoo k=%d failed: %s\n", k, klsh_last_error());
      return 1;
    }
    std::vector<uint32_t> sorted = order;
    std::sort(sorted.begin(), sorted.end());
    for (size_t i = 0; i < sorted.size(); ++i)
      if (sorted[i] != i) {
        fprintf(stderr, "cuckoo k=%d: not a permutation\n", k);
        return 1;
      }
  }
  uint32_t none = 0;
  if (klsh_cuckoo_order(nullptr, 0, 21, &none) < 0) return 1;
  printf("cuckoo ok\n");
  return 0;
}

int cmd_rng() {
  for (int d : {1, 3, 8, 64, 513}) {
    uint64_t counter = 5;
    std::vector<float> t((size_t)7 * d);
    if (klsh_hyperplanes(12345u, &counter, 7, d, t.data()) != KLSH_OK || counter != 12) return 1;
  }
  for (int d : {1, 8, 64}) {
    const uint64_t n = 1000;
    std::vector<uint16_t> c(n * d);
    std::vector<double> cov(d);
    if (klsh_synth_counts(n, d, 3, 0, 2, c.data(), cov.data()) != KLSH_OK) return 1;
  }
  printf("rng ok\n");
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: asan_host fastq DIR FILE... | kmc NAME... | ttest | cuckoo | rng\n");
    return 2;
  }
  const std::string cmd = argv[1];
  if (cmd == "fastq" && argc >= 3) return cmd_fastq(argc, argv);
  if (cmd == "kmc") return cmd_kmc(argc, argv);
  if (cmd == "ttest") return cmd_ttest();
  if (cmd == "cuckoo") return cmd_cuckoo();
  if (cmd == "rng") return cmd_rng();
  fprintf(stderr, "unknown command\n");
  return 2;
}
