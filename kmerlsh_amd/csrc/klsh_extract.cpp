// Mode E behind the C ABI (include/klsh.h): the differential test of the clusters and the read
// extraction that consumes them (reference app/kmerLSH.cc:521-580).
//
//   klsh_ttest2 / klsh_wrs   AB::WRS (function/funcAB.cc:73-109): per cluster with more than
//                            size_thresh members, ALGLIB's pooled two-sample Student t-test of the
//                            centroid's first n1 samples against the next n2.  Host code: one test
//                            per cluster is microseconds of scalar work.  ALGLIB 3.15.0 (vendored
//                            by the reference, utils/alglib-3.15.0) is restated below in the same
//                            operation order, with glibc's libm, so the p-values are its bits.
//   klsh_fastq_*             FastqFile + the reference's kseq variant (utils/fastq.cc,
//                            kmer/kseq.h:153-200): the exact record rules, gzip or plain.
//   klsh_kset_* /            IOFQ::CheckRead (io/ioFastQ.cc:5-76) on the GPU (klsh_extract.hip):
//   klsh_check_reads         the k-mer set as a device hash table, one wave per read.
//   klsh_extract_fastq       IOFQ::ReadExtract (io/ioFastQ.cc:78-159): parse a batch on the host
//                            while the GPU checks the previous one, write the selected records.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <zlib.h>

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

// ============================================ ALGLIB 3.15.0 restated (Cephes algorithms) ======
// Constants of utils/alglib-3.15.0/src/ap.h:1008-1011.
constexpr double kMachEps = 5E-16, kMaxReal = 1E300, kMinReal = 1E-300;
constexpr double kPi = 3.1415926535897932384626433832795;

// gammafunc_gammastirf, specialfunctions.cpp:3672-3698
double gamma_stirling(double x) {
  double w = 1 / x;
  double stir = 7.87311395793093628397E-4;
  stir = -2.29549961613378126380E-4 + w * stir;
  stir = -2.68132617805781232825E-3 + w * stir;
  stir = 3.47222221605458667310E-3 + w * stir;
  stir = 8.33333333333482257126E-2 + w * stir;
  w = 1 + w * stir;
  double y = std::exp(x);
  if (x > 143.01608) {
    const double v = std::pow(x, 0.5 * x - 0.25);
    y = v * (v / y);
  } else {
    y = std::pow(x, x - 0.5) / y;
  }
  return 2.50662827463100050242 * y * w;
}

// gammafunction, specialfunctions.cpp:3419-3512
double gamma_fn(double x) {
  double sgngam = 1;
  const double q = std::fabs(x);
  if (q > 33.0) {
    double z;
    if (x < 0.0) {
      double p = (double)(int64_t)std::floor(q);
      const int64_t i = (int64_t)std::floor(p + 0.5);
      if (i % 2 == 0) sgngam = -1;
      z = q - p;
      if (z > 0.5) {
        p = p + 1;
        z = q - p;
      }
      z = q * std::sin(kPi * z);
      z = std::fabs(z);
      z = kPi / (z * gamma_stirling(q));
    } else {
      z = gamma_stirling(x);
    }
    return sgngam * z;
  }
  double z = 1;
  while (x >= 3) {
    x = x - 1;
    z = z * x;
  }
  while (x < 0) {
    if (x > -0.000000001) return z / ((1 + 0.5772156649015329 * x) * x);
    z = z / x;
    x = x + 1;
  }
  while (x < 2) {
    if (x < 0.000000001) return z / ((1 + 0.5772156649015329 * x) * x);
    z = z / x;
    x = x + 1.0;
  }
  if (x == 2) return z;
  x = x - 2.0;
  double pp = 1.60119522476751861407E-4;
  pp = 1.19135147006586384913E-3 + x * pp;
  pp = 1.04213797561761569935E-2 + x * pp;
  pp = 4.76367800457137231464E-2 + x * pp;
  pp = 2.07448227648435975150E-1 + x * pp;
  pp = 4.94214826801497100753E-1 + x * pp;
  pp = 9.99999999999999996796E-1 + x * pp;
  double qq = -2.31581873324120129819E-5;
  qq = 5.39605580493303397842E-4 + x * qq;
  qq = -4.45641913851797240494E-3 + x * qq;
  qq = 1.18139785222060435552E-2 + x * qq;
  qq = 3.58236398605498653373E-2 + x * qq;
  qq = -2.34591795718243348568E-1 + x * qq;
  qq = 7.14304917030273074085E-2 + x * qq;
  qq = 1.00000000000000000320 + x * qq;
  return z * pp / qq;
}

// lngamma, specialfunctions.cpp:3548-3662 (the sign output is unused by the callers here)
double lngamma_fn(double x) {
  const double logpi = 1.14472988584940017414, ls2pi = 0.91893853320467274178;
  if (x < -34.0) {
    const double q = -x;
    const double w = lngamma_fn(q);
    double p = (double)(int64_t)std::floor(q);
    double z = q - p;
    if (z > 0.5) {
      p = p + 1;
      z = p - q;
    }
    z = q * std::sin(kPi * z);
    return logpi - std::log(z) - w;
  }
  if (x < 13) {
    double z = 1, p = 0, u = x;
    while (u >= 3) {
      p = p - 1;
      u = x + p;
      z = z * u;
    }
    while (u < 2) {
      z = z / u;
      p = p + 1;
      u = x + p;
    }
    if (z < 0) z = -z;
    if (u == 2) return std::log(z);
    p = p - 2;
    x = x + p;
    double b = -1378.25152569120859100;
    b = -38801.6315134637840924 + x * b;
    b = -331612.992738871184744 + x * b;
    b = -1162370.97492762307383 + x * b;
    b = -1721737.00820839662146 + x * b;
    b = -853555.664245765465627 + x * b;
    double c = 1;
    c = -351.815701436523470549 + x * c;
    c = -17064.2106651881159223 + x * c;
    c = -220528.590553854454839 + x * c;
    c = -1139334.44367982507207 + x * c;
    c = -2532523.07177582951285 + x * c;
    c = -2018891.41433532773231 + x * c;
    p = x * b / c;
    return std::log(z) + p;
  }
  double q = (x - 0.5) * std::log(x) - x + ls2pi;
  if (x > 100000000) return q;
  const double p = 1 / (x * x);
  if (x >= 1000.0) {
    q = q + ((7.9365079365079365079365 * 0.0001 * p - 2.7777777777777777777778 * 0.001) * p +
             0.0833333333333333333333) / x;
  } else {
    double a = 8.11614167470508450300 * 0.0001;
    a = -5.95061904284301438324 * 0.0001 + p * a;
    a = 7.93650340457716943945 * 0.0001 + p * a;
    a = -2.77777777730099687205 * 0.001 + p * a;
    a = 8.33333333333331927722 * 0.01 + p * a;
    q = q + a / x;
  }
  return q;
}

// ibetaf_incompletebetafe / _fe2 (continued fractions), specialfunctions.cpp:7584-7812.
// fe2 is the same recurrence with z = x/(1-x) and the (k2, k6) roles exchanged.
double ibeta_cf(double a, double b, double x, bool second) {
  const double big = 4.503599627370496e15, biginv = 2.22044604925031308085e-16;
  double k1 = a, k2 = second ? b - 1.0 : a + b, k3 = a, k4 = a + 1.0, k5 = 1.0,
         k6 = second ? a + b : b - 1.0, k7 = second ? a + 1.0 : k4, k8 = a + 2.0;
  double pkm2 = 0.0, qkm2 = 1.0, pkm1 = 1.0, qkm1 = 1.0;
  const double z = second ? x / (1.0 - x) : x;
  double ans = 1.0, r = 1.0, t;
  const double thresh = 3.0 * kMachEps;
  int n = 0;
  do {
    double xk = -z * k1 * k2 / (k3 * k4);
    double pk = pkm1 + pkm2 * xk;
    double qk = qkm1 + qkm2 * xk;
    pkm2 = pkm1;
    pkm1 = pk;
    qkm2 = qkm1;
    qkm1 = qk;
    xk = z * k5 * k6 / (k7 * k8);
    pk = pkm1 + pkm2 * xk;
    qk = qkm1 + qkm2 * xk;
    pkm2 = pkm1;
    pkm1 = pk;
    qkm2 = qkm1;
    qkm1 = qk;
    if (qk != 0) r = pk / qk;
    if (r != 0) {
      t = std::fabs((ans - r) / r);
      ans = r;
    } else {
      t = 1.0;
    }
    if (t < thresh) break;
    k1 = k1 + 1.0;
    k2 = second ? k2 - 1.0 : k2 + 1.0;
    k3 = k3 + 2.0;
    k4 = k4 + 2.0;
    k5 = k5 + 1.0;
    k6 = second ? k6 + 1.0 : k6 - 1.0;
    k7 = k7 + 2.0;
    k8 = k8 + 2.0;
    if (std::fabs(qk) + std::fabs(pk) > big) {
      pkm2 = pkm2 * biginv;
      pkm1 = pkm1 * biginv;
      qkm2 = qkm2 * biginv;
      qkm1 = qkm1 * biginv;
    }
    if (std::fabs(qk) < biginv || std::fabs(pk) < biginv) {
      pkm2 = pkm2 * big;
      pkm1 = pkm1 * big;
      qkm2 = qkm2 * big;
      qkm1 = qkm1 * big;
    }
    n = n + 1;
  } while (n != 300);
  return ans;
}

// ibetaf_incompletebetaps (power series), specialfunctions.cpp:7818-7870
double ibeta_ps(double a, double b, double x, double maxgam) {
  const double ai = 1.0 / a;
  double u = (1.0 - b) * x;
  double v = u / (a + 1.0);
  const double t1 = v;
  double t = u, n = 2.0, s = 0.0;
  const double z = kMachEps * ai;
  while (std::fabs(v) > z) {
    u = (n - b) * x / n;
    t = t * u;
    v = t / (a + n);
    s = s + v;
    n = n + 1.0;
  }
  s = s + t1;
  s = s + ai;
  u = a * std::log(x);
  if (a + b < maxgam && std::fabs(u) < std::log(kMaxReal)) {
    t = gamma_fn(a + b) / (gamma_fn(a) * gamma_fn(b));
    s = s * t * std::pow(x, a);
  } else {
    t = lngamma_fn(a + b) - lngamma_fn(a) - lngamma_fn(b) + u + std::log(s);
    s = t < std::log(kMinReal) ? 0.0 : std::exp(t);
  }
  return s;
}

// incompletebeta, specialfunctions.cpp:6975-7096
double incomplete_beta(double a, double b, double x) {
  const double maxgam = 171.624376956302725;
  const double minlog = std::log(kMinReal), maxlog = std::log(kMaxReal);
  if (x == 0) return 0;
  if (x == 1) return 1;
  if (b * x <= 1.0 && x <= 0.95) return ibeta_ps(a, b, x, maxgam);
  double w = 1.0 - x, xc, t;
  int flag = 0;
  if (x > a / (a + b)) {
    flag = 1;
    t = a;
    a = b;
    b = t;
    xc = x;
    x = w;
  } else {
    xc = w;
  }
  if ((flag == 1 && b * x <= 1.0) && x <= 0.95) {
    t = ibeta_ps(a, b, x, maxgam);
    return t <= kMachEps ? 1.0 - kMachEps : 1.0 - t;
  }
  double y = x * (a + b - 2.0) - (a - 1.0);
  w = y < 0.0 ? ibeta_cf(a, b, x, false) : ibeta_cf(a, b, x, true) / xc;
  y = a * std::log(x);
  t = b * std::log(xc);
  if ((a + b < maxgam && std::fabs(y) < maxlog) && std::fabs(t) < maxlog) {
    t = std::pow(xc, b);
    t = t * std::pow(x, a);
    t = t / a;
    t = t * w;
    t = t * (gamma_fn(a + b) / (gamma_fn(a) * gamma_fn(b)));
    if (flag == 1) return t <= kMachEps ? 1.0 - kMachEps : 1.0 - t;
    return t;
  }
  y = y + t + lngamma_fn(a + b) - lngamma_fn(a) - lngamma_fn(b);
  y = y + std::log(w / a);
  t = y < minlog ? 0.0 : std::exp(y);
  if (flag == 1) t = t <= kMachEps ? 1.0 - kMachEps : 1.0 - t;
  return t;
}

// studenttdistribution, specialfunctions.cpp:9559-9630
double student_t_cdf(int64_t k, double t) {
  if (t == 0) return 0.5;
  if (t < -2.0) {
    const double rk = (double)k;
    const double z = rk / (rk + t * t);
    return 0.5 * incomplete_beta(0.5 * rk, 0.5, z);
  }
  const double x = t < 0 ? -t : t;
  const double rk = (double)k;
  const double z = 1.0 + x * x / rk;
  double p, f, tz;
  if (k % 2 != 0) {
    const double xsqk = x / std::sqrt(rk);
    p = std::atan(xsqk);
    if (k > 1) {
      f = 1.0;
      tz = 1.0;
      int64_t j = 3;
      while (j <= k - 2 && tz / f > kMachEps) {
        tz = tz * ((j - 1) / (z * j));
        f = f + tz;
        j = j + 2;
      }
      p = p + f * xsqk / z;
    }
    p = p * 2.0 / kPi;
  } else {
    f = 1.0;
    tz = 1.0;
    int64_t j = 2;
    while (j <= k - 2 && tz / f > kMachEps) {
      tz = tz * ((j - 1) / (z * j));
      f = f + tz;
      j = j + 2;
    }
    p = f * x / std::sqrt(z * rk);
  }
  if (t < 0) p = -p;
  return 0.5 + 0.5 * p;
}

// studentttest2, statistics.cpp:12502-12620
void student_t_test2(const double* x, int64_t n, const double* y, int64_t m, double* both,
                     double* left, double* right) {
  if (n <= 0 || m <= 0) {
    *both = *left = *right = 1.0;
    return;
  }
  double xmean = 0, ymean = 0;
  const double x0 = x[0], y0 = y[0];
  bool samex = true, samey = true;
  for (int64_t i = 0; i < n; ++i) {
    xmean = xmean + x[i];
    samex = samex && x[i] == x0;
  }
  xmean = samex ? x0 : xmean / n;
  for (int64_t i = 0; i < m; ++i) {
    ymean = ymean + y[i];
    samey = samey && y[i] == y0;
  }
  ymean = samey ? y0 : ymean / m;
  double s = 0;
  if (n + m > 2) {
    for (int64_t i = 0; i < n; ++i) s = s + (x[i] - xmean) * (x[i] - xmean);
    for (int64_t i = 0; i < m; ++i) s = s + (y[i] - ymean) * (y[i] - ymean);
    s = std::sqrt(s * ((double)1 / (double)n + (double)1 / (double)m) / (n + m - 2));
  }
  if (s == 0) {
    *both = xmean == ymean ? 1.0 : 0.0;
    *left = xmean >= ymean ? 1.0 : 0.0;
    *right = xmean <= ymean ? 1.0 : 0.0;
    return;
  }
  const double stat = (xmean - ymean) / s;
  const double p = student_t_cdf(n + m - 2, stat);
  *both = 2 * (p > 1 - p ? 1 - p : p);
  *left = p;
  *right = 1 - p;
}

// ============================================================ FASTQ (the reference's kseq) ====
// kmer/kseq.h:60-200 as the reference uses it: the name is the whole header line after '@'/'>'
// (up to '\n'); sequence characters are the isgraph() ones up to the next '>', '+' or '@'; the
// quality is the next seq.l characters in [33, 127] after the '+' line, plus one more character
// consumed; a record whose quality is short ends the file (-2).  Characters are read as signed
// chars, so a 0xFF byte reads as end of input where the reference compares with -1.
struct FastqReader {
  gzFile fp = nullptr;
  std::vector<char> buf;
  int begin = 0, end = 0;
  bool is_eof = false;
  int last_char = 0;
  bool done = false;

  // batch storage (reader-owned; valid until the next batch)
  std::vector<char> seq, name, qual;
  std::vector<uint64_t> seq_off, name_off, qual_off;

  bool open(const char* path) {
    fp = gzopen(path, "r");
    if (!fp) return false;
    (void)gzbuffer(fp, 1 << 20);
    buf.resize(1 << 20);
    return true;
  }
  ~FastqReader() {
    if (fp) gzclose(fp);
  }
  bool fill() {
    if (is_eof) return false;
    begin = 0;
    end = gzread(fp, buf.data(), (unsigned)buf.size());
    if (end < (int)buf.size()) is_eof = true;  // a short read is the end (ks_getc)
    if (end < 0) end = 0;
    return end > 0;
  }
  int getc() {  // ks_getc, kseq.h:60-68
    if (is_eof && begin >= end) return -1;
    if (begin >= end && !fill()) return -1;
    return (int)(signed char)buf[begin++];
  }
  // one record appended to the batch: >= 0 (its sequence length), -1 end, -2 truncated
  int next() {  // kseq_read, kseq.h:153-200
    int c;
    if (last_char == 0) {
      while ((c = getc()) != -1 && c != '>' && c != '@') {
      }
      if (c == -1) return -1;
      last_char = c;
    }
    // name: ks_getuntil(ks, '\n', ...) — -1 only when nothing is left
    if (begin >= end && is_eof) return -1;
    const size_t n0 = name.size(), s0 = seq.size(), q0 = qual.size();
    while (true) {
      if (begin >= end && !fill()) break;
      const char* b = buf.data() + begin;
      const void* nl = memchr(b, '\n', (size_t)(end - begin));
      const int stop = nl ? (int)((const char*)nl - buf.data()) : end;
      name.insert(name.end(), b, (const char*)buf.data() + stop);
      begin = stop + (nl ? 1 : 0);
      if (nl) break;
    }
    // (a header line ending at EOF would read a comment here: nothing is left to read)
    while ((c = getc()) != -1 && c != '>' && c != '+' && c != '@')
      if (c >= 33 && c <= 126) seq.push_back((char)c);  // isgraph in the C locale
    if (c == '>' || c == '@') last_char = c;
    const size_t sl = seq.size() - s0;
    if (c != '+') {  // no quality: the reference would copy a stale buffer; we keep it empty
      commit();
      return (int)sl;
    }
    while ((c = getc()) != -1 && c != '\n') {
    }
    if (c == -1) {
      rollback(n0, s0, q0);
      return -2;
    }
    size_t ql = 0;
    while ((c = getc()) != -1 && ql < sl)
      if (c >= 33 && c <= 127) {
        qual.push_back((char)c);
        ++ql;
      }
    last_char = 0;
    if (sl != ql) {
      rollback(n0, s0, q0);
      return -2;
    }
    commit();
    return (int)sl;
  }
  void commit() {
    seq_off.push_back(seq.size());
    name_off.push_back(name.size());
    qual_off.push_back(qual.size());
  }
  void rollback(size_t n0, size_t s0, size_t q0) {
    name.resize(n0);
    seq.resize(s0);
    qual.resize(q0);
  }
  // up to max_reads records (or until ~max_bases sequence bytes): FastqFile::read
  // (utils/fastq.cc:54-67) with larger parts — part boundaries change nothing downstream
  uint64_t batch(uint64_t max_reads, uint64_t max_bases) {
    seq.clear();
    name.clear();
    qual.clear();
    seq_off.assign(1, 0);
    name_off.assign(1, 0);
    qual_off.assign(1, 0);
    uint64_t n = 0;
    while (!done && n < max_reads && seq.size() < max_bases) {
      if (next() < 0) {
        done = true;  // -1 (end) and -2 (truncated record) both end the file (fastq.cc:59-66)
        break;
      }
      ++n;
    }
    return n;
  }
};

}  // namespace

struct klsh_fastq {
  FastqReader r;
};

struct klsh_kset {
  klsh_ctx* ctx = nullptr;
  uint64_t* tab = nullptr;
  uint64_t mask = 0;
  uint64_t n = 0;
};

#define KLSH_XHIP(call)                                                          \
  do {                                                                           \
    hipError_t e_ = (call);                                                      \
    if (e_ != hipSuccess)                                                        \
      return set_error(KLSH_E_HIP, (std::string(#call) + " -> " + hipGetErrorString(e_)).c_str()); \
  } while (0)

extern "C" {

int klsh_ttest2(const double* x, int64_t n, const double* y, int64_t m, double* bothtails,
                double* lefttail, double* righttail) {
  if ((n > 0 && !x) || (m > 0 && !y) || !bothtails || !lefttail || !righttail)
    return set_error(KLSH_E_ARG, "null argument");
  student_t_test2(x, n, y, m, bothtails, lefttail, righttail);
  return KLSH_OK;
}

int klsh_wrs(const float* centroids, uint64_t n_clusters, int n1, int n2,
             const uint64_t* member_counts, float pvalue_thresh, int size_thresh, uint8_t* group) {
  if ((n_clusters && (!centroids || !member_counts || !group)) || n1 < 0 || n2 < 0)
    return set_error(KLSH_E_ARG, "bad argument");
  const int d = n1 + n2;
  std::vector<double> x(n1 > 0 ? n1 : 1), y(n2 > 0 ? n2 : 1);
  for (uint64_t c = 0; c < n_clusters; ++c) {
    group[c] = 0;
    // ids.size() > size_thresh, compared as size_t against the int (funcAB.cc:85)
    if (!(member_counts[c] > (uint64_t)(int64_t)size_thresh)) continue;
    const float* v = centroids + c * (uint64_t)d;
    for (int i = 0; i < n1; ++i) x[i] = (double)v[i];
    for (int j = 0; j < n2; ++j) y[j] = (double)v[n1 + j];
    double both, left, right;
    student_t_test2(x.data(), n1, y.data(), n2, &both, &left, &right);
    // float threshold promoted to double in the comparisons (funcAB.cc:102-106)
    if (left <= (double)pvalue_thresh) group[c] = 2;
    else if (right <= (double)pvalue_thresh) group[c] = 1;
  }
  return KLSH_OK;
}

klsh_fastq* klsh_fastq_open(const char* path, int* err) {
  if (err) *err = KLSH_OK;
  if (!path) {
    set_error(KLSH_E_ARG, "null path");
    if (err) *err = KLSH_E_ARG;
    return nullptr;
  }
  klsh_fastq* f = new klsh_fastq();
  if (!f->r.open(path)) {
    delete f;
    set_error(KLSH_E_ARG, (std::string("cannot open ") + path).c_str());
    if (err) *err = KLSH_E_ARG;
    return nullptr;
  }
  return f;
}

int64_t klsh_fastq_next(klsh_fastq* f, uint64_t max_reads, const char** seq,
                        const uint64_t** seq_off, const char** name, const uint64_t** name_off,
                        const char** qual, const uint64_t** qual_off) {
  if (!f) return set_error(KLSH_E_ARG, "null reader");
  const uint64_t n = f->r.batch(max_reads ? max_reads : 1, ~0ull);
  if (seq) *seq = f->r.seq.data();
  if (seq_off) *seq_off = f->r.seq_off.data();
  if (name) *name = f->r.name.data();
  if (name_off) *name_off = f->r.name_off.data();
  if (qual) *qual = f->r.qual.data();
  if (qual_off) *qual_off = f->r.qual_off.data();
  return (int64_t)n;
}

void klsh_fastq_close(klsh_fastq* f) { delete f; }

klsh_kset* klsh_kset_create(klsh_ctx* ctx, const uint64_t* kmers, uint64_t n, int* err) {
  auto bad = [&](int e) -> klsh_kset* {
    if (err) *err = e;
    return nullptr;
  };
  if (!ctx || (n && !kmers)) return bad(set_error(KLSH_E_ARG, "null argument"));
  if (hipSetDevice(klsh::ctx_device(ctx)) != hipSuccess) return bad(set_error(KLSH_E_HIP, "hipSetDevice"));
  const hipStream_t s = klsh::ctx_stream(ctx);
  uint64_t cap = 1024;
  while (cap < 2 * n) cap <<= 1;  // load factor <= 1/2
  klsh_kset* ks = new klsh_kset();
  ks->ctx = ctx;
  ks->mask = cap - 1;
  ks->n = n;
  uint64_t* dk = nullptr;
  bool ok = hipMalloc((void**)&ks->tab, cap * 8) == hipSuccess;
  ok = ok && (n == 0 || hipMalloc((void**)&dk, n * 8) == hipSuccess);
  ok = ok && hipMemsetAsync(ks->tab, 0xFF, cap * 8, s) == hipSuccess;
  ok = ok && (n == 0 || hipMemcpyAsync(dk, kmers, n * 8, hipMemcpyHostToDevice, s) == hipSuccess);
  if (ok) {
    klsh::launch_kset_insert(dk, n, ks->tab, ks->mask, s);
    ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(s) == hipSuccess;
  }
  if (dk) (void)hipFree(dk);
  if (!ok) {
    if (ks->tab) (void)hipFree(ks->tab);
    delete ks;
    return bad(set_error(KLSH_E_NOMEM, "k-mer set allocation / upload failed"));
  }
  if (err) *err = KLSH_OK;
  return ks;
}

void klsh_kset_destroy(klsh_kset* ks) {
  if (!ks) return;
  (void)hipSetDevice(klsh::ctx_device(ks->ctx));
  if (ks->tab) (void)hipFree(ks->tab);
  delete ks;
}

int klsh_check_reads(klsh_ctx* ctx, const klsh_kset* ks, const char* seq,
                     const uint64_t* read_offsets, uint64_t n_reads, int k, float kmer_vote,
                     uint32_t* hits, uint8_t* flags) {
  if (!ctx || !ks || ks->ctx != ctx || (n_reads && (!seq || !read_offsets || !flags)))
    return set_error(KLSH_E_ARG, "bad argument");
  if (k < 1 || k > 32) return set_error(KLSH_E_RANGE, "k must be in [1, 32] (Kmer::MAX_K)");
  if (n_reads == 0) return KLSH_OK;
  KLSH_XHIP(hipSetDevice(klsh::ctx_device(ctx)));
  const hipStream_t s = klsh::ctx_stream(ctx);
  const uint64_t nb = read_offsets[n_reads] - read_offsets[0];
  std::vector<uint64_t> off(read_offsets, read_offsets + n_reads + 1);
  for (auto& o : off) o -= read_offsets[0];
  uint8_t *dseq = nullptr, *dflag = nullptr;
  uint64_t* doff = nullptr;
  uint32_t* dhit = nullptr;
  bool ok = hipMalloc((void**)&dseq, nb + 64) == hipSuccess &&
            hipMalloc((void**)&doff, (n_reads + 1) * 8) == hipSuccess &&
            hipMalloc((void**)&dhit, n_reads * 4) == hipSuccess &&
            hipMalloc((void**)&dflag, n_reads) == hipSuccess;
  ok = ok && hipMemcpyAsync(dseq, seq + read_offsets[0], nb, hipMemcpyHostToDevice, s) == hipSuccess &&
       hipMemcpyAsync(doff, off.data(), off.size() * 8, hipMemcpyHostToDevice, s) == hipSuccess;
  if (ok) {
    klsh::launch_check_reads(dseq, doff, n_reads, k, kmer_vote, ks->tab, ks->mask, dhit, dflag, s);
    ok = hipGetLastError() == hipSuccess;
  }
  ok = ok && (!hits || hipMemcpyAsync(hits, dhit, n_reads * 4, hipMemcpyDeviceToHost, s) == hipSuccess) &&
       hipMemcpyAsync(flags, dflag, n_reads, hipMemcpyDeviceToHost, s) == hipSuccess &&
       hipStreamSynchronize(s) == hipSuccess;
  (void)hipFree(dseq);
  (void)hipFree(doff);
  (void)hipFree(dhit);
  (void)hipFree(dflag);
  if (!ok) return set_error(KLSH_E_HIP, "check_reads: allocation, copy or launch failed");
  return KLSH_OK;
}

int klsh_extract_fastq(klsh_ctx* ctx, const klsh_kset* ks, const char* in_path,
                       const char* out_path, int k, float kmer_vote, klsh_extract_stats* st) {
  if (!ctx || !ks || ks->ctx != ctx || !in_path || !out_path)
    return set_error(KLSH_E_ARG, "bad argument");
  if (k < 1 || k > 32) return set_error(KLSH_E_RANGE, "k must be in [1, 32] (Kmer::MAX_K)");
  const double t_start = now_ms();
  if (st && st->struct_size != sizeof(klsh_extract_stats))
    return set_error(KLSH_E_ARG, "klsh_extract_stats.struct_size != sizeof: built against another klsh.h");
  klsh_extract_stats local{};
  local.struct_size = sizeof(local);
  KLSH_XHIP(hipSetDevice(klsh::ctx_device(ctx)));
  const hipStream_t s = klsh::ctx_stream(ctx);
  FastqReader rdr;
  if (!rdr.open(in_path)) return set_error(KLSH_E_ARG, (std::string("cannot open ") + in_path).c_str());
  FILE* of = fopen(out_path, "wb");
  if (!of) return set_error(KLSH_E_ARG, (std::string("cannot open for writing ") + out_path).c_str());
  // Two batch slots: the host parses batch i+1 (slot (i+1)&1) while the GPU checks batch i.
  constexpr uint64_t kReads = 1u << 18, kBases = 64ull << 20;
  struct Slot {
    uint8_t* dseq = nullptr;
    uint64_t* doff = nullptr;
    uint32_t* dhit = nullptr;
    uint8_t* dflag = nullptr;
    uint8_t* hflag = nullptr;
    uint64_t cap_b = 0;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    hipEvent_t done = nullptr;  // after the flag copy: finish() waits for this batch only
    uint64_t n = 0;
  } slot[2];
  int rc = KLSH_OK;
  auto cleanup = [&]() {
    for (auto& sl : slot) {
      if (sl.dseq) (void)hipFree(sl.dseq);
      if (sl.doff) (void)hipFree(sl.doff);
      if (sl.dhit) (void)hipFree(sl.dhit);
      if (sl.dflag) (void)hipFree(sl.dflag);
      if (sl.hflag) (void)hipHostFree(sl.hflag);
      if (sl.e0) (void)hipEventDestroy(sl.e0);
      if (sl.e1) (void)hipEventDestroy(sl.e1);
      if (sl.done) (void)hipEventDestroy(sl.done);
    }
  };
  for (auto& sl : slot) {
    bool ok = hipMalloc((void**)&sl.doff, (kReads + 1) * 8) == hipSuccess &&
              hipMalloc((void**)&sl.dhit, kReads * 4) == hipSuccess &&
              hipMalloc((void**)&sl.dflag, kReads) == hipSuccess &&
              hipHostMalloc((void**)&sl.hflag, kReads, hipHostMallocDefault) == hipSuccess &&
              hipEventCreate(&sl.e0) == hipSuccess && hipEventCreate(&sl.e1) == hipSuccess &&
              hipEventCreateWithFlags(&sl.done, hipEventDisableTiming) == hipSuccess;
    if (!ok) {
      cleanup();
      fclose(of);
      return set_error(KLSH_E_NOMEM, "extract: batch buffers");
    }
  }
  // The reader parses every batch; its storage is swapped into a per-slot copy so the next parse
  // can proceed while the previous batch's records wait for their flags.
  FastqReader keep[2];
  std::vector<char> out;
  out.reserve(1 << 22);
  auto launch = [&](int si) -> int {
    Slot& sl = slot[si];
    FastqReader& b = keep[si];
    sl.n = b.seq_off.size() - 1;
    const uint64_t nb = b.seq.size();
    if (nb + 64 > sl.cap_b) {
      if (sl.dseq) (void)hipFree(sl.dseq);
      sl.dseq = nullptr;
      sl.cap_b = nb + 64 > kBases + (64u << 10) ? nb + 64 : kBases + (64u << 10);
      KLSH_XHIP(hipMalloc((void**)&sl.dseq, sl.cap_b));
    }
    if (nb) KLSH_XHIP(hipMemcpyAsync(sl.dseq, b.seq.data(), nb, hipMemcpyHostToDevice, s));
    KLSH_XHIP(hipMemcpyAsync(sl.doff, b.seq_off.data(), (sl.n + 1) * 8, hipMemcpyHostToDevice, s));
    KLSH_XHIP(hipEventRecord(sl.e0, s));
    klsh::launch_check_reads(sl.dseq, sl.doff, sl.n, k, kmer_vote, ks->tab, ks->mask, sl.dhit,
                             sl.dflag, s);
    KLSH_XHIP(hipGetLastError());
    KLSH_XHIP(hipEventRecord(sl.e1, s));
    KLSH_XHIP(hipMemcpyAsync(sl.hflag, sl.dflag, sl.n, hipMemcpyDeviceToHost, s));
    KLSH_XHIP(hipEventRecord(sl.done, s));
    return KLSH_OK;
  };
  auto finish = [&](int si) -> int {
    Slot& sl = slot[si];
    FastqReader& b = keep[si];
    KLSH_XHIP(hipEventSynchronize(sl.e1));
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, sl.e0, sl.e1);
    local.kernel_ms += ms;
    // the flag copy behind this batch's kernel — not the stream, which by now also holds the next
    // batch: waiting for that would serialise the host parse behind every kernel
    KLSH_XHIP(hipEventSynchronize(sl.done));
    out.clear();
    for (uint64_t i = 0; i < sl.n; ++i) {
      const uint64_t len = b.seq_off[i + 1] - b.seq_off[i];
      if (len == 0) {  // io/ioFastQ.cc:20-24
        printf("\nabnormal read entry skipped\n");
        fwrite(b.name.data() + b.name_off[i], 1, b.name_off[i + 1] - b.name_off[i], stdout);
        printf("\n");
        local.abnormal += 1;
        continue;
      }
      if (len >= (uint64_t)k + 10u) {
        local.reads_tested += 1;
        local.kmers_checked += len - (uint64_t)k + 1u;
      }
      if (!sl.hflag[i]) continue;
      local.reads_extracted += 1;
      // "@name\nseq\n+\nqual\n" (io/ioFastQ.cc:110-128)
      out.push_back('@');
      out.insert(out.end(), b.name.data() + b.name_off[i], b.name.data() + b.name_off[i + 1]);
      out.push_back('\n');
      out.insert(out.end(), b.seq.data() + b.seq_off[i], b.seq.data() + b.seq_off[i + 1]);
      out.push_back('\n');
      out.push_back('+');
      out.push_back('\n');
      out.insert(out.end(), b.qual.data() + b.qual_off[i], b.qual.data() + b.qual_off[i + 1]);
      out.push_back('\n');
    }
    if (!out.empty() && fwrite(out.data(), 1, out.size(), of) != out.size())
      return set_error(KLSH_E_ARG, "extract: write failed");
    return KLSH_OK;
  };
  int cur = 0;
  bool pending = false;
  while (true) {
    const double tp = now_ms();
    const uint64_t n = rdr.batch(kReads, kBases);
    local.parse_ms += now_ms() - tp;
    if (n > 0) {
      std::swap(keep[cur].seq, rdr.seq);
      std::swap(keep[cur].seq_off, rdr.seq_off);
      std::swap(keep[cur].name, rdr.name);
      std::swap(keep[cur].name_off, rdr.name_off);
      std::swap(keep[cur].qual, rdr.qual);
      std::swap(keep[cur].qual_off, rdr.qual_off);
      local.reads += n;
      local.bases += keep[cur].seq.size();
      if ((rc = launch(cur))) break;
    }
    if (pending && (rc = finish(cur ^ 1))) break;  // the previous batch, while this one runs
    pending = n > 0;
    if (n == 0) break;
    cur ^= 1;
  }
  if (rc == KLSH_OK && pending) rc = finish(cur);
  cleanup();
  if (fclose(of) != 0 && rc == KLSH_OK) rc = set_error(KLSH_E_ARG, "extract: close failed");
  local.total_ms = now_ms() - t_start;
  if (st) *st = local;
  return rc;
}

}  // extern "C"
