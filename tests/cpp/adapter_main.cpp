// Drives include/klsh_cluster.hpp (the reference-signature adapter) the way the reference's
// app/kmerLSH.cc would: a vector<Abundance*> in, Cluster(...) in place, results written out.
//   adapter_main ROWS.f32 N D MINSIM ITERS BTHR OUT.f32 OUT.clust
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "klsh_cluster.hpp"

#ifdef KLSH_REF_ABUNDANCE  // the reference's own data model, included in place (-D path)
#include KLSH_REF_ABUNDANCE
using Abundance = Core::Abundance;
#else
struct Abundance {  // same public members as the reference's Core::Abundance
  std::vector<float> _values;
  std::vector<uint64_t> _ids;
};
#endif

int main(int argc, char** argv) {
  if (argc < 9) return 1;
  const size_t n = strtoull(argv[2], nullptr, 10);
  const int d = atoi(argv[3]);
  std::vector<float> x(n * d);
  FILE* f = fopen(argv[1], "rb");
  if (!f || fread(x.data(), 4, x.size(), f) != x.size()) return 2;
  fclose(f);
  std::vector<Abundance*> v;
  for (size_t i = 0; i < n; ++i) {
    Abundance* a = new Abundance();
    a->_values.assign(x.begin() + i * d, x.begin() + (i + 1) * d);
    a->_ids.push_back(i);
    v.push_back(a);
  }
  klsh::Cluster(&v, (float)atof(argv[4]), atoi(argv[5]), 1, d, atoi(argv[6]), false);
  FILE* fo = fopen(argv[7], "wb");
  FILE* fc = fopen(argv[8], "wb");
  for (Abundance* a : v) {
    fwrite(a->_values.data(), 4, d, fo);
    fprintf(fc, "%zu", a->_ids.size());
    for (uint64_t id : a->_ids) fprintf(fc, "\t%llu", (unsigned long long)id);
    fputc('\n', fc);
    delete a;
  }
  fclose(fo);
  fclose(fc);
  return 0;
}
