// Loads a uid,sid CSV with frecsys::Dataset and prints its tuples and CSR
// checksums (tests/test_dataset_cpu.py compares thread counts and Python).
#include <cstdio>
#include <cstdint>

#include "frecsys/dataset.h"

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  frecsys::Dataset d(argv[1]);
  uint64_t h = 1469598103934665603ull;
  auto mix = [&](int64_t v) { h = (h ^ (uint64_t)v) * 1099511628211ull; };
  for (int k = 0; k < d.num_tuples(); ++k) {
    mix(d.users()[k]);
    mix(d.items()[k]);
  }
  const frecsys::Csr& u = d.user_csr();
  for (int64_t x : u.ptr) mix(x);
  for (int32_t x : u.col) mix(x);
  printf("%d %d %d %llu\n", d.num_tuples(), d.max_user(), d.max_item(), (unsigned long long)h);
  return 0;
}
