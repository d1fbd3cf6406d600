// Host check of FastDiv (csrc/common.h): n / d as (umulhi(n, m) + n) >> l for every divisor d < 5000
// (all n < 1000, 20000 sampled n < 2^31 and n = 2^31 - 1) and for the engine's map sizes (2M samples).
// usage: g++ -O2 -std=c++17 tools/fastdiv_check.cpp -o /tmp/fdc && /tmp/fdc   (tests/test_host.py runs it)
#include <cstdint>
#include <cstdio>
#include <random>

struct FastDiv {
  unsigned m;
  int l;
};
// same construction as fast_div() in csrc/common.h
static FastDiv fast_div(unsigned d) {
  int l = 0;
  while ((1u << l) < d) ++l;
  return FastDiv{(unsigned)(((1ull << 32) * ((1ull << l) - d)) / d + 1), l};
}
static unsigned fdiv(unsigned n, FastDiv f) { return (unsigned)((((uint64_t)n * f.m) >> 32) + n) >> f.l; }

int main() {
  std::mt19937 rng(1);
  long bad = 0;
  for (unsigned d = 1; d < 5000; ++d) {
    const FastDiv f = fast_div(d);
    for (int i = 0; i < 21000; ++i) {
      const unsigned n = i < 1000 ? (unsigned)i : (rng() & 0x7fffffffu);
      bad += fdiv(n, f) != n / d;
    }
    bad += fdiv(0x7fffffffu, f) != 0x7fffffffu / d;
  }
  for (unsigned d : {49u, 196u, 784u, 3136u, 12544u, 100352u, 1u << 20, 3000017u}) {
    const FastDiv f = fast_div(d);
    for (int i = 0; i < 2000000; ++i) {
      const unsigned n = rng() & 0x7fffffffu;
      bad += fdiv(n, f) != n / d;
    }
  }
  printf("fastdiv mismatches: %ld\n", bad);
  return bad != 0;
}
