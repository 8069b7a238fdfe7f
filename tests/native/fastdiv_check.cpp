// Host check of ops/csrc/fastdiv.h against the `/` operator (tests/test_fastdiv.py).
#include <cstdio>
#include <cstdlib>
#include <random>

#include "fastdiv.h"

static int check(uint32_t d, uint32_t n) {
  const uint32_t q = fastdiv(n, fastdiv_make(d));
  if (q != n / d) {
    std::printf("MISMATCH d=%u n=%u got=%u want=%u\n", d, n, q, n / d);
    return 1;
  }
  return 0;
}

int main() {
  int bad = 0;
  std::mt19937_64 rng(1234);
  // every n < 2^16 for small divisors (the kernels' pixel / row / item geometry)
  for (uint32_t d = 1; d <= 2048 && !bad; ++d)
    for (uint32_t n = 0; n < 65536u && !bad; ++n) bad |= check(d, n);
  // around multiples of d up to 2^32 - 1, and random divisors up to 2^31
  for (int it = 0; it < 2000000 && !bad; ++it) {
    const uint32_t d = it & 1 ? (uint32_t)(rng() % 100000u) + 1u : (uint32_t)(rng() % (1u << 31)) + 1u;
    const uint64_t k = rng() % ((0xffffffffull / d) + 1);
    const uint64_t base = k * d;
    for (int o = -1; o <= 1 && !bad; ++o) {
      const int64_t n = (int64_t)base + o;
      if (n >= 0 && n <= 0xffffffffll) bad |= check(d, (uint32_t)n);
    }
    bad |= check(d, 0xffffffffu);
  }
  for (uint32_t s = 0; s < 31 && !bad; ++s) bad |= check(1u << s, 0xffffffffu) | check((1u << s) + 1u, 0xfffffffeu);
  if (bad) return 1;
  std::printf("fastdiv: ok\n");
  return 0;
}
