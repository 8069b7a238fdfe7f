// Sanitizer driver for the engine's host staging pool (engine/csrc/staging_core.h), no Python:
// built with -fsanitize=thread and with -fsanitize=address,undefined by
// tests/test_native_sanitizers.py.  Several submitter threads share one pool (the batcher's
// executor threads sharing an engine) and hammer gather() with batches of varying shape; every
// destination byte is checked after each call, and pools are created / destroyed repeatedly
// (late-waking workers, shutdown while idle).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "../../mlmicroservicetemplate_amd/engine/csrc/staging_core.h"

static int check_batch(mls_staging::Stager& st, std::mt19937& rng, int iters) {
  for (int it = 0; it < iters; ++it) {
    const size_t n = 1 + rng() % 12;
    const size_t each = 1 + rng() % (700 * 1024);  // crosses the 256 KiB chunk size both ways
    std::vector<std::vector<unsigned char>> srcs(n, std::vector<unsigned char>(each));
    std::vector<uintptr_t> ptrs;
    for (auto& s : srcs) {
      const unsigned char v = static_cast<unsigned char>(rng());
      for (size_t i = 0; i < each; i += 4096) s[i] = static_cast<unsigned char>(v + i / 4096);
      s[each - 1] = v ^ 0x5a;
      ptrs.push_back(reinterpret_cast<uintptr_t>(s.data()));
    }
    std::vector<unsigned char> dst(n * each + 64, 0xee);
    st.gather(reinterpret_cast<uintptr_t>(dst.data()), ptrs, each);
    for (size_t r = 0; r < n; ++r)
      if (std::memcmp(dst.data() + r * each, srcs[r].data(), each) != 0) return 1;
    for (size_t i = n * each; i < dst.size(); ++i)
      if (dst[i] != 0xee) return 2;  // nothing written past the batch
  }
  return 0;
}

int main() {
  int failures = 0;
  for (int round = 0; round < 3; ++round) {
    mls_staging::Stager st(round + 1);  // 1, 2, 3 pool threads
    std::vector<std::thread> ts;
    std::vector<int> rc(4, 0);
    for (int t = 0; t < 4; ++t)
      ts.emplace_back([&, t] {
        std::mt19937 rng(1234 + 17 * t + round);
        rc[t] = check_batch(st, rng, 40);
      });
    for (auto& t : ts) t.join();
    for (int r : rc) failures += r != 0;
  }
  {
    mls_staging::Stager idle(4);  // destroyed without ever being used
  }
  mls_staging::Stager none(0);  // caller-only copies
  std::mt19937 rng(7);
  failures += check_batch(none, rng, 10) != 0;
  std::printf("staging sanitize: %s\n", failures ? "FAIL" : "ok");
  return failures ? 1 : 0;
}
