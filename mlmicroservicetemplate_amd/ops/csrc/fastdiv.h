// Division by a launch-constant divisor as a multiply-high and three shifts/adds (Granlund &
// Montgomery's round-up method with a 33-bit multiplier), exact for every 32-bit unsigned n and
// 1 <= d < 2^31.  hipcc lowers `n / d` with a runtime d to a ~30-instruction v_rcp_iflag_f32 sequence;
// the kernels' prologues (per-lane pixel -> (image, row, column) geometry) and per-item decodes did a
// dozen of those before their first DMA.  The host builds the FastDiv once per launch and passes it
// in the kernel arguments (two SGPRs; the divisor itself stays a separate field where it is needed).
//
// Plain C++ on purpose: tests/native/fastdiv_check.cpp compiles this header with the host compiler and
// checks it exhaustively against `/` (tests/test_fastdiv.py).
#pragma once
#include <stdint.h>

#if defined(__HIP__)
#define MLS_FD_FN __host__ __device__ __forceinline__
#else
#define MLS_FD_FN inline
#endif

struct FastDiv {
  uint32_t m;   // floor(2^32 * (2^l - d) / d) + 1, l = ceil(log2 d)
  uint32_t sh;  // min(l, 1) << 8 | max(l - 1, 0)
};

inline FastDiv fastdiv_make(uint32_t d) {
  uint32_t l = 0;
  while (l < 32 && (1ull << l) < d) ++l;
  FastDiv f;
  f.m = (uint32_t)(((1ull << 32) * ((1ull << l) - d)) / d + 1);
  f.sh = (l ? 1u : 0u) << 8 | (l ? l - 1 : 0u);
  return f;
}

// n / d
MLS_FD_FN uint32_t fastdiv(uint32_t n, FastDiv f) {
  const uint32_t t = (uint32_t)(((uint64_t)n * f.m) >> 32);
  return (t + ((n - t) >> (f.sh >> 8))) >> (f.sh & 0xffu);
}
MLS_FD_FN int fastdiv(int n, FastDiv f) { return (int)fastdiv((uint32_t)n, f); }
