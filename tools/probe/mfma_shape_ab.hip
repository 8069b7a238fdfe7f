// MFMA shape A/B on gfx950: v_mfma_f32_16x16x32_bf16 vs v_mfma_f32_32x32x16_bf16 at the SAME wave
// tile (64 x 64 outputs per wave, 64 fp32 accumulators per lane) and the same LDS fragment traffic
// (8 ds_read_b128 per wave per 32-deep k-step for either shape), on random bf16 operands.
// Question (VERDICT r3 "A second MFMA shape"): does 32x32x16 run the projection / conv k-loops
// faster?  Per k32-step a wave issues 16 x 16x16x32 (16 cycles each) or 8 x 32x32x16 (32 cycles
// each) = 256 MFMA cycles either way; the LDS bytes per FLOP are set by the wave tile, not the shape.
//
// Build + run (one GPU):  hipcc -O3 --offload-arch=gfx950 -o /tmp/mfma_ab tools/probe/mfma_shape_ab.hip && /tmp/mfma_ab
// Prints one JSON line per (shape, operand source, waves per SIMD).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int KSTEPS = 4096;       // 32-deep k-steps per wave
constexpr int LDS_ROWS = 128;      // operand image rows (64 A + 64 B), 64 B (32 bf16) each... x8 k-steps
constexpr int LDS_KS = 8;          // distinct k-steps held in LDS (cycled)
constexpr int LDS_BYTES = LDS_KS * LDS_ROWS * 64;

// SHAPE 0: 16x16x32, SHAPE 1: 32x32x16.  FROM_LDS: re-read every fragment from LDS each k-step.
template <int SHAPE, bool FROM_LDS>
__global__ __launch_bounds__(512) void mfma_loop(const __bf16* __restrict__ src, float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < LDS_BYTES / 16; i += blockDim.x)
    reinterpret_cast<uint4*>(lds)[i] = reinterpret_cast<const uint4*>(src)[(blockIdx.x * 7 + i) % (LDS_BYTES / 16)];
  __syncthreads();
  // a fragment read: 16 B per lane from a 64-B row of k-step `ks`; rows swizzled so the 16-lane groups
  // of ds_read_b128 hit distinct banks (row r, chunk c -> c ^ (r & 3))
  auto frag = [&](int ks, int row0, int q) -> bf16x8 {
    const int r = row0 + (lane & 15), c = q ^ (r & 3);
    return *reinterpret_cast<const bf16x8*>(lds + (ks % LDS_KS) * LDS_ROWS * 64 + r * 64 + c * 16);
  };
  float sum = 0.f;
  if constexpr (SHAPE == 0) {
    f32x4 acc[4][4];
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 a[4], b[4];
    for (int i = 0; i < 4; ++i) {
      a[i] = frag(0, i * 16, lane >> 4);
      b[i] = frag(0, 64 + i * 16, lane >> 4);
    }
    for (int ks = 0; ks < KSTEPS; ++ks) {
      if constexpr (FROM_LDS) {
        for (int i = 0; i < 4; ++i) {
          a[i] = frag(ks, i * 16, lane >> 4);
          b[i] = frag(ks, 64 + i * 16, lane >> 4);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) sum += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
  } else {
    f32x16 acc[2][2];
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 2; ++j)
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    bf16x8 a[2][2], b[2][2];  // [k16 half][32-row block]
    auto frag32 = [&](int ks, int row0, int h) -> bf16x8 {  // 32 rows x 16 k: lane row = lane & 31, k-half by lane >> 5
      const int r = row0 + (lane & 31), c = (h * 2 + (lane >> 5)) ^ (r & 3);
      return *reinterpret_cast<const bf16x8*>(lds + (ks % LDS_KS) * LDS_ROWS * 64 + r * 64 + c * 16);
    };
    for (int h = 0; h < 2; ++h)
      for (int i = 0; i < 2; ++i) {
        a[h][i] = frag32(0, i * 32, h);
        b[h][i] = frag32(0, 64 + i * 32, h);
      }
    for (int ks = 0; ks < KSTEPS; ++ks) {
      if constexpr (FROM_LDS) {
        for (int h = 0; h < 2; ++h)
          for (int i = 0; i < 2; ++i) {
            a[h][i] = frag32(ks, i * 32, h);
            b[h][i] = frag32(ks, 64 + i * 32, h);
          }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[h][i], b[h][j], acc[i][j], 0, 0, 0);
    }
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 2; ++j)
        for (int e = 0; e < 16; ++e) sum += acc[i][j][e];
  }
  out[blockIdx.x * blockDim.x + tid] = sum;
}

template <int SHAPE, bool FROM_LDS>
void run(const char* name, const __bf16* src, float* out, int waves_per_simd) {
  const int threads = 256 * waves_per_simd, blocks = 256 * 4;
  hipLaunchKernelGGL((mfma_loop<SHAPE, FROM_LDS>), dim3(blocks), dim3(threads), 0, 0, src, out);  // warm
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int reps = 5;
  hipEventRecord(e0);
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((mfma_loop<SHAPE, FROM_LDS>), dim3(blocks), dim3(threads), 0, 0, src, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  const double flop = 2.0 * 64 * 64 * 32 * (double)KSTEPS * (threads / 64) * blocks * reps;
  printf("{\"shape\": \"%s\", \"operands\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"tflops\": %.1f}\n", name,
         FROM_LDS ? "lds" : "registers", waves_per_simd, ms / reps, flop / (ms * 1e-3) / 1e12);
  fflush(stdout);
}

int main() {
  std::vector<unsigned short> h(LDS_BYTES / 2);
  srand(1);
  for (auto& v : h) {  // random bf16 in [-1, 1): never zero-filled (clock behaviour differs)
    const float f = (rand() / (float)RAND_MAX) * 2.f - 1.f;
    unsigned u;
    std::memcpy(&u, &f, 4);
    v = (unsigned short)(u >> 16);
  }
  __bf16* src;
  float* out;
  hipMalloc(&src, LDS_BYTES);
  hipMalloc(&out, 256 * 4 * 512 * sizeof(float));
  hipMemcpy(src, h.data(), LDS_BYTES, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; ++rep)
    for (int w = 1; w <= 2; ++w) {
      run<0, false>("16x16x32", src, out, w);
      run<1, false>("32x32x16", src, out, w);
      run<0, true>("16x16x32", src, out, w);
      run<1, true>("32x32x16", src, out, w);
    }
  hipFree(src);
  hipFree(out);
  return 0;
}
