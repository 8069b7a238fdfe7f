// Standalone check of the LN-fold building blocks on gfx950: bf16 dot2 row sums and the ^16 / ^32
// lane swaps (prints max errors vs a float reference).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include "../../../mlmicroservicetemplate_amd/ops/csrc/common.h"

typedef short bf16x2 __attribute__((ext_vector_type(2)));  // the builtin takes the bf16 pairs as raw i16x2
typedef unsigned u32x4v __attribute__((ext_vector_type(4)));

__global__ void k(const uint4* x, float* o) {
  const int l = threadIdx.x;
  const bf16x8 a = __builtin_bit_cast(bf16x8, x[l]);
  const u32x4v q = __builtin_bit_cast(u32x4v, a);
  const bf16x2 one = __builtin_bit_cast(bf16x2, 0x3F803F80u);
  float s1 = 0.f, s2 = 0.f, f1 = 0.f, f2 = 0.f;
  for (int d = 0; d < 4; ++d) {
    const bf16x2 v = __builtin_bit_cast(bf16x2, q[d]);
    s1 = __builtin_amdgcn_fdot2_f32_bf16(v, one, s1, false);
    s2 = __builtin_amdgcn_fdot2_f32_bf16(v, v, s2, false);
  }
  for (int e = 0; e < 8; ++e) { const float f = (float)a[e]; f1 += f; f2 += f * f; }
  o[l * 6 + 0] = s1; o[l * 6 + 1] = f1; o[l * 6 + 2] = s2; o[l * 6 + 3] = f2;
  float r = f1;
  r += xor16_f(r);
  r += xor32_f(r);
  o[l * 6 + 4] = r;
  o[l * 6 + 5] = xor16_f((float)l) * 100.f + xor32_f((float)l);
}

int main() {
  uint16_t h[64 * 8];
  float ref[64 * 8];
  srand(1);
  for (int i = 0; i < 64 * 8; ++i) {
    float f = (rand() / (float)RAND_MAX - 0.3f) * 4.f;
    uint32_t u; std::memcpy(&u, &f, 4); u &= 0xFFFF0000u; std::memcpy(&f, &u, 4);
    h[i] = (uint16_t)(u >> 16); ref[i] = f;
  }
  void *dx, *dout;
  hipMalloc(&dx, sizeof(h)); hipMalloc(&dout, 64 * 6 * 4);
  hipMemcpy(dx, h, sizeof(h), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, (const uint4*)dx, (float*)dout);
  float o[64 * 6];
  hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost);
  double e1 = 0, e2 = 0, er = 0; int bad_perm = 0;
  for (int l = 0; l < 64; ++l) {
    double r1 = 0, r2 = 0;
    for (int e = 0; e < 8; ++e) { r1 += ref[l * 8 + e]; r2 += ref[l * 8 + e] * ref[l * 8 + e]; }
    e1 = fmax(e1, fabs(o[l * 6] - r1)); e2 = fmax(e2, fabs(o[l * 6 + 2] - r2));
    double rr = 0;
    for (int q = 0; q < 4; ++q) { int m = (l & 15) + 16 * q; for (int e = 0; e < 8; ++e) rr += ref[m * 8 + e]; }
    er = fmax(er, fabs(o[l * 6 + 4] - rr));
    const float want = (float)((l ^ 16) * 100 + (l ^ 32));
    if (o[l * 6 + 5] != want) { if (bad_perm < 4) printf("lane %d perm got %.0f want %.0f\n", l, o[l * 6 + 5], want); ++bad_perm; }
    if (l < 3) printf("lane %d dot2 s1 %.5f float %.5f ref %.5f | s2 %.5f float %.5f ref %.5f\n", l, o[l*6], o[l*6+1], r1, o[l*6+2], o[l*6+3], r2);
  }
  printf("max err dot2 sum %.3g sumsq %.3g, lane-reduced sum %.3g, bad perms %d\n", e1, e2, er, bad_perm);
  return 0;
}
