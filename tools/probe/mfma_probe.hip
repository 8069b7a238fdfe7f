// Probe: verify the gfx950 bf16 MFMA operand/accumulator lane maps used by ops/csrc.
#include <hip/hip_runtime.h>
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
// A row-major [16][32] bf16, B row-major [32][16] (k-major), D [16][16] f32
extern "C" __global__ void probe16(const __bf16* A, const __bf16* B, float* D) {
  int l = threadIdx.x;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = A[(l & 15) * 32 + 8 * (l >> 4) + j];
    b[j] = B[(8 * (l >> 4) + j) * 16 + (l & 15)];
  }
  f32x4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  for (int j = 0; j < 4; ++j) D[((l >> 4) * 4 + j) * 16 + (l & 15)] = acc[j];
}
// A [32][16], B [16][32], D [32][32]
extern "C" __global__ void probe32(const __bf16* A, const __bf16* B, float* D) {
  int l = threadIdx.x, r = l & 31, h = l >> 5;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = A[r * 16 + 8 * h + j];
    b[j] = B[(8 * h + j) * 32 + r];
  }
  f32x16 acc = {};
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  for (int g = 0; g < 16; ++g) D[((g & 3) + 8 * (g >> 2) + 4 * h) * 32 + r] = acc[g];
}
extern "C" int launch_probe(int which, const void* A, const void* B, void* D, void* stream) {
  if (which == 16) hipLaunchKernelGGL(probe16, dim3(1), dim3(64), 0, (hipStream_t)stream, (const __bf16*)A, (const __bf16*)B, (float*)D);
  else hipLaunchKernelGGL(probe32, dim3(1), dim3(64), 0, (hipStream_t)stream, (const __bf16*)A, (const __bf16*)B, (float*)D);
  return (int)hipGetLastError();
}
