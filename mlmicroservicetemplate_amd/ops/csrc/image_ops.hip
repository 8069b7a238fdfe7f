// K11 (max / global-average pooling), K12 (uint8 HWC -> normalised bf16 NHWC) and a
// standalone inference BatchNorm (K3, the unfused path; the fast path folds BN into K1's epilogue).
// All memory-bound: 16-B vector accesses per lane (cdna_hip_programming.md Guideline 13),
// grid-stride loops capped at 256 CUs x 8 blocks.
#include "common.h"

namespace {

inline int grid_for(long work, int block) {
  long g = (work + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

// 4 pixels per thread: 12 input bytes (3 dwords) -> 4 x (4 x bf16) = 32 output bytes.
// out channel 3 is zero (Cin padded 3 -> 4 so the stem conv reads 8-byte taps).
__global__ __launch_bounds__(256) void normalize_u8_kernel(const uint8_t* __restrict__ in, bf16* __restrict__ out,
                                                           long npix, float m0, float m1, float m2, float s0,
                                                           float s1, float s2) {
  const long nq = npix / 4;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < nq; q += (long)gridDim.x * blockDim.x) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(in + q * 12);
    const uint32_t w0 = src[0], w1 = src[1], w2 = src[2];
    uint8_t b[12];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      b[i] = (w0 >> (8 * i)) & 0xff;
      b[4 + i] = (w1 >> (8 * i)) & 0xff;
      b[8 + i] = (w2 >> (8 * i)) & 0xff;
    }
    float f[16];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      f[4 * p + 0] = ((float)b[3 * p + 0] - m0) * s0;
      f[4 * p + 1] = ((float)b[3 * p + 1] - m1) * s1;
      f[4 * p + 2] = ((float)b[3 * p + 2] - m2) * s2;
      f[4 * p + 3] = 0.f;
    }
    float lo[8], hi[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      lo[i] = f[i];
      hi[i] = f[8 + i];
    }
    st16(out + q * 16, pack8(lo));
    st16(out + q * 16 + 8, pack8(hi));
  }
  // tail pixels (npix % 4)
  const long tail0 = nq * 4;
  const long t = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (t < npix - tail0) {
    const long p = tail0 + t;
    const uint8_t* s = in + p * 3;
    bf16* d = out + p * 4;
    d[0] = f2bf(((float)s[0] - m0) * s0);
    d[1] = f2bf(((float)s[1] - m1) * s1);
    d[2] = f2bf(((float)s[2] - m2) * s2);
    d[3] = f2bf(0.f);
  }
}

// NHWC max pool; thread = (b, oh, ow, 8 channels)
__global__ __launch_bounds__(256) void maxpool_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int B, int H,
                                                      int W, int C, int Ho, int Wo, int k, int s, int p) {
  const int c8n = C / 8;
  const long total = (long)B * Ho * Wo * c8n;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(q % c8n);
    long r = q / c8n;
    const int ow = (int)(r % Wo);
    r /= Wo;
    const int oh = (int)(r % Ho);
    const int b = (int)(r / Ho);
    float m[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) m[e] = -INFINITY;
    for (int kh = 0; kh < k; ++kh) {
      const int ih = oh * s - p + kh;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int kw = 0; kw < k; ++kw) {
        const int iw = ow * s - p + kw;
        if ((unsigned)iw >= (unsigned)W) continue;
        float v[8];
        unpack8(ld16(x + (((long)b * H + ih) * W + iw) * C + c8 * 8), v);
#pragma unroll
        for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], v[e]);
      }
    }
    st16(y + (((long)b * Ho + oh) * Wo + ow) * C + c8 * 8, pack8(m));
  }
}

// global average pool [B][HW][C] -> [B][C]; thread = (b, 8 channels)
__global__ __launch_bounds__(256) void avgpool_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int B, int HW,
                                                      int C, float inv) {
  const int c8n = C / 8;
  const long total = (long)B * c8n;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(q % c8n);
    const int b = (int)(q / c8n);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const bf16* src = x + (long)b * HW * C + c8 * 8;
    for (int i = 0; i < HW; ++i) {
      float v[8];
      unpack8(ld16(src + (long)i * C), v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] *= inv;
    st16(y + (long)b * C + c8 * 8, pack8(acc));
  }
}

// inference BatchNorm (+optional ReLU) over NHWC: y = x * scale[c] + bias[c]
__global__ __launch_bounds__(256) void bn_act_kernel(const bf16* __restrict__ x, bf16* __restrict__ y,
                                                     const float* __restrict__ scale, const float* __restrict__ bias,
                                                     long rows, int C, int relu) {
  const int c8n = C / 8;
  const long total = rows * c8n;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const int c = (int)(q % c8n) * 8;
    float v[8];
    unpack8(ld16(x + q * 8), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float t = v[e] * scale[c + e] + bias[c + e];
      v[e] = relu ? fmaxf(t, 0.f) : t;
    }
    st16(y + q * 8, pack8(v));
  }
}

}  // namespace

extern "C" {

int mls_normalize_u8(const void* in, void* out, long npix, const float* mean3, const float* std3, void* stream) {
  if (npix <= 0) return MLS_BAD_ARG;
  const long nq = npix / 4;
  int g = grid_for(nq > 0 ? nq : 1, 256);
  hipLaunchKernelGGL(normalize_u8_kernel, dim3(g), dim3(256), 0, (hipStream_t)stream, (const uint8_t*)in, (bf16*)out,
                     npix, mean3[0], mean3[1], mean3[2], 1.f / std3[0], 1.f / std3[1], 1.f / std3[2]);
  return (int)hipGetLastError();
}

int mls_maxpool2d(const void* x, void* y, int B, int H, int W, int C, int k, int s, int p, void* stream) {
  if (C % 8) return MLS_BAD_ARG;
  const int Ho = (H + 2 * p - k) / s + 1, Wo = (W + 2 * p - k) / s + 1;
  const long total = (long)B * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(maxpool_kernel, dim3(grid_for(total, 256)), dim3(256), 0, (hipStream_t)stream, (const bf16*)x,
                     (bf16*)y, B, H, W, C, Ho, Wo, k, s, p);
  return (int)hipGetLastError();
}

int mls_avgpool_global(const void* x, void* y, int B, int HW, int C, void* stream) {
  if (C % 8) return MLS_BAD_ARG;
  const long total = (long)B * (C / 8);
  hipLaunchKernelGGL(avgpool_kernel, dim3(grid_for(total, 256)), dim3(256), 0, (hipStream_t)stream, (const bf16*)x,
                     (bf16*)y, B, HW, C, 1.f / (float)HW);
  return (int)hipGetLastError();
}

int mls_bn_act(const void* x, void* y, const float* scale, const float* bias, long rows, int C, int relu, void* stream) {
  if (C % 8) return MLS_BAD_ARG;
  const long total = rows * (C / 8);
  hipLaunchKernelGGL(bn_act_kernel, dim3(grid_for(total, 256)), dim3(256), 0, (hipStream_t)stream, (const bf16*)x,
                     (bf16*)y, scale, bias, rows, C, relu);
  return (int)hipGetLastError();
}

}  // extern "C"
