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

// uint8 [B,H,W,3] -> bf16 [B,H+2p,W+2p,4]: ((x - mean) / std, 0) with a zero border of p pixels
// (the stem conv then needs no bounds checks) and channel 3 zero (Cin padded 3 -> 4 so the stem
// reads two 4-channel taps per 16-B chunk).  One thread per output pixel, 8-B stores.
__global__ __launch_bounds__(256) void normalize_u8_kernel(const uint8_t* __restrict__ in, bf16* __restrict__ out,
                                                           int B, int H, int W, int pad, float m0, float m1,
                                                           float m2, float s0, float s1, float s2) {
  const int Hp = H + 2 * pad, Wp = W + 2 * pad;
  const long total = (long)B * Hp * Wp;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const int x = (int)(q % Wp);
    const long r = q / Wp;
    const int y = (int)(r % Hp);
    const int b = (int)(r / Hp);
    const int iy = y - pad, ix = x - pad;
    bf16x4 v;
    if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W) {
      const uint8_t* p = in + (((long)b * H + iy) * W + ix) * 3;
      v[0] = (bf16)(((float)p[0] - m0) * s0);
      v[1] = (bf16)(((float)p[1] - m1) * s1);
      v[2] = (bf16)(((float)p[2] - m2) * s2);
      v[3] = (bf16)0.f;
    } else {
      v[0] = v[1] = v[2] = v[3] = (bf16)0.f;
    }
    *reinterpret_cast<uint2*>(out + q * 4) = __builtin_bit_cast(uint2, v);
  }
}

// NHWC max pool; thread = (b, oh, ow, 8 channels).  All k*k taps are loaded with clamped
// (always valid) addresses and masked afterwards, so the loads issue back to back.
template <int KS>
__global__ __launch_bounds__(256) void maxpool_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int B, int H,
                                                      int W, int C, int Ho, int Wo, int s, int p) {
  const int c8n = C / 8;
  const long total = (long)B * Ho * Wo * c8n;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(q % c8n);
    long r = q / c8n;
    const int ow = (int)(r % Wo);
    r /= Wo;
    const int oh = (int)(r % Ho);
    const int b = (int)(r / Ho);
    uint4 raw[KS * KS];
    bool ok[KS * KS];
#pragma unroll
    for (int kh = 0; kh < KS; ++kh)
#pragma unroll
      for (int kw = 0; kw < KS; ++kw) {
        const int ih = oh * s - p + kh, iw = ow * s - p + kw;
        const bool v = (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
        const int cih = v ? ih : 0, ciw = v ? iw : 0;
        ok[kh * KS + kw] = v;
        raw[kh * KS + kw] = ld16(x + (((long)b * H + cih) * W + ciw) * C + c8 * 8);
      }
    float m[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) m[e] = -INFINITY;
#pragma unroll
    for (int t = 0; t < KS * KS; ++t) {
      float v[8];
      unpack8(raw[t], v);
#pragma unroll
      for (int e = 0; e < 8; ++e) m[e] = ok[t] ? fmaxf(m[e], v[e]) : m[e];
    }
    st16(y + (((long)b * Ho + oh) * Wo + ow) * C + c8 * 8, pack8(m));
  }
}

// global average pool [B][HW][C] -> [B][C].  Block = (batch, 64 x 8 channels); its 4 waves
// split the HW positions (independent 16-B loads, unrolled) and combine through LDS.
__global__ __launch_bounds__(256) void avgpool_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int B, int HW,
                                                      int C, float inv) {
  __shared__ float part[3][64][8];
  const int c8n = C / 8;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int groups = (c8n + 63) / 64;
  const int b = blockIdx.x / groups;
  const int c8 = (blockIdx.x % groups) * 64 + lane;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c8 < c8n) {
    const bf16* src = x + (long)b * HW * C + c8 * 8;
    int i = wid;
    for (; i + 12 < HW; i += 16) {
      float v0[8], v1[8], v2[8], v3[8];
      unpack8(ld16(src + (long)i * C), v0);
      unpack8(ld16(src + (long)(i + 4) * C), v1);
      unpack8(ld16(src + (long)(i + 8) * C), v2);
      unpack8(ld16(src + (long)(i + 12) * C), v3);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += (v0[e] + v1[e]) + (v2[e] + v3[e]);
    }
    for (; i < HW; i += 4) {
      float v[8];
      unpack8(ld16(src + (long)i * C), v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
  }
  if (wid > 0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) part[wid - 1][lane][e] = acc[e];
  }
  __syncthreads();
  if (wid == 0 && c8 < c8n) {
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = (acc[e] + part[0][lane][e] + part[1][lane][e] + part[2][lane][e]) * inv;
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

__global__ __launch_bounds__(256) void silu_mul_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, long groups) {
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < groups; q += (long)gridDim.x * blockDim.x) {
    float g[8], u[8], o[8];
    unpack8(ld16(x + q * 16), g);
    unpack8(ld16(x + q * 16 + 8), u);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = silu(g[e]) * u[e];
    st16(y + q * 8, pack8(o));
  }
}

}  // namespace

extern "C" {

int mls_normalize_u8(const void* in, void* out, int B, int H, int W, int pad, const float* mean3, const float* std3,
                     void* stream) {
  if (B <= 0 || H <= 0 || W <= 0 || pad < 0) return MLS_BAD_ARG;
  const long total = (long)B * (H + 2 * pad) * (W + 2 * pad);
  hipLaunchKernelGGL(normalize_u8_kernel, dim3(grid_for(total, 256)), dim3(256), 0, (hipStream_t)stream,
                     (const uint8_t*)in, (bf16*)out, B, H, W, pad, mean3[0], mean3[1], mean3[2], 1.f / std3[0],
                     1.f / std3[1], 1.f / std3[2]);
  return (int)hipGetLastError();
}

int mls_maxpool2d(const void* x, void* y, int B, int H, int W, int C, int k, int s, int p, void* stream) {
  if (C % 8) return MLS_BAD_ARG;
  const int Ho = (H + 2 * p - k) / s + 1, Wo = (W + 2 * p - k) / s + 1;
  const long total = (long)B * Ho * Wo * (C / 8);
  if (k == 3)
    hipLaunchKernelGGL(maxpool_kernel<3>, dim3(grid_for(total, 256)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16*)x, (bf16*)y, B, H, W, C, Ho, Wo, s, p);
  else if (k == 2)
    hipLaunchKernelGGL(maxpool_kernel<2>, dim3(grid_for(total, 256)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16*)x, (bf16*)y, B, H, W, C, Ho, Wo, s, p);
  else
    return MLS_UNSUPPORTED;
  return (int)hipGetLastError();
}

int mls_avgpool_global(const void* x, void* y, int B, int HW, int C, void* stream) {
  if (C % 8) return MLS_BAD_ARG;
  const int groups = (C / 8 + 63) / 64;
  hipLaunchKernelGGL(avgpool_kernel, dim3(B * groups), dim3(256), 0, (hipStream_t)stream, (const bf16*)x, (bf16*)y, B,
                     HW, C, 1.f / (float)HW);
  return (int)hipGetLastError();
}

// SiLU-mul over a gate/up-interleaved GEMM output (groups of 8: gate 0-7, up 0-7, ...):
// y[m][8j+e] = silu(x[m][16j+e]) * x[m][16j+8+e]; the epilogue of a library (hipBLASLt) gate/up GEMM.
int mls_silu_mul_interleaved(const void* x, void* y, long rows, int n_out, void* stream) {
  if (n_out % 8) return MLS_BAD_ARG;
  const long total = rows * (n_out / 8);
  hipLaunchKernelGGL(silu_mul_kernel, dim3(grid_for(total, 256)), dim3(256), 0, (hipStream_t)stream, (const bf16*)x,
                     (bf16*)y, total);
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
