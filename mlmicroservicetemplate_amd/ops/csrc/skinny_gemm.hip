// Skinny GEMM for decode-shaped products (M = batch <= 16 rows by default dispatch): out[M][N] = act(A[M][K] W[N][K]^T + b).
// Memory-bound on W (every weight byte is read exactly once per call), so -- per
// cdna_hip_programming.md §5 "GEMV / M <= 16 decode weights" -- W goes straight to VGPRs with
// 16-B buffer loads (no LDS round trip), many loads in flight per lane (unrolled k loop), and
// the math on v_mfma_f32_16x16x32_bf16 (A = the few activation rows, padded to 16 by the
// descriptor range check; B = 16 weight rows).  Block = 8 waves on one 16-column tile, each
// wave every 8th 32-wide k-step, reduced through LDS; when N/16 tiles cannot fill the chip the grid also
// splits K across blocks (fp32 slabs + a finishing epilogue kernel).  The epilogue fuses bias,
// activation, residual and the SiLU-mul of the interleaved gate/up projection (a 16-column
// tile = 8 gate + 8 up columns).
#include "common.h"

namespace {

struct SkArgs {
  const bf16* a;  // [M][lda]
  const bf16* w;  // [N][K]
  const float* bias;
  const bf16* res;  // [M][N]
  bf16* out;        // [M][ldo]
  float* ws;        // [nsplit][M][N]
  int M, N, K, lda, ldo, act, nsplit, ksteps_per_split;
  uint32_t a_bytes, w_bytes;
};

MLS_DEV float epi(float v, int n, const SkArgs& s) { return v + (s.bias ? s.bias[n] : 0.f); }

template <int TMS, int UNROLL, int NWV>
__global__ __launch_bounds__(NWV * 64) void skinny_gemm_kernel(const SkArgs s) {
  __shared__ float red[NWV][TMS * 16][17];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nr = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const int split = blockIdx.y;
  const int ks_beg = split * s.ksteps_per_split;
  const int ksteps = (s.K + 31) / 32;
  const int ks_end = min(ksteps, ks_beg + s.ksteps_per_split);
  const rsrc_t ar = make_rsrc(s.a, s.a_bytes);
  const rsrc_t wr = make_rsrc(s.w, s.w_bytes);
  const int wbase = ((n0 + nr) * s.K + 8 * g) * 2;
  int abase[TMS];
#pragma unroll
  for (int t = 0; t < TMS; ++t) {
    const int m = 16 * t + nr;
    abase[t] = m < s.M ? (m * s.lda + 8 * g) * 2 : OOB;
  }
  f32x4 acc[TMS];
#pragma unroll
  for (int t = 0; t < TMS; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  int ks = ks_beg + wid;
  for (; ks + NWV * (UNROLL - 1) < ks_end; ks += NWV * UNROLL) {
    uint4 wv[UNROLL], av[UNROLL][TMS];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int k = (ks + NWV * u) * 32;
      const bool kin = k + 8 * g < s.K;
      wv[u] = bload16(wr, kin ? wbase + k * 2 : OOB);
#pragma unroll
      for (int t = 0; t < TMS; ++t) av[u][t] = bload16(ar, (kin && abase[t] != OOB) ? abase[t] + k * 2 : OOB);
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
#pragma unroll
      for (int t = 0; t < TMS; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, av[u][t]),
                                                         __builtin_bit_cast(bf16x8, wv[u]), acc[t], 0, 0, 0);
  }
  for (; ks < ks_end; ks += NWV) {
    const int k = ks * 32;
    const bool kin = k + 8 * g < s.K;
    const uint4 wv = bload16(wr, kin ? wbase + k * 2 : OOB);
#pragma unroll
    for (int t = 0; t < TMS; ++t) {
      const uint4 av = bload16(ar, (kin && abase[t] != OOB) ? abase[t] + k * 2 : OOB);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, av), __builtin_bit_cast(bf16x8, wv),
                                                       acc[t], 0, 0, 0);
    }
  }
  // C layout: acc[t][j] = out[m = 16t + 4g + j][n = n0 + nr]
#pragma unroll
  for (int t = 0; t < TMS; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) red[wid][16 * t + 4 * g + j][nr] = acc[t][j];
  __syncthreads();
  const bool glu = s.act == ACT_SILU_MUL;
  for (int q = tid; q < TMS * 16 * 16; q += NWV * 64) {
    const int m = q >> 4, c = q & 15;
    if (m >= s.M) continue;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NWV; ++w) v += red[w][m][c];
    const int n = n0 + c;
    if (s.nsplit > 1) {
      s.ws[((size_t)split * s.M + m) * s.N + n] = v;
      continue;
    }
    if (glu) {
      if (c < 8) {
        float up = 0.f;
#pragma unroll
        for (int w = 0; w < NWV; ++w) up += red[w][m][c + 8];
        const float gt = epi(v, n, s);
        s.out[(size_t)m * s.ldo + (n0 >> 1) + c] = (bf16)(silu(gt) * epi(up, n + 8, s));
      }
      continue;
    }
    float o = epi(v, n, s);
    if (s.res) o += (float)s.res[(size_t)m * s.N + n];
    s.out[(size_t)m * s.ldo + n] = (bf16)apply_act(o, s.act);
  }
}

__global__ __launch_bounds__(256) void skinny_finish_kernel(const SkArgs s) {
  const bool glu = s.act == ACT_SILU_MUL;
  const int ncols = glu ? s.N / 2 : s.N;
  const long total = (long)s.M * ncols;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const int m = (int)(q / ncols), c = (int)(q % ncols);
    const int n = glu ? (c / 8) * 16 + (c % 8) : c;
    float v = 0.f, u = 0.f;
    for (int sp = 0; sp < s.nsplit; ++sp) {
      const float* row = s.ws + ((size_t)sp * s.M + m) * s.N;
      v += row[n];
      if (glu) u += row[n + 8];
    }
    if (glu) {
      s.out[(size_t)m * s.ldo + c] = (bf16)(silu(epi(v, n, s)) * epi(u, n + 8, s));
    } else {
      float o = epi(v, n, s);
      if (s.res) o += (float)s.res[(size_t)m * s.N + n];
      s.out[(size_t)m * s.ldo + n] = (bf16)apply_act(o, s.act);
    }
  }
}

}  // namespace

extern "C" {

// M <= 32, N % 16 == 0, K % 8 == 0.  nsplit <= 0: auto (fill the chip).  ws: >= nsplit*M*N floats.
int mls_skinny_gemm(const void* A, const void* W, const float* bias, const void* res, void* out, void* ws,
                    size_t ws_bytes, int M, int N, int K, int act, int nsplit, void* stream) {
  if (M <= 0 || M > 32 || N % 16 || K % 8 || K <= 0) return MLS_BAD_ARG;
  SkArgs s{};
  s.a = (const bf16*)A;
  s.w = (const bf16*)W;
  s.bias = bias;
  s.res = (const bf16*)res;
  s.out = (bf16*)out;
  s.ws = (float*)ws;
  s.M = M; s.N = N; s.K = K; s.lda = K;
  s.act = act;
  s.ldo = act == ACT_SILU_MUL ? N / 2 : N;
  const size_t ab = (size_t)M * K * 2, wb = (size_t)N * K * 2;
  if (ab >= 0x7FFFFFFFull || wb >= 0x7FFFFFFFull) return MLS_UNSUPPORTED;
  s.a_bytes = (uint32_t)ab;
  s.w_bytes = (uint32_t)wb;
  const int tiles = N / 16;
  const int ksteps = (K + 31) / 32;
  if (nsplit <= 0) {  // 8 waves split K inside a block; split across blocks only below 256 tiles
    nsplit = 1;
    while (tiles * nsplit < 256 && ksteps / (nsplit * 2) >= 32) nsplit *= 2;
  }
  if (nsplit > 1 && (ws == nullptr || ws_bytes < (size_t)nsplit * M * N * 4)) nsplit = 1;
  s.nsplit = nsplit;
  s.ksteps_per_split = (ksteps + nsplit - 1) / nsplit;
  dim3 grid(tiles, nsplit);
  hipStream_t st = (hipStream_t)stream;
  if (M <= 16)
    hipLaunchKernelGGL((skinny_gemm_kernel<1, 8, 8>), grid, dim3(512), 0, st, s);
  else
    hipLaunchKernelGGL((skinny_gemm_kernel<2, 4, 8>), grid, dim3(512), 0, st, s);
  if (nsplit > 1) {
    const long total = (long)M * (act == ACT_SILU_MUL ? N / 2 : N);
    int blocks = (int)((total + 255) / 256);
    blocks = blocks > 2048 ? 2048 : blocks;
    hipLaunchKernelGGL(skinny_finish_kernel, dim3(blocks), dim3(256), 0, st, s);
  }
  return (int)hipGetLastError();
}

}  // extern "C"
