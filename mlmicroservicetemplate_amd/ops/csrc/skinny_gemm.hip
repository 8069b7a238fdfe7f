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
//
// Fused pre-norm (decode): with `norm` set the kernel computes RMSNorm(a + a2) on the fly -- the
// RMSNorm gain is folded into W's columns at load time, so x_norm @ W^T = rstd[m] * ((a+a2) @ W'^T)
// and rstd only scales the epilogue.  Each block already streams every element of its rows of
// (a + a2) through registers for the MFMA, so the sum of squares costs nothing extra; blocks of
// column tile 0 also write the updated residual stream a + a2 to a_out (a separate buffer: other
// blocks still read a).  This removes the standalone RMSNorm launch (2 per layer) from decode.
#include <type_traits>

#include "common.h"
#include "ar_protocol.h"
#include "fastdiv.h"

namespace {

struct SkArgs {
  const bf16* a;   // [M][lda]
  const bf16* a2;  // optional [M][lda] added to a (residual-stream update)
  bf16* a_out;     // optional [M][lda] <- a + a2 (written by column-tile-0 blocks)
  const bf16* w;   // [N][K]
  const float* bias;
  const bf16* res;  // [M][N]
  bf16* out;        // [M][ldo]
  float* ws;        // [nsplit][M][N]
  int M, N, K, lda, ldo, act, nsplit, ksteps_per_split, norm;
  float eps;
  uint32_t a_bytes, w_bytes;
  // FUSE_COMBINE (packed LDS kernel): A = the split-KV decode attention's merged output, combined
  // here from its fp32 partials (o [M][Hq][nsplit][D], (m, l) [M][Hq][nsplit][2]); rows whose
  // sequence fit one split were written to `a` directly by the attention kernel
  const float* cws;
  const float* cml;
  const int* lens;
  int c_nsplit, c_chunk, c_hq, c_hd;
  const float* wscale;  // fp8 weights: per-output-channel dequantisation scale [N]
  // fused tensor-parallel all-reduce of `out` (ar_protocol.h; world == 0: none): the row-parallel
  // decode projections reduce their partial sums across ranks in their own epilogue
  ArFuse arf;
  // runtime divisors of the A staging loops (fastdiv.h): K / 8 chunks per row, combine head dim
  FastDiv fd_kch, fd_hd;
};

// fusion modes of the A prologue (template parameter, so the unrolled k loop has no runtime
// branches -- a branch there makes hipcc drain vmcnt(0) per k-step, cdna_hip_programming.md item 4c)
enum { FUSE_NONE = 0, FUSE_NORM = 1, FUSE_ADD_NORM = 2, FUSE_COMBINE = 3 };

MLS_DEV uint4 add_round(uint4 a, uint4 b) {  // bf16 + bf16 -> bf16 (the residual stream's precision)
  float x[8], y[8];
  unpack8(a, x);
  unpack8(b, y);
#pragma unroll
  for (int e = 0; e < 8; ++e) x[e] += y[e];
  return pack8(x);
}

MLS_DEV float sumsq8(uint4 v) {
  float x[8];
  unpack8(v, x);
  float r = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) r += x[e] * x[e];
  return r;
}

MLS_DEV float epi(float v, int n, const SkArgs& s) { return v + (s.bias ? s.bias[n] : 0.f); }

// NT 16-column tiles per block: every A fragment a wave loads feeds NT MFMAs, so the activation
// traffic from L2 (M rows x K per block) is amortised over NT weight tiles -- at M = 16 it equals
// the weight traffic when NT = 1.
template <int TMS, int UNROLL, int NWV, int FUSE, int NT>
__global__ __launch_bounds__(NWV * 64) void skinny_gemm_kernel(const SkArgs s) {
  __shared__ float red[NWV][TMS * 16][NT * 16 + 1];
  __shared__ float ssq_red[NWV][TMS * 16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nr = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16 * NT;
  const int split = blockIdx.y;
  const int ks_beg = split * s.ksteps_per_split;
  const int ksteps = (s.K + 31) / 32;
  const int ks_end = min(ksteps, ks_beg + s.ksteps_per_split);
  const rsrc_t ar = make_rsrc(s.a, s.a_bytes);
  const rsrc_t wr = make_rsrc(s.w, s.w_bytes);
  const rsrc_t a2r = make_rsrc(s.a2, FUSE == FUSE_ADD_NORM ? s.a_bytes : 0);
  const bool wr_res = FUSE == FUSE_ADD_NORM && s.a_out && blockIdx.x == 0;
  int wbase[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) wbase[j] = ((n0 + 16 * j + nr) * s.K + 8 * g) * 2;
  int abase[TMS];
#pragma unroll
  for (int t = 0; t < TMS; ++t) {
    const int m = 16 * t + nr;
    abase[t] = m < s.M ? (m * s.lda + 8 * g) * 2 : OOB;
  }
  f32x4 acc[TMS][NT];
  float ssq[TMS];
#pragma unroll
  for (int t = 0; t < TMS; ++t) {
    ssq[t] = 0.f;
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[t][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  // U k-steps per trip: issue every load first, then the math, then (tile-0 blocks) the
  // residual-stream stores
  auto body = [&](int ks0, auto U_) {
    constexpr int U = decltype(U_)::value;
    uint4 wv[U][NT], av[U][TMS], a2v[U][TMS];
    int aoff[U][TMS];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = (ks0 + NWV * u) * 32;
      const bool kin = k + 8 * g < s.K;
#pragma unroll
      for (int j = 0; j < NT; ++j) wv[u][j] = bload16(wr, kin ? wbase[j] + k * 2 : OOB);
#pragma unroll
      for (int t = 0; t < TMS; ++t) {
        aoff[u][t] = (kin && abase[t] != OOB) ? abase[t] + k * 2 : OOB;
        av[u][t] = bload16(ar, aoff[u][t]);
        if constexpr (FUSE == FUSE_ADD_NORM) a2v[u][t] = bload16(a2r, aoff[u][t]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < TMS; ++t) {
        if constexpr (FUSE == FUSE_ADD_NORM) av[u][t] = add_round(av[u][t], a2v[u][t]);
        if constexpr (FUSE != FUSE_NONE) ssq[t] += sumsq8(av[u][t]);
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, av[u][t]),
                                                              __builtin_bit_cast(bf16x8, wv[u][j]), acc[t][j], 0, 0, 0);
      }
    if constexpr (FUSE == FUSE_ADD_NORM) {
      if (wr_res) {
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int t = 0; t < TMS; ++t)
            if (aoff[u][t] != OOB) st16(s.a_out + aoff[u][t] / 2, av[u][t]);
      }
    }
  };
  int ks = ks_beg + wid;
  for (; ks + NWV * (UNROLL - 1) < ks_end; ks += NWV * UNROLL) body(ks, std::integral_constant<int, UNROLL>{});
  for (; ks < ks_end; ks += NWV) body(ks, std::integral_constant<int, 1>{});

  // C layout: acc[t][j][i] = out[m = 16t + 4g + i][n = n0 + 16j + nr]
#pragma unroll
  for (int t = 0; t < TMS; ++t)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[wid][16 * t + 4 * g + i][16 * j + nr] = acc[t][j][i];
  if constexpr (FUSE != FUSE_NONE) {
    // lanes nr, nr+16, nr+32, nr+48 hold row nr's four 8-element k slices
#pragma unroll
    for (int t = 0; t < TMS; ++t) {
      float v = ssq[t];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      if (g == 0) ssq_red[wid][16 * t + nr] = v;
    }
  }
  __syncthreads();
  const bool glu = s.act == ACT_SILU_MUL;
  constexpr int COLS = NT * 16;
  for (int q = tid; q < TMS * 16 * COLS; q += NWV * 64) {
    const int m = q / COLS, c = q % COLS;
    if (m >= s.M) continue;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NWV; ++w) v += red[w][m][c];
    const int n = n0 + c;
    float rs = 1.f;
    if constexpr (FUSE != FUSE_NONE) {
      float t2 = 0.f;
#pragma unroll
      for (int w = 0; w < NWV; ++w) t2 += ssq_red[w][m];
      if (s.nsplit > 1) {  // partial square sums ride after the slabs; the finisher combines them
        if (blockIdx.x == 0 && c == 0) s.ws[(size_t)s.nsplit * s.M * s.N + split * s.M + m] = t2;
      } else {
        rs = rsqrtf(t2 / (float)s.K + s.eps);
      }
    }
    if (s.nsplit > 1) {
      s.ws[((size_t)split * s.M + m) * s.N + n] = v;
      continue;
    }
    v *= rs;
    if (glu) {
      if ((c & 15) < 8) {
        float up = 0.f;
#pragma unroll
        for (int w = 0; w < NWV; ++w) up += red[w][m][c + 8];
        up *= rs;
        const float gt = epi(v, n, s);
        s.out[(size_t)m * s.ldo + (n >> 4) * 8 + (n & 7)] = (bf16)(silu(gt) * epi(up, n + 8, s));
      }
      continue;
    }
    float o = epi(v, n, s);
    if (s.res) o += (float)s.res[(size_t)m * s.N + n];
    s.out[(size_t)m * s.ldo + n] = (bf16)apply_act(o, s.act);
  }
}

// Few-row variant (M <= 4, whole K per block): the activation rows -- with the fused prologue,
// a + a2 rounded to the bf16 residual stream -- are staged ONCE per block into LDS (M*K*2 bytes,
// dynamic) together with their square sums, so the k loop is the plain weight stream with the
// A fragments read from LDS; the block's first weight loads are issued before that prologue and
// every later trip's loads are in flight while the previous trip's MFMAs run (register double
// buffer).  Measured motivation: the register-path fused kernel streamed gate_up ~20 % slower
// than the plain one (profiles/r1_decode_cold_weight_stream_probe.jsonl).
template <int UNROLL, int NWV, int FUSE, int NT>
__global__ __launch_bounds__(NWV * 64) void skinny_lds_kernel(const SkArgs s) {
  extern __shared__ __attribute__((aligned(16))) uint4 a_lds[];  // [M][K/8]
  __shared__ float red[NWV][16][NT * 16 + 1];
  __shared__ float ssq_s[4];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nr = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16 * NT;
  const int ksteps = s.K >> 5;
  const int kch = s.K >> 3;  // 16-B chunks per row
  const rsrc_t wr = make_rsrc(s.w, s.w_bytes);
  int wbase[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) wbase[j] = ((n0 + 16 * j + nr) * s.K + 8 * g) * 2;

  auto load_trip = [&](int ks0, uint4 (&wv)[UNROLL][NT]) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int ks = ks0 + NWV * u;
#pragma unroll
      for (int j = 0; j < NT; ++j) wv[u][j] = bload16(wr, ks < ksteps ? wbase[j] + ks * 64 : OOB);
    }
  };
  uint4 wnext[UNROLL][NT];
  int ks = wid;
  load_trip(ks, wnext);  // in flight during the prologue

  // prologue: A (+ A2) -> LDS, residual write-back (column-tile-0 blocks), square sums
  constexpr bool NORM = FUSE == FUSE_NORM || FUSE == FUSE_ADD_NORM;
  if (tid < 4) ssq_s[tid] = 0.f;
  __syncthreads();
  float part[4] = {0.f, 0.f, 0.f, 0.f};
  const bool wr_res = FUSE == FUSE_ADD_NORM && s.a_out && blockIdx.x == 0;
  int lens4[4] = {0, 0, 0, 0};
  if constexpr (FUSE == FUSE_COMBINE) {
    // block-uniform reads (scalar loads): they do not queue behind the weight loads in flight
#pragma unroll
    for (int mm = 0; mm < 4; ++mm) lens4[mm] = mm < s.M ? __builtin_nontemporal_load(s.lens + mm) : 0;
  }
  for (int q = tid; q < s.M * kch; q += NWV * 64) {
    const int m = fastdiv(q, s.fd_kch), c = q - m * kch;
    uint4 v;
    if constexpr (FUSE == FUSE_COMBINE) {
      // the decode_combine_kernel arithmetic for this row's 8 dims of one head
      const int h = fastdiv(c * 8, s.fd_hd), d0 = c * 8 - h * s.c_hd;
      const int L = m == 0 ? lens4[0] : m == 1 ? lens4[1] : m == 2 ? lens4[2] : lens4[3];
      const int ns = min(s.c_nsplit, (L + s.c_chunk - 1) / s.c_chunk);
      if (ns <= 1) {
        v = ld16(s.a + (size_t)m * s.lda + c * 8);
      } else {
        const long rec = ((long)m * s.c_hq + h) * s.c_nsplit;
        // online merge in groups of 4 splits: each group's (m, l, o) loads are issued together
        // (one memory round trip per group, not two per split)
        float mx = -INFINITY, l = 0.f, o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int s0 = 0; s0 < ns; s0 += 4) {
          float2 ml[4];
          float4 x0[4], x1[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const bool in = s0 + j < ns;
            const long r = rec + (in ? s0 + j : 0);
            ml[j] = in ? *reinterpret_cast<const float2*>(s.cml + r * 2) : make_float2(-INFINITY, 0.f);
            x0[j] = in ? *reinterpret_cast<const float4*>(s.cws + r * s.c_hd + d0) : make_float4(0.f, 0.f, 0.f, 0.f);
            x1[j] = in ? *reinterpret_cast<const float4*>(s.cws + r * s.c_hd + d0 + 4)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
          }
          float gm = mx;
#pragma unroll
          for (int j = 0; j < 4; ++j) gm = fmaxf(gm, ml[j].x);
          if (gm == -INFINITY) continue;
          const float al = __builtin_amdgcn_exp2f(mx - gm);
          l *= al;
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] *= al;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float w = __builtin_amdgcn_exp2f(ml[j].x - gm);
            l += ml[j].y * w;
            o[0] += x0[j].x * w; o[1] += x0[j].y * w; o[2] += x0[j].z * w; o[3] += x0[j].w * w;
            o[4] += x1[j].x * w; o[5] += x1[j].y * w; o[6] += x1[j].z * w; o[7] += x1[j].w * w;
          }
          mx = gm;
        }
        const float inv = l > 0.f ? 1.f / l : 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] *= inv;
        v = pack8(o);
      }
    } else {
      v = ld16(s.a + (size_t)m * s.lda + c * 8);
    }
    if constexpr (FUSE == FUSE_ADD_NORM) {
      v = add_round(v, ld16(s.a2 + (size_t)m * s.lda + c * 8));
      if (wr_res) st16(s.a_out + (size_t)m * s.lda + c * 8, v);
    }
    a_lds[q] = v;
    if constexpr (NORM) {
      const float sq = sumsq8(v);
#pragma unroll
      for (int mm = 0; mm < 4; ++mm) part[mm] += mm == m ? sq : 0.f;
    }
  }
  if constexpr (NORM) {
#pragma unroll
    for (int mm = 0; mm < 4; ++mm) {
      const float t = wave_sum(part[mm]);
      if (lane == 0 && mm < s.M) atomicAdd(&ssq_s[mm], t);
    }
  }
  __syncthreads();

  f32x4 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool arow = nr < s.M;
  for (; ks < ksteps; ks += NWV * UNROLL) {
    uint4 wv[UNROLL][NT];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
#pragma unroll
      for (int j = 0; j < NT; ++j) wv[u][j] = wnext[u][j];
    if (ks + NWV * UNROLL < ksteps) load_trip(ks + NWV * UNROLL, wnext);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int k = ks + NWV * u;
      const uint4 av = (arow && k < ksteps) ? a_lds[nr * kch + k * 4 + g] : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int j = 0; j < NT; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, av),
                                                         __builtin_bit_cast(bf16x8, wv[u][j]), acc[j], 0, 0, 0);
    }
  }
  // reduce the waves' partial sums; C layout: acc[j][i] = out[m = 4g + i][n = n0 + 16j + nr]
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[wid][4 * g + i][16 * j + nr] = acc[j][i];
  __syncthreads();
  const bool glu = s.act == ACT_SILU_MUL;
  constexpr int COLS = NT * 16;
  for (int q = tid; q < s.M * COLS; q += NWV * 64) {
    const int m = q / COLS, c = q % COLS;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NWV; ++w) v += red[w][m][c];
    const float rs = FUSE != FUSE_NONE ? rsqrtf(ssq_s[m] / (float)s.K + s.eps) : 1.f;
    const int n = n0 + c;
    v *= rs;
    if (glu) {
      if ((c & 15) < 8) {
        float up = 0.f;
#pragma unroll
        for (int w = 0; w < NWV; ++w) up += red[w][m][c + 8];
        up *= rs;
        s.out[(size_t)m * s.ldo + (n >> 4) * 8 + (n & 7)] = (bf16)(silu(epi(v, n, s)) * epi(up, n + 8, s));
      }
      continue;
    }
    float o = epi(v, n, s);
    if (s.res) o += (float)s.res[(size_t)m * s.N + n];
    s.out[(size_t)m * s.ldo + n] = (bf16)apply_act(o, s.act);
  }
}

// Packed-weight variant of skinny_lds_kernel (M <= 4).  W is re-laid out once at load time
// (pack_skinny_weight) so the 64 lanes' MFMA B fragments of one (16-row tile, 32-wide k-step) are
// one contiguous 1 KiB granule: [tile][kstep][g][nr][8].  Each wave then streams a CONTIGUOUS
// range of granules (its 1/NWV of the tile's k-steps), so every load instruction reads 1 KiB of
// consecutive bytes and consecutive instructions continue the same run -- instead of 16 rows x
// 64 B scattered K*2 bytes apart per instruction in the row-major layout.  NTL: non-temporal
// cache policy on the weight stream (read exactly once per call).
template <int NTL>
MLS_DEV uint4 bload16_pol(rsrc_t r, int byte_off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, NTL ? 2 : 0));
}

template <int UNROLL, int NWV, int FUSE, int NTL>
__global__ __launch_bounds__(NWV * 64) void skinny_packed_kernel(const SkArgs s) {
  extern __shared__ __attribute__((aligned(16))) uint4 a_lds[];  // [M][K/8]
  __shared__ float red[NWV][16][17];
  __shared__ float ssq_s[4];
  constexpr int T = NWV * 64;
  constexpr bool NORM = FUSE == FUSE_NORM || FUSE == FUSE_ADD_NORM;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nr = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const int ksteps = s.K >> 5;
  const int kch = s.K >> 3;
  const int nq = s.M * kch;
  const int kpw = (ksteps + NWV - 1) / NWV;
  const int kb = wid * kpw, ke = min(ksteps, kb + kpw);
  const rsrc_t wr = make_rsrc(s.w, s.w_bytes);
  const rsrc_t ar = make_rsrc(s.a, s.a_bytes);
  const rsrc_t a2r = make_rsrc(s.a2, FUSE == FUSE_ADD_NORM ? s.a_bytes : 0);
  const int wbase = blockIdx.x * ksteps * 1024 + lane * 16;

  auto load_trip = [&](int ks0, uint4 (&wv)[UNROLL]) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) wv[u] = bload16_pol<NTL>(wr, ks0 + u < ke ? wbase + (ks0 + u) * 1024 : OOB);
  };
  // The first QPT A (+ A2) chunks per thread -- all of A up to 2048 chunks, e.g. 4 rows at K = 4096
  // -- are loaded BEFORE the first weight trip: the vector memory counter retires in order, so
  // consuming them then does not wait for the weights, and the barriers below are LDS-only (a
  // __syncthreads would drain the weight loads too).  Larger A goes through the loop after.
  constexpr int QPT = 2048 / T;
  uint4 a0[QPT], a20[QPT];
#pragma unroll
  for (int j = 0; j < QPT; ++j) {
    const int q = tid + j * T;
    const int m = fastdiv(q, s.fd_kch), c = q - m * kch;
    const int off = q < nq ? (m * s.lda + c * 8) * 2 : OOB;
    a0[j] = bload16(ar, off);
    if constexpr (FUSE == FUSE_ADD_NORM) a20[j] = bload16(a2r, off);
  }
  uint4 wnext[UNROLL];
  load_trip(kb, wnext);  // in flight during the prologue

  if (tid < 4) ssq_s[tid] = 0.f;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  float part[4] = {0.f, 0.f, 0.f, 0.f};
  const bool wr_res = FUSE == FUSE_ADD_NORM && s.a_out && blockIdx.x == 0;
  int lens4[4] = {0, 0, 0, 0};
  if constexpr (FUSE == FUSE_COMBINE) {
    // block-uniform reads (scalar loads): they do not queue behind the weight loads in flight
#pragma unroll
    for (int mm = 0; mm < 4; ++mm) lens4[mm] = mm < s.M ? __builtin_nontemporal_load(s.lens + mm) : 0;
  }
  auto stage = [&](int q, uint4 v, uint4 v2) {
    const int m = fastdiv(q, s.fd_kch), c = q - m * kch;
    if constexpr (FUSE == FUSE_COMBINE) {
      // the decode_combine_kernel arithmetic for this row's 8 dims of one head
      const int h = fastdiv(c * 8, s.fd_hd), d0 = c * 8 - h * s.c_hd;
      const int L = m == 0 ? lens4[0] : m == 1 ? lens4[1] : m == 2 ? lens4[2] : lens4[3];
      const int ns = min(s.c_nsplit, (L + s.c_chunk - 1) / s.c_chunk);
      if (ns > 1) {
        const long rec = ((long)m * s.c_hq + h) * s.c_nsplit;
        // online merge in groups of 4 splits: each group's (m, l, o) loads are issued together
        float mx = -INFINITY, l = 0.f, o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int s0 = 0; s0 < ns; s0 += 4) {
          float2 ml[4];
          float4 x0[4], x1[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const bool in = s0 + j < ns;
            const long r = rec + (in ? s0 + j : 0);
            ml[j] = in ? *reinterpret_cast<const float2*>(s.cml + r * 2) : make_float2(-INFINITY, 0.f);
            x0[j] = in ? *reinterpret_cast<const float4*>(s.cws + r * s.c_hd + d0) : make_float4(0.f, 0.f, 0.f, 0.f);
            x1[j] = in ? *reinterpret_cast<const float4*>(s.cws + r * s.c_hd + d0 + 4)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
          }
          float gm = mx;
#pragma unroll
          for (int j = 0; j < 4; ++j) gm = fmaxf(gm, ml[j].x);
          if (gm == -INFINITY) continue;
          const float al = __builtin_amdgcn_exp2f(mx - gm);
          l *= al;
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] *= al;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float w = __builtin_amdgcn_exp2f(ml[j].x - gm);
            l += ml[j].y * w;
            o[0] += x0[j].x * w; o[1] += x0[j].y * w; o[2] += x0[j].z * w; o[3] += x0[j].w * w;
            o[4] += x1[j].x * w; o[5] += x1[j].y * w; o[6] += x1[j].z * w; o[7] += x1[j].w * w;
          }
          mx = gm;
        }
        const float inv = l > 0.f ? 1.f / l : 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] *= inv;
        v = pack8(o);
      }
    }
    if constexpr (FUSE == FUSE_ADD_NORM) {
      v = add_round(v, v2);
      if (wr_res) st16(s.a_out + (size_t)m * s.lda + c * 8, v);
    }
    a_lds[q] = v;
    if constexpr (NORM) {
      const float sq = sumsq8(v);
#pragma unroll
      for (int mm = 0; mm < 4; ++mm) part[mm] += mm == m ? sq : 0.f;
    }
  };
#pragma unroll
  for (int j = 0; j < QPT; ++j)
    if (tid + j * T < nq) stage(tid + j * T, a0[j], a20[j]);
  for (int q = tid + QPT * T; q < nq; q += T) {
    const int m = fastdiv(q, s.fd_kch), c = q - m * kch;
    stage(q, ld16(s.a + (size_t)m * s.lda + c * 8),
          FUSE == FUSE_ADD_NORM ? ld16(s.a2 + (size_t)m * s.lda + c * 8) : make_uint4(0, 0, 0, 0));
  }
  if constexpr (NORM) {
#pragma unroll
    for (int mm = 0; mm < 4; ++mm) {
      const float t = wave_sum(part[mm]);
      if (lane == 0 && mm < s.M) atomicAdd(&ssq_s[mm], t);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool arow = nr < s.M;
  for (int ks = kb; ks < ke; ks += UNROLL) {
    uint4 wv[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) wv[u] = wnext[u];
    if (ks + UNROLL < ke) load_trip(ks + UNROLL, wnext);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int k = ks + u;
      const uint4 av = (arow && k < ke) ? a_lds[nr * kch + k * 4 + g] : make_uint4(0, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, av), __builtin_bit_cast(bf16x8, wv[u]),
                                                    acc, 0, 0, 0);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) red[wid][4 * g + i][nr] = acc[i];
  __syncthreads();
  const bool glu = s.act == ACT_SILU_MUL;
  for (int q = tid; q < s.M * 16; q += NWV * 64) {
    const int m = q >> 4, c = q & 15;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NWV; ++w) v += red[w][m][c];
    const float rs = NORM ? rsqrtf(ssq_s[m] / (float)s.K + s.eps) : 1.f;
    const int n = n0 + c;
    v *= rs;
    if (glu) {
      if (c < 8) {
        float up = 0.f;
#pragma unroll
        for (int w = 0; w < NWV; ++w) up += red[w][m][c + 8];
        up *= rs;
        s.out[(size_t)m * s.ldo + (n >> 4) * 8 + (n & 7)] = (bf16)(silu(epi(v, n, s)) * epi(up, n + 8, s));
      }
      continue;
    }
    float o = epi(v, n, s);
    if (s.res) o += (float)s.res[(size_t)m * s.N + n];
    s.out[(size_t)m * s.ldo + n] = (bf16)apply_act(o, s.act);
  }
  if (s.arf.world) ar_fused_tail(s.arf, s.out, s.M, s.N, n0, 16);
}

// Packed weights, M <= 16 (or A too large for LDS): the A fragments (+ A2) ride beside the weight
// granules in registers, read per k-step from L2 (every block re-reads A; at M = 16 that is half
// the weight bytes, all L2 / MALL hits), register double-buffered like the weight stream.  Each
// wave folds its own k range of the RMSNorm square sums; the block reduces them through LDS.
template <int UNROLL, int NWV, int FUSE, int NTL, int NT, int TMS>
__global__ __launch_bounds__(NWV * 64) void skinny_packed_reg_kernel(const SkArgs s) {
  __shared__ float red[NWV][16 * TMS][NT * 16 + 1];
  __shared__ float ssq_red[NWV][16 * TMS];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nr = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16 * NT;
  const int ksteps = s.K >> 5;
  const int kpw = (ksteps + NWV - 1) / NWV;
  const int kb = wid * kpw, ke = min(ksteps, kb + kpw);
  const rsrc_t wr = make_rsrc(s.w, s.w_bytes);
  const rsrc_t ar = make_rsrc(s.a, s.a_bytes);
  const rsrc_t a2r = make_rsrc(s.a2, FUSE == FUSE_ADD_NORM ? s.a_bytes : 0);
  const int wbase = blockIdx.x * NT * ksteps * 1024 + lane * 16;  // tile j: + j * ksteps * 1024
  int abase[TMS];
#pragma unroll
  for (int t = 0; t < TMS; ++t) abase[t] = 16 * t + nr < s.M ? ((16 * t + nr) * s.lda + 8 * g) * 2 : OOB;
  const bool wr_res = FUSE == FUSE_ADD_NORM && s.a_out && blockIdx.x == 0;

  struct Trip {
    uint4 w[UNROLL][NT], a[UNROLL][TMS], a2[UNROLL][TMS];
  };
  auto load_trip = [&](int ks0, Trip& tr) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const bool in = ks0 + u < ke;
#pragma unroll
      for (int j = 0; j < NT; ++j)
        tr.w[u][j] = bload16_pol<NTL>(wr, in ? wbase + (j * ksteps + ks0 + u) * 1024 : OOB);
#pragma unroll
      for (int t = 0; t < TMS; ++t) {
        const int ao = (in && abase[t] != OOB) ? abase[t] + (ks0 + u) * 64 : OOB;
        tr.a[u][t] = bload16(ar, ao);
        if constexpr (FUSE == FUSE_ADD_NORM) tr.a2[u][t] = bload16(a2r, ao);
      }
    }
  };
  Trip nxt;
  load_trip(kb, nxt);
  f32x4 acc[TMS][NT];
  float ssq[TMS];
#pragma unroll
  for (int t = 0; t < TMS; ++t) {
    ssq[t] = 0.f;
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[t][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  for (int ks = kb; ks < ke; ks += UNROLL) {
    Trip cur = nxt;
    if (ks + UNROLL < ke) load_trip(ks + UNROLL, nxt);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
#pragma unroll
      for (int t = 0; t < TMS; ++t) {
        uint4 av = cur.a[u][t];
        if constexpr (FUSE == FUSE_ADD_NORM) {
          av = add_round(av, cur.a2[u][t]);
          if (wr_res && abase[t] != OOB && ks + u < ke)
            st16(s.a_out + (16 * t + nr) * s.lda + (ks + u) * 32 + 8 * g, av);
        }
        if constexpr (FUSE != FUSE_NONE) ssq[t] += sumsq8(av);
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, av),
                                                              __builtin_bit_cast(bf16x8, cur.w[u][j]), acc[t][j], 0, 0, 0);
      }
  }
#pragma unroll
  for (int t = 0; t < TMS; ++t)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[wid][16 * t + 4 * g + i][16 * j + nr] = acc[t][j][i];
  if constexpr (FUSE != FUSE_NONE) {
#pragma unroll
    for (int t = 0; t < TMS; ++t) {
      float v = ssq[t];  // lanes nr, nr+16, nr+32, nr+48 hold row 16t+nr's k slices
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      if (g == 0) ssq_red[wid][16 * t + nr] = v;
    }
  }
  __syncthreads();
  const bool glu = s.act == ACT_SILU_MUL;
  constexpr int COLS = NT * 16;
  for (int q = tid; q < s.M * COLS; q += NWV * 64) {
    const int m = q / COLS, c = q % COLS;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NWV; ++w) v += red[w][m][c];
    float rs = 1.f;
    if constexpr (FUSE != FUSE_NONE) {
      float t2 = 0.f;
#pragma unroll
      for (int w = 0; w < NWV; ++w) t2 += ssq_red[w][m];
      rs = rsqrtf(t2 / (float)s.K + s.eps);
    }
    const int n = n0 + c;
    v *= rs;
    if (glu) {
      if ((c & 15) < 8) {
        float up = 0.f;
#pragma unroll
        for (int w = 0; w < NWV; ++w) up += red[w][m][c + 8];
        up *= rs;
        s.out[(size_t)m * s.ldo + (n >> 4) * 8 + (n & 7)] = (bf16)(silu(epi(v, n, s)) * epi(up, n + 8, s));
      }
      continue;
    }
    float o = epi(v, n, s);
    if (s.res) o += (float)s.res[(size_t)m * s.N + n];
    s.out[(size_t)m * s.ldo + n] = (bf16)apply_act(o, s.act);
  }  if (s.arf.world) ar_fused_tail(s.arf, s.out, s.M, s.N, n0, COLS);
}


// FP8 (OCP e4m3) weight-and-activation decode GEMM, M <= 4: W8A8 with a per-output-channel weight
// scale and a per-row dynamic activation scale, on v_mfma_f32_16x16x32_fp8_fp8.  Half the weight
// bytes of the bf16 stream (decode is weight-bandwidth bound).  W is packed in 1 KiB granules of
// 16 rows x 64 k ([N/16][K/64][g][nr][2 k-steps][8]), so one 16-B load per lane feeds two MFMAs.
// Prologue: A (+ A2) staged in LDS as bf16 with the row square sums and |max|, then requantised
// in place to fp8 with scale |max| / 448; epilogue: acc * s_a[m] * s_w[n] (* rstd[m]).
template <int UNROLL, int NWV, int FUSE>
__global__ __launch_bounds__(NWV * 64) void skinny_fp8_kernel(const SkArgs s) {
  extern __shared__ __attribute__((aligned(16))) uint4 a_lds[];  // bf16 [M][K], then fp8 [M][K]
  __shared__ float red[NWV][16][17];
  __shared__ float ssq_s[4];
  __shared__ int amax_s[4];
  constexpr int T = NWV * 64;
  constexpr bool NORM = FUSE == FUSE_NORM || FUSE == FUSE_ADD_NORM;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nr = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const int kgs = s.K >> 6;  // 64-wide granules per row
  const int kch = s.K >> 3;
  const int nq = s.M * kch;
  const int kpw = (kgs + NWV - 1) / NWV;
  const int kb = wid * kpw, ke = min(kgs, kb + kpw);
  const rsrc_t wr = make_rsrc(s.w, s.w_bytes);
  const rsrc_t ar = make_rsrc(s.a, s.a_bytes);
  const rsrc_t a2r = make_rsrc(s.a2, FUSE == FUSE_ADD_NORM ? s.a_bytes : 0);
  const int wbase = blockIdx.x * kgs * 1024 + lane * 16;

  auto load_trip = [&](int kg0, uint4 (&wv)[UNROLL]) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) wv[u] = bload16_pol<1>(wr, kg0 + u < ke ? wbase + (kg0 + u) * 1024 : OOB);
  };
  constexpr int QPT = 2048 / T;
  uint4 a0[QPT], a20[QPT];
#pragma unroll
  for (int j = 0; j < QPT; ++j) {
    const int q = tid + j * T;
    const int m = fastdiv(q, s.fd_kch), c = q - m * kch;
    const int off = q < nq ? (m * s.lda + c * 8) * 2 : OOB;
    a0[j] = bload16(ar, off);
    if constexpr (FUSE == FUSE_ADD_NORM) a20[j] = bload16(a2r, off);
  }
  uint4 wnext[UNROLL];
  load_trip(kb, wnext);

  if (tid < 4) {
    ssq_s[tid] = 0.f;
    amax_s[tid] = 0;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  float part[4] = {0.f, 0.f, 0.f, 0.f}, amx[4] = {0.f, 0.f, 0.f, 0.f};
  const bool wr_res = FUSE == FUSE_ADD_NORM && s.a_out && blockIdx.x == 0;
  auto stage = [&](int q, uint4 v, uint4 v2) {
    const int m = fastdiv(q, s.fd_kch), c = q - m * kch;
    if constexpr (FUSE == FUSE_ADD_NORM) {
      v = add_round(v, v2);
      if (wr_res) st16(s.a_out + (size_t)m * s.lda + c * 8, v);
    }
    a_lds[q] = v;
    float x[8];
    unpack8(v, x);
    float sq = 0.f, mx = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sq += x[e] * x[e];
      mx = fmaxf(mx, fabsf(x[e]));
    }
#pragma unroll
    for (int mm = 0; mm < 4; ++mm) {
      part[mm] += mm == m ? sq : 0.f;
      amx[mm] = mm == m ? fmaxf(amx[mm], mx) : amx[mm];
    }
  };
#pragma unroll
  for (int j = 0; j < QPT; ++j)
    if (tid + j * T < nq) stage(tid + j * T, a0[j], a20[j]);
  for (int q = tid + QPT * T; q < nq; q += T) {
    const int m = fastdiv(q, s.fd_kch), c = q - m * kch;
    stage(q, ld16(s.a + (size_t)m * s.lda + c * 8),
          FUSE == FUSE_ADD_NORM ? ld16(s.a2 + (size_t)m * s.lda + c * 8) : make_uint4(0, 0, 0, 0));
  }
#pragma unroll
  for (int mm = 0; mm < 4; ++mm) {
    const float t = wave_sum(part[mm]);
    const float mxw = wave_max(amx[mm]);
    if (lane == 0 && mm < s.M) {
      if constexpr (NORM) atomicAdd(&ssq_s[mm], t);
      atomicMax(&amax_s[mm], __float_as_int(mxw));  // non-negative floats order as their bits
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  // requantise A to fp8 in place: every thread first reads its chunks, then (after a barrier) writes
  float inv[4];
#pragma unroll
  for (int mm = 0; mm < 4; ++mm) {
    const float amax = __int_as_float(amax_s[mm]);
    inv[mm] = amax > 0.f ? 448.f / amax : 0.f;
  }
  constexpr int QMAX = 4096 / T;  // M * K / 8 <= 4096 chunks (host: M * K * 2 <= 64 KiB)
  uint4 hold[QMAX];
#pragma unroll
  for (int j = 0; j < QMAX; ++j) {
    const int q = tid + j * T;
    hold[j] = q < nq ? a_lds[q] : make_uint4(0, 0, 0, 0);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  uint2* a8 = reinterpret_cast<uint2*>(a_lds);  // fp8 [M][K]: chunk q -> 8 bytes at q * 8
#pragma unroll
  for (int j = 0; j < QMAX; ++j) {
    const int q = tid + j * T;
    if (q < nq) {
      const int m = fastdiv(q, s.fd_kch);
      const float sc = m == 0 ? inv[0] : m == 1 ? inv[1] : m == 2 ? inv[2] : inv[3];
      float x[8];
      unpack8(hold[j], x);
      int lo = __builtin_amdgcn_cvt_pk_fp8_f32(x[0] * sc, x[1] * sc, 0, false);
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(x[2] * sc, x[3] * sc, lo, true);
      int hi = __builtin_amdgcn_cvt_pk_fp8_f32(x[4] * sc, x[5] * sc, 0, false);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(x[6] * sc, x[7] * sc, hi, true);
      a8[q] = make_uint2((uint32_t)lo, (uint32_t)hi);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool arow = nr < s.M;
  const char* a8b = reinterpret_cast<const char*>(a_lds) + nr * s.K + 8 * g;
  for (int kg = kb; kg < ke; kg += UNROLL) {
    uint4 wv[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) wv[u] = wnext[u];
    if (kg + UNROLL < ke) load_trip(kg + UNROLL, wnext);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int k = kg + u;
      const bool ok = arow && k < ke;
      const long x0 = ok ? *reinterpret_cast<const long*>(a8b + k * 64) : 0;
      const long x1 = ok ? *reinterpret_cast<const long*>(a8b + k * 64 + 32) : 0;
      const long w0 = (long)(((unsigned long)wv[u].y << 32) | wv[u].x);
      const long w1 = (long)(((unsigned long)wv[u].w << 32) | wv[u].z);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(x0, w0, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(x1, w1, acc, 0, 0, 0);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) red[wid][4 * g + i][nr] = acc[i];
  __syncthreads();
  const bool glu = s.act == ACT_SILU_MUL;
  for (int q = tid; q < s.M * 16; q += T) {
    const int m = q >> 4, c = q & 15;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NWV; ++w) v += red[w][m][c];
    const float sa = __int_as_float(amax_s[m]) * (1.f / 448.f);
    const float rs = (NORM ? rsqrtf(ssq_s[m] / (float)s.K + s.eps) : 1.f) * sa;
    const int n = n0 + c;
    v *= rs * s.wscale[n];
    if (glu) {
      if (c < 8) {
        float up = 0.f;
#pragma unroll
        for (int w = 0; w < NWV; ++w) up += red[w][m][c + 8];
        up *= rs * s.wscale[n + 8];
        s.out[(size_t)m * s.ldo + (n >> 4) * 8 + (n & 7)] = (bf16)(silu(epi(v, n, s)) * epi(up, n + 8, s));
      }
      continue;
    }
    float o = epi(v, n, s);
    if (s.res) o += (float)s.res[(size_t)m * s.N + n];
    s.out[(size_t)m * s.ldo + n] = (bf16)apply_act(o, s.act);
  }
}

// [N][K] row-major -> [N/16][K/32][4][16][8] (the packed granule layout above)
__global__ __launch_bounds__(256) void pack_skinny_kernel(const bf16* __restrict__ w, bf16* __restrict__ wp, int N,
                                                          int K) {
  const int ksteps = K >> 5;
  const long total = (long)N * (K >> 3);  // 16-B chunks
  for (long q = blockIdx.x * 256L + threadIdx.x; q < total; q += (long)gridDim.x * 256) {
    const int lane = (int)(q & 63);
    const long gr = q >> 6;  // granule = tile * ksteps + ks
    const int ks = (int)(gr % ksteps), tile = (int)(gr / ksteps);
    const int n = tile * 16 + (lane & 15), k = ks * 32 + 8 * (lane >> 4);
    st16(wp + q * 8, ld16(w + (size_t)n * K + k));
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
    if (s.norm) {
      float t2 = 0.f;
      for (int sp = 0; sp < s.nsplit; ++sp) t2 += s.ws[(size_t)s.nsplit * s.M * s.N + sp * s.M + m];
      const float rs = rsqrtf(t2 / (float)s.K + s.eps);
      v *= rs;
      u *= rs;
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

int g_skinny_no_lds = 0;     // A/B switch for probes (mls_skinny_set_variant)
int g_skinny_max_split = 0;  // cap on the automatic cross-block K split (0: none)

extern "C" {

int mls_ar_fuse_desc(void* ctx, long n, ArFuse* f);  // custom_allreduce.hip

int mls_skinny_set_variant(int no_lds) {
  g_skinny_no_lds = no_lds;
  return 0;
}

int mls_skinny_set_max_split(int cap) {
  g_skinny_max_split = cap;
  return 0;
}

// M <= 32, N % 16 == 0, K % 8 == 0.  nsplit <= 0: auto (fill the chip).  ws: >= nsplit*M*(N+1) floats.
// A2 / A_out / norm: the fused residual-add + RMSNorm prologue (header comment); A_out must not alias A/A2.
int mls_skinny_gemm_norm(const void* A, const void* A2, void* A_out, const void* W, const float* bias, const void* res,
                         void* out, void* ws, size_t ws_bytes, int M, int N, int K, int act, int nsplit, int norm,
                         float eps, void* stream) {
  if (M <= 0 || M > 32 || N % 16 || K % 8 || K <= 0) return MLS_BAD_ARG;
  if (A_out && (A_out == A || A_out == A2)) return MLS_BAD_ARG;
  SkArgs s{};
  s.a = (const bf16*)A;
  s.a2 = (const bf16*)A2;
  s.a_out = (bf16*)A_out;
  s.norm = norm;
  s.eps = eps;
  s.w = (const bf16*)W;
  s.bias = bias;
  s.res = (const bf16*)res;
  s.out = (bf16*)out;
  s.ws = (float*)ws;
  s.M = M; s.N = N; s.K = K; s.lda = K;
  s.fd_kch = fastdiv_make((uint32_t)(K >> 3));
  s.act = act;
  s.ldo = act == ACT_SILU_MUL ? N / 2 : N;
  const size_t ab = (size_t)M * K * 2, wb = (size_t)N * K * 2;
  if (ab >= 0x7FFFFFFFull || wb >= 0x7FFFFFFFull) return MLS_UNSUPPORTED;
  s.a_bytes = (uint32_t)ab;
  s.w_bytes = (uint32_t)wb;
  // M > 2: NT tiles per block while that still leaves >= 384 blocks (1.5 per CU) -- measured: NT = 4
  // halves gate_up at M = 16 but costs ~10 % at M = 1, where the activation traffic is negligible
  // and the deeper single-tile unroll wins (profiles/r1_decode_probe.jsonl).  K is split across
  // blocks only when even single-tile blocks cannot cover 256 CUs.
  int nt = 1;
  while (M > 2 && nt < 4 && N % (32 * nt) == 0 && N / (32 * nt) >= 384) nt *= 2;
  const int tiles = N / (16 * nt);
  const int ksteps = (K + 31) / 32;
  if (nsplit <= 0) {  // 8 waves split K inside a block; split across blocks only below 256 blocks
    nsplit = 1;
    // M <= 4 with >= 32 column tiles: never split -- the finish launch costs more than the idle
    // CUs (emulated TP = 8 rank, batch 1: 1.55 -> 1.44 ms/token; TP = 1 unchanged, its GEMMs
    // already have >= 256 tiles).  At M = 8 the split still wins (1.67 vs 1.73 ms/token).
    const bool no_split = M <= 4 && tiles >= 32;
    while (!no_split && tiles * nsplit < 256 && ksteps / (nsplit * 2) >= 32) nsplit *= 2;
    if (g_skinny_max_split > 0 && nsplit > g_skinny_max_split) nsplit = g_skinny_max_split;
  }
  if (nsplit > 1 && (ws == nullptr || ws_bytes < (size_t)nsplit * M * (N + 1) * 4)) nsplit = 1;
  s.nsplit = nsplit;
  s.ksteps_per_split = (ksteps + nsplit - 1) / nsplit;
  dim3 grid(tiles, nsplit);
  hipStream_t st = (hipStream_t)stream;
  if ((A2 || A_out) && !norm) return MLS_UNSUPPORTED;  // the residual add exists only as the norm prologue
  const int mode = A2 ? FUSE_ADD_NORM : norm ? FUSE_NORM : FUSE_NONE;
  const size_t a_lds_bytes = (size_t)M * K * 2;
  if (M <= 4 && nsplit == 1 && K % 32 == 0 && a_lds_bytes <= 65536 && !g_skinny_no_lds) {
#define MLS_SKL(UN, NT_)                                                                                        \
  switch (mode) {                                                                                               \
    case FUSE_NONE:                                                                                             \
      hipLaunchKernelGGL((skinny_lds_kernel<UN, 8, FUSE_NONE, NT_>), grid, dim3(512), a_lds_bytes, st, s); break; \
    case FUSE_NORM:                                                                                             \
      hipLaunchKernelGGL((skinny_lds_kernel<UN, 8, FUSE_NORM, NT_>), grid, dim3(512), a_lds_bytes, st, s); break; \
    default:                                                                                                    \
      hipLaunchKernelGGL((skinny_lds_kernel<UN, 8, FUSE_ADD_NORM, NT_>), grid, dim3(512), a_lds_bytes, st, s);    \
      break;                                                                                                    \
  }
    if (nt == 4) {
      MLS_SKL(4, 4)
    } else if (nt == 2) {
      MLS_SKL(4, 2)
    } else {
      MLS_SKL(8, 1)
    }
#undef MLS_SKL
    return (int)hipGetLastError();
  }
#define MLS_SKINNY_F(TMS, UN, NT_)                                                                             \
  switch (mode) {                                                                                              \
    case FUSE_NONE:                                                                                            \
      hipLaunchKernelGGL((skinny_gemm_kernel<TMS, UN, 8, FUSE_NONE, NT_>), grid, dim3(512), 0, st, s); break;   \
    case FUSE_NORM:                                                                                            \
      hipLaunchKernelGGL((skinny_gemm_kernel<TMS, UN, 8, FUSE_NORM, NT_>), grid, dim3(512), 0, st, s); break;   \
    default:                                                                                                   \
      hipLaunchKernelGGL((skinny_gemm_kernel<TMS, UN, 8, FUSE_ADD_NORM, NT_>), grid, dim3(512), 0, st, s); break; \
  }
#define MLS_SKINNY(TMS, UN)                      \
  if (nt == 4) {                                 \
    MLS_SKINNY_F(TMS, (UN > 4 ? 4 : UN), 4)      \
  } else if (nt == 2) {                          \
    MLS_SKINNY_F(TMS, UN, 2)                     \
  } else {                                       \
    MLS_SKINNY_F(TMS, UN, 1)                     \
  }
  if (M <= 16) {
    MLS_SKINNY(1, 8)
  } else {
    MLS_SKINNY(2, 4)
  }
#undef MLS_SKINNY
#undef MLS_SKINNY_F
  if (nsplit > 1) {
    const long total = (long)M * (act == ACT_SILU_MUL ? N / 2 : N);
    int blocks = (int)((total + 255) / 256);
    blocks = blocks > 2048 ? 2048 : blocks;
    hipLaunchKernelGGL(skinny_finish_kernel, dim3(blocks), dim3(256), 0, st, s);
  }
  return (int)hipGetLastError();
}

// W [N][K] -> packed granules (N % 16 == 0, K % 32 == 0); Wp must not alias W.
int mls_skinny_pack(const void* W, void* Wp, int N, int K, void* stream) {
  if (N <= 0 || K <= 0 || N % 16 || K % 32 || W == Wp) return MLS_BAD_ARG;
  const long chunks = (long)N * (K / 8);
  int blocks = (int)((chunks + 255) / 256);
  blocks = blocks > 4096 ? 4096 : blocks;
  hipLaunchKernelGGL(pack_skinny_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const bf16*)W, (bf16*)Wp,
                     N, K);
  return (int)hipGetLastError();
}

// Packed-weight skinny GEMM (+ optional fused add + RMSNorm prologue), M <= 32.  M <= 4 with A
// within 64 KiB stages A in LDS (skinny_packed_kernel), otherwise A rides in registers
// (skinny_packed_reg_kernel; variant | 16 forces it).  variant = probe knob, (granules per trip,
// waves, non-temporal): 0 (8,8,no) 1 (8,8,nt) 2 (8,4,no) 3 (8,4,nt) 4 (16,8,no) 5 (16,8,nt)
// 6 (16,4,no) 7 (16,4,nt) 8 (8,16,nt) 9 (4,16,nt; the measured default) 10 (4,8,nt); register
// path only: 11 / 12 = (4,8) over 2 / 4 column tiles per block, 13 = (4,16) over 2.
static int skinny_packed_impl(const void* A, const void* A2, void* A_out, const void* Wp, const float* bias,
                              const void* res, void* out, int M, int N, int K, int act, int norm, float eps, int variant,
                              void* stream, const ArFuse* arf) {
  if (M <= 0 || M > 32 || N % 16 || K % 32 || K <= 0) return MLS_BAD_ARG;
  if (A_out && (A_out == A || A_out == A2)) return MLS_BAD_ARG;
  if ((A2 || A_out) && !norm) return MLS_UNSUPPORTED;
  const size_t ab = (size_t)M * K * 2, wb = (size_t)N * K * 2;
  if (wb >= 0x7FFFFFFFull) return MLS_UNSUPPORTED;
  SkArgs s{};
  s.a = (const bf16*)A;
  s.a2 = (const bf16*)A2;
  s.a_out = (bf16*)A_out;
  s.norm = norm;
  s.eps = eps;
  s.w = (const bf16*)Wp;
  s.bias = bias;
  s.res = (const bf16*)res;
  s.out = (bf16*)out;
  s.M = M; s.N = N; s.K = K; s.lda = K;
  s.fd_kch = fastdiv_make((uint32_t)(K >> 3));
  s.act = act;
  s.ldo = act == ACT_SILU_MUL ? N / 2 : N;
  s.a_bytes = (uint32_t)ab;
  s.w_bytes = (uint32_t)wb;
  s.nsplit = 1;
  if (arf) s.arf = *arf;
  const int mode = A2 ? FUSE_ADD_NORM : norm ? FUSE_NORM : FUSE_NONE;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid(N / 16);
  if (M > 4 || ab > 65536 || (variant & 16)) {  // A fragments from L2 in registers (16: forced)
#define MLS_SKR3(UN, NW, NT_, TM)                                                                               \
  switch (mode) {                                                                                                 \
    case FUSE_NONE:                                                                                               \
      hipLaunchKernelGGL((skinny_packed_reg_kernel<UN, NW, FUSE_NONE, 1, NT_, TM>), dim3(N / (16 * NT_)),          \
                         dim3(NW * 64), 0, st, s);                                                                \
      break;                                                                                                      \
    case FUSE_NORM:                                                                                               \
      hipLaunchKernelGGL((skinny_packed_reg_kernel<UN, NW, FUSE_NORM, 1, NT_, TM>), dim3(N / (16 * NT_)),          \
                         dim3(NW * 64), 0, st, s);                                                                \
      break;                                                                                                      \
    default:                                                                                                      \
      hipLaunchKernelGGL((skinny_packed_reg_kernel<UN, NW, FUSE_ADD_NORM, 1, NT_, TM>), dim3(N / (16 * NT_)),      \
                         dim3(NW * 64), 0, st, s);                                                                \
      break;                                                                                                      \
  }
#define MLS_SKR(UN, NW, NT_) MLS_SKR3(UN, NW, NT_, 1)
    int v = variant & 15;
    if (M > 16) {  // two 16-row A fragments per granule
      if (N / 16 >= 384 && N % 32 == 0 && v != 10) {
        MLS_SKR3(4, 8, 2, 2)  // 8 waves: the double-buffered 2-tile trip needs > 128 VGPRs
      } else if (v == 10) {
        MLS_SKR3(4, 8, 1, 2)
      } else {
        MLS_SKR3(4, 16, 1, 2)
      }
      return (int)hipGetLastError();
    }
    // default: two column tiles per block once there are >= 384 tiles (A fragments amortised over
    // two weight granules; M = 8: QKV 14.3 -> 12.1 us, gate_up 47.0 -> 43.4), else one tile, 16 waves
    // (profiles/r2_decode_packed_weight_probe.jsonl)
    if (v == 9 && N / 16 >= 384) v = 11;
    if ((v == 11 || v == 13) && N % 32) v = 9;
    if (v == 12 && N % 64) v = 9;
    switch (v) {
      case 1: MLS_SKR(8, 8, 1) break;
      case 10: MLS_SKR(4, 8, 1) break;
      case 11: MLS_SKR(4, 8, 2) break;
      case 12: MLS_SKR(4, 8, 4) break;
      case 13: MLS_SKR(4, 16, 2) break;
      default: MLS_SKR(4, 16, 1) break;
    }
#undef MLS_SKR
#undef MLS_SKR3
    return (int)hipGetLastError();
  }
#define MLS_SKP(UN, NW, NTL_)                                                                                 \
  switch (mode) {                                                                                               \
    case FUSE_NONE:                                                                                             \
      hipLaunchKernelGGL((skinny_packed_kernel<UN, NW, FUSE_NONE, NTL_>), grid, dim3(NW * 64), ab, st, s); break; \
    case FUSE_NORM:                                                                                             \
      hipLaunchKernelGGL((skinny_packed_kernel<UN, NW, FUSE_NORM, NTL_>), grid, dim3(NW * 64), ab, st, s); break; \
    default:                                                                                                    \
      hipLaunchKernelGGL((skinny_packed_kernel<UN, NW, FUSE_ADD_NORM, NTL_>), grid, dim3(NW * 64), ab, st, s);    \
      break;                                                                                                    \
  }
  switch (variant) {
    case 0: MLS_SKP(8, 8, 0) break;
    case 2: MLS_SKP(8, 4, 0) break;
    case 3: MLS_SKP(8, 4, 1) break;
    case 4: MLS_SKP(16, 8, 0) break;
    case 5: MLS_SKP(16, 8, 1) break;
    case 6: MLS_SKP(16, 4, 0) break;
    case 7: MLS_SKP(16, 4, 1) break;
    case 8: MLS_SKP(8, 16, 1) break;
    case 9: MLS_SKP(4, 16, 1) break;
    case 10: MLS_SKP(4, 8, 1) break;
    default: MLS_SKP(8, 8, 1) break;  // 1: the measured default
  }
#undef MLS_SKP
  return (int)hipGetLastError();
}

// Packed-weight decode GEMM whose A operand is the split-KV decode attention's output, merged
// from its partials in the prologue (FUSE_COMBINE; the attention launch then skips its combine
// kernel).  M <= 4, M * K * 2 <= 64 KiB, K == Hq * D, D % 8 == 0.
static int skinny_packed_combine_impl(const void* A, const float* cws, const float* cml, const int* lens, int nsplit,
                                      int chunk, int Hq, int D, const void* Wp, const float* bias, const void* res,
                                      void* out, int M, int N, int K, int act, int variant, void* stream,
                                      const ArFuse* arf) {
  if (M <= 0 || M > 4 || N % 16 || K % 32 || K != Hq * D || D % 8 || nsplit <= 0 || chunk <= 0) return MLS_BAD_ARG;
  const size_t ab = (size_t)M * K * 2, wb = (size_t)N * K * 2;
  if (wb >= 0x7FFFFFFFull || ab > 65536) return MLS_UNSUPPORTED;
  SkArgs s{};
  s.a = (const bf16*)A;
  s.w = (const bf16*)Wp;
  s.bias = bias;
  s.res = (const bf16*)res;
  s.out = (bf16*)out;
  s.M = M; s.N = N; s.K = K; s.lda = K;
  s.fd_kch = fastdiv_make((uint32_t)(K >> 3));
  s.act = act;
  s.ldo = act == ACT_SILU_MUL ? N / 2 : N;
  s.a_bytes = (uint32_t)ab;
  s.w_bytes = (uint32_t)wb;
  s.nsplit = 1;
  s.cws = cws;
  s.cml = cml;
  s.lens = lens;
  s.c_nsplit = nsplit;
  s.c_chunk = chunk;
  s.c_hq = Hq;
  s.c_hd = D;
  s.fd_hd = fastdiv_make((uint32_t)D);
  if (arf) s.arf = *arf;
  hipStream_t st = (hipStream_t)stream;
  if (variant == 1)
    hipLaunchKernelGGL((skinny_packed_kernel<8, 8, FUSE_COMBINE, 1>), dim3(N / 16), dim3(512), ab, st, s);
  else
    hipLaunchKernelGGL((skinny_packed_kernel<4, 16, FUSE_COMBINE, 1>), dim3(N / 16), dim3(1024), ab, st, s);
  return (int)hipGetLastError();
}

int mls_skinny_packed(const void* A, const void* A2, void* A_out, const void* Wp, const float* bias, const void* res,
                      void* out, int M, int N, int K, int act, int norm, float eps, int variant, void* stream) {
  return skinny_packed_impl(A, A2, A_out, Wp, bias, res, out, M, N, K, act, norm, eps, variant, stream, nullptr);
}

int mls_skinny_packed_combine(const void* A, const float* cws, const float* cml, const int* lens, int nsplit,
                              int chunk, int Hq, int D, const void* Wp, const float* bias, const void* res, void* out,
                              int M, int N, int K, int act, int variant, void* stream) {
  return skinny_packed_combine_impl(A, cws, cml, lens, nsplit, chunk, Hq, D, Wp, bias, res, out, M, N, K, act, variant,
                                    stream, nullptr);
}

// Row-parallel tensor-parallel projection with its all-reduce FUSED (ar_protocol.h): out = the sum
// over the ranks of A . Wp^T, reduced in this launch through the one-shot IPC context ar_ctx
// (custom_allreduce.hip) -- no bias / residual / activation (they would be summed world times).
// out must be contiguous [M][N] with M * N * 2 <= the context's one-shot cap.
static int ar_fuse_check(void* ar_ctx, const float* bias, const void* res, int act, int M, int N, ArFuse* f) {
  if (!ar_ctx || bias || res || act != ACT_NONE) return MLS_BAD_ARG;
  return mls_ar_fuse_desc(ar_ctx, (long)M * N, f);
}

int mls_skinny_packed_ar(const void* A, const void* A2, void* A_out, const void* Wp, const void* out_, int M, int N,
                         int K, int norm, float eps, int variant, void* ar_ctx, void* stream) {
  ArFuse f;
  const int rc = ar_fuse_check(ar_ctx, nullptr, nullptr, ACT_NONE, M, N, &f);
  if (rc) return rc;
  return skinny_packed_impl(A, A2, A_out, Wp, nullptr, nullptr, const_cast<void*>(out_), M, N, K, ACT_NONE, norm, eps,
                            variant, stream, &f);
}

int mls_skinny_packed_combine_ar(const void* A, const float* cws, const float* cml, const int* lens, int nsplit,
                                 int chunk, int Hq, int D, const void* Wp, void* out, int M, int N, int K, int variant,
                                 void* ar_ctx, void* stream) {
  ArFuse f;
  const int rc = ar_fuse_check(ar_ctx, nullptr, nullptr, ACT_NONE, M, N, &f);
  if (rc) return rc;
  return skinny_packed_combine_impl(A, cws, cml, lens, nsplit, chunk, Hq, D, Wp, nullptr, nullptr, out, M, N, K,
                                    ACT_NONE, variant, stream, &f);
}

// FP8 (e4m3) decode GEMM (W8A8, see skinny_fp8_kernel): M <= 4, K % 64 == 0, M * K * 2 <= 64 KiB.
// Wq: packed fp8 granules; wscale [N] fp32.  Same fusion options as mls_skinny_packed.
int mls_skinny_fp8(const void* A, const void* A2, void* A_out, const void* Wq, const float* wscale, const float* bias,
                   const void* res, void* out, int M, int N, int K, int act, int norm, float eps, int variant,
                   void* stream) {
  if (M <= 0 || M > 4 || N % 16 || K % 64 || K <= 0 || !wscale) return MLS_BAD_ARG;
  if (A_out && (A_out == A || A_out == A2)) return MLS_BAD_ARG;
  if ((A2 || A_out) && !norm) return MLS_UNSUPPORTED;
  const size_t ab = (size_t)M * K * 2, wb = (size_t)N * K;
  if (wb >= 0x7FFFFFFFull || ab > 65536) return MLS_UNSUPPORTED;
  SkArgs s{};
  s.a = (const bf16*)A;
  s.a2 = (const bf16*)A2;
  s.a_out = (bf16*)A_out;
  s.norm = norm;
  s.eps = eps;
  s.w = (const bf16*)Wq;
  s.wscale = wscale;
  s.bias = bias;
  s.res = (const bf16*)res;
  s.out = (bf16*)out;
  s.M = M; s.N = N; s.K = K; s.lda = K;
  s.fd_kch = fastdiv_make((uint32_t)(K >> 3));
  s.act = act;
  s.ldo = act == ACT_SILU_MUL ? N / 2 : N;
  s.a_bytes = (uint32_t)ab;
  s.w_bytes = (uint32_t)wb;
  s.nsplit = 1;
  const int mode = A2 ? FUSE_ADD_NORM : norm ? FUSE_NORM : FUSE_NONE;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid(N / 16);
#define MLS_SK8(UN, NW)                                                                                     \
  switch (mode) {                                                                                           \
    case FUSE_NONE: hipLaunchKernelGGL((skinny_fp8_kernel<UN, NW, FUSE_NONE>), grid, dim3(NW * 64), ab, st, s); break; \
    case FUSE_NORM: hipLaunchKernelGGL((skinny_fp8_kernel<UN, NW, FUSE_NORM>), grid, dim3(NW * 64), ab, st, s); break; \
    default: hipLaunchKernelGGL((skinny_fp8_kernel<UN, NW, FUSE_ADD_NORM>), grid, dim3(NW * 64), ab, st, s); break;    \
  }
  // variant: 1 (default) 4 granules per trip x 8 waves; 0: 4 x 16; 2: 2 x 16
  // (profiles/r2_decode_fp8_weight_probe.jsonl: 1 is fastest on every Llama-3-8B shape)
  if (variant == 0) {
    MLS_SK8(4, 16)
  } else if (variant == 2) {
    MLS_SK8(2, 16)
  } else {
    MLS_SK8(4, 8)
  }
#undef MLS_SK8
  return (int)hipGetLastError();
}

int mls_skinny_gemm(const void* A, const void* W, const float* bias, const void* res, void* out, void* ws,
                    size_t ws_bytes, int M, int N, int K, int act, int nsplit, void* stream) {
  return mls_skinny_gemm_norm(A, nullptr, nullptr, W, bias, res, out, ws, ws_bytes, M, N, K, act, nsplit, 0, 0.f,
                              stream);
}

}  // extern "C"
