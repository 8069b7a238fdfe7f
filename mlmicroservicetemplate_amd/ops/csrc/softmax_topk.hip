// K6 (row softmax, numerically stable, optional additive mask) and K7 (row top-k), plus the
// fused classifier head softmax -> top-k that ResNet-50 / BERT serving emit per request.
// One 256-thread workgroup (4 waves) per row; the row is staged once in LDS as fp32, so the k
// selection rounds re-read LDS, never HBM (cdna_hip_programming.md App. B "Reduction").
#include "common.h"

namespace {

struct KV {
  float v;
  int i;
};

MLS_DEV KV better(KV a, KV b) {  // larger value wins; ties -> smaller index (stable)
  if (b.v > a.v || (b.v == a.v && b.i < a.i && b.i >= 0)) return b;
  return a;
}

MLS_DEV KV wave_argmax(KV x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    KV y;
    y.v = __shfl_xor(x.v, o, 64);
    y.i = __shfl_xor(x.i, o, 64);
    x = better(x, y);
  }
  return x;
}

MLS_DEV KV block_argmax(KV x, float* rv, int* ri) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  x = wave_argmax(x);
  __syncthreads();
  if (lane == 0) {
    rv[wid] = x.v;
    ri[wid] = x.i;
  }
  __syncthreads();
  KV t{-INFINITY, -1};
  if (lane < nw) t = KV{rv[lane], ri[lane]};
  return wave_argmax(t);
}

template <typename Tin>
MLS_DEV float load_as_f32(const Tin* p, long i);
template <>
MLS_DEV float load_as_f32<bf16>(const bf16* p, long i) { return (float)p[i]; }
template <>
MLS_DEV float load_as_f32<float>(const float* p, long i) { return p[i]; }

// softmax (optional) + top-k per row.  `apply_softmax`: 1 -> values are probabilities,
// 0 -> raw logits (plain top-k).  Dynamic LDS: N floats.
template <typename Tin>
__global__ __launch_bounds__(256) void softmax_topk_kernel(const Tin* __restrict__ x, float* __restrict__ vals,
                                                           int* __restrict__ idx, int N, int k, int apply_softmax,
                                                           float temperature) {
  extern __shared__ __attribute__((aligned(16))) float row[];
  __shared__ float rv[16];
  __shared__ int ri[16];
  const long r = blockIdx.x;
  const Tin* src = x + r * (long)N;
  const float invt = 1.f / temperature;
  float mx = -INFINITY;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    const float v = load_as_f32<Tin>(src, i) * invt;
    row[i] = v;
    mx = fmaxf(mx, v);
  }
  float denom = 1.f;
  if (apply_softmax) {
    mx = block_max(mx, rv);
    float s = 0.f;
    for (int i = threadIdx.x; i < N; i += blockDim.x) s += __expf(row[i] - mx);
    denom = block_sum(s, rv);
  }
  __syncthreads();
  for (int j = 0; j < k; ++j) {
    KV best{-INFINITY, -1};
    for (int i = threadIdx.x; i < N; i += blockDim.x) best = better(best, KV{row[i], i});
    best = block_argmax(best, rv, ri);
    if (threadIdx.x == 0) {
      const float v = apply_softmax ? __expf(best.v - mx) / denom : best.v;
      vals[r * k + j] = v;
      idx[r * k + j] = best.i;
      if (best.i >= 0) row[best.i] = -INFINITY;
    }
    __syncthreads();
  }
}

// Wave-per-row variant for rows up to 4096 (the classifier heads): no block barriers, the k
// selection rounds are pure wave shuffles.  4 rows per 256-thread block, LDS N floats per wave.
template <typename Tin>
__global__ __launch_bounds__(256) void softmax_topk_wave_kernel(const Tin* __restrict__ x, float* __restrict__ vals,
                                                                int* __restrict__ idx, int rows, int N, int k,
                                                                int apply_softmax, float temperature) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const long r = (long)blockIdx.x * 4 + wid;
  if (r >= rows) return;
  float* row = lds + wid * N;
  const Tin* src = x + r * (long)N;
  const float invt = 1.f / temperature;
  float mx = -INFINITY;
  for (int i = lane; i < N; i += 64) {
    const float v = load_as_f32<Tin>(src, i) * invt;
    row[i] = v;
    mx = fmaxf(mx, v);
  }
  float denom = 1.f;
  if (apply_softmax) {
    mx = wave_max(mx);
    float s = 0.f;
    for (int i = lane; i < N; i += 64) s += __expf(row[i] - mx);
    denom = wave_sum(s);
  }
  for (int j = 0; j < k; ++j) {
    KV best{-INFINITY, -1};
    for (int i = lane; i < N; i += 64) best = better(best, KV{row[i], i});
    best = wave_argmax(best);
    if (lane == 0) {
      vals[r * k + j] = apply_softmax ? __expf(best.v - mx) / denom : best.v;
      idx[r * k + j] = best.i;
    }
    if (best.i >= 0 && (best.i & 63) == lane) row[best.i] = -INFINITY;
  }
}

// Register-resident variant for bf16 rows with N % 8 == 0, N <= 512 * CPL (the ResNet / BERT
// classifier heads): a wave owns a row, every lane issues all its 16-B loads up front (one memory
// round trip, where the strided scalar loop above paid one per element group), and the k selection
// rounds scan registers + wave shuffles -- no LDS at all.
template <int CPL>
__global__ __launch_bounds__(256) void softmax_topk_reg_kernel(const bf16* __restrict__ x, float* __restrict__ vals,
                                                               int* __restrict__ idx, int rows, int N, int k,
                                                               int apply_softmax, float temperature, int chunks,
                                                               int valid) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const long r = (long)blockIdx.x * 4 + wid;
  if (r >= rows) return;
  const int nch = N >> 3;
  // rows may be `chunks` equal pieces of one longer row: columns at or past `valid` of that row
  // (a vocab shard's padded tail) are excluded before the selection
  const int limit = valid - (int)(r % chunks) * N;
  const bf16* src = x + r * (long)N;
  const float invt = 1.f / temperature;
  float v[CPL][8];
  uint4 raw[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int ch = lane + 64 * c;
    raw[c] = ch < nch ? ld16(src + ch * 8) : make_uint4(0, 0, 0, 0);
  }
  float mx = -INFINITY;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const bool ok = lane + 64 * c < nch;
    unpack8(raw[c], v[c]);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[c][e] = ok && (lane + 64 * c) * 8 + e < limit ? v[c][e] * invt : -INFINITY;
      mx = fmaxf(mx, v[c][e]);
    }
  }
  float denom = 1.f;
  if (apply_softmax) {
    mx = wave_max(mx);
    float sum = 0.f;
#pragma unroll
    for (int c = 0; c < CPL; ++c)
#pragma unroll
      for (int e = 0; e < 8; ++e) sum += v[c][e] == -INFINITY ? 0.f : __expf(v[c][e] - mx);
    denom = wave_sum(sum);
  }
  for (int j = 0; j < k; ++j) {
    KV best{-INFINITY, -1};
#pragma unroll
    for (int c = 0; c < CPL; ++c)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int i = (lane + 64 * c) * 8 + e;
        if (lane + 64 * c < nch) best = better(best, KV{v[c][e], i});
      }
    best = wave_argmax(best);
    if (lane == 0) {
      vals[r * k + j] = apply_softmax ? __expf(best.v - mx) / denom : best.v;
      idx[r * k + j] = best.i;
    }
    if (best.i >= 0 && ((best.i >> 3) & 63) == lane) {  // owner lane retires the winner
      const int c = (best.i >> 3) >> 6, e = best.i & 7;
#pragma unroll
      for (int cc = 0; cc < CPL; ++cc)
#pragma unroll
        for (int ee = 0; ee < 8; ++ee)
          if (cc == c && ee == e) v[cc][ee] = -INFINITY;
    }
  }
}

// y = softmax(x * scale + mask) row-wise, bf16 in/out; mask (fp32, additive) is indexed
// [row / rows_per_mask][N] (e.g. one padding mask per sequence shared by all heads/queries).
__global__ __launch_bounds__(256) void softmax_rows_kernel(const bf16* __restrict__ x, bf16* __restrict__ y,
                                                           const float* __restrict__ mask, int N, int rows_per_mask,
                                                           float scale) {
  extern __shared__ __attribute__((aligned(16))) float row[];
  __shared__ float red[16];
  const long r = blockIdx.x;
  const bf16* src = x + r * (long)N;
  const float* mk = mask ? mask + (r / rows_per_mask) * (long)N : nullptr;
  float mx = -INFINITY;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    float v = (float)src[i] * scale;
    if (mk) v += mk[i];
    row[i] = v;
    mx = fmaxf(mx, v);
  }
  mx = block_max(mx, red);
  float s = 0.f;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    const float e = (mx == -INFINITY) ? 0.f : __expf(row[i] - mx);
    row[i] = e;
    s += e;
  }
  s = block_sum(s, red);
  const float inv = s > 0.f ? 1.f / s : 0.f;
  for (int i = threadIdx.x; i < N; i += blockDim.x) y[r * (long)N + i] = f2bf(row[i] * inv);
}

// Second stage of the large-vocabulary top-k (LM heads): row r holds C chunks' k candidates each
// (value, chunk-local index); the winners get their shard-global index chunk * L + local + lo, and
// candidates at or past `valid` (the zero-padded vocabulary tail of a TP shard) are dropped BEFORE
// the selection.  One block per row, candidates staged once in LDS, k block-argmax rounds.
__global__ __launch_bounds__(256) void topk_merge_kernel(const float* __restrict__ cv, const int* __restrict__ ci,
                                                         float* __restrict__ vals, int* __restrict__ idx, int C, int k,
                                                         int L, int lo, int valid) {
  extern __shared__ __attribute__((aligned(16))) float cand[];  // [n] values, then [n] global indices
  __shared__ float rv[16];
  __shared__ int ri[16];
  const long r = blockIdx.x;
  const int n = C * k;
  int* gidx = reinterpret_cast<int*>(cand + n);
  for (int j = threadIdx.x; j < n; j += blockDim.x) {
    const int local = ci[r * n + j];
    const int g = (j / k) * L + local;
    const bool ok = local >= 0 && g < valid;
    cand[j] = ok ? cv[r * n + j] : -INFINITY;
    gidx[j] = ok ? g : -1;
  }
  __syncthreads();
  for (int j = 0; j < k; ++j) {
    KV best{-INFINITY, -1};
    for (int i = threadIdx.x; i < n; i += blockDim.x)
      if (gidx[i] >= 0) best = better(best, KV{cand[i], i});
    best = block_argmax(best, rv, ri);
    if (threadIdx.x == 0) {
      vals[r * k + j] = best.i >= 0 ? best.v : -INFINITY;
      idx[r * k + j] = best.i >= 0 ? gidx[best.i] + lo : lo;
      if (best.i >= 0) gidx[best.i] = -1;
    }
    __syncthreads();
  }
}

}  // namespace

extern "C" {

// x: [rows][N] (dtype 0 = bf16, 1 = fp32); vals fp32 [rows][k]; idx int32 [rows][k]
int mls_softmax_topk(const void* x, int dtype, float* vals, int* idx, int rows, int N, int k, int apply_softmax,
                     float temperature, void* stream) {
  if (rows <= 0 || N <= 0 || k <= 0 || k > N || N > 32768 || temperature <= 0.f) return MLS_BAD_ARG;
  if (dtype == 0 && N % 8 == 0 && N <= 2048 && k <= 64) {
    dim3 g((rows + 3) / 4);
    if (N <= 512)
      hipLaunchKernelGGL(softmax_topk_reg_kernel<1>, g, dim3(256), 0, (hipStream_t)stream, (const bf16*)x, vals, idx,
                         rows, N, k, apply_softmax, temperature, 1, N);
    else if (N <= 1024)
      hipLaunchKernelGGL(softmax_topk_reg_kernel<2>, g, dim3(256), 0, (hipStream_t)stream, (const bf16*)x, vals, idx,
                         rows, N, k, apply_softmax, temperature, 1, N);
    else
      hipLaunchKernelGGL(softmax_topk_reg_kernel<4>, g, dim3(256), 0, (hipStream_t)stream, (const bf16*)x, vals, idx,
                         rows, N, k, apply_softmax, temperature, 1, N);
    return (int)hipGetLastError();
  }
  if (N <= 4096) {
    const size_t lds4 = (size_t)4 * N * sizeof(float);
    dim3 g((rows + 3) / 4);
    if (dtype == 0)
      hipLaunchKernelGGL(softmax_topk_wave_kernel<bf16>, g, dim3(256), lds4, (hipStream_t)stream, (const bf16*)x, vals,
                         idx, rows, N, k, apply_softmax, temperature);
    else
      hipLaunchKernelGGL(softmax_topk_wave_kernel<float>, g, dim3(256), lds4, (hipStream_t)stream, (const float*)x,
                         vals, idx, rows, N, k, apply_softmax, temperature);
    return (int)hipGetLastError();
  }
  const size_t lds = (size_t)N * sizeof(float);
  if (dtype == 0)
    hipLaunchKernelGGL(softmax_topk_kernel<bf16>, dim3(rows), dim3(256), lds, (hipStream_t)stream, (const bf16*)x,
                       vals, idx, N, k, apply_softmax, temperature);
  else
    hipLaunchKernelGGL(softmax_topk_kernel<float>, dim3(rows), dim3(256), lds, (hipStream_t)stream, (const float*)x,
                       vals, idx, N, k, apply_softmax, temperature);
  return (int)hipGetLastError();
}

int mls_softmax_rows(const void* x, void* y, const float* mask, int rows, int N, int rows_per_mask, float scale,
                     void* stream) {
  if (rows <= 0 || N <= 0 || N > 32768 || (mask && rows_per_mask <= 0)) return MLS_BAD_ARG;
  hipLaunchKernelGGL(softmax_rows_kernel, dim3(rows), dim3(256), (size_t)N * sizeof(float), (hipStream_t)stream,
                     (const bf16*)x, (bf16*)y, mask, N, rows_per_mask > 0 ? rows_per_mask : 1, scale);
  return (int)hipGetLastError();
}

// Large-vocabulary raw-logit top-k, stage 1: x [rows][C * L] bf16 viewed as rows * C chunks of L
// (L % 8 == 0, L <= 2048), columns >= valid excluded; cv / ci [rows][C * k] chunk-local winners.
int mls_topk_chunks(const void* x, float* cv, int* ci, int rows, int C, int L, int k, int valid, void* stream) {
  if (rows <= 0 || C <= 0 || L <= 0 || L % 8 || L > 2048 || k <= 0 || k > 64 || k > L) return MLS_BAD_ARG;
  const int R = rows * C;
  dim3 g((R + 3) / 4);
  if (L <= 512)
    hipLaunchKernelGGL(softmax_topk_reg_kernel<1>, g, dim3(256), 0, (hipStream_t)stream, (const bf16*)x, cv, ci, R, L,
                       k, 0, 1.f, C, valid);
  else if (L <= 1024)
    hipLaunchKernelGGL(softmax_topk_reg_kernel<2>, g, dim3(256), 0, (hipStream_t)stream, (const bf16*)x, cv, ci, R, L,
                       k, 0, 1.f, C, valid);
  else
    hipLaunchKernelGGL(softmax_topk_reg_kernel<4>, g, dim3(256), 0, (hipStream_t)stream, (const bf16*)x, cv, ci, R, L,
                       k, 0, 1.f, C, valid);
  return (int)hipGetLastError();
}

// cv / ci: [rows][C * k] per-chunk candidates (chunk-local indices) -> vals / idx [rows][k]
int mls_topk_merge(const float* cv, const int* ci, float* vals, int* idx, int rows, int C, int k, int L, int lo,
                   int valid, void* stream) {
  if (rows <= 0 || C <= 0 || k <= 0 || L <= 0 || (size_t)C * k * 8 > 65536) return MLS_BAD_ARG;
  hipLaunchKernelGGL(topk_merge_kernel, dim3(rows), dim3(256), (size_t)C * k * 8, (hipStream_t)stream, cv, ci, vals,
                     idx, C, k, L, lo, valid);
  return (int)hipGetLastError();
}

}  // extern "C"
