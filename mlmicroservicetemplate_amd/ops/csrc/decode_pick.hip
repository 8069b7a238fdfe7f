// X4 tail on device: merge the tensor-parallel ranks' top-k candidates and pick each sequence's
// next token inside the captured decode step, so a TP decode loop never waits on the host.
//
// cand_v / cand_i: [tp][B][k] (the one-shot all-gather of every rank's local top-k; rank-major, so
// candidate j = r * k + c of row b is the host's `permute(1, 0, 2).reshape(B, -1)` order).
// Per row (params per row: top_k, temperature, seed):
//   greedy (top_k <= 1): the candidate at the FIRST maximum (torch.argmax order);
//   sampled: the top_k largest (ties -> lower j first, = a stable descending sort), p =
//   softmax(v / temperature), u = uniform(seed, step), the first i with cdf_i > u * cdf_last.
// uniform(seed, step) = (splitmix64(seed * 0x9E3779B97F4A7C15 + step) >> 40) * 2^-24: a counter-
// based draw the host reproduces bit-exactly (models/llama.py sample_uniform), independent of the
// row's position in the batch -- so a sequence's tokens do not depend on what else is in flight.
// Then the step's static inputs advance in place: tok[b] = token, pos[b] += 1, lens[b] += 1,
// hist[b][step[b]] = token, step[b] += 1 -- the next graph replay decodes the next position.
#include "common.h"

namespace {

constexpr int PICK_MAX_CAND = 512;  // tp * k
constexpr int PICK_MAX_TOPK = 64;

MLS_DEV unsigned long long splitmix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

struct VI {
  float v;
  int j;
};
// larger value first; ties: lower candidate index first
MLS_DEV bool vi_better(VI a, VI b) { return a.v > b.v || (a.v == b.v && a.j < b.j); }

MLS_DEV VI wave_best(VI x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    VI y{__shfl_xor(x.v, o, 64), __shfl_xor(x.j, o, 64)};
    if (vi_better(y, x)) x = y;
  }
  return x;
}

__global__ __launch_bounds__(64) void decode_pick_kernel(const float* __restrict__ cv, const int* __restrict__ ci,
                                                         int tp, int B, int k, const int* __restrict__ topk,
                                                         const float* __restrict__ temp,
                                                         const long long* __restrict__ seed, int* tok, int* pos,
                                                         int* lens, int* hist, int hist_cols, int* step,
                                                         const int* __restrict__ rows,
                                                         const int* __restrict__ active, int* emit) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const int n = tp * k;
  // per-sequence state row of candidate row b: rows[b] (a prefill of new sequences into their
  // serving slots) or b; inactive state rows (an idle serving slot) are left untouched
  const int sr = rows ? rows[b] : b;
  if (active && !active[sr]) return;
  __shared__ float sv[PICK_MAX_CAND];
  __shared__ int sj[PICK_MAX_CAND];
  for (int j = lane; j < n; j += 64) {
    const int r = j / k, c = j - r * k;
    sv[j] = cv[((long)r * B + b) * k + c];
    sj[j] = ci[((long)r * B + b) * k + c];
  }
  __syncthreads();
  const int want = topk ? topk[sr] : 1;
  int token;
  if (want <= 1) {
    VI best{-INFINITY, 0x7fffffff};
    for (int j = lane; j < n; j += 64) best = vi_better(VI{sv[j], j}, best) ? VI{sv[j], j} : best;
    best = wave_best(best);
    token = sj[best.j < n ? best.j : 0];
  } else {
    const int kk = want < n ? (want < PICK_MAX_TOPK ? want : PICK_MAX_TOPK) : n;
    __shared__ float tv[PICK_MAX_TOPK];
    __shared__ int tj[PICK_MAX_TOPK];
    for (int s = 0; s < kk; ++s) {  // kk rounds of wave argmax, each removes its winner
      VI best{-INFINITY, 0x7fffffff};
      for (int j = lane; j < n; j += 64)
        if (sj[j] >= 0 || sv[j] > -INFINITY) best = vi_better(VI{sv[j], j}, best) ? VI{sv[j], j} : best;
      best = wave_best(best);
      if (lane == 0) {
        tv[s] = best.v;
        tj[s] = best.j;
        if (best.j < n) sv[best.j] = -INFINITY, sj[best.j] = -1;
      }
      __syncthreads();
    }
    if (lane == 0) {
      const float t = fmaxf(temp ? temp[sr] : 1.f, 1e-5f);
      const float mx = tv[0];
      float p[PICK_MAX_TOPK];
      float cdf = 0.f;
      for (int s = 0; s < kk; ++s) {
        p[s] = expf((tv[s] - mx) / t);
        cdf += p[s];
        p[s] = cdf;  // running sum (same order as the host's cumsum)
      }
      const unsigned long long h =
          splitmix64((unsigned long long)(seed ? seed[sr] : 0) * 0x9E3779B97F4A7C15ull + (unsigned long long)step[sr]);
      const float u = (float)(h >> 40) * (1.f / 16777216.f);
      int pick = kk - 1;
      for (int s = 0; s < kk; ++s)
        if (p[s] > u * cdf) {
          pick = s;
          break;
        }
      const int jj = tj[pick];
      // the winners' ids were cleared in sj: re-read the candidate id from global memory
      const int r = jj / k, c = jj - r * k;
      sj[0] = ci[((long)r * B + b) * k + c];
    }
    __syncthreads();
    token = sj[0];
  }
  if (lane == 0) {
    const int s = step[sr];
    if (hist && s < hist_cols) hist[(long)sr * hist_cols + s] = token;
    step[sr] = s + 1;
    tok[sr] = token;
    pos[sr] += 1;
    lens[sr] += 1;
    if (emit) emit[sr] = token;
  }
}

}  // namespace

extern "C" {

// cv [tp][B][k] f32, ci [tp][B][k] i32; per-row params topk / temp / seed (nullptr: greedy, 1.0, 0);
// tok / pos / lens [B] i32 advanced in place; hist [B][hist_cols] (nullable); step [B] i32.
// Serving extensions (all nullable): rows [B] i32 maps candidate row b to state row rows[b] (the
// state arrays then have the serving batch's size, indices < state_rows); active [state rows] i32
// skips idle state rows; emit [state rows] i32 receives each picked token (a per-iteration
// read-back buffer next to the decode graph's own tok).
int mls_decode_pick(const float* cv, const int* ci, int tp, int B, int k, const int* topk, const float* temp,
                    const long long* seed, int* tok, int* pos, int* lens, int* hist, int hist_cols, int* step,
                    const int* rows, const int* active, int* emit, void* stream) {
  if (tp <= 0 || B <= 0 || k <= 0 || tp * k > PICK_MAX_CAND || !tok || !pos || !lens || !step) return MLS_BAD_ARG;
  hipLaunchKernelGGL(decode_pick_kernel, dim3(B), dim3(64), 0, (hipStream_t)stream, cv, ci, tp, B, k, topk, temp, seed,
                     tok, pos, lens, hist, hist_cols, step, rows, active, emit);
  return (int)hipGetLastError();
}

}  // extern "C"
