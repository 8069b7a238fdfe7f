// Fused classifier head of ResNet-50 (K2 + K6 + K7 of SURVEY.md §2.E.1 in ONE launch):
//   logits = pooled . W^T + b  ->  softmax  ->  top-k  (+ per-row decode-error flags)
// where `pooled` [B][K] fp32 is the global average pool, accumulated by the LAST convolution's
// epilogue (conv_gemm.hip, ConvArgs::pool: per-image column sums of the post-ReLU tile, one fp32
// atomic per (image segment, column) of a tile) -- the [B][7][7][2048] block output is never written
// to HBM nor read back, and avgpool / FC / softmax-top-k stop being three launches (~31 us serial,
// round 3's profiles/r3_resnet50_b32_serial_kernel_summary_final.txt).
//
// Grid (ceil(N / 16) class groups) x (ceil(B / 4) row groups), 8 waves.  A block computes the
// 16-class x 4-row logit tile of its classes x rows on MFMA (D = W_tile . pooled^T, K split over the waves,
// pooled converted to bf16 on load -- the precision of the unfused bf16 GEMM), reduces the waves
// through LDS, adds the bias and writes the tile through (sc1) to `logits`.  One ticket per row
// group: the block that completes a row group (the last of its class groups) runs softmax + top-k
// for those rows (one row per wave) from the written-through logits (sc1 loads, no acquire: guide §6 Guideline 16 R1)
// and zeroes the rows' pooled sums for the next launch (the convolution accumulates into them).
// Counters are this stream's self-resetting split-K counters (conv_gemm.hip).
#include "common.h"

#include <cstdlib>
#include <mutex>
#include <unordered_map>
#include <vector>
#include <utility>

int* mls_stream_splitk_counters(void* stream, long ntiles);  // conv_gemm.hip

namespace {

constexpr int HT = 16;     // classes x rows per block tile
constexpr int MAXV = 32;   // logits per lane in the finishing pass (N <= 2048)

struct HeadArgs {
  const float* pooled;  // [B][K] fp32 (zeroed again by this kernel)
  const bf16* w;        // [N][K]
  const float* bias;    // [N] or null
  float* logits;        // [B][N] fp32 scratch / output
  float* vals;          // [B][k] fp32 (k > 0)
  int* idx;             // [B][k] int32
  const int* err;       // [B] int32 or null: rows flagged nonzero get idx -1, vals NaN
  int* cnt;             // [ceil(B/16)] arrival counters, zero between launches
  int B, N, K, k, softmax;
  uint32_t pooled_bytes, w_bytes, logits_bytes;
};

typedef unsigned int head_u32x4 __attribute__((__vector_size__(16)));

constexpr int HW = 8;   // waves per block
constexpr int HR = 4;   // rows per row group: the finisher of a group runs one row per wave, so its
                        // latency is one write-through load round trip + one top-k, not 16 rows' worth

// softmax + top-k of one row (a whole wave): the row's logits are loaded in one round trip, each
// lane keeps its MAXV candidates, and k rounds of wave arg-max pick the winners
template <int MAXV>
MLS_DEV void head_finish_row(const HeadArgs& a, const rsrc_t& lr, int row, int lane) {
  float v[MAXV];
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {  // unconditional loads (OOB offset), masked after (see below)
    const int c = lane + 64 * j;
    const bool ok = c < a.N;
    const float x = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(lr, ok ? (row * a.N + c) * 4 : OOB, 0, 16));
    v[j] = ok ? x : -INFINITY;
  }
  float m = -INFINITY;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) m = fmaxf(m, v[j]);
  m = wave_max(m);
  float s = 0.f;
  if (a.softmax) {
#pragma unroll
    for (int j = 0; j < MAXV; ++j) s += v[j] == -INFINITY ? 0.f : __expf(v[j] - m);
    s = wave_sum(s);
  }
  const bool bad = a.err && a.err[row] != 0;
  float wv = 0.f;
  int wc = -1;
  for (int t = 0; t < a.k; ++t) {
    float bv = -INFINITY;
    int bj = 0;
#pragma unroll
    for (int j = 0; j < MAXV; ++j)
      if (v[j] > bv) {
        bv = v[j];
        bj = j;
      }
    int bc = bv == -INFINITY ? 0x7fffffff : lane + 64 * bj;
    // wave arg-max: larger value wins, ties to the smaller class id
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oc = __shfl_xor(bc, o, 64);
      if (ov > bv || (ov == bv && oc < bc)) {
        bv = ov;
        bc = oc;
      }
    }
    if (lane == (bc & 63)) {  // the owner removes the winner from its candidates
#pragma unroll
      for (int j = 0; j < MAXV; ++j)
        if (lane + 64 * j == bc) v[j] = -INFINITY;
    }
    if (lane == 0) {
      const float p = a.softmax ? __expf(bv - m) / s : bv;
      a.vals[row * a.k + t] = bad ? __builtin_nanf("") : p;
      a.idx[row * a.k + t] = bad ? -1 : (bc < a.N ? bc : -1);
    }
  }
}

__global__ __launch_bounds__(HW * 64) void fc_head_kernel(const HeadArgs a) {
  __shared__ float red[HW][HT][HT + 1];
  __shared__ int flag;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int c0 = blockIdx.x * HT, r0 = blockIdx.y * HR;
  const rsrc_t wr = make_rsrc(a.w, a.w_bytes);
  const rsrc_t pr = make_rsrc(a.pooled, a.pooled_bytes);
  const rsrc_t lr = make_rsrc(a.logits, a.logits_bytes);

  // ---- 16 classes x HR rows (a 16 x 16 MFMA tile, rows past HR read as zero): wave w sums k in
  //      [w * K/8, (w + 1) * K/8), every load of its range issued before the first MFMA ----
  const int kw = a.K / HW;  // host: K % 256 == 0, K <= 2048
  const int kb = wid * kw;
  const int cl = c0 + fr, rw = r0 + fr;
  const int woff = cl < a.N ? (cl * a.K + kb + fq * 8) * 2 : OOB;
  const int poff = fr < HR && rw < a.B ? (rw * a.K + kb + fq * 8) * 4 : OOB;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  uint4 wv[8];
  float4 pv[8][2];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const bool in = 32 * s < kw;
    wv[s] = bload16(wr, woff == OOB || !in ? OOB : woff + 32 * s * 2);
    pv[s][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(pr, poff == OOB || !in ? OOB : poff + 32 * s * 4, 0, 0));
    pv[s][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(pr, poff == OOB || !in ? OOB : poff + 32 * s * 4 + 16, 0, 0));
  }
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    bf16x8 b;
    b[0] = (bf16)pv[s][0].x; b[1] = (bf16)pv[s][0].y; b[2] = (bf16)pv[s][0].z; b[3] = (bf16)pv[s][0].w;
    b[4] = (bf16)pv[s][1].x; b[5] = (bf16)pv[s][1].y; b[6] = (bf16)pv[s][1].z; b[7] = (bf16)pv[s][1].w;
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wv[s]), b, acc, 0, 0, 0);
  }
  // D[class fq*4 + i][row fr]
#pragma unroll
  for (int i = 0; i < 4; ++i) red[wid][fq * 4 + i][fr] = acc[i];
  __syncthreads();
  if (tid < HT * HR) {
    const int c = tid / HR, r = tid % HR;
    const int cg = c0 + c, rg = r0 + r;
    float v = a.bias && cg < a.N ? a.bias[cg] : 0.f;
#pragma unroll
    for (int w = 0; w < HW; ++w) v += red[w][c][r];
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), lr, cg < a.N && rg < a.B ? (rg * a.N + cg) * 4 : OOB, 0, 16);
  }
  // publish: every wave's write-through stores drained, then one ticket for this row group
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    int* c = a.cnt + blockIdx.y;
    const int prev = __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == (int)gridDim.x - 1;
    if (last) __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for the next launch
    flag = last;
  }
  __syncthreads();
  if (!flag) return;

  // ---- the row group's finisher: wave w < HR takes row r0 + w.  Every logit load is issued
  //      unconditionally (out-of-range columns read the OOB offset and are masked to -inf after
  //      the load): a load behind a per-element condition makes hipcc branch around it and wait
  //      vmcnt(0) per element -- dependent write-through round trips, ~30 us per group measured ----
  const int row = r0 + wid;
  if (a.k > 0 && wid < HR && row < a.B) {
    if (a.N <= 1024) head_finish_row<16>(a, lr, row, lane);
    else head_finish_row<MAXV>(a, lr, row, lane);
  }
  // zero the row group's pooled sums for the next launch (every class group has read them: they
  // arrived before this ticket)
  const int nrows = min(HR, a.B - r0);
  const int n4 = nrows * (a.K / 4);
  float4* pz = reinterpret_cast<float4*>(const_cast<float*>(a.pooled) + (long)r0 * a.K);
  for (int i = tid; i < n4; i += HW * 64) pz[i] = float4{0.f, 0.f, 0.f, 0.f};
}


// ---------------------------------------------------------------------------------------------
// v2 (default; MLS_HEAD_V2=0 runs the one-launch kernel above).  That kernel took 20.7 us at B = 32
// (profiles/r5_head_probe.jsonl): 14.7 us of it the FC alone, because 504 blocks re-read the 4 MB
// weight 8 times (once per 4-row group) and the fp32 pooled rows 63 times -- ~49 MB for a 0.13
// GFLOP product -- and then the last block of each row group ran its rows' softmax / top-k.
// v2 is two launches with no inter-block hand-off inside either:
//  * head_fc_kernel: grid (class groups of 32) x (K slices of 256) x (row groups of 32); 4 waves,
//    wave = 16 rows x 16 classes x K 256 = 8 MFMAs with every operand load issued up front; each
//    weight byte is read by one block per row group; the fp32 partial tile goes to slab
//    [slice][row][class] (16-B stores: the swapped product gives a lane 4 consecutive classes);
//  * head_finish_kernel: one block per row sums the slabs in slice order (deterministic), adds the
//    bias, writes the logits, runs softmax + top-k as block arg-max rounds, and zeroes the row's
//    pooled sums for the next forward.
constexpr int HV2_CG = 32, HV2_KS = 256, HV2_RG = 32;

struct HeadV2Args {
  const float* pooled;
  const bf16* w;
  const float* bias;
  float* slabs;  // [K / HV2_KS][B][N]
  float* logits;
  float* vals;
  int* idx;
  const int* err;
  int B, N, K, k, softmax;
  uint32_t pooled_bytes, w_bytes;
};

__global__ __launch_bounds__(256) void head_fc_kernel(const HeadV2Args a) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int c0 = blockIdx.x * HV2_CG + (wid & 1) * 16, k0 = blockIdx.y * HV2_KS;
  const int r0 = blockIdx.z * HV2_RG + (wid >> 1) * 16;
  const rsrc_t wr = make_rsrc(a.w, a.w_bytes), pr = make_rsrc(a.pooled, a.pooled_bytes);
  const int cl = c0 + fr, rw = r0 + fr;
  const int woff = cl < a.N ? (cl * a.K + k0 + fq * 8) * 2 : OOB;
  const int poff = rw < a.B ? (rw * a.K + k0 + fq * 8) * 4 : OOB;
  uint4 wv[HV2_KS / 32];
  float4 pv[HV2_KS / 32][2];
#pragma unroll
  for (int s = 0; s < HV2_KS / 32; ++s) {
    wv[s] = bload16(wr, woff == OOB ? OOB : woff + 64 * s);
    pv[s][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(pr, poff == OOB ? OOB : poff + 128 * s, 0, 0));
    pv[s][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(pr, poff == OOB ? OOB : poff + 128 * s + 16, 0, 0));
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < HV2_KS / 32; ++s) {
    bf16x8 b;
    b[0] = (bf16)pv[s][0].x; b[1] = (bf16)pv[s][0].y; b[2] = (bf16)pv[s][0].z; b[3] = (bf16)pv[s][0].w;
    b[4] = (bf16)pv[s][1].x; b[5] = (bf16)pv[s][1].y; b[6] = (bf16)pv[s][1].z; b[7] = (bf16)pv[s][1].w;
    // D[class fq*4 + i][row fr]: lane (fr, fq) holds classes c0 + fq*4 .. +3 of row r0 + fr
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wv[s]), b, acc, 0, 0, 0);
  }
  const int row = r0 + fr, col = c0 + fq * 4;
  if (row < a.B && col < a.N) {
    float* dst = a.slabs + ((long)blockIdx.y * a.B + row) * a.N + col;
    if (col + 4 <= a.N && (a.N & 3) == 0) {
      *reinterpret_cast<float4*>(dst) = float4{acc[0], acc[1], acc[2], acc[3]};
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float e = acc[i];  // through a named float (ext-vector element bit-cast hazard)
        if (col + i < a.N) dst[i] = e;
      }
    }
  }
}

// block-wide arg-max over (value, class): larger value wins, ties to the smaller class
MLS_DEV void block_argmax(float& bv, int& bc, float* sv, int* sc) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oc = __shfl_xor(bc, o, 64);
    if (ov > bv || (ov == bv && oc < bc)) {
      bv = ov;
      bc = oc;
    }
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    sv[wid] = bv;
    sc[wid] = bc;
  }
  __syncthreads();
  bv = sv[0];
  bc = sc[0];
#pragma unroll
  for (int w = 1; w < 4; ++w)
    if (sv[w] > bv || (sv[w] == bv && sc[w] < bc)) {
      bv = sv[w];
      bc = sc[w];
    }
  __syncthreads();  // sv / sc are reused by the next round
}

// DPP / lane-swap wave reductions (no LDS traffic: the ds_bpermute form costs ~12 dependent LDS
// round trips per arg-max)
MLS_DEV float hv2_wave_max(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));   // lane ^ 1
  v = fmaxf(v, dpp_f<0x4E>(v));   // lane ^ 2
  v = fmaxf(v, dpp_f<0x141>(v));  // row_half_mirror: the other quad of the 8
  v = fmaxf(v, dpp_f<0x140>(v));  // row_mirror: the other half of the 16
  v = fmaxf(v, xor16_f(v));
  return fmaxf(v, xor32_f(v));
}
MLS_DEV float hv2_wave_sum(float v) {
  v = group_sum<16>(v);
  v += xor16_f(v);
  return v + xor32_f(v);
}
MLS_DEV int hv2_wave_min(int c) {
  float v = __int_as_float(c);  // moved as bits; compared as ints
  auto mn = [](float a, float b) { return __int_as_float(min(__float_as_int(a), __float_as_int(b))); };
  v = mn(v, dpp_f<0xB1>(v));
  v = mn(v, dpp_f<0x4E>(v));
  v = mn(v, dpp_f<0x141>(v));
  v = mn(v, dpp_f<0x140>(v));
  v = mn(v, xor16_f(v));
  return __float_as_int(mn(v, xor32_f(v)));
}
// wave arg-max of (v, c): larger v wins, ties to the smaller class; every lane gets the winner
MLS_DEV void hv2_wave_argmax(float& v, int& c) {
  const float m = hv2_wave_max(v);
  c = hv2_wave_min(v == m ? c : 0x7fffffff);
  v = m;
}

constexpr int HV2_PER_T = 4;  // classes per thread in the finisher (N <= 1024)
constexpr int HV2_FAST_K = 16;  // top-k up to this: wave-local top-k + one barrier + a one-wave merge
constexpr int HV2_MAXS = 8;   // K slices summed with all loads in flight (K <= 2048)

__global__ __launch_bounds__(256) void head_finish_kernel(const HeadV2Args a) {
  __shared__ float sv[4];
  __shared__ int sc[4];
  __shared__ float sred[4];
  const int row = blockIdx.x, tid = threadIdx.x;
  const int nks = a.K / HV2_KS;
  const int c = tid * HV2_PER_T;
  float v[HV2_PER_T];
  const bool full = c + HV2_PER_T <= a.N && (a.N & 3) == 0;
#pragma unroll
  for (int i = 0; i < HV2_PER_T; ++i) v[i] = 0.f;
  if (full && nks <= HV2_MAXS) {
    // every slice's 16 B issued before the first is summed (a runtime-count loop waited for each
    // load in turn: 8 dependent L2 round trips, ~8 of the finisher's 11 us); slices past nks read
    // zero through the range check; summed in slice order -> the same bits on every launch
    const rsrc_t sr = make_rsrc(a.slabs, (uint32_t)((size_t)nks * a.B * a.N * 4));
    float4 x[HV2_MAXS];
#pragma unroll
    for (int s = 0; s < HV2_MAXS; ++s)
      x[s] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                            sr, s < nks ? (int)((((size_t)s * a.B + row) * a.N + c) * 4) : OOB, 0, 0));
#pragma unroll
    for (int s = 0; s < HV2_MAXS; ++s) {
      v[0] += x[s].x; v[1] += x[s].y; v[2] += x[s].z; v[3] += x[s].w;
    }
  } else {
    for (int s = 0; s < nks; ++s) {  // slice order: the same sum on every launch
      const float* src = a.slabs + ((long)s * a.B + row) * a.N + c;
      for (int i = 0; i < HV2_PER_T; ++i)
        if (c + i < a.N) v[i] += src[i];
    }
  }
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < HV2_PER_T; ++i) {
    if (c + i < a.N) {
      v[i] += a.bias ? a.bias[c + i] : 0.f;
      m = fmaxf(m, v[i]);
    } else {
      v[i] = -INFINITY;
    }
  }
  float lg[HV2_PER_T];  // the logits, stored at the end: a store pending at the reductions'
#pragma unroll          // barriers would make each of them wait for it (vmcnt(0))
  for (int i = 0; i < HV2_PER_T; ++i) lg[i] = v[i];
  auto epilogue = [&]() {
#pragma unroll
    for (int i = 0; i < HV2_PER_T; ++i)
      if (c + i < a.N) a.logits[(long)row * a.N + c + i] = lg[i];
    // zero this row's pooled sums for the next forward (the FC kernel, an earlier launch, read them)
    float4* pz = reinterpret_cast<float4*>(const_cast<float*>(a.pooled) + (long)row * a.K);
    for (int i = tid; i < a.K / 4; i += 256) pz[i] = float4{0.f, 0.f, 0.f, 0.f};
  };
  if (a.k <= 0) {
    epilogue();
    return;
  }
  const bool bad = a.err && a.err[row] != 0;
  if (a.k <= HV2_FAST_K) {
    // each wave: its max / exp-sum and its own top-k (k rounds of DPP arg-max, no barrier); one
    // barrier hands the 4 waves' candidates to wave 0, which merges them with k more rounds.  The
    // softmax sum combines the waves' sums rescaled to the global max.
    __shared__ float cv[4 * HV2_FAST_K], wm[4], ws[4];
    __shared__ int cc[4 * HV2_FAST_K];
    const int lane = tid & 63, wid = tid >> 6;
    const float mw = hv2_wave_max(m);
    float sw = 0.f;
    if (a.softmax) {
#pragma unroll
      for (int i = 0; i < HV2_PER_T; ++i) sw += v[i] == -INFINITY ? 0.f : __expf(v[i] - mw);
      sw = hv2_wave_sum(sw);
    }
    for (int t = 0; t < a.k; ++t) {
      float bv = -INFINITY;
      int bj = 0;
#pragma unroll
      for (int i = 0; i < HV2_PER_T; ++i)
        if (v[i] > bv) {
          bv = v[i];
          bj = i;
        }
      int bc = bv == -INFINITY ? 0x7fffffff : c + bj;
      hv2_wave_argmax(bv, bc);
      if (bc >= c && bc < c + HV2_PER_T) v[bc - c] = -INFINITY;  // the owner drops the winner
      if (lane == t) {
        cv[wid * a.k + t] = bv;
        cc[wid * a.k + t] = bc;
      }
    }
    if (lane == 0) {
      wm[wid] = mw;
      ws[wid] = sw;
    }
    __syncthreads();
    if (wid == 0) {
      const int nc = 4 * a.k;
      float bv0 = lane < nc ? cv[lane] : -INFINITY;
      int bc0 = lane < nc ? cc[lane] : 0x7fffffff;
      const float gm = fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]));
      float gs = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) gs += ws[w] * __expf(wm[w] - gm);
      float ov = 0.f;
      int oc = -1;
      for (int t = 0; t < a.k; ++t) {
        float bv = bv0;
        int bc = bc0;
        hv2_wave_argmax(bv, bc);
        if (bc0 == bc && bv0 == bv) bv0 = -INFINITY, bc0 = 0x7fffffff;  // the holder drops it
        if (lane == t) {
          ov = a.softmax ? __expf(bv - gm) / gs : bv;
          oc = bc;
        }
      }
      if (lane < a.k) {
        a.vals[row * a.k + lane] = bad ? __builtin_nanf("") : ov;
        a.idx[row * a.k + lane] = bad ? -1 : (oc < a.N ? oc : -1);
      }
    }
    epilogue();
    return;
  }
  m = block_max(m, sred);
  float ssum = 0.f;
  if (a.softmax) {
#pragma unroll
    for (int i = 0; i < HV2_PER_T; ++i) ssum += v[i] == -INFINITY ? 0.f : __expf(v[i] - m);
    ssum = block_sum(ssum, sred);
  }
  float wv = 0.f;
  int wc = -1;
  for (int t = 0; t < a.k; ++t) {
    float bv = -INFINITY;
    int bj = 0;
#pragma unroll
    for (int i = 0; i < HV2_PER_T; ++i)
      if (v[i] > bv) {
        bv = v[i];
        bj = i;
      }
    int bc = bv == -INFINITY ? 0x7fffffff : c + bj;
    block_argmax(bv, bc, sv, sc);
    if (bc >= c && bc < c + HV2_PER_T) v[bc - c] = -INFINITY;  // the owner drops the winner
    if (tid == t) {  // thread t keeps winner t; all k written after the last round
      wv = a.softmax ? __expf(bv - m) / ssum : bv;
      wc = bc;
    }
  }
  if (tid < a.k) {
    a.vals[row * a.k + tid] = bad ? __builtin_nanf("") : wv;
    a.idx[row * a.k + tid] = bad ? -1 : (wc < a.N ? wc : -1);
  }
  epilogue();
}

// Fallback slab store for callers that pass no workspace: one slab per stream, grown outside any
// capture.  A replaced slab is never freed -- a graph captured earlier on the stream (engines share
// the pooled CU-masked streams) keeps writing to it, and hipFree would synchronize the device while
// other slots run -- it is retired and stays allocated.  ops.fc_head passes a workspace from the
// torch allocator (in a capture: the graph's pool), so this store is only for raw-ABI callers.
float* head_slabs(hipStream_t st, size_t bytes) {
  static std::mutex mu;
  static std::unordered_map<hipStream_t, std::pair<float*, size_t>> bufs;
  static std::vector<float*> retired;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> g(mu);
  auto it = bufs.find(st);
  if (it != bufs.end() && it->second.second >= bytes) return it->second.first;
  if (cs != hipStreamCaptureStatusNone) return nullptr;  // no allocation inside a capture
  float* p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;  // the old slab (if any) stays valid
  if (it != bufs.end()) retired.push_back(it->second.first);
  bufs[st] = {p, bytes};
  return p;
}
}  // namespace

extern "C" {

// pooled [B][K] fp32 (averages, zeroed on return), w [N][K] bf16, bias [N] fp32 or null ->
// logits [B][N] fp32 (caller's scratch or output) and, for k > 0, vals / idx [B][k] of the
// (softmax of the) logits' top-k.  err [B] int32 or null.  K % 256 == 0, K <= 2048, N <= 2048, k <= 64.
// ws: fp32 workspace of ws_bytes >= (K / 256) * B * N * 4 for the v2 kernels' partial slabs (the
// caller's allocator: in a capture, the graph's pool), or null for the per-stream fallback store.
int mls_fc_head(const float* pooled, const void* w, const float* bias, float* logits, float* vals, int* idx,
                const int* err, int B, int N, int K, int k, int softmax, float* ws, long long ws_bytes,
                void* stream) {
  if (B <= 0 || N <= 0 || N > 64 * MAXV || K <= 0 || K % 256 || K > 2048 || k < 0 || k > 64 || k > N) return MLS_BAD_ARG;
  if (k > 0 && (!vals || !idx)) return MLS_BAD_ARG;
  const long pb = (long)B * K * 4, wb = (long)N * K * 2, lb = (long)B * N * 4;
  if (pb >= 0x7fffffffL || wb >= 0x7fffffffL || lb >= 0x7fffffffL) return MLS_UNSUPPORTED;
  static const bool v2 = [] {  // MLS_HEAD_V2=0: the one-launch kernel (A/B)
    const char* e = getenv("MLS_HEAD_V2");
    return !(e && e[0] == '0');
  }();
  if (v2 && N <= 256 * HV2_PER_T && K % HV2_KS == 0) {
    const size_t sb = (size_t)(K / HV2_KS) * B * N * sizeof(float);
    if (ws && ws_bytes < (long long)sb) return MLS_BAD_ARG;
    float* slabs = ws ? ws : head_slabs((hipStream_t)stream, sb);
    if (slabs) {
      HeadV2Args a2;
      a2.pooled = pooled;
      a2.w = (const bf16*)w;
      a2.bias = bias;
      a2.slabs = slabs;
      a2.logits = logits;
      a2.vals = vals;
      a2.idx = idx;
      a2.err = err;
      a2.B = B, a2.N = N, a2.K = K, a2.k = k, a2.softmax = softmax;
      a2.pooled_bytes = (uint32_t)pb;
      a2.w_bytes = (uint32_t)wb;
      hipLaunchKernelGGL(head_fc_kernel, dim3((N + HV2_CG - 1) / HV2_CG, K / HV2_KS, (B + HV2_RG - 1) / HV2_RG),
                         dim3(256), 0, (hipStream_t)stream, a2);
      hipLaunchKernelGGL(head_finish_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, a2);
      return (int)hipGetLastError();
    }
  }
  const int nrg = (B + HR - 1) / HR;
  int* cnt = mls_stream_splitk_counters(stream, nrg);
  if (!cnt) return MLS_UNSUPPORTED;  // counters must exist before graph capture (eager warm-up)
  HeadArgs a;
  a.pooled = pooled;
  a.w = (const bf16*)w;
  a.bias = bias;
  a.logits = logits;
  a.vals = vals;
  a.idx = idx;
  a.err = err;
  a.cnt = cnt;
  a.B = B, a.N = N, a.K = K, a.k = k, a.softmax = softmax;
  a.pooled_bytes = (uint32_t)pb;
  a.w_bytes = (uint32_t)wb;
  a.logits_bytes = (uint32_t)lb;
  hipLaunchKernelGGL(fc_head_kernel, dim3((N + HT - 1) / HT, nrg), dim3(HW * 64), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

}  // extern "C"
