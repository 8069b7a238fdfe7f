// K8: fused attention on gfx950.
//
// (1) flash_fwd_kernel<D>: prefill / encoder attention, O = softmax(Q K^T * scale + mask) V,
//     never materialising the S x S scores.  BERT: bidirectional + key-padding mask (per-batch
//     valid length), Hq == Hkv, D = 64.  Llama: causal, GQA (Hq / Hkv query heads share a KV
//     head), D = 128.  Q/K/V are read in place from the fused QKV projection output (strided).
//
//     Block = NW waves = 16 NW query rows (16 per wave), K/V tiles of 64 keys staged in LDS.  NW = 4
//     in general; BERT (D = 64, 64 < S <= 128) uses NW = 8 so one block holds a whole
//     (sequence, head) and its K/V rows are fetched once (-8 % kernel time at B=128).
//     Per wave and tile, with v_mfma_f32_16x16x32_bf16:
//       S^T = K . Q^T   (A = K rows from LDS, B = Q^T fragments kept in registers): the key is
//                       on the accumulator row, the query on the lane -> softmax statistics of
//                       one query live in one lane column (4 register values x 4 lane groups);
//       O  += P . V     (A = P straight from the S^T accumulators, packed to bf16 -- the key
//                       order inside each 32-key k-step is permuted, so the V fragment is read in
//                       the SAME permuted order with ds_read_b64_tr_b16 from a row-major V tile).
//     K tile: 16-B chunk XOR-swizzle (chunk ^ row & (CPR-1)) -> conflict-free ds_read_b128;
//     V tile: rows padded by 32 B -> conflict-free transposed reads (checked against the gfx950
//     LDS lane groups).  Online softmax in exp2 with the scale folded in.
//
// (2) decode: q_len = 1 per sequence against the KV cache (memory-bound).  Split-KV
//     ("flash-decoding"): grid (splits, Hkv, B); each wave walks keys with 16-B loads, one key
//     row per D/8 lanes, all G = Hq/Hkv query heads of the KV head at once (GQA: every K/V byte
//     is read once for the G heads); partial (m, l, O) per split, then a combine kernel.
#include <cstdlib>

#include "common.h"

typedef short short4v __attribute__((ext_vector_type(4)));
#define LDS_AS __attribute__((address_space(3)))

namespace {

struct AttnArgs {
  const bf16* q;
  const bf16* k;
  const bf16* v;
  bf16* o;
  int q_stride, k_stride, v_stride, o_stride;  // token-row strides (elements)
  int B, S, Hq, Hkv;
  int q_rows;          // query rows per sequence (positions 0 .. q_rows - 1; == S for full attention)
  int pre;             // 8- / 1-wave blocks: tile 1's K/V loads issued with tile 0's (MLS_FLASH_PRE=0: off)
  const int* kv_lens;  // [B] valid keys per sequence (nullptr -> S)
  int causal;
  float scale_log2;  // softmax scale * log2(e)
  uint32_t q_bytes, k_bytes, v_bytes;
};

MLS_DEV float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

template <int D, int NW = 4>
__global__ __launch_bounds__(64 * NW) void flash_fwd_kernel(const AttnArgs a) {
  constexpr int NT = 64 * NW;            // threads; NW waves x 16 query rows
  constexpr int BQ = 16 * NW, BKV = 64;
  constexpr int CPR = D / 8;             // 16-B chunks per row
  constexpr int KK = D / 32;             // k-steps of the S^T MFMA
  constexpr int DT = D / 16;             // 16-wide d tiles of O
  constexpr int VST = D * 2 + 32;        // padded V row stride (bytes)
  constexpr int K_BYTES = BKV * D * 2;
  constexpr int V_BYTES = BKV * VST;
  __shared__ __attribute__((aligned(16))) char smem[K_BYTES + V_BYTES];
  char* Ks = smem;
  char* Vs = smem + K_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, fr = lane & 15;
  const int b = blockIdx.z, h = blockIdx.y;
  const int hk = h / (a.Hq / a.Hkv);
  const int q0 = blockIdx.x * BQ;
  const int qw = q0 + wid * 16;
  MLS_CHECK(!a.kv_lens || a.kv_lens[b] <= a.S, 301);
  const int L = a.kv_lens ? min(a.kv_lens[b], a.S) : a.S;
  const long tok0 = (long)b * a.S, tokq = (long)b * a.q_rows;  // first K/V row, first Q / O row

  const rsrc_t qr = make_rsrc(a.q, a.q_bytes);
  const rsrc_t kr = make_rsrc(a.k, a.k_bytes);
  const rsrc_t vr = make_rsrc(a.v, a.v_bytes);

  // Q^T fragments (B operand): lane holds Q[q = qw + fr][d = 32kk + 8g .. +7]
  bf16x8 qf[KK];
  {
    const int q = qw + fr;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const int off = q < a.q_rows ? (int)(((tokq + q) * a.q_stride + (long)h * D + 32 * kk + 8 * g) * 2) : OOB;
      qf[kk] = __builtin_bit_cast(bf16x8, bload16(qr, off));
    }
  }

  f32x4 acc_o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) acc_o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;

  int kv_end = L;
  if (a.causal) kv_end = min(kv_end, q0 + BQ);
  const int ntiles = (kv_end + BKV - 1) / BKV;

  // K / V tiles (zero rows past L via OOB loads) are register double-buffered: tile kt + 1's loads
  // are issued right after tile kt is in LDS and land while tile kt's MFMAs run (one global
  // round trip per kernel instead of one per tile: BERT S=128 has 2 tiles, Llama S=512 has 8)
  constexpr int NI = (BKV * CPR) / NT;
  static_assert(NI * NT == BKV * CPR, "tile chunks split evenly over the block");
  uint4 kreg[NI], vreg[NI];
  auto load_into = [&](int kt, uint4 (&kd)[NI], uint4 (&vd)[NI]) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int idx = tid + NT * i;
      const int row = idx / CPR, ch = idx % CPR;
      const int kv = kt * BKV + row;
      const bool ok = kv < L;
      kd[i] = bload16(kr, ok ? (int)(((tok0 + kv) * a.k_stride + (long)hk * D + ch * 8) * 2) : OOB);
      vd[i] = bload16(vr, ok ? (int)(((tok0 + kv) * a.v_stride + (long)hk * D + ch * 8) * 2) : OOB);
    }
  };
  auto load_tile = [&](int kt) { load_into(kt, kreg, vreg); };
  // NW = 8 (BERT, S <= 128: two tiles) and NW = 1 (the [CLS] rows): tile 1's loads go out right
  // behind tile 0's instead of one round trip later (co-running at B=128: 8-wave kernel 28.1 -> 26.3
  // and 25.4 -> 26.4 us on two boxes, 1-wave 23.7 -> 19.8 us; engine level: r5_bert_flash_prefetch_ab.txt)
  const bool pre = (NW == 8 || NW == 1) && a.pre;
  uint4 kpre[NI], vpre[NI];
  if (ntiles > 0) load_tile(0);
  if (pre && ntiles > 1) load_into(1, kpre, vpre);

  for (int kt = 0; kt < ntiles; ++kt) {
    const int kv0 = kt * BKV;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int idx = tid + NT * i;
      const int row = idx / CPR, ch = idx % CPR;
      *reinterpret_cast<uint4*>(Ks + row * (D * 2) + ((ch ^ (row & (CPR - 1))) * 16)) = kreg[i];
      *reinterpret_cast<uint4*>(Vs + row * VST + ch * 16) = vreg[i];
    }
    __syncthreads();
    if (kt + 1 < ntiles) {
      if (pre && kt == 0) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          kreg[i] = kpre[i];
          vreg[i] = vpre[i];
        }
      } else {
        load_tile(kt + 1);
      }
    }

    // ---- S^T = K Q^T : 4 sub-tiles of 16 keys ----
    f32x4 s[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int row = 16 * t + fr;
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const int ch = 4 * kk + g;
        const bf16x8 kf = __builtin_bit_cast(
            bf16x8, *reinterpret_cast<const uint4*>(Ks + row * (D * 2) + ((ch ^ (row & (CPR - 1))) * 16)));
        s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[kk], s[t], 0, 0, 0);
      }
    }
    // ---- mask + scale + online softmax (query = qw + fr, key = kv0 + 16t + 4g + j) ----
    const int qabs = qw + fr;
    float mt = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kv = kv0 + 16 * t + 4 * g + j;
        float x = s[t][j] * a.scale_log2;
        if (kv >= L || (a.causal && kv > qabs)) x = -INFINITY;
        s[t][j] = x;
        mt = fmaxf(mt, x);
      }
    mt = fmaxf(mt, xor16_f(mt));  // v_permlane swaps, not LDS round trips
    mt = fmaxf(mt, xor32_f(mt));
    const float m_new = fmaxf(m_run, mt);
    const float alpha = (m_new == -INFINITY) ? 1.f : fast_exp2(m_run - m_new);
    float ls = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float p = (m_new == -INFINITY) ? 0.f : fast_exp2(s[t][j] - m_new);
        s[t][j] = p;
        ls += p;
      }
    ls += xor16_f(ls);
    ls += xor32_f(ls);
    l_run = l_run * alpha + ls;
    m_run = m_new;
    // rescale O rows q = 4g + j by alpha of query lane (4g + j)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float aj = __shfl(alpha, 4 * g + j, 64);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) acc_o[dt][j] *= aj;
    }
    // ---- O += P V : two 32-key k-steps, key order permuted identically in A and B ----
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      bf16x8 pf;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pf[j] = (bf16)s[2 * st][j];
        pf[4 + j] = (bf16)s[2 * st + 1][j];
      }
      const int qq = fr >> 2, pp = fr & 3;
      const int row0 = 32 * st + 4 * g + qq;  // run 0 rows: keys 32st + 4g + (0..3)
      const int row1 = row0 + 16;             // run 1 rows: keys 32st + 16 + 4g + (0..3)
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int colb = (16 * dt + 4 * pp) * 2;
        const short4v r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS short4v*)(Vs + row0 * VST + colb));
        const short4v r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS short4v*)(Vs + row1 * VST + colb));
        typedef short short8v __attribute__((ext_vector_type(8)));
        const short8v vv = {r0[0], r0[1], r0[2], r0[3], r1[0], r1[1], r1[2], r1[3]};
        acc_o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf, __builtin_bit_cast(bf16x8, vv), acc_o[dt], 0, 0, 0);
      }
    }
    __syncthreads();
  }

  // ---- normalise and store: O rows q = qw + 4g + j, cols d = 16dt + fr
  const float inv_l = l_run > 0.f ? 1.f / l_run : 0.f;
  if constexpr (D == 64) {  // BERT: 2-B stores straight from the accumulators (the LDS-staged 16-B
                            // row stores below measured -0.8 % at B=32, level at B=128)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float il = __shfl(inv_l, 4 * g + j, 64);
      const int q = qw + 4 * g + j;
      if (q < a.q_rows) {
        bf16* dst = a.o + (tokq + q) * a.o_stride + (long)h * D + fr;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) dst[16 * dt] = (bf16)(acc_o[dt][j] * il);
      }
    }
  } else {
    // D = 128 (Llama prefill, +1-2 % at B=1x512): the wave's [16][D] tile through LDS (the K tile's
    // space: every wave is past the loop's last barrier), then 16-B row stores
    bf16* Os = reinterpret_cast<bf16*>(smem) + wid * 16 * D;
    static_assert(NW * 16 * D * 2 <= K_BYTES, "output tiles fit the K tile");
  #pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float il = __shfl(inv_l, 4 * g + j, 64);
  #pragma unroll
      for (int dt = 0; dt < DT; ++dt) Os[(4 * g + j) * D + 16 * dt + fr] = (bf16)(acc_o[dt][j] * il);
    }
    __syncthreads();
  #pragma unroll
    for (int c = lane; c < 16 * CPR; c += 64) {
      const int r = c / CPR, ch = c % CPR;
      const int q = qw + r;
      if (q < a.q_rows) st16(a.o + (tokq + q) * a.o_stride + (long)h * D + ch * 8, ld16(Os + r * D + ch * 8));
    }
  }
}

// flash_fwd2_kernel<D>: the prefill kernel with the O accumulator transposed and the per-score VALU cut
// (Llama prefill, D = 128: the v1 loop issued ~450 VALU + ~170 SALU per wave per 64-key tile against
// 32 MFMAs -- 193 TFLOP/s at B = 8 x 512, profiles/r6_flash_llama_probe.txt).  Same tiling, loads and
// LDS layouts as flash_fwd_kernel; per tile and wave:
//   * O^T += V^T P^T: the PV MFMA with its operands swapped (the V fragment read by ds_read_tr16 is the
//     A operand's layout as well), so the accumulator holds O[q = lane column][d rows] and the softmax
//     rescale / final 1 / l are lane-local -- no cross-lane shuffles of alpha or 1 / l;
//   * the row sum l stays a per-lane partial over the lane's own keys (combined once, at the end);
//   * scores stay unscaled: the row max is taken raw, one FMA per score forms x * scale - m;
//     -1e30 instead of -inf for the running max removes every "no key yet" select;
//   * the key-range / causal mask runs only on the tiles that need it (wave-uniform branch), where
//     16-key sub-tiles wholly above the diagonal also skip their MFMAs;
//   * tile load offsets are computed once and advanced by one add per tile.
// One tile body with wave-uniform branches, 158 VGPRs: 3 waves per SIMD.  (Full and edge tiles as
// two straight-line copies of the body took 196 VGPRs -- 2 waves per SIMD -- and measured 71-73 vs
// 62 us at B = 8 x 512: profiles/r6_flash_v2_vs_v1.jsonl.)
template <int D, int NW = 4>
__global__ __launch_bounds__(64 * NW, NW == 8 ? 2 : 3) void flash_fwd2_kernel(const AttnArgs a) {
  constexpr int NT = 64 * NW;
  constexpr int BQ = 16 * NW, BKV = 64;
  constexpr int CPR = D / 8;
  constexpr int KK = D / 32;
  constexpr int DT = D / 16;
  constexpr int VST = D * 2 + 32;
  constexpr int K_BYTES = BKV * D * 2;
  constexpr int V_BYTES = BKV * VST;
  __shared__ __attribute__((aligned(16))) char smem[K_BYTES + V_BYTES];
  char* Ks = smem;
  char* Vs = smem + K_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, fr = lane & 15;
  const int b = blockIdx.z, h = blockIdx.y;
  const int hk = h / (a.Hq / a.Hkv);
  const int q0 = blockIdx.x * BQ;
  const int qw = q0 + wid * 16;
  MLS_CHECK(!a.kv_lens || a.kv_lens[b] <= a.S, 302);
  const int L = a.kv_lens ? min(a.kv_lens[b], a.S) : a.S;
  const long tok0 = (long)b * a.S, tokq = (long)b * a.q_rows;

  const rsrc_t qr = make_rsrc(a.q, a.q_bytes);
  const rsrc_t kr = make_rsrc(a.k, a.k_bytes);
  const rsrc_t vr = make_rsrc(a.v, a.v_bytes);

  bf16x8 qf[KK];  // Q^T fragments (B operand of S^T = K Q^T): Q[q = qw + fr][d = 32kk + 8g .. +7]
  {
    const int q = qw + fr;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const int off = q < a.q_rows ? (int)(((tokq + q) * a.q_stride + (long)h * D + 32 * kk + 8 * g) * 2) : OOB;
      qf[kk] = __builtin_bit_cast(bf16x8, bload16(qr, off));
    }
  }

  f32x4 acc_o[DT];  // acc_o[dt][j] = O[q = qw + fr][d = 16dt + 4g + j] (unnormalised)
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) acc_o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float c = a.scale_log2;
  float m_run = -1e30f;  // running max of the scaled scores of query fr (log2 units)
  float l_run = 0.f;     // this lane's partial of the row sum (its own keys only)

  int kv_end = L;
  if (a.causal) kv_end = min(kv_end, q0 + BQ);
  const int ntiles = (kv_end + BKV - 1) / BKV;

  constexpr int NI = (BKV * CPR) / NT;
  static_assert(NI * NT == BKV * CPR, "tile chunks split evenly over the block");
  int krow[NI], koff[NI], voff[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int idx = tid + NT * i;
    const int row = idx / CPR, ch = idx % CPR;
    krow[i] = row;
    koff[i] = (int)(((tok0 + row) * a.k_stride + (long)hk * D + ch * 8) * 2);
    voff[i] = (int)(((tok0 + row) * a.v_stride + (long)hk * D + ch * 8) * 2);
  }
  const int kstep = BKV * a.k_stride * 2, vstep = BKV * a.v_stride * 2;
  uint4 kreg[NI], vreg[NI];
  auto load_into = [&](int kt, uint4 (&kd)[NI], uint4 (&vd)[NI]) {
    const int kv0 = kt * BKV;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const bool ok = kv0 + krow[i] < L;
      kd[i] = bload16(kr, ok ? koff[i] + kt * kstep : OOB);
      vd[i] = bload16(vr, ok ? voff[i] + kt * vstep : OOB);
    }
  };
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  auto tile_body = [&](int kv0, bool EDGE) {
    f32x4 s[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      // a causal sub-tile wholly above the wave's diagonal: no MFMAs (masked to -inf below)
      if (EDGE && a.causal && kv0 + 16 * t > qw + 15) continue;
      const int row = 16 * t + fr;
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const int ch = 4 * kk + g;
        const bf16x8 kf = __builtin_bit_cast(
            bf16x8, *reinterpret_cast<const uint4*>(Ks + row * (D * 2) + ((ch ^ (row & (CPR - 1))) * 16)));
        s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[kk], s[t], 0, 0, 0);
      }
    }
    if (EDGE) {
      const int qabs = qw + fr;
      const int lim = a.causal ? min(L - 1, qabs) : L - 1;  // last visible key of this query
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (kv0 + 16 * t + 4 * g + j > lim) s[t][j] = -INFINITY;
    }
    float mt = fmaxf(fmaxf(fmaxf(s[0][0], s[0][1]), fmaxf(s[0][2], s[0][3])),
                     fmaxf(fmaxf(s[1][0], s[1][1]), fmaxf(s[1][2], s[1][3])));
    mt = fmaxf(mt, fmaxf(fmaxf(fmaxf(s[2][0], s[2][1]), fmaxf(s[2][2], s[2][3])),
                         fmaxf(fmaxf(s[3][0], s[3][1]), fmaxf(s[3][2], s[3][3]))));
    mt = fmaxf(mt, xor16_f(mt));
    mt = fmaxf(mt, xor32_f(mt));
    const float m_new = fmaxf(m_run, mt * c);  // -inf * c stays -inf; m_run >= -1e30
    const float alpha = fast_exp2(m_run - m_new);
    m_run = m_new;
    // x * scale - m as packed FMAs (v_pk_fma_f32), two scores per instruction
    const f32x2 c2 = {c, c}, nm2 = {-m_new, -m_new};
    f32x2 ls2 = {0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        f32x2 x = {s[t][2 * jj], s[t][2 * jj + 1]};
        x = __builtin_elementwise_fma(x, c2, nm2);
        const f32x2 p = {fast_exp2(x[0]), fast_exp2(x[1])};  // masked: exp2(-inf) = 0
        s[t][2 * jj] = p[0];
        s[t][2 * jj + 1] = p[1];
        ls2 += p;
      }
    l_run = fmaf(l_run, alpha, ls2[0] + ls2[1]);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) acc_o[dt] *= alpha;
    // ---- O^T += V^T P^T: two 32-key k-steps, key order permuted identically in both operands ----
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      if (EDGE && a.causal && kv0 + 32 * st > qw + 15) continue;  // both sub-tiles above the diagonal
      bf16x8 pf;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pf[j] = (bf16)s[2 * st][j];
        pf[4 + j] = (bf16)s[2 * st + 1][j];
      }
      const int qq = fr >> 2, pp = fr & 3;
      const int row0 = 32 * st + 4 * g + qq;
      const int row1 = row0 + 16;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int colb = (16 * dt + 4 * pp) * 2;
        const short4v r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS short4v*)(Vs + row0 * VST + colb));
        const short4v r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS short4v*)(Vs + row1 * VST + colb));
        typedef short short8v __attribute__((ext_vector_type(8)));
        const short8v vv = {r0[0], r0[1], r0[2], r0[3], r1[0], r1[1], r1[2], r1[3]};
        acc_o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, vv), pf, acc_o[dt], 0, 0, 0);
      }
    }
  };
  // 8-wave blocks (BERT, S <= 128: two tiles): tile 1's loads go out right behind tile 0's, as in v1
  const bool pre = NW == 8 && a.pre;
  uint4 kpre[NI], vpre[NI];
  if (ntiles > 0) load_into(0, kreg, vreg);
  if (pre && ntiles > 1) load_into(1, kpre, vpre);

  for (int kt = 0; kt < ntiles; ++kt) {
    const int kv0 = kt * BKV;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int idx = tid + NT * i;
      const int row = idx / CPR, ch = idx % CPR;
      *reinterpret_cast<uint4*>(Ks + row * (D * 2) + ((ch ^ (row & (CPR - 1))) * 16)) = kreg[i];
      *reinterpret_cast<uint4*>(Vs + row * VST + ch * 16) = vreg[i];
    }
    __syncthreads();
    if (kt + 1 < ntiles) {
      if (pre && kt == 0) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          kreg[i] = kpre[i];
          vreg[i] = vpre[i];
        }
      } else {
        load_into(kt + 1, kreg, vreg);
      }
    }

    // keys kv0 + 16t + 4g + j against query qw + fr; the mask (and the causal sub-tile skip) only
    // where the tile crosses the key range end or the wave's diagonal
    tile_body(kv0, kv0 + BKV > L || (a.causal && kv0 + BKV - 1 > qw));
    __syncthreads();
  }

  // ---- normalise (lane-local 1 / l of query fr) and store through LDS as 16-B row stores
  float l = l_run + xor16_f(l_run);
  l += xor32_f(l);
  const float inv_l = l > 0.f ? 1.f / l : 0.f;
  // rows padded by 16 B: the 16 query rows of one 8-B write land in different banks
  constexpr int OST = D + 8;
  bf16* Os = reinterpret_cast<bf16*>(smem) + wid * 16 * OST;  // K / V tile space: past the last barrier
  static_assert(NW * 16 * OST * 2 <= K_BYTES + V_BYTES, "output tiles fit the K / V tiles");
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    bf16x4 o4;
#pragma unroll
    for (int j = 0; j < 4; ++j) o4[j] = (bf16)(acc_o[dt][j] * inv_l);
    *reinterpret_cast<bf16x4*>(Os + fr * OST + 16 * dt + 4 * g) = o4;
  }
  __syncthreads();
#pragma unroll
  for (int cc = lane; cc < 16 * CPR; cc += 64) {
    const int r = cc / CPR, ch = cc % CPR;
    const int q = qw + r;
    if (q < a.q_rows) st16(a.o + (tokq + q) * a.o_stride + (long)h * D + ch * 8, ld16(Os + r * OST + ch * 8));
  }
}

// ------------------------------------------------------------------------------- decode
struct DecodeArgs {
  const bf16* q;   // [B][q_stride], head h at h*D (rope mode: the fused QKV row, K at Hq*D, V at (Hq+Hkv)*D)
  bf16* kc;        // [B][max_len][Hkv][D]
  bf16* vc;
  bf16* o;         // [B][o_stride]
  float* ws;       // [B][Hq][nsplit][D]
  float* ws_ml;    // [B][Hq][nsplit][2]
  int* counters;   // [B][Hkv], zero between launches (the last arriver resets its entry)
  int q_stride, o_stride;
  long seq_stride;  // elements per sequence in the cache (max_len * Hkv * D)
  const int* lens;
  const int* page_table;  // paged cache: [B][pages_per_seq] page ids, a page = one split's CHUNK rows
  int pages_per_seq;
  int hm_rows;  // 0: row-major cache rows [row][Hkv][D]; R: head-major blocks [row / R][Hkv][R][D]
  const int* positions;  // rope mode: query position per sequence (== lens[b] - 1)
  const float* cos_t;    // [max_pos][D/2]
  const float* sin_t;
  int Hq, Hkv, nsplit, max_pos;
  float scale_log2;
};

// rotate-half RoPE of this lane's 8 dims (d = gl*8 + e) given the partner lane's 8 (d +- D/2)
template <int D>
MLS_DEV void rope8(float (&x)[8], const float (&xp)[8], const float* cos_t, const float* sin_t, int pos, int gl) {
  constexpr int HALF = D / 2, HL = D / 16;  // HL = lanes per half row
  const int i0 = (gl % HL) * 8;
  const float4 c0 = *reinterpret_cast<const float4*>(cos_t + (long)pos * HALF + i0);
  const float4 c1 = *reinterpret_cast<const float4*>(cos_t + (long)pos * HALF + i0 + 4);
  const float4 s0 = *reinterpret_cast<const float4*>(sin_t + (long)pos * HALF + i0);
  const float4 s1 = *reinterpret_cast<const float4*>(sin_t + (long)pos * HALF + i0 + 4);
  const float c[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
  const float sn[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
  const float sgn = gl < HL ? -1.f : 1.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) x[e] = x[e] * c[e] + sgn * xp[e] * sn[e];
}

// Decode attention: grid (splits, Hkv, B), 4 waves; the G query heads of a KV head share every
// K/V row load.  A lane owns 8 of a row's D dims (LPR lanes per row, RPW rows per wave, ROWS =
// 4*RPW rows per block pass); all NIT passes' K/V loads are issued before any math (one memory
// round trip per block).  Rope mode also applies RoPE to q and to the new token's K (row lens-1,
// taken from the QKV row, not the cache) and appends that K/V to the cache -- the standalone
// rope/KV-append kernel is gone from decode.  The RPW row groups of a wave merge by shuffles, the
// 4 waves through LDS; a sequence that fits one split writes its output directly, otherwise each
// split writes an fp32 partial (m, l, o) for decode_combine_kernel.  (An in-launch last-arriver
// merge was measured slower: its per-block release fences serialise per XCD, and write-through
// partials read back serially cost more than the extra launch.)
template <int D, int G, int NIT>
__global__ __launch_bounds__(256) void decode_attn_kernel(const DecodeArgs a) {
  constexpr int LPR = D / 8;      // lanes per key row
  constexpr int RPW = 64 / LPR;   // rows per wave step
  constexpr int ROWS = 4 * RPW;   // rows per block pass
  constexpr int CHUNK = ROWS * NIT;
  __shared__ float sm_m[4][G], sm_l[4][G];
  __shared__ __attribute__((aligned(16))) float sm_o[4][G][D];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int grp = lane / LPR, gl = lane % LPR, glp = gl ^ (LPR / 2);
  // grid (Hkv, splits, B): the Hkv blocks of one (split, sequence) dispatch back to back, so the
  // 256-B head slices of each 2 KiB cache row are read together (one DRAM row open, not Hkv)
  const int b = blockIdx.z, hk = blockIdx.x, sp = blockIdx.y;
  const int L0 = a.lens[b];
  // keys past the split grid are never visited: a host context bound below lens is a caller bug
  MLS_CHECK(sp != 0 || L0 <= a.nsplit * CHUNK, 201);
  const int L = min(L0, a.nsplit * CHUNK);
  const int start = sp * CHUNK;
  if (start >= L) {
    if (L <= 0 && sp == 0)
      for (int idx = tid; idx < G * D; idx += 256) a.o[(long)b * a.o_stride + (long)hk * G * D + idx] = (bf16)0.f;
    return;
  }
  const int end = min(L, start + CHUNK);
  const bool rope = a.positions != nullptr;
  const int pos = rope ? a.positions[b] : 0;
  MLS_CHECK(!rope || (pos >= 0 && pos < a.max_pos && pos == L0 - 1), 202);
  const bf16* qrow = a.q + (long)b * a.q_stride;
  // row r of this split lives at cbase + r * rstride: contiguous per sequence, or (paged) in the page
  // the table maps this split to -- a page holds exactly one split's CHUNK rows.  Head-major caches
  // keep one head's rows contiguous (rstride = D): the block streams one 64 x 256 B run.
  const long rstride = a.hm_rows > 0 ? (long)D : (long)a.Hkv * D;
  long cbase;
  if (a.hm_rows > 0) {
    const long blk = a.page_table ? (long)a.page_table[b * a.pages_per_seq + sp] : (long)b;
    const long r0 = a.page_table ? (long)start : 0;  // row index of the block's first row
    cbase = ((blk * a.Hkv + hk) * a.hm_rows - r0) * D + gl * 8;
  } else {
    const long sbase = a.page_table ? ((long)a.page_table[b * a.pages_per_seq + sp] * CHUNK - start) * rstride
                                    : (long)b * a.seq_stride;
    cbase = sbase + (long)hk * D + gl * 8;
  }

  // issue every K/V row load of this block first
  uint4 kraw[NIT], vraw[NIT];
#pragma unroll
  for (int i = 0; i < NIT; ++i) {
    const int r = start + i * ROWS + wid * RPW + grp;
    const bool ld = r < end && !(rope && r == L - 1);
    kraw[i] = ld ? ld16(a.kc + cbase + r * rstride) : make_uint4(0, 0, 0, 0);
    vraw[i] = ld ? ld16(a.vc + cbase + r * rstride) : make_uint4(0, 0, 0, 0);
  }
  // every small operand (the G query heads, their RoPE partners, the position's cos / sin, the new
  // token's K / V) is loaded in the same batch as the cache rows, before any of it is used: one
  // memory round trip per block instead of a dependent q -> rope chain per head
  uint4 qraw[G], qpraw[G], knew = make_uint4(0, 0, 0, 0), kpnew = knew, vnew = knew;
  float4 cs[4] = {};
#pragma unroll
  for (int hh = 0; hh < G; ++hh) {
    const bf16* qh = qrow + (long)(hk * G + hh) * D;
    qraw[hh] = ld16(qh + gl * 8);
    qpraw[hh] = rope ? ld16(qh + glp * 8) : make_uint4(0, 0, 0, 0);
  }
  const bool has_new = rope && L - 1 >= start && L - 1 < end;
  if (rope) {
    const int i0 = (gl % (D / 16)) * 8;
    const float* cp = a.cos_t + (long)pos * (D / 2) + i0;
    const float* sp_ = a.sin_t + (long)pos * (D / 2) + i0;
    cs[0] = *reinterpret_cast<const float4*>(cp);
    cs[1] = *reinterpret_cast<const float4*>(cp + 4);
    cs[2] = *reinterpret_cast<const float4*>(sp_);
    cs[3] = *reinterpret_cast<const float4*>(sp_ + 4);
    // (every block of the sequence loads the new row, so the loads batch with the rest unbranched)
    const bf16* kh = qrow + (long)(a.Hq + hk) * D;
    knew = ld16(kh + gl * 8);
    kpnew = ld16(kh + glp * 8);
    vnew = ld16(qrow + (long)(a.Hq + a.Hkv + hk) * D + gl * 8);
  }
  auto rope_regs = [&](float (&x)[8], const float (&xp)[8]) {
    const float c[8] = {cs[0].x, cs[0].y, cs[0].z, cs[0].w, cs[1].x, cs[1].y, cs[1].z, cs[1].w};
    const float sn[8] = {cs[2].x, cs[2].y, cs[2].z, cs[2].w, cs[3].x, cs[3].y, cs[3].z, cs[3].w};
    const float sgn = gl < D / 16 ? -1.f : 1.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = x[e] * c[e] + sgn * xp[e] * sn[e];
  };
  float qv[G][8];
#pragma unroll
  for (int hh = 0; hh < G; ++hh) {
    unpack8(qraw[hh], qv[hh]);
    if (rope) {
      float xp[8];
      unpack8(qpraw[hh], xp);
      rope_regs(qv[hh], xp);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) qv[hh][e] = (float)(bf16)qv[hh][e] * a.scale_log2;  // bf16 q, as the cache path
  }
  if (has_new) {  // the new token's row, appended to the cache
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int r = start + i * ROWS + wid * RPW + grp;
      if (r == L - 1) {
        float kx[8], kp[8];
        unpack8(knew, kx);
        unpack8(kpnew, kp);
        rope_regs(kx, kp);
        kraw[i] = pack8(kx);
        vraw[i] = vnew;
        st16(a.kc + cbase + r * rstride, kraw[i]);
        st16(a.vc + cbase + r * rstride, vraw[i]);
      }
    }
  }

  float m[G], l[G], acc[G][8];
#pragma unroll
  for (int hh = 0; hh < G; ++hh) {
    m[hh] = -INFINITY;
    l[hh] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[hh][e] = 0.f;
  }
#pragma unroll
  for (int i = 0; i < NIT; ++i) {
    if (start + i * ROWS >= end) break;  // block-uniform
    const int r = start + i * ROWS + wid * RPW + grp;
    float kf[8], vf[8];
    unpack8(kraw[i], kf);
    unpack8(vraw[i], vf);
    const bool valid = r < end;
#pragma unroll
    for (int hh = 0; hh < G; ++hh) {
      float d = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) d += qv[hh][e] * kf[e];
      d = group_sum<LPR>(d);  // the row's LPR lanes (DPP, no LDS round trips)
      const float sc = valid ? d : -INFINITY;
      const float mn = fmaxf(m[hh], sc);
      if (mn == -INFINITY) continue;
      const float al = __builtin_amdgcn_exp2f(m[hh] - mn);
      const float p = __builtin_amdgcn_exp2f(sc - mn);
      l[hh] = l[hh] * al + p;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[hh][e] = acc[hh][e] * al + p * vf[e];
      m[hh] = mn;
    }
  }
  // merge the wave's RPW row groups (lanes gl + LPR*grp) by shuffles
#pragma unroll
  for (int hh = 0; hh < G; ++hh) {
    // partner lanes (lane ^ o) by DPP row rotation / v_permlane swaps
    auto xchg = [](float v, int o) { return o == 8 ? xor8_f(v) : o == 16 ? xor16_f(v) : xor32_f(v); };
#pragma unroll
    for (int o = LPR; o < 64; o <<= 1) {
      const float m2 = xchg(m[hh], o), l2 = xchg(l[hh], o);
      const float mn = fmaxf(m[hh], m2);
      const float w1 = mn == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m[hh] - mn);
      const float w2 = mn == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m2 - mn);
      l[hh] = l[hh] * w1 + l2 * w2;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[hh][e] = acc[hh][e] * w1 + xchg(acc[hh][e], o) * w2;
      m[hh] = mn;
    }
    if (grp == 0) {
      if (gl == 0) {
        sm_m[wid][hh] = m[hh];
        sm_l[wid][hh] = l[hh];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) sm_o[wid][hh][gl * 8 + e] = acc[hh][e];
    }
  }
  __syncthreads();
  const bool direct = L <= CHUNK;
  for (int idx = tid; idx < G * D; idx += 256) {
    const int hh = idx / D, d = idx % D;
    float M = -INFINITY;
#pragma unroll
    for (int p = 0; p < 4; ++p) M = fmaxf(M, sm_m[p][hh]);
    float Ls = 0.f, O = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const float w = __builtin_amdgcn_exp2f(sm_m[p][hh] - M);
        Ls += sm_l[p][hh] * w;
        O += sm_o[p][hh][d] * w;
      }
    }
    if (direct) {
      a.o[(long)b * a.o_stride + (long)(hk * G + hh) * D + d] = (bf16)(Ls > 0.f ? O / Ls : 0.f);
    } else {
      const long base = ((long)b * a.Hq + hk * G + hh) * a.nsplit + sp;
      a.ws[base * D + d] = O;
      if (d == 0) {
        a.ws_ml[base * 2] = M;
        a.ws_ml[base * 2 + 1] = Ls;
      }
    }
  }
}

// Decode attention on the matrix cores (D = 128, chunk = 32 keys per wave).  The VALU kernel
// above spends ~850 VALU instructions per wave on a 64-key split (per key and head: the 8-lane
// dot, its DPP reduction, the online-softmax rescale of 8 accumulators), which is what bounds it
// at large batch (batch 128: 55M VALU instructions per layer, ~2.3 TB/s of KV).  Here, per wave:
//   S^T = K . Q^T  (A = 32 key rows straight from the cache, 16-B loads; B = the G roped query
//                  heads from LDS, head on the lane column, padded to 16 with zeros): 8 MFMAs
//   O   = P . V    (A = P packed from the S^T accumulators, B = V through a per-wave row-major
//                  LDS image read with ds_read_b64_tr_b16, keys in the same permuted order):
//                  8 MFMAs, one softmax pass (all 32 keys are in registers, no rescale)
// RoPE of q / the new key and the KV append run once per block in an LDS prologue.  Partials
// (m, l, O) are merged over the block's waves and written exactly as the VALU kernel does, so
// decode_combine_kernel and the fused combine of mls_skinny_packed_combine are shared.
template <int G, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void decode_attn_mfma_kernel(const DecodeArgs a) {
  constexpr int D = 128, KK = D / 32, DT = D / 16;
  constexpr int NT = WAVES * 64, CHUNK = WAVES * 32;
  constexpr int VST = D * 2 + 32;          // padded V row (bytes): conflict-free transposed reads
  constexpr int NPRO = (G + 1) * 16;       // prologue tasks: G query heads + the new key row, 16-B chunks
  constexpr int PIT = (NPRO + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) char vs[WAVES][32 * VST];
  __shared__ __attribute__((aligned(16))) bf16 qimg[G + 2][D];  // roped q heads, roped new K, new V
  __shared__ float sm_m[WAVES][G], sm_l[WAVES][G];
  __shared__ __attribute__((aligned(16))) float sm_o[WAVES][G][D];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, fr = lane & 15;
  const int b = blockIdx.z, hk = blockIdx.x, sp = blockIdx.y;
  const int L0 = a.lens[b];
  MLS_CHECK(sp != 0 || L0 <= a.nsplit * CHUNK, 201);
  const int L = min(L0, a.nsplit * CHUNK);
  const int start = sp * CHUNK;
  if (start >= L) {
    if (L <= 0 && sp == 0)
      for (int idx = tid; idx < G * D; idx += NT) a.o[(long)b * a.o_stride + (long)hk * G * D + idx] = (bf16)0.f;
    return;
  }
  const int end = min(L, start + CHUNK);
  const bool rope = a.positions != nullptr;
  const int pos = rope ? a.positions[b] : 0;
  MLS_CHECK(!rope || (pos >= 0 && pos < a.max_pos && pos == L0 - 1), 202);
  const bf16* qrow = a.q + (long)b * a.q_stride;
  const long rstride = a.hm_rows > 0 ? (long)D : (long)a.Hkv * D;
  long cbase;
  if (a.hm_rows > 0) {
    const long blk = a.page_table ? (long)a.page_table[b * a.pages_per_seq + sp] : (long)b;
    const long r0 = a.page_table ? (long)start : 0;
    cbase = ((blk * a.Hkv + hk) * a.hm_rows - r0) * D;
  } else {
    cbase = a.page_table ? ((long)a.page_table[b * a.pages_per_seq + sp] * CHUNK - start) * rstride
                         : (long)b * a.seq_stride;
    cbase += (long)hk * D;
  }
  const bool has_new = rope && L - 1 >= start && L - 1 < end;
  const int w0 = start + wid * 32;  // this wave's first key

  // small operands first (so their vmcnt waits leave the cache rows in flight), then the rows
  uint4 px[PIT], pxp[PIT], pv[PIT];
  float4 pcs[PIT][4];
#pragma unroll
  for (int it = 0; it < PIT; ++it) {
    const int t = tid + it * NT, r = t >> 4, c = t & 15;
    px[it] = pxp[it] = pv[it] = make_uint4(0, 0, 0, 0);
    pcs[it][0] = pcs[it][1] = pcs[it][2] = pcs[it][3] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (t < NPRO && (r < G || rope)) {
      const bf16* src = qrow + (long)(r < G ? hk * G + r : a.Hq + hk) * D;
      px[it] = ld16(src + c * 8);
      if (rope) {
        pxp[it] = ld16(src + ((c + 8) & 15) * 8);
        const float* cp = a.cos_t + (long)pos * (D / 2) + (c & 7) * 8;
        const float* sq = a.sin_t + (long)pos * (D / 2) + (c & 7) * 8;
        pcs[it][0] = *reinterpret_cast<const float4*>(cp);
        pcs[it][1] = *reinterpret_cast<const float4*>(cp + 4);
        pcs[it][2] = *reinterpret_cast<const float4*>(sq);
        pcs[it][3] = *reinterpret_cast<const float4*>(sq + 4);
        if (r == G) pv[it] = ld16(qrow + (long)(a.Hq + a.Hkv + hk) * D + c * 8);
      }
    }
  }
  uint4 kraw[2][KK], vraw[8];
#pragma unroll
  for (int t2 = 0; t2 < 2; ++t2) {
    const int key = w0 + 16 * t2 + fr;
    const bool ok = key < end && !(rope && key == L - 1);
#pragma unroll
    for (int kk = 0; kk < KK; ++kk)
      kraw[t2][kk] = ok ? ld16(a.kc + cbase + key * rstride + 32 * kk + 8 * g) : make_uint4(0, 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int key = w0 + 4 * i + g;
    const bool ok = key < end && !(rope && key == L - 1);
    vraw[i] = ok ? ld16(a.vc + cbase + key * rstride + fr * 8) : make_uint4(0, 0, 0, 0);
  }

  // prologue: RoPE'd q heads (bf16, as the cache path rounds them) and the new key row -> LDS;
  // the block holding row L-1 appends the new K / V to the cache
#pragma unroll
  for (int it = 0; it < PIT; ++it) {
    const int t = tid + it * NT, r = t >> 4, c = t & 15;
    if (t < NPRO && (r < G || rope)) {
      float x[8];
      unpack8(px[it], x);
      if (rope) {
        float xp[8];
        unpack8(pxp[it], xp);
        const float cc[8] = {pcs[it][0].x, pcs[it][0].y, pcs[it][0].z, pcs[it][0].w,
                             pcs[it][1].x, pcs[it][1].y, pcs[it][1].z, pcs[it][1].w};
        const float sn[8] = {pcs[it][2].x, pcs[it][2].y, pcs[it][2].z, pcs[it][2].w,
                             pcs[it][3].x, pcs[it][3].y, pcs[it][3].z, pcs[it][3].w};
        const float sgn = c < 8 ? -1.f : 1.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = x[e] * cc[e] + sgn * xp[e] * sn[e];
      }
      const uint4 xb = pack8(x);
      *reinterpret_cast<uint4*>(&qimg[r][c * 8]) = xb;
      if (r == G) {
        *reinterpret_cast<uint4*>(&qimg[G + 1][c * 8]) = pv[it];
        if (has_new) {
          st16(a.kc + cbase + (long)(L - 1) * rstride + c * 8, xb);
          st16(a.vc + cbase + (long)(L - 1) * rstride + c * 8, pv[it]);
        }
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  bf16x8 qf[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk)
    qf[kk] = fr < G ? __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(&qimg[fr < G ? fr : 0][32 * kk + 8 * g]))
                    : __builtin_bit_cast(bf16x8, make_uint4(0, 0, 0, 0));
  f32x4 s[2];
#pragma unroll
  for (int t2 = 0; t2 < 2; ++t2) {
    if (rope && w0 + 16 * t2 + fr == L - 1) {
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) kraw[t2][kk] = *reinterpret_cast<const uint4*>(&qimg[G][32 * kk + 8 * g]);
    }
    s[t2] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KK; ++kk)
      s[t2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kraw[t2][kk]), qf[kk], s[t2], 0, 0, 0);
  }
  // softmax over the wave's 32 keys (key = w0 + 16 t2 + 4g + j on accumulator row, head fr on the lane)
  float mt = -INFINITY;
#pragma unroll
  for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float x = w0 + 16 * t2 + 4 * g + j < end ? s[t2][j] * a.scale_log2 : -INFINITY;
      s[t2][j] = x;
      mt = fmaxf(mt, x);
    }
  mt = fmaxf(mt, xor16_f(mt));
  mt = fmaxf(mt, xor32_f(mt));
  float ls = 0.f;
#pragma unroll
  for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float p = mt == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(s[t2][j] - mt);
      s[t2][j] = p;
      ls += p;
    }
  ls += xor16_f(ls);
  ls += xor32_f(ls);

  // V rows -> this wave's LDS image (row-major, padded); the new row from the prologue image
  char* V = vs[wid];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint4 v = vraw[i];
    if (rope && w0 + 4 * i + g == L - 1) v = *reinterpret_cast<const uint4*>(&qimg[G + 1][fr * 8]);
    *reinterpret_cast<uint4*>(V + (4 * i + g) * VST + fr * 16) = v;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's image, read back by the same wave
  bf16x8 pf;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    pf[j] = (bf16)s[0][j];
    pf[4 + j] = (bf16)s[1][j];
  }
  const int row0 = 4 * g + (fr >> 2), row1 = row0 + 16;
  f32x4 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    const int colb = (16 * dt + 4 * (fr & 3)) * 2;
    const short4v r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS short4v*)(V + row0 * VST + colb));
    const short4v r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS short4v*)(V + row1 * VST + colb));
    typedef short short8v __attribute__((ext_vector_type(8)));
    const short8v vv = {r0[0], r0[1], r0[2], r0[3], r1[0], r1[1], r1[2], r1[3]};
    o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf, __builtin_bit_cast(bf16x8, vv), f32x4{0.f, 0.f, 0.f, 0.f},
                                                    0, 0, 0);
  }
  // O rows = heads 4g + j, columns d = 16 dt + fr
  if (g == 0 && fr < G) {
    sm_m[wid][fr] = mt;
    sm_l[wid][fr] = ls;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int h = 4 * g + j;
    if (h < G) {
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) sm_o[wid][h < G ? h : 0][16 * dt + fr] = o[dt][j];
    }
  }
  __syncthreads();
  const bool direct = L <= CHUNK;
  for (int idx = tid; idx < G * D; idx += NT) {
    const int hh = idx / D, d = idx % D;
    float M = -INFINITY;
#pragma unroll
    for (int p = 0; p < WAVES; ++p) M = fmaxf(M, sm_m[p][hh]);
    float Ls = 0.f, O = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int p = 0; p < WAVES; ++p) {
        const float w = __builtin_amdgcn_exp2f(sm_m[p][hh] - M);
        Ls += sm_l[p][hh] * w;
        O += sm_o[p][hh][d] * w;
      }
    }
    if (direct) {
      a.o[(long)b * a.o_stride + (long)(hk * G + hh) * D + d] = (bf16)(Ls > 0.f ? O / Ls : 0.f);
    } else {
      const long base = ((long)b * a.Hq + hk * G + hh) * a.nsplit + sp;
      a.ws[base * D + d] = O;
      if (d == 0) {
        a.ws_ml[base * 2] = M;
        a.ws_ml[base * 2 + 1] = Ls;
      }
    }
  }
}

// merge the splits of one (b, q-head): block of D threads; the (m, l) of every split are read
// once into LDS (one round trip), then each thread's O loads are issued 8 at a time
template <int D>
__global__ __launch_bounds__(D) void decode_combine_kernel(const DecodeArgs a, int chunk) {
  __shared__ float sw[1024];
  __shared__ float s_inv;
  const int bh = blockIdx.x;  // b * Hq + h
  const int b = bh / a.Hq, h = bh % a.Hq;
  const int d = threadIdx.x;
  const int L = a.lens[b];
  const int ns = min(a.nsplit, (L + chunk - 1) / chunk);
  if (ns <= 1) return;  // the split kernel wrote this row directly
  const long rec = (long)bh * a.nsplit;
  // independent loads first, one round trip: the first 8 splits' partial O (clamped index, used
  // below only for s < ns) and, when every split has a lane (ns <= D: always at the 64 / 128-row
  // chunks up to 8k contexts), this lane's (m, l) pair -- kept for the second pass
  const bool one = ns <= D;  // block-uniform
  float vpre[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) vpre[j] = a.ws[(rec + min(j, ns - 1)) * D + d];
  float2 mine = make_float2(-INFINITY, 0.f);
  float mloc = -INFINITY;
  if (one) {
    mine = *reinterpret_cast<const float2*>(a.ws_ml + (rec + min(d, ns - 1)) * 2);
    if (d >= ns) mine = make_float2(-INFINITY, 0.f);
    mloc = mine.x;
  } else {
    for (int s = d; s < ns; s += D) mloc = fmaxf(mloc, a.ws_ml[(rec + s) * 2]);
  }
  __shared__ float red[D / 64];
  mloc = wave_max(mloc);
  if ((d & 63) == 0) red[d >> 6] = mloc;
  __syncthreads();
  float M = red[0];
#pragma unroll
  for (int w = 1; w < D / 64; ++w) M = fmaxf(M, red[w]);
  float lloc = 0.f;
  if (one) {
    const float w = (M == -INFINITY || d >= ns) ? 0.f : __builtin_amdgcn_exp2f(mine.x - M);
    if (d < ns) sw[d] = w;
    lloc = mine.y * w;
  } else {
    for (int s = d; s < ns; s += D) {
      const float w = M == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(a.ws_ml[(rec + s) * 2] - M);
      sw[s] = w;
      lloc += a.ws_ml[(rec + s) * 2 + 1] * w;
    }
  }
  lloc = wave_sum(lloc);
  __syncthreads();
  if ((d & 63) == 0) red[d >> 6] = lloc;
  __syncthreads();
  if (d == 0) {
    float Ls = 0.f;
#pragma unroll
    for (int w = 0; w < D / 64; ++w) Ls += red[w];
    s_inv = Ls > 0.f ? 1.f / Ls : 0.f;
  }
  __syncthreads();
  float O = 0.f;
  const int nf = min(ns, 8);
#pragma unroll
  for (int j = 0; j < 8; ++j)
    if (j < nf) O += vpre[j] * sw[j];
  int s = nf;
  for (; s + 8 <= ns; s += 8) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = a.ws[(rec + s + j) * D + d];
#pragma unroll
    for (int j = 0; j < 8; ++j) O += v[j] * sw[s + j];
  }
  for (; s < ns; ++s) O += a.ws[(rec + s) * D + d] * sw[s];
  a.o[(long)b * a.o_stride + (long)h * D + d] = (bf16)(O * s_inv);
}

}  // namespace

// D = 128 (Llama prefill): 2 = the transposed-O kernel (default), 1 = the v1 loop (A/B; MLS_FLASH_V)
static int g_flash_ver = [] {
  const char* e = getenv("MLS_FLASH_V");
  return e ? atoi(e) : 2;
}();

extern "C" {

int mls_flash_set_version(int v) {  // returns the previous version
  if (v != 1 && v != 2) return MLS_BAD_ARG;
  const int old = g_flash_ver;
  g_flash_ver = v;
  return old;
}

// q/k/v point at the first element of head 0 of token 0; strides are token-row strides.  q_rows:
// query (and output) rows per sequence -- S for full attention; fewer = the first q_rows positions
// of each sequence only, against all of its keys (BERT's last layer: the [CLS] row), q / o then
// hold B * q_rows rows.
int mls_flash_attention_rows(const void* q, const void* k, const void* v, void* o, int q_stride, int k_stride,
                             int v_stride, int o_stride, int B, int S, int q_rows, int Hq, int Hkv, int D,
                             const int* kv_lens, int causal, float scale, void* stream) {
  if (B <= 0 || S <= 0 || Hq <= 0 || Hkv <= 0 || Hq % Hkv || q_rows <= 0 || q_rows > S) return MLS_BAD_ARG;
  if (q_stride % 8 || k_stride % 8 || v_stride % 8) return MLS_BAD_ARG;
  if (o_stride % 8 || (reinterpret_cast<uintptr_t>(o) & 15)) return MLS_BAD_ARG;  // 16-B row stores
  AttnArgs a{};
  a.q = (const bf16*)q;
  a.k = (const bf16*)k;
  a.v = (const bf16*)v;
  a.o = (bf16*)o;
  a.q_stride = q_stride; a.k_stride = k_stride; a.v_stride = v_stride; a.o_stride = o_stride;
  a.B = B; a.S = S; a.Hq = Hq; a.Hkv = Hkv;
  a.q_rows = q_rows;
  a.kv_lens = kv_lens;
  a.causal = causal;
  a.scale_log2 = scale * 1.4426950408889634f;
  const long T = (long)B * S, TQ = (long)B * q_rows;
  const size_t qb = ((size_t)(TQ - 1) * q_stride + (size_t)Hq * D) * 2;
  const size_t kb = ((size_t)(T - 1) * k_stride + (size_t)Hkv * D) * 2;
  const size_t vb = ((size_t)(T - 1) * v_stride + (size_t)Hkv * D) * 2;
  if (qb >= 0x7FFFFFFFull || kb >= 0x7FFFFFFFull || vb >= 0x7FFFFFFFull) return MLS_UNSUPPORTED;
  a.q_bytes = (uint32_t)qb; a.k_bytes = (uint32_t)kb; a.v_bytes = (uint32_t)vb;
  static const int pre_env = [] {
    const char* e = getenv("MLS_FLASH_PRE");
    return e ? atoi(e) : 1;
  }();
  a.pre = pre_env;
  if (D == 64 && q_rows <= 16) {  // a few rows per sequence: one wave per (sequence, head)
    hipLaunchKernelGGL((flash_fwd_kernel<64, 1>), dim3(1, Hq, B), dim3(64), 0, (hipStream_t)stream, a);
    return (int)hipGetLastError();
  }
  // BERT (D = 64, S <= 128): one 8-wave block holds all 128 queries of a (sequence, head), so the
  // head's K/V rows are fetched once instead of once per 64-query tile (MLS_FLASH_NW=4 restores
  // the 4-wave tiling for A/B)
  static const int nw_env = [] {
    const char* e = getenv("MLS_FLASH_NW");
    return e ? atoi(e) : 8;
  }();
  if (D == 64 && q_rows > 64 && q_rows <= 128 && nw_env == 8) {
    if (g_flash_ver == 2)
      hipLaunchKernelGGL((flash_fwd2_kernel<64, 8>), dim3(1, Hq, B), dim3(512), 0, (hipStream_t)stream, a);
    else
      hipLaunchKernelGGL((flash_fwd_kernel<64, 8>), dim3(1, Hq, B), dim3(512), 0, (hipStream_t)stream, a);
    return (int)hipGetLastError();
  }
  dim3 grid((q_rows + 63) / 64, Hq, B);
  if (D == 64)
    hipLaunchKernelGGL(flash_fwd_kernel<64>, grid, dim3(256), 0, (hipStream_t)stream, a);
  else if (D == 128 && g_flash_ver == 2)
    hipLaunchKernelGGL(flash_fwd2_kernel<128>, grid, dim3(256), 0, (hipStream_t)stream, a);
  else if (D == 128)
    hipLaunchKernelGGL(flash_fwd_kernel<128>, grid, dim3(256), 0, (hipStream_t)stream, a);
  else
    return MLS_UNSUPPORTED;
  return (int)hipGetLastError();
}

int mls_flash_attention(const void* q, const void* k, const void* v, void* o, int q_stride, int k_stride,
                        int v_stride, int o_stride, int B, int S, int Hq, int Hkv, int D, const int* kv_lens,
                        int causal, float scale, void* stream) {
  return mls_flash_attention_rows(q, k, v, o, q_stride, k_stride, v_stride, o_stride, B, S, S, Hq, Hkv, D, kv_lens,
                                  causal, scale, stream);
}

// workspace: ws >= B*Hq*nsplit*D floats, ws_ml >= B*Hq*nsplit*2 floats, nsplit = ceil(max_len/chunk);
// page_table (optional): [B][pages_per_seq] ids of chunk-row pages of the caches (paged KV).
// hm_rows: 0 = row-major cache [rows][Hkv][D]; R = head-major [rows / R][Hkv][R][D] (R = max_len
// per sequence, or the page rows when paged).
// skip_combine: leave multi-split rows as partials in ws / ws_ml (a consumer merges them, e.g.
// mls_skinny_packed_combine); rows that fit one split are still written to `o`.
// counters: B*Hkv zero-initialised ints.  chunk: rows per split (D=128: 16..256; D=64: 32..512).
// positions/cos/sin non-null: rope mode (q = the fused QKV rows, positions[b] == lens[b] - 1).
int mls_decode_attention(const void* q, void* k_cache, void* v_cache, void* o, float* ws, float* ws_ml, int* counters,
                         int q_stride, int o_stride, long seq_stride, const int* lens, const int* positions,
                         const float* cos_t, const float* sin_t, int max_pos, int B, int Hq, int Hkv, int D,
                         int max_len, int chunk, float scale, const int* page_table, int pages_per_seq,
                         int skip_combine, int hm_rows, int impl, void* stream) {
  if (B <= 0 || Hq % Hkv || chunk <= 0 || max_len <= 0) return MLS_BAD_ARG;
  if (page_table && (long)pages_per_seq * chunk < max_len) return MLS_BAD_ARG;
  (void)counters;  // reserved (in-launch merge variants); the combine runs as its own launch
  if (positions && (!cos_t || !sin_t)) return MLS_BAD_ARG;
  DecodeArgs a{};
  a.q = (const bf16*)q;
  a.kc = (bf16*)k_cache;
  a.vc = (bf16*)v_cache;
  a.o = (bf16*)o;
  a.ws = ws;
  a.ws_ml = ws_ml;
  a.counters = counters;
  a.q_stride = q_stride;
  a.o_stride = o_stride;
  a.seq_stride = seq_stride;
  a.lens = lens;
  a.page_table = page_table;
  a.pages_per_seq = pages_per_seq;
  a.hm_rows = hm_rows;
  if (page_table && hm_rows > 0 && hm_rows != chunk) return MLS_BAD_ARG;  // a page = one split
  a.positions = positions;
  a.cos_t = cos_t;
  a.sin_t = sin_t;
  a.max_pos = max_pos;
  a.Hq = Hq;
  a.Hkv = Hkv;
  a.nsplit = (max_len + chunk - 1) / chunk;
  a.scale_log2 = scale * 1.4426950408889634f;
  const int G = Hq / Hkv;
  const int rows = D == 128 ? 16 : 32;  // rows per block pass
  const int nit = chunk / rows;
  if (chunk % rows || (nit != 1 && nit != 2 && nit != 4 && nit != 8 && nit != 16)) return MLS_BAD_ARG;
  if (a.nsplit > 1024) return MLS_UNSUPPORTED;  // combine keeps one weight per split in LDS
  dim3 grid(Hkv, a.nsplit, B);
  hipStream_t st = (hipStream_t)stream;
  // impl: 0 auto, 1 VALU kernel, 2 matrix-core kernel (D = 128, 64- / 128- / 256-key splits, G <= 8)
  const bool mfma_ok = D == 128 && (chunk == 64 || chunk == 128 || chunk == 256) && (G == 1 || G == 2 || G == 4 || G == 8);
  if (impl == 2 && !mfma_ok) return MLS_UNSUPPORTED;
  if (impl != 1 && mfma_ok) {
#define DECM(GG)                                                                                            \
  if (chunk == 64) hipLaunchKernelGGL((decode_attn_mfma_kernel<GG, 2>), grid, dim3(128), 0, st, a);        \
  else if (chunk == 128) hipLaunchKernelGGL((decode_attn_mfma_kernel<GG, 4>), grid, dim3(256), 0, st, a);  \
  else hipLaunchKernelGGL((decode_attn_mfma_kernel<GG, 8>), grid, dim3(512), 0, st, a);
    if (G == 1) { DECM(1) }
    else if (G == 2) { DECM(2) }
    else if (G == 4) { DECM(4) }
    else { DECM(8) }
#undef DECM
    if (a.nsplit > 1 && !skip_combine)
      hipLaunchKernelGGL(decode_combine_kernel<128>, dim3(B * Hq), dim3(128), 0, st, a, chunk);
    return (int)hipGetLastError();
  }
#define DEC(DD, GG)                                                                                        \
  switch (nit) {                                                                                           \
    case 1: hipLaunchKernelGGL((decode_attn_kernel<DD, GG, 1>), grid, dim3(256), 0, st, a); break;        \
    case 2: hipLaunchKernelGGL((decode_attn_kernel<DD, GG, 2>), grid, dim3(256), 0, st, a); break;        \
    case 4: hipLaunchKernelGGL((decode_attn_kernel<DD, GG, 4>), grid, dim3(256), 0, st, a); break;        \
    case 8: hipLaunchKernelGGL((decode_attn_kernel<DD, GG, 8>), grid, dim3(256), 0, st, a); break;        \
    default: hipLaunchKernelGGL((decode_attn_kernel<DD, GG, 16>), grid, dim3(256), 0, st, a); break;      \
  }
  if (D == 128) {
    if (G == 1) { DEC(128, 1) }
    else if (G == 2) { DEC(128, 2) }
    else if (G == 4) { DEC(128, 4) }
    else if (G == 8) { DEC(128, 8) }
    else return MLS_UNSUPPORTED;
    if (a.nsplit > 1 && !skip_combine)
      hipLaunchKernelGGL(decode_combine_kernel<128>, dim3(B * Hq), dim3(128), 0, st, a, chunk);
  } else if (D == 64) {
    if (G == 1) { DEC(64, 1) }
    else if (G == 4) { DEC(64, 4) }
    else return MLS_UNSUPPORTED;
    if (a.nsplit > 1 && !skip_combine)
      hipLaunchKernelGGL(decode_combine_kernel<64>, dim3(B * Hq), dim3(64), 0, st, a, chunk);
  } else {
    return MLS_UNSUPPORTED;
  }
#undef DEC
  return (int)hipGetLastError();
}

}  // extern "C"

MLS_DEBUG_EXPORT(attention)
