// K8: fused attention on gfx950.
//
// (1) flash_fwd_kernel<D>: prefill / encoder attention, O = softmax(Q K^T * scale + mask) V,
//     never materialising the S x S scores.  BERT: bidirectional + key-padding mask (per-batch
//     valid length), Hq == Hkv, D = 64.  Llama: causal, GQA (Hq / Hkv query heads share a KV
//     head), D = 128.  Q/K/V are read in place from the fused QKV projection output (strided).
//
//     Block = 4 waves = 64 query rows (16 per wave), K/V tiles of 64 keys staged in LDS.
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
  const int* kv_lens;  // [B] valid keys per sequence (nullptr -> S)
  int causal;
  float scale_log2;  // softmax scale * log2(e)
  uint32_t q_bytes, k_bytes, v_bytes;
};

MLS_DEV float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

template <int D>
__global__ __launch_bounds__(256) void flash_fwd_kernel(const AttnArgs a) {
  constexpr int BQ = 64, BKV = 64;
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
  const int L = a.kv_lens ? min(a.kv_lens[b], a.S) : a.S;
  const long tok0 = (long)b * a.S;

  const rsrc_t qr = make_rsrc(a.q, a.q_bytes);
  const rsrc_t kr = make_rsrc(a.k, a.k_bytes);
  const rsrc_t vr = make_rsrc(a.v, a.v_bytes);

  // Q^T fragments (B operand): lane holds Q[q = qw + fr][d = 32kk + 8g .. +7]
  bf16x8 qf[KK];
  {
    const int q = qw + fr;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const int off = q < a.S ? (int)(((tok0 + q) * a.q_stride + (long)h * D + 32 * kk + 8 * g) * 2) : OOB;
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

  for (int kt = 0; kt < ntiles; ++kt) {
    const int kv0 = kt * BKV;
    // ---- stage K and V tiles (zero rows past L via OOB loads) ----
#pragma unroll
    for (int i = 0; i < (BKV * CPR) / 256; ++i) {
      const int idx = tid + 256 * i;
      const int row = idx / CPR, ch = idx % CPR;
      const int kv = kv0 + row;
      const bool ok = kv < L;
      const uint4 kvec = bload16(kr, ok ? (int)(((tok0 + kv) * a.k_stride + (long)hk * D + ch * 8) * 2) : OOB);
      const uint4 vvec = bload16(vr, ok ? (int)(((tok0 + kv) * a.v_stride + (long)hk * D + ch * 8) * 2) : OOB);
      *reinterpret_cast<uint4*>(Ks + row * (D * 2) + ((ch ^ (row & (CPR - 1))) * 16)) = kvec;
      *reinterpret_cast<uint4*>(Vs + row * VST + ch * 16) = vvec;
    }
    __syncthreads();

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
    mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
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
    ls += __shfl_xor(ls, 16, 64);
    ls += __shfl_xor(ls, 32, 64);
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

  // ---- normalise and store: O rows q = qw + 4g + j, cols d = 16dt + fr ----
  const float inv_l = l_run > 0.f ? 1.f / l_run : 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float il = __shfl(inv_l, 4 * g + j, 64);
    const int q = qw + 4 * g + j;
    if (q < a.S) {
      bf16* dst = a.o + (tok0 + q) * a.o_stride + (long)h * D + fr;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) dst[16 * dt] = (bf16)(acc_o[dt][j] * il);
    }
  }
}

// ------------------------------------------------------------------------------- decode
struct DecodeArgs {
  const bf16* q;   // [B][q_stride], head h at h*D
  const bf16* kc;  // [B][max_len][Hkv][D]
  const bf16* vc;
  bf16* o;         // [B][o_stride]
  float* ws;       // [B][Hq][nsplit][D]
  float* ws_ml;    // [B][Hq][nsplit][2]
  int q_stride, o_stride;
  long seq_stride;  // elements per sequence in the cache (max_len * Hkv * D)
  const int* lens;
  int Hq, Hkv, chunk, nsplit;
  float scale_log2;
};

template <int D, int G>
__global__ __launch_bounds__(256) void decode_split_kernel(const DecodeArgs a) {
  constexpr int LPR = D / 8;      // lanes per key row
  constexpr int RPW = 64 / LPR;   // rows per wave step
  constexpr int NPART = 4 * RPW;  // partial states per block
  __shared__ float sm_m[NPART][G], sm_l[NPART][G];
  __shared__ __attribute__((aligned(16))) float sm_o[NPART][G][D];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int grp = lane / LPR, gl = lane % LPR;
  const int b = blockIdx.z, hk = blockIdx.y, sp = blockIdx.x;
  const int L = a.lens[b];
  const int start = sp * a.chunk, end = min(L, start + a.chunk);

  float qv[G][8];
#pragma unroll
  for (int hh = 0; hh < G; ++hh) unpack8(ld16(a.q + (long)b * a.q_stride + (long)(hk * G + hh) * D + gl * 8), qv[hh]);
  float m[G], l[G], acc[G][8];
#pragma unroll
  for (int hh = 0; hh < G; ++hh) {
    m[hh] = -INFINITY;
    l[hh] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[hh][e] = 0.f;
  }
  const bf16* kbase = a.kc + (long)b * a.seq_stride + (long)hk * D + gl * 8;
  const bf16* vbase = a.vc + (long)b * a.seq_stride + (long)hk * D + gl * 8;
  const long rstride = (long)a.Hkv * D;
  for (int r = start + wid * RPW + grp; r < end; r += 4 * RPW) {
    float kf[8], vf[8];
    unpack8(ld16(kbase + r * rstride), kf);
    unpack8(ld16(vbase + r * rstride), vf);
#pragma unroll
    for (int hh = 0; hh < G; ++hh) {
      float d = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) d += qv[hh][e] * kf[e];
#pragma unroll
      for (int o = LPR / 2; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
      const float sc = d * a.scale_log2;
      const float mn = fmaxf(m[hh], sc);
      const float al = __builtin_amdgcn_exp2f(m[hh] - mn);
      const float p = __builtin_amdgcn_exp2f(sc - mn);
      l[hh] = l[hh] * al + p;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[hh][e] = acc[hh][e] * al + p * vf[e];
      m[hh] = mn;
    }
  }
  const int part = wid * RPW + grp;
#pragma unroll
  for (int hh = 0; hh < G; ++hh) {
    if (gl == 0) {
      sm_m[part][hh] = m[hh];
      sm_l[part][hh] = l[hh];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) sm_o[part][hh][gl * 8 + e] = acc[hh][e];
  }
  __syncthreads();
  for (int idx = tid; idx < G * D; idx += 256) {
    const int hh = idx / D, d = idx % D;
    float M = -INFINITY;
    for (int p = 0; p < NPART; ++p) M = fmaxf(M, sm_m[p][hh]);
    float Ls = 0.f, O = 0.f;
    if (M != -INFINITY) {
      for (int p = 0; p < NPART; ++p) {
        const float w = __builtin_amdgcn_exp2f(sm_m[p][hh] - M);
        Ls += sm_l[p][hh] * w;
        O += sm_o[p][hh][d] * w;
      }
    }
    const long base = (((long)b * a.Hq + hk * G + hh) * a.nsplit + sp);
    a.ws[base * D + d] = O;
    if (d == 0) {
      a.ws_ml[base * 2] = M;
      a.ws_ml[base * 2 + 1] = Ls;
    }
  }
}

template <int D>
__global__ __launch_bounds__(D) void decode_combine_kernel(const DecodeArgs a) {
  const int bh = blockIdx.x;  // b * Hq + h
  const int b = bh / a.Hq, h = bh % a.Hq;
  const int d = threadIdx.x;
  const int ns = min(a.nsplit, (a.lens[b] + a.chunk - 1) / a.chunk);
  float M = -INFINITY;
  for (int s = 0; s < ns; ++s) M = fmaxf(M, a.ws_ml[((long)bh * a.nsplit + s) * 2]);
  float Ls = 0.f, O = 0.f;
  if (M != -INFINITY) {
    for (int s = 0; s < ns; ++s) {
      const long base = (long)bh * a.nsplit + s;
      const float w = __builtin_amdgcn_exp2f(a.ws_ml[base * 2] - M);
      Ls += a.ws_ml[base * 2 + 1] * w;
      O += a.ws[base * D + d] * w;
    }
  }
  a.o[(long)b * a.o_stride + (long)h * D + d] = (bf16)(Ls > 0.f ? O / Ls : 0.f);
}

}  // namespace

extern "C" {

// q/k/v point at the first element of head 0 of token 0; strides are token-row strides.
int mls_flash_attention(const void* q, const void* k, const void* v, void* o, int q_stride, int k_stride,
                        int v_stride, int o_stride, int B, int S, int Hq, int Hkv, int D, const int* kv_lens,
                        int causal, float scale, void* stream) {
  if (B <= 0 || S <= 0 || Hq <= 0 || Hkv <= 0 || Hq % Hkv) return MLS_BAD_ARG;
  if (q_stride % 8 || k_stride % 8 || v_stride % 8) return MLS_BAD_ARG;
  AttnArgs a{};
  a.q = (const bf16*)q;
  a.k = (const bf16*)k;
  a.v = (const bf16*)v;
  a.o = (bf16*)o;
  a.q_stride = q_stride; a.k_stride = k_stride; a.v_stride = v_stride; a.o_stride = o_stride;
  a.B = B; a.S = S; a.Hq = Hq; a.Hkv = Hkv;
  a.kv_lens = kv_lens;
  a.causal = causal;
  a.scale_log2 = scale * 1.4426950408889634f;
  const long T = (long)B * S;
  const size_t qb = ((size_t)(T - 1) * q_stride + (size_t)Hq * D) * 2;
  const size_t kb = ((size_t)(T - 1) * k_stride + (size_t)Hkv * D) * 2;
  const size_t vb = ((size_t)(T - 1) * v_stride + (size_t)Hkv * D) * 2;
  if (qb >= 0x7FFFFFFFull || kb >= 0x7FFFFFFFull || vb >= 0x7FFFFFFFull) return MLS_UNSUPPORTED;
  a.q_bytes = (uint32_t)qb; a.k_bytes = (uint32_t)kb; a.v_bytes = (uint32_t)vb;
  dim3 grid((S + 63) / 64, Hq, B);
  if (D == 64)
    hipLaunchKernelGGL(flash_fwd_kernel<64>, grid, dim3(256), 0, (hipStream_t)stream, a);
  else if (D == 128)
    hipLaunchKernelGGL(flash_fwd_kernel<128>, grid, dim3(256), 0, (hipStream_t)stream, a);
  else
    return MLS_UNSUPPORTED;
  return (int)hipGetLastError();
}

// workspace: ws >= B*Hq*nsplit*D floats, ws_ml >= B*Hq*nsplit*2 floats; nsplit = ceil(max_len/chunk)
int mls_decode_attention(const void* q, const void* k_cache, const void* v_cache, void* o, float* ws, float* ws_ml,
                         int q_stride, int o_stride, long seq_stride, const int* lens, int B, int Hq, int Hkv, int D,
                         int max_len, int chunk, float scale, void* stream) {
  if (B <= 0 || Hq % Hkv || chunk <= 0 || max_len <= 0) return MLS_BAD_ARG;
  DecodeArgs a{};
  a.q = (const bf16*)q;
  a.kc = (const bf16*)k_cache;
  a.vc = (const bf16*)v_cache;
  a.o = (bf16*)o;
  a.ws = ws;
  a.ws_ml = ws_ml;
  a.q_stride = q_stride;
  a.o_stride = o_stride;
  a.seq_stride = seq_stride;
  a.lens = lens;
  a.Hq = Hq;
  a.Hkv = Hkv;
  a.chunk = chunk;
  a.nsplit = (max_len + chunk - 1) / chunk;
  a.scale_log2 = scale * 1.4426950408889634f;
  const int G = Hq / Hkv;
  dim3 grid(a.nsplit, Hkv, B);
  hipStream_t st = (hipStream_t)stream;
#define DEC(DD, GG) hipLaunchKernelGGL((decode_split_kernel<DD, GG>), grid, dim3(256), 0, st, a)
  if (D == 128) {
    if (G == 1) DEC(128, 1);
    else if (G == 2) DEC(128, 2);
    else if (G == 4) DEC(128, 4);
    else if (G == 8) DEC(128, 8);
    else return MLS_UNSUPPORTED;
    hipLaunchKernelGGL(decode_combine_kernel<128>, dim3(B * Hq), dim3(128), 0, st, a);
  } else if (D == 64) {
    if (G == 1) DEC(64, 1);
    else if (G == 4) DEC(64, 4);
    else return MLS_UNSUPPORTED;
    hipLaunchKernelGGL(decode_combine_kernel<64>, dim3(B * Hq), dim3(64), 0, st, a);
  } else {
    return MLS_UNSUPPORTED;
  }
#undef DEC
  return (int)hipGetLastError();
}

}  // extern "C"
