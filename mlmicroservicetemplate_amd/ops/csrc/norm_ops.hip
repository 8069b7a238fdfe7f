// K4 LayerNorm (+fused residual add), K5 RMSNorm (+fused residual add), K10 embedding gathers
// (BERT word+position+type fused with the embedding LayerNorm; Llama vocab-parallel rows that
// zero out-of-shard ids before the TP all-reduce), K9 RoPE (in place on the Q/K heads of the
// fused QKV buffer) and K13 KV-cache append.
//
// Row kernels: one wave64 per row, 16-B (8 x bf16) vector accesses, the row held in registers
// (<= CPL chunks per lane), fp32 statistics via wave shuffles; 4 rows per 256-thread block.
#include "common.h"

namespace {

constexpr int ROWS_PER_BLOCK = 4;

template <int CPL>  // 16-B chunks per lane: D <= 64 * 8 * CPL
__global__ __launch_bounds__(256) void layernorm_kernel(const bf16* __restrict__ x, const bf16* __restrict__ res,
                                                        const bf16* __restrict__ gamma, const bf16* __restrict__ beta,
                                                        bf16* __restrict__ out, bf16* __restrict__ res_out, long rows,
                                                        int D, float eps, int rms) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nch = D >> 3;
  float v[CPL][8];
  // Every load of the row is issued before any is consumed, at clamped (always valid) chunk
  // offsets; the tail lanes' values are dropped below.  With the loads behind per-chunk
  // `ch < nch` guards hipcc waited vmcnt(0) per chunk: 3 dependent round trips per 16-B chunk.
  // gamma / beta go with x up to 8 chunks per lane (register budget), after the statistics above.
  constexpr bool EARLY_GB = CPL <= 8;
  const bf16* xrow = x + row * D;
  const bf16* rrow = res ? res + row * D : xrow;
  const bf16* bsrc = beta ? beta : gamma;
  uint4 xv[CPL], rv[CPL], graw[CPL], braw[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int off = min(lane + 64 * c, nch - 1) * 8;
    xv[c] = ld16(xrow + off);
    rv[c] = ld16(rrow + off);
    if constexpr (EARLY_GB) {
      graw[c] = ld16(gamma + off);
      braw[c] = ld16(bsrc + off);
    }
  }
  float s = 0.f, ss = 0.f;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int ch = lane + 64 * c;
    const bool live = ch < nch;
    // consumed unconditionally (a tail lane works on a clamped duplicate, zeroed below): a use
    // under `live` lets hipcc sink the load into the branch and wait for it there
    unpack8(xv[c], v[c]);
    if (res) {
      float r[8];
      unpack8(rv[c], r);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[c][e] += r[e];
    }
    if (res_out) {
      // the residual stream is carried in bf16; normalise what the next layer will see
      uint4 p = pack8(v[c]);
      if (live) st16(res_out + row * D + ch * 8, p);
      unpack8(p, v[c]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[c][e] = live ? v[c][e] : 0.f;
      s += v[c][e];
      ss += v[c][e] * v[c][e];
    }
  }
  if constexpr (!EARLY_GB) {
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int off = min(lane + 64 * c, nch - 1) * 8;
      graw[c] = ld16(gamma + off);
      braw[c] = ld16(bsrc + off);
    }
  }
  s = wave_sum(s);
  ss = wave_sum(ss);
  const float inv_d = 1.f / (float)D;
  float mean, rstd;
  if (rms) {
    mean = 0.f;
    rstd = rsqrtf(ss * inv_d + eps);
  } else {
    mean = s * inv_d;
    const float var = fmaxf(ss * inv_d - mean * mean, 0.f);
    rstd = rsqrtf(var + eps);
  }
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nch) {
      float g[8], b[8], o[8];
      unpack8(graw[c], g);
      unpack8(braw[c], b);
      if (!beta) {
#pragma unroll
        for (int e = 0; e < 8; ++e) b[e] = 0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (v[c][e] - mean) * rstd * g[e] + b[e];
      st16(out + row * D + ch * 8, pack8(o));
    }
  }
}

// Few long rows (decode-batch RMSNorm of Llama: 32-128 rows of 4096): one 256-thread block per
// row, CPT 16-B chunks per thread, block-wide statistics.  The wave-per-row kernel puts 128 rows
// on 32 CUs with 8 dependent 16-B chunks per lane (11.5 us per call at 128 x 4096).
template <int CPT>
__global__ __launch_bounds__(256) void layernorm_rowblock_kernel(const bf16* __restrict__ x, const bf16* __restrict__ res,
                                                                 const bf16* __restrict__ gamma,
                                                                 const bf16* __restrict__ beta, bf16* __restrict__ out,
                                                                 bf16* __restrict__ res_out, int D, float eps, int rms) {
  __shared__ float red[16];
  const long row = blockIdx.x;
  const int t = threadIdx.x;
  const int nch = D >> 3;
  // all loads issued unconditionally at clamped offsets before any use (as layernorm_kernel: the
  // per-chunk guarded loads made hipcc wait vmcnt(0) per chunk); tail chunks are zeroed below
  const bf16* xrow = x + row * D;
  const bf16* rrow = res ? res + row * D : xrow;
  uint4 xraw[CPT], rraw[CPT], graw[CPT], braw[CPT];
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int off = min(t + 256 * c, nch - 1) * 8;
    xraw[c] = ld16(xrow + off);
    rraw[c] = ld16(rrow + off);
    graw[c] = ld16(gamma + off);
    braw[c] = ld16((beta ? beta : gamma) + off);
  }
  float v[CPT][8];
  float s = 0.f, ss = 0.f;
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int ch = t + 256 * c;
    const bool live = ch < nch;
    unpack8(xraw[c], v[c]);
    if (res) {
      float r[8];
      unpack8(rraw[c], r);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[c][e] += r[e];
    }
    if (res_out) {
      const uint4 p = pack8(v[c]);
      if (live) st16(res_out + row * D + ch * 8, p);
      unpack8(p, v[c]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[c][e] = live ? v[c][e] : 0.f;
      s += v[c][e];
      ss += v[c][e] * v[c][e];
    }
  }
  s = block_sum(s, red);
  ss = block_sum(ss, red + 8);
  const float inv_d = 1.f / (float)D;
  float mean, rstd;
  if (rms) {
    mean = 0.f;
    rstd = rsqrtf(ss * inv_d + eps);
  } else {
    mean = s * inv_d;
    rstd = rsqrtf(fmaxf(ss * inv_d - mean * mean, 0.f) + eps);
  }
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int ch = t + 256 * c;
    if (ch < nch) {
      float g[8], b[8], o[8];
      unpack8(graw[c], g);
      unpack8(braw[c], b);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (v[c][e] - mean) * rstd * g[e] + (beta ? b[e] : 0.f);
      st16(out + row * D + ch * 8, pack8(o));
    }
  }
}

// A projection's split-K reduce fused with the residual add + RMSNorm that follows it (Llama-3-8B
// above 24 tokens per step: o_proj -> the gate_up pre-norm, down_proj -> the next qkv pre-norm).  One
// block per row; the same arithmetic as conv_gemm.hip's reduce (fp32 slabs summed in slice order,
// rounded to bf16) followed by layernorm_rowblock_kernel (+ residual, rounded and written back,
// RMS statistics of the rounded row, x * rstd * gamma): one launch instead of two.  Slices past
// `split` read zero through the buffer range check, so all slab loads are in flight together.
template <int CPT, int MAXS>
__global__ __launch_bounds__(256) void splitk_add_rmsnorm_kernel(const float* __restrict__ ws, uint32_t ws_bytes,
                                                                 int split, int M, bf16* __restrict__ res,
                                                                 const bf16* __restrict__ gamma, bf16* __restrict__ out,
                                                                 int D, float eps) {
  __shared__ float red[16];
  const long row = blockIdx.x;
  const int t = threadIdx.x;
  const int nch = D >> 3;
  const rsrc_t wr = make_rsrc(ws, ws_bytes);
  uint4 rraw[CPT], graw[CPT];
  float4 x[MAXS][CPT][2];
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int off = min(t + 256 * c, nch - 1) * 8;
    rraw[c] = ld16(res + row * D + off);
    graw[c] = ld16(gamma + off);
#pragma unroll
    for (int s2 = 0; s2 < MAXS; ++s2) {
      const int b = s2 < split ? (int)((((size_t)s2 * M + row) * D + off) * 4) : OOB;
      x[s2][c][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(wr, b, 0, 0));
      x[s2][c][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(wr, b == OOB ? OOB : b + 16, 0, 0));
    }
  }
  float v[CPT][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int ch = t + 256 * c;
    const bool live = ch < nch;
    float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s2 = 0; s2 < MAXS; ++s2) {
      o[0] += x[s2][c][0].x; o[1] += x[s2][c][0].y; o[2] += x[s2][c][0].z; o[3] += x[s2][c][0].w;
      o[4] += x[s2][c][1].x; o[5] += x[s2][c][1].y; o[6] += x[s2][c][1].z; o[7] += x[s2][c][1].w;
    }
    unpack8(pack8(o), v[c]);  // the projection's bf16 output
    float r[8];
    unpack8(rraw[c], r);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[c][e] += r[e];
    const uint4 p = pack8(v[c]);
    if (live) st16(res + row * D + ch * 8, p);
    unpack8(p, v[c]);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[c][e] = live ? v[c][e] : 0.f;
      ss += v[c][e] * v[c][e];
    }
  }
  ss = block_sum(ss, red + 8);
  const float rstd = rsqrtf(ss * (1.f / (float)D) + eps);
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int ch = t + 256 * c;
    if (ch < nch) {
      float g[8], o[8];
      unpack8(graw[c], g);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (v[c][e] - 0.f) * rstd * g[e] + 0.f;
      st16(out + row * D + ch * 8, pack8(o));
    }
  }
}

// BERT embeddings: out[t] = LN(word[id] + pos[t % S] + type[tt]) ; one wave per token
template <int CPL>
// ids / type_ids: token t of sequence t / S at (t / S) * id_stride + t % S -- contiguous [B][S] with
// id_stride == S, or read in place from the engine's packed request rows [ids | type ids | len]
// (id_stride = 2S + 1): no unpacking copies.  lens_src / lens_out (optional): sequence b's length at
// lens_src[b * id_stride] copied to lens_out[b] (contiguous, for the attention kernel).
__global__ __launch_bounds__(256) void embed_ln_kernel(const int* __restrict__ ids, const int* __restrict__ type_ids,
                                                       const bf16* __restrict__ word, const bf16* __restrict__ pos,
                                                       const bf16* __restrict__ typ, const bf16* __restrict__ gamma,
                                                       const bf16* __restrict__ beta, bf16* __restrict__ out,
                                                       long rows, int S, int D, int vocab, float eps, int id_stride,
                                                       const int* __restrict__ lens_src, int* __restrict__ lens_out) {
  const int lane = threadIdx.x & 63;
  const long t = (long)blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6);
  if (t >= rows) return;
  const long seq = t / S;
  const long at = seq * id_stride + (t - seq * S);
  if (lens_out && lane == 0 && t == seq * S) lens_out[seq] = lens_src[seq * id_stride];
  int id = ids[at];
  id = (id < 0 || id >= vocab) ? 0 : id;
  const int tt = type_ids ? type_ids[at] : 0;
  const int p = (int)(t % S);
  const int nch = D >> 3;
  float v[CPL][8];
  float s = 0.f, ss = 0.f;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nch) {
      float a[8], b[8], d[8];
      unpack8(ld16(word + (long)id * D + ch * 8), a);
      unpack8(ld16(pos + (long)p * D + ch * 8), b);
      unpack8(ld16(typ + (long)tt * D + ch * 8), d);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[c][e] = a[e] + b[e] + d[e];
        s += v[c][e];
        ss += v[c][e] * v[c][e];
      }
    }
  }
  s = wave_sum(s);
  ss = wave_sum(ss);
  const float mean = s / D;
  const float rstd = rsqrtf(fmaxf(ss / D - mean * mean, 0.f) + eps);
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nch) {
      float g[8], b[8], o[8];
      unpack8(ld16(gamma + ch * 8), g);
      unpack8(ld16(beta + ch * 8), b);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (v[c][e] - mean) * rstd * g[e] + b[e];
      st16(out + t * D + ch * 8, pack8(o));
    }
  }
}

// vocab-parallel embedding: rows of ids outside [lo, hi) are zero (summed by the all-reduce)
__global__ __launch_bounds__(256) void embedding_kernel(const int* __restrict__ ids, const bf16* __restrict__ table,
                                                        bf16* __restrict__ out, long rows, int D, int lo, int hi) {
  const int nch = D >> 3;
  const long total = rows * nch;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const long t = q / nch;
    const int ch = (int)(q - t * nch);
    const int id = ids[t];
    uint4 v = make_uint4(0, 0, 0, 0);
    if (id >= lo && id < hi) v = ld16(table + (long)(id - lo) * D + ch * 8);
    st16(out + t * D + ch * 8, v);
  }
}

// Prefill KV-cache row of every token (models/llama.py prefill into continuous-batching slots /
// through the page table; replaces a dozen torch index launches per call): token t = (batch b =
// t / S, position p = pos[t]) -> -1 unless p < lens[b]; slot = slot_ids ? slot_ids[b] : b; paged:
// table[slot][p / page_rows] * page_rows + p % page_rows, plain: slot * max_seq + p.
__global__ __launch_bounds__(256) void prefill_slots_kernel(const int* __restrict__ pos, const int* __restrict__ lens,
                                                            const int* __restrict__ slot_ids,
                                                            const int* __restrict__ table, int table_stride,
                                                            int page_rows, int max_seq, int S, long T,
                                                            int* __restrict__ out) {
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < T; t += (long)gridDim.x * blockDim.x) {
    const int b = (int)(t / S), p = pos[t];
    int row = -1;
    if (p >= 0 && p < lens[b]) {
      const int slot = slot_ids ? slot_ids[b] : b;
      row = table ? table[(long)slot * table_stride + p / page_rows] * page_rows + p % page_rows
                  : slot * max_seq + p;
    }
    out[t] = row;
  }
}

// Last valid token row of each sequence: out[b] = src[b * S + lens[b] - 1] (and the same rows of
// src2 into out2 when given) -- the prefill's hand-off to the LM head.
__global__ __launch_bounds__(256) void last_rows_kernel(const bf16* __restrict__ src, const bf16* __restrict__ src2,
                                                        const int* __restrict__ lens, int B, int S, int D,
                                                        bf16* __restrict__ out, bf16* __restrict__ out2) {
  const int nch = D >> 3;
  const long total = (long)B * nch;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const int b = (int)(q / nch), ch = (int)(q - (long)b * nch);
    const int l = lens[b];
    const long row = (long)b * S + (l >= 1 && l <= S ? l - 1 : S - 1);
    st16(out + (long)b * D + ch * 8, ld16(src + row * D + ch * 8));
    if (src2) st16(out2 + (long)b * D + ch * 8, ld16(src2 + row * D + ch * 8));
  }
}

// Element offset of (cache slot, head, dim chunk) in a KV cache.  hm_rows == 0: row-major
// [slot][Hkv][D]; hm_rows = R > 0: head-major blocks of R rows, [slot / R][Hkv][R][D] -- a
// sequence's (R = max_seq) or a page's (R = page rows) rows of one head are contiguous, so the
// decode-attention block reading one head streams one contiguous run.
MLS_DEV long kv_offset(long slot, int h, int d, int Hkv, int D, int hm_rows) {
  if (hm_rows <= 0) return (slot * Hkv + h) * D + d;
  return (((slot / hm_rows) * Hkv + h) * hm_rows + slot % hm_rows) * D + d;
}

// RoPE + KV-cache append in one pass (decode / prefill): Q and K heads rotated in place, then
// the (rotated) K heads and the V heads of each token copied to cache slot slots[t]; one launch
// instead of two.  Block = one token; threads: (head, pair-quad) for the rotation, then 16-B copies.
__global__ __launch_bounds__(256) void rope_kv_kernel(bf16* __restrict__ qkv, const int* __restrict__ positions,
                                                      const float* __restrict__ cos_t, const float* __restrict__ sin_t,
                                                      int row_stride, int Hq, int Hkv, int D,
                                                      const int* __restrict__ slots, bf16* __restrict__ kc,
                                                      bf16* __restrict__ vc, const int* __restrict__ lens, int S,
                                                      int max_seq, long cache_rows, int max_pos, int hm_rows) {
  const long t = blockIdx.x;
  const int half = D >> 1, quads = half >> 2;
  const int p = positions[t];
  const bool p_ok = p >= 0 && p < max_pos;
  MLS_CHECK(p_ok, 102);
  if (!p_ok) return;  // no RoPE row for this position: leave the token untouched
  bf16* row = qkv + t * row_stride;
  const int nrot = Hq + Hkv;
  for (int q = threadIdx.x; q < nrot * quads; q += blockDim.x) {
    const int h = q / quads, i = (q % quads) * 4;
    bf16* base = row + (long)h * D;
    const bf16x4 a = __builtin_bit_cast(bf16x4, *reinterpret_cast<const uint2*>(base + i));
    const bf16x4 b = __builtin_bit_cast(bf16x4, *reinterpret_cast<const uint2*>(base + half + i));
    const float4 c = *reinterpret_cast<const float4*>(cos_t + (long)p * half + i);
    const float4 sn = *reinterpret_cast<const float4*>(sin_t + (long)p * half + i);
    const float cc[4] = {c.x, c.y, c.z, c.w}, ss[4] = {sn.x, sn.y, sn.z, sn.w};
    bf16x4 oa, ob;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float x0 = (float)a[e], x1 = (float)b[e];
      oa[e] = (bf16)(x0 * cc[e] - x1 * ss[e]);
      ob[e] = (bf16)(x1 * cc[e] + x0 * ss[e]);
    }
    *reinterpret_cast<uint2*>(base + i) = __builtin_bit_cast(uint2, oa);
    *reinterpret_cast<uint2*>(base + half + i) = __builtin_bit_cast(uint2, ob);
  }
  // cache slot: explicit, or derived -- token t is (batch t / S, position p) in a [B][max_seq] cache,
  // written only while p < lens[b] (prefill padding skipped; decode: lens = position + 1)
  int slot = -1;
  if (slots) {
    slot = slots[t];
  } else if (max_seq > 0) {
    const int b = (int)(t / S);
    if (p < max_seq && (!lens || p < lens[b])) slot = b * max_seq + p;
  }
  if (slot < 0 || !kc) return;
  MLS_CHECK(slot < cache_rows, 101);
  if (slot >= cache_rows) return;
  __syncthreads();  // rotated K visible to the copy below (LDS-free: same block, global memory)
  __threadfence_block();
  const int nch = (Hkv * D) >> 3, hch = D >> 3;
  for (int q = threadIdx.x; q < 2 * nch; q += blockDim.x) {
    const int which = q / nch, ch = q % nch;
    const bf16* src = row + (long)(Hq + which * Hkv) * D + ch * 8;
    bf16* dst = (which ? vc : kc) + kv_offset(slot, ch / hch, (ch % hch) * 8, Hkv, D, hm_rows);
    st16(dst, ld16(src));
  }
}

// RoPE (rotate-half convention) in place on the first n_rot_heads heads of each token row:
// x[i] <- x[i] cos - x[i + D/2] sin ; x[i + D/2] <- x[i + D/2] cos + x[i] sin
// cos/sin table: [max_pos][D/2] fp32.  One thread per (token, head, 4 pairs).
__global__ __launch_bounds__(256) void rope_kernel(bf16* __restrict__ qkv, const int* __restrict__ positions,
                                                   const float* __restrict__ cos_t, const float* __restrict__ sin_t,
                                                   long tokens, int row_stride, int n_rot_heads, int D) {
  const int half = D >> 1;
  const int quads = half >> 2;
  const long total = tokens * n_rot_heads * quads;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const int i4 = (int)(q % quads);
    const long th = q / quads;
    const int h = (int)(th % n_rot_heads);
    const long t = th / n_rot_heads;
    const int p = positions[t];
    bf16* base = qkv + t * row_stride + (long)h * D;
    const int i = i4 * 4;
    const uint2 a_raw = *reinterpret_cast<const uint2*>(base + i);
    const uint2 b_raw = *reinterpret_cast<const uint2*>(base + half + i);
    const bf16x4 a = __builtin_bit_cast(bf16x4, a_raw);
    const bf16x4 b = __builtin_bit_cast(bf16x4, b_raw);
    const float4 c = *reinterpret_cast<const float4*>(cos_t + (long)p * half + i);
    const float4 s = *reinterpret_cast<const float4*>(sin_t + (long)p * half + i);
    const float cc[4] = {c.x, c.y, c.z, c.w}, sn[4] = {s.x, s.y, s.z, s.w};
    bf16x4 oa, ob;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float x0 = (float)a[e], x1 = (float)b[e];
      oa[e] = (bf16)(x0 * cc[e] - x1 * sn[e]);
      ob[e] = (bf16)(x1 * cc[e] + x0 * sn[e]);
    }
    *reinterpret_cast<uint2*>(base + i) = __builtin_bit_cast(uint2, oa);
    *reinterpret_cast<uint2*>(base + half + i) = __builtin_bit_cast(uint2, ob);
  }
}

// KV-cache append: cache[slot[t]][h][:] = src[t][col0 + h*D : ...]; k and v in one launch.
// cache layout [num_slots][Hkv][D] (slot = page * page_size + offset, or seq * max_len + pos).
__global__ __launch_bounds__(256) void kv_append_kernel(const bf16* __restrict__ qkv, int row_stride, int k_col,
                                                        int v_col, const int* __restrict__ slots,
                                                        bf16* __restrict__ kc, bf16* __restrict__ vc, long tokens,
                                                        int Hkv, int D, int hm_rows) {
  const int nch = (Hkv * D) >> 3, hch = D >> 3;
  const long total = tokens * nch * 2;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const int which = (int)(q & 1);
    const long r = q >> 1;
    const long t = r / nch;
    const int ch = (int)(r - t * nch);
    const int slot = slots[t];
    if (slot < 0) continue;
    const bf16* src = qkv + t * row_stride + (which ? v_col : k_col) + ch * 8;
    bf16* dst = (which ? vc : kc) + kv_offset(slot, ch / hch, (ch % hch) * 8, Hkv, D, hm_rows);
    st16(dst, ld16(src));
  }
}

inline int grid_for(long work, int block) {
  long g = (work + block - 1) / block;
  return (int)(g > 4096 ? 4096 : (g < 1 ? 1 : g));
}

}  // namespace

extern "C" {

int mls_layernorm(const void* x, const void* res, const void* gamma, const void* beta, void* out, void* res_out,
                  long rows, int D, float eps, int rms, void* stream) {
  if (D % 8 || D > 64 * 8 * 16 || rows <= 0) return MLS_BAD_ARG;
  const int cpl = (D / 8 + 63) / 64;
  hipStream_t st = (hipStream_t)stream;
  if (rows < 1024 && D >= 2048) {  // too few rows to fill the chip a wave per row
    const int cpt = (D / 8 + 255) / 256;
#define LNB_LAUNCH(C)                                                                                          \
  hipLaunchKernelGGL(layernorm_rowblock_kernel<C>, dim3((unsigned)rows), dim3(256), 0, st, (const bf16*)x,     \
                     (const bf16*)res, (const bf16*)gamma, (const bf16*)beta, (bf16*)out, (bf16*)res_out, D, eps, rms)
    if (cpt <= 2) LNB_LAUNCH(2);
    else if (cpt <= 4) LNB_LAUNCH(4);
    else LNB_LAUNCH(8);
#undef LNB_LAUNCH
    return (int)hipGetLastError();
  }
  dim3 grid((unsigned)((rows + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK));
#define LN_LAUNCH(C)                                                                                           \
  hipLaunchKernelGGL(layernorm_kernel<C>, grid, dim3(256), 0, st, (const bf16*)x, (const bf16*)res,           \
                     (const bf16*)gamma, (const bf16*)beta, (bf16*)out, (bf16*)res_out, rows, D, eps, rms)
  if (cpl <= 1) LN_LAUNCH(1);
  else if (cpl <= 2) LN_LAUNCH(2);
  else if (cpl <= 4) LN_LAUNCH(4);
  else if (cpl <= 8) LN_LAUNCH(8);
  else LN_LAUNCH(16);
#undef LN_LAUNCH
  return (int)hipGetLastError();
}

int mls_embed_ln2(const int* ids, const int* type_ids, int id_stride, const int* lens_src, int* lens_out,
                  const void* word, const void* pos, const void* typ, const void* gamma, const void* beta, void* out,
                  long rows, int S, int D, int vocab, float eps, void* stream) {
  if (D % 8 || D > 64 * 8 * 4 || rows <= 0 || S <= 0 || id_stride < S || (lens_out && !lens_src) || rows % S)
    return MLS_BAD_ARG;
  const int cpl = (D / 8 + 63) / 64;
  dim3 grid((unsigned)((rows + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK));
  hipStream_t st = (hipStream_t)stream;
#define EL_LAUNCH(C)                                                                                                 \
  hipLaunchKernelGGL(embed_ln_kernel<C>, grid, dim3(256), 0, st, ids, type_ids, (const bf16*)word, (const bf16*)pos, \
                     (const bf16*)typ, (const bf16*)gamma, (const bf16*)beta, (bf16*)out, rows, S, D, vocab, eps, \
                     id_stride, lens_src, lens_out)
  if (cpl <= 1) EL_LAUNCH(1);
  else if (cpl <= 2) EL_LAUNCH(2);
  else EL_LAUNCH(4);
#undef EL_LAUNCH
  return (int)hipGetLastError();
}

int mls_embed_ln(const int* ids, const int* type_ids, const void* word, const void* pos, const void* typ,
                 const void* gamma, const void* beta, void* out, long rows, int S, int D, int vocab, float eps,
                 void* stream) {
  if (S <= 0 || rows % S) {  // a partial last sequence: contiguous ids, plain t % S positions
    if (D % 8 || D > 64 * 8 * 4 || rows <= 0 || S <= 0) return MLS_BAD_ARG;
    const long full = rows / S * S;
    if (full) {
      const int rc = mls_embed_ln2(ids, type_ids, S, nullptr, nullptr, word, pos, typ, gamma, beta, out, full, S, D,
                                   vocab, eps, stream);
      if (rc) return rc;
    }
    return mls_embed_ln2(ids + full, type_ids ? type_ids + full : nullptr, (int)(rows - full), nullptr, nullptr, word,
                         pos, typ, gamma, beta, (bf16*)out + full * D, rows - full, (int)(rows - full), D, vocab, eps,
                         stream);
  }
  return mls_embed_ln2(ids, type_ids, S, nullptr, nullptr, word, pos, typ, gamma, beta, out, rows, S, D, vocab, eps,
                       stream);
}

int mls_embedding(const int* ids, const void* table, void* out, long rows, int D, int lo, int hi, void* stream) {
  if (D % 8 || rows <= 0) return MLS_BAD_ARG;
  hipLaunchKernelGGL(embedding_kernel, dim3(grid_for(rows * (D / 8), 256)), dim3(256), 0, (hipStream_t)stream, ids,
                     (const bf16*)table, (bf16*)out, rows, D, lo, hi);
  return (int)hipGetLastError();
}

int mls_prefill_slots(const int* pos, const int* lens, const int* slot_ids, const int* table, int table_stride,
                      int page_rows, int max_seq, int B, int S, int* out, void* stream) {
  if (B <= 0 || S <= 0 || (table && (page_rows <= 0 || table_stride <= 0)) || (!table && max_seq <= 0))
    return MLS_BAD_ARG;
  const long T = (long)B * S;
  hipLaunchKernelGGL(prefill_slots_kernel, dim3(grid_for(T, 256)), dim3(256), 0, (hipStream_t)stream, pos, lens,
                     slot_ids, table, table_stride, page_rows, max_seq, S, T, out);
  return (int)hipGetLastError();
}

int mls_last_rows(const void* src, const void* src2, const int* lens, int B, int S, int D, void* out, void* out2,
                  void* stream) {
  if (B <= 0 || S <= 0 || D % 8 || (src2 && !out2)) return MLS_BAD_ARG;
  hipLaunchKernelGGL(last_rows_kernel, dim3(grid_for((long)B * (D / 8), 256)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)src, (const bf16*)src2, lens, B, S, D, (bf16*)out, (bf16*)out2);
  return (int)hipGetLastError();
}

int mls_rope(void* qkv, const int* positions, const float* cos_t, const float* sin_t, long tokens, int row_stride,
             int n_rot_heads, int D, void* stream) {
  if (D % 8 || tokens <= 0) return MLS_BAD_ARG;
  const long work = tokens * n_rot_heads * (D / 8);
  hipLaunchKernelGGL(rope_kernel, dim3(grid_for(work, 256)), dim3(256), 0, (hipStream_t)stream, (bf16*)qkv,
                     positions, cos_t, sin_t, tokens, row_stride, n_rot_heads, D);
  return (int)hipGetLastError();
}

int mls_rope_kv(void* qkv, const int* positions, const float* cos_t, const float* sin_t, long tokens, int row_stride,
                int Hq, int Hkv, int D, const int* slots, void* k_cache, void* v_cache, const int* lens, int S,
                int max_seq, long cache_rows, int max_pos, int hm_rows, void* stream) {
  if (D % 8 || tokens <= 0 || row_stride % 8 || (!slots && max_seq > 0 && S <= 0)) return MLS_BAD_ARG;
  if (hm_rows > 0 && cache_rows % hm_rows) return MLS_BAD_ARG;
  hipLaunchKernelGGL(rope_kv_kernel, dim3((unsigned)tokens), dim3(256), 0, (hipStream_t)stream, (bf16*)qkv, positions,
                     cos_t, sin_t, row_stride, Hq, Hkv, D, slots, (bf16*)k_cache, (bf16*)v_cache, lens, S, max_seq,
                     cache_rows, max_pos, hm_rows);
  return (int)hipGetLastError();
}

int mls_kv_append(const void* qkv, int row_stride, int k_col, int v_col, const int* slots, void* k_cache,
                  void* v_cache, long tokens, int Hkv, int D, int hm_rows, void* stream) {
  if ((Hkv * D) % 8 || D % 8 || tokens <= 0 || k_col % 8 || v_col % 8 || row_stride % 8) return MLS_BAD_ARG;
  const long work = tokens * (Hkv * D / 8) * 2;
  hipLaunchKernelGGL(kv_append_kernel, dim3(grid_for(work, 256)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)qkv, row_stride, k_col, v_col, slots, (bf16*)k_cache, (bf16*)v_cache, tokens, Hkv,
                     D, hm_rows);
  return (int)hipGetLastError();
}


// ws: split-K fp32 slabs [split][M][D] (conv_gemm.hip mls_gemm_slabs), split 1..8; res [M][D] bf16 is
// updated in place (res += the reduced projection, rounded to bf16); out [M][D] = RMSNorm(res) * gamma.
int mls_splitk_add_rmsnorm(const float* ws, size_t ws_bytes, int split, int M, int D, void* res, const void* gamma,
                           void* out, float eps, void* stream) {
  if (!ws || !res || !gamma || !out || M <= 0 || D <= 0 || D % 8 || D > 256 * 8 * 2 || split < 1 || split > 8 ||
      ws_bytes < (size_t)split * M * D * 4 || (size_t)split * M * D * 4 >= 0x7FFFFFF0ull)
    return MLS_BAD_ARG;
  const uint32_t wb = (uint32_t)((size_t)split * M * D * 4);
  hipStream_t st = (hipStream_t)stream;
#define SRN_LAUNCH(C, S)                                                                                       \
  hipLaunchKernelGGL((splitk_add_rmsnorm_kernel<C, S>), dim3((unsigned)M), dim3(256), 0, st, ws, wb, split, M, \
                     (bf16*)res, (const bf16*)gamma, (bf16*)out, D, eps)
  const bool one = D / 8 <= 256;
  if (split <= 4) {
    if (one) SRN_LAUNCH(1, 4); else SRN_LAUNCH(2, 4);
  } else {
    if (one) SRN_LAUNCH(1, 8); else SRN_LAUNCH(2, 8);
  }
#undef SRN_LAUNCH
  return (int)hipGetLastError();
}

}  // extern "C"

MLS_DEBUG_EXPORT(norm_ops)
