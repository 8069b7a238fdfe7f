// K2 of SURVEY.md §2.E.1 for large M: the transformer projection GEMM on gfx950 MFMA,
//     out[M][N] = act(A[M][K] . W[N][K]^T + bias[N]) (+ residual[M][N])
// (BERT QKV / O / FFN at T = B*S tokens, Llama prefill QKV / O / gate_up / down / lm_head).  This is
// the kernel that replaces the hipBLASLt call ops.linear used to make for M >= 33.
//
// Design (cdna_hip_programming.md §5, "glds vs register staging" and "Pipelining across barriers"):
//  * both operands are K-contiguous (activations [M][K], weights [N][K]), so every MFMA fragment is
//    one 16-B ds_read_b128 of 8 consecutive k from a 128-B LDS row (BK = 64);
//  * operands reach LDS by LDS-DMA (buffer_load ... lds, 16 B per lane): no VGPR staging, no
//    ds_write pass; the LDS image is lane-linear, so the bank swizzle is applied on the SOURCE
//    address and the same involution on the read (rule 21): 16-B chunk c of row r lives at chunk
//    c ^ ((r >> 1) & 7), conflict-free for the gfx950 ds_read_b128 lane groups over the 16 rows of
//    a fragment read (checked against the 4 x 16-lane group table);
//  * a STAGES-deep ring (2 for the 256 x 256 tile = 128 KB, 3 for the smaller tiles): stage t + S - 1
//    is issued right after the barrier that retires stage t, one barrier per K-step, counted
//    `s_waitcnt vmcnt(N)` (never 0 in steady state) and a raw s_barrier, so the DMA of the next
//    stages stays in flight across the barrier while the MFMAs of this one run;
//  * swapped product: the MFMA computes D = W_tile . A_tile^T, so each lane's 4 accumulators are 4
//    consecutive OUTPUT COLUMNS of one row -> 8-B bias / residual loads and output stores per lane,
//    and the SiLU-mul pairing (gate / up interleaved in groups of 8 columns) is one lane^32 swap;
//  * XCD-aware bijective block remap, tiles ordered N-fastest inside an XCD so the blocks sharing
//    an A panel (and the whole, L2-sized weight matrix of a BERT projection) share one L2;
//  * rows past M read as zero through the buffer range check (offset OOB) and are never stored.
#include "common.h"

namespace {

constexpr int GBK = 64;
#define GLDS3 __attribute__((address_space(3)))

struct GemmTileArgs {
  const bf16* a;
  const bf16* w;
  const float* bias;  // [N] or nullptr
  const bf16* res;    // [M][ldr] or nullptr
  bf16* out;          // [M][ldo]
  int M, N, K, act, ldo, ldr;
  uint32_t a_bytes, w_bytes;
  int tiles_n;
  int flags;  // probe-only ablations (GT_ABL_*), 0 in every real call
  int splitk;  // K splits per output tile (>= 1); > 1: fp32 slabs in ws + per-tile arrival counters
  float* ws;   // [tiles][splitk][BM * BN] fp32 partial tiles (fragment-linear)
  int* cnt;    // [tiles] arrival counters: zero before the launch, reset to zero by each tile's reducer
  // LayerNorm folding (see "LayerNorm folding" below)
  const float* fold_c;    // EPI 4: [N] sum_k W'[n][k] of the gamma-folded weight
  const float* ln_part;   // EPI 3 / 4: [M][P][2] row partials (sum, sum of squares) of the LN'd operand,
                          // P = its width / 128 (as a PART epilogue wrote them)
  const float* ln_g;      // EPI 3: [N] fp32 gamma of the residual's LN (its beta is folded into bias)
  float* stats_part;      // PART: [M][N / 128][2] partials of the OUTPUT rows, one per 128-column block
                          // (its two 64-column waves combined through LDS): M * N / 64 floats
  float eps;
};
// ablation flags (tools/gemm_tile_probe.py --ablate; cfg bits 8+ of mls_gemm_tile): timing-only builds
// of the same instruction stream (cdna_hip_programming.md §7, "price ONE buffer's traffic")
constexpr int GT_ABL_NOLOAD = 1;   // zero-record A / W descriptors: every DMA dropped by the range check
constexpr int GT_ABL_NOSTORE = 2;  // epilogue stores land on a zero-record descriptor (dropped)
constexpr int GT_ABL_NOBIAS = 4;   // epilogue skips the bias loads

MLS_DEV void gt_glds16(rsrc_t r, char* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (GLDS3 void*)lds, 16, voff, soff, 0, 0);
}

template <int N>
MLS_DEV void gt_wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt field");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

MLS_DEV void gt_barrier() {
  // LDS-only wait + raw barrier: __syncthreads() would also wait vmcnt(0) and drain the ring
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// 16-B chunk swizzle of an LDS row: BK = 64 (128-B rows, 8 chunks): chunk ^ ((r >> 1) & 7); BK = 32
// (64-B rows, 4 chunks): chunk ^ ((r & 1) | ((r >> 1) & 2)).  Both make the 16-row fragment reads
// conflict-free for the four gfx950 ds_read_b128 lane groups.
template <int BKS>
MLS_DEV int gt_swz(int row) {
  if constexpr (BKS == 64) return (row >> 1) & 7;
  else return (row & 1) | ((row >> 1) & 2);
}

// Logical tile t -> (tm, tn) in GROUP_M-row bands walked column by column: t = band * (GM * tiles_n)
// + tn * gm + (tm - band * GM).  A persistent round hands each XCD 32 consecutive t = a 4 x 8 block
// of tiles (4 A panels + 8 W panels live in that XCD's L2 instead of 1 + 32 for a row-major walk:
// profiles/r3_gemm_tile_pmc.txt measured the row-major order at a 50 % L2 hit rate, 2.7x the HBM
// bytes of hipBLASLt on the same 256 x 256 tile).
constexpr int GT_GROUP_M = 4;
MLS_DEV void gt_tile(int t, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int per_band = GT_GROUP_M * tiles_n;
  const int band = t / per_band, first = band * GT_GROUP_M;
  const int gm = tiles_m - first < GT_GROUP_M ? tiles_m - first : GT_GROUP_M;
  const int r = t - band * per_band;
  tn = r / gm;
  tm = first + (r - tn * gm);
}

// wait until at most N of this wave's DMA groups are outstanding, N = LOADS * min(S - 2, left)
template <int STAGES, int LOADS>
MLS_DEV void gt_wait_ring(int left) {
  if constexpr (STAGES == 2) {
    gt_wait_vmcnt<0>();
  } else if constexpr (STAGES == 3) {
    if (left >= 1) gt_wait_vmcnt<LOADS>();
    else gt_wait_vmcnt<0>();
  } else {
    static_assert(STAGES == 4, "ring depth");
    if (left >= 2) gt_wait_vmcnt<2 * LOADS>();
    else if (left == 1) gt_wait_vmcnt<LOADS>();
    else gt_wait_vmcnt<0>();
  }
}

// Tile epilogue shared by every variant: lane (fr, fq) holds D[n = 4*fq + e][m = fr] of each 16 x 16
// MFMA tile = row m, 4 consecutive output columns.  Written so no memory op sits behind a per-element
// branch (cdna_hip_programming.md §5 item 4(c): hipcc would wait vmcnt(0) per element -- one
// dependent L2 round trip per (i, jn), ~32 per tile, measured as ~15 us of a 40 us BERT GEMM):
//  * bias: 16 values per 16-column tile, uniform per wave -> scalar loads (constant address space),
//    the lane picks its 4 -- no VMEM op, so no vmcnt wait that would drain the DMA ring;
//  * residual: range-checked buffer loads (OOB -> 0) issued as one batch of MT per column tile;
//  * stores: range-checked buffer stores (rows >= M and columns >= N land on the OOB offset).
#define GCONST4 __attribute__((address_space(4)))
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
// EPI: 0 bias (+ act), 1 bias + residual (+ act), 2 SiLU-mul.  One specialisation per kind so the
// unrolled (i, pair) body is straight-line code: a runtime act / residual / SiLU branch inside it made
// hipcc re-home all 128 accumulator registers at every join (~500 instructions per store, measured
// by in-kernel stamps at 31-60k cycles per 256 x 256 tile epilogue).
// 16-B stores (T21, on the 16x16 fragment): v_permlane16_swap over the column tiles (2p, 2p + 1)
// gives each lane 8 consecutive columns of its row -- fq 0: tile 2p cols 0-7, fq 1: tile 2p+1 cols
// 0-7, fq 2: tile 2p cols 8-15, fq 3: tile 2p+1 cols 8-15 -- so a wave stores 16 rows x 64 B per
// instruction: half the store instructions of the bf16x4-per-lane layout (the tail is store-ISSUE
// bound: MI355X_MICROARCH.md, 'attention epilogue store tail').  Bias and residual are loaded in
// the same layout (16-B range-checked buffer loads, OOB -> 0).
// Row statistics of this lane's MT epilogue rows from the [M][P][2] partials a PART epilogue wrote
// (P = width / 128 <= 8 partials per row, 128 columns each, P even): lane fq loads partials 2fq and 2fq + 1
// with one 16-B load (issued first, beside the bias loads), then two lane swaps finish the row in a
// fixed order -- deterministic.  gt_row_stats_finish returns rmu = -mu * rstd and rrs = rstd.
template <int MT>
MLS_DEV void gt_row_stats_issue(const float* part, int width, int m0, int rows, int wrow, uint4 (&t)[MT]) {
  const int lane = threadIdx.x & 63, fr = lane & 15, fq = lane >> 4;
  const int P = width >> 7;
  const rsrc_t rp = make_rsrc(part + (size_t)m0 * P * 2, (uint32_t)(rows * P * 8));
#pragma unroll
  for (int i = 0; i < MT; ++i) t[i] = bload16(rp, 2 * fq < P ? ((wrow + i * 16 + fr) * P + 2 * fq) * 8 : OOB);
}
template <int MT>
MLS_DEV void gt_row_stats_finish(const uint4 (&t)[MT], int width, float eps, float (&rmu)[MT], float (&rrs)[MT]) {
  const float invn = 1.f / (float)width;
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    float s1 = __uint_as_float(t[i].x) + __uint_as_float(t[i].z);
    float s2 = __uint_as_float(t[i].y) + __uint_as_float(t[i].w);
    s1 += xor16_f(s1);
    s2 += xor16_f(s2);
    s1 += xor32_f(s1);
    s2 += xor32_f(s2);
    const float mu = s1 * invn;
    const float r = rsqrtf(fmaxf(s2 * invn - mu * mu, 0.f) + eps);
    rrs[i] = r;
    rmu[i] = -mu * r;
  }
}

// EPI 3: bias + LayerNorm(residual) (row statistics from g.ln_part, fp32 gamma per column; the LN's
// beta is folded into the bias by the caller);
// EPI 4: LN-folded A: rstd * (acc - mu * fold_c) + bias (+ act), A-row statistics from g.ln_part.
// PART: also accumulate each output row's sum / sum of squares over this wave's columns (of the bf16
// values stored); the two waves of each 128-column block combine theirs through LDS (pscr: [WN][BM]
// float2 past the ring, one block barrier) and one thread per (row, block) stores the pair to
// g.stats_part.  Every wave of the block runs the same epilogue, so the barrier is uniform.
template <int MT, int NTL, int EPI, int ACT, bool PART = false, int BM = 256, int WN = 4>
MLS_DEV void gt_epilogue_t(f32x4 (&acc)[MT][NTL], const GemmTileArgs& g, int m0, int n0, int wrow, int wcol,
                           float* pscr = nullptr) {
  static_assert(NTL % 2 == 0, "column tiles pair up");
  constexpr bool RES = EPI == 1 || EPI == 3;
  // the LayerNorm forms hold per-row values (stats, partial sums) across the column loop: the 256-row
  // tile (MT = 8) walks its rows in two halves, each re-reading the (L1-resident) column vectors, so
  // the per-row arrays stay at 4 entries (the whole tile at once spilled 8-19 VGPRs)
  constexpr int RH = (EPI >= 3 || PART) && MT >= 8 ? 2 : 1, MH = MT / RH;
  const int lane = threadIdx.x & 63, fr = lane & 15, fq = lane >> 4;
  const int ldo2 = g.ldo * 2, ldr2 = g.ldr * 2;
  const int rows = g.M - m0 < 256 ? g.M - m0 : 256;  // valid rows of this tile (tiles are <= 256 tall)
  const bool nostore = g.flags & GT_ABL_NOSTORE;
  const rsrc_t ro = make_rsrc(g.out + (size_t)m0 * g.ldo, nostore ? 0u : (uint32_t)(rows * ldo2));
  const rsrc_t rr = make_rsrc(RES ? g.res + (size_t)m0 * g.ldr : g.out, RES ? (uint32_t)(rows * ldr2) : 0u);
  const bool use_bias = g.bias && !(g.flags & GT_ABL_NOBIAS);
  const rsrc_t rb = make_rsrc(use_bias ? (const void*)g.bias : (const void*)g.out, use_bias ? (uint32_t)g.N * 4u : 0u);
  const rsrc_t rg = EPI == 3 || EPI == 4 ? make_rsrc(EPI == 3 ? g.ln_g : g.fold_c, (uint32_t)g.N * 4u) : rb;
  const int sub = (fq & 1) * 16 + (fq >> 1) * 8;  // this lane's 8 columns within the 32-column pair
#pragma unroll
  for (int h = 0; h < RH; ++h) {
    const int hrow = wrow + h * MH * 16;  // first row of this half (within the tile)
    // per-row (-mu * rstd, rstd) of this lane's rows (EPI 3 / 4) and partial sums (PART)
    float rmu[MH], rrs[MH], ps1[MH], ps2[MH];
#pragma unroll
    for (int i = 0; i < MH; ++i) ps1[i] = ps2[i] = 0.f;
    constexpr bool STATS = EPI == 3 || EPI == 4;
    const int lnw = EPI == 3 ? g.N : g.K;  // the LN'd rows' width: the residual's (N) or A's (K)
    uint4 st[MH];
    if constexpr (STATS) gt_row_stats_issue<MH>(g.ln_part, lnw, m0, rows, hrow, st);
#pragma unroll
    for (int p = 0; p < NTL / 2; ++p) {
      const int c0 = n0 + wcol + p * 32, c = c0 + sub;
      const bool col_ok = c < g.N;  // N % 16 == 0: an 8-column run is wholly in or out
      const f32x4 b_lo = __builtin_bit_cast(f32x4, bload16(rb, col_ok ? c * 4 : OOB));
      const f32x4 b_hi = __builtin_bit_cast(f32x4, bload16(rb, col_ok ? c * 4 + 16 : OOB));
      f32x4 g_lo = {0.f, 0.f, 0.f, 0.f}, g_hi = g_lo;
      if constexpr (STATS) {
        g_lo = __builtin_bit_cast(f32x4, bload16(rg, col_ok ? c * 4 : OOB));
        g_hi = __builtin_bit_cast(f32x4, bload16(rg, col_ok ? c * 4 + 16 : OOB));
        if (p == 0) gt_row_stats_finish<MH>(st, lnw, g.eps, rmu, rrs);  // its loads flew beside the bias
      }
      // residual rows two 16-row blocks ahead (a whole column of them live would cost 32 VGPRs and
      // spill the 256 x 256 tile)
      const int roff = col_ok ? (hrow + fr) * ldr2 + c * 2 : OOB;
      uint4 rv0 = {0, 0, 0, 0}, rv1 = {0, 0, 0, 0};
      if constexpr (RES) {
        rv0 = bload16(rr, roff);
        if (MH > 1) rv1 = bload16(rr, col_ok ? roff + 16 * ldr2 : OOB);
      }
#pragma unroll
      for (int i = 0; i < MH; ++i) {
        const int ia = h * MH + i;        // accumulator row block
        const int r = hrow + i * 16 + fr;  // row within the tile
        uint4 rcur = rv0;
        if constexpr (RES) {
          rv0 = rv1;
          if (i + 2 < MH) rv1 = bload16(rr, col_ok ? roff + (i + 2) * 16 * ldr2 : OOB);
        }
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          // __float_as_uint, not __builtin_bit_cast: hipcc (ROCm 7.2) folds a bit_cast of an ext-vector
          // element feeding this builtin to element 0 -- one swap for all four (checked in the .s)
          const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[ia][2 * p][e]),
                                                           __float_as_uint(acc[ia][2 * p + 1][e]), false, false);
          if constexpr (EPI == 4) {  // rstd * (acc - mu * c) + b
            v[e] = fmaf(rrs[i], __uint_as_float(sw[0]), fmaf(rmu[i], g_lo[e], b_lo[e]));
            v[4 + e] = fmaf(rrs[i], __uint_as_float(sw[1]), fmaf(rmu[i], g_hi[e], b_hi[e]));
          } else {
            v[e] = __uint_as_float(sw[0]) + b_lo[e];
            v[4 + e] = __uint_as_float(sw[1]) + b_hi[e];
          }
        }
        bf16x8 o;
        int off;
        if constexpr (EPI == 2) {
          // gate lanes fq 0/1 (tile 2p / 2p+1 cols 0-7) pair with their up columns on lanes fq 2/3
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = (bf16)(silu_fast(v[e]) * xor32_f(v[e]));
          off = fq < 2 && col_ok ? r * ldo2 + ((c0 >> 1) + fq * 8) * 2 : OOB;
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float x = v[e];
            v[e] = ACT == ACT_GELU ? gelu_fast(x) : ACT == ACT_RELU ? fmaxf(x, 0.f) : ACT == ACT_SILU ? silu_fast(x)
                   : ACT == ACT_TANH ? tanhf(x) : x;
          }
          if constexpr (EPI == 1) {
            const bf16x8 rb8 = __builtin_bit_cast(bf16x8, rcur);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += (float)rb8[e];
          } else if constexpr (EPI == 3) {
            const bf16x8 rb8 = __builtin_bit_cast(bf16x8, rcur);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float n = fmaf((float)rb8[e], rrs[i], rmu[i]);  // (r - mu) * rstd
              v[e] = fmaf(n, e < 4 ? g_lo[e] : g_hi[e - 4], v[e]);
            }
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = (bf16)v[e];
          if constexpr (PART) {  // columns >= N read as zero (residual / accumulators) and add nothing
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float q = col_ok ? (float)o[e] : 0.f;
              ps1[i] += q;
              ps2[i] = fmaf(q, q, ps2[i]);
            }
          }
          off = col_ok ? r * ldo2 + c * 2 : OOB;
        }
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), ro, off, 0, 0);
        __builtin_amdgcn_sched_barrier(0);  // keep each row block's live range to itself
      }
    }
    if constexpr (PART) {
      // the 4 lanes fq of a row hold different columns: finish the wave's sums, lanes fq 0 park them
      static_assert(NTL * 16 == 64, "two 64-column waves per 128-column partial");
      const int wn = wcol / 64;
#pragma unroll
      for (int i = 0; i < MH; ++i) {
        float a = ps1[i], b = ps2[i];
        a += xor16_f(a);
        b += xor16_f(b);
        a += xor32_f(a);
        b += xor32_f(b);
        if (fq == 0) {
          float2 v;
          v.x = a;
          v.y = b;
          reinterpret_cast<float2*>(pscr)[wn * BM + hrow + i * 16 + fr] = v;
        }
      }
    }
  }
  if constexpr (PART) {
    // one thread per (row, 128-column block of this tile): add the block's two waves, store the pair
    constexpr int BN = WN * 64, QB = BN / 128;
    static_assert(QB >= 1, "tile covers whole 128-column blocks");
    const int P = g.N >> 7;
    gt_barrier();
    const rsrc_t rp = make_rsrc(g.stats_part + (size_t)m0 * P * 2, (uint32_t)(rows * P * 8));
    for (int t = threadIdx.x; t < BM * QB; t += blockDim.x) {
      const int r = t % BM, q = t / BM;
      const float2 a = reinterpret_cast<const float2*>(pscr)[(2 * q) * BM + r];
      const float2 b = reinterpret_cast<const float2*>(pscr)[(2 * q + 1) * BM + r];
      const u32x2 v = {__float_as_uint(a.x + b.x), __float_as_uint(a.y + b.y)};
      const int part = (n0 >> 7) + q;
      __builtin_amdgcn_raw_buffer_store_b64(v, rp, part < P ? (r * P + part) * 8 : OOB, 0, 0);
    }
  }
}

// The bf16x4-per-lane form of the epilogue (one 8-B store per (i, jn), scalar-loaded bias): kept as
// the A/B arm of the 16-B form (cfg 19 = cfg 1 with it) -- probe only.
template <int MT, int NTL, int EPI, int ACT>
MLS_DEV void gt_epilogue_x2(f32x4 (&acc)[MT][NTL], const GemmTileArgs& g, int m0, int n0, int wrow, int wcol) {
  const int lane = threadIdx.x & 63, fr = lane & 15, fq = lane >> 4;
  const int ldo2 = g.ldo * 2, ldr2 = g.ldr * 2;
  const int rows = g.M - m0 < 256 ? g.M - m0 : 256;
  const bool nostore = g.flags & GT_ABL_NOSTORE;
  const rsrc_t ro = make_rsrc(g.out + (size_t)m0 * g.ldo, nostore ? 0u : (uint32_t)(rows * ldo2));
  const rsrc_t rr = make_rsrc(EPI == 1 ? g.res + (size_t)m0 * g.ldr : g.out, EPI == 1 ? (uint32_t)(rows * ldr2) : 0u);
#pragma unroll
  for (int jn = 0; jn < NTL; ++jn) {
    const int nt0 = n0 + wcol + jn * 16, n = nt0 + 4 * fq;
    const bool col_ok = nt0 < g.N;
    f32x4 bv = {0.f, 0.f, 0.f, 0.f}, bu = {0.f, 0.f, 0.f, 0.f};
    if (g.bias && col_ok && !(g.flags & GT_ABL_NOBIAS)) {
      const GCONST4 f32x4* bp = (const GCONST4 f32x4*)(g.bias + nt0);
      const f32x4 b0 = bp[0], b1 = bp[1], b2 = bp[2], b3 = bp[3];
      bv = fq == 0 ? b0 : fq == 1 ? b1 : fq == 2 ? b2 : b3;
      bu = fq == 0 ? b2 : b3;
    }
    uint2 rv[MT];
    if constexpr (EPI == 1) {
#pragma unroll
      for (int i = 0; i < MT; ++i) rv[i] = bload8(rr, col_ok ? (wrow + i * 16 + fr) * ldr2 + n * 2 : OOB);
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int r = wrow + i * 16 + fr;
      const f32x4 v = acc[i][jn];
      bf16x4 b;
      int off;
      if constexpr (EPI == 2) {
#pragma unroll
        for (int e = 0; e < 4; ++e) b[e] = (bf16)(silu_fast(v[e] + bv[e]) * (xor32_f(v[e]) + bu[e]));
        off = fq < 2 && col_ok ? r * ldo2 + ((nt0 >> 1) + 4 * fq) * 2 : OOB;
      } else {
        f32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float x = v[e] + bv[e];
          o[e] = ACT == ACT_GELU ? gelu_fast(x) : ACT == ACT_RELU ? fmaxf(x, 0.f) : ACT == ACT_SILU ? silu_fast(x)
                 : ACT == ACT_TANH ? tanhf(x) : x;
        }
        if constexpr (EPI == 1) {
          const bf16x4 rb = __builtin_bit_cast(bf16x4, rv[i]);
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] += (float)rb[e];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) b[e] = (bf16)o[e];
        off = col_ok ? r * ldo2 + n * 2 : OOB;
      }
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, b), ro, off, 0, 0);
    }
  }
}

#define GT_EPI_CALL(ACTV)                                                   \
  do {                                                                      \
    if constexpr (X2) gt_epilogue_x2<MT, NTL, EPI, ACTV>(acc, g, m0, n0, wrow, wcol); \
    else gt_epilogue_t<MT, NTL, EPI, ACTV>(acc, g, m0, n0, wrow, wcol);    \
  } while (0)
template <int MT, int NTL, int EPI, bool X2>
MLS_DEV void gt_epilogue_a(f32x4 (&acc)[MT][NTL], const GemmTileArgs& g, int m0, int n0, int wrow, int wcol) {
  switch (g.act) {
    case ACT_GELU: GT_EPI_CALL(ACT_GELU); break;
    case ACT_RELU: GT_EPI_CALL(ACT_RELU); break;
    case ACT_SILU: GT_EPI_CALL(ACT_SILU); break;
    case ACT_TANH: GT_EPI_CALL(ACT_TANH); break;
    default: GT_EPI_CALL(ACT_NONE); break;
  }
}

// dispatch once per tile, then zero the accumulators for the next tile in one straight run.  LN: the
// LayerNorm-folding epilogues (EPI 3 / 4, + row statistics) -- gemm_tile_kernel instantiations only
// LNK 1: the folded projection (EPI 4, act none / gelu); LNK 2: the residual projection (EPI 1 / 3,
// + PART when g.stats_part) -- one instantiation per kind keeps each kernel's register peak to its own
template <int MT, int NTL, int LNK, int BM, int WN>
MLS_DEV void gt_epilogue_ln(f32x4 (&acc)[MT][NTL], const GemmTileArgs& g, int m0, int n0, int wrow, int wcol,
                            float* pscr) {
  if constexpr (LNK == 1) {
    if (g.act == ACT_GELU) gt_epilogue_t<MT, NTL, 4, ACT_GELU>(acc, g, m0, n0, wrow, wcol);
    else gt_epilogue_t<MT, NTL, 4, ACT_NONE>(acc, g, m0, n0, wrow, wcol);
  } else if (g.stats_part) {
    if (g.ln_part) gt_epilogue_t<MT, NTL, 3, ACT_NONE, true, BM, WN>(acc, g, m0, n0, wrow, wcol, pscr);
    else gt_epilogue_t<MT, NTL, 1, ACT_NONE, true, BM, WN>(acc, g, m0, n0, wrow, wcol, pscr);
  } else {
    if (g.ln_part) gt_epilogue_t<MT, NTL, 3, ACT_NONE>(acc, g, m0, n0, wrow, wcol);
    else gt_epilogue_t<MT, NTL, 1, ACT_NONE>(acc, g, m0, n0, wrow, wcol);
  }
}
// LNK != 0: pscr = the LDS scratch past the ring that a PART epilogue combines its waves through
template <int MT, int NTL, bool X2 = false, int LNK = 0, int BM = 256, int WN = 4>
MLS_DEV void gt_epilogue(f32x4 (&acc)[MT][NTL], const GemmTileArgs& g, int m0, int n0, int wrow, int wcol,
                         float* pscr = nullptr) {
  if constexpr (LNK != 0) {
    gt_epilogue_ln<MT, NTL, LNK, BM, WN>(acc, g, m0, n0, wrow, wcol, pscr);
  } else if (g.act == ACT_SILU_MUL) {
    if constexpr (X2) gt_epilogue_x2<MT, NTL, 2, ACT_NONE>(acc, g, m0, n0, wrow, wcol);
    else gt_epilogue_t<MT, NTL, 2, ACT_NONE>(acc, g, m0, n0, wrow, wcol);
  } else if (g.res) {
    gt_epilogue_a<MT, NTL, 1, X2>(acc, g, m0, n0, wrow, wcol);
  } else {
    gt_epilogue_a<MT, NTL, 0, X2>(acc, g, m0, n0, wrow, wcol);
  }
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int jn = 0; jn < NTL; ++jn) acc[i][jn] = f32x4{0.f, 0.f, 0.f, 0.f};
  // retire the epilogue's VMEM ops with the BUILTIN wait (hipcc's waitcnt pass sees it; an asm one it
  // does not): otherwise the pass carries the bias / residual load registers as possibly pending
  // around the k-loop back edge and emits vmcnt(0) before the first ds_read of EVERY k-step --
  // draining the DMA ring each step (+25-40 % k-step cycles, measured by stamps vs the x2 arm)
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
}

// In-launch split-K combine (cdna_hip_programming.md §5 "Projection GEMM", item 2): each K-split
// block writes its fp32 partial tile as a fragment-linear slab (lane-contiguous 16 B, 1 KB per wave
// instruction), retires it, and one lane releases at agent scope and draws a ticket from the tile's
// counter; the split that draws S - 1 is the reducer: acquire, add the other S - 1 slabs into its
// accumulators, reset the counter for the next launch, and run the normal epilogue.  Returns true
// for the reducer; the others return with zeroed accumulators.  Correct for any placement of a
// tile's splits (adjacent units -> same XCD in practice, the fast case).
template <int TILE_ELEMS, int MT, int NTL>
MLS_DEV bool gt_splitk_arrive(f32x4 (&acc)[MT][NTL], const GemmTileArgs& g, int tile, int split, int* flag) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, S = g.splitk;
  f32x4* const tile_ws = reinterpret_cast<f32x4*>(g.ws + (size_t)tile * S * TILE_ELEMS);
  const int frag0 = wid * MT * NTL * 64 + lane;  // this lane's first f32x4 in a slab
  f32x4* mine = tile_ws + (size_t)split * (TILE_ELEMS / 4) + frag0;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int jn = 0; jn < NTL; ++jn) mine[(i * NTL + jn) * 64] = acc[i][jn];
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // every wave: its slab stores (and the ring's DMAs) retired
  gt_barrier();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __builtin_amdgcn_s_waitcnt(0x0F70);
    const int old = __hip_atomic_fetch_add(g.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == S - 1;
    if (last) {
      __hip_atomic_store(g.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __builtin_amdgcn_s_waitcnt(0x0F70);
    }
    *flag = last;
  }
  gt_barrier();
  const bool last = __builtin_amdgcn_readfirstlane(*flag) != 0;
  gt_barrier();  // flag read by every wave before it can be rewritten by this block's next unit
  if (!last) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn) acc[i][jn] = f32x4{0.f, 0.f, 0.f, 0.f};
    return false;
  }
  // sum ALL S slabs (its own re-read too) in split order: the result does not depend on which
  // split arrived last, so repeated launches are bit-identical
  for (int s2 = 0; s2 < S; ++s2) {
    const f32x4* slab = tile_ws + (size_t)s2 * (TILE_ELEMS / 4) + frag0;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      f32x4 t[NTL];
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn) t[jn] = slab[(i * NTL + jn) * 64];
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn) acc[i][jn] = s2 == 0 ? t[jn] : acc[i][jn] + t[jn];
      __builtin_amdgcn_sched_barrier(0);  // NTL loads in flight at a time: the accumulators fill the file
    }
  }
  return true;
}

// In-kernel stamps (cdna_hip_programming.md §7) for the STAMP build of the tile kernel (cfg 13/14 =
// cfg 1/2 + stamps, probe only): s_memtime with its own lgkmcnt wait, fenced by sched_barriers.
MLS_DEV unsigned long long gt_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
MLS_DEV unsigned long long gt_realtime() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

// LayerNorm folding (BERT post-LN: x = LN(h) feeds the next projection AND the residual add after
// it).  No LN kernel runs and x is never formed:
//  * the producer of h (O / FFN-down projection, residual epilogue) stores h and, per output row and
//    128-column block, the sum and sum of squares of the bf16 values it stored (PART: [M][N/128][2],
//    the block's two 64-column waves combined through LDS);
//  * the projection that consumes x reads A = h and W' = W . diag(gamma): x . W^T = rstd * (h . W'^T -
//    mu * c) + beta . W^T with c[n] = sum_k W'[n][k], applied to the accumulator in the epilogue
//    (EPI 4);
//  * the residual add after it normalizes its residual operand in the epilogue: (h - mu) * rstd *
//    gamma + beta (EPI 3);
//  * both consumers finish each row's (mu, rstd) from the partials themselves (gt_row_stats; the
//    loads ride beside the bias loads) -- the kernel boundary orders them after the producer, so no
//    cross-block protocol or extra launch is needed.
// Removes the LN launch and its T x H read + write per LayerNorm.
template <int BM, int BN, int WM, int WN, int STAGES, int BKS, bool STAMP = false, bool PIPE = false, bool X2 = false,
          int LNK = 0>
__global__ __launch_bounds__(WM * WN * 64) void gemm_tile_kernel(const GemmTileArgs g0) {
  static_assert(LNK == 0 || (!STAMP && !X2 && BN / WN == 64), "LayerNorm-folding builds: 64-column wave tiles");
  // STAMP: g0.res is the stamp buffer [grid][8] (u64): t0 start, t1 first k-step landed, t2 first
  // tile's last MFMA, t3 its epilogue issued, t4 all stores retired, t5/t6 realtime at t0/t4, t7 tiles
  unsigned long long st[5] = {0, 0, 0, 0, 0}, rt0 = 0;
  GemmTileArgs g = g0;
  if constexpr (STAMP) {
    g.res = nullptr;
    st[0] = gt_stamp();
    rt0 = gt_realtime();
  }
  constexpr int NT = WM * WN * 64;
  constexpr int WTM = BM / WM, WTN = BN / WN;  // wave tile: WTM rows (m) x WTN columns (n)
  constexpr int MT = WTM / 16, NTL = WTN / 16;
  constexpr int ROWB = BKS * 2, CPR = ROWB / 16;  // bytes / 16-B chunks per LDS row
  constexpr int A_BYTES = BM * ROWB, B_BYTES = BN * ROWB, STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int A_LD = A_BYTES / (NT * 16), B_LD = B_BYTES / (NT * 16), LOADS = A_LD + B_LD;
  static_assert(A_BYTES % (NT * 16) == 0 && B_BYTES % (NT * 16) == 0, "stage must split into whole DMA rounds");
  static_assert(BKS == 32 || BKS == 64, "stage depth");
  // + 16 B: the split-K "last arriver" flag -- in the SAME __shared__ object as the ring (a second
  // one can make hipcc wait vmcnt(0) before every k-step's first ds_read: §5 item 4(a))
  // LNK == 2: [WN][BM] float2 scratch past the ring for the PART epilogue's cross-wave combine
  constexpr int PSCR_BYTES = LNK == 2 ? WN * BM * 8 : 0;
  static_assert(STAGES * STAGE_BYTES + 16 + PSCR_BYTES <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[STAGES * STAGE_BYTES + 16 + PSCR_BYTES];
  float* const pscr = reinterpret_cast<float*>(smem + STAGES * STAGE_BYTES + 16);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid - wm * WN;
  const int tiles_m = (g.M + BM - 1) / BM, ntiles = tiles_m * g.tiles_n;
  // work unit = (tile, K split): unit u -> tile u / S, split u % S (the S splits of a tile are
  // adjacent units, so they land on one XCD and its reducer reads same-XCD slabs).  Persistent:
  // block b takes units b', b' + G, ... where b' = XCD-contiguous remap of b
  const int S = g.splitk, nunits = ntiles * S;
  const int G = gridDim.x, bq = xcd_remap(blockIdx.x, G);
  const int my_tiles = bq < nunits ? (nunits - 1 - bq) / G + 1 : 0;  // units of this block
  const int nk = g.K / BKS / S, nsteps = my_tiles * nk;              // k-steps per unit

  const rsrc_t ra = make_rsrc(g.a, g.a_bytes), rw = make_rsrc(g.w, g.w_bytes);
  // DMA source: LDS byte p = i*NT*16 + tid*16 of a stage image is row p / 128, lane-linear chunk
  // tid & 7 = source chunk (tid & 7) ^ swz(row); the tile row / k-step base rides in soffset
  int a_row[A_LD], a_col[A_LD], w_row[B_LD], w_col[B_LD];
#pragma unroll
  for (int i = 0; i < A_LD; ++i) {
    a_row[i] = (i * NT + tid) / CPR;
    a_col[i] = ((tid % CPR) ^ gt_swz<BKS>(a_row[i])) * 16;
  }
#pragma unroll
  for (int i = 0; i < B_LD; ++i) {
    w_row[i] = (i * NT + tid) / CPR;
    w_col[i] = ((tid % CPR) ^ gt_swz<BKS>(w_row[i])) * 16;
  }
  const int K2 = g.K * 2;

  // unit ui of this block -> tile origin (m0, n0) and its first k-step k0
  auto tile_mn = [&](int ti, int& m0, int& n0, int& k0) {
    const int u = bq + ti * G, t = S == 1 ? u : u / S;
    int tm, tn;
    gt_tile(t, tiles_m, g.tiles_n, tm, tn);
    m0 = tm * BM;
    n0 = tn * BN;
    k0 = (u - t * S) * nk;
  };
  // loader cursor: the (unit, k-step) of the next DMA, advanced without divisions
  int l_ti = 0, l_kt = 0, l_m0 = 0, l_n0 = 0, l_k0 = 0, l_slot = 0;
  if (nsteps > 0) tile_mn(0, l_m0, l_n0, l_k0);
  auto stage = [&]() {  // DMA the loader cursor's k-step into ring slot l_slot, then advance it
    const int kt = l_k0 + l_kt, m0 = l_m0, n0 = l_n0;
    char* base = smem + l_slot * STAGE_BYTES + wid * 1024;
    l_slot = l_slot + 1 == STAGES ? 0 : l_slot + 1;
    if (++l_kt == nk) {
      l_kt = 0;
      if (++l_ti < my_tiles) tile_mn(l_ti, l_m0, l_n0, l_k0);
    }
    const int sa = m0 * K2 + kt * ROWB, sb = n0 * K2 + kt * ROWB;
#pragma unroll
    for (int i = 0; i < A_LD; ++i)
      gt_glds16(ra, base + i * NT * 16, m0 + a_row[i] < g.M ? a_row[i] * K2 + a_col[i] : OOB, sa);
#pragma unroll
    for (int i = 0; i < B_LD; ++i)
      gt_glds16(rw, base + A_BYTES + i * NT * 16, n0 + w_row[i] < g.N ? w_row[i] * K2 + w_col[i] : OOB, sb);
  };

  f32x4 acc[MT][NTL];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTL; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment reads inside a stage image (row r, 16-B chunk c -> r*128 + (c ^ swz(r))*16)
  const int fr = lane & 15, fq = lane >> 4;
  const int sw = gt_swz<BKS>(fr);  // tile rows are 16-aligned: swz(r) depends on r & 15 only
  const int a_rd = (wm * WTM + fr) * ROWB, w_rd = A_BYTES + (wn * WTN + fr) * ROWB;


#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nsteps) stage();

  int c_kt = 0, c_ti = 0, c_slot = 0;  // compute cursor
  for (int j = 0; j < nsteps; ++j) {
    gt_wait_ring<STAGES, LOADS>(nsteps - 1 - j);  // step j landed; later ones may still fly
    gt_barrier();  // step j visible to every wave; step j - 1 fully read by every wave
    if constexpr (STAMP)
      if (j == 0) st[1] = gt_stamp();
    if (j + STAGES - 1 < nsteps) stage();
    const char* base = smem + c_slot * STAGE_BYTES;
    c_slot = c_slot + 1 == STAGES ? 0 : c_slot + 1;
    if constexpr (PIPE && BKS == 64) {
      // fragment pipeline across the two 32-deep halves of the step: the k 32-63 W fragments are
      // read up front, each A fragment of k 32-63 right after the last MFMA that reads its k 0-31
      // register -- the second half's LDS latency hides under the first half's MFMAs instead of
      // stalling both waves of the SIMD after them
      const int coff0 = (fq ^ sw) << 4, coff1 = ((4 + fq) ^ sw) << 4;
      bf16x8 af[MT], w0[NTL], w1[NTL];
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn) w0[jn] = *reinterpret_cast<const bf16x8*>(base + w_rd + jn * 16 * ROWB + coff0);
#pragma unroll
      for (int i = 0; i < MT; ++i) af[i] = *reinterpret_cast<const bf16x8*>(base + a_rd + i * 16 * ROWB + coff0);
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn) w1[jn] = *reinterpret_cast<const bf16x8*>(base + w_rd + jn * 16 * ROWB + coff1);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
#pragma unroll
        for (int jn = 0; jn < NTL; ++jn)
          acc[i][jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0[jn], af[i], acc[i][jn], 0, 0, 0);
        af[i] = *reinterpret_cast<const bf16x8*>(base + a_rd + i * 16 * ROWB + coff1);
      }
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int jn = 0; jn < NTL; ++jn)
          acc[i][jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[jn], af[i], acc[i][jn], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    } else {
#pragma unroll
    for (int ks = 0; ks < BKS / 32; ++ks) {
      const int coff = ((ks * 4 + fq) ^ sw) << 4;
      bf16x8 af[MT], wf[NTL];
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn) wf[jn] = *reinterpret_cast<const bf16x8*>(base + w_rd + jn * 16 * ROWB + coff);
#pragma unroll
      for (int i = 0; i < MT; ++i) af[i] = *reinterpret_cast<const bf16x8*>(base + a_rd + i * 16 * ROWB + coff);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int jn = 0; jn < NTL; ++jn)
          acc[i][jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[jn], af[i], acc[i][jn], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    }
    if (++c_kt < nk) continue;
    c_kt = 0;

    // ---- epilogue of this unit (the next unit's first k-steps are already in flight) ----
    int m0, n0, k0;
    if constexpr (STAMP)
      if (c_ti == 0) st[2] = gt_stamp();
    const int cu = bq + c_ti * G;
    tile_mn(c_ti++, m0, n0, k0);
    // LNK: the LayerNorm-folding epilogues live in their own instantiations (all of them in one
    // kernel cost ~30 VGPRs + ~60 SGPRs kernel-wide and spilled the 256 x 256 tile)
    const bool reducer = S == 1 || gt_splitk_arrive<BM * BN, MT, NTL>(acc, g, cu / S, cu - (cu / S) * S,
                                                                        (int*)(smem + STAGES * STAGE_BYTES));
    if (reducer) gt_epilogue<MT, NTL, X2, LNK, BM, WN>(acc, g, m0, n0, wm * WTM, wn * WTN, pscr);
    if constexpr (STAMP)
      if (c_ti == 1) st[3] = gt_stamp();
  }
  if constexpr (STAMP) {
    gt_wait_vmcnt<0>();
    st[4] = gt_stamp();
    const unsigned long long rt1 = gt_realtime();
    if (threadIdx.x == 0) {
      unsigned long long* o = (unsigned long long*)g0.res + blockIdx.x * 8;
#pragma unroll
      for (int k = 0; k < 5; ++k) o[k] = st[k];
      o[5] = rt0;
      o[6] = rt1;
      o[7] = (unsigned long long)my_tiles;
    }
  }
}


// ---------------------------------------------------------------------------------------------
// Ping-pong variant (cfg 8 / 9): the 8 waves are two groups of 4 -- group 0 = waves 0-3, group 1 =
// waves 4-7, one wave of each per SIMD -- and group 1 runs one barrier behind group 0.  Each wave's
// k-step is an L section (DMA issue + every ds_read of the step's fragments) and an M section (its
// MFMAs only), separated by block barriers; with the one-barrier stagger, in every barrier interval
// one wave per SIMD is in its M section while the other loads, so the MFMA pipe never waits on LDS
// latency or the barrier (the structure of cdna_hip_programming.md §5's 256^2 template, at k-step
// granularity).  Barrier intervals I_k: group 0 reads stage s in I_{2s-1} and multiplies in I_{2s};
// group 1 reads in I_{2s} and multiplies in I_{2s+1}.  Stage s + 1 (same buffer as s - 1, free once
// group 1 finished reading s - 1 in I_{2s-2}) is DMA'd in two halves: group 0 issues the A tile in
// its L section (I_{2s-1}), group 1 the W tile in its M section of step s - 1 (I_{2s-1}); both
// retire their half with vmcnt(0) before barrier B_{2s+1}, the first after which stage s + 1 is
// read -- ~1.5 intervals of slack for every DMA.
template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(512) void gemm_pp_kernel(const GemmTileArgs g) {
  static_assert(WM * WN == 8, "8 waves");
  constexpr int WTM = BM / WM, WTN = BN / WN, MT = WTM / 16, NTL = WTN / 16;
  constexpr int ROWB = 128, A_BYTES = BM * ROWB, B_BYTES = BN * ROWB, STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int A_LD = A_BYTES / (256 * 16), B_LD = B_BYTES / (256 * 16);  // per thread of its group
  static_assert(A_BYTES % (256 * 16) == 0 && B_BYTES % (256 * 16) == 0, "whole DMA rounds per group");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int grp = __builtin_amdgcn_readfirstlane(wid >> 2), gt = tid & 255, gw = (tid >> 6) & 3;
  const int wm = wid / WN, wn = wid - wm * WN;
  const int tiles_m = (g.M + BM - 1) / BM, ntiles = tiles_m * g.tiles_n;
  const int G = gridDim.x, bq = xcd_remap(blockIdx.x, G);
  const int my_tiles = bq < ntiles ? (ntiles - 1 - bq) / G + 1 : 0;
  const int nk = g.K / 64, nsteps = my_tiles * nk;
  const rsrc_t ra = make_rsrc(g.a, g.a_bytes), rw = make_rsrc(g.w, g.w_bytes);
  const int K2 = g.K * 2;
  // this thread's DMA pieces: group 0 copies the A tile, group 1 the W tile of a stage
  constexpr int LD = A_LD > B_LD ? A_LD : B_LD;
  const int nld = grp == 0 ? A_LD : B_LD;
  int d_row[LD], d_col[LD];
#pragma unroll
  for (int i = 0; i < LD; ++i) {
    d_row[i] = (i * 256 + gt) >> 3;
    d_col[i] = ((gt & 7) ^ gt_swz<64>(d_row[i])) * 16;
  }
  auto tile_mn = [&](int ti, int& m0, int& n0) {
    int tm, tn;
    gt_tile(bq + ti * G, tiles_m, g.tiles_n, tm, tn);
    m0 = tm * BM;
    n0 = tn * BN;
  };
  auto dma_half = [&](int j) {  // this group's half of stage j
    const int ti = j / nk, kt = j - ti * nk;
    int m0, n0;
    tile_mn(ti, m0, n0);
    char* base = smem + (j & 1) * STAGE_BYTES + gw * 1024;
    if (grp == 0) {
      const int sa = m0 * K2 + kt * ROWB;
#pragma unroll
      for (int i = 0; i < A_LD; ++i)
        gt_glds16(ra, base + i * 4096, m0 + d_row[i] < g.M ? d_row[i] * K2 + d_col[i] : OOB, sa);
    } else {
      const int sb = n0 * K2 + kt * ROWB;
#pragma unroll
      for (int i = 0; i < B_LD; ++i)
        gt_glds16(rw, base + A_BYTES + i * 4096, n0 + d_row[i] < g.N ? d_row[i] * K2 + d_col[i] : OOB, sb);
    }
  };
  (void)nld;

  f32x4 acc[MT][NTL];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTL; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4, sw = gt_swz<64>(fr);
  const int a_rd = (wm * WTM + fr) * ROWB, w_rd = A_BYTES + (wn * WTN + fr) * ROWB;


  // prologue: stage 0 (both halves), group 1's half of stage 1; stage 0 visible to all
  if (nsteps > 0) dma_half(0);
  if (grp == 1 && nsteps > 1) dma_half(1);
  if (grp == 0) gt_wait_vmcnt<0>();
  else if (nsteps > 1) gt_wait_vmcnt<B_LD>();
  else gt_wait_vmcnt<0>();
  gt_barrier();
  if (grp == 1) gt_barrier();  // the stagger

  bf16x8 af[2][MT], wf[2][NTL];
  for (int j = 0; j < nsteps; ++j) {
    // ---- L section: DMA (group 0: A of stage j + 1) + all fragment reads of stage j ----
    if (grp == 0 && j + 1 < nsteps) dma_half(j + 1);
    const char* base = smem + (j & 1) * STAGE_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int coff = ((ks * 4 + fq) ^ sw) << 4;
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn) wf[ks][jn] = *reinterpret_cast<const bf16x8*>(base + w_rd + jn * 2048 + coff);
#pragma unroll
      for (int i = 0; i < MT; ++i) af[ks][i] = *reinterpret_cast<const bf16x8*>(base + a_rd + i * 2048 + coff);
    }
    if (grp == 1) gt_wait_vmcnt<0>();  // group 1's W half of stage j + 1 (issued in its last M section)
    gt_barrier();
    // ---- M section: group 1 issues its W half of stage j + 2, then every MFMA of step j ----
    if (grp == 1 && j + 2 < nsteps) dma_half(j + 2);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int jn = 0; jn < NTL; ++jn)
          acc[i][jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ks][jn], af[ks][i], acc[i][jn], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    if (j % nk == nk - 1) {
      int m0, n0;
      tile_mn(j / nk, m0, n0);
      gt_epilogue<MT, NTL>(acc, g, m0, n0, wm * WTM, wn * WTN);
    }
    if (grp == 0) gt_wait_vmcnt<0>();  // group 0's A half of stage j + 1
    gt_barrier();
  }
  if (grp == 0) gt_barrier();  // balance group 1's stagger barrier
}

// ---------------------------------------------------------------------------------------------
// Ring variant (cfg 10-12): the ping-pong stagger of gemm_pp_kernel on a DEEP LDS-DMA ring.
//
// Measured on the kernels above (profiles/r3_gemm_tile_probe_*.jsonl): the 2-stage 256 x 256 loop
// runs at ~48 % of MFMA peak on 8192^3 -- the DMA of step j + 1 has one k-step (~0.85 us of MFMA)
// to land, less than a loaded L2-miss round trip -- and the ping-pong kernel, whose DMA had even
// less lead, was slower still.  This kernel keeps the stagger (one wave per SIMD in its MFMA section
// while the other reads fragments, so barriers never empty the MFMA pipe) and gives every DMA
// R - 1 sub-steps of lead:
//  * sub-step = 32 of K: one 16x16x32 MFMA per (i, jn) per wave (32 per wave on the 256^2 tile);
//    ring slot = A[BM][32] + W[BN][32] (24-32 KB, 64-B rows), R slots (160 KB for 256^2 x 5);
//  * group 0 = waves 0-3, group 1 = waves 4-7 (one of each per SIMD); group 1 runs one barrier
//    behind.  Barrier interval 2u: G0 reads slot u (L section) while G1 multiplies u - 1 (M
//    section); interval 2u + 1: G0 multiplies u, G1 reads u;
//  * G0 DMAs the A half of sub-step u + R - 1 in its L section of u, G1 the W half of u + R in its M
//    section of u -- both into slot (u - 1) % R / u % R, free since the barrier that closed the
//    last read of it; each wave retires its half of sub-step u + 1 (counted vmcnt, never 0 in steady
//    state) before the barrier that precedes the first read of it, so a DMA has ~2(R - 2) barrier
//    intervals of lead instead of 2;
//  * epilogue bias through the scalar cache (constant address space, uniform per wave): a vector
//    load there would make hipcc drain the whole DMA ring with vmcnt(0) at every tile end.
template <int L, int MAXN>
MLS_DEV void gt_wait_groups(int n) {  // wait until <= L * min(n, MAXN) of this wave's loads are in flight
  if constexpr (MAXN == 0) {
    gt_wait_vmcnt<0>();
  } else {
    if (n >= MAXN) gt_wait_vmcnt<L * MAXN>();
    else gt_wait_groups<L, MAXN - 1>(n);
  }
}

template <int BM, int BN, int WM, int WN, int R>
__global__ __launch_bounds__(512) void gemm_ring_kernel(const GemmTileArgs g) {
  static_assert(WM * WN == 8, "8 waves");
  constexpr int WTM = BM / WM, WTN = BN / WN, MT = WTM / 16, NTL = WTN / 16;
  constexpr int ROWB = 64;  // 32 k of bf16
  constexpr int A_BYTES = BM * ROWB, SLOT = (BM + BN) * ROWB;
  constexpr int LA = A_BYTES / (256 * 16), LB = BN * ROWB / (256 * 16);  // DMAs per thread per half
  static_assert(LA * 256 * 16 == A_BYTES && LB * 256 * 16 == BN * ROWB, "whole DMA rounds per group");
  static_assert(R * SLOT <= 160 * 1024 && R >= 3, "ring");
  static_assert(WTN == 64 || WTN == 32, "bias slice");
  __shared__ __attribute__((aligned(16))) char smem[R * SLOT];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int grp = __builtin_amdgcn_readfirstlane(wid >> 2), gt = tid & 255, gw = wid & 3;
  const int wm = wid / WN, wn = wid - wm * WN;
  const int tiles_m = (g.M + BM - 1) / BM, ntiles = tiles_m * g.tiles_n;
  const int G = gridDim.x, bq = xcd_remap(blockIdx.x, G);
  const int my_tiles = bq < ntiles ? (ntiles - 1 - bq) / G + 1 : 0;
  const int nk = g.K / 32, nsub = my_tiles * nk;
  const rsrc_t ra = make_rsrc(g.a, g.a_bytes), rw = make_rsrc(g.w, g.w_bytes);
  const int K2 = g.K * 2;

  auto tile_mn = [&](int ti, int& m0, int& n0) {
    int tm, tn;
    gt_tile(bq + ti * G, tiles_m, g.tiles_n, tm, tn);
    m0 = tm * BM;
    n0 = tn * BN;
  };
  // this thread's DMA pieces (group 0: A rows, group 1: W rows): LDS byte i*4096 + gt*16 of the
  // half = row (i*4096 + gt*16) / 64, lane-linear chunk gt & 3 = source chunk (gt & 3) ^ swz(row)
  constexpr int LD = LA > LB ? LA : LB;
  int d_off[LD];
  const int lim = grp == 0 ? g.M : g.N;
#pragma unroll
  for (int i = 0; i < LD; ++i) {
    const int row = i * 64 + (gt >> 2);
    d_off[i] = row * K2 + (((gt & 3) ^ gt_swz<32>(row)) << 4);
  }
  // loader cursor of this group (its half of sub-step l_u goes to slot l_u % R)
  int l_u = 0, l_kt = 0, l_ti = 0, l_m0 = 0, l_n0 = 0, l_slot = 0;
  tile_mn(0, l_m0, l_n0);
  auto issue = [&]() {
    char* base = smem + l_slot * SLOT + gw * 1024;
    if (grp == 0) {
      const int so = l_m0 * K2 + l_kt * ROWB;
#pragma unroll
      for (int i = 0; i < LA; ++i)
        gt_glds16(ra, base + i * 4096, l_m0 + i * 64 + (gt >> 2) < lim ? d_off[i] : OOB, so);
    } else {
      const int so = l_n0 * K2 + l_kt * ROWB;
#pragma unroll
      for (int i = 0; i < LB; ++i)
        gt_glds16(rw, base + A_BYTES + i * 4096, l_n0 + i * 64 + (gt >> 2) < lim ? d_off[i] : OOB, so);
    }
    ++l_u;
    l_slot = l_slot + 1 == R ? 0 : l_slot + 1;
    if (++l_kt == nk) {
      l_kt = 0;
      if (++l_ti < my_tiles) tile_mn(l_ti, l_m0, l_n0);
    }
  };

  f32x4 acc[MT][NTL];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTL; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4;
  const int coff = (fq ^ gt_swz<32>(fr)) << 4;
  const int a_rd = (wm * WTM + fr) * ROWB + coff, w_rd = A_BYTES + (wn * WTN + fr) * ROWB + coff;


  // prologue: G0 A halves of 0 .. R-2, G1 W halves of 0 .. R-1; sub-step 0 retired; G1 staggers
  {
    const int n_pro = grp == 0 ? R - 1 : R;
    for (int u = 0; u < n_pro && u < nsub; ++u) issue();
    const int after = l_u - 1;  // loads issued after sub-step 0's
    if (grp == 0) gt_wait_groups<LA, R - 2>(after);
    else gt_wait_groups<LB, R - 1>(after);
  }
  gt_barrier();
  if (grp == 1) gt_barrier();

  int c_slot = 0, c_kt = 0, c_ti = 0;
  bf16x8 af[MT], wf[NTL];
  for (int u = 0; u < nsub; ++u) {
    // ---- L section ----
    if (grp == 0 && l_u < nsub) issue();  // A half of u + R - 1
    {
      const char* base = smem + c_slot * SLOT;
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn) wf[jn] = *reinterpret_cast<const bf16x8*>(base + w_rd + jn * 16 * ROWB);
#pragma unroll
      for (int i = 0; i < MT; ++i) af[i] = *reinterpret_cast<const bf16x8*>(base + a_rd + i * 16 * ROWB);
    }
    c_slot = c_slot + 1 == R ? 0 : c_slot + 1;
    if (grp == 1 && u + 1 < nsub) gt_wait_groups<LB, R - 2>(l_u - 1 - (u + 1));  // W half of u + 1 retired
    gt_barrier();
    // ---- M section ----
    if (grp == 1 && l_u < nsub) issue();  // W half of u + R
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn)
        acc[i][jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[jn], af[i], acc[i][jn], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    if (++c_kt == nk) {
      c_kt = 0;
      int m0, n0;
      tile_mn(c_ti++, m0, n0);
      gt_epilogue<MT, NTL>(acc, g, m0, n0, wm * WTM, wn * WTN);
    }
    if (grp == 0 && u + 1 < nsub) gt_wait_groups<LA, R - 2>(l_u - 1 - (u + 1));  // A half of u + 1 retired
    gt_barrier();
  }
  if (grp == 0) gt_barrier();  // balance group 1's stagger barrier
}

struct GtCfg {
  int bm, bn, threads;
};

// cfg ids (ops.GEMM_TILE_CFGS), tile / waves / ring (stages x K depth) / LDS:
//   1: 256x256, 8 waves 2x4, 2 x 64, 128 KB      6: 256x256, 8 waves 2x4, 4 x 32, 128 KB
//   2: 256x128, 8 waves 4x2, 3 x 64, 144 KB      7: 256x128, 8 waves 4x2, 4 x 32,  96 KB
//   3: 128x128, 4 waves 2x2, 2 x 64,  64 KB (2 blocks / CU)
//   4: 128x128, 4 waves 2x2, 3 x 64,  96 KB      5: 128x256, 8 waves 2x4, 3 x 64, 144 KB
//   8: 256x256 ping-pong (gemm_pp_kernel), 2 x 64, 128 KB    9: 256x128 ping-pong, 2 x 64, 96 KB
//  10: 256x256 ring (gemm_ring_kernel), 5 x 32, 160 KB      11: 256x256 ring, 4 x 32, 128 KB
//  12: 256x128 ring, 6 x 32, 144 KB
//  21: 192x192, 8 waves 4x2, 3 x 64, 144 KB (a 3-deep ring at ~the 256^2 tile's reuse)   22: + PIPE
//  (a 4-wave 256x256 tile -- one wave per SIMD, 128x128 wave tile, 256 accumulators -- spills
//   101-138 VGPRs in the k-loop under hipcc 7.2; not kept: docs/PERF_NOTES.md Round 4)
GtCfg gt_cfg(int cfg) {
  switch (cfg) {
    case 1: return {256, 256, 512};
    case 2: return {256, 128, 512};
    case 3: return {128, 128, 256};
    case 4: return {128, 128, 256};
    case 5: return {128, 256, 512};
    case 6: return {256, 256, 512};
    case 7: return {256, 128, 512};
    case 8: return {256, 256, 512};
    case 9: return {256, 128, 512};
    case 10: return {256, 256, 512};
    case 11: return {256, 256, 512};
    case 12: return {256, 128, 512};
    case 13: return {256, 256, 512};
    case 14: return {256, 128, 512};
    case 15: return {256, 256, 512};
    case 16: return {256, 128, 512};
    case 17: return {256, 256, 512};
    case 18: return {256, 128, 512};
    case 19: return {256, 256, 512};
    case 20: return {256, 256, 512};
    case 21: return {192, 192, 512};
    case 22: return {192, 192, 512};
    default: return {0, 0, 0};
  }
}

int gt_num_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
        hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}

int gt_launch(const GemmTileArgs& g0, int cfg, int grid_cap, hipStream_t st) {
  const GtCfg c = gt_cfg(cfg);
  if (!c.bm) return MLS_BAD_ARG;
  GemmTileArgs g = g0;
  const int tiles_m = (g.M + c.bm - 1) / c.bm;
  g.tiles_n = (g.N + c.bn - 1) / c.bn;
  // persistent grid: one resident wave of blocks (cfg 3 fits 2 per CU), each walking its tiles with
  // the LDS-DMA ring running ahead across tile boundaries
  const int per_cu = cfg == 3 ? 2 : 1;
  int cap = grid_cap > 0 ? grid_cap : gt_num_cus() * per_cu;
  const int ntiles = tiles_m * g.tiles_n;
  // split-K: tile-kernel cfgs only; whole k-steps per split, room for every slab and counter
  const bool sk_ok = cfg <= 7 || cfg >= 13;
  const int bks = cfg == 6 || cfg == 7 ? 32 : 64;
  if (g.splitk < 1) g.splitk = 1;
  if (g.splitk > 1 && (!sk_ok || (g.K / bks) % g.splitk || !g.ws || !g.cnt)) return MLS_BAD_ARG;
  const int units = ntiles * g.splitk;
  const dim3 grid(units < cap ? units : cap), block(c.threads);
  if (g.fold_c || g.ln_part || g.stats_part) {  // LayerNorm folding (mls_gemm_tile_ln maps the cfg)
#define GT_LN_LAUNCH(K)                                                                                              \
  switch (cfg) {                                                                                                     \
    case 15: hipLaunchKernelGGL((gemm_tile_kernel<256, 256, 2, 4, 2, 64, false, true, false, K>), grid, block, 0, st, g); break; \
    case 16: hipLaunchKernelGGL((gemm_tile_kernel<256, 128, 4, 2, 3, 64, false, true, false, K>), grid, block, 0, st, g); break; \
    case 5: hipLaunchKernelGGL((gemm_tile_kernel<128, 256, 2, 4, 3, 64, false, false, false, K>), grid, block, 0, st, g); break; \
    case 4: hipLaunchKernelGGL((gemm_tile_kernel<128, 128, 2, 2, 3, 64, false, false, false, K>), grid, block, 0, st, g); break; \
    default: return MLS_BAD_ARG;                                                                                     \
  }
    if (g.fold_c) {
      GT_LN_LAUNCH(1)
    } else {
      GT_LN_LAUNCH(2)
    }
#undef GT_LN_LAUNCH
    return hipGetLastError() == hipSuccess ? MLS_OK : MLS_BAD_ARG;
  }
  switch (cfg) {
    case 1: hipLaunchKernelGGL((gemm_tile_kernel<256, 256, 2, 4, 2, 64>), grid, block, 0, st, g); break;
    case 2: hipLaunchKernelGGL((gemm_tile_kernel<256, 128, 4, 2, 3, 64>), grid, block, 0, st, g); break;
    case 3: hipLaunchKernelGGL((gemm_tile_kernel<128, 128, 2, 2, 2, 64>), grid, block, 0, st, g); break;
    case 4: hipLaunchKernelGGL((gemm_tile_kernel<128, 128, 2, 2, 3, 64>), grid, block, 0, st, g); break;
    case 5: hipLaunchKernelGGL((gemm_tile_kernel<128, 256, 2, 4, 3, 64>), grid, block, 0, st, g); break;
    case 6: hipLaunchKernelGGL((gemm_tile_kernel<256, 256, 2, 4, 4, 32>), grid, block, 0, st, g); break;
    case 7: hipLaunchKernelGGL((gemm_tile_kernel<256, 128, 4, 2, 4, 32>), grid, block, 0, st, g); break;
    case 8: hipLaunchKernelGGL((gemm_pp_kernel<256, 256, 2, 4>), grid, block, 0, st, g); break;
    case 9: hipLaunchKernelGGL((gemm_pp_kernel<256, 128, 4, 2>), grid, block, 0, st, g); break;
    case 10: hipLaunchKernelGGL((gemm_ring_kernel<256, 256, 2, 4, 5>), grid, block, 0, st, g); break;
    case 11: hipLaunchKernelGGL((gemm_ring_kernel<256, 256, 2, 4, 4>), grid, block, 0, st, g); break;
    case 12: hipLaunchKernelGGL((gemm_ring_kernel<256, 128, 4, 2, 6>), grid, block, 0, st, g); break;
    case 13: hipLaunchKernelGGL((gemm_tile_kernel<256, 256, 2, 4, 2, 64, true>), grid, block, 0, st, g); break;
    case 14: hipLaunchKernelGGL((gemm_tile_kernel<256, 128, 4, 2, 3, 64, true>), grid, block, 0, st, g); break;
    case 15: hipLaunchKernelGGL((gemm_tile_kernel<256, 256, 2, 4, 2, 64, false, true>), grid, block, 0, st, g); break;
    case 16: hipLaunchKernelGGL((gemm_tile_kernel<256, 128, 4, 2, 3, 64, false, true>), grid, block, 0, st, g); break;
    case 17: hipLaunchKernelGGL((gemm_tile_kernel<256, 256, 2, 4, 2, 64, true, true>), grid, block, 0, st, g); break;
    case 18: hipLaunchKernelGGL((gemm_tile_kernel<256, 128, 4, 2, 3, 64, true, true>), grid, block, 0, st, g); break;
    case 19: hipLaunchKernelGGL((gemm_tile_kernel<256, 256, 2, 4, 2, 64, false, false, true>), grid, block, 0, st, g); break;
    case 20: hipLaunchKernelGGL((gemm_tile_kernel<256, 256, 2, 4, 2, 64, true, false, true>), grid, block, 0, st, g); break;
    case 21: hipLaunchKernelGGL((gemm_tile_kernel<192, 192, 4, 2, 3, 64>), grid, block, 0, st, g); break;
    case 22: hipLaunchKernelGGL((gemm_tile_kernel<192, 192, 4, 2, 3, 64, false, true>), grid, block, 0, st, g); break;
  }
  return hipGetLastError() == hipSuccess ? MLS_OK : MLS_BAD_ARG;
}

// default tile by shape: the largest tile that still gives the chip >= ~1 block per CU, else the
// one with the most blocks (the projection GEMMs run under 4-5-way stream concurrency in serving)
int gt_pick(int M, int N) {
  auto blocks = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
  if (blocks(256, 256) >= 256) return 15;  // cfg 1 + fragment pipeline (>= cfg 1 on every probed shape)
  if (blocks(256, 128) >= 256) return 16;
  if (blocks(128, 256) >= 256) return 5;
  return 4;
}

}  // namespace

extern "C" {

// out[M][N] = act(A[M][K] . W[N][K]^T + bias (+ res));  ACT_SILU_MUL: W rows gate/up interleaved in
// groups of 8, out [M][N/2].  K % 64 == 0, N % 16 == 0; cfg 0 = pick by shape; grid_cap 0 = one
// resident wave of persistent blocks.  splitk > 1: K in that many whole-k-step splits combined in
// the launch -- ws >= tiles * splitk * BM * BN fp32, cnt >= tiles int32, all ZERO before the first
// launch (each tile's reducer resets its counter).
int mls_gemm_tile(const void* A, const void* W, const float* bias, const void* res, void* out, int M, int N, int K,
                  int act, int ldo, int ldr, int cfg, int grid_cap, int splitk, void* ws, long long ws_elems,
                  void* cnt, int cnt_elems, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || K % 64 || N % 16 || (res && act == ACT_SILU_MUL)) return MLS_BAD_ARG;
  const size_t ab = (size_t)M * K * 2, wb = (size_t)N * K * 2;
  if (ab >= 0x7FFFFFFFull || wb >= 0x7FFFFFFFull || (size_t)M * ldo >= 0x7FFFFFFFFFull) return MLS_UNSUPPORTED;
  GemmTileArgs g{};
  g.flags = cfg >> 8;
  cfg &= 0xFF;
  g.a = (const bf16*)A;
  g.w = (const bf16*)W;
  g.bias = bias;
  g.res = (const bf16*)res;
  g.out = (bf16*)out;
  g.M = M; g.N = N; g.K = K; g.act = act;
  g.ldo = ldo > 0 ? ldo : (act == ACT_SILU_MUL ? N / 2 : N);
  g.ldr = ldr > 0 ? ldr : N;
  g.a_bytes = g.flags & GT_ABL_NOLOAD ? 0u : (uint32_t)ab;
  g.w_bytes = g.flags & GT_ABL_NOLOAD ? 0u : (uint32_t)wb;
  const int c = cfg > 0 ? cfg : gt_pick(M, N);
  g.splitk = splitk > 1 ? splitk : 1;
  if (g.splitk > 1) {
    const GtCfg t = gt_cfg(c);
    if (!t.bm) return MLS_BAD_ARG;
    const long long tiles = (long long)((M + t.bm - 1) / t.bm) * ((N + t.bn - 1) / t.bn);
    if (!ws || !cnt || tiles > cnt_elems || tiles * g.splitk * t.bm * t.bn > ws_elems) return MLS_BAD_ARG;
    g.ws = (float*)ws;
    g.cnt = (int*)cnt;
  }
  return gt_launch(g, c, grid_cap, (hipStream_t)stream);
}

int mls_gemm_tile_pick(int M, int N) { return gt_pick(M, N); }

// LayerNorm-folding forms of mls_gemm_tile (module comment "LayerNorm folding"; no split-K, ldo = ldr = N).
// Row statistics travel as [M][width / 128][2] partials (sum, sum of squares) written by a PART launch.
//  * fold_c != null: A = the raw pre-LN rows, W = W . diag(gamma), bias = b + W . beta (ops.fold_layernorm);
//    out = act(rstd * (A . W^T - mu * fold_c) + bias), A-row statistics from ln_part (K / 128 partials).
//    act: none / gelu;
//  * res != null: out = A . W^T + bias + res', res' = res, or (res - mu) * rstd * ln_g with ln_part (N / 128
//    partials) given -- the LN's beta must be folded into bias; stats_part != null: also write the OUTPUT
//    rows' partials there
//    ([M][N / 128][2]: >= M * N / 64 floats in total; N % 128 == 0).
// The LN'd widths must be multiples of 256 and at most 1024.  cfg: 0 = by shape; the folding kernels
// are the 256 x 256 / 256 x 128 PIPE tiles (15 / 16) and the 128 x 256 / 128 x 128 tiles (5 / 4).
int mls_gemm_tile_ln(const void* A, const void* W, const float* bias, const void* res, void* out, int M, int N,
                     int K, int act, int cfg, const float* fold_c, const float* ln_part, const float* ln_g,
                     float* stats_part, long long part_elems, float eps, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || K % 64 || N % 16) return MLS_BAD_ARG;
  // the LN'd rows' partials are read two per lane with 16-B loads (gt_row_stats_issue): their width
  // must be a multiple of 256 (an even partial count) and at most 1024
  if (fold_c && (res || !ln_part || stats_part || (act != ACT_NONE && act != ACT_GELU) || K % 256 || K > 1024))
    return MLS_BAD_ARG;
  if (!fold_c && (!res || act != ACT_NONE)) return MLS_BAD_ARG;
  if (ln_part && !fold_c && (!ln_g || N % 256 || N > 1024)) return MLS_BAD_ARG;
  if (stats_part && (N % 128 || (long long)M * (N / 128) * 2 > part_elems)) return MLS_BAD_ARG;
  const size_t ab = (size_t)M * K * 2, wb = (size_t)N * K * 2;
  if (ab >= 0x7FFFFFFFull || wb >= 0x7FFFFFFFull || (size_t)M * N >= 0x3FFFFFFFull) return MLS_UNSUPPORTED;
  int c = (cfg & 0xFF) > 0 ? (cfg & 0xFF) : gt_pick(M, N);
  switch (c) {
    case 15: case 16: case 5: case 4: break;
    case 3: c = 4; break;
    default: c = gt_cfg(c).bn == 128 ? 16 : 15; break;
  }
  GemmTileArgs g{};
  g.a = (const bf16*)A;
  g.w = (const bf16*)W;
  g.bias = bias;
  g.res = (const bf16*)res;
  g.out = (bf16*)out;
  g.M = M; g.N = N; g.K = K; g.act = act;
  g.ldo = N;
  g.ldr = N;
  g.a_bytes = (uint32_t)ab;
  g.w_bytes = (uint32_t)wb;
  g.splitk = 1;
  g.fold_c = fold_c;
  g.ln_part = ln_part;
  g.ln_g = ln_g;
  g.stats_part = stats_part;
  g.eps = eps;
  return gt_launch(g, c, 0, (hipStream_t)stream);
}

}  // extern "C"
