// K1 + K2 of SURVEY.md §2.E.1: implicit-GEMM NHWC convolution and plain GEMM on gfx950 MFMA,
// with a fused epilogue  y = act(acc * scale[n] + bias[n] (+ residual[m][n])).
//
// GEMM view:  M = B*Ho*Wo (or rows),  N = Cout,  K = KH*KW*Cin,  out[M][N] row-major (= NHWC).
//   A[m][k] = x[b][oh*s - p + kh][ow*s - p + kw][c]   with k = (kh*KW + kw)*Cin + c
//   B[k][n] = w[n][k]                                  (weights stored [Cout][KH][KW][Cin])
//
// Design (MI355X-first, see /opt/skills/guides/cdna_hip_programming.md §5):
//  * 256 threads = 4 waves in a 2x2 wave grid; each wave owns a (BM/2)x(BN/2) sub-tile built
//    from v_mfma_f32_16x16x32_bf16 (the bf16 shape that holds the higher clock on random data).
//  * BK = 64: one 128-byte row per tile row.  LDS images are [rows][8 x 16 B] with the 16-B
//    chunk XOR-swizzled by (row & 7): the MFMA fragment reads (ds_read_b128, 16 rows x 1 chunk
//    per lane group) are bank-conflict-free (checked exhaustively against the gfx950 lane groups).
//  * register-staged double buffer with the async-STAGE split (T14): global loads of tile k+1
//    are issued before the MFMAs of tile k and written to the other LDS buffer after them; one
//    barrier per K-step.  Register staging (not LDS-DMA) because the implicit-GEMM gather needs
//    per-lane zero-fill for the conv padding.
//  * the im2col gather is never materialised: for Cin % 64 == 0 a whole BK step lies inside one
//    filter tap, so the tap decomposition is wave-uniform scalar work per K-step.
//  * stem mode (Cin padded 3->4, KW padded 7->8 in the weights): one 16-B chunk = 2 taps x 4 ch.
//  * epilogue through LDS: accumulators are parked as fp32, then every thread emits whole
//    16-B rows (8 channels) so residual reads and output writes are coalesced dwordx4.
//  * split-K for the small-M / large-K layers (ResNet layer3/4, FC): fp32 slabs + a separate
//    reduce-epilogue kernel (deterministic; the launch boundary is captured in the hipGraph).
//  * XCD-aware bijective block remap so neighbouring tiles share an XCD's L2.
#include "common.h"
#include "fastdiv.h"

#include <cstdlib>
#include <mutex>
#include <unordered_map>

namespace {

constexpr int BK = 64;
constexpr int NTHREADS = 256;

enum ConvMode : int { MODE_GENERIC = 0, MODE_1X1 = 1, MODE_STEM = 2, MODE_DUAL = 3 };

// MODE_DUAL: two 1x1 convolutions summed into one output, i.e. one GEMM over the concatenated
// reduction  [y | x(strided)] . [W_y ; W_x]^T  -- a ResNet bottleneck's conv3 together with its
// downsample projection.  k < K1 reads y (the block's 1x1 input, stride 1), k >= K1 reads x at
// stride `stride2`; the identity branch is never written to or re-read from HBM.

struct ConvArgs {
  const bf16* x;
  const bf16* w;
  const float* scale;  // [N] or nullptr
  const float* bias;   // [N] or nullptr
  const bf16* res;     // [M][ldr] or nullptr
  bf16* out;           // [M][ldo]
  float* ws;           // split-K slabs [splitk][M][N]
  int B, H, W, Cin, Ho, Wo, N, KH, KW, stride, pad;
  int M, K;            // K = reduction length == weight row stride
  int act;
  int splitk, kchunk;
  int ldo, ldr;
  uint32_t o_bytes;
  uint32_t x_bytes, w_bytes, r_bytes;  // extents of x, w, res for the buffer-load range check
  int dbg;  // diagnostics only (ablation): 1 = skip MFMAs, 2 = skip output stores, 4 = skip operand DMA
  // MODE_DUAL second operand: x2 [B][H2][W2][Cin2], sampled at stride2; reduction split at K1
  const bf16* x2;
  uint32_t x2_bytes;
  int H2, W2, Cin2, stride2, K1;
  // split-K arrival counters (one per output tile, zero between launches): non-null -> the last
  // slice block of each tile sums the slabs and runs the epilogue in-launch (no reduce kernel)
  int* cnt;
  uint32_t ws_bytes;  // slab extent (sc1 buffer accesses of the in-launch reduction)
  // fused global average pool (the network's last convolution): pool[b][n] += pool_scale * sum of
  // the image's post-activation rows (one fp32 atomic per image segment and column of a tile);
  // pool_only: the output itself is not stored.  splitk == 1 only.
  float* pool;
  float pool_scale;
  int pool_hw, pool_only;
  // the kernels' runtime divisors (fastdiv.h; set by set_fastdivs for the launched tile width):
  // Ho*Wo, Wo, splitk, column tiles, Cin, KW, k-steps per tile (persistent), pool_hw
  FastDiv fd_howo, fd_wo, fd_split, fd_ntn, fd_cin, fd_kw, fd_nk, fd_pool;
};

void set_fastdivs(ConvArgs& a, int bn) {
  a.fd_howo = fastdiv_make((uint32_t)(a.Ho * a.Wo));
  a.fd_wo = fastdiv_make((uint32_t)a.Wo);
  a.fd_split = fastdiv_make((uint32_t)(a.splitk > 0 ? a.splitk : 1));
  a.fd_ntn = fastdiv_make((uint32_t)((a.N + bn - 1) / bn));
  a.fd_cin = fastdiv_make((uint32_t)a.Cin);
  a.fd_kw = fastdiv_make((uint32_t)(a.KW > 0 ? a.KW : 1));
  a.fd_nk = fastdiv_make((uint32_t)((a.K + BK - 1) / BK));
  a.fd_pool = fastdiv_make((uint32_t)(a.pool_hw > 0 ? a.pool_hw : 1));
}

int g_dbg_flags = 0;  // set via mls_set_debug_flags (tools/conv_ablate.py); 0 in production

#define LDS3 __attribute__((address_space(3)))

MLS_DEV void glds16(rsrc_t r, char* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDS3 void*)lds, 16, voff, soff, 0, 0);
}

template <int N>
MLS_DEV void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt field");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// LDS chunk swizzle of a tile row: BK = 64 (128-B rows, 8 chunks): chunk ^ (row & 7);
// BK = 32 (64-B rows, 4 chunks): chunk ^ f(row & 15), f = (r0 | r2 << 1) -- conflict-free for the
// gfx950 ds_read_b128 lane groups over the MFMA fragment rows (checked exhaustively, 96 such linear
// maps exist; this is one of them).
template <int BKT>
MLS_DEV int row_swz(int r) {
  if constexpr (BKT == 64) return r & 7;
  else return (r & 1) | ((r >> 1) & 2);
}

// Split-K finish for 8 outputs of row m starting at column n: sum the fp32 slabs, then
// act(sum * scale + bias (+ res)) -> bf16.  SiLU-mul (gate/up interleaved in 8-column groups):
// columns n..n+15 -> 8 outputs at n / 2.  Used by the separate reduce kernel and by the in-launch
// reducer (the last-arriving slice block of a tile).
typedef unsigned int u32x4v __attribute__((__vector_size__(16)));

// SC1: the slabs were written through (sc1 stores) by other workgroups of this launch -> read them
// with sc1 loads through `wr` (no acquire fence); otherwise plain loads (a later launch).
template <bool SC1>
MLS_DEV float4 slab_ld(const ConvArgs& a, rsrc_t wr, size_t idx) {
  if constexpr (SC1) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(wr, (int)(idx * 4), 0, 16));
  } else {
    return *reinterpret_cast<const float4*>(a.ws + idx);
  }
}

template <bool SC1>
MLS_DEV void splitk_finish_chunk(const ConvArgs& a, rsrc_t wr, int m, int n, bool glu) {
  float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (glu) {
    float u[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int s = 0; s < a.splitk; ++s) {
      const size_t i0 = ((size_t)s * a.M + m) * a.N + n;
      const float4 g0 = slab_ld<SC1>(a, wr, i0), g1 = slab_ld<SC1>(a, wr, i0 + 4);
      const float4 u0 = slab_ld<SC1>(a, wr, i0 + 8), u1 = slab_ld<SC1>(a, wr, i0 + 12);
      v[0] += g0.x; v[1] += g0.y; v[2] += g0.z; v[3] += g0.w; v[4] += g1.x; v[5] += g1.y; v[6] += g1.z; v[7] += g1.w;
      u[0] += u0.x; u[1] += u0.y; u[2] += u0.z; u[3] += u0.w; u[4] += u1.x; u[5] += u1.y; u[6] += u1.z; u[7] += u1.w;
    }
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float gt = v[e] + (a.bias ? a.bias[n + e] : 0.f);
      const float up = u[e] + (a.bias ? a.bias[n + 8 + e] : 0.f);
      o[e] = silu(gt) * up;
    }
    st16(a.out + (size_t)m * a.ldo + (n >> 1), pack8(o));
    return;
  }
  for (int s = 0; s < a.splitk; ++s) {
    const size_t i0 = ((size_t)s * a.M + m) * a.N + n;
    const float4 x0 = slab_ld<SC1>(a, wr, i0), x1 = slab_ld<SC1>(a, wr, i0 + 4);
    v[0] += x0.x; v[1] += x0.y; v[2] += x0.z; v[3] += x0.w; v[4] += x1.x; v[5] += x1.y; v[6] += x1.z; v[7] += x1.w;
  }
  if (a.scale) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= a.scale[n + e];
  }
  if (a.bias) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += a.bias[n + e];
  }
  if (a.res) {
    float r[8];
    unpack8(ld16(a.res + (size_t)m * a.ldr + n), r);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += r[e];
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = apply_act(v[e], a.act);
  st16(a.out + (size_t)m * a.ldo + n, pack8(v));
}

// MFMA operand order of conv_gemm_kernel.  1: D = B_tile . A_tile^T, so a lane's 4 accumulators
// are 4 consecutive OUTPUT CHANNELS of one output pixel and parking a 16 x 16 fragment in LDS for
// the epilogue is ONE ds_write_b128 per lane (row stride C_LD = BN + 4 floats: the 8-lane groups
// of the write hit disjoint bank quads) instead of four ds_write_b32 down a column.  0 (default):
// D = A_tile . B_tile^T -- the swapped build measured 2 % SLOWER over the forward's conv calls
// co-running (397 vs 389 us, profiles/r3_swap_epilogue_component_costs.jsonl), so it stays an
// A/B build option (-DMLS_CONV_SWAP=1).
#ifndef MLS_CONV_SWAP
#define MLS_CONV_SWAP 0
#endif

// Park one 16 x 16 fp32 accumulator fragment at (row0, col0) of the row-major LDS tile Cs.
MLS_DEV void park_frag(float* Cs, int ld, int row0, int col0, int fr, int fq, const f32x4& v) {
  if (MLS_CONV_SWAP) {
    *reinterpret_cast<float4*>(Cs + (row0 + fr) * ld + col0 + fq * 4) = float4{v[0], v[1], v[2], v[3]};
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float e = v[r];  // through a named float (ext-vector element bit-cast hazard)
      Cs[(row0 + fq * 4 + r) * ld + col0 + fr] = e;
    }
  }
}

// v2: LDS-DMA (buffer_load ... lds) into a STAGES-deep ring, counted vmcnt + raw s_barrier.
// BKT (64 or 32) is the K depth of a stage: 32 halves the LDS ring, and with the accumulators
// parked for the epilogue in EPI_PASSES row blocks, a block's LDS can shrink to ~24 KB -- twice
// the resident blocks per CU for the latency-bound layers (guide: residency hides DMA latency).
template <int BM, int BN, int WM, int WN, int STAGES, int MODE, int BKT = 64, int EPI_PASSES = 1>
__global__ __launch_bounds__(WM * WN * 64) void conv_gemm_kernel(const ConvArgs a) {
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int CPK = BKT / 8;   // 16-B chunks per tile row
  constexpr int RPP = 64 / CPK;  // tile rows per 1-KiB DMA piece
  constexpr int A_BYTES = BM * BKT * 2, B_BYTES = BN * BKT * 2;
  constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int AI = BM / RPP / NW, BI = BN / RPP / NW;  // 1-KiB DMA pieces per wave per stage
  static_assert(AI * RPP * NW == BM && BI * RPP * NW == BN, "tile / wave mismatch");
  static_assert(TM >= 1 && TN >= 1, "wave tile too small");
  static_assert(BKT == 64 || BKT == 32, "BK");
  constexpr int LPS = AI + BI;  // vmcnt units per stage
  constexpr int C_LD = BN + 4;
  constexpr int PASS_ROWS = BM / EPI_PASSES;
  static_assert(PASS_ROWS % 16 == 0 && PASS_ROWS * EPI_PASSES == BM, "epilogue passes");
  constexpr int EPI_BYTES = PASS_ROWS * C_LD * 4;
  constexpr int LDS_BYTES = (STAGES * STAGE_BYTES > EPI_BYTES) ? STAGES * STAGE_BYTES : EPI_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;

  const int ntn = (a.N + BN - 1) / BN;
  int t = xcd_remap(blockIdx.x, gridDim.x);
  const int tq = fastdiv(t, a.fd_split);
  const int split = t - tq * a.splitk;
  t = tq;
  const int tmi = fastdiv(t, a.fd_ntn), tn = t - tmi * ntn;
  const int m0 = tmi * BM, n0 = tn * BN;
  const int kbeg = split * a.kchunk;
  const int kend = min(a.K, kbeg + a.kchunk);
  const int nk = kend > kbeg ? (kend - kbeg + BKT - 1) / BKT : 0;

  // lane -> (row within an RPP-row DMA piece, logical 16-B chunk).  The DMA writes LDS lane-
  // linearly (base + 16*lane), so the XOR swizzle is applied to the SOURCE chunk instead:
  // physical chunk (lane % CPK) of row r holds logical chunk (lane % CPK) ^ row_swz(r).
  const int r8 = lane / CPK;
  const int lc = (lane % CPK) ^ row_swz<BKT>(r8);

  int a_v[AI], a_v2[AI];
  uint32_t a_msk[AI];
  const int HoWo = a.Ho * a.Wo;
#pragma unroll
  for (int j = 0; j < AI; ++j) {
    const int m = m0 + (wid * AI + j) * RPP + r8;
    a_msk[j] = 0u;
    a_v[j] = OOB;
    a_v2[j] = OOB;
    if (m < a.M) {
      const int b = fastdiv(m, a.fd_howo);
      const int rem = m - b * HoWo;
      const int oh = fastdiv(rem, a.fd_wo);
      const int ow = rem - oh * a.Wo;
      if (MODE == MODE_DUAL) {
        a_v[j] = (((b * a.H + oh) * a.W + ow) * a.Cin + lc * 8) * 2;
        a_v2[j] = (((b * a.H2 + oh * a.stride2) * a.W2 + ow * a.stride2) * a.Cin2 + lc * 8) * 2;
      } else if (MODE == MODE_1X1) {
        a_v[j] = (((b * a.H + oh * a.stride) * a.W + ow * a.stride) * a.Cin + lc * 8) * 2;
      } else if (MODE == MODE_STEM) {  // pre-padded image, Cin 4, chunk = 2 taps: kh = lc>>2, kw = 2*(lc&3)
        a_v[j] = (((b * a.H + oh * a.stride + (lc >> 2)) * a.W + ow * a.stride + 2 * (lc & 3)) * 4) * 2;
      } else {  // generic: per-row validity bitmask over the KH*KW taps
        const int ih0 = oh * a.stride - a.pad, iw0 = ow * a.stride - a.pad;
        uint32_t msk = 0u;
        for (int kh = 0; kh < a.KH; ++kh)
          for (int kw = 0; kw < a.KW; ++kw)
            if ((unsigned)(ih0 + kh) < (unsigned)a.H && (unsigned)(iw0 + kw) < (unsigned)a.W)
              msk |= 1u << (kh * a.KW + kw);
        a_msk[j] = msk;
        a_v[j] = ((b * a.H * a.W + ih0 * a.W + iw0) * a.Cin + lc * 8) * 2;
      }
    }
  }
  int b_v[BI];
#pragma unroll
  for (int j = 0; j < BI; ++j) {
    const int n = n0 + (wid * BI + j) * RPP + r8;
    b_v[j] = n < a.N ? (n * a.K + lc * 8) * 2 : OOB;
  }

  const rsrc_t xr = make_rsrc(a.x, a.x_bytes);
  const rsrc_t wr = make_rsrc(a.w, a.w_bytes);
  const rsrc_t xr2 = make_rsrc(a.x2, MODE == MODE_DUAL ? a.x2_bytes : 0);

  auto issue = [&](int kt, int buf) {
    const int k0 = kbeg + kt * BKT;
    char* sA = smem + buf * STAGE_BYTES;
    char* sB = sA + A_BYTES;
    const int left = kend - k0;  // < BKT only on a K tail
    const bool lane_kin = lc * 8 < left;
    if (MODE == MODE_DUAL) {  // K1 % 64 == 0: a step lies wholly in one operand (wave-uniform branch)
      if (k0 < a.K1) {
#pragma unroll
        for (int j = 0; j < AI; ++j) glds16(xr, sA + (wid * AI + j) * 1024, lane_kin ? a_v[j] : OOB, k0 * 2);
      } else {
#pragma unroll
        for (int j = 0; j < AI; ++j)
          glds16(xr2, sA + (wid * AI + j) * 1024, lane_kin ? a_v2[j] : OOB, (k0 - a.K1) * 2);
      }
    } else if (MODE == MODE_1X1) {
#pragma unroll
      for (int j = 0; j < AI; ++j) glds16(xr, sA + (wid * AI + j) * 1024, lane_kin ? a_v[j] : OOB, k0 * 2);
    } else if (MODE == MODE_STEM) {
      const int soff = (k0 >> 5) * a.W * 8;  // kh base rows (K rows of 32 = one kh)
#pragma unroll
      for (int j = 0; j < AI; ++j) glds16(xr, sA + (wid * AI + j) * 1024, a_v[j], soff);
    } else {
      const int tap = fastdiv(k0, a.fd_cin);  // the whole BKT-wide step is inside one tap
      const int c0 = k0 - tap * a.Cin;
      const int kh = fastdiv(tap, a.fd_kw);
      const int kw = tap - kh * a.KW;
      const int uni = ((kh * a.W + kw) * a.Cin + c0) * 2;
#pragma unroll
      for (int j = 0; j < AI; ++j) {
        const bool ok = (a_msk[j] >> tap) & 1u;
        glds16(xr, sA + (wid * AI + j) * 1024, ok ? a_v[j] + uni : OOB, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < BI; ++j) glds16(wr, sB + (wid * BI + j) * 1024, lane_kin ? b_v[j] : OOB, k0 * 2);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // residual prefetch: issued before the operand DMA so its latency overlaps the K loop instead
  // of serialising after it (the small-K layers are latency-bound).  Same thread->chunk map as
  // the epilogue below.
  constexpr int CPR = BN / 8;
  constexpr int EPI_IT = (BM * CPR + NT - 1) / NT;
  uint4 resv[EPI_IT];
  const bool pre_res = a.res != nullptr && a.splitk == 1 && a.act != ACT_SILU_MUL;
  if (pre_res) {
    const rsrc_t rr = make_rsrc(a.res, a.r_bytes);
#pragma unroll
    for (int it = 0; it < EPI_IT; ++it) {
      const int q = tid + it * NT;
      const int row = q / CPR, c8 = q - (q / CPR) * CPR;
      const int m = m0 + row, n = n0 + c8 * 8;
      const bool ok = q < BM * CPR && m < a.M && n < a.N;
      resv[it] = bload16(rr, ok ? (m * a.ldr + n) * 2 : OOB);
    }
  }

  // bias / scale prefetch: NT % CPR == 0, so every epilogue iteration of this thread touches
  // the same 8 output columns -> one 32-B chunk of each, loaded up front.
  static_assert(NT % CPR == 0, "epilogue column mapping");
  const int my_n = n0 + (tid % CPR) * 8;
  float bias8[8], scale8[8];
  {
    const bool nok = my_n < a.N;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      bias8[e] = 0.f;
      scale8[e] = 1.f;
    }
    if (nok && a.bias) {
      const float4 b0 = *reinterpret_cast<const float4*>(a.bias + my_n);
      const float4 b1 = *reinterpret_cast<const float4*>(a.bias + my_n + 4);
      bias8[0] = b0.x; bias8[1] = b0.y; bias8[2] = b0.z; bias8[3] = b0.w;
      bias8[4] = b1.x; bias8[5] = b1.y; bias8[6] = b1.z; bias8[7] = b1.w;
    }
    if (nok && a.scale) {
      const float4 s0 = *reinterpret_cast<const float4*>(a.scale + my_n);
      const float4 s1 = *reinterpret_cast<const float4*>(a.scale + my_n + 4);
      scale8[0] = s0.x; scale8[1] = s0.y; scale8[2] = s0.z; scale8[3] = s0.w;
      scale8[4] = s1.x; scale8[5] = s1.y; scale8[6] = s1.z; scale8[7] = s1.w;
    }
  }

  const int npro = nk < STAGES - 1 ? nk : STAGES - 1;
  if (!(a.dbg & 4))
    for (int s = 0; s < npro; ++s) issue(s, s);

  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int issued = (kt + STAGES - 1 < nk) ? kt + STAGES - 1 : nk;
    const int ahead = issued - (kt + 1);  // stages still allowed in flight (<= STAGES - 2)
    switch (ahead) {  // counted wait: stage kt landed, the younger `ahead` stages stay in flight
      case 4: if constexpr (STAGES >= 6) { wait_vmcnt<4 * LPS>(); break; } [[fallthrough]];
      case 3: if constexpr (STAGES >= 5) { wait_vmcnt<3 * LPS>(); break; } [[fallthrough]];
      case 2: if constexpr (STAGES >= 4) { wait_vmcnt<2 * LPS>(); break; } [[fallthrough]];
      case 1: wait_vmcnt<LPS>(); break;
      default: wait_vmcnt<0>(); break;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + STAGES - 1 < nk && !(a.dbg & 4)) issue(kt + STAGES - 1, (kt + STAGES - 1) % STAGES);
    if (a.dbg & 1) continue;
    const int cur = kt % STAGES;
    const uint4* As = reinterpret_cast<const uint4*>(smem + cur * STAGE_BYTES);
    const uint4* Bs = reinterpret_cast<const uint4*>(smem + cur * STAGE_BYTES + A_BYTES);
#pragma unroll
    for (int kk = 0; kk < BKT / 32; ++kk) {
      const int ch = fq + 4 * kk;
      bf16x8 af[TM], bfv[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * WTM + i * 16 + fr;
        af[i] = __builtin_bit_cast(bf16x8, As[r * CPK + (ch ^ row_swz<BKT>(r))]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wn * WTN + j * 16 + fr;
        bfv[j] = __builtin_bit_cast(bf16x8, Bs[r * CPK + (ch ^ row_swz<BKT>(r))]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = MLS_CONV_SWAP ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfv[j], af[i], acc[i][j], 0, 0, 0)
                                    : __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfv[j], acc[i][j], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  // ---- epilogue: park fp32 accumulators in LDS (EPI_PASSES row blocks), then emit 16-B rows ----
  float* Cs = reinterpret_cast<float*>(smem);
  if (EPI_PASSES == 1 && a.act == ACT_SILU_MUL && a.splitk == 1) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) park_frag(Cs, C_LD, wm * WTM + i * 16, wn * WTN + j * 16, fr, fq, acc[i][j]);
    __syncthreads();
    // gate/up interleaved in 8-column groups: chunk 2p = gate, 2p+1 = up -> 8 outputs at n/2
    for (int q = tid; q < BM * (CPR / 2); q += NT) {
      const int row = q / (CPR / 2), p = q - (q / (CPR / 2)) * (CPR / 2);
      const int m = m0 + row, n = n0 + p * 16;
      if (m >= a.M || n >= a.N) continue;
      const float* src = Cs + row * C_LD + p * 16;
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float gt = src[e], up = src[8 + e];
        if (a.bias) {
          gt += a.bias[n + e];
          up += a.bias[n + 8 + e];
        }
        o[e] = silu(gt) * up;
      }
      st16(a.out + (size_t)m * a.ldo + (n >> 1), pack8(o));
    }
    return;
  }
  const rsrc_t wsr = make_rsrc(a.ws, a.cnt != nullptr ? a.ws_bytes : 0u);
#pragma unroll
  for (int pass = 0; pass < EPI_PASSES; ++pass) {
    const int row_lo = pass * PASS_ROWS;
    if (pass > 0) __syncthreads();  // the previous pass's rows have been read
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int frag_row = wm * WTM + i * 16;  // a fragment's 16 rows fall in one pass
      if (EPI_PASSES > 1 && (frag_row < row_lo || frag_row >= row_lo + PASS_ROWS)) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j) park_frag(Cs, C_LD, frag_row - row_lo, wn * WTN + j * 16, fr, fq, acc[i][j]);
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < EPI_IT; ++it) {
      const int q = tid + it * NT;
      const int row = q / CPR, c8 = q - (q / CPR) * CPR;
      if (EPI_PASSES > 1 && (row < row_lo || row >= row_lo + PASS_ROWS)) continue;
      const int m = m0 + row, n = n0 + c8 * 8;
      if (q >= BM * CPR || m >= a.M || n >= a.N) continue;
      const float4 v0 = *reinterpret_cast<const float4*>(Cs + (row - row_lo) * C_LD + c8 * 8);
      const float4 v1 = *reinterpret_cast<const float4*>(Cs + (row - row_lo) * C_LD + c8 * 8 + 4);
      if (a.splitk > 1) {
        const size_t widx = ((size_t)split * a.M + m) * a.N + n;
        if (a.cnt != nullptr) {  // write-through: visible to this tile's reducer with no release fence
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, v0), wsr, (int)(widx * 4), 0, 16);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, v1), wsr, (int)(widx * 4 + 16), 0, 16);
        } else {
          *reinterpret_cast<float4*>(a.ws + widx) = v0;
          *reinterpret_cast<float4*>(a.ws + widx + 4) = v1;
        }
        continue;
      }
      float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = v[e] * scale8[e] + bias8[e];
      if (pre_res) {
        float r[8];
        unpack8(resv[it], r);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += r[e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = apply_act(v[e], a.act);
      if (a.dbg & 2) {
        if (v[0] == 12345.678f) st16(a.out, pack8(v));  // keep the value live, never true
        continue;
      }
      if (a.pool) {  // the pooled values: post-activation, back into this thread's own LDS slots
        float* cp = Cs + (row - row_lo) * C_LD + c8 * 8;
        *reinterpret_cast<float4*>(cp) = float4{v[0], v[1], v[2], v[3]};
        *reinterpret_cast<float4*>(cp + 4) = float4{v[4], v[5], v[6], v[7]};
        if (a.pool_only) continue;
      }
      st16(a.out + (size_t)m * a.ldo + n, pack8(v));
    }
    if (a.pool && a.splitk == 1) {
      // global average pool: a thread per column walks the pass's rows in order (a fixed summation
      // order per image segment: with <= 2 segments per image per column the fp32 atomics commute,
      // so the pooled sums are bit-identical run to run), one atomic per image segment.  The LDS
      // reads are issued 8 at a time and the image boundary is tracked instead of divided per row
      // (the plain per-row walk cost the last conv 3-6 us: profiles/r4_resnet50_serial_head_ab.txt).
      __syncthreads();
      const int n = n0 + tid;
      const int rows = min(PASS_ROWS, a.M - (m0 + row_lo));
      if (tid < BN && n < a.N && rows > 0) {
        int cur = fastdiv(m0 + row_lo, a.fd_pool);
        int next = (cur + 1) * a.pool_hw - (m0 + row_lo);  // first pass row of the next image
        float sum = 0.f;
        for (int r0 = 0; r0 < rows; r0 += 8) {
          float x[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] = Cs[min(r0 + j, PASS_ROWS - 1) * C_LD + tid];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int r = r0 + j;
            if (r < rows) {
              if (r == next) {
                atomicAdd(a.pool + (size_t)cur * a.N + n, sum * a.pool_scale);
                sum = 0.f;
                ++cur;
                next += a.pool_hw;
              }
              sum += x[j];
            }
          }
        }
        atomicAdd(a.pool + (size_t)cur * a.N + n, sum * a.pool_scale);
      }
    }
  }
  if (a.splitk > 1 && a.cnt != nullptr) {
    // In-launch split-K reduction (guide §5 item 2): publish this slice's slab with one agent-scope
    // release, take a ticket; the tile's last arriver acquires once and finishes the tile.
    // sc1 (write-through) slabs: drained stores need no release fence, sc1 loads no acquire (guide
    // §5 item 2, §6 Guideline 16 R1).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(smem);  // the one LDS array (no second __shared__ object)
    if (tid == 0) {
      const int prev = __hip_atomic_fetch_add(a.cnt + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = prev == a.splitk - 1;
      if (last) __hip_atomic_store(a.cnt + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for the next launch
      flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
    const bool glu = a.act == ACT_SILU_MUL;
    const int cpr = glu ? CPR / 2 : CPR;  // output chunks of 8 per tile row
    const int cw = glu ? 16 : 8;          // input columns per chunk
    for (int q = tid; q < BM * cpr; q += NT) {
      const int row = q / cpr, c = q - (q / cpr) * cpr;
      const int m = m0 + row, n = n0 + c * cw;
      if (m < a.M && n < a.N) splitk_finish_chunk<true>(a, wsr, m, n, glu);
    }
  }
}

// v3: persistent + software-pipelined across tiles.  Each block walks tiles lb, lb+G, ...; the
// LDS-DMA ring (3 stages) runs continuously over the flattened (tile, k-step) sequence, so the
// next tile's operands -- and, with its last k-step, its residual tile -- are in flight while the
// current tile's epilogue runs.  Epilogue in place: acc*scale + bias + residual -> act -> bf16
// written over the residual tile in LDS, then 16-B buffer stores (always issued, OOB-dropped, so
// the hand-counted vmcnt stays exact).  Bias comes from a per-block LDS copy.  No split-K.
template <int BM, int BN, int WM, int WN, int MODE>
__global__ __launch_bounds__(WM * WN * 64) void conv_gemm_persistent(const ConvArgs a) {
  constexpr int STAGES = 3;
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, R_BYTES = BM * BN * 2;
  constexpr int STAGE_BYTES = A_BYTES + B_BYTES + R_BYTES;
  constexpr int AI = BM / 8 / NW, BI = BN / 8 / NW;
  constexpr int RCPR = BN / 8;     // 16-B chunks per output / residual row
  constexpr int RPP = 64 / RCPR;   // rows per 1-KiB DMA piece
  constexpr int RI = BM / RPP / NW;
  constexpr int EPI2 = BM * RCPR / NT;  // 16-B output stores per thread per tile
  static_assert(AI * 8 * NW == BM && BI * 8 * NW == BN && RI * RPP * NW == BM && EPI2 * NT == BM * RCPR, "tile");
  constexpr int LPS = AI + BI;
  constexpr int BIAS_MAX = 2048;
  __shared__ __attribute__((aligned(16))) char smem[STAGES * STAGE_BYTES + BIAS_MAX * 4];
  float* sbias = reinterpret_cast<float*>(smem + STAGES * STAGE_BYTES);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int ntm = (a.M + BM - 1) / BM, ntn = (a.N + BN - 1) / BN, T = ntm * ntn;
  const int G = gridDim.x;
  const int lb = xcd_remap(blockIdx.x, G);
  if (lb >= T) return;
  const int my_tiles = (T - lb + G - 1) / G;
  const int nk = (a.K + BK - 1) / BK;
  const int S_tot = my_tiles * nk;
  const bool has_res = a.res != nullptr;
  const bool bias_lds = a.bias != nullptr && a.N <= BIAS_MAX;
  if (bias_lds)
    for (int i = tid; i < a.N; i += NT) sbias[i] = a.bias[i];

  const int r8 = lane >> 3, lc = (lane & 7) ^ r8;
  const int rrow = lane / RCPR, rpc = lane % RCPR;
  const rsrc_t xr = make_rsrc(a.x, a.x_bytes);
  const rsrc_t wr = make_rsrc(a.w, a.w_bytes);
  const rsrc_t rr = make_rsrc(a.res, a.r_bytes);
  const rsrc_t orr = make_rsrc(a.out, a.o_bytes);
  const int HoWo = a.Ho * a.Wo;

  int a_v[AI], b_v[BI], r_v[RI];
  uint32_t a_msk[AI];
  auto setup_tile = [&](int k) {  // issue-side per-tile precompute (once per tile)
    const int t = lb + k * G;
    const int tq = fastdiv(t, a.fd_ntn);
    const int m0 = tq * BM, n0 = (t - tq * ntn) * BN;
#pragma unroll
    for (int j = 0; j < AI; ++j) {
      const int m = m0 + (wid * AI + j) * 8 + r8;
      a_msk[j] = 0u;
      a_v[j] = OOB;
      if (m < a.M) {
        const int b = fastdiv(m, a.fd_howo);
        const int rem = m - b * HoWo;
        const int oh = fastdiv(rem, a.fd_wo);
        const int ow = rem - oh * a.Wo;
        if (MODE == MODE_1X1) {
          a_v[j] = (((b * a.H + oh * a.stride) * a.W + ow * a.stride) * a.Cin + lc * 8) * 2;
        } else if (MODE == MODE_STEM) {
          a_v[j] = (((b * a.H + oh * a.stride + (lc >> 2)) * a.W + ow * a.stride + 2 * (lc & 3)) * 4) * 2;
        } else {
          const int ih0 = oh * a.stride - a.pad, iw0 = ow * a.stride - a.pad;
          uint32_t msk = 0u;
          for (int kh = 0; kh < a.KH; ++kh)
            for (int kw = 0; kw < a.KW; ++kw)
              if ((unsigned)(ih0 + kh) < (unsigned)a.H && (unsigned)(iw0 + kw) < (unsigned)a.W)
                msk |= 1u << (kh * a.KW + kw);
          a_msk[j] = msk;
          a_v[j] = ((b * a.H * a.W + ih0 * a.W + iw0) * a.Cin + lc * 8) * 2;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < BI; ++j) {
      const int n = n0 + (wid * BI + j) * 8 + r8;
      b_v[j] = n < a.N ? (n * a.K + lc * 8) * 2 : OOB;
    }
#pragma unroll
    for (int j = 0; j < RI; ++j) {
      const int row = (wid * RI + j) * RPP + rrow;
      const int lch = rpc ^ (row & (RCPR - 1));
      const int m = m0 + row, n = n0 + lch * 8;
      r_v[j] = (m < a.M && n < a.N) ? (m * a.ldr + n) * 2 : OOB;
    }
  };

  auto issue = [&](int sidx, int buf) {
    const int k = fastdiv(sidx, a.fd_nk), ks = sidx - k * nk;
    if (ks == 0) setup_tile(k);
    const int k0 = ks * BK;
    char* sA = smem + buf * STAGE_BYTES;
    char* sB = sA + A_BYTES;
    char* sR = sB + B_BYTES;
    const int left = a.K - k0;
    const bool lane_kin = lc * 8 < left;
    if (MODE == MODE_1X1) {
#pragma unroll
      for (int j = 0; j < AI; ++j) glds16(xr, sA + (wid * AI + j) * 1024, lane_kin ? a_v[j] : OOB, k0 * 2);
    } else if (MODE == MODE_STEM) {
      const int soff = (k0 >> 5) * a.W * 8;
#pragma unroll
      for (int j = 0; j < AI; ++j) glds16(xr, sA + (wid * AI + j) * 1024, a_v[j], soff);
    } else {
      const int tap = fastdiv(k0, a.fd_cin);
      const int c0 = k0 - tap * a.Cin;
      const int kh = fastdiv(tap, a.fd_kw);
      const int kw = tap - kh * a.KW;
      const int uni = ((kh * a.W + kw) * a.Cin + c0) * 2;
#pragma unroll
      for (int j = 0; j < AI; ++j) {
        const bool ok = (a_msk[j] >> tap) & 1u;
        glds16(xr, sA + (wid * AI + j) * 1024, ok ? a_v[j] + uni : OOB, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < BI; ++j) glds16(wr, sB + (wid * BI + j) * 1024, lane_kin ? b_v[j] : OOB, k0 * 2);
    if (has_res && ks == nk - 1) {
#pragma unroll
      for (int j = 0; j < RI; ++j) glds16(rr, sR + (wid * RI + j) * 1024, r_v[j], 0);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  int issued = 0;
  for (; issued < S_tot && issued < STAGES - 1; ++issued) issue(issued, issued);

  const int fr = lane & 15, fq = lane >> 4;
  bool prev_epi = false;
  for (int s = 0; s < S_tot; ++s) {
    // exact count of the VMEM ops younger than stage s: stage s+1's DMA (+ its residual pieces)
    // and the previous epilogue's stores
    if (issued > s + 1) {
      const bool nr = has_res && (s + 1 - fastdiv(s + 1, a.fd_nk) * nk == nk - 1);
      if (nr && prev_epi)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPS + RI + EPI2) : "memory");
      else if (nr)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPS + RI) : "memory");
      else if (prev_epi)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPS + EPI2) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPS) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (issued < S_tot) {
      issue(issued, issued % STAGES);
      ++issued;
    }
    const int buf = s % STAGES;
    const uint4* As = reinterpret_cast<const uint4*>(smem + buf * STAGE_BYTES);
    const uint4* Bs = reinterpret_cast<const uint4*>(smem + buf * STAGE_BYTES + A_BYTES);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = fq + 4 * kk;
      bf16x8 af[TM], bfv[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * WTM + i * 16 + fr;
        af[i] = __builtin_bit_cast(bf16x8, As[r * 8 + (ch ^ (r & 7))]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wn * WTN + j * 16 + fr;
        bfv[j] = __builtin_bit_cast(bf16x8, Bs[r * 8 + (ch ^ (r & 7))]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfv[j], acc[i][j], 0, 0, 0);
    }
    prev_epi = false;
    const int sq = fastdiv(s, a.fd_nk);
    if (s - sq * nk == nk - 1) {
      const int t = lb + sq * G;
      const int tq = fastdiv(t, a.fd_ntn);
      const int m0 = tq * BM, n0 = (t - tq * ntn) * BN;
      char* sR = smem + buf * STAGE_BYTES + A_BYTES + B_BYTES;
      // pass 1: in place over the residual tile (each element owned by exactly one lane)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * WTN + j * 16 + fr;
        const int n = n0 + col;
        float bb = 0.f, sc = 1.f;
        if (n < a.N) {
          if (bias_lds) bb = sbias[n];
          else if (a.bias) bb = a.bias[n];
          if (a.scale) sc = a.scale[n];
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = wm * WTM + i * 16 + fq * 4 + r;
            const int off = row * (BN * 2) + ((((col >> 3) ^ (row & (RCPR - 1)))) << 4) + (col & 7) * 2;
            bf16* p = reinterpret_cast<bf16*>(sR + off);
            float v = acc[i][j][r] * sc + bb;
            if (has_res) v += (float)*p;
            *p = (bf16)apply_act(v, a.act);
          }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      // pass 2: whole 16-B rows out
#pragma unroll
      for (int it = 0; it < EPI2; ++it) {
        const int q = tid + it * NT;
        const int row = q / RCPR, c8 = q % RCPR;
        const int m = m0 + row, n = n0 + c8 * 8;
        const uint4 v = *reinterpret_cast<const uint4*>(sR + row * (BN * 2) + ((c8 ^ (row & (RCPR - 1))) << 4));
        const int off = (m < a.M && n < a.N) ? (m * a.ldo + n) * 2 : OOB;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v),
                                               orr, off, 0, 0);
      }
      prev_epi = true;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// sum split-K slabs + epilogue; one thread per 8 outputs
__global__ __launch_bounds__(256) void splitk_epilogue_kernel(const ConvArgs a) {
  const bool glu = a.act == ACT_SILU_MUL;
  const int nc = glu ? a.N / 16 : a.N / 8;  // output chunks of 8 per row
  const long total = (long)a.M * nc;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const int m = (int)(q / nc), c = (int)(q - (q / nc) * nc);
    splitk_finish_chunk<false>(a, make_rsrc(nullptr, 0), m, glu ? c * 16 : c * 8, glu);
  }
}

struct TileCfg {
  int bm, bn, threads;
};
// id: 0 = heuristic; 1..8 = explicit (BM x BN, waves, LDS stages)
constexpr TileCfg kCfgs[] = {{0, 0, 0},       {128, 128, 256}, {128, 64, 256}, {64, 128, 256},
                             {64, 64, 256},   {128, 128, 512}, {64, 64, 256},  {128, 64, 512},
                             {64, 128, 512},  {64, 128, 512},  {128, 64, 512}, {64, 64, 256},
                             {128, 128, 512}, {128, 128, 512}, {128, 128, 512}, {64, 64, 256},
                             {128, 64, 256},  {64, 128, 256},  {128, 128, 256},
                             // 19, 23..28: deep rings (3-4 stages in flight); 20..22 = persistent kernel
                             {128, 128, 512}, {64, 64, 256},  {128, 64, 512}, {64, 128, 512},
                             {128, 128, 512}, {64, 128, 256}, {128, 64, 256}, {64, 64, 256},
                             {128, 128, 512}, {64, 128, 512},
                             // 29..31: 256-wide tiles for the large plain GEMMs (BERT projections, prefill)
                             {256, 128, 512}, {256, 128, 512}, {128, 256, 512}};
constexpr int kNumCfgs = 32;
// cfgs 13..19 and 23..26 stage K in 32-deep steps (BK = 32): not for the stem layout or the SiLU-mul epilogue
constexpr bool cfg_bk32(int c) { return (c >= 13 && c <= 19) || (c >= 23 && c <= 26); }

template <int MODE>
void launch_mode(int cfg, dim3 grid, hipStream_t st, const ConvArgs& a) {
  switch (cfg) {
    case 1: hipLaunchKernelGGL((conv_gemm_kernel<128, 128, 2, 2, 2, MODE>), grid, dim3(256), 0, st, a); break;
    case 2: hipLaunchKernelGGL((conv_gemm_kernel<128, 64, 2, 2, 3, MODE>), grid, dim3(256), 0, st, a); break;
    case 3: hipLaunchKernelGGL((conv_gemm_kernel<64, 128, 2, 2, 3, MODE>), grid, dim3(256), 0, st, a); break;
    case 5: hipLaunchKernelGGL((conv_gemm_kernel<128, 128, 4, 2, 3, MODE>), grid, dim3(512), 0, st, a); break;
    case 6: hipLaunchKernelGGL((conv_gemm_kernel<64, 64, 2, 2, 4, MODE>), grid, dim3(256), 0, st, a); break;
    case 7: hipLaunchKernelGGL((conv_gemm_kernel<128, 64, 4, 2, 3, MODE>), grid, dim3(512), 0, st, a); break;
    case 8: hipLaunchKernelGGL((conv_gemm_kernel<64, 128, 2, 4, 3, MODE>), grid, dim3(512), 0, st, a); break;
    // 2-stage variants: half the LDS ring -> more resident blocks for the latency-bound small-K layers
    case 9: hipLaunchKernelGGL((conv_gemm_kernel<64, 128, 2, 4, 2, MODE>), grid, dim3(512), 0, st, a); break;
    case 10: hipLaunchKernelGGL((conv_gemm_kernel<128, 64, 4, 2, 2, MODE>), grid, dim3(512), 0, st, a); break;
    case 11: hipLaunchKernelGGL((conv_gemm_kernel<64, 64, 2, 2, 2, MODE>), grid, dim3(256), 0, st, a); break;
    case 12: hipLaunchKernelGGL((conv_gemm_kernel<128, 128, 4, 2, 2, MODE>), grid, dim3(512), 0, st, a); break;
    // BK = 32 + multi-pass epilogue: 24-48 KB of LDS per block instead of 48-68 KB
    case 13: hipLaunchKernelGGL((conv_gemm_kernel<128, 128, 4, 2, 2, MODE, 32, 4>), grid, dim3(512), 0, st, a); break;
    case 14: hipLaunchKernelGGL((conv_gemm_kernel<128, 128, 4, 2, 3, MODE, 32, 2>), grid, dim3(512), 0, st, a); break;
    case 15: hipLaunchKernelGGL((conv_gemm_kernel<64, 64, 2, 2, 3, MODE, 32, 1>), grid, dim3(256), 0, st, a); break;
    case 16: hipLaunchKernelGGL((conv_gemm_kernel<128, 64, 2, 2, 3, MODE, 32, 1>), grid, dim3(256), 0, st, a); break;
    case 17: hipLaunchKernelGGL((conv_gemm_kernel<64, 128, 2, 2, 3, MODE, 32, 1>), grid, dim3(256), 0, st, a); break;
    case 18: hipLaunchKernelGGL((conv_gemm_kernel<128, 128, 2, 2, 3, MODE, 32, 2>), grid, dim3(256), 0, st, a); break;
    // deep rings: more K-steps of operands in flight per block (the latency-bound small-M layers)
    case 19: hipLaunchKernelGGL((conv_gemm_kernel<128, 128, 4, 2, 4, MODE, 32, 2>), grid, dim3(512), 0, st, a); break;
    case 23: hipLaunchKernelGGL((conv_gemm_kernel<128, 128, 4, 2, 5, MODE, 32, 2>), grid, dim3(512), 0, st, a); break;
    case 24: hipLaunchKernelGGL((conv_gemm_kernel<64, 128, 2, 2, 4, MODE, 32, 1>), grid, dim3(256), 0, st, a); break;
    case 25: hipLaunchKernelGGL((conv_gemm_kernel<128, 64, 2, 2, 4, MODE, 32, 1>), grid, dim3(256), 0, st, a); break;
    case 26: hipLaunchKernelGGL((conv_gemm_kernel<64, 64, 2, 2, 5, MODE, 32, 1>), grid, dim3(256), 0, st, a); break;
    case 27: hipLaunchKernelGGL((conv_gemm_kernel<128, 128, 4, 2, 4, MODE>), grid, dim3(512), 0, st, a); break;
    case 28: hipLaunchKernelGGL((conv_gemm_kernel<64, 128, 2, 4, 4, MODE>), grid, dim3(512), 0, st, a); break;
    case 29: hipLaunchKernelGGL((conv_gemm_kernel<256, 128, 4, 2, 2, MODE, 64, 2>), grid, dim3(512), 0, st, a); break;
    case 30: hipLaunchKernelGGL((conv_gemm_kernel<256, 128, 4, 2, 3, MODE, 64, 2>), grid, dim3(512), 0, st, a); break;
    case 31: hipLaunchKernelGGL((conv_gemm_kernel<128, 256, 2, 4, 2, MODE, 64, 2>), grid, dim3(512), 0, st, a); break;
    default: hipLaunchKernelGGL((conv_gemm_kernel<64, 64, 2, 2, 3, MODE>), grid, dim3(256), 0, st, a); break;
  }
}

// Heuristic tile choice: fill 256 CUs x 2 resident blocks, penalise padding waste and small tiles.
void choose_cfg(int M, int N, int K, int& cfg, int& splitk) {
  const float tile_eff[kNumCfgs] = {0.f,  1.0f, 0.86f, 0.86f, 0.68f, 1.0f, 0.68f, 0.86f, 0.86f, 0.86f,
                                    0.86f, 0.68f, 1.0f, 1.0f, 1.0f, 0.68f, 0.86f, 0.86f, 1.0f};
  float best = -1.f;
  int bc = 4;
  for (int c = 1; c <= 4; ++c) {
    const int bm = kCfgs[c].bm, bn = kCfgs[c].bn;
    const long tm = (M + bm - 1) / bm, tn = (N + bn - 1) / bn, tiles = tm * tn;
    const float pad = (float)M * N / ((float)tiles * bm * bn);
    const long waves = (tiles + 511) / 512;
    const float fill = (float)tiles / (float)(waves * 512);
    const float score = tile_eff[c] * pad * (tiles >= 256 ? fill : fill * 0.5f);
    if (score > best) {
      best = score;
      bc = c;
    }
  }
  cfg = bc;
  const long tiles = (long)((M + kCfgs[bc].bm - 1) / kCfgs[bc].bm) * ((N + kCfgs[bc].bn - 1) / kCfgs[bc].bn);
  splitk = 1;
  while (tiles * splitk < 384 && K / (splitk * 2) >= 256 && splitk < 8) splitk *= 2;
}

int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

template <int MODE>
void launch_persistent(int cfg, hipStream_t st, ConvArgs a) {
  set_fastdivs(a, cfg == 21 ? 64 : cfg == 22 ? 128 : 64);
  auto grid = [&](int bm, int bn, int per_cu) {
    const long T = (long)((a.M + bm - 1) / bm) * ((a.N + bn - 1) / bn);
    const long g = (long)num_cus() * per_cu;
    return dim3((unsigned)(T < g ? T : g));
  };
  switch (cfg) {
    case 21: hipLaunchKernelGGL((conv_gemm_persistent<128, 64, 4, 2, MODE>), grid(128, 64, 1), dim3(512), 0, st, a); break;
    case 22: hipLaunchKernelGGL((conv_gemm_persistent<64, 128, 2, 4, MODE>), grid(64, 128, 1), dim3(512), 0, st, a); break;
    default: hipLaunchKernelGGL((conv_gemm_persistent<64, 64, 2, 2, MODE>), grid(64, 64, 2), dim3(256), 0, st, a); break;
  }
}

// Split-K arrival counters: one zeroed array per HIP stream, reset by each tile's last arriver,
// so it is zero again whenever the next launch on that stream starts.  A launch captured into a
// hipGraph keeps the capture stream's array; that is safe under the same rule the split-K slabs
// (StreamWorkspace, keyed by stream) already follow: graphs captured on one stream are replayed on
// that stream only (the engine's per-slot streams).  Arrays are allocated outside capture only (the
// eager warm-up); a stream without one uses the separate reduce kernel.  MLS_SPLITK_INLAUNCH=0
// disables the in-launch path.
constexpr int kStreamCounters = 1 << 16;

int* splitk_counters(hipStream_t st, long ntiles) {
  static std::mutex mu;
  static std::unordered_map<hipStream_t, int*> arrays;
  static const bool enabled = [] {
    const char* e = getenv("MLS_SPLITK_INLAUNCH");
    return !(e && e[0] == '0');
  }();
  if (!enabled || ntiles <= 0 || ntiles > kStreamCounters) return nullptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> g(mu);
  auto it = arrays.find(st);
  if (it != arrays.end()) return it->second;
  if (cs != hipStreamCaptureStatusNone) return nullptr;  // no allocation inside a capture
  int* p = nullptr;
  if (hipMalloc(&p, kStreamCounters * sizeof(int)) != hipSuccess) return nullptr;
  if (hipMemset(p, 0, kStreamCounters * sizeof(int)) != hipSuccess) {
    (void)hipFree(p);
    return nullptr;
  }
  arrays[st] = p;
  return p;
}

// defer_split != null: leave the split-K fp32 slabs [split][M][N] in `ws` for the caller to reduce
// (mls_splitk_add_rmsnorm: the reduce fused with the next residual add + RMSNorm) -- no in-launch or
// separate reduce, no bf16 output; *defer_split = the split used.  MLS_UNSUPPORTED (nothing launched)
// when the shape would not split.
int launch_conv(ConvArgs a, int mode, int cfg, int splitk, size_t ws_bytes, hipStream_t st,
                int* defer_split = nullptr) {
  if (a.act == ACT_SILU_MUL && a.N % 16 != 0) return MLS_BAD_ARG;
  if (a.N % 8 != 0 || a.M <= 0 || a.N <= 0 || a.K <= 0 || a.K % 8 != 0) return MLS_BAD_ARG;
  {
    const size_t ob = ((size_t)(a.M - 1) * a.ldo + (a.act == ACT_SILU_MUL ? a.N / 2 : a.N)) * 2;
    if (ob >= 0x7FFFFFFFull) return MLS_UNSUPPORTED;
    a.o_bytes = (uint32_t)ob;
  }
  if (cfg >= 20 && cfg <= 22 && mode == MODE_DUAL) cfg = 0;  // persistent kernel: no dual mode
  if (defer_split && cfg >= 20 && cfg <= 22) return MLS_UNSUPPORTED;  // persistent: never splits
  if (cfg >= 20 && cfg <= 22) {
    if (a.act != ACT_SILU_MUL && (splitk <= 1)) {
      a.splitk = 1;
      a.kchunk = a.K;
      a.dbg = g_dbg_flags;
      const size_t rb = a.res ? ((size_t)(a.M - 1) * a.ldr + a.N) * 2 : 0;
      if (rb >= 0x7FFFFFFFull) return MLS_UNSUPPORTED;
      a.r_bytes = (uint32_t)rb;
      switch (mode) {
        case MODE_1X1: launch_persistent<MODE_1X1>(cfg, st, a); break;
        case MODE_GENERIC: launch_persistent<MODE_GENERIC>(cfg, st, a); break;
        case MODE_STEM: launch_persistent<MODE_STEM>(cfg, st, a); break;
        default: return MLS_UNSUPPORTED;
      }
      return (int)hipGetLastError();
    }
    cfg = 4;  // persistent kernel has no split-K / SiLU-mul: fall back
  }
  int acfg = 0, asplit = 1;
  choose_cfg(a.M, a.N, a.K, acfg, asplit);
  if (cfg <= 0 || cfg >= kNumCfgs) cfg = acfg;
  if (cfg_bk32(cfg) && (mode == MODE_STEM || a.act == ACT_SILU_MUL)) cfg = acfg;
  if (splitk <= 0) splitk = asplit;
  // K per split: multiple of BK (so MODE_GENERIC steps never straddle a tap)
  int kchunk = ((a.K + splitk - 1) / splitk + BK - 1) / BK * BK;
  splitk = (a.K + kchunk - 1) / kchunk;
  if (splitk > 1 && (a.ws == nullptr || ws_bytes < (size_t)splitk * a.M * a.N * sizeof(float))) {
    // not enough workspace: fall back to no split
    splitk = 1;
    kchunk = (a.K + BK - 1) / BK * BK;
  }
  a.splitk = splitk;
  a.kchunk = kchunk;
  a.dbg = g_dbg_flags;
  {
    const size_t rb = a.res ? ((size_t)(a.M - 1) * a.ldr + a.N) * 2 : 0;
    if (rb >= 0x7FFFFFFFull) return MLS_UNSUPPORTED;
    a.r_bytes = (uint32_t)rb;
  }
  const int bm = kCfgs[cfg].bm, bn = kCfgs[cfg].bn;
  const long otiles = (long)((a.M + bm - 1) / bm) * ((a.N + bn - 1) / bn);
  const long ntiles = otiles * splitk;
  if (ntiles > 0x7fffffffL) return MLS_BAD_ARG;
  a.cnt = nullptr;
  if (defer_split) {
    if (splitk <= 1 || a.act != ACT_NONE || a.res || a.scale || a.bias) return MLS_UNSUPPORTED;
    *defer_split = splitk;
  } else if (splitk > 1 && (size_t)splitk * a.M * a.N * sizeof(float) < 0x7FFFFFF0ull) {
    a.cnt = splitk_counters(st, otiles);
    a.ws_bytes = (uint32_t)((size_t)splitk * a.M * a.N * sizeof(float));
  }
  dim3 grid((unsigned)ntiles);
  set_fastdivs(a, bn);
  switch (mode) {
    case MODE_1X1: launch_mode<MODE_1X1>(cfg, grid, st, a); break;
    case MODE_GENERIC: launch_mode<MODE_GENERIC>(cfg, grid, st, a); break;
    case MODE_STEM: launch_mode<MODE_STEM>(cfg, grid, st, a); break;
    case MODE_DUAL: launch_mode<MODE_DUAL>(cfg, grid, st, a); break;
    default: return MLS_UNSUPPORTED;
  }
  if (splitk > 1 && a.cnt == nullptr && !defer_split) {
    const long total = (long)a.M * (a.N / 8);
    int blocks = (int)((total + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(splitk_epilogue_kernel, dim3(blocks), dim3(256), 0, st, a);
  }
  return (int)hipGetLastError();
}

}  // namespace

// Per-stream split-K arrival counters for other translation units (conv3x3_halo.hip): the same
// arrays, so kernels of different kinds on one stream share them (each launch leaves them zero).
int* mls_stream_splitk_counters(void* stream, long ntiles) { return splitk_counters((hipStream_t)stream, ntiles); }

extern "C" {

// NHWC conv2d with fused epilogue. Weights [Cout][KH][KW][Cin] bf16; for the stem mode
// (Cin == 4, KH > 1) the weights are [Cout][KH][8][4] (KW zero-padded to 8).
int mls_conv2d(const void* x, const void* w, const float* scale, const float* bias, const void* res, void* out,
               void* ws, size_t ws_bytes, int B, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
               int pad, int act, int cfg, int splitk, void* stream) {
  ConvArgs a{};
  a.x = (const bf16*)x;
  a.w = (const bf16*)w;
  a.scale = scale;
  a.bias = bias;
  a.res = (const bf16*)res;
  a.out = (bf16*)out;
  a.ws = (float*)ws;
  a.B = B; a.H = H; a.W = W; a.Cin = Cin; a.N = Cout; a.KH = KH; a.KW = KW; a.stride = stride; a.pad = pad;
  a.Ho = (H + 2 * pad - KH) / stride + 1;
  a.Wo = (W + 2 * pad - KW) / stride + 1;
  a.M = B * a.Ho * a.Wo;
  a.act = act;
  a.ldo = Cout;
  a.ldr = Cout;
  const size_t xb = (size_t)B * H * W * Cin * 2;
  if (xb >= 0x7FFFFFFFull) return MLS_UNSUPPORTED;  // 32-bit buffer offsets
  a.x_bytes = (uint32_t)xb;
  int mode;
  if (Cin == 4 && KH > 1) {
    // pre-padded image (the normalise kernel writes the zero border): no bounds checks;
    // taps up to KW padded to 8 must stay inside the row
    if (KW > 8 || pad != 0 || (a.Wo - 1) * stride + 8 > W || (a.Ho - 1) * stride + 8 > H) return MLS_UNSUPPORTED;
    mode = MODE_STEM;
    a.K = KH * 32;
  } else if (KH == 1 && KW == 1 && pad == 0) {
    mode = MODE_1X1;
    a.K = Cin;
  } else if (Cin % 64 == 0 && KH * KW <= 32) {
    mode = MODE_GENERIC;
    a.K = KH * KW * Cin;
  } else {
    return MLS_UNSUPPORTED;
  }
  const size_t wb = (size_t)Cout * a.K * 2;
  if (wb >= 0x7FFFFFFFull) return MLS_UNSUPPORTED;
  a.w_bytes = (uint32_t)wb;
  return launch_conv(a, mode, cfg, splitk, ws_bytes, (hipStream_t)stream);
}

// mls_conv2d + the fused global average pool of the output: pool [B][Cout] fp32 += mean over the
// Ho*Wo pixels of each image (the caller zeroes it; ops.fc_head does so after reading it);
// pool_only: `out` is not written (may be null).  No split-K, no persistent config.
int mls_conv2d_pool(const void* x, const void* w, const float* scale, const float* bias, const void* res, void* out,
                    float* pool, int pool_only, int B, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                    int pad, int act, int cfg, void* stream) {
  if (!pool || act == ACT_SILU_MUL || (!out && !pool_only)) return MLS_BAD_ARG;
  if (cfg >= 20 && cfg <= 22) cfg = 0;
  ConvArgs a{};
  a.x = (const bf16*)x;
  a.w = (const bf16*)w;
  a.scale = scale;
  a.bias = bias;
  a.res = (const bf16*)res;
  a.out = (bf16*)out;
  a.B = B; a.H = H; a.W = W; a.Cin = Cin; a.N = Cout; a.KH = KH; a.KW = KW; a.stride = stride; a.pad = pad;
  a.Ho = (H + 2 * pad - KH) / stride + 1;
  a.Wo = (W + 2 * pad - KW) / stride + 1;
  a.M = B * a.Ho * a.Wo;
  a.act = act;
  a.ldo = Cout;
  a.ldr = Cout;
  a.pool = pool;
  a.pool_hw = a.Ho * a.Wo;
  a.pool_scale = 1.f / (float)(a.Ho * a.Wo);
  a.pool_only = pool_only;
  const size_t xb = (size_t)B * H * W * Cin * 2;
  if (xb >= 0x7FFFFFFFull) return MLS_UNSUPPORTED;
  a.x_bytes = (uint32_t)xb;
  int mode;
  if (KH == 1 && KW == 1 && pad == 0) {
    mode = MODE_1X1;
    a.K = Cin;
  } else if (Cin % 64 == 0 && KH * KW <= 32 && Cin != 4) {
    mode = MODE_GENERIC;
    a.K = KH * KW * Cin;
  } else {
    return MLS_UNSUPPORTED;
  }
  const size_t wb = (size_t)Cout * a.K * 2;
  if (wb >= 0x7FFFFFFFull) return MLS_UNSUPPORTED;
  a.w_bytes = (uint32_t)wb;
  return launch_conv(a, mode, cfg, 1, 0, (hipStream_t)stream);
}

// out = act(conv1x1(y, W[:, :Cin1]) + conv1x1_stride2(x, W[:, Cin1:]) + bias): y [B][Ho][Wo][Cin1],
// x [B][H2][W2][Cin2] with Ho = ceil(H2 / stride2); W [Cout][Cin1 + Cin2]; Cin1 % 64 == 0.
int mls_conv2d_dual(const void* y, const void* x, const void* w, const float* bias, void* out, void* ws,
                    size_t ws_bytes, int B, int Ho, int Wo, int Cin1, int H2, int W2, int Cin2, int stride2, int Cout,
                    int act, int cfg, int splitk, void* stream) {
  if (Cin1 % 64 || Cin2 % 8 || stride2 < 1 || (Ho - 1) * stride2 >= H2 || (Wo - 1) * stride2 >= W2) return MLS_BAD_ARG;
  ConvArgs a{};
  a.x = (const bf16*)y;
  a.x2 = (const bf16*)x;
  a.w = (const bf16*)w;
  a.bias = bias;
  a.out = (bf16*)out;
  a.ws = (float*)ws;
  a.B = B; a.H = Ho; a.W = Wo; a.Cin = Cin1; a.Ho = Ho; a.Wo = Wo; a.N = Cout; a.KH = 1; a.KW = 1;
  a.stride = 1; a.pad = 0;
  a.H2 = H2; a.W2 = W2; a.Cin2 = Cin2; a.stride2 = stride2; a.K1 = Cin1;
  a.M = B * Ho * Wo;
  a.K = Cin1 + Cin2;
  a.act = act;
  a.ldo = Cout;
  a.ldr = Cout;
  const size_t yb = (size_t)a.M * Cin1 * 2, xb = (size_t)B * H2 * W2 * Cin2 * 2, wb = (size_t)Cout * a.K * 2;
  if (yb >= 0x7FFFFFFFull || xb >= 0x7FFFFFFFull || wb >= 0x7FFFFFFFull) return MLS_UNSUPPORTED;
  a.x_bytes = (uint32_t)yb;
  a.x2_bytes = (uint32_t)xb;
  a.w_bytes = (uint32_t)wb;
  return launch_conv(a, MODE_DUAL, cfg, splitk, ws_bytes, (hipStream_t)stream);
}

// out[M][N] = act(A[M][K] . W[N][K]^T * scale + bias (+ res[M][N]))
int mls_gemm(const void* A, const void* W, const float* scale, const float* bias, const void* res, void* out, void* ws,
             size_t ws_bytes, int M, int N, int K, int act, int cfg, int splitk, void* stream) {
  ConvArgs a{};
  a.x = (const bf16*)A;
  a.w = (const bf16*)W;
  a.scale = scale;
  a.bias = bias;
  a.res = (const bf16*)res;
  a.out = (bf16*)out;
  a.ws = (float*)ws;
  a.B = M; a.H = 1; a.W = 1; a.Cin = K; a.Ho = 1; a.Wo = 1; a.N = N; a.KH = 1; a.KW = 1; a.stride = 1; a.pad = 0;
  a.M = M;
  a.K = K;
  a.act = act;
  a.ldo = act == ACT_SILU_MUL ? N / 2 : N;
  a.ldr = N;
  const size_t xb = (size_t)M * K * 2, wb = (size_t)N * K * 2;
  if (xb >= 0x7FFFFFFFull || wb >= 0x7FFFFFFFull) return MLS_UNSUPPORTED;
  a.x_bytes = (uint32_t)xb;
  a.w_bytes = (uint32_t)wb;
  return launch_conv(a, MODE_1X1, cfg, splitk, ws_bytes, (hipStream_t)stream);
}

// out-less GEMM: A [M][K] . W[N][K]^T as split-K fp32 slabs [split][M][N] in ws, reduced by the
// caller (mls_splitk_add_rmsnorm).  *split_used = the split; MLS_UNSUPPORTED when it would be 1.
int mls_gemm_slabs(const void* A, const void* W, void* ws, size_t ws_bytes, int M, int N, int K, int cfg, int splitk,
                   int* split_used, void* stream) {
  if (!split_used || !ws) return MLS_BAD_ARG;
  ConvArgs a{};
  a.x = (const bf16*)A;
  a.w = (const bf16*)W;
  a.ws = (float*)ws;
  a.B = M; a.H = 1; a.W = 1; a.Cin = K; a.Ho = 1; a.Wo = 1; a.N = N; a.KH = 1; a.KW = 1; a.stride = 1; a.pad = 0;
  a.M = M;
  a.K = K;
  a.act = ACT_NONE;
  a.ldo = N;
  a.ldr = N;
  const size_t xb = (size_t)M * K * 2, wb = (size_t)N * K * 2;
  if (xb >= 0x7FFFFFFFull || wb >= 0x7FFFFFFFull) return MLS_UNSUPPORTED;
  a.x_bytes = (uint32_t)xb;
  a.w_bytes = (uint32_t)wb;
  return launch_conv(a, MODE_1X1, cfg, splitk, ws_bytes, (hipStream_t)stream, split_used);
}

// the tile config / split-K the heuristic would pick (for the autotuner and tests)
int mls_gemm_heuristic(int M, int N, int K, int* cfg, int* splitk) {
  choose_cfg(M, N, K, *cfg, *splitk);
  return 0;
}

int mls_gemm_num_cfgs() { return kNumCfgs; }

void mls_set_debug_flags(int flags) { g_dbg_flags = flags; }

}  // extern "C"
