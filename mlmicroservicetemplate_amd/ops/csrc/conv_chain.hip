// Bottleneck boundary chain: one ResNet bottleneck's last 1x1 conv (+ residual + ReLU) and the NEXT
// bottleneck's first 1x1 conv in ONE kernel, so the block output y -- the widest tensor of the
// network (56x56x256 / 28x28x512 at bs=32: 51 / 26 MB) -- is written once and never re-read:
//
//   y  = relu(A1 . W3^T + b3 (+ res))      [M][N1]   stored (the next block's residual)
//   t1 = relu(y  . W1^T + b1)              [M][N2]   stored (the next block's conv2 input)
//
// A1 is the conv3 input [M][Ka] or, for a stage's first block, the dual operand [t2 | x_strided]
// (conv3 + downsample projection as one reduction, conv_gemm.hip MODE_DUAL) with no residual.
//
// Why: at bs = 32 the layer1 / layer2 1x1 convs run at 4-5 TB/s of HBM under concurrent streams
// (docs/PERF_NOTES.md, r2 PMC): bytes, not MFMAs, are their cost.  Unchained, y is written by conv3
// and read back by the next conv1 (+51 MB per layer1 boundary); here it stays in LDS.
//
// Structure (per block: one BM-row tile, 8 waves as 4 (M) x 2 (N)):
//   * A1 tile staged once into LDS (KS 64-wide slabs, 128-B rows, 16-B chunks XOR-swizzled by
//     row & 7 on the SOURCE address so the LDS-DMA stays lane-linear; conflict-free ds_read_b128).
//   * loop over the N1 / 64 output-channel chunks j, a 2-deep LDS-DMA ring of stages
//     {W3 rows j*64.. (64 x K1), W1 columns j*64.. (N2 x 64), residual chunk (BM x 64)}, stage j+1
//     in flight during chunk j (counted vmcnt + raw s_barrier, never a full drain in the loop):
//       GEMM1  acc1[BM x 64] = A1 . W3_j^T                       (MFMA 16x16x32 bf16)
//       pass 1 y = relu(acc1 + b3 + res) -> bf16, IN PLACE over the residual chunk in LDS
//       y chunk -> HBM with 16-B buffer stores
//       GEMM2  acc2[BM x N2] += y_j . W1_j^T   (the y chunk in LDS is exactly GEMM2's K-slab j)
//   * epilogue: t1 = relu(acc2 + b1) -> bf16 through LDS -> 16-B stores.
// Numerics: y rounds once exactly as conv_gemm.hip's epilogue (acc + bias + res, ReLU, bf16); t1
// accumulates the same K order in fp32.
#include "common.h"
#include "fastdiv.h"

namespace {

#define LDS3 __attribute__((address_space(3)))

MLS_DEV void glds16(rsrc_t r, char* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDS3 void*)lds, 16, voff, soff, 0, 0);
}

typedef unsigned int u32x4v __attribute__((__vector_size__(16)));

// SW (template parameter): MFMA operand order.  true: D = W . A^T, so a lane's 4 accumulators are
// 4 consecutive output channels of one row -- pass 1 reads the residual and writes y as one 8-B
// LDS access per fragment (instead of four 2-B read-modify-writes), the t1 epilogue parks 8 B per
// fragment, and the biases come from wave-uniform scalar loads (no VGPR-resident bias table, no
// VMEM op beside the DMA ring); false: D = A . W^T.  Per boundary from the per-call A/B
// (profiles/r3_swap_epilogue_component_costs.jsonl): the single-slab (KS = 1) layer1 boundaries
// take SW (layer1.1 -> 1.2: 27.4 -> 23.2 us co-running), the others measured level or slower.
// MLS_CHAIN_SWAP=0/1 at build time forces one order everywhere (A/B builds).
#define CONST4 __attribute__((address_space(4)))

// the 4 biases of lane group fq in the 16 output channels starting at the wave-uniform nt0
MLS_DEV f32x4 bias4(const float* b, int nt0, int fq) {
  if (!b) return f32x4{0.f, 0.f, 0.f, 0.f};
  const CONST4 f32x4* bp = (const CONST4 f32x4*)(b + nt0);
  const f32x4 b0 = bp[0], b1 = bp[1], b2 = bp[2], b3 = bp[3];
  return fq == 0 ? b0 : fq == 1 ? b1 : fq == 2 ? b2 : b3;
}

struct ChainArgs {
  const bf16* a1;   // [M][Ka]            (conv3 input, stride 1)
  const bf16* a2;   // [B][H2][W2][Kb]    (dual: the block input, sampled at stride2) or null
  const bf16* w3;   // [N1][Ka + Kb]
  const float* b3;  // [N1]
  const bf16* res;  // [M][N1] or null
  bf16* y;          // [M][N1]
  const bf16* w1;   // [N2][N1]
  const float* b1;  // [N2]
  bf16* t1;         // [M][N2]
  int M, Ka, Kb, N1, N2;
  int Ho, Wo, H2, W2, stride2;  // dual geometry (M = B * Ho * Wo)
  FastDiv fd_howo, fd_wo;       // Ho * Wo, Wo (fastdiv.h)
  uint32_t a1_bytes, a2_bytes, w3_bytes, res_bytes, y_bytes, w1_bytes, t1_bytes;
};

// 16-B chunk swizzle of an LDS image row: 128-B rows (8 chunks): chunk ^ (r & 7); 64-B rows (4
// chunks): chunk ^ f(r & 7), f = (r0 | r2 << 1) -- conflict-free for the 16x16x32 fragment reads
// (conv_gemm.hip row_swz).  The LDS-DMA writes lane-linearly, so the swizzle goes on the SOURCE.
template <int CPR>
MLS_DEV int row_swz(int r) {
  if constexpr (CPR == 8) return r & 7;
  else return (r & 1) | ((r >> 1) & 2);
}

// KS = (Ka + Kb) / 64 A1 slabs; KSA = Ka / 64 of them from a1, the rest from a2 (dual).  CW = the
// output-channel chunk of GEMM1 = the K slab of GEMM2 (64, or 32 where the weights of a 64-wide
// stage would not fit the LDS next to the A tile: layer2 -> 3 and layer3).  N1 is a template
// parameter so the chunk loop unrolls and every bias lives in registers, loaded before the first
// LDS-DMA: a plain global load consumed beside in-flight DMA makes hipcc wait vmcnt(0) and drain
// the ring (cdna_hip_programming.md §5, "Projection GEMM" item 4(b)).  OCC = waves per SIMD the
// register allocation must allow: 4 where the LDS footprint lets two blocks share a CU (<= 80 KB).
template <int BM, int KS, int N1, int N2, int CW, int OCC, bool SW>
__global__ __launch_bounds__(512, OCC) void conv_chain_kernel(const ChainArgs a) {
  constexpr int NW = 8, NT = 512, WM = 4, WN = 2;
  constexpr int WTM = BM / WM, TM = WTM / 16;  // GEMM1 / GEMM2 wave rows
  constexpr int TN = CW / WN / 16;             // GEMM1 column fragments per wave
  constexpr int TN2 = N2 / WN / 16;            // GEMM2 column fragments per wave
  constexpr int CPR = CW / 8;                  // 16-B chunks per row of the W1 / residual / y images
  constexpr int RPP = 64 / CPR;                // rows of those images per 1-KiB DMA piece
  constexpr int A1_BYTES = BM * KS * 128;
  constexpr int W3_BYTES = CW * KS * 128;
  constexpr int W1_BYTES = N2 * CW * 2;
  constexpr int R_BYTES = BM * CW * 2;
  constexpr int STAGE = W3_BYTES + W1_BYTES + R_BYTES;
  constexpr int EPI_BYTES = BM * N2 * 2;
  constexpr int RING = A1_BYTES + 2 * STAGE;
  constexpr int LDS_BYTES = RING > EPI_BYTES ? RING : EPI_BYTES;
  constexpr int A1_PW = BM / 8 * KS / NW;  // 1-KiB DMA pieces per wave
  constexpr int W3_PW = CW / 8 * KS / NW;
  constexpr int W1_PW = N2 / RPP / NW;
  constexpr int R_PW = BM / RPP / NW;
  constexpr int Y_ST = BM * CPR / NT;     // 16-B y stores per thread per chunk
  constexpr int T_ST = BM * N2 / 8 / NT;  // 16-B t1 stores per thread
  constexpr int NJ = N1 / CW;
  static_assert(TM >= 1 && TN >= 1 && TN2 >= 1 && (CW == 64 || CW == 32), "tile");
  static_assert(A1_PW * NW * 8 == BM * KS && W3_PW * NW * 8 == CW * KS, "A1 / W3 DMA split");
  static_assert(W1_PW * NW * RPP == N2 && R_PW * NW * RPP == BM, "W1 / residual DMA split");
  static_assert(Y_ST * NT == BM * CPR && T_ST * NT == BM * N2 / 8, "epilogue split");
  static_assert(LDS_BYTES <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int fr = lane & 15, fq = lane >> 4;
  const int m0 = xcd_remap(blockIdx.x, gridDim.x) * BM;
  const int K1 = a.Ka + a.Kb, KSA = a.Ka / 64;
  const bool has_res = a.res != nullptr;

  // (original order) biases of every column this lane touches, before any DMA is in flight
  float b3v[SW ? 1 : NJ][TN], b1v[TN2];
  if constexpr (!SW) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int jn = 0; jn < TN; ++jn) b3v[j][jn] = a.b3 ? a.b3[j * CW + wn * (CW / 2) + jn * 16 + fr] : 0.f;
#pragma unroll
    for (int jn = 0; jn < TN2; ++jn) b1v[jn] = a.b1 ? a.b1[wn * (N2 / 2) + jn * 16 + fr] : 0.f;
  }

  // DMA lane geometry.  128-B rows (A1, W3): 8 rows x 8 chunks per piece; CW-wide rows (W1,
  // residual): RPP rows x CPR chunks.  LDS chunk c of row r holds the logical chunk c ^ swz(r).
  const int r8 = lane >> 3, lc = (lane & 7) ^ r8;
  const int rq = lane / CPR, lq = (lane % CPR) ^ row_swz<CPR>(rq);

  const rsrc_t a1r = make_rsrc(a.a1, a.a1_bytes);
  const rsrc_t a2r = make_rsrc(a.a2, a.a2_bytes);
  const rsrc_t w3r = make_rsrc(a.w3, a.w3_bytes);
  const rsrc_t w1r = make_rsrc(a.w1, a.w1_bytes);
  const rsrc_t rr = make_rsrc(a.res, a.res_bytes);
  const rsrc_t yr = make_rsrc(a.y, a.y_bytes);
  const rsrc_t tr = make_rsrc(a.t1, a.t1_bytes);

  char* const sA1 = smem;
  auto stage_base = [&](int buf) { return smem + A1_BYTES + buf * STAGE; };

  // ---- A1 tile: slab s, row block rb; wave w issues pieces q = w * A1_PW + i
#pragma unroll
  for (int i = 0; i < A1_PW; ++i) {
    const int q = wid * A1_PW + i;
    const int s = q / (BM / 8), rb = q - s * (BM / 8);
    const int m = m0 + rb * 8 + r8;
    char* dst = sA1 + q * 1024;
    if (s < KSA) {
      glds16(a1r, dst, m < a.M ? (m * a.Ka + s * 64 + lc * 8) * 2 : OOB, 0);
    } else {  // dual operand: row m of the output grid samples the block input at stride2
      int off = OOB;
      if (m < a.M) {
        const int b = fastdiv(m, a.fd_howo), rem = m - b * (a.Ho * a.Wo);
        const int oh = fastdiv(rem, a.fd_wo), ow = rem - oh * a.Wo;
        off = (((b * a.H2 + oh * a.stride2) * a.W2 + ow * a.stride2) * a.Kb + (s - KSA) * 64 + lc * 8) * 2;
      }
      glds16(a2r, dst, off, 0);
    }
  }

  auto issue = [&](int j, int buf) {
    char* sW3 = stage_base(buf);
    char* sW1 = sW3 + W3_BYTES;
    char* sR = sW1 + W1_BYTES;
#pragma unroll
    for (int i = 0; i < W3_PW; ++i) {  // W3 rows j*CW + rb*8 + r8 of K slab s ([KS][CW][64] image)
      const int q = wid * W3_PW + i;
      const int s = q / (CW / 8), rb = q - s * (CW / 8);
      glds16(w3r, sW3 + q * 1024, ((j * CW + rb * 8 + r8) * K1 + s * 64 + lc * 8) * 2, 0);
    }
#pragma unroll
    for (int i = 0; i < W1_PW; ++i) {  // W1 rows n2 = q*RPP + rq, columns j*CW..
      const int q = wid * W1_PW + i;
      glds16(w1r, sW1 + q * 1024, ((q * RPP + rq) * N1 + j * CW + lq * 8) * 2, 0);
    }
    if (has_res) {
#pragma unroll
      for (int i = 0; i < R_PW; ++i) {
        const int q = wid * R_PW + i;
        const int m = m0 + q * RPP + rq;
        glds16(rr, sR + q * 1024, m < a.M ? (m * N1 + j * CW + lq * 8) * 2 : OOB, 0);
      }
    }
  };
  issue(0, 0);

  f32x4 acc2[TM][TN2];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int jn = 0; jn < TN2; ++jn) acc2[i][jn] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    // stage j landed: the only younger VMEM ops are chunk j-1's y stores
    if (j == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // the biases are retired too: pin their first use here, before stage 1 is issued
      if constexpr (!SW) {
#pragma unroll
        for (int jj = 0; jj < NJ; ++jj)
#pragma unroll
          for (int jn = 0; jn < TN; ++jn) asm volatile("" ::"v"(b3v[jj][jn]));
#pragma unroll
        for (int jn = 0; jn < TN2; ++jn) asm volatile("" ::"v"(b1v[jn]));
      }
    } else {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(Y_ST) : "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (j + 1 < NJ) issue(j + 1, (j + 1) & 1);
    char* sW3 = stage_base(j & 1);
    char* sW1 = sW3 + W3_BYTES;
    char* sR = sW1 + W1_BYTES;

    // ---- GEMM1: acc1[BM x CW] = A1 . W3_j^T
    f32x4 acc1[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int jn = 0; jn < TN; ++jn) acc1[i][jn] = f32x4{0.f, 0.f, 0.f, 0.f};
    const uint4* A1s = reinterpret_cast<const uint4*>(sA1);
    const uint4* W3s = reinterpret_cast<const uint4*>(sW3);
#pragma unroll
    for (int kk = 0; kk < 2 * KS; ++kk) {
      const int s = kk >> 1, ch = fq + 4 * (kk & 1);
      bf16x8 af[TM], bfv[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * WTM + i * 16 + fr;
        af[i] = __builtin_bit_cast(bf16x8, A1s[s * BM * 8 + r * 8 + (ch ^ (r & 7))]);
      }
#pragma unroll
      for (int jn = 0; jn < TN; ++jn) {
        const int n = wn * (CW / 2) + jn * 16 + fr;
        bfv[jn] = __builtin_bit_cast(bf16x8, W3s[s * CW * 8 + n * 8 + (ch ^ (n & 7))]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int jn = 0; jn < TN; ++jn)
          acc1[i][jn] = SW ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfv[jn], af[i], acc1[i][jn], 0, 0, 0)
                                       : __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfv[jn], acc1[i][jn], 0, 0, 0);
    }

    // ---- pass 1: y = relu(acc1 + b3 (+ res)) -> bf16, in place over the residual chunk
    if constexpr (SW) {
#pragma unroll
      for (int jn = 0; jn < TN; ++jn) {
        const int nt0 = wn * (CW / 2) + jn * 16, col = nt0 + fq * 4;  // col % 8 in {0, 4}: 8 B in one chunk
        const f32x4 bb = bias4(a.b3, j * CW + nt0, fq);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = wm * WTM + i * 16 + fr;
          uint2* p = reinterpret_cast<uint2*>(sR + row * (CW * 2) + (((col >> 3) ^ row_swz<CPR>(row)) << 4) +
                                              (col & 7) * 2);
          float rs[4] = {0.f, 0.f, 0.f, 0.f};
          if (has_res) {
            const bf16x4 rv = __builtin_bit_cast(bf16x4, *p);
#pragma unroll
            for (int r = 0; r < 4; ++r) rs[r] = (float)rv[r];
          }
          bf16x4 q;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float e = acc1[i][jn][r];  // through a named float (ext-vector element bit-cast hazard)
            q[r] = (bf16)fmaxf(e + bb[r] + rs[r], 0.f);
          }
          *p = __builtin_bit_cast(uint2, q);
        }
      }
    } else
#pragma unroll
    for (int jn = 0; jn < TN; ++jn) {
      const int col = wn * (CW / 2) + jn * 16 + fr;
      const float bb = b3v[j][jn];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = wm * WTM + i * 16 + fq * 4 + r;
          bf16* p = reinterpret_cast<bf16*>(sR + row * (CW * 2) + (((col >> 3) ^ row_swz<CPR>(row)) << 4) +
                                            (col & 7) * 2);
          const float e = acc1[i][jn][r];  // through a named float (ext-vector element bit-cast hazard)
          float v = e + bb;
          if (has_res) v += (float)*p;
          *p = (bf16)fmaxf(v, 0.f);
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();

    // ---- y chunk -> HBM (16-B rows), issued before GEMM2 so the stores drain under its MFMAs
#pragma unroll
    for (int it = 0; it < Y_ST; ++it) {
      const int q = tid + it * NT;
      const int row = q / CPR, c = q % CPR;
      const uint4 v = *reinterpret_cast<const uint4*>(sR + row * (CW * 2) + ((c ^ row_swz<CPR>(row)) << 4));
      const int m = m0 + row;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, v), yr,
                                             m < a.M ? (m * N1 + j * CW + c * 8) * 2 : OOB, 0, 0);
    }

    // ---- GEMM2: acc2[BM x N2] += y_j . W1_j^T
    const uint4* Ys = reinterpret_cast<const uint4*>(sR);
    const uint4* W1s = reinterpret_cast<const uint4*>(sW1);
#pragma unroll
    for (int kk = 0; kk < CW / 32; ++kk) {
      const int ch = fq + 4 * kk;
      bf16x8 af[TM], bfv[TN2];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * WTM + i * 16 + fr;
        af[i] = __builtin_bit_cast(bf16x8, Ys[r * CPR + (ch ^ row_swz<CPR>(r))]);
      }
#pragma unroll
      for (int jn = 0; jn < TN2; ++jn) {
        const int n = wn * (N2 / 2) + jn * 16 + fr;
        bfv[jn] = __builtin_bit_cast(bf16x8, W1s[n * CPR + (ch ^ row_swz<CPR>(n))]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int jn = 0; jn < TN2; ++jn)
          acc2[i][jn] = SW ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfv[jn], af[i], acc2[i][jn], 0, 0, 0)
                                       : __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfv[jn], acc2[i][jn], 0, 0, 0);
    }
  }

  // ---- epilogue: t1 = relu(acc2 + b1) -> bf16 tile in LDS -> 16-B stores
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // every wave is done reading the ring
  constexpr int TPR = N2 / 8;    // 16-B chunks per t1 row
  bf16* to = reinterpret_cast<bf16*>(smem);
  if constexpr (SW) {
#pragma unroll
    for (int jn = 0; jn < TN2; ++jn) {
      const int nt0 = wn * (N2 / 2) + jn * 16, col = nt0 + fq * 4;
      const f32x4 bb = bias4(a.b1, nt0, fq);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WTM + i * 16 + fr;
        bf16x4 q;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = acc2[i][jn][r];
          q[r] = (bf16)fmaxf(e + bb[r], 0.f);
        }
        *reinterpret_cast<uint2*>(to + row * N2 + ((((col >> 3) ^ (row & 7))) << 3) + (col & 7)) =
            __builtin_bit_cast(uint2, q);
      }
    }
  } else
#pragma unroll
  for (int jn = 0; jn < TN2; ++jn) {
    const int col = wn * (N2 / 2) + jn * 16 + fr;
    const float bb = b1v[jn];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * WTM + i * 16 + fq * 4 + r;
        const float e = acc2[i][jn][r];
        // chunk swizzle by row (TPR >= 8) keeps the 16-lane column groups on distinct banks
        to[row * N2 + ((((col >> 3) ^ (row & 7))) << 3) + (col & 7)] = (bf16)fmaxf(e + bb, 0.f);
      }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int it = 0; it < T_ST; ++it) {
    const int q = tid + it * NT;
    const int row = q / TPR, c = q - (q / TPR) * TPR;
    const uint4 v = *reinterpret_cast<const uint4*>(to + row * N2 + ((c ^ (row & 7)) << 3));
    const int m = m0 + row;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, v), tr, m < a.M ? (m * a.N2 + c * 8) * 2 : OOB,
                                           0, 0);
  }
}

// The ResNet-50 boundaries (BM = 128):          KS   N1   N2  CW
//   layer1.0 (dual) -> layer1.1                  2   256   64  64
//   layer1.1 -> layer1.2                         1   256   64  64
//   layer1.2 -> layer2.0                         1   256  128  64
//   layer2.1 -> 2.2, 2.2 -> 2.3                  2   512  128  64 (or 32: 80 KB, two blocks per CU)
//   layer2.3 -> layer3.0                         2   512  256  32
//   layer3.1 -> 3.2 ... layer3.4 -> 3.5          4  1024  256  32
template <int KS, int N1, int N2, int CW, int BM = 128>
int launch_chain(const ChainArgs& a, hipStream_t st) {
  constexpr int LDS = BM * KS * 128 + 2 * (CW * KS * 128 + N2 * CW * 2 + BM * CW * 2);
  constexpr int OCC = LDS <= 80 * 1024 ? 4 : 2;
#ifdef MLS_CHAIN_SWAP
  constexpr bool SW = MLS_CHAIN_SWAP;
#else
  constexpr bool SW = KS == 1;
#endif
  hipLaunchKernelGGL((conv_chain_kernel<BM, KS, N1, N2, CW, OCC, SW>), dim3((unsigned)((a.M + BM - 1) / BM)),
                     dim3(512), 0, st, a);
  return (int)hipGetLastError();
}

int g_chain_cw_l2 = 0;  // layer2 chunk width override (0 = default 64; mls_chain_set_l2_cw for A/B)
int g_chain_bm_l2 = 128;  // layer2 boundaries' row tile (64: 392 blocks instead of 196 at B = 32)

}  // namespace

extern "C" {

// y = relu(conv1x1([a1 | a2 strided]) + b3 (+ res)); t1 = relu(conv1x1(y, w1) + b1).
// a1 [M][Ka] (M = B*Ho*Wo), a2 [B][H2][W2][Kb] sampled at stride2 (Kb = 0: none), w3 [N1][Ka+Kb],
// res [M][N1] or null, w1 [N2][N1]; y [M][N1], t1 [M][N2].  (KS = (Ka + Kb) / 64, N1, N2) one of
// (1, 256, 64), (2, 256, 64), (1, 256, 128), (2, 512, 128), (2, 512, 256), (4, 1024, 256);
// anything else MLS_UNSUPPORTED.
int mls_conv_chain(const void* a1, const void* a2, const void* w3, const float* b3, const void* res, void* y,
                   const void* w1, const float* b1, void* t1, int B, int Ho, int Wo, int Ka, int H2, int W2, int Kb,
                   int stride2, int N1, int N2, void* stream) {
  if (B <= 0 || Ho <= 0 || Wo <= 0 || Ka <= 0 || Ka % 64 || Kb < 0 || Kb % 64 || N1 <= 0 || N1 % 64 || N2 <= 0)
    return MLS_BAD_ARG;
  if (Kb > 0 && (stride2 < 1 || (Ho - 1) * stride2 >= H2 || (Wo - 1) * stride2 >= W2 || res)) return MLS_BAD_ARG;
  ChainArgs a{};
  a.a1 = (const bf16*)a1;
  a.a2 = (const bf16*)a2;
  a.w3 = (const bf16*)w3;
  a.b3 = b3;
  a.res = (const bf16*)res;
  a.y = (bf16*)y;
  a.w1 = (const bf16*)w1;
  a.b1 = b1;
  a.t1 = (bf16*)t1;
  a.M = B * Ho * Wo;
  a.Ka = Ka;
  a.Kb = Kb;
  a.N1 = N1;
  a.N2 = N2;
  a.Ho = Ho, a.Wo = Wo, a.H2 = H2, a.W2 = W2, a.stride2 = stride2;
  a.fd_howo = fastdiv_make((uint32_t)(Ho * Wo));
  a.fd_wo = fastdiv_make((uint32_t)Wo);
  const long M = a.M;
  const long sizes[7] = {M * Ka * 2, (long)B * H2 * W2 * Kb * 2, (long)N1 * (Ka + Kb) * 2, res ? M * N1 * 2 : 0,
                         M * N1 * 2, (long)N2 * N1 * 2, M * N2 * 2};
  for (long s : sizes)
    if (s >= 0x7fffffffL) return MLS_UNSUPPORTED;
  a.a1_bytes = (uint32_t)sizes[0];
  a.a2_bytes = (uint32_t)sizes[1];
  a.w3_bytes = (uint32_t)sizes[2];
  a.res_bytes = (uint32_t)sizes[3];
  a.y_bytes = (uint32_t)sizes[4];
  a.w1_bytes = (uint32_t)sizes[5];
  a.t1_bytes = (uint32_t)sizes[6];
  const hipStream_t st = (hipStream_t)stream;
  const int ks = (Ka + Kb) / 64;
  if (ks == 1 && N1 == 256 && N2 == 64) return launch_chain<1, 256, 64, 64>(a, st);
  if (ks == 2 && N1 == 256 && N2 == 64) return launch_chain<2, 256, 64, 64>(a, st);
  if (ks == 1 && N1 == 256 && N2 == 128) return launch_chain<1, 256, 128, 64>(a, st);
  if (ks == 2 && N1 == 512 && N2 == 128) {
    if (g_chain_bm_l2 == 64) return launch_chain<2, 512, 128, 64, 64>(a, st);
    return g_chain_cw_l2 == 32 ? launch_chain<2, 512, 128, 32>(a, st) : launch_chain<2, 512, 128, 64>(a, st);
  }
  if (ks == 2 && N1 == 512 && N2 == 256)
    return g_chain_bm_l2 == 64 ? launch_chain<2, 512, 256, 64, 64>(a, st) : launch_chain<2, 512, 256, 32>(a, st);
  if (ks == 4 && N1 == 1024 && N2 == 256) return launch_chain<4, 1024, 256, 32>(a, st);
  return MLS_UNSUPPORTED;
}

// A/B switch for the layer2 boundaries' chunk width (64 = 128 KB of LDS, one block per CU; 32 =
// 80 KB, two per CU).
void mls_chain_set_l2_cw(int cw) { g_chain_cw_l2 = (cw == 32 || cw == 64) ? cw : 0; }

// A/B switch for the layer2 boundaries' row tile: 128 (default) or 64 (twice the blocks).
void mls_chain_set_l2_bm(int bm) { g_chain_bm_l2 = bm == 64 ? 64 : 128; }

}  // extern "C"

MLS_DEBUG_EXPORT(conv_chain)
