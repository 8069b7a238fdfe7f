// ResNet-50 input block as ONE kernel: uint8 image -> normalise -> 7x7/2 stem conv (BN folded)
// -> ReLU -> 3x3/2 max pool, bf16 NHWC [B][56][56][64] out.  Replaces three launches
// (normalize_u8 -> conv_gemm_kernel MODE_STEM -> maxpool_kernel) and keeps the 112x112x64 stem
// activation (51 MB per batch of 32, written once and re-read once) entirely on chip.
//
// Block = up to 4 consecutive 4 x 8 tiles of pooled outputs along one pooled-row strip (weights
// loaded to VGPRs once per block; the next tile's image bytes are fetched during the current
// tile's math).  A tile  Its pooling windows cover 9 x 17 stem pixels (one row /
// column shared with the neighbouring tile, recomputed instead of exchanged), whose receptive
// fields form one 23 x 40 pixel patch of the image: staged ONCE in LDS as normalised bf16 x 4
// channels (zero outside the image = the conv padding), so every image pixel is read from memory
// once per tile instead of once per tap (the implicit-GEMM stem re-gathers each ~12 times).
// GEMM view per tile: M = 153 stem pixels (padded to 160 = 10 MFMA row blocks), N = 64, K = 7 kh
// x 32 (kw padded 7 -> 8, Cin 3 -> 4: one v_mfma_f32_16x16x32_bf16 k-slab per kernel row, each
// lane's 16-byte A fragment = 2 adjacent taps x 4 channels, one ds_read_b128 from the patch).
// Weights (28 KB, L2-resident) go straight to VGPRs.  Epilogue: bias + ReLU -> bf16 tile in LDS
// (stem pixels outside the image forced to 0, which cannot win a max of ReLU outputs), then each
// thread max-reduces one pooled pixel x 8 channels and stores 16 bytes.  Rounding to bf16 before
// the max equals rounding after it (monotone), so the result matches the three-kernel path.
#include "common.h"

#include <cstdlib>

namespace {

constexpr int TPH = 4, TPW = 8;                    // pooled outputs per block
constexpr int SR = 2 * TPH + 1, SC = 2 * TPW + 1;  // stem pixels per block: 9 x 17
constexpr int SP = SR * SC;                        // 153
constexpr int MROWS = 160;                         // 10 row blocks of 16
constexpr int PR = 2 * (SR - 1) + 7;               // patch rows: 23
constexpr int PC = 2 * (SC - 1) + 8;               // patch cols: 40 (taps padded to 8)
constexpr int COUT = 64, KTOT = 7 * 32;
constexpr int PATCH_BYTES = PR * PC * 8;           // 7360
constexpr int TSTR = COUT + 8;                      // stem tile row stride (bf16): 144 B spreads the
                                                    // epilogue's 4 row groups and the pool's rows over banks
constexpr int TILE_BYTES = MROWS * TSTR * 2;       // 23040
constexpr int NPOOL = TPH * TPW;                   // 32 pooled pixels per tile
constexpr int POOL_BYTES = NPOOL * COUT * 2;       // 4096: the pooled tile as the 1x1 conv's A operand

// TILES_PER_BLOCK = consecutive tiles of one pooled-row strip per block.  CONV1: also run the first
// bottleneck's 1x1 conv (64 -> 64, BN folded, ReLU) on each pooled tile while it is in LDS and
// store its output t1 -- the layer1.0.conv1 launch and its 12.8 MB re-read of the pooled map go
// away (the pooled map itself is still stored: the block's downsample branch reads it).
// SWAP: the MFMA computes D = W . Patch^T instead of Patch . W, so each lane holds 4 consecutive
// output channels of one stem pixel and the epilogue writes 8 B per (row block, column block) --
// 10 ds_write_b64 per lane per tile instead of 40 single-bf16 writes, one pixel-validity test per
// row block instead of per element.
// LDS-only block barrier: this wave's LDS accesses done, then s_barrier.  __syncthreads() would also
// drain vmcnt -- the next tile's image bytes (fetched a tile ahead) and the pooled stores would
// then complete at every barrier, exposing a full memory round trip per tile instead of hiding it.
MLS_DEV void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// RAWB: the tile loop's barriers as lds_barrier() (default) instead of __syncthreads() (A/B,
// MLS_STEM_RAWBAR=0).
template <int TILES_PER_BLOCK, bool CONV1, bool SWAP = true, bool RAWB = true>
__global__ __launch_bounds__(256, 3) void stem_pool_kernel(const uint8_t* __restrict__ img, const bf16* __restrict__ w,
                                                        const float* __restrict__ bias, bf16* __restrict__ out, int B,
                                                        int H, int W, int Po, float m0, float m1, float m2, float s0,
                                                        float s1, float s2, int dbg, const bf16* __restrict__ w1,
                                                        const float* __restrict__ b1, bf16* __restrict__ t1) {
  __shared__ __attribute__((aligned(16))) char smem[PATCH_BYTES + TILE_BYTES + (CONV1 ? 2 * POOL_BYTES : 0)];
  bf16* tile = reinterpret_cast<bf16*>(smem + PATCH_BYTES);  // [MROWS][TSTR]
  char* sPool = smem + PATCH_BYTES + TILE_BYTES;             // [32 px][8 x 16 B], chunk ^ (px & 7)
  char* sT1 = sPool + POOL_BYTES;                            // [32 px][8 x 16 B], chunk ^ (px & 7)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int tw = Po / TPW, th = Po / TPH;
  const int nparts = (tw + TILES_PER_BLOCK - 1) / TILES_PER_BLOCK;
  int t = blockIdx.x;
  const int part = t % nparts;
  t /= nparts;
  const int by = t % th;
  const int b = t / th;
  MLS_CHECK(b < B, 401);
  const int bx0 = part * TILES_PER_BLOCK, bx1 = min(tw, bx0 + TILES_PER_BLOCK);
  const int ph0 = by * TPH;
  const int sr0 = 2 * ph0 - 1;     // first stem row of the strip (may be -1)
  const int ir0 = 2 * sr0 - 3;     // first image row of the patch (stride 2, pad 3)

  // weight fragments straight to registers, once per block (2 x 2 waves, a wave = 80 rows x 32 cols)
  const int wm = wid >> 1, wn = wid & 1;
  const int fr = lane & 15, fq = lane >> 4;
  bf16x8 bw[2][7];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = wn * 32 + j * 16 + fr;
#pragma unroll
    for (int kh = 0; kh < 7; ++kh)
      bw[j][kh] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(w + (long)n * KTOT + kh * 32 + fq * 8));
  }
  float bj[2];      // !SWAP: this lane's output channel per column block
  float bq[2][4];   // SWAP: this lane's 4 consecutive output channels per column block
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    bj[j] = bias[wn * 32 + j * 16 + fr];
#pragma unroll
    for (int r = 0; r < 4; ++r) bq[j][r] = bias[wn * 32 + j * 16 + fq * 4 + r];
  }
  // CONV1: wave w owns t1 columns w*16 .. w*16+15 of both 16-pixel row blocks; its B fragments
  // (64 input channels = 2 k-steps) and bias in registers for the whole block
  bf16x8 bw1[2];
  float bb1 = 0.f;
  if constexpr (CONV1) {
#pragma unroll
    for (int k = 0; k < 2; ++k)
      bw1[k] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(w1 + (wid * 16 + fr) * COUT + k * 32 + fq * 8));
    bb1 = b1 ? b1[wid * 16 + fr] : 0.f;
  }
  int abase[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int p = min(wm * 80 + i * 16 + fr, SP - 1);  // padded rows read a valid pixel, never stored
    const int sr = p / SC, sc = p - (p / SC) * SC;
    abase[i] = ((2 * sr) * PC + 2 * sc + 2 * fq) * 8;
  }

  // epilogue row masks (bit i * 4 + r): padded rows, stem row 0, stem column 0 -- kept as bits so the
  // tile loop does not hold 20 row / column pairs in registers
  // (SWAP: one bit per row block i -- the lane's pixel is wm * 80 + i * 16 + fr)
  uint32_t m_pad = 0, m_sr0 = 0, m_sc0 = 0;
#pragma unroll
  for (int i = 0; i < 5; ++i)
#pragma unroll
    for (int r = 0; r < (SWAP ? 1 : 4); ++r) {
      const int row = wm * 80 + i * 16 + (SWAP ? fr : fq * 4 + r);
      const int sr = row / SC, sc = row - (row / SC) * SC;
      const int bit = SWAP ? i : i * 4 + r;
      m_pad |= (uint32_t)(row >= SP) << bit;
      m_sr0 |= (uint32_t)(sr == 0) << bit;
      m_sc0 |= (uint32_t)(sc == 0) << bit;
    }

  // image bytes of a tile's patch -> registers (issued a tile ahead: software pipelined)
  constexpr int PIT = (PR * PC + 255) / 256;  // 4
  uint8_t px[PIT][3];
  bool in[PIT];
  auto fetch = [&](int bx) {
    const int ic0 = 2 * (2 * (bx * TPW) - 1) - 3;
#pragma unroll
    for (int it = 0; it < PIT; ++it) {
      const int q = tid + it * 256;
      const int pr = q / PC, pc = q - (q / PC) * PC;
      const int iy = ir0 + pr, ix = ic0 + pc;
      in[it] = q < PR * PC && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W && !(dbg & 1);
      const uint8_t* p = img + (((long)b * H + (in[it] ? iy : 0)) * W + (in[it] ? ix : 0)) * 3;
      px[it][0] = p[0];
      px[it][1] = p[1];
      px[it][2] = p[2];
    }
  };
  fetch(bx0);
  for (int bx = bx0; bx < bx1; ++bx) {
    const int pw0 = bx * TPW;
    const int sc0 = 2 * pw0 - 1;
    if constexpr (RAWB) lds_barrier();  // the previous tile's patch / tile reads are done
    else __syncthreads();
    // patch: normalised bf16 x 4 channels, zero outside the image
#pragma unroll
    for (int it = 0; it < PIT; ++it) {
      const int q = tid + it * 256;
      if (q >= PR * PC) break;
      bf16x4 v;
      v[0] = (bf16)(in[it] ? ((float)px[it][0] - m0) * s0 : 0.f);
      v[1] = (bf16)(in[it] ? ((float)px[it][1] - m1) * s1 : 0.f);
      v[2] = (bf16)(in[it] ? ((float)px[it][2] - m2) * s2 : 0.f);
      v[3] = (bf16)0.f;
      *reinterpret_cast<uint2*>(smem + q * 8) = __builtin_bit_cast(uint2, v);
    }
    if (bx + 1 < bx1) fetch(bx + 1);  // next tile's bytes fly during this tile's math
    if constexpr (RAWB) lds_barrier();
    else __syncthreads();

    // MFMA over the 7 kernel rows
    f32x4 acc[5][2];
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kh = 0; kh < 7; ++kh) {
      if (dbg & 2) break;
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        const bf16x8 av = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(smem + abase[i] + kh * PC * 8));
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = SWAP ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[j][kh], av, acc[i][j], 0, 0, 0)
                           : __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bw[j][kh], acc[i][j], 0, 0, 0);
      }
    }

    // bias + ReLU -> bf16 stem tile in LDS; stem pixels outside the image (row / column -1) -> 0
    const uint32_t zero = (sr0 < 0 ? m_sr0 : 0u) | (sc0 < 0 ? m_sc0 : 0u);
    if constexpr (SWAP) {
      // lane: stem pixel wm*80 + i*16 + fr, channels wn*32 + j*16 + fq*4 .. +3 -> one 8-B write
      // (pixel stride 144 B: the 16 lanes of a ds_write_b64 group land on disjoint bank pairs)
      bf16* tp = tile + (wm * 80 + fr) * TSTR + wn * 32 + fq * 4;
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        if ((m_pad >> i) & 1u) continue;
        const bool z = (zero >> i) & 1u;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          bf16x4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float e = acc[i][j][r];  // through a named float (ext-vector element bit-cast hazard)
            v[r] = (bf16)(z ? 0.f : fmaxf(e + bq[j][r], 0.f));
          }
          *reinterpret_cast<uint2*>(tp + i * 16 * TSTR + j * 16) = __builtin_bit_cast(uint2, v);
        }
      }
    } else {
      bf16* trow = tile + (wm * 80 + fq * 4) * TSTR + wn * 32 + fr;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 5; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int k = i * 4 + r;
            if (!((m_pad >> k) & 1u))
              trow[(i * 16 + r) * TSTR + j * 16] = (bf16)(((zero >> k) & 1u) ? 0.f : fmaxf(acc[i][j][r] + bj[j], 0.f));
          }
    }
    if constexpr (RAWB) lds_barrier();
    else __syncthreads();

    // 3x3 / 2 max pool: thread = one pooled pixel x 8 channels
    const int pp = tid >> 3, c8 = tid & 7;
    const int pr = pp / TPW, pc = pp - (pp / TPW) * TPW;
    float m[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const int row = (2 * pr + dy) * SC + 2 * pc + dx;
        float v[8];
        unpack8(*reinterpret_cast<const uint4*>(tile + row * TSTR + c8 * 8), v);
#pragma unroll
        for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], v[e]);
      }
    if (dbg & 4) {
      if (m[0] == 12345.f) st16(out, pack8(m));  // keep the work live; never true
      continue;
    }
    const uint4 pooled = pack8(m);
    st16(out + (((long)b * Po + ph0 + pr) * Po + pw0 + pc) * COUT + c8 * 8, pooled);
    if constexpr (CONV1) {
      // t1 = relu(pooled . W1^T + b1): the pooled tile [32 px][64 ch] in LDS is the A operand
      *reinterpret_cast<uint4*>(sPool + pp * 128 + ((c8 ^ (pp & 7)) << 4)) = pooled;
      __syncthreads();
      f32x4 acc1[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        acc1[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int r = i * 16 + fr;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int ch = fq + 4 * k;
          const bf16x8 av = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sPool + r * 128 + ((ch ^ (r & 7)) << 4)));
          acc1[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bw1[k], acc1[i], 0, 0, 0);
        }
      }
      const int col = wid * 16 + fr;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = i * 16 + fq * 4 + r;
          const float e = acc1[i][r];  // through a named float (ext-vector element bit-cast hazard)
          *reinterpret_cast<bf16*>(sT1 + row * 128 + (((col >> 3) ^ (row & 7)) << 4) + (col & 7) * 2) =
              (bf16)fmaxf(e + bb1, 0.f);
        }
      __syncthreads();
      st16(t1 + (((long)b * Po + ph0 + pr) * Po + pw0 + pc) * COUT + c8 * 8,
           *reinterpret_cast<const uint4*>(sT1 + pp * 128 + ((c8 ^ (pp & 7)) << 4)));
    }
  }
}


// ---------------------------------------------------------------------------------------------
// v2 (default; MLS_STEM_V2=0 runs the kernel above).  What the v1 tile loop cost, read from its
// ISA: the next tile's image bytes were fetched as ubyte / ushort loads that hipcc merges right
// after issue (s_waitcnt vmcnt(6..1) straight behind the fetch), so every tile paid a full memory
// round trip before its MFMAs; 448 blocks of 7 tiles left 64 CUs with one block and 192 with two
// (the kernel lasts two blocks); the pool unpacked 9 x 8 bf16 to fp32 per thread.  v2:
//  * tile = 7 x 4 pooled outputs (15 x 9 = 135 stem pixels, 9 MFMA row blocks); a block runs 7
//    tiles along a pooled-row strip, the grid is 32 images x 8 strips x 2 halves = 512 blocks =
//    exactly 2 per CU, all resident;
//  * the patch (35 image rows x 28 columns, 4-pixel groups aligned to 4) is fetched as one 12-B
//    load per thread and kept as raw dwords until the next tile writes it -- the fetch of tile t+1
//    really flies under tile t's MFMAs;
//  * waves = 2 row halves (5 / 4 row blocks) x 2 channel halves (2 column blocks): each A
//    fragment read from LDS feeds two MFMAs;
//  * 3x3/2 max pool on the raw bf16 bits with v_pk_max_u16 (post-ReLU values are >= 0, so their
//    bf16 patterns order like unsigned integers), 4 packed maxes per tap instead of 16 fp32 ops.
namespace v2 {
constexpr int TPH = 7, TPW = 4;                 // pooled outputs per tile
constexpr int SR = 2 * TPH + 1, SC = 2 * TPW + 1;  // 15 x 9 stem pixels
constexpr int SP = SR * SC;                     // 135
constexpr int RB = 9;                           // 16-row MFMA blocks (144 rows)
constexpr int PRW = 2 * (SR - 1) + 7;           // patch image rows: 35
constexpr int PG = 7;                           // 4-pixel column groups: 28 image columns
constexpr int PSTR = 30;                        // patch row stride in pixels (240 B; col 0 unused)
constexpr int PATCH_BYTES = (PRW + 2) * PSTR * 8;  // 8880: + 2 dummy rows that threads >= 245 write
constexpr int TSTR = 72;                        // stem tile row stride (bf16): 144 B
constexpr int TILE_BYTES = RB * 16 * TSTR * 2;  // 20736
constexpr int TILES = 7;                        // per block
constexpr int COUT = 64, KTOT = 7 * 32;
}  // namespace v2

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4s __attribute__((__vector_size__(16)));

__global__ __launch_bounds__(256, 2) void stem_pool_v2_kernel(const uint8_t* __restrict__ img, const bf16* __restrict__ w,
                                                           const float* __restrict__ bias, bf16* __restrict__ out,
                                                           uint32_t img_bytes, int B, float m0, float m1, float m2,
                                                           float s0, float s1, float s2, long long* stamps,
                                                           int stagger, int* arrive) {
  // stamps (diagnostics, MLS_STEM_STAMPS=1 via mls_stem_set_stamps): s_memtime of lane 0 of every
  // wave at the kernel start, after the first loads, and at each phase boundary of each tile
  constexpr int H = 224, W = 224, Po = 56;
  __shared__ __attribute__((aligned(16))) char smem[v2::PATCH_BYTES + v2::TILE_BYTES];
  bf16* tile = reinterpret_cast<bf16*>(smem + v2::PATCH_BYTES);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int half = blockIdx.x & 1, strip = (blockIdx.x >> 1) & 7, b = blockIdx.x >> 4;
  const int ph0 = strip * v2::TPH;
  const int sr0 = 2 * ph0 - 1;   // first stem row (may be -1)
  const int ir0 = 2 * sr0 - 3;   // first image row of the patch
  const rsrc_t ir = make_rsrc(img, img_bytes);

  const int wm = wid >> 1, wn = wid & 1;  // row half (blocks 0-4 / 5-8), channel half
  const int fr = lane & 15, fq = lane >> 4;
  bf16x8 bw[2][7];
  float bq[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = wn * 32 + j * 16 + fr;
#pragma unroll
    for (int kh = 0; kh < 7; ++kh)
      bw[j][kh] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(w + (long)n * v2::KTOT + kh * 32 + fq * 8));
#pragma unroll
    for (int r = 0; r < 4; ++r) bq[j][r] = bias[wn * 32 + j * 16 + fq * 4 + r];
  }
  // A-fragment offsets of this wave's row blocks: stem pixel p = (r, c) reads patch rows 2r + kh,
  // columns 4 + 2c + 2fq (+1): the tap pair (2fq, 2fq + 1) of kernel row kh, 4 channels each
  int abase[5];
  uint32_t m_pad = 0, m_r0 = 0, m_c0 = 0;  // per row block: padding row, stem row 0, stem column 0
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int rb = wm * 5 + i;
    const int p0 = rb * 16 + fr;
    const int p = p0 < v2::SP ? p0 : v2::SP - 1;
    const int r = p / v2::SC, c = p - (p / v2::SC) * v2::SC;
    abase[i] = ((2 * r) * v2::PSTR + 4 + 2 * c + 2 * fq) * 8;
    m_pad |= (uint32_t)(p0 >= v2::SP) << i;
    m_r0 |= (uint32_t)(r == 0) << i;
    m_c0 |= (uint32_t)(c == 0) << i;
  }

  // patch fetch: thread q -> patch row q / 7, 4-pixel group q % 7 (12 bytes, 4-B aligned); threads
  // >= 245 land in the two dummy rows (every thread writes: no divergent branch in the loop)
  const int q = tid;
  const int prow = q / v2::PG, pgrp = q - (q / v2::PG) * v2::PG;
  uint32_t raw[3];
  float valid;  // 1 / 0: a multiplier, not a select (a per-element select made hipcc branch + wait)
  auto fetch = [&](int t) {
    const int pc0 = half * (v2::TILES * v2::TPW) + t * v2::TPW;  // first pooled column of tile t
    const int ix = 4 * pc0 - 8 + 4 * pgrp;           // 16 k - 8 + 4 g: a group is all in or all out
    const int iy = ir0 + prow;
    const bool ok = prow < v2::PRW && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
    valid = ok ? 1.f : 0.f;
    const int off = ok ? ((b * H + iy) * W + ix) * 3 : OOB;
#pragma unroll
    for (int k = 0; k < 3; ++k) raw[k] = __builtin_amdgcn_raw_buffer_load_b32(ir, off + 4 * k, 0, 0);
  };
  // stagger (MLS_STEM_STAGGER=<cycles>): the second block to arrive on a CU starts that much later,
  // so the two blocks' MFMA phases do not coincide (arrival parity per CU from a global counter
  // indexed by the CU's hardware id; never reset, the parity alternates)
  if (stagger > 0 && arrive) {
    __shared__ int s_par;
    if (tid == 0) {
      const unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_REG_HW_ID
      const unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));  // HW_REG_XCC_ID[3:0]
      const unsigned cu = ((hw >> 8) & 15u) | (((hw >> 12) & 1u) << 4) | (((hw >> 13) & 7u) << 5);
      s_par = atomicAdd(arrive + ((xcc & 7u) << 8 | (cu & 255u)), 1) & 1;
    }
    __syncthreads();
    if (s_par) {
      const long long t0 = __builtin_amdgcn_s_memtime();
      while (__builtin_amdgcn_s_memtime() - t0 < stagger) __builtin_amdgcn_s_sleep(4);
    }
  }
  long long* st = stamps ? stamps + ((long)blockIdx.x * 4 + wid) * 64 : nullptr;
  if (st && lane == 0) st[0] = __builtin_amdgcn_s_memtime();
  fetch(0);
  // tile 0's bytes (used at once anyway) and the weight / bias loads complete here: left pending,
  // hipcc's wait pass merges them into the loop head's state and waits vmcnt(0) there (the
  // previous tile's pooled store included) instead of vmcnt(1) for the prefetched bytes
  __builtin_amdgcn_s_waitcnt(0);
  if (st && lane == 0) st[1] = __builtin_amdgcn_s_memtime();
  // pool: thread = pooled pixel pp (< 28) x 8-channel chunk; threads >= 224 redo pixel 27 and
  // store out of range (dropped): every thread stores, so the loop head waits vmcnt(1) for the
  // prefetched patch bytes, not vmcnt(0) behind a divergent store
  const int pp = min(tid >> 3, v2::TPH * v2::TPW - 1), c8 = tid & 7;
  const int pr = pp / v2::TPW, pc = pp - (pp / v2::TPW) * v2::TPW;
  const rsrc_t orr = make_rsrc(out, (uint32_t)((long)B * Po * Po * v2::COUT * 2));

  for (int t = 0; t < v2::TILES; ++t) {
    const int pc0 = half * (v2::TILES * v2::TPW) + t * v2::TPW;
    const int sc0 = 2 * pc0 - 1;
    lds_barrier();  // the previous tile's patch / tile reads are done
    if (st && lane == 0) st[2 + 6 * t] = __builtin_amdgcn_s_memtime();
    {  // normalised bf16 x 4 channels (channel 3 = 0), zero outside the image; the same
       // arithmetic as v1 ((x - mean) * inv_std, +0 outside), so both kernels give identical bits
      const float ss[3] = {s0, s1, s2};
      const float mm[3] = {m0, m1, m2};
      const bool ok = valid != 0.f;
      char* dst = smem + (prow * v2::PSTR + 1 + 4 * pgrp) * 8;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bf16x4 v;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const int byte = 3 * j + c;
          const float x = (float)((raw[byte >> 2] >> (8 * (byte & 3))) & 0xffu);
          const float nv = (x - mm[c]) * ss[c];
          v[c] = (bf16)(ok ? nv : 0.f);
        }
        v[3] = (bf16)0.f;
        *reinterpret_cast<uint2*>(dst + j * 8) = __builtin_bit_cast(uint2, v);
      }
    }
    if (t + 1 < v2::TILES) fetch(t + 1);  // lands under this tile's MFMAs
    if (st && lane == 0) st[3 + 6 * t] = __builtin_amdgcn_s_memtime();
    lds_barrier();
    if (st && lane == 0) st[4 + 6 * t] = __builtin_amdgcn_s_memtime();

    f32x4 acc[5][2];
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // every wave runs 5 row blocks (wave row half 1's fifth is padding, dropped by m_pad): no
    // branch between the fragment reads and the MFMAs, and the critical wave does 5 anyway.  The
    // next kernel row's 5 fragments are read while this row's 10 MFMAs run (register double buffer)
    bf16x8 av[2][5];
#pragma unroll
    for (int i = 0; i < 5; ++i)
      av[0][i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(smem + abase[i]));
#pragma unroll
    for (int kh = 0; kh < 7; ++kh) {
      if (kh + 1 < 7) {
#pragma unroll
        for (int i = 0; i < 5; ++i)
          av[(kh + 1) & 1][i] = __builtin_bit_cast(
              bf16x8, *reinterpret_cast<const uint4*>(smem + abase[i] + (kh + 1) * v2::PSTR * 8));
      }
#pragma unroll
      for (int i = 0; i < 5; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[j][kh], av[kh & 1][i], acc[i][j], 0, 0, 0);
    }
    if (st && lane == 0) st[5 + 6 * t] = __builtin_amdgcn_s_memtime();
    // bias + ReLU -> bf16 stem tile; stem pixels outside the image (row / column -1) -> 0
    const uint32_t zero = (sr0 < 0 ? m_r0 : 0u) | (sc0 < 0 ? m_c0 : 0u);
    bf16* tp = tile + (wm * 80 + fr) * v2::TSTR + wn * 32 + fq * 4;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      if ((m_pad >> i) & 1u) continue;
      const bool z = (zero >> i) & 1u;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        bf16x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = acc[i][j][r];  // through a named float (ext-vector element bit-cast hazard)
          v[r] = (bf16)(z ? 0.f : fmaxf(e + bq[j][r], 0.f));
        }
        *reinterpret_cast<uint2*>(tp + i * 16 * v2::TSTR + j * 16) = __builtin_bit_cast(uint2, v);
      }
    }
    if (st && lane == 0) st[6 + 6 * t] = __builtin_amdgcn_s_memtime();
    lds_barrier();

    {
      u16x2 mx[4] = {u16x2{0, 0}, u16x2{0, 0}, u16x2{0, 0}, u16x2{0, 0}};
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const uint4 v = *reinterpret_cast<const uint4*>(tile + ((2 * pr + dy) * v2::SC + 2 * pc + dx) * v2::TSTR + c8 * 8);
          mx[0] = __builtin_elementwise_max(mx[0], __builtin_bit_cast(u16x2, v.x));
          mx[1] = __builtin_elementwise_max(mx[1], __builtin_bit_cast(u16x2, v.y));
          mx[2] = __builtin_elementwise_max(mx[2], __builtin_bit_cast(u16x2, v.z));
          mx[3] = __builtin_elementwise_max(mx[3], __builtin_bit_cast(u16x2, v.w));
        }
      const uint4 o{__builtin_bit_cast(uint32_t, mx[0]), __builtin_bit_cast(uint32_t, mx[1]),
                    __builtin_bit_cast(uint32_t, mx[2]), __builtin_bit_cast(uint32_t, mx[3])};
      const int ooff = tid < v2::TPH * v2::TPW * 8 ? ((((b * Po + ph0 + pr) * Po + pc0 + pc) * v2::COUT + c8 * 8) * 2) : OOB;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4s, o), orr, ooff, 0, 0);
    }
    if (st && lane == 0) st[7 + 6 * t] = __builtin_amdgcn_s_memtime();
  }
  if (st && lane == 0) st[2 + 6 * v2::TILES] = __builtin_amdgcn_s_memtime();
}

// ---------------------------------------------------------------------------------------------
// v3 (MLS_STEM_VER=3 / mls_stem_set_version): v2's tiles, weights, fragment layout and arithmetic
// -- bit-identical output -- with the tile loop software-pipelined.  v2's stamps put a tile at
// patch 620 + MFMA 2300 + epilogue 1300 + pool 930 cycles per wave, phases separated by three
// block barriers, so the matrix pipe idles for ~60 % of the loop, and the two blocks of a CU run
// their phases in lockstep.  v3 double-buffers the patch and the stem tile in LDS (2 x 8880 +
// 2 x 20736 B, still 2 blocks per CU) and runs, between ONE barrier per tile:
//   patch(t+1) written from the bytes fetched a tile earlier, fetch(t+2) issued,
//   MFMA(t) on patch[t&1] with pool(t-1) on tile[(t-1)&1] interleaved into its kernel rows,
//   epilogue(t) -> tile[t&1].
// Tile -1's pool and tile 7's patch run on dummy data (stores dropped by the range check, loads
// zero-filled), so the loop body has no branches.
__global__ __launch_bounds__(256, 2) void stem_pool_v3_kernel(const uint8_t* __restrict__ img, const bf16* __restrict__ w,
                                                           const float* __restrict__ bias, bf16* __restrict__ out,
                                                           uint32_t img_bytes, int B, float m0, float m1, float m2,
                                                           float s0, float s1, float s2) {
  constexpr int H = 224, W = 224, Po = 56;
  constexpr int NT = v2::TILES;
  __shared__ __attribute__((aligned(16))) char smem[2 * v2::PATCH_BYTES + 2 * v2::TILE_BYTES];
  auto patch_buf = [&](int i) { return smem + (i & 1) * v2::PATCH_BYTES; };
  auto tile_buf = [&](int i) { return reinterpret_cast<bf16*>(smem + 2 * v2::PATCH_BYTES + (i & 1) * v2::TILE_BYTES); };
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int half = blockIdx.x & 1, strip = (blockIdx.x >> 1) & 7, b = blockIdx.x >> 4;
  const int ph0 = strip * v2::TPH;
  const int sr0 = 2 * ph0 - 1;
  const int ir0 = 2 * sr0 - 3;
  const rsrc_t ir = make_rsrc(img, img_bytes);

  const int wm = wid >> 1, wn = wid & 1;
  const int fr = lane & 15, fq = lane >> 4;
  bf16x8 bw[2][7];
  float bq[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = wn * 32 + j * 16 + fr;
#pragma unroll
    for (int kh = 0; kh < 7; ++kh)
      bw[j][kh] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(w + (long)n * v2::KTOT + kh * 32 + fq * 8));
#pragma unroll
    for (int r = 0; r < 4; ++r) bq[j][r] = bias[wn * 32 + j * 16 + fq * 4 + r];
  }
  int abase[5];
  uint32_t m_r0 = 0, m_c0 = 0;  // per row block: stem row 0, stem column 0
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int rb = wm * 5 + i;
    const int p0 = rb * 16 + fr;
    const int p = p0 < v2::SP ? p0 : v2::SP - 1;
    const int r = p / v2::SC, c = p - (p / v2::SC) * v2::SC;
    abase[i] = ((2 * r) * v2::PSTR + 4 + 2 * c + 2 * fq) * 8;
    m_r0 |= (uint32_t)(r == 0) << i;
    m_c0 |= (uint32_t)(c == 0) << i;
  }

  const int q = tid;
  const int prow = q / v2::PG, pgrp = q - (q / v2::PG) * v2::PG;
  uint32_t raw[3];
  float valid;
  auto fetch = [&](int t) {  // t >= NT: nothing to fetch (zero bytes, valid = 0)
    const int pc0 = half * (NT * v2::TPW) + t * v2::TPW;
    const int ix = 4 * pc0 - 8 + 4 * pgrp;
    const int iy = ir0 + prow;
    const bool ok = t < NT && prow < v2::PRW && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
    valid = ok ? 1.f : 0.f;
    const int off = ok ? ((b * H + iy) * W + ix) * 3 : OOB;
#pragma unroll
    for (int k = 0; k < 3; ++k) raw[k] = __builtin_amdgcn_raw_buffer_load_b32(ir, off + 4 * k, 0, 0);
  };
  // normalised bf16 x 4 channels from raw[]: x * s + (-m * s) as one FMA per value with both
  // terms zeroed for pixels outside the image (their bytes load as 0), 2 VALU per value instead
  // of v2's subtract / multiply / select
  const float nb0 = -m0 * s0, nb1 = -m1 * s1, nb2 = -m2 * s2;
  auto write_patch = [&](char* pb) {
    const float ss[3] = {s0 * valid, s1 * valid, s2 * valid};
    const float bb[3] = {nb0 * valid, nb1 * valid, nb2 * valid};
    char* dst = pb + (prow * v2::PSTR + 1 + 4 * pgrp) * 8;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bf16x4 v;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int byte = 3 * j + c;
        const float x = (float)((raw[byte >> 2] >> (8 * (byte & 3))) & 0xffu);
        v[c] = (bf16)__builtin_fmaf(x, ss[c], bb[c]);
      }
      v[3] = (bf16)0.f;
      *reinterpret_cast<uint2*>(dst + j * 8) = __builtin_bit_cast(uint2, v);
    }
  };

  const int pp = min(tid >> 3, v2::TPH * v2::TPW - 1), c8 = tid & 7;
  const int pr = pp / v2::TPW, pc = pp - (pp / v2::TPW) * v2::TPW;
  const rsrc_t orr = make_rsrc(out, (uint32_t)((long)B * Po * Po * v2::COUT * 2));
  const bool pool_lane = tid < v2::TPH * v2::TPW * 8;

  fetch(0);
  __builtin_amdgcn_s_waitcnt(0);
  write_patch(patch_buf(0));
  fetch(1);
  lds_barrier();

  for (int t = 0; t < NT; ++t) {
    // patch of tile t+1 (bytes fetched one tile ago), then the bytes of tile t+2
    write_patch(patch_buf(t + 1));
    fetch(t + 2);

    // MFMA(t) with pool(t-1) interleaved: 9 pool taps spread over the 7 kernel rows
    const char* pb = patch_buf(t);
    const bf16* tp_prev = tile_buf(t + 1);
    i16x2 mx[4] = {i16x2{0, 0}, i16x2{0, 0}, i16x2{0, 0}, i16x2{0, 0}};
    f32x4 acc[5][2];
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{bq[j][0], bq[j][1], bq[j][2], bq[j][3]};  // bias as C
    bf16x8 av[2][5];
#pragma unroll
    for (int i = 0; i < 5; ++i)
      av[0][i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(pb + abase[i]));
#pragma unroll
    for (int kh = 0; kh < 7; ++kh) {
      // the next kernel row's A fragments and this row's pool taps (kh 0-1 two taps, the rest one:
      // 9 over 7) are issued, then this row's 10 MFMAs, then the taps are max-reduced; the
      // scheduling barriers keep hipcc from sinking the loads next to their first use (it did:
      // each fragment read was waited for right after its issue)
      uint4 tv[2];
      if (kh + 1 < 7) {
#pragma unroll
        for (int i = 0; i < 5; ++i)
          av[(kh + 1) & 1][i] = __builtin_bit_cast(
              bf16x8, *reinterpret_cast<const uint4*>(pb + abase[i] + (kh + 1) * v2::PSTR * 8));
      }
      const int tap0 = kh < 2 ? 2 * kh : kh + 2, ntap = kh < 2 ? 2 : 1;
#pragma unroll
      for (int u = 0; u < ntap; ++u) {
        const int tap = tap0 + u, dy = tap / 3, dx = tap % 3;
        tv[u] = *reinterpret_cast<const uint4*>(tp_prev + ((2 * pr + dy) * v2::SC + 2 * pc + dx) * v2::TSTR + c8 * 8);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 5; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[j][kh], av[kh & 1][i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < ntap; ++u) {
        mx[0] = __builtin_elementwise_max(mx[0], __builtin_bit_cast(i16x2, tv[u].x));
        mx[1] = __builtin_elementwise_max(mx[1], __builtin_bit_cast(i16x2, tv[u].y));
        mx[2] = __builtin_elementwise_max(mx[2], __builtin_bit_cast(i16x2, tv[u].z));
        mx[3] = __builtin_elementwise_max(mx[3], __builtin_bit_cast(i16x2, tv[u].w));
      }
    }
    {  // pooled tile t-1 out (tile -1: dropped)
      const int pc0p = half * (NT * v2::TPW) + (t - 1) * v2::TPW;
      const uint4 o{__builtin_bit_cast(uint32_t, mx[0]), __builtin_bit_cast(uint32_t, mx[1]),
                    __builtin_bit_cast(uint32_t, mx[2]), __builtin_bit_cast(uint32_t, mx[3])};
      const int ooff = (t > 0 && pool_lane) ? ((((b * Po + ph0 + pr) * Po + pc0p + pc) * v2::COUT + c8 * 8) * 2) : OOB;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4s, o), orr, ooff, 0, 0);
    }
    // epilogue(t): pre-activation -> bf16 stem tile t (the bias rode in as the MFMA's C).  The ReLU
    // is the pool's: a max of bf16 bit patterns as SIGNED 16-bit integers starting from 0 orders
    // the positive values correctly and sends every negative one (sign bit set) below the 0, so
    // max(0, taps) = ReLU(max(taps)) = max(ReLU(taps)) -- no per-value op here.  Stem pixels outside
    // the image (row / column -1, only in the first strip / first tile of a row) are forced to 0.
    const int sc0 = 2 * (half * (NT * v2::TPW) + t * v2::TPW) - 1;
    bf16* tp = tile_buf(t) + (wm * 80 + fr) * v2::TSTR + wn * 32 + fq * 4;
    const int wm_u = __builtin_amdgcn_readfirstlane(wm);  // wave-uniform: scalar branches below
    if (sr0 < 0 || sc0 < 0) {  // block-uniform
      const uint32_t zero = (sr0 < 0 ? m_r0 : 0u) | (sc0 < 0 ? m_c0 : 0u);
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        if (i == 4 && wm_u == 1) continue;  // row block 9: past the tile (rows 135-143 of block 8 are
                                            // written too; the pool never reads them)
        const int keep = ((zero >> i) & 1u) ? 0 : -1;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          bf16x4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float e = acc[i][j][r];
            v[r] = (bf16)__builtin_bit_cast(float, __builtin_bit_cast(int, e) & keep);
          }
          *reinterpret_cast<uint2*>(tp + i * 16 * v2::TSTR + j * 16) = __builtin_bit_cast(uint2, v);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        if (i == 4 && wm_u == 1) continue;  // row block 9: past the tile (rows 135-143 of block 8 are
                                            // written too; the pool never reads them)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          bf16x4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float e = acc[i][j][r];
            v[r] = (bf16)e;
          }
          *reinterpret_cast<uint2*>(tp + i * 16 * v2::TSTR + j * 16) = __builtin_bit_cast(uint2, v);
        }
      }
    }
    lds_barrier();
  }
  {  // the last tile's pool
    const bf16* tpl = tile_buf(NT - 1);
    i16x2 mx[4] = {i16x2{0, 0}, i16x2{0, 0}, i16x2{0, 0}, i16x2{0, 0}};
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const uint4 v = *reinterpret_cast<const uint4*>(tpl + ((2 * pr + dy) * v2::SC + 2 * pc + dx) * v2::TSTR + c8 * 8);
        mx[0] = __builtin_elementwise_max(mx[0], __builtin_bit_cast(i16x2, v.x));
        mx[1] = __builtin_elementwise_max(mx[1], __builtin_bit_cast(i16x2, v.y));
        mx[2] = __builtin_elementwise_max(mx[2], __builtin_bit_cast(i16x2, v.z));
        mx[3] = __builtin_elementwise_max(mx[3], __builtin_bit_cast(i16x2, v.w));
      }
    const int pc0 = half * (NT * v2::TPW) + (NT - 1) * v2::TPW;
    const uint4 o{__builtin_bit_cast(uint32_t, mx[0]), __builtin_bit_cast(uint32_t, mx[1]),
                  __builtin_bit_cast(uint32_t, mx[2]), __builtin_bit_cast(uint32_t, mx[3])};
    const int ooff = pool_lane ? ((((b * Po + ph0 + pr) * Po + pc0 + pc) * v2::COUT + c8 * 8) * 2) : OOB;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4s, o), orr, ooff, 0, 0);
  }
}
}  // namespace

extern "C" {

// per-CU arrival counters of the v2 stagger (2048 = 8 XCCs x 256 hardware CU ids), allocated once
static int* stem_arrivals() {
  static int* p = [] {
    int* q = nullptr;
    if (hipMalloc(&q, 2048 * sizeof(int)) != hipSuccess || hipMemset(q, 0, 2048 * sizeof(int)) != hipSuccess)
      return (int*)nullptr;
    (void)hipDeviceSynchronize();
    return q;
  }();
  return p;
}

// diagnostics: v2 writes per-wave phase stamps ([blocks][4 waves][64] int64) here while set
long long* g_stem_stamps = nullptr;
// which tile loop runs (3: software-pipelined v3, the default; 2: phase-serial v2, also taken
// while stamps or a stagger are set); MLS_STEM_VER overrides the default, mls_stem_set_version
// switches at run time (tests compare the two).  v3 vs v2 (profiles/r6_stem_v3_ab.jsonl): alone
// 22.3 vs 24.7 us per B=32 call, bench 20 steps 55.5-56.0k vs 55.3-55.5k (3 of 3 pairs), 200 level
static int g_stem_ver = [] {
  const char* e = getenv("MLS_STEM_VER");
  return e && (e[0] == '2' || e[0] == '3') ? e[0] - '0' : 3;
}();
int mls_stem_set_version(int v) {
  const int old = g_stem_ver;
  if (v == 2 || v == 3) g_stem_ver = v;
  return old;
}
int mls_stem_set_stamps(void* buf) {
  g_stem_stamps = (long long*)buf;
  return 0;
}

int mls_stem_pool_conv1(const void* images, const void* w, const float* bias, void* out, int B, int H, int W,
                        const float* mean3, const float* std3, const void* w1, const float* b1, void* t1,
                        void* stream);

// images uint8 [B][H][W][3]; w = the packed stem weights [64][7][8][4] bf16 (BN scale folded);
// bias fp32 [64]; out bf16 [B][Po][Po][64] with Po = H / 4.  224 x 224 (ResNet) only.
int mls_stem_pool(const void* images, const void* w, const float* bias, void* out, int B, int H, int W,
                  const float* mean3, const float* std3, void* stream) {
  return mls_stem_pool_conv1(images, w, bias, out, B, H, W, mean3, std3, nullptr, nullptr, nullptr, stream);
}

// ... and, with w1 [64][64] (BN folded) / b1 [64] / t1 [B][Po][Po][64] given, the first bottleneck's
// 1x1 conv + ReLU on the pooled map in the same kernel.
int mls_stem_pool_conv1(const void* images, const void* w, const float* bias, void* out, int B, int H, int W,
                        const float* mean3, const float* std3, const void* w1, const float* b1, void* t1,
                        void* stream) {
  if (B <= 0 || H != 224 || W != 224) return MLS_UNSUPPORTED;
  const int Po = H / 4;  // stem 112 -> pool 56
  if (Po % TPH || Po % TPW) return MLS_UNSUPPORTED;
  static const int dbg = [] {  // ablation flags for tools/probe/stem_pool_probe.py: 1 no image loads, 2 no MFMA, 4 no stores
    const char* e = getenv("MLS_STEM_DBG");
    return e ? atoi(e) : 0;
  }();
  // tiles per block (1, 2, 4 or 7; MLS_STEM_TPB overrides for the probe).  7 = a whole pooled-row
  // strip: 25.9 us vs 28.9 (1 tile) with 4 copies co-running, 35.0 vs 32.0 alone
  // (profiles/r1_stem_pool_tiles_per_block.jsonl); the engine runs 5 batches in flight.
  static const int tpb = [] {
    const char* e = getenv("MLS_STEM_TPB");
    const int v = e ? atoi(e) : 7;
    return v == 1 || v == 2 || v == 4 ? v : 7;
  }();
  const long blocks = (long)B * (Po / TPH) * ((Po / TPW + tpb - 1) / tpb);
  if (blocks > 0x7fffffffL) return MLS_BAD_ARG;
  const bool c1 = w1 != nullptr && t1 != nullptr;
  static const bool use_v2 = [] {  // MLS_STEM_V2=0: the v1 kernel (A/B)
    const char* e = getenv("MLS_STEM_V2");
    return !(e && e[0] == '0');
  }();
  const long img_bytes = (long)B * H * W * 3;
  static const int stagger = [] {
    const char* e = getenv("MLS_STEM_STAGGER");
    return e ? atoi(e) : 0;
  }();
  if (use_v2 && !c1 && img_bytes < 0x7fffffffL && g_stem_ver == 3 && !g_stem_stamps && stagger <= 0) {
    hipLaunchKernelGGL(stem_pool_v3_kernel, dim3((unsigned)(B * 16)), dim3(256), 0, (hipStream_t)stream,
                       (const uint8_t*)images, (const bf16*)w, bias, (bf16*)out, (uint32_t)img_bytes, B, mean3[0],
                       mean3[1], mean3[2], 1.f / std3[0], 1.f / std3[1], 1.f / std3[2]);
    return (int)hipGetLastError();
  }
  if (use_v2 && !c1 && img_bytes < 0x7fffffffL) {
    hipLaunchKernelGGL(stem_pool_v2_kernel, dim3((unsigned)(B * 16)), dim3(256), 0, (hipStream_t)stream,
                       (const uint8_t*)images, (const bf16*)w, bias, (bf16*)out, (uint32_t)img_bytes, B, mean3[0],
                       mean3[1], mean3[2], 1.f / std3[0], 1.f / std3[1], 1.f / std3[2], g_stem_stamps, stagger,
                       stagger > 0 ? stem_arrivals() : nullptr);
    return (int)hipGetLastError();
  }
  static const bool swap = [] {  // MLS_STEM_SWAP=0: the per-element epilogue (A/B)
    const char* e = getenv("MLS_STEM_SWAP");
    return !(e && e[0] == '0');
  }();
  auto kernel = c1 ? (tpb == 1 ? stem_pool_kernel<1, true> : tpb == 2 ? stem_pool_kernel<2, true>
                                         : tpb == 7 ? stem_pool_kernel<7, true> : stem_pool_kernel<4, true>)
                   : (tpb == 1 ? stem_pool_kernel<1, false> : tpb == 2 ? stem_pool_kernel<2, false>
                                         : tpb == 7 ? stem_pool_kernel<7, false> : stem_pool_kernel<4, false>);
  if (!swap && !c1 && tpb == 7) kernel = stem_pool_kernel<7, false, false>;
  static const bool rawbar = [] {  // MLS_STEM_RAWBAR=0: __syncthreads() in the tile loop (A/B)
    const char* e = getenv("MLS_STEM_RAWBAR");
    return !(e && e[0] == '0');
  }();
  if (!rawbar && !c1 && swap)
    kernel = tpb == 1 ? stem_pool_kernel<1, false, true, false> : tpb == 2 ? stem_pool_kernel<2, false, true, false>
           : tpb == 7 ? stem_pool_kernel<7, false, true, false> : stem_pool_kernel<4, false, true, false>;
  hipLaunchKernelGGL(kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, (const uint8_t*)images,
                     (const bf16*)w, bias, (bf16*)out, B, H, W, Po, mean3[0], mean3[1], mean3[2], 1.f / std3[0],
                     1.f / std3[1], 1.f / std3[2], dbg, (const bf16*)w1, b1, (bf16*)t1);
  return (int)hipGetLastError();
}

}  // extern "C"

MLS_DEBUG_EXPORT(stem_pool)
