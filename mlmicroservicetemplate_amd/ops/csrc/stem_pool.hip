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
template <int TILES_PER_BLOCK, bool CONV1, bool SWAP = true>
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
    __syncthreads();  // the previous tile's patch / tile reads are done
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
    __syncthreads();

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
    __syncthreads();

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

}  // namespace

extern "C" {

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
  static const bool swap = [] {  // MLS_STEM_SWAP=0: the per-element epilogue (A/B)
    const char* e = getenv("MLS_STEM_SWAP");
    return !(e && e[0] == '0');
  }();
  auto kernel = c1 ? (tpb == 1 ? stem_pool_kernel<1, true> : tpb == 2 ? stem_pool_kernel<2, true>
                                         : tpb == 7 ? stem_pool_kernel<7, true> : stem_pool_kernel<4, true>)
                   : (tpb == 1 ? stem_pool_kernel<1, false> : tpb == 2 ? stem_pool_kernel<2, false>
                                         : tpb == 7 ? stem_pool_kernel<7, false> : stem_pool_kernel<4, false>);
  if (!swap && !c1 && tpb == 7) kernel = stem_pool_kernel<7, false, false>;
  hipLaunchKernelGGL(kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, (const uint8_t*)images,
                     (const bf16*)w, bias, (bf16*)out, B, H, W, Po, mean3[0], mean3[1], mean3[2], 1.f / std3[0],
                     1.f / std3[1], 1.f / std3[2], dbg, (const bf16*)w1, b1, (bf16*)t1);
  return (int)hipGetLastError();
}

}  // extern "C"

MLS_DEBUG_EXPORT(stem_pool)
