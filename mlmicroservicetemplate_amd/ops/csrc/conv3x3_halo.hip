// Halo-tiled direct 3x3 / stride 1 / pad 1 convolution, NHWC bf16, for the ResNet bottleneck conv2
// layers (56x56x64, 28x28x128, 14x14x256, 7x7x512).
//
// Why not the implicit GEMM of conv_gemm.hip: there every k-step re-gathers a BM x 64 slice of the
// input for ONE tap, so each input pixel crosses L2 -> LDS nine times, and a 128x128 tile at BK 64
// needs ~150 GB/s per CU of L2 bandwidth to keep its MFMAs busy -- about what a CU gets
// (docs/PERF_NOTES.md).  Here a block owns a whole spatial tile -- nb images x th output rows x the
// full width W (<= 256 output pixels, contiguous in the NHWC output) -- and per 32-channel chunk
// stages the input patch WITH its 1-pixel halo once ((th + 2) x (W + 2) pixels x 64 B) plus the
// 9 taps' weights for 64 output channels (36 KB); all 9 taps then read their A fragments from the
// same patch at a (kh, kw) pixel offset.  Per chunk: ~60 KB of LDS-DMA for 2 x 16 x 64 x 9 x 32
// MACs -- ~2.5x the arithmetic intensity of the 128x128 implicit-GEMM tile.
//
// Layout: patch [pixel][4 x 16-B chunks] (a fragment row = one pixel's 64 B); weights
// [tap][64 cols][4 chunks], chunk-swizzled so the B reads are conflict-free (the A reads of a row
// block that wraps a patch row cannot be swizzled for every alignment and stay <= 2-way).  Both are
// staged through registers: chunk c + 1's buffer loads are in flight during chunk c's MFMAs and
// land in LDS after the next barrier (MLS_HALO_RS=0: LDS DMA per chunk instead; level end to end,
// faster per layer at c4 -- profiles/r1_halo_regstage_probe.jsonl); out-of-image halo pixels get
// an out-of-range offset and read as zero = the conv padding.  One stage per block so several blocks share a CU and
// overlap each other's loads (a double-buffered 120 KB first version, one block per CU, measured
// slower under concurrency: profiles/r1_halo_probe_stages.jsonl).  A tap's fragments are read
// while the previous tap's MFMAs run.  Epilogue: bias + activation (+ optional residual) -> bf16
// tile in LDS -> 16-B coalesced stores.
//
// Selected per layer by the tuning table (ops.CFG_HALO); at bs=32 under 4-way concurrency it wins
// 12 of the 13 stride-1 3x3 layers (13.5 vs 19.1 us on layer1, profiles/r1_halo_vs_table_c4.jsonl)
// and lifts bench.py from 48.0k to 49.6k req/s.
#include "common.h"
#include "fastdiv.h"

#include <cstdlib>

int* mls_stream_splitk_counters(void* stream, long ntiles);  // conv_gemm.hip

namespace {

constexpr int CK = 32;                           // input channels per chunk = one MFMA k-slab
constexpr int MAX_ROWS = 256;                    // output pixels per block (16 MFMA row blocks)
constexpr int PATCH_MAX = 384;                   // input pixels per patch
// the XL tile (variant 2): 512 output pixels x 64 channels, each wave a 4 x 4 grid of MFMA tiles
// (half the LDS fragment reads per MFMA of the 2 x 4 grid: at 2 x 4 the fragment reads alone need
// ~190 of the CU's 256 LDS bytes / clk), weights amortised over twice the pixels
constexpr int XL_ROWS = 512;
constexpr int XL_PATCH = 648;                    // 8 images of 9 x 9, or 10 x 58 rows of a 56-wide map

#define LDS3 __attribute__((address_space(3)))

// MFMA operand order: 1 D = W_tile . Patch^T -- a lane holds 4 consecutive output channels of one
// pixel, so the epilogue parks a fragment with one 8-B LDS write (and a split-K slice with one
// 16-B store) instead of four 2-B / 4-B ones.  0 (default): Patch . W_tile^T -- the swapped build
// was level-to-slower on every 3x3 layer (layer1 12.6 vs 12.1 us co-running,
// profiles/r3_swap_epilogue_component_costs.jsonl): the epilogue runs once per 2-16 chunks here,
// unlike the stem's once per 70 MFMAs.  A/B build option (-DMLS_HALO_SWAP=1).
#ifndef MLS_HALO_SWAP
#define MLS_HALO_SWAP 0
#endif
typedef unsigned int halo_u32x4 __attribute__((__vector_size__(16)));

MLS_DEV void glds16(rsrc_t r, char* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDS3 void*)lds, 16, voff, soff, 0, 0);
}

struct HaloArgs {
  const bf16* x;     // [B][H][W][Cin]
  const bf16* w;     // [N][3][3][Cin]
  const float* bias; // [N] fp32 or null
  const bf16* res;   // [B][H][W][N] or null
  bf16* out;         // [B][H][W][N]
  float* ws;         // split-K slabs [ksplit][B*H*W][N] fp32 (ksplit > 1)
  int* cnt;          // per-tile arrival counters of this stream (ksplit > 1)
  int B, H, W, Cin, N, th, nb, act, ksplit;
  uint32_t x_bytes, w_bytes, ws_bytes;
  // runtime divisors (fastdiv.h): ksplit, tiles, H / th, th * W, W, (th + 2) * (W + 2), W + 2
  FastDiv fd_ks, fd_tiles, fd_tpi, fd_r, fd_w, fd_p2, fd_w2;
};

// Weight image swizzle: 16-B chunk ch of column n sits at ch ^ h((n >> 2) & 3), h = {0, 2, 3, 1}:
// the four 16-lane groups of a ds_read_b128 ({0-3,12-15,20-27}, ...) then hit 16 distinct bank
// quads (MI355X_MICROARCH.md, LDS table); unswizzled they conflict 2-way.
MLS_DEV int wswz(int n) { return (0x78 >> (2 * ((n >> 2) & 3))) & 3; }

// BN output channels per block, NW waves; wave w owns MFMA row blocks w, w + NW, ... (16 / NW of
// them) x all BN / 16 column blocks.  <64, 8>: 60 KB of LDS (2 blocks per CU); <32, 4>: 42 KB
// (3 per CU), half the MFMA work per staged patch.
// ROWS / PMAX: output pixels / patch pixels per block.  CONTIG (the XL tile): wave w owns the row
// blocks w*RBW .. w*RBW+RBW-1 and skips (wave-uniformly) the ones past the tile's last pixel;
// otherwise row blocks w, w + NW, ... and padded blocks are computed and dropped.
template <int BN, int NW, int ROWS = MAX_ROWS, int PMAX = PATCH_MAX>
struct HaloCfg {
  static constexpr int NTHR = NW * 64;
  static constexpr int PATCH_BYTES = (PMAX + 15) / 16 * 1024;  // whole 16-pixel DMA pieces (the last may be partial)
  static constexpr int W_BYTES = 9 * BN * CK * 2;
  static constexpr int W_PIECES = W_BYTES / 1024;
  static constexpr int STAGE = PATCH_BYTES + W_BYTES;
  static constexpr int EPI_LD = BN + 8;  // bf16 row stride of the epilogue tile
  static constexpr int RBW = ROWS / 16 / NW;  // row blocks per wave
  static constexpr int CB = BN / 16;          // column blocks
  static constexpr bool CONTIG = ROWS > MAX_ROWS;
  static constexpr int PP_WAVE = ((PMAX + 15) / 16 + NW - 1) / NW;  // patch DMA pieces per wave
  static constexpr int WP_WAVE = (W_PIECES + NW - 1) / NW;
  static_assert(ROWS * EPI_LD * 2 <= STAGE, "epilogue tile fits the stage buffer");
  static_assert(RBW * NW * 16 == ROWS && CB * 16 == BN, "tile split");
  static_assert(STAGE <= 160 * 1024, "LDS");
};

template <int BN, int NW, bool RS, int ROWS = MAX_ROWS, int PMAX = PATCH_MAX>
__global__ __launch_bounds__(NW * 64) void conv3x3_halo_kernel(const HaloArgs a) {
  using C = HaloCfg<BN, NW, ROWS, PMAX>;
  constexpr int RBW = C::RBW, CB = C::CB;
  constexpr int PATCH_BYTES = C::PATCH_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[C::STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int W2 = a.W + 2, TH2 = a.th + 2;
  const int R = a.nb * a.th * a.W;  // output pixels of the tile
  const int P = a.nb * TH2 * W2;    // patch pixels
  const int tiles = (a.B / a.nb) * (a.H / a.th);
  int t = xcd_remap(blockIdx.x, gridDim.x);
  const int tq = fastdiv(t, a.fd_ks);
  const int split = t - tq * a.ksplit;  // split-K slices of a tile are neighbours (one XCD's L2)
  t = tq;
  const int tn = fastdiv(t, a.fd_tiles), tile = t - tn * tiles;  // column-block-major: neighbours share weights
  MLS_CHECK(tn * BN < a.N, 501);
  const int n0 = tn * BN;
  const int tpi = a.H / a.th;  // tiles per image (nb == 1)
  const int ti = fastdiv(tile, a.fd_tpi);
  const int b0 = a.nb > 1 ? tile * a.nb : ti;
  const int oh0 = a.nb > 1 ? 0 : (tile - ti * tpi) * a.th;
  const long m_base = (long)tile * R;  // the tile's output pixels are contiguous rows

  auto rb_of = [&](int i) { return C::CONTIG ? wid * RBW + i : wid + NW * i; };
  // A fragments: patch pixel of tap (0, 0) for this lane's row in each of the wave's row blocks
  int pb[RBW];
  bool rb_on[RBW];
#pragma unroll
  for (int i = 0; i < RBW; ++i) {
    const int rb = rb_of(i);
    rb_on[i] = rb * 16 < R;
    const int r = min(rb * 16 + fr, R - 1);  // padded rows read a valid pixel, never stored
    const int img = fastdiv(r, a.fd_r);
    const int rem = r - img * (a.th * a.W);
    const int ohl = fastdiv(rem, a.fd_w), ow = rem - ohl * a.W;
    pb[i] = (img * TH2 + ohl) * W2 + ow;
  }

  // DMA source offsets without the chunk's channel base (added as the scalar offset)
  const int npieces = (P + 15) / 16;
  int xoff[C::PP_WAVE];
#pragma unroll
  for (int s = 0; s < C::PP_WAVE; ++s) {
    const int j = wid + NW * s;
    const int px = j * 16 + (lane >> 2), ch = lane & 3;
    xoff[s] = OOB;
    if (px < P) {
      const int img = fastdiv(px, a.fd_p2);
      const int rem = px - img * (TH2 * W2);
      const int pr = fastdiv(rem, a.fd_w2), pc = rem - pr * W2;
      const int b = b0 + img, ih = oh0 + pr - 1, iw = pc - 1;
      if (b < a.B && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W)
        xoff[s] = (((b * a.H + ih) * a.W + iw) * a.Cin + ch * 8) * 2;
    }
  }
  const int K = 9 * a.Cin;
  int woff[C::WP_WAVE];
#pragma unroll
  for (int s = 0; s < C::WP_WAVE; ++s) {
    const int j = wid + NW * s;
    const int q = j * 64 + lane;
    const int n = (q >> 2) & (BN - 1), tap = q / (4 * BN);
    const int ch = (q & 3) ^ wswz(n);  // LDS slot (q & 3) holds source chunk ch (DMA writes lane-linearly)
    woff[s] = j < C::W_PIECES ? ((n0 + n) * K + tap * a.Cin + ch * 8) * 2 : OOB;
  }
  const rsrc_t xr = make_rsrc(a.x, a.x_bytes);
  const rsrc_t wr = make_rsrc(a.w, a.w_bytes);
  char* sP = smem;
  char* sW = smem + PATCH_BYTES;

  f32x4 acc[RBW][CB];
#pragma unroll
  for (int i = 0; i < RBW; ++i)
#pragma unroll
    for (int j = 0; j < CB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nchunks = a.Cin / CK / a.ksplit;  // host: divisible
  const int cfirst = split * nchunks;
  const int bsw = (fq ^ wswz(fr)) * 16;  // this lane's B chunk slot (j * 16 keeps (n >> 2) & 3)
  // RS: register-staged -- chunk c + 1's patch and weights are loaded into VGPRs while chunk c's
  // MFMAs run and written to LDS after the next barrier, so the L2 / HBM latency hides behind
  // the math instead of stalling every chunk; otherwise LDS-DMA issued and awaited per chunk.
  uint4 px[C::PP_WAVE], pw[C::WP_WAVE];
  auto fetch = [&](int c) {
    const int cb = c * CK * 2;
#pragma unroll
    for (int s = 0; s < C::PP_WAVE; ++s) px[s] = bload16(xr, xoff[s] + cb);  // OOB (halo, tail) -> 0
#pragma unroll
    for (int s = 0; s < C::WP_WAVE; ++s) pw[s] = bload16(wr, woff[s] + cb);
  };
  if (RS) fetch(cfirst);
  for (int c = cfirst; c < cfirst + nchunks; ++c) {
    if (c > cfirst) __syncthreads();  // every wave is done reading chunk c - 1
    if (RS) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int s = 0; s < C::PP_WAVE; ++s) {
        const int j = wid + NW * s;
        if (j < npieces) *reinterpret_cast<uint4*>(sP + j * 1024 + lane * 16) = px[s];
      }
#pragma unroll
      for (int s = 0; s < C::WP_WAVE; ++s) {
        const int j = wid + NW * s;
        if (j < C::W_PIECES) *reinterpret_cast<uint4*>(sW + j * 1024 + lane * 16) = pw[s];
      }
      __syncthreads();  // chunk c is in LDS for every wave
      if (c + 1 < cfirst + nchunks) fetch(c + 1);
    } else {
      const int cb = c * CK * 2;
#pragma unroll
      for (int s = 0; s < C::PP_WAVE; ++s) {
        const int j = wid + NW * s;
        if (j < npieces) glds16(xr, sP + j * 1024, xoff[s], cb);
      }
#pragma unroll
      for (int s = 0; s < C::WP_WAVE; ++s) {
        const int j = wid + NW * s;
        if (j < C::W_PIECES) glds16(wr, sW + j * 1024, woff[s], cb);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // chunk c landed for every wave
    }
    // fragments of tap t + 1 are read while tap t's MFMAs run (register double buffer); every
    // row block is computed (a padded one reads clamped pixels and is not stored) so the tap
    // loop has no branches for the scheduler to stop at
    const char* pB = sW + fr * 64 + bsw;
    bf16x8 af[2][RBW], bf[2][CB];
    auto load = [&](int tap, int slot) {
      const int toff = ((tap / 3) * W2 + (tap % 3)) * 64;
#pragma unroll
      for (int i = 0; i < RBW; ++i)
        af[slot][i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sP + (pb[i] * 4 + fq) * 16 + toff));
#pragma unroll
      for (int j = 0; j < CB; ++j)
        bf[slot][j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(pB + (tap * BN + j * 16) * 64));
    };
    load(0, 0);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int cur = tap & 1;
      if (tap + 1 < 9) load(tap + 1, cur ^ 1);
#pragma unroll
      for (int i = 0; i < RBW; ++i) {
        if (C::CONTIG && !rb_on[i]) continue;  // wave-uniform: this row block is all padding
#pragma unroll
        for (int j = 0; j < CB; ++j)
          acc[i][j] = MLS_HALO_SWAP ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[cur][j], af[cur][i], acc[i][j], 0, 0, 0)
                                    : __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[cur][i], bf[cur][j], acc[i][j], 0, 0, 0);
      }
    }
  }

  const long M = (long)a.B * a.H * a.W;
  if (a.ksplit > 1) {
    // In-launch split-K: write this slice's fp32 partial through to the slabs (sc1), take a
    // ticket on the tile's counter; the last arriver sums the slices and runs the epilogue
    // (the conv_gemm.hip reducer's protocol).
    const rsrc_t wsr = make_rsrc(a.ws, a.ws_bytes);
#pragma unroll
    for (int i = 0; i < RBW; ++i) {
      const int rb = rb_of(i);
#pragma unroll
      for (int j = 0; j < CB; ++j) {
        if (MLS_HALO_SWAP) {  // lane: pixel rb*16 + fr, 4 consecutive channels -> one 16-B store
          const int row = rb * 16 + fr;
          const long idx = ((long)split * M + m_base + row) * a.N + n0 + j * 16 + fq * 4;
          const float v0 = acc[i][j][0], v1 = acc[i][j][1], v2 = acc[i][j][2], v3 = acc[i][j][3];
          const halo_u32x4 q = {__float_as_uint(v0), __float_as_uint(v1), __float_as_uint(v2), __float_as_uint(v3)};
          __builtin_amdgcn_raw_buffer_store_b128(q, wsr, row < R ? (int)(idx * 4) : OOB, 0, 16);
          continue;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rb * 16 + fq * 4 + r;
          const long idx = ((long)split * M + m_base + row) * a.N + n0 + j * 16 + fr;
          // (the element goes through a named float: __builtin_bit_cast of the vector element
          // expression itself stored element 0 for every r with this compiler)
          const float v = acc[i][j][r];
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), wsr, row < R ? (int)(idx * 4) : OOB, 0, 16);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(smem);
    if (tid == 0) {
      int* c = a.cnt + tn * tiles + tile;
      const int prev = __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = prev == a.ksplit - 1;
      if (last) __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for the next launch
      flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
    constexpr int CPR8 = BN / 8;
    for (int q = tid; q < R * CPR8; q += C::NTHR) {
      const int row = q / CPR8, c8 = q - (q / CPR8) * CPR8;
      const long o = (m_base + row) * a.N + n0 + c8 * 8;
      float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int sl = 0; sl < a.ksplit; ++sl) {
        const int off = (int)(((long)sl * M * a.N + o) * 4);
        const float4 x0 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(wsr, off, 0, 16));
        const float4 x1 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(wsr, off + 16, 0, 16));
        v[0] += x0.x; v[1] += x0.y; v[2] += x0.z; v[3] += x0.w;
        v[4] += x1.x; v[5] += x1.y; v[6] += x1.z; v[7] += x1.w;
      }
      float g[8];
      if (a.res) unpack8(*reinterpret_cast<const uint4*>(a.res + o), g);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float bb = a.bias ? a.bias[n0 + c8 * 8 + e] : 0.f;
        v[e] = apply_act(v[e] + bb + (a.res ? g[e] : 0.f), a.act);
      }
      st16(a.out + o, pack8(v));
    }
    return;
  }

  // epilogue: bias + act -> bf16 tile in LDS (reusing the stage buffer) -> 16-B stores
  // bias of this lane's output channel(s): MLS_HALO_SWAP -> 4 consecutive channels fq*4 .. +3 per
  // column block (the lane holds one pixel x 4 channels: one 8-B LDS write per fragment, pixel
  // stride EPI_LD = BN + 8 bf16 so the 16-lane groups of a ds_write_b64 hit disjoint bank pairs)
  float bj[CB][MLS_HALO_SWAP ? 4 : 1];
#pragma unroll
  for (int j = 0; j < CB; ++j)
#pragma unroll
    for (int r = 0; r < (MLS_HALO_SWAP ? 4 : 1); ++r)
      bj[j][r] = a.bias ? a.bias[n0 + j * 16 + (MLS_HALO_SWAP ? fq * 4 + r : fr)] : 0.f;
  __syncthreads();  // every wave is done with the last chunk
  bf16* to = reinterpret_cast<bf16*>(smem);
#pragma unroll
  for (int i = 0; i < RBW; ++i) {
    if (!rb_on[i]) continue;
    const int rb = rb_of(i);
#pragma unroll
    for (int j = 0; j < CB; ++j) {
      if (MLS_HALO_SWAP) {
        bf16x4 q;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][j][r];  // through a named float (ext-vector element bit-cast hazard)
          v += bj[j][r];
          if (!a.res) v = apply_act(v, a.act);
          q[r] = (bf16)v;
        }
        *reinterpret_cast<uint2*>(to + (rb * 16 + fr) * C::EPI_LD + j * 16 + fq * 4) = __builtin_bit_cast(uint2, q);
        continue;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rb * 16 + fq * 4 + r;
        float v = acc[i][j][r] + bj[j][0];
        if (!a.res) v = apply_act(v, a.act);
        to[row * C::EPI_LD + j * 16 + fr] = (bf16)v;
      }
    }
  }
  __syncthreads();
  constexpr int CPR = BN / 8;  // 16-B chunks per output row
  for (int q = tid; q < R * CPR; q += C::NTHR) {
    const int row = q / CPR, c8 = q - (q / CPR) * CPR;
    const long o = (m_base + row) * a.N + n0 + c8 * 8;
    uint4 v = *reinterpret_cast<const uint4*>(to + row * C::EPI_LD + c8 * 8);
    if (a.res) {  // act(conv + bias + residual)
      float f[8], g[8];
      unpack8(v, f);
      unpack8(*reinterpret_cast<const uint4*>(a.res + o), g);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = apply_act(f[e] + g[e], a.act);
      v = pack8(f);
    }
    st16(a.out + o, v);
  }
}

// Tile geometry for an H x W image: the largest th dividing H with th * W <= 256 output pixels
// and (th + 2) * (W + 2) <= PATCH_MAX patch pixels; whole images (th == H) are packed nb per
// block (nb | B).  Returns false when no geometry fits.
bool halo_geometry(int B, int H, int W, int* th, int* nb, int max_rows = MAX_ROWS, int patch_max = PATCH_MAX) {
  for (int t = H; t >= 1; --t) {
    if (H % t || t * W > max_rows || (t + 2) * (W + 2) > patch_max) continue;
    int n = 1;
    if (t == H)
      for (int c = 8; c >= 1; --c)
        if (B % c == 0 && c * H * W <= max_rows && c * (H + 2) * (W + 2) <= patch_max) {
          n = c;
          break;
        }
    *th = t;
    *nb = n;
    return true;
  }
  return false;
}

}  // namespace

extern "C" {

// 3x3 / stride 1 / pad 1 conv: x [B][H][W][Cin] bf16, w [N][3][3][Cin] bf16 (the packed conv
// layout), bias fp32 [N] (BN folded), optional residual [B][H][W][N]; out [B][H][W][N] bf16.
// Cin % 32 == 0; variant 0: 64 output channels x 8 waves per block (N % 64 == 0), variant 1:
// 32 x 4 (N % 32 == 0).
int mls_conv3x3_halo(const void* x, const void* w, const float* bias, const void* res, void* out, void* ws,
                     size_t ws_bytes, int B, int H, int W, int Cin, int N, int act, int variant, int splitk,
                     void* stream) {
  const int bn = variant == 1 ? 32 : 64;
  if (B <= 0 || H <= 0 || W <= 0 || Cin % CK || Cin <= 0 || N % bn || N <= 0 || variant < 0 || variant > 2)
    return MLS_BAD_ARG;
  int th = 0, nb = 0;
  const bool xl = variant == 2;
  if (!halo_geometry(B, H, W, &th, &nb, xl ? XL_ROWS : MAX_ROWS, xl ? XL_PATCH : PATCH_MAX)) return MLS_UNSUPPORTED;
  const long xb = (long)B * H * W * Cin * 2, wb = (long)N * 9 * Cin * 2;
  if (xb >= 0x7fffffffL || wb >= 0x7fffffffL || (long)B * H * W * N >= 0x7fffffffL) return MLS_UNSUPPORTED;
  HaloArgs a;
  a.x = (const bf16*)x;
  a.w = (const bf16*)w;
  a.bias = bias;
  a.res = (const bf16*)res;
  a.out = (bf16*)out;
  a.B = B, a.H = H, a.W = W, a.Cin = Cin, a.N = N, a.th = th, a.nb = nb, a.act = act;
  a.x_bytes = (uint32_t)xb;
  a.w_bytes = (uint32_t)wb;
  const int tiles = (B / nb) * (H / th);
  // split-K over input-channel chunks: needs the slabs, this stream's counters (allocated outside
  // graph capture, like conv_gemm's) and an even chunk split; otherwise one slice
  a.ksplit = 1;
  a.ws = nullptr;
  a.cnt = nullptr;
  a.ws_bytes = 0;
  const long slab = (long)splitk * B * H * W * N * 4;
  if (splitk > 1 && (Cin / CK) % splitk == 0 && ws && (long)ws_bytes >= slab && slab < 0x7fffffffL) {
    int* cnt = mls_stream_splitk_counters(stream, (long)tiles * (N / bn));
    if (cnt) {
      a.ksplit = splitk;
      a.ws = (float*)ws;
      a.cnt = cnt;
      a.ws_bytes = (uint32_t)slab;
    }
  }
  a.fd_ks = fastdiv_make((uint32_t)a.ksplit);
  a.fd_tiles = fastdiv_make((uint32_t)tiles);
  a.fd_tpi = fastdiv_make((uint32_t)(H / th));
  a.fd_r = fastdiv_make((uint32_t)(th * W));
  a.fd_w = fastdiv_make((uint32_t)W);
  a.fd_p2 = fastdiv_make((uint32_t)((th + 2) * (W + 2)));
  a.fd_w2 = fastdiv_make((uint32_t)(W + 2));
  const dim3 grid((unsigned)((long)tiles * (N / bn) * a.ksplit));
  static const bool rs = [] {  // MLS_HALO_RS=0: LDS-DMA staging (A/B)
    const char* e = getenv("MLS_HALO_RS");
    return !(e && e[0] == '0');
  }();
  // (a 64-channel x 4-wave variant -- 4 x 4 MFMA tiles per wave, half the LDS reads per MFMA --
  // measured 15-25 % slower than <64, 8>: profiles/r1_halo_w4_probe.jsonl)
  if (variant == 2) {
    hipLaunchKernelGGL((conv3x3_halo_kernel<64, 8, true, XL_ROWS, XL_PATCH>), grid, dim3(512), 0, (hipStream_t)stream,
                       a);
  } else if (variant == 1) {
    if (rs) hipLaunchKernelGGL((conv3x3_halo_kernel<32, 4, true>), grid, dim3(256), 0, (hipStream_t)stream, a);
    else hipLaunchKernelGGL((conv3x3_halo_kernel<32, 4, false>), grid, dim3(256), 0, (hipStream_t)stream, a);
  } else {
    if (rs) hipLaunchKernelGGL((conv3x3_halo_kernel<64, 8, true>), grid, dim3(512), 0, (hipStream_t)stream, a);
    else hipLaunchKernelGGL((conv3x3_halo_kernel<64, 8, false>), grid, dim3(512), 0, (hipStream_t)stream, a);
  }
  return (int)hipGetLastError();
}

// The geometry the kernel would use (for tests / the tuner): returns 0 and fills th, nb.
int mls_conv3x3_halo_geometry(int B, int H, int W, int* th, int* nb) {
  return halo_geometry(B, H, W, th, nb) ? 0 : MLS_UNSUPPORTED;
}

// ... for a given variant (2 = the 512-pixel XL tile)
int mls_conv3x3_halo_geometry_v(int B, int H, int W, int variant, int* th, int* nb) {
  const bool xl = variant == 2;
  return halo_geometry(B, H, W, th, nb, xl ? XL_ROWS : MAX_ROWS, xl ? XL_PATCH : PATCH_MAX) ? 0 : MLS_UNSUPPORTED;
}

}  // extern "C"

MLS_DEBUG_EXPORT(conv3x3_halo)
