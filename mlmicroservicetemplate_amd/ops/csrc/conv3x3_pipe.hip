// Pipelined halo-tiled 3x3 / stride 1 / pad 1 convolution, NHWC bf16 -- the ResNet bottleneck
// conv2 layers (56x56x64, 28x28x128, 14x14x256, 7x7x512) at serving batch sizes.
//
// What limits conv3x3_halo.hip (the round-1 kernel this replaces on the 3x3 layers): every block
// owns ONE tile and runs  load chunk -> wait -> compute -> epilogue  with a single LDS stage, so
//  * blocks that start together move through their phases in lock step: the chip first streams
//    every tile's patch (bandwidth-bound), then computes (MFMA-bound), then stores -- the sum of the
//    phases instead of their max (layer1: 448 tiles of 2 chunks each, ~18 us alone for ~5 us of
//    bytes and ~4 us of MFMA work);
//  * the 14x14 / 7x7 layers launch only 128 / 64 tiles of 64 channels: half or three quarters of
//    the 256 CUs idle when the layer runs alone (27.7 / 43 us per call, 12-13 % of bf16 peak);
//  * the A-fragment reads of a 64-B-per-pixel patch image are 2-way bank conflicted.
//
// This kernel:
//  * an LDS-DMA ring (`buffer_load ... lds`) of STAGES chunk stages {patch with halo, 9 taps'
//    weights} that runs over the flattened (item, chunk) sequence of the block: chunk c + 1 (or the
//    next item's first chunk) lands while chunk c's MFMAs run, counted `s_waitcnt vmcnt(N)` and raw
//    `s_barrier` (guide §5 "Pipelining across barriers"), the epilogue's stores are left in flight
//    across the next wait (they are the youngest vector-memory ops and the count allows for them);
//  * a block may take several consecutive items (IPB) so its prologue load overlaps earlier work;
//    items are (tile, 16*CB output channels, K split) -- BN = 32 and an in-launch split-K over the
//    input-channel chunks give the small-M layers >= 256 items;
//  * MFMA operands swapped (D = W_tile . Patch^T): a lane's 4 accumulators are 4 consecutive
//    output channels of one pixel, so the epilogue stores 8 B of bf16 per fragment straight from
//    registers (no LDS pass) and a split-K slice writes 16-B fp32 slab pieces;
//  * patch image [pixel][4 x 16 B] with chunk ^ (((p >> 2) & 1) << 1): the 16 pixels x 2 chunks
//    of every ds_read_b128 lane group hit 16 distinct 16-B bank slots for ANY tap offset (checked
//    exhaustively over pixel bases 0..63, tools/probe/pipe_swizzle_check.py); weights
//    [tap][col][4 x 16 B] with conv3x3_halo.hip's column swizzle;
//  * wave tile RBW row blocks x CB column blocks (4 x 4 at NW = 4: 8 ds_read_b128 per 16 MFMAs).
//
// Contract as mls_conv3x3_halo (no residual: the ResNet 3x3 convs have none).  Selected per layer
// through the tuning table (ops.CFG_PIPE + variant).
#include "common.h"
#include "fastdiv.h"

int* mls_stream_splitk_counters(void* stream, long ntiles);  // conv_gemm.hip

namespace {

constexpr int CK = 32;         // input channels per chunk (one MFMA k-slab, 64 B per pixel)
constexpr int PMAX = 384;      // patch pixels per item (the largest patch area: PPC = 24 pieces)
constexpr int MAX_ROWS = 256;  // output pixels per item (16 row blocks)
constexpr int NMAX = 512;      // output channels (bias staged in LDS)

#define LDS3 __attribute__((address_space(3)))

struct PipeArgs {
  const bf16* x;      // [B][H][W][Cin]
  const bf16* w;      // [N][3][3][Cin]
  const float* bias;  // [N] fp32 or null
  bf16* out;          // [B][H][W][N]
  float* ws;          // split-K slabs [ksplit][B*H*W][N] fp32 (ksplit > 1)
  int* cnt;           // per-tile arrival counters of this stream (ksplit > 1)
  int B, H, W, Cin, N, th, nb, act, ksplit;
  int tiles, ntn, nitems, ipb;
  int nck, tpi;  // input-channel chunks per item, tiles per image (H / th)
  uint32_t x_bytes, w_bytes, ws_bytes, o_bytes;
  // every runtime divisor of the kernel as a FastDiv: patch pixels per image ((th+2)*(W+2)), patch
  // row (W+2), output pixels per image-tile (th*W), W, ksplit, ntn, nck, tpi (fastdiv.h: with `/`
  // the prologue's per-lane geometry was ~500 VALU ops before the first DMA)
  FastDiv mg_p2, mg_w2, mg_r, mg_w, mg_ks, mg_ntn, mg_nck, mg_tpi;
};

MLS_DEV void glds16(rsrc_t r, char* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDS3 void*)lds, 16, voff, soff, 0, 0);
}
MLS_DEV int wswz(int n) { return (0x78 >> (2 * ((n >> 2) & 3))) & 3; }
// byte offset of logical 16-B chunk `ch` of patch pixel p
MLS_DEV int patch_addr(int p, int ch) { return ((p << 6) | (ch << 4)) ^ ((p << 3) & 32); }

template <int N>
MLS_DEV void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt field");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

typedef unsigned int pipe_u32x4 __attribute__((__vector_size__(16)));
typedef unsigned int pipe_u32x2 __attribute__((__vector_size__(8)));

// PPC: 1-KiB patch DMA pieces per stage (16 px each): 24 (<= 384 patch pixels) or 16 (<= 256,
// smaller items but a 3rd stage fits; no all-padding pieces issued for the 14x14 layer)
template <int BN, int NW, int RBW, int STAGES, int PPC>
struct PipeCfg {
  static constexpr int PP = PPC;
  static constexpr int CB = BN / 16;
  static constexpr int W_PIECES = 9 * BN * CK * 2 / 1024;  // 36 (BN 64) / 18 (BN 32)
  static constexpr int PATCH_BYTES = PP * 1024;
  static constexpr int STAGE = PATCH_BYTES + W_PIECES * 1024;
  static constexpr int PPW = PP / NW;                        // patch pieces per wave per stage
  static constexpr int WPW = (W_PIECES + NW - 1) / NW;       // weight pieces per wave (excess = duplicates)
  static constexpr int LPS = PPW + WPW;                      // vmcnt units per stage per wave
  static constexpr int NST = RBW * CB;                       // epilogue stores per wave per item
  static constexpr int BIAS_OFF = STAGES * STAGE;
  static constexpr int FLAG_OFF = BIAS_OFF + NMAX * 4;
  static constexpr int DUMMY_OFF = FLAG_OFF + 16;  // 1-KiB sink of the branch-free tail DMAs
  static constexpr int LDS = DUMMY_OFF + 1024;
  static_assert(PP % NW == 0 || PP < NW, "patch pieces split evenly over the waves");
  static_assert(RBW * NW >= 1 && RBW * NW * 16 <= 2 * MAX_ROWS, "row blocks");
  static_assert(LDS <= 160 * 1024, "LDS");
  static_assert(LPS * (STAGES - 1) + NST < 64, "vmcnt range");
};

template <int BN, int NW, int RBW, int STAGES, int PPC>
__global__ __launch_bounds__(NW * 64) void conv3x3_pipe_kernel(const PipeArgs a) {
  using C = PipeCfg<BN, NW, RBW, STAGES, PPC>;
  constexpr int CB = C::CB, LPS = C::LPS, NST = C::NST;
  __shared__ __attribute__((aligned(16))) char smem[C::LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int W2 = a.W + 2, TH2 = a.th + 2;
  const int R = a.nb * a.th * a.W;  // output pixels of an item
  const int P = a.nb * TH2 * W2;    // patch pixels of an item
  const int nck = a.nck;
  const long M = (long)a.B * a.H * a.W;

  // items [first, first + mine) of this block, consecutive (the XCD remap keeps neighbouring
  // items -- same tile, other channels / K slices -- on one XCD's L2)
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int first = lb * a.ipb;
  const int mine = min(a.ipb, a.nitems - first);
  if (mine <= 0) return;
  const int nsteps = mine * nck;

  // bias of every output channel -> LDS (plain loads, drained once before the ring starts)
  float* sbias = reinterpret_cast<float*>(smem + C::BIAS_OFF);
  for (int i = tid; i < a.N; i += NW * 64) sbias[i] = a.bias ? a.bias[i] : 0.f;

  // per-lane, item-independent geometry of the patch DMA pieces: pixel -> (row in patch, column),
  // relative source offset; the item adds its base and the row validity
  int prel[C::PPW], prow[C::PPW];
  bool pok[C::PPW];
#pragma unroll
  for (int s = 0; s < C::PPW; ++s) {
    const int px = (wid + NW * s) * 16 + (lane >> 2);
    const int slot = lane & 3;
    const int ch = slot ^ (((px >> 2) & 1) << 1);  // LDS slot `slot` of pixel px holds chunk ch
    const int img = fastdiv(px, a.mg_p2);
    const int rem = px - img * (TH2 * W2);
    const int pr = fastdiv(rem, a.mg_w2), pc = rem - pr * W2;
    pok[s] = px < P && pc >= 1 && pc <= a.W;
    prow[s] = pr;  // ih = oh0 + pr - 1
    prel[s] = (((img * a.H + pr - 1) * a.W + (pc - 1)) * a.Cin + ch * 8) * 2;
  }
  // weight pieces: [tap][col][slot] lane-linear; excess pieces of the last wave repeat one of its
  // own earlier pieces (same bytes to the same place) so every wave issues exactly WPW DMAs
  int woff[C::WPW], wdst[C::WPW];
#pragma unroll
  for (int s = 0; s < C::WPW; ++s) {
    int j = wid + NW * s;
    if (j >= C::W_PIECES) j -= NW;
    const int q = j * 64 + lane;
    const int n = (q >> 2) & (BN - 1), tap = q / (4 * BN);
    const int ch = (q & 3) ^ wswz(n);
    woff[s] = (n * 9 * a.Cin + tap * a.Cin + ch * 8) * 2;
    wdst[s] = j * 1024;
  }
  const rsrc_t xr = make_rsrc(a.x, a.x_bytes);
  const rsrc_t wr = make_rsrc(a.w, a.w_bytes);

  // item -> (tile, column block, K slice); items are tile-major
  auto decode = [&](int item, int& tile, int& tn, int& split) {
    const int t2 = fastdiv(item, a.mg_ks);
    split = item - t2 * a.ksplit;
    tile = fastdiv(t2, a.mg_ntn);
    tn = t2 - tile * a.ntn;
  };
  // issue cursor: the item whose patch offsets are cached
  int iss_item = -1, iss_wbase = 0, iss_cbase = 0;
  int xoff[C::PPW];
  // the DMA of `step`: prep() once (source offsets of a new item), then pieces 0 .. LPS-1 -- in the
  // main loop spread over the 9 taps of the current step (issue cost among the MFMAs, not in a
  // burst at the step start)
  auto prep = [&](int step, char*& st, int& cb) {
    const int sq = fastdiv(step, a.mg_nck);
    const int it = first + sq, c = step - sq * nck;
    if (it != iss_item) {
      iss_item = it;
      int tile, tn, split;
      decode(it, tile, tn, split);
      const int ti = fastdiv(tile, a.mg_tpi);
      const int b0 = a.nb > 1 ? tile * a.nb : ti;
      const int oh0 = a.nb > 1 ? 0 : (tile - ti * a.tpi) * a.th;
      const int iss_xbase = ((b0 * a.H + oh0) * a.W) * a.Cin * 2;
      iss_wbase = tn * BN * 9 * a.Cin * 2;
      iss_cbase = split * nck;
#pragma unroll
      for (int s = 0; s < C::PPW; ++s) {
        const int ih = oh0 + prow[s] - 1;
        // absolute (non-negative) voffset: the buffer range check sees the halo zero-fill as OOB
        xoff[s] = pok[s] && (unsigned)ih < (unsigned)a.H ? iss_xbase + prel[s] : OOB;
      }
    }
    st = smem + (step % STAGES) * C::STAGE;
    cb = (iss_cbase + c) * CK * 2;
  };
  // s: compile-time after unrolling.  `live` false (no next stage: the block's last steps): the
  // DMA still issues -- a zero-fill into a 1-KiB dummy slot -- so there is no branch in the tap
  // loop (a branch there makes hipcc's waitcnt pass drain every fragment read, lgkmcnt(0))
  auto piece = [&](int s, char* st, int cb, bool live) {
    char* dummy = smem + C::DUMMY_OFF;
    if (s < C::PPW) glds16(xr, live ? st + (wid + NW * s) * 1024 : dummy, live ? xoff[s] : OOB, cb);
    else glds16(wr, live ? st + C::PATCH_BYTES + wdst[s - C::PPW] : dummy, live ? woff[s - C::PPW] : OOB, iss_wbase + cb);
  };

  // A/B fragment bases: patch pixel of tap (0, 0) for this lane's output row in each row block
  // (padded rows read a valid pixel and are never stored)
  int pb[RBW];
#pragma unroll
  for (int i = 0; i < RBW; ++i) {
    const int r = min((wid + NW * i) * 16 + fr, R - 1);
    const int img = fastdiv(r, a.mg_r);
    const int rem = r - img * (a.th * a.W);
    const int ohl = fastdiv(rem, a.mg_w), ow = rem - ohl * a.W;
    pb[i] = (img * TH2 + ohl) * W2 + ow;
  }
  const int wfo = (fr * 4 + (fq ^ wswz(fr))) * 16;  // this lane's weight-fragment byte offset

  f32x4 acc[RBW][CB];
#pragma unroll
  for (int i = 0; i < RBW; ++i)
#pragma unroll
    for (int j = 0; j < CB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the bias loads (before any DMA is in flight)
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nsteps) {
      char* st;
      int cb;
      prep(s, st, cb);
#pragma unroll
      for (int q = 0; q < LPS; ++q) piece(q, st, cb, true);
    }

  bool st_pending = false;  // the previous step ended with an item epilogue (its stores in flight)
  for (int step = 0; step < nsteps; ++step) {
    const int ahead = min(nsteps - 1, step + STAGES - 2) - step;  // younger stages allowed in flight
    if (st_pending) {
      if (STAGES > 2 && ahead > 0) wait_vm<(STAGES > 2 ? LPS : 0) + NST>();
      else wait_vm<NST>();
    } else {
      if (STAGES > 2 && ahead > 0) wait_vm<(STAGES > 2 ? LPS : 0)>();
      else wait_vm<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // stage `step` landed for every wave; stage step-1 fully read
    const bool nxt = step + STAGES - 1 < nsteps;  // block-uniform
    char* nst = smem;
    int ncb = 0;
    if (nxt) prep(step + STAGES - 1, nst, ncb);
    st_pending = false;

    const char* sP = smem + (step % STAGES) * C::STAGE;
    const char* sW = sP + C::PATCH_BYTES + wfo;
    bf16x8 wf[2][CB], pf[2][RBW];
    auto load = [&](int tap, int buf) {
      const int toff = (tap / 3) * W2 + (tap % 3);
#pragma unroll
      for (int j = 0; j < CB; ++j)
        wf[buf][j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sW + (tap * BN + j * 16) * 64));
#pragma unroll
      for (int i = 0; i < RBW; ++i)
        pf[buf][i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sP + patch_addr(pb[i] + toff, fq)));
    };
    load(0, 0);
    // software pipeline over the taps: tap t + 1's fragments are read (and this tap's share of the
    // next stage's DMA issued) before tap t's MFMAs; the sched barriers keep hipcc from sinking the
    // reads next to their MFMAs (it otherwise re-uses one fragment set and waits lgkmcnt(0) per tap)
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int cur = tap & 1;
      if (tap + 1 < 9) load(tap + 1, cur ^ 1);
#pragma unroll
      for (int q = 0; q < LPS; ++q)
        if (q * 9 / LPS == tap) piece(q, nst, ncb, nxt);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < RBW; ++i)
#pragma unroll
        for (int j = 0; j < CB; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[cur][j], pf[cur][i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }

    const int sq = fastdiv(step, a.mg_nck);
    if (step - sq * nck != nck - 1) continue;  // not the item's last chunk

    // ---- item epilogue: lane = output pixel (rb*16 + fr) x 4 consecutive channels per column block
    int tile, tn, split;
    decode(first + sq, tile, tn, split);
    const long m_base = (long)tile * R;
    const int n0 = tn * BN;
    if (a.ksplit > 1) {
      const rsrc_t wsr = make_rsrc(a.ws, a.ws_bytes);
#pragma unroll
      for (int i = 0; i < RBW; ++i) {
        const int r = (wid + NW * i) * 16 + fr;
#pragma unroll
        for (int j = 0; j < CB; ++j) {
          const long idx = ((long)split * M + m_base + r) * a.N + n0 + j * 16 + fq * 4;
          const float v0 = acc[i][j][0], v1 = acc[i][j][1], v2 = acc[i][j][2], v3 = acc[i][j][3];
          const pipe_u32x4 q = {__float_as_uint(v0), __float_as_uint(v1), __float_as_uint(v2), __float_as_uint(v3)};
          __builtin_amdgcn_raw_buffer_store_b128(q, wsr, r < R ? (int)(idx * 4) : OOB, 0, 16);  // sc1
        }
      }
      // every wave's slab stores (and the ring's in-flight DMA) drained, then one ticket
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      int* flag = reinterpret_cast<int*>(smem + C::FLAG_OFF);
      if (tid == 0) {
        int* c = a.cnt + tn * a.tiles + tile;
        const int prev = __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = prev == a.ksplit - 1;
        if (last) __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
        *flag = last;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      const bool last = *reinterpret_cast<volatile int*>(flag) != 0;
      __builtin_amdgcn_s_barrier();  // the flag is read before the next item can reuse it
      if (!last) {
#pragma unroll
        for (int i = 0; i < RBW; ++i)
#pragma unroll
          for (int j = 0; j < CB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        continue;
      }
      // last arriver: add the other slices' slabs (sc1 loads: no acquire needed)
      for (int sl = 0; sl < a.ksplit; ++sl) {
        if (sl == split) continue;
#pragma unroll
        for (int i = 0; i < RBW; ++i) {
          const int r = (wid + NW * i) * 16 + fr;
#pragma unroll
          for (int j = 0; j < CB; ++j) {
            const long idx = ((long)sl * M + m_base + r) * a.N + n0 + j * 16 + fq * 4;
            const float4 v = __builtin_bit_cast(
                float4, __builtin_amdgcn_raw_buffer_load_b128(wsr, r < R ? (int)(idx * 4) : OOB, 0, 16));
            acc[i][j][0] += v.x;
            acc[i][j][1] += v.y;
            acc[i][j][2] += v.z;
            acc[i][j][3] += v.w;
          }
        }
      }
    }
    const rsrc_t orr = make_rsrc(a.out, a.o_bytes);
    const float lo = a.act == ACT_RELU ? 0.f : -INFINITY;  // host: ACT_NONE / ACT_RELU only
#pragma unroll
    for (int j = 0; j < CB; ++j) {
      const float4 bb = *reinterpret_cast<const float4*>(sbias + n0 + j * 16 + fq * 4);
#pragma unroll
      for (int i = 0; i < RBW; ++i) {
        const int r = (wid + NW * i) * 16 + fr;
        const float v0 = acc[i][j][0], v1 = acc[i][j][1], v2 = acc[i][j][2], v3 = acc[i][j][3];
        bf16x4 q;
        q[0] = (bf16)fmaxf(v0 + bb.x, lo);
        q[1] = (bf16)fmaxf(v1 + bb.y, lo);
        q[2] = (bf16)fmaxf(v2 + bb.z, lo);
        q[3] = (bf16)fmaxf(v3 + bb.w, lo);
        const long o = (m_base + r) * a.N + n0 + j * 16 + fq * 4;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(pipe_u32x2, q), orr, r < R ? (int)(o * 2) : OOB, 0, 0);
        acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    st_pending = a.ksplit == 1;  // split-K drained its stores above
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Item geometry as conv3x3_halo.hip: the largest th dividing H with th * W <= max_rows and
// (th + 2) * (W + 2) <= PMAX; whole images (th == H) packed nb per item (nb | B).
bool pipe_geometry(int B, int H, int W, int max_rows, int pmax, int* th, int* nb) {
  for (int t = H; t >= 1; --t) {
    if (H % t || t * W > max_rows || (t + 2) * (W + 2) > pmax) continue;
    int n = 1;
    if (t == H)
      for (int c = 8; c >= 1; --c)
        if (B % c == 0 && c * H * W <= max_rows && c * (H + 2) * (W + 2) <= pmax) {
          n = c;
          break;
        }
    *th = t;
    *nb = n;
    return true;
  }
  return false;
}

// variant -> (BN, NW, RBW, STAGES, PPC); max_rows of the geometry = 16 * NW * RBW (<= 256),
// patch pixels <= 16 * PPC
struct PipeVariant {
  int bn, nw, rbw, stages, ppc;
};
constexpr PipeVariant kPipeVariants[] = {
    {64, 4, 4, 2, 24},  // 0: 256-pixel items x 64 channels, 4 waves of 4 x 4 tiles
    {32, 4, 4, 2, 24},  // 1: x 32 channels (2x the items of the small-M layers)
    {32, 4, 4, 3, 24},  // 2: x 32 channels, 3-stage ring
    {64, 8, 2, 2, 24},  // 3: 8 waves of 2 x 4 tiles
    {64, 4, 2, 2, 24},  // 4: 128-pixel items x 64 channels (layer1 / layer2: 2x the items)
    {32, 4, 2, 3, 24},  // 5: 128-pixel items x 32 channels, 3 stages
    {64, 8, 2, 3, 16},  // 6: <= 256-pixel patches, 8 waves, 3 stages (52 KB each)
    {64, 4, 2, 3, 16},  // 7: 128-pixel items, 4 waves of 2 x 4, 3 stages
    {64, 8, 1, 3, 16},  // 8: 128-pixel items, 8 waves of 1 x 4, 3 stages
    {32, 8, 2, 3, 16},  // 9: x 32 channels, 8 waves, 3 stages
    {32, 8, 2, 4, 16},  // 10: x 32 channels, 8 waves, 4 stages (34 KB each)
    {64, 8, 2, 2, 16},  // 11: variant 6 with 2 stages
};
constexpr int kNumPipeVariants = sizeof(kPipeVariants) / sizeof(kPipeVariants[0]);

template <int BN, int NW, int RBW, int STAGES, int PPC>
void launch_pipe(dim3 grid, hipStream_t st, const PipeArgs& a) {
  hipLaunchKernelGGL((conv3x3_pipe_kernel<BN, NW, RBW, STAGES, PPC>), grid, dim3(NW * 64), 0, st, a);
}

}  // namespace

extern "C" {

// 3x3 / stride 1 / pad 1 conv: x [B][H][W][Cin] bf16, w [N][3][3][Cin] bf16, bias fp32 [N] or null;
// out [B][H][W][N] bf16 = act(conv + bias).  Cin % 32 == 0, N % BN == 0, N <= 512.  splitk > 1:
// input-channel chunks split over that many items per tile, reduced in the same launch through fp32
// slabs in ws (>= splitk * B*H*W*N floats) and this stream's arrival counters; ipb = items per block.
int mls_conv3x3_pipe(const void* x, const void* w, const float* bias, void* out, void* ws, size_t ws_bytes, int B,
                     int H, int W, int Cin, int N, int act, int variant, int splitk, int ipb, void* stream) {
  if (variant < 0 || variant >= kNumPipeVariants) return MLS_BAD_ARG;
  const PipeVariant v = kPipeVariants[variant];
  if (B <= 0 || H <= 0 || W <= 0 || Cin <= 0 || Cin % CK || N <= 0 || N % v.bn || N > NMAX || ipb < 1)
    return MLS_BAD_ARG;
  if (act != ACT_NONE && act != ACT_RELU) return MLS_UNSUPPORTED;
  int th = 0, nb = 0;
  const int max_rows = 16 * v.nw * v.rbw;
  if (!pipe_geometry(B, H, W, max_rows < MAX_ROWS ? max_rows : MAX_ROWS, 16 * v.ppc, &th, &nb)) return MLS_UNSUPPORTED;
  const long xb = (long)B * H * W * Cin * 2, wb = (long)N * 9 * Cin * 2, ob = (long)B * H * W * N * 2;
  if (xb >= 0x7fffffffL || wb >= 0x7fffffffL || ob >= 0x7fffffffL) return MLS_UNSUPPORTED;
  PipeArgs a;
  a.x = (const bf16*)x;
  a.w = (const bf16*)w;
  a.bias = bias;
  a.out = (bf16*)out;
  a.B = B, a.H = H, a.W = W, a.Cin = Cin, a.N = N, a.th = th, a.nb = nb, a.act = act;
  a.x_bytes = (uint32_t)xb;
  a.w_bytes = (uint32_t)wb;
  a.o_bytes = (uint32_t)ob;
  a.tiles = (B / nb) * (H / th);
  a.ntn = N / v.bn;
  a.ksplit = 1;
  a.ws = nullptr;
  a.cnt = nullptr;
  a.ws_bytes = 0;
  const long slab = (long)splitk * B * H * W * N * 4;
  if (splitk > 1 && (Cin / CK) % splitk == 0 && ws && (long)ws_bytes >= slab && slab < 0x7fffffffL) {
    int* cnt = mls_stream_splitk_counters(stream, (long)a.tiles * a.ntn);
    if (cnt) {
      a.ksplit = splitk;
      a.ws = (float*)ws;
      a.cnt = cnt;
      a.ws_bytes = (uint32_t)slab;
    }
  }
  a.nitems = a.tiles * a.ntn * a.ksplit;
  a.ipb = ipb;
  a.nck = Cin / CK / a.ksplit;
  a.tpi = H / th;
  a.mg_p2 = fastdiv_make((th + 2) * (W + 2));
  a.mg_w2 = fastdiv_make(W + 2);
  a.mg_r = fastdiv_make(th * W);
  a.mg_w = fastdiv_make(W);
  a.mg_ks = fastdiv_make(a.ksplit);
  a.mg_ntn = fastdiv_make(a.ntn);
  a.mg_nck = fastdiv_make(a.nck);
  a.mg_tpi = fastdiv_make(a.tpi);

  const dim3 grid((unsigned)((a.nitems + ipb - 1) / ipb));
  hipStream_t st = (hipStream_t)stream;
  switch (variant) {
    case 0: launch_pipe<64, 4, 4, 2, 24>(grid, st, a); break;
    case 1: launch_pipe<32, 4, 4, 2, 24>(grid, st, a); break;
    case 2: launch_pipe<32, 4, 4, 3, 24>(grid, st, a); break;
    case 3: launch_pipe<64, 8, 2, 2, 24>(grid, st, a); break;
    case 4: launch_pipe<64, 4, 2, 2, 24>(grid, st, a); break;
    case 5: launch_pipe<32, 4, 2, 3, 24>(grid, st, a); break;
    case 6: launch_pipe<64, 8, 2, 3, 16>(grid, st, a); break;
    case 7: launch_pipe<64, 4, 2, 3, 16>(grid, st, a); break;
    case 8: launch_pipe<64, 8, 1, 3, 16>(grid, st, a); break;
    case 9: launch_pipe<32, 8, 2, 3, 16>(grid, st, a); break;
    case 10: launch_pipe<32, 8, 2, 4, 16>(grid, st, a); break;
    case 11: launch_pipe<64, 8, 2, 2, 16>(grid, st, a); break;
    default: return MLS_BAD_ARG;
  }
  return (int)hipGetLastError();
}

// The item geometry (output rows per item, images per item) a variant uses: 0 + th, nb.
int mls_conv3x3_pipe_geometry(int B, int H, int W, int variant, int* th, int* nb) {
  if (variant < 0 || variant >= kNumPipeVariants) return MLS_BAD_ARG;
  const PipeVariant v = kPipeVariants[variant];
  const int max_rows = 16 * v.nw * v.rbw;
  return pipe_geometry(B, H, W, max_rows < MAX_ROWS ? max_rows : MAX_ROWS, 16 * v.ppc, th, nb) ? 0 : MLS_UNSUPPORTED;
}

int mls_conv3x3_pipe_num_variants() { return kNumPipeVariants; }

}  // extern "C"
