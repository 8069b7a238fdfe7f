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
};

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

template <int BM, int BN, int WM, int WN, int STAGES, int BKS>
__global__ __launch_bounds__(WM * WN * 64) void gemm_tile_kernel(const GemmTileArgs g) {
  constexpr int NT = WM * WN * 64;
  constexpr int WTM = BM / WM, WTN = BN / WN;  // wave tile: WTM rows (m) x WTN columns (n)
  constexpr int MT = WTM / 16, NTL = WTN / 16;
  constexpr int ROWB = BKS * 2, CPR = ROWB / 16;  // bytes / 16-B chunks per LDS row
  constexpr int A_BYTES = BM * ROWB, B_BYTES = BN * ROWB, STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int A_LD = A_BYTES / (NT * 16), B_LD = B_BYTES / (NT * 16), LOADS = A_LD + B_LD;
  static_assert(A_BYTES % (NT * 16) == 0 && B_BYTES % (NT * 16) == 0, "stage must split into whole DMA rounds");
  static_assert(BKS == 32 || BKS == 64, "stage depth");
  __shared__ __attribute__((aligned(16))) char smem[STAGES * STAGE_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid - wm * WN;
  const int tiles_m = (g.M + BM - 1) / BM, ntiles = tiles_m * g.tiles_n;
  // persistent: block b takes logical tiles b', b' + G, b' + 2G, ... where b' = XCD-contiguous
  // remap of b -- at every round an XCD works on a contiguous (N-fastest) run of tiles
  const int G = gridDim.x, bq = xcd_remap(blockIdx.x, G);
  const int my_tiles = bq < ntiles ? (ntiles - 1 - bq) / G + 1 : 0;
  const int nk = g.K / BKS, nsteps = my_tiles * nk;

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

  auto tile_mn = [&](int ti, int& m0, int& n0) {
    int tm, tn;
    gt_tile(bq + ti * G, tiles_m, g.tiles_n, tm, tn);
    m0 = tm * BM;
    n0 = tn * BN;
  };
  // loader cursor: the (tile, k-step) of the next DMA, advanced without divisions
  int l_ti = 0, l_kt = 0, l_m0 = 0, l_n0 = 0, l_slot = 0;
  if (nsteps > 0) tile_mn(0, l_m0, l_n0);
  auto stage = [&]() {  // DMA the loader cursor's k-step into ring slot l_slot, then advance it
    const int kt = l_kt, m0 = l_m0, n0 = l_n0;
    char* base = smem + l_slot * STAGE_BYTES + wid * 1024;
    l_slot = l_slot + 1 == STAGES ? 0 : l_slot + 1;
    if (++l_kt == nk) {
      l_kt = 0;
      if (++l_ti < my_tiles) tile_mn(l_ti, l_m0, l_n0);
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
  const bool glu = g.act == ACT_SILU_MUL;

#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nsteps) stage();

  int c_kt = 0, c_ti = 0, c_slot = 0;  // compute cursor
  for (int j = 0; j < nsteps; ++j) {
    gt_wait_ring<STAGES, LOADS>(nsteps - 1 - j);  // step j landed; later ones may still fly
    gt_barrier();  // step j visible to every wave; step j - 1 fully read by every wave
    if (j + STAGES - 1 < nsteps) stage();
    const char* base = smem + c_slot * STAGE_BYTES;
    c_slot = c_slot + 1 == STAGES ? 0 : c_slot + 1;
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
    if (++c_kt < nk) continue;
    c_kt = 0;

    // ---- epilogue of this tile (the next tile's first k-steps are already in flight) ----
    // lane holds D[n = 4*fq + r][m = fr] of each 16 x 16 tile -> row m, 4 consecutive columns
    int m0, n0;
    tile_mn(c_ti++, m0, n0);
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int m = m0 + wm * WTM + i * 16 + fr;
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn) {
        const int nt0 = n0 + wn * WTN + jn * 16;  // first column of this 16-column tile
        const int n = nt0 + 4 * fq;
        float v[4] = {acc[i][jn][0], acc[i][jn][1], acc[i][jn][2], acc[i][jn][3]};
        acc[i][jn] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (glu) {
          // columns nt0..nt0+7 are gate, nt0+8..nt0+15 up: lane l < 32 holds gate, lane l + 32 its up
          float u[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) u[e] = xor32_f(v[e]);
          if (fq < 2 && m < g.M && nt0 < g.N) {
            float o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float gt = v[e] + (g.bias ? g.bias[n + e] : 0.f);
              const float up = u[e] + (g.bias ? g.bias[n + 8 + e] : 0.f);
              o[e] = silu(gt) * up;
            }
            bf16x4 b = {(bf16)o[0], (bf16)o[1], (bf16)o[2], (bf16)o[3]};
            *reinterpret_cast<bf16x4*>(g.out + (size_t)m * g.ldo + (nt0 >> 1) + 4 * fq) = b;
          }
          continue;
        }
        if (m >= g.M || n >= g.N) continue;
        if (g.bias) {
          const float4 b = *reinterpret_cast<const float4*>(g.bias + n);
          v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
        }
        if (g.act != ACT_NONE) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = apply_act(v[e], g.act);
        }
        if (g.res) {
          const bf16x4 r = *reinterpret_cast<const bf16x4*>(g.res + (size_t)m * g.ldr + n);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += (float)r[e];
        }
        bf16x4 b = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
        *reinterpret_cast<bf16x4*>(g.out + (size_t)m * g.ldo + n) = b;
      }
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
  const bool glu = g.act == ACT_SILU_MUL;

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
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int m = m0 + wm * WTM + i * 16 + fr;
#pragma unroll
        for (int jn = 0; jn < NTL; ++jn) {
          const int nt0 = n0 + wn * WTN + jn * 16, n = nt0 + 4 * fq;
          float v[4] = {acc[i][jn][0], acc[i][jn][1], acc[i][jn][2], acc[i][jn][3]};
          acc[i][jn] = f32x4{0.f, 0.f, 0.f, 0.f};
          if (glu) {
            float u[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) u[e] = xor32_f(v[e]);
            if (fq < 2 && m < g.M && nt0 < g.N) {
              float o[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const float gt_ = v[e] + (g.bias ? g.bias[n + e] : 0.f);
                const float up = u[e] + (g.bias ? g.bias[n + 8 + e] : 0.f);
                o[e] = silu(gt_) * up;
              }
              bf16x4 b = {(bf16)o[0], (bf16)o[1], (bf16)o[2], (bf16)o[3]};
              *reinterpret_cast<bf16x4*>(g.out + (size_t)m * g.ldo + (nt0 >> 1) + 4 * fq) = b;
            }
            continue;
          }
          if (m >= g.M || n >= g.N) continue;
          if (g.bias) {
            const float4 b = *reinterpret_cast<const float4*>(g.bias + n);
            v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
          }
          if (g.act != ACT_NONE) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = apply_act(v[e], g.act);
          }
          if (g.res) {
            const bf16x4 r = *reinterpret_cast<const bf16x4*>(g.res + (size_t)m * g.ldr + n);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += (float)r[e];
          }
          bf16x4 b = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
          *reinterpret_cast<bf16x4*>(g.out + (size_t)m * g.ldo + n) = b;
        }
      }
    }
    if (grp == 0) gt_wait_vmcnt<0>();  // group 0's A half of stage j + 1
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
  const dim3 grid(ntiles < cap ? ntiles : cap), block(c.threads);
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
  }
  return hipGetLastError() == hipSuccess ? MLS_OK : MLS_BAD_ARG;
}

// default tile by shape: the largest tile that still gives the chip >= ~1 block per CU, else the
// one with the most blocks (the projection GEMMs run under 4-5-way stream concurrency in serving)
int gt_pick(int M, int N) {
  auto blocks = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
  if (blocks(256, 256) >= 256) return 1;
  if (blocks(256, 128) >= 256) return 2;
  if (blocks(128, 256) >= 256) return 5;
  return 4;
}

}  // namespace

extern "C" {

// out[M][N] = act(A[M][K] . W[N][K]^T + bias (+ res));  ACT_SILU_MUL: W rows gate/up interleaved in
// groups of 8, out [M][N/2].  K % 64 == 0, N % 16 == 0; cfg 0 = pick by shape; grid_cap 0 = one
// resident wave of persistent blocks.
int mls_gemm_tile(const void* A, const void* W, const float* bias, const void* res, void* out, int M, int N, int K,
                  int act, int ldo, int ldr, int cfg, int grid_cap, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || K % 64 || N % 16 || (res && act == ACT_SILU_MUL)) return MLS_BAD_ARG;
  const size_t ab = (size_t)M * K * 2, wb = (size_t)N * K * 2;
  if (ab >= 0x7FFFFFFFull || wb >= 0x7FFFFFFFull || (size_t)M * ldo >= 0x7FFFFFFFFFull) return MLS_UNSUPPORTED;
  GemmTileArgs g{};
  g.a = (const bf16*)A;
  g.w = (const bf16*)W;
  g.bias = bias;
  g.res = (const bf16*)res;
  g.out = (bf16*)out;
  g.M = M; g.N = N; g.K = K; g.act = act;
  g.ldo = ldo > 0 ? ldo : (act == ACT_SILU_MUL ? N / 2 : N);
  g.ldr = ldr > 0 ? ldr : N;
  g.a_bytes = (uint32_t)ab;
  g.w_bytes = (uint32_t)wb;
  return gt_launch(g, cfg > 0 ? cfg : gt_pick(M, N), grid_cap, (hipStream_t)stream);
}

int mls_gemm_tile_pick(int M, int N) { return gt_pick(M, N); }

}  // extern "C"
