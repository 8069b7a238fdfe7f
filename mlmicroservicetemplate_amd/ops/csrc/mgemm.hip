// Medium-M weight-streaming GEMM for the 17..256-row decode projections of continuous batching
// (Llama-3-8B at 128-256 slots): out[M][N] = act(A[M][K] . W[N][K]^T + bias) (+ residual).
//
// Why a third GEMM shape: at M = 256 a projection reads its weights once (33.5 MB for o_proj) and
// does 2 * 256 FLOP per weight element, so it should run at the HBM rate (~5 us for o_proj); the
// tile kernels run the shape at 1.4 TB/s (23.5 us, conv_gemm 128x64 split 2, README route table):
// with W staged through the same LDS ring as A and 2-3 stages in flight per block, each k-step waits
// a full HBM round trip.  The skinny kernel (W straight to VGPRs) holds at most 32 rows.
//
// Layout (256 threads = 4 waves, one block per 64-column slice of N and K slice of the split):
//  * every wave owns 16 output columns and ALL M rows (RT 16-row tiles): per 32-wide k-step it
//    issues ONE 16-B weight load per lane straight into a register ring LW steps deep -- weights
//    never touch LDS and ~LW x 4 KB of them are in flight per block;
//  * A (the activations, L2-resident, shared by the 4 waves) goes through a 4-stage LDS-DMA ring
//    (buffer_load ... lds, 16 rows x 64 B per 1-KiB piece, chunks XOR-swizzled on the source side
//    so the ds_read_b128 fragment reads are conflict-free), counted vmcnt + one barrier per k-step;
//  * v_mfma_f32_16x16x32_bf16 with A as the row operand: a lane's 4 accumulators are 4 rows of one
//    output column;
//  * split 1: the block's 16 x RT-row x 64 tile is parked in LDS and written as 16-B bf16 rows with
//    bias / act / SiLU-mul (gate/up interleaved in 8-column groups) / residual fused; split > 1:
//    fp32 slabs [split][M][N] and mgemm_finish_kernel (slice order -> deterministic).
#include "common.h"

namespace {

#define LDS3 __attribute__((address_space(3)))

struct MgArgs {
  const bf16* a;     // [M][lda]
  const bf16* w;     // [N][K]
  const float* bias;  // [N] or null
  const bf16* res;   // [M][ldo] or null
  bf16* out;         // [M][ldo]  (ldo = N, or N / 2 with SiLU-mul)
  float* ws;         // [split][M][N] fp32 slabs (split > 1)
  int M, N, K, lda, ldo, act, split, kchunk;
  uint32_t a_bytes, w_bytes;
};

constexpr int MG_BN = 64;   // columns per block (4 waves x 16)
constexpr int MG_SA = 4;    // A ring stages (k-steps of 32)
constexpr int MG_LW = 8;    // weight register ring depth (k-steps)
constexpr int MG_UNR = 8;   // k-loop unroll = lcm(MG_SA, MG_LW): static ring indices
constexpr int MG_CLD = MG_BN + 4;  // parked-tile row stride (floats)

MLS_DEV int mg_swz(int r) { return (r & 1) | ((r >> 1) & 2); }  // 64-B rows: conv_gemm.hip row_swz<32>

MLS_DEV void mg_glds16(rsrc_t r, char* lds, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDS3 void*)lds, 16, voff, 0, 0, 0);
}

template <int RT>
__global__ __launch_bounds__(256) void mgemm_kernel(const MgArgs g) {
  constexpr int A_ST = RT * 16 * 64;  // one k-step of A: RT*16 rows x 32 bf16
  constexpr int PPW = RT / 4;         // 1-KiB DMA pieces per wave per stage
  static_assert(PPW * 4 == RT, "RT multiple of 4");
  constexpr int RING = MG_SA * A_ST;
  constexpr int PARK = RT * 16 * MG_CLD * 4;
  constexpr int LDS = RING > PARK ? RING : PARK;
  __shared__ __attribute__((aligned(16))) char smem[LDS];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int n0 = blockIdx.x * MG_BN;
  const int split = blockIdx.y;
  const int kbeg = split * g.kchunk;
  const int nk = g.kchunk / 32;

  const rsrc_t ar = make_rsrc(g.a, g.a_bytes);
  const rsrc_t wr = make_rsrc(g.w, g.w_bytes);

  // A DMA lane geometry: piece = 16 rows x 4 chunks; lane -> row r4, physical chunk pc holds the
  // source's logical chunk pc ^ swz(r4)
  const int r4 = lane >> 2, pc = lane & 3;
  const int lsrc = ((pc ^ mg_swz(r4)) * 8) * 2;
  int a_row_off[PPW];
#pragma unroll
  for (int j = 0; j < PPW; ++j) {
    const int m = (wid * PPW + j) * 16 + r4;
    a_row_off[j] = m < g.M ? m * g.lda * 2 + lsrc : OOB;
  }
  // weight fragment of this lane: column n0 + 16 wid + fr, k group fq
  const int wn = n0 + wid * 16 + fr;
  const int w_off0 = wn < g.N ? (wn * g.K + kbeg + fq * 8) * 2 : OOB;

  auto issue_a = [&](int kt) {  // stage kt % MG_SA (kt >= nk: zeros, no traffic)
    char* dst = smem + (kt % MG_SA) * A_ST;
    const bool live = kt < nk;
    const int kb = (kbeg + kt * 32) * 2;
#pragma unroll
    for (int j = 0; j < PPW; ++j)
      mg_glds16(ar, dst + (wid * PPW + j) * 1024, live && a_row_off[j] != OOB ? a_row_off[j] + kb : OOB);
  };
  auto load_w = [&](int kt) -> uint4 {
    return bload16(wr, kt < nk && w_off0 != OOB ? w_off0 + kt * 64 : OOB);
  };

  f32x4 acc[RT];
#pragma unroll
  for (int i = 0; i < RT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: the weight ring runs MG_LW - (MG_SA - 1) steps further ahead than the A ring; then
  // (A(j), W(j + MG_LW - MG_SA + 1)) pairs -- the steady-state order, so one vmcnt count fits every step
  uint4 wreg[MG_LW];
  constexpr int WLEAD = MG_LW - (MG_SA - 1);
#pragma unroll
  for (int j = 0; j < WLEAD; ++j) wreg[j] = load_w(j);
#pragma unroll
  for (int j = 0; j < MG_SA - 1; ++j) {
    issue_a(j);
    wreg[j + WLEAD] = load_w(j + WLEAD);
  }
  // at the top of step kt, issued after A(kt): W(kt + WLEAD) and (MG_SA - 2) more (A, W) pairs
  constexpr int WAIT_A = 1 + (MG_SA - 2) * (PPW + 1);

  for (int kt0 = 0; kt0 < nk; kt0 += MG_UNR) {
#pragma unroll
    for (int u = 0; u < MG_UNR; ++u) {
      const int kt = kt0 + u;
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WAIT_A) : "memory");
      __builtin_amdgcn_s_barrier();  // stage kt complete (all waves' pieces); stage kt - 1 free
      const uint4 wcur = wreg[u % MG_LW];
      issue_a(kt + MG_SA - 1);
      wreg[u % MG_LW] = load_w(kt + MG_LW);
      const char* st = smem + (kt % MG_SA) * A_ST;
      const bf16x8 wf = __builtin_bit_cast(bf16x8, wcur);
#pragma unroll
      for (int i = 0; i < RT; ++i) {
        const int row = i * 16 + fr;
        const bf16x8 af = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(st + row * 64 + ((fq ^ mg_swz(fr)) << 4)));
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, wf, acc[i], 0, 0, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // the look-ahead (zero) DMA landed
  __syncthreads();

  // D[row 4 fq + r][col fr] of row tile i -> parked tile Cs[row][16 wid + fr]
  float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < RT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float e = acc[i][r];  // through a named float (ext-vector element bit-cast hazard)
      Cs[(i * 16 + fq * 4 + r) * MG_CLD + wid * 16 + fr] = e;
    }
  __syncthreads();

  const int rows = min(RT * 16, g.M);
  if (g.split > 1) {  // fp32 slab rows of 8 columns
    for (int q = tid; q < rows * (MG_BN / 8); q += 256) {
      const int m = q / (MG_BN / 8), c = q % (MG_BN / 8);
      const int n = n0 + c * 8;
      if (n >= g.N) continue;
      const float* src = Cs + m * MG_CLD + c * 8;
      float* dst = g.ws + ((size_t)split * g.M + m) * g.N + n;
      *reinterpret_cast<float4*>(dst) = *reinterpret_cast<const float4*>(src);
      *reinterpret_cast<float4*>(dst + 4) = *reinterpret_cast<const float4*>(src + 4);
    }
    return;
  }
  if (g.act == ACT_SILU_MUL) {  // 8 gate + 8 up columns -> 8 outputs at n / 2
    for (int q = tid; q < rows * (MG_BN / 16); q += 256) {
      const int m = q / (MG_BN / 16), p = q % (MG_BN / 16);
      const int n = n0 + p * 16;
      if (n >= g.N) continue;
      const float* src = Cs + m * MG_CLD + p * 16;
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float gt = src[e] + (g.bias ? g.bias[n + e] : 0.f);
        const float up = src[8 + e] + (g.bias ? g.bias[n + 8 + e] : 0.f);
        o[e] = silu(gt) * up;
      }
      st16(g.out + (size_t)m * g.ldo + (n >> 1), pack8(o));
    }
    return;
  }
  for (int q = tid; q < rows * (MG_BN / 8); q += 256) {
    const int m = q / (MG_BN / 8), c = q % (MG_BN / 8);
    const int n = n0 + c * 8;
    if (n >= g.N) continue;
    const float* src = Cs + m * MG_CLD + c * 8;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = src[e] + (g.bias ? g.bias[n + e] : 0.f);
    if (g.res) {
      float r[8];
      unpack8(ld16(g.res + (size_t)m * g.ldo + n), r);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += r[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = apply_act(v[e], g.act);
    st16(g.out + (size_t)m * g.ldo + n, pack8(v));
  }
}

// split > 1: sum the slabs in slice order, then the same epilogue as split 1
__global__ __launch_bounds__(256) void mgemm_finish_kernel(const MgArgs g) {
  const bool glu = g.act == ACT_SILU_MUL;
  const int cw = glu ? 16 : 8;
  const int cpr = g.N / cw;
  const long q = (long)blockIdx.x * 256 + threadIdx.x;
  if (q >= (long)g.M * cpr) return;
  const int m = (int)(q / cpr), n = (int)(q % cpr) * cw;
  float v[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) v[e] = 0.f;
  for (int s = 0; s < g.split; ++s) {
    const float* src = g.ws + ((size_t)s * g.M + m) * g.N + n;
    const float4 x0 = *reinterpret_cast<const float4*>(src), x1 = *reinterpret_cast<const float4*>(src + 4);
    v[0] += x0.x; v[1] += x0.y; v[2] += x0.z; v[3] += x0.w; v[4] += x1.x; v[5] += x1.y; v[6] += x1.z; v[7] += x1.w;
    if (glu) {
      const float4 y0 = *reinterpret_cast<const float4*>(src + 8), y1 = *reinterpret_cast<const float4*>(src + 12);
      v[8] += y0.x; v[9] += y0.y; v[10] += y0.z; v[11] += y0.w; v[12] += y1.x; v[13] += y1.y; v[14] += y1.z; v[15] += y1.w;
    }
  }
  float o[8];
  if (glu) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float gt = v[e] + (g.bias ? g.bias[n + e] : 0.f);
      const float up = v[8 + e] + (g.bias ? g.bias[n + 8 + e] : 0.f);
      o[e] = silu(gt) * up;
    }
    st16(g.out + (size_t)m * g.ldo + (n >> 1), pack8(o));
    return;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = v[e] + (g.bias ? g.bias[n + e] : 0.f);
  if (g.res) {
    float r[8];
    unpack8(ld16(g.res + (size_t)m * g.ldo + n), r);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] += r[e];
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = apply_act(o[e], g.act);
  st16(g.out + (size_t)m * g.ldo + n, pack8(o));
}

template <int RT>
void launch_mg(const MgArgs& g, hipStream_t st) {
  hipLaunchKernelGGL((mgemm_kernel<RT>), dim3(g.N / MG_BN, g.split), dim3(256), 0, st, g);
}

}  // namespace

extern "C" {

// The split the launcher picks for split <= 0: the most K slices (each a multiple of 256 dividing K)
// that keep the grid within `blocks` (default 256, one per CU: every extra slice adds an fp32 slab
// of M x N to write and read back).
int mls_mgemm_auto_split(int N, int K, int blocks) {
  const int cols = N / MG_BN;
  if (blocks <= 0) blocks = 256;
  int best = 1;
  for (int s = 1; s <= 16; ++s) {
    if (K % (s * 32 * MG_UNR)) continue;
    if (cols * s <= blocks) best = s;
  }
  return best;
}

// A [M][lda] bf16 (0 < M <= 256, lda >= K, lda % 8 == 0), W [N][K] bf16 (N % 64 == 0, K % 256 == 0),
// bias fp32 [N] or null, res [M][N] bf16 or null (not with SiLU-mul), out [M][N] (act SiLU-mul:
// [M][N/2], gate/up interleaved in 8-column groups of W).  split <= 0: auto; K % (split * 256) == 0;
// split > 1 needs ws of >= split * M * N floats (ws_bytes).
int mls_mgemm(const void* A, const void* W, const float* bias, const void* res, void* out, void* ws,
              size_t ws_bytes, int M, int N, int K, int lda, int act, int split, void* stream) {
  if (!A || !W || !out || M <= 0 || M > 256 || N <= 0 || N % MG_BN || K <= 0 || K % (32 * MG_UNR) || lda < K ||
      lda % 8)
    return MLS_BAD_ARG;
  const bool glu = act == ACT_SILU_MUL;
  if (glu && res) return MLS_BAD_ARG;
  if (split <= 0) split = mls_mgemm_auto_split(N, K, 0);
  if (K % (split * 32 * MG_UNR)) return MLS_BAD_ARG;
  const size_t wbytes = (size_t)N * K * 2, abytes = ((size_t)(M - 1) * lda + K) * 2;
  if (wbytes >= 0x80000000ull || abytes >= 0x80000000ull) return MLS_UNSUPPORTED;
  if (split > 1 && (!ws || ws_bytes < (size_t)split * M * N * 4)) return MLS_BAD_ARG;
  MgArgs g{};
  g.a = (const bf16*)A;
  g.w = (const bf16*)W;
  g.bias = bias;
  g.res = (const bf16*)res;
  g.out = (bf16*)out;
  g.ws = (float*)ws;
  g.M = M, g.N = N, g.K = K, g.lda = lda, g.ldo = glu ? N / 2 : N, g.act = act;
  g.split = split, g.kchunk = K / split;
  g.a_bytes = (uint32_t)abytes, g.w_bytes = (uint32_t)wbytes;
  const hipStream_t st = (hipStream_t)stream;
  if (M <= 64) launch_mg<4>(g, st);
  else if (M <= 128) launch_mg<8>(g, st);
  else launch_mg<16>(g, st);
  if (split > 1) {
    const long items = (long)M * (N / (glu ? 16 : 8));
    hipLaunchKernelGGL(mgemm_finish_kernel, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, st, g);
  }
  return (int)hipGetLastError();
}

}  // extern "C"
