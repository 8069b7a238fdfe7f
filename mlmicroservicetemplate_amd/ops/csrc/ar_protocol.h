// One-shot IPC all-reduce protocol pieces shared by the standalone collective
// (custom_allreduce.hip) and the GEMMs that run it in their own epilogue (skinny_gemm.hip: the
// tensor-parallel decode's row-parallel projections -- o and down -- reduce their partial output
// across ranks in the SAME launch, no separate all-reduce kernel).
//
// Chunk c of a message (AR_ELEMS_PER_BLOCK bf16 elements) is owned by AR block c in both users and
// advances the same per-chunk device epoch, so standalone and fused calls interleave freely as long
// as every rank issues the same sequence of calls.  Allocation layout of each rank's IPC buffer:
// [2][cap] staging | ready[AR_MAX_RANKS][max_blocks] | done[...] | epochs | err (| two-shot region).
#pragma once
#include "common.h"

constexpr int AR_MAX_RANKS = 8;
constexpr int AR_THREADS = 256;
constexpr int AR_ELEMS_PER_BLOCK = AR_THREADS * 8;  // 4 KiB of bf16 per block per call

__host__ __device__ inline size_t ar_flags_off(size_t cap) { return 2 * cap; }

MLS_DEV int* ar_ready(char* base, size_t cap, int max_blocks, int src, int b) {
  return reinterpret_cast<int*>(base + ar_flags_off(cap)) + src * max_blocks + b;
}
MLS_DEV int* ar_done(char* base, size_t cap, int max_blocks, int src, int b) {
  return reinterpret_cast<int*>(base + ar_flags_off(cap)) + (AR_MAX_RANKS + src) * max_blocks + b;
}

MLS_DEV bool ar_wait_ge(int* flag, int want, long long timeout) {
  for (long long i = 0; i < timeout; ++i) {
    if (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) >= want) return true;
    __builtin_amdgcn_s_sleep(2);
  }
  return false;
}

MLS_DEV uint4 load_sys16(const void* p) {  // system-coherent 16-B load (peer memory over xGMI)
  const rsrc_t r = make_rsrc(p, 16);
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, 0, 0, 17));
}

// What a fusing kernel needs of a rank's all-reduce context (filled on the host by
// mls_ar_fuse_desc, passed by value in the kernel arguments; world == 0: no fused all-reduce).
struct ArFuse {
  char* bufs[AR_MAX_RANKS];
  size_t cap;
  int rank, world, max_blocks;
  int* epochs;     // per-chunk epochs (shared with the standalone one-shot kernel)
  int* err;        // timeout word
  int* cnt;        // [max_blocks] per-chunk arrival counters of the fusing GEMM: zero between launches
  long long timeout;
};

// One-shot all-reduce of chunk c of an n-element bf16 message (`in` -> `out`, which may alias),
// run by a whole block of any size (the element loops stride by blockDim.x):
//   wait until every peer finished reading this staging half two epochs ago, stage the chunk,
//   publish ready everywhere, wait for every peer's ready, sum the chunk over all ranks (fp32, the
//   same peer order on every rank -> identical bytes everywhere), publish done.
// `timeout` bounds each peer wait (spin iterations); returns false when one of them ran out (the
// error word is set too), so a caller running several chunks can stop waiting on a lost peer.
MLS_DEV bool ar_oneshot_chunk(const ArFuse& f, const bf16* in, bf16* out, long n, int c, long long timeout) {
  __shared__ int s_epoch, s_ok;
  const int tid = threadIdx.x, nt = blockDim.x;
  if (tid == 0) {
    s_epoch = f.epochs[c] + 1;
    s_ok = 1;
  }
  __syncthreads();
  const int e = s_epoch, parity = e & 1;
  const long lo = (long)c * AR_ELEMS_PER_BLOCK, hi = lo + AR_ELEMS_PER_BLOCK < n ? lo + AR_ELEMS_PER_BLOCK : n;
  if (tid < f.world && e > 2) {
    if (!ar_wait_ge(ar_done(f.bufs[f.rank], f.cap, f.max_blocks, tid, c), e - 2, timeout)) s_ok = 0;
  }
  __syncthreads();
  bf16* stage = reinterpret_cast<bf16*>(f.bufs[f.rank] + parity * f.cap);
  for (long i = lo + tid * 8; i < hi; i += (long)nt * 8) st16(stage + i, ld16(in + i));
  __threadfence_system();
  __syncthreads();
  if (tid < f.world)
    __hip_atomic_store(ar_ready(f.bufs[tid], f.cap, f.max_blocks, f.rank, c), e, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  if (tid < f.world) {
    if (!ar_wait_ge(ar_ready(f.bufs[f.rank], f.cap, f.max_blocks, tid, c), e, timeout)) s_ok = 0;
  }
  __syncthreads();
  for (long i = lo + tid * 8; i < hi; i += (long)nt * 8) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < f.world; ++r) {
      const int src = (f.rank + r) % f.world;  // stagger the peers each rank hits first
      float x[8];
      unpack8(load_sys16(reinterpret_cast<const bf16*>(f.bufs[src] + parity * f.cap) + i), x);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += x[k];
    }
    st16(out + i, pack8(acc));
  }
  __syncthreads();
  if (tid < f.world)
    __hip_atomic_store(ar_done(f.bufs[tid], f.cap, f.max_blocks, f.rank, c), e, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  const bool ok = s_ok != 0;
  if (tid == 0) {
    f.epochs[c] = e;
    if (!ok) atomicOr(f.err, 1);
  }
  __syncthreads();  // s_epoch / s_ok are rewritten by the block's next chunk
  return ok;
}

// The fused all-reduce tail of a GEMM whose output `out` [M][N] (row stride N, bf16) is this rank's
// partial sum.  Every block calls it after its stores, with every thread, covering rows [0, M) x
// columns [c0, c0 + cols).  Each block publishes its stores (agent-scope release), then counts the
// elements it contributed to every chunk its rows touch; the block whose count completes a chunk
// (acquire) runs that chunk's one-shot all-reduce -- chunks reduce as soon as the blocks producing
// them are done, inside this launch.
MLS_DEV void ar_fused_tail(const ArFuse& f, bf16* out, int M, int N, int c0, int cols) {
  constexpr int MAXL = 64;
  __shared__ int s_last[MAXL];
  __shared__ int s_nlast;
  const long n = (long)M * N;
  // publish (MI355X_MICROARCH.md, Valid forms: Producer): every storing wave drains its stores,
  // the block meets, then ONE lane releases at agent scope and waits for the write-back before
  // its counter adds (the asm wait: hipcc may drop the fence's own, Guideline 16 Pitfall 12)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int nl = 0;
    for (int m = 0; m < M; ++m) {
      const long lo = (long)m * N + c0, hi = lo + cols;
      for (long c = lo / AR_ELEMS_PER_BLOCK; c * AR_ELEMS_PER_BLOCK < hi; ++c) {
        const long clo = lo > c * AR_ELEMS_PER_BLOCK ? lo : c * AR_ELEMS_PER_BLOCK;
        const long chi = hi < (c + 1) * AR_ELEMS_PER_BLOCK ? hi : (c + 1) * AR_ELEMS_PER_BLOCK;
        const long total = n - c * AR_ELEMS_PER_BLOCK < AR_ELEMS_PER_BLOCK ? n - c * AR_ELEMS_PER_BLOCK : AR_ELEMS_PER_BLOCK;
        const int add = (int)(chi - clo);
        const int old = __hip_atomic_fetch_add(f.cnt + c, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old + add == total) {
          __hip_atomic_store(f.cnt + c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
          if (nl < MAXL) s_last[nl++] = (int)c;
        }
      }
    }
    if (nl) {  // Consumer: one agent acquire, its invalidate completed before the barrier
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_nlast = nl;
  }
  __syncthreads();
  const int nl = s_nlast;
  // a chunk whose peer wait ran out means a lost peer: the block's later chunks do not spin the
  // full bound again (each would cost ~timeout); they still publish so the epochs stay in step
  bool alive = true;
  for (int i = 0; i < nl; ++i) alive = ar_oneshot_chunk(f, out, out, n, s_last[i], alive ? f.timeout : 1) && alive;
}
