// X2: one-shot all-reduce over HIP IPC for the small, latency-bound
// tensor-parallel messages of Llama decode (8 KiB per all-reduce at T = 1, 65 of them per token).
//
// A ring all-reduce over point-to-point xGMI pays 2(N-1) dependent link hops per call; here every
// rank reads every peer's buffer directly -- all 7 links at once, one hop -- and sums locally:
//
//   1. each block b stages its chunk of the local input into this rank's IPC buffer (half
//      `parity` = epoch & 1), then publishes `ready[rank][b] = epoch` in every peer's flag array;
//   2. it waits until every peer has published chunk b of this epoch, reads chunk b from all
//      ranks' buffers over xGMI, sums in fp32 and writes the output;
//   3. it publishes `done[rank][b] = epoch` everywhere; before restaging a buffer half (two
//      epochs later) a block first waits for every peer's `done` of that half's last epoch.
//
// The epoch lives on the device, one counter per block, so a captured hipGraph replays correctly
// (every rank issues the same sequence of calls, hence the same per-block epochs).  Buffers and
// flags are uncached device memory; flags are system-scope atomics, peer data is read with
// system-coherent (sc0 sc1) loads.  Every spin-wait is bounded: on timeout the block records an
// error (read by mls_ar_error) and finishes, so a missing peer can never hang the GPU; the Python
// side self-tests the path at start-up against RCCL and keeps RCCL if anything is off.
#include <cstring>

#include "ar_protocol.h"

namespace {

struct ArCtx {
  int rank, world, max_blocks;
  size_t cap;                    // bytes per buffer half
  char* local;                   // this rank's allocation
  char* peers[AR_MAX_RANKS];     // every rank's allocation mapped here (peers[rank] == local)
  int* epochs;                   // [max_blocks] device-side per-block epoch (local)
  int* err;                      // local error word
  bool opened;
  // two-shot region (its own staging halves, flags and epochs: the protocols never share memory)
  size_t cap2;                   // bytes per two-shot staging half (0 = no two-shot path)
  size_t off2;                   // byte offset of the region in every rank's allocation
  int max_blocks2;
  int* epochs2;
  int* fuse_cnt;                 // [max_blocks] arrival counters of the GEMMs that fuse the one-shot
  long long timeout;             // peer-wait bound (spin iterations) of the GEMM-fused one-shot
};

// allocation layout: [2][cap] staging | ready[AR_MAX_RANKS][max_blocks] | done[...] | epochs | err
// | (4 KiB aligned, off2) [2][cap2] two-shot staging | ready2 / red2 / done2 [AR_MAX_RANKS][max_blocks2] | epochs2

struct ArArgs {
  const bf16* in;
  bf16* out;
  long n;
  int rank, world, max_blocks;
  size_t cap;
  char* bufs[AR_MAX_RANKS];
  int* epochs;
  int* err;
  long long timeout;  // spin iterations
};

MLS_DEV ArFuse ar_view(const ArArgs& a) {
  ArFuse f{};
  for (int r = 0; r < AR_MAX_RANKS; ++r) f.bufs[r] = a.bufs[r];
  f.cap = a.cap;
  f.rank = a.rank;
  f.world = a.world;
  f.max_blocks = a.max_blocks;
  f.epochs = a.epochs;
  f.err = a.err;
  f.cnt = nullptr;
  f.timeout = a.timeout;
  return f;
}

__global__ __launch_bounds__(AR_THREADS) void oneshot_allreduce_kernel(const ArArgs a) {
  ar_oneshot_chunk(ar_view(a), a.in, a.out, a.n, blockIdx.x, a.timeout);
}

// X4: one-shot all-gather of `nbytes` per rank (the decode step's top-k candidates, a few KB):
// the same stage -> publish -> wait -> read protocol and per-block epochs as the all-reduce (every
// rank issues the same sequence of calls, so block b's epoch advances identically everywhere), but
// chunk b of every rank is copied to out[src] instead of summed.
__global__ __launch_bounds__(AR_THREADS) void oneshot_allgather_kernel(const ArArgs a, const char* in, char* out,
                                                                        long nbytes) {
  const int b = blockIdx.x, tid = threadIdx.x;
  __shared__ int s_epoch, s_ok;
  if (tid == 0) {
    s_epoch = a.epochs[b] + 1;
    s_ok = 1;
  }
  __syncthreads();
  const int e = s_epoch;
  const int parity = e & 1;
  const long off = (long)b * AR_THREADS * 16 + tid * 16;
  const bool mine = off < nbytes;  // nbytes % 16 == 0 (host-checked)
  if (tid < a.world && e > 2) {
    if (!ar_wait_ge(ar_done(a.bufs[a.rank], a.cap, a.max_blocks, tid, b), e - 2, a.timeout)) s_ok = 0;
  }
  __syncthreads();
  char* stage = a.bufs[a.rank] + parity * a.cap;
  if (mine) st16(stage + off, ld16(in + off));
  __threadfence_system();
  __syncthreads();
  if (tid < a.world)
    __hip_atomic_store(ar_ready(a.bufs[tid], a.cap, a.max_blocks, a.rank, b), e, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  if (tid < a.world) {
    if (!ar_wait_ge(ar_ready(a.bufs[a.rank], a.cap, a.max_blocks, tid, b), e, a.timeout)) s_ok = 0;
  }
  __syncthreads();
  if (mine) {
    for (int r = 0; r < a.world; ++r) {
      const int src = (a.rank + r) % a.world;
      st16(out + (long)src * nbytes + off, load_sys16(a.bufs[src] + parity * a.cap + off));
    }
  }
  __syncthreads();
  if (tid < a.world)
    __hip_atomic_store(ar_done(a.bufs[tid], a.cap, a.max_blocks, a.rank, b), e, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  if (tid == 0) {
    a.epochs[b] = e;
    if (!s_ok) atomicOr(a.err, 1);
  }
}

// Two-shot all-reduce (reduce-scatter + all-gather in one launch) for the mid-size messages -- TP
// decode at 32-256 rows (0.25-2 MiB per all-reduce) -- where the one-shot's (N - 1) x n bytes of
// peer reads per rank outgrow xGMI: here each rank reads 2 (N - 1) / N x n.  The n elements are
// N segments of n / N; block b owns chunk b of EVERY segment:
//   1. stage chunk b of all N segments into this rank's two-shot buffer (half `parity`), publish
//      ready2[rank][b] everywhere;
//   2. once every peer's ready2 arrived, sum chunk b of segment `rank` over all ranks' buffers
//      (fp32), write the bf16 result to `out` AND back into this rank's own staging copy of that
//      chunk (no peer reads it during step 2: peer p reads segment p), publish red2[rank][b];
//   3. once every peer's red2 arrived, copy chunk b of every other segment s from rank s's buffer
//      (its reduced copy) to `out`; publish done2[rank][b] -- the restage guard two epochs later.
// Every rank writes identical bf16 bytes for every element (one reducer per segment).  Same epoch,
// bounded-spin and error-word rules as the one-shot kernel, in a disjoint region of the allocation.
constexpr int AR2_CH = AR_THREADS * 8;  // elements of each segment per block

struct Ar2Args {
  const bf16* in;
  bf16* out;
  long n, seg;
  int rank, world, max_blocks;
  size_t cap, off;
  char* bufs[AR_MAX_RANKS];
  int* epochs;
  int* err;
  long long timeout;
};

MLS_DEV int* ar2_flag(char* base, const Ar2Args& a, int kind, int src, int b) {
  return reinterpret_cast<int*>(base + a.off + 2 * a.cap) + (kind * AR_MAX_RANKS + src) * a.max_blocks + b;
}

__global__ __launch_bounds__(AR_THREADS) void twoshot_allreduce_kernel(const Ar2Args a) {
  const int b = blockIdx.x, tid = threadIdx.x;
  __shared__ int s_epoch, s_ok;
  if (tid == 0) {
    s_epoch = a.epochs[b] + 1;
    s_ok = 1;
  }
  __syncthreads();
  const int e = s_epoch, parity = e & 1;
  const long c0 = (long)b * AR2_CH + tid * 8;  // this lane's 8 elements within each segment
  const bool mine = c0 < a.seg;                // seg % 8 == 0 (host-checked)
  char* const own = a.bufs[a.rank] + a.off + parity * a.cap;
  if (tid < a.world && e > 2) {
    if (!ar_wait_ge(ar2_flag(a.bufs[a.rank], a, 2, tid, b), e - 2, a.timeout)) s_ok = 0;
  }
  __syncthreads();
  // (1) stage chunk b of every segment
  if (mine)
    for (int s = 0; s < a.world; ++s) {
      const long i = s * a.seg + c0;
      st16(reinterpret_cast<bf16*>(own) + i, ld16(a.in + i));
    }
  __threadfence_system();
  __syncthreads();
  if (tid < a.world)
    __hip_atomic_store(ar2_flag(a.bufs[tid], a, 0, a.rank, b), e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (tid < a.world) {
    if (!ar_wait_ge(ar2_flag(a.bufs[a.rank], a, 0, tid, b), e, a.timeout)) s_ok = 0;
  }
  __syncthreads();
  // (2) reduce this rank's segment
  if (mine) {
    const long i = a.rank * a.seg + c0;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < a.world; ++r) {
      const int src = (a.rank + r) % a.world;
      float x[8];
      unpack8(load_sys16(reinterpret_cast<const bf16*>(a.bufs[src] + a.off + parity * a.cap) + i), x);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += x[k];
    }
    const uint4 v = pack8(acc);
    st16(a.out + i, v);
    st16(reinterpret_cast<bf16*>(own) + i, v);
  }
  __threadfence_system();
  __syncthreads();
  if (tid < a.world)
    __hip_atomic_store(ar2_flag(a.bufs[tid], a, 1, a.rank, b), e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (tid < a.world) {
    if (!ar_wait_ge(ar2_flag(a.bufs[a.rank], a, 1, tid, b), e, a.timeout)) s_ok = 0;
  }
  __syncthreads();
  // (3) gather the other segments' reduced chunks from their owners
  if (mine)
    for (int r = 1; r < a.world; ++r) {
      const int src = (a.rank + r) % a.world;
      const long i = src * a.seg + c0;
      st16(a.out + i, load_sys16(reinterpret_cast<const bf16*>(a.bufs[src] + a.off + parity * a.cap) + i));
    }
  __syncthreads();
  if (tid < a.world)
    __hip_atomic_store(ar2_flag(a.bufs[tid], a, 2, a.rank, b), e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (tid == 0) {
    a.epochs[b] = e;
    if (!s_ok) atomicOr(a.err, 1);
  }
}

// fault injection for tests: hold the stream for `us` microseconds (bounded: <= 10 s)
__global__ void gpu_sleep_kernel(long long ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

// copy the (sticky) error word into a device int32 -- capturable, so a serving decode graph
// reports its collectives' peer timeouts in the iteration's one read-back (models/llama_serving.py)
__global__ void ar_error_peek_kernel(const int* err, int* dst) {
  if (threadIdx.x == 0) dst[0] = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

extern "C" {

// cap: bytes per message (messages above it use RCCL); returns an opaque context
static size_t ar_region1_bytes(const ArCtx* c) {
  const size_t flags = (size_t)2 * AR_MAX_RANKS * c->max_blocks * sizeof(int);
  return 2 * c->cap + flags + (size_t)c->max_blocks * sizeof(int) + 64;
}
static size_t ar_region2_bytes(const ArCtx* c) {
  const size_t flags = (size_t)3 * AR_MAX_RANKS * c->max_blocks2 * sizeof(int);
  return 2 * c->cap2 + flags + (size_t)c->max_blocks2 * sizeof(int);
}

// cap: bytes per one-shot message; cap2: bytes per two-shot message (0 = none; messages above the
// caps use RCCL); returns an opaque context
int mls_ar_create2(int rank, int world, long cap, long cap2, void** ctx_out) {
  if (world < 1 || world > AR_MAX_RANKS || rank < 0 || rank >= world || cap <= 0 || cap % 4096 || cap2 < 0 ||
      cap2 % 4096)
    return MLS_BAD_ARG;
  ArCtx* c = new ArCtx{};
  c->timeout = 1LL << 24;
  c->rank = rank;
  c->world = world;
  c->cap = (size_t)cap;
  c->max_blocks = (int)((cap / 2 + AR_ELEMS_PER_BLOCK - 1) / AR_ELEMS_PER_BLOCK);
  c->cap2 = (size_t)cap2;
  // a segment is <= cap2 / 2 / world elements; one block per AR2_CH of it
  c->max_blocks2 = cap2 ? (int)((cap2 / 2 / world + AR2_CH - 1) / AR2_CH) : 0;
  c->off2 = (ar_region1_bytes(c) + 4095) / 4096 * 4096;
  const size_t bytes = c->off2 + (cap2 ? ar_region2_bytes(c) : 0);
  if (hipExtMallocWithFlags((void**)&c->local, bytes, hipDeviceMallocUncached) != hipSuccess) {
    delete c;
    return MLS_UNSUPPORTED;
  }
  if (hipMemset(c->local, 0, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    hipFree(c->local);
    delete c;
    return MLS_UNSUPPORTED;
  }
  const size_t flags = (size_t)2 * AR_MAX_RANKS * c->max_blocks * sizeof(int);
  c->epochs = reinterpret_cast<int*>(c->local + 2 * c->cap + flags);
  c->err = c->epochs + c->max_blocks;
  c->epochs2 = cap2 ? reinterpret_cast<int*>(c->local + c->off2 + 2 * c->cap2 +
                                             (size_t)3 * AR_MAX_RANKS * c->max_blocks2 * sizeof(int))
                    : nullptr;
  if (hipMalloc((void**)&c->fuse_cnt, (size_t)c->max_blocks * sizeof(int)) != hipSuccess ||
      hipMemset(c->fuse_cnt, 0, (size_t)c->max_blocks * sizeof(int)) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    hipFree(c->local);
    delete c;
    return MLS_UNSUPPORTED;
  }
  for (int i = 0; i < AR_MAX_RANKS; ++i) c->peers[i] = nullptr;
  c->peers[rank] = c->local;
  *ctx_out = c;
  return 0;
}

// The descriptor a GEMM needs to run the one-shot all-reduce of its own n-element output in its
// epilogue (ar_protocol.h ar_fused_tail); MLS_BAD_ARG when n does not fit the one-shot buffer.
int mls_ar_fuse_desc(void* ctx, long n, ArFuse* f) {
  ArCtx* c = (ArCtx*)ctx;
  if (!c || (!c->opened && c->world > 1) || n <= 0 || n % 8 || (size_t)n * 2 > c->cap) return MLS_BAD_ARG;
  *f = ArFuse{};
  for (int r = 0; r < AR_MAX_RANKS; ++r) f->bufs[r] = c->peers[r];
  f->cap = c->cap;
  f->rank = c->rank;
  f->world = c->world;
  f->max_blocks = c->max_blocks;
  f->epochs = c->epochs;
  f->err = c->err;
  f->cnt = c->fuse_cnt;
  f->timeout = c->timeout;
  return 0;
}

// The peer-wait bound the GEMM-fused all-reduce uses (CustomAllReduce.timeout, MLS_AR_TIMEOUT_ITERS):
// the standalone kernels take theirs per call.
int mls_ar_set_timeout(void* ctx, long long iters) {
  ArCtx* c = (ArCtx*)ctx;
  if (!c || iters <= 0) return MLS_BAD_ARG;
  c->timeout = iters;
  return 0;
}

int mls_ar_create(int rank, int world, long cap, void** ctx_out) { return mls_ar_create2(rank, world, cap, 0, ctx_out); }

int mls_ar_handle(void* ctx, void* handle_out /* HIP_IPC_HANDLE_SIZE bytes */) {
  ArCtx* c = (ArCtx*)ctx;
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, c->local) != hipSuccess) return MLS_UNSUPPORTED;
  memcpy(handle_out, &h, sizeof(h));
  return 0;
}

int mls_ar_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

// handles: world * handle_size bytes (this rank's entry is ignored)
int mls_ar_open(void* ctx, const void* handles) {
  ArCtx* c = (ArCtx*)ctx;
  for (int r = 0; r < c->world; ++r) {
    if (r == c->rank) continue;
    hipIpcMemHandle_t h;
    memcpy(&h, (const char*)handles + (size_t)r * sizeof(h), sizeof(h));
    void* p = nullptr;
    if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) return MLS_UNSUPPORTED;
    c->peers[r] = (char*)p;
  }
  c->opened = true;
  return 0;
}

// in/out: n bf16 elements (n % 8 == 0, n * 2 <= cap); in may alias out
int mls_ar_allreduce(void* ctx, const void* in, void* out, long n, long long timeout, void* stream) {
  ArCtx* c = (ArCtx*)ctx;
  if (!c->opened && c->world > 1) return MLS_BAD_ARG;
  if (n <= 0 || n % 8 || (size_t)n * 2 > c->cap) return MLS_BAD_ARG;
  ArArgs a{};
  a.in = (const bf16*)in;
  a.out = (bf16*)out;
  a.n = n;
  a.rank = c->rank;
  a.world = c->world;
  a.max_blocks = c->max_blocks;
  a.cap = c->cap;
  for (int r = 0; r < AR_MAX_RANKS; ++r) a.bufs[r] = c->peers[r];
  a.epochs = c->epochs;
  a.err = c->err;
  a.timeout = timeout > 0 ? timeout : (1LL << 24);
  const int blocks = (int)((n + AR_ELEMS_PER_BLOCK - 1) / AR_ELEMS_PER_BLOCK);
  hipLaunchKernelGGL(oneshot_allreduce_kernel, dim3(blocks), dim3(AR_THREADS), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

// two-shot: in/out n bf16 elements, n % (8 * world) == 0, n * 2 <= cap2; in may alias out
int mls_ar_allreduce2(void* ctx, const void* in, void* out, long n, long long timeout, void* stream) {
  ArCtx* c = (ArCtx*)ctx;
  if (!c->opened && c->world > 1) return MLS_BAD_ARG;
  if (!c->cap2 || n <= 0 || n % (8L * c->world) || (size_t)n * 2 > c->cap2) return MLS_BAD_ARG;
  Ar2Args a{};
  a.in = (const bf16*)in;
  a.out = (bf16*)out;
  a.n = n;
  a.seg = n / c->world;
  a.rank = c->rank;
  a.world = c->world;
  a.max_blocks = c->max_blocks2;
  a.cap = c->cap2;
  a.off = c->off2;
  for (int r = 0; r < AR_MAX_RANKS; ++r) a.bufs[r] = c->peers[r];
  a.epochs = c->epochs2;
  a.err = c->err;
  a.timeout = timeout > 0 ? timeout : (1LL << 24);
  const int blocks = (int)((a.seg + AR2_CH - 1) / AR2_CH);
  if (blocks > c->max_blocks2) return MLS_BAD_ARG;
  hipLaunchKernelGGL(twoshot_allreduce_kernel, dim3(blocks), dim3(AR_THREADS), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

// X4: out[world][nbytes] = every rank's `in` (nbytes % 16 == 0, nbytes <= cap, out != in)
int mls_ar_allgather(void* ctx, const void* in, void* out, long nbytes, long long timeout, void* stream) {
  ArCtx* c = (ArCtx*)ctx;
  if (!c->opened && c->world > 1) return MLS_BAD_ARG;
  if (nbytes <= 0 || nbytes % 16 || (size_t)nbytes > c->cap) return MLS_BAD_ARG;
  ArArgs a{};
  a.rank = c->rank;
  a.world = c->world;
  a.max_blocks = c->max_blocks;
  a.cap = c->cap;
  for (int r = 0; r < AR_MAX_RANKS; ++r) a.bufs[r] = c->peers[r];
  a.epochs = c->epochs;
  a.err = c->err;
  a.timeout = timeout > 0 ? timeout : (1LL << 24);
  const int blocks = (int)((nbytes + AR_THREADS * 16 - 1) / (AR_THREADS * 16));
  if (blocks > c->max_blocks) return MLS_BAD_ARG;
  hipLaunchKernelGGL(oneshot_allgather_kernel, dim3(blocks), dim3(AR_THREADS), 0, (hipStream_t)stream, a,
                     (const char*)in, (char*)out, nbytes);
  return (int)hipGetLastError();
}

// After a peer-wait timeout the per-block epochs of the ranks may disagree: every rank calls this
// between two process-group barriers (no kernel of the group in flight) to restart the protocol.
int mls_ar_reset(void* ctx) {
  ArCtx* c = (ArCtx*)ctx;
  if (hipDeviceSynchronize() != hipSuccess) return MLS_UNSUPPORTED;
  const size_t flags = (size_t)2 * AR_MAX_RANKS * c->max_blocks * sizeof(int);
  const size_t bytes = flags + (size_t)c->max_blocks * sizeof(int) + 64;
  if (hipMemset(c->local + 2 * c->cap, 0, bytes) != hipSuccess) return MLS_UNSUPPORTED;
  if (c->fuse_cnt && hipMemset(c->fuse_cnt, 0, (size_t)c->max_blocks * sizeof(int)) != hipSuccess) return MLS_UNSUPPORTED;
  if (c->cap2) {
    const size_t f2 = (size_t)3 * AR_MAX_RANKS * c->max_blocks2 * sizeof(int) + (size_t)c->max_blocks2 * sizeof(int);
    if (hipMemset(c->local + c->off2 + 2 * c->cap2, 0, f2) != hipSuccess) return MLS_UNSUPPORTED;
  }
  return (int)hipDeviceSynchronize();
}

int mls_gpu_sleep(long us, void* stream) {
  if (us < 0 || us > 10000000) return MLS_BAD_ARG;
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) !=
      hipSuccess || khz <= 0)
    khz = 100000;  // the gfx9 constant clock: 100 MHz
  hipLaunchKernelGGL(gpu_sleep_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (long long)us * khz / 1000);
  return (int)hipGetLastError();
}

// error word (1 = a wait timed out since the last reset); resets it
int mls_ar_error(void* ctx, int* out) {
  ArCtx* c = (ArCtx*)ctx;
  if (hipMemcpy(out, c->err, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return MLS_UNSUPPORTED;
  const int zero = 0;
  return (int)hipMemcpy(c->err, &zero, sizeof(int), hipMemcpyHostToDevice);
}

// dst (device int32) <- the error word, on `stream`, without resetting it (mls_ar_error resets)
int mls_ar_error_peek(void* ctx, int* dst, void* stream) {
  ArCtx* c = (ArCtx*)ctx;
  if (!c || !dst) return MLS_BAD_ARG;
  hipLaunchKernelGGL(ar_error_peek_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (const int*)c->err, dst);
  return (int)hipGetLastError();
}

int mls_ar_destroy(void* ctx) {
  ArCtx* c = (ArCtx*)ctx;
  if (!c) return 0;
  hipDeviceSynchronize();
  for (int r = 0; r < c->world; ++r)
    if (r != c->rank && c->peers[r]) hipIpcCloseMemHandle(c->peers[r]);
  hipFree(c->local);
  if (c->fuse_cnt) hipFree(c->fuse_cnt);
  delete c;
  return 0;
}

}  // extern "C"
