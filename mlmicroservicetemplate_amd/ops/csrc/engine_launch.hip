// The serving engine's per-batch enqueue in one native call (engine/worker.py GpuEngine.launch):
// pinned host rows -> device input (hipMemcpyAsync), the captured forward (hipGraphLaunch of the
// slot's graph exec), device outputs -> pinned host buffers, the slot's done event -- all on the
// slot's stream, in that order.  The Python sequence of the same calls (torch copy_, replay, event
// record / wait, stream contexts) costs 85-100 us of host time per batch and 250-290 us for the
// first batch after the pipeline drained (profiles/r4_engine_first_submit_timeline.jsonl): host
// time that delays every refill of a freed slot and the whole first wave of the bench's window.
#include "common.h"

#include <cstdlib>
#include <time.h>

typedef unsigned int u32x4v_e __attribute__((__vector_size__(16)));

namespace {
inline long long now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (long long)ts.tv_sec * 1000000000LL + ts.tv_nsec;
}
}  // namespace

// Zero-copy H2D: a few workgroups pull a pinned host buffer (mapped in the GPU's address space)
// over PCIe into device memory -- a kernel in the slot's own stream (and captured into its graph),
// so no SDMA copy-engine queue takes part: the SDMA H2D of a 4.8 MB batch occasionally blocked the
// enqueue ~6 ms with every queue of the process stalled (tools/probe/r5_stall.sh: 4 of ~60 20-step
// runs; none with HSA_ENABLE_SDMA=0, whose blit kernels cost 7 %).  U 16-B loads in flight per
// lane; offsets past `bytes` read zero / store nothing (buffer range check), so no tail branch.
template <int U>
__global__ __launch_bounds__(256) void h2d_pull_kernel(const void* src, void* dst, uint32_t bytes, int iters) {
  const rsrc_t s = make_rsrc(src, bytes), d = make_rsrc(dst, bytes);
  const int stride = (int)gridDim.x * 256 * 16;
  int off = ((int)blockIdx.x * 256 + (int)threadIdx.x) * 16;
  for (int it = 0; it < iters; ++it) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(s, off + u * stride, 0, 2));  // nt
#pragma unroll
    for (int u = 0; u < U; ++u)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v_e, v[u]), d, off + u * stride, 0, 0);
    off += U * stride;
  }
}

// The same pull with the source read at run time from a pinned host cell the host writes before
// the graph launch: cell[0] = source address (pinned host memory, or device memory), cell[1] = how
// many of the launch's workgroups copy (0 = all).  A captured graph thus pulls whichever buffer a
// batch was staged in (GpuEngine.prepare): a pre-staged batch needs no host memcpy into the slot's
// own buffer, and a batch already pulled to the device ahead of its launch (GpuEngine prepull) is
// a device-to-device copy by all of the workgroups -- PCIe sets the host pull's ~90 us with 8 of
// them, HBM wants more.  The cell is read with system-scope loads (no cache may hold the previous
// launch's words) and made wave-uniform for the buffer descriptor.
// SA: cache-policy bits of the device-side stores (0 = default; 2 = nt: stream past the L2 the
// co-running batches' convolutions work out of -- MLS_PULL_STORE_AUX, an A/B knob)
template <int U, int SA = 0>
__global__ __launch_bounds__(256) void h2d_pull_cell_kernel(const unsigned long long* src_cell, void* dst,
                                                            uint32_t bytes) {
  const unsigned long long a = __hip_atomic_load(src_cell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const unsigned long long nb = __hip_atomic_load(src_cell + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  const int nblk_req = (int)__builtin_amdgcn_readfirstlane((unsigned)nb);
  const int nblk = nblk_req > 0 && nblk_req < (int)gridDim.x ? nblk_req : (int)gridDim.x;
  if ((int)blockIdx.x >= nblk) return;
  const void* src = (const void*)(((unsigned long long)hi << 32) | lo);
  const rsrc_t s = make_rsrc(src, bytes), d = make_rsrc(dst, bytes);
  const int stride = nblk * 256 * 16;
  const int iters = (int)((bytes + (uint32_t)(stride * U) - 1) / (uint32_t)(stride * U));
  int off = ((int)blockIdx.x * 256 + (int)threadIdx.x) * 16;
  for (int it = 0; it < iters; ++it) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(s, off + u * stride, 0, 2));  // nt
#pragma unroll
    for (int u = 0; u < U; ++u)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v_e, v[u]), d, off + u * stride, 0, SA);
    off += U * stride;
  }
}

static int pull_store_aux() {
  static const int v = [] {
    const char* e = getenv("MLS_PULL_STORE_AUX");
    return e ? atoi(e) : 0;
  }();
  return v;
}

extern "C" {
int mls_engine_launch_after(void* wait_event, void* stream, void* h2d_dst, const void* h2d_src, long long h2d_bytes,
                            void* graph_exec, int n_d2h, void* const* d2h_dst, void* const* d2h_src,
                            const long long* d2h_bytes, void* event, long long* t_ns);

// src_cell: pinned host words {source address (`bytes` readable), workgroups to copy with (0 = all
// `blocks`)}.
int mls_h2d_pull_cell(const void* src_cell, void* dst, long long bytes, int blocks, void* stream) {
  if (!src_cell || !dst || bytes <= 0 || bytes % 16 || bytes >= (1LL << 30) || blocks <= 0 || blocks > 1024)
    return MLS_BAD_ARG;
  constexpr int U = 8;
  const int sa = pull_store_aux();
  if (sa == 2)
    hipLaunchKernelGGL((h2d_pull_cell_kernel<U, 2>), dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       (const unsigned long long*)src_cell, dst, (uint32_t)bytes);
  else if (sa == 3)
    hipLaunchKernelGGL((h2d_pull_cell_kernel<U, 3>), dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       (const unsigned long long*)src_cell, dst, (uint32_t)bytes);
  else
    hipLaunchKernelGGL(h2d_pull_cell_kernel<U>, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       (const unsigned long long*)src_cell, dst, (uint32_t)bytes);
  return (int)hipGetLastError();
}

// src: pinned host memory (hipHostMalloc / torch pin_memory), dst: device memory (or the other way
// round: any two GPU-addressable buffers), bytes % 16 == 0, < 1 GiB.  blocks: workgroups copying
// (each lane keeps 8 x 16 B in flight).
int mls_h2d_pull(const void* src, void* dst, long long bytes, int blocks, void* stream) {
  if (!src || !dst || bytes <= 0 || bytes % 16 || bytes >= (1LL << 30) || blocks <= 0 || blocks > 1024)
    return MLS_BAD_ARG;
  constexpr int U = 8;
  const long long step = (long long)blocks * 256 * 16 * U;
  const int iters = (int)((bytes + step - 1) / step);
  hipLaunchKernelGGL(h2d_pull_kernel<U>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, src, dst,
                     (uint32_t)bytes, iters);
  return (int)hipGetLastError();
}

// The same copy kernel the other way: device memory -> pinned host memory (the engine's per-batch
// results, pushed at the end of the slot's graph instead of D2H hipMemcpyAsync on an SDMA queue).
int mls_d2h_push(const void* src, void* dst, long long bytes, int blocks, void* stream) {
  return mls_h2d_pull(src, dst, bytes, blocks, stream);
}

// d2h_*: n_d2h (<= 8) destination / source / byte-count triples.  t_ns (optional, 5 entries):
// CLOCK_MONOTONIC before the H2D, after it, after the graph launch, after the D2H copies and after
// the event record -- which HIP call a host stall sits in (engine/worker.py Ticket.launch_ns).
// Returns 0 or the HIP error.
int mls_engine_launch(void* stream, void* h2d_dst, const void* h2d_src, long long h2d_bytes, void* graph_exec,
                      int n_d2h, void* const* d2h_dst, void* const* d2h_src, const long long* d2h_bytes,
                      void* event, long long* t_ns) {
  return mls_engine_launch_after(nullptr, stream, h2d_dst, h2d_src, h2d_bytes, graph_exec, n_d2h, d2h_dst, d2h_src,
                                 d2h_bytes, event, t_ns);
}

// the same, the slot's stream first waiting for `wait_event` (recorded on another stream: the
// early pull of a pre-staged batch, GpuEngine prepull), or no wait when it is null
int mls_engine_launch_after(void* wait_event, void* stream, void* h2d_dst, const void* h2d_src, long long h2d_bytes,
                            void* graph_exec, int n_d2h, void* const* d2h_dst, void* const* d2h_src,
                            const long long* d2h_bytes, void* event, long long* t_ns) {
  if (!graph_exec || n_d2h < 0 || n_d2h > 8) return MLS_BAD_ARG;
  hipStream_t st = (hipStream_t)stream;
  hipError_t e = hipSuccess;
  if (wait_event) e = hipStreamWaitEvent(st, (hipEvent_t)wait_event, 0);
  if (t_ns) t_ns[0] = now_ns();
  if (h2d_bytes > 0 && e == hipSuccess) e = hipMemcpyAsync(h2d_dst, h2d_src, (size_t)h2d_bytes, hipMemcpyHostToDevice, st);
  if (t_ns) t_ns[1] = now_ns();
  if (e == hipSuccess) e = hipGraphLaunch((hipGraphExec_t)graph_exec, st);
  if (t_ns) t_ns[2] = now_ns();
  for (int i = 0; i < n_d2h && e == hipSuccess; ++i)
    e = hipMemcpyAsync(d2h_dst[i], d2h_src[i], (size_t)d2h_bytes[i], hipMemcpyDeviceToHost, st);
  if (t_ns) t_ns[3] = now_ns();
  if (e == hipSuccess && event) e = hipEventRecord((hipEvent_t)event, st);
  if (t_ns) t_ns[4] = now_ns();
  return (int)e;
}

}  // extern "C"
