// The serving engine's per-batch enqueue in one native call (engine/worker.py GpuEngine.launch):
// pinned host rows -> device input (hipMemcpyAsync), the captured forward (hipGraphLaunch of the
// slot's graph exec), device outputs -> pinned host buffers, the slot's done event -- all on the
// slot's stream, in that order.  The Python sequence of the same calls (torch copy_, replay, event
// record / wait, stream contexts) costs 85-100 us of host time per batch and 250-290 us for the
// first batch after the pipeline drained (profiles/r4_engine_first_submit_timeline.jsonl): host
// time that delays every refill of a freed slot and the whole first wave of the bench's window.
#include "common.h"

#include <time.h>

namespace {
inline long long now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (long long)ts.tv_sec * 1000000000LL + ts.tv_nsec;
}
}  // namespace

extern "C" {

// d2h_*: n_d2h (<= 8) destination / source / byte-count triples.  t_ns (optional, 5 entries):
// CLOCK_MONOTONIC before the H2D, after it, after the graph launch, after the D2H copies and after
// the event record -- which HIP call a host stall sits in (engine/worker.py Ticket.launch_ns).
// Returns 0 or the HIP error.
int mls_engine_launch(void* stream, void* h2d_dst, const void* h2d_src, long long h2d_bytes, void* graph_exec,
                      int n_d2h, void* const* d2h_dst, void* const* d2h_src, const long long* d2h_bytes,
                      void* event, long long* t_ns) {
  if (!graph_exec || n_d2h < 0 || n_d2h > 8) return MLS_BAD_ARG;
  hipStream_t st = (hipStream_t)stream;
  hipError_t e = hipSuccess;
  if (t_ns) t_ns[0] = now_ns();
  if (h2d_bytes > 0) e = hipMemcpyAsync(h2d_dst, h2d_src, (size_t)h2d_bytes, hipMemcpyHostToDevice, st);
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
