// Spatial partitioning of the GPU between the engine's in-flight batches.
//
// The serving engine runs several batches at once, one per slot stream.  By default every slot's
// kernels may run on all 256 CUs, so the co-running batches interleave over every XCD: each
// kernel's output leaves its producer XCD's L2 and the next kernel reads it back from the
// Infinity Cache / HBM, and the small late-layer kernels (ResNet layer3 / 4: 64-200 tiles) share
// the chip in time with tails and ramps of their own.  A CU-masked slot stream
// (hipExtStreamCreateWithCUMask) pins one batch to a subset of the XCDs instead: its kernels fill
// their partition (4x the tiles per CU of the whole chip), and activations produced and consumed
// inside one partition stay in that partition's L2s.
//
// mls_cu_census records, per block, the XCC id (HW_REG_XCC_ID) and HW_ID register of the CU it ran
// on, so the host can learn how the logical CU-mask bits map to XCDs on this part (the mask
// layout is not documented per XCC) and verify a mask.
#include "common.h"

namespace {

__global__ __launch_bounds__(64) void cu_census_kernel(int* out, int spin) {
  if (threadIdx.x == 0) {
    // s_getreg_b32 simm16 = (size - 1) << 11 | offset << 6 | id: whole 32-bit HW_ID (id 4) and
    // XCC_ID (id 20).  Scalar register reads only; the results leave through a vector store.
    const int hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    const int xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    for (int i = 0; i < spin; ++i) __builtin_amdgcn_s_sleep(8);  // keep blocks resident so the grid spreads
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = hw;
  }
}

}  // namespace

extern "C" {

// A new stream whose kernels run only on the CUs whose bits are set in mask[0..words).
int mls_stream_create_cumask(const uint32_t* mask, int words, void** stream) {
  if (!mask || words <= 0 || !stream) return MLS_BAD_ARG;
  hipStream_t s = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask);
  if (e != hipSuccess) return (int)e;
  *stream = (void*)s;
  return 0;
}

int mls_stream_get_cumask(void* stream, uint32_t* mask, int words) {
  if (!mask || words <= 0) return MLS_BAD_ARG;
  return (int)hipExtStreamGetCUMask((hipStream_t)stream, (uint32_t)words, mask);
}

int mls_stream_destroy(void* stream) { return (int)hipStreamDestroy((hipStream_t)stream); }

// out: int32 [blocks][2] = (XCC_ID, HW_ID) per block
int mls_cu_census(int* out, int blocks, int spin, void* stream) {
  if (!out || blocks <= 0) return MLS_BAD_ARG;
  hipLaunchKernelGGL(cu_census_kernel, dim3(blocks), dim3(64), 0, (hipStream_t)stream, out, spin);
  return (int)hipGetLastError();
}

}  // extern "C"
