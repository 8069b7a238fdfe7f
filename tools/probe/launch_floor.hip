// Probe: per-dispatch floor on MI355X (empty kernel, tiny grid vs full-chip grid), eager vs graph.
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void empty_k(int* p) { if (p && threadIdx.x == 9999) p[0] = 1; }
__global__ void touch_k(float* p, int n) { int i = blockIdx.x * blockDim.x + threadIdx.x; if (i < n) p[i] += 1.f; }
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
int main() {
  hipStream_t s; CK(hipStreamCreate(&s));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  float* buf; CK(hipMalloc(&buf, 64 << 20));
  const int N = 2000;
  struct Case { const char* name; int grid; int block; int kind; };
  Case cases[] = {{"empty 1x64", 1, 64, 0}, {"empty 2048x256", 2048, 256, 0}, {"empty 8192x256", 8192, 256, 0},
                  {"touch 1M floats", 4096, 256, 1}, {"touch 16M floats", 65536, 256, 1}};
  for (auto& c : cases) {
    for (int graph = 0; graph < 2; ++graph) {
      auto launch = [&]() {
        if (c.kind == 0) hipLaunchKernelGGL(empty_k, dim3(c.grid), dim3(c.block), 0, s, nullptr);
        else hipLaunchKernelGGL(touch_k, dim3(c.grid), dim3(c.block), 0, s, buf, c.grid * c.block);
      };
      hipGraphExec_t ge = nullptr;
      if (graph) {
        hipGraph_t g;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int i = 0; i < N; ++i) launch();
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s));
      } else {
        for (int i = 0; i < 100; ++i) launch();
      }
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(a, s));
      if (graph) CK(hipGraphLaunch(ge, s)); else for (int i = 0; i < N; ++i) launch();
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b));
      printf("%-18s %s: %.2f us/kernel\n", c.name, graph ? "graph" : "eager", ms * 1000.f / N);
    }
  }
  return 0;
}
