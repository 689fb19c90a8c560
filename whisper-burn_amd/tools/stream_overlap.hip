// stream_overlap.hip -- do hipGraph replays on different streams overlap?
//   hipcc --offload-arch=gfx950 -O3 tools/stream_overlap.hip -o build/stream_overlap
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void tiny(int* p) {
  if (threadIdx.x == 0) atomicAdd(p + blockIdx.x % 64, 1);
}
__global__ void spin(int* p, long long cycles) {  // occupies one CU per block for `cycles`
  const long long t0 = clock64();
  while (clock64() - t0 < cycles) {
  }
  if (threadIdx.x == 0) atomicAdd(p, 1);
}

#define CK(x)                                                  \
  do {                                                         \
    hipError_t e = (x);                                        \
    if (e != hipSuccess) {                                     \
      printf("%s failed: %s\n", #x, hipGetErrorString(e));     \
      return 1;                                                \
    }                                                          \
  } while (0)

int main() {
  const int S = 4, N = 100;
  hipStream_t st[S];
  hipGraphExec_t ge[2][S];
  int* c;
  CK(hipMalloc(&c, 4096));
  for (int i = 0; i < S; ++i) CK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
  for (int kind = 0; kind < 2; ++kind)
    for (int i = 0; i < S; ++i) {
      hipGraph_t g;
      CK(hipStreamBeginCapture(st[i], hipStreamCaptureModeThreadLocal));
      for (int k = 0; k < N; ++k) {
        if (kind == 0) hipLaunchKernelGGL(tiny, dim3(64), dim3(64), 0, st[i], c + 64 * i);
        else hipLaunchKernelGGL(spin, dim3(32), dim3(64), 0, st[i], c + 64 * i, 10000LL);  // ~4 us, 32 CUs
      }
      CK(hipStreamEndCapture(st[i], &g));
      CK(hipGraphInstantiate(&ge[kind][i], g, nullptr, nullptr, 0));
    }
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int kind = 0; kind < 2; ++kind)
    for (int ns = 1; ns <= S; ns *= 2) {
      for (int i = 0; i < ns; ++i) CK(hipGraphLaunch(ge[kind][i], st[i]));
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(a, 0));
      for (int i = 0; i < ns; ++i) CK(hipStreamWaitEvent(st[i], a, 0));
      for (int r = 0; r < 5; ++r)
        for (int i = 0; i < ns; ++i) CK(hipGraphLaunch(ge[kind][i], st[i]));
      for (int i = 0; i < ns; ++i) {
        hipEvent_t ev;
        CK(hipEventCreate(&ev));
        CK(hipEventRecord(ev, st[i]));
        CK(hipStreamWaitEvent(0, ev, 0));
      }
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      printf("%s graphs on %d streams: %.1f us per replay round (%.2f us per kernel per stream)\n",
             kind == 0 ? "tiny" : "spin4us", ns, ms * 1e3 / 5, ms * 1e3 / 5 / N);
    }
  return 0;
}
