// launch_floor.hip -- per-kernel cost of dependent launches on one stream:
// hipGraph replay vs eager launches, tiny kernels vs kernels that dirty L2.
//   hipcc --offload-arch=gfx950 -O3 tools/launch_floor.hip -o build/launch_floor
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ void tiny(int* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1;
}
__global__ void dirty(float* p, int n) {  // writes n floats (dirties L2)
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = (float)i;
}

// ~4 KB of straight-line code per instance (I-cache experiment)
template <int ID>
__global__ void bigcode(float* p) {
  float v0 = threadIdx.x, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3;
#pragma unroll
  for (int i = 0; i < 128; ++i) {
    v0 = v0 * 1.0001f + (float)(ID + i);
    v1 = v1 * 0.9999f + (float)(ID - i);
    v2 = v2 * 1.0002f + (float)(ID * i);
    v3 = v3 * 0.9998f + (float)(ID ^ i);
  }
  if (v0 + v1 + v2 + v3 == 12345.0f) p[threadIdx.x] = v0;
}

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e = (x);                                                   \
    if (e != hipSuccess) {                                                \
      printf("%s failed: %s\n", #x, hipGetErrorString(e));                \
      return 1;                                                           \
    }                                                                     \
  } while (0)

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int* c;
  float* buf;
  CK(hipMalloc(&c, 4));
  CK(hipMalloc(&buf, 64 << 20));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int N = 200;
  for (int mode = 0; mode < 8; ++mode) {
    // 0: tiny 1 WG, 1: tiny 256 WG, 2: dirty 128 KB, 3: dirty 4 MB; 4,5: tiny 1 WG / dirty 128KB eager
    const bool graph = mode < 4 || mode >= 6;
    auto launch = [&](int i) {
      switch (mode) {
        case 0: case 4: hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, c); break;
        case 1: hipLaunchKernelGGL(tiny, dim3(256), dim3(256), 0, s, c); break;
        case 2: case 5: hipLaunchKernelGGL(dirty, dim3(128), dim3(256), 0, s, buf + (i % 64) * 32768, 32768); break;
        case 3: hipLaunchKernelGGL(dirty, dim3(512), dim3(256), 0, s, buf + (i % 4) * (1 << 20), 1 << 20); break;
        case 6: hipLaunchKernelGGL(bigcode<0>, dim3(256), dim3(256), 0, s, buf); break;
        case 7:
          switch (i % 8) {
            case 0: hipLaunchKernelGGL(bigcode<0>, dim3(256), dim3(256), 0, s, buf); break;
            case 1: hipLaunchKernelGGL(bigcode<1>, dim3(256), dim3(256), 0, s, buf); break;
            case 2: hipLaunchKernelGGL(bigcode<2>, dim3(256), dim3(256), 0, s, buf); break;
            case 3: hipLaunchKernelGGL(bigcode<3>, dim3(256), dim3(256), 0, s, buf); break;
            case 4: hipLaunchKernelGGL(bigcode<4>, dim3(256), dim3(256), 0, s, buf); break;
            case 5: hipLaunchKernelGGL(bigcode<5>, dim3(256), dim3(256), 0, s, buf); break;
            case 6: hipLaunchKernelGGL(bigcode<6>, dim3(256), dim3(256), 0, s, buf); break;
            default: hipLaunchKernelGGL(bigcode<7>, dim3(256), dim3(256), 0, s, buf); break;
          }
          break;
      }
    };
    float ms = 0;
    if (graph) {
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      for (int i = 0; i < N; ++i) launch(i);
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(a, s));
      for (int r = 0; r < 5; ++r) CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      ms /= 5;
    } else {
      for (int i = 0; i < N; ++i) launch(i);
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(a, s));
      for (int i = 0; i < N; ++i) launch(i);
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
    }
    static const char* names[] = {"graph tiny 1WG", "graph tiny 256WG", "graph dirty 128KB", "graph dirty 4MB",
                                  "eager tiny 1WG", "eager dirty 128KB", "graph bigcode same", "graph bigcode x8"};
    printf("%-20s %7.2f us per kernel\n", names[mode], ms * 1e3 / N);
  }
  return 0;
}
