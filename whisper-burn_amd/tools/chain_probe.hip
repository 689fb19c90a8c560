// chain_probe.hip -- what a dependent kernel costs in a graph, and whether
// graphs on several streams overlap (decode-step design evidence).
//   hipcc --offload-arch=gfx950 -O3 tools/chain_probe.hip -o build/chain_probe
// Modes (all hipGraph-replayed, N kernels per chain):
//   tiny      1 WG x 64 threads, no memory
//   gemv40    40 WGs x 512 threads, 64 KiB LDS, each WG reads 24 KiB of a
//             1 GiB pool (cold, 16-B loads, all in flight), reduces, writes
//             32 floats -- the shape of a K = 1280 decode GEMM
//   gemv160   the same at 160 WGs
// each run with 1, 2 and 4 streams replaying their own graph concurrently.
// Prints wall microseconds per kernel (total wall / kernels of all streams).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ void tiny(int* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1;
}

__global__ __launch_bounds__(512) void gemv(const uint4* __restrict__ w, size_t pool_u4, size_t off_u4,
                                            float* __restrict__ out) {
  __shared__ float red[16384];  // 64 KiB
  const int tid = threadIdx.x;
  // 24 KiB per WG = 1536 uint4 = 3 per thread
  const size_t base = (off_u4 + (size_t)blockIdx.x * 1536) % pool_u4;
  uint4 v[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) v[i] = w[(base + i * 512 + tid) % pool_u4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 3; ++i) s += (float)(v[i].x ^ v[i].y) * 1e-9f + (float)(v[i].z ^ v[i].w) * 1e-9f;
  red[tid] = s;
  __syncthreads();
  if (tid < 32) {
    float t = 0.f;
    for (int j = tid; j < 512; j += 32) t += red[j];
    out[blockIdx.x * 32 + tid] = t;
  }
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
  const int N = 200;
  const size_t pool_bytes = (size_t)1 << 30;
  const size_t pool_u4 = pool_bytes / 16;
  uint4* pool;
  float* out;
  int* c;
  CK(hipMalloc(&pool, pool_bytes));
  CK(hipMemset(pool, 1, pool_bytes));
  CK(hipMalloc(&out, 4 * 160 * 32 * 4 * 8));
  CK(hipMalloc(&c, 64));
  const char* names[] = {"tiny", "gemv40", "gemv160"};
  for (int mode = 0; mode < 3; ++mode) {
    for (int ns : {1, 2, 4}) {
      std::vector<hipStream_t> st(ns);
      std::vector<hipGraphExec_t> ge(ns);
      for (int s = 0; s < ns; ++s) {
        CK(hipStreamCreateWithFlags(&st[s], hipStreamNonBlocking));
        hipGraph_t g;
        CK(hipStreamBeginCapture(st[s], hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < N; ++i) {
          if (mode == 0) {
            hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, st[s], c + s);
          } else {
            const int wgs = mode == 1 ? 40 : 160;
            // walk the pool so every kernel reads cold lines
            const size_t off = ((size_t)(s * N + i) * 160 * 1536 * 7) % pool_u4;
            hipLaunchKernelGGL(gemv, dim3(wgs), dim3(512), 0, st[s], pool, pool_u4, off, out + s * 160 * 32);
          }
        }
        CK(hipStreamEndCapture(st[s], &g));
        CK(hipGraphInstantiate(&ge[s], g, nullptr, nullptr, 0));
        CK(hipGraphDestroy(g));
      }
      for (int s = 0; s < ns; ++s) CK(hipGraphLaunch(ge[s], st[s]));
      CK(hipDeviceSynchronize());
      float best = 1e30f;
      for (int rep = 0; rep < 5; ++rep) {
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a, nullptr));
        CK(hipDeviceSynchronize());
        for (int s = 0; s < ns; ++s) CK(hipGraphLaunch(ge[s], st[s]));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(b, nullptr));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
      }
      printf("%-8s streams %d: %6.2f us per kernel-slot (chain of %d per stream), %6.2f us per kernel overall\n",
             names[mode], ns, best * 1e3 / N, N, best * 1e3 / (N * ns));
      for (int s = 0; s < ns; ++s) {
        CK(hipGraphExecDestroy(ge[s]));
        CK(hipStreamDestroy(st[s]));
      }
    }
  }
  return 0;
}
