// Price of an in-launch grid barrier against a kernel boundary on this chip,
// at the workgroup counts of the batch-1 decode GEMMs (40-160), before
// building a persistent decode layer on them:
//   launches  ROUNDS empty kernels of G workgroups, captured in one HIP graph
//             (the decode step replays its kernels the same way)
//   flat      one launch of G workgroups crossing ROUNDS barriers on one
//             monotonic device-scope counter (relaxed atomic add, relaxed
//             vector-load poll, release / acquire fences)
//   xcd       the same through per-XCD counters (workgroup b on XCD b % 8)
//             whose last arriver bumps a top counter (fewer far atomics)
//   flat-gen  one counter; its last arriver stores a generation word that
//             the others poll (polls and atomics on different lines)
//   xcd-gen   per-XCD counters -> top counter -> generation word
// Every spin gives up after kSpinCap polls and raises an error flag, so a
// wrong barrier ends the launch instead of hanging the GPU.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/barrier_bench tools/barrier_bench.hip
//   ./tools/barrier_bench [rounds]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

constexpr unsigned kSpinCap = 1u << 22;

__global__ void empty_kernel(int* sink) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && sink[1] == 12345) sink[0] = 1;
}

__device__ __forceinline__ unsigned poll(unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// flat: arrival k of every workgroup adds 1; round r completes at (r + 1) * G
__global__ void flat_kernel(unsigned* ctr, int rounds, int* err) {
  const unsigned G = gridDim.x;
  for (int r = 0; r < rounds; ++r) {
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (unsigned)(r + 1) * G;
      unsigned n = 0;
      while (poll(ctr) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++n > kSpinCap) {
          atomicExch(err, 1);
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
  }
}

// xcd: ctr[0..7] per XCD, ctr[8] top.  The last of XCD x's workgroups in
// round r bumps the top; everyone polls the top.
__global__ void xcd_kernel(unsigned* ctr, int rounds, int* err) {
  const unsigned G = gridDim.x, x = blockIdx.x & 7;
  const unsigned nx = G / 8 + ((G & 7) > x ? 1u : 0u);  // workgroups on this XCD
  unsigned nxcd = G < 8 ? G : 8;
  for (int r = 0; r < rounds; ++r) {
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      const unsigned prev = __hip_atomic_fetch_add(&ctr[x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (prev + 1 == (unsigned)(r + 1) * nx)
        __hip_atomic_fetch_add(&ctr[8], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (unsigned)(r + 1) * nxcd;
      unsigned n = 0;
      while (poll(&ctr[8]) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++n > kSpinCap) {
          atomicExch(err, 1);
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
  }
}

// generation forms: counters at ctr[32 x] (one 128-B line each), top at
// ctr[256], generation word at ctr[288]
template <bool XCD>
__global__ void gen_kernel(unsigned* ctr, int rounds, int* err) {
  const unsigned G = gridDim.x, x = blockIdx.x & 7;
  const unsigned nx = G / 8 + ((G & 7) > x ? 1u : 0u);
  const unsigned nxcd = G < 8 ? G : 8;
  unsigned* gen = ctr + 288;
  for (int r = 0; r < rounds; ++r) {
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      bool last;
      if (XCD) {
        const unsigned p = __hip_atomic_fetch_add(&ctr[32 * x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = false;
        if (p + 1 == (unsigned)(r + 1) * nx) {
          const unsigned q = __hip_atomic_fetch_add(&ctr[256], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          last = q + 1 == (unsigned)(r + 1) * nxcd;
        }
      } else {
        const unsigned p = __hip_atomic_fetch_add(&ctr[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = p + 1 == (unsigned)(r + 1) * G;
      }
      if (last) {
        __hip_atomic_store(gen, (unsigned)(r + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        unsigned n = 0;
        while (poll(gen) < (unsigned)(r + 1)) {
          __builtin_amdgcn_s_sleep(1);
          if (++n > kSpinCap) {
            atomicExch(err, 1);
            break;
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
  }
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 200;
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  unsigned* ctr;
  int* err;
  int* sink;
  CHECK(hipMalloc(&ctr, 512 * sizeof(unsigned)));
  CHECK(hipMalloc(&err, sizeof(int)));
  CHECK(hipMalloc(&sink, 2 * sizeof(int)));
  CHECK(hipMemset(sink, 0, 2 * sizeof(int)));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int G : {40, 80, 160, 256}) {
    // launches: graph of `rounds` empty kernels
    hipGraph_t gr;
    hipGraphExec_t ge;
    CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < rounds; ++i) hipLaunchKernelGGL(empty_kernel, dim3(G), dim3(512), 0, st, sink);
    CHECK(hipStreamEndCapture(st, &gr));
    CHECK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
    std::vector<float> tl, tm[4];
    for (int rep = 0; rep < 6; ++rep) {
      float ms = 0;
      CHECK(hipEventRecord(a, st));
      CHECK(hipGraphLaunch(ge, st));
      CHECK(hipEventRecord(b, st));
      CHECK(hipEventSynchronize(b));
      CHECK(hipEventElapsedTime(&ms, a, b));
      tl.push_back(ms * 1000.0f / rounds);
      for (int mode = 0; mode < 4; ++mode) {
        CHECK(hipMemsetAsync(ctr, 0, 512 * sizeof(unsigned), st));
        CHECK(hipMemsetAsync(err, 0, sizeof(int), st));
        CHECK(hipEventRecord(a, st));
        if (mode == 0)
          hipLaunchKernelGGL(flat_kernel, dim3(G), dim3(512), 0, st, ctr, rounds, err);
        else if (mode == 1)
          hipLaunchKernelGGL(xcd_kernel, dim3(G), dim3(512), 0, st, ctr, rounds, err);
        else if (mode == 2)
          hipLaunchKernelGGL(gen_kernel<false>, dim3(G), dim3(512), 0, st, ctr, rounds, err);
        else
          hipLaunchKernelGGL(gen_kernel<true>, dim3(G), dim3(512), 0, st, ctr, rounds, err);
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(b, st));
        CHECK(hipEventSynchronize(b));
        CHECK(hipEventElapsedTime(&ms, a, b));
        int e = 0;
        CHECK(hipMemcpy(&e, err, sizeof(int), hipMemcpyDeviceToHost));
        if (e) {
          fprintf(stderr, "G=%d mode %d: barrier gave up\n", G, mode);
          return 1;
        }
        tm[mode].push_back(ms * 1000.0f / rounds);
      }
    }
    auto med = [](std::vector<float> v) {
      std::sort(v.begin() + 1, v.end());
      return v[1 + (v.size() - 1) / 2];
    };
    printf("G=%3d workgroups x 512 threads: kernel boundary (graph) %.2f us; barrier flat %.2f, xcd %.2f, "
           "flat-gen %.2f, xcd-gen %.2f us (median of 5, per round over %d rounds)\n",
           G, med(tl), med(tm[0]), med(tm[1]), med(tm[2]), med(tm[3]), rounds);
    CHECK(hipGraphExecDestroy(ge));
    CHECK(hipGraphDestroy(gr));
  }
  return 0;
}
