// mfma_cycles.hip -- issue cost of the f16 MFMA shapes on gfx950 (one wave,
// back-to-back independent accumulators), measured with s_memtime.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_cycles.hip -o build/mfma_cycles && build/mfma_cycles
#include <hip/hip_runtime.h>

#include <cstdio>

typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kIters = 256;

template <int KIND>
__global__ void bench(float* out, long long* cyc) {
  floatx4 a4[4] = {};
  floatx16 a16[2] = {};
  half4 x4 = {(_Float16)threadIdx.x, 1, 2, 3};
  half8 x8 = {(_Float16)threadIdx.x, 1, 2, 3, 4, 5, 6, 7};
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (KIND == 0) a4[j] = __builtin_amdgcn_mfma_f32_16x16x16f16(x4, x4, a4[j], 0, 0, 0);
      if (KIND == 1) a4[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(x8, x8, a4[j], 0, 0, 0);
      if (KIND == 2) a16[j & 1] = __builtin_amdgcn_mfma_f32_32x32x8f16(x4, x4, a16[j & 1], 0, 0, 0);
      if (KIND == 3) a16[j & 1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(x8, x8, a16[j & 1], 0, 0, 0);
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int j = 0; j < 4; ++j) s += a4[j][0];
  for (int j = 0; j < 2; ++j) s += a16[j][0];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

int main() {
  float* out;
  long long* cyc;
  (void)hipMalloc(&out, 256 * 4);
  (void)hipMalloc(&cyc, 8);
  const char* names[4] = {"16x16x16f16", "16x16x32_f16", "32x32x8f16", "32x32x16_f16"};
  for (int k = 0; k < 4; ++k) {
    for (int rep = 0; rep < 2; ++rep) {
      if (k == 0) hipLaunchKernelGGL(bench<0>, dim3(1), dim3(64), 0, 0, out, cyc);
      if (k == 1) hipLaunchKernelGGL(bench<1>, dim3(1), dim3(64), 0, 0, out, cyc);
      if (k == 2) hipLaunchKernelGGL(bench<2>, dim3(1), dim3(64), 0, 0, out, cyc);
      if (k == 3) hipLaunchKernelGGL(bench<3>, dim3(1), dim3(64), 0, 0, out, cyc);
      (void)hipDeviceSynchronize();
    }
    long long c = 0;
    (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    // s_memtime ticks at the shader clock (MI355X_MICROARCH.md cycle table)
    printf("%-14s %.1f cycles per MFMA\n", names[k], (double)c / (kIters * 4));
  }
  return 0;
}
