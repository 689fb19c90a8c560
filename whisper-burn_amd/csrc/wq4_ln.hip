// wq4_ln.hip -- LayerNorm writing the A-tiled operand of the next Q4 GEMM
// (or f32 rows): src/model/layers.rs:12-32 (eps 1e-5, biased variance).
#include <hip/hip_runtime.h>

#include "wq4_kernels.hpp"
#include "wq4_lnmath.hpp"

namespace wq4 {

// ------------------------------------------------------------------ LN --
// One wave per row; the row stays in registers (D <= 64 * 4 * kLnMaxV).
// Arithmetic in wq4_lnmath.hpp, shared with the decode GEMM's residual + LN tail.
template <int NS, bool TILED>
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                        const float* __restrict__ bb, int M, int D,
                                                        _Float16* __restrict__ tiled, float* __restrict__ out) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int kbp = kbp_of(D);
  const int rows_total = TILED ? ((M + 31) / 32) * 32 : M;
  const int row = blockIdx.x * 4 + wave;
  if (row >= rows_total) return;
  if (row >= M) {  // padded rows of the last m-tile: finite zeros
    if constexpr (TILED)
      for (int k = lane * 4; k < D; k += 256) atile_store4<NS>(tiled, row, k, kbp, 0.f, 0.f, 0.f, 0.f);
    return;
  }
  const float* xr = x + (size_t)row * D;
  floatx4 v[kLnMaxV];
#pragma unroll
  for (int i = 0; i < kLnMaxV; ++i) {
    const int k = lane * 4 + 256 * i;
    v[i] = k < D ? *reinterpret_cast<const floatx4*>(xr + k) : floatx4{0.f, 0.f, 0.f, 0.f};
  }
  float mean, den;
  ln_row_stats(v, D, lane, mean, den);
#pragma unroll
  for (int i = 0; i < kLnMaxV; ++i) {
    const int k = lane * 4 + 256 * i;
    if (k < D) {
      const floatx4 g = *reinterpret_cast<const floatx4*>(w + k);
      const floatx4 be = *reinterpret_cast<const floatx4*>(bb + k);
      float y[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) y[j] = ln_apply(v[i][j], mean, den, g[j], be[j]);
      if constexpr (TILED)
        atile_store4<NS>(tiled, row, k, kbp, y[0], y[1], y[2], y[3]);
      else
        *reinterpret_cast<floatx4*>(out + (size_t)row * D + k) = floatx4{y[0], y[1], y[2], y[3]};
    }
  }
}

hipError_t launch_layernorm(const float* x, const float* w, const float* b, int M, int D, _Float16* tiled, int ns,
                            float* out, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (D % 4 != 0 || D > 256 * kLnMaxV) return hipErrorInvalidValue;
  const int rows_total = tiled ? ((M + 31) / 32) * 32 : M;
  const dim3 grid((rows_total + 3) / 4), block(256);
  if (tiled) {
    if (ns == 2)
      hipLaunchKernelGGL((layernorm_kernel<2, true>), grid, block, 0, st, x, w, b, M, D, tiled, out);
    else
      hipLaunchKernelGGL((layernorm_kernel<1, true>), grid, block, 0, st, x, w, b, M, D, tiled, out);
  } else {
    hipLaunchKernelGGL((layernorm_kernel<2, false>), grid, block, 0, st, x, w, b, M, D, tiled, out);
  }
  return hipGetLastError();
}

}  // namespace wq4
