// wq4_lnmath.hpp -- LayerNorm arithmetic shared bit-for-bit by the model's
// LayerNorm kernel (whisper/wa_kernels.hip) and the LN-fused decode GEMM
// (wq4_q4gemm.hip): src/model/layers.rs:12-32 (eps 1e-5, biased variance,
// two-pass mean / variance).  One wave owns a row; lane l holds the float4s
// at k = 4 l + 256 i.  Both kernels call exactly these functions, so the
// fused and unfused decode paths produce identical operands.
#pragma once
#include <hip/hip_runtime.h>

#include "wq4_device.hpp"

namespace wq4 {

constexpr int kLnMaxV = 8;  // D <= 2048

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// mean and sqrt(var + eps) of the row held in v (zeros past D).
__device__ __forceinline__ void ln_row_stats(const floatx4 (&v)[kLnMaxV], int D, int lane, float& mean,
                                             float& den) {
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < kLnMaxV; ++i) s += (v[i][0] + v[i][1]) + (v[i][2] + v[i][3]);
  mean = wave_sum(s) / (float)D;
  float s2 = 0.0f;
#pragma unroll
  for (int i = 0; i < kLnMaxV; ++i) {
    const int k = lane * 4 + 256 * i;
    if (k < D) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float c = v[i][j] - mean;
        s2 += c * c;
      }
    }
  }
  den = sqrtf(wave_sum(s2) / (float)D + 1e-5f);
}

__device__ __forceinline__ float ln_apply(float v, float mean, float den, float g, float b) {
  return ((v - mean) / den) * g + b;
}

}  // namespace wq4
