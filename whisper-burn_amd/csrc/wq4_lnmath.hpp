// wq4_lnmath.hpp -- LayerNorm arithmetic shared bit-for-bit by the
// LayerNorm kernel (wq4_ln.hip) and the residual + LayerNorm tail of the
// decode GEMM (wq4_q4gemm.hip), plus the A-tiled operand store helpers: src/model/layers.rs:12-32 (eps 1e-5, biased variance,
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

// Index (in halves) of element (row, k) of an A-tiled operand with kbp
// (even) Q4 blocks per row, split s.
__device__ __forceinline__ size_t atile_index(int row, int k, int kbp, int ns, int s) {
  const int mt = row >> 5, r = row & 31;
  const int b = k >> 5, kk = (k >> 4) & 1, hh = (k >> 3) & 1, j = k & 7;
  return (((((size_t)mt * kbp + b) * 2 + kk) * ns + s) * 64 + (r + 32 * hh)) * 8 + j;
}

// Write 4 consecutive k (k % 4 == 0) of one row into the A-tiled operand.
template <int NS>
__device__ __forceinline__ void atile_store4(_Float16* t, int row, int k, int kbp, float a, float b, float c,
                                             float d) {
  typedef _Float16 half4 __attribute__((ext_vector_type(4)));
  half4 hi, lo;
  const float v[4] = {a, b, c, d};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    _Float16 x, y;
    split_act(v[j], x, y);
    hi[j] = x;
    lo[j] = y;
  }
  *reinterpret_cast<half4*>(t + atile_index(row, k, kbp, NS, 0)) = hi;
  if constexpr (NS == 2) *reinterpret_cast<half4*>(t + atile_index(row, k, kbp, NS, 1)) = lo;
}

// Attention-output store: four consecutive columns k .. k + 3 of row `row`
// as the A-tiled operand of the output projection, or -- range tier 3
// (wa_model: an attention output beyond the f16 pair's range) -- as f32 rows
// [row][ld] into o32 when it is non-null (wave-uniform).
template <int NS>
__device__ __forceinline__ void attn_store4(_Float16* t, float* o32, int ld, int row, int k, int kbp, float a, float b,
                                            float c, float d) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  if (o32) {
    *reinterpret_cast<f4*>(o32 + (size_t)row * ld + k) = f4{a, b, c, d};
    return;
  }
  atile_store4<NS>(t, row, k, kbp, a, b, c, d);
}

// LayerNorm-fold consumer: a row's mean and sqrt(var + eps) from its
// `tiles` 16-column tile statistics (tile mean m_j, sum of squared
// deviations q_j), spread over 16 consecutive lanes (part p holds tiles p,
// p + 16, ...; zeros past `tiles`).  Every tile holds 16 values, so the
// exact merge is the equal-count one:
//   mean = (sum_j m_j) / T,   M2 = sum_j q_j + 16 sum_j (m_j - mean)^2
// -- two passes, two divisions per row (the per-step divisions of a
// pairwise merge cost ~1.7 us per launch on the decode critical path,
// tools/warm_cold.py).  The cross-lane sums are xor butterflies; a + b is
// commutative bit-for-bit, so every lane and every workgroup gets the same
// bits, and the result depends on (K, the statistics) only.
template <int NPER>
__device__ __forceinline__ void lnf_merge_tiles(const floatx2 (&st)[NPER], int part, int tiles, float& mean,
                                                float& den) {
  float s = 0.0f;
#pragma unroll
  for (int v = 0; v < NPER; ++v) s += part + 16 * v < tiles ? st[v][0] : 0.0f;
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) s += __shfl_xor(s, o, 64);
  mean = s / (float)tiles;
  float q = 0.0f;
#pragma unroll
  for (int v = 0; v < NPER; ++v) {
    const float d = st[v][0] - mean;
    q += part + 16 * v < tiles ? st[v][1] + 16.0f * (d * d) : 0.0f;
  }
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) q += __shfl_xor(q, o, 64);
  den = sqrtf(q / (float)(16 * tiles) + 1e-5f);
}

__host__ __device__ inline int kbp_of(int k) { return ((k / 32 + 1) / 2) * 2; }

// The LayerNorm-fold consumer's correction (a - mean * (W gamma)[n]) / den
// with the product-difference as ONE explicit fma: every kernel implementing
// the consumer (the 8-wave decode kernel, the decode-step kernel) shares it,
// so floating-point contraction cannot make their bits differ.
__device__ __forceinline__ float lnf_apply(float a, float mean, float wg, float den) {
  return fmaf(-mean, wg, a) / den;
}

__device__ __forceinline__ float ln_apply(float v, float mean, float den, float g, float b) {
  return ((v - mean) / den) * g + b;
}

}  // namespace wq4
