// wq4_ln.hip -- LayerNorm writing the A-tiled operand of the next Q4 GEMM
// (or f32 rows): src/model/layers.rs:12-32 (eps 1e-5, biased variance).
#include <hip/hip_runtime.h>

#include "wq4_kernels.hpp"
#include "wq4_lnmath.hpp"

namespace wq4 {

// ------------------------------------------------------------------ LN --
// One wave per row; the row stays in registers (D <= 64 * 4 * kLnMaxV).
// Arithmetic in wq4_lnmath.hpp, shared with the decode GEMM's LayerNorm-on-
// load and with layernorm_tiled_kernel below (the A-tiled form for large M).
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

// A-tiled output, one workgroup per 32-row m-tile: wave w normalises rows
// 4w .. 4w+3 in registers (the per-row arithmetic of layernorm_kernel, so
// the bits are the same), then per 512-column chunk the waves stage the f16
// pairs in LDS and write whole 1 KiB fragments (one 16-B store per lane)
// instead of 8-B pieces scattered over the fragments.  Rows >= M and columns
// >= D of the tile are written as zeros.
constexpr int kLnTileKc = 512;
constexpr int kLnTileMinRows = 2048;
template <int NS>
__global__ __launch_bounds__(512) void layernorm_tiled_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                              const float* __restrict__ bb, int M, int D,
                                                              _Float16* __restrict__ tiled) {
  constexpr int LDR = kLnTileKc + 8;  // halves per staged row
  __shared__ __attribute__((aligned(16))) _Float16 sh[NS][32 * LDR];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int mt = blockIdx.x, kbp = kbp_of(D);
  floatx4 v[4][kLnMaxV];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int row = mt * 32 + 4 * wave + q;
    const float* xr = x + (size_t)(row < M ? row : 0) * D;
#pragma unroll
    for (int i = 0; i < kLnMaxV; ++i) {
      const int k = lane * 4 + 256 * i;
      v[q][i] = (row < M && k < D) ? *reinterpret_cast<const floatx4*>(xr + k) : floatx4{0.f, 0.f, 0.f, 0.f};
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int row = mt * 32 + 4 * wave + q;
    if (row < M) {  // wave-uniform
      float mean, den;
      ln_row_stats(v[q], D, lane, mean, den);
#pragma unroll
      for (int i = 0; i < kLnMaxV; ++i) {
        const int k = lane * 4 + 256 * i;
        if (k < D) {
          const floatx4 g = *reinterpret_cast<const floatx4*>(w + k);
          const floatx4 be = *reinterpret_cast<const floatx4*>(bb + k);
#pragma unroll
          for (int j = 0; j < 4; ++j) v[q][i][j] = ln_apply(v[q][i][j], mean, den, g[j], be[j]);
        }
      }
    }
  }
  half8* dst = reinterpret_cast<half8*>(tiled);
  for (int k0 = 0; k0 < D; k0 += kLnTileKc) {
    const int kc = min(kLnTileKc, D - k0);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < kLnMaxV; ++i) {
        const int k = lane * 4 + 256 * i;
        if (k >= k0 && k < k0 + kc) {
          typedef _Float16 half4 __attribute__((ext_vector_type(4)));
          half4 hi, lo;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            _Float16 a, c;
            split_act(v[q][i][j], a, c);
            hi[j] = a;
            lo[j] = c;
          }
          *reinterpret_cast<half4*>(&sh[0][(4 * wave + q) * LDR + (k - k0)]) = hi;
          if constexpr (NS == 2) *reinterpret_cast<half4*>(&sh[NS - 1][(4 * wave + q) * LDR + (k - k0)]) = lo;
        }
      }
    __syncthreads();
    // fragments (block, kk) of this chunk: lane (r, h) = row r, columns
    // 32 block + 16 kk + 8 h .. + 7
    const int nb = (kc + 31) / 32, r = lane & 31, h = lane >> 5;
    for (int f = wave; f < 2 * nb; f += 8) {
      const int bl = f >> 1, kk = f & 1, kl = bl * 32 + kk * 16 + 8 * h;
#pragma unroll
      for (int p = 0; p < NS; ++p) {
        half8 val = *reinterpret_cast<const half8*>(&sh[p][r * LDR + (kl < kc ? kl : 0)]);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (kl + j >= kc) val[j] = (_Float16)0.0f;  // columns >= D (D % 8 != 0)
        dst[((((size_t)mt * kbp + k0 / 32 + bl) * 2 + kk) * NS + p) * 64 + lane] = val;
      }
    }
    __syncthreads();
  }
}

hipError_t launch_layernorm(const float* x, const float* w, const float* b, int M, int D, _Float16* tiled, int ns,
                            float* out, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (D % 4 != 0 || D > 256 * kLnMaxV) return hipErrorInvalidValue;
  // A-tiled output: the m-tile kernel (whole-fragment stores) once there are
  // enough m-tiles to fill the chip (encoder: 1500 at 32 clips; 21 % faster
  // than one wave per row, PMC r02), one wave per row below (prompt and
  // decode rows: 2 m-tiles would run on 2 CUs).  Same bits either way.
  const dim3 grid((((M + 31) / 32) * 32 + 3) / 4), block(256);
  if (tiled && M > kLnTileMinRows) {
    const dim3 gt((M + 31) / 32);
    if (ns == 2)
      hipLaunchKernelGGL((layernorm_tiled_kernel<2>), gt, dim3(512), 0, st, x, w, b, M, D, tiled);
    else
      hipLaunchKernelGGL((layernorm_tiled_kernel<1>), gt, dim3(512), 0, st, x, w, b, M, D, tiled);
  } else if (tiled) {
    if (ns == 2)
      hipLaunchKernelGGL((layernorm_kernel<2, true>), grid, block, 0, st, x, w, b, M, D, tiled, out);
    else
      hipLaunchKernelGGL((layernorm_kernel<1, true>), grid, block, 0, st, x, w, b, M, D, tiled, out);
  } else {
    hipLaunchKernelGGL((layernorm_kernel<2, false>), dim3((M + 3) / 4), block, 0, st, x, w, b, M, D, tiled, out);
  }
  return hipGetLastError();
}

}  // namespace wq4
