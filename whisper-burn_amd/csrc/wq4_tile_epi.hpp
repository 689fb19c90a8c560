// wq4_tile_epi.hpp -- epilogue of the encoder-size Q4 GEMM kernels (the
// prefill tile kernel and the 8-wave wide kernel): one wave's TM x TN tiles
// of 32 x 32 accumulators, v_mfma_f32_32x32x16_* C/D layout, written as f32
// rows (bias / GELU / residual, linear.rs:34-40, layers.rs:35-58), head-major
// f32 (the cross K / V caches) or the A-tiled f16 operand of the next GEMM.
#pragma once
#include "wq4_device.hpp"

namespace wq4 {

constexpr int kStageLd = 68;  // padded f32 row stride of the transpose stage

// acc[i] of a 32x32 tile: row (i&3) + 8*(i>>2) + 4*h, column r (C/D layout of
// v_mfma_f32_32x32x16_*, cdna_hip_programming.md §3).
__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// Writes one wave's 32-row slab (TN n-tiles of 32 cols) held in `stage`
// ([32][kStageLd] f32, already epilogue-applied) as A-tiled f16 fragments.
template <int NS, int TN>
__device__ __forceinline__ void store_tiled_slab(const float* stage, const EpiArgs& e, int mt_g, int nt_g0,
                                                 int lane) {
  const int r = lane & 31, h = lane >> 5;
  half8* dst = reinterpret_cast<half8*>(e.out_tiled);
  const size_t kbp_next = (size_t)e.nbp_next * 2;
#pragma unroll
  for (int nt = 0; nt < TN; ++nt) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const float* src = stage + r * kStageLd + nt * 32 + kk * 16 + h * 8;
      const floatx4 a = *reinterpret_cast<const floatx4*>(src);
      const floatx4 c = *reinterpret_cast<const floatx4*>(src + 4);
      half8 hi, lo;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        _Float16 x, y;
        split_act(a[j], x, y);
        hi[j] = x;
        lo[j] = y;
        split_act(c[j], x, y);
        hi[4 + j] = x;
        lo[4 + j] = y;
      }
      const size_t frag = (((size_t)mt_g * kbp_next + (nt_g0 + nt)) * 2 + kk) * NS;
      dst[(frag + 0) * 64 + lane] = hi;
      if constexpr (NS == 2) dst[(frag + 1) * 64 + lane] = lo;
    }
  }
}

// The epilogue of one wave's tiles: acc[mt][nt] holds global m-tile
// mt_base + mt (rows 32 (mt_base + mt) + acc_row) and n-tile nt0 + nt.
// y = epi(acc * colscale[col] * act_inv).  `stage` is this wave's own
// [32][kStageLd] f32 LDS region (EPI == kEpiTiled only); `mtiles_out` bounds
// the A-tiled m-tiles written (the output operand's allocation).
template <int NS, int EPI, int TM, int TN>
__device__ __forceinline__ void tile_epilogue(const floatx16 (&acc)[TM][TN], int mt_base, int nt0, bool active,
                                              int mtiles_out, const float* __restrict__ colscale, float* stage,
                                              int lane, const EpiArgs& e) {
  const int r = lane & 31, h = lane >> 5;
  float cs[TN];
  const float ainv = e.act_inv ? *e.act_inv : kActScaleInv;  // A operand scale (exact power of two)
#pragma unroll
  for (int nt = 0; nt < TN; ++nt) cs[nt] = active ? colscale[(nt0 + nt) * 32 + r] * ainv : 1.0f;

  if constexpr (EPI == kEpiF32) {
    if (active) {
#pragma unroll
      for (int mt = 0; mt < TM; ++mt)
#pragma unroll
        for (int nt = 0; nt < TN; ++nt)
          epi_store_tile(
              acc[mt][nt], cs[nt], (nt0 + nt) * 32 + r, [&](int i) { return (mt_base + mt) * 32 + acc_row(i, h); },
              [&](int row, int col) { return (size_t)row * e.ldo + col; }, e);
    }
  } else if constexpr (EPI == kEpiHeadMajor) {
    if (active) {
      // one division per m-tile and n-tile, not per element (out_index)
      size_t cofs[TN];
#pragma unroll
      for (int nt = 0; nt < TN; ++nt) {
        const int col = (nt0 + nt) * 32 + r;
        const int part = col / e.hm_d, c = col - part * e.hm_d;
        cofs[nt] = (size_t)part * e.m * e.hm_d + (size_t)(c >> 6) * e.hm_t * 64 + (c & 63);
      }
      const size_t gstride = (size_t)(e.hm_d >> 6) * e.hm_t * 64;
#pragma unroll
      for (int mt = 0; mt < TM; ++mt) {
        const int r0 = (mt_base + mt) * 32;
        const int g0 = r0 / e.hm_t, t0 = r0 - g0 * e.hm_t;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int rl = acc_row(i, h), row = r0 + rl;
          int t = t0 + rl, g = g0;
          while (t >= e.hm_t) {  // at most one step when hm_t >= 32
            t -= e.hm_t;
            ++g;
          }
          const size_t rofs = (size_t)g * gstride + (size_t)t * 64;
#pragma unroll
          for (int nt = 0; nt < TN; ++nt) {
            const int col = (nt0 + nt) * 32 + r;
            if (row < e.m && col < e.n) e.out[rofs + cofs[nt]] = epi_value(acc[mt][nt][i] * cs[nt], row, col, e);
          }
        }
      }
    }
  } else {
#pragma unroll
    for (int mt = 0; mt < TM; ++mt) {
      if (active && mt_base + mt < mtiles_out) {
#pragma unroll
        for (int nt = 0; nt < TN; ++nt)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int rl = acc_row(i, h);
            const int row = (mt_base + mt) * 32 + rl;
            const int col = (nt0 + nt) * 32 + r;
            const float v = (row < e.m && col < e.n) ? epi_value(acc[mt][nt][i] * cs[nt], row, col, e) : 0.0f;
            stage[rl * kStageLd + nt * 32 + r] = v;
          }
        // the stage is this wave's own (the K loop's last barrier freed the
        // A buffers under it): a wave-local hand-off, no workgroup barrier
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): stage writes visible to this wave
        __builtin_amdgcn_wave_barrier();
        store_tiled_slab<NS, TN>(stage, e, mt_base + mt, nt0, lane);
        __builtin_amdgcn_wave_barrier();
      }
    }
  }
}

}  // namespace wq4
