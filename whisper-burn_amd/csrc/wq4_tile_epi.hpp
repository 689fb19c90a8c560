// wq4_tile_epi.hpp -- epilogue of the encoder-size Q4 GEMM kernels (the
// prefill tile kernel and the 8-wave wide kernel): one wave's TM x TN tiles
// of 32 x 32 accumulators, v_mfma_f32_32x32x16_* C/D layout, written as f32
// rows (bias / GELU / residual, linear.rs:34-40, layers.rs:35-58), head-major
// f32 (the cross K / V caches) or the A-tiled f16 operand of the next GEMM.
#pragma once
#include <type_traits>

#include "wq4_device.hpp"

namespace wq4 {

constexpr int kStageLd = 68;  // padded f32 row stride of the transpose stage

// Branch-free epilogue memory operations: a buffer descriptor over `bytes`
// (0 for an absent operand: its loads read 0, its stores are dropped) and a
// voffset past any descriptor for masked columns (descriptors < 2 GiB, so
// voffset + soffset cannot wrap).
constexpr uint32_t kEpiOob = 0x80000000u;
// cache-policy bits of the f32 epilogue's buffer stores (A/B builds only:
// 0 = default, 2 = nt streaming)
#ifndef WQ4_EPI_STORE_AUX
#define WQ4_EPI_STORE_AUX 0
#endif
__device__ __forceinline__ __amdgpu_buffer_rsrc_t epi_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

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
// the A-tiled m-tiles written (the output operand's allocation).  `pre`
// (optional, LDS): this wave's columns' colscale x act_inv at pre[nt * 32 +
// r] and bias at pre[256 + nt * 32 + r], staged by the kernel before its K
// loop ended (the same products: the same bits); otherwise both are loaded
// here, two memory round trips.
template <int NS, int EPI, int TM, int TN>
__device__ __forceinline__ void tile_epilogue(const floatx16 (&acc)[TM][TN], int mt_base, int nt0, bool active,
                                              int mtiles_out, const float* __restrict__ colscale, float* stage,
                                              int lane, const EpiArgs& e, const float* pre = nullptr) {
  const int r = lane & 31, h = lane >> 5;
  float cs[TN], b[TN];
  if (pre) {
#pragma unroll
    for (int nt = 0; nt < TN; ++nt) {
      cs[nt] = active ? pre[nt * 32 + r] : 1.0f;
      b[nt] = pre[256 + nt * 32 + r];
    }
  } else {
    const float ainv = e.act_inv ? *e.act_inv : kActScaleInv;  // A operand scale (exact power of two)
    const __amdgpu_buffer_rsrc_t rb = epi_rsrc(e.bias, e.bias ? (uint32_t)e.n * 4 : 0);
#pragma unroll
    for (int nt = 0; nt < TN; ++nt) {
      const int col = (nt0 + nt) * 32 + r;
      cs[nt] = active ? colscale[col] * ainv : 1.0f;
      b[nt] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rb, col < e.n ? col * 4 : kEpiOob, 0, 0));
    }
    // landed before the first store (vmcnt(0) with nothing else in flight):
    // otherwise hipcc waits for them, behind every earlier store, at the top
    // of each exec-masked head-major store
    __builtin_amdgcn_s_waitcnt(0x0F70);
  }

  if constexpr (EPI == kEpiF32) {
    // Buffer loads and stores, masked by offset instead of by branch: a
    // load or store under an exec branch made hipcc drain vmcnt(0) at every
    // join -- one wait for all earlier stores per element, 25-31 us of a
    // 256 x 256 tile's epilogue in the wide kernel (tools/wide_stamps.py).
    // Residuals of half the m-tiles in flight at once, all loaded before any
    // store of theirs (out may alias residual: same element, same lane).
    const uint64_t obytes = (uint64_t)e.m * (uint64_t)e.ldo * 4;
    // padded rows (< 256 past m) add to soffset: kEpiOob + soffset must not
    // wrap past 2^32 back into the descriptor
    if (active && obytes + (uint64_t)256 * (uint64_t)e.ldo * 4 < (1ull << 31)) {
      const __amdgpu_buffer_rsrc_t rr = epi_rsrc(e.residual, e.residual ? (uint32_t)obytes : 0);
      const __amdgpu_buffer_rsrc_t ro = epi_rsrc(e.out, (uint32_t)obytes);
      // element (mt, nt, i) at voff[nt] (this lane's column and row half h;
      // masked columns past every descriptor) + soff(mt, i) (wave-uniform
      // row part); rows >= m land past the descriptor by themselves
      uint32_t voff[TN];
#pragma unroll
      for (int nt = 0; nt < TN; ++nt) {
        const int col = (nt0 + nt) * 32 + r;
        voff[nt] = col < e.n ? ((uint32_t)(4 * h) * (uint32_t)e.ldo + (uint32_t)col) * 4 : kEpiOob;
      }
      const uint32_t ld4 = (uint32_t)e.ldo * 4;
      auto soff = [&](int mt, int i) -> uint32_t {
        return ((uint32_t)(mt_base + mt) * 32 + (uint32_t)((i & 3) + 8 * (i >> 2))) * ld4;
      };
      if (e.residual) {
        constexpr int HM = TM > 1 ? TM / 2 : 1;  // m-tiles per round of residual loads
#pragma unroll
        for (int m0 = 0; m0 < TM; m0 += HM) {
          float res[HM][TN][16];
#pragma unroll
          for (int mt = 0; mt < HM; ++mt)
#pragma unroll
            for (int nt = 0; nt < TN; ++nt)
#pragma unroll
              for (int i = 0; i < 16; ++i)
                res[mt][nt][i] =
                    __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rr, voff[nt], soff(m0 + mt, i), 0));
#pragma unroll
          for (int mt = 0; mt < HM; ++mt)
#pragma unroll
            for (int nt = 0; nt < TN; ++nt)
#pragma unroll
              for (int i = 0; i < 16; ++i)
                __builtin_amdgcn_raw_buffer_store_b32(
                    __builtin_bit_cast(uint32_t, epi_value_pre(acc[m0 + mt][nt][i] * cs[nt], b[nt], res[mt][nt][i], e)),
                    ro, voff[nt], soff(m0 + mt, i), WQ4_EPI_STORE_AUX);
        }
      } else {
#pragma unroll
        for (int mt = 0; mt < TM; ++mt)
#pragma unroll
          for (int nt = 0; nt < TN; ++nt)
#pragma unroll
            for (int i = 0; i < 16; ++i)
              __builtin_amdgcn_raw_buffer_store_b32(
                  __builtin_bit_cast(uint32_t, epi_value_pre(acc[mt][nt][i] * cs[nt], b[nt], 0.0f, e)), ro, voff[nt],
                  soff(mt, i), WQ4_EPI_STORE_AUX);
      }
    } else if (active) {  // outputs past 2 GiB: pointer stores
#pragma unroll
      for (int mt = 0; mt < TM; ++mt)
#pragma unroll
        for (int nt = 0; nt < TN; ++nt)
          epi_store_tile(
              acc[mt][nt], cs[nt], (nt0 + nt) * 32 + r, [&](int i) { return (mt_base + mt) * 32 + acc_row(i, h); },
              [&](int row, int col) { return (size_t)row * e.ldo + col; }, e);
    }
  } else if constexpr (EPI == kEpiHeadMajor) {
    // RES: with a residual the element-wise epi_value (pointer loads); without
    // (the K / V cache GEMMs) the preloaded bias and no load at all
    auto run = [&](auto res_c) {
      constexpr bool RES = decltype(res_c)::value;
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
            if (row < e.m && col < e.n)
              e.out[rofs + cofs[nt]] = RES ? epi_value(acc[mt][nt][i] * cs[nt], row, col, e)
                                           : epi_value_pre(acc[mt][nt][i] * cs[nt], b[nt], 0.0f, e);
          }
        }
      }
    };
    if (active) {
      if (e.residual) run(std::true_type{});
      else run(std::false_type{});
    }
  } else {
    // RES as above (the GELU GEMM has no residual: no memory access before
    // the slab stores)
    auto run = [&](auto res_c) {
      constexpr bool RES = decltype(res_c)::value;
#pragma unroll
      for (int mt = 0; mt < TM; ++mt) {
        if (mt_base + mt < mtiles_out) {
#pragma unroll
          for (int nt = 0; nt < TN; ++nt)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int rl = acc_row(i, h);
              const int row = (mt_base + mt) * 32 + rl;
              const int col = (nt0 + nt) * 32 + r;
              const float v = !(row < e.m && col < e.n) ? 0.0f
                              : RES ? epi_value(acc[mt][nt][i] * cs[nt], row, col, e)
                                    : epi_value_pre(acc[mt][nt][i] * cs[nt], b[nt], 0.0f, e);
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
    };
    if (active) {
      if (e.residual) run(std::true_type{});
      else run(std::false_type{});
    }
  }
}

}  // namespace wq4
