// wa_headproj.hpp -- a LayerNorm-folded Q4_0 projection of a few activation
// rows formed inside an attention launch (decode steps).
//
// A decode step is a chain of short launches; where an
// attention workgroup owns whole heads it can form the head's projection
// itself instead of waiting for a GEMM launch:
//   * the fused decoder self-attention of a few-clip group (q, k, v of its
//     head, one clip: 12 subtiles of 16 columns, ROWS = 1; decoder.rs:77-112,
//     attention.rs:93-125),
//   * the K / V cross-attention of a few-clip group (q of its head, one clip:
//     4 subtiles, ROWS = 1; attention.rs:208-236),
//   * the cross-attention query transform of a 16-clip group (q of its head
//     for all 16 clips: 4 subtiles, ROWS = 16; wa_xattn.hip).
// The arithmetic is that of the decode-step GEMM (wq4_skinny.hip,
// skinny_gemm_kernel) as a LayerNorm-fold consumer (wq4_gemm_tiled_lnfold),
// bit for bit: per Q4 block t = MFMA(x_hi, q-8) + MFMA(x_lo, q-8) on
// v_mfma_f32_16x16x32_f16, acc = fma(t, d, acc); 8 (virtual) waves take the
// blocks [w kb/8, (w+1) kb/8) and are summed in wave order; then
//   y = ((sum * 2^-4) - mean * (W gamma)[n]) / sqrt(var + 1e-5) + (W beta + b)[n]
// with (mean, var) merged from the producer's 16-column tile statistics
// (lnf_merge_tiles).  So a fused launch produces exactly the values the GEMM
// launch it replaces would under kernel policy 3
// (tests/test_fused_decode_gpu.py compares the two paths bit for bit).
//
// Memory: the weights of the projection's subtiles (decode-step layout: 1 KiB
// of nibbles per (subtile, 4 blocks), 128 B of scales), the rows' A-tiled
// fragments, their tile statistics and the fold vectors are brought into LDS
// by LDS-DMA (buffer_load ... lds: no registers, every piece in flight at
// once) while the caller's own loads stay in flight behind them (counted
// vmcnt).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../wq4_device.hpp"
#include "../wq4_lnmath.hpp"
#include "wa_kernels.hpp"

namespace wa {

// HeadProj (the kernel argument): wa_kernels.hpp.

constexpr int kHpVW = 8;     // virtual waves (the decode-step kernel's 8 waves)
constexpr int kHpMaxK = 1280;
constexpr int kHpLnPer = 5;  // tile statistics per thread: 16 x 5 = 80 >= K / 16

typedef __attribute__((address_space(3))) void hp_lds_void;

// The LDS image, in 16-B pieces, one DMA instruction per 64 consecutive
// pieces (1 KiB), every region padded to whole instructions:
//   W  weights     [s][u][lane]                 NSUB * ku * 64
//   D  scales      [s][u][8]                    NSUB * ku * 8
//   A  activations [b][kk][plane][half][row]    kb * 8 * ROWS
//   S  statistics  [row][tile] (8 B each)       ROWS * K / 32
//   G  W gamma, B  W beta + bias: 1 KiB each (columns 4 lane .. + 3)
// then (ROWS == 1) the partial sums red[8 virtual waves][NSUB][16]; with
// ROWS == 16 the partials red[8][NSUB][64 lanes][4] overwrite W / D / A once
// every wave is past its MFMAs (hp_store_red).
__host__ __device__ constexpr int hp_pad64(int n) { return (n + 63) / 64 * 64; }
__host__ __device__ constexpr int hp_w_pieces(int nsub, int ku) { return nsub * ku * 64; }
__host__ __device__ constexpr int hp_d_pieces(int nsub, int ku) { return nsub * ku * 8; }
__host__ __device__ constexpr int hp_a_pieces(int rows, int ku) { return ku * 4 * 8 * rows; }
__host__ __device__ constexpr int hp_s_pieces(int rows, int ku) { return rows * ku * 4; }  // rows * (K / 16) / 2
__host__ __device__ constexpr int hp_a_off(int nsub, int ku) {
  return (hp_pad64(hp_w_pieces(nsub, ku)) + hp_pad64(hp_d_pieces(nsub, ku))) * 16;
}
__host__ __device__ constexpr int hp_s_off(int rows, int nsub, int ku) {
  return hp_a_off(nsub, ku) + hp_pad64(hp_a_pieces(rows, ku)) * 16;
}
__host__ __device__ constexpr int hp_g_off(int rows, int nsub, int ku) {
  return hp_s_off(rows, nsub, ku) + hp_pad64(hp_s_pieces(rows, ku)) * 16;
}
__host__ __device__ constexpr int hp_red_off(int rows, int nsub, int ku) {
  return rows == 1 ? hp_g_off(rows, nsub, ku) + 2048 : 0;
}
__host__ __device__ constexpr int hp_red_bytes(int rows, int nsub) {
  return rows == 1 ? kHpVW * nsub * 16 * 4 : kHpVW * nsub * 256 * 4;
}
__host__ __device__ constexpr int hp_lds_bytes(int rows, int nsub, int ku) {
  return rows == 1 ? hp_red_off(rows, nsub, ku) + hp_red_bytes(rows, nsub) : hp_g_off(rows, nsub, ku) + 2048;
}
// Whether a projection fits the scheme: the decode-step layout (K % 128 ==
// 0), the statistics merge (K / 16 <= 80 tiles), the G / B slots (<= 256
// columns), the partials aliasing W / D / A (ROWS == 16), 156 KiB of LDS.
__host__ __device__ constexpr bool hp_supported(int rows, int nsub, int K) {
  return K % 128 == 0 && K >= 128 && K <= kHpMaxK && nsub * 16 <= 256 &&
         (rows == 1 || hp_red_bytes(rows, nsub) <= hp_s_off(rows, nsub, K / 128)) &&
         hp_lds_bytes(rows, nsub, K / 128) <= 156 * 1024;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t hp_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

// Issue every LDS-DMA instruction of the projection: NSUB subtiles (global
// subtile index sub_of(s)), A-tiled rows row0 .. row0 + ROWS - 1 of which the
// first nrows are real (the others read zeros), instructions i = wave, wave
// + nwaves, ...  Pieces past a region read zeros.
template <int ROWS, int NSUB, class SubOf>
__device__ __forceinline__ void hp_issue(const HeadProj& p, SubOf sub_of, int row0, int nrows, uint8_t* lds, int wave,
                                         int nwaves, int lane) {
  const int ku = p.ku, kb = ku * 4, tiles = p.K / 16;
  const int nw = hp_w_pieces(NSUB, ku), nd = hp_d_pieces(NSUB, ku), na = hp_a_pieces(ROWS, ku);
  const int ns = hp_s_pieces(ROWS, ku);
  const int iw = hp_pad64(nw) / 64, id = iw + hp_pad64(nd) / 64, ia = id + hp_pad64(na) / 64,
            is = ia + hp_pad64(ns) / 64;
  const __amdgpu_buffer_rsrc_t rw = hp_rsrc(p.q16, 0x7FFFFFF0u);
  const __amdgpu_buffer_rsrc_t rd = hp_rsrc(p.d16, 0x7FFFFFF0u);
  const __amdgpu_buffer_rsrc_t ra = hp_rsrc(p.at, (uint32_t)kb * 4u * 1024u);  // m-tile 0, f16 pairs
  const __amdgpu_buffer_rsrc_t rs = hp_rsrc(p.stats, (uint32_t)(row0 + nrows) * (uint32_t)tiles * 8u);
  const __amdgpu_buffer_rsrc_t rg = hp_rsrc(p.wg, 0x7FFFFFF0u);
  const __amdgpu_buffer_rsrc_t rb = hp_rsrc(p.b2, 0x7FFFFFF0u);
  constexpr uint32_t kOob = 0x7FFFFFF0u;
  for (int i = wave; i < is + 2; i += nwaves) {  // i is wave-uniform: every branch below is too
    void* dst = lds + (size_t)i * 1024;
    if (i < iw) {
      const int pc = i * 64 + lane, s = pc / (ku * 64), within = pc - s * (ku * 64);
      const uint32_t off = pc < nw ? (uint32_t)(((size_t)sub_of(s) * ku * 64 + within) * 16) : kOob;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (hp_lds_void*)dst, 16, off, 0, 0, 0);
    } else if (i < id) {
      const int q = (i - iw) * 64 + lane, s = q / (ku * 8), within = q - s * (ku * 8);
      const uint32_t off = q < nd ? (uint32_t)(((size_t)sub_of(s) * ku * 8 + within) * 16) : kOob;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rd, (hp_lds_void*)dst, 16, off, 0, 0, 0);
    } else if (i < ia) {
      // piece (((b * 2 + kk) * 2 + plane) * 2 + half) * ROWS + r: A-tiled
      // fragment ((b * 2 + kk) * 2 + plane), lane' row0 + r + 32 half
      const int q = (i - id) * 64 + lane, r = q % ROWS, f = q / ROWS;
      const int h = f & 1, fr = f >> 1;  // fr = (b * 2 + kk) * 2 + plane
      const uint32_t off = q < na && r < nrows ? (uint32_t)((fr * 64 + row0 + r + 32 * h) * 16) : kOob;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (hp_lds_void*)dst, 16, off, 0, 0, 0);
    } else if (i < is) {  // the rows' (mean, M2) tile statistics, contiguous [row][tile]
      const int q = (i - ia) * 64 + lane;
      const uint32_t off = q < ns ? (uint32_t)(row0 * tiles * 8 + q * 16) : kOob;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (hp_lds_void*)dst, 16, off, 0, 0, 0);
    } else {  // W gamma / W beta + bias of columns 4 lane .. + 3
      const int c = lane * 4, sl = c >> 4;
      const uint32_t off = c < NSUB * 16 ? (uint32_t)((sub_of(sl) * 16 + (c & 15)) * 4) : kOob;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(i == is ? rg : rb, (hp_lds_void*)dst, 16, off, 0, 0, 0);
    }
  }
}

// LayerNorm statistics (mean, den) of local row `r` from its tile statistics
// in LDS: the 16 lanes of a 16-lane group (part = lane & 15) merge tiles
// part, part + 16, ... exactly as the decode-step kernel (lnf_merge_tiles);
// every lane of the group gets the result.
template <int ROWS, int NSUB>
__device__ __forceinline__ void hp_row_stats(const HeadProj& p, const uint8_t* lds, int r, int lane, float& mean,
                                             float& den) {
  const int tiles = p.K / 16, part = lane & 15;
  const float* st = reinterpret_cast<const float*>(lds + hp_s_off(ROWS, NSUB, p.ku)) + (size_t)r * tiles * 2;
  wq4::floatx2 v[kHpLnPer];
#pragma unroll
  for (int u = 0; u < kHpLnPer; ++u) {
    const int j = part + 16 * u;
    v[u] = j < tiles ? wq4::floatx2{st[2 * j], st[2 * j + 1]} : wq4::floatx2{0.0f, 0.0f};
  }
  wq4::lnf_merge_tiles<kHpLnPer>(v, part, tiles, mean, den);
}

// Compute: wave `wave` of `nwaves` (VPW = kHpVW / nwaves virtual waves per
// wave) runs virtual waves wave + nwaves * v; each takes blocks [vw kb / 8,
// (vw + 1) kb / 8) of every subtile (the decode-step kernel's split at K <=
// 1280).  acc[v][s]: the 16x16 output tile (lane l: rows 4 (l >> 4) + j,
// column l & 15).  The pieces must have landed (caller: counted vmcnt +
// barrier after hp_issue).
template <int ROWS, int NSUB, int VPW>
__device__ __forceinline__ void hp_compute(const HeadProj& p, const uint8_t* lds, int wave, int nwaves, int lane,
                                           wq4::floatx4 (&acc)[VPW][NSUB]) {
  const int ku = p.ku, kb = ku * 4;
  const uint8_t* wl = lds;
  const uint8_t* dl = lds + (size_t)hp_pad64(hp_w_pieces(NSUB, ku)) * 16;
  const uint8_t* al = lds + hp_a_off(NSUB, ku);
  const int r = lane & 15, g = lane >> 4;
#pragma unroll
  for (int v = 0; v < VPW; ++v) {
    const int vw = wave + nwaves * v;
    const int b0 = (vw * kb) / kHpVW, b1 = ((vw + 1) * kb) / kHpVW;
#pragma unroll
    for (int s = 0; s < NSUB; ++s) acc[v][s] = wq4::floatx4{0.f, 0.f, 0.f, 0.f};
    // unit by unit (4 blocks): one conflict-free ds_read_b128 of the lane's
    // nibble words and one ds_read_b64 of its column's scales per subtile
    for (int u = b0 >> 2; u * 4 < b1; ++u) {
      wq4::u32x4 wv[NSUB];
      wq4::u32x2 dv[NSUB];
#pragma unroll
      for (int s = 0; s < NSUB; ++s) {
        wv[s] = *reinterpret_cast<const wq4::u32x4*>(wl + ((size_t)(s * ku + u) * 64 + lane) * 16);
        dv[s] = *reinterpret_cast<const wq4::u32x2*>(dl + ((size_t)(s * ku + u) * 16 + (lane & 15)) * 8);
      }
      const int bs = max(b0, 4 * u), be = min(b1, 4 * u + 4);
      for (int b = bs; b < be; ++b) {
        // A fragments: lane (r, g) = row r of the MFMA tile, k = 32 b + 8 g ..;
        // with ROWS == 1 only row 0 is real, the other rows are zero
        wq4::half8 a[2];
#pragma unroll
        for (int pl = 0; pl < 2; ++pl) {
          const int piece = ((((b * 2 + (g >> 1)) * 2 + pl) * 2 + (g & 1)) * ROWS) + (ROWS == 1 ? 0 : r);
          const wq4::half8 x = *reinterpret_cast<const wq4::half8*>(al + (size_t)piece * 16);
          a[pl] = (ROWS == 1 && r != 0) ? wq4::half8{} : x;
        }
        const int bi = b & 3;
#pragma unroll
        for (int s = 0; s < NSUB; ++s) {
          const uint32_t w = bi == 0 ? wv[s][0] : bi == 1 ? wv[s][1] : bi == 2 ? wv[s][2] : wv[s][3];
          const uint32_t dw = (bi >> 1) ? dv[s][1] : dv[s][0];
          const float d = (float)__builtin_bit_cast(_Float16, (uint16_t)((bi & 1) ? (dw >> 16) : (dw & 0xffffu)));
          const wq4::half8 q = wq4::deq8(w);  // exact q - 8
          wq4::floatx4 tmp = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], q, wq4::floatx4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          tmp = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[1], q, tmp, 0, 0, 0);
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[v][s][j] = fmaf(tmp[j], d, acc[v][s][j]);
        }
      }
    }
  }
}

// The partials to red (ROWS == 16: call after a barrier that follows every
// wave's hp_compute -- red overwrites W / D / A).
template <int ROWS, int NSUB, int VPW>
__device__ __forceinline__ void hp_store_red(const HeadProj& p, uint8_t* lds, int wave, int nwaves, int lane,
                                             const wq4::floatx4 (&acc)[VPW][NSUB]) {
  float* red = reinterpret_cast<float*>(lds + hp_red_off(ROWS, NSUB, p.ku));
#pragma unroll
  for (int v = 0; v < VPW; ++v) {
    const int vw = wave + nwaves * v;
#pragma unroll
    for (int s = 0; s < NSUB; ++s) {
      if constexpr (ROWS == 1) {
        if (lane < 16) red[(vw * NSUB + s) * 16 + lane] = acc[v][s][0];  // row 0 = element 0 of lanes 0 .. 15
      } else {
        *reinterpret_cast<wq4::floatx4*>(&red[((vw * NSUB + s) * 64 + lane) * 4]) = acc[v][s];
      }
    }
  }
}

// Output (local row rr, column c < 16 NSUB): the virtual waves' partials in
// wave order, the activation scale, the LayerNorm-fold correction and the
// bias -- skinny_gemm_kernel's epilogue for a consumer with bias (y = a + b2).
template <int ROWS, int NSUB>
__device__ __forceinline__ float hp_finish(const HeadProj& p, const uint8_t* lds, int rr, int c, float mean, float den) {
  const float* red = reinterpret_cast<const float*>(lds + hp_red_off(ROWS, NSUB, p.ku));
  const float* gb = reinterpret_cast<const float*>(lds + hp_g_off(ROWS, NSUB, p.ku));
  const int idx = ROWS == 1 ? c : (((c >> 4) * 64 + (c & 15) + 16 * (rr >> 2)) * 4 + (rr & 3));
  constexpr int stride = ROWS == 1 ? NSUB * 16 : NSUB * 256;
  float v = red[idx];
#pragma unroll
  for (int w = 1; w < kHpVW; ++w) v = v + red[w * stride + idx];
  const float a = wq4::lnf_apply(v * wq4::kActScaleInv, mean, gb[c], den);
  return a + gb[256 + c];
}

}  // namespace wa
