// wa_headproj.hpp -- a LayerNorm-folded Q4_0 projection of ONE activation row
// formed inside an attention launch (few-clip decode steps).
//
// A decode step of a few clips is a chain of short launches;
// where an attention workgroup owns whole heads it can form the head's
// projection itself instead of waiting for a GEMM launch:
//   * the fused decoder self-attention (q, k, v of its head: 12 subtiles of
//     16 columns; decoder.rs:77-112, attention.rs:93-125),
//   * the K / V cross-attention (q of its head: 4 subtiles; attention.rs:
//     208-236).
// The arithmetic is that of the decode-step GEMM (wq4_skinny.hip,
// skinny_gemm_kernel) as a LayerNorm-fold consumer (wq4_gemm_tiled_lnfold),
// bit for bit: per Q4 block t = MFMA(x_hi, q-8) + MFMA(x_lo, q-8) on
// v_mfma_f32_16x16x32_f16, acc = fma(t, d, acc); 8 (virtual) waves take the
// blocks [w kb/8, (w+1) kb/8) and are summed in wave order; then
//   y = ((sum * 2^-4) - mean * (W gamma)[n]) / sqrt(var + 1e-5) + (W beta + b)[n]
// with (mean, var) merged from the producer's 16-column tile statistics
// (lnf_merge_tiles).  So a fused launch produces exactly the values the
// GEMM launch it replaces would (tests/test_fused_decode_gpu.py compares the
// two paths bit for bit under kernel policy 3).
//
// Memory: the weights of the projection's subtiles (decode-step layout: 1 KiB
// of nibbles per (subtile, 4 blocks), 128 B of scales) and the row's A-tiled
// fragments are brought into LDS by LDS-DMA (buffer_load ... lds: no
// registers, every piece in flight at once) while the caller's own loads
// (the first K / V pass) stay in flight behind them (counted vmcnt).
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
// pieces (1 KiB): [weights: s, u, lane][scales: s, u, 8][A: block, kk,
// plane, half], each region padded to whole instructions, then three 1-KiB
// aux slots (the row's tile statistics, the
// NSUB * 16 columns' W gamma, their W beta + bias), then the partial sums
// red[8 virtual waves][NSUB][16] f32.
__host__ __device__ constexpr int hp_w_pieces(int nsub, int ku) { return nsub * ku * 64; }
__host__ __device__ constexpr int hp_d_pieces(int nsub, int ku) { return nsub * ku * 8; }
__host__ __device__ constexpr int hp_a_pieces(int ku) { return ku * 4 * 8; }  // kb blocks x (kk, plane, half)
__host__ __device__ constexpr int hp_pad64(int n) { return (n + 63) / 64 * 64; }
__host__ __device__ constexpr int hp_main_instr(int nsub, int ku) {
  return (hp_pad64(hp_w_pieces(nsub, ku)) + hp_pad64(hp_d_pieces(nsub, ku)) + hp_pad64(hp_a_pieces(ku))) / 64;
}
__host__ __device__ constexpr int hp_aux_off(int nsub, int ku) { return hp_main_instr(nsub, ku) * 1024; }
__host__ __device__ constexpr int hp_red_off(int nsub, int ku) { return hp_aux_off(nsub, ku) + 3 * 1024; }
__host__ __device__ constexpr int hp_lds_bytes(int nsub, int ku) { return hp_red_off(nsub, ku) + kHpVW * nsub * 16 * 4; }
// Whether a projection of this K fits the scheme: the decode-step layout
// (K % 128 == 0), the statistics slot (K / 16 <= 80 tiles), the aux slots
// (<= 256 columns).
__host__ __device__ constexpr bool hp_supported(int nsub, int K) {
  return K % 128 == 0 && K >= 128 && K <= kHpMaxK && nsub * 16 <= 256;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t hp_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

// Issue every LDS-DMA instruction of the projection (NSUB subtiles, global
// subtile index sub_of(s), A-tiled row `row`), instructions i = wave, wave +
// nwaves, ...  Returns how many THIS wave issued (for a counted vmcnt).
// Pieces past a region read zeros.
template <int NSUB, class SubOf>
__device__ __forceinline__ int hp_issue(const HeadProj& p, SubOf sub_of, int row, uint8_t* lds, int wave, int nwaves,
                                        int lane) {
  const int ku = p.ku, kb = ku * 4, tiles = p.K / 16;
  const int nw = hp_w_pieces(NSUB, ku), nd = hp_d_pieces(NSUB, ku), na = hp_a_pieces(ku);
  const int nwp = hp_pad64(nw), ndp = hp_pad64(nd);
  const int nmain = hp_main_instr(NSUB, ku);
  const __amdgpu_buffer_rsrc_t rw = hp_rsrc(p.q16, 0x7FFFFFF0u);
  const __amdgpu_buffer_rsrc_t rd = hp_rsrc(p.d16, 0x7FFFFFF0u);
  const __amdgpu_buffer_rsrc_t ra = hp_rsrc(p.at, (uint32_t)kb * 4u * 1024u);  // m-tile 0, f16 pairs
  const __amdgpu_buffer_rsrc_t rs = hp_rsrc(p.stats, (uint32_t)(row + 1) * (uint32_t)tiles * 8u);
  const __amdgpu_buffer_rsrc_t rg = hp_rsrc(p.wg, 0x7FFFFFF0u);
  const __amdgpu_buffer_rsrc_t rb = hp_rsrc(p.b2, 0x7FFFFFF0u);
  int mine = 0;
  for (int i = wave; i < nmain + 3; i += nwaves) {
    void* dst = lds + (size_t)i * 1024;
    const int pc = i * 64 + lane;  // this lane's piece
    if (i >= nmain) {
      const int k = i - nmain;
      if (k == 0) {  // the row's (mean, M2) tile statistics: 2 tiles per piece
        const uint32_t off = lane * 2 < tiles ? (uint32_t)((row * tiles + lane * 2) * 8) : 0x7FFFFFF0u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (hp_lds_void*)dst, 16, off, 0, 0, 0);
      } else {  // W gamma / W beta + bias of columns 4 lane .. + 3
        const int c = lane * 4, sl = c >> 4;
        const uint32_t off = c < NSUB * 16 ? (uint32_t)((sub_of(sl) * 16 + (c & 15)) * 4) : 0x7FFFFFF0u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(k == 1 ? rg : rb, (hp_lds_void*)dst, 16, off, 0, 0, 0);
      }
    } else if (i * 64 < nwp) {
      const int s = pc / (ku * 64), within = pc - s * (ku * 64);
      const uint32_t off = pc < nw ? (uint32_t)(((size_t)sub_of(s) * ku * 64 + within) * 16) : 0x7FFFFFF0u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (hp_lds_void*)dst, 16, off, 0, 0, 0);
    } else if (i * 64 < nwp + ndp) {
      const int q = pc - nwp, s = q / (ku * 8), within = q - s * (ku * 8);
      const uint32_t off = q < nd ? (uint32_t)(((size_t)sub_of(s) * ku * 8 + within) * 16) : 0x7FFFFFF0u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rd, (hp_lds_void*)dst, 16, off, 0, 0, 0);
    } else {
      // A piece (block b, kk, plane pl, half h) of row `row`: A-tiled
      // fragment ((b * 2 + kk) * 2 + pl), lane' row + 32 h
      const int q = pc - nwp - ndp;
      const int b = q >> 3, kk = (q >> 2) & 1, pl = (q >> 1) & 1, h = q & 1;
      const uint32_t off = q < na ? (uint32_t)(((((b * 2 + kk) * 2 + pl) * 64) + row + 32 * h) * 16) : 0x7FFFFFF0u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (hp_lds_void*)dst, 16, off, 0, 0, 0);
    }
    ++mine;
  }
  return mine;
}

// The row's LayerNorm statistics (mean, den) from the producer's tile
// statistics in LDS: lanes 0 .. 15 of one wave (part = lane & 15) merge tiles
// part, part + 16, ... exactly as the decode-step kernel (lnf_merge_tiles);
// every lane of the wave returns the result of its 16-lane group (use lane < 16).
template <int NSUB>
__device__ __forceinline__ void hp_row_stats(const HeadProj& p, const uint8_t* lds, int lane, float& mean, float& den) {
  const float* st = reinterpret_cast<const float*>(lds + hp_aux_off(NSUB, p.ku));
  wq4::floatx2 v[kHpLnPer];
  const int part = lane & 15, tiles = p.K / 16;
#pragma unroll
  for (int u = 0; u < kHpLnPer; ++u) {
    const int j = part + 16 * u;
    v[u] = j < tiles ? wq4::floatx2{st[2 * j], st[2 * j + 1]} : wq4::floatx2{0.0f, 0.0f};
  }
  wq4::lnf_merge_tiles<kHpLnPer>(v, part, tiles, mean, den);
}

// Compute: wave `wave` of `nwaves` (nwaves divides kHpVW) runs virtual waves
// wave, wave + nwaves, ...; virtual wave vw takes blocks [vw kb / 8, (vw + 1)
// kb / 8) of every subtile (the decode-step kernel's split at K <= 1280) and
// leaves row 0's 16 columns per subtile in red[vw][s][16].  The pieces must
// have landed (caller: counted vmcnt + barrier after hp_issue).
template <int NSUB>
__device__ __forceinline__ void hp_compute(const HeadProj& p, uint8_t* lds, int wave, int nwaves, int lane) {
  const int ku = p.ku, kb = ku * 4;
  const int nwp = hp_pad64(hp_w_pieces(NSUB, ku)), ndp = hp_pad64(hp_d_pieces(NSUB, ku));
  const uint32_t* wl = reinterpret_cast<const uint32_t*>(lds);
  const uint16_t* dl = reinterpret_cast<const uint16_t*>(lds + (size_t)nwp * 16);
  const uint8_t* al = lds + (size_t)(nwp + ndp) * 16;
  float* red = reinterpret_cast<float*>(lds + hp_red_off(NSUB, ku));
  const int r = lane & 15, g = lane >> 4;
  for (int vw = wave; vw < kHpVW; vw += nwaves) {
    const int b0 = (vw * kb) / kHpVW, b1 = ((vw + 1) * kb) / kHpVW;
    wq4::floatx4 acc[NSUB];
#pragma unroll
    for (int s = 0; s < NSUB; ++s) acc[s] = wq4::floatx4{0.f, 0.f, 0.f, 0.f};
    for (int b = b0; b < b1; ++b) {
      // A fragments: lane (r, g) = row r of the MFMA tile, k = 32 b + 8 g ..;
      // only row 0 is real, the other rows are zero
      wq4::half8 a[2];
#pragma unroll
      for (int pl = 0; pl < 2; ++pl) {
        const wq4::half8 v =
            *reinterpret_cast<const wq4::half8*>(al + (size_t)(((b * 2 + (g >> 1)) * 2 + pl) * 2 + (g & 1)) * 16);
        a[pl] = r == 0 ? v : wq4::half8{};
      }
#pragma unroll
      for (int s = 0; s < NSUB; ++s) {
        const uint32_t w = wl[((s * ku + (b >> 2)) * 64 + lane) * 4 + (b & 3)];
        const float d = (float)__builtin_bit_cast(_Float16, dl[((s * ku + (b >> 2)) * 16 + (lane & 15)) * 4 + (b & 3)]);
        const wq4::half8 q = wq4::deq8(w);  // exact q - 8
        wq4::floatx4 tmp = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], q, wq4::floatx4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        tmp = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[1], q, tmp, 0, 0, 0);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[s][j] = fmaf(tmp[j], d, acc[s][j]);
      }
    }
    if (lane < 16) {  // row 0 = element 0 of lanes 0 .. 15 (column = lane)
#pragma unroll
      for (int s = 0; s < NSUB; ++s) red[(vw * NSUB + s) * 16 + lane] = acc[s][0];
    }
  }
}

// Output column c (< 16 NSUB): the virtual waves' partials in wave order,
// the activation scale, the LayerNorm-fold correction and the bias --
// skinny_gemm_kernel's epilogue for a consumer with bias (y = a + b2).
template <int NSUB>
__device__ __forceinline__ float hp_finish(const HeadProj& p, const uint8_t* lds, int c, float mean, float den) {
  const float* red = reinterpret_cast<const float*>(lds + hp_red_off(NSUB, p.ku));
  const float* aux = reinterpret_cast<const float*>(lds + hp_aux_off(NSUB, p.ku));
  float v = red[c];
#pragma unroll
  for (int w = 1; w < kHpVW; ++w) v = v + red[w * NSUB * 16 + c];
  float a = v * wq4::kActScaleInv;
  a = (a - mean * aux[256 + c]) / den;
  return a + aux[512 + c];
}

}  // namespace wa
