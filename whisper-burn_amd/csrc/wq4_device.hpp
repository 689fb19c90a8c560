// wq4_device.hpp -- CDNA4 (gfx950) device helpers for the Q4_0 GEMM path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wq4_epi.hpp"

namespace wq4 {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef float floatx2 __attribute__((ext_vector_type(2)));

// tanh-approximate GELU, src/model/layers.rs:35-41:
//   x * 0.5 * (tanh(u) + 1),  u = sqrt(2/pi) * (x + 0.044715 x^3),
// evaluated as the identical x / (1 + exp(-2u)) = x / (1 + 2^t),
// t = x * (c0 + c1 x^2): one v_exp_f32 and one v_rcp_f32 (~8 VALU) instead
// of the ~36 of tanhf -- at fc1's 246 M outputs per encoder layer that was
// the A-tiled epilogue's largest cost.  No cancellation where tanh(u) -> -1
// (the f32 tanh form loses its relative precision there); u -> -inf gives
// 2^t = inf, x * 0 = -0; u -> +inf gives x; NaN stays NaN.
__device__ __forceinline__ float gelu_tanh(float x) {
  constexpr float c0 = -2.0f * 0.7978845608028654f * 1.4426950408889634f;  // -2 sqrt(2/pi) log2(e)
  constexpr float c1 = c0 * 0.044715f;
  const float t = x * __builtin_fmaf(x * x, c1, c0);
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(t));
}

__device__ __forceinline__ float epi_value(float acc, int row, int col, const EpiArgs& e) {
  float v = acc;
  if (e.bias) v = v + e.bias[col];
  if (e.gelu) v = gelu_tanh(v);
  if (e.residual) v = e.residual[(size_t)row * e.ldo + col] + v;
  return v;
}

// epi_value with bias[col] / residual[row][col] already loaded (same
// arithmetic, same order).
__device__ __forceinline__ float epi_value_pre(float acc, float bias, float res, const EpiArgs& e) {
  float v = acc;
  if (e.bias) v = v + bias;
  if (e.gelu) v = gelu_tanh(v);
  if (e.residual) v = res + v;
  return v;
}

// f32 epilogue of one 32 x 32 accumulator tile (this lane: column col,
// element i at row row_of(i), stored at out[idx(row, col)]): the bias and
// all 16 residuals are loaded before the first store.  Element by element
// (epi_value) the compiler cannot move a residual load above the previous
// element's store -- y may alias residual (in-place residual adds) -- so the
// tile paid 16 dependent memory round trips; this way it pays one.  Same
// arithmetic as epi_value: the same bits.
// DRAIN: one vmcnt(0) after the loads, before the first store -- without it
// hipcc re-waits (vmcnt(0), behind every earlier store) at the top of each
// exec-masked store, i.e. per element (the encoder ring kernel's epilogue).
template <bool DRAIN = false, class RowOf, class Idx>
__device__ __forceinline__ void epi_store_tile(const floatx16& acc, float cs, int col, RowOf row_of, Idx idx,
                                               const EpiArgs& e) {
  const bool cok = col < e.n;
  const float b = (e.bias && cok) ? e.bias[col] : 0.0f;
  float res[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = row_of(i);
    res[i] = (e.residual && cok && row < e.m) ? e.residual[(size_t)row * e.ldo + col] : 0.0f;
  }
  if constexpr (DRAIN) __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = row_of(i);
    if (cok && row < e.m) e.out[idx(row, col)] = epi_value_pre(acc[i] * cs, b, res[i], e);
  }
}

// One repacked u32 (8 nibbles, see wq4_layout.hpp) -> 8 exact f16 (q - 8),
// element order j = 0..7:
//   (w & 0x000F000F) | 0x64006400 = f16 pair (1024 + q_a, 1024 + q_b)
//   (w & 0x00F000F0) | 0x64006400 = f16 pair (1024 + 16 q_a, ...)
// then -1032 resp. *(1/16) - 72; every step is exact in f16.
__device__ __forceinline__ half8 deq8(uint32_t w) {
  const uint32_t C = 0x64006400u;
  const uint32_t w8 = w >> 8;
  const uint32_t p0 = (w & 0x000F000Fu) | C;
  const uint32_t p1 = (w & 0x00F000F0u) | C;
  const uint32_t p2 = (w8 & 0x000F000Fu) | C;
  const uint32_t p3 = (w8 & 0x00F000F0u) | C;
  const half2v off1 = {(_Float16)1032.0f, (_Float16)1032.0f};
  const half2v inv16 = {(_Float16)0.0625f, (_Float16)0.0625f};
  const half2v off16 = {(_Float16)72.0f, (_Float16)72.0f};
  half2v h0 = __builtin_bit_cast(half2v, p0) - off1;
  half2v h1 = __builtin_bit_cast(half2v, p1) * inv16 - off16;
  half2v h2 = __builtin_bit_cast(half2v, p2) - off1;
  half2v h3 = __builtin_bit_cast(half2v, p3) * inv16 - off16;
  half8 r;
  r[0] = h0[0]; r[1] = h0[1];
  r[2] = h1[0]; r[3] = h1[1];
  r[4] = h2[0]; r[5] = h2[1];
  r[6] = h3[0]; r[7] = h3[1];
  return r;
}

// MFMA B operand for one k-half: B = (q - 8) * d' as the exact f16 pair
// hi = RN(B), lo = B - hi (the fma is exact: B has <= 14 significant bits).
template <int NB>
__device__ __forceinline__ void deq_scaled(uint32_t w, uint32_t dbits, half8& hi, half8& lo) {
  const half8 q = deq8(w);
  const _Float16 d = __builtin_bit_cast(_Float16, (uint16_t)dbits);
  const half8 dv = {d, d, d, d, d, d, d, d};
  hi = q * dv;
  if constexpr (NB == 2) lo = __builtin_elementwise_fma(q, dv, -hi);
}

__device__ __forceinline__ floatx16 mfma32(const half8& a, const half8& b, const floatx16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// f32 -> (hi, lo) f16 split; hi = RNE(x), lo = RNE(x - hi).  x - hi is exact.
__device__ __forceinline__ void split_f16(float x, _Float16& hi, _Float16& lo) {
  hi = (_Float16)x;
  lo = (_Float16)(x - (float)hi);
}

// The MFMAs flush f16 subnormal inputs (measured on gfx950 with denormals
// enabled in the kernel descriptor: scripts/attn_precision_probe.py), so the
// lo half of a pair is lost once |lo| < 2^-14 -- for an unscaled N(0, 1)
// operand that is most elements below 4.  Every split operand is therefore
// scaled by a power of two that keeps lo normal over its range, and the
// product's scale is undone in f32 (exact).  GEMM A operands (activations,
// the A-tiled layout): x * 2^4, |x| < 4094; undone through the column scale.
constexpr float kActScale = 16.0f, kActScaleInv = 1.0f / 16.0f;
__device__ __forceinline__ void split_act(float x, _Float16& hi, _Float16& lo) { split_f16(x * kActScale, hi, lo); }

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming
// §5 T1): blocks L, L+8, L+16, ... (one XCD under round-robin dispatch) get
// consecutive logical ids, so neighbouring tiles share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int L, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = L % 8, idx = L / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// DPP lane read inside a row of 16 lanes -- a VALU operand modifier, no LDS
// round trip as with ds_bpermute (__shfl_xor).  CTRL: 0xB1 quad_perm
// [1,0,3,2] (lane ^ 1), 0x4E quad_perm [2,3,0,1] (lane ^ 2), 0x141
// row_half_mirror (lane 7 - i of its 8), 0x140 row_mirror (lane 15 - i).
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xf, 0xf, false));
}

// Butterfly sum / max over each aligned 16-lane group, result in every lane.
// Bit-identical to the __shfl_xor butterfly over offsets 1, 2, 4, 8: after
// the lane^1 and lane^2 steps a quad holds one value, so the half-mirror
// partner (another quad of the 8) carries exactly what lane^4 would; after
// that an 8-lane group holds one value and the mirror stands in for lane^8.
__device__ __forceinline__ float sum16(float v) {
  v += dpp_f32<0xB1>(v);
  v += dpp_f32<0x4E>(v);
  v += dpp_f32<0x141>(v);
  v += dpp_f32<0x140>(v);
  return v;
}
__device__ __forceinline__ float max16(float v) {
  v = fmaxf(v, dpp_f32<0xB1>(v));
  v = fmaxf(v, dpp_f32<0x4E>(v));
  v = fmaxf(v, dpp_f32<0x141>(v));
  v = fmaxf(v, dpp_f32<0x140>(v));
  return v;
}

// Async 16-B-per-lane global -> LDS copy (global_load_lds_dwordx4): lane l's
// 16 bytes land at lds_base + 16 * l (lds_base wave-uniform).
__device__ __forceinline__ void glds16(const void* gsrc, void* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc,
                                   (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

}  // namespace wq4
