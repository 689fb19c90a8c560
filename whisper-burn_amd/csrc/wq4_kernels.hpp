// wq4_kernels.hpp -- host-visible launchers of the Q4 GEMM kernels.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include "wq4_epi.hpp"
#include "wq4_layout.hpp"

namespace wq4 {

// LayerNorm (layers.rs:12-32) of M rows of D: A-tiled f16 split operand
// (tiled != null, ns = 1 or 2) or f32 rows (out).
hipError_t launch_layernorm(const float* x, const float* w, const float* b, int M, int D, _Float16* tiled, int ns,
                            float* out, hipStream_t st);

// f32 [M, ld] row-major -> A-tiled f16 split (ns = 1 or 2).
// scale: device [2] = {s, 1/s} written by launch_act_scale (x is tiled as x * s),
// or nullptr: the fixed kActScale.
hipError_t launch_tile_activations(const float* x, _Float16* at, int M, int K, int ld, int ns, hipStream_t st,
                                   const float* scale = nullptr);
// Per-call activation scale for the f32 entry points: s = the power of two
// min(2^4, 2^floor(log2(16384 / max|x|))) keeps every hi half finite (|x s| <
// 2^15) and the lo halves of the largest values normal; out[0] = s,
// out[1] = 1 / s.
hipError_t launch_act_scale(const float* x, int M, int K, int ld, float* out, hipStream_t st);

// Split-K workspace of the decode kernel, one per (device, stream): partial
// tiles and per-n-tile arrival counters (zeroed once, re-armed by the kernel).
constexpr int64_t kDecodeWsFloats = (int64_t)4 << 20;  // 16 MiB of partials
constexpr int64_t kDecodeMaxTiles = 1 << 16;            // counters
constexpr int kDecodeMaxPer = 4;                        // block pairs per wave (4-wave split-K)
constexpr int kDecodeMaxPer8 = 3;                       // block pairs per wave (8-wave, whole K)
constexpr int kDecodeMaxMTiles = 4;                     // rows <= 128 (launches of 2 m-tiles)
struct DecodeWs {
  float* part;
  int* counters;
  float* act_scale;  // [2]: the f32 entry points' per-call activation scale (launch_act_scale)
};
struct DecodePlan {
  int per;    // kernel instance: max block pairs per wave
  int ks;     // workgroups (K slices) per n-tile
  int chunk;  // block pairs per wave (<= per)
  int w;      // waves per workgroup (4: split-K, 8: whole K per workgroup)
};
DecodePlan plan_decode(int64_t ntiles, int64_t nbp, int mreal);

// y = epi((A W^T) * colscale).  epi_mode: 0 = f32 row-major, 1 = A-tiled f16
// operand of a following GEMM.  ws != null selects the split-K decode kernel
// (rows <= 128; larger row counts or unsupported shapes use the tile kernel).
// wtype: kWeightsQ4 (nib/sc/colscale of wq4_layout.hpp) or kWeightsF16
// (nib = repack_f16 fragments, sc unused, colscale = 1).
constexpr int kWeightsQ4 = 0, kWeightsF16 = 1;
// Whether launch_q4_gemm can build the A operand by LayerNorm-on-load
// (EpiArgs::lnx) for this weight and row count: 8-wave decode plans.
bool decode_ln_supported(const Q4Geom& g, int rows);
hipError_t launch_q4_gemm(const Q4Geom& g, const uint8_t* nib, const uint32_t* sc, const float* colscale,
                          const _Float16* at, int rows, const EpiArgs& e, int epi_mode, int ns, const DecodeWs* ws,
                          hipStream_t st, int wtype);

}  // namespace wq4
