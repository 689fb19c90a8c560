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
  float* act_scale;  // [8]: the f32 entry points' per-call operand scales, two {s, 1/s, max bits} slots (launch_act_scale)
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

// The encoder-size GEMM ring kernel (wq4_enc.hip): Q4_0 weights, f16x2
// operands, f32 or A-tiled outputs, rows > 128 -- bit-identical to the
// prefill tile kernel's results.  enc_gemm_pick: 0 = use the tile kernel,
// else the geometry (2 = L, 3 = S) to pass to launch_enc_gemm, or 5 = the
// wide kernel (launch_wide_gemm).
int enc_gemm_pick(const Q4Geom& g, int rows, int epi_mode, int ns, int wtype);
hipError_t launch_enc_gemm(const Q4Geom& g, const uint8_t* nib, const uint32_t* sc, const float* cs,
                           const _Float16* at, int rows, const EpiArgs& e, int epi_mode, int geo, hipStream_t st);
// The 8-wave wide kernel (wq4_wide.hip, enc_gemm_pick geometry 5): Q4_0
// weights, rows > 128, NS = 1 or 2 -- bit-identical to the tile kernel.
bool wide_gemm_supported(const Q4Geom& g, int rows, int ns, int wtype);
hipError_t launch_wide_gemm(const Q4Geom& g, const uint8_t* nib, const uint32_t* sc, const float* cs,
                            const _Float16* at, int rows, const EpiArgs& e, int epi_mode, int ns, hipStream_t st);

// The decode-step GEMM (wq4_skinny.hip): rows <= 32, 16-column workgroups on
// 16x16x32 MFMAs, one Q4 block per MFMA with the scale applied per block in
// f32.  Its own weight layout (q16 / d16, or f16s for f16 weights) is built
// at upload next to the prefill kernel's.  LayerNorm-fold statistics are per
// 16-column tile (EpiArgs::lnf_tiles = K / 16), K <= 1280 for a consumer.
inline int64_t skinny_units(const Q4Geom& g) { return (g.kb + 3) / 4; }
inline size_t skinny_q_bytes(const Q4Geom& g) { return (size_t)(g.np / 16) * skinny_units(g) * 1024; }
inline size_t skinny_d_bytes(const Q4Geom& g) { return (size_t)(g.np / 16) * skinny_units(g) * 128; }
inline size_t skinny_f16_bytes(const Q4Geom& g) { return (size_t)(g.np / 16) * g.kb * 1024; }
void repack_q4_skinny(const uint8_t* raw, const Q4Geom& g, uint32_t* q16, uint16_t* d16);
void repack_f16_skinny(const uint16_t* w, const Q4Geom& g, uint16_t* f16s);
bool skinny_supported(const Q4Geom& g, int rows);
constexpr int kSkinnyMaxLnTiles = 80;  // LayerNorm-fold consumer: K / 16 tile statistics per row
// ws: the stream's split-K workspace (partials + arrival counters) for the
// K splits of large K (fc2).
hipError_t launch_skinny_gemm(const Q4Geom& g, const uint32_t* wq, const uint16_t* wd, const _Float16* at, int rows,
                              const EpiArgs& e, int epi_mode, int ns, int wtype, const DecodeWs* ws, hipStream_t st);

}  // namespace wq4
