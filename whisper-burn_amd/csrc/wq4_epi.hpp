// wq4_epi.hpp -- epilogue description shared by host launchers and kernels.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace wq4 {

struct EpiArgs {
  const float* bias;      // [N] or nullptr                    (linear.rs:36-38)
  const float* residual;  // [M][ldo] f32 or nullptr (may == out)
  float* out;             // f32 row-major [M][ldo]
  _Float16* out_tiled;    // A-tiled operand of the next GEMM (K' = N)
  int ldo;                // row stride of out / residual
  int nbp_next;           // block pairs of the next GEMM's K (ceil(N/64))
  int gelu;               // tanh-GELU after bias (layers.rs:35-41)
  int m;                  // real rows
  int n;                  // real cols
  int hm_t;               // > 0: head-major f32 output, rows grouped by hm_t (see out_index)
  int hm_d;               //      columns per part (K | V), heads of 64
  // LayerNorm-on-load (decode kernel, LNA variants): the A operand is
  // LayerNorm(lnx rows; lng, lnb) (layers.rs:12-32) built in registers instead
  // of read from a pre-tiled operand.  lnx: [M][lnd] f32.
  const float* lnx;
  const float* lng;
  const float* lnb;
  int lnd;
  // LayerNorm folded into the GEMMs around it (decode-step kernel, or the
  // decode kernel's 8-wave plans; wq4_gemm_tiled_lnfold).  Producer (a
  // residual GEMM whose output x feeds LayerNorm(x; gamma, beta)): also
  // writes the A-tiled operand of x * gamma (lnf_at, K' = N, lnf_nbp block
  // pairs) and per (row, 16-column tile) the tile mean and sum of squared
  // deviations (lnf_stats_out [M][N/16][2]).
  // Consumer (a GEMM on LayerNorm(x)): A = tiled(x * gamma); merges the
  // lnf_tiles tile statistics of each row (exact equal-count merge of
  // 16-value tiles, wq4_lnmath.hpp lnf_merge_tiles) and applies
  // out = (acc - mean * lnf_wg[n]) / sqrt(var + 1e-5) + bias[n] before the
  // rest of the epilogue (bias = W beta + linear bias, lnf_wg = W gamma).
  const float* lnf_g;
  _Float16* lnf_at;
  float* lnf_stats_out;
  int lnf_nbp;
  const float* lnf_stats_in;
  const float* lnf_wg;
  int lnf_tiles;
  // Inverse scale of the A operand (device scalar) when the operand was tiled
  // with a per-call scale (wq4_matmul / linear / ffn entry points: wide
  // activation range); nullptr = the fixed kActScale of every internal
  // producer (wq4_device.hpp split_act).
  const float* act_inv;
  // timing diagnostics (WQ4_STAMP builds only): the decode kernel's launch slot
  int stamp_id;
};

// Output element index.  Row-major by default; head-major (hm_t > 0) writes
// out[part][g][head][t][64] for row = g * hm_t + t, col = part * hm_d +
// head * 64 + d -- the [B, H, T, 64] K/V view the attention reads
// (reference: src/model/attention.rs:254-263, reshape + swap_dims of k, v).
#if defined(__HIPCC__)
__host__ __device__
#endif
inline size_t out_index(const EpiArgs& e, int row, int col) {
  if (e.hm_t <= 0) return (size_t)row * e.ldo + col;
  const int g = row / e.hm_t, t = row - g * e.hm_t;
  const int part = col / e.hm_d, c = col - part * e.hm_d;
  return (size_t)part * e.m * e.hm_d + (((size_t)g * (e.hm_d >> 6) + (c >> 6)) * e.hm_t + t) * 64 + (c & 63);
}

enum EpiMode { kEpiF32 = 0, kEpiTiled = 1, kEpiHeadMajor = 2 };  // head-major: f32 via out_index

}  // namespace wq4
