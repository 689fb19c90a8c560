// wq4_epi.hpp -- epilogue description shared by host launchers and kernels.
#pragma once
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
};

enum EpiMode { kEpiF32 = 0, kEpiTiled = 1 };

}  // namespace wq4
