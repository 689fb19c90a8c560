// wq4_kernels.hpp -- host-visible launchers of the Q4 GEMM kernels.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include "wq4_epi.hpp"
#include "wq4_layout.hpp"

namespace wq4 {

// f32 [M, ld] row-major -> A-tiled f16 split (ns = 1 or 2).
hipError_t launch_tile_activations(const float* x, _Float16* at, int M, int K, int ld, int ns, hipStream_t st);

// y = epi((A W^T) * colscale).  epi_mode: 0 = f32 row-major, 1 = A-tiled f16
// operand of a following GEMM.  decode selects the K-split kernel.
hipError_t launch_q4_gemm(const Q4Geom& g, const uint8_t* nib, const uint32_t* sc, const float* colscale,
                          const _Float16* at, int rows, const EpiArgs& e, int epi_mode, int ns, bool decode,
                          hipStream_t st);

}  // namespace wq4
