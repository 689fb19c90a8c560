// wq4_q4gemm.hip -- MI355X (gfx950) kernels of the fused Q4_0 dequant + GEMM.
//
// Replaces the reference's single WGSL shader (src/gguf/shader.wgsl:51-92,
// one thread per output, scalar f32 FMA, 18 dependent u32 loads per block)
// with MFMA kernels over the repacked weights and A-tiled activations of
// wq4_layout.hpp:
//
//  q4_gemm_prefill  M >= ~64 rows (encoder, cross-K/V): 128 x 256 workgroup
//                   tile, 4 waves x (128 x 64), A streamed into a double-
//                   buffered LDS ring by global_load_lds (lane-linear images,
//                   conflict-free ds_read_b128), B (weights) straight to VGPRs
//                   as one 1 KiB coalesced load per (n-tile, block pair).
//  q4_gemm_decode   M <= ~64 rows (decoder tokens, prompt): one 32-column
//                   n-tile per workgroup, the K range split over 4 waves and
//                   reduced through LDS in a fixed order; A rows beyond M are
//                   never loaded.
//
// Arithmetic (both kernels, every output):  with x = x_hi + x_lo (f16 pair)
// and the exact weight B = (q - 8) * d' = B_hi + B_lo (f16 pair, d' the
// row-prescaled f16 scale, wq4_layout.hpp),
//   acc += MFMA(x_hi, B_hi) + MFMA(x_lo, B_hi) + MFMA(x_hi, B_lo)
// per 16-k half, in k order, f32 accumulation, then y = acc * 2^-s_n.  The
// dropped x_lo * B_lo term is < 2^-22 relative.  WQ4_PREC_F16 keeps only
// MFMA(x_hi, B_hi).  Per-row instruction order depends on (N, K) only, never
// on M or the tile position: a row's result is identical at batch 1 and 256.
#include <hip/hip_runtime.h>

#include "wq4_device.hpp"
#include "wq4_kernels.hpp"

namespace wq4 {

// ------------------------------------------------------------------------
// f32 row-major [M, K] -> A-tiled f16 (hi[, lo]) operand.  One thread per
// (m-tile, block, kk, lane) = 8 elements.
// ------------------------------------------------------------------------
template <int NS, bool ALIGNED>
__global__ __launch_bounds__(256) void tile_activations_kernel(const float* __restrict__ x,
                                                               _Float16* __restrict__ at, int M, int K,
                                                               int ld, int mtiles, int kbp) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)mtiles * kbp * 2 * 64;
  if (idx >= total) return;
  const int lane = (int)(idx & 63);
  int64_t rest = idx >> 6;
  const int kk = (int)(rest & 1);
  rest >>= 1;
  const int b = (int)(rest % kbp);
  const int mt = (int)(rest / kbp);
  const int r = lane & 31, h = lane >> 5;
  const int m = mt * 32 + r;
  const int k0 = b * 32 + kk * 16 + h * 8;
  float v[8];
  if (m < M && k0 < K) {
    if constexpr (ALIGNED) {
      const floatx4* src = reinterpret_cast<const floatx4*>(x + (size_t)m * ld + k0);
      const floatx4 a = src[0], c = src[1];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = a[j];
        v[4 + j] = c[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = x[(size_t)m * ld + k0 + j];
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.0f;
  }
  half8 hi, lo;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    _Float16 a, c;
    split_f16(v[j], a, c);
    hi[j] = a;
    lo[j] = c;
  }
  const size_t frag = (((size_t)mt * kbp + b) * 2 + kk) * NS;
  half8* dst = reinterpret_cast<half8*>(at);
  dst[(frag + 0) * 64 + lane] = hi;
  if constexpr (NS == 2) dst[(frag + 1) * 64 + lane] = lo;
}

// ------------------------------------------------------------------------
// Epilogue helpers.
// ------------------------------------------------------------------------
constexpr int kStageLd = 68;  // padded f32 row stride of the transpose stage

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
        split_f16(a[j], x, y);
        hi[j] = x;
        lo[j] = y;
        split_f16(c[j], x, y);
        hi[4 + j] = x;
        lo[4 + j] = y;
      }
      const size_t frag = (((size_t)mt_g * kbp_next + (nt_g0 + nt)) * 2 + kk) * NS;
      dst[(frag + 0) * 64 + lane] = hi;
      if constexpr (NS == 2) dst[(frag + 1) * 64 + lane] = lo;
    }
  }
}

// acc[i] of a 32x32 tile: row (i&3) + 8*(i>>2) + 4*h, column r (C/D layout of
// v_mfma_f32_32x32x16_*, cdna_hip_programming.md §3).
__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// ------------------------------------------------------------------------
// Prefill / encoder kernel.
// ------------------------------------------------------------------------
constexpr int kPrefillTM = 4;  // m-tiles (32 rows) per workgroup
constexpr int kPrefillTN = 2;  // n-tiles (32 cols) per wave; 4 waves

template <int NS, int EPI>
__global__ __launch_bounds__(256, 2) void q4_gemm_prefill_kernel(const uint8_t* __restrict__ nib,
                                                                 const uint32_t* __restrict__ sc,
                                                                 const float* __restrict__ colscale,
                                                                 const _Float16* __restrict__ at, int mtiles,
                                                                 int nbp, int ntiles, EpiArgs e) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int TM = kPrefillTM, TN = kPrefillTN;
  constexpr int CHUNK = 4096 * NS;   // one (m-tile, block pair) of A
  constexpr int BUF = TM * CHUNK;    // one K-step of A for the workgroup
  constexpr int SEGS = BUF / 1024;   // 1 KiB glds segments per K-step
  constexpr int SEGS_PER_WAVE = SEGS / 4;
  constexpr int SEGS_PER_CHUNK = CHUNK / 1024;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int ngroups = (ntiles + 4 * TN - 1) / (4 * TN);
  const int mgroups = mtiles / TM;
  const int wg = xcd_remap(blockIdx.x, ngroups * mgroups);
  const int mg = wg / ngroups, ng = wg % ngroups;
  const int nt0 = ng * (4 * TN) + wave * TN;
  const bool active = nt0 < ntiles;  // wave-uniform

  const uint8_t* abase = reinterpret_cast<const uint8_t*>(at);
  const size_t mtile_stride = (size_t)nbp * CHUNK;
  const uint8_t* arow = abase + (size_t)(TM * mg) * mtile_stride;

  auto issue_a = [&](int bp, int buf) {
#pragma unroll
    for (int i = 0; i < SEGS_PER_WAVE; ++i) {
      const int seg = i * 4 + wave;
      const int ml = seg / SEGS_PER_CHUNK, so = seg % SEGS_PER_CHUNK;
      const uint8_t* src = arow + ml * mtile_stride + (size_t)bp * CHUNK + so * 1024 + lane * 16;
      glds16(src, smem + buf * BUF + seg * 1024);
    }
  };

  u32x4 braw[TN];
  uint32_t bsc[TN];
  auto load_b = [&](int bp, u32x4* br, uint32_t* bs) {
#pragma unroll
    for (int nt = 0; nt < TN; ++nt) {
      const size_t t = (size_t)(nt0 + nt) * nbp + bp;
      br[nt] = *reinterpret_cast<const u32x4*>(nib + (t * 64 + lane) * 16);
      bs[nt] = sc[t * 32 + r];
    }
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.0f;

  issue_a(0, 0);
  if (active) load_b(0, braw, bsc);
  __syncthreads();

  for (int bp = 0; bp < nbp; ++bp) {
    const bool more = bp + 1 < nbp;
    u32x4 braw_n[TN];
    uint32_t bsc_n[TN];
    if (more) {
      issue_a(bp + 1, (bp + 1) & 1);
      if (active) load_b(bp + 1, braw_n, bsc_n);
    }
    if (active) {
      const uint8_t* abuf = smem + (bp & 1) * BUF;
#pragma unroll
      for (int blk = 0; blk < 2; ++blk) {
        half8 bh[TN][2], bl[TN][2];
#pragma unroll
        for (int nt = 0; nt < TN; ++nt) {
          const uint32_t dbits = blk ? (bsc[nt] >> 16) : (bsc[nt] & 0xffffu);
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) deq_scaled<NS>(braw[nt][blk * 2 + kk], dbits, bh[nt][kk], bl[nt][kk]);
        }
#pragma unroll
        for (int mt = 0; mt < TM; ++mt) {
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) {
            const uint8_t* fa = abuf + mt * CHUNK + ((blk * 2 + kk) * NS) * 1024 + lane * 16;
            const half8 ahi = *reinterpret_cast<const half8*>(fa);
            half8 alo;
            if constexpr (NS == 2) alo = *reinterpret_cast<const half8*>(fa + 1024);
#pragma unroll
            for (int nt = 0; nt < TN; ++nt) {
              acc[mt][nt] = mfma32(ahi, bh[nt][kk], acc[mt][nt]);
              if constexpr (NS == 2) {
                acc[mt][nt] = mfma32(alo, bh[nt][kk], acc[mt][nt]);
                acc[mt][nt] = mfma32(ahi, bl[nt][kk], acc[mt][nt]);
              }
            }
          }
        }
      }
    }
    if (more) {
#pragma unroll
      for (int nt = 0; nt < TN; ++nt) {
        braw[nt] = braw_n[nt];
        bsc[nt] = bsc_n[nt];
      }
    }
    __syncthreads();  // drains this step's global_load_lds before the next read
  }

  float cs[TN];
#pragma unroll
  for (int nt = 0; nt < TN; ++nt) cs[nt] = active ? colscale[(nt0 + nt) * 32 + r] : 1.0f;

  if constexpr (EPI == kEpiF32) {
    if (active) {
#pragma unroll
      for (int mt = 0; mt < TM; ++mt)
#pragma unroll
        for (int nt = 0; nt < TN; ++nt)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int row = (TM * mg + mt) * 32 + acc_row(i, h);
            const int col = (nt0 + nt) * 32 + r;
            if (row < e.m && col < e.n)
              e.out[(size_t)row * e.ldo + col] = epi_value(acc[mt][nt][i] * cs[nt], row, col, e);
          }
    }
  } else {
    float* stage = reinterpret_cast<float*>(smem) + wave * (32 * kStageLd);
#pragma unroll
    for (int mt = 0; mt < TM; ++mt) {
      if (active) {
#pragma unroll
        for (int nt = 0; nt < TN; ++nt)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int rl = acc_row(i, h);
            const int row = (TM * mg + mt) * 32 + rl;
            const int col = (nt0 + nt) * 32 + r;
            const float v = (row < e.m && col < e.n) ? epi_value(acc[mt][nt][i] * cs[nt], row, col, e) : 0.0f;
            stage[rl * kStageLd + nt * 32 + r] = v;
          }
      }
      __syncthreads();
      if (active) store_tiled_slab<NS, TN>(stage, e, TM * mg + mt, nt0, lane);
      __syncthreads();
    }
  }
}

// ------------------------------------------------------------------------
// Decode / small-M kernel.
// ------------------------------------------------------------------------
constexpr int kDecodeMTG = 2;     // m-tiles held in registers per pass
constexpr int kDecodeWaves = 8;   // waves per workgroup, each a contiguous K range
constexpr int kDecodeMaxBp = 12;  // block pairs whose weights a wave keeps in flight

template <int NS, int EPI>
__global__ __launch_bounds__(512) void q4_gemm_decode_kernel(const uint8_t* __restrict__ nib,
                                                             const uint32_t* __restrict__ sc,
                                                             const float* __restrict__ colscale,
                                                             const _Float16* __restrict__ at, int mtiles,
                                                             int nbp, int ntiles, EpiArgs e) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int W = kDecodeWaves;
  float* red = reinterpret_cast<float*>(smem);                        // [W-1][16][64]
  float* stage = reinterpret_cast<float*>(smem) + (W - 1) * 16 * 64;  // [32][kStageLd]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int nt = blockIdx.x;
  const int chunk = (nbp + W - 1) / W;
  const int bp0 = wave * chunk;
  const int cnt = max(0, min(nbp, bp0 + chunk) - bp0);
  const size_t kbp = (size_t)nbp * 2;
  const half8* afr = reinterpret_cast<const half8*>(at);
  const float cs = colscale[nt * 32 + r];

  for (int mt0 = 0; mt0 < mtiles; mt0 += kDecodeMTG) {
    floatx16 acc[kDecodeMTG];
#pragma unroll
    for (int a = 0; a < kDecodeMTG; ++a)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][i] = 0.0f;

    for (int base = 0; base < cnt; base += kDecodeMaxBp) {
      const int n = min(kDecodeMaxBp, cnt - base);
      // every weight load of this pass in flight at once (memory-level parallelism)
      u32x4 br[kDecodeMaxBp];
      uint32_t bs[kDecodeMaxBp];
#pragma unroll
      for (int i = 0; i < kDecodeMaxBp; ++i) {
        if (i < n) {
          const size_t t = (size_t)nt * nbp + bp0 + base + i;
          br[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(nib + (t * 64 + lane) * 16));
          bs[i] = __builtin_nontemporal_load(sc + t * 32 + r);
        }
      }
#pragma unroll
      for (int i = 0; i < kDecodeMaxBp; ++i) {
        if (i < n) {
          const int bp = bp0 + base + i;
#pragma unroll
          for (int blk = 0; blk < 2; ++blk) {
            const uint32_t dbits = blk ? (bs[i] >> 16) : (bs[i] & 0xffffu);
            half8 bh[2], bl[2];
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) deq_scaled<NS>(br[i][blk * 2 + kk], dbits, bh[kk], bl[kk]);
#pragma unroll
            for (int mi = 0; mi < kDecodeMTG; ++mi) {
              const int mt = mt0 + mi;
              if (mt < mtiles) {
                const bool row_ok = mt * 32 + r < e.m;
#pragma unroll
                for (int kk = 0; kk < 2; ++kk) {
                  const size_t frag = (((size_t)mt * kbp + 2 * bp + blk) * 2 + kk) * NS;
                  half8 ahi, alo;
#pragma unroll
                  for (int j = 0; j < 8; ++j) {
                    ahi[j] = (_Float16)0.0f;
                    alo[j] = (_Float16)0.0f;
                  }
                  if (row_ok) {
                    ahi = afr[frag * 64 + lane];
                    if constexpr (NS == 2) alo = afr[(frag + 1) * 64 + lane];
                  }
                  acc[mi] = mfma32(ahi, bh[kk], acc[mi]);
                  if constexpr (NS == 2) {
                    acc[mi] = mfma32(alo, bh[kk], acc[mi]);
                    acc[mi] = mfma32(ahi, bl[kk], acc[mi]);
                  }
                }
              }
            }
          }
        }
      }
    }

    // Fixed-order reduction over the W waves, one m-tile at a time.
#pragma unroll
    for (int mi = 0; mi < kDecodeMTG; ++mi) {
      const int mt = mt0 + mi;
      if (mt >= mtiles) break;  // uniform across the workgroup
      if (wave > 0) {
#pragma unroll
        for (int i = 0; i < 16; ++i) red[((wave - 1) * 16 + i) * 64 + lane] = acc[mi][i];
      }
      __syncthreads();
      if (wave == 0) {
        floatx16 s = acc[mi];
#pragma unroll
        for (int w = 0; w < W - 1; ++w)
#pragma unroll
          for (int i = 0; i < 16; ++i) s[i] = s[i] + red[(w * 16 + i) * 64 + lane];
        if constexpr (EPI == kEpiF32) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int row = mt * 32 + acc_row(i, h);
            const int col = nt * 32 + r;
            if (row < e.m && col < e.n) e.out[(size_t)row * e.ldo + col] = epi_value(s[i] * cs, row, col, e);
          }
        } else {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int rl = acc_row(i, h);
            const int row = mt * 32 + rl;
            const int col = nt * 32 + r;
            stage[rl * kStageLd + r] = (row < e.m && col < e.n) ? epi_value(s[i] * cs, row, col, e) : 0.0f;
          }
          __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): stage writes visible to this wave
          __builtin_amdgcn_wave_barrier();
          store_tiled_slab<NS, 1>(stage, e, mt, nt, lane);
        }
      }
      __syncthreads();
    }
  }
}

// ------------------------------------------------------------------------
// Launchers.
// ------------------------------------------------------------------------
static size_t prefill_lds_bytes(int ns, int epi) {
  const size_t a = (size_t)2 * kPrefillTM * 4096 * ns;
  const size_t s = epi == kEpiTiled ? (size_t)4 * 32 * kStageLd * 4 : 0;
  return a > s ? a : s;
}

static size_t decode_lds_bytes() {
  return (size_t)(kDecodeWaves - 1) * 16 * 64 * 4 + (size_t)32 * kStageLd * 4;
}

hipError_t launch_tile_activations(const float* x, _Float16* at, int M, int K, int ld, int ns, hipStream_t st) {
  const int mtiles = (int)(round_up(M < 1 ? 1 : M, kMPad) / kMTile);
  const int kbp = (int)(((K / kBlock) + 1) / 2) * 2;
  const int64_t total = (int64_t)mtiles * kbp * 2 * 64;
  const int grid = (int)((total + 255) / 256);
  const bool aligned = (ld % 4 == 0) && ((reinterpret_cast<uintptr_t>(x) & 15u) == 0);
#define WQ4_TILE(NS_, AL_)                                                                                   \
  hipLaunchKernelGGL((tile_activations_kernel<NS_, AL_>), dim3(grid), dim3(256), 0, st, x, at, M, K, ld, mtiles, \
                     kbp)
  if (ns == 2) {
    if (aligned) WQ4_TILE(2, true); else WQ4_TILE(2, false);
  } else {
    if (aligned) WQ4_TILE(1, true); else WQ4_TILE(1, false);
  }
#undef WQ4_TILE
  return hipGetLastError();
}

template <int NS, int EPI>
static hipError_t launch_gemm_t(const Q4Geom& g, const uint8_t* nib, const uint32_t* sc, const float* cs,
                                const _Float16* at, int rows, const EpiArgs& e, bool decode, hipStream_t st) {
  const int mtiles = (int)(round_up(rows < 1 ? 1 : rows, kMPad) / kMTile);
  if (decode) {
    const int mreal = (int)((rows + kMTile - 1) / kMTile);  // never touch padded m-tiles
    hipLaunchKernelGGL((q4_gemm_decode_kernel<NS, EPI>), dim3((unsigned)g.ntiles), dim3(64 * kDecodeWaves),
                       decode_lds_bytes(), st, nib, sc, cs, at, mreal, (int)g.nbp, (int)g.ntiles, e);
  } else {
    const int ngroups = (int)((g.ntiles + 4 * kPrefillTN - 1) / (4 * kPrefillTN));
    const int mgroups = mtiles / kPrefillTM;
    hipLaunchKernelGGL((q4_gemm_prefill_kernel<NS, EPI>), dim3((unsigned)(ngroups * mgroups)), dim3(256),
                       prefill_lds_bytes(NS, EPI), st, nib, sc, cs, at, mtiles, (int)g.nbp, (int)g.ntiles, e);
  }
  return hipGetLastError();
}

hipError_t launch_q4_gemm(const Q4Geom& g, const uint8_t* nib, const uint32_t* sc, const float* colscale,
                          const _Float16* at, int rows, const EpiArgs& e, int epi_mode, int ns, bool decode,
                          hipStream_t st) {
  if (ns == 2) {
    return epi_mode == kEpiF32 ? launch_gemm_t<2, kEpiF32>(g, nib, sc, colscale, at, rows, e, decode, st)
                               : launch_gemm_t<2, kEpiTiled>(g, nib, sc, colscale, at, rows, e, decode, st);
  }
  return epi_mode == kEpiF32 ? launch_gemm_t<1, kEpiF32>(g, nib, sc, colscale, at, rows, e, decode, st)
                             : launch_gemm_t<1, kEpiTiled>(g, nib, sc, colscale, at, rows, e, decode, st);
}

}  // namespace wq4
