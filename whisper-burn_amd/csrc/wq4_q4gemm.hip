// wq4_q4gemm.hip -- MI355X (gfx950) kernels of the fused Q4_0 dequant + GEMM.
//
// Replaces the reference's single WGSL shader (src/gguf/shader.wgsl:51-92,
// one thread per output, scalar f32 FMA, 18 dependent u32 loads per block)
// with two MFMA kernels over the repacked weights and A-tiled activations of
// wq4_layout.hpp:
//
//  q4_gemm_prefill  M >= ~64 rows (encoder, cross-K/V): 64 x 256 workgroup
//                   tile, 4 waves x (64 x 64), A staged through LDS (double
//                   buffer, register staging), B (weights) straight to VGPRs
//                   as one 1 KiB coalesced load per (n-tile, block pair).
//  q4_gemm_decode   M <= ~64 rows (decoder tokens, prompt): one 32-column
//                   n-tile per workgroup, the K range split over 4 waves and
//                   reduced through LDS in a fixed order; A rows beyond M are
//                   never loaded.
//
// Per output and Q4 block b the arithmetic is identical in both kernels and
// independent of M and of the tile position:
//    P_b = sum_{kk=0,1} sum_{s in splits} MFMA_32x32x16_f16(A[kk][s], B_b[kk])
//    acc = fma(d_b, P_b, acc)            (d_b = f16 scale in f32)
// with B_b[kk] the exact f16 (q - 8) and A[kk][s] the f16 hi/lo split of x.
// The prefill kernel sums blocks in order 0..Kb-1; the decode kernel sums
// each wave's contiguous block range in order and adds the 4 wave partials
// in wave order.  Both orders depend only on (N, K), never on M, so a row's
// result is the same at batch 1 and batch 256.
#include <hip/hip_runtime.h>

#include "wq4_device.hpp"
#include "wq4_kernels.hpp"

namespace wq4 {

// ------------------------------------------------------------------------
// f32 row-major [M, K] -> A-tiled f16 (hi[, lo]) operand.  One thread per
// (m-tile, block, kk, lane) = 8 elements.
// ------------------------------------------------------------------------
template <int NS>
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
    const floatx4* src = reinterpret_cast<const floatx4*>(x + (size_t)m * ld + k0);
    floatx4 a = src[0], c = src[1];
    v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
    v[4] = c[0]; v[5] = c[1]; v[6] = c[2]; v[7] = c[3];
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

// Scalar-input variant used when a row is not 16-B aligned (ld % 4 != 0).
template <int NS>
__global__ __launch_bounds__(256) void tile_activations_unaligned_kernel(const float* __restrict__ x,
                                                                         _Float16* __restrict__ at, int M,
                                                                         int K, int ld, int mtiles, int kbp) {
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
  half8 hi, lo;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float v = (m < M && k0 < K) ? x[(size_t)m * ld + k0 + j] : 0.0f;
    _Float16 a, c;
    split_f16(v, a, c);
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

// ------------------------------------------------------------------------
// Prefill / encoder kernel.
// ------------------------------------------------------------------------
template <int NS, int EPI>
__global__ __launch_bounds__(256, 2) void q4_gemm_prefill_kernel(const uint8_t* __restrict__ nib,
                                                                 const uint32_t* __restrict__ sc,
                                                                 const _Float16* __restrict__ at, int mtiles,
                                                                 int nbp, int ntiles, EpiArgs e) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int CHUNK = 4096 * NS;  // one (m-tile, block pair) of A
  constexpr int BUF = 2 * CHUNK;    // two m-tiles per workgroup
  constexpr int LOADS = BUF / (256 * 16);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int ngroups = (ntiles + 7) / 8;
  const int mgroups = mtiles / 2;
  const int wg = xcd_remap(blockIdx.x, ngroups * mgroups);
  const int mg = wg / ngroups, ng = wg % ngroups;
  const int nt0 = ng * 8 + wave * 2;
  const bool active = nt0 < ntiles;  // wave-uniform

  const uint8_t* abase = reinterpret_cast<const uint8_t*>(at);
  const size_t mtile_stride = (size_t)nbp * CHUNK;
  const uint8_t* arow = abase + (size_t)(2 * mg) * mtile_stride;

  u32x4 areg[LOADS];
  auto load_a = [&](int bp) {
#pragma unroll
    for (int i = 0; i < LOADS; ++i) {
      const int o = (i * 256 + tid) * 16;
      const int ml = o / CHUNK, rest = o % CHUNK;
      areg[i] = *reinterpret_cast<const u32x4*>(arow + ml * mtile_stride + (size_t)bp * CHUNK + rest);
    }
  };
  auto store_a = [&](int buf) {
#pragma unroll
    for (int i = 0; i < LOADS; ++i)
      *reinterpret_cast<u32x4*>(smem + buf * BUF + (i * 256 + tid) * 16) = areg[i];
  };

  u32x4 braw[2];
  uint32_t bsc[2];
  auto load_b = [&](int bp, u32x4* br, uint32_t* bs) {
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const size_t t = (size_t)(nt0 + nt) * nbp + bp;
      br[nt] = *reinterpret_cast<const u32x4*>(nib + (t * 64 + lane) * 16);
      bs[nt] = sc[t * 32 + r];
    }
  };

  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.0f;

  load_a(0);
  if (active) load_b(0, braw, bsc);
  store_a(0);
  __syncthreads();

  for (int bp = 0; bp < nbp; ++bp) {
    const bool more = bp + 1 < nbp;
    u32x4 braw_n[2];
    uint32_t bsc_n[2];
    if (more) {
      load_a(bp + 1);
      if (active) load_b(bp + 1, braw_n, bsc_n);
    }
    if (active) {
      const uint8_t* abuf = smem + (bp & 1) * BUF;
#pragma unroll
      for (int blk = 0; blk < 2; ++blk) {
        half8 bf[2][2];
        float d[2];
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          bf[nt][0] = deq8(braw[nt][blk * 2 + 0]);
          bf[nt][1] = deq8(braw[nt][blk * 2 + 1]);
          d[nt] = f16bits_to_f32(blk ? (bsc[nt] >> 16) : (bsc[nt] & 0xffffu));
        }
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          half8 a[2][NS];
#pragma unroll
          for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int s = 0; s < NS; ++s)
              a[kk][s] = *reinterpret_cast<const half8*>(abuf + mt * CHUNK + ((blk * 2 + kk) * NS + s) * 1024 +
                                                         lane * 16);
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) {
            floatx16 p;
#pragma unroll
            for (int i = 0; i < 16; ++i) p[i] = 0.0f;
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
#pragma unroll
              for (int s = 0; s < NS; ++s) p = mfma32(a[kk][s], bf[nt][kk], p);
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[mt][nt][i] = __builtin_fmaf(d[nt], p[i], acc[mt][nt][i]);
          }
        }
      }
    }
    if (more) {
      store_a((bp + 1) & 1);
      braw[0] = braw_n[0];
      braw[1] = braw_n[1];
      bsc[0] = bsc_n[0];
      bsc[1] = bsc_n[1];
    }
    __syncthreads();
  }

  if constexpr (EPI == kEpiF32) {
    if (active) {
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int row = (2 * mg + mt) * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
            const int col = (nt0 + nt) * 32 + r;
            if (row < e.m && col < e.n) e.out[(size_t)row * e.ldo + col] = epi_value(acc[mt][nt][i], row, col, e);
          }
    }
  } else {
    float* stage = reinterpret_cast<float*>(smem) + wave * (32 * kStageLd);
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      if (active) {
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int rl = (i & 3) + 8 * (i >> 2) + 4 * h;
            const int row = (2 * mg + mt) * 32 + rl;
            const int col = (nt0 + nt) * 32 + r;
            const float v = (row < e.m && col < e.n) ? epi_value(acc[mt][nt][i], row, col, e) : 0.0f;
            stage[rl * kStageLd + nt * 32 + r] = v;
          }
      }
      __syncthreads();
      if (active) store_tiled_slab<NS, 2>(stage, e, 2 * mg + mt, nt0, lane);
      __syncthreads();
    }
  }
}

// ------------------------------------------------------------------------
// Decode / small-M kernel.
// ------------------------------------------------------------------------
constexpr int kDecodeMTG = 2;  // m-tiles held in registers per pass

template <int NS, int EPI>
__global__ __launch_bounds__(256) void q4_gemm_decode_kernel(const uint8_t* __restrict__ nib,
                                                             const uint32_t* __restrict__ sc,
                                                             const _Float16* __restrict__ at, int mtiles,
                                                             int nbp, int ntiles, EpiArgs e) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  float* red = reinterpret_cast<float*>(smem);              // [3][16][64]
  float* stage = reinterpret_cast<float*>(smem) + 3 * 16 * 64;  // [32][kStageLd]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int nt = blockIdx.x;
  const int chunk = (nbp + 3) / 4;
  const int bp0 = wave * chunk;
  const int bp1 = min(nbp, bp0 + chunk);
  const size_t kbp = (size_t)nbp * 2;
  const half8* afr = reinterpret_cast<const half8*>(at);

  for (int mt0 = 0; mt0 < mtiles; mt0 += kDecodeMTG) {
    floatx16 acc[kDecodeMTG];
#pragma unroll
    for (int a = 0; a < kDecodeMTG; ++a)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][i] = 0.0f;

    u32x4 br;
    uint32_t bs = 0;
    if (bp0 < bp1) {
      const size_t t = (size_t)nt * nbp + bp0;
      br = *reinterpret_cast<const u32x4*>(nib + (t * 64 + lane) * 16);
      bs = sc[t * 32 + r];
    }
    for (int bp = bp0; bp < bp1; ++bp) {
      u32x4 br_n;
      uint32_t bs_n = 0;
      if (bp + 1 < bp1) {
        const size_t t = (size_t)nt * nbp + bp + 1;
        br_n = *reinterpret_cast<const u32x4*>(nib + (t * 64 + lane) * 16);
        bs_n = sc[t * 32 + r];
      }
#pragma unroll
      for (int blk = 0; blk < 2; ++blk) {
        const half8 b0 = deq8(br[blk * 2 + 0]);
        const half8 b1 = deq8(br[blk * 2 + 1]);
        const float d = f16bits_to_f32(blk ? (bs >> 16) : (bs & 0xffffu));
#pragma unroll
        for (int mi = 0; mi < kDecodeMTG; ++mi) {
          const int mt = mt0 + mi;
          if (mt < mtiles) {
            const bool row_ok = mt * 32 + r < e.m;
            half8 a[2][NS];
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
#pragma unroll
              for (int s = 0; s < NS; ++s) {
                const size_t frag = (((size_t)mt * kbp + 2 * bp + blk) * 2 + kk) * NS + s;
                half8 v;
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = (_Float16)0.0f;
                if (row_ok) v = afr[frag * 64 + lane];
                a[kk][s] = v;
              }
            floatx16 p;
#pragma unroll
            for (int i = 0; i < 16; ++i) p[i] = 0.0f;
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
              const half8& bk = kk ? b1 : b0;
#pragma unroll
              for (int s = 0; s < NS; ++s) p = mfma32(a[kk][s], bk, p);
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[mi][i] = __builtin_fmaf(d, p[i], acc[mi][i]);
          }
        }
      }
      br = br_n;
      bs = bs_n;
    }

    // Fixed-order reduction over the 4 waves, one m-tile at a time.
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
        for (int w = 0; w < 3; ++w)
#pragma unroll
          for (int i = 0; i < 16; ++i) s[i] = s[i] + red[(w * 16 + i) * 64 + lane];
        if constexpr (EPI == kEpiF32) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int row = mt * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
            const int col = nt * 32 + r;
            if (row < e.m && col < e.n) e.out[(size_t)row * e.ldo + col] = epi_value(s[i], row, col, e);
          }
        } else {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int rl = (i & 3) + 8 * (i >> 2) + 4 * h;
            const int row = mt * 32 + rl;
            const int col = nt * 32 + r;
            stage[rl * kStageLd + r] = (row < e.m && col < e.n) ? epi_value(s[i], row, col, e) : 0.0f;
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
size_t prefill_lds_bytes(int ns, int epi) {
  size_t a = (size_t)2 * 2 * 4096 * ns;
  size_t s = epi == kEpiTiled ? (size_t)4 * 32 * kStageLd * 4 : 0;
  return a > s ? a : s;
}

size_t decode_lds_bytes() { return (size_t)3 * 16 * 64 * 4 + (size_t)32 * kStageLd * 4; }

hipError_t launch_tile_activations(const float* x, _Float16* at, int M, int K, int ld, int ns, hipStream_t st) {
  const int mtiles = (int)(round_up(M < 1 ? 1 : M, kMPad) / kMTile);
  const int kbp = (int)(((K / kBlock) + 1) / 2) * 2;
  const int64_t total = (int64_t)mtiles * kbp * 2 * 64;
  const int grid = (int)((total + 255) / 256);
  const bool aligned = (ld % 4 == 0) && ((reinterpret_cast<uintptr_t>(x) & 15u) == 0);
  if (aligned) {
    if (ns == 2)
      hipLaunchKernelGGL(tile_activations_kernel<2>, dim3(grid), dim3(256), 0, st, x, at, M, K, ld, mtiles, kbp);
    else
      hipLaunchKernelGGL(tile_activations_kernel<1>, dim3(grid), dim3(256), 0, st, x, at, M, K, ld, mtiles, kbp);
  } else {
    if (ns == 2)
      hipLaunchKernelGGL(tile_activations_unaligned_kernel<2>, dim3(grid), dim3(256), 0, st, x, at, M, K, ld,
                         mtiles, kbp);
    else
      hipLaunchKernelGGL(tile_activations_unaligned_kernel<1>, dim3(grid), dim3(256), 0, st, x, at, M, K, ld,
                         mtiles, kbp);
  }
  return hipGetLastError();
}

template <int NS, int EPI>
static hipError_t launch_gemm_t(const Q4Geom& g, const uint8_t* nib, const uint32_t* sc, const _Float16* at,
                                int rows, const EpiArgs& e, bool decode, hipStream_t st) {
  const int mtiles = (int)(round_up(rows < 1 ? 1 : rows, kMPad) / kMTile);
  if (decode) {
    hipLaunchKernelGGL((q4_gemm_decode_kernel<NS, EPI>), dim3((unsigned)g.ntiles), dim3(256), decode_lds_bytes(),
                       st, nib, sc, at, mtiles, (int)g.nbp, (int)g.ntiles, e);
  } else {
    const int ngroups = (int)((g.ntiles + 7) / 8);
    const int mgroups = mtiles / 2;
    hipLaunchKernelGGL((q4_gemm_prefill_kernel<NS, EPI>), dim3((unsigned)(ngroups * mgroups)), dim3(256),
                       prefill_lds_bytes(NS, EPI), st, nib, sc, at, mtiles, (int)g.nbp, (int)g.ntiles, e);
  }
  return hipGetLastError();
}

hipError_t launch_q4_gemm(const Q4Geom& g, const uint8_t* nib, const uint32_t* sc, const _Float16* at, int rows,
                          const EpiArgs& e, int epi_mode, int ns, bool decode, hipStream_t st) {
  if (ns == 2) {
    return epi_mode == kEpiF32 ? launch_gemm_t<2, kEpiF32>(g, nib, sc, at, rows, e, decode, st)
                               : launch_gemm_t<2, kEpiTiled>(g, nib, sc, at, rows, e, decode, st);
  }
  return epi_mode == kEpiF32 ? launch_gemm_t<1, kEpiF32>(g, nib, sc, at, rows, e, decode, st)
                             : launch_gemm_t<1, kEpiTiled>(g, nib, sc, at, rows, e, decode, st);
}

}  // namespace wq4
