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
// Arithmetic, x = x_hi + x_lo (f16 pair):
//   prefill, Q4_0 weights -- block-scaled: per Q4 block t = sum over its 32 k
//     of MFMA(x_hi, q - 8) + MFMA(x_lo, q - 8) (q - 8 exact in f16, f32
//     accumulation from zero), acc = t * d' + acc, then y = acc * 2^-s_n:
//     two MFMAs per multiply-add;
//   decode, and f16 weights -- with the exact weight B = (q - 8) * d' = B_hi +
//     B_lo (f16 pair, d' the row-prescaled f16 scale, wq4_layout.hpp),
//     acc += MFMA(x_hi, B_hi) + MFMA(x_lo, B_hi) + MFMA(x_hi, B_lo) per 16-k
//     half (f16 weights: B_lo = 0), f32 accumulation; the dropped x_lo * B_lo
//     term is < 2^-22 relative.
// WQ4_PREC_F16 keeps only the x_hi terms.  Per-row instruction order depends
// on (N, K) only, never on M or the tile position: a row's result is
// identical at batch 1 and 256.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "wq4_device.hpp"
#include "wq4_kernels.hpp"
#include "wq4_lnmath.hpp"
#include "wq4_tile_epi.hpp"

namespace wq4 {

// WQ4_PF_DIAG (timing diagnostics of the prefill kernel only; 0 in the
// product): 1 no scale FMAs, 2 no dequantisation, 3 scalar v_fma_f32 scale,
// 4 = 1 + 2.
#ifndef WQ4_PF_DIAG
#define WQ4_PF_DIAG 0
#endif

// ------------------------------------------------------------------------
// f32 row-major [M, K] -> A-tiled f16 (hi[, lo]) operand.  One thread per
// (m-tile, block, kk, lane) = 8 elements.
// ------------------------------------------------------------------------
template <int NS, bool ALIGNED>
__global__ __launch_bounds__(256) void tile_activations_kernel(const float* __restrict__ x,
                                                               _Float16* __restrict__ at, int M, int K,
                                                               int ld, int mtiles, int kbp,
                                                               const float* __restrict__ scale) {
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
  const float s = scale ? scale[0] : kActScale;
  half8 hi, lo;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    _Float16 a, c;
    split_f16(v[j] * s, a, c);
    hi[j] = a;
    lo[j] = c;
  }
  const size_t frag = (((size_t)mt * kbp + b) * 2 + kk) * NS;
  half8* dst = reinterpret_cast<half8*>(at);
  dst[(frag + 0) * 64 + lane] = hi;
  if constexpr (NS == 2) dst[(frag + 1) * 64 + lane] = lo;
}

// ------------------------------------------------------------------------
// Prefill / encoder kernel.
// ------------------------------------------------------------------------
constexpr int kPrefillTM = 4;  // m-tiles (32 rows) per workgroup
constexpr int kPrefillTN = 2;  // n-tiles (32 cols) per wave; 4 waves

template <int NS, int EPI, int WK>
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
  const int r = lane & 31;
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

  // B: Q4 -> 16 B nibbles + a scale word per (n-tile, bp); F16 weights ->
  // four 16 B fragments (blk, kk) per (n-tile, bp), used as they are
  constexpr int BW = WK == kWeightsF16 ? 4 : 1;
  u32x4 braw[TN][BW];
  uint32_t bsc[TN];
  auto load_b = [&](int bp, u32x4 (*br)[BW], uint32_t* bs) {
#pragma unroll
    for (int nt = 0; nt < TN; ++nt) {
      const size_t t = (size_t)(nt0 + nt) * nbp + bp;
      if constexpr (WK == kWeightsF16) {
#pragma unroll
        for (int q = 0; q < 4; ++q) br[nt][q] = *reinterpret_cast<const u32x4*>(nib + (t * 64 + lane) * 64 + q * 16);
        bs[nt] = 0;
      } else {
        br[nt][0] = *reinterpret_cast<const u32x4*>(nib + (t * 64 + lane) * 16);
        bs[nt] = sc[t * 32 + r];
      }
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
    u32x4 braw_n[TN][BW];
    uint32_t bsc_n[TN];
    if (more) {
      issue_a(bp + 1, (bp + 1) & 1);
      if (active) load_b(bp + 1, braw_n, bsc_n);
    }
    if (active) {
      const uint8_t* abuf = smem + (bp & 1) * BUF;
#pragma unroll
      for (int blk = 0; blk < 2; ++blk) {
        if constexpr (WK == kWeightsF16) {
          // exact f16 weights: acc += x_hi * w + x_lo * w per 16-k half
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
                const half8 bw = __builtin_bit_cast(half8, braw[nt][blk * 2 + kk]);
                acc[mt][nt] = mfma32(ahi, bw, acc[mt][nt]);
                if constexpr (NS == 2) acc[mt][nt] = mfma32(alo, bw, acc[mt][nt]);
              }
            }
          }
        } else {
          // Q4_0, block-scaled: t = sum over the block's 32 k of x * (q - 8)
          // (exact f16 integers, f32 MFMA accumulation from zero), then
          // acc += t * d' -- two MFMAs per multiply-add with NS = 2 instead
          // of three for an f16-pair weight
          half8 qf[TN][2];
          float dsc[TN];
#pragma unroll
          for (int nt = 0; nt < TN; ++nt) {
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) qf[nt][kk] = deq8(braw[nt][0][blk * 2 + kk]);
            dsc[nt] = (float)__builtin_bit_cast(_Float16, (uint16_t)(blk ? (bsc[nt] >> 16) : (bsc[nt] & 0xffffu)));
          }
          // two temporaries in flight: tile (mt, 1)'s MFMA chain runs under
          // the scale FMAs of (mt, 0), and (mt + 1, 0)'s under those of
          // (mt, 1), so no FMA waits on the MFMA it reads
          static_assert(TN == 2, "the interleave below pairs the two n-tiles of a wave");
          floatx16 t0, t1;
#if WQ4_PF_DIAG == 2 || WQ4_PF_DIAG == 4  // timing diagnostics: no dequantisation (raw bits as B)
#pragma unroll
          for (int nt = 0; nt < TN; ++nt)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) qf[nt][kk] = __builtin_bit_cast(half8, braw[nt][0]);
#endif
          auto chain = [&](const half8 (&ah)[2], const half8 (&al)[2], int nt) {
            floatx16 t = mfma32(ah[0], qf[nt][0], floatx16{});
            if constexpr (NS == 2) t = mfma32(al[0], qf[nt][0], t);
            t = mfma32(ah[1], qf[nt][1], t);
            if constexpr (NS == 2) t = mfma32(al[1], qf[nt][1], t);
            return t;
          };
#pragma unroll
          for (int mt = 0; mt < TM; ++mt) {
            const uint8_t* fa = abuf + mt * CHUNK + (blk * 2 * NS) * 1024 + lane * 16;
            half8 ahi[2], alo[2];
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
              ahi[kk] = *reinterpret_cast<const half8*>(fa + kk * NS * 1024);
              if constexpr (NS == 2) alo[kk] = *reinterpret_cast<const half8*>(fa + kk * NS * 1024 + 1024);
            }
#if WQ4_PF_DIAG == 1 || WQ4_PF_DIAG == 4  // timing diagnostics: no scale FMAs (chains add into acc)
            t0 = chain(ahi, alo, 0);
            t1 = chain(ahi, alo, 1);
            acc[mt][0] += t0;  // one v_add per element instead of an FMA would still be VALU: keep adds
            acc[mt][1] += t1;
#elif WQ4_PF_DIAG == 3  // scalar v_fma_f32 per element (build with -fno-slp-vectorize)
            t0 = chain(ahi, alo, 0);
            if (mt > 0) {
#pragma unroll
              for (int i = 0; i < 16; ++i) acc[mt - 1][1][i] = __builtin_fmaf(t1[i], dsc[1], acc[mt - 1][1][i]);
            }
            t1 = chain(ahi, alo, 1);
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[mt][0][i] = __builtin_fmaf(t0[i], dsc[0], acc[mt][0][i]);
#else
            t0 = chain(ahi, alo, 0);
            if (mt > 0) acc[mt - 1][1] = t1 * dsc[1] + acc[mt - 1][1];
            t1 = chain(ahi, alo, 1);
            acc[mt][0] = t0 * dsc[0] + acc[mt][0];
#endif
            // issue order: the m-tile's 4 A reads, then MFMA / 2 VALU pairs
            __builtin_amdgcn_sched_group_barrier(0x100, 2 * NS, 0);
#pragma unroll
            for (int i = 0; i < 4 * NS; ++i) {
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
              __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
            }
          }
#if WQ4_PF_DIAG == 3
#pragma unroll
          for (int i = 0; i < 16; ++i) acc[TM - 1][1][i] = __builtin_fmaf(t1[i], dsc[1], acc[TM - 1][1][i]);
#elif WQ4_PF_DIAG != 1 && WQ4_PF_DIAG != 4
          acc[TM - 1][1] = t1 * dsc[1] + acc[TM - 1][1];
#endif
        }
      }
    }
    if (more) {
#pragma unroll
      for (int nt = 0; nt < TN; ++nt) {
#pragma unroll
        for (int q = 0; q < BW; ++q) braw[nt][q] = braw_n[nt][q];
        bsc[nt] = bsc_n[nt];
      }
    }
    __syncthreads();  // drains this step's global_load_lds before the next read
  }

  tile_epilogue<NS, EPI, TM, TN>(acc, TM * mg, nt0, active, mtiles, colscale,
                                 reinterpret_cast<float*>(smem) + wave * (32 * kStageLd), lane, e);
}

// ------------------------------------------------------------------------
// Decode / small-M kernel (M <= 64: decoder tokens, prompt).
//
// Latency-bound GEMV-like shape: the weight bytes of one launch (~1-4 MB)
// are far too few to fill HBM from a handful of workgroups, and every output
// column needs the whole activation operand.  So the K range is split twice:
//   * over KS workgroups per 32-column n-tile (grid = ntiles * KS, chosen so
//     the grid covers most of the 256 CUs), and
//   * over the 4 waves of a workgroup (<= PER block pairs per wave).
// Every wave issues all of its weight and activation loads at once (one
// memory latency, no serial prefetch chain), runs two MFMA chains (k-half
// kk = 0 / 1), and the wave partials are summed through LDS in wave order.
// With KS > 1 each workgroup stores its 32 x 32 partial to a workspace; the
// last workgroup of the n-tile to arrive (device-scope counter) sums the KS
// partials in slice order, applies the epilogue and re-arms the counter.
// Summation order is a function of (N, K) only -> deterministic and batch
// invariant.
// ------------------------------------------------------------------------
constexpr int kDecodeWaves = 4;
constexpr int kDecodeMaxKs = 8;  // K slices per n-tile (fix-up keeps all slabs in flight)

// Branch-free loads through buffer resources: an out-of-range offset reads
// zeros, so masked rows and the ragged end of a wave's K range need no exec
// branches (which would make the compiler drain vmcnt between load groups).
constexpr int kOob = 0x7fffff00;
#ifndef WQ4_WEIGHT_AUX  // compile-time only (tuning builds): cache policy of the decode weight stream
#define WQ4_WEIGHT_AUX 2  // nt
#endif
constexpr int kWeightAux = WQ4_WEIGHT_AUX;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
template <int AUX>
__device__ __forceinline__ half8 bload_h8(__amdgpu_buffer_rsrc_t rs, int off) {
  return __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, AUX));
}

template <int NS, int EPI>
__device__ __forceinline__ void decode_epilogue(const floatx16& s, float cs, int mt, int nt, int lane, float* stage,
                                                const EpiArgs& e) {
  const int r = lane & 31, h = lane >> 5;
  const int col = nt * 32 + r;
  if constexpr (EPI != kEpiTiled) {
    epi_store_tile(
        s, cs, col, [&](int i) { return mt * 32 + acc_row(i, h); },
        [&](int row, int c) { return EPI == kEpiHeadMajor ? out_index(e, row, c) : (size_t)row * e.ldo + c; }, e);
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int rl = acc_row(i, h);
      const int row = mt * 32 + rl;
      stage[rl * kStageLd + r] = (row < e.m && col < e.n) ? epi_value(s[i] * cs, row, col, e) : 0.0f;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): stage writes visible to this wave
    __builtin_amdgcn_wave_barrier();
    store_tiled_slab<NS, 1>(stage, e, mt, nt, lane);
    __builtin_amdgcn_wave_barrier();
  }
}

__host__ __device__ constexpr size_t decode_lds_bytes_dev(int w) {
  return (size_t)(w == 8 ? w : w - 1) * 16 * 64 * 4 + (size_t)32 * kStageLd * 4;
}
// + LNA row stats, + LayerNorm-fold mean / den [32] each and the producer's x stage [32][33]
__host__ __device__ constexpr size_t decode_lds_bytes_all(int w) {
  return decode_lds_bytes_dev(w) + 2 * 64 * 4 + (64 + 32 * 33) * 4;
}


#ifndef WQ4_DIAG
#define WQ4_DIAG 0
#endif
// WQ4_STAMP (timing diagnostics only: make variant V=stamp DEFS=-DWQ4_STAMP=1,
// scripts/skinny_stamps.py with GETTER=decode; 0 in the product): the 8-wave
// plans record per launch and workgroup s_memrealtime at the start, after
// every operand load landed, after the MFMA loop, after the reduction
// barrier and at the end of the epilogue, plus s_memtime cycles.
#ifndef WQ4_STAMP
#define WQ4_STAMP 0
#endif
constexpr int kDStampLaunches = 512, kDStampWgs = 256, kDStampSlots = 8;
#if WQ4_STAMP
__device__ unsigned long long g_dec_stamps[kDStampLaunches * kDStampWgs * kDStampSlots];
#endif
__device__ __forceinline__ unsigned long long dstamp_rt() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
__device__ __forceinline__ unsigned long long dstamp_cyc() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
// Q4_0 weights at f16x2: block-scaled products (1, the product) -- per Q4
// block t = MFMA(x_hi, q0) + MFMA(x_lo, q0) + MFMA(x_hi, q1) + MFMA(x_lo, q1)
// (q - 8 exact in f16, f32 accumulation), then acc = fma(t, d', acc) for the
// accumulator rows that hold real rows only -- the arithmetic of the prefill
// and decode-step kernels: two MFMAs per 16 k and no weight-side split,
// where B = (q - 8) d' = B_hi + B_lo (0, the round-2 form) needs three
// MFMAs and the split's VALU.  Compile-time switch for A/B builds.
#ifndef WQ4_DECODE_BS
#define WQ4_DECODE_BS 1
#endif
template <int NS, int EPI, int PER, int MT, int W, int WK, bool LNA = false>
__global__ __launch_bounds__(64 * W) void q4_gemm_decode_kernel(const uint8_t* __restrict__ nib,
                                                              const uint32_t* __restrict__ sc,
                                                              const float* __restrict__ colscale,
                                                              const _Float16* __restrict__ at, int mt0, int nbp, int ks,
                                                              int chunk, float* __restrict__ part,
                                                              int* __restrict__ counters, EpiArgs e) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int mtiles = MT;
  constexpr int kRedWaves = W == 8 ? W : W - 1;
  unsigned long long st_[kDStampSlots] = {};
  if constexpr (WQ4_STAMP && W == 8) {
    st_[0] = dstamp_rt();
    st_[5] = dstamp_cyc();
  }
  float* red = reinterpret_cast<float*>(smem);                          // [kRedWaves][16][64]
  float* stage = reinterpret_cast<float*>(smem) + kRedWaves * 16 * 64;  // [32][kStageLd]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: scalar buffer descriptors
  const int r = lane & 31;
  const int nt = blockIdx.x / ks;
  const int slice = blockIdx.x - nt * ks;
  const int bp0 = min(nbp, (slice * W + wave) * chunk);  // chunk <= PER (launcher)
  const int cnt = max(0, min(nbp, bp0 + chunk) - bp0);
  // weight row scale x A operand scale (exact powers of two)
  const float cs = colscale[nt * 32 + r] * (e.act_inv ? *e.act_inv : kActScaleInv);
  // 8-wave plans: the epilogue operands of this lane's two outputs (rows
  // acc_row(2 wave + q, h), column nt * 32 + r) are loaded up front so they
  // are not a memory round trip after the MFMAs (bias, residual: never
  // written by this launch before its own epilogue reads them).
  // All of these are branch-free buffer loads (an absent operand is a
  // zero-size resource, an out-of-range element an out-of-range offset: both
  // read 0): a load under an exec branch made the compiler drain vmcnt(0)
  // at the join, one full memory latency before the weight stream was even
  // issued (+1.9 us per LayerNorm-fold consumer launch, tools/warm_cold.py).
  float pre_bias = 0.0f, pre_res[2] = {0.0f, 0.0f};
  float pre_wg = 0.0f, pre_g = 0.0f;  // LayerNorm fold: W gamma[col] (consumer), gamma[col] (producer)
  if constexpr (W == 8 && EPI != kEpiHeadMajor) {
    const int col = nt * 32 + r;
    const int coff = col < e.n ? col * 4 : kOob;
    const uint32_t nb = (uint32_t)e.n * 4;
    pre_bias = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(brsrc(e.bias, e.bias ? nb : 0), coff, 0, 0));
    pre_wg = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                           brsrc(e.lnf_wg, e.lnf_stats_in ? nb : 0), coff, 0, 0));
    pre_g = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(brsrc(e.lnf_g, e.lnf_at ? nb : 0), coff, 0, 0));
    const __amdgpu_buffer_rsrc_t rres = brsrc(e.residual, e.residual ? (uint32_t)e.m * (uint32_t)e.ldo * 4 : 0);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int row = mt0 * 32 + acc_row(2 * wave + q, lane >> 5);
      pre_res[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                 rres, row < e.m && col < e.n ? (row * e.ldo + col) * 4 : kOob, 0, 0));
    }
  }
  // LayerNorm fold, consumer: thread (row tid / 16, part tid % 16) loads the
  // row's tile statistics j = part, part + 16, ... first, so they land before
  // the weight / operand stream; merged below while that stream is in flight.
  constexpr int kLnfPer = 5;  // <= 80 16-column tiles (D <= 1280)
  floatx2 lnf_st[kLnfPer];
  const int lnf_row = tid >> 4, lnf_part = tid & 15;
  if constexpr (W == 8) {
    const int grow = mt0 * 32 + lnf_row;
    const __amdgpu_buffer_rsrc_t rst =
        brsrc(e.lnf_stats_in, e.lnf_stats_in ? (uint32_t)e.m * (uint32_t)e.lnf_tiles * 8 : 0);
#pragma unroll
    for (int u = 0; u < kLnfPer; ++u) {
      const int j = lnf_part + 16 * u;
      lnf_st[u] = __builtin_bit_cast(floatx2, __builtin_amdgcn_raw_buffer_load_b64(
                                                  rst, grow < e.m && j < e.lnf_tiles ? (grow * e.lnf_tiles + j) * 8 : kOob, 0, 0));
    }
  }
  // keep every epilogue-operand / statistics load above the weight stream
  // (the merge below then waits for them with a counted vmcnt)
  __builtin_amdgcn_sched_barrier(0);

  // this wave's weights (once-read stream: nt) -- zeros past cnt
  const size_t t0 = (size_t)nt * nbp + bp0;
  // WQ4_DIAG (timing diagnostics only, make diag + scripts/gpu.sh libs; 0 in the product):
  // 1 no MFMAs, 2 no A loads, 3 no weight loads, 4 no epilogue
  constexpr int kDiag = WQ4_DIAG;
  constexpr int BW = WK == kWeightsF16 ? 4 : 1;  // 16 B weight loads per lane per bp
  const __amdgpu_buffer_rsrc_t rw = brsrc(nib + t0 * 1024 * BW, (uint32_t)cnt * 1024 * BW);
  u32x4 br[PER][BW];
  uint32_t bs[PER];
  if constexpr (WK == kWeightsF16) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
#pragma unroll
      for (int q = 0; q < 4; ++q) br[i][q] = __builtin_amdgcn_raw_buffer_load_b128(rw, (i * 64 + lane) * 64 + q * 16, 0, kWeightAux);
      bs[i] = 0;
    }
  } else {
    const __amdgpu_buffer_rsrc_t rsc = brsrc(sc + t0 * 32, (uint32_t)cnt * 128);
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      br[i][0] = kDiag == 3 ? u32x4{0u, 0u, 0u, 0u} : __builtin_amdgcn_raw_buffer_load_b128(rw, (i * 64 + lane) * 16, 0, kWeightAux);
      bs[i] = kDiag == 3 ? 0u : __builtin_amdgcn_raw_buffer_load_b32(rsc, (i * 32 + r) * 4, 0, kWeightAux);
    }
  }
  // activation fragments of every m-tile, rows >= M read as zeros
  half8 a[MT][PER][2][2][NS];
  if constexpr (LNA) {
    // LayerNorm on load: row statistics exactly as layernorm_kernel (one
    // wave per row, ln_row_stats), then lane (r, hh) builds its fragments
    // y = ((x - mean) / den) * g + b of row r, columns 32 b + 16 kk + 8 hh + j
    // -- bit-identical to LayerNorm -> A-tiled operand -> this kernel.
    float* lnst = reinterpret_cast<float*>(smem + decode_lds_bytes_dev(W));  // [MT * 32][2]
    constexpr int RPW = MT * 32 / W;  // rows per wave: all their loads in flight at once
    floatx4 v[RPW][kLnMaxV];
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      const int row = mt0 * 32 + wave * RPW + q;
      const float* xr = e.lnx + (size_t)(row < e.m ? row : 0) * e.lnd;
#pragma unroll
      for (int i = 0; i < kLnMaxV; ++i) {
        const int k = lane * 4 + 256 * i;
        v[q][i] = (row < e.m && k < e.lnd) ? *reinterpret_cast<const floatx4*>(xr + k) : floatx4{0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      const int rr = wave * RPW + q;
      float mean = 0.0f, den = 1.0f;
      if (mt0 * 32 + rr < e.m) ln_row_stats(v[q], e.lnd, lane, mean, den);
      if (lane == 0) {
        lnst[2 * rr] = mean;
        lnst[2 * rr + 1] = den;
      }
    }
    __syncthreads();
    const int hh = lane >> 5;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int row = (mt0 + mt) * 32 + r;
      const bool row_ok = row < e.m;
      const float mean = lnst[2 * (mt * 32 + r)], den = lnst[2 * (mt * 32 + r) + 1];
      const float* xr = e.lnx + (size_t)(row_ok ? row : 0) * e.lnd;
#pragma unroll
      for (int i = 0; i < PER; ++i)
#pragma unroll
        for (int blk = 0; blk < 2; ++blk)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) {
            const int k0 = (bp0 + i) * 64 + blk * 32 + kk * 16 + 8 * hh;
            half8 hi, lo;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              hi[j] = (_Float16)0.0f;
              lo[j] = (_Float16)0.0f;
            }
            if (i < cnt && row_ok && k0 < e.lnd) {
              const floatx4 x0 = *reinterpret_cast<const floatx4*>(xr + k0);
              const floatx4 x1 = *reinterpret_cast<const floatx4*>(xr + k0 + 4);
              const floatx4 g0 = *reinterpret_cast<const floatx4*>(e.lng + k0);
              const floatx4 g1 = *reinterpret_cast<const floatx4*>(e.lng + k0 + 4);
              const floatx4 b0 = *reinterpret_cast<const floatx4*>(e.lnb + k0);
              const floatx4 b1 = *reinterpret_cast<const floatx4*>(e.lnb + k0 + 4);
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                _Float16 h0, l0, h1, l1;
                split_act(ln_apply(x0[j], mean, den, g0[j], b0[j]), h0, l0);
                split_act(ln_apply(x1[j], mean, den, g1[j], b1[j]), h1, l1);
                hi[j] = h0;
                lo[j] = l0;
                hi[4 + j] = h1;
                lo[4 + j] = l1;
              }
            }
            a[mt][i][blk][kk][0] = hi;
            if constexpr (NS == 2) a[mt][i][blk][kk][NS - 1] = lo;
          }
    }
  } else {
    const size_t slab = (size_t)nbp * 2 * 2 * NS * 1024;  // bytes of one m-tile (kbp = 2 nbp)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const __amdgpu_buffer_rsrc_t ra = brsrc(reinterpret_cast<const uint8_t*>(at) + (mt0 + mt) * slab + (size_t)bp0 * 4 * NS * 1024,
                                              (uint32_t)cnt * 4 * NS * 1024);
      const bool row_ok = (mt0 + mt) * 32 + r < e.m;
#pragma unroll
      for (int i = 0; i < PER; ++i)
#pragma unroll
        for (int blk = 0; blk < 2; ++blk)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int q = 0; q < NS; ++q) {
              const int frag = ((2 * i + blk) * 2 + kk) * NS + q;
              a[mt][i][blk][kk][q] = kDiag == 2 ? half8{} : bload_h8<0>(ra, row_ok ? frag * 1024 + lane * 16 : kOob);
            }
    }
  }

  // LayerNorm fold, consumer: the row statistics from its tile statistics
  // (lnf_merge_tiles, wq4_lnmath.hpp)
  float* lnf_mu = reinterpret_cast<float*>(smem + decode_lds_bytes_dev(W) + 2 * 64 * 4);  // [32]
  float* lnf_den = lnf_mu + 32;                                                           // [32]
  float* lnf_x = lnf_den + 32;                                                            // [32][33]
  if constexpr (W == 8) {
    if (e.lnf_stats_in) {
      float m_a, den_a;
      lnf_merge_tiles<kLnfPer>(lnf_st, lnf_part, e.lnf_tiles, m_a, den_a);
      if (lnf_part == 0) {
        lnf_mu[lnf_row] = m_a;
        lnf_den[lnf_row] = den_a;
      }
    }
  }

  if constexpr (WQ4_STAMP && W == 8) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st_[1] = dstamp_rt();
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    floatx16 acc0, acc1;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      acc0[i] = 0.0f;
      acc1[i] = 0.0f;
    }
    // block-scaled form: accumulator elements j < jmax hold this m-tile's
    // real rows (element j: row (j & 3) + 8 (j >> 2) + 4 h); the rest stay 0
    // and are never stored.  Wave-uniform, and a row's arithmetic does not
    // depend on it.
    const int mrows = e.m - (mt0 + mt) * 32;
    const int jmax = mrows <= 8 ? 4 : mrows <= 16 ? 8 : mrows <= 24 ? 12 : 16;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      if constexpr (WQ4_DECODE_BS && WK == kWeightsQ4 && NS == 2) {
        if (kDiag != 1 && i < cnt) {
#pragma unroll
          for (int blk = 0; blk < 2; ++blk) {
            const half8 q0 = deq8(br[i][0][blk * 2 + 0]);  // exact q - 8, k-half 0 / 1
            const half8 q1 = deq8(br[i][0][blk * 2 + 1]);
            const float d = (float)__builtin_bit_cast(_Float16, (uint16_t)(blk ? (bs[i] >> 16) : (bs[i] & 0xffffu)));
            floatx16 t = mfma32(a[mt][i][blk][0][0], q0, floatx16{});
            t = mfma32(a[mt][i][blk][0][1], q0, t);
            t = mfma32(a[mt][i][blk][1][0], q1, t);
            t = mfma32(a[mt][i][blk][1][1], q1, t);
            floatx16& acc = blk ? acc1 : acc0;  // two chains: even / odd blocks
#pragma unroll
            for (int j = 0; j < 16; ++j)
              if (j < jmax) acc[j] = fmaf(t[j], d, acc[j]);
          }
        }
        continue;
      }
      if (kDiag != 1 && i < cnt) {
#pragma unroll
        for (int blk = 0; blk < 2; ++blk) {
          half8 bh0, bl0, bh1, bl1;
          if constexpr (WK == kWeightsF16) {
            bh0 = __builtin_bit_cast(half8, br[i][blk * 2 + 0]);
            bh1 = __builtin_bit_cast(half8, br[i][blk * 2 + 1]);
          } else {
            const uint32_t dbits = blk ? (bs[i] >> 16) : (bs[i] & 0xffffu);
            deq_scaled<NS>(br[i][0][blk * 2 + 0], dbits, bh0, bl0);
            deq_scaled<NS>(br[i][0][blk * 2 + 1], dbits, bh1, bl1);
          }
          acc0 = mfma32(a[mt][i][blk][0][0], bh0, acc0);
          acc1 = mfma32(a[mt][i][blk][1][0], bh1, acc1);
          if constexpr (NS == 2) {
            acc0 = mfma32(a[mt][i][blk][0][1], bh0, acc0);
            acc1 = mfma32(a[mt][i][blk][1][1], bh1, acc1);
            if constexpr (WK != kWeightsF16) {
              acc0 = mfma32(a[mt][i][blk][0][0], bl0, acc0);
              acc1 = mfma32(a[mt][i][blk][1][0], bl1, acc1);
            }
          }
        }
      }
    }
    floatx16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = acc0[i] + acc1[i];

    if constexpr (kDiag == 4) {  // diagnostics: no reduction / epilogue at all
      if (acc[0] == 12345.0f) e.out[0] = acc[1];
      return;
    }
    if constexpr (W == 8) {
      // whole K in this workgroup: every wave finalises 2 of the 16
      // accumulator registers (same wave-order sum as the 4-wave path) and
      // applies their epilogue -- the reduction and epilogue run 8-wide
      if constexpr (WQ4_STAMP) st_[2] = dstamp_rt();
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (i < jmax) red[(wave * 16 + i) * 64 + lane] = acc[i];  // registers of real rows only
      __syncthreads();
      if constexpr (WQ4_STAMP) st_[3] = dstamp_rt();
      const int h = lane >> 5;
      const int col = nt * 32 + r;
      float v[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int i = 2 * wave + q;
        v[q] = 0.0f;  // rows past M: 0 (never stored)
        if (i < jmax) {
          v[q] = red[i * 64 + lane];
#pragma unroll
          for (int w = 1; w < W; ++w) v[q] = v[q] + red[(w * 16 + i) * 64 + lane];
        }
      }
      typedef __attribute__((address_space(1))) int gint;
      gint* ctr = (gint*)(counters + nt);
      if (ks > 1) {
        // split-K: every wave publishes its 2 registers write-through (sc1),
        // drains, and one lane takes the ticket; the slice drawing ks-1 sums
        // the slabs in slice order (cdna_hip_programming.md Guideline 16, R1)
        const __amdgpu_buffer_rsrc_t rs = brsrc(part + ((size_t)nt * ks + slice) * 1024, 4096);
        const floatx2 f2 = {v[0], v[1]};
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, f2), rs, (wave * 64 + lane) * 8, 0, 16);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // every storing wave drained before the ticket; red[] free again
        if (tid == 0) {
          const int prev = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          red[0] = prev == ks - 1 ? 1.0f : 0.0f;
        }
        __syncthreads();
        if (red[0] == 0.0f) return;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler-only: loads stay below the ticket
        const __amdgpu_buffer_rsrc_t ra = brsrc(part + (size_t)nt * ks * 1024, (uint32_t)ks * 4096);
        u32x2 pv[kDecodeMaxKs];
#pragma unroll
        for (int sl = 0; sl < kDecodeMaxKs; ++sl)
          pv[sl] = __builtin_amdgcn_raw_buffer_load_b64(ra, sl < ks ? sl * 4096 + (wave * 64 + lane) * 8 : kOob, 0,
                                                        16);
        floatx2 t = __builtin_bit_cast(floatx2, pv[0]);
#pragma unroll
        for (int sl = 1; sl < kDecodeMaxKs; ++sl)
          if (sl < ks) t = t + __builtin_bit_cast(floatx2, pv[sl]);
        v[0] = t[0];
        v[1] = t[1];
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int i = 2 * wave + q;
        const int rl = acc_row(i, h);
        const int row = (mt0 + mt) * 32 + rl;
        float a = v[q] * cs;
        if (e.lnf_stats_in) a = lnf_apply(a, lnf_mu[rl], pre_wg, lnf_den[rl]);  // LayerNorm fold, consumer
        if constexpr (EPI == kEpiTiled) {
          stage[rl * kStageLd + r] = (row < e.m && col < e.n) ? epi_value_pre(a, pre_bias, pre_res[q], e) : 0.0f;
        } else if constexpr (EPI == kEpiHeadMajor) {
          if (row < e.m && col < e.n) e.out[out_index(e, row, col)] = epi_value(a, row, col, e);
        } else {
          const bool ok = row < e.m && col < e.n;
          const float y = epi_value_pre(a, pre_bias, pre_res[q], e);
          if (ok) e.out[(size_t)row * e.ldo + col] = y;
          if (e.lnf_at) {  // LayerNorm fold, producer: x (statistics) and x * gamma (next operand)
            lnf_x[rl * 33 + r] = ok ? y : 0.0f;
            stage[rl * kStageLd + r] = ok ? y * pre_g : 0.0f;
          }
        }
      }
      if constexpr (EPI == kEpiTiled) {
        __syncthreads();
        if (wave == 0) store_tiled_slab<NS, 1>(stage, e, mt0 + mt, nt, lane);
      }
      if constexpr (EPI == kEpiF32) {
        if (e.lnf_at) {
          __syncthreads();
          if (wave == 0) {
            EpiArgs e2 = e;
            e2.out_tiled = e.lnf_at;
            e2.nbp_next = e.lnf_nbp;
            store_tiled_slab<NS, 1>(stage, e2, mt0 + mt, nt, lane);
          } else if (wave == 1) {  // lane (row, half): the 16-column tile statistics
            const int rl = lane & 31, hf = lane >> 5, row = (mt0 + mt) * 32 + rl;
            if (row < e.m && 2 * nt + hf < e.n / 16) {  // never a slot past N / 16
              float sum = 0.0f;
#pragma unroll
              for (int c = 0; c < 16; ++c) sum += lnf_x[rl * 33 + 16 * hf + c];
              const float mean = sum * (1.0f / 16.0f);
              float m2 = 0.0f;
#pragma unroll
              for (int c = 0; c < 16; ++c) {
                const float d = lnf_x[rl * 33 + 16 * hf + c] - mean;
                m2 += d * d;
              }
              *reinterpret_cast<floatx2*>(e.lnf_stats_out + ((size_t)row * (e.n / 16) + 2 * nt + hf) * 2) =
                  floatx2{mean, m2};
            }
          }
        }
      }
      if (ks > 1 && tid == 0) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
#if WQ4_STAMP
      if (tid == 0 && e.stamp_id >= 0 && e.stamp_id < kDStampLaunches && blockIdx.x < kDStampWgs) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        st_[4] = dstamp_rt();
        st_[6] = dstamp_cyc();
        st_[7] = (unsigned long long)cnt;
        for (int q = 0; q < kDStampSlots; ++q)
          g_dec_stamps[((size_t)e.stamp_id * kDStampWgs + blockIdx.x) * kDStampSlots + q] = st_[q];
      }
#endif
      continue;  // MT == 1 for 8-wave plans
    }

    // fixed-order reduction over the W waves
    if (wave > 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i) red[((wave - 1) * 16 + i) * 64 + lane] = acc[i];
    }
    __syncthreads();
    if (wave == 0) {
      floatx16 s = acc;
#pragma unroll
      for (int w = 0; w < W - 1; ++w)
#pragma unroll
        for (int i = 0; i < 16; ++i) s[i] = s[i] + red[(w * 16 + i) * 64 + lane];
      if (W == 8 || ks == 1) {  // 8-wave plan: always the whole K (no split-K code at all)
        decode_epilogue<NS, EPI>(s, cs, mt0 + mt, nt, lane, stage, e);
      } else {
        // write-through (sc1) slab stores: visible device-wide once drained,
        // no release fence (cdna_hip_programming.md Guideline 16, R1)
        const __amdgpu_buffer_rsrc_t rs = brsrc(part + (((size_t)nt * mtiles + mt) * ks + slice) * 1024, 4096);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          // whole-vector bit casts only: clang's __builtin_bit_cast of an
          // ext-vector ELEMENT reads element 0 (ROCm 7.2)
          const floatx4 f = {s[4 * q], s[4 * q + 1], s[4 * q + 2], s[4 * q + 3]};
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, f), rs, (q * 64 + lane) * 16, 0, 16);
        }
      }
    }
    __syncthreads();
  }
  if (W == 8 || ks == 1 || wave != 0) return;

  // split-K fix-up: wave 0 of each slice drained its sc1 stores, one ticket
  // per slice; the slice drawing ks-1 sums all slabs in slice order with sc1
  // loads (no acquire needed: every handed-off byte is stored and loaded sc1).
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  typedef __attribute__((address_space(1))) int gint;
  gint* ctr = (gint*)(counters + nt);
  int prev = 0;
  if (lane == 0) prev = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  prev = __shfl(prev, 0);
  if (prev != ks - 1) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler-only: keep the loads below the ticket
#pragma unroll
  for (int mt = 0; mt < mtiles; ++mt) {
    const __amdgpu_buffer_rsrc_t rs = brsrc(part + ((size_t)nt * mtiles + mt) * ks * 1024, (uint32_t)ks * 4096);
    u32x4 v[kDecodeMaxKs][4];  // every slab load in flight at once
#pragma unroll
    for (int sl = 0; sl < kDecodeMaxKs; ++sl)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        v[sl][q] = __builtin_amdgcn_raw_buffer_load_b128(rs, sl < ks ? sl * 4096 + (q * 64 + lane) * 16 : kOob, 0, 16);
    floatx16 s;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const floatx4 f = __builtin_bit_cast(floatx4, v[0][q]);
#pragma unroll
      for (int j = 0; j < 4; ++j) s[4 * q + j] = f[j];
    }
#pragma unroll
    for (int sl = 1; sl < kDecodeMaxKs; ++sl)
      if (sl < ks) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const floatx4 f = __builtin_bit_cast(floatx4, v[sl][q]);
#pragma unroll
          for (int j = 0; j < 4; ++j) s[4 * q + j] = s[4 * q + j] + f[j];
        }
      }
    decode_epilogue<NS, EPI>(s, cs, mt0 + mt, nt, lane, stage, e);
  }
  if (lane == 0) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
}

// ------------------------------------------------------------------------
// Launchers.
// ------------------------------------------------------------------------
static size_t prefill_lds_bytes(int ns, int epi) {
  const size_t a = (size_t)2 * kPrefillTM * 4096 * ns;
  const size_t s = epi == kEpiTiled ? (size_t)4 * 32 * kStageLd * 4 : 0;
  return a > s ? a : s;
}

static size_t decode_lds_bytes(int w) { return decode_lds_bytes_all(w); }



DecodePlan plan_decode(int64_t ntiles, int64_t nbp, int mreal) {
  // Smallest per-wave depth whose grid still covers ~all CUs, then balance.
  static const int pers[3] = {4, 2, 1};
  DecodePlan p{1, 1, 1, kDecodeWaves};
  (void)mreal;  // the plan depends on (N, K) only: batch-invariant rows
  // K <= 1536: one 8-wave workgroup per n-tile holds the whole K range (no
  // split-K hand-off at all); the grid is N / 32 workgroups.  Measured and
  // not kept (DESIGN.md dead ends): 4-wave plans and more, smaller K slices
  // (fewer block pairs per wave) for every Whisper decode shape.
  constexpr int per8 = kDecodeMaxPer8;
  if (nbp <= 8 * per8 * kDecodeMaxKs && ntiles <= kDecodeMaxTiles) {
    // larger K: the same 8-wave workgroups over ks K slices (sc1 slabs +
    // last-arriver merge); ks depends on K only
    p.w = 8;
    p.ks = (int)((nbp + 8 * per8 - 1) / (8 * per8));
    while (p.ks > 1 && ntiles * p.ks * 1024 > (int64_t)kDecodeWsFloats) --p.ks;  // workspace bound
    p.chunk = (int)((nbp + 8 * p.ks - 1) / (8 * p.ks));
    p.per = p.chunk;
    if (p.per <= kDecodeMaxPer8) return p;
    p = DecodePlan{1, 1, 1, kDecodeWaves};  // does not fit: 4-wave plan below
  }
  const int max_per = kDecodeMaxPer;
  int per = 1;
  for (int c : pers) {
    if (c > max_per) continue;
    const int64_t ks = (nbp + (int64_t)kDecodeWaves * c - 1) / ((int64_t)kDecodeWaves * c);
    if (ntiles * ks >= 192) {
      per = c;
      break;
    }
  }
  int64_t ks = (nbp + (int64_t)kDecodeWaves * per - 1) / ((int64_t)kDecodeWaves * per);
  if (ks > kDecodeMaxKs) ks = kDecodeMaxKs;
  while (ks > 1 && ntiles * ks * 2 * 1024 > (int64_t)kDecodeWsFloats) --ks;  // workspace bound (2 m-tiles)
  if (ntiles > kDecodeMaxTiles) ks = 1;
  int64_t chunk = (nbp + (int64_t)kDecodeWaves * ks - 1) / ((int64_t)kDecodeWaves * ks);
  while (chunk > per) per *= 2;  // ks shrank: deepen the waves
  p.per = per;
  p.ks = (int)ks;
  p.chunk = (int)chunk;
  return p;
}

__global__ __launch_bounds__(256) void act_max_kernel(const float* __restrict__ x, int M, int K, int ld,
                                                      unsigned* __restrict__ max_bits) {
  float mx = 0.0f;
  for (int m = blockIdx.x; m < M; m += gridDim.x)
    for (int c = threadIdx.x; c < K; c += 256) mx = fmaxf(mx, fabsf(x[(size_t)m * ld + c]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  // |x| >= 0: the f32 bit patterns order like the values, so an unsigned
  // maximum (a vector atomic, order-independent) gives the exact maximum
  if ((threadIdx.x & 63) == 0)
    __hip_atomic_fetch_max(max_bits, __float_as_uint(mx), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void act_scale_finish_kernel(float* __restrict__ out) {
  const float mx = __uint_as_float(reinterpret_cast<const unsigned*>(out)[2]);
  int e = 4;  // the internal producers' 2^4, unless the range needs less
  if (mx > 0.0f && mx < INFINITY) e = min(4, (int)floorf(log2f(16384.0f / mx)));
  out[0] = ldexpf(1.0f, e);
  out[1] = ldexpf(1.0f, -e);
}

hipError_t launch_act_scale(const float* x, int M, int K, int ld, float* out, hipStream_t st) {
  // out[2] holds the running maximum's bits; zeroed per call on the stream
  hipError_t e = hipMemsetAsync(out + 2, 0, sizeof(unsigned), st);
  if (e != hipSuccess) return e;
  const int grid = M < 2048 ? (M < 1 ? 1 : M) : 2048;
  hipLaunchKernelGGL(act_max_kernel, dim3(grid), dim3(256), 0, st, x, M, K, ld,
                     reinterpret_cast<unsigned*>(out + 2));
  hipLaunchKernelGGL(act_scale_finish_kernel, dim3(1), dim3(1), 0, st, out);
  return hipGetLastError();
}

hipError_t launch_tile_activations(const float* x, _Float16* at, int M, int K, int ld, int ns, hipStream_t st,
                                   const float* scale) {
  const int mtiles = (int)(round_up(M < 1 ? 1 : M, kMPad) / kMTile);
  const int kbp = (int)(((K / kBlock) + 1) / 2) * 2;
  const int64_t total = (int64_t)mtiles * kbp * 2 * 64;
  const int grid = (int)((total + 255) / 256);
  const bool aligned = (ld % 4 == 0) && ((reinterpret_cast<uintptr_t>(x) & 15u) == 0);
#define WQ4_TILE(NS_, AL_)                                                                                   \
  hipLaunchKernelGGL((tile_activations_kernel<NS_, AL_>), dim3(grid), dim3(256), 0, st, x, at, M, K, ld, mtiles, \
                     kbp, scale)
  if (ns == 2) {
    if (aligned) WQ4_TILE(2, true); else WQ4_TILE(2, false);
  } else {
    if (aligned) WQ4_TILE(1, true); else WQ4_TILE(1, false);
  }
#undef WQ4_TILE
  return hipGetLastError();
}

// Stamp bookkeeping (WQ4_STAMP builds): launch slot -> (N, K, rows).
static int g_dstamp_next = 0;
static int g_dstamp_meta[kDStampLaunches][3];

template <int NS, int EPI, int WK>
static hipError_t launch_gemm_t(const Q4Geom& g, const uint8_t* nib, const uint32_t* sc, const float* cs,
                                const _Float16* at, int rows, const EpiArgs& e, const DecodeWs* ws,
                                hipStream_t st) {
  const int mtiles = (int)(round_up(rows < 1 ? 1 : rows, kMPad) / kMTile);
  const int mreal0 = (int)((rows + kMTile - 1) / kMTile);
  const DecodePlan p = plan_decode(g.ntiles, g.nbp, 2);
  const bool dec_ok = ws && mreal0 <= kDecodeMaxMTiles && p.per <= (p.w == 8 ? kDecodeMaxPer8 : kDecodeMaxPer);
  if (e.lnx) {  // LayerNorm-on-load: 8-wave decode plans only (the caller falls back otherwise)
    if (!dec_ok || p.w != 8) return hipErrorNotSupported;
    const dim3 grid((unsigned)(g.ntiles * p.ks));
#define WQ4_DECLN(PER_)                                                                                      \
  hipLaunchKernelGGL((q4_gemm_decode_kernel<NS, EPI, PER_, 1, 8, WK, true>), grid, dim3(512), decode_lds_bytes(8), \
                     st, nib, sc, cs, at, mt0, (int)g.nbp, p.ks, p.chunk, ws->part, ws->counters, e)
    for (int mt0 = 0; mt0 < mreal0; ++mt0) {
      if (p.per == 1) WQ4_DECLN(1);
      else if (p.per == 2) WQ4_DECLN(2);
      else WQ4_DECLN(3);
    }
#undef WQ4_DECLN
    return hipGetLastError();
  }
  if (dec_ok) {
    const dim3 grid((unsigned)(g.ntiles * p.ks));
    EpiArgs es = e;
    es.stamp_id = -1;
    if (WQ4_STAMP && p.w == 8 && g_dstamp_next < kDStampLaunches) {
      es.stamp_id = g_dstamp_next++;
      g_dstamp_meta[es.stamp_id][0] = (int)g.n;
      g_dstamp_meta[es.stamp_id][1] = (int)g.k;
      g_dstamp_meta[es.stamp_id][2] = rows;
    }
#define WQ4_DEC(PER_, MT_, W_)                                                                               \
  hipLaunchKernelGGL((q4_gemm_decode_kernel<NS, EPI, PER_, MT_, W_, WK>), grid, dim3(64 * W_), decode_lds_bytes(W_), \
                     st, nib, sc, cs, at, mt0, (int)g.nbp, p.ks, p.chunk, ws->part, ws->counters, es)
    // 8-wave plans: one m-tile per launch (two would not fit the registers);
    // 4-wave plans: m-tiles in launches of <= 2.  Launches on one stream
    // complete in order, so they share the workspace and counters.
    if (p.w == 8) {
      for (int mt0 = 0; mt0 < mreal0; ++mt0) {
        if (p.per == 1) WQ4_DEC(1, 1, 8);
        else if (p.per == 2) WQ4_DEC(2, 1, 8);
        else WQ4_DEC(3, 1, 8);
      }
    } else {
      for (int mt0 = 0; mt0 < mreal0; mt0 += 2) {
        if (mreal0 - mt0 == 1) {
          if (p.per == 1) WQ4_DEC(1, 1, 4);
          else if (p.per == 2) WQ4_DEC(2, 1, 4);
          else WQ4_DEC(4, 1, 4);
        } else {
          if (p.per == 1) WQ4_DEC(1, 2, 4);
          else if (p.per == 2) WQ4_DEC(2, 2, 4);
          else WQ4_DEC(4, 2, 4);
        }
      }
    }
#undef WQ4_DEC
  } else if (const int geo = enc_gemm_pick(g, rows, EPI, NS, WK)) {
    if (geo == 5) return launch_wide_gemm(g, nib, sc, cs, at, rows, e, EPI, NS, st);
    return launch_enc_gemm(g, nib, sc, cs, at, rows, e, EPI, geo, st);
  } else {
    const int ngroups = (int)((g.ntiles + 4 * kPrefillTN - 1) / (4 * kPrefillTN));
    const int mgroups = mtiles / kPrefillTM;
    hipLaunchKernelGGL((q4_gemm_prefill_kernel<NS, EPI, WK>), dim3((unsigned)(ngroups * mgroups)), dim3(256),
                       prefill_lds_bytes(NS, EPI), st, nib, sc, cs, at, mtiles, (int)g.nbp, (int)g.ntiles, e);
  }
  return hipGetLastError();
}

bool decode_ln_supported(const Q4Geom& g, int rows) {
  const int mreal0 = (int)((rows + kMTile - 1) / kMTile);
  const DecodePlan p = plan_decode(g.ntiles, g.nbp, 2);
  return rows >= 1 && mreal0 <= kDecodeMaxMTiles && p.w == 8 && p.per <= kDecodeMaxPer8;
}

hipError_t launch_q4_gemm(const Q4Geom& g, const uint8_t* nib, const uint32_t* sc, const float* colscale,
                          const _Float16* at, int rows, const EpiArgs& e, int epi_mode, int ns, const DecodeWs* ws,
                          hipStream_t st, int wtype) {
#define WQ4_GEMM(NS_, WK_)                                                                                   \
  switch (epi_mode) {                                                                                        \
    case kEpiF32: return launch_gemm_t<NS_, kEpiF32, WK_>(g, nib, sc, colscale, at, rows, e, ws, st);        \
    case kEpiTiled: return launch_gemm_t<NS_, kEpiTiled, WK_>(g, nib, sc, colscale, at, rows, e, ws, st);    \
    default: return launch_gemm_t<NS_, kEpiHeadMajor, WK_>(g, nib, sc, colscale, at, rows, e, ws, st);       \
  }
  if (wtype == kWeightsF16) {
    if (ns == 2) WQ4_GEMM(2, kWeightsF16);
    WQ4_GEMM(1, kWeightsF16);
  }
  if (ns == 2) WQ4_GEMM(2, kWeightsQ4);
  WQ4_GEMM(1, kWeightsQ4);
#undef WQ4_GEMM
}

}  // namespace wq4

// Timing diagnostics (WQ4_STAMP builds only; returns 0 launches otherwise):
// copies [launches][kDStampWgs][8] stamps of the 8-wave decode kernel and
// [launches][3] (N, K, rows).
extern "C" int wq4_diag_decode_stamps(unsigned long long* out, int* meta, int max_launches) {
#if WQ4_STAMP
  const int n = wq4::g_dstamp_next < max_launches ? wq4::g_dstamp_next : max_launches;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(wq4::g_dec_stamps),
                          (size_t)n * wq4::kDStampWgs * wq4::kDStampSlots * sizeof(unsigned long long)) != hipSuccess)
    return -1;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < 3; ++j) meta[i * 3 + j] = wq4::g_dstamp_meta[i][j];
  return n;
#else
  (void)out;
  (void)meta;
  (void)max_launches;
  return 0;
#endif
}
