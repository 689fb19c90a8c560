// wa_xattn.hip -- decoder cross-attention computed over the encoder output
// itself (no per-layer cross K/V caches).
//
// Reference: CrossAttention::forward_with_cache (src/model/attention.rs:
// 204-236) + scaled_dot_product_attention (:243-298):
//     K = enc Wk^T + bk,  V = enc Wv^T + bv   (cached per layer, [T, D])
//     out_h = softmax(q_h K_h^T / 8) V_h
// Restated (exact in real arithmetic):
//     qt_h  = Wk_h^T q_h / 8                        [D]    (xattn_q_kernel)
//     s_t   = qt_h . enc_t     (q_h . bk_h is the same for every t: softmax-
//                               invariant, dropped)
//     Z_h   = sum_t softmax(s)_t enc_t              [D]    (xattn_main_kernel)
//     out_h = Wv_h Z_h + bv_h  (softmax weights sum to 1) (xattn_out_kernel)
// Every layer streams the clip's encoder output once -- T*D values shared by
// all heads -- instead of its K and V (2*T*D), halving the HBM bytes of the
// decode step's dominant kernel, and the 32 layers' K/V caches (15.7 GB for
// 32 Large-V3 clips) and their projection GEMMs disappear.
//
// Numerics: enc and qt are f16 hi/lo pairs (x = hi + lo to 2^-22) and every
// product runs as three f16 MFMAs (hi*hi + lo*hi + hi*lo, f32 accumulate) --
// the f32-faithful arithmetic of the Q4 GEMMs; NS = 1 (WQ4_PREC_F16) keeps
// only the hi planes.  Softmax is the online (flash) form in f32 with expf.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "../wq4_device.hpp"
#include "../wq4_lnmath.hpp"
#include "wa_kernels.hpp"

namespace wa {
namespace {

using wq4::atile_store4;
using wq4::attn_store4;
using wq4::kbp_of;
using wq4::split_f16;
using wq4::half2v;
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx2 __attribute__((ext_vector_type(2)));

constexpr int kWtQ4 = 0, kWtF16 = 1;  // raw weight formats (wa_model wtype)
constexpr int kTc = 16;          // keys (encoder frames) per sub-chunk
constexpr int kMaxD = 1280;
constexpr float kXqScale = 0.125f * 1.4426950408889634f;  // 1 / sqrt(64) * log2(e)
// Operand scales of the f16-pair MFMAs (the MFMAs flush f16 subnormal inputs:
// wq4_device.hpp split_act), all powers of two, undone in f32 (exact):
//   xattn_q   q rows x 2^4 (split_act), Wk x 2^12 (|w| < 16), product x 2^-16
//   main      qt x 2^5, encoder planes x 2^5 (|x| < 2047): scores x 2^10;
//             p in (0, 2] x 2^14 (the lazy reference maximum, softmax_entry): Z x 2^19
//   out       Zn x 2^5, Wv scale d x 2^12 (d < 16): product x 2^-17
constexpr float kWkScale = 4096.0f, kXqInv = 1.0f / (16.0f * 4096.0f);
constexpr float kQtScale = 32.0f, kEncScale = 32.0f, kSInv = 1.0f / 1024.0f;
constexpr float kPScale = 16384.0f, kZInv = 1.0f / (16384.0f * 32.0f);
constexpr float kZnScale = 32.0f, kWvScale = 4096.0f, kOutInv = 1.0f / (32.0f * 4096.0f);
#ifndef WA_XATTN_SPLITS  // compile-time only: tuning builds (A/B: scripts/gpu.sh libs)
#define WA_XATTN_SPLITS 8
#endif
// Frame ranges per query row.  Measured: 8 beat 4, 6, 12 and 16 in round 1;
// in round 2's model (two concurrent decode groups of 16 clips) 12 and 16 ran
// the isolated 16-clip launch faster (50.5 us vs 55.7 at 12) but the decode
// slower (926 / 1073 ms vs 873): more workgroups crowd out the other group.
// Round 5 (after the xattn_out merge rewrite): 12 splits 30.1 vs 36.2 us
// isolated at 16 rows, decode 909 vs 856 ms.
constexpr int kXattnSplits = WA_XATTN_SPLITS;
// Timing attribution builds of tools/xattn_micro.hip only (wrong results):
// 1 = no encoder fetch after the first sub-chunk, 2 = no Z phase, 3 = no
// score MFMAs, 4 = no softmax, 5 = never rescale Z, 6 = no barrier after the
// score partials, 7 = no barrier after the softmax, 8 = softmax computed but
// P stored as zeros, 9 = no softmax, P = 1, 10 = no sub-chunk loop (fixed
// cost: qt loads, LDS init, partial stores).  0 (the product)
// compiles none of them.
#ifndef WA_XATTN_DIAG
#define WA_XATTN_DIAG 0
#endif
// Frames whose encoder-plane sub-chunks xattn_main loads with the default
// cache policy; the rest use WA_XATTN_STREAM_AUX (nontemporal).  >= 1500:
// all default (tuning builds: scripts/gpu.sh libs).
#ifndef WA_XATTN_CACHE_FRAMES
#define WA_XATTN_CACHE_FRAMES 1500
#endif
#ifndef WA_XATTN_STREAM_AUX
#define WA_XATTN_STREAM_AUX 2
#endif
constexpr int kMaxFrames = 1500;
// WA_XATTN_STAMP (tools/xattn_micro.hip only): the clock at the phase
// boundaries of every sub-chunk of workgroup (0, 0), waves 0 and NW - 1,
// into g_xstamp (read back with hipMemcpyFromSymbol; results unchanged).
#ifndef WA_XATTN_STAMP
#define WA_XATTN_STAMP 0
#endif
#if WA_XATTN_STAMP
constexpr int kXsPhases = 8, kXsChunks = 16;
__device__ unsigned long long g_xstamp[2][kXsChunks][kXsPhases];
#endif
// xattn_out attribution builds (tools/xattn_micro.hip only, wrong results):
// 1 = no Wv stage, 2 = no split-partial loads, 3 = no projection MFMAs.
#ifndef WA_XATTN_ODIAG
#define WA_XATTN_ODIAG 0
#endif

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __fp16 fp16x4_t __attribute__((__vector_size__(4 * sizeof(__fp16))));

// gfx950: the K=32 / K=16 forms run at twice the FLOP rate of the older
// 16x16x16 / 32x32x8 forms (same cycles per instruction, tools/mfma_cycles.hip)
__device__ __forceinline__ floatx4 mfma16x32(half8 a, half8 b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ floatx16 mfma32x16(half8 a, half8 b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
// ds_read_b64_tr_b16 (cdna_hip_programming.md T10): per 16-lane group a 4-row
// x 16-column block, lane i receiving column i (row q in element q)
__device__ __forceinline__ half4 lds_tr4(const _Float16* p) {
  return __builtin_bit_cast(half4, __builtin_amdgcn_ds_read_tr16_b64_v4f16(
                                       (__attribute__((address_space(3))) fp16x4_t*)(p)));
}

// Weight element (o, c) of a [rows, K] linear weight in its raw GGUF form:
// Q4_0 blocks (tests.rs:60-87: (nibble - 8) * d, f32) or f16.
template <int WK>
__device__ __forceinline__ void load_w32(const uint8_t* __restrict__ w, int K, int o, int kb, float* out) {
  if (WK == kWtQ4) {
    const uint16_t* blk = reinterpret_cast<const uint16_t*>(w + ((size_t)o * (K / 32) + kb) * 18);
    const float d = (float)__builtin_bit_cast(_Float16, blk[0]);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t two = blk[1 + i];  // bytes 2i, 2i+1 of the 16 nibble bytes
      out[2 * i] = (float)((int)(two & 15u) - 8) * d;
      out[2 * i + 1] = (float)((int)((two >> 8) & 15u) - 8) * d;
      out[16 + 2 * i] = (float)((int)((two >> 4) & 15u) - 8) * d;
      out[16 + 2 * i + 1] = (float)((int)((two >> 12) & 15u) - 8) * d;
    }
  } else {
    const _Float16* p = reinterpret_cast<const _Float16*>(w) + (size_t)o * K + kb * 32;
#pragma unroll
    for (int i = 0; i < 32; ++i) out[i] = (float)p[i];
  }
}

// ------------------------------------------------------------- qt = Wk^T q --
// grid (H, D / 64, ceil(R / 32)), 128 threads: 64 columns of one head for up
// to 32 rows.  qt: [R][NS][HP][D] f16 planes (rows of padded heads h >= H are
// never written: zeroed once at allocation).  out[r][c] = sum_d
// q[r][h*64+d] Wk[h*64+d][c] as a 32 x 64 x 64 f16x2 product (A = q rows
// split hi + lo from f32, B = the exact Wk values split hi + lo; the dropped
// lo * lo term is < 2^-22 relative).  The 64 x 64 Wk block is dequantised
// once into LDS transposed ([c][d], row stride 72 halves: conflict-free
// fragment reads); wave w computes columns c0 + 32 w .. + 31.
template <int NS, int WK>
__global__ __launch_bounds__(128) void xattn_q_mfma_kernel(const float* __restrict__ q, int R, int D,
                                                           const uint8_t* __restrict__ wk, int HP,
                                                           _Float16* __restrict__ qt) {
  constexpr int LD = 72;
  __shared__ __attribute__((aligned(16))) _Float16 wth[64 * LD];
  __shared__ __attribute__((aligned(16))) _Float16 wtl[64 * LD];
  const int h = blockIdx.x, c0 = blockIdx.y * 64, r0 = blockIdx.z * 32, tid = threadIdx.x;
  const int w = tid >> 6, l = tid & 63, l32 = l & 31, kh = l >> 5;
  // A fragments: row l32, d = 16 ks + 8 kh .. + 7 (rows >= R read as zeros)
  const int row = r0 + l32;
  floatx4 xa[4][2];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int u = 0; u < 2; ++u)
      xa[ks][u] = row < R ? *reinterpret_cast<const floatx4*>(q + (size_t)row * D + h * 64 + ks * 16 + 8 * kh + 4 * u)
                          : floatx4{0.0f, 0.0f, 0.0f, 0.0f};
  {  // thread (row d, block b) of the 64 x 2 Q4 blocks: exact values, split, stored transposed
    const int d = tid >> 1, b = tid & 1;
    float v[32];
    load_w32<WK>(wk, D, h * 64 + d, (c0 >> 5) + b, v);
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      _Float16 hi, lo;
      split_f16(v[i] * kWkScale, hi, lo);
      wth[(b * 32 + i) * LD + d] = hi;
      wtl[(b * 32 + i) * LD + d] = lo;
    }
  }
  half8 ah[4], al[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      _Float16 x, y;
      wq4::split_act(xa[ks][j >> 2][j & 3], x, y);
      ah[ks][j] = x;
      al[ks][j] = y;
    }
  __syncthreads();
  floatx16 acc = {};
  const int c = 32 * w + l32;
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const half8 bh = *reinterpret_cast<const half8*>(&wth[c * LD + ks * 16 + 8 * kh]);
    const half8 bl = *reinterpret_cast<const half8*>(&wtl[c * LD + ks * 16 + 8 * kh]);
    acc = mfma32x16(ah[ks], bh, acc);
    acc = mfma32x16(al[ks], bh, acc);
    acc = mfma32x16(ah[ks], bl, acc);
  }
  // acc[i]: row (i & 3) + 8 (i >> 2) + 4 kh, column c.  / sqrt(64)
  // (attention.rs:262) * log2(e): scores in base-2 units for v_exp_f32
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int r = r0 + (i & 3) + 8 * (i >> 2) + 4 * kh;
    if (r < R) {
      _Float16 x, y;
      split_f16(acc[i] * kXqInv * kXqScale * kQtScale, x, y);
      qt[(((size_t)r * NS + 0) * HP + h) * D + c0 + c] = x;
      if (NS == 2) qt[(((size_t)r * NS + 1) * HP + h) * D + c0 + c] = y;
    }
  }
}

// One (head, frame) entry of the online softmax over a 16-frame sub-chunk,
// shared by the fused and the split-phase kernels (their bits must agree):
// the head's 16 lanes form one DPP row.  Scores carry the 2^10 operand scale.
// Lazy reference maximum: the running reference M only moves when the
// sub-chunk's maximum exceeds it by more than 1 (base 2), so p <= 2 and most
// sub-chunks need no rescale of Z (alpha == 1 exactly); any reference gives
// the same softmax, and xattn_out's merge uses the references it is given.
constexpr float kLazyMax = 1024.0f;  // 1.0 in base-2 units x 2^10
__device__ __forceinline__ void softmax_entry(float sv, bool valid, float& M, float& L, float& alpha, float& p) {
  sv = valid ? sv : -INFINITY;
  const float cm = wq4::max16(sv);  // DPP butterfly over the head's 16 frames
  float mn = fmaxf(M, cm);
  if (M != -INFINITY && mn - M <= kLazyMax) mn = M;
  alpha = 1.0f;
  p = 0.0f;
  if (mn != -INFINITY) {
    alpha = __builtin_amdgcn_exp2f((M - mn) * kSInv);
    p = valid ? __builtin_amdgcn_exp2f((sv - mn) * kSInv) : 0.0f;
  }
  const float ps = wq4::sum16(p);
  L = L * alpha + ps;
  M = mn;
}

// ------------------------------------------------------------ main stream --
// grid (S, R), NW waves; wave w owns columns [w*D/NW, (w+1)*D/NW).
// Per sub-chunk of 16 frames: the frames' enc rows go to LDS; scores
// S[t][h] = sum_c enc[t][c] qt[h][c] (16x16x32 MFMA, m = frame, n = head,
// per-wave column slice, summed over waves through LDS); online softmax per
// head; Z[h][c] += P[h][t] enc[t][c] (32x32x16 MFMA, m = the 32 padded
// heads, k = the 16 frames read transposed from the same LDS image by
// ds_read_b64_tr_b16; accumulators stay in registers).  Writes per (row,
// split): Z [H][D] and (max, sum) [H].
template <int D, int HT, int NS, int NW, int PF>
__global__ __launch_bounds__(64 * NW) void xattn_main_kernel(const _Float16* __restrict__ qt,
                                                             const _Float16* __restrict__ enc, int Tq, int T,
                                                             int H, int S, int CH, float* __restrict__ zpart,
                                                             float* __restrict__ mlpart, int R) {
  constexpr int kThreads = 64 * NW;
  constexpr int CW = D / NW;      // columns per wave
  constexpr int KS = CW / 32;     // 32-column steps per wave (score k-steps = Z column tiles)
  constexpr int HP = HT * 16;     // padded heads of the score tiles
  constexpr int ROW = NS * D;     // halves per encoder row (hi plane | lo plane)
  constexpr int RS = ROW + 32;    // LDS row stride: == 16 dwords (mod 64) -> conflict-free transposed reads
  constexpr int NV = kTc * ROW / 8;  // 16-byte vectors per sub-chunk
  constexpr int NLD = (NV + kThreads - 1) / kThreads;
  constexpr int HR = HT == 2 ? 1 : HT;  // score head tiles held in registers
  static_assert(CW * NW == D && CW % 32 == 0 && HT <= 2 && (PF == 1 || PF == 2), "bad column split");
  __shared__ __attribute__((aligned(16))) _Float16 se[kTc * RS];
  __shared__ __attribute__((aligned(16))) float red[NW][HT][16][20];  // row stride 20: conflict-free b128 stores
  __shared__ __attribute__((aligned(16))) _Float16 sp[NS][32][kTc + 8];  // row stride 12 dwords: conflict-free P reads
  __shared__ float salpha[32];
  __shared__ int srescale[2];
  // heads 16..19 (H in (16, 20]) in rows 0..3, row 4 zeros: the padding lanes
  // of the second head tile read row 4 at the same immediate offsets
  __shared__ __attribute__((aligned(16))) _Float16 sq1[HT == 2 ? NS : 1][5][HT == 2 ? D + 16 : 8];

  const int s = blockIdx.x, r = blockIdx.y;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int l16 = l & 15, lq = l >> 4, l32 = l & 31, lh = l >> 5;
  const _Float16* E = enc + (size_t)(r / Tq) * T * ROW;
  const int c0 = w * CW;
  const int ts = s * CH * kTc;
  const int te = min(T, ts + CH * kTc);
  const int nch = WA_XATTN_DIAG == 10 ? 0 : te > ts ? (te - ts + kTc - 1) / kTc : 0;
#if WA_XATTN_STAMP
  const int stamp_w = (s == 0 && r == 0 && l == 0) ? (w == 0 ? 0 : w == NW - 1 ? 1 : -1) : -1;
  auto stamp = [&](int chi, int ph) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    const unsigned long long t = __builtin_readcyclecounter();
    if (stamp_w >= 0 && chi < kXsChunks) g_xstamp[stamp_w][chi][ph] = t;
  };
#else
  auto stamp = [](int, int) {};
#endif

  // qt operands (B of the score MFMA: k = column, n = head): head tile 0 in
  // registers; for H in (16, 20] the 4 heads of tile 1 from LDS (registers of
  // a mostly-padding tile would not fit beside the Z accumulators)
  half8 qb[HR][KS][NS];
#pragma unroll
  for (int ht = 0; ht < HR; ++ht)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int p = 0; p < NS; ++p)
        qb[ht][ks][p] = *reinterpret_cast<const half8*>(
            qt + (((size_t)r * NS + p) * HP + ht * 16 + l16) * D + c0 + ks * 32 + 8 * lq);
  if (HT == 2) {
    for (int i = tid; i < NS * 5 * (D / 8); i += kThreads) {
      const int p = i / (5 * (D / 8)), rem = i - p * 5 * (D / 8), hr = rem / (D / 8), c8 = rem - hr * (D / 8);
      *reinterpret_cast<half8*>(&sq1[p][hr][8 * c8]) =
          hr < 4 ? *reinterpret_cast<const half8*>(qt + (((size_t)r * NS + p) * HP + 16 + hr) * D + 8 * c8) : half8{};
    }
  }
  // rows of P past the score tiles stay 0, their alpha 1
  for (int i = tid; i < NS * 32 * (kTc + 8); i += kThreads) (&sp[0][0][0])[i] = (_Float16)(WA_XATTN_DIAG == 9 ? 1.0f : 0.0f);
  if (tid < 32) salpha[tid] = 1.0f;
  if (tid < 2) srescale[tid] = 0;

  floatx16 zacc[KS];
#pragma unroll
  for (int ct = 0; ct < KS; ++ct)
#pragma unroll
    for (int j = 0; j < 16; ++j) zacc[ct][j] = 0.0f;
  // softmax state: thread owns (head, frame) entries tid + e * kThreads
  constexpr int SMX = (HT * 256 + kThreads - 1) / kThreads;
  float M[SMX], L[SMX];
#pragma unroll
  for (int e = 0; e < SMX; ++e) {
    M[e] = -INFINITY;
    L[e] = 0.0f;
  }

  // this range's frames through a buffer resource: rows past te read as
  // zeros, no branches.  Wave w fetches only its own column slice (16 frames
  // x CW columns x NS planes): lane item v = plane-major, then frame, then
  // 16-B piece, so one load instruction covers runs of CW * 2 contiguous
  // bytes.  PF sub-chunks are in flight in registers while one is computed.
  typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
  constexpr int PPR = CW / 8;  // 16-B pieces per frame row of the slice (one plane)
  static_assert(NLD * 64 == NS * kTc * PPR, "the slice is a whole number of loads per lane");
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<_Float16*>(E + (size_t)ts * ROW), 0, nch > 0 ? (te - ts) * ROW * 2 : 0, 0x00020000);
  auto item = [&](int i, int& row, int& col) {  // col: halves within the row (plane included)
    const int v = l + 64 * i;
    const int p = v / (kTc * PPR), rem = v - p * (kTc * PPR);
    row = rem / PPR;
    col = p * D + c0 + (rem - row * PPR) * 8;
  };
  // Infinity Cache policy (WA_XATTN_CACHE_FRAMES): the sub-chunks of frames
  // below the bound load with the default policy, the rest nontemporal, so
  // that the part of every clip's planes that fits stays cached from one
  // layer to the next instead of the whole set thrashing it (both decode
  // groups' planes, 245 MB at 32 clips, against 256 MB).  Same values either
  // way; one wave-uniform branch per sub-chunk.
  auto fetch_aux = [&](u32x4v(&buf)[NLD], int chi, auto aux_c) {
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      int row, col;
      item(i, row, col);
      buf[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(((chi * kTc + row) * ROW + col) * 2), 0,
                                                     decltype(aux_c)::value);
    }
  };
  auto fetch = [&](u32x4v (&buf)[NLD], int chi) {
    if (WA_XATTN_CACHE_FRAMES >= kMaxFrames || ts + chi * kTc < WA_XATTN_CACHE_FRAMES)
      fetch_aux(buf, chi, std::integral_constant<int, 0>{});
    else
      fetch_aux(buf, chi, std::integral_constant<int, WA_XATTN_STREAM_AUX>{});
  };

  // transposed-read lane geometry (Z phase): 16-lane group g reads rows
  // 8*(g>>1) + 4*half + (0..3), columns 16*(g&1) + (0..15) of a 32-column
  // tile; lane 4q+pp addresses row q, columns 4pp..4pp+3
  const int g = l >> 4, gi = l & 15;
  const int trow = 8 * (g >> 1) + (gi >> 2), tcol = 16 * (g & 1) + 4 * (gi & 3);
  // se swizzle: frame row t keeps its 16-B slots at slot ^ sw(t), sw(t) = 3
  // for t >= 8 (a permutation inside each aligned 4-slot block; slices start
  // on 4-slot boundaries).  With the row stride == 4 slots (mod 16) it spreads
  // the score reads' 16-lane ds_read_b128 groups over all 16 slots of the
  // bank row and leaves the transposed reads' 32-lane groups and the 8-lane
  // store groups conflict-free.  Every wave touches only its own slice, so
  // the stores need no barrier before this wave's reads.
  auto sw = [](int t) { return (t & 8) ? 3 : 0; };
  const int lq_sw = lq ^ sw(l16);
  auto write_se = [&](const u32x4v (&buf)[NLD]) {
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      int row, col;
      item(i, row, col);
      *reinterpret_cast<u32x4v*>(&se[row * RS + (((col >> 3) ^ sw(row)) << 3)]) = buf[i];
    }
  };

  // scores of this wave's column slice: A = enc (m = frame, k = column) from
  // afrag(ks, plane), B = qt (k = column, n = head); partial sums to red
  const int q1row = l16 < 4 ? l16 : 4;
  auto b1frag = [&](int ks, int p) {  // heads 16..19; the padding lanes read the zero row (no exec branch)
    return *reinterpret_cast<const half8*>(&sq1[p][q1row][c0 + ks * 32 + 8 * lq]);
  };
  auto scores = [&](auto&& afrag) {
    floatx4 sacc[HT];
#pragma unroll
    for (int ht = 0; ht < HT; ++ht) sacc[ht] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int ks = 0; ks < (WA_XATTN_DIAG == 3 ? 0 : KS); ++ks) {
      half8 a[NS], b1[NS];
#pragma unroll
      for (int p = 0; p < NS; ++p) {
        a[p] = afrag(ks, p);
        if (HT > HR) b1[p] = b1frag(ks, p);
      }
#pragma unroll
      for (int ht = 0; ht < HT; ++ht) {
        half8 b[NS];
#pragma unroll
        for (int p = 0; p < NS; ++p) b[p] = ht < HR ? qb[ht < HR ? ht : 0][ks][p] : b1[p];
        sacc[ht] = mfma16x32(a[0], b[0], sacc[ht]);
        if constexpr (NS == 2) {
          sacc[ht] = mfma16x32(a[1], b[0], sacc[ht]);
          sacc[ht] = mfma16x32(a[0], b[1], sacc[ht]);
        }
      }
    }
#pragma unroll
    for (int ht = 0; ht < HT; ++ht) *reinterpret_cast<floatx4*>(&red[w][ht][l16][4 * lq]) = sacc[ht];
  };
  // online softmax of the sub-chunk's scores (red): P to sp, alpha to salpha
  auto softmax_phase = [&](int chi, int t0) {
    // entry (head tile, head, frame); 16 lanes per head
#pragma unroll
    for (int e = 0; e < SMX; ++e) {
      const int idx = tid + e * kThreads;
      if (idx < HT * 256 && WA_XATTN_DIAG != 4 && WA_XATTN_DIAG != 9) {
        const int ht = idx >> 8, hh = (idx >> 4) & 15, t = idx & 15;
        const int h = ht * 16 + hh;
        float sv = 0.0f;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) sv += red[ww][ht][hh][t];
        const bool valid = h < H && t0 + t < te;
        float alpha, p;
        softmax_entry(sv, valid, M[e], L[e], alpha, p);
        _Float16 phi, plo;
        split_f16(p * kPScale, phi, plo);  // p * 2^14: the lo half stays a normal f16 (undone at the store)
        if (WA_XATTN_DIAG == 8) phi = plo = (_Float16)0.0f;
        sp[0][h][t] = phi;
        if (NS == 2) sp[1][h][t] = plo;
        if (t == 0) salpha[h] = alpha;
        if (alpha != 1.0f && WA_XATTN_DIAG != 5) srescale[chi & 1] = 1;  // benign race: every writer stores 1
      }
    }
  };
  // the Z update of sub-chunk chi from se (rows at swizzle swz) and sp; call
  // after the barrier that follows softmax_phase(chi)
  auto z_phase = [&](int chi) {
    // alpha == 1 for every head (no running maximum moved, the steady state)
    // makes the rescale a multiplication by 1: skipped, bit-identical
    const bool rescale = srescale[chi & 1] != 0;
    if (tid == 0) srescale[(chi + 1) & 1] = 0;  // next sub-chunk's flag; its writers come after the next barrier
    // A = P (m = head, k = frame), B = enc (k = frame, n = column)
    half8 pa[NS];
#pragma unroll
    for (int p = 0; p < NS; ++p) pa[p] = *reinterpret_cast<const half8*>(&sp[p][l32][8 * lh]);
    if (rescale) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const float al = salpha[(j & 3) + 8 * (j >> 2) + 4 * lh];
#pragma unroll
        for (int ct = 0; ct < KS; ++ct) zacc[ct][j] *= al;
      }
    }
    stamp(chi, 6);
    const int tc0 = ((((tcol >> 3) ^ sw(trow)) << 3) | (tcol & 7));
    const int tc1 = ((((tcol >> 3) ^ sw(trow + 4)) << 3) | (tcol & 7));
#pragma unroll
    for (int ct = 0; ct < (WA_XATTN_DIAG == 2 ? 0 : KS); ++ct) {
      half8 eb[NS];
#pragma unroll
      for (int p = 0; p < NS; ++p) {
        const half4 x0 = lds_tr4(&se[trow * RS + p * D + c0 + ct * 32 + tc0]);
        const half4 x1 = lds_tr4(&se[(trow + 4) * RS + p * D + c0 + ct * 32 + tc1]);
        eb[p] = half8{x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
      }
      zacc[ct] = mfma32x16(pa[0], eb[0], zacc[ct]);
      if (NS == 2) {
        zacc[ct] = mfma32x16(pa[1], eb[0], zacc[ct]);
        zacc[ct] = mfma32x16(pa[0], eb[1], zacc[ct]);
      }
    }
  };
  // One sub-chunk: this wave's slice to se, the next fetch, the scores from
  // se, then one barrier for the score partials and one inside tail().
  auto step = [&](u32x4v (&buf)[NLD], int chi) {
    const int t0 = ts + chi * kTc;
    stamp(chi, 0);
    write_se(buf);
    stamp(chi, 1);
    if (chi + PF < nch && WA_XATTN_DIAG != 1) fetch(buf, chi + PF);  // in flight during the next PF sub-chunks
    scores([&](int ks, int p) {
      return *reinterpret_cast<const half8*>(&se[l16 * RS + p * D + c0 + ks * 32 + 8 * lq_sw]);
    });
    stamp(chi, 2);
    if (WA_XATTN_DIAG != 6) __syncthreads();  // every wave's score partials in red
    stamp(chi, 3);
    softmax_phase(chi, t0);
    stamp(chi, 4);
    if (WA_XATTN_DIAG != 7) __syncthreads();
    stamp(chi, 5);
    z_phase(chi);
    stamp(chi, 7);
  };
  u32x4v pre0[NLD];
  u32x4v pre1[PF == 2 ? NLD : 1];
  if (nch > 0) fetch(pre0, 0);
  __syncthreads();  // sq1, sp, salpha, srescale initialised
  if constexpr (PF == 2) {
    if (nch > 1) fetch(pre1, 1);
    for (int chi = 0; chi < nch; chi += 2) {
      step(pre0, chi);
      if (chi + 1 < nch) step(pre1, chi + 1);
    }
  } else {
    for (int chi = 0; chi < nch; ++chi) step(pre0, chi);
  }

  // partials of this (row, split)
  const size_t base = (size_t)r * S + s;
#pragma unroll
  for (int e = 0; e < SMX; ++e) {
    const int idx = tid + e * kThreads;
    if (idx < HT * 256 && (idx & 15) == 0) {
      const int h = (idx >> 8) * 16 + ((idx >> 4) & 15);
      if (h < H) {
        mlpart[(base * H + h) * 2] = M[e] * kSInv;  // unscaled base-2 maximum (xattn_out's merge)
        mlpart[(base * H + h) * 2 + 1] = L[e];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int h = (j & 3) + 8 * (j >> 2) + 4 * lh;
    if (h < H) {
#pragma unroll
      for (int ct = 0; ct < KS; ++ct) zpart[(base * H + h) * D + c0 + ct * 32 + l32] = zacc[ct][j] * kZInv;
    }
  }
}

// Wv (Q4_0) repacked once at model load into the projection's lane order,
// the same bytes as the Q4 blocks: per (head, block kb, m-tile) one u32 per
// lane -- lane l = (n = l & 15, lq = l >> 4) gets the nibbles of elements
// 8 lq .. + 7 of weight row 16 m-tile + n, element 2i in bits 8i .. 8i + 3,
// 2i + 1 in bits 8i + 4 .. 8i + 7 -- then the 16 rows' f16 scales:
// [h][kb][m-tile][64 u32 | 16 u16].  xattn_out loads them straight into
// registers: no LDS stage, no per-launch byte shuffling.
constexpr int kWvPackU32 = 64 + 8;  // u32 words per (h, kb, m-tile)
__global__ __launch_bounds__(256) void wv_pack_kernel(const uint8_t* __restrict__ wv, int H, int D,
                                                      uint32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int nkb = D / 32;
  if (i >= (int64_t)H * nkb * 4 * 64) return;
  const int l = (int)(i & 63), mt = (int)((i >> 6) & 3);
  const int64_t hk = i >> 8;
  const int kb = (int)(hk % nkb), h = (int)(hk / nkb);
  const int n = l & 15, lq = l >> 4;
  const uint8_t* blk = wv + ((size_t)h * 64 + mt * 16 + n) * ((size_t)nkb * 18) + (size_t)kb * 18;
  // element e of the block: low nibble of byte 2 + e (e < 16), else high nibble of byte 2 + e - 16
  uint32_t wd = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int e = 8 * lq + j;
    const uint32_t q = e < 16 ? (blk[2 + e] & 15u) : (blk[2 + e - 16] >> 4);
    wd |= q << (4 * j);
  }
  uint32_t* o = out + (((size_t)h * nkb + kb) * 4 + mt) * kWvPackU32;
  o[l] = wd;
  if (lq == 0) reinterpret_cast<uint16_t*>(o + 64)[n] = (uint16_t)(blk[0] | (blk[1] << 8));
}

// ---------------------------------------- merge + out = Wv Zn + bv --
// grid (H, ceil(R / RPW)), 512 threads: the head's 64 raw Wv rows (46 KB of
// Q4_0 blocks, LDS-DMA) and RPW rows of Zn in LDS.  Q4 weights: the
// projection runs on 16x16x32 MFMA (f16x2, waves split the K blocks, 8
// partials per output); f16 weights: thread (row pair d, d + 32; blocks b,
// b + 16, b + 32) on VALU, 16 partials.  The partials are added through LDS
// in a fixed order and out[r][h*64 + d] + bv goes into the A-tiled operand of
// the output projection.  Fewer rows per workgroup spread the split-partial
// stream (S * 5 KB per row and head) over more CUs.  MTG > 1 (few rows, Q4
// weights): the head's 64 outputs go to MTG workgroups (grid z), each staging
// only its 64 / MTG weight rows and merging the rows' splits itself; every
// output keeps its wave split and sum order, so its bits do not change.
template <int NS, int WK, int RPW, int SM, int MTG>
__global__ __launch_bounds__(512) void xattn_out_kernel(const float* __restrict__ zpart,
                                                        const float* __restrict__ mlpart, int R, int H, int D, int S,
                                                        const uint8_t* __restrict__ wv,
                                                        const uint32_t* __restrict__ wvp,
                                                        const float* __restrict__ bv, _Float16* __restrict__ tiled,
                                                        float* __restrict__ out32) {
  // Zn of the RPW rows: f32 [column][row] (f16 weights, VALU projection) or
  // f16 hi / lo planes [row][column] (Q4 weights, MFMA projection)
  constexpr int ZLD = kMaxD + 8;  // halves; == 4 dwords (mod 64): conflict-free B fragment reads
  __shared__ __attribute__((aligned(16))) uint8_t zbuf[WK == kWtQ4 ? 2 * RPW * ZLD * 2 : kMaxD * RPW * 4];
  float* zs = reinterpret_cast<float*>(zbuf);
  _Float16* zh = reinterpret_cast<_Float16*>(zbuf);
  _Float16* zl = zh + RPW * ZLD;
  __shared__ __attribute__((aligned(16))) _Float16 zzero[8];
  __shared__ float red[16][64][RPW + 1];
  static_assert(MTG == 1 || WK == kWtQ4, "output groups need the Q4 MFMA projection");
  constexpr int NMT = 4 / MTG;  // 16-output m-tiles per workgroup
  const int h = blockIdx.x, rbase = blockIdx.y * RPW, rstep = 1, mt0 = blockIdx.z * NMT;
  const int tid = threadIdx.x;
  const int nkb = D / 32;
  // the value bias of this thread's final outputs, loaded up front
  const float bias1 = tid < 16 * NMT * RPW ? bv[h * 64 + 16 * mt0 + (tid & (16 * NMT - 1))] : 0.0f;
  // Q4: this wave's packed nibbles and scales (blocks kb = w, w + 8, ...,
  // its m-tiles), issued before the merge's loads: both in flight together
  constexpr int KPW = kMaxD / 32 / 8;  // blocks per wave
  uint32_t wq[WK == kWtQ4 ? KPW : 1][WK == kWtQ4 ? NMT : 1], wd[WK == kWtQ4 ? KPW : 1][WK == kWtQ4 ? NMT : 1];
  if constexpr (WK == kWtQ4) {
    const int l = tid & 63, w = tid >> 6;
#pragma unroll
    for (int u = 0; u < KPW; ++u) {
      const int kb = w + 8 * u < nkb ? w + 8 * u : 0;
#pragma unroll
      for (int mt = 0; mt < NMT; ++mt) {
        const uint32_t* o = wvp + (((size_t)h * nkb + kb) * 4 + mt0 + mt) * kWvPackU32;
        wq[u][mt] = WA_XATTN_ODIAG == 1 ? 0u : o[l];
        wd[u][mt] = WA_XATTN_ODIAG == 1 ? 0u : reinterpret_cast<const uint16_t*>(o + 64)[l & 15];
      }
    }
  }
  // merge of the S frame ranges (flash-attention merge, fixed split order):
  // Zn[c] = (sum_s w_s Z_s[c]) / (sum_s w_s L_s), w_s = exp(M_s - max_s M_s).
  // The weights depend on the row only: thread (row j < RPW) computes its
  // row's w_s and the denominator (split order) into LDS while every
  // thread's Z loads are in flight -- one memory round trip for the merge and
  // no per-item copies of (M_s, L_s) in registers (at 12-16 splits those
  // spilled: xattn_out 16-36 us, profiles/r05_xattn_micro.log).  Item (row j,
  // 4 columns): every split's float4, all NIT items loaded before any is
  // merged (fixed unrolled counts; splits >= S read nothing); rows >= R give
  // zeros.
  __shared__ float swt[RPW][SM + 1];  // w_s per row, [SM] = the denominator
  {
    const int nq = D / 4;
    constexpr int NIT = (RPW * (kMaxD / 4) + 511) / 512;
    floatx4 zv[NIT][SM];
#pragma unroll
    for (int u = 0; u < NIT; ++u) {
      const int it = tid + 512 * u;
      const int j = it / nq, q = it - j * nq;
      const bool ok = it < RPW * nq && rbase + rstep * j < R;
      const size_t rb = (size_t)(ok ? rbase + rstep * j : 0) * S;
      const floatx4* zp = reinterpret_cast<const floatx4*>(zpart + (rb * H + h) * D) + (ok ? q : 0);
#pragma unroll
      for (int s = 0; s < SM; ++s)
        if (s < S) zv[u][s] = WA_XATTN_ODIAG == 2 ? floatx4{0.0f, 0.0f, 0.0f, 0.0f} : zp[(size_t)s * H * (D / 4)];
    }
    if (tid < RPW) {
      const int j = tid;
      const size_t rb = (size_t)(rbase + rstep * j < R ? rbase + rstep * j : 0) * S;
      const floatx2* mp = reinterpret_cast<const floatx2*>(mlpart) + rb * H + h;
      floatx2 ml[SM];
#pragma unroll
      for (int s = 0; s < SM; ++s)
        if (s < S) ml[s] = WA_XATTN_ODIAG == 2 ? floatx2{0.0f, 1.0f} : mp[(size_t)s * H];
      float mx = -INFINITY;
#pragma unroll
      for (int s = 0; s < SM; ++s)
        if (s < S) mx = fmaxf(mx, ml[s][0]);
      float lsum = 0.0f;
#pragma unroll
      for (int s = 0; s < SM; ++s)
        if (s < S) {
          const float w = ml[s][0] == -INFINITY ? 0.0f : __builtin_amdgcn_exp2f(ml[s][0] - mx);  // base-2 units
          lsum = fmaf(w, ml[s][1], lsum);
          swt[j][s] = w;
        }
      swt[j][SM] = lsum;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NIT; ++u) {
      const int it = tid + 512 * u;
      if (it >= RPW * nq) break;
      const int j = it / nq, q = it - j * nq;
      const bool rok = rbase + rstep * j < R;
      floatx4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int s = 0; s < SM; ++s)
        if (s < S) {
          const float w = swt[j][s];
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[e] = fmaf(w, zv[u][s][e], acc[e]);
        }
      const float lsum = swt[j][SM];
      if constexpr (WK == kWtQ4) {
        half4 hi, lo;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          _Float16 x, y;
          split_f16(rok ? acc[e] / lsum * kZnScale : 0.0f, x, y);
          hi[e] = x;
          lo[e] = y;
        }
        *reinterpret_cast<half4*>(&zh[j * ZLD + 4 * q]) = hi;
        *reinterpret_cast<half4*>(&zl[j * ZLD + 4 * q]) = lo;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) zs[(4 * q + e) * RPW + j] = rok ? acc[e] / lsum : 0.0f;
      }
    }
  }
  if (tid < 8) zzero[tid] = (_Float16)0.0f;
  __syncthreads();
  constexpr int NPART = WK == kWtQ4 ? 8 : 16;  // partials per output in red
  if constexpr (WK == kWtQ4) {
    // out^T (d x row) = Wv_h (64 x D) Zn^T on 16x16x32 MFMA: m = 16 outputs d
    // (4 tiles), n = the rows (RPW real of 16), k = one Q4 block of 32
    // columns.  Wave w takes blocks w, w + 8, ...; A = the exact weights
    // (q - 8) d split hi + lo, B = Zn hi / lo: three products as elsewhere.
    // Lane l: A row d = 16 mt + (l & 15), elements 8 (l >> 4) .. + 7 of the
    // block = low (l >> 4 < 2) or high nibbles of nibble bytes 8 ((l >> 4) & 1)
    // .. + 7; B row n = l & 15, the same 8 columns.
    const int w = tid >> 6, l = tid & 63, n = l & 15, lq = l >> 4;
    floatx4 acc[4];
#pragma unroll
    for (int mt = 0; mt < NMT; ++mt) acc[mt] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int u = 0; u < KPW; ++u) {
      const int kb = w + 8 * u;
      if (kb >= (WA_XATTN_ODIAG == 3 ? 0 : nkb)) break;
      const _Float16* zhp = n < RPW ? &zh[n * ZLD + kb * 32 + 8 * lq] : zzero;
      const _Float16* zlp = n < RPW ? &zl[n * ZLD + kb * 32 + 8 * lq] : zzero;
      const half8 bh = *reinterpret_cast<const half8*>(zhp);
      const half8 bl = *reinterpret_cast<const half8*>(zlp);
#pragma unroll
      for (int mt = 0; mt < NMT; ++mt) {  // local m-tile: outputs 16 (mt0 + mt) ..
        const _Float16 d = __builtin_bit_cast(_Float16, (uint16_t)wd[u][mt]) * (_Float16)kWvScale;  // exact: d < 16
        const half2v off = {(_Float16)1032.0f, (_Float16)1032.0f};
        const half2v dv = {d, d};
        half8 ah, al;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t x = wq[u][mt] >> (8 * i);  // elements 2i, 2i + 1 in its low two nibbles
          const uint32_t pr = (x & 0xFu) | ((x << 12) & 0xF0000u) | 0x64006400u;
          const half2v qv = __builtin_bit_cast(half2v, pr) - off;  // exact q - 8
          const half2v hv = qv * dv;
          const half2v lv = __builtin_elementwise_fma(qv, dv, -hv);  // exact remainder
          ah[2 * i] = hv[0];
          ah[2 * i + 1] = hv[1];
          al[2 * i] = lv[0];
          al[2 * i + 1] = lv[1];
        }
        acc[mt] = mfma16x32(ah, bh, acc[mt]);
        acc[mt] = mfma16x32(ah, bl, acc[mt]);
        acc[mt] = mfma16x32(al, bh, acc[mt]);
      }
    }
    // acc[mt][i]: output d = 16 (mt0 + mt) + 4 lq + i, row n (red indexed locally)
    if (n < RPW) {
#pragma unroll
      for (int mt = 0; mt < NMT; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) red[w][16 * mt + 4 * lq + i][n] = acc[mt][i];
    }
  } else {
    const int dp = tid & 31, bg = tid >> 5;  // rows dp, dp + 32; blocks bg, bg + 16, bg + 32
    float acc0[RPW], acc1[RPW];
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      acc0[j] = 0.0f;
      acc1[j] = 0.0f;
    }
#pragma unroll 1
    for (int kb = bg; kb < nkb; kb += 16) {
      float w0[32], w1[32];
      load_w32<WK>(wv, D, h * 64 + dp, kb, w0);
      load_w32<WK>(wv, D, h * 64 + dp + 32, kb, w1);
#pragma unroll
      for (int i = 0; i < 32; ++i) {
        const float* z = &zs[(kb * 32 + i) * RPW];
#pragma unroll
        for (int j = 0; j < RPW; ++j) {
          acc0[j] = fmaf(w0[i], z[j], acc0[j]);
          acc1[j] = fmaf(w1[i], z[j], acc1[j]);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      red[bg][dp][j] = acc0[j];
      red[bg][dp + 32][j] = acc1[j];
    }
  }
  __syncthreads();
  if (tid < 16 * NMT * RPW) {  // thread (row j, output d): the block-group sum in group order, then 4-wide stores
    const int j = tid / (16 * NMT), d = tid & (16 * NMT - 1), r = rbase + rstep * j;
    float sacc = bias1;
#pragma unroll
    for (int g = 0; g < NPART; ++g) sacc += red[g][d][j] * (WK == kWtQ4 ? kOutInv : 1.0f);  // exact rescale
    const float v1 = __shfl_down(sacc, 1, 64), v2 = __shfl_down(sacc, 2, 64), v3 = __shfl_down(sacc, 3, 64);
    if (r < R && (d & 3) == 0) attn_store4<NS>(tiled, out32, D, r, h * 64 + 16 * mt0 + d, kbp_of(D), sacc, v1, v2, v3);
  }
}

// f32 rows [rows][D] -> [rows][NS][D] f16 planes (hi | lo)
template <int NS>
__global__ __launch_bounds__(256) void enc_planes_kernel(const float* __restrict__ x, int64_t n, int D,
                                                         _Float16* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int64_t row = i / D;
  const int c = (int)(i - row * D);
  _Float16 hi, lo;
  split_f16(x[i] * kEncScale, hi, lo);
  out[(row * NS) * D + c] = hi;
  if (NS == 2) out[(row * NS + 1) * D + c] = lo;
}

// 8 waves (4 when D / 8 is not a multiple of 32: D = 384)
// A-tiled operand rows [R][K] -> f32 (diagnostics)
template <int NS>
__global__ __launch_bounds__(256) void untile_kernel(const _Float16* __restrict__ t, int R, int K,
                                                     float* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= R * K) return;
  const int r = i / K, k = i - r * K;
  float v = (float)t[wq4::atile_index(r, k, kbp_of(K), NS, 0)];
  if (NS == 2) v += (float)t[wq4::atile_index(r, k, kbp_of(K), NS, 1)];
  out[i] = v * wq4::kActScaleInv;
}

// ------------------------------------------- few query rows: split phases --
// With R query rows the fused xattn_main_kernel runs S * R workgroups (8 at
// one clip), each walking its CH sub-chunks in series (2.7 us each at 16
// clips).  For R <= xattn_small_rows() the same arithmetic runs as two
// launches that spread over sub-chunks and columns instead:
//   scores   one workgroup per (row, sub-chunk): the fused kernel's score
//            MFMA sequence per wave column slice, its wave-order partial sum;
//   z        one workgroup per (row, split, 128 columns): the fused kernel's
//            online softmax of the split (recomputed per workgroup while its
//            encoder loads are in flight), then per wave one 32-column tile's
//            rescale + three MFMAs per sub-chunk.
// Every partial (Z, max, sum) therefore has the fused path's bits, so a
// clip's tokens do not depend on the batch (test_xattn_small_rows_bit_identical).
constexpr int kSmallMaxCH = 12;   // sub-chunks per split the softmax/z kernels preload (T <= 1536 at 8 splits)
constexpr int kSmallRowsMax = 8;  // scratch is sized for up to this many rows

template <int D, int HT, int NS, int NW>
__global__ __launch_bounds__(64 * NW) void xattn_scores_kernel(const _Float16* __restrict__ qt,
                                                               const _Float16* __restrict__ enc, int Tq, int T,
                                                               int NG, float* __restrict__ sbuf) {
  constexpr int CW = D / NW, KS = CW / 32, HP = HT * 16, ROW = NS * D;
  __shared__ __attribute__((aligned(16))) float red[NW][HT][16][20];
  const int g = blockIdx.x, r = blockIdx.y;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, l16 = l & 15, lq = l >> 4;
  const int c0 = w * CW, f = g * kTc + l16;
  const _Float16* E = enc + (size_t)(r / Tq) * T * ROW;
  // A = this wave's column slice of the sub-chunk's frames (frames >= T are
  // zeros, as the fused kernel's buffer loads give); B = qt, the second head
  // tile's padding lanes zero
  half8 a[KS][NS];
  const int fc = f < T ? f : T - 1;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int p = 0; p < NS; ++p)
      a[ks][p] = *reinterpret_cast<const half8*>(E + (size_t)fc * ROW + p * D + c0 + ks * 32 + 8 * lq);
  if (f >= T) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int p = 0; p < NS; ++p) a[ks][p] = half8{};
  }
  half8 qb[KS][HT][NS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int ht = 0; ht < HT; ++ht) {
      // padding lanes of the second head tile read their group's real row
      // (no extra bytes fetched) and are zeroed below
      const int hr = (HT == 2 && ht == 1) ? 16 + (l16 & 3) : ht * 16 + l16;
#pragma unroll
      for (int p = 0; p < NS; ++p)
        qb[ks][ht][p] = *reinterpret_cast<const half8*>(qt + (((size_t)r * NS + p) * HP + hr) * D + c0 + ks * 32 + 8 * lq);
    }
  __builtin_amdgcn_sched_barrier(0);  // every load above in flight before the first MFMA
  floatx4 sacc[HT];
#pragma unroll
  for (int ht = 0; ht < HT; ++ht) sacc[ht] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int ht = 0; ht < HT; ++ht) {
      const bool ok = !(HT == 2 && ht == 1) || l16 < 4;
      half8 b[NS];
#pragma unroll
      for (int p = 0; p < NS; ++p) b[p] = ok ? qb[ks][ht][p] : half8{};
      sacc[ht] = mfma16x32(a[ks][0], b[0], sacc[ht]);
      if constexpr (NS == 2) {
        sacc[ht] = mfma16x32(a[ks][1], b[0], sacc[ht]);
        sacc[ht] = mfma16x32(a[ks][0], b[1], sacc[ht]);
      }
    }
#pragma unroll
  for (int ht = 0; ht < HT; ++ht) *reinterpret_cast<floatx4*>(&red[w][ht][l16][4 * lq]) = sacc[ht];
  __syncthreads();
  for (int idx = tid; idx < HT * 256; idx += 64 * NW) {
    const int ht = idx >> 8, hh = (idx >> 4) & 15, t = idx & 15;
    float sv = 0.0f;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) sv += red[ww][ht][hh][t];
    sbuf[(((size_t)r * NG + g) * HP + ht * 16 + hh) * 16 + t] = sv;
  }
}

// grid (S, D / 128, R), 4 waves: wave w owns columns cb .. cb + 31 of split
// s.  The split's online softmax (the fused kernel's, step by step: same
// lanes, DPP reductions, rescale flag) is recomputed by every workgroup of
// the split from the scores while its encoder loads are in flight; the
// workgroup of column group 0 writes the split's (max, sum).
template <int D, int HT, int NS>
__global__ __launch_bounds__(256) void xattn_z_kernel(const _Float16* __restrict__ enc,
                                                      const float* __restrict__ sbuf, int Tq, int T, int H, int S,
                                                      int CH, int NG, float* __restrict__ zpart,
                                                      float* __restrict__ mlpart) {
  constexpr int ROW = NS * D, ZR = 32, HP = HT * 16;  // staged plane: 16 frames x 32 columns, rows of 64 B
  constexpr int SMX = 512 / 256;                      // softmax entries (head 0..31, frame) per thread
  __shared__ __attribute__((aligned(16))) _Float16 sp[kSmallMaxCH][NS][32][kTc];
  __shared__ float sal[kSmallMaxCH][32];
  __shared__ int sfl[kSmallMaxCH];
  __shared__ __attribute__((aligned(16))) _Float16 stg[4][NS][16 * ZR];
  const int s = blockIdx.x, r = blockIdx.z, tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int l32 = l & 31, lh = l >> 5;
  const int cb = blockIdx.y * 128 + w * 32;
  const int ts = s * CH * kTc, te = min(T, ts + CH * kTc);
  const int nch = te > ts ? (te - ts + kTc - 1) / kTc : 0;
  const size_t g0 = (size_t)r * NG + s * CH;
  // this wave's enc pieces of every sub-chunk (lane: frame l >> 2, 8 columns
  // 8 (l & 3)), frames past the split read as zeros
  typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
  const _Float16* E = enc + (size_t)(r / Tq) * T * ROW;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<_Float16*>(E + (size_t)ts * ROW), 0, nch > 0 ? (te - ts) * ROW * 2 : 0, 0x00020000);
  u32x4v ev[kSmallMaxCH][NS];
#pragma unroll
  for (int c = 0; c < kSmallMaxCH; ++c)
#pragma unroll
    for (int p = 0; p < NS; ++p)  // unconditional: past the split's frames the buffer gives zeros
      ev[c][p] = __builtin_amdgcn_raw_buffer_load_b128(
          rs, (uint32_t)((((c * kTc + (l >> 2)) * ROW) + p * D + cb + 8 * (l & 3)) * 2), 0, 0);
  // the split's scores (every load issued up front)
  float sv_all[kSmallMaxCH][SMX];
#pragma unroll
  for (int c = 0; c < kSmallMaxCH; ++c)
#pragma unroll
    for (int e = 0; e < SMX; ++e) {
      const int idx = tid + e * 256, h = idx >> 4, t = idx & 15;
      const int cc = c < nch ? c : 0, hc = h < HP ? h : 0;
      sv_all[c][e] = sbuf[((g0 + cc) * HP + hc) * 16 + t];
    }
  if (tid < kSmallMaxCH) sfl[tid] = 0;
  __syncthreads();
  float M[SMX], L[SMX];
#pragma unroll
  for (int e = 0; e < SMX; ++e) {
    M[e] = -INFINITY;
    L[e] = 0.0f;
  }
#pragma unroll
  for (int chi = 0; chi < kSmallMaxCH; ++chi) {
    if (chi >= nch) continue;
    const int t0 = ts + chi * kTc;
#pragma unroll
    for (int e = 0; e < SMX; ++e) {
      const int idx = tid + e * 256, h = idx >> 4, t = idx & 15;
      _Float16 phi = (_Float16)0.0f, plo = (_Float16)0.0f;
      float alpha = 1.0f;
      if (h < HP) {  // the fused kernel's softmax entry
        float p;
        softmax_entry(sv_all[chi][e], h < H && t0 + t < te, M[e], L[e], alpha, p);
        split_f16(p * kPScale, phi, plo);
      }
      sp[chi][0][h][t] = phi;
      if (NS == 2) sp[chi][1][h][t] = plo;
      if (t == 0) sal[chi][h] = alpha;
      if (alpha != 1.0f) sfl[chi] = 1;  // benign race: every writer stores 1
    }
  }
  if (blockIdx.y == 0) {
    const size_t base = (size_t)r * S + s;
#pragma unroll
    for (int e = 0; e < SMX; ++e) {
      const int idx = tid + e * 256, h = idx >> 4;
      if ((idx & 15) == 0 && h < H && h < HP) {
        mlpart[(base * H + h) * 2] = M[e] * kSInv;
        mlpart[(base * H + h) * 2 + 1] = L[e];
      }
    }
  }
  __syncthreads();
  const int g = l >> 4, gi = l & 15;
  const int trow = 8 * (g >> 1) + (gi >> 2), tcol = 16 * (g & 1) + 4 * (gi & 3);
  floatx16 zacc;
#pragma unroll
  for (int j = 0; j < 16; ++j) zacc[j] = 0.0f;
#pragma unroll
  for (int chi = 0; chi < kSmallMaxCH; ++chi) {
    if (chi >= nch) continue;
#pragma unroll
    for (int p = 0; p < NS; ++p)
      *reinterpret_cast<u32x4v*>(&stg[w][p][(l >> 2) * ZR + 8 * (l & 3)]) = ev[chi][p];
    half8 pa[NS];
#pragma unroll
    for (int p = 0; p < NS; ++p) pa[p] = *reinterpret_cast<const half8*>(&sp[chi][p][l32][8 * lh]);
    if (sfl[chi]) {
#pragma unroll
      for (int j = 0; j < 16; ++j) zacc[j] *= sal[chi][(j & 3) + 8 * (j >> 2) + 4 * lh];
    }
    half8 eb[NS];
#pragma unroll
    for (int p = 0; p < NS; ++p) {
      const half4 x0 = lds_tr4(&stg[w][p][trow * ZR + tcol]);
      const half4 x1 = lds_tr4(&stg[w][p][(trow + 4) * ZR + tcol]);
      eb[p] = half8{x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
    }
    zacc = mfma32x16(pa[0], eb[0], zacc);
    if (NS == 2) {
      zacc = mfma32x16(pa[1], eb[0], zacc);
      zacc = mfma32x16(pa[0], eb[1], zacc);
    }
  }
  const size_t base = (size_t)r * S + s;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int h = (j & 3) + 8 * (j >> 2) + 4 * lh;
    if (h < H) zpart[(base * H + h) * D + cb + l32] = zacc[j] * kZInv;
  }
}

template <int D, int HT, int NS>
void launch_small(int R, int Tq, int T, int H, const XattnPlan& p, const _Float16* qt, const _Float16* enc,
                  float* z, float* ml, float* scratch, hipStream_t st) {
  constexpr int NW = (D / 8) % 32 == 0 ? 8 : 4;
  const int NG = p.splits * p.ch;
  float* sb = scratch;  // R * NG * 32 * 16 floats
  hipLaunchKernelGGL((xattn_scores_kernel<D, HT, NS, NW>), dim3(NG, R), dim3(64 * NW), 0, st, qt, enc, Tq, T, NG, sb);
  hipLaunchKernelGGL((xattn_z_kernel<D, HT, NS>), dim3(p.splits, D / 128, R), dim3(256), 0, st, enc, sb, Tq, T, H,
                     p.splits, p.ch, NG, z, ml);
}

// Query rows at or below which the split phases run (WA_XATTN_SMALL_ROWS
// overrides it: 0 = always fused; tests force each path).
int xattn_small_rows() {
  int v = 4;
  if (const char* e = getenv("WA_XATTN_SMALL_ROWS")) v = atoi(e);
  return std::max(0, std::min(kSmallRowsMax, v));
}

// 8 waves (two per SIMD, 256 registers each: the Z accumulators of an
// eighth of the columns + one sub-chunk in flight); 4 when D / 8 is not a
// multiple of 32 (D = 384).  A second sub-chunk in flight (PF = 2) does not
// fit the register file at Large-V3 f16x2.  Measured and removed (round 5):
// the scores of sub-chunk j + 1 straight from the fetched registers beside
// sub-chunk j's Z update (one LDS write less, the MFMAs of two sub-chunks
// interleaved) -- 45.3 vs 36.2 us at 16 rows, decode 970 vs 856 ms.
template <int D, int HT, int NS>
void launch_main(dim3 g, const _Float16* qt, const _Float16* enc, int Tq, int T, int H, int S, int CH, float* z,
                 float* ml, int R, hipStream_t st) {
  constexpr int NW = (D / 8) % 32 == 0 ? 8 : 4;
  hipLaunchKernelGGL((xattn_main_kernel<D, HT, NS, NW, 1>), g, dim3(64 * NW), 0, st, qt, enc, Tq, T, H, S, CH, z, ml,
                     R);
}

// Rows of Zn per xattn_out workgroup: 4.  Isolated, 2 rows per workgroup is
// faster at 16 rows (9.6 vs 11.0 us) and slower at 32 (14.3 vs 11.1); in the
// model (two concurrent 16-row decode groups) 2 rows made the decode slower
// (893-898 vs 874-878 ms, scripts/gpu.sh libs): the doubled grid
// crowds the other group.  1 and 8 are slower everywhere.  A row's bits do
// not depend on its workgroup's rows (each is its own MFMA column).
#ifndef WA_XATTN_OUT_ROWS  // compile-time override: tuning builds (scripts/xattn_micro.sh)
#define WA_XATTN_OUT_ROWS 4
#endif
int out_rows(int R) {
  (void)R;
  return WA_XATTN_OUT_ROWS;
}
template <int NS, int WK, int RPW>
void launch_out_rpw(int R, int H, const float* z, const float* ml, int D, int S, const uint8_t* wv,
                    const uint32_t* wvp, const float* bv, _Float16* tiled, float* out32, hipStream_t st,
                    bool split_outputs) {
  const dim3 go(H, (R + RPW - 1) / RPW);
  if constexpr (WK == kWtQ4) {
    if (split_outputs) {  // few rows: 4 workgroups per head
      hipLaunchKernelGGL((xattn_out_kernel<NS, WK, RPW, kXattnSplits, 4>), dim3(go.x, go.y, 4), dim3(512), 0, st, z,
                         ml, R, H, D, S, wv, wvp, bv, tiled, out32);
      return;
    }
  }
  hipLaunchKernelGGL((xattn_out_kernel<NS, WK, RPW, kXattnSplits, 1>), go, dim3(512), 0, st, z, ml, R, H, D, S, wv,
                     wvp, bv, tiled, out32);
}
template <int NS, int WK>
void launch_out(int R, int H, const float* z, const float* ml, int D, int S, const uint8_t* wv, const uint32_t* wvp,
                const float* bv, _Float16* tiled, float* out32, hipStream_t st, bool split_outputs = false) {
  switch (out_rows(R)) {
    case 1: launch_out_rpw<NS, WK, 1>(R, H, z, ml, D, S, wv, wvp, bv, tiled, out32, st, split_outputs); break;
    case 2: launch_out_rpw<NS, WK, 2>(R, H, z, ml, D, S, wv, wvp, bv, tiled, out32, st, split_outputs); break;
    case 8: launch_out_rpw<NS, WK, 8>(R, H, z, ml, D, S, wv, wvp, bv, tiled, out32, st, split_outputs); break;
    default: launch_out_rpw<NS, WK, 4>(R, H, z, ml, D, S, wv, wvp, bv, tiled, out32, st, split_outputs); break;
  }
}

}  // namespace

// The frame split depends on T only -- never on the number of query rows --
// so every row's arithmetic (and its tokens) is independent of the batch.
// 8 ranges of 12 sub-chunks for T = 1500: 256 workgroups at 32 rows.
XattnPlan xattn_plan(int R, int T) {
  (void)R;
  const int nchunk = (T + kTc - 1) / kTc;
  const int S = std::max(1, std::min(kXattnSplits, nchunk));
  XattnPlan p;
  p.ch = (nchunk + S - 1) / S;
  p.splits = (nchunk + p.ch - 1) / p.ch;
  return p;
}

size_t xattn_part_floats(int R, int H, int D, int T) {
  const XattnPlan p = xattn_plan(R, T);
  size_t n = (size_t)R * p.splits * H * ((size_t)D + 2) + (size_t)R * H * D;
  if (R <= kSmallRowsMax) {  // split-phase scratch: the scores (+ 16-B alignment)
    const size_t ng = (size_t)p.splits * p.ch;
    n = (n + 3) / 4 * 4 + (size_t)R * ng * 32 * 16 + 4;
  }
  return n;
}

hipError_t launch_untile(const _Float16* tiled, int R, int K, int ns, float* out, hipStream_t st) {
  const dim3 g((R * K + 255) / 256);
  if (ns == 2)
    hipLaunchKernelGGL(untile_kernel<2>, g, dim3(256), 0, st, tiled, R, K, out);
  else
    hipLaunchKernelGGL(untile_kernel<1>, g, dim3(256), 0, st, tiled, R, K, out);
  return hipGetLastError();
}

hipError_t launch_enc_planes(const float* x, int64_t rows, int D, int ns, _Float16* out, hipStream_t st) {
  const int64_t n = rows * D;
  const dim3 g((unsigned)((n + 255) / 256));
  if (ns == 2)
    hipLaunchKernelGGL(enc_planes_kernel<2>, g, dim3(256), 0, st, x, n, D, out);
  else
    hipLaunchKernelGGL(enc_planes_kernel<1>, g, dim3(256), 0, st, x, n, D, out);
  return hipGetLastError();
}

size_t wv_pack_words(int H, int D) { return (size_t)H * (D / 32) * 4 * kWvPackU32; }

hipError_t launch_wv_pack(const uint8_t* wv, int H, int D, uint32_t* out, hipStream_t st) {
  if (D % 32 != 0 || D > kMaxD) return hipErrorInvalidValue;
  const int64_t n = (int64_t)H * (D / 32) * 4 * 64;
  hipLaunchKernelGGL(wv_pack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, wv, H, D, out);
  return hipGetLastError();
}

hipError_t launch_xattn(const float* q, const uint8_t* wk, const uint8_t* wv, const uint32_t* wvp, const float* bv,
                        int wtype, const _Float16* enc, int B, int Tq, int T, int H, int D, _Float16* qt, float* part,
                        _Float16* tiled, int ns, hipStream_t st, float* out32) {
  const int R = B * Tq;
  const int HT = (H + 15) / 16, HP = HT * 16;
  if (D != H * 64 || D % 128 != 0 || D > kMaxD || H > 20 || !q) return hipErrorInvalidValue;
  if (wtype == kWtQ4 && !wvp) return hipErrorInvalidValue;  // Q4: the load-time packed Wv (launch_wv_pack)
  const XattnPlan p = xattn_plan(R, T);
  float* z = part;
  float* ml = part + (size_t)R * p.splits * H * D;
  // qt = Wk^T q / 8
  const dim3 gq(H, D / 64, (R + 31) / 32);
#define WA_XQ(NS_, WK_) hipLaunchKernelGGL((xattn_q_mfma_kernel<NS_, WK_>), gq, dim3(128), 0, st, q, R, D, wk, HP, qt)
  if (wtype == kWtQ4) {
    if (ns == 2) WA_XQ(2, kWtQ4); else WA_XQ(1, kWtQ4);
  } else {
    if (ns == 2) WA_XQ(2, kWtF16); else WA_XQ(1, kWtF16);
  }
#undef WA_XQ
  // stream the encoder output: fused, or in split phases for few rows
  const dim3 gm(p.splits, R);
  const bool small = R <= xattn_small_rows() && p.ch <= kSmallMaxCH;
  float* scratch = part + ((size_t)R * p.splits * H * ((size_t)D + 2) + (size_t)R * H * D + 3) / 4 * 4;
#define WA_XMAIN(DD, HH)                                                                   \
  if (D == DD && HT == HH) {                                                               \
    if (small) {                                                                           \
      if (ns == 2)                                                                         \
        launch_small<DD, HH, 2>(R, Tq, T, H, p, qt, enc, z, ml, scratch, st);              \
      else                                                                                 \
        launch_small<DD, HH, 1>(R, Tq, T, H, p, qt, enc, z, ml, scratch, st);              \
    } else if (ns == 2)                                                                    \
      launch_main<DD, HH, 2>(gm, qt, enc, Tq, T, H, p.splits, p.ch, z, ml, R, st);          \
    else                                                                                   \
      launch_main<DD, HH, 1>(gm, qt, enc, Tq, T, H, p.splits, p.ch, z, ml, R, st);          \
  } else
  WA_XMAIN(1280, 2)
  WA_XMAIN(1024, 1)
  WA_XMAIN(768, 1)
  WA_XMAIN(512, 1)
  WA_XMAIN(384, 1)
  return hipErrorInvalidValue;
#undef WA_XMAIN
  // merge the splits and project with Wv into the output projection's operand
  if (wtype == kWtQ4) {
    if (ns == 2)
      launch_out<2, kWtQ4>(R, H, z, ml, D, p.splits, wv, wvp, bv, tiled, out32, st, small);
    else
      launch_out<1, kWtQ4>(R, H, z, ml, D, p.splits, wv, wvp, bv, tiled, out32, st, small);
  } else {
    if (ns == 2)
      launch_out<2, kWtF16>(R, H, z, ml, D, p.splits, wv, wvp, bv, tiled, out32, st, small);
    else
      launch_out<1, kWtF16>(R, H, z, ml, D, p.splits, wv, wvp, bv, tiled, out32, st, small);
  }
  return hipGetLastError();
}

}  // namespace wa
