// wa_kernels.hip -- gfx950 kernels of the Whisper model around the Q4 path.
//
// Reference semantics (zerr0o/whisper-burn):
//   LayerNorm        src/model/layers.rs:12-32   (eps 1e-5, biased variance)
//   GELU (tanh)      src/model/layers.rs:35-41
//   Conv1D + GELU    src/model/layers.rs:62-132, encoder.rs:87-106
//   SDPA             src/model/attention.rs:243-298 (scores / sqrt(64),
//                    causal mask only when q_len > 1, softmax over keys)
//   KV-cached decode src/model/attention.rs:93-125, decoder.rs:77-112
//   logits / argmax  src/model/decoder.rs:289-292, 342-347; whisper.rs:131-138
// Every product here is f32 x f32 (v_mfma_f32_32x32x2_f32: exact products,
// f32 accumulation) or f32 VALU; only the operands handed to the Q4 GEMMs
// are written in the f16 hi/lo A-tiled layout (wq4_layout.hpp).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdlib>

#include "../wq4_device.hpp"
#include "../wq4_lnmath.hpp"
#include "wa_kernels.hpp"

// WA_LOGITS_NT (default on): the decode step's 266-MB embedding-table stream
// (logits_argmax_f16_k32_kernel) with the nontemporal policy, so it does not
// push the encoder planes the next step's cross-attention re-reads out of the
// Infinity Cache: decode 928 -> 920 ms at 32 clips, RTF +0.7 % (two A/B runs
// bracketed by the base build, profiles/r06af_libs.txt, r06ag_libs.txt).
#ifndef WA_LOGITS_NT
#define WA_LOGITS_NT 1
#endif

namespace wa {

using wq4::floatx16;
using wq4::floatx4;
using wq4::half8;

constexpr int kEOT = 50257;
// attention scores scaled by 1/sqrt(64) * log2(e) (attention.rs:262): the
// softmax runs in base 2, one v_exp_f32 (2^x) per exponential
constexpr float kEaQScale = 0.125f * 1.4426950408889634f;
// Operand scales of the f16-pair MFMAs (the MFMAs flush f16 subnormal inputs,
// wq4_device.hpp split_act): q / 8 (base 2), k and v enter as x * 2^5 (|x| <
// 2047), the softmax weights p in (0, 2] (lazy reference maximum) as p * 2^14
// (<= 32768 < 65504); the scores come out x 2^10 and the output x 2^19 --
// undone in f32, exactly.
constexpr float kQKScale = 32.0f, kSInv = 1.0f / 1024.0f;
constexpr float kPScale = 16384.0f, kPVInv = 1.0f / (16384.0f * 32.0f);
constexpr float kEaLazyMax = 1024.0f;  // 1.0 in base-2 units x 2^10 (the scores' operand scale)
// the conv front-end: input x 2^4, weights x 2^10 (|w| < 64), product x 2^-14
constexpr float kCvAScale = 16.0f, kCvBScale = 1024.0f, kCvInv = 1.0f / (16.0f * 1024.0f);
// logits: hidden rows as GEMM activations (x 2^4), the f16-pair table x 2^8
// (|e| < 255), logits x 2^-12
constexpr float kEmbScale = 256.0f, kLgInv = 1.0f / (16.0f * 256.0f);

using wq4::kLnMaxV;
using wq4::wave_sum;

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ floatx16 mfma_f32(float a, float b, const floatx16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

using wq4::atile_store4;
using wq4::attn_store4;
using wq4::kbp_of;
using wq4::split_f16;



// ------------------------------------ encoder attention, f16x2 MFMA --
// Encoder self-attention (attention.rs:243-298, non-causal; scores use q / 8,
// an exact power-of-two scaling of attention.rs:266-267's division), flash
// style: products on v_mfma_f32_32x32x16_f16 with every operand an
// exact-to-2^-22 f16 pair (x = hi + lo; hi*hi + lo*hi + hi*lo, f32
// accumulation -- the arithmetic of the Q4 GEMMs).  Both products are
// computed transposed (S^T = K Q^T, O^T = V^T P^T) so that a lane owns one
// query and the online-softmax statistics are lane-local.  Workgroup = 8
// waves x 32 queries of one (clip, head); 64-key tiles of K and V are converted to f16
// pairs into LDS (row stride 72 halves: conflict-free b128 and transposed
// reads), the next tile's f32 loads in flight meanwhile.
//   S^T = K Q^T   A = K (m = key, k = dim) ds_read_b128; B = Q^T from registers
//   O^T += V^T P^T  A = V^T via ds_read_b64_tr_b16 of row-major V, in the key
//                 order of the S^T accumulator; B = P^T = that accumulator.
typedef _Float16 ea_half4 __attribute__((ext_vector_type(4)));
typedef __fp16 ea_fp16x4 __attribute__((__vector_size__(4 * sizeof(__fp16))));
__device__ __forceinline__ ea_half4 ea_tr4(const _Float16* p) {
  return __builtin_bit_cast(ea_half4, __builtin_amdgcn_ds_read_tr16_b64_v4f16(
                                          (__attribute__((address_space(3))) ea_fp16x4*)(p)));
}
__device__ __forceinline__ floatx16 ea_mfma(half8 a, half8 b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// Two split_f16 at once: hi = RNE(x) of both by one v_cvt_pk_f16_f32, the
// exact remainders x - hi by one packed subtract, lo = their RNE -- five
// instructions per pair where two split_f16 take eight; the same bits.
typedef _Float16 ea_half2 __attribute__((ext_vector_type(2)));
typedef float ea_float2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split2(float a, float b, ea_half2& hi, ea_half2& lo) {
  hi = __builtin_convertvector((ea_float2){a, b}, ea_half2);
  const ea_float2 r = (ea_float2){a, b} - __builtin_convertvector(hi, ea_float2);
  lo = __builtin_convertvector(r, ea_half2);
}

constexpr int kEaKeys = 64;  // keys per LDS tile
constexpr int kEaLd = 72;    // LDS row stride (halves)

// Registers held to 128 (4 waves per SIMD: two 8-wave workgroups per CU,
// one's staging beside the other's MFMAs); WA_EA_WAVES: A/B builds.
#ifndef WA_EA_WAVES
#define WA_EA_WAVES 4
#endif
template <int NS, int NW>
__global__ __launch_bounds__(64 * NW, WA_EA_WAVES) void encoder_attention_f16_kernel(const float* __restrict__ qkv,
                                                                                    int T, int H,
                                                                                    _Float16* __restrict__ tiled,
                                                                                    float* __restrict__ out32) {
  // two tile buffers: tile kt + 1 is staged into the other one while tile
  // kt is read, one barrier per tile
  __shared__ __attribute__((aligned(16))) _Float16 klsb[2][NS][kEaKeys * kEaLd];
  __shared__ __attribute__((aligned(16))) _Float16 vlsb[2][NS][kEaKeys * kEaLd];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, lh = lane >> 5;
  const int head = blockIdx.y, b = blockIdx.z;
  const int D = H * 64, ld = 3 * D;
  const float* base = qkv + (size_t)b * T * ld;
  const int q = blockIdx.x * (32 * NW) + wave * 32 + l32;

  // Q^T operand (k = dim, n = query): lane (query l32, dims 16 ks + 8 lh + 0..7), scaled by 1/8 (exact)
  half8 qb[4][NS];
  {
    const float* qr = base + (size_t)(q < T ? q : 0) * ld + head * 64;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const floatx4 x0 = *reinterpret_cast<const floatx4*>(qr + 16 * ks + 8 * lh);
      const floatx4 x1 = *reinterpret_cast<const floatx4*>(qr + 16 * ks + 8 * lh + 4);
      half8 hi, lo;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        // q / 8 * log2(e): the scores come out in base-2 units, so the
        // softmax exponentials are single v_exp_f32 (2^x) instructions
        const float v = q < T ? (j < 4 ? x0[j] : x1[j - 4]) * kEaQScale : 0.0f;
        _Float16 a, c;
        split_f16(v * kQKScale, a, c);
        hi[j] = a;
        lo[j] = c;
      }
      qb[ks][0] = hi;
      if constexpr (NS == 2) qb[ks][1] = lo;
    }
  }
  // staging: thread (key tid / TPK, dims EPT (tid % TPK) + 0..EPT-1) of K and V
  constexpr int EPT = 64 * kEaKeys / (64 * NW);  // elements per thread and tensor (16 or 8)
  constexpr int TPK = 64 / EPT;                  // threads per key
  const int skey = tid / TPK, sd = (tid % TPK) * EPT;
  floatx4 kreg[EPT / 4], vreg[EPT / 4];
  auto fetch = [&](int key0) {
    const int key = key0 + skey;
    const bool ok = key < T;
    const float* kr = base + (size_t)(ok ? key : 0) * ld + D + head * 64 + sd;
#pragma unroll
    for (int i = 0; i < EPT / 4; ++i) {
      kreg[i] = ok ? *reinterpret_cast<const floatx4*>(kr + 4 * i) : floatx4{0.f, 0.f, 0.f, 0.f};
      vreg[i] = ok ? *reinterpret_cast<const floatx4*>(kr + D + 4 * i) : floatx4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto stage = [&](int buf) {
    _Float16(*kls)[kEaKeys * kEaLd] = klsb[buf];
    _Float16(*vls)[kEaKeys * kEaLd] = vlsb[buf];
    half8 kh[EPT / 8], kl[EPT / 8], vh[EPT / 8], vl[EPT / 8];
#pragma unroll
    for (int i = 0; i < EPT; i += 2) {
      ea_half2 h2, l2;
      split2(kreg[i >> 2][i & 3] * kQKScale, kreg[i >> 2][(i & 3) + 1] * kQKScale, h2, l2);
      kh[i >> 3][i & 7] = h2[0];
      kh[i >> 3][(i & 7) + 1] = h2[1];
      kl[i >> 3][i & 7] = l2[0];
      kl[i >> 3][(i & 7) + 1] = l2[1];
      split2(vreg[i >> 2][i & 3] * kQKScale, vreg[i >> 2][(i & 3) + 1] * kQKScale, h2, l2);
      vh[i >> 3][i & 7] = h2[0];
      vh[i >> 3][(i & 7) + 1] = h2[1];
      vl[i >> 3][i & 7] = l2[0];
      vl[i >> 3][(i & 7) + 1] = l2[1];
    }
#pragma unroll
    for (int u = 0; u < EPT / 8; ++u) {
      *reinterpret_cast<half8*>(&kls[0][skey * kEaLd + sd + 8 * u]) = kh[u];
      *reinterpret_cast<half8*>(&vls[0][skey * kEaLd + sd + 8 * u]) = vh[u];
      if constexpr (NS == 2) {
        *reinterpret_cast<half8*>(&kls[NS - 1][skey * kEaLd + sd + 8 * u]) = kl[u];
        *reinterpret_cast<half8*>(&vls[NS - 1][skey * kEaLd + sd + 8 * u]) = vl[u];
      }
    }
  };

  float m = -INFINITY, l = 0.0f;
  floatx16 o[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    o[0][i] = 0.0f;
    o[1][i] = 0.0f;
  }
  // transposed-read geometry: 16-lane group g = lane / 16 covers dims
  // 16 (g & 1) + 0..15 and keys 4 (g >> 1) + 0..3 (+ 8): the S^T
  // accumulator's key order for lanes < 32 / >= 32
  const int g = lane >> 4, gi = lane & 15;
  const int trow = 4 * (g >> 1) + (gi >> 2), tcol = 16 * (g & 1) + 4 * (gi & 3);
  const int ntile = (T + kEaKeys - 1) / kEaKeys;
  fetch(0);
  stage(0);
  __syncthreads();
  if (ntile > 1) fetch(kEaKeys);  // tile 1 in flight during tile 0
  for (int kt = 0; kt < ntile; ++kt) {
    const int key0 = kt * kEaKeys;
    const _Float16(*kls)[kEaKeys * kEaLd] = klsb[kt & 1];
    const _Float16(*vls)[kEaKeys * kEaLd] = vlsb[kt & 1];
#pragma unroll
    for (int sub = 0; sub < kEaKeys / 32; ++sub) {
      floatx16 st;
#pragma unroll
      for (int i = 0; i < 16; ++i) st[i] = 0.0f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int off = (sub * 32 + l32) * kEaLd + 16 * ks + 8 * lh;
        const half8 ah = *reinterpret_cast<const half8*>(&kls[0][off]);
        st = ea_mfma(ah, qb[ks][0], st);
        if constexpr (NS == 2) {
          const half8 al = *reinterpret_cast<const half8*>(&kls[1][off]);
          st = ea_mfma(al, qb[ks][0], st);
          st = ea_mfma(ah, qb[ks][1], st);
        }
      }
      // online softmax of query l32 over these 32 keys (16 here, 16 in lane ^ 32)
      if (key0 + sub * 32 + 32 > T) {  // only the last tile holds keys past T (wave-uniform)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = key0 + sub * 32 + (i & 3) + 8 * (i >> 2) + 4 * lh;
          if (key >= T) st[i] = -INFINITY;
        }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int i = 0; i < 16; ++i) mx = fmaxf(mx, st[i]);
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      // lazy reference maximum (as the decoder cross-attention's softmax_entry):
      // the running reference m only moves when the tile's maximum exceeds
      // it by more than 1 (base 2), so p <= 2 and most tiles need no rescale
      // of o (alpha == 1 exactly, skipped when the whole wave agrees); any
      // reference gives the same softmax.  Scores (and m) carry the 2^10
      // operand scale.
      float mn = fmaxf(m, mx);
      if (m != -INFINITY && mn - m <= kEaLazyMax) mn = m;
      const float alpha = __builtin_amdgcn_exp2f((m - mn) * kSInv);  // exp2(-inf) = 0; 1 when mn == m
      float rs = 0.0f;
      // mn is finite: the first 32 keys of tile 0 hold key 0 (< T)
      const float nmn = -mn * kSInv;  // exact (power-of-two scale)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        st[i] = __builtin_amdgcn_exp2f(fmaf(st[i], kSInv, nmn));
        rs += st[i];
      }
      rs += __shfl_xor(rs, 32, 64);
      l = l * alpha + rs;
      m = mn;
      if (__builtin_amdgcn_ballot_w64(alpha != 1.0f) != 0) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          o[0][i] *= alpha;
          o[1][i] *= alpha;
        }
      }
      // P^T operands: MFMA t takes accumulator registers 8 t .. 8 t + 7.
      // p in (0, 2] is split at p * 2^14 (exact scaling; undone at the end)
      // so that the lo part of a small p stays a normal f16: 22 bits for
      // every p >= 2^-17 instead of an absolute 2^-24 floor
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        half8 ph, pl;
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          ea_half2 h2, l2;
          split2(st[8 * t + j] * kPScale, st[8 * t + j + 1] * kPScale, h2, l2);
          ph[j] = h2[0];
          ph[j + 1] = h2[1];
          pl[j] = l2[0];
          pl[j + 1] = l2[1];
        }
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          half8 va[NS];
#pragma unroll
          for (int pp = 0; pp < NS; ++pp) {
            const _Float16* vb = &vls[pp][(sub * 32 + 16 * t + trow) * kEaLd + dt * 32 + tcol];
            const ea_half4 x0 = ea_tr4(vb);
            const ea_half4 x1 = ea_tr4(vb + 8 * kEaLd);
            va[pp] = half8{x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
          }
          o[dt] = ea_mfma(va[0], ph, o[dt]);
          if constexpr (NS == 2) {
            o[dt] = ea_mfma(va[1], ph, o[dt]);
            o[dt] = ea_mfma(va[0], pl, o[dt]);
          }
        }
      }
    }
    // the next tile into the other buffer (its last readers, tile kt - 1,
    // passed the barrier below one iteration ago), then the one after it
    // into registers
    if (kt + 1 < ntile) {
      stage((kt + 1) & 1);
      if (kt + 2 < ntile) fetch(key0 + 2 * kEaKeys);
    }
    __syncthreads();
  }
  if (q < T) {
    const int row = b * T + q;
    const int kbp = kbp_of(D);
    const float inv = (1.0f / l) * kPVInv;  // exact power-of-two rescale of 1 / l
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const int d = dt * 32 + 8 * gg + 4 * lh;
        attn_store4<NS>(tiled, out32, H * 64, row, head * 64 + d, kbp, o[dt][4 * gg] * inv,
                        o[dt][4 * gg + 1] * inv, o[dt][4 * gg + 2] * inv, o[dt][4 * gg + 3] * inv);
      }
  }
}

hipError_t launch_encoder_attention(const float* qkv, int B, int T, int H, _Float16* tiled, int ns,
                                    hipStream_t st, float* out32) {
  // 8 waves x 32 queries per workgroup; when that grid leaves most CUs idle
  // (one or two clips: 120 / 240 workgroups at Large-V3) 4 waves, twice the
  // workgroups (each query's arithmetic is the same either way)
  const bool few = (int64_t)B * H * ((T + 255) / 256) < 256;
  if (few) {
    const dim3 g4((T + 127) / 128, H, B);
    if (ns == 2)
      hipLaunchKernelGGL((encoder_attention_f16_kernel<2, 4>), g4, dim3(256), 0, st, qkv, T, H, tiled, out32);
    else
      hipLaunchKernelGGL((encoder_attention_f16_kernel<1, 4>), g4, dim3(256), 0, st, qkv, T, H, tiled, out32);
    return hipGetLastError();
  }
  const dim3 g2((T + 255) / 256, H, B);
  if (ns == 2)
    hipLaunchKernelGGL((encoder_attention_f16_kernel<2, 8>), g2, dim3(512), 0, st, qkv, T, H, tiled, out32);
  else
    hipLaunchKernelGGL((encoder_attention_f16_kernel<1, 8>), g2, dim3(512), 0, st, qkv, T, H, tiled, out32);
  return hipGetLastError();
}

// ---------------------------------------------- decode-step attention --
// Shared by self- and cross-attention of the decoder (Tq <= 4 queries per
// clip): 16 lanes share one key (4 dims each), 4 keys per load instruction,
// U instructions in flight per wave, online softmax per 16-lane group, then a
// fixed-order merge over the groups of a wave and over the 4 waves.

// Online-softmax scan of keys [k0, k1).  rows(j, kp, vp) yields this lane's
// 4-float K / V pointers of key j; vis(t, j) says whether query t sees key j.
// attn_fetch issues one pass's loads (4 U keys per wave), attn_update folds
// them in; attn_scan alternates the two.  A caller may issue the first pass's
// loads itself before its queries exist.
template <int TQ>
__device__ __forceinline__ void attn_init(float (&m)[TQ], float (&l)[TQ], floatx4 (&o)[TQ]) {
#pragma unroll
  for (int t = 0; t < TQ; ++t) {
    m[t] = -INFINITY;
    l[t] = 0.0f;
    o[t] = floatx4{0.f, 0.f, 0.f, 0.f};
  }
}

template <int U, class Rows>
__device__ __forceinline__ void attn_fetch(int j0, int k1, int grp, Rows rows, floatx4 (&kk)[U], floatx4 (&vv)[U]) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int j = max(0, min(j0 + 4 * u + grp, k1 - 1));  // clamped: loads never branch
    const float *kp, *vp;
    rows(j, kp, vp);
    kk[u] = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(kp));
    vv[u] = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(vp));
  }
}

template <int TQ, int U, class Vis>
__device__ __forceinline__ void attn_update(const floatx4 (&qv)[TQ], int Tq, int j0, int k1, int grp, Vis vis,
                                            const floatx4 (&kk)[U], const floatx4 (&vv)[U], float (&m)[TQ],
                                            float (&l)[TQ], floatx4 (&o)[TQ]) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int j = j0 + 4 * u + grp;
#pragma unroll
    for (int t = 0; t < TQ; ++t) {
      if (t < Tq) {
        const float dot =
            wq4::sum16(qv[t][0] * kk[u][0] + qv[t][1] * kk[u][1] + qv[t][2] * kk[u][2] + qv[t][3] * kk[u][3]);
        if (j < k1 && vis(t, j)) {
          const float mn = fmaxf(m[t], dot);
          const float alpha = __builtin_amdgcn_exp2f(m[t] - mn);  // base-2 units
          const float p = __builtin_amdgcn_exp2f(dot - mn);
          l[t] = l[t] * alpha + p;
          o[t] = o[t] * alpha + vv[u] * p;
          m[t] = mn;
        }
      }
    }
  }
}

template <int TQ, int U, class Rows, class Vis>
__device__ __forceinline__ void attn_scan(const floatx4 (&qv)[TQ], int Tq, int k0, int k1, int grp, Rows rows,
                                          Vis vis, float (&m)[TQ], float (&l)[TQ], floatx4 (&o)[TQ]) {
  attn_init<TQ>(m, l, o);
  for (int j0 = k0; j0 < k1; j0 += 4 * U) {
    floatx4 kk[U], vv[U];
    attn_fetch<U>(j0, k1, grp, rows, kk, vv);
    attn_update<TQ, U>(qv, Tq, j0, k1, grp, vis, kk, vv, m, l, o);
  }
}

// Merge the 4 groups of each wave, then the NWV waves, in a fixed order.  Wave
// t (< Tq) returns query t's (mn, ls, os = unnormalised o[lane]).
template <int TQ, int NWV>
__device__ __forceinline__ void attn_merge(int Tq, int wave, int lane, float (&m)[TQ], float (&l)[TQ],
                                           floatx4 (&o)[TQ], float (&wm)[NWV][TQ], float (&wl)[NWV][TQ],
                                           float (&wo)[NWV][TQ][64], float& mn, float& ls, float& os) {
  const int sub = lane & 15, grp = lane >> 4;
#pragma unroll
  for (int t = 0; t < TQ; ++t) {
    if (t >= Tq) break;
#pragma unroll
    for (int off = 16; off < 64; off <<= 1) {
      const float m2 = __shfl_xor(m[t], off, 64), l2 = __shfl_xor(l[t], off, 64);
      floatx4 o2;
#pragma unroll
      for (int e = 0; e < 4; ++e) o2[e] = __shfl_xor(o[t][e], off, 64);
      const float mx = fmaxf(m[t], m2);
      const float a1 = m[t] == -INFINITY ? 0.0f : __builtin_amdgcn_exp2f(m[t] - mx);
      const float a2 = m2 == -INFINITY ? 0.0f : __builtin_amdgcn_exp2f(m2 - mx);
      l[t] = l[t] * a1 + l2 * a2;
      o[t] = o[t] * a1 + o2 * a2;
      m[t] = mx;
    }
    if (grp == 0) {
#pragma unroll
      for (int e = 0; e < 4; ++e) wo[wave][t][sub * 4 + e] = o[t][e];
    }
    if (lane == 0) {
      wm[wave][t] = m[t];
      wl[wave][t] = l[t];
    }
  }
  __syncthreads();
  mn = -INFINITY;
  ls = 0.0f;
  os = 0.0f;
  if (wave < Tq) {
    const int t = wave;
#pragma unroll
    for (int w = 0; w < NWV; ++w) mn = fmaxf(mn, wm[w][t]);
#pragma unroll
    for (int w = 0; w < NWV; ++w) {
      const float a = wm[w][t] == -INFINITY ? 0.0f : __builtin_amdgcn_exp2f(wm[w][t] - mn);
      ls += wl[w][t] * a;
      os += wo[w][t][lane] * a;
    }
  }
}

// ------------------------------------------ decoder self-attention --
// One workgroup per (head, clip); the 4 waves split the keys 0 .. kv_len +
// Tq - 1 (causal inside the new tokens).  Self-K/V caches are head-major
// [clip][head][ctx][64] (contiguous per (clip, head)); the Tq new keys are
// appended there for later steps and read here straight from the qkv rows.
constexpr int kMaxCtx = 448;

template <int NS, int TQ>
__global__ __launch_bounds__(256) void dec_self_attn_kernel(const float* __restrict__ qkv, float* __restrict__ ck,
                                                            float* __restrict__ cv, int Tq_, int H, int ctx,
                                                            const DecodeState* state, int kv_len_host,
                                                            _Float16* __restrict__ tiled, float* __restrict__ out32) {
  const int Tq = TQ == 1 ? 1 : Tq_;
  __shared__ float wm[4][TQ], wl[4][TQ];
  __shared__ float wo[4][TQ][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int head = blockIdx.x, b = blockIdx.y;
  const int D = H * 64;
  const int sub = lane & 15, grp = lane >> 4;
  const int kv_len = state ? state->kv_len : kv_len_host;
  const size_t hb = ((size_t)b * H + head) * ctx * 64;
  floatx4 qv[TQ];
  const float* kb = ck + hb + sub * 4;
  const float* vb = cv + hb + sub * 4;
  const float* newb = qkv + (size_t)b * Tq * 3 * D + D + head * 64 + sub * 4;
  // append the new keys / values (decoder.rs:77-112 via Tensor::cat)
  if (tid < Tq * 16) {
    const int t = tid >> 4, s4 = (tid & 15) * 4;
    const float* src = qkv + (size_t)(b * Tq + t) * 3 * D + head * 64 + s4;
    *reinterpret_cast<floatx4*>(ck + hb + (size_t)(kv_len + t) * 64 + s4) = *reinterpret_cast<const floatx4*>(src + D);
    *reinterpret_cast<floatx4*>(cv + hb + (size_t)(kv_len + t) * 64 + s4) =
        *reinterpret_cast<const floatx4*>(src + 2 * D);
  }
#pragma unroll
  for (int t = 0; t < TQ; ++t)
    qv[t] = t < Tq ? *reinterpret_cast<const floatx4*>(qkv + (size_t)(b * Tq + t) * 3 * D + head * 64 + sub * 4) *
                         kEaQScale
                   : floatx4{0.f, 0.f, 0.f, 0.f};
  const int nk = kv_len + Tq;
  const int per_wave = (nk + 3) / 4;
  const int k0 = min(nk, wave * per_wave), k1 = min(nk, k0 + per_wave);
  float m[TQ], l[TQ];
  floatx4 o[TQ];
  attn_scan<TQ, 8>(
      qv, Tq, k0, k1, grp,
      [&](int j, const float*& kp, const float*& vp) {
        if (j < kv_len) {
          kp = kb + (size_t)j * 64;
          vp = vb + (size_t)j * 64;
        } else {  // this step's own keys: not yet visible through the cache
          kp = newb + (size_t)(j - kv_len) * 3 * D;
          vp = kp + D;
        }
      },
      [&](int t, int j) { return j <= kv_len + t; }, m, l, o);
  float mn, ls, os;
  attn_merge<TQ, 4>(Tq, wave, lane, m, l, o, wm, wl, wo, mn, ls, os);
  if (wave < Tq) {
    const int t = wave;
    const float val = os / ls;
    const float v1 = __shfl_down(val, 1, 64), v2 = __shfl_down(val, 2, 64), v3 = __shfl_down(val, 3, 64);
    if ((lane & 3) == 0) attn_store4<NS>(tiled, out32, D, b * Tq + t, head * 64 + lane, kbp_of(D), val, v1, v2, v3);
  }
}

hipError_t launch_decoder_self_attention(const float* qkv, float* cache_k, float* cache_v, int B, int Tq, int H,
                                         int ctx, const DecodeState* state, int kv_len_host, _Float16* tiled,
                                         int ns, hipStream_t st, float* out32) {
  if (Tq > 4 || ctx > kMaxCtx) return hipErrorInvalidValue;
  const dim3 grid(H, B), block(256);
#define WA_SELF(NS_, TQ_)                                                                                     \
  hipLaunchKernelGGL((dec_self_attn_kernel<NS_, TQ_>), grid, block, 0, st, qkv, cache_k, cache_v, Tq, H, ctx, \
                     state, kv_len_host, tiled, out32)
  if (ns == 2) {
    if (Tq == 1) { WA_SELF(2, 1); } else { WA_SELF(2, 4); }
  } else {
    if (Tq == 1) { WA_SELF(1, 1); } else { WA_SELF(1, 4); }
  }
#undef WA_SELF
  return hipGetLastError();
}

// ------------------------- cross-attention over cached K / V (few clips) --
// The reference's own formulation (attention.rs:177-206 forward_init_cache:
// K = enc Wk^T, V = enc Wv^T + bv cached per layer; :208-236 / 243-298
// forward_with_cache: softmax(q K^T / 8) V), for decode groups of a few
// clips: there the step is a latency chain, and one GEMV launch over the
// cached K / V (f32, head-major [clip][head][T][64], written by the
// head-major Q4 GEMM after the encoder) replaces the four launches of the
// cache-free form (wa_xattn.hip).  Products are f32 x f32 (exact), sums and
// softmax f32, as the reference's.
//
// Grid (H * S, B): the T keys of each (head, clip) are split over S
// workgroups (S from T only: a clip's bits do not depend on its batch).
// Each publishes (o[64], m, l) per query write-through (sc1 stores); the
// last arriver of the (clip, head), told by its counter ticket, merges the S
// partials in split order (sc1 loads; MI355X_MICROARCH.md hand-off table,
// row 1) and writes the A-tiled operand of the output projection.
constexpr int kXkvMaxSplit = 32;
constexpr int kXkvPart = 68;  // floats per (query) partial: o[64], m, l, pad

// 188 keys per split (8 splits at T = 1500, <= 47 keys per wave: one
// 12-deep scan pass); measured at one clip (Large-V3, in the decode step):
// 9.2 us per launch vs 9.9 at 96 keys, 11.1 at 375, 13.4 at 48 (r03).  A
// function of T only: a clip's bits do not depend on its batch.
constexpr int kXkvKeys = 188;
int cross_attention_kv_splits(int T) {
  const int s = (T + kXkvKeys - 1) / kXkvKeys;
  return s < 1 ? 1 : (s > kXkvMaxSplit ? kXkvMaxSplit : s);
}

template <int NS, int TQ>
__global__ __launch_bounds__(256) void cross_attn_kv_kernel(const float* __restrict__ q, const float* __restrict__ kc,
                                                            const float* __restrict__ vc, int Tq_, int T, int H,
                                                            int S, float* __restrict__ part,
                                                            int* __restrict__ counters,
                                                            _Float16* __restrict__ tiled, float* __restrict__ out32) {
  constexpr int U = TQ == 1 ? 12 : 8;  // <= 48 keys per wave in flight at once (decode step)
  const int Tq = TQ == 1 ? 1 : Tq_;
  __shared__ float wm[4][TQ], wl[4][TQ];
  __shared__ float wo[4][TQ][64];
  __shared__ int last_flag;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int head = blockIdx.x / S, split = blockIdx.x - head * S, b = blockIdx.y;
  const int D = H * 64;
  const int sub = lane & 15, grp = lane >> 4;
  const int per_split = (T + S - 1) / S;
  const int s0 = min(T, split * per_split), s1 = min(T, s0 + per_split);
  const int per_wave = (s1 - s0 + 3) / 4;
  const int k0 = min(s1, s0 + wave * per_wave), k1 = min(s1, k0 + per_wave);
  const size_t hofs = ((size_t)b * H + head) * T * 64 + sub * 4;
  const float* kb = kc + hofs;
  const float* vb = vc + hofs;
  auto rows = [&](int j, const float*& kp, const float*& vp) {
    kp = kb + (size_t)j * 64;
    vp = vb + (size_t)j * 64;
  };
  float m[TQ], l[TQ];
  floatx4 o[TQ];
  floatx4 qv[TQ];
  attn_init<TQ>(m, l, o);
#pragma unroll
  for (int t = 0; t < TQ; ++t)
    qv[t] = t < Tq ? *reinterpret_cast<const floatx4*>(q + (size_t)(b * Tq + t) * D + head * 64 + sub * 4) *
                         kEaQScale
                   : floatx4{0.f, 0.f, 0.f, 0.f};
  for (int j0 = k0; j0 < k1; j0 += 4 * U) {
    floatx4 kk[U], vv[U];
    attn_fetch<U>(j0, k1, grp, rows, kk, vv);
    attn_update<TQ, U>(qv, Tq, j0, k1, grp, [](int, int) { return true; }, kk, vv, m, l, o);
  }
  float mn, ls, os;
  attn_merge<TQ, 4>(Tq, wave, lane, m, l, o, wm, wl, wo, mn, ls, os);
  if (S > 1) {
    typedef __attribute__((address_space(1))) float gfloat;
    typedef __attribute__((address_space(1))) int gint;
    const size_t bh = (size_t)b * H + head;
    if (wave < Tq) {  // this split's partial, write-through
      gfloat* pp = (gfloat*)(part + ((bh * S + split) * 4 + wave) * kXkvPart);
      __hip_atomic_store(pp + lane, os, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (lane == 0) __hip_atomic_store(pp + 64, mn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (lane == 1) __hip_atomic_store(pp + 65, ls, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains before the ticket
    __syncthreads();
    if (tid == 0) {
      const int prev = __hip_atomic_fetch_add((gint*)(counters + bh), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last_flag = prev == S - 1;
      if (prev == S - 1) __hip_atomic_store((gint*)(counters + bh), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!last_flag || wave >= Tq) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler-only: the loads stay below the ticket
    // merge the S partials in split order (sc1 loads of sc1-stored bytes)
    float po[kXkvMaxSplit], pm[kXkvMaxSplit], pl[kXkvMaxSplit];
#pragma unroll
    for (int sp = 0; sp < kXkvMaxSplit; ++sp) {
      if (sp < S) {
        gfloat* pp = (gfloat*)(part + ((bh * S + sp) * 4 + wave) * kXkvPart);
        po[sp] = __hip_atomic_load(pp + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        pm[sp] = __hip_atomic_load(pp + 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        pl[sp] = __hip_atomic_load(pp + 65, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    mn = -INFINITY;
#pragma unroll
    for (int sp = 0; sp < kXkvMaxSplit; ++sp)
      if (sp < S) mn = fmaxf(mn, pm[sp]);
    ls = 0.0f;
    os = 0.0f;
#pragma unroll
    for (int sp = 0; sp < kXkvMaxSplit; ++sp) {
      if (sp < S) {
        const float a = pm[sp] == -INFINITY ? 0.0f : __builtin_amdgcn_exp2f(pm[sp] - mn);
        ls += pl[sp] * a;
        os += po[sp] * a;
      }
    }
  }
  if (wave < Tq) {
    const int t = wave;
    const float val = os / ls;
    const float v1 = __shfl_down(val, 1, 64), v2 = __shfl_down(val, 2, 64), v3 = __shfl_down(val, 3, 64);
    if ((lane & 3) == 0) attn_store4<NS>(tiled, out32, D, b * Tq + t, head * 64 + lane, kbp_of(D), val, v1, v2, v3);
  }
}

size_t cross_attention_kv_part_floats(int B, int H, int T) {
  return (size_t)B * H * cross_attention_kv_splits(T) * 4 * kXkvPart;
}

hipError_t launch_cross_attention_kv(const float* q, const float* k, const float* v, int B, int Tq, int T, int H,
                                     float* part, int* counters, _Float16* tiled, int ns, hipStream_t st,
                                     float* out32) {
  if (Tq < 1 || Tq > 4 || B < 1 || T < 1 || H < 1 || !q) return hipErrorInvalidValue;
  const int S = cross_attention_kv_splits(T);
  const dim3 grid(H * S, B), block(256);
#define WA_XKV(NS_, TQ_)                                                                                           \
  hipLaunchKernelGGL((cross_attn_kv_kernel<NS_, TQ_>), grid, block, 0, st, q, k, v, Tq, T, H, S, part, counters, \
                     tiled, out32)
  if (ns == 2) {
    if (Tq == 1) { WA_XKV(2, 1); } else { WA_XKV(2, 4); }
  } else {
    if (Tq == 1) { WA_XKV(1, 1); } else { WA_XKV(1, 4); }
  }
#undef WA_XKV
  return hipGetLastError();
}

// ------------------------------------------------------ conv + GELU --
// out[b, t, n] = gelu(bias[n] + sum_{kk, c} in(b, c, t*S + kk - 1) W[n, c, kk])
// (+ pos[t, n]).  GEMM view: rows (b, t), cols n, K = 3C (k = kk*C + c, the
// reference's im2col order, layers.rs:92-121).
constexpr int kCvLd = 40;
template <int NS>
__global__ __launch_bounds__(256) void conv_gelu_f16_kernel(const float* __restrict__ in, long in_bs, long in_cs,
                                                            long in_ts, int B, int C, int T_in, int S,
                                                            const float* __restrict__ wt,
                                                            const float* __restrict__ bias,
                                                            const float* __restrict__ pos, int N,
                                                            float* __restrict__ out, int T_out) {
  __shared__ __attribute__((aligned(16))) _Float16 as[NS][128 * kCvLd];
  __shared__ __attribute__((aligned(16))) _Float16 bs[NS][128 * kCvLd];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, lh = lane >> 5;
  const int M = B * T_out, K = 3 * C;
  const int m0 = blockIdx.x * 128, n0 = blockIdx.y * 128;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][c][i] = 0.0f;
  auto put = [&](_Float16 (&dst)[NS][128 * kCvLd], int row, int kl, floatx4 v, float scale) {
    ea_half4 hi, lo;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      _Float16 a, b;
      split_f16(v[j] * scale, a, b);
      hi[j] = a;
      lo[j] = b;
    }
    *reinterpret_cast<ea_half4*>(&dst[0][row * kCvLd + kl]) = hi;
    if constexpr (NS == 2) *reinterpret_cast<ea_half4*>(&dst[NS - 1][row * kCvLd + kl]) = lo;
  };
  for (int kc = 0; kc < K; kc += 32) {
    // stage A (im2col gather) and B: 128 rows x 32 k each, (row, 4 k) per item
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int e = it * 256 + tid;
      const int ml = e >> 3, kl = (e & 7) * 4;
      const int m = m0 + ml, k = kc + kl;
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      if (m < M && k < K) {
        const int bb = m / T_out, t = m - bb * T_out;
        if (in_cs == 1) {  // 4 consecutive channels of one tap (C % 4 == 0)
          const int kk = k / C, c = k - kk * C;
          const int ti = t * S + kk - 1;
          if (ti >= 0 && ti < T_in) v = *reinterpret_cast<const floatx4*>(in + bb * in_bs + c + (long)ti * in_ts);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int kj = k + j, kk = kj / C, c = kj - kk * C;
            const int ti = t * S + kk - 1;
            if (kj < K && ti >= 0 && ti < T_in) v[j] = in[bb * in_bs + c * in_cs + (long)ti * in_ts];
          }
        }
      }
      put(as, ml, kl, v, kCvAScale);
    }
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int e = it * 256 + tid;
      const int nl = e >> 3, kl = (e & 7) * 4;
      const int n = n0 + nl, k = kc + kl;
      const floatx4 v = (n < N && k + 3 < K) ? *reinterpret_cast<const floatx4*>(wt + (size_t)n * K + k)
                                             : floatx4{0.f, 0.f, 0.f, 0.f};
      put(bs, nl, kl, v, kCvBScale);
    }
    __syncthreads();
#pragma unroll
    for (int k16 = 0; k16 < 2; ++k16) {
      half8 a[2][NS], b[2][NS];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int p = 0; p < NS; ++p) {
          a[i][p] = *reinterpret_cast<const half8*>(&as[p][(wm + 32 * i + l32) * kCvLd + 16 * k16 + 8 * lh]);
          b[i][p] = *reinterpret_cast<const half8*>(&bs[p][(wn + 32 * i + l32) * kCvLd + 16 * k16 + 8 * lh]);
        }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = ea_mfma(a[i][0], b[j][0], acc[i][j]);
          if constexpr (NS == 2) {
            acc[i][j] = ea_mfma(a[i][1], b[j][0], acc[i][j]);
            acc[i][j] = ea_mfma(a[i][0], b[j][1], acc[i][j]);
          }
        }
    }
    __syncthreads();
  }
  // acc[i][j]: A = rows (m), B = cols (n): lane holds column n = l32, rows (r & 3) + 8 (r >> 2) + 4 lh
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int m = m0 + wm + 32 * a + (i & 3) + 8 * (i >> 2) + 4 * lh;
        const int n = n0 + wn + 32 * c + l32;
        if (m < M && n < N) {
          float v = wq4::gelu_tanh(acc[a][c][i] * kCvInv + bias[n]);
          if (pos) v = v + pos[(size_t)(m % T_out) * N + n];
          out[(size_t)m * N + n] = v;
        }
      }
}

hipError_t launch_conv_gelu(const float* in, long in_bs, long in_cs, long in_ts, int B, int C, int T_in,
                            int stride, const float* w_t, const float* bias, const float* pos, int N, float* out,
                            hipStream_t st) {
  if (C % 4 != 0) return hipErrorInvalidValue;  // float4 channel staging (n_mels 80 / 128, D)
  const int T_out = (T_in + 2 - 3) / stride + 1;
  const dim3 grid((B * T_out + 127) / 128, (N + 127) / 128), block(256);
  hipLaunchKernelGGL(conv_gelu_f16_kernel<2>, grid, block, 0, st, in, in_bs, in_cs, in_ts, B, C, T_in, stride, w_t,
                     bias, pos, N, out, T_out);
  return hipGetLastError();
}

// ----------------------------------------------------------- embedding --
__global__ void embed_kernel(const int* __restrict__ tokens, const float* __restrict__ te,
                             const float* __restrict__ pe, int Tq, int D, const DecodeState* state, int pos0,
                             float* __restrict__ x) {
  const int row = blockIdx.x;  // b * Tq + t
  const int t = row % Tq;
  const int p = (state ? state->position : pos0) + t;
  const int tok = tokens[row];
  for (int d = threadIdx.x; d < D; d += blockDim.x)
    x[(size_t)row * D + d] = te[(size_t)tok * D + d] + pe[(size_t)p * D + d];
}

hipError_t launch_embed(const int* tokens, const float* tok_emb, const float* pos_emb, int B, int Tq, int D,
                        const DecodeState* state, int pos0_host, float* x, hipStream_t st) {
  hipLaunchKernelGGL(embed_kernel, dim3(B * Tq), dim3(256), 0, st, tokens, tok_emb, pos_emb, Tq, D, state,
                     pos0_host, x);
  return hipGetLastError();
}

// Embedding + the LayerNorm-fold producer of the first decoder layer's
// attn_ln (wq4_gemm_tiled_lnfold): x rows as embed_kernel, plus the A-tiled
// operand of x * gamma and per (row, 32-column tile) the tile mean and sum
// of squared deviations.  One workgroup per row; thread t owns the float4 at
// columns 4 t + 1024 i, so a tile is 8 consecutive lanes.
template <int NS>
__global__ __launch_bounds__(256) void embed_fold_kernel(const int* __restrict__ tokens, const float* __restrict__ te,
                                                         const float* __restrict__ pe, int Tq, int D,
                                                         const DecodeState* state, int pos0, float* __restrict__ x,
                                                         const float* __restrict__ gamma, _Float16* __restrict__ at,
                                                         float* __restrict__ stats) {
  const int row = blockIdx.x;  // b * Tq + t
  const int t = row % Tq;
  const int p = (state ? state->position : pos0) + t;
  const int tok = tokens[row];
  const int kbp = kbp_of(D);
  for (int c = 4 * threadIdx.x; c < ((D + 1023) / 1024) * 1024; c += 1024) {
    const bool in = c < D;  // D % 32 == 0: a tile is wholly in or out
    floatx4 v = {0.f, 0.f, 0.f, 0.f}, g = {0.f, 0.f, 0.f, 0.f};
    if (in) {
      const floatx4 a = *reinterpret_cast<const floatx4*>(te + (size_t)tok * D + c);
      const floatx4 b = *reinterpret_cast<const floatx4*>(pe + (size_t)p * D + c);
      g = *reinterpret_cast<const floatx4*>(gamma + c);
      v = a + b;
      *reinterpret_cast<floatx4*>(x + (size_t)row * D + c) = v;
      atile_store4<NS>(at, row, c, kbp, v[0] * g[0], v[1] * g[1], v[2] * g[2], v[3] * g[3]);
    }
    // statistics per 16-column tile (the decode-step GEMM's LayerNorm fold)
    float sum = (v[0] + v[1]) + (v[2] + v[3]);
#pragma unroll
    for (int o = 1; o < 4; o <<= 1) sum += __shfl_xor(sum, o, 64);
    const float mean = sum * (1.0f / 16.0f);
    float m2 = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) m2 += (v[j] - mean) * (v[j] - mean);
#pragma unroll
    for (int o = 1; o < 4; o <<= 1) m2 += __shfl_xor(m2, o, 64);
    if (in && (threadIdx.x & 3) == 0) {
      float* st = stats + ((size_t)row * (D / 16) + c / 16) * 2;
      st[0] = mean;
      st[1] = m2;
    }
  }
}

hipError_t launch_embed_fold(const int* tokens, const float* tok_emb, const float* pos_emb, int B, int Tq, int D,
                             const DecodeState* state, int pos0_host, float* x, const float* gamma, _Float16* at,
                             float* stats, int ns, hipStream_t st) {
  if (D % 32 != 0) return hipErrorInvalidValue;
  if (ns == 2)
    hipLaunchKernelGGL(embed_fold_kernel<2>, dim3(B * Tq), dim3(256), 0, st, tokens, tok_emb, pos_emb, Tq, D, state,
                       pos0_host, x, gamma, at, stats);
  else
    hipLaunchKernelGGL(embed_fold_kernel<1>, dim3(B * Tq), dim3(256), 0, st, tokens, tok_emb, pos_emb, Tq, D, state,
                       pos0_host, x, gamma, at, stats);
  return hipGetLastError();
}

// -------------------------------------------------------------- logits --
// logits[b, v] = sum_d h[b, d] E[v, d]; B <= 32 clips per call.  One wave =
// 32 vocabulary rows; h staged in LDS in 256-wide k chunks.
__global__ __launch_bounds__(256) void logits_kernel(const float* __restrict__ hid, int B, int D, long ldh,
                                                     const float* __restrict__ emb, int V,
                                                     float* __restrict__ logits) {
  __shared__ float hs[32][256 + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int n = blockIdx.x * 128 + wave * 32 + r;
  const float* er = emb + (size_t)(n < V ? n : 0) * D;
  floatx16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
  for (int kc = 0; kc < D; kc += 256) {
    const int kw = min(256, D - kc);
    __syncthreads();
    for (int e = tid; e < 32 * 256; e += 256) {
      const int row = e >> 8, k = e & 255;
      hs[row][k] = (row < B && k < kw) ? hid[(size_t)row * ldh + kc + k] : 0.0f;
    }
    __syncthreads();
    for (int k8 = 0; k8 < kw; k8 += 8) {
      const floatx4 e4 = n < V ? *reinterpret_cast<const floatx4*>(er + kc + k8 + 4 * h) : floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = mfma_f32(hs[r][k8 + 4 * h + s], e4[s], acc);
    }
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
    if (row < B && n < V) logits[(size_t)row * V + n] = acc[i];
  }
}

hipError_t launch_logits(const float* h, int B, int D, long ldh, const float* emb, int V, float* logits,
                         hipStream_t st) {
  for (int b0 = 0; b0 < B; b0 += 32) {
    const int nb = min(32, B - b0);
    hipLaunchKernelGGL(logits_kernel, dim3((V + 127) / 128), dim3(256), 0, st, h + (size_t)b0 * ldh, nb, D, ldh,
                       emb, V, logits + (size_t)b0 * V);
  }
  return hipGetLastError();
}

// -------------------------------------------------------------- argmax --
// Rust `max_by(partial_cmp)` keeps the LAST of equal maxima (whisper.rs:131-138).
__device__ __forceinline__ void better(float& bv, int& bi, float v, int i) {
  if (v > bv || (v == bv && i > bi)) {
    bv = v;
    bi = i;
  }
}

__global__ __launch_bounds__(256) void argmax_kernel(const float* __restrict__ logits, int V, int lo, int hi,
                                                     int suppress_fixed, int min_tokens, const DecodeState* state,
                                                     int* __restrict__ out, int out_stride, int* __restrict__ range_flag) {
  __shared__ float sv[4];
  __shared__ int si[4];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* lg = logits + (size_t)b * V;
  const int suppress = state ? (state->step + 1 < min_tokens) : suppress_fixed;
  float bv = -INFINITY;
  int bi = -1;
  bool bad = false;
  for (int i = lo + tid; i < hi; i += 256) {
    float v = lg[i];
    bad |= !__builtin_isfinite(v);
    if (suppress && i == kEOT) v = -INFINITY;
    better(bv, bi, v, i);
  }
  if (bad && range_flag) *range_flag = 1;  // plain vector store: every writer stores 1
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float v = __shfl_xor(bv, o, 64);
    const int i = __shfl_xor(bi, o, 64);
    better(bv, bi, v, i);
  }
  if (lane == 0) {
    sv[wave] = bv;
    si[wave] = bi;
  }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < 4; ++w) better(bv, bi, sv[w], si[w]);
    out[(size_t)b * out_stride] = bi < 0 ? lo : bi;
  }
}

hipError_t launch_argmax(const float* logits, int B, int V, int lo, int hi, int suppress_eot,
                         const DecodeState* state, int* out_tok, int out_stride, int* range_flag, hipStream_t st) {
  hipLaunchKernelGGL(argmax_kernel, dim3(B), dim3(256), 0, st, logits, V, lo, hi, suppress_eot, 0,
                     (const DecodeState*)nullptr, out_tok, out_stride, range_flag);
  (void)state;
  return hipGetLastError();
}

hipError_t launch_argmax_step(const float* logits, int B, int V, int min_tokens, const DecodeState* state,
                              int* out_tok, int* range_flag, hipStream_t st) {
  hipLaunchKernelGGL(argmax_kernel, dim3(B), dim3(256), 0, st, logits, V, 0, V, 0, min_tokens, state, out_tok, 1,
                     range_flag);
  return hipGetLastError();
}

// ------------------------------------------------ logits + greedy pick --
// Decode step (B <= 32 clips): logits[b, v] = h[b] . E[v] (decoder.rs:289-292)
// fused with the greedy argmax (whisper.rs:119-124, 131-138) -- the logits
// never reach HBM (logits_argmax_f16_k32_kernel below).  Each workgroup
// leaves one (max, index) candidate per clip; the last-arriving workgroup
// (agent-scope ticket, write-through partials: cdna_hip_programming.md
// Guideline 16 R1) reduces them.  (value, index) is compared
// lexicographically -- the largest value, the LARGEST index among equal
// maxima -- so the result equals the sequential Rust max_by scan whatever the
// reduction order.

__device__ __forceinline__ void better_pair(float& bv, int& bi, float v, int i) {
  if (v > bv || (v == bv && i > bi)) {
    bv = v;
    bi = i;
  }
}

// Greedy pick of a workgroup's 32 x 128 logits block lg[clip][kLgPickLd]
// (already masked), then the last-arriving workgroup's pick over all
// workgroups' candidates.
constexpr int kLgPickLd = 132;
__device__ __forceinline__ void pick_from_lds(const float* lg, int B, int V, float* __restrict__ pval,
                                              int* __restrict__ pidx, int* __restrict__ counter,
                                              int* __restrict__ out_tok, int* ticket) {
  const int tid = threadIdx.x, nwg = gridDim.x;
  __syncthreads();
  const int row = tid >> 3, part = tid & 7;
  float bv = -INFINITY;
  int bi = -1;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int c = part * 16 + j;
    const int idx = blockIdx.x * 128 + c;
    if (idx < V) better_pair(bv, bi, lg[row * kLgPickLd + c], idx);
  }
#pragma unroll
  for (int o = 1; o < 8; o <<= 1) {
    const float v2 = __shfl_xor(bv, o, 64);
    const int i2 = __shfl_xor(bi, o, 64);
    better_pair(bv, bi, v2, i2);
  }
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(pval, 0, 32 * nwg * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc(pidx, 0, 32 * nwg * 4, 0x00020000);
  if (part == 0 && row < B) {
    const uint32_t off = (uint32_t)(row * nwg + blockIdx.x) * 4;
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, bv), rv, off, 0, 16);  // sc1
    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)bi, ri, off, 0, 16);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    typedef __attribute__((address_space(1))) int gint;
    const int prev = __hip_atomic_fetch_add((gint*)counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *ticket = prev == nwg - 1;
  }
  __syncthreads();
  if (!*ticket) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler-only: loads stay below the ticket
  bv = -INFINITY;
  bi = -1;
  if (row < B) {
    for (int j = part; j < nwg; j += 8) {
      const uint32_t off = (uint32_t)(row * nwg + j) * 4;
      const float v = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rv, off, 0, 16));
      const int i = (int)__builtin_amdgcn_raw_buffer_load_b32(ri, off, 0, 16);
      better_pair(bv, bi, v, i);
    }
  }
#pragma unroll
  for (int o = 1; o < 8; o <<= 1) {
    const float v2 = __shfl_xor(bv, o, 64);
    const int i2 = __shfl_xor(bi, o, 64);
    better_pair(bv, bi, v2, i2);
  }
  if (part == 0 && row < B) out_tok[row] = bi < 0 ? 0 : bi;
  if (tid == 0) {
    typedef __attribute__((address_space(1))) int gint;
    __hip_atomic_store((gint*)counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
  }
}

constexpr int kLg2Chunk = 128;
// 16-row groups of the fragment-tiled table (V padded to 128-row workgroups)
__host__ __device__ inline int64_t emb_groups16(int V) { return (int64_t)(V + 127) / 128 * 8; }

// Tied-embedding logits of the decode step on f16 MFMA, fused with the greedy
// pick: the embedding as exact-to-2^-22 f16 pairs E = hi + lo in a
// fragment-tiled table (launch_emb_tiled: a lane's fragment is 8 dims of one
// of 16 rows, one load instruction reads 1 KiB contiguous), the hidden rows
// as the A-tiled f16-pair operand the final LayerNorm writes (wq4_layernorm,
// the same split as the GEMMs); three 16x16x32 f16 MFMAs per product
// (hi*hi + lo*hi + hi*lo), f32 accumulation.  Wave = 32 vocabulary rows as
// two 16-row m-tiles, the 32 clips as two n-tiles.  Per 128-dim chunk the
// hidden fragments (32 rows x 128 dims, 8 or 16 KiB) come into an LDS double
// buffer through registers one chunk ahead, beside the next chunk's table
// fragments in registers: one barrier per chunk, no conversion.  trace_out
// (diagnostics, null in the product graph): the logits of
// trace_ids[clip][step + 1][0..trace_k) are written to the same slots of
// trace_out, as the pick sees them (EOT already masked).
template <int NS>
__global__ __launch_bounds__(256) void logits_argmax_f16_k32_kernel(
    const _Float16* __restrict__ htiled, int B, int D, const _Float16* __restrict__ emb2, int V, int min_tokens,
    const DecodeState* __restrict__ state, float* __restrict__ pval, int* __restrict__ pidx, int* __restrict__ counter,
    int* __restrict__ out_tok, const int* __restrict__ trace_ids, float* __restrict__ trace_out, int trace_s1,
    int trace_k, int* __restrict__ range_flag) {
  constexpr int KS = kLg2Chunk / 32;             // Q4-block-sized k-steps per chunk
  constexpr int HCH = KS * 2 * NS * 1024;        // bytes of hidden fragments per chunk
  static_assert(HCH % (256 * 16) == 0, "whole glds rounds");
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * HCH + 32 * kLgPickLd * 4 + 16];
  float* lg = reinterpret_cast<float*>(smem + 2 * HCH);
  int* ticket = reinterpret_cast<int*>(smem + 2 * HCH + 32 * kLgPickLd * 4);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l16 = lane & 15, lq = lane >> 4;
  const int v0 = blockIdx.x * 128 + wave * 32;
  // chunk-major table (launch_emb_tiled): this wave's two 16-row groups are
  // 2 KS NS KiB contiguous per chunk, and a chunk of the whole table is one
  // contiguous stretch (every wave streams the same region at once)
  const int nch = D / kLg2Chunk;
  const size_t chunk_halves = (size_t)emb_groups16(V) * KS * NS * 512;
  const _Float16* er = emb2 + (size_t)(v0 / 16) * KS * NS * 512 + lane * 8;
  floatx4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
  half8 ec[2][KS][NS], en[2][KS][NS];
  auto load_e = [&](half8 (&e)[2][KS][NS], int kc) {
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int p = 0; p < NS; ++p)  // D % kLg2Chunk == 0 (launcher): always in range
          e[mt][ks][p] = WA_LOGITS_NT ? __builtin_nontemporal_load(reinterpret_cast<const half8*>(
                                            er + (kc / kLg2Chunk) * chunk_halves + ((mt * KS + ks) * NS + p) * 512))
                                      : *reinterpret_cast<const half8*>(er + (kc / kLg2Chunk) * chunk_halves +
                                                                         ((mt * KS + ks) * NS + p) * 512);
  };
  // the hidden fragments of chunk c: A-tiled m-tile 0, blocks 4c .. 4c + 3
  // (kk, plane, lane: 1 KiB each, contiguous), staged through registers into
  // LDS buffer c & 1 lane-linear.  Not global_load_lds: while an LDS DMA is in
  // flight hipcc waits vmcnt(0) at the first use of any ordinary load result
  // (cdna_hip_programming.md "Pipelining across barriers"), which would drain
  // the next chunk's table loads at the first MFMA of every chunk.
  constexpr int HPT = HCH / (256 * 16);  // 16-B pieces per thread per chunk
  half8 hr[HPT];
  auto load_h = [&](int c) {
    const uint8_t* src = reinterpret_cast<const uint8_t*>(htiled) + (size_t)c * HCH;
#pragma unroll
    for (int i = 0; i < HPT; ++i) hr[i] = *reinterpret_cast<const half8*>(src + (i * 256 + tid) * 16);
  };
  auto store_h = [&](int c) {
#pragma unroll
    for (int i = 0; i < HPT; ++i) *reinterpret_cast<half8*>(smem + (c & 1) * HCH + (i * 256 + tid) * 16) = hr[i];
  };
  load_h(0);
  load_e(ec, 0);
  store_h(0);
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    // hidden c + 1 first (its wait after the MFMAs then leaves the table loads
    // in flight), the next chunk's table second
    if (c + 1 < nch) load_h(c + 1);
    load_e(en, c + 1 < nch ? (c + 1) * kLg2Chunk : c * kLg2Chunk);  // the last chunk re-loads itself
    // keep the loads here: left to itself the scheduler sinks them below the
    // MFMAs (fewer live registers), and every chunk then waits a full latency
    __builtin_amdgcn_sched_barrier(0);
    const uint8_t* hb = smem + (c & 1) * HCH;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        // B: clip 16 nt + l16, dims 32 ks + 8 lq .. + 7 = fragment (ks, kk = lq >> 1),
        // lane' = clip + 32 (lq & 1)
        const int off = ((ks * 2 + (lq >> 1)) * NS) * 1024 + (16 * nt + l16 + 32 * (lq & 1)) * 16;
        const half8 bh = *reinterpret_cast<const half8*>(hb + off);
        half8 bl;
        if constexpr (NS == 2) bl = *reinterpret_cast<const half8*>(hb + off + 1024);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ec[mt][ks][0], bh, acc[mt][nt], 0, 0, 0);
          if constexpr (NS == 2) {
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ec[mt][ks][1], bh, acc[mt][nt], 0, 0, 0);
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ec[mt][ks][0], bl, acc[mt][nt], 0, 0, 0);
          }
        }
      }
    }
    // buffer (c + 1) & 1 was last read in chunk c - 1, before the previous barrier
    if (c + 1 < nch) store_h(c + 1);
    __syncthreads();  // no LDS DMA in flight: a bare s_barrier, the table loads survive it
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int p = 0; p < NS; ++p) ec[mt][ks][p] = en[mt][ks][p];
  }
  // acc[mt][nt]: lane holds clip 16 nt + l16, vocab v0 + 16 mt + 4 lq + j
  const int suppress = state->step + 1 < min_tokens;
  bool bad = false;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int vl = 16 * mt + 4 * lq + j;
        const int n = v0 + vl;
        float v = acc[mt][nt][j] * kLgInv;
        bad |= n < V && 16 * nt + l16 < B && !__builtin_isfinite(v);
        if (n >= V || (suppress && n == kEOT)) v = -INFINITY;
        lg[(16 * nt + l16) * kLgPickLd + wave * 32 + vl] = v;
      }
  // an MFMA operand out of the f16-pair range upstream turns every logit of
  // the clip into inf / NaN: flag it (plain vector store, every writer stores 1)
  if (bad && range_flag) *range_flag = 1;
  if (trace_out) {  // diagnostics only: uniform branch
    __syncthreads();
    const int slot = state->step + 1;
    if (slot < trace_s1)
      for (int e = tid; e < B * trace_k; e += 256) {
        const int b = e / trace_k;
        const size_t o = ((size_t)b * trace_s1 + slot) * trace_k + (e - b * trace_k);
        const int id = trace_ids[o] - (int)blockIdx.x * 128;
        if (id >= 0 && id < 128) trace_out[o] = lg[b * kLgPickLd + id];
      }
  }
  pick_from_lds(lg, B, V, pval, pidx, counter, out_tok, ticket);
}

int logits_argmax_groups(int V) { return (V + 127) / 128; }

// f32 rows -> fragment-tiled f16 planes, chunk-major: fragment
// f = (chunk * groups + g) * KS + ks holds rows 16 g .. + 15, dims
// 128 chunk + 32 ks + 8 (lane >> 4) .. + 7; thread = (fragment, lane): 8 values
template <int NS>
__global__ __launch_bounds__(256) void emb_tiled_kernel(const float* __restrict__ x, int V, int D, int64_t nfrag,
                                                        _Float16* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nfrag * 64) return;
  const int lane = (int)(i & 63);
  constexpr int KS = kLg2Chunk / 32;
  const int64_t f = i >> 6;
  const int64_t groups = emb_groups16(V);
  const int64_t cg = f / KS;  // chunk * groups + g
  const int64_t chunk = cg / groups, g = cg - chunk * groups;
  const int s = (int)(chunk * KS + (f - cg * KS));
  const int64_t v = g * 16 + (lane & 15);
  const int k = s * 32 + 8 * (lane >> 4);
  half8 hi, lo;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    _Float16 a = (_Float16)0.0f, b = (_Float16)0.0f;
    if (v < V) split_f16(x[v * D + k + j] * kEmbScale, a, b);
    hi[j] = a;
    lo[j] = b;
  }
  *reinterpret_cast<half8*>(out + (f * NS + 0) * 512 + lane * 8) = hi;
  if constexpr (NS == 2) *reinterpret_cast<half8*>(out + (f * NS + 1) * 512 + lane * 8) = lo;
}

bool emb_tiled_supported(int D) { return D % kLg2Chunk == 0; }
int64_t emb_tiled_rows(int V) { return (int64_t)logits_argmax_groups(V) * 128; }

hipError_t launch_emb_tiled(const float* emb, int V, int D, int ns, _Float16* out, hipStream_t st) {
  if (!emb_tiled_supported(D) || (ns != 1 && ns != 2)) return hipErrorInvalidValue;
  const int64_t nfrag = emb_tiled_rows(V) / 16 * (D / 32);
  const dim3 g((unsigned)((nfrag * 64 + 255) / 256));
  if (ns == 2)
    hipLaunchKernelGGL(emb_tiled_kernel<2>, g, dim3(256), 0, st, emb, V, D, nfrag, out);
  else
    hipLaunchKernelGGL(emb_tiled_kernel<1>, g, dim3(256), 0, st, emb, V, D, nfrag, out);
  return hipGetLastError();
}

hipError_t launch_logits_argmax(const _Float16* htiled, int B, int D, const _Float16* emb2, int ns, int V,
                                int min_tokens, const DecodeState* state, float* pval, int* pidx, int* counter,
                                int* out_tok, const int* trace_ids, float* trace_out, int trace_s1, int trace_k,
                                int* range_flag, hipStream_t st) {
  if (B < 1 || B > 32 || !emb_tiled_supported(D) || !state || !emb2 || !htiled) return hipErrorInvalidValue;
  const dim3 grid(logits_argmax_groups(V));
  if (ns == 2)
    hipLaunchKernelGGL(logits_argmax_f16_k32_kernel<2>, grid, dim3(256), 0, st, htiled, B, D, emb2, V, min_tokens,
                       state, pval, pidx, counter, out_tok, trace_ids, trace_out, trace_s1, trace_k, range_flag);
  else
    hipLaunchKernelGGL(logits_argmax_f16_k32_kernel<1>, grid, dim3(256), 0, st, htiled, B, D, emb2, V, min_tokens,
                       state, pval, pidx, counter, out_tok, trace_ids, trace_out, trace_s1, trace_k, range_flag);
  return hipGetLastError();
}

// ------------------------------------------------------------ bookkeep --
__global__ void bookkeep_kernel(const int* __restrict__ next, int* __restrict__ tokens, int* __restrict__ ntok,
                                int* __restrict__ done, int B, int max_tokens, int eot_stop, DecodeState* state) {
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    if (!done[b]) {
      const int tk = next[b];
      if (eot_stop && tk == kEOT) {
        done[b] = 1;
        atomicAdd(&state->n_done, 1);
      } else if (ntok[b] < max_tokens) {
        tokens[(size_t)b * max_tokens + ntok[b]] = tk;
        ntok[b] += 1;
      }
    }
  }
  if (threadIdx.x == 0) {
    state->position += 1;
    state->kv_len += 1;
    state->step += 1;
  }
}

hipError_t launch_bookkeep(const int* next_tok, int* tokens, int* n_tokens, int* done, int B, int max_tokens,
                           int eot_stop, DecodeState* state, hipStream_t st) {
  hipLaunchKernelGGL(bookkeep_kernel, dim3(1), dim3(256), 0, st, next_tok, tokens, n_tokens, done, B, max_tokens,
                     eot_stop, state);
  return hipGetLastError();
}

}  // namespace wa
