// wq4_skinny.hip -- the decode-step Q4 GEMM (M <= 32 rows): 16-column
// workgroups on v_mfma_f32_16x16x32_f16 with one Q4 block per MFMA.
//
// Replaces, for the greedy decode step, the WGSL shader's per-output loop
// (src/gguf/shader.wgsl:72-89): out[m][n] = sum_blk d[n][blk] * sum_i
// (q[n][k]-8) * x[m][k].  The Q4 block structure is kept in the arithmetic
// ("block-scaled"): per (row, column, block)
//     t = MFMA(x_hi, q - 8) + MFMA(x_lo, q - 8)       (q - 8 exact in f16,
//                                                     x = hi + lo, products
//                                                     exact, f32 accumulate)
//     acc = fma(t, d, acc)                            (d: the GGUF f16 scale)
// -- two MFMAs per block where the B = (q-8) d hi/lo form needs three, and
// no weight-side rounding at all.  Per row the order is fixed by K only
// (waves take fixed block ranges, summed in wave order), so a clip's result
// does not depend on how many rows share the launch.
//
// Why 16 columns: a K = 1280 decode GEMM at 32 columns per workgroup runs on
// 40 of 256 CUs and its dependent MFMA chain alone took 2.4 us of a 7.2 us
// kernel (WQ4_DIAG = 1 timing build); 16 columns double the CUs and
// the 16x16x32 shape does not pad 16 rows to 32.
//
// Weight layout (built once at upload, beside the prefill kernel's):
//   q16[nt16][u][lane][4 x u32]   nt16 = 16 output columns, u = 4 Q4 blocks
//     lane l: n = 16 nt16 + (l & 15), g = l >> 4: u32 i = block 4u + i,
//     elements 8g .. 8g + 7, packed as wq4_device.hpp deq8() reads them
//   d16[nt16][u][16 n][4 blocks]  f16 scales (the raw GGUF d)
// F16 weights (config 5): f16s[nt16][blk][lane][8 halves] = w[n][32 blk +
// 8 g + j] * 2^8 (exact; keeps small weights out of the f16 subnormals the
// MFMA flushes), undone with the activation scale.
#include <hip/hip_runtime.h>

#include <cstring>

#include "wq4_device.hpp"
#include "wq4_kernels.hpp"
#include "wq4_lnmath.hpp"

namespace wq4 {

// ------------------------------------------------------------------ host --
static inline uint32_t skinny_pack(const uint8_t* bytes, int hi_nibbles) {
  uint32_t w = 0;  // element j = 2i at nibble i, j = 2i + 1 at nibble 4 + i (deq8 order)
  for (int i = 0; i < 4; ++i) {
    const uint32_t a = hi_nibbles ? (bytes[2 * i] >> 4) : (bytes[2 * i] & 0x0f);
    const uint32_t b = hi_nibbles ? (bytes[2 * i + 1] >> 4) : (bytes[2 * i + 1] & 0x0f);
    w |= (a << (4 * i)) | (b << (16 + 4 * i));
  }
  return w;
}

void repack_q4_skinny(const uint8_t* raw, const Q4Geom& g, uint32_t* q16, uint16_t* d16) {
  const int64_t nt16 = g.np / 16, ku = skinny_units(g);
  std::memset(q16, 0, skinny_q_bytes(g));
  std::memset(d16, 0, skinny_d_bytes(g));
  for (int64_t t = 0; t < nt16; ++t)
    for (int64_t u = 0; u < ku; ++u)
      for (int l = 0; l < 64; ++l) {
        const int64_t n = 16 * t + (l & 15);
        const int gq = l >> 4;
        for (int i = 0; i < 4; ++i) {
          const int64_t b = 4 * u + i;
          if (n >= g.n || b >= g.kb) continue;
          const uint8_t* blk = raw + (n * g.kb + b) * kBlockBytes;
          q16[((t * ku + u) * 64 + l) * 4 + i] = skinny_pack(blk + 2 + 8 * (gq & 1), gq >> 1);
          if (gq == 0) d16[((t * ku + u) * 16 + (l & 15)) * 4 + i] = (uint16_t)(blk[0] | (blk[1] << 8));
        }
      }
}

void repack_f16_skinny(const uint16_t* w, const Q4Geom& g, uint16_t* f16s) {
  const int64_t nt16 = g.np / 16;
  std::memset(f16s, 0, skinny_f16_bytes(g));
  for (int64_t t = 0; t < nt16; ++t)
    for (int64_t b = 0; b < g.kb; ++b)
      for (int l = 0; l < 64; ++l) {
        const int64_t n = 16 * t + (l & 15);
        if (n >= g.n) continue;
        for (int j = 0; j < 8; ++j) {
          const int64_t k = 32 * b + 8 * (l >> 4) + j;
          const _Float16 v = __builtin_bit_cast(_Float16, w[n * g.k + k]) * (_Float16)256.0f;  // exact
          f16s[((t * g.kb + b) * 64 + l) * 8 + j] = __builtin_bit_cast(uint16_t, v);
        }
      }
}

// ---------------------------------------------------------------- device --
namespace {

// WQ4_STAMP (timing diagnostics only: make stamp, scripts/skinny_stamps.py;
// 0 in the product): per launch and workgroup, s_memrealtime at the start,
// after the first unit's loads landed, after the MFMA loop, after the
// reduction barrier and at the end, plus s_memtime cycles start -> end.
#ifndef WQ4_STAMP
#define WQ4_STAMP 0
#endif
constexpr int kStampLaunches = 512, kStampWgs = 512, kStampSlots = 8;
#if WQ4_STAMP
__device__ unsigned long long g_sk_stamps[kStampLaunches * kStampWgs * kStampSlots];
#endif
__device__ __forceinline__ unsigned long long stamp_rt() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
__device__ __forceinline__ unsigned long long stamp_cyc() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

constexpr int kSkW = 8;        // waves per workgroup (they split the K blocks)
constexpr int kSkLnPer = 5;    // LayerNorm-fold tile statistics per thread: 16 x 5 = 80 >= D / 16
constexpr int kOobS = 0x7fffff00;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, bytes, 0x00020000);
}
__device__ __forceinline__ floatx4 mfma16(const half8& a, const half8& b, const floatx4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

constexpr int kSkBpw = 5;  // Q4 blocks per wave at most (the launcher splits K over workgroups to fit)
constexpr int kSkOut = 1024;  // outputs per workgroup at most: 16 rows x 64 columns (split-K slab stride)

// One Q4 block of a wave's operands: the weights of its NT 16-column
// subtiles and the A fragments of its MT 16-row tiles.
template <int NT, int MT, int NS, int WK>
struct SkBlock {
  uint32_t w[NT][WK == kWeightsF16 ? 4 : 1];  // Q4: 8 nibbles; f16: 8 halves
  float d[NT];                                // Q4 block scale
  half8 a[MT][NS];
};

template <int NT, int MT, int NS, int WK>
__device__ __forceinline__ void sk_load(SkBlock<NT, MT, NS, WK>& B, int b, int lane, int ku, int kb,
                                        __amdgpu_buffer_rsrc_t rw, __amdgpu_buffer_rsrc_t rd,
                                        __amdgpu_buffer_rsrc_t ra, int m, int r0) {
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    if constexpr (WK == kWeightsF16) {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rw, ((t * kb + b) * 64 + lane) * 16, 0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) B.w[t][j] = v[j];
      B.d[t] = 1.0f;
    } else {
      B.w[t][0] = __builtin_amdgcn_raw_buffer_load_b32(rw, (((t * ku + (b >> 2)) * 64 + lane) * 4 + (b & 3)) * 4, 0, 0);
      const uint16_t db = __builtin_amdgcn_raw_buffer_load_b16(rd, (((t * ku + (b >> 2)) * 16 + (lane & 15)) * 4 + (b & 3)) * 2, 0, 0);
      B.d[t] = (float)__builtin_bit_cast(_Float16, db);
    }
  }
  // (weights and scales with the default cache policy: non-temporal loads
  // measured 3 % slower over the decode step, r02 chain trace)
  // A-tiled (32x32x16 fragment) layout read as 16x16x32 fragments: lane
  // (r, g) = row 16 mt + r, k = 32 b + 8 g .. + 7 -> fragment (b, kk = g >> 1),
  // lane' = row + 32 (g & 1).  Rows >= m are not read (zeros).
  const int r = lane & 15, g = lane >> 4;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int row = r0 + 16 * mt + r;
      const int off = ((((b * 2 + (g >> 1)) * NS + s) * 64) + row + 32 * (g & 1)) * 16;
      B.a[mt][s] = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(ra, row < m ? off : kOobS, 0, 0));
    }
}

template <int NT, int MT, int NS, int WK>
__device__ __forceinline__ void sk_compute(const SkBlock<NT, MT, NS, WK>& B, floatx4 (&acc)[NT][MT]) {
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    if constexpr (WK == kWeightsF16) {
      const half8 w = __builtin_bit_cast(half8, u32x4{B.w[t][0], B.w[t][1], B.w[t][2], B.w[t][3]});
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        acc[t][mt] = mfma16(B.a[mt][0], w, acc[t][mt]);
        if constexpr (NS == 2) acc[t][mt] = mfma16(B.a[mt][1], w, acc[t][mt]);
      }
    } else {
      const half8 q = deq8(B.w[t][0]);  // exact q - 8
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        floatx4 tmp = mfma16(B.a[mt][0], q, floatx4{0.f, 0.f, 0.f, 0.f});
        if constexpr (NS == 2) tmp = mfma16(B.a[mt][1], q, tmp);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[t][mt][j] = fmaf(tmp[j], B.d[t], acc[t][mt][j]);
      }
    }
  }
}

// grid = (np / (16 NT)) x mtl x ks workgroups (n-tile major, then the
// 16-row tile, then the K slice), 512 threads.  The
// workgroup's K slice (kb / ks blocks) is split over the 8 waves, <= 5
// blocks each, every load of a wave in flight at once.  With ks > 1 the
// slices' partial sums meet through write-through (sc1) slabs and an
// arrival counter; the last arriver adds them in slice order
// (cdna_hip_programming.md Guideline 16, R1) and runs the epilogue.
template <int NS, int EPI, int NT, int WK>
__global__ __launch_bounds__(64 * kSkW) void skinny_gemm_kernel(const uint32_t* __restrict__ wq,
                                                                const uint16_t* __restrict__ wd,
                                                                const _Float16* __restrict__ at, int K, int ku,
                                                                int kbp, int ks, int mtl, float binv,
                                                                float* __restrict__ part, int* __restrict__ counters,
                                                                EpiArgs e, int stamp_id) {
  constexpr int MT = 1, ROWS = 16, COLS = 16 * NT, OUT = ROWS * COLS;
  __shared__ __attribute__((aligned(16))) float red[kSkW * NT * MT * 256];
  __shared__ __attribute__((aligned(16))) float stage[ROWS * (COLS + 1)];
  __shared__ float lnf_mu[ROWS], lnf_den[ROWS];
  __shared__ int last;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // workgroup = (16-row tile mi of mtl, 16 NT columns nt, K slice): rows are
  // split over workgroups so that each streams half the A operand when there
  // are 32 rows (the load of A from L2 is this kernel's longest phase)
  const int tt = blockIdx.x / ks, slice = blockIdx.x - tt * ks;
  const int nt = tt / mtl, mi = tt - nt * mtl, r0 = 16 * mi;
  const int kb = K / 32, nbk = kb / ks;
  const int bw0 = slice * nbk + (wave * nbk) / kSkW, bw1 = slice * nbk + ((wave + 1) * nbk) / kSkW;
  unsigned long long st_[kStampSlots] = {};
  if constexpr (WQ4_STAMP) {
    st_[0] = stamp_rt();
    st_[5] = stamp_cyc();
  }

  // epilogue operands of this thread's outputs (row o / COLS, column o %
  // COLS, o = tid + 512 j), loaded up front (never written by this launch
  // before its own epilogue)
  // All of them branch-free buffer loads (an absent operand is a zero-size
  // resource, an element out of range an out-of-range offset: both read 0):
  // a load under an exec branch makes the compiler drain vmcnt at the join,
  // a whole memory round trip before the weight stream is issued (the
  // 8-wave decode kernel's finding, tools/warm_cold.py; here the stamped
  // operand phase fell from 3.3-4.0 us to ~2.3 at one clip).
  constexpr int OPT = (OUT + 511) / 512;
  float pre_bias[OPT], pre_res[OPT], pre_wg[OPT], pre_g[OPT];
  {
    const uint32_t nb = (uint32_t)e.n * 4;
    const __amdgpu_buffer_rsrc_t rbias = rsrc(e.bias, e.bias ? nb : 0);
    const __amdgpu_buffer_rsrc_t rwg = rsrc(e.lnf_wg, e.lnf_stats_in ? nb : 0);
    const __amdgpu_buffer_rsrc_t rg = rsrc(e.lnf_g, e.lnf_at ? nb : 0);
    const __amdgpu_buffer_rsrc_t rres = rsrc(e.residual, e.residual ? (uint32_t)e.m * (uint32_t)e.ldo * 4u : 0);
#pragma unroll
    for (int j = 0; j < OPT; ++j) {
      const int o = tid + 512 * j, orow = r0 + o / COLS, n = nt * COLS + o % COLS;
      const bool ok = o < OUT && orow < e.m && n < e.n;
      const int coff = ok ? n * 4 : kOobS;
      pre_bias[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rbias, coff, 0, 0));
      pre_wg[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rwg, coff, 0, 0));
      pre_g[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rg, coff, 0, 0));
      pre_res[j] = __builtin_bit_cast(
          float, __builtin_amdgcn_raw_buffer_load_b32(rres, ok ? (orow * e.ldo + n) * 4 : kOobS, 0, 0));
    }
  }
  const float ainv = (e.act_inv ? *e.act_inv : kActScaleInv) * binv;
  // LayerNorm fold, consumer: thread (row tid / 16, part tid % 16) loads the
  // row's 16-column tile statistics j = part, part + 16, ... first
  floatx2 lnf_st[kSkLnPer];
  const int lrow = r0 + (tid >> 4), lpart = tid & 15;  // threads tid < 256: this tile's 16 rows
  {
    const __amdgpu_buffer_rsrc_t rst =
        rsrc(e.lnf_stats_in, e.lnf_stats_in ? (uint32_t)e.m * (uint32_t)e.lnf_tiles * 8u : 0);
#pragma unroll
    for (int v = 0; v < kSkLnPer; ++v) {
      const int j = lpart + 16 * v;
      lnf_st[v] = __builtin_bit_cast(
          floatx2, __builtin_amdgcn_raw_buffer_load_b64(
                       rst, (tid < 256 && lrow < e.m && j < e.lnf_tiles) ? (lrow * e.lnf_tiles + j) * 8 : kOobS, 0, 0));
    }
  }
  // keep every epilogue-operand / statistics load above the weight stream
  __builtin_amdgcn_sched_barrier(0);

  const int nt16 = nt * NT;
  const __amdgpu_buffer_rsrc_t rw =
      WK == kWeightsF16 ? rsrc(wq + (size_t)nt16 * kb * 256, (uint32_t)(NT * kb) * 1024u)
                        : rsrc(wq + (size_t)nt16 * ku * 256, (uint32_t)(NT * ku) * 1024u);
  const __amdgpu_buffer_rsrc_t rd = rsrc(wd + (size_t)nt16 * ku * 64, (uint32_t)(NT * ku) * 128u);
  const __amdgpu_buffer_rsrc_t ra = rsrc(at, (uint32_t)kbp * 2u * NS * 1024u);
  floatx4 acc[NT][MT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[t][mt] = floatx4{0.f, 0.f, 0.f, 0.f};
  SkBlock<NT, MT, NS, WK> Bk[kSkBpw];
#pragma unroll
  for (int i = 0; i < kSkBpw; ++i)
    if (bw0 + i < bw1) sk_load<NT, MT, NS, WK>(Bk[i], bw0 + i, lane, ku, kb, rw, rd, ra, e.m, r0);
  if constexpr (WQ4_STAMP) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st_[1] = stamp_rt();
  }
#pragma unroll
  for (int i = 0; i < kSkBpw; ++i)
    if (bw0 + i < bw1) sk_compute<NT, MT, NS, WK>(Bk[i], acc);
  if constexpr (WQ4_STAMP) st_[2] = stamp_rt();

  // LayerNorm fold, consumer: the row statistics from its 16-column tile
  // statistics (lnf_merge_tiles, wq4_lnmath.hpp)
  if (e.lnf_stats_in) {
    float m_a, den_a;
    lnf_merge_tiles<kSkLnPer>(lnf_st, lpart, e.lnf_tiles, m_a, den_a);
    if (lpart == 0 && tid < 256) {
      lnf_mu[lrow - r0] = m_a;
      lnf_den[lrow - r0] = den_a;
    }
  }

  // fixed-order reduction over the waves: red[w][t][mt][lane][i]
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
      *reinterpret_cast<floatx4*>(&red[(((wave * NT + t) * MT + mt) * 64 + lane) * 4]) = acc[t][mt];
  __syncthreads();
  if constexpr (WQ4_STAMP) st_[3] = stamp_rt();
  float sum[OPT];
#pragma unroll
  for (int j = 0; j < OPT; ++j) {
    // output (row, col) sits in subtile col / 16, m-tile row / 16, lane
    // col % 16 + 16 ((row % 16) / 4), element row % 4
    const int o = tid + 512 * j, orow = o / COLS, ocol = o % COLS;
    const int t = ocol >> 4, mt = orow >> 4, rr = orow & 15;
    const int idx = ((t * MT + mt) * 64 + (ocol & 15) + 16 * (rr >> 2)) * 4 + (rr & 3);
    float v = 0.0f;
    if (o < OUT) {
      v = red[idx];
#pragma unroll
      for (int w = 1; w < kSkW; ++w) v = v + red[w * NT * MT * 256 + idx];
    }
    sum[j] = v;
  }
  if (ks > 1) {
    // this slice's partials, write-through; one ticket per workgroup
    const __amdgpu_buffer_rsrc_t rp = rsrc(part + (size_t)tt * ks * kSkOut, (uint32_t)ks * kSkOut * 4u);
#pragma unroll
    for (int j = 0; j < OPT; ++j) {
      const int o = tid + 512 * j;
      if (o < OUT) __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, sum[j]), rp, (slice * kSkOut + o) * 4, 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every storing wave drained before the ticket
    typedef __attribute__((address_space(1))) int gint;
    gint* ctr = (gint*)(counters + tt);
    if (tid == 0) last = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ks - 1;
    __syncthreads();
    if (!last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler-only: the loads stay below the ticket
#pragma unroll
    for (int j = 0; j < OPT; ++j) {
      const int o = tid + 512 * j;
      float v = 0.0f;
      if (o < OUT) {
        for (int sl = 0; sl < ks; ++sl)  // slice order: the same bits whatever arrived last
          v = v + __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rp, (sl * kSkOut + o) * 4, 0, 16));
      }
      sum[j] = v;
    }
    if (tid == 0) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
  }

  const bool tiled_out = EPI == kEpiTiled || e.lnf_at != nullptr;
  float y[OPT];
#pragma unroll
  for (int j = 0; j < OPT; ++j) {
    const int o = tid + 512 * j, lr = o / COLS, orow = r0 + lr, ocol = o % COLS, n = nt * COLS + ocol;
    const bool ok = o < OUT && orow < e.m && n < e.n;
    float a = sum[j] * ainv;
    if (e.lnf_stats_in && o < OUT) a = lnf_apply(a, lnf_mu[lr], pre_wg[j], lnf_den[lr]);  // LayerNorm fold, consumer
    y[j] = ok ? epi_value_pre(a, pre_bias[j], pre_res[j], e) : 0.0f;
    if constexpr (EPI == kEpiF32) {
      if (ok) e.out[(size_t)orow * e.ldo + n] = y[j];
    }
    if (tiled_out && o < OUT) stage[lr * (COLS + 1) + ocol] = EPI == kEpiTiled ? y[j] : y[j] * pre_g[j];
    // LayerNorm fold, producer: (mean, M2) of each row's 16 values per
    // subtile -- 16 consecutive lanes (COLS is a multiple of 16)
    if (e.lnf_at != nullptr && o - (tid & 63) < OUT) {  // wave-uniform
      const float mean = sum16(y[j]) * (1.0f / 16.0f);
      const float dv = y[j] - mean;
      const float m2 = sum16(dv * dv);
      // padding subtiles (N % 64 == 32: n >= N) own no statistics slot
      if ((ocol & 15) == 0 && o < OUT && orow < e.m && n < e.n)
        *reinterpret_cast<floatx2*>(e.lnf_stats_out + ((size_t)orow * (e.n / 16) + nt * NT + (ocol >> 4)) * 2) =
            floatx2{mean, m2};
    }
  }
  // A-tiled outputs: each 16-column subtile is one k-half (kk) of one Q4
  // block of the next GEMM's operand: lane' (row, h) holds columns 8h..8h+7
  if (tiled_out) {
    __syncthreads();
    if (tid < 32 * NT) {  // (row of the tile, half h, subtile t)
      const int lr = tid & 15, h = (tid >> 4) & 1, t = tid >> 5, row = r0 + lr;
      _Float16* dst = EPI == kEpiTiled ? e.out_tiled : e.lnf_at;
      half8 hi, lo;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        _Float16 x0 = (_Float16)0.0f, x1 = (_Float16)0.0f;
        if (row < e.m) split_act(stage[lr * (COLS + 1) + 16 * t + 8 * h + j], x0, x1);
        hi[j] = x0;
        lo[j] = x1;
      }
      const size_t frag = (size_t)(nt * NT + t) * NS;  // m-tile 0 (rows < 32): (block, kk) = nt16 / 2, nt16 % 2
      half8* d8 = reinterpret_cast<half8*>(dst);
      d8[(frag + 0) * 64 + row + 32 * h] = hi;
      if constexpr (NS == 2) d8[(frag + 1) * 64 + row + 32 * h] = lo;
    }
  }
#if WQ4_STAMP
  if (tid == 0 && stamp_id >= 0 && stamp_id < kStampLaunches && blockIdx.x < kStampWgs) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st_[4] = stamp_rt();
    st_[6] = stamp_cyc();
    st_[7] = (unsigned long long)(bw1 - bw0);
    for (int i = 0; i < kStampSlots; ++i) g_sk_stamps[((size_t)stamp_id * kStampWgs + blockIdx.x) * kStampSlots + i] = st_[i];
  }
#endif
  (void)stamp_id;
  (void)st_;
}

}  // namespace

// K split over workgroups: the smallest of 1, 2, 4, 8 that divides the block
// count and leaves <= kSkBpw blocks per wave (a function of K only, so the
// per-row arithmetic never depends on M); 0 = unsupported.
static int skinny_ks(const Q4Geom& g) {
  for (int ks = 1; ks <= 8; ks *= 2)
    if (g.kb % ks == 0 && (g.kb / ks + kSkW - 1) / kSkW <= kSkBpw) return ks;
  return 0;
}

// 16-column subtiles per workgroup: the fewest (1, 2, 4) that keep the grid
// within one workgroup per CU.  Only the work split changes with it, never
// an output's arithmetic.
static int skinny_nt(const Q4Geom& g, int rows) {
  const int64_t per = (int64_t)skinny_ks(g) * ((rows + 15) / 16);
  for (int nt = 1; nt < 4; nt *= 2)
    if (g.np / (16 * nt) * per <= 256) return nt;
  return 4;
}

bool skinny_supported(const Q4Geom& g, int rows) {
  if (rows < 1 || rows > 32 || g.k % 128 != 0 || g.n % 16 != 0 || skinny_ks(g) == 0) return false;
  const int64_t tiles = g.np / (16 * skinny_nt(g, rows)) * ((rows + 15) / 16);
  return tiles * skinny_ks(g) * kSkOut <= kDecodeWsFloats && tiles <= kDecodeMaxTiles;
}

// Stamp bookkeeping (WQ4_STAMP builds): launch id -> (N, K, rows).
static int g_stamp_next = 0;
static int g_stamp_meta[kStampLaunches][3];

hipError_t launch_skinny_gemm(const Q4Geom& g, const uint32_t* wq, const uint16_t* wd, const _Float16* at, int rows,
                              const EpiArgs& e, int epi_mode, int ns, int wtype, const DecodeWs* ws, hipStream_t st) {
  if (!skinny_supported(g, rows) || !ws) return hipErrorInvalidValue;
  int stamp_id = -1;
  if (WQ4_STAMP && g_stamp_next < kStampLaunches) {
    stamp_id = g_stamp_next++;
    g_stamp_meta[stamp_id][0] = (int)g.n;
    g_stamp_meta[stamp_id][1] = (int)g.k;
    g_stamp_meta[stamp_id][2] = rows;
  }
  const int ku = (int)skinny_units(g), ks = skinny_ks(g), nt = skinny_nt(g, rows), mtl = (rows + 15) / 16;
  const int kbp = (int)(2 * g.nbp);
  const float binv = wtype == kWeightsF16 ? 1.0f / 256.0f : 1.0f;
  const dim3 grid((unsigned)(g.np / (16 * nt) * mtl * ks));
#define WQ4_SK(NS_, EPI_, NT_, WK_)                                                                   \
  hipLaunchKernelGGL((skinny_gemm_kernel<NS_, EPI_, NT_, WK_>), grid, dim3(64 * kSkW), 0, st, wq, wd, at, \
                     (int)g.k, ku, kbp, ks, mtl, binv, ws->part, ws->counters, e, stamp_id)
#define WQ4_SK_NT(NS_, EPI_, WK_) \
  if (nt == 4) { WQ4_SK(NS_, EPI_, 4, WK_); } else if (nt == 2) { WQ4_SK(NS_, EPI_, 2, WK_); } else { WQ4_SK(NS_, EPI_, 1, WK_); }
#define WQ4_SK_WK(NS_, EPI_) \
  if (wtype == kWeightsF16) { WQ4_SK_NT(NS_, EPI_, kWeightsF16); } else { WQ4_SK_NT(NS_, EPI_, kWeightsQ4); }
  if (ns == 2) {
    if (epi_mode == kEpiTiled) { WQ4_SK_WK(2, kEpiTiled); } else { WQ4_SK_WK(2, kEpiF32); }
  } else {
    if (epi_mode == kEpiTiled) { WQ4_SK_WK(1, kEpiTiled); } else { WQ4_SK_WK(1, kEpiF32); }
  }
#undef WQ4_SK_WK
#undef WQ4_SK_NT
#undef WQ4_SK
  return hipGetLastError();
}

}  // namespace wq4

// Timing diagnostics (WQ4_STAMP builds only; returns 0 launches otherwise):
// copies [launches][kStampWgs][8] stamps and [launches][3] (N, K, rows).
extern "C" int wq4_diag_skinny_stamps(unsigned long long* out, int* meta, int max_launches) {
#if WQ4_STAMP
  const int n = wq4::g_stamp_next < max_launches ? wq4::g_stamp_next : max_launches;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(wq4::g_sk_stamps),
                          (size_t)n * wq4::kStampWgs * wq4::kStampSlots * sizeof(unsigned long long)) != hipSuccess)
    return -1;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < 3; ++j) meta[i * 3 + j] = wq4::g_stamp_meta[i][j];
  return n;
#else
  (void)out;
  (void)meta;
  (void)max_launches;
  return 0;
#endif
}
