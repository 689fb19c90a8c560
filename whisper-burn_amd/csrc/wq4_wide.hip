// wq4_wide.hip -- the encoder-size Q4_0 GEMM on one 8-wave workgroup per CU.
//
// Same arithmetic as q4_gemm_prefill_kernel (wq4_q4gemm.hip), bit for bit:
// per Q4 block t = MFMA(x_hi, q - 8) + MFMA(x_lo, q - 8) over its two 16-k
// halves (f32 accumulation from zero), acc = fma(t, d', acc), blocks in K
// order, y = epi(acc * 2^-s_n * act_inv) -- the reference's
// shader.wgsl:72-89 contraction with exact products.  What differs is the
// pipeline around it:
//
//  * 256 x 256 output tile per workgroup, 8 waves as 2 (M) x 4 (N), each
//    wave 128 x 64 (4 x 2 tiles of 32 x 32): one workgroup per CU, two waves
//    per SIMD, so one wave's block-scale FMAs and dequantisation issue beside
//    its partner's MFMAs.
//  * EVERY operand is staged by LDS-DMA (buffer ..._lds loads through
//    per-row descriptors): the A fragments, the repacked nibbles and the
//    block scales.  No ordinary global load in the K loop, so hipcc never
//    drains vmcnt(0) there (cdna_hip_programming.md §5, "Projection GEMM at
//    M = 256" item 4b).
//  * The K loop runs in half steps of one Q4 block (32 k) through a ring of
//    four LDS slots; each wave waits with a counted vmcnt (never 0 in the
//    loop) for its own copies, one raw s_barrier publishes them, and the
//    copies of half step h + 3 are issued into the slot the barrier freed.
//    In the product schedule (WQ4_WIDE_CARRY) the barrier at half step h
//    publishes slot h + 1: the last two chains of h already read the next
//    half step's first A fragments and nibbles, and the scale FMAs of h's
//    last two tiles ride in h + 1's first chains -- no drain between half
//    steps ("Pipelining across barriers").
//  * Epilogue (wq4_tile_epi.hpp) without memory drains: column scales and
//    bias staged in LDS during the loop, buffer stores masked by offset.
//
// LDS: slots 0 / 2 hold A (8 m-tiles x 2 NS KiB) + nibbles (8 n-tiles x 1
// KiB, both blocks of the pair) + scales (8 n-tiles x 128 B, twice); slots
// 1 / 3 hold A only -- the odd half step's weights are read into registers
// with the even one's.  148 KiB at NS = 2.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "wq4_device.hpp"
#include "wq4_kernels.hpp"
#include "wq4_tile_epi.hpp"

namespace wq4 {

// WQ4_WIDE_DIAG (timing diagnostics only, `make widediag`; 0 in the
// product): 1 no block-scale FMAs (the MFMA chains accumulate straight into
// acc), 2 = 1 + no dequantisation (raw nibble words as the B operand).
#ifndef WQ4_WIDE_DIAG
#define WQ4_WIDE_DIAG 0
#endif
// WQ4_WIDE_STAMP (timing diagnostics only; 0 in the product): per
// workgroup, waves 0 and 4 record the s_memtime cycles spent in the K loop's
// vmcnt waits, barriers, LDS-DMA issue and compute, and the loop's total
// (wq4_diag_wide_stamps).
#ifndef WQ4_WIDE_STAMP
#define WQ4_WIDE_STAMP 0
#endif
[[maybe_unused]] constexpr int kWideStampWgs = 4096;
#if WQ4_WIDE_STAMP
__device__ unsigned long long g_wide_stamps[kWideStampWgs * 2 * 10];
#endif

// WQ4_WIDE_SCHED: the half step's instruction order (A/B builds): 0 the
// plain two-temporary loop left to the scheduler, 1 three rotating
// temporaries, the order pinned by sched_barrier, 2 the same order in asm
// statements (one MFMA + its scale FMAs each).
#ifndef WQ4_WIDE_SCHED
#define WQ4_WIDE_SCHED 2
#endif
// WQ4_WIDE_PRIO: waves 4-7 at s_setprio 1 for the whole kernel (A/B; off:
// -4 to +2 %, profiles/r06_wide_prio_andor.log);
// WQ4_WIDE_ANDOR (default on: +1-5 %, profiles/r06_wide_prio_andor.log): the
// nibble dequantisation with v_and_or_b32 (one VALU
// instruction per AND + OR pair; A/B).
#ifndef WQ4_WIDE_PRIO
#define WQ4_WIDE_PRIO 0
#endif
#ifndef WQ4_WIDE_ANDOR
#define WQ4_WIDE_ANDOR 1
#endif

// deq8 (wq4_device.hpp) with each (w & mask) | C as one v_and_or_b32: the
// same bits.
__device__ __forceinline__ half8 deq8_andor(uint32_t w, uint32_t mlo, uint32_t mhi, uint32_t c) {
  const uint32_t w8 = w >> 8;
  uint32_t p0, p1, p2, p3;
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(p0) : "v"(w), "s"(mlo), "v"(c));
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(p1) : "v"(w), "s"(mhi), "v"(c));
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(p2) : "v"(w8), "s"(mlo), "v"(c));
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(p3) : "v"(w8), "s"(mhi), "v"(c));
  const half2v off1 = {(_Float16)1032.0f, (_Float16)1032.0f};
  const half2v inv16 = {(_Float16)0.0625f, (_Float16)0.0625f};
  const half2v off16 = {(_Float16)72.0f, (_Float16)72.0f};
  const half2v h0 = __builtin_bit_cast(half2v, p0) - off1;
  const half2v h1 = __builtin_bit_cast(half2v, p1) * inv16 - off16;
  const half2v h2 = __builtin_bit_cast(half2v, p2) - off1;
  const half2v h3 = __builtin_bit_cast(half2v, p3) * inv16 - off16;
  half8 r;
  r[0] = h0[0]; r[1] = h0[1];
  r[2] = h1[0]; r[3] = h1[1];
  r[4] = h2[0]; r[5] = h2[1];
  r[6] = h3[0]; r[7] = h3[1];
  return r;
}

// WQ4_WIDE_SPREAD (with WQ4_WIDE_SCHED 2): the next half step's LDS-DMA
// copies issued one per MFMA chain (1) instead of all after the barrier (0).
#ifndef WQ4_WIDE_SPREAD
#define WQ4_WIDE_SPREAD 1
#endif
// WQ4_WIDE_CARRY (with the pinned, spread schedule at NS = 2): no drain at a
// half step's end -- the scale FMAs of its last two tiles ride behind the
// next half step's first two chains (the temporaries rotate by two per half
// step), and the next half step's first A fragments, nibbles and its
// dequantisation are done under the last two chains, so a half step opens
// straight into MFMAs.  The barrier at half step h then publishes slot h + 1.
#ifndef WQ4_WIDE_CARRY
#define WQ4_WIDE_CARRY 1
#endif

// One MFMA of a block chain, t = A B + (first ? 0 : t); nop: open with
// s_nop 1 (the B operand may have been written by the VALU just before).
__device__ __forceinline__ void grp_mfma(floatx16& t, const half8& a, const half8& b, bool first, bool nop) {
  if (first && nop)
    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=&v"(t) : "v"(a), "v"(b));
  else if (first)
    asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=&v"(t) : "v"(a), "v"(b));
  else
    asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(t) : "v"(a), "v"(b));
}
// The same MFMA followed by four scale FMAs c_i = fma(u_i, d, c_i) of an
// older tile (u: a temporary whose chain has completed).
__device__ __forceinline__ void grp_mfma_fma(floatx16& t, const half8& a, const half8& b, bool first, bool nop,
                                             float& c0, float& c1, float& c2, float& c3, float u0, float u1,
                                             float u2, float u3, float d) {
  if (first && nop)
    asm volatile(
        "s_nop 1\n\t"
        "v_mfma_f32_32x32x16_f16 %0, %5, %6, 0\n\t"
        "v_fma_f32 %1, %7, %11, %1\n\t"
        "v_fma_f32 %2, %8, %11, %2\n\t"
        "v_fma_f32 %3, %9, %11, %3\n\t"
        "v_fma_f32 %4, %10, %11, %4"
        : "=&v"(t), "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3)
        : "v"(a), "v"(b), "v"(u0), "v"(u1), "v"(u2), "v"(u3), "v"(d));
  else if (first)
    asm volatile(
        "v_mfma_f32_32x32x16_f16 %0, %5, %6, 0\n\t"
        "v_fma_f32 %1, %7, %11, %1\n\t"
        "v_fma_f32 %2, %8, %11, %2\n\t"
        "v_fma_f32 %3, %9, %11, %3\n\t"
        "v_fma_f32 %4, %10, %11, %4"
        : "=&v"(t), "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3)
        : "v"(a), "v"(b), "v"(u0), "v"(u1), "v"(u2), "v"(u3), "v"(d));
  else
    asm volatile(
        "v_mfma_f32_32x32x16_f16 %0, %5, %6, %0\n\t"
        "v_fma_f32 %1, %7, %11, %1\n\t"
        "v_fma_f32 %2, %8, %11, %2\n\t"
        "v_fma_f32 %3, %9, %11, %3\n\t"
        "v_fma_f32 %4, %10, %11, %4"
        : "+v"(t), "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3)
        : "v"(a), "v"(b), "v"(u0), "v"(u1), "v"(u2), "v"(u3), "v"(d));
}

template <int NS>
struct WideGeo {
  static constexpr int FR = 2 * NS;                // A fragments (1 KiB) per m-tile and Q4 block
  static constexpr int AH = 8 * FR * 1024;          // A bytes of one half step
  static constexpr int BH = 8 * 1024 + 8 * 256;     // nibbles of 8 n-tiles (one block pair) + 8 scale copies
  static constexpr int PAIR = 2 * AH + BH;          // slot 2p (A + B) then slot 2p + 1 (A)
  static constexpr int RING = 2 * PAIR;
  static constexpr int STAGE = 8 * 32 * kStageLd * 4;  // tiled epilogue stage (reuses the ring)
  static constexpr int MAIN = RING > STAGE ? RING : STAGE;
  // + the workgroup's 256 columns' colscale x act_inv and bias (tile_epilogue's `pre`)
  static constexpr int LDS = MAIN + 2 * 256 * 4;
  static constexpr int CNT0 = FR + 2, CNT1 = FR;    // LDS-DMA copies per wave: even / odd half step
};

// 4 B per lane: lane l's dword lands at lds_base + 4 l.  (The sub-dword
// forms also land one dword per lane, so a 2-byte copy is not packed.)
__device__ __forceinline__ void glds4(const void* gsrc, void* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc,
                                   (__attribute__((address_space(3))) void*)lds_base, 4, 0, 0);
}

// A raw buffer descriptor over `bytes` bytes at a wave-uniform base (the
// inputs readfirstlane'd so hipcc keeps it in SGPRs, guide T8 / T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wide_rsrc(const void* p, uint32_t bytes) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
// buffer LDS-DMA of `size` (4 / 16) bytes per lane: lane l's bytes land at
// lds_base + size l (counted in vmcnt like global_load_lds).
__device__ __forceinline__ void blds(__amdgpu_buffer_rsrc_t r, void* lds_base, int size, uint32_t voff,
                                     uint32_t soff) {
  if (size == 16)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_base, 16, voff, soff, 0, 0);
  else
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_base, 4, voff, soff, 0, 0);
}

// This lane's id, recomputed at every call (volatile: never CSE'd into a
// value hipcc keeps live across the K loop).
__device__ __forceinline__ uint32_t fresh_lane() {
  uint32_t l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// s_waitcnt vmcnt(N), the other counters untouched (gfx9 encoding).
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt(0x0F70 | (N & 15) | ((N >> 4) << 14));
}

__device__ __forceinline__ void ring_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's reads of the slot being recycled are done
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <int NS, int EPI>
__global__ __launch_bounds__(512, 1) void q4_gemm_wide_kernel(const uint8_t* __restrict__ nib,
                                                              const uint32_t* __restrict__ sc,
                                                              const float* __restrict__ colscale,
                                                              const _Float16* __restrict__ at, int mtiles, int nbp,
                                                              int ntiles, EpiArgs e) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
#if WQ4_WIDE_STAMP
  const unsigned long long st_entry = __builtin_amdgcn_s_memrealtime();
#endif
  using G = WideGeo<NS>;
  constexpr int TM = 4, TN = 2, FR = G::FR;
  constexpr int CHUNK = 4096 * NS;  // A bytes per (m-tile, block pair) in global memory

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  if (WQ4_WIDE_PRIO && wave >= 4) __builtin_amdgcn_s_setprio(1);  // the second-dispatched half of each SIMD pair
  // deq8_andor's constants: the masks in SGPRs, the OR constant in a VGPR
  // (gfx9 VOP3 takes no literal and one SGPR)
  const uint32_t kMaskLo = __builtin_amdgcn_readfirstlane(0x000F000Fu), kMaskHi = __builtin_amdgcn_readfirstlane(0x00F000F0u);
  uint32_t kOrC = 0x64006400u;
  asm volatile("" : "+v"(kOrC));
  const int r = lane & 31;
  const int ngroups = (ntiles + 7) / 8, mgroups = (mtiles + 7) / 8;
  const int wg = xcd_remap(blockIdx.x, ngroups * mgroups);
  const int mg = wg / ngroups, ng = wg % ngroups;
  const int nt0 = ng * 8 + wn * TN;
  const bool active = nt0 < ntiles;  // wave-uniform (ntiles is even)
  // The epilogue's per-column operands, staged in LDS while the K loop runs
  // (loaded under the first copies, written before the first barrier): the
  // epilogue starts without a memory round trip.  Thread t: column
  // 256 ng + (t & 255), colscale (waves 0-3) or bias (waves 4-7).
  float* pre = reinterpret_cast<float*>(smem + G::MAIN);
  auto pre_load = [&]() {
    const int col = ng * 256 + (tid & 255);
    const bool isb = wave >= 4;
    const uint32_t lim = isb ? (e.bias ? (uint32_t)e.n : 0u) : (uint32_t)ntiles * 32;
    const __amdgpu_buffer_rsrc_t rs = isb ? wide_rsrc(e.bias, e.bias ? (uint32_t)e.n * 4 : 0)
                                          : wide_rsrc(colscale, (uint32_t)ntiles * 128);
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (uint32_t)col < lim ? col * 4 : 0x80000000u, 0, 0));
  };
  auto pre_store = [&](float v) {
    const float ainv = e.act_inv ? *e.act_inv : kActScaleInv;  // A operand scale (exact power of two)
    pre[tid] = wave >= 4 ? v : v * ainv;
  };

  // Loader role: wave w copies m-tile 8 mg + w, the nibbles of n-tile
  // 8 ng + w and the scales of n-tiles 8 ng + 2 (w & 3) + {0, 1} (waves 4-7
  // copy those of 0-3 again, so every wave issues the same count); indices
  // are clamped to the last tile: the duplicate rows / columns are never
  // stored.
  // The copies are buffer LDS-DMA loads: a descriptor per operand row in
  // SGPRs, the half step's offset in soffset, one shared 32-bit per-lane
  // voffset -- flat global_load_lds would keep 64-bit VGPR addresses live
  // across the loop, which the carried schedule cannot afford.
  const uint32_t abytes = (uint32_t)nbp * CHUNK, nbytes = (uint32_t)nbp * 1024;
  const __amdgpu_buffer_rsrc_t arsrc =
      wide_rsrc(reinterpret_cast<const uint8_t*>(at) + (size_t)min(mg * 8 + wave, mtiles - 1) * abytes, abytes);
  const __amdgpu_buffer_rsrc_t nrsrc = wide_rsrc(nib + (size_t)min(ng * 8 + wave, ntiles - 1) * nbytes, nbytes);
  // scales: lanes 32-63 copy the second n-tile of the wave's pair (voffset < 4 GiB: N K / 16 bytes)
  const __amdgpu_buffer_rsrc_t srsrc = wide_rsrc(sc, (uint32_t)ntiles * nbp * 128);
  const uint32_t lane16 = lane * 16;
  // the scale copy's per-lane offset, rebuilt from a fresh lane id at each
  // use (held in a VGPR across the loop, it is one too many for the carried
  // schedule): lanes 32-63 copy the pair's second n-tile (clamped)
  const int snt0 = min(ng * 8 + 2 * (wave & 3), ntiles - 1), snt1 = min(ng * 8 + 2 * (wave & 3) + 1, ntiles - 1);
  const uint32_t sbase = (uint32_t)snt0 * nbp * 128, sdelta = (uint32_t)(snt1 - snt0) * nbp * 128;
  auto soff = [&]() {
    const uint32_t l = fresh_lane();
    return sbase + (l >> 5) * sdelta + ((l & 31) << 2);
  };

  // copy n (0 .. FR + 1) of half step h's CNT0 / CNT1 copies into its slot
  auto issue_part = [&](int h, int n) {
    const int bp = h >> 1, blk = h & 1;
    uint8_t* base = smem + (h >> 1 & 1) * G::PAIR + blk * (G::AH + G::BH);
    if (n < FR)
      blds(arsrc, base + wave * (FR * 1024) + n * 1024, 16, lane16, bp * CHUNK + (blk * FR + n) * 1024);
    else if (blk == 0 && n == FR)
      blds(nrsrc, base + G::AH + wave * 1024, 16, lane16, bp * 1024);
    else if (blk == 0 && n == FR + 1)
      blds(srsrc, base + G::AH + 8192 + wave * 256, 4, soff(), bp * 128);
  };
  auto issue = [&](int h) {
#pragma unroll
    for (int n = 0; n < FR + 2; ++n) issue_part(h, n);
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.0f;

  u32x4 braw[TN];   // this wave's nibbles of the block pair (both blocks)
  uint32_t bsc[TN]; // and its column's two f16 scales

  // one half step: Q4 block 2 bp + BLK out of the slot at `base`
  // pend >= 0: the half step whose LDS-DMA copies this one issues (into the
  // slot the barrier freed); the pinned schedule spreads them over its
  // first chains, the other forms issue them up front
  auto compute = [&](const uint8_t* base, auto blk_c, int pend) {
    constexpr int BLK = decltype(blk_c)::value;
    constexpr bool kSpread = WQ4_WIDE_SPREAD && WQ4_WIDE_SCHED == 2 && NS == 2 && !WQ4_WIDE_DIAG;
    if (!kSpread && pend >= 0) issue(pend);
    if constexpr (BLK == 0) {
#pragma unroll
      for (int nt = 0; nt < TN; ++nt) {
        braw[nt] = *reinterpret_cast<const u32x4*>(base + G::AH + (wn * TN + nt) * 1024 + lane * 16);
        bsc[nt] = *reinterpret_cast<const uint32_t*>(base + G::AH + 8192 + wn * 256 + nt * 128 + r * 4);
      }
    }
    half8 qf[TN][2];
    float dsc[TN];
#pragma unroll
    for (int nt = 0; nt < TN; ++nt) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        qf[nt][kk] = WQ4_WIDE_DIAG == 2 ? __builtin_bit_cast(half8, braw[nt])
                     : WQ4_WIDE_ANDOR ? deq8_andor(braw[nt][BLK * 2 + kk], kMaskLo, kMaskHi, kOrC)
                                      : deq8(braw[nt][BLK * 2 + kk]);
      dsc[nt] = (float)__builtin_bit_cast(_Float16, (uint16_t)(BLK ? (bsc[nt] >> 16) : (bsc[nt] & 0xffffu)));
    }
    auto chain = [&](const half8 (&ah)[2], const half8 (&al)[2], int nt) {
      floatx16 t = mfma32(ah[0], qf[nt][0], floatx16{});
      if constexpr (NS == 2) t = mfma32(al[0], qf[nt][0], t);
      t = mfma32(ah[1], qf[nt][1], t);
      if constexpr (NS == 2) t = mfma32(al[1], qf[nt][1], t);
      return t;
    };
#if WQ4_WIDE_DIAG
    floatx16 t0, t1;
#pragma unroll
    for (int mt = 0; mt < TM; ++mt) {
      const uint8_t* fa = base + (wm * TM + mt) * (FR * 1024) + lane * 16;
      half8 ahi[2], alo[2];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        ahi[kk] = *reinterpret_cast<const half8*>(fa + kk * NS * 1024);
        if constexpr (NS == 2) alo[kk] = *reinterpret_cast<const half8*>(fa + kk * NS * 1024 + 1024);
      }
      (void)t0;
      (void)t1;
#pragma unroll
      for (int nt = 0; nt < TN; ++nt) {
        acc[mt][nt] = mfma32(ahi[0], qf[nt][0], acc[mt][nt]);
        if constexpr (NS == 2) acc[mt][nt] = mfma32(alo[0], qf[nt][0], acc[mt][nt]);
        acc[mt][nt] = mfma32(ahi[1], qf[nt][1], acc[mt][nt]);
        if constexpr (NS == 2) acc[mt][nt] = mfma32(alo[1], qf[nt][1], acc[mt][nt]);
      }
    }
    asm volatile("" ::"v"(dsc[0]), "v"(dsc[1]));
#elif WQ4_WIDE_SCHED == 0
    // two temporaries in flight: tile (mt, 1)'s MFMA chain runs under the
    // scale FMAs of (mt, 0), and (mt + 1, 0)'s under those of (mt, 1)
    floatx16 t0, t1;
#pragma unroll
    for (int mt = 0; mt < TM; ++mt) {
      const uint8_t* fa = base + (wm * TM + mt) * (FR * 1024) + lane * 16;
      half8 ahi[2], alo[2];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        ahi[kk] = *reinterpret_cast<const half8*>(fa + kk * NS * 1024);
        if constexpr (NS == 2) alo[kk] = *reinterpret_cast<const half8*>(fa + kk * NS * 1024 + 1024);
      }
      t0 = chain(ahi, alo, 0);
      if (mt > 0) acc[mt - 1][1] = t1 * dsc[1] + acc[mt - 1][1];
      t1 = chain(ahi, alo, 1);
      acc[mt][0] = t0 * dsc[0] + acc[mt][0];
    }
    acc[TM - 1][1] = t1 * dsc[1] + acc[TM - 1][1];
#elif WQ4_WIDE_SCHED == 1
    // Tiles j = 0..7 (m-tile j / 2, n-tile j % 2) through three rotating
    // temporaries: between the MFMAs of tile j's chain sit the scale FMAs of
    // tile j - 2 (a chain two tiles old has completed: no FMA waits on an
    // MFMA) and, in the first chain of each m-tile, the reads of the next
    // m-tile's A fragments; sched_barrier pins that order (left to itself
    // the scheduler bunches the FMAs behind the MFMAs, and the two waves of
    // a SIMD then idle the matrix pipe together).  Same per-element
    // arithmetic in the same order: the tile kernel's bits.
    constexpr int NM = 2 * NS;        // MFMAs per chain
    constexpr int FPM = 16 / NM;      // scale FMAs (elements) per MFMA
    floatx16 tt[3];
    half8 a[2][2][NS];  // [m-tile parity][kk][hi, lo]
    auto afrag = [&](int mt, int kk, int q) {
      return *reinterpret_cast<const half8*>(base + (wm * TM + mt) * (FR * 1024) + (kk * NS + q) * 1024 + lane * 16);
    };
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int q = 0; q < NS; ++q) a[0][kk][q] = afrag(0, kk, q);
#pragma unroll
    for (int j = 0; j < 2 * TM; ++j) {
      const int mt = j >> 1, nt = j & 1, pb = mt & 1;
#pragma unroll
      for (int i = 0; i < NM; ++i) {
        const int kk = i / NS, q = i % NS;
        tt[j % 3] = mfma32(a[pb][kk][q], qf[nt][kk], i == 0 ? floatx16{} : tt[j % 3]);
        if (nt == 0 && mt + 1 < TM) a[pb ^ 1][kk][q] = afrag(mt + 1, kk, q);
        if (j >= 2) {
          const int p = j - 2;
#pragma unroll
          for (int e = i * FPM; e < (i + 1) * FPM; ++e)
            acc[p >> 1][p & 1][e] = __builtin_fmaf(tt[p % 3][e], dsc[p & 1], acc[p >> 1][p & 1][e]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int p = 2 * TM - 2; p < 2 * TM; ++p)
#pragma unroll
      for (int e = 0; e < 16; ++e)
        acc[p >> 1][p & 1][e] = __builtin_fmaf(tt[p % 3][e], dsc[p & 1], acc[p >> 1][p & 1][e]);
#else
    // WQ4_WIDE_SCHED == 2: the order of WQ4_WIDE_SCHED == 1, pinned by
    // writing each MFMA together with the scale FMAs that ride behind it as
    // one asm statement (grp_mfma_fma): asm statements keep their order, and
    // hipcc cannot pull the FMAs together behind the MFMAs.  Hazards inside
    // the statements (hipcc pads none, cdna_hip_programming.md §5.7): an FMA
    // reads a temporary whose chain ended >= 2 NS statements (>= 12 states)
    // earlier; the first MFMA on a freshly dequantised B operand opens with
    // s_nop 1; a chain's MFMAs accumulate in place (0 states).
    // (f16 operands, NS = 1: the plain loop)
    if constexpr (NS == 1) {
      floatx16 t0, t1;
#pragma unroll
      for (int mt = 0; mt < TM; ++mt) {
        const uint8_t* fa = base + (wm * TM + mt) * (FR * 1024) + lane * 16;
        half8 ahi[2], alo[2];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) ahi[kk] = *reinterpret_cast<const half8*>(fa + kk * NS * 1024);
        t0 = chain(ahi, alo, 0);
        if (mt > 0) acc[mt - 1][1] = t1 * dsc[1] + acc[mt - 1][1];
        t1 = chain(ahi, alo, 1);
        acc[mt][0] = t0 * dsc[0] + acc[mt][0];
      }
      acc[TM - 1][1] = t1 * dsc[1] + acc[TM - 1][1];
      return;
    }
    floatx16 tt[3];
    half8 a[2][2][2];  // [m-tile parity][kk][hi, lo]
    auto afrag = [&](int mt, int kk, int q) {
      return *reinterpret_cast<const half8*>(base + (wm * TM + mt) * (FR * 1024) + (kk * NS + q) * 1024 + lane * 16);
    };
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int q = 0; q < 2; ++q) a[0][kk][q] = afrag(0, kk, q);
#pragma unroll
    for (int j = 0; j < 2 * TM; ++j) {
      const int mt = j >> 1, nt = j & 1, pb = mt & 1;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int kk = i >> 1, q = i & 1;
        if (j >= 2) {
          const int p = j - 2;
          floatx16& c = acc[p >> 1][p & 1];
          const floatx16& t = tt[p % 3];
          float c0 = c[4 * i], c1 = c[4 * i + 1], c2 = c[4 * i + 2], c3 = c[4 * i + 3];
          grp_mfma_fma(tt[j % 3], a[pb][kk][q], qf[nt][kk], i == 0, false, c0, c1, c2, c3, t[4 * i], t[4 * i + 1],
                       t[4 * i + 2], t[4 * i + 3], dsc[p & 1]);
          c[4 * i] = c0;
          c[4 * i + 1] = c1;
          c[4 * i + 2] = c2;
          c[4 * i + 3] = c3;
        } else {
          grp_mfma(tt[j % 3], a[pb][kk][q], qf[nt][kk], i == 0, i == 0);
        }
        if (nt == 0 && mt + 1 < TM) a[pb ^ 1][kk][q] = afrag(mt + 1, kk, q);
        if (kSpread && i == 1 && j < FR + 2 && pend >= 0) issue_part(pend, j);  // one copy per chain
      }
    }
#pragma unroll
    for (int p = 2 * TM - 2; p < 2 * TM; ++p)
#pragma unroll
      for (int e = 0; e < 16; ++e)
        acc[p >> 1][p & 1][e] = __builtin_fmaf(tt[p % 3][e], dsc[p & 1], acc[p >> 1][p & 1][e]);
#endif
  };

  const int H = 2 * nbp;
#if WQ4_WIDE_STAMP
  unsigned long long st_acc[4] = {0, 0, 0, 0}, st_t = 0;
  const unsigned long long st_begin = __builtin_amdgcn_s_memtime();
  const unsigned long long st_rbegin = __builtin_amdgcn_s_memrealtime();
#define WIDE_STAMP(k)                                            \
  {                                                              \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    if (k >= 0) st_acc[k < 0 ? 0 : k] += now_ - st_t;            \
    st_t = now_;                                                 \
  }
#else
#define WIDE_STAMP(k)
#endif
  constexpr bool kCarry = WQ4_WIDE_CARRY && WQ4_WIDE_SCHED == 2 && WQ4_WIDE_SPREAD && NS == 2 && !WQ4_WIDE_DIAG;
  if constexpr (kCarry) {
    // WQ4_WIDE_CARRY.  Every wave computes, inactive ones (n-tiles past
    // ntiles, partial last n-group only) on the clamped duplicate columns
    // their epilogue never stores: no active / inactive branch in the loop,
    // whose joins cost hipcc's allocator spills.
    // State that lives across half steps -- the three
    // temporaries (the last two tiles' FMAs are still owed), the next half
    // step's dequantised nibbles, its first m-tile's A fragments and the
    // block scales of this and the previous half step.
    floatx16 tt[3];
    half8 a[2][2];  // [kk][hi, lo] of one m-tile, each fragment replaced by the next m-tile's after its last MFMA
    half8 qf[TN][2];
    float dcur[TN], dprev[TN];
#pragma unroll
    for (int x = 0; x < 3; ++x)
#pragma unroll
      for (int i = 0; i < 16; ++i) tt[x][i] = 0.0f;  // half step 0 "carries" fma(0, 0, +0) = +0 into acc[3][*]
    dprev[0] = dprev[1] = 0.0f;
    auto afrag = [&](const uint8_t* b, int mt, int kk, int q) {
      return *reinterpret_cast<const half8*>(b + (wm * TM + mt) * (FR * 1024) + (kk * NS + q) * 1024 + lane * 16);
    };
    // the nibble words of ONE block (read just before their dequantisation)
    // and the pair's scale word: 6 VGPRs fewer than holding the pair's
    uint32_t bw[TN][2], bs[TN];
    auto load_b = [&](const uint8_t* pb, int nt, int blk) {  // pb: the pair's even slot (still unrecycled)
      const uint32_t* w = reinterpret_cast<const uint32_t*>(pb + G::AH + (wn * TN + nt) * 1024 + lane * 16) + blk * 2;
      bw[nt][0] = w[0];
      bw[nt][1] = w[1];
      bs[nt] = *reinterpret_cast<const uint32_t*>(pb + G::AH + 8192 + wn * 256 + nt * 128 + ((fresh_lane() & 31) << 2));
    };
    auto deq = [&](int nt) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) qf[nt][kk] = deq8_andor(bw[nt][kk], kMaskLo, kMaskHi, kOrC);
    };
    auto scale = [&](int nt, int blk) {
      return (float)__builtin_bit_cast(_Float16, (uint16_t)(blk ? (bs[nt] >> 16) : (bs[nt] & 0xffffu)));
    };
    // One half step (block BLK of its pair) out of the slot at `base`, its
    // temporaries rotated by OFF; nbase: the next half step's slot (next:
    // there is one).  Tile j = (m-tile j / 2, n-tile j % 2) runs in
    // tt[(j + OFF) % 3]; chains 0 / 1 carry the FMAs of the previous half
    // step's tiles 6 / 7 (its OFF was OFF + 1 mod 3), chains j >= 2 those of
    // tile j - 2.  Hazards as in the SCHED 2 path; chain 0 opens with s_nop
    // 1 (its B operand was dequantised at the previous half step's end).
    // mid_sync: the first half step, which runs without a barrier at its top
    // (slot 0 was published by the prologue's), and so waits for and
    // publishes slot 1 only before the chains that read it.
    auto mid_sync = [&]() {
      if (nbp > 1) vm_wait<G::CNT0 + G::CNT1>();  // only the copies of half steps 2 and 3 may be outstanding
      else vm_wait<0>();
      ring_barrier();
    };
    auto step = [&](const uint8_t* base, const uint8_t* nbase, auto blk_c, auto off_c, auto ms_c, int pend,
                    bool next) __attribute__((always_inline)) {
      constexpr int BLK = decltype(blk_c)::value, OFF = decltype(off_c)::value;
      constexpr bool MS = decltype(ms_c)::value;
#pragma unroll
      for (int j = 0; j < 2 * TM; ++j) {
        const int mt = j >> 1, nt = j & 1;
        if (MS && j == 2 * TM - 2) mid_sync();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int kk = i >> 1, q = i & 1;
          const int p = j >= 2 ? j - 2 : 6 + j;
          floatx16& c = acc[p >> 1][p & 1];
          const floatx16& t = tt[j >= 2 ? (p + OFF) % 3 : (j + OFF + 1) % 3];
          const float d = j >= 2 ? dcur[p & 1] : dprev[j];
          float c0 = c[4 * i], c1 = c[4 * i + 1], c2 = c[4 * i + 2], c3 = c[4 * i + 3];
          grp_mfma_fma(tt[(j + OFF) % 3], a[kk][q], qf[nt][kk], i == 0, j == 0 && i == 0, c0, c1, c2, c3,
                       t[4 * i], t[4 * i + 1], t[4 * i + 2], t[4 * i + 3], d);
          c[4 * i] = c0;
          c[4 * i + 1] = c1;
          c[4 * i + 2] = c2;
          c[4 * i + 3] = c3;
          if (nt == 1) a[kk][q] = mt + 1 < TM ? afrag(base, mt + 1, kk, q) : afrag(nbase, 0, kk, q);
          // the next half step's nibbles: the next pair's even slot, or this one's
          if (j == 2 * TM - 2 && i >= 2) load_b(BLK ? nbase : base, i - 2, 1 - BLK);
          if (i == 1 && j < FR + 2 && pend >= 0) issue_part(pend, j);  // one copy per chain
        }
        // the next half step's nibbles, each n-tile once its last chain here is issued
        if (j >= 2 * TM - 2) deq(nt);
      }
      (void)next;  // the last half step prefetches from a valid slot too; its tiles 6 / 7 are finished after the loop
#pragma unroll
      for (int nt = 0; nt < TN; ++nt) {
        dprev[nt] = dcur[nt];
        dcur[nt] = scale(nt, 1 - BLK);
      }
    };
    // the last half step's tiles 6 / 7 (its OFF = 2 (H - 1) mod 3)
    auto finish = [&](auto off_c) {
      constexpr int OFF = decltype(off_c)::value;
      // the last chain's MFMA result is read by the VALU right behind it:
      // pad the MFMA-write -> VALU-read window (18 states for 16 passes)
      asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" : "+v"(tt[(6 + OFF) % 3]), "+v"(tt[(7 + OFF) % 3]));
#pragma unroll
      for (int p = 2 * TM - 2; p < 2 * TM; ++p)
#pragma unroll
        for (int e = 0; e < 16; ++e)
          acc[p >> 1][p & 1][e] = __builtin_fmaf(tt[(p + OFF) % 3][e], dprev[p & 1], acc[p >> 1][p & 1][e]);
    };
    // Ring protocol: the barrier at half step h publishes slot h + 1 (each
    // wave has waited for its own copies of h + 1, only those of h + 2 may
    // be outstanding) and frees slot h - 1 (read by half step h - 1 and by
    // h - 2's prefetch), into which h's chains issue the copies of h + 3.
    issue(0);
    const float pv = pre_load();  // lands with slot 0
    if (H > 1) issue(1);
    if (H > 2) issue(2);
    if (H > 2) vm_wait<G::CNT0 + G::CNT1>();
    else vm_wait<G::CNT1>();
    pre_store(pv);
    ring_barrier();
    {
#pragma unroll
      for (int nt = 0; nt < TN; ++nt) {
        load_b(smem, nt, 0);
        deq(nt);
        dcur[nt] = scale(nt, 0);
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int q = 0; q < 2; ++q) a[kk][q] = afrag(smem, 0, kk, q);
    }
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using NoMs = std::integral_constant<bool, false>;
    // more_c: true when the caller knows a block pair follows (the loop
    // body: no branch on it there)
    auto pair = [&](int bp, auto offe, auto first_c, auto more_c) __attribute__((always_inline)) {
      constexpr int OE = decltype(offe)::value, OO = (OE + 2) % 3;
      constexpr bool FIRST = decltype(first_c)::value;
      const bool more = decltype(more_c)::value || bp + 1 < nbp;
      const uint8_t* b0 = smem + (bp & 1) * G::PAIR;
      const uint8_t* b1 = b0 + G::AH + G::BH;
      const uint8_t* bn = smem + ((bp + 1) & 1) * G::PAIR;
      WIDE_STAMP(-1);
      if constexpr (!FIRST) {
        if (more) vm_wait<G::CNT0>();
        else vm_wait<0>();
        WIDE_STAMP(0);
        ring_barrier();
        WIDE_STAMP(1);
      }
      WIDE_STAMP(2);
      step(b0, b1, I0{}, std::integral_constant<int, OE>{}, first_c, more ? 2 * bp + 3 : -1, true);
      WIDE_STAMP(3);
      if (more) vm_wait<G::CNT1>();
      else vm_wait<0>();
      WIDE_STAMP(0);
      ring_barrier();
      WIDE_STAMP(1);
      WIDE_STAMP(2);
      step(b1, bn, I1{}, std::integral_constant<int, OO>{}, NoMs{}, more ? 2 * bp + 4 : -1, more);
      WIDE_STAMP(3);
    };
    // half step h runs with OFF = 2 h mod 3: even (2 bp) -> bp mod 3, odd ->
    // bp + 2 mod 3.  The first pair is peeled (no barrier at its top), then
    // three pairs per trip, so the rotation is straight code (a branch
    // between the rotations costs hipcc's allocator ~1000 spilled VGPRs),
    // then the last one to three pairs.
    using Yes = std::integral_constant<bool, true>;
    pair(0, I0{}, Yes{}, NoMs{});
    int bp = 1;
    for (; bp + 3 < nbp; bp += 3) {  // every pair here has a successor
      pair(bp, I1{}, NoMs{}, Yes{});
      pair(bp + 1, I2{}, NoMs{}, Yes{});
      pair(bp + 2, I0{}, NoMs{}, Yes{});
    }
    if (bp < nbp) pair(bp, I1{}, NoMs{}, NoMs{});
    if (bp + 1 < nbp) pair(bp + 1, I2{}, NoMs{}, NoMs{});
    if (bp + 2 < nbp) pair(bp + 2, I0{}, NoMs{}, NoMs{});
    {
      const int ol = (2 * (H - 1)) % 3;
      if (ol == 0) finish(std::integral_constant<int, 0>{});
      else if (ol == 1) finish(std::integral_constant<int, 1>{});
      else finish(std::integral_constant<int, 2>{});
    }
  } else {
  issue(0);
  if (H > 1) issue(1);
  if (H > 2) issue(2);
  for (int bp = 0; bp < nbp; ++bp) {
    const bool more = bp + 1 < nbp;
    const uint8_t* b0 = smem + (bp & 1) * G::PAIR;
    // even half step: block 2 bp (slot 2 (bp & 1))
    WIDE_STAMP(-1);
    if (more) vm_wait<G::CNT0 + G::CNT1>();
    else vm_wait<G::CNT1>();
    WIDE_STAMP(0);
    ring_barrier();
    WIDE_STAMP(1);
    WIDE_STAMP(2);
    if (active) compute(b0, std::integral_constant<int, 0>{}, more ? 2 * bp + 3 : -1);
    else if (more) issue(2 * bp + 3);
    WIDE_STAMP(3);
    // odd half step: block 2 bp + 1 (slot 2 (bp & 1) + 1)
    if (more) vm_wait<G::CNT0 + G::CNT1>();
    else vm_wait<0>();
    WIDE_STAMP(0);
    ring_barrier();
    WIDE_STAMP(1);
    WIDE_STAMP(2);
    if (active) compute(b0 + G::AH + G::BH, std::integral_constant<int, 1>{}, 2 * bp + 4 < H ? 2 * bp + 4 : -1);
    else if (2 * bp + 4 < H) issue(2 * bp + 4);
    WIDE_STAMP(3);
  }
  }
#undef WIDE_STAMP
  if constexpr (!kCarry) pre_store(pre_load());  // (the A/B path: after its loop)
  __syncthreads();  // the ring is drained and read: the epilogue stage may reuse it
#if WQ4_WIDE_STAMP
  if (lane == 0 && (wave == 0 || wave == 4) && blockIdx.x < kWideStampWgs) {
    unsigned long long* o = g_wide_stamps + ((size_t)blockIdx.x * 2 + (wave >> 2)) * 10;
    for (int k = 0; k < 4; ++k) o[k] = st_acc[k];
    o[4] = __builtin_amdgcn_s_memtime() - st_begin;
    o[5] = __builtin_amdgcn_s_memrealtime() - st_rbegin;  // 100 MHz ticks
    o[6] = st_entry;
    o[8] = __builtin_amdgcn_s_memrealtime();  // the K loop's end, absolute
  }
#endif

  tile_epilogue<NS, EPI, TM, TN>(acc, mg * 8 + wm * TM, nt0, active, mtiles, colscale,
                                 reinterpret_cast<float*>(smem) + wave * (32 * kStageLd), lane, e, pre + wn * TN * 32);
#if WQ4_WIDE_STAMP
  {
    const unsigned long long issued = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_waitcnt(0);  // the epilogue's stores completed
    if (lane == 0 && (wave == 0 || wave == 4) && blockIdx.x < kWideStampWgs) {
      g_wide_stamps[((size_t)blockIdx.x * 2 + (wave >> 2)) * 10 + 9] = issued;
      g_wide_stamps[((size_t)blockIdx.x * 2 + (wave >> 2)) * 10 + 7] = __builtin_amdgcn_s_memrealtime();
    }
  }
#endif
}

bool wide_gemm_supported(const Q4Geom& g, int rows, int ns, int wtype) {
  return wtype == kWeightsQ4 && (ns == 1 || ns == 2) && rows > 128 && g.kb >= 1 && g.ntiles % 2 == 0;
}

template <int NS>
static hipError_t launch_wide_t(const Q4Geom& g, const uint8_t* nib, const uint32_t* sc, const float* cs,
                                const _Float16* at, int rows, const EpiArgs& e, int epi_mode, hipStream_t st) {
  const int mtiles = (int)(round_up(rows < 1 ? 1 : rows, kMPad) / kMTile);
  const int ngroups = (int)((g.ntiles + 7) / 8);
  const int mgroups = (mtiles + 7) / 8;
  const dim3 grid((unsigned)(ngroups * mgroups));
  const size_t lds = WideGeo<NS>::LDS;
  if (epi_mode == kEpiTiled)
    hipLaunchKernelGGL((q4_gemm_wide_kernel<NS, kEpiTiled>), grid, dim3(512), lds, st, nib, sc, cs, at, mtiles,
                       (int)g.nbp, (int)g.ntiles, e);
  else if (epi_mode == kEpiHeadMajor)
    hipLaunchKernelGGL((q4_gemm_wide_kernel<NS, kEpiHeadMajor>), grid, dim3(512), lds, st, nib, sc, cs, at, mtiles,
                       (int)g.nbp, (int)g.ntiles, e);
  else
    hipLaunchKernelGGL((q4_gemm_wide_kernel<NS, kEpiF32>), grid, dim3(512), lds, st, nib, sc, cs, at, mtiles,
                       (int)g.nbp, (int)g.ntiles, e);
  return hipGetLastError();
}

hipError_t launch_wide_gemm(const Q4Geom& g, const uint8_t* nib, const uint32_t* sc, const float* cs,
                            const _Float16* at, int rows, const EpiArgs& e, int epi_mode, int ns, hipStream_t st) {
  if (ns == 2) return launch_wide_t<2>(g, nib, sc, cs, at, rows, e, epi_mode, st);
  return launch_wide_t<1>(g, nib, sc, cs, at, rows, e, epi_mode, st);
}

}  // namespace wq4

// Timing diagnostics (WQ4_WIDE_STAMP builds only; 0 workgroups otherwise):
// copies [wgs][2 waves][10] loop-phase cycle sums of the last wide launch
// (vmcnt, barrier, issue, compute, loop total; then the loop's s_memrealtime,
// the absolute s_memrealtime at kernel entry and after the epilogue's stores
// completed; the K loop's end; the epilogue's last store issued).
extern "C" int wq4_diag_wide_stamps(unsigned long long* out, int max_wgs) {
#if WQ4_WIDE_STAMP
  const int n = max_wgs < wq4::kWideStampWgs ? max_wgs : wq4::kWideStampWgs;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(wq4::g_wide_stamps), (size_t)n * 2 * 10 * sizeof(unsigned long long)) !=
      hipSuccess)
    return -1;
  return n;
#else
  (void)out;
  (void)max_wgs;
  return 0;
#endif
}
