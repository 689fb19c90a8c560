// wq4_enc.hip -- the encoder (large-M) Q4_0 GEMM: a deep LDS-DMA ring.
//
// Replaces the contraction of the reference's WGSL shader (src/gguf/
// shader.wgsl:72-89: per output, per Q4 block, 16 low + 16 high nibbles times
// x, scaled by the block's f16 d) for the encoder's M = B * 1500 rows with
// the arithmetic of q4_gemm_prefill_kernel (wq4_q4gemm.hip), bit for bit:
//   per Q4 block  t = MFMA(x_hi0, q0) + MFMA(x_lo0, q0) + MFMA(x_hi1, q1) +
//                     MFMA(x_lo1, q1)       (q = nibble - 8, exact f16; f32
//                                            accumulation from zero)
//                 acc = t * d' + acc        (f32, blocks in order)
//   y = acc * colscale * 2^-4 -> epilogue
// so a row's result never depends on the tile shape, the grid or M.
//
// What changes is the memory pipeline (r02 profile: the old kernel's 48 %
// MFMA-busy came from the structure, not the VALU -- removing every scale FMA
// and the dequantisation gained only 11 %, tools/pf_variants.py).  The old
// kernel staged one 64-k block pair of A per barrier into a 2-deep ring and
// drained it (vmcnt(0)) every step, so each step waited for the NEXT step's
// loads.  Here the ring holds single Q4 blocks (32 k):
//   * A: 4 slots, loaded 3 blocks ahead by buffer_load ... lds (OOB rows read
//     as zeros: partial m-groups need no guard),
//   * B: the repacked nibbles (wq4_layout.hpp, 1 KiB per n-tile and block
//     pair) in 3 block-pair slots, loaded 1.5 block pairs ahead,
//   * the per-block f16 scales with them (1 KiB per block pair),
// and each block ends in ONE raw s_barrier preceded by a COUNTED
// s_waitcnt vmcnt(N) that retires only the slot about to be read
// (cdna_hip_programming.md §5 'Pipelining across barriers', T3+T4): the loads
// of the next three blocks stay in flight across it.  All LDS is one
// __shared__ array (§5 'Three .s-level traps' (a)).
//
// Two geometries (rows choose; the per-element arithmetic is the same):
//   L  8 waves = 2 (M) x 4 (N), each 128 x 64 (4 x 2 tiles of 32x32):
//      256 x 256 per workgroup, 155 KiB LDS, one workgroup per CU;
//   S  4 waves = 1 x 4, each 64 x 32 (2 x 1 tiles): 64 x 128 per workgroup,
//      47 KiB LDS -- one clip (M = 1500) still fills the 256 CUs.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>
#include <type_traits>

#include "wq4_device.hpp"
#include "wq4_kernels.hpp"
#include "wq4_tile_epi.hpp"

namespace wq4 {

// WQ4_ENC_DIAG (timing diagnostics only, tools/pf_variants.py; 0 in the
// product): 1 = no scale FMAs (chains accumulate straight into acc), 2 = 1 +
// no dequantisation.
#ifndef WQ4_ENC_DIAG
#define WQ4_ENC_DIAG 0
#endif

namespace {

typedef __attribute__((address_space(3))) void lds_void;

// One 16-B-per-lane LDS-DMA piece: lane l's 16 bytes from rsrc + voff land
// at lds_base + 16 l (lds_base wave-uniform).  Offsets past the resource's
// size read zeros.
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, uint32_t voff, void* lds_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)lds_base, 16, voff, 0, 0, 0);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_bytes(const void* base, uint64_t bytes) {
  const uint32_t n = bytes > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)n, 0x00020000);
}

constexpr int kStageLdE = 68;  // padded f32 row stride of the tiled-epilogue stage (as wq4_q4gemm.hip)

__device__ __forceinline__ int acc_row_e(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// s_waitcnt vmcnt(N) with N a compile-time count (the immediate is part of
// the instruction)
template <int N>
__device__ __forceinline__ void vmcnt_wait() {
  static_assert(N >= 0 && N <= 12, "vmcnt immediate out of the listed range");
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 7) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 9) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
  else if constexpr (N == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else if constexpr (N == 11) asm volatile("s_waitcnt vmcnt(11)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
}

}  // namespace

// The ring geometry of one configuration.
template <int WM, int TM, int TN>
struct EncGeo {
  static constexpr int WN = 4;
  static constexpr int WAVES = WM * WN;
  static constexpr int THREADS = 64 * WAVES;
  static constexpr int MT = WM * TM;             // m-tiles per workgroup
  static constexpr int NT = WN * TN;             // n-tiles per workgroup
  static constexpr int A_SLOT = MT * 4096;       // one Q4 block of A (hi, lo; kk 0, 1)
  static constexpr int B_SLOT = NT * 1024;       // one block pair of nibbles
  static constexpr int SC_SLOT = WAVES * 256;    // one block pair of scales: 256 B per wave piece
  static constexpr int A_SLOTS = 4, B_SLOTS = 3;
  static constexpr int B_OFF = A_SLOTS * A_SLOT;
  static constexpr int SC_OFF = B_OFF + B_SLOTS * B_SLOT;
  static constexpr int LDS = SC_OFF + B_SLOTS * SC_SLOT;
  static constexpr int NA = MT * 4 / WAVES;      // A pieces per wave per block (= TM)
  static constexpr int NB = NT / WAVES;          // nibble pieces per wave per block pair
  static_assert(NA * WAVES == MT * 4 && NB * WAVES == NT && NB >= 1, "uneven ring split");
  static_assert(NT <= 2 * WAVES, "one scale piece per wave covers <= 2 n-tiles");
  static constexpr int STAGE = WAVES * 32 * kStageLdE * 4;  // tiled epilogue stage (reuses the ring)
  static_assert(STAGE <= LDS || STAGE <= 160 * 1024, "stage");
};

template <int WM, int TM, int TN, int EPI>
__global__ __launch_bounds__(64 * WM * 4, WM == 2 ? 2 : 3) void q4_gemm_enc_kernel(const uint8_t* __restrict__ nib,
                                                                     const uint32_t* __restrict__ sc,
                                                                     const float* __restrict__ colscale,
                                                                     const _Float16* __restrict__ at, int mtiles,
                                                                     int nbp, int ntiles, EpiArgs e) {
  using G = EncGeo<WM, TM, TN>;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int wr = wave / G::WN, wc = wave % G::WN;
  const int ngroups = (ntiles + G::NT - 1) / G::NT;
  const int mgroups = (mtiles + G::MT - 1) / G::MT;
  const int wg = xcd_remap(blockIdx.x, ngroups * mgroups);
  const int mg = wg / ngroups, ng = wg % ngroups;
  const int kb = 2 * nbp;  // Q4 blocks (padded to even, as the A-tiled operand)

  // buffer resources: A from this group's first m-tile (rows past the
  // operand read as zeros), nibbles and scales over the whole tensor
  const uint8_t* abase = reinterpret_cast<const uint8_t*>(at) + (size_t)mg * G::MT * kb * 4096;
  const int64_t mrem = (int64_t)mtiles - (int64_t)mg * G::MT;
  const __amdgpu_buffer_rsrc_t ra = rsrc_bytes(abase, (uint64_t)(mrem < 0 ? 0 : mrem) * kb * 4096);
  const __amdgpu_buffer_rsrc_t rb = rsrc_bytes(nib, (uint64_t)ntiles * nbp * 1024);
  const __amdgpu_buffer_rsrc_t rsc = rsrc_bytes(sc, (uint64_t)ntiles * nbp * 128);

  // A piece j of block b (j = wave + WAVES * i): m-tile j / 4, fragment j % 4
  auto issue_a = [&](int b) {
    uint8_t* slot = smem + (b & 3) * G::A_SLOT;
#pragma unroll
    for (int i = 0; i < G::NA; ++i) {
      const int j = wave + G::WAVES * i;
      const uint32_t off = b < kb ? (uint32_t)(((j >> 2) * kb + b) * 4096 + (j & 3) * 1024 + lane * 16) : 0xFFFFFFF0u;
      dma16(ra, off, slot + j * 1024);
    }
  };
  // nibbles of block pair p: n-tile wave + WAVES * i (1 KiB each), then the
  // scales: every wave one 4-B-per-lane piece, lanes 0..31 = the 32 u32 of
  // n-tile `wave`'s (n-tile, pair) record, lanes 32..63 those of n-tile
  // wave + WAVES (n-tiles past the group read zeros into padding).  Loads past the last block / pair are
  // issued too, as zero-reads (out-of-range offsets) into slots nobody reads
  // any more: every block issues the same count, so one vmcnt fits all.
  auto issue_b = [&](int p) {
    const int s = p % G::B_SLOTS;
    const bool live = p < nbp;
#pragma unroll
    for (int i = 0; i < G::NB; ++i) {
      const int t = wave + G::WAVES * i;
      const uint32_t off = live ? (uint32_t)((((size_t)(ng * G::NT + t)) * nbp + p) * 1024 + lane * 16) : 0xFFFFFFF0u;
      dma16(rb, off, smem + G::B_OFF + s * G::B_SLOT + t * 1024);
    }
    const int st = wave + G::WAVES * (lane >> 5);  // lanes 32..63: a second n-tile when NT > WAVES
    const uint32_t soff = (live && st < G::NT)
                              ? (uint32_t)((((size_t)(ng * G::NT + st)) * nbp + p) * 128 + (lane & 31) * 4)
                              : 0xFFFFFFF0u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsc, (lds_void*)(smem + G::SC_OFF + s * G::SC_SLOT + wave * 256), 4, soff,
                                             0, 0, 0);
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.0f;

  // prologue = the issues of virtual blocks -4 .. -1 (see the schedule below)
  issue_b(0);
  issue_a(0);
  issue_a(1);
  issue_b(1);
  issue_a(2);

  // B operand of block hb: per n-tile the dequantised nibbles (kk 0, 1) and
  // the block's f16 scale (slot of block pair hb / 2)
  half8 qf[TN][2];
  float dsc[TN], dprev[TN];
  auto load_b = [&](int hb) {
    const int bs = (hb >> 1) % G::B_SLOTS, blk = hb & 1;
#pragma unroll
    for (int nt = 0; nt < TN; ++nt) {
      const int t = wc * TN + nt;
      const u32x2 w2 = *reinterpret_cast<const u32x2*>(smem + G::B_OFF + bs * G::B_SLOT + t * 1024 + lane * 16 + blk * 8);
      const uint32_t s2 = *reinterpret_cast<const uint32_t*>(smem + G::SC_OFF + bs * G::SC_SLOT +
                                                             (t % G::WAVES) * 256 + (t / G::WAVES) * 128 + r * 4);
#if WQ4_ENC_DIAG >= 2  // timing diagnostics: no dequantisation
      qf[nt][0] = __builtin_bit_cast(half8, u32x4{w2[0], w2[1], w2[0], w2[1]});
      qf[nt][1] = __builtin_bit_cast(half8, u32x4{w2[1], w2[0], w2[1], w2[0]});
#else
      qf[nt][0] = deq8(w2[0]);
      qf[nt][1] = deq8(w2[1]);
#endif
      dsc[nt] = (float)__builtin_bit_cast(_Float16, (uint16_t)(blk ? (s2 >> 16) : (s2 & 0xffffu)));
    }
  };
  // every wave: NA A pieces per block, NB + 1 B pieces every second block
  auto wait_block = [&]() {
    vmcnt_wait<2 * G::NA + G::NB + 1>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");  // no LDS read of this block moves above the barrier
    __builtin_amdgcn_sched_barrier(0);
  };

  // Two chain temporaries: chain c (m-tile c / TN, n-tile c % TN) writes
  // tt[c & 1] while the scale FMAs of chain c - 1 (the other one) fill its
  // MFMA gaps; the last chain of a block (odd: TM * TN is even) is scaled in
  // the first chain of the next one.  Every acc element still gets its
  // blocks' FMAs in block order: the arithmetic of q4_gemm_prefill_kernel.
  static_assert((TM * TN) % 2 == 0, "chain parity must repeat per block");
  floatx16 tt[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    tt[0][i] = 0.0f;
    tt[1][i] = 0.0f;
  }
#pragma unroll
  for (int nt = 0; nt < TN; ++nt) dprev[nt] = 0.0f;  // "block -1": acc += 0 * 0, an exact no-op

  // Schedule, block h: [wait] -> s_barrier -> build block h's B operand ->
  // issue A(h+3) (slot (h+3)%4 = (h-1)%4, last read by block h-1: every
  // wave is past it) and, at even h, B(h/2 + 2) (slot last read by block
  // h-2) -> compute block h.  Block h's wait must retire A(h) and B(h/2).
  // Issue order: per block an A group (NA pieces), at even blocks then a B
  // group (NB' = NB + 1 scale piece); B(p) goes out at block 2p - 4.  At each
  // wait the loads issued after the oldest one it needs are two A groups and
  // one B group: vmcnt(2 NA + NB') retires exactly what the block reads
  // while the following blocks' loads stay in flight; past the end every
  // block still issues its (zero-read) pieces, so the counts hold.
  for (int hb = 0; hb < kb; ++hb) {
    wait_block();
    load_b(hb);
    issue_a(hb + 3);
    if (!(hb & 1)) issue_b(hb / 2 + 2);
    const uint8_t* aslot = smem + (hb & 3) * G::A_SLOT + (wr * TM) * 4096 + lane * 16;
    half8 ah[2], al[2];
#pragma unroll
    for (int c = 0; c < TM * TN; ++c) {
      const int mt = c / TN, nt = c % TN;
      if (nt == 0) {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          ah[kk] = *reinterpret_cast<const half8*>(aslot + mt * 4096 + (kk * 2 + 0) * 1024);
          al[kk] = *reinterpret_cast<const half8*>(aslot + mt * 4096 + (kk * 2 + 1) * 1024);
        }
      }
      // pending chain c - 1 (the previous block's last chain for c = 0)
      const int pm = c == 0 ? TM - 1 : (c - 1) / TN, pn = c == 0 ? TN - 1 : (c - 1) % TN;
      const float pd = c == 0 ? dprev[TN - 1] : dsc[pn];
      floatx16& t = tt[c & 1];
      const floatx16& tp = tt[(c + 1) & 1];
#if WQ4_ENC_DIAG >= 1  // timing diagnostics (wrong results): chains accumulate into acc, no VALU scale
      (void)t; (void)tp; (void)pd; (void)pm; (void)pn;
      acc[mt][nt] = mfma32(ah[0], qf[nt][0], acc[mt][nt]);
      acc[mt][nt] = mfma32(al[0], qf[nt][0], acc[mt][nt]);
      acc[mt][nt] = mfma32(ah[1], qf[nt][1], acc[mt][nt]);
      acc[mt][nt] = mfma32(al[1], qf[nt][1], acc[mt][nt]);
#else
      // the chain of q4_gemm_prefill_kernel, in its order
      t = mfma32(ah[0], qf[nt][0], floatx16{});
      t = mfma32(al[0], qf[nt][0], t);
      t = mfma32(ah[1], qf[nt][1], t);
      t = mfma32(al[1], qf[nt][1], t);
      acc[pm][pn] = tp * pd + acc[pm][pn];
#endif
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
      }
    }
#pragma unroll
    for (int nt = 0; nt < TN; ++nt) dprev[nt] = dsc[nt];
  }
  // the last block's last chain
  acc[TM - 1][TN - 1] = tt[1] * dprev[TN - 1] + acc[TM - 1][TN - 1];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // ring drained (vmcnt(0) above), every wave done reading: the stage may reuse it

  const int mt0 = mg * G::MT + wr * TM;  // first m-tile of this wave
  const int nt0 = ng * G::NT + wc * TN;  // first n-tile of this wave
  float cs[TN];
  const float ainv = e.act_inv ? *e.act_inv : kActScaleInv;
  // bias preloaded once (branch-free buffer loads): with no residual the
  // epilogue then reads nothing, and hipcc has no load to drain vmcnt(0)
  // for between the stores (it did so per element: wq4_tile_epi.hpp)
  float b[TN];
  {
    const __amdgpu_buffer_rsrc_t rb = epi_rsrc(e.bias, e.bias ? (uint32_t)e.n * 4 : 0);
#pragma unroll
    for (int nt = 0; nt < TN; ++nt) {
      const int col = (nt0 + nt) * 32 + r;
      cs[nt] = nt0 + nt < ntiles ? colscale[col] * ainv : 1.0f;
      b[nt] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rb, col < e.n ? col * 4 : kEpiOob, 0, 0));
    }
    // landed before the first store: otherwise hipcc waits for them (vmcnt(0),
    // behind every earlier store) at the top of each exec-masked store below
    __builtin_amdgcn_s_waitcnt(0x0F70);
  }

  if constexpr (EPI == kEpiF32 || EPI == kEpiHeadMajor) {
    auto idx = [&](int row, int col) {
      return EPI == kEpiHeadMajor ? out_index(e, row, col) : (size_t)row * e.ldo + col;
    };
    if (e.residual) {  // element-wise residual reads (all 16 of a tile before its stores)
#pragma unroll
      for (int mt = 0; mt < TM; ++mt)
#pragma unroll
        for (int nt = 0; nt < TN; ++nt)
          epi_store_tile<true>(
              acc[mt][nt], cs[nt], (nt0 + nt) * 32 + r, [&](int i) { return (mt0 + mt) * 32 + acc_row_e(i, h); },
              idx, e);
    } else {
#pragma unroll
      for (int mt = 0; mt < TM; ++mt)
#pragma unroll
        for (int nt = 0; nt < TN; ++nt) {
          const int col = (nt0 + nt) * 32 + r;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int row = (mt0 + mt) * 32 + acc_row_e(i, h);
            if (col < e.n && row < e.m) e.out[idx(row, col)] = epi_value_pre(acc[mt][nt][i] * cs[nt], b[nt], 0.0f, e);
          }
        }
    }
  } else {
    static_assert(EPI == kEpiTiled, "f32, head-major f32 or A-tiled outputs");
    float* stage = reinterpret_cast<float*>(smem) + wave * (32 * kStageLdE);
    const size_t kbp_next = (size_t)e.nbp_next * 2;
    half8* dst = reinterpret_cast<half8*>(e.out_tiled);
    // RES: residual reads element by element; without (the GELU GEMM) the
    // preloaded bias and no memory read before the fragment stores
    auto run = [&](auto res_c) {
      constexpr bool RES = decltype(res_c)::value;
#pragma unroll
      for (int mt = 0; mt < TM; ++mt) {
#pragma unroll
        for (int nt = 0; nt < TN; ++nt)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int rl = acc_row_e(i, h);
            const int row = (mt0 + mt) * 32 + rl;
            const int col = (nt0 + nt) * 32 + r;
            stage[rl * kStageLdE + nt * 32 + r] =
                !(row < e.m && col < e.n) ? 0.0f
                : RES                   ? epi_value(acc[mt][nt][i] * cs[nt], row, col, e)
                                        : epi_value_pre(acc[mt][nt][i] * cs[nt], b[nt], 0.0f, e);
          }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's stage writes land before its reads
        __builtin_amdgcn_wave_barrier();
        // the slab as A-tiled fragments: lane (r, h) of (m-tile, n-tile = block
        // of the next GEMM, kk) holds columns 16 kk + 8 h .. + 7 of row r
        if ((mt0 + mt) < mtiles) {
#pragma unroll
          for (int nt = 0; nt < TN; ++nt) {
            if (nt0 + nt >= ntiles) continue;  // padding n-tiles (N % 64 == 32) are written: zeros
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
              const float* src = stage + r * kStageLdE + nt * 32 + kk * 16 + h * 8;
              const floatx4 a = *reinterpret_cast<const floatx4*>(src);
              const floatx4 c = *reinterpret_cast<const floatx4*>(src + 4);
              half8 hi, lo;
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                _Float16 x, y;
                split_act(a[j], x, y);
                hi[j] = x;
                lo[j] = y;
                split_act(c[j], x, y);
                hi[4 + j] = x;
                lo[4 + j] = y;
              }
              const size_t frag = (((size_t)(mt0 + mt) * kbp_next + (nt0 + nt)) * 2 + kk) * 2;
              dst[(frag + 0) * 64 + lane] = hi;
              dst[(frag + 1) * 64 + lane] = lo;
            }
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
    };
    if (e.residual) run(std::true_type{});
    else run(std::false_type{});
  }
}

// ------------------------------------------------------------------------
// Launcher.
// ------------------------------------------------------------------------
// 0 = off (the prefill tile kernel), 1 = by rows (enc_gemm_pick), 2 = always
// L, 3 = always S, 5 = always the wide kernel (wq4_wide.hip).
// Initialised from WQ4_ENC_KERNEL (default 1); wq4_debug_set_enc_kernel
// switches it at run time (A/B and bit-equality tests in one process).
static std::atomic<int> g_enc_mode{[] {
  const char* env = getenv("WQ4_ENC_KERNEL");
  return env ? atoi(env) : 1;
}()};

// Which kernel runs a rows > 128 Q4_0 GEMM: 0 = the prefill tile kernel,
// 2 = the ring kernel's L geometry, 3 = its S geometry, 5 = the 8-wave wide
// kernel (wq4_wide.hip).  Measured (r03, tools/enc_ab.py, Large-V3 encoder
// shapes): at M = 1500 the tile kernel's 60-240 workgroups leave the chip
// idle and S runs 1.1-2.4x faster (one layer's four GEMMs 0.191 vs 0.349
// ms); crossover at M = 1500, 3000, 6000, 12000 (profiles/r03_enc_ab.log):
// S while the tile kernel's grid has < 400 workgroups.  r06
// (profiles/r06_enc_ab_rows.log, tile vs wide interleaved in one process):
// at M = 48000 the wide kernel is 1-7 % faster on every shape (457 / 454 /
// 488 / 562 TF/s against 453 / 424 / 471 / 530), at 24000 and 12000 on 7 of
// 8, at 6000 only where its own grid is >= 480 workgroups.  After the wide
// kernel's carried schedule and drain-free epilogue (profiles/r06ab_enc_ab_*.log,
// r06aa_enc_ab_*.log, M = 3000 .. 24000, modes 0 / 2 / 3 / 5): the wide
// kernel is fastest from ~170 of its workgroups up (+9-21 % where that moved
// the choice: M = 3000 / N = 3840, 5120; M = 9000 / N = 1280; M = 12000 /
// N = 1280), 3 % behind the tile kernel at M = 6000 / 9000, N = 3840 (a
// third round of 256 workgroups 40 % full); below, the ring kernel's S.
int enc_gemm_pick(const Q4Geom& g, int rows, int epi_mode, int ns, int wtype) {
  const int mode = g_enc_mode.load();
  if (mode == 0 || wtype != kWeightsQ4 || rows <= 128 || g.kb < 1) return 0;
  if (mode == 5) return wide_gemm_supported(g, rows, ns, wtype) ? 5 : 0;
  const int64_t mt = round_up(rows, kMPad) / kMTile;
  const int64_t tile_grid = ((mt + 3) / 4) * ((g.ntiles + 7) / 8);
  const int64_t wide_grid = ((mt + 7) / 8) * ((g.ntiles + 7) / 8);
  if (mode == 1 && wide_grid >= 170 && wide_gemm_supported(g, rows, ns, wtype)) return 5;
  if (ns != 2) return 0;  // the ring kernel: f16x2 operands only
  if (mode >= 2) return mode;
  return tile_grid < 400 ? 3 : 0;
}

template <int WM, int TM, int TN>
static hipError_t launch_enc_t(const Q4Geom& g, const uint8_t* nib, const uint32_t* sc, const float* cs,
                               const _Float16* at, int rows, const EpiArgs& e, int epi_mode, hipStream_t st) {
  using G = EncGeo<WM, TM, TN>;
  const int mtiles = (int)(round_up(rows < 1 ? 1 : rows, kMPad) / kMTile);
  const int ngroups = (int)((g.ntiles + G::NT - 1) / G::NT);
  const int mgroups = (mtiles + G::MT - 1) / G::MT;
  const size_t lds = G::LDS > G::STAGE ? (size_t)G::LDS : (size_t)G::STAGE;
  const dim3 grid((unsigned)(ngroups * mgroups));
  if (epi_mode == kEpiTiled)
    hipLaunchKernelGGL((q4_gemm_enc_kernel<WM, TM, TN, kEpiTiled>), grid, dim3(G::THREADS), lds, st, nib, sc, cs, at,
                       mtiles, (int)g.nbp, (int)g.ntiles, e);
  else if (epi_mode == kEpiHeadMajor)  // the cross K / V cache GEMMs (wq4_gemm_tiled_headmajor)
    hipLaunchKernelGGL((q4_gemm_enc_kernel<WM, TM, TN, kEpiHeadMajor>), grid, dim3(G::THREADS), lds, st, nib, sc, cs,
                       at, mtiles, (int)g.nbp, (int)g.ntiles, e);
  else
    hipLaunchKernelGGL((q4_gemm_enc_kernel<WM, TM, TN, kEpiF32>), grid, dim3(G::THREADS), lds, st, nib, sc, cs, at,
                       mtiles, (int)g.nbp, (int)g.ntiles, e);
  return hipGetLastError();
}

hipError_t launch_enc_gemm(const Q4Geom& g, const uint8_t* nib, const uint32_t* sc, const float* cs,
                           const _Float16* at, int rows, const EpiArgs& e, int epi_mode, int geo, hipStream_t st) {
  if (geo == 2) return launch_enc_t<2, 4, 2>(g, nib, sc, cs, at, rows, e, epi_mode, st);
  if (geo == 4) return launch_enc_t<1, 1, 2>(g, nib, sc, cs, at, rows, e, epi_mode, st);
  return launch_enc_t<1, 2, 1>(g, nib, sc, cs, at, rows, e, epi_mode, st);
}

}  // namespace wq4

extern "C" int wq4_debug_set_enc_kernel(int mode) {
  if (mode < 0 || mode > 5) return -1;
  const int prev = wq4::g_enc_mode.load();
  wq4::g_enc_mode.store(mode);
  return prev;
}
