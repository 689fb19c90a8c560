// wq4_layout.hpp -- on-device data layouts of the Q4_0 path (host + device).
//
// Weights (Q4Tensor, src/gguf/tensor.rs:21-27) arrive as raw GGUF Q4_0 bytes:
// row-major [N, K], K/32 blocks of 18 B per row (f16 scale LE + 16 nibble
// bytes; low nibble = element i, high nibble = element i+16; shader.wgsl:7-21).
// On upload they are repacked, losslessly and at the same 4.5 bits/weight,
// into the fragment order of v_mfma_f32_32x32x16_f16:
//
//   n-tile  = 32 output rows n, block pair bp = 2 Q4 blocks (64 k)
//   nib[nt][bp][lane 0..63][16 B]        1 KiB per (nt, bp): ONE coalesced
//                                        global_load_dwordx4 per wave
//   lane l: r = l & 31 -> n = 32*nt + r ; h = l >> 5 -> raw bytes 8h..8h+7
//   16 B = { blk0.kk0, blk0.kk1, blk1.kk0, blk1.kk1 } as u32 words, where
//   kk0 = the 8 LOW nibbles (elements 8h+j), kk1 = the 8 HIGH nibbles
//   (elements 16+8h+j), j = 0..7, packed so that
//     w = sum_i q[j=2i] << 4i | q[j=2i+1] << (16+4i),  i = 0..3
//   which turns into the MFMA B operand (8 x f16 (q-8), order j) with
//   4 v_and_or + 1 shift + 4 packed-f16 ops (wq4_device.hpp deq8()).
//   sc[nt][bp][32 n] : u32 = { f16 d'(blk 2bp), f16 d'(blk 2bp+1) }
//   colscale[n]      : f32 2^-s_n
// where d' = d * 2^s_n exactly (a pure exponent shift of the GGUF f16 scale)
// and s_n is chosen per output row so that 8 * max_b d'_{n,b} <= 2^15: the
// kernels build the MFMA B operand as the exact two-term f16 sum
//   B_hi + B_lo = (q - 8) * d'      (B_hi = f16 RN, B_lo = f16 remainder)
// and multiply each output column by colscale once, in the epilogue.  If a
// row's scales span more than the f16 range allows (d_max/d_min > 2^26) its
// s_n is 0 and d' = d.  The repack stays lossless (unrepack_q4 recovers d).
//
// N is padded to a multiple of 64 and the block count to a multiple of 2 with
// d = 0 blocks (they contribute exactly 0).
//
// Activations feeding a Q4 GEMM ("A-tiled"): per 32-row m-tile, per Q4 block
// b, per k-half kk (16 k), per split s (hi, lo) one 1 KiB MFMA A fragment:
//   At[mt][b][kk][s][lane][8 x f16],  lane l: r = l & 31 -> m = 32*mt + r,
//   h = l >> 5 -> k = 32*b + 16*kk + 8*h + j,  j = 0..7
// so one (m-tile, block pair) is 4*NS KiB contiguous and every fragment read
// is lane-linear (conflict-free ds_read_b128, coalesced global loads).
// x = hi + lo with hi = f16(x), lo = f16(x - hi)  (NS = 2), or hi only (NS=1).
#pragma once
#include <cstddef>
#include <cstdint>

namespace wq4 {

constexpr int kBlock = 32;       // Q4_0 elements per block
constexpr int kBlockBytes = 18;  // f16 scale + 16 nibble bytes
constexpr int kNTile = 32;       // output rows per MFMA n-tile
constexpr int kNPad = 64;        // N padding granule
constexpr int kMTile = 32;       // activation rows per m-tile
constexpr int kMPad = 128;       // M padding granule of A-tiled buffers

struct Q4Geom {
  int64_t n = 0, k = 0;   // logical [N, K]
  int64_t np = 0;         // padded N (multiple of 64)
  int64_t kb = 0;         // K / 32 blocks
  int64_t nbp = 0;        // block pairs = ceil(kb / 2)
  int64_t ntiles = 0;     // np / 32
  size_t nib_bytes() const { return (size_t)ntiles * nbp * 1024; }
  size_t sc_bytes() const { return (size_t)ntiles * nbp * 32 * 4; }
  size_t colscale_bytes() const { return (size_t)np * 4; }
  size_t f16_frag_bytes() const { return (size_t)ntiles * nbp * 4096; }  // F16 weights
};

inline int64_t round_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }

inline Q4Geom make_geom(int64_t n, int64_t k) {
  Q4Geom g;
  g.n = n;
  g.k = k;
  g.np = round_up(n, kNPad);
  g.kb = k / kBlock;
  g.nbp = (g.kb + 1) / 2;
  g.ntiles = g.np / kNTile;
  return g;
}

// Bytes of an A-tiled buffer holding `rows` rows of a K-wide operand.
inline size_t atiled_bytes(int64_t rows, int64_t k, int ns) {
  int64_t mp = round_up(rows < 1 ? 1 : rows, kMPad);
  int64_t nbp = (k / kBlock + 1) / 2;
  return (size_t)(mp / kMTile) * (size_t)nbp * 4096u * (size_t)ns;
}

// Host-side repack of raw GGUF Q4_0 bytes into nib/sc (see header comment).
void repack_q4(const uint8_t* raw, const Q4Geom& g, uint8_t* nib, uint32_t* sc, float* colscale);
// Exact inverse (for Q4Tensor::dequantize and the lossless check).
void unrepack_q4(const uint8_t* nib, const uint32_t* sc, const float* colscale, const Q4Geom& g, uint8_t* raw);

// Unquantized f16 weights (BASELINE config 5; GGUF F16 linear tensors):
// row-major [N, K] IEEE halves repacked into the same MFMA B-fragment order,
//   frag[nt][bp][lane][blk][kk][8 halves]  (4 KiB per (nt, bp), 64 B a lane)
//   lane l: n = 32 nt + (l & 31), k = 64 bp + 32 blk + 16 kk + 8 (l >> 5) + j
// (zero beyond N / K): the kernels feed these halves to the MFMA as they are.
void repack_f16(const uint16_t* w, const Q4Geom& g, uint16_t* frag);
void unrepack_f16(const uint16_t* frag, const Q4Geom& g, uint16_t* w);

}  // namespace wq4
