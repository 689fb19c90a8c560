// wq4_layout.cpp -- host repack of GGUF Q4_0 blocks into MFMA fragment order
// and its exact inverse.  Layout spec: wq4_layout.hpp.
#include "wq4_layout.hpp"

#include <cmath>
#include <cstring>
#include <vector>

namespace wq4 {

static inline float h2f(uint16_t b) { return (float)__builtin_bit_cast(_Float16, b); }
static inline uint16_t f2h(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }

static inline uint32_t pack_half(const uint8_t* bytes, int kk) {
  // bytes -> 8 raw nibble bytes (8h..8h+7 of one block); kk selects the
  // low (elements 8h+j) or high (16+8h+j) nibble of each byte.
  uint32_t w = 0;
  for (int i = 0; i < 4; ++i) {
    uint32_t a = kk ? (bytes[2 * i] >> 4) : (bytes[2 * i] & 0x0f);
    uint32_t b = kk ? (bytes[2 * i + 1] >> 4) : (bytes[2 * i + 1] & 0x0f);
    w |= (a << (4 * i)) | (b << (16 + 4 * i));
  }
  return w;
}

static inline void unpack_half(uint32_t w, int kk, uint8_t* bytes) {
  for (int i = 0; i < 4; ++i) {
    uint32_t a = (w >> (4 * i)) & 0x0f;
    uint32_t b = (w >> (16 + 4 * i)) & 0x0f;
    if (kk) {
      bytes[2 * i] = (uint8_t)((bytes[2 * i] & 0x0f) | (a << 4));
      bytes[2 * i + 1] = (uint8_t)((bytes[2 * i + 1] & 0x0f) | (b << 4));
    } else {
      bytes[2 * i] = (uint8_t)((bytes[2 * i] & 0xf0) | a);
      bytes[2 * i + 1] = (uint8_t)((bytes[2 * i + 1] & 0xf0) | b);
    }
  }
}

// Exponent shift s for one output row: 8 * max d' <= 2^15, every nonzero
// d * 2^s still an exact f16 (else 0, i.e. no shift).
static int row_shift(const uint8_t* row, int64_t kb) {
  float dmax = 0.0f;
  for (int64_t b = 0; b < kb; ++b) {
    const float d = std::fabs(h2f((uint16_t)(row[b * kBlockBytes] | (row[b * kBlockBytes + 1] << 8))));
    if (!std::isfinite(d)) return 0;
    dmax = d > dmax ? d : dmax;
  }
  if (dmax == 0.0f) return 0;
  const int s = (int)std::floor(std::log2(4096.0 / (double)dmax));  // dmax * 2^s in (2^11, 2^12]
  for (int64_t b = 0; b < kb; ++b) {
    const uint16_t bits = (uint16_t)(row[b * kBlockBytes] | (row[b * kBlockBytes + 1] << 8));
    const float d = h2f(bits);
    const float ds = std::ldexp(d, s);
    if (std::fabs(ds) > 4096.0f) return 0;
    const uint16_t hb = f2h(ds);
    if (std::ldexp(h2f(hb), -s) != d || f2h(std::ldexp(h2f(hb), -s)) != bits) return 0;
  }
  return s;
}

void repack_q4(const uint8_t* raw, const Q4Geom& g, uint8_t* nib, uint32_t* sc, float* colscale) {
  std::memset(nib, 0, g.nib_bytes());
  std::memset(sc, 0, g.sc_bytes());
  for (int64_t n = 0; n < g.np; ++n) colscale[n] = 1.0f;
  for (int64_t n = 0; n < g.n; ++n) {
    const int64_t nt = n / kNTile, r = n % kNTile;
    const uint8_t* row = raw + n * g.kb * kBlockBytes;
    const int s = row_shift(row, g.kb);
    colscale[n] = std::ldexp(1.0f, -s);
    for (int64_t b = 0; b < g.kb; ++b) {
      const uint8_t* blk = row + b * kBlockBytes;
      const int64_t bp = b / 2, bi = b % 2;
      const uint16_t dbits = (uint16_t)(blk[0] | (blk[1] << 8));
      const uint32_t d = s ? f2h(std::ldexp(h2f(dbits), s)) : dbits;
      uint32_t& w = sc[(nt * g.nbp + bp) * 32 + r];
      w |= d << (16 * bi);
      for (int h = 0; h < 2; ++h) {
        const int lane = (int)r + 32 * h;
        uint32_t* dst = reinterpret_cast<uint32_t*>(nib + ((nt * g.nbp + bp) * 64 + lane) * 16);
        for (int kk = 0; kk < 2; ++kk) dst[bi * 2 + kk] = pack_half(blk + 2 + 8 * h, kk);
      }
    }
  }
}

void unrepack_q4(const uint8_t* nib, const uint32_t* sc, const float* colscale, const Q4Geom& g, uint8_t* raw) {
  for (int64_t n = 0; n < g.n; ++n) {
    const int64_t nt = n / kNTile, r = n % kNTile;
    const int s = -(int)std::lround(std::log2((double)colscale[n]));
    for (int64_t b = 0; b < g.kb; ++b) {
      uint8_t* blk = raw + (n * g.kb + b) * kBlockBytes;
      const int64_t bp = b / 2, bi = b % 2;
      const uint16_t ds = (uint16_t)((sc[(nt * g.nbp + bp) * 32 + r] >> (16 * bi)) & 0xffffu);
      const uint16_t d = s ? f2h(std::ldexp(h2f(ds), -s)) : ds;
      blk[0] = (uint8_t)(d & 0xff);
      blk[1] = (uint8_t)(d >> 8);
      for (int h = 0; h < 2; ++h) {
        const int lane = (int)r + 32 * h;
        const uint32_t* src = reinterpret_cast<const uint32_t*>(nib + ((nt * g.nbp + bp) * 64 + lane) * 16);
        for (int kk = 0; kk < 2; ++kk) unpack_half(src[bi * 2 + kk], kk, blk + 2 + 8 * h);
      }
    }
  }
}

static inline size_t f16_frag_index(const Q4Geom& g, int64_t n, int64_t k) {
  const int64_t nt = n / 32, r = n % 32, bp = k / 64, kb = k % 64;
  const int64_t blk = kb / 32, kk = (kb / 16) % 2, h = (kb / 8) % 2, j = kb % 8;
  const int64_t lane = r + 32 * h;
  return (size_t)(((nt * g.nbp + bp) * 64 + lane) * 32 + (blk * 2 + kk) * 8 + j);
}

void repack_f16(const uint16_t* w, const Q4Geom& g, uint16_t* frag) {
  std::memset(frag, 0, g.f16_frag_bytes());
  for (int64_t n = 0; n < g.n; ++n)
    for (int64_t k = 0; k < g.k; ++k) frag[f16_frag_index(g, n, k)] = w[n * g.k + k];
}

void unrepack_f16(const uint16_t* frag, const Q4Geom& g, uint16_t* w) {
  for (int64_t n = 0; n < g.n; ++n)
    for (int64_t k = 0; k < g.k; ++k) w[n * g.k + k] = frag[f16_frag_index(g, n, k)];
}

}  // namespace wq4
