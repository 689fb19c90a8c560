// wq4_layout.cpp -- host repack of GGUF Q4_0 blocks into MFMA fragment order
// and its exact inverse.  Layout spec: wq4_layout.hpp.
#include "wq4_layout.hpp"

#include <cstring>

namespace wq4 {

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

void repack_q4(const uint8_t* raw, const Q4Geom& g, uint8_t* nib, uint32_t* sc) {
  std::memset(nib, 0, g.nib_bytes());
  std::memset(sc, 0, g.sc_bytes());
  for (int64_t n = 0; n < g.n; ++n) {
    const int64_t nt = n / kNTile, r = n % kNTile;
    for (int64_t b = 0; b < g.kb; ++b) {
      const uint8_t* blk = raw + (n * g.kb + b) * kBlockBytes;
      const int64_t bp = b / 2, bi = b % 2;
      const uint32_t d = (uint32_t)blk[0] | ((uint32_t)blk[1] << 8);
      uint32_t& s = sc[(nt * g.nbp + bp) * 32 + r];
      s |= d << (16 * bi);
      for (int h = 0; h < 2; ++h) {
        const int lane = (int)r + 32 * h;
        uint32_t* dst = reinterpret_cast<uint32_t*>(nib + ((nt * g.nbp + bp) * 64 + lane) * 16);
        for (int kk = 0; kk < 2; ++kk) dst[bi * 2 + kk] = pack_half(blk + 2 + 8 * h, kk);
      }
    }
  }
}

void unrepack_q4(const uint8_t* nib, const uint32_t* sc, const Q4Geom& g, uint8_t* raw) {
  for (int64_t n = 0; n < g.n; ++n) {
    const int64_t nt = n / kNTile, r = n % kNTile;
    for (int64_t b = 0; b < g.kb; ++b) {
      uint8_t* blk = raw + (n * g.kb + b) * kBlockBytes;
      const int64_t bp = b / 2, bi = b % 2;
      const uint32_t d = (sc[(nt * g.nbp + bp) * 32 + r] >> (16 * bi)) & 0xffffu;
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

}  // namespace wq4
