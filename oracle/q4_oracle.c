/*
 * q4_oracle.c -- CPU restatement of the reference's Q4_0 dequant+GEMM path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (whisper-burn_amd/, the
 * C-ABI library libwq4.so) links, loads or calls this file.  It is the checker
 * that tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use.
 *
 * Parity pinning: the quantizer restatement q4o_quantize_convert() is pinned
 * byte-for-byte against golden vectors produced by importing the reference's
 * own scripts/convert_whisper.py:quantize_q4_0 in the build container
 * (tests/golden/make_golden.py -> tests/golden/q4_golden.npz).  The rest is
 * pinned against the reference's known-answer assertions in
 * src/gguf/tests.rs (tolerances 0.08 / 1e-5 / 1e-3 / 1e-2) re-expressed in
 * tests/test_oracle.py.  The reference crate itself cannot be compiled here
 * (no Rust toolchain), so there is no oracle/_ref build for this path.
 *
 * Every function cites the reference file:line it restates.  Compiled with
 * -O2 -ffp-contract=off so that a*b+c is never fused (Rust and numpy do not
 * fuse either); the summation order of each loop is the reference's.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define Q4_BLOCK 32
#define Q4_BYTES 18

/* ---- IEEE binary16 <-> binary32 (round-to-nearest-even), exact ----------
 * Stand-in for half::f16::from_f32 / to_f32 (half 2.7.1, used at
 * src/gguf/tensor.rs:99 and src/gguf/tests.rs:44,75) and np.float16()
 * (scripts/convert_whisper.py:55).  Exhaustively checked against numpy in
 * tests/test_oracle.py. */
static inline uint32_t f32_bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float bits_f32(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

float q4o_f16_to_f32(uint16_t h) {
  uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  uint32_t exp = (h >> 10) & 0x1f;
  uint32_t man = h & 0x3ffu;
  if (exp == 0) {
    if (man == 0) return bits_f32(sign);
    /* subnormal: value = man * 2^-24, exact in f32 */
    float v = (float)man * 5.9604644775390625e-08f;
    return sign ? -v : v;
  }
  if (exp == 31) return bits_f32(sign | 0x7f800000u | (man << 13));
  return bits_f32(sign | ((exp + 112u) << 23) | (man << 13));
}

uint16_t q4o_f32_to_f16(float f) {
  uint32_t u = f32_bits(f);
  uint32_t sign = (u >> 16) & 0x8000u;
  uint32_t abs = u & 0x7fffffffu;
  if (abs >= 0x7f800000u) { /* inf / nan */
    if (abs > 0x7f800000u) return (uint16_t)(sign | 0x7e00u | ((abs >> 13) & 0x3ffu));
    return (uint16_t)(sign | 0x7c00u);
  }
  if (abs >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u); /* rounds to >= 65520 -> inf */
  if (abs < 0x38800000u) {                                   /* below 2^-14: subnormal */
    if (abs < 0x33000000u) return (uint16_t)sign;            /* < 2^-25: rounds to 0 (tie at 2^-25 -> even 0) */
    uint32_t e = abs >> 23;
    uint32_t m = (abs & 0x7fffffu) | 0x800000u;
    uint32_t shift = 126u - e; /* 14..24 */
    uint32_t r = m >> shift;
    uint32_t rem = m & ((1u << shift) - 1u);
    uint32_t half = 1u << (shift - 1u);
    if (rem > half || (rem == half && (r & 1u))) r++;
    return (uint16_t)(sign | r);
  }
  uint32_t r = abs - 0x38000000u; /* rebias exponent 127 -> 15 */
  uint32_t low = r & 0x1fffu;
  r >>= 13;
  if (low > 0x1000u || (low == 0x1000u && (r & 1u))) r++;
  return (uint16_t)(sign | r);
}

/* ---- round half to even, f32 (numpy np.round semantics) ---------------- */
static float round_half_even(float x) {
  float r = nearbyintf(x); /* default rounding mode is to-nearest-even */
  return r;
}

/* ---- quantizers ---------------------------------------------------------
 * q4o_quantize_test: src/gguf/tests.rs:24-57 (the reference test quantizer).
 *   amax = max |v| (fold from 0.0, f32::max), d = amax / 7.0 (f32),
 *   id = d != 0 ? 1/d : 0, q = ((v*id + 8.5) as u8).min(15)  -- Rust `as u8`
 *   saturates (negative -> 0, NaN -> 0).  Low nibble = elements 0..15,
 *   high nibble = elements 16..31 (tests.rs:48-53).  Scale f16 LE first. */
static uint8_t rust_as_u8(float v) {
  if (!(v > 0.0f)) return 0; /* negative, -0, NaN */
  if (v >= 255.0f) return 255;
  return (uint8_t)v; /* truncation toward zero */
}

void q4o_quantize_test(const float* data, int64_t n, uint8_t* out) {
  int64_t nb = n / Q4_BLOCK;
  for (int64_t b = 0; b < nb; ++b) {
    const float* blk = data + b * Q4_BLOCK;
    float amax = 0.0f;
    for (int i = 0; i < Q4_BLOCK; ++i) amax = fmaxf(amax, fabsf(blk[i])); /* tests.rs:39 */
    float d = amax / 7.0f;                                                 /* tests.rs:40 */
    float id = d != 0.0f ? 1.0f / d : 0.0f;                                /* tests.rs:41 */
    uint16_t h = q4o_f32_to_f16(d);                                        /* tests.rs:44 */
    uint8_t* o = out + b * Q4_BYTES;
    o[0] = (uint8_t)(h & 0xff);
    o[1] = (uint8_t)(h >> 8);
    for (int i = 0; i < 16; ++i) { /* tests.rs:48-54 */
      uint8_t q0 = rust_as_u8(blk[i] * id + 8.5f);
      uint8_t q1 = rust_as_u8(blk[i + 16] * id + 8.5f);
      if (q0 > 15) q0 = 15;
      if (q1 > 15) q1 = 15;
      o[2 + i] = (uint8_t)(q0 | (q1 << 4));
    }
  }
}

/* q4o_quantize_convert: scripts/convert_whisper.py:33-74 (the product
 * quantizer that produced the shipped GGUF files), under numpy 2 (NEP 50)
 * scalar semantics: amax float32, d = amax / 7.0 stays float32 (:52),
 * scale stored np.float16(d) (:55), q = np.round(block / d) half-to-even in
 * float32 (:60) then astype(int8), nibble = (q + 8) & 0x0F (:67-68). */
void q4o_quantize_convert(const float* data, int64_t n, uint8_t* out) {
  int64_t nb = n / Q4_BLOCK;
  for (int64_t b = 0; b < nb; ++b) {
    const float* blk = data + b * Q4_BLOCK;
    float amax = 0.0f;
    for (int i = 0; i < Q4_BLOCK; ++i) {
      float a = fabsf(blk[i]);
      if (a > amax || isnan(a)) amax = a; /* np.max propagates NaN */
    }
    float d = (amax > 0.0f) ? amax / 7.0f : 0.0f; /* :52 */
    uint16_t h = q4o_f32_to_f16(d);              /* :55 */
    uint8_t* o = out + b * Q4_BYTES;
    o[0] = (uint8_t)(h & 0xff);
    o[1] = (uint8_t)(h >> 8);
    int q[Q4_BLOCK];
    for (int i = 0; i < Q4_BLOCK; ++i) {
      if (d > 0.0f) {
        float r = round_half_even(blk[i] / d); /* :60 */
        q[i] = (int)(int8_t)(int)r;            /* astype(np.int8): in range for finite input */
      } else {
        q[i] = 0; /* :62 */
      }
    }
    for (int i = 0; i < 16; ++i) { /* :65-69 */
      int lo = (q[i] + 8) & 0x0f;
      int hi = (q[i + 16] + 8) & 0x0f;
      o[2 + i] = (uint8_t)(lo | (hi << 4));
    }
  }
}

/* ---- dequantize: src/gguf/tests.rs:60-87 == src/gguf/tensor.rs:96-109 ---- */
void q4o_dequantize(const uint8_t* q4, int64_t n, float* out) {
  int64_t nb = n / Q4_BLOCK;
  for (int64_t b = 0; b < nb; ++b) {
    const uint8_t* o = q4 + b * Q4_BYTES;
    float d = q4o_f16_to_f32((uint16_t)(o[0] | (o[1] << 8)));
    float* dst = out + b * Q4_BLOCK;
    for (int i = 0; i < 16; ++i) {
      uint8_t byte = o[2 + i];
      float lo = (float)(byte & 0x0f) - 8.0f;
      float hi = (float)((byte >> 4) & 0x0f) - 8.0f;
      dst[i] = lo * d;
      dst[i + 16] = hi * d;
    }
  }
}

/* ---- naive f32 matmul: src/gguf/tests.rs:172-184 -------------------------
 * out[M,N] = a[M,K] . bt[N,K]^T, i-j-l loops, acc += a*b (no fma). */
void q4o_reference_matmul(const float* a, const float* bt, int64_t m, int64_t k, int64_t n, float* out) {
  for (int64_t i = 0; i < m; ++i)
    for (int64_t j = 0; j < n; ++j) {
      float acc = 0.0f;
      const float* ar = a + i * k;
      const float* br = bt + j * k;
      for (int64_t l = 0; l < k; ++l) acc += ar[l] * br[l];
      out[i * n + j] = acc;
    }
}

/* ---- the WGSL kernel's arithmetic: src/gguf/shader.wgsl:51-92 -----------
 * One output per (b, m, n).  Per block: d = f16->f32 scale (:37-42, :77);
 * for i in 0..16: lo = (f32(byte & 0xF) - 8) * d; hi likewise (:84-85);
 * acc += lo * x[i]; acc += hi * x[i+16] (:86-87).  No fma (WGSL leaves
 * contraction to the implementation; the restatement does not fuse). */
void q4o_shader_matmul(const uint8_t* q4, const float* x, int64_t B, int64_t M, int64_t K, int64_t N,
                       float* out) {
  int64_t bpr = K / 32; /* :69 */
  for (int64_t b = 0; b < B; ++b)
    for (int64_t m = 0; m < M; ++m) {
      const float* xin = x + (b * M + m) * K; /* :68 */
      for (int64_t n = 0; n < N; ++n) {
        float acc = 0.0f;
        for (int64_t blk = 0; blk < bpr; ++blk) {
          const uint8_t* o = q4 + (n * bpr + blk) * Q4_BYTES; /* :73-74 */
          float d = q4o_f16_to_f32((uint16_t)(o[0] | (o[1] << 8)));
          int64_t k0 = blk * 32;
          for (int i = 0; i < 16; ++i) {
            uint8_t byte = o[2 + i];
            float lo = ((float)(byte & 0x0f) - 8.0f) * d;
            float hi = ((float)((byte >> 4) & 0x0f) - 8.0f) * d;
            acc += lo * xin[k0 + i];
            acc += hi * xin[k0 + i + 16];
          }
        }
        out[(b * M + m) * N + n] = acc; /* :91 */
      }
    }
}

/* ---- Q4Linear::forward: src/gguf/linear.rs:34-40 -------------------------
 * y = q4_matmul(x, W) (+ bias broadcast over [B, M]). */
void q4o_linear(const uint8_t* q4, const float* bias, const float* x, int64_t B, int64_t M, int64_t K,
                int64_t N, float* out) {
  q4o_shader_matmul(q4, x, B, M, K, N, out);
  if (bias)
    for (int64_t r = 0; r < B * M; ++r)
      for (int64_t n = 0; n < N; ++n) out[r * N + n] = out[r * N + n] + bias[n];
}

/* ---- gelu: src/model/layers.rs:35-41 (tanh approximation) ---------------
 * x3 = x*x*x; inner = (x + x3*0.044715) * sqrt(2/pi); x*0.5*(tanh(inner)+1). */
float q4o_gelu1(float x) {
  const float s = 0.7978845608028654f; /* (2/PI as f32).sqrt() */
  float x3 = x * x * x;
  float inner = (x + x3 * 0.044715f) * s;
  return x * 0.5f * (tanhf(inner) + 1.0f);
}

void q4o_gelu(float* x, int64_t n) {
  for (int64_t i = 0; i < n; ++i) x[i] = q4o_gelu1(x[i]);
}

/* ---- Q4FFN::forward: src/model/layers.rs:54-58 ----------------------------
 * h = fc1(x) (+b1); h = gelu(h); y = fc2(h) (+b2).  h: caller scratch
 * [B*M*F]. */
void q4o_ffn(const uint8_t* fc1, const float* b1, const uint8_t* fc2, const float* b2, const float* x,
             int64_t B, int64_t M, int64_t D, int64_t F, float* h, float* out) {
  q4o_linear(fc1, b1, x, B, M, D, F, h);
  q4o_gelu(h, B * M * F);
  q4o_linear(fc2, b2, h, B, M, F, D, out);
}

/* ---- the CPU baseline leg: dequantize + naive matmul ---------------------
 * The reference's CPU dequant->GEMM path (tests.rs:60-87 then :172-184),
 * one thread, as bench.py's cpu_baseline times it.  deq: caller scratch
 * [N*K]. */
void q4o_cpu_dequant_gemm(const uint8_t* q4, const float* x, int64_t M, int64_t K, int64_t N, float* deq,
                          float* out) {
  q4o_dequantize(q4, N * K, deq);
  q4o_reference_matmul(x, deq, M, K, N, out);
}

/* ---- the CPU baseline of SURVEY.md §8(d), run (i) and run (ii) -----------
 * Q4Linear::forward on the CPU path the reference has: dequantize
 * (tests.rs:60-87) + naive i-j-l f32 matmul (tests.rs:172-184) + bias
 * (linear.rs:37-39); Q4FFN::forward = fc1 -> gelu -> fc2 (layers.rs:54-58).
 * nthreads = 1 is the reference's single-threaded loop (run (i)); nthreads > 1
 * is this build's OpenMP parallelisation (run (ii)): dequant blocks and the
 * (row, column) outputs of the matmul are shared out statically, each output
 * still summed in the reference's l order, so both runs give the same bits.
 * deq: caller scratch [N*K]; the FFN's h: [M*F]. */
static void cpu_dequant_mt(const uint8_t* q4, int64_t n, float* out, int nthreads) {
  int64_t nb = n / Q4_BLOCK;
#pragma omp parallel for schedule(static) num_threads(nthreads)
  for (int64_t b = 0; b < nb; ++b) q4o_dequantize(q4 + b * Q4_BYTES, Q4_BLOCK, out + b * Q4_BLOCK);
}

static void cpu_matmul_mt(const float* a, const float* bt, int64_t m, int64_t k, int64_t n, float* out,
                          int nthreads) {
#pragma omp parallel for collapse(2) schedule(static) num_threads(nthreads)
  for (int64_t i = 0; i < m; ++i)
    for (int64_t j = 0; j < n; ++j) {
      float acc = 0.0f;
      const float* ar = a + i * k;
      const float* br = bt + j * k;
      for (int64_t l = 0; l < k; ++l) acc += ar[l] * br[l];
      out[i * n + j] = acc;
    }
}

void q4o_cpu_linear(const uint8_t* q4, const float* bias, const float* x, int64_t M, int64_t K, int64_t N,
                    float* deq, float* out, int nthreads) {
  cpu_dequant_mt(q4, N * K, deq, nthreads);
  cpu_matmul_mt(x, deq, M, K, N, out, nthreads);
  if (bias)
    for (int64_t r = 0; r < M; ++r)
      for (int64_t c = 0; c < N; ++c) out[r * N + c] = out[r * N + c] + bias[c];
}

void q4o_cpu_ffn(const uint8_t* fc1, const float* b1, const uint8_t* fc2, const float* b2, const float* x,
                 int64_t M, int64_t D, int64_t F, float* deq, float* h, float* out, int nthreads) {
  q4o_cpu_linear(fc1, b1, x, M, D, F, deq, h, nthreads);
  q4o_gelu(h, M * F);
  q4o_cpu_linear(fc2, b2, h, M, F, D, deq, out, nthreads);
}

/* ---- closed-form inputs of the reference tests (Rust f32 sin/cos) -------
 * kind 0: ((i*0.001).sin()*0.1)          tests.rs:432-434, 493-495, 515-517
 * kind 1: ((i*0.0007).cos()*0.05)        tests.rs:436-438
 * kind 2: ((i*0.1).sin()*0.5)            tests.rs:377
 * kind 3: (i*0.1)                        tests.rs:383, 533
 * kind 4: ((i*0.05-6.4).sin()*0.3)       tests.rs:337-339
 * kind 5: ((i*0.003-3.0).sin()*0.5)      tests.rs:669-671
 * kind 6: ((i*0.001-1.0).sin())          tests.rs:283-285
 * kind 7: ((i*0.001).sin()*0.05)         tests.rs:580-582
 * kind 8: (i*0.01)                       tests.rs:522 (bias)
 * Rust f32::sin/cos call the platform libm sinf/cosf, as here. */
void q4o_closed_form(int kind, int64_t n, float* out) {
  for (int64_t i = 0; i < n; ++i) {
    float fi = (float)i;
    float v;
    switch (kind) {
      case 0: v = sinf(fi * 0.001f) * 0.1f; break;
      case 1: v = cosf(fi * 0.0007f) * 0.05f; break;
      case 2: v = sinf(fi * 0.1f) * 0.5f; break;
      case 3: v = fi * 0.1f; break;
      case 4: v = sinf(fi * 0.05f - 6.4f) * 0.3f; break;
      case 5: v = sinf(fi * 0.003f - 3.0f) * 0.5f; break;
      case 6: v = sinf(fi * 0.001f - 1.0f); break;
      case 7: v = sinf(fi * 0.001f) * 0.05f; break;
      case 8: v = fi * 0.01f; break;
      default: v = 0.0f;
    }
    out[i] = v;
  }
}
