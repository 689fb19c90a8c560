/*
 * wq4.h -- C ABI of the MI355X-native fused Q4_0 dequant + GEMM path.
 *
 * Drop-in boundary for the reference's Q4 operator surface
 * (zerr0o/whisper-burn, src/gguf/{tensor,op,linear}.rs, src/model/layers.rs).
 * Every entry point names the reference item it replaces (file:line).  The
 * reference binds this path in-process through Burn/CubeCL; a Rust maintainer
 * would bind these symbols with `extern "C"`.
 *
 * Conventions
 *  - Plain pointers and sizes only.  `stream` is a hipStream_t passed as
 *    void* (NULL = the device's null stream).  Device pointers (`*_dev`) are
 *    hipMalloc'd memory on the tensor's device.
 *  - Shapes follow the reference: weights [N, K] = [out_features, in_features]
 *    (tensor.rs:29-33), activations [B, M, K] f32 contiguous, outputs
 *    [B, M, N] f32 contiguous (op.rs:41-46, :73).
 *  - Every call returns a wq4_status; on failure wq4_last_error() returns a
 *    thread-local message.  Nothing aborts (the reference panics at
 *    op.rs:53,58-61,106 -- here those are WQ4_ESHAPE / WQ4_EHIP).
 *  - Calls are stream-ordered and asynchronous: no implicit device sync, no
 *    allocation inside the *_ws entry points (graph-capturable).  Distinct
 *    streams may be used concurrently from distinct host threads.
 *  - Result precision: products are formed from f16 hi/lo splits of the f32
 *    activations against the exact f16 value (q - 8) of each nibble,
 *    accumulated in f32 by MFMA; the per-block f16 scale is applied in f32
 *    (see DESIGN.md "Numerics").  The split is of x * s, s a power of two
 *    (2^4 for the internal producers; at these f32 entry points picked per
 *    call from max |x|: s = min(2^4, 2^floor(log2(16384 / max|x|)))), and
 *    the MFMA flushes f16 subnormal inputs, so an element x carries
 *      ~22 significant bits (x = hi + lo)  when |x s| >= 2^-3,
 *      11 bits (hi alone: lo is an f16 subnormal) when 2^-14 <= |x s| < 2^-3,
 *      nothing (flushed to 0)              when |x s| < 2^-14;
 *    i.e. an absolute error floor of 2^-14 / s per element (2^-18 at s = 2^4)
 *    below which the relative precision falls from 2^-22 to 2^-11.  In a dot
 *    product the deficit is weighted by the small elements' share of
 *    sum |x w| (tests/test_q4_gpu.py test_gelu_epilogue_vs_float64 holds an
 *    identity-weight GEMM to exactly these terms).  WQ4_PREC_F16 keeps hi
 *    only: 11 bits for every |x s| >= 2^-14.
 */
#ifndef WQ4_H
#define WQ4_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WQ4_ABI_VERSION 1

typedef enum wq4_status {
  WQ4_OK = 0,
  WQ4_EINVAL = 1,      /* null pointer / bad argument                         */
  WQ4_ESHAPE = 2,      /* shape rule violated (tensor.rs:38-42, op.rs:53-61) */
  WQ4_EBYTES = 3,      /* byte count != N*K/32*18 (tensor.rs:43-48)          */
  WQ4_EHIP = 4,        /* HIP runtime error (launch, memcpy, malloc)         */
  WQ4_ENOMEM = 5,      /* workspace too small / allocation failed            */
  WQ4_EUNSUPPORTED = 6, /* valid request this build does not implement       */
  WQ4_ERANGE = 7        /* an activation left the MFMA operand range (the
                           model runtime's overflow guard, whisper_amd.h)   */
} wq4_status;

/* Activation precision of the product (see header comment).             */
typedef enum wq4_precision {
  WQ4_PREC_F16X2 = 0, /* default: x = hi + lo, two f16 MFMA passes           */
  WQ4_PREC_F16 = 1    /* fast: x rounded to f16, one MFMA pass               */
} wq4_precision;

/* Epilogue flags for the *_ex entry points.                              */
#define WQ4_EPI_GELU 1u     /* tanh-GELU after bias (layers.rs:35-41)       */
#define WQ4_EPI_RESIDUAL 2u /* y = residual + (x W^T + b); residual may == y */

typedef struct wq4_tensor wq4_tensor; /* Q4Tensor (src/gguf/tensor.rs:21-27) */

/* ---- library -------------------------------------------------------- */
const char* wq4_last_error(void);
int wq4_abi_version(void);
wq4_status wq4_device_count(int* count);
/* Process-wide default precision for calls that do not pass one. */
wq4_status wq4_set_precision(wq4_precision prec);
wq4_precision wq4_get_precision(void);

/* ---- Q4Tensor (src/gguf/tensor.rs) ------------------------------------ */
/* Q4Tensor::from_q4_bytes (tensor.rs:35-71).  `raw` = host bytes exactly as
 * stored in GGUF: N*K/32 blocks of 18 B (f16 scale LE, 16 nibble bytes; low
 * nibble = elements 0..15, high = 16..31).  Errors: WQ4_ESHAPE if N*K % 32
 * (tensor.rs:38-42); WQ4_EBYTES if nbytes != N*K/32*18 (tensor.rs:43-48).
 * The bytes are repacked on upload into the MFMA fragment order (lossless;
 * wq4_tensor_raw_bytes returns them again).  Like Q4Tensor, a tensor whose
 * K % 32 != 0 (blocks straddle rows) is accepted and can be dequantized, but
 * every GEMM entry point rejects it with WQ4_ESHAPE (the shader needs whole
 * blocks per row, shader.wgsl:69). */
wq4_status wq4_tensor_create(int device, const uint8_t* raw, size_t nbytes, int64_t n, int64_t k,
                             wq4_tensor** out);
void wq4_tensor_destroy(wq4_tensor* t);
/* Unquantized weights (BASELINE config 5; GGUF F16 linear tensors, which the
 * reference loader rejects, loader.rs:131-134): w = host IEEE halves [N, K]
 * row-major, K % 32 == 0.  The same GEMM entry points then run the MFMA
 * kernels on the f16 weights directly (x = hi + lo against the exact f16 w:
 * two MFMA passes instead of three).  dequantize() returns the f16 values
 * as f32; raw_bytes() the 2*N*K bytes as given. */
wq4_status wq4_tensor_create_f16(int device, const uint16_t* w, int64_t n, int64_t k, wq4_tensor** out);
/* Creation flags of the _ex forms.  By default a tensor with K % 128 == 0
 * and N % 16 == 0 also gets the decode-step (<= 32 rows) kernel's weight
 * layout, a second device copy of the weights; WQ4_TENSOR_NO_DECODE_STEP
 * skips it for tensors that never run at <= 32 rows (encoder weights), and
 * such tensors use the other kernels at every row count. */
#define WQ4_TENSOR_NO_DECODE_STEP 1u
wq4_status wq4_tensor_create_ex(int device, const uint8_t* raw, size_t nbytes, int64_t n, int64_t k, unsigned flags,
                                wq4_tensor** out);
wq4_status wq4_tensor_create_f16_ex(int device, const uint16_t* w, int64_t n, int64_t k, unsigned flags,
                                    wq4_tensor** out);
/* 1 if the tensor holds the decode-step kernel's layout (see above; for f16
 * weights also only when max |w| * 256 stays finite in f16). */
int wq4_tensor_has_decode_step(const wq4_tensor* t);
/* 0 = Q4_0 blocks, 1 = f16 weights. */
int wq4_tensor_weight_type(const wq4_tensor* t);
/* Q4Tensor::shape (tensor.rs:74-76): [N, K]. */
wq4_status wq4_tensor_shape(const wq4_tensor* t, int64_t* n, int64_t* k);
/* Q4Tensor::num_blocks (tensor.rs:79-81). */
int64_t wq4_tensor_num_blocks(const wq4_tensor* t);
int wq4_tensor_device(const wq4_tensor* t);
/* Q4Tensor::dequantize (tensor.rs:88-113): D2H read then host dequant into
 * `host_out` [N*K] f32 (synchronous, diagnostics only, as in the reference). */
wq4_status wq4_tensor_dequantize(const wq4_tensor* t, float* host_out);
/* D2H read of the device copy, un-repacked to the original GGUF bytes
 * [N*K/32*18] (synchronous; proves the repack is lossless). */
wq4_status wq4_tensor_raw_bytes(const wq4_tensor* t, uint8_t* host_out);
/* Bytes of device memory the tensor holds. */
size_t wq4_tensor_device_bytes(const wq4_tensor* t);

/* ---- q4_matmul (src/gguf/op.rs:47-117) ---------------------------------- */
/* y[B,M,N] = x[B,M,K] . W[N,K]^T.  x_dev, y_dev: f32 device buffers on the
 * tensor's device.  K must equal W's K (op.rs:58-61).  Uses an internal,
 * grow-only per-device workspace (allocation happens only on growth). */
wq4_status wq4_matmul(const wq4_tensor* w, const float* x_dev, float* y_dev, int64_t b, int64_t m, int64_t k,
                      void* stream);

/* Q4Linear::forward (src/gguf/linear.rs:34-40): y = x W^T (+ bias[N]).
 * bias_dev may be NULL (cross-attention key has none, loader.rs:205-210). */
wq4_status wq4_linear_forward(const wq4_tensor* w, const float* bias_dev, const float* x_dev, float* y_dev,
                              int64_t b, int64_t m, int64_t k, void* stream);

/* Q4FFN::forward (src/model/layers.rs:54-58): y = fc2(gelu(fc1(x))), with
 * the GELU fused into fc1's epilogue and the intermediate kept in the
 * MFMA operand layout (never materialised as f32). */
wq4_status wq4_ffn_forward(const wq4_tensor* fc1, const float* b1_dev, const wq4_tensor* fc2,
                           const float* b2_dev, const float* x_dev, float* y_dev, int64_t b, int64_t m,
                           void* stream);

/* ---- explicit-workspace / extended forms (graph-capturable) ----------- */
/* Workspace bytes needed by wq4_linear_forward_ws for these sizes. */
size_t wq4_linear_workspace_bytes(const wq4_tensor* w, int64_t rows);
/* Workspace bytes needed by wq4_ffn_forward_ws. */
size_t wq4_ffn_workspace_bytes(const wq4_tensor* fc1, const wq4_tensor* fc2, int64_t rows);
/* y = epi(x W^T + bias); flags = WQ4_EPI_*; residual_dev used iff
 * WQ4_EPI_RESIDUAL (may alias y_dev).  rows = B*M.  No allocation. */
wq4_status wq4_linear_forward_ws(const wq4_tensor* w, const float* bias_dev, const float* x_dev,
                                 const float* residual_dev, float* y_dev, int64_t rows, int64_t k,
                                 unsigned flags, wq4_precision prec, void* workspace, size_t ws_bytes,
                                 void* stream);
wq4_status wq4_ffn_forward_ws(const wq4_tensor* fc1, const float* b1_dev, const wq4_tensor* fc2,
                              const float* b2_dev, const float* x_dev, const float* residual_dev, float* y_dev,
                              int64_t rows, unsigned flags, wq4_precision prec, void* workspace,
                              size_t ws_bytes, void* stream);

/* ---- operand-layout entry points (producers that emit A-tiled) -------- */
/* Bytes of an A-tiled operand buffer for `rows` x `k` activations.       */
size_t wq4_atiled_bytes(int64_t rows, int64_t k, wq4_precision prec);
/* f32 [rows, k] (row stride ld floats) -> A-tiled operand (f16 hi[/lo]).  */
wq4_status wq4_tile_activations(const float* x_dev, int64_t rows, int64_t k, int64_t ld, wq4_precision prec,
                                void* at_dev, size_t at_bytes, void* stream);
/* y = epi(A W^T + bias) from an A-tiled operand (no conversion pass).     */
wq4_status wq4_linear_forward_tiled(const wq4_tensor* w, const float* bias_dev, const void* at_dev,
                                    const float* residual_dev, float* y_dev, int64_t rows, unsigned flags,
                                    wq4_precision prec, void* stream);
/* Same, writing the result as the A-tiled operand of a following GEMM whose
 * K equals this N (used for fc1 -> fc2; bias/GELU applied first).          */
wq4_status wq4_linear_forward_tiled_out(const wq4_tensor* w, const float* bias_dev, const void* at_dev,
                                        void* at_out_dev, size_t at_out_bytes, int64_t rows, unsigned flags,
                                        wq4_precision prec, void* stream);

/* Extended operand-layout GEMM used by the model runtime: explicit kernel
 * (0 = automatic by rows, 1 = MFMA tile "prefill", 2 = K-split "decode",
 * 3 = the decode-step kernel: rows <= 32, K % 128 == 0, N % 16 == 0),
 * output f32 row-major y_dev, or, with WQ4_EPI_TILED_OUT, the A-tiled
 * operand at_out_dev of a following GEMM (K' = N; N % 32 == 0).           */
#define WQ4_EPI_TILED_OUT 4u
/* wq4_gemm_ln_tiled only: LayerNorm inside the decode GEMM (see there). */
#define WQ4_EPI_LN_FUSED 8u
wq4_status wq4_gemm_tiled(const wq4_tensor* w, const float* bias_dev, const void* at_dev, const float* residual_dev,
                          float* y_dev, void* at_out_dev, int64_t rows, unsigned flags, wq4_precision prec,
                          int kernel, void* stream);

/* LayerNorm (layers.rs:12-32) of x rows [rows, K] f32 followed by the GEMM
 * of wq4_gemm_tiled (same flags / outputs) -- the attn_ln / mlp_ln ->
 * Q4Linear pairs of encoder.rs:37-49 and decoder.rs:77-112.  By default
 * wq4_layernorm writes at_scratch_dev (wq4_atiled_bytes(rows, K, prec)) and
 * the GEMM reads it.  With WQ4_EPI_LN_FUSED in flags and a decode-sized row
 * count the LayerNorm runs inside the GEMM instead (the A operand built from
 * x in registers, bit-identical to the two-step path; slower on MI355X for
 * the Whisper shapes, where every n-tile repeats the row statistics). */
wq4_status wq4_gemm_ln_tiled(const wq4_tensor* w, const float* bias_dev, const float* x_dev, const float* ln_w_dev,
                             const float* ln_b_dev, void* at_scratch_dev, const float* residual_dev, float* y_dev,
                             void* at_out_dev, int64_t rows, unsigned flags, wq4_precision prec, int kernel,
                             void* stream);

/* LayerNorm folded into the decoder GEMMs around it (rows <= 32: the
 * 8-wave decode kernel where its 8-wave plan applies, else -- or under
 * kernel policy 3 -- the decode-step kernel; replaces the wq4_layernorm launch between a
 * residual GEMM and the GEMM that reads LayerNorm of its output -- the
 * attn_ln / cross_attn_ln / mlp_ln -> Q4Linear pairs of decoder.rs:77-112).
 * LN(x) = (x - mean) / sqrt(var + 1e-5) * gamma + beta (layers.rs:12-32), so
 *   W LN(x) + bias = (W (x * gamma) - mean * (W gamma)) / sqrt(var + 1e-5)
 *                    + (W beta + bias).
 * Producer (set gamma_dev, at_out_dev, stats_out_dev): a residual GEMM
 * (WQ4_EPI_RESIDUAL, f32 output x) also writes the A-tiled operand of
 * x * gamma (wq4_atiled_bytes(rows, N, prec)) and, per (row, 16-column
 * tile), the tile mean and sum of squared deviations (stats_out_dev,
 * rows * N/16 * 2 floats).  Consumer (set stats_in_dev, wg_dev): at_dev is
 * that operand; the row statistics are merged (the exact equal-count
 * merge of 16-value tiles, a fixed order: every workgroup gets the same
 * bits) and the correction applied before bias / GELU / tiled output; bias_dev is
 * W beta + bias and wg_dev W gamma (wq4_ln_fold_vectors).  A launch may be
 * both.  Not bit-identical to wq4_layernorm -> wq4_gemm_tiled (re-associated
 * sums; tolerance in tests/test_q4_gpu.py). */
typedef struct wq4_ln_fold {
  const float* gamma_dev;     /* producer: gamma of the LayerNorm that follows */
  void* at_out_dev;           /* producer: A-tiled x * gamma */
  float* stats_out_dev;       /* producer: [rows][N/16][2] */
  const float* stats_in_dev;  /* consumer: the producer's statistics (K/16 tiles) */
  const float* wg_dev;        /* consumer: W gamma [N] */
} wq4_ln_fold;
wq4_status wq4_gemm_tiled_lnfold(const wq4_tensor* w, const float* bias_dev, const void* at_dev,
                                 const float* residual_dev, float* y_dev, void* at_out_dev, int64_t rows,
                                 unsigned flags, wq4_precision prec, const wq4_ln_fold* fold, void* stream);
/* Host: wg = W gamma and bias_out = W beta + bias (bias may be NULL) for a
 * consumer of wq4_gemm_tiled_lnfold, accumulated in double from the
 * dequantized weights.  gamma / beta: K floats; outputs N floats. */
wq4_status wq4_ln_fold_vectors(const wq4_tensor* w, const float* gamma, const float* beta, const float* bias,
                               float* wg_out, float* bias_out);
/* Whether wq4_gemm_tiled_lnfold supports w at this row count (a consumer
 * also needs K <= 1280). */
int wq4_lnfold_supported(const wq4_tensor* w, int64_t rows);

/* Allocate (once) the per-(device, stream) split-K workspace that small-M
 * GEMMs on `stream` use.  The first small-M GEMM on a stream does this
 * itself, which is not allowed inside a graph capture: call this first when
 * capturing such GEMMs into a hipGraph. */
wq4_status wq4_prepare_stream(int device, void* stream);

/* LayerNorm (src/model/layers.rs:12-32: eps 1e-5, biased variance) of
 * rows x d f32 rows, written either as the A-tiled operand of a following
 * GEMM with K = d (at_out_dev, wq4_atiled_bytes(rows, d, prec) bytes) or as
 * f32 rows (y_dev); exactly one of the two is non-NULL.  d % 4 == 0,
 * d <= 2048. */
wq4_status wq4_layernorm(const float* x_dev, const float* w_dev, const float* b_dev, int64_t rows, int64_t d,
                         wq4_precision prec, void* at_out_dev, float* y_dev, void* stream);

/* Fused K|V projection written head-major for attention: w is [parts * d, K]
 * (parts stacked projections of d = heads * 64 columns each), rows =
 * groups * group_rows; y_dev[part][group][head][t][64] (the [B, H, T, 64]
 * view of the cross-attention k / v after reshape + swap_dims(1, 2),
 * zerr0o/whisper-burn src/model/attention.rs:177-206, 254-263).
 * d % 64 == 0.                                                          */
wq4_status wq4_gemm_tiled_headmajor(const wq4_tensor* w, const float* bias_dev, const void* at_dev, float* y_dev,
                                    int64_t rows, int group_rows, int d, wq4_precision prec, int kernel,
                                    void* stream);

/* ---- conversion (scripts/convert_whisper.py:33-74) -------------------- */
/* Q4_0-quantize n f32 values (n % 32 == 0) exactly as the reference's
 * converter does under numpy 2: d = amax/7 (f32), f16 scale, round-half-even
 * of v/d, nibble = (q + 8) & 0xF, low nibble = elements 0..15.             */
wq4_status wq4_quantize_q4_0(const float* x, int64_t n, uint8_t* out);

/* ---- kernel selection (exposed for tests and the bench) -------------- */
/* 0 = automatic (by rows), 1 = force the MFMA tile kernel ("prefill"),
 * 2 = force the K-split streaming kernel ("decode"), 3 = force the
 * decode-step kernel (rows <= 32).  Each computes every output row with an
 * M-independent instruction sequence. */
wq4_status wq4_set_kernel_policy(int policy);
/* Name of the kernel a Q4_0 GEMM of `rows` rows over [n, k] weights runs
 * under the current policy and encoder-kernel mode ("skinny_gemm_kernel",
 * "q4_gemm_decode_kernel", "q4_gemm_enc_kernel", "q4_gemm_prefill_kernel";
 * "" for a shape no GEMM accepts).  Host only (bench.py's roofline label). */
const char* wq4_gemm_kernel_name(int64_t n, int64_t k, int64_t rows);

/* ---- host-only diagnostics (no GPU needed) ---------------------------- */
/* Sizes of the repacked nibble / scale / column-scale arrays for [N, K]. */
wq4_status wq4_debug_repacked_bytes(int64_t n, int64_t k, size_t* nib_bytes, size_t* sc_bytes, size_t* cs_bytes);
/* The repack wq4_tensor_create applies on upload, run on the host. */
wq4_status wq4_debug_repack(const uint8_t* raw, int64_t n, int64_t k, uint8_t* nib_out, uint32_t* sc_out,
                            float* colscale_out);
/* Its inverse (raw GGUF bytes from the repacked arrays). */
wq4_status wq4_debug_unrepack(const uint8_t* nib, const uint32_t* sc, const float* colscale, int64_t n, int64_t k,
                              uint8_t* raw_out);

/* Diagnostics: which kernel runs the encoder-size (rows > 128) Q4_0 GEMMs.
 * 0 = the prefill tile kernel, 1 = by rows (default; WQ4_ENC_KERNEL
 * overrides at load): the LDS-DMA ring kernel's 64 x 128 geometry while the
 * tile kernel's grid would leave CUs idle (one clip), else the tile kernel;
 * 2 = the ring kernel's 256 x 256 geometry, 3 = its 64 x 128 geometry,
 * 4 = its 32 x 256 geometry.  All give bit-identical results.
 * Returns the previous mode, -1 on a bad argument. */
int wq4_debug_set_enc_kernel(int mode);

#ifdef __cplusplus
}
#endif
#endif /* WQ4_H */
