// wa_kernels.hpp -- launchers of the Whisper model kernels around the Q4 path
// (LayerNorm, attention, conv front-end, embedding, logits, greedy argmax).
// Reference semantics: src/model/{layers,attention,encoder,decoder,whisper}.rs.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace wa {

// Device-resident decode state (read by kernels, advanced on the device so a
// captured step graph can be replayed without host involvement).
struct DecodeState {
  int position;  // positional-embedding index of the current token
  int kv_len;    // entries in the self-attention KV cache before this step
  int step;      // greedy-loop step index (whisper.rs:104)
  int n_done;    // clips that have emitted EOT
};

// Encoder self-attention (attention.rs:243-298, non-causal), flash-style,
// f32 MFMA.  qkv: [B*T, 3D] f32 (q | k | v).  Writes the A-tiled operand of
// the output projection (rows b*T + t, K = D) -- or, with out32 non-null
// (range tier 3, wa_model), f32 rows [B*T][D] there instead.  The same holds
// for every attention launcher below.
hipError_t launch_encoder_attention(const float* qkv, int B, int T, int H, _Float16* tiled, int ns,
                                    hipStream_t st, float* out32 = nullptr);

// Decoder self-attention with KV cache (attention.rs:62-125).  qkv [B*Tq, 3D];
// appends k, v of the Tq new tokens at cache index kv_len (+ kv_base_extra)
// and attends over kv_len + Tq entries, causal inside the new tokens when
// Tq > 1 (attention.rs:270-287).  cache_k/v: [B, ctx, D].
hipError_t launch_decoder_self_attention(const float* qkv, float* cache_k, float* cache_v, int B, int Tq, int H,
                                         int ctx, const DecodeState* state, int kv_len_host, _Float16* tiled,
                                         int ns, hipStream_t st, float* out32 = nullptr);

// Cross-attention over cached K / V (attention.rs:177-236, the reference's
// form; used for decode groups of a few clips): q [B*Tq, D] f32, k / v
// head-major [B][H][T][64] f32 (wq4_gemm_tiled_headmajor of the encoder
// output), Tq <= 4; part: cross_attention_kv_part_floats floats, counters:
// B * H ints zeroed once (re-armed by the kernel).  Writes the A-tiled
// operand of the output projection.
int cross_attention_kv_splits(int T);
size_t cross_attention_kv_part_floats(int B, int H, int T);
hipError_t launch_cross_attention_kv(const float* q, const float* k, const float* v, int B, int Tq, int T, int H,
                                     float* part, int* counters, _Float16* tiled, int ns, hipStream_t st,
                                     float* out32 = nullptr);

// Cross-attention over the encoder output (wa_xattn.hip; attention.rs:
// 204-298 restated without K/V caches): q [B*Tq, D] f32 (rows b*Tq + i),
// wk / wv: the layer's raw key / value weights [D, D] (wtype: Q4_0 blocks or
// f16), bv: value bias, enc: [B][T][ns][D] f16 planes (launch_enc_planes),
// qt: [B*Tq][ns][ceil16(H)][D] f16 scratch zeroed once, part:
// xattn_part_floats floats.  Writes the A-tiled operand of the output
// projection.  Needs D == 64 * H, D % 128 == 0, D <= 1280.
struct XattnPlan {
  int splits;  // frame ranges per query row (workgroups per row)
  int ch;      // 16-frame sub-chunks per range
};
XattnPlan xattn_plan(int R, int T);
size_t xattn_part_floats(int R, int H, int D, int T);
// Q4_0 Wv repacked once at model load into the cross-attention
// projection's lane order (same bytes; wv_pack_words u32 words).
size_t wv_pack_words(int H, int D);
hipError_t launch_wv_pack(const uint8_t* wv, int H, int D, uint32_t* out, hipStream_t st);
// wvp: the launch_wv_pack words of wv (Q4 weights; ignored for f16 weights).
hipError_t launch_xattn(const float* q, const uint8_t* wk, const uint8_t* wv, const uint32_t* wvp, const float* bv,
                        int wtype, const _Float16* enc, int B, int Tq, int T, int H, int D, _Float16* qt, float* part,
                        _Float16* tiled, int ns, hipStream_t st, float* out32 = nullptr);
// A-tiled operand [R][K] (hi + lo) -> f32 rows (diagnostics).
hipError_t launch_untile(const _Float16* tiled, int R, int K, int ns, float* out, hipStream_t st);
// f32 rows [rows][D] -> [rows][ns][D] f16 planes (hi | lo) for launch_xattn.
hipError_t launch_enc_planes(const float* x, int64_t rows, int D, int ns, _Float16* out, hipStream_t st);

// Conv1D (layers.rs:77-132) as an implicit-im2col f32 MFMA GEMM + bias +
// GELU (encoder.rs:89-94) (+ pos[t] if pos != nullptr).  Input element
// (b, c, t) at in[b*in_bs + c*in_cs + t*in_ts]; output [B, T_out, N].
// w_t: weights re-laid as [N][3*C] with k = kk*C + c.
hipError_t launch_conv_gelu(const float* in, long in_bs, long in_cs, long in_ts, int B, int C, int T_in,
                            int stride, const float* w_t, const float* bias, const float* pos, int N, float* out,
                            hipStream_t st);

// x[b*Tq + t] = tok_emb[tokens[b*Tq + t]] + pos_emb[pos0 + t]   (decoder.rs:326-343)
// pos0 = state ? state->position : pos0_host.
hipError_t launch_embed(const int* tokens, const float* tok_emb, const float* pos_emb, int B, int Tq, int D,
                        const DecodeState* state, int pos0_host, float* x, hipStream_t st);

// launch_embed + the LayerNorm-fold producer for gamma (wq4_gemm_tiled_lnfold):
// also writes at = A-tiled x * gamma and stats [rows][D/32][2]; D % 32 == 0.
hipError_t launch_embed_fold(const int* tokens, const float* tok_emb, const float* pos_emb, int B, int Tq, int D,
                             const DecodeState* state, int pos0_host, float* x, const float* gamma, _Float16* at,
                             float* stats, int ns, hipStream_t st);

// logits[b, v] = h[b * ldh] . E[v]  (decoder.rs:289-292, 342-343), f32
// products and accumulation (v_mfma_f32_32x32x2_f32).
hipError_t launch_logits(const float* h, int B, int D, long ldh, const float* emb, int V, float* logits,
                         hipStream_t st);

// Greedy pick per clip (whisper.rs:119-124, 131-138): argmax with the LAST
// maximum winning ties (Rust max_by), EOT (50257) masked when suppress != 0,
// or restricted to [lo, hi) for language detection (whisper.rs:76-83).
// Writes out_tok[b * out_stride].
// range_flag (nullable): set to 1 when a logit of [lo, hi) is not finite --
// an MFMA operand left the f16-pair range somewhere upstream (the
// overflow propagates to every logit of the clip); wa_transcribe checks it.
hipError_t launch_argmax(const float* logits, int B, int V, int lo, int hi, int suppress_eot,
                         const DecodeState* state, int* out_tok, int out_stride, int* range_flag, hipStream_t st);

// Decode-step logits fused with the greedy pick (launch_logits +
// launch_argmax_step in one kernel, logits never stored): B <= 32 rows,
// D % 8 == 0; pval / pidx: 32 * logits_argmax_groups(V) scratch each,
// counter: one int zeroed once (re-armed by the kernel).
int logits_argmax_groups(int V);
// htiled: the B hidden rows as the A-tiled operand (wq4 layout, m-tile 0,
// ns planes -- what wq4_layernorm writes with at_out); emb2: the f16-pair
// table, fragment-tiled (launch_emb_tiled); D % 128 == 0.
// trace_ids / trace_out (diagnostics; null in the product): [B][trace_s1]
// [trace_k] -- the logits of the listed ids at slot state->step + 1.
// range_flag (nullable): as launch_argmax, for every logit of the B rows.
hipError_t launch_logits_argmax(const _Float16* htiled, int B, int D, const _Float16* emb2, int ns, int V,
                                int min_tokens, const DecodeState* state, float* pval, int* pidx, int* counter,
                                int* out_tok, const int* trace_ids, float* trace_out, int trace_s1, int trace_k,
                                int* range_flag, hipStream_t st);
// Whether the logits kernel reads a fragment-tiled table for this width.
bool emb_tiled_supported(int D);
// Rows of the fragment-tiled table (V padded to the kernel's 128-row groups).
int64_t emb_tiled_rows(int V);
// f32 [V][D] -> fragment-tiled f16 planes, chunk-major: per 128-column
// chunk c, 16-row group g (G = emb_tiled_rows(V) / 16 of them), 32-column
// step ks < 4 and plane p, the 16x16x32 MFMA operand of 64 lanes x 8 halves
// is 1 KiB contiguous at (((c * G + g) * 4 + ks) * ns + p) KiB (lane =
// 16 (k / 8 % 4) + row % 16), rows >= V zero -- every load instruction of
// the logits kernel reads 1 KiB contiguous and one chunk of the whole table
// is one contiguous stretch.  out: emb_tiled_rows(V) * ns * D halves.
hipError_t launch_emb_tiled(const float* emb, int V, int D, int ns, _Float16* out, hipStream_t st);

// Greedy-loop bookkeeping at the top of each step (whisper.rs:104-115):
// for every clip not yet done, EOT -> done (eot_stop != 0), else append the
// next token; then advance position / kv_len / step.
hipError_t launch_bookkeep(const int* next_tok, int* tokens, int* n_tokens, int* done, int B, int max_tokens,
                           int eot_stop, DecodeState* state, hipStream_t st);

// Step-dependent EOT suppression (whisper.rs:120-122) folded into argmax:
// suppress iff state->step < min_tokens - 1 (state->step already advanced).
hipError_t launch_argmax_step(const float* logits, int B, int V, int min_tokens, const DecodeState* state,
                              int* out_tok, int* range_flag, hipStream_t st);

}  // namespace wa
