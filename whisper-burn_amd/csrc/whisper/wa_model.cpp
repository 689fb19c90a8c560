// wa_model.cpp -- Whisper model runtime around the Q4 path (host side).
//
// Re-builds, MI355X-first, the module graph that calls the Q4 operator in the
// reference (zerr0o/whisper-burn):
//   WhisperEncoder::forward        src/model/encoder.rs:87-115
//   EncoderBlock::forward          src/model/encoder.rs:37-49
//   DecoderBlock::forward_*        src/model/decoder.rs:77-283
//   WhisperDecoder::forward_prompt src/model/decoder.rs:251-296
//   WhisperDecoder::decode_step    src/model/decoder.rs:306-348
//   WhisperModel::transcribe       src/model/whisper.rs:51-128
// Design points: clips are batched through every kernel; q/k/v
// (and cross k/v) projections run as ONE Q4 GEMM over row-concatenated Q4
// weights (bitwise identical per output to separate GEMMs); bias, GELU and
// the residual add are fused into the Q4 GEMM epilogues; LayerNorm and the
// attention kernels write the Q4 GEMM operand (A-tiled f16 hi/lo) directly;
// the KV caches are preallocated (no Tensor::cat); the greedy loop keeps
// tokens, positions and the done flags on the device and each decode step is
// one replayed hipGraph.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/whisper_amd.h"
#include "../../../include/wq4.h"
#include "wa_gguf.hpp"
#include "wa_kernels.hpp"
#include "wa_mel.hpp"

namespace {

thread_local std::string g_err;

wq4_status fail(wq4_status s, const std::string& m) {
  g_err = m;
  return s;
}

#define WA_HIP(expr)                                                                            \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess) return fail(WQ4_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)
#define WA_WQ4(expr)                                                                \
  do {                                                                              \
    wq4_status s_ = (expr);                                                         \
    if (s_ != WQ4_OK) return fail(s_, std::string(#expr) + ": " + wq4_last_error()); \
  } while (0)

constexpr int kSOT = 50258;
constexpr int kMaxTokens = 224;  // whisper.rs:20
constexpr int kMinTokens = 3;    // whisper.rs:97
// Pipelined transcribes (transcribe_pipelined): CUs of the encoder stream
// that runs beside a decode, the encoder layers it covers in the first
// overlapped batch, and the share of the last decode's length its part is
// sized to afterwards (WA_ENC_CUS / WA_ENC_OVERLAP / WA_ENC_FILL override).
// Fill measured at 32 clips (scripts/r05ad.sh): RTF 959 at 0.92, 966 at 0.98
// / 1.0 / 1.02, 948 at 1.04 (the masked part then outlasts the decode);
// 0.98 keeps ~30 ms of slack.
constexpr int kEncOverlapCUs = 32;
constexpr int kEncOverlapLayers0 = 16;
constexpr double kEncOverlapFill = 0.98;

struct Config {  // WhisperConfig, src/model/config.rs:5-30
  int n_mels, n_audio_ctx, n_audio_state, n_audio_head, n_audio_layer;
  int n_text_ctx, n_text_state, n_text_head, n_text_layer, n_vocab, n_lang;
  int transcribe_token() const { return 50260 + n_lang; }      // config.rs:66-69
  int no_timestamps_token() const { return transcribe_token() + 4; }  // config.rs:72-74
};

Config preset(int variant) {
  switch (variant) {
    case WA_LARGE_V3:  // config.rs:32-47; vocab = rows of the HF/GGUF embedding
      return {128, 1500, 1280, 20, 32, 448, 1280, 20, 32, 51866, 100};
    case WA_MEDIUM:  // config.rs:49-63
      return {80, 1500, 1024, 16, 24, 448, 1024, 16, 24, 51865, 99};
    default:  // parity-test configuration (not a released model)
      return {80, 1500, 384, 6, 2, 448, 384, 6, 2, 51866, 100};
  }
}

// ----------------------------------------------- synthetic weights --
uint64_t fnv1a64(const char* s) {
  uint64_t h = 0xCBF29CE484222325ull;
  for (; *s; ++s) {
    h ^= (uint8_t)*s;
    h *= 0x100000001B3ull;
  }
  return h;
}

inline uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

template <class F>
void parallel_for(int64_t n, F fn) {
  unsigned nt = std::max(1u, std::min(32u, std::thread::hardware_concurrency()));
  if (n < (1 << 16)) nt = 1;
  std::vector<std::thread> th;
  const int64_t chunk = (n + nt - 1) / nt;
  for (unsigned t = 0; t < nt; ++t) {
    const int64_t a = t * chunk, b = std::min(n, a + chunk);
    if (a >= b) break;
    th.emplace_back([=] { fn(a, b); });
  }
  for (auto& x : th) x.join();
}

// oracle/oracle.py:synth_uniform -- bit-identical (compiled -ffp-contract=off).
void synth_uniform(uint64_t seed, const std::string& name, int64_t n, float lo, float hi, float* out) {
  const uint64_t key = seed ^ fnv1a64(name.c_str());
  const float span = (float)((double)hi - (double)lo);
  parallel_for(n, [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) {
      const float u = (float)(splitmix64(key + (uint64_t)i) >> 40);
      const float unit = u * (float)(1.0 / 16777216.0);
      const float t = unit * span;
      out[i] = lo + t;
    }
  });
}

float lin_scale(int k) { return (float)(1.5 / std::sqrt((double)k)); }

struct Dev {
  std::vector<void*> ptrs;
  ~Dev() {
    for (void* p : ptrs) (void)hipFree(p);
  }
  template <class T>
  T* alloc(size_t n) {
    void* p = nullptr;
    if (hipMalloc(&p, n * sizeof(T) + 256) != hipSuccess) return nullptr;
    ptrs.push_back(p);
    return static_cast<T*>(p);
  }
  // frees one pointer alloc() returned (null: no-op)
  void release(void* p) {
    if (!p) return;
    for (void*& q : ptrs)
      if (q == p) {
        (void)hipFree(q);
        q = ptrs.back();
        ptrs.pop_back();
        return;
      }
  }
};

struct EncLayer {
  float *ln1_w, *ln1_b, *ln2_w, *ln2_b, *qkv_b, *out_b, *fc1_b, *fc2_b;
  wq4_tensor *qkv = nullptr, *out = nullptr, *fc1 = nullptr, *fc2 = nullptr;
};
struct DecLayer {
  float *ln1_w, *ln1_b, *ln2_w, *ln2_b, *ln3_w, *ln3_b;
  float *qkv_b, *out_b, *cq_b, *cv_b, *cout_b, *fc1_b, *fc2_b;
  wq4_tensor *qkv = nullptr, *out = nullptr, *cq = nullptr, *cout = nullptr, *fc1 = nullptr, *fc2 = nullptr;
  // LayerNorm fold (wq4_gemm_tiled_lnfold) of the GEMMs that read a
  // LayerNorm: W gamma and W beta + bias of qkv (attn_ln), cq
  // (cross_attn_ln), fc1 (mlp_ln)
  float *qkv_wg = nullptr, *qkv_b2 = nullptr, *cq_wg = nullptr, *cq_b2 = nullptr, *fc1_wg = nullptr,
        *fc1_b2 = nullptr;
  // cross-attention key / value weights in raw GGUF form (Q4_0 blocks or
  // f16), read by the K/V-cache-free cross-attention (wa_xattn.hip)
  uint8_t *ck_raw = nullptr, *cv_raw = nullptr;
  uint32_t* cv_p = nullptr;  // Q4_0: cv_raw in the projection's lane order (wa::launch_wv_pack)
  float *cache_k, *cache_v;
  // few-clip decode groups (wa_model::kv_clips): the reference's per-layer
  // cross K / V caches, head-major [clip][head][T][64] f32, written by the
  // head-major GEMMs of ck / cv over the encoder output (cross_kv_forward)
  wq4_tensor *ck = nullptr, *cv = nullptr;
  float *xk = nullptr, *xv = nullptr;
};

// One decode group: a contiguous range of clips [b0, b0 + nb) decoded on its
// own stream with its own activations, DecodeState and step graph.  The
// decode step is a chain of ~350 small dependent kernels (latency-bound);
// groups on separate streams overlap one another's launch gaps and let the
// HBM-bound cross-attention of one group run beside the latency-bound GEMMs
// of another.  Per-clip results do not depend on the grouping (every
// kernel's per-row arithmetic is independent of the batch).
constexpr int kMaxGroups = 4;
struct DecGroup {
  hipStream_t st = nullptr;
  int b0 = 0, nb = 0;
  float *xd, *qkvd, *qd, *hid, *logits;
  _Float16 *atd_dec, *atf_dec;
  int *prompt_tok, *next_tok, *tokens, *ntok, *done;
  _Float16* xqt;    // cross-attention Wk^T q operands [rows][ns][16*ceil(H/16)][D]
  float* xattn_part;  // cross-attention split partials (Z, max, sum)
  float* xkv_part;    // cross-attention over cached K / V: split partials
  int* xkv_ctr;       //   and the per-(clip, head) arrival counters
  _Float16* atd_ln;   // LayerNorm fold: A-tiled x * gamma of the next LayerNorm
  float* ln_stats;    //                 its per (row, 32-column tile) mean / M2
  _Float16* hid_t;    // fused logits + argmax: the final LN, A-tiled (m-tile 0)
  float* lg_val;      //                        per-workgroup candidates [32][groups]
  int *lg_idx, *lg_ctr;
  wa::DecodeState* state;
  void* ffn_ws = nullptr;  // wide_ffn: wq4_ffn_forward_ws workspace (4 * nb rows)
  size_t ffn_ws_bytes = 0;
  int* host_ndone = nullptr;  // pinned ring
  hipGraphExec_t graph = nullptr;
  int64_t graph_key = -1;  // (b0, nb, eot mode, trace) the graph was captured for
};

}  // namespace


struct wa_model {
  int device = 0;
  Config cfg{};
  wq4_precision prec = WQ4_PREC_F16X2;
  int ns = 2;
  int bmax = 1;
  Dev dev;
  size_t bytes = 0;
  // globals
  float *conv1_wt, *conv1_b, *conv2_wt, *conv2_b, *enc_pos, *lnp_w, *lnp_b;
  float *tok_emb, *dec_pos, *dln_w, *dln_b;
  _Float16* tok_emb2 = nullptr;  // tied embedding as fragment-tiled f16 pairs (wa::launch_emb_tiled)
  std::vector<EncLayer> enc;
  std::vector<DecLayer> dec;
  // encoder activations
  float *h1, *x, *qkv;
  _Float16 *at_d, *at_f;
  // encoder output as f16 planes [clip][T][ns][D], the cross-attention's
  // only per-clip state (no per-layer K/V caches)
  _Float16* enc_planes = nullptr;
  const float* enc_f32 = nullptr;  // ln_post output of the last encoder pass
  // decode groups: the clips of a transcribe split over up to kMaxGroups
  // independent streams, each replaying its own step graph (see DecGroup)
  std::vector<DecGroup> groups;
  int wtype = 0;     // linear weights: 0 Q4_0, 1 f16 (BASELINE config 5)
  int kv_batch = 0;  // clips of the last encoder pass (enc_planes valid for [0, kv_batch))
  // Cross K / V caches (capacity kv_clips clips) for transcribes of at most
  // kv_small clips -- their decode steps are launch-latency chains: one GEMV
  // launch over the caches replaces the cache-free cross-attention's four,
  // wa_kernels.hip.  kv_n: clips [0, kv_n) of the last encoder pass have
  // caches; a decode group entirely inside them reads the caches.
  int kv_clips = 0, kv_small = 0;
  int kv_n = 0;
  bool kv_alloc_ok = false;  // every layer's xk / xv allocated (cross_kv_forward)
  bool group_kv(const DecGroup& g) const { return g.nb > 0 && g.b0 + g.nb <= kv_n; }
  hipStream_t own_stream = nullptr;  // encoder / encoder planes (graph capture needs a non-null stream)
  // pipelined transcribes (wa_transcribe_batches): the CU-masked stream of
  // the encoder part that runs beside a decode, its CU count, the encoder
  // layers that part covers (adapted per batch) and the last call's stats
  hipStream_t enc_stream = nullptr;
  int enc_cus = 0;
  int overlap_k = -1;
  int overlap_b = 0, overlap_eot = -1;  // the batch shape overlap_k was adapted to
  float pipe[4] = {0, 0, 0, 0};
  // Activation-range guard.  Every internal producer writes MFMA operands as
  // f16 pairs of x * 2^4 (wq4_device.hpp split_act), finite for |x| < 4094;
  // beyond that the f16 half overflows and the clip's logits become inf /
  // NaN.  The pick kernels set *range_flag on any non-finite logit.  After a
  // flagged transcribe the model retries it once with the LayerNorm fold off
  // (wide_range: the fold feeds the RAW residual stream x * gamma to the MFMAs,
  // where the LayerNorm path feeds LayerNorm(x), bounded by sqrt(D) |gamma| +
  // |beta|); still flagged -> WQ4_ERANGE, never NaN tokens.
  int* range_flag = nullptr;
  bool wide_range = false;
  // second tier (wide_range still flagged): the encoder and decoder FFNs run
  // as Q4FFN::forward at the ABI (wq4_ffn_forward_ws: LayerNorm output in
  // f32, fc1 + GELU to f32, each GEMM operand scaled by a power of two picked
  // per call from its max |x|), so fc1 / GELU outputs of any f32-finite size
  // reach fc2 finite.  Workspaces allocated when the tier is entered:
  // ffn_ws for the encoder's B * T rows, g.ffn_ws per decode group.
  bool wide_ffn = false;
  // third tier (wide_ffn still flagged): every attention output (encoder
  // self-attention, decoder self- and cross-attention) is written as f32
  // rows instead of the f16-pair operand, and the output projections run as
  // Q4Linear::forward at the ABI (wq4_linear_forward_ws: per-call operand
  // scale).  Scratch: m->h1 (free during the encoder layers) / g.hid, with
  // the layer's own A-tiled buffer as the ABI workspace.
  bool wide_attn = false;
  int range_tier() const { return wide_attn ? 3 : wide_ffn ? 2 : wide_range ? 1 : 0; }
  void* ffn_ws = nullptr;
  size_t ffn_ws_bytes = 0;
  float timings[5] = {0, 0, 0, 0, 0};
  // decode-step logit trace (wa_transcribe_trace; null otherwise): device
  // [clip][trace_s1][trace_k] ids and their logits
  const int* trace_ids = nullptr;
  float* trace_out = nullptr;
  int trace_s1 = 0, trace_k = 0;
  // live kernel timing (wa_profile_*)
  struct Pending {
    hipEvent_t a, b;
    int cat;
    double gflop, gb;
  };
  bool profile = false;
  std::vector<Pending> pending;
  double prof[WA_PROF_CATEGORIES][4] = {};

  void resolve_profile() {
    for (auto& p : pending) {
      float ms = 0.0f;
      if (hipEventSynchronize(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
        prof[p.cat][0] += 1;
        prof[p.cat][1] += ms;
        prof[p.cat][2] += p.gflop;
        prof[p.cat][3] += p.gb;
      }
      (void)hipEventDestroy(p.a);
      (void)hipEventDestroy(p.b);
    }
    pending.clear();
  }

  ~wa_model() {
    resolve_profile();
    for (auto& g : groups) {
      if (g.graph) (void)hipGraphExecDestroy(g.graph);
      if (g.st) (void)hipStreamDestroy(g.st);
      if (g.host_ndone) (void)hipHostFree(g.host_ndone);
    }
    if (own_stream) (void)hipStreamDestroy(own_stream);
    if (enc_stream) (void)hipStreamDestroy(enc_stream);
    for (auto& l : enc)
      for (wq4_tensor* t : {l.qkv, l.out, l.fc1, l.fc2}) wq4_tensor_destroy(t);
    for (auto& l : dec)
      for (wq4_tensor* t : {l.qkv, l.out, l.cq, l.cout, l.fc1, l.fc2, l.ck, l.cv}) wq4_tensor_destroy(t);
  }
};

namespace {

// Where the weights come from: the synthetic generator (no checkpoint is
// available offline) or a GGUF file (loader.rs).  Names are the GGUF names.
struct Source {
  virtual ~Source() = default;
  // n f32 values of `name`; false (no error) when an optional tensor is absent
  virtual bool f32(const std::string& name, int64_t n, float lo, float hi, bool optional, std::vector<float>& out) = 0;
  // raw Q4_0 bytes of the [rows, k] weight `name` written at dst
  virtual bool q4(const std::string& name, int rows, int k, uint8_t* dst) = 0;
  // f16 halves of the [rows, k] weight `name` written at dst (config 5)
  virtual bool f16(const std::string& name, int rows, int k, uint16_t* dst) = 0;
  std::string err;
};

struct SynthSource : Source {
  uint64_t seed;
  explicit SynthSource(uint64_t s) : seed(s) {}
  bool f32(const std::string& name, int64_t n, float lo, float hi, bool optional, std::vector<float>& out) override {
    // Whisper's attention key projections have no bias (loader.rs:205-210)
    if (optional && name.size() > 9 && name.compare(name.size() - 9, 9, ".key.bias") == 0) return false;
    out.resize((size_t)n);
    synth_uniform(seed, name, n, lo, hi, out.data());
    return true;
  }
  bool q4(const std::string& name, int rows, int k, uint8_t* dst) override {
    std::vector<float> w((size_t)rows * k);
    synth_uniform(seed, name, (int64_t)rows * k, -lin_scale(k), lin_scale(k), w.data());
    const int64_t nblk = (int64_t)rows * k / 32;
    parallel_for(nblk, [&](int64_t a, int64_t b) {
      (void)wq4_quantize_q4_0(w.data() + a * 32, (b - a) * 32, dst + a * 18);
    });
    return true;
  }
  bool f16(const std::string& name, int rows, int k, uint16_t* dst) override {
    std::vector<float> w((size_t)rows * k);
    synth_uniform(seed, name, (int64_t)rows * k, -lin_scale(k), lin_scale(k), w.data());
    for (size_t i = 0; i < w.size(); ++i) dst[i] = __builtin_bit_cast(uint16_t, (_Float16)w[i]);
    return true;
  }
};

// f16 (IEEE binary16, little-endian) -> f32, exact (half 2.7.1 semantics).
float f16_to_f32(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }

struct GgufSource : Source {
  const wa::GgufFile& g;
  explicit GgufSource(const wa::GgufFile& f) : g(f) {}
  bool bad(const std::string& m) {
    err = m;
    return false;
  }
  // loader.rs:47-104 (F32 / F16 1-D and 2-D tensors, 3-D conv weights)
  bool f32(const std::string& name, int64_t n, float, float, bool optional, std::vector<float>& out) override {
    const wa::GgufTensor* t = g.find(name);
    if (!t) return optional ? false : bad("Tensor '" + name + "' not found");
    if (t->type != wa::kGgmlF32 && t->type != wa::kGgmlF16)
      return bad("Expected F32/F16 for '" + name + "', got Q4_0");
    if ((int64_t)t->elements() != n)
      return bad("Tensor '" + name + "' has " + std::to_string(t->elements()) + " elements, expected " +
                 std::to_string(n));
    const uint8_t* p = g.data(*t);
    if (!p) return bad("Tensor '" + name + "' data lies outside the file");
    out.resize((size_t)n);
    if (t->type == wa::kGgmlF32) {
      std::memcpy(out.data(), p, (size_t)n * 4);
    } else {
      for (int64_t i = 0; i < n; ++i) out[(size_t)i] = f16_to_f32((uint16_t)(p[2 * i] | (p[2 * i + 1] << 8)));
    }
    return true;
  }
  // loader.rs:106-144: Q4_0 only; GGUF dims are [in_features, out_features]
  bool q4(const std::string& name, int rows, int k, uint8_t* dst) override {
    const wa::GgufTensor* t = g.find(name);
    if (!t) return bad("Tensor '" + name + "' not found");
    if (t->type != wa::kGgmlQ4_0)
      return bad("Expected Q4_0 for weight '" + name + "', got " + (t->type == wa::kGgmlF32 ? "F32" : "F16") +
                 ". Use the conversion script.");
    if (t->dims.size() != 2 || t->dims[0] != (uint64_t)k || t->dims[1] != (uint64_t)rows)
      return bad("Q4 weight '" + name + "' has the wrong shape (expected [" + std::to_string(rows) + ", " +
                 std::to_string(k) + "])");
    const uint8_t* p = g.data(*t);
    if (!p) return bad("Tensor '" + name + "' data lies outside the file");
    std::memcpy(dst, p, t->nbytes());
    return true;
  }
  // config 5: F16 linear weights (the reference loader rejects them)
  bool f16(const std::string& name, int rows, int k, uint16_t* dst) override {
    const wa::GgufTensor* t = g.find(name);
    if (!t) return bad("Tensor '" + name + "' not found");
    if (t->type != wa::kGgmlF16)
      return bad("Expected F16 for weight '" + name + "' (an F16 checkpoint), got " +
                 (t->type == wa::kGgmlF32 ? "F32" : "Q4_0"));
    if (t->dims.size() != 2 || t->dims[0] != (uint64_t)k || t->dims[1] != (uint64_t)rows)
      return bad("F16 weight '" + name + "' has the wrong shape (expected [" + std::to_string(rows) + ", " +
                 std::to_string(k) + "])");
    const uint8_t* p = g.data(*t);
    if (!p) return bad("Tensor '" + name + "' data lies outside the file");
    std::memcpy(dst, p, t->nbytes());
    return true;
  }
};

struct Builder {
  wa_model* m;
  Source& src;
  wq4_status st = WQ4_OK;

  float* upload(const std::vector<float>& v) {
    float* p = m->dev.alloc<float>(v.size());
    if (!p || hipMemcpy(p, v.data(), v.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
      st = fail(WQ4_ENOMEM, "upload failed");
      return nullptr;
    }
    m->bytes += v.size() * 4;
    return p;
  }
  std::vector<float> get(const std::string& name, int64_t n, float lo, float hi) {
    std::vector<float> v;
    if (st == WQ4_OK && !src.f32(name, n, lo, hi, false, v)) st = fail(WQ4_EINVAL, src.err);
    if (v.size() != (size_t)n) v.assign((size_t)n, 0.0f);
    return v;
  }
  float* vec(const std::string& name, int64_t n, float lo, float hi) { return upload(get(name, n, lo, hi)); }
  // Linear weights of several GGUF tensors [n_i, k], row-concatenated (a
  // fused projection): Q4_0 blocks, or f16 halves for an F16 model.
  // decode_step = false: the tensor never runs at <= 32 rows (encoder), so
  // the decode-step kernel's second weight copy is not built.
  wq4_tensor* q4(const std::vector<std::string>& names, const std::vector<int>& rows, int k, bool decode_step = true) {
    const unsigned cflags = decode_step ? 0u : WQ4_TENSOR_NO_DECODE_STEP;
    if (st != WQ4_OK) return nullptr;
    int64_t total = 0;
    for (int r : rows) total += r;
    if (m->wtype == 1) {
      std::vector<uint16_t> h((size_t)(total * k));
      size_t off = 0;
      for (size_t i = 0; i < names.size(); ++i) {
        if (!src.f16(names[i], rows[i], k, h.data() + off)) {
          st = fail(WQ4_EINVAL, src.err);
          return nullptr;
        }
        off += (size_t)rows[i] * k;
      }
      wq4_tensor* t = nullptr;
      wq4_status s = wq4_tensor_create_f16_ex(m->device, h.data(), total, k, cflags, &t);
      if (s != WQ4_OK) st = fail(s, std::string("F16 weight upload: ") + wq4_last_error());
      m->bytes += wq4_tensor_device_bytes(t);
      return t;
    }
    std::vector<uint8_t> raw((size_t)(total * k / 32 * 18));
    size_t off = 0;
    for (size_t i = 0; i < names.size(); ++i) {
      if (!src.q4(names[i], rows[i], k, raw.data() + off)) {
        st = fail(WQ4_EINVAL, src.err);
        return nullptr;
      }
      off += (size_t)rows[i] * k / 32 * 18;
    }
    wq4_tensor* t = nullptr;
    wq4_status s = wq4_tensor_create_ex(m->device, raw.data(), raw.size(), total, k, cflags, &t);
    if (s != WQ4_OK) st = fail(s, std::string("Q4 upload: ") + wq4_last_error());
    m->bytes += wq4_tensor_device_bytes(t);
    return t;
  }
  // One linear weight [rows, k] uploaded in its raw GGUF form (Q4_0 blocks,
  // or f16 halves for an F16 model) for kernels that dequantize it directly.
  uint8_t* raw(const std::string& name, int rows, int k) {
    if (st != WQ4_OK) return nullptr;
    const size_t n = m->wtype == 1 ? (size_t)rows * k * 2 : (size_t)rows * k / 32 * 18;
    std::vector<uint8_t> h(n);
    const bool ok = m->wtype == 1 ? src.f16(name, rows, k, reinterpret_cast<uint16_t*>(h.data()))
                                  : src.q4(name, rows, k, h.data());
    if (!ok) {
      st = fail(WQ4_EINVAL, src.err);
      return nullptr;
    }
    uint8_t* p = m->dev.alloc<uint8_t>(n);
    if (!p || hipMemcpy(p, h.data(), n, hipMemcpyHostToDevice) != hipSuccess) {
      st = fail(WQ4_ENOMEM, "upload failed");
      return nullptr;
    }
    m->bytes += n;
    return p;
  }
  // bias vector of a fused projection: absent biases (attention key) are 0.
  float* bias_cat(const std::vector<std::string>& names, int n) {
    std::vector<float> v;
    for (const auto& nm : names) {
      std::vector<float> b;
      if (st == WQ4_OK && src.f32(nm, n, -0.02f, 0.02f, true, b)) {
        v.insert(v.end(), b.begin(), b.end());
      } else {
        if (!src.err.empty()) st = fail(WQ4_EINVAL, src.err);
        v.insert(v.end(), n, 0.0f);
      }
    }
    return upload(v);
  }
  // conv weight [N, C, 3] (GGUF dims [3, C, N], loader.rs:254-268) ->
  // [N][kk*C + c] (im2col order, layers.rs:118-121)
  float* conv(const std::string& name, int N, int C) {
    auto w = get(name, (int64_t)N * C * 3, -lin_scale(3 * C), lin_scale(3 * C));
    std::vector<float> t((size_t)N * 3 * C);
    for (int n = 0; n < N; ++n)
      for (int c = 0; c < C; ++c)
        for (int kk = 0; kk < 3; ++kk) t[(size_t)n * 3 * C + kk * C + c] = w[((size_t)n * C + c) * 3 + kk];
    return upload(t);
  }
};

// Every weight of the model (loader.rs:279-377 load_encoder / load_decoder).
wq4_status build_model(wa_model* m, Source& src) {
  const Config& c = m->cfg;
  const int D = c.n_audio_state, F = 4 * D, Dt = c.n_text_state, Ft = 4 * Dt;
  Builder B{m, src};
  m->conv1_wt = B.conv("encoder.conv1.weight", D, c.n_mels);
  m->conv1_b = B.vec("encoder.conv1.bias", D, -0.02f, 0.02f);
  m->conv2_wt = B.conv("encoder.conv2.weight", D, D);
  m->conv2_b = B.vec("encoder.conv2.bias", D, -0.02f, 0.02f);
  m->enc_pos = B.vec("encoder.positional_embedding", (int64_t)c.n_audio_ctx * D, -0.1f, 0.1f);
  m->enc.resize(c.n_audio_layer);
  for (int i = 0; i < c.n_audio_layer; ++i) {
    const std::string p = "encoder.blocks." + std::to_string(i);
    EncLayer& L = m->enc[i];
    L.ln1_w = B.vec(p + ".attn_ln.weight", D, 0.9f, 1.1f);
    L.ln1_b = B.vec(p + ".attn_ln.bias", D, -0.05f, 0.05f);
    L.qkv = B.q4({p + ".attn.query.weight", p + ".attn.key.weight", p + ".attn.value.weight"}, {D, D, D}, D, false);
    L.qkv_b = B.bias_cat({p + ".attn.query.bias", p + ".attn.key.bias", p + ".attn.value.bias"}, D);
    L.out = B.q4({p + ".attn.out.weight"}, {D}, D, false);
    L.out_b = B.vec(p + ".attn.out.bias", D, -0.02f, 0.02f);
    L.ln2_w = B.vec(p + ".mlp_ln.weight", D, 0.9f, 1.1f);
    L.ln2_b = B.vec(p + ".mlp_ln.bias", D, -0.05f, 0.05f);
    L.fc1 = B.q4({p + ".mlp.0.weight"}, {F}, D, false);
    L.fc1_b = B.vec(p + ".mlp.0.bias", F, -0.02f, 0.02f);
    L.fc2 = B.q4({p + ".mlp.2.weight"}, {D}, F, false);
    L.fc2_b = B.vec(p + ".mlp.2.bias", D, -0.02f, 0.02f);
    if (B.st != WQ4_OK) return B.st;
  }
  m->lnp_w = B.vec("encoder.ln_post.weight", D, 0.9f, 1.1f);
  m->lnp_b = B.vec("encoder.ln_post.bias", D, -0.05f, 0.05f);
  m->tok_emb = B.vec("decoder.token_embedding.weight", (int64_t)c.n_vocab * Dt, -lin_scale(Dt), lin_scale(Dt));
  m->dec_pos = B.vec("decoder.positional_embedding", (int64_t)c.n_text_ctx * Dt, -0.02f, 0.02f);
  m->dec.resize(c.n_text_layer);
  for (int i = 0; i < c.n_text_layer; ++i) {
    const std::string p = "decoder.blocks." + std::to_string(i);
    DecLayer& L = m->dec[i];
    L.ln1_w = B.vec(p + ".attn_ln.weight", Dt, 0.9f, 1.1f);
    L.ln1_b = B.vec(p + ".attn_ln.bias", Dt, -0.05f, 0.05f);
    L.qkv = B.q4({p + ".attn.query.weight", p + ".attn.key.weight", p + ".attn.value.weight"}, {Dt, Dt, Dt}, Dt);
    L.qkv_b = B.bias_cat({p + ".attn.query.bias", p + ".attn.key.bias", p + ".attn.value.bias"}, Dt);
    L.out = B.q4({p + ".attn.out.weight"}, {Dt}, Dt);
    L.out_b = B.vec(p + ".attn.out.bias", Dt, -0.02f, 0.02f);
    L.ln2_w = B.vec(p + ".cross_attn_ln.weight", Dt, 0.9f, 1.1f);
    L.ln2_b = B.vec(p + ".cross_attn_ln.bias", Dt, -0.05f, 0.05f);
    L.cq = B.q4({p + ".cross_attn.query.weight"}, {Dt}, Dt);
    L.cq_b = B.vec(p + ".cross_attn.query.bias", Dt, -0.02f, 0.02f);
    // cross-attention key / value (loader.rs:205-210; the key bias, absent
    // in Whisper, cancels in the softmax and is not needed)
    L.ck_raw = B.raw(p + ".cross_attn.key.weight", Dt, D);
    L.cv_raw = B.raw(p + ".cross_attn.value.weight", Dt, D);
    if (L.cv_raw && m->wtype == 0) {
      const size_t nw = wa::wv_pack_words(m->cfg.n_text_head, Dt);
      L.cv_p = m->dev.alloc<uint32_t>(nw);
      if (!L.cv_p || wa::launch_wv_pack(L.cv_raw, m->cfg.n_text_head, Dt, L.cv_p, nullptr) != hipSuccess)
        return fail(WQ4_ENOMEM, "cross-attention Wv repack");
      m->bytes += nw * 4;
    }
    L.cv_b = B.bias_cat({p + ".cross_attn.value.bias"}, Dt);
    if (m->kv_clips > 0) {  // the cache GEMMs run at encoder row counts only: no decode-step copy
      L.ck = B.q4({p + ".cross_attn.key.weight"}, {Dt}, D, false);
      L.cv = B.q4({p + ".cross_attn.value.weight"}, {Dt}, D, false);
    }
    L.cout = B.q4({p + ".cross_attn.out.weight"}, {Dt}, Dt);
    L.cout_b = B.vec(p + ".cross_attn.out.bias", Dt, -0.02f, 0.02f);
    L.ln3_w = B.vec(p + ".mlp_ln.weight", Dt, 0.9f, 1.1f);
    L.ln3_b = B.vec(p + ".mlp_ln.bias", Dt, -0.05f, 0.05f);
    L.fc1 = B.q4({p + ".mlp.0.weight"}, {Ft}, Dt);
    L.fc1_b = B.vec(p + ".mlp.0.bias", Ft, -0.02f, 0.02f);
    L.fc2 = B.q4({p + ".mlp.2.weight"}, {Dt}, Ft);
    L.fc2_b = B.vec(p + ".mlp.2.bias", Dt, -0.02f, 0.02f);
    if (B.st != WQ4_OK) return B.st;
  }
  m->dln_w = B.vec("decoder.ln.weight", Dt, 0.9f, 1.1f);
  m->dln_b = B.vec("decoder.ln.bias", Dt, -0.05f, 0.05f);
  return B.st;
}

// W gamma and W beta + bias of every decoder GEMM that reads a LayerNorm
// (wq4_ln_fold_vectors, double accumulation from the dequantized weights),
// layers spread over host threads.
wq4_status build_ln_fold(wa_model* m) {
  const int Dt = m->cfg.n_text_state;
  struct Job {
    wq4_tensor* w;
    const float *g, *b, *bias;
    float **wg, **b2;
  };
  std::vector<Job> jobs;
  for (DecLayer& L : m->dec) {
    jobs.push_back({L.qkv, L.ln1_w, L.ln1_b, L.qkv_b, &L.qkv_wg, &L.qkv_b2});
    jobs.push_back({L.cq, L.ln2_w, L.ln2_b, L.cq_b, &L.cq_wg, &L.cq_b2});
    jobs.push_back({L.fc1, L.ln3_w, L.ln3_b, L.fc1_b, &L.fc1_wg, &L.fc1_b2});
  }
  for (Job& j : jobs) {
    int64_t n = 0, k = 0;
    (void)wq4_tensor_shape(j.w, &n, &k);
    *j.wg = m->dev.alloc<float>((size_t)n);
    *j.b2 = m->dev.alloc<float>((size_t)n);
    if (!*j.wg || !*j.b2) return fail(WQ4_ENOMEM, "LayerNorm-fold vector allocation failed");
    m->bytes += (size_t)n * 8;
  }
  std::atomic<size_t> next{0};
  std::atomic<int> bad{0};
  auto work = [&]() {
    (void)hipSetDevice(m->device);
    for (size_t i = next++; i < jobs.size(); i = next++) {
      const Job& j = jobs[i];
      int64_t n = 0, k = 0;
      (void)wq4_tensor_shape(j.w, &n, &k);
      std::vector<float> g(Dt), b(Dt), bias((size_t)n), wg((size_t)n), b2((size_t)n);
      if (hipMemcpy(g.data(), j.g, Dt * 4, hipMemcpyDeviceToHost) != hipSuccess ||
          hipMemcpy(b.data(), j.b, Dt * 4, hipMemcpyDeviceToHost) != hipSuccess ||
          hipMemcpy(bias.data(), j.bias, (size_t)n * 4, hipMemcpyDeviceToHost) != hipSuccess ||
          wq4_ln_fold_vectors(j.w, g.data(), b.data(), bias.data(), wg.data(), b2.data()) != WQ4_OK ||
          hipMemcpy(*j.wg, wg.data(), (size_t)n * 4, hipMemcpyHostToDevice) != hipSuccess ||
          hipMemcpy(*j.b2, b2.data(), (size_t)n * 4, hipMemcpyHostToDevice) != hipSuccess)
        bad = 1;
    }
  };
  const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t) th.emplace_back(work);
  for (auto& t : th) t.join();
  if (bad) return fail(WQ4_EHIP, "LayerNorm-fold vectors failed");
  return WQ4_OK;
}

wq4_status alloc_activations(wa_model* m) {
  const Config& c = m->cfg;
  const int D = c.n_audio_state, F = 4 * D, Dt = c.n_text_state, Ft = 4 * Dt;
  const int B = m->bmax, T = c.n_audio_ctx;
  const int64_t renc = (int64_t)B * T, rdec = (int64_t)B * 4;
  Dev& d = m->dev;
  auto tiled = [&](int64_t rows, int k) {
    const size_t n = wq4_atiled_bytes(rows, k, m->prec);
    m->bytes += n;
    return d.alloc<_Float16>(n / 2);
  };
  auto f32 = [&](int64_t n) {
    m->bytes += (size_t)n * 4;
    return d.alloc<float>((size_t)n);
  };
  m->h1 = f32((int64_t)B * 2 * T * D);
  m->x = f32(renc * D);
  m->qkv = f32(renc * 3 * D);
  m->at_d = tiled(renc, D);
  m->at_f = tiled(renc, F);
  m->enc_planes = d.alloc<_Float16>((size_t)renc * m->ns * D);
  m->bytes += (size_t)renc * m->ns * D * 2;
  for (auto& L : m->dec) {
    L.cache_k = f32((int64_t)B * c.n_text_ctx * Dt);
    L.cache_v = f32((int64_t)B * c.n_text_ctx * Dt);
  }  // the cross K / V caches: on the first transcribe that reads them (cross_kv_forward)
  // f16-pair tied embedding for the decode step's fused logits + pick,
  // fragment-tiled (1 KiB contiguous per load instruction)
  if (!wa::emb_tiled_supported(Dt)) return fail(WQ4_EINVAL, "n_text_state must be a multiple of 128");
  const size_t erows = (size_t)wa::emb_tiled_rows(c.n_vocab);
  m->tok_emb2 = d.alloc<_Float16>(erows * m->ns * Dt);
  if (!m->tok_emb2) return fail(WQ4_ENOMEM, "embedding plane allocation failed");
  m->bytes += erows * m->ns * Dt * 2;
  WA_HIP(wa::launch_emb_tiled(m->tok_emb, c.n_vocab, Dt, m->ns, m->tok_emb2, nullptr));
  // cross-attention scratch, sized for the largest plan over 1..4B rows
  const int HP = (c.n_text_head + 15) / 16 * 16;
  size_t xpart = 0;
  for (int r = 1; r <= rdec; ++r) xpart = std::max(xpart, wa::xattn_part_floats(r, c.n_text_head, Dt, T));
  m->groups.resize(kMaxGroups);
  for (DecGroup& g : m->groups) {  // each group sized for the whole batch (small)
    g.xd = f32(rdec * Dt);
    g.qkvd = f32(rdec * 3 * Dt);
    g.qd = f32(rdec * Dt);
    g.hid = f32(rdec * Dt);
    g.logits = f32((int64_t)B * c.n_vocab);
    g.atd_dec = tiled(rdec, Dt);
    g.atf_dec = tiled(rdec, Ft);
    g.prompt_tok = d.alloc<int>(rdec);
    g.next_tok = d.alloc<int>(B);
    g.tokens = d.alloc<int>((size_t)B * kMaxTokens);
    g.ntok = d.alloc<int>(B);
    g.done = d.alloc<int>(B);
    g.state = d.alloc<wa::DecodeState>(1);
    g.xattn_part = f32((int64_t)xpart);
    const int kvc = std::max(1, m->kv_clips);
    g.xkv_part = f32((int64_t)wa::cross_attention_kv_part_floats(kvc, c.n_text_head, T));
    g.xkv_ctr = d.alloc<int>((size_t)kvc * c.n_text_head);
    g.xqt = d.alloc<_Float16>((size_t)rdec * m->ns * HP * Dt);
    g.atd_ln = tiled(rdec, Dt);
    g.ln_stats = f32(rdec * (Dt / 16) * 2);  // per 16-column tile (the decode-step GEMM)
    g.hid_t = tiled(rdec, Dt);
    g.lg_val = f32((int64_t)32 * wa::logits_argmax_groups(c.n_vocab));
    g.lg_idx = d.alloc<int>((size_t)32 * wa::logits_argmax_groups(c.n_vocab));
    g.lg_ctr = d.alloc<int>(1);
    m->bytes += (size_t)rdec * m->ns * HP * Dt * 2;
    for (void* p : {(void*)g.xd, (void*)g.qkvd, (void*)g.qd, (void*)g.hid, (void*)g.logits, (void*)g.atd_dec,
                    (void*)g.atf_dec, (void*)g.prompt_tok, (void*)g.next_tok, (void*)g.tokens, (void*)g.ntok,
                    (void*)g.done, (void*)g.state, (void*)g.xattn_part, (void*)g.xqt, (void*)g.lg_val,
                    (void*)g.lg_idx, (void*)g.lg_ctr, (void*)g.atd_ln, (void*)g.ln_stats, (void*)g.hid_t,
                    (void*)g.xkv_part, (void*)g.xkv_ctr})
      if (!p) return fail(WQ4_ENOMEM, "decode-group allocation failed");
    WA_HIP(hipMemset(g.xkv_ctr, 0, (size_t)kvc * c.n_text_head * sizeof(int)));
    WA_HIP(hipMemset(g.atd_ln, 0, wq4_atiled_bytes(rdec, Dt, m->prec)));
    WA_HIP(hipMemset(g.hid_t, 0, wq4_atiled_bytes(rdec, Dt, m->prec)));  // padded clips stay 0
    WA_HIP(hipMemset(g.lg_ctr, 0, sizeof(int)));
    WA_HIP(hipMemset(g.xqt, 0, (size_t)rdec * m->ns * HP * Dt * 2));  // padded heads stay 0
    WA_HIP(hipMemset(g.atd_dec, 0, wq4_atiled_bytes(rdec, Dt, m->prec)));
    WA_HIP(hipMemset(g.atf_dec, 0, wq4_atiled_bytes(rdec, Ft, m->prec)));
    WA_HIP(hipHostMalloc(reinterpret_cast<void**>(&g.host_ndone), 8 * sizeof(int), 0));
    WA_HIP(hipStreamCreateWithFlags(&g.st, hipStreamNonBlocking));
  }
  m->range_flag = d.alloc<int>(1);
  for (void* p : {(void*)m->h1, (void*)m->x, (void*)m->qkv, (void*)m->at_d, (void*)m->at_f, (void*)m->enc_planes,
                  (void*)m->range_flag})
    if (!p) return fail(WQ4_ENOMEM, "activation allocation failed");
  WA_HIP(hipMemset(m->range_flag, 0, sizeof(int)));
  for (auto& L : m->dec)
    if (!L.cache_k || !L.cache_v) return fail(WQ4_ENOMEM, "KV cache allocation failed");
  // zero the A-tiled buffers once: padded rows stay finite forever
  WA_HIP(hipMemset(m->at_d, 0, wq4_atiled_bytes(renc, D, m->prec)));
  WA_HIP(hipMemset(m->at_f, 0, wq4_atiled_bytes(renc, F, m->prec)));
  return WQ4_OK;
}

// ------------------------------------------------------------ forward --
// HIP-event bracket of one launch (only when m->profile).
struct Prof {
  wa_model* m;
  hipStream_t st;
  int cat;
  double gflop, gb;
  hipEvent_t a = nullptr, b = nullptr;
  Prof(wa_model* m_, hipStream_t st_, int cat_, double gflop_, double gb_)
      : m(m_), st(st_), cat(cat_), gflop(gflop_), gb(gb_) {
    // the CU-masked stream of a pipelined transcribe is not timed: the
    // events measure the kernels at full width
    if (m->profile && st != m->enc_stream && hipEventCreate(&a) == hipSuccess && hipEventCreate(&b) == hipSuccess)
      (void)hipEventRecord(a, st);
  }
  ~Prof() {
    if (a && b) {
      (void)hipEventRecord(b, st);
      m->pending.push_back({a, b, cat, gflop, gb});
    }
  }
};

// Algorithmic cost of one Q4 GEMM: 2*rows*N*K flops;
// N*K*18/32 weight bytes + rows*K*4 (x, f32 at the ABI) + rows*N*4 (y).
Prof q4prof(wa_model* m, hipStream_t st, const wq4_tensor* w, int64_t rows) {
  int64_t n = 0, k = 0;
  (void)wq4_tensor_shape(w, &n, &k);
  return Prof(m, st, 0, 2.0 * rows * n * k * 1e-9, ((double)n * k * 18 / 32 + 4.0 * rows * k + 4.0 * rows * n) * 1e-9);
}

// WhisperEncoder::forward (encoder.rs:87-115) in three parts, so that a
// pipelined transcribe (wa_transcribe_batches) can run the front and the
// first layers of the next batch's encoder on a CU-masked stream beside the
// current batch's decode: encoder_front (the conv stem), encoder_layers
// [l0, l1) and encoder_post (ln_post, f32, into enc_out_f32 or the conv
// scratch; m->enc_f32 points at it).
wq4_status encoder_front(wa_model* m, const float* mel, int B, hipStream_t st) {
  const Config& c = m->cfg;
  const int D = c.n_audio_state, T = c.n_audio_ctx;
  const int T_mel = 2 * T;
  const int64_t rows = (int64_t)B * T;
  {  // conv1 + GELU: mel [B, n_mels, 3000] -> h1 [B, 3000, D]   (encoder.rs:89-90)
    Prof p(m, st, 2, 2.0 * B * T_mel * D * 3.0 * c.n_mels * 1e-9, 4.0 * B * T_mel * (c.n_mels + D) * 1e-9);
    WA_HIP(wa::launch_conv_gelu(mel, (long)c.n_mels * T_mel, T_mel, 1, B, c.n_mels, T_mel, 1, m->conv1_wt,
                                m->conv1_b, nullptr, D, m->h1, st));
  }
  {  // conv2 (stride 2) + GELU + positional embedding -> x [B, 1500, D]   (:93-106)
    Prof p(m, st, 2, 2.0 * rows * D * 3.0 * D * 1e-9, 4.0 * B * (T_mel + T) * D * 1e-9);
    WA_HIP(wa::launch_conv_gelu(m->h1, (long)T_mel * D, 1, D, B, D, T_mel, 2, m->conv2_wt, m->conv2_b, m->enc_pos,
                                D, m->x, st));
  }
  return WQ4_OK;
}

wq4_status encoder_layers(wa_model* m, int B, int l0, int l1, hipStream_t st) {
  const Config& c = m->cfg;
  const int D = c.n_audio_state, T = c.n_audio_ctx, H = c.n_audio_head;
  const int64_t rows = (int64_t)B * T;
  const double ln_gb = 8.0 * rows * D * 1e-9;
  for (int li = l0; li < l1; ++li) {  // EncoderBlock::forward (encoder.rs:37-49)
    const EncLayer& L = m->enc[li];
    {
      Prof p(m, st, 3, 0.0, ln_gb);
      WA_WQ4(wq4_layernorm(m->x, L.ln1_w, L.ln1_b, rows, D, m->prec, m->at_d, nullptr, st));
    }
    {
      Prof p = q4prof(m, st, L.qkv, rows);
      WA_WQ4(wq4_gemm_tiled(L.qkv, L.qkv_b, m->at_d, nullptr, m->qkv, nullptr, rows, 0u, m->prec, 1, st));
    }
    {
      Prof p(m, st, 1, 4.0 * B * H * (double)T * T * 64 * 1e-9, 16.0 * rows * D * 1e-9);
      WA_HIP(wa::launch_encoder_attention(m->qkv, B, T, H, m->at_d, m->ns, st, m->wide_attn ? m->h1 : nullptr));
    }
    if (m->wide_attn) {  // range tier 3: the f32 attention output through Q4Linear::forward (m->at_d: workspace)
      WA_WQ4(wq4_linear_forward_ws(L.out, L.out_b, m->h1, m->x, m->x, rows, D, WQ4_EPI_RESIDUAL, m->prec, m->at_d,
                                   wq4_atiled_bytes(rows, D, m->prec), st));
    } else {
      Prof p = q4prof(m, st, L.out, rows);
      WA_WQ4(wq4_gemm_tiled(L.out, L.out_b, m->at_d, m->x, m->x, nullptr, rows, WQ4_EPI_RESIDUAL, m->prec, 1, st));
    }
    if (m->wide_ffn) {  // range tier 2: Q4FFN::forward with per-call operand scales (m->qkv: f32 scratch)
      WA_WQ4(wq4_layernorm(m->x, L.ln2_w, L.ln2_b, rows, D, WQ4_PREC_F16X2, nullptr, m->qkv, st));
      WA_WQ4(wq4_ffn_forward_ws(L.fc1, L.fc1_b, L.fc2, L.fc2_b, m->qkv, m->x, m->x, rows, WQ4_EPI_RESIDUAL, m->prec,
                                m->ffn_ws, m->ffn_ws_bytes, st));
      continue;
    }
    {
      Prof p(m, st, 3, 0.0, ln_gb);
      WA_WQ4(wq4_layernorm(m->x, L.ln2_w, L.ln2_b, rows, D, m->prec, m->at_d, nullptr, st));
    }
    {
      Prof p = q4prof(m, st, L.fc1, rows);
      WA_WQ4(wq4_gemm_tiled(L.fc1, L.fc1_b, m->at_d, nullptr, nullptr, m->at_f, rows,
                            WQ4_EPI_GELU | WQ4_EPI_TILED_OUT, m->prec, 1, st));
    }
    {
      Prof p = q4prof(m, st, L.fc2, rows);
      WA_WQ4(wq4_gemm_tiled(L.fc2, L.fc2_b, m->at_f, m->x, m->x, nullptr, rows, WQ4_EPI_RESIDUAL, m->prec, 1, st));
    }
  }
  return WQ4_OK;
}

wq4_status encoder_post(wa_model* m, int B, hipStream_t st, float* enc_out_f32) {
  const Config& c = m->cfg;
  const int D = c.n_audio_state;
  const int64_t rows = (int64_t)B * c.n_audio_ctx;
  {
    Prof p(m, st, 3, 0.0, 8.0 * rows * D * 1e-9);
    float* out = enc_out_f32 ? enc_out_f32 : m->h1;
    WA_WQ4(wq4_layernorm(m->x, m->lnp_w, m->lnp_b, rows, D, WQ4_PREC_F16X2, nullptr, out, st));
    m->enc_f32 = out;
  }
  return WQ4_OK;
}

wq4_status encoder_forward(wa_model* m, const float* mel, int B, hipStream_t st, float* enc_out_f32) {
  wq4_status s = encoder_front(m, mel, B, st);
  if (s == WQ4_OK) s = encoder_layers(m, B, 0, (int)m->enc.size(), st);
  if (s == WQ4_OK) s = encoder_post(m, B, st, enc_out_f32);
  return s;
}

// The cross-attention state of every decoder layer: the reference caches
// K = enc Wk^T and V = enc Wv^T per layer (attention.rs:177-206
// forward_init_cache); here one copy of encoder_out as f16 planes serves all
// layers (wa_xattn.hip).
// Transcribes of at most kv_clips clips also get the reference's own
// per-layer caches, K = enc Wk^T and V = enc Wv^T + bv, head-major (the
// few-clip decode reads them: launch_cross_attention_kv).
// `caches` false (wa_encode: no decode follows it) fills the planes only.
// The caches (f32, kv_clips x n_audio_ctx x n_text_state per layer and
// tensor: 3.9 GB for Large-V3 at 8 clips) are allocated on the first
// transcribe of at most kv_small clips, so batches past that never hold them.
wq4_status cross_kv_forward(wa_model* m, int B, hipStream_t st, bool caches) {
  const Config& c = m->cfg;
  const int64_t rows = (int64_t)B * c.n_audio_ctx;
  m->kv_batch = B;
  WA_HIP(wa::launch_enc_planes(m->enc_f32, rows, c.n_audio_state, m->ns, m->enc_planes, st));
  m->kv_n = caches && B <= m->kv_small ? B : 0;
  if (m->kv_n > 0 && !m->kv_alloc_ok) {
    // all layers or none: a partial failure frees what it got, so the next
    // transcribe retries the allocation (or fails the same way) instead of
    // running the cache GEMMs on a null layer
    const size_t n = (size_t)m->kv_clips * c.n_audio_ctx * c.n_text_state;
    bool ok = true;
    for (DecLayer& L : m->dec) {
      if (!L.xk) L.xk = m->dev.alloc<float>(n);
      if (!L.xv) L.xv = m->dev.alloc<float>(n);
      if (!L.xk || !L.xv) {
        ok = false;
        break;
      }
    }
    if (!ok) {
      for (DecLayer& L : m->dec) {
        m->dev.release(L.xk);
        m->dev.release(L.xv);
        L.xk = L.xv = nullptr;
      }
      m->kv_n = 0;
      return fail(WQ4_ENOMEM, "cross K/V cache allocation failed");
    }
    m->bytes += n * 8 * m->dec.size();
    m->kv_alloc_ok = true;
  }
  if (m->kv_n > 0) {
    // ln_post again, as the GEMMs' A-tiled operand (m->x still holds its
    // input); the caches of clips [0, kv_n): a prefix of the rows
    const int64_t kv_rows = (int64_t)m->kv_n * c.n_audio_ctx;
    WA_WQ4(wq4_layernorm(m->x, m->lnp_w, m->lnp_b, kv_rows, c.n_audio_state, m->prec, m->at_d, nullptr, st));
    for (DecLayer& L : m->dec) {
      WA_WQ4(wq4_gemm_tiled_headmajor(L.ck, nullptr, m->at_d, L.xk, kv_rows, c.n_audio_ctx, c.n_text_state, m->prec,
                                      0, st));
      WA_WQ4(wq4_gemm_tiled_headmajor(L.cv, L.cv_b, m->at_d, L.xv, kv_rows, c.n_audio_ctx, c.n_text_state, m->prec,
                                      0, st));
    }
  }
  return WQ4_OK;
}

// LayerNorm fold for this decoder pass: decode steps (Tq = 1) whose GEMMs
// all run the 8-wave decode plans (WA_LN_FOLD=0 disables, for A/B runs).
bool lnfold_on(const wa_model* m, int Tq, const wa::DecodeState* state, int64_t rows) {
  static const bool enabled = [] {
    const char* e = getenv("WA_LN_FOLD");
    return e ? atoi(e) != 0 : true;
  }();
  if (!enabled || m->wide_range || state == nullptr || Tq != 1 || m->dec.empty()) return false;
  const DecLayer& L = m->dec[0];
  for (const wq4_tensor* w : {L.qkv, L.out, L.cq, L.cout, L.fc1, L.fc2})
    if (!wq4_lnfold_supported(w, rows)) return false;
  return true;
}

// A greedy decode step of <= 32 clips picks its tokens inside the logits
// kernel (wa::launch_logits_argmax); prompts and larger groups keep the
// stored logits + separate argmax.
bool fused_pick(const DecGroup& g, int Tq, const wa::DecodeState* state) {
  return state != nullptr && Tq == 1 && g.nb <= 32;
}

// Decoder pass over Tq new tokens for the clips of group g (forward_prompt
// when state == nullptr, decode_step otherwise), ending in last-position
// logits.  Self-KV and the encoder planes are addressed at the group's clip offset.
wq4_status decoder_forward(wa_model* m, DecGroup& g, const int* tokens, int Tq, const wa::DecodeState* state,
                           int pos0, int kv0, hipStream_t st) {
  const Config& c = m->cfg;
  const int D = c.n_text_state, H = c.n_text_head, T = c.n_audio_ctx;
  const int B = g.nb;
  const int64_t rows = (int64_t)B * Tq;
  const size_t self_ofs = (size_t)g.b0 * H * c.n_text_ctx * 64;
  const _Float16* enc = m->enc_planes + (size_t)g.b0 * T * m->ns * c.n_audio_state;
  // Decode steps fold every decoder LayerNorm into the GEMMs around it
  // (wq4_gemm_tiled_lnfold): the residual GEMM producing x also writes
  // tiled(x * gamma) and tile statistics, the GEMM reading LN(x) corrects
  // its epilogue -- no LayerNorm launches inside the layer loop.
  const bool fold = lnfold_on(m, Tq, state, rows);
  if (fold)
    WA_HIP(wa::launch_embed_fold(tokens, m->tok_emb, m->dec_pos, B, Tq, D, state, pos0, g.xd, m->dec[0].ln1_w,
                                 g.atd_ln, g.ln_stats, m->ns, st));
  else
    WA_HIP(wa::launch_embed(tokens, m->tok_emb, m->dec_pos, B, Tq, D, state, pos0, g.xd, st));
  const int nl = (int)m->dec.size();
  for (int li = 0; li < nl; ++li) {  // DecoderBlock (decoder.rs:77-112 / 140-183)
    DecLayer& L = m->dec[li];
    if (fold) {
      const wq4_ln_fold cons1{nullptr, nullptr, nullptr, g.ln_stats, L.qkv_wg};
      WA_WQ4(wq4_gemm_tiled_lnfold(L.qkv, L.qkv_b2, g.atd_ln, nullptr, g.qkvd, nullptr, rows, 0u, m->prec, &cons1,
                                   st));
    } else {
      WA_WQ4(wq4_layernorm(g.xd, L.ln1_w, L.ln1_b, rows, D, m->prec, g.atd_dec, nullptr, st));
      WA_WQ4(wq4_gemm_tiled(L.qkv, L.qkv_b, g.atd_dec, nullptr, g.qkvd, nullptr, rows, 0u, m->prec, 2, st));
    }
    // range tier 3: attention outputs as f32 rows in g.hid, projected through
    // Q4Linear::forward at the ABI (g.atd_dec: its workspace); tier >= 1 has
    // the fold off
    float* const a32 = m->wide_attn ? g.hid : nullptr;
    const size_t a32_ws = wq4_atiled_bytes(rows, D, m->prec);
    WA_HIP(wa::launch_decoder_self_attention(g.qkvd, L.cache_k + self_ofs, L.cache_v + self_ofs, B, Tq, H,
                                             c.n_text_ctx, state, kv0, g.atd_dec, m->ns, st, a32));
    if (a32) {
      WA_WQ4(wq4_linear_forward_ws(L.out, L.out_b, a32, g.xd, g.xd, rows, D, WQ4_EPI_RESIDUAL, m->prec, g.atd_dec,
                                   a32_ws, st));
      WA_WQ4(wq4_layernorm(g.xd, L.ln2_w, L.ln2_b, rows, D, m->prec, g.atd_dec, nullptr, st));
      WA_WQ4(wq4_gemm_tiled(L.cq, L.cq_b, g.atd_dec, nullptr, g.qd, nullptr, rows, 0u, m->prec, 2, st));
    } else if (fold) {
      const wq4_ln_fold prod2{L.ln2_w, g.atd_ln, g.ln_stats, nullptr, nullptr};
      WA_WQ4(wq4_gemm_tiled_lnfold(L.out, L.out_b, g.atd_dec, g.xd, g.xd, nullptr, rows, WQ4_EPI_RESIDUAL, m->prec,
                                   &prod2, st));
      const wq4_ln_fold cons2{nullptr, nullptr, nullptr, g.ln_stats, L.cq_wg};
      WA_WQ4(wq4_gemm_tiled_lnfold(L.cq, L.cq_b2, g.atd_ln, nullptr, g.qd, nullptr, rows, 0u, m->prec, &cons2, st));
    } else {
      WA_WQ4(wq4_gemm_tiled(L.out, L.out_b, g.atd_dec, g.xd, g.xd, nullptr, rows, WQ4_EPI_RESIDUAL, m->prec, 2, st));
      WA_WQ4(wq4_layernorm(g.xd, L.ln2_w, L.ln2_b, rows, D, m->prec, g.atd_dec, nullptr, st));
      WA_WQ4(wq4_gemm_tiled(L.cq, L.cq_b, g.atd_dec, nullptr, g.qd, nullptr, rows, 0u, m->prec, 2, st));
    }
    if (m->group_kv(g)) {  // few clips: one GEMV launch over the cached K / V
      const size_t kofs = (size_t)g.b0 * T * D;
      WA_HIP(wa::launch_cross_attention_kv(g.qd, L.xk + kofs, L.xv + kofs, B, Tq, T, H, g.xkv_part, g.xkv_ctr,
                                           g.atd_dec, m->ns, st, a32));
    } else {
      WA_HIP(wa::launch_xattn(g.qd, L.ck_raw, L.cv_raw, L.cv_p, L.cv_b, m->wtype, enc, B, Tq, T, H, D, g.xqt,
                              g.xattn_part, g.atd_dec, m->ns, st, a32));
    }
    if (a32)  // range tier 3: the cross-attention output projection at the ABI
      WA_WQ4(wq4_linear_forward_ws(L.cout, L.cout_b, a32, g.xd, g.xd, rows, D, WQ4_EPI_RESIDUAL, m->prec, g.atd_dec,
                                   a32_ws, st));
    if (fold) {
      const wq4_ln_fold prod3{L.ln3_w, g.atd_ln, g.ln_stats, nullptr, nullptr};
      WA_WQ4(wq4_gemm_tiled_lnfold(L.cout, L.cout_b, g.atd_dec, g.xd, g.xd, nullptr, rows, WQ4_EPI_RESIDUAL,
                                   m->prec, &prod3, st));
      const wq4_ln_fold cons3{nullptr, nullptr, nullptr, g.ln_stats, L.fc1_wg};
      WA_WQ4(wq4_gemm_tiled_lnfold(L.fc1, L.fc1_b2, g.atd_ln, nullptr, nullptr, g.atf_dec, rows,
                                   WQ4_EPI_GELU | WQ4_EPI_TILED_OUT, m->prec, &cons3, st));
      // the next layer's attn_ln (none after the last layer: decoder.ln below)
      const bool nxt = li + 1 < nl;
      const wq4_ln_fold prod1{nxt ? m->dec[li + 1].ln1_w : nullptr, nxt ? g.atd_ln : nullptr,
                              nxt ? g.ln_stats : nullptr, nullptr, nullptr};
      WA_WQ4(wq4_gemm_tiled_lnfold(L.fc2, L.fc2_b, g.atf_dec, g.xd, g.xd, nullptr, rows, WQ4_EPI_RESIDUAL, m->prec,
                                   &prod1, st));
    } else {
      if (!a32)
        WA_WQ4(wq4_gemm_tiled(L.cout, L.cout_b, g.atd_dec, g.xd, g.xd, nullptr, rows, WQ4_EPI_RESIDUAL, m->prec, 2,
                              st));
      if (m->wide_ffn) {  // range tier 2: Q4FFN::forward with per-call operand scales (g.hid: f32 scratch)
        WA_WQ4(wq4_layernorm(g.xd, L.ln3_w, L.ln3_b, rows, D, WQ4_PREC_F16X2, nullptr, g.hid, st));
        WA_WQ4(wq4_ffn_forward_ws(L.fc1, L.fc1_b, L.fc2, L.fc2_b, g.hid, g.xd, g.xd, rows, WQ4_EPI_RESIDUAL,
                                  m->prec, g.ffn_ws, g.ffn_ws_bytes, st));
        continue;
      }
      WA_WQ4(wq4_layernorm(g.xd, L.ln3_w, L.ln3_b, rows, D, m->prec, g.atd_dec, nullptr, st));
      WA_WQ4(wq4_gemm_tiled(L.fc1, L.fc1_b, g.atd_dec, nullptr, nullptr, g.atf_dec, rows,
                            WQ4_EPI_GELU | WQ4_EPI_TILED_OUT, m->prec, 2, st));
      WA_WQ4(wq4_gemm_tiled(L.fc2, L.fc2_b, g.atf_dec, g.xd, g.xd, nullptr, rows, WQ4_EPI_RESIDUAL, m->prec, 2, st));
    }
  }
  // final LN (decoder.rs:286 / 340) and tied-embedding logits of the last
  // position of every clip (decoder.rs:289-292, 342-343)
  if (fused_pick(g, Tq, state)) {  // decode step: logits + greedy pick in one kernel, into next_tok
    // the final LN writes the pick's operand directly (A-tiled, the
    // embedding planes' precision)
    WA_WQ4(wq4_layernorm(g.xd, m->dln_w, m->dln_b, rows, D, m->prec, g.hid_t, nullptr, st));
    const size_t tofs = (size_t)g.b0 * m->trace_s1 * m->trace_k;
    WA_HIP(wa::launch_logits_argmax(g.hid_t, B, D, m->tok_emb2, m->ns, c.n_vocab, kMinTokens, state, g.lg_val,
                                    g.lg_idx, g.lg_ctr, g.next_tok, m->trace_out ? m->trace_ids + tofs : nullptr,
                                    m->trace_out ? m->trace_out + tofs : nullptr, m->trace_s1, m->trace_k,
                                    m->range_flag, st));
    return WQ4_OK;
  }
  WA_WQ4(wq4_layernorm(g.xd, m->dln_w, m->dln_b, rows, D, WQ4_PREC_F16X2, nullptr, g.hid, st));
  WA_HIP(wa::launch_logits(g.hid + (size_t)(Tq - 1) * D, B, D, (int64_t)Tq * D, m->tok_emb, c.n_vocab, g.logits,
                           st));
  return WQ4_OK;
}

// One greedy step (whisper.rs:104-125): bookkeeping, decode_step, argmax.
wq4_status decode_step(wa_model* m, DecGroup& g, int eot_stop, hipStream_t st) {
  WA_HIP(wa::launch_bookkeep(g.next_tok, g.tokens, g.ntok, g.done, g.nb, kMaxTokens, eot_stop, g.state, st));
  wq4_status s = decoder_forward(m, g, g.next_tok, 1, g.state, 0, 0, st);
  if (s != WQ4_OK) return s;
  if (!fused_pick(g, 1, g.state))
    WA_HIP(wa::launch_argmax_step(g.logits, g.nb, m->cfg.n_vocab, kMinTokens, g.state, g.next_tok, m->range_flag, st));
  return WQ4_OK;
}

// Prompt of group g (whisper.rs:60-99), leaving the first greedy token in
// next_tok and the DecodeState ready for the step graph.
wq4_status prompt_group(wa_model* m, DecGroup& g, int lang_token, hipStream_t st) {
  const Config& c = m->cfg;
  const int B = g.nb;
  std::vector<int> ptok((size_t)B * 4);
  int pos0, kv0;
  wq4_status s;
  if (lang_token >= 0) {
    for (int b = 0; b < B; ++b) {
      ptok[b * 4 + 0] = kSOT;
      ptok[b * 4 + 1] = lang_token;
      ptok[b * 4 + 2] = c.transcribe_token();
      ptok[b * 4 + 3] = c.no_timestamps_token();
    }
    WA_HIP(hipMemcpyAsync(g.prompt_tok, ptok.data(), (size_t)B * 4 * 4, hipMemcpyHostToDevice, st));
    s = decoder_forward(m, g, g.prompt_tok, 4, nullptr, 0, 0, st);
    if (s != WQ4_OK) return s;
    pos0 = 4;
    kv0 = 4;
  } else {
    // decode_step(SOT, 0) fills a 1-entry cache; the language is the last max
    // over the language-token range (whisper.rs:73-83) ...
    for (int b = 0; b < B; ++b) {
      ptok[b * 3 + 0] = kSOT;
      ptok[b * 3 + 1] = c.transcribe_token();
      ptok[b * 3 + 2] = c.no_timestamps_token();
    }
    WA_HIP(hipMemcpyAsync(g.prompt_tok, ptok.data(), (size_t)B * 3 * 4, hipMemcpyHostToDevice, st));
    // SOT rows: embed reads tokens[b * Tq + t] with Tq = 1 -> a contiguous [B]
    // array: next_tok as scratch
    std::vector<int> sot(B, kSOT);
    WA_HIP(hipMemcpyAsync(g.next_tok, sot.data(), (size_t)B * 4, hipMemcpyHostToDevice, st));
    s = decoder_forward(m, g, g.next_tok, 1, nullptr, 0, 0, st);
    if (s != WQ4_OK) return s;
    WA_HIP(wa::launch_argmax(g.logits, B, c.n_vocab, 50259, 50259 + c.n_lang, 0, nullptr, g.prompt_tok, 3,
                             m->range_flag, st));
    // ... then forward_prompt([lang, TRANSCRIBE, NO_TIMESTAMPS]) OVERWRITES the
    // cache from index 0 with positions 0..2 (decoder.rs:272-283) while the
    // position counter continues at 1 + 3 = 4 (whisper.rs:74,93).
    s = decoder_forward(m, g, g.prompt_tok, 3, nullptr, 0, 0, st);
    if (s != WQ4_OK) return s;
    pos0 = 4;
    kv0 = 3;
  }
  // first token: EOT suppressed (whisper.rs:97-99)
  WA_HIP(wa::launch_argmax(g.logits, B, c.n_vocab, 0, c.n_vocab, 1, nullptr, g.next_tok, 1, m->range_flag, st));
  const wa::DecodeState init{pos0 - 1, kv0 - 1, -1, 0};
  WA_HIP(hipMemcpyAsync(g.state, &init, sizeof(init), hipMemcpyHostToDevice, st));
  WA_HIP(hipMemsetAsync(g.ntok, 0, (size_t)B * 4, st));
  WA_HIP(hipMemsetAsync(g.done, 0, (size_t)B * 4, st));
  WA_HIP(hipMemsetAsync(g.tokens, 0, (size_t)B * kMaxTokens * 4, st));
  return WQ4_OK;
}

// Capture (once per group size / eot mode) the step graph of group g.
wq4_status ensure_graph(wa_model* m, DecGroup& g, int eot_stop) {
  // everything the captured step bakes in: the clip range (self-KV and
  // encoder-plane offsets), the EOT mode and the trace buffers
  // buffers, the range tier; one explicit field per mixed-radix digit
  const int64_t key =
      (((((int64_t)g.b0 * 512 + g.nb) * 2 + (eot_stop ? 1 : 0)) * 2 + (m->trace_out ? 1 : 0)) * 2 +
       (m->group_kv(g) ? 1 : 0)) * 4 + m->range_tier();
  if (g.graph && g.graph_key == key) return WQ4_OK;
  if (g.graph) {
    (void)hipGraphExecDestroy(g.graph);
    g.graph = nullptr;
  }
  WA_WQ4(wq4_prepare_stream(m->device, g.st));  // split-K workspace exists before capture
  hipGraph_t gr;
  WA_HIP(hipStreamBeginCapture(g.st, hipStreamCaptureModeThreadLocal));
  wq4_status s = decode_step(m, g, eot_stop, g.st);
  hipError_t ce = hipStreamEndCapture(g.st, &gr);
  if (s != WQ4_OK) return s;
  if (ce != hipSuccess) return fail(WQ4_EHIP, std::string("graph capture: ") + hipGetErrorString(ce));
  ce = hipGraphInstantiate(&g.graph, gr, nullptr, nullptr, 0);
  (void)hipGraphDestroy(gr);
  if (ce != hipSuccess) return fail(WQ4_EHIP, std::string("graph instantiate: ") + hipGetErrorString(ce));
  g.graph_key = key;
  return WQ4_OK;
}

// Clips up to which a transcribe decodes over cross K / V caches
// (WA_XATTN_KV_CLIPS overrides; 0 = never; measured in DESIGN.md §4).
void kv_config(wa_model* m, int max_batch) {
  static const int small = [] {
    const char* e = getenv("WA_XATTN_KV_CLIPS");
    return e ? std::max(0, atoi(e)) : 8;
  }();
  m->kv_small = std::min(small, max_batch);
  m->kv_clips = m->kv_small;
}

// Range tier 2's workspaces (wq4_ffn_forward_ws): the encoder's B * T rows
// and 4 * B rows per decode group (prompts), allocated once.
wq4_status ensure_ffn_ws(wa_model* m) {
  if (m->ffn_ws) return WQ4_OK;
  const DecLayer& Ld = m->dec.front();
  const EncLayer& Le = m->enc.front();
  const size_t ne = wq4_ffn_workspace_bytes(Le.fc1, Le.fc2, (int64_t)m->bmax * m->cfg.n_audio_ctx);
  const size_t nd = wq4_ffn_workspace_bytes(Ld.fc1, Ld.fc2, (int64_t)m->bmax * 4);
  if (ne == 0 || nd == 0) return fail(WQ4_EINVAL, "FFN workspace size");
  // all or nothing: a partial failure releases what it got, so a later
  // tier-2 entry allocates (or fails) afresh instead of leaking the first set
  void* e = m->dev.alloc<uint8_t>(ne);
  bool ok = e != nullptr;
  for (DecGroup& g : m->groups) {
    g.ffn_ws = ok ? m->dev.alloc<uint8_t>(nd) : nullptr;
    ok = ok && g.ffn_ws != nullptr;
  }
  if (!ok) {
    m->dev.release(e);
    for (DecGroup& g : m->groups) {
      m->dev.release(g.ffn_ws);
      g.ffn_ws = nullptr;
      g.ffn_ws_bytes = 0;
    }
    return fail(WQ4_ENOMEM, "range tier 2: FFN workspace allocation failed");
  }
  for (DecGroup& g : m->groups) {
    g.ffn_ws_bytes = nd;
    m->bytes += nd;
  }
  m->ffn_ws = e;
  m->ffn_ws_bytes = ne;
  m->bytes += ne;
  return WQ4_OK;
}

// Number of decode groups for a batch (WA_DECODE_GROUPS overrides).
int decode_groups(int B) {
  static const int forced = [] {
    const char* env = getenv("WA_DECODE_GROUPS");
    return env ? atoi(env) : 0;
  }();
  int G = forced > 0 ? forced : (B >= 16 ? 2 : 1);
  if (G > kMaxGroups) G = kMaxGroups;
  if (G > B) G = B;
  return G;
}

}  // namespace

// ================================================================= C ABI ==
extern "C" {

const char* wa_last_error(void) { return g_err.c_str(); }

wq4_status wa_synth_uniform(uint64_t seed, const char* name, int64_t n, float lo, float hi, float* out) {
  if (!name || !out || n < 0) return fail(WQ4_EINVAL, "bad argument");
  synth_uniform(seed, name, n, lo, hi, out);
  return WQ4_OK;
}

wq4_status wa_model_create_synthetic_ex(int device, int variant, uint64_t seed, int max_batch, wq4_precision prec,
                                        int weight_type, wa_model** out) {
  if (!out) return fail(WQ4_EINVAL, "out is null");
  *out = nullptr;
  if (variant < 0 || variant > 2) return fail(WQ4_EINVAL, "unknown variant");
  if (max_batch < 1 || max_batch > 256) return fail(WQ4_EINVAL, "max_batch must be in [1, 256]");
  if (prec != WQ4_PREC_F16X2 && prec != WQ4_PREC_F16) return fail(WQ4_EINVAL, "unknown precision");
  if (weight_type != 0 && weight_type != 1) return fail(WQ4_EINVAL, "weight_type must be 0 (Q4_0) or 1 (F16)");
  WA_HIP(hipSetDevice(device));
  std::unique_ptr<wa_model> m(new wa_model());
  m->device = device;
  m->cfg = preset(variant);
  m->prec = prec;
  m->ns = prec == WQ4_PREC_F16 ? 1 : 2;
  m->bmax = max_batch;
  kv_config(m.get(), max_batch);
  m->wtype = weight_type;
  SynthSource src(seed);
  wq4_status s = build_model(m.get(), src);
  if (s != WQ4_OK) return s;
  s = build_ln_fold(m.get());
  if (s != WQ4_OK) return s;
  s = alloc_activations(m.get());
  if (s != WQ4_OK) return s;
  WA_HIP(hipStreamCreateWithFlags(&m->own_stream, hipStreamNonBlocking));
  WA_HIP(hipDeviceSynchronize());
  *out = m.release();
  return WQ4_OK;
}

wq4_status wa_model_create_synthetic(int device, int variant, uint64_t seed, int max_batch, wq4_precision prec,
                                     wa_model** out) {
  return wa_model_create_synthetic_ex(device, variant, seed, max_batch, prec, 0, out);
}

wq4_status wa_model_create_from_gguf(int device, const char* path, int variant, int max_batch, wq4_precision prec,
                                     wa_model** out) {
  if (!out || !path) return fail(WQ4_EINVAL, "null argument");
  *out = nullptr;
  if (variant < 0 || variant > 2) return fail(WQ4_EINVAL, "unknown variant");
  if (max_batch < 1 || max_batch > 256) return fail(WQ4_EINVAL, "max_batch must be in [1, 256]");
  if (prec != WQ4_PREC_F16X2 && prec != WQ4_PREC_F16) return fail(WQ4_EINVAL, "unknown precision");
  wa::GgufFile file;
  if (!file.open(path)) return fail(WQ4_EINVAL, "Failed to parse GGUF: " + file.error());
  WA_HIP(hipSetDevice(device));
  std::unique_ptr<wa_model> m(new wa_model());
  m->device = device;
  m->cfg = preset(variant);
  m->prec = prec;
  m->ns = prec == WQ4_PREC_F16 ? 1 : 2;
  m->bmax = max_batch;
  kv_config(m.get(), max_batch);
  const wa::GgufTensor* probe = file.find("encoder.blocks.0.attn.query.weight");
  m->wtype = probe && probe->type == wa::kGgmlF16 ? 1 : 0;  // an F16 checkpoint (config 5)
  GgufSource src(file);
  wq4_status s = build_model(m.get(), src);
  if (s != WQ4_OK) return s;
  s = build_ln_fold(m.get());
  if (s != WQ4_OK) return s;
  s = alloc_activations(m.get());
  if (s != WQ4_OK) return s;
  WA_HIP(hipStreamCreateWithFlags(&m->own_stream, hipStreamNonBlocking));
  WA_HIP(hipDeviceSynchronize());
  *out = m.release();
  return WQ4_OK;
}

void wa_model_destroy(wa_model* m) { delete m; }

wq4_status wa_gguf_open(const char* path, wa_gguf** out) {
  if (!path || !out) return fail(WQ4_EINVAL, "null argument");
  *out = nullptr;
  auto* f = new wa::GgufFile();
  if (!f->open(path)) {
    const std::string e = f->error();
    delete f;
    return fail(WQ4_EINVAL, "Failed to parse GGUF: " + e);
  }
  *out = reinterpret_cast<wa_gguf*>(f);
  return WQ4_OK;
}

void wa_gguf_close(wa_gguf* g) { delete reinterpret_cast<wa::GgufFile*>(g); }

int wa_gguf_version(const wa_gguf* g) { return g ? (int)reinterpret_cast<const wa::GgufFile*>(g)->version() : -1; }

int64_t wa_gguf_tensor_count(const wa_gguf* g) {
  return g ? (int64_t)reinterpret_cast<const wa::GgufFile*>(g)->tensors().size() : -1;
}

wq4_status wa_gguf_tensor_info(const wa_gguf* g, int64_t index, char* name, size_t name_cap, int* ndims,
                               uint64_t* dims, int* type, uint64_t* offset, uint64_t* nbytes) {
  if (!g) return fail(WQ4_EINVAL, "null gguf");
  const auto& ts = reinterpret_cast<const wa::GgufFile*>(g)->tensors();
  if (index < 0 || index >= (int64_t)ts.size()) return fail(WQ4_EINVAL, "tensor index out of range");
  const wa::GgufTensor& t = ts[(size_t)index];
  if (name && name_cap) {
    const size_t n = std::min(name_cap - 1, t.name.size());
    std::memcpy(name, t.name.data(), n);
    name[n] = 0;
  }
  if (ndims) *ndims = (int)t.dims.size();
  if (dims)
    for (size_t i = 0; i < t.dims.size(); ++i) dims[i] = t.dims[i];
  if (type) *type = (int)t.type;
  if (offset) *offset = t.offset;
  if (nbytes) *nbytes = t.nbytes();
  return WQ4_OK;
}

wq4_status wa_gguf_tensor_data(const wa_gguf* g, const char* name, uint8_t* out, size_t cap) {
  if (!g || !name || !out) return fail(WQ4_EINVAL, "null argument");
  const auto* f = reinterpret_cast<const wa::GgufFile*>(g);
  const wa::GgufTensor* t = f->find(name);
  if (!t) return fail(WQ4_EINVAL, std::string("Tensor '") + name + "' not found in GGUF");
  const uint8_t* p = f->data(*t);
  if (!p) return fail(WQ4_EINVAL, std::string("Tensor '") + name + "' data lies outside the file");
  if (cap < t->nbytes()) return fail(WQ4_ENOMEM, "output buffer too small");
  std::memcpy(out, p, t->nbytes());
  return WQ4_OK;
}

int wa_model_weight_type(const wa_model* m) { return m ? m->wtype : -1; }

wq4_status wa_model_config(const wa_model* m, int32_t* cfg) {
  if (!m || !cfg) return fail(WQ4_EINVAL, "null argument");
  const Config& c = m->cfg;
  const int32_t v[WA_CFG_COUNT] = {c.n_mels,       c.n_audio_ctx,  c.n_audio_state, c.n_audio_head,
                                   c.n_audio_layer, c.n_text_ctx,   c.n_text_state,  c.n_text_head,
                                   c.n_text_layer,  c.n_vocab,      c.n_lang};
  std::memcpy(cfg, v, sizeof(v));
  return WQ4_OK;
}

size_t wa_model_device_bytes(const wa_model* m) { return m ? m->bytes : 0; }

wq4_status wa_last_timings(const wa_model* m, float* out) {
  if (!m || !out) return fail(WQ4_EINVAL, "null argument");
  std::memcpy(out, m->timings, sizeof(m->timings));
  return WQ4_OK;
}

wq4_status wa_profile_enable(wa_model* m, int enable) {
  if (!m) return fail(WQ4_EINVAL, "null model");
  m->profile = enable != 0;
  return WQ4_OK;
}

wq4_status wa_profile_read(wa_model* m, double* out, int reset) {
  if (!m || !out) return fail(WQ4_EINVAL, "null argument");
  m->resolve_profile();
  std::memcpy(out, m->prof, sizeof(m->prof));
  if (reset) std::memset(m->prof, 0, sizeof(m->prof));
  return WQ4_OK;
}

wq4_status wa_encode(wa_model* m, const float* mel_dev, int n_clips, float* enc_out_dev, void* stream) {
  if (!m || !mel_dev) return fail(WQ4_EINVAL, "null argument");
  if (n_clips < 1 || n_clips > m->bmax) return fail(WQ4_EINVAL, "n_clips out of range");
  WA_HIP(hipSetDevice(m->device));
  hipStream_t st = static_cast<hipStream_t>(stream);
  wq4_status s = encoder_forward(m, mel_dev, n_clips, st, enc_out_dev);
  if (s != WQ4_OK) return s;
  return cross_kv_forward(m, n_clips, st, false);
}

wq4_status wa_prompt_logits(wa_model* m, const int32_t* prompt_dev, int n_clips, int plen, float* logits_dev,
                            void* stream) {
  if (!m || !prompt_dev || !logits_dev) return fail(WQ4_EINVAL, "null argument");
  if (n_clips < 1 || n_clips > m->bmax || plen < 1 || plen > 4) return fail(WQ4_EINVAL, "bad n_clips / plen");
  if (n_clips > m->kv_batch) return fail(WQ4_EINVAL, "wa_encode the clips first");
  WA_HIP(hipSetDevice(m->device));
  hipStream_t st = static_cast<hipStream_t>(stream);
  DecGroup& g = m->groups[0];
  g.b0 = 0;
  g.nb = n_clips;
  wq4_status s = decoder_forward(m, g, prompt_dev, plen, nullptr, 0, 0, st);
  if (s != WQ4_OK) return s;
  WA_HIP(hipMemcpyAsync(logits_dev, g.logits, (size_t)n_clips * m->cfg.n_vocab * 4, hipMemcpyDeviceToDevice, st));
  return WQ4_OK;
}

}  // extern "C"

namespace {

// HIP events destroyed with the set.
struct EventSet {
  std::vector<hipEvent_t> e;
  EventSet() = default;
  EventSet(const EventSet&) = delete;
  EventSet& operator=(const EventSet&) = delete;
  ~EventSet() {
    for (hipEvent_t x : e) (void)hipEventDestroy(x);
  }
  hipError_t make(hipEvent_t* out, bool timing = true) {
    hipError_t r = hipEventCreateWithFlags(out, timing ? hipEventDefault : hipEventDisableTiming);
    if (r == hipSuccess) e.push_back(*out);
    return r;
  }
};

// Prompt + greedy loop (whisper.rs:60-125) of every decode group of a batch
// of B clips, each group's stream first waiting on `ready` (the encoder
// planes of the batch).  Records gprompt[i] after group i's prompt and
// gdone[i] after its last step; the host blocks only for the lagged EOT
// polls (eot_stop).
wq4_status run_decode(wa_model* m, int B, int lang_token, int max_tokens, int eot_stop, hipEvent_t ready,
                      const hipEvent_t* gprompt, const hipEvent_t* gdone, int* steps_out) {
  const int G = decode_groups(B);
  for (int i = 0; i < G; ++i) {
    DecGroup& g = m->groups[i];
    g.b0 = (int)((int64_t)B * i / G);
    g.nb = (int)((int64_t)B * (i + 1) / G) - g.b0;
    WA_HIP(hipStreamWaitEvent(g.st, ready, 0));
    wq4_status s = prompt_group(m, g, lang_token, g.st);
    if (s != WQ4_OK) return s;
    WA_HIP(hipEventRecord(gprompt[i], g.st));
    s = ensure_graph(m, g, eot_stop);
    if (s != WQ4_OK) return s;
  }
  // greedy loop (whisper.rs:104-125): each step replays every live group's
  // graph; a group stops once all its clips emitted EOT (polled with a lag)
  EventSet ev;
  hipEvent_t ring[kMaxGroups][8];
  if (eot_stop)
    for (int i = 0; i < G; ++i)
      for (auto& e : ring[i]) WA_HIP(ev.make(&e, false));
  int steps = 0;
  const int lag = 4;
  bool live[kMaxGroups] = {};
  int nlive = G;
  for (int i = 0; i < G; ++i) live[i] = true;
  for (int step = 0; step < max_tokens && nlive > 0; ++step) {
    for (int i = 0; i < G; ++i) {
      if (!live[i]) continue;
      DecGroup& g = m->groups[i];
      WA_HIP(hipGraphLaunch(g.graph, g.st));
      if (eot_stop) {
        const int slot = step % 8;
        WA_HIP(hipMemcpyAsync(&g.host_ndone[slot], &g.state->n_done, sizeof(int), hipMemcpyDeviceToHost, g.st));
        WA_HIP(hipEventRecord(ring[i][slot], g.st));
      }
    }
    ++steps;
    if (eot_stop && step >= lag) {
      const int old = (step - lag) % 8;
      for (int i = 0; i < G; ++i) {
        if (!live[i]) continue;
        WA_HIP(hipEventSynchronize(ring[i][old]));
        if (m->groups[i].host_ndone[old] >= m->groups[i].nb) {  // every clip had emitted EOT by then
          live[i] = false;
          --nlive;
        }
      }
    }
  }
  // the loop's bookkeeping for tokens chosen by the last step happens at the
  // top of a step that the reference never runs: nothing to add.
  for (int i = 0; i < G; ++i) WA_HIP(hipEventRecord(gdone[i], m->groups[i].st));
  *steps_out = steps;
  return WQ4_OK;
}

// `st` waits for every group of the batch, then copies the groups' tokens /
// counts (kMaxTokens per clip) and the range flag to (pinned) host memory.
wq4_status collect_batch(wa_model* m, int B, const hipEvent_t* gdone, hipStream_t st, int32_t* tok, int32_t* nt,
                         int* flag) {
  const int G = decode_groups(B);
  for (int i = 0; i < G; ++i) WA_HIP(hipStreamWaitEvent(st, gdone[i], 0));
  for (int i = 0; i < G; ++i) {
    const DecGroup& g = m->groups[i];
    WA_HIP(hipMemcpyAsync(tok + (size_t)g.b0 * kMaxTokens, g.tokens, (size_t)g.nb * kMaxTokens * 4,
                          hipMemcpyDeviceToHost, st));
    WA_HIP(hipMemcpyAsync(nt + g.b0, g.ntok, (size_t)g.nb * 4, hipMemcpyDeviceToHost, st));
  }
  WA_HIP(hipMemcpyAsync(flag, m->range_flag, sizeof(int), hipMemcpyDeviceToHost, st));
  return WQ4_OK;
}

void copy_tokens(const int32_t* tok, const int32_t* nt, int B, int max_tokens, int32_t* tokens_out,
                 int32_t* n_tokens_out) {
  for (int b = 0; b < B; ++b) {
    n_tokens_out[b] = std::min(nt[b], max_tokens);
    std::memcpy(tokens_out + (size_t)b * max_tokens, tok + (size_t)b * kMaxTokens, (size_t)max_tokens * 4);
  }
}

// One transcribe (whisper.rs:51-128 for a batch of clips); *overflow = the
// range flag of this run (see wa_model::range_flag).
wq4_status transcribe_once(wa_model* m, const float* mel_dev, int n_clips, int lang_token, int max_tokens,
                           int eot_stop, int32_t* tokens_out, int32_t* n_tokens_out, void* stream, bool* overflow) {
  // all work on the model's own stream, ordered after the caller's stream
  hipStream_t st = m->own_stream;
  const int B = n_clips;
  const int G = decode_groups(B);
  EventSet ev;
  hipEvent_t e_in, e_enc, e_kv, e_ready, e_end, gprompt[kMaxGroups], gdone[kMaxGroups];
  for (hipEvent_t* e : {&e_in, &e_enc, &e_kv, &e_ready, &e_end}) WA_HIP(ev.make(e));
  for (int i = 0; i < G; ++i) {
    WA_HIP(ev.make(&gprompt[i]));
    WA_HIP(ev.make(&gdone[i]));
  }
  WA_HIP(hipEventRecord(e_in, static_cast<hipStream_t>(stream)));
  WA_HIP(hipStreamWaitEvent(st, e_in, 0));
  WA_HIP(hipMemsetAsync(m->range_flag, 0, sizeof(int), st));

  WA_HIP(hipEventRecord(e_enc, st));
  wq4_status s = encoder_forward(m, mel_dev, B, st, nullptr);
  if (s != WQ4_OK) return s;
  WA_HIP(hipEventRecord(e_kv, st));
  s = cross_kv_forward(m, B, st, true);
  if (s != WQ4_OK) return s;
  WA_HIP(hipEventRecord(e_ready, st));
  // decode groups: contiguous clip ranges on their own streams, started
  // after the encoder-planes pass, joined back into `st` at the end
  int steps = 0;
  s = run_decode(m, B, lang_token, max_tokens, eot_stop, e_ready, gprompt, gdone, &steps);
  if (s != WQ4_OK) return s;
  std::vector<int32_t> tok((size_t)B * kMaxTokens), nt(B);
  int flag = 0;
  s = collect_batch(m, B, gdone, st, tok.data(), nt.data(), &flag);
  if (s != WQ4_OK) return s;
  WA_HIP(hipEventRecord(e_end, st));
  WA_HIP(hipStreamSynchronize(st));
  *overflow = flag != 0;
  copy_tokens(tok.data(), nt.data(), B, max_tokens, tokens_out, n_tokens_out);
  // phases: encoder, encoder planes (the cross-attention state), prompt (slowest group), decode loop
  float t_enc = 0.0f, t_kv = 0.0f, tp = 0.0f, tall = 0.0f;
  WA_HIP(hipEventElapsedTime(&t_enc, e_enc, e_kv));
  WA_HIP(hipEventElapsedTime(&t_kv, e_kv, e_ready));
  for (int i = 0; i < G; ++i) {
    float t = 0.0f;
    WA_HIP(hipEventElapsedTime(&t, e_ready, gprompt[i]));
    tp = std::max(tp, t);
  }
  WA_HIP(hipEventElapsedTime(&tall, e_ready, e_end));
  m->timings[0] = t_enc;
  m->timings[1] = t_kv;
  m->timings[2] = tp;
  m->timings[3] = tall - tp;
  m->timings[4] = (float)steps;
  return WQ4_OK;
}

// The CU-masked stream of the pipelined transcribe's overlapped encoder
// part: bits 0 .. n-1 of the mask, which the driver spreads over the XCDs
// (bit i -> XCD i mod 8), n / 8 CUs of each; created on first use.
wq4_status ensure_enc_stream(wa_model* m) {
  if (m->enc_stream) return WQ4_OK;
  hipDeviceProp_t prop;
  WA_HIP(hipGetDeviceProperties(&prop, m->device));
  const int total = prop.multiProcessorCount;
  int n = kEncOverlapCUs;
  if (const char* e = getenv("WA_ENC_CUS")) n = atoi(e);
  n = std::max(8, std::min(total, n));
  std::vector<uint32_t> mask((total + 31) / 32, 0u);
  for (int i = 0; i < n; ++i) mask[i / 32] |= 1u << (i % 32);
  WA_HIP(hipExtStreamCreateWithCUMask(&m->enc_stream, (uint32_t)mask.size(), mask.data()));
  m->enc_cus = n;
  return WQ4_OK;
}

// wa_transcribe over n_batches batches of n_clips clips, software-pipelined:
// while batch i decodes (its groups' streams), the conv stem and the first
// k encoder layers of batch i + 1 run on the CU-masked stream (a few CUs of
// every XCD; the decode keeps the rest), and once batch i's decode is done
// the remaining layers, ln_post and the encoder planes of batch i + 1 run
// at full width on the model stream.  The encoder buffers are free during a
// decode (it reads only the planes, rewritten after the decode it serves),
// so nothing is double-buffered.  k adapts per batch to the last decode's
// length over the masked stream's measured time per layer.  Every kernel
// computes what it computes in wa_transcribe: the same tokens.  flags[i] =
// batch i's range flag (the caller re-runs flagged batches).
wq4_status transcribe_pipelined(wa_model* m, const float* mel_dev, int NB, int B, int lang_token, int max_tokens,
                                int eot_stop, int32_t* tokens_out, int32_t* n_tokens_out, void* stream, int* flags) {
  WA_WQ4(ensure_enc_stream(m));
  hipStream_t st = m->own_stream, es = m->enc_stream;
  const int L = (int)m->enc.size(), G = decode_groups(B);
  const size_t mel_stride = (size_t)B * m->cfg.n_mels * 2 * m->cfg.n_audio_ctx;
  // pinned result staging: per batch the groups' tokens, counts and range flag
  int32_t* host = nullptr;
  const size_t per = (size_t)B * kMaxTokens + B + 1;
  WA_HIP(hipHostMalloc(reinterpret_cast<void**>(&host), (size_t)NB * per * 4, 0));
  struct HostGuard {  // an early error return may leave copies into `p` queued: drain this model's streams first
    wa_model* m;
    int32_t* p;
    bool done = false;  // success: the model stream was synchronised after the last copy
    ~HostGuard() {
      if (!done) {
        (void)hipStreamSynchronize(m->own_stream);
        if (m->enc_stream) (void)hipStreamSynchronize(m->enc_stream);
        for (DecGroup& g : m->groups)
          if (g.st) (void)hipStreamSynchronize(g.st);
      }
      (void)hipHostFree(p);
    }
  } hg{m, host};
  EventSet ev;
  struct Batch {
    hipEvent_t ready, mstart, mend, pstart, gprompt[kMaxGroups], gdone[kMaxGroups];
    int k = 0, steps = 0;
  };
  std::vector<Batch> bt(NB);
  for (Batch& b : bt) {
    for (hipEvent_t* e : {&b.ready, &b.mstart, &b.mend, &b.pstart}) WA_HIP(ev.make(e));
    for (int i = 0; i < G; ++i) {
      WA_HIP(ev.make(&b.gprompt[i]));
      WA_HIP(ev.make(&b.gdone[i]));
    }
  }
  hipEvent_t e_in, e_enc0;
  WA_HIP(ev.make(&e_in));
  WA_HIP(ev.make(&e_enc0));
  WA_HIP(hipEventRecord(e_in, static_cast<hipStream_t>(stream)));
  WA_HIP(hipStreamWaitEvent(st, e_in, 0));
  // batch 0: the whole encoder at full width
  WA_HIP(hipEventRecord(e_enc0, st));
  wq4_status s = encoder_forward(m, mel_dev, B, st, nullptr);
  if (s == WQ4_OK) s = cross_kv_forward(m, B, st, true);
  if (s != WQ4_OK) return s;
  WA_HIP(hipMemsetAsync(m->range_flag, 0, sizeof(int), st));
  WA_HIP(hipEventRecord(bt[0].ready, st));
  // the adapted depth belongs to a batch shape: a call with another clip
  // count or EOT mode starts again from the default
  if (m->overlap_k < 0 || m->overlap_b != B || m->overlap_eot != eot_stop) m->overlap_k = std::min(L, kEncOverlapLayers0);
  m->overlap_b = B;
  m->overlap_eot = eot_stop;
  double t_exposed = 0.0, t_masked = 0.0, t_decode = 0.0, t_prompt = 0.0, k_sum = 0.0;
  int32_t steps_all = 0;
  for (int i = 0; i < NB; ++i) {
    Batch& b = bt[i];
    if (i >= 1) {
      // batch i - 1 is decoded (and batch i's masked part done) before batch
      // i's decode is enqueued: the GPU meanwhile runs batch i's remaining
      // layers; adapt k to the finished decode
      Batch& p = bt[i - 1];
      for (int g = 0; g < G; ++g) WA_HIP(hipEventSynchronize(p.gdone[g]));
      WA_HIP(hipEventSynchronize(p.mend));
      float td = 0.0f, tm = 0.0f;
      for (int g = 0; g < G; ++g) {
        float t = 0.0f;
        WA_HIP(hipEventElapsedTime(&t, p.ready, p.gdone[g]));
        td = std::max(td, t);
      }
      WA_HIP(hipEventElapsedTime(&tm, p.mstart, p.mend));
      if (!getenv("WA_ENC_OVERLAP")) {
        const double per_layer = tm / (double)(p.k + 1);  // the conv stem counts as one layer
        double fill = kEncOverlapFill;
        if (const char* e = getenv("WA_ENC_FILL")) fill = atof(e);  // A/B only
        m->overlap_k = std::max(0, std::min(L, (int)(fill * td / per_layer) - 1));
      }
    }
    if (const char* e = getenv("WA_ENC_OVERLAP")) m->overlap_k = std::max(0, std::min(L, atoi(e)));
    if (i + 1 < NB) {  // the masked part of batch i + 1, beside batch i's decode
      b.k = m->overlap_k;
      WA_HIP(hipStreamWaitEvent(es, b.ready, 0));
      WA_HIP(hipEventRecord(b.mstart, es));
      s = encoder_front(m, mel_dev + (i + 1) * mel_stride, B, es);
      if (s == WQ4_OK) s = encoder_layers(m, B, 0, b.k, es);
      if (s != WQ4_OK) return s;
      WA_HIP(hipEventRecord(b.mend, es));
    }
    s = run_decode(m, B, lang_token, max_tokens, eot_stop, b.ready, b.gprompt, b.gdone, &b.steps);
    if (s != WQ4_OK) return s;
    int32_t* hb = host + (size_t)i * per;
    s = collect_batch(m, B, b.gdone, st, hb, hb + (size_t)B * kMaxTokens, hb + (size_t)B * kMaxTokens + B);
    if (s != WQ4_OK) return s;
    if (i + 1 < NB) {  // the rest of batch i + 1's encoder at full width
      WA_HIP(hipStreamWaitEvent(st, b.mend, 0));
      WA_HIP(hipEventRecord(b.pstart, st));
      s = encoder_layers(m, B, b.k, L, st);
      if (s == WQ4_OK) s = encoder_post(m, B, st, nullptr);
      if (s == WQ4_OK) s = cross_kv_forward(m, B, st, true);
      if (s != WQ4_OK) return s;
      WA_HIP(hipMemsetAsync(m->range_flag, 0, sizeof(int), st));
      WA_HIP(hipEventRecord(bt[i + 1].ready, st));
    }
  }
  WA_HIP(hipStreamSynchronize(st));
  hg.done = true;
  for (int i = 0; i < NB; ++i) {
    const int32_t* hb = host + (size_t)i * per;
    copy_tokens(hb, hb + (size_t)B * kMaxTokens, B, max_tokens, tokens_out + (size_t)i * B * max_tokens,
                n_tokens_out + (size_t)i * B);
    flags[i] = hb[(size_t)B * kMaxTokens + B];
    // per-batch phases (averaged below)
    Batch& b = bt[i];
    float t = 0.0f, tp = 0.0f, td = 0.0f;
    if (i == 0) {
      WA_HIP(hipEventElapsedTime(&t, e_enc0, b.ready));
    } else {
      WA_HIP(hipEventElapsedTime(&t, bt[i - 1].pstart, b.ready));
      float tm = 0.0f;
      WA_HIP(hipEventElapsedTime(&tm, bt[i - 1].mstart, bt[i - 1].mend));
      t_masked += tm;
      k_sum += bt[i - 1].k;
    }
    t_exposed += t;
    for (int g = 0; g < G; ++g) {
      float a = 0.0f, d = 0.0f;
      WA_HIP(hipEventElapsedTime(&a, b.ready, b.gprompt[g]));
      WA_HIP(hipEventElapsedTime(&d, b.ready, b.gdone[g]));
      tp = std::max(tp, a);
      td = std::max(td, d);
    }
    t_prompt += tp;
    t_decode += td - tp;
    steps_all += b.steps;
  }
  m->timings[0] = (float)(t_exposed / NB);
  m->timings[1] = 0.0f;
  m->timings[2] = (float)(t_prompt / NB);
  m->timings[3] = (float)(t_decode / NB);
  m->timings[4] = (float)steps_all / NB;
  m->pipe[0] = (float)NB;
  m->pipe[1] = NB > 1 ? (float)(k_sum / (NB - 1)) : 0.0f;
  m->pipe[2] = NB > 1 ? (float)(t_masked / (NB - 1)) : 0.0f;
  m->pipe[3] = (float)m->enc_cus;
  return WQ4_OK;
}

}  // namespace

extern "C" {

wq4_status wa_transcribe(wa_model* m, const float* mel_dev, int n_clips, int lang_token, int max_tokens,
                         int eot_stop, int32_t* tokens_out, int32_t* n_tokens_out, void* stream) {
  if (!m || !mel_dev || !tokens_out || !n_tokens_out) return fail(WQ4_EINVAL, "null argument");
  if (n_clips < 1 || n_clips > m->bmax) return fail(WQ4_EINVAL, "n_clips out of range");
  if (max_tokens < 1 || max_tokens > kMaxTokens) return fail(WQ4_EINVAL, "max_tokens must be in [1, 224]");
  WA_HIP(hipSetDevice(m->device));
  bool overflow = false;
  wq4_status s = transcribe_once(m, mel_dev, n_clips, lang_token, max_tokens, eot_stop, tokens_out, n_tokens_out,
                                 stream, &overflow);
  if (s != WQ4_OK) return s;
  if (overflow && !m->wide_range) {
    // the LayerNorm fold feeds the raw residual stream to the MFMAs: retry on
    // the LayerNorm path, and keep it for this model (sticky: its activations
    // evidently exceed the fold's range)
    m->wide_range = true;
    s = transcribe_once(m, mel_dev, n_clips, lang_token, max_tokens, eot_stop, tokens_out, n_tokens_out, stream,
                        &overflow);
    if (s != WQ4_OK) return s;
  }
  if (overflow && !m->wide_ffn) {
    // the FFN hidden layer (fc1 + GELU) feeds fc2 unnormalised: retry with
    // every FFN on per-call operand scales (sticky, like tier 1)
    s = ensure_ffn_ws(m);
    if (s != WQ4_OK) return s;
    m->wide_ffn = true;
    s = transcribe_once(m, mel_dev, n_clips, lang_token, max_tokens, eot_stop, tokens_out, n_tokens_out, stream,
                        &overflow);
    if (s != WQ4_OK) return s;
  }
  if (overflow && !m->wide_attn) {
    // an attention output feeds its output projection unnormalised: retry
    // with f32 attention outputs and per-call operand scales on those
    // projections (sticky; needs tier 2's workspaces, already allocated)
    m->wide_attn = true;
    s = transcribe_once(m, mel_dev, n_clips, lang_token, max_tokens, eot_stop, tokens_out, n_tokens_out, stream,
                        &overflow);
    if (s != WQ4_OK) return s;
  }
  if (overflow)
    return fail(WQ4_ERANGE,
                "activation overflow: an MFMA operand left the f16-pair range (|x| >= 4094 after every range tier: "
                "LayerNorm path, per-call FFN and attention-projection operand scales) and the logits are not finite");
  return WQ4_OK;
}

wq4_status wa_transcribe_batches(wa_model* m, const float* mel_dev, int n_batches, int n_clips, int lang_token,
                                 int max_tokens, int eot_stop, int32_t* tokens_out, int32_t* n_tokens_out,
                                 void* stream) {
  if (!m || !mel_dev || !tokens_out || !n_tokens_out) return fail(WQ4_EINVAL, "null argument");
  if (n_batches < 1) return fail(WQ4_EINVAL, "n_batches must be >= 1");
  if (n_clips < 1 || n_clips > m->bmax) return fail(WQ4_EINVAL, "n_clips out of range");
  if (max_tokens < 1 || max_tokens > kMaxTokens) return fail(WQ4_EINVAL, "max_tokens must be in [1, 224]");
  WA_HIP(hipSetDevice(m->device));
  std::vector<int> flags(n_batches, 0);
  wq4_status s = transcribe_pipelined(m, mel_dev, n_batches, n_clips, lang_token, max_tokens, eot_stop, tokens_out,
                                      n_tokens_out, stream, flags.data());
  if (s != WQ4_OK) return s;
  const size_t mel_stride = (size_t)n_clips * m->cfg.n_mels * 2 * m->cfg.n_audio_ctx;
  // the pipeline decoded every batch at the tier the model had on entry
  const int tier0 = m->range_tier();
  for (int i = 0; i < n_batches; ++i) {
    // a flagged batch goes through wa_transcribe's range tiers on its own;
    // once that raised the (sticky) tier, the later batches are re-run at it
    // too -- one wa_transcribe per batch would have decoded them there
    if (!flags[i] && m->range_tier() == tier0) continue;
    s = wa_transcribe(m, mel_dev + i * mel_stride, n_clips, lang_token, max_tokens, eot_stop,
                      tokens_out + (size_t)i * n_clips * max_tokens, n_tokens_out + (size_t)i * n_clips, stream);
    if (s != WQ4_OK) return s;
  }
  return WQ4_OK;
}

wq4_status wa_last_pipeline_stats(const wa_model* m, float* out) {
  if (!m || !out) return fail(WQ4_EINVAL, "null argument");
  std::memcpy(out, m->pipe, sizeof(m->pipe));
  return WQ4_OK;
}

int wa_model_wide_range(const wa_model* m) { return m ? m->range_tier() : -1; }

wq4_status wa_transcribe_trace(wa_model* m, const float* mel_dev, int n_clips, int lang_token, int max_tokens,
                               int eot_stop, int32_t* tokens_out, int32_t* n_tokens_out, const int32_t* trace_ids_dev,
                               int trace_k, float* trace_out_dev, void* stream) {
  if (!m || !trace_ids_dev || !trace_out_dev || trace_k < 1) return fail(WQ4_EINVAL, "bad trace arguments");
  m->trace_ids = trace_ids_dev;
  m->trace_out = trace_out_dev;
  m->trace_s1 = max_tokens + 1;
  m->trace_k = trace_k;
  const wq4_status s = wa_transcribe(m, mel_dev, n_clips, lang_token, max_tokens, eot_stop, tokens_out,
                                     n_tokens_out, stream);
  m->trace_ids = nullptr;
  m->trace_out = nullptr;
  m->trace_s1 = m->trace_k = 0;
  for (DecGroup& g : m->groups) {  // the trace graphs bake in the caller's buffers: never replay them again
    if (g.graph) (void)hipGraphExecDestroy(g.graph);
    g.graph = nullptr;
    g.graph_key = -1;
  }
  return s;
}

int wa_decode_group_rows(int n_clips) {
  if (n_clips < 1) return 0;
  const int G = decode_groups(n_clips);
  return (n_clips + G - 1) / G;  // the largest group (groups split [0, B) evenly, transcribe_batch)
}

constexpr int kProbeOut = WA_PROBE_OUT;

wq4_status wa_probe_kernels(wa_model* m, int n_clips, int iters, double* out, int out_len) {
  if (!m || !out) return fail(WQ4_EINVAL, "null argument");
  if (out_len < kProbeOut) return fail(WQ4_EINVAL, "out holds fewer than 6 doubles");
  if (n_clips < 1 || n_clips > m->bmax || iters < 1) return fail(WQ4_EINVAL, "bad n_clips / iters");
  if (n_clips > m->kv_batch) return fail(WQ4_EINVAL, "run wa_transcribe / wa_encode on n_clips clips first");
  WA_HIP(hipSetDevice(m->device));
  hipStream_t st = m->own_stream;
  const Config& c = m->cfg;
  const int B = n_clips, D = c.n_text_state, T = c.n_audio_ctx, H = c.n_text_head;
  DecLayer& L = m->dec[0];
  DecGroup g = m->groups[0];  // group 0's buffers, a clip range of its own
  const _Float16* enc = m->enc_planes;
  hipEvent_t a, b;
  WA_HIP(hipEventCreate(&a));
  WA_HIP(hipEventCreate(&b));
  float ms = 0.0f;
  // cross-attention of one decode step (Tq = 1) in the form a decode group of
  // n_clips clips runs: over the cached K / V (few clips) or streaming every
  // clip's encoder output
  g.b0 = 0;
  g.nb = B;
  const bool kv = m->group_kv(g);
  auto xattn = [&]() -> hipError_t {
    if (kv)
      return wa::launch_cross_attention_kv(g.qd, L.xk, L.xv, B, 1, T, H, g.xkv_part, g.xkv_ctr, g.atd_dec, m->ns, st);
    return wa::launch_xattn(g.qd, L.ck_raw, L.cv_raw, L.cv_p, L.cv_b, m->wtype, enc, B, 1, T, H, D, g.xqt,
                            g.xattn_part, g.atd_dec, m->ns, st);
  };
  WA_HIP(xattn());
  WA_HIP(hipEventRecord(a, st));
  for (int i = 0; i < iters; ++i) WA_HIP(xattn());
  WA_HIP(hipEventRecord(b, st));
  WA_HIP(hipEventSynchronize(b));
  WA_HIP(hipEventElapsedTime(&ms, a, b));
  out[0] = ms * 1e3 / iters;
  // algorithmic bytes: the cached K and V (f32) of every clip, or the
  // encoder output planes of every clip + Wk, Wv (raw); + q + output operand
  const double wbytes = m->wtype == 1 ? 2.0 * D * D * 2 : 2.0 * D * D * 18 / 32;
  out[1] = kv ? (double)B * T * D * 4 * 2 + (double)B * D * (4 + 2 * m->ns)
              : (double)B * T * D * 2 * m->ns + wbytes + (double)B * D * (4 + 2 * m->ns);
  out[5] = kv ? 1.0 : 0.0;
  // fc1 of one decode step (M = n_clips rows, decode kernel, GELU + tiled out)
  const int F = 4 * D;
  WA_WQ4(wq4_gemm_tiled(L.fc1, L.fc1_b, g.atd_dec, nullptr, nullptr, g.atf_dec, B, WQ4_EPI_GELU | WQ4_EPI_TILED_OUT,
                        m->prec, 2, st));
  WA_HIP(hipEventRecord(a, st));
  for (int i = 0; i < iters; ++i)
    WA_WQ4(wq4_gemm_tiled(L.fc1, L.fc1_b, g.atd_dec, nullptr, nullptr, g.atf_dec, B,
                          WQ4_EPI_GELU | WQ4_EPI_TILED_OUT, m->prec, 2, st));
  WA_HIP(hipEventRecord(b, st));
  WA_HIP(hipEventSynchronize(b));
  WA_HIP(hipEventElapsedTime(&ms, a, b));
  out[2] = ms * 1e3 / iters;
  out[3] = (double)F * D * 18 / 32 + (double)B * D * 2 * m->ns + (double)B * F * 2 * m->ns;
  out[4] = 2.0 * B * F * D;
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return WQ4_OK;
}

wq4_status wa_xattn_check(int device, const float* q_dev, const uint8_t* wk_dev, const uint8_t* wv_dev,
                          const float* bv_dev, int weight_type, const float* enc_dev, int n_clips, int Tq, int T,
                          int H, wq4_precision prec, float* out_dev) {
  if (!q_dev || !wk_dev || !wv_dev || !bv_dev || !enc_dev || !out_dev) return fail(WQ4_EINVAL, "null argument");
  if (n_clips < 1 || Tq < 1 || T < 1 || H < 1) return fail(WQ4_EINVAL, "bad sizes");
  const int D = 64 * H, ns = prec == WQ4_PREC_F16 ? 1 : 2, R = n_clips * Tq;
  const int HP = (H + 15) / 16 * 16;
  WA_HIP(hipSetDevice(device));
  Dev d;
  auto* planes = d.alloc<_Float16>((size_t)n_clips * T * ns * D);
  auto* qt = d.alloc<_Float16>((size_t)R * ns * HP * D);
  auto* part = d.alloc<float>(wa::xattn_part_floats(R, H, D, T));
  const size_t tb = wq4_atiled_bytes(R, D, prec);
  auto* tiled = d.alloc<_Float16>(tb / 2);
  if (!planes || !qt || !part || !tiled) return fail(WQ4_ENOMEM, "allocation failed");
  WA_HIP(hipMemset(qt, 0, (size_t)R * ns * HP * D * 2));
  WA_HIP(hipMemset(tiled, 0, tb));
  WA_HIP(wa::launch_enc_planes(enc_dev, (int64_t)n_clips * T, D, ns, planes, nullptr));
  uint32_t* wvp = nullptr;
  if (weight_type == 0) {
    wvp = d.alloc<uint32_t>(wa::wv_pack_words(H, D));
    if (!wvp) return fail(WQ4_ENOMEM, "allocation failed");
    WA_HIP(wa::launch_wv_pack(wv_dev, H, D, wvp, nullptr));
  }
  WA_HIP(wa::launch_xattn(q_dev, wk_dev, wv_dev, wvp, bv_dev, weight_type, planes, n_clips, Tq, T, H, D, qt, part,
                          tiled, ns, nullptr));
  WA_HIP(wa::launch_untile(tiled, R, D, ns, out_dev, nullptr));
  WA_HIP(hipDeviceSynchronize());
  return WQ4_OK;
}

wq4_status wa_xattn_kv_check(int device, const float* q_dev, const float* k_dev, const float* v_dev, int n_clips,
                             int Tq, int T, int H, wq4_precision prec, float* out_dev) {
  if (!q_dev || !k_dev || !v_dev || !out_dev) return fail(WQ4_EINVAL, "null argument");
  if (n_clips < 1 || Tq < 1 || Tq > 4 || T < 1 || H < 1) return fail(WQ4_EINVAL, "bad sizes");
  const int D = 64 * H, ns = prec == WQ4_PREC_F16 ? 1 : 2, R = n_clips * Tq;
  WA_HIP(hipSetDevice(device));
  Dev d;
  auto* part = d.alloc<float>(wa::cross_attention_kv_part_floats(n_clips, H, T));
  auto* ctr = d.alloc<int>((size_t)n_clips * H);
  const size_t tb = wq4_atiled_bytes(R, D, prec);
  auto* tiled = d.alloc<_Float16>(tb / 2);
  if (!part || !ctr || !tiled) return fail(WQ4_ENOMEM, "allocation failed");
  WA_HIP(hipMemset(ctr, 0, (size_t)n_clips * H * sizeof(int)));
  WA_HIP(hipMemset(tiled, 0, tb));
  WA_HIP(wa::launch_cross_attention_kv(q_dev, k_dev, v_dev, n_clips, Tq, T, H, part, ctr, tiled, ns, nullptr));
  WA_HIP(wa::launch_untile(tiled, R, D, ns, out_dev, nullptr));
  WA_HIP(hipDeviceSynchronize());
  return WQ4_OK;
}

wq4_status wa_encoder_attention_check(int device, const float* qkv_dev, int n_clips, int T, int H, wq4_precision prec,
                                      float* out_dev) {
  if (!qkv_dev || !out_dev) return fail(WQ4_EINVAL, "null argument");
  if (n_clips < 1 || T < 1 || H < 1) return fail(WQ4_EINVAL, "bad sizes");
  const int D = 64 * H, ns = prec == WQ4_PREC_F16 ? 1 : 2;
  const int64_t R = (int64_t)n_clips * T;
  WA_HIP(hipSetDevice(device));
  Dev d;
  const size_t tb = wq4_atiled_bytes(R, D, prec);
  auto* tiled = d.alloc<_Float16>(tb / 2);
  if (!tiled) return fail(WQ4_ENOMEM, "allocation failed");
  WA_HIP(hipMemset(tiled, 0, tb));
  WA_HIP(wa::launch_encoder_attention(qkv_dev, n_clips, T, H, tiled, ns, nullptr));
  WA_HIP(wa::launch_untile(tiled, (int)R, D, ns, out_dev, nullptr));
  WA_HIP(hipDeviceSynchronize());
  return WQ4_OK;
}

wq4_status wa_self_attention_check(int device, const float* qkv_dev, float* cache_k_dev, float* cache_v_dev,
                                   int n_clips, int Tq, int H, int ctx, int kv_len, wq4_precision prec,
                                   float* out_dev) {
  if (!qkv_dev || !cache_k_dev || !cache_v_dev || !out_dev) return fail(WQ4_EINVAL, "null argument");
  if (n_clips < 1 || Tq < 1 || Tq > 4 || H < 1 || ctx < 1 || ctx > 448 || kv_len < 0 || kv_len + Tq > ctx)
    return fail(WQ4_EINVAL, "bad sizes");
  const int D = 64 * H, ns = prec == WQ4_PREC_F16 ? 1 : 2, R = n_clips * Tq;
  WA_HIP(hipSetDevice(device));
  Dev d;
  const size_t tb = wq4_atiled_bytes(R, D, prec);
  auto* tiled = d.alloc<_Float16>(tb / 2);
  if (!tiled) return fail(WQ4_ENOMEM, "allocation failed");
  WA_HIP(hipMemset(tiled, 0, tb));
  WA_HIP(wa::launch_decoder_self_attention(qkv_dev, cache_k_dev, cache_v_dev, n_clips, Tq, H, ctx, nullptr, kv_len,
                                           tiled, ns, nullptr));
  WA_HIP(wa::launch_untile(tiled, R, D, ns, out_dev, nullptr));
  WA_HIP(hipDeviceSynchronize());
  return WQ4_OK;
}

wq4_status wa_logits_argmax_check(int device, const float* hid_dev, const float* emb_dev, int n_clips, int D, int V,
                                  int step, wq4_precision prec, int32_t* tok_dev, float* logits_dev) {
  if (!hid_dev || !emb_dev || !tok_dev) return fail(WQ4_EINVAL, "null argument");
  if (n_clips < 1 || n_clips > 32 || V < 1 || !wa::emb_tiled_supported(D)) return fail(WQ4_EINVAL, "bad sizes");
  const int ns = prec == WQ4_PREC_F16 ? 1 : 2;
  WA_HIP(hipSetDevice(device));
  Dev d;
  const int64_t erows = wa::emb_tiled_rows(V);
  const int ng = wa::logits_argmax_groups(V);
  auto* emb2 = d.alloc<_Float16>((size_t)erows * ns * D);
  auto* st = d.alloc<wa::DecodeState>(1);
  auto* pval = d.alloc<float>((size_t)32 * ng);
  auto* pidx = d.alloc<int>((size_t)32 * ng);
  auto* ctr = d.alloc<int>(1);
  const size_t tb = wq4_atiled_bytes(n_clips, D, prec);
  auto* ht = d.alloc<_Float16>(tb / 2);
  int* ids = nullptr;
  if (logits_dev) ids = d.alloc<int>((size_t)n_clips * 2 * V);
  if (!emb2 || !st || !pval || !pidx || !ctr || !ht || (logits_dev && !ids))
    return fail(WQ4_ENOMEM, "allocation failed");
  WA_HIP(wa::launch_emb_tiled(emb_dev, V, D, ns, emb2, nullptr));
  WA_WQ4(wq4_tile_activations(hid_dev, n_clips, D, D, prec, ht, tb, nullptr));
  // A trace writes slot state->step + 1 of [clip][2][V] (every id listed at
  // slot 1): the state's step is then 0 and the EOT suppression of `step`
  // (step + 1 < 3, whisper.rs:120-122) is passed through min_tokens instead.
  const wa::DecodeState s0{0, 0, logits_dev ? 0 : step, 0};
  const int min_tokens = !logits_dev ? kMinTokens : (step + 1 < kMinTokens ? 1 << 30 : 0);
  WA_HIP(hipMemcpy(st, &s0, sizeof(s0), hipMemcpyHostToDevice));
  WA_HIP(hipMemset(ctr, 0, sizeof(int)));
  float* tr = nullptr;
  if (logits_dev) {
    std::vector<int> h((size_t)n_clips * 2 * V, 0);
    for (int b = 0; b < n_clips; ++b)
      for (int v = 0; v < V; ++v) h[((size_t)b * 2 + 1) * V + v] = v;
    WA_HIP(hipMemcpy(ids, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    tr = d.alloc<float>((size_t)n_clips * 2 * V);
    if (!tr) return fail(WQ4_ENOMEM, "allocation failed");
  }
  WA_HIP(wa::launch_logits_argmax(ht, n_clips, D, emb2, ns, V, min_tokens, st, pval, pidx, ctr, tok_dev,
                                  ids, tr, 2, V, nullptr, nullptr));
  if (logits_dev)
    for (int b = 0; b < n_clips; ++b)
      WA_HIP(hipMemcpy(logits_dev + (size_t)b * V, tr + ((size_t)b * 2 + 1) * V, (size_t)V * 4,
                       hipMemcpyDeviceToDevice));
  WA_HIP(hipDeviceSynchronize());
  return WQ4_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- log-mel --
// Per-device constants (window, filterbank, twiddles; per n_mels) and the
// per-workgroup-max scratch, allocated on first use outside stream capture.
namespace {
struct MelDevice {
  std::map<int, uint8_t*> consts;
  float* part = nullptr;
  int part_clips = 0;
};
std::mutex g_mel_mu;
std::map<int, MelDevice> g_mel;
}  // namespace

extern "C" {

wq4_status wa_log_mel(int device, const float* audio_dev, int n_clips, int64_t n_samples, int64_t ld_audio,
                      int n_mels, float* mel_dev, void* stream) {
  if (!mel_dev || (!audio_dev && n_samples > 0)) return fail(WQ4_EINVAL, "null argument");
  if (n_clips < 1) return fail(WQ4_EINVAL, "n_clips must be >= 1");
  if (n_samples < 0 || ld_audio < n_samples) return fail(WQ4_EINVAL, "need 0 <= n_samples <= ld_audio");
  if (n_mels < 1 || n_mels > wa::kMelMaxMels) return fail(WQ4_EINVAL, "n_mels must be in [1, 256]");
  WA_HIP(hipSetDevice(device));
  hipStream_t st = static_cast<hipStream_t>(stream);
  std::lock_guard<std::mutex> lk(g_mel_mu);
  MelDevice& md = g_mel[device];
  uint8_t*& c = md.consts[n_mels];
  if (!c || md.part_clips < n_clips) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    WA_HIP(hipStreamIsCapturing(st, &cs));
    if (cs != hipStreamCaptureStatusNone)
      return fail(WQ4_EINVAL, "wa_log_mel: run once outside stream capture first (allocates constants)");
  }
  if (!c) {
    const wa::MelBank bank = wa::make_mel_bank(n_mels);
    std::vector<uint8_t> host(wa::mel_const_bytes(n_mels));
    wa::mel_pack_consts(bank, host.data());
    WA_HIP(hipMalloc(reinterpret_cast<void**>(&c), host.size()));
    WA_HIP(hipMemcpy(c, host.data(), host.size(), hipMemcpyHostToDevice));
  }
  if (md.part_clips < n_clips) {
    WA_HIP(hipDeviceSynchronize());
    if (md.part) WA_HIP(hipFree(md.part));
    md.part = nullptr;
    md.part_clips = 0;
    WA_HIP(hipMalloc(reinterpret_cast<void**>(&md.part), (size_t)n_clips * wa::kMelWgPerClip * sizeof(float)));
    md.part_clips = n_clips;
  }
  WA_HIP(wa::launch_log_mel(audio_dev, n_clips, n_samples, ld_audio, n_mels, c, md.part, mel_dev, st));
  return WQ4_OK;
}

wq4_status wa_mel_filterbank(int n_mels, float* filters_out, float* window_out) {
  if (n_mels < 1 || n_mels > wa::kMelMaxMels) return fail(WQ4_EINVAL, "n_mels must be in [1, 256]");
  const wa::MelBank bank = wa::make_mel_bank(n_mels);
  if (filters_out) std::memcpy(filters_out, bank.filters.data(), bank.filters.size() * sizeof(float));
  if (window_out) std::memcpy(window_out, bank.window.data(), bank.window.size() * sizeof(float));
  return WQ4_OK;
}

}  // extern "C"
