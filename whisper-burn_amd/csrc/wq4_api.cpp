// wq4_api.cpp -- C ABI (include/wq4.h) over the MI355X Q4_0 kernels.
//
// Mirrors the reference operator surface:
//   Q4Tensor::{from_q4_bytes, shape, num_blocks, dequantize}  src/gguf/tensor.rs
//   q4_matmul                                                 src/gguf/op.rs:47-117
//   Q4Linear::forward                                         src/gguf/linear.rs:34-40
//   Q4FFN::forward (+ gelu)                                   src/model/layers.rs:35-58
// Differences by design: no hidden per-call uploads (op.rs:67-70 uploads an
// info buffer and flushes the queue on every call), caller-owned outputs,
// status codes instead of panics.
#include <hip/hip_runtime_api.h>

#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "../../include/wq4.h"
#include "wq4_kernels.hpp"
#include "wq4_layout.hpp"

struct wq4_tensor {
  int device = 0;
  wq4::Q4Geom g;
  bool flat = false;         // K % 32 != 0: stored as raw blocks, no GEMM (see create)
  uint8_t* nib = nullptr;    // device, g.nib_bytes()
  uint32_t* sc = nullptr;    // device, g.sc_bytes()
  float* cs = nullptr;       // device, g.colscale_bytes()
  uint8_t* raw = nullptr;    // device, raw GGUF bytes (flat tensors only)
  size_t raw_bytes = 0;
  int wtype = 0;             // wq4::kWeightsQ4, or kWeightsF16 (nib = f16 fragments, sc unused, cs = 1)
  uint32_t* q16 = nullptr;   // device, the decode-step kernel's layout (wq4_skinny.hip): Q4 nibbles or f16s
  uint16_t* d16 = nullptr;   // device, its f16 block scales (Q4 only)
};

namespace {

thread_local std::string g_err;
std::atomic<int> g_prec{WQ4_PREC_F16X2};
// WQ4_KERNEL_POLICY initialises it (A/B runs of whole programs, e.g. bench.py);
// wq4_set_kernel_policy changes it at run time.
std::atomic<int> g_policy{[] {
  const char* env = getenv("WQ4_KERNEL_POLICY");
  const int v = env ? atoi(env) : 0;
  return v >= 0 && v <= 3 ? v : 0;
}()};

wq4_status fail(wq4_status s, const std::string& msg) {
  g_err = msg;
  return s;
}

wq4_status hip_fail(hipError_t e, const char* what) {
  return fail(WQ4_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

// RAII device switch (hipSetDevice is per host thread).
struct DeviceGuard {
  int prev = -1;
  bool ok = true;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// Grow-only workspace per (device, stream) for the convenience entry points.
struct Arena {
  void* ptr = nullptr;
  size_t bytes = 0;
};
std::mutex g_arena_mu;
std::map<std::pair<int, void*>, Arena> g_arenas;

wq4_status arena_get(int dev, void* stream, size_t need, void** out) {
  std::lock_guard<std::mutex> lk(g_arena_mu);
  Arena& a = g_arenas[{dev, stream}];
  if (a.bytes < need) {
    if (a.ptr) {
      // pending work on this stream may still read the old buffer
      hipError_t e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
      if (e != hipSuccess) return hip_fail(e, "arena sync");
      (void)hipFree(a.ptr);
      a.ptr = nullptr;
      a.bytes = 0;
    }
    size_t sz = need < ((size_t)1 << 20) ? ((size_t)1 << 20) : need;
    hipError_t e = hipMalloc(&a.ptr, sz);
    if (e != hipSuccess) return fail(WQ4_ENOMEM, std::string("workspace hipMalloc: ") + hipGetErrorString(e));
    a.bytes = sz;
  }
  *out = a.ptr;
  return WQ4_OK;
}

// Split-K workspace of the decode kernel per (device, stream); never freed
// (tiny, and kernels in flight or captured graphs may still reference it).
std::map<std::pair<int, void*>, wq4::DecodeWs> g_decode_ws;

wq4_status decode_ws_get(int dev, void* stream, const wq4::DecodeWs** out) {
  std::lock_guard<std::mutex> lk(g_arena_mu);
  auto it = g_decode_ws.find({dev, stream});
  if (it == g_decode_ws.end()) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(static_cast<hipStream_t>(stream), &cs) == hipSuccess &&
        cs != hipStreamCaptureStatusNone)
      return fail(WQ4_EINVAL,
                  "the first small-M GEMM on a stream must run outside graph capture (it allocates the split-K "
                  "workspace)");
    wq4::DecodeWs ws{nullptr, nullptr, nullptr};
    hipError_t e = hipMalloc(&ws.part, (size_t)wq4::kDecodeWsFloats * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&ws.act_scale, 32);  // two [scale, 1/scale, max bits] slots
    if (e == hipSuccess) e = hipMalloc(&ws.counters, (size_t)wq4::kDecodeMaxTiles * sizeof(int));
    if (e == hipSuccess)
      e = hipMemsetAsync(ws.counters, 0, (size_t)wq4::kDecodeMaxTiles * sizeof(int),
                         static_cast<hipStream_t>(stream));
    if (e != hipSuccess) {
      if (ws.part) (void)hipFree(ws.part);
      if (ws.counters) (void)hipFree(ws.counters);
      if (ws.act_scale) (void)hipFree(ws.act_scale);
      return fail(WQ4_ENOMEM, std::string("decode workspace: ") + hipGetErrorString(e));
    }
    it = g_decode_ws.emplace(std::make_pair(dev, stream), ws).first;
  }
  *out = &it->second;
  return WQ4_OK;
}

int ns_of(wq4_precision p) { return p == WQ4_PREC_F16 ? 1 : 2; }

bool use_decode(int64_t rows) {
  const int pol = g_policy.load();
  if (pol == 1) return false;
  if (pol == 2) return true;
  return rows <= 32 * wq4::kDecodeMaxMTiles;
}

wq4::EpiArgs make_epi(const float* bias, const float* residual, float* out, int ldo, int m, int n, bool gelu) {
  wq4::EpiArgs e{};
  e.bias = bias;
  e.residual = residual;
  e.out = out;
  e.out_tiled = nullptr;
  e.ldo = ldo;
  e.nbp_next = 0;
  e.gelu = gelu ? 1 : 0;
  e.m = m;
  e.n = n;
  return e;
}

wq4_status check_prec(wq4_precision p) {
  if (p != WQ4_PREC_F16X2 && p != WQ4_PREC_F16) return fail(WQ4_EINVAL, "unknown precision");
  return WQ4_OK;
}

wq4_status check_gemm_tensor(const wq4_tensor* w) {
  if (!w) return fail(WQ4_EINVAL, "weights are null");
  if (w->flat)  // the reference shader needs whole blocks per row (shader.wgsl:69)
    return fail(WQ4_ESHAPE, "q4_matmul needs K % 32 == 0, weights are [" + std::to_string(w->g.n) + ", " +
                                std::to_string(w->g.k) + "]");
  return WQ4_OK;
}

bool skinny_ok(const wq4_tensor* w, int64_t rows) {
  return w && w->q16 && wq4::skinny_supported(w->g, (int)rows);
}

// kernel 0 = by row count (<= 32 and a skinny layout: the decode-step kernel;
// <= 128: the 8-wave decode kernel; else the prefill tile kernel), 1 =
// prefill, 2 = decode, 3 = decode-step (skinny) kernel.
int pick_kernel(const wq4_tensor* w, int64_t rows, int kernel) {
  if (kernel != 0) return kernel;
  const int pol = g_policy.load();
  if (pol != 0) return pol == 3 && !skinny_ok(w, rows) ? 2 : pol;
  if (skinny_ok(w, rows)) return 3;
  return use_decode(rows) ? 2 : 1;
}

// The kernel of a LayerNorm-fold GEMM (16-column tile statistics, K <= 1280
// for a consumer): the 8-wave decode kernel (2) where its 8-wave plan applies
// -- in the model's decode step, two groups' chains run concurrently and its
// 40-160 workgroup grids left room for the other group's kernels: decode
// 875 ms against 905-914 ms with the decode-step kernel's 80-240 workgroups
// (Large-V3, 32 clips, bench A/B, r02) -- else the decode-step
// kernel (3), which policy 3 also forces; 0 = unsupported.
int lnfold_kernel(const wq4_tensor* w, int64_t rows) {
  if (!w || w->flat || rows < 1 || rows > 32) return 0;
  const bool old_ok = wq4::decode_ln_supported(w->g, (int)rows);
  if (g_policy.load() == 3) return skinny_ok(w, rows) ? 3 : 0;
  if (old_ok) return 2;
  return skinny_ok(w, rows) ? 3 : 0;
}

wq4_status gemm(const wq4_tensor* w, const _Float16* at, int64_t rows, const wq4::EpiArgs& e, int mode, int ns,
                hipStream_t st, bool dec, bool skinny = false) {
  if (skinny) {
    if (!skinny_ok(w, rows)) return fail(WQ4_ESHAPE, "the decode-step kernel needs rows <= 32, K % 128 == 0, N % 16 == 0");
    const wq4::DecodeWs* ws = nullptr;
    wq4_status s = decode_ws_get(w->device, st, &ws);
    if (s != WQ4_OK) return s;
    hipError_t he = wq4::launch_skinny_gemm(w->g, w->q16, w->d16, at, (int)rows, e, mode, ns, w->wtype, ws, st);
    if (he != hipSuccess) return hip_fail(he, "skinny gemm launch");
    return WQ4_OK;
  }
  const wq4::DecodeWs* ws = nullptr;
  if (dec) {
    wq4_status s = decode_ws_get(w->device, st, &ws);
    if (s != WQ4_OK) return s;
  }
  hipError_t he = wq4::launch_q4_gemm(w->g, w->nib, w->sc, w->cs, at, (int)rows, e, mode, ns, ws, st, w->wtype);
  if (he != hipSuccess) return hip_fail(he, "q4_gemm launch");
  return WQ4_OK;
}

}  // namespace

extern "C" {

const char* wq4_last_error(void) { return g_err.c_str(); }
int wq4_abi_version(void) { return WQ4_ABI_VERSION; }

wq4_status wq4_device_count(int* count) {
  if (!count) return fail(WQ4_EINVAL, "count is null");
  hipError_t e = hipGetDeviceCount(count);
  if (e != hipSuccess) {
    *count = 0;
    return hip_fail(e, "hipGetDeviceCount");
  }
  return WQ4_OK;
}

wq4_status wq4_set_precision(wq4_precision prec) {
  wq4_status s = check_prec(prec);
  if (s != WQ4_OK) return s;
  g_prec.store(prec);
  return WQ4_OK;
}

wq4_precision wq4_get_precision(void) { return static_cast<wq4_precision>(g_prec.load()); }

wq4_status wq4_set_kernel_policy(int policy) {
  if (policy < 0 || policy > 3) return fail(WQ4_EINVAL, "policy must be 0, 1, 2 or 3");
  g_policy.store(policy);
  return WQ4_OK;
}

const char* wq4_gemm_kernel_name(int64_t n, int64_t k, int64_t rows) {
  if (n < 1 || k < 32 || k % 32 != 0 || rows < 1) return "";
  const wq4::Q4Geom g = wq4::make_geom(n, k);
  // the decode-step layout exists for K % 128 == 0, N % 16 == 0 (upload)
  const bool skinny = k % 128 == 0 && n % 16 == 0 && wq4::skinny_supported(g, (int)rows);
  const int pol = g_policy.load();
  int kern = pol != 0 ? (pol == 3 && !skinny ? 2 : pol) : skinny ? 3 : use_decode(rows) ? 2 : 1;
  switch (kern) {
    case 3: return "skinny_gemm_kernel";
    case 2: return "q4_gemm_decode_kernel";
    default:
      switch (wq4::enc_gemm_pick(g, (int)rows, 0, g_prec.load() == WQ4_PREC_F16X2 ? 2 : 1, 0)) {
        case 0: return "q4_gemm_prefill_kernel";
        case 5: return "q4_gemm_wide_kernel";
        default: return "q4_gemm_enc_kernel";
      }
  }
}

// Q4Tensor::from_q4_bytes, src/gguf/tensor.rs:35-71.
wq4_status wq4_tensor_create(int device, const uint8_t* raw, size_t nbytes, int64_t n, int64_t k,
                             wq4_tensor** out) {
  return wq4_tensor_create_ex(device, raw, nbytes, n, k, 0u, out);
}

wq4_status wq4_tensor_create_ex(int device, const uint8_t* raw, size_t nbytes, int64_t n, int64_t k, unsigned flags,
                                wq4_tensor** out) {
  if (!out) return fail(WQ4_EINVAL, "out is null");
  *out = nullptr;
  if (n <= 0 || k <= 0)
    return fail(WQ4_ESHAPE, "Q4_0 shape must be positive, got [" + std::to_string(n) + ", " + std::to_string(k) + "]");
  const int64_t elems = n * k;
  if (elems % 32 != 0)  // tensor.rs:38-42
    return fail(WQ4_ESHAPE, "Q4_0 requires element count divisible by 32, got " + std::to_string(elems));
  const int64_t nblocks = elems / 32;
  const size_t expected = (size_t)nblocks * 18;
  if (nbytes != expected)  // tensor.rs:43-48
    return fail(WQ4_EBYTES, "Q4_0 byte count mismatch: expected " + std::to_string(expected) + " for " +
                                std::to_string(nblocks) + " blocks, got " + std::to_string(nbytes));
  if (!raw) return fail(WQ4_EINVAL, "raw is null");
  if (n > (1 << 24) || k > (1 << 24)) return fail(WQ4_ESHAPE, "dimension too large for this build (> 2^24)");

  DeviceGuard dg(device);
  if (!dg.ok) return fail(WQ4_EHIP, "hipSetDevice(" + std::to_string(device) + ") failed");
  auto* t = new wq4_tensor();
  t->device = device;
  t->g = wq4::make_geom(n, k);
  hipError_t e = hipSuccess;
  if (k % 32 != 0) {
    // Accepted like the reference (only N*K % 32 is checked, tensor.rs:38-42)
    // and kept as raw blocks: dequantize() works, GEMM entry points refuse.
    t->flat = true;
    t->raw_bytes = nbytes;
    e = hipMalloc(&t->raw, nbytes);
    if (e == hipSuccess) e = hipMemcpy(t->raw, raw, nbytes, hipMemcpyHostToDevice);
  } else {
    std::vector<uint8_t> nib(t->g.nib_bytes());
    std::vector<uint32_t> sc(t->g.sc_bytes() / 4);
    std::vector<float> cs(t->g.np);
    wq4::repack_q4(raw, t->g, nib.data(), sc.data(), cs.data());
    e = hipMalloc(&t->nib, nib.size());
    if (e == hipSuccess) e = hipMalloc(&t->sc, t->g.sc_bytes());
    if (e == hipSuccess) e = hipMalloc(&t->cs, t->g.colscale_bytes());
    if (e == hipSuccess) e = hipMemcpy(t->nib, nib.data(), nib.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(t->sc, sc.data(), t->g.sc_bytes(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(t->cs, cs.data(), t->g.colscale_bytes(), hipMemcpyHostToDevice);
    if (e == hipSuccess && k % 128 == 0 && n % 16 == 0 && !(flags & WQ4_TENSOR_NO_DECODE_STEP)) {
      // the decode-step kernel's layout
      std::vector<uint32_t> q16(wq4::skinny_q_bytes(t->g) / 4);
      std::vector<uint16_t> d16(wq4::skinny_d_bytes(t->g) / 2);
      wq4::repack_q4_skinny(raw, t->g, q16.data(), d16.data());
      e = hipMalloc(&t->q16, wq4::skinny_q_bytes(t->g));
      if (e == hipSuccess) e = hipMalloc(&t->d16, wq4::skinny_d_bytes(t->g));
      if (e == hipSuccess) e = hipMemcpy(t->q16, q16.data(), wq4::skinny_q_bytes(t->g), hipMemcpyHostToDevice);
      if (e == hipSuccess) e = hipMemcpy(t->d16, d16.data(), wq4::skinny_d_bytes(t->g), hipMemcpyHostToDevice);
    }
  }
  if (e != hipSuccess) {
    wq4_tensor_destroy(t);
    return hip_fail(e, "Q4Tensor upload");
  }
  *out = t;
  return WQ4_OK;
}

void wq4_tensor_destroy(wq4_tensor* t) {
  if (!t) return;
  DeviceGuard dg(t->device);
  if (t->nib) (void)hipFree(t->nib);
  if (t->sc) (void)hipFree(t->sc);
  if (t->cs) (void)hipFree(t->cs);
  if (t->raw) (void)hipFree(t->raw);
  if (t->q16) (void)hipFree(t->q16);
  if (t->d16) (void)hipFree(t->d16);
  delete t;
}

wq4_status wq4_tensor_shape(const wq4_tensor* t, int64_t* n, int64_t* k) {
  if (!t || !n || !k) return fail(WQ4_EINVAL, "null argument");
  *n = t->g.n;
  *k = t->g.k;
  return WQ4_OK;
}

int64_t wq4_tensor_num_blocks(const wq4_tensor* t) { return t ? t->g.n * t->g.k / 32 : -1; }
int wq4_tensor_device(const wq4_tensor* t) { return t ? t->device : -1; }
size_t wq4_tensor_device_bytes(const wq4_tensor* t) {
  if (!t) return 0;
  const size_t sk = !t->q16 ? 0 : t->wtype == wq4::kWeightsF16 ? wq4::skinny_f16_bytes(t->g)
                                                                : wq4::skinny_q_bytes(t->g) + wq4::skinny_d_bytes(t->g);
  if (t->wtype == wq4::kWeightsF16) return t->g.f16_frag_bytes() + t->g.colscale_bytes() + sk;
  return t->flat ? t->raw_bytes : t->g.nib_bytes() + t->g.sc_bytes() + t->g.colscale_bytes() + sk;
}

wq4_status wq4_tensor_create_f16(int device, const uint16_t* w, int64_t n, int64_t k, wq4_tensor** out) {
  return wq4_tensor_create_f16_ex(device, w, n, k, 0u, out);
}

int wq4_tensor_has_decode_step(const wq4_tensor* t) { return t && t->q16 ? 1 : 0; }

// The decode-step kernel keeps f16 weights as w * 2^8 (wq4_skinny.hip): only
// when that stays finite in f16 (|w| < 255.875).
static bool f16_skinny_in_range(const uint16_t* w, size_t count) {
  for (size_t i = 0; i < count; ++i) {
    const float v = std::fabs((float)__builtin_bit_cast(_Float16, w[i]));
    if (!(v * 256.0f <= 65504.0f)) return false;  // also rejects inf / NaN
  }
  return true;
}

wq4_status wq4_tensor_create_f16_ex(int device, const uint16_t* w, int64_t n, int64_t k, unsigned flags,
                                    wq4_tensor** out) {
  if (!out) return fail(WQ4_EINVAL, "out is null");
  *out = nullptr;
  if (n <= 0 || k <= 0 || k % 32 != 0)
    return fail(WQ4_ESHAPE, "F16 weights need n > 0 and k % 32 == 0, got [" + std::to_string(n) + ", " +
                                std::to_string(k) + "]");
  if (n > (1 << 24) || k > (1 << 24)) return fail(WQ4_ESHAPE, "dimension too large for this build (> 2^24)");
  if (!w) return fail(WQ4_EINVAL, "weights are null");
  DeviceGuard dg(device);
  if (!dg.ok) return fail(WQ4_EHIP, "hipSetDevice(" + std::to_string(device) + ") failed");
  auto* t = new wq4_tensor();
  t->device = device;
  t->g = wq4::make_geom(n, k);
  t->wtype = wq4::kWeightsF16;
  std::vector<uint16_t> frag(t->g.f16_frag_bytes() / 2);
  wq4::repack_f16(w, t->g, frag.data());
  std::vector<float> ones(t->g.np, 1.0f);
  hipError_t e = hipMalloc(&t->nib, t->g.f16_frag_bytes());
  if (e == hipSuccess) e = hipMalloc(&t->cs, t->g.colscale_bytes());
  if (e == hipSuccess) e = hipMemcpy(t->nib, frag.data(), t->g.f16_frag_bytes(), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(t->cs, ones.data(), t->g.colscale_bytes(), hipMemcpyHostToDevice);
  if (e == hipSuccess && k % 128 == 0 && n % 16 == 0 && !(flags & WQ4_TENSOR_NO_DECODE_STEP) &&
      f16_skinny_in_range(w, (size_t)(n * k))) {  // the decode-step kernel's layout
    std::vector<uint16_t> f16s(wq4::skinny_f16_bytes(t->g) / 2);
    wq4::repack_f16_skinny(w, t->g, f16s.data());
    e = hipMalloc(&t->q16, wq4::skinny_f16_bytes(t->g));
    if (e == hipSuccess) e = hipMemcpy(t->q16, f16s.data(), wq4::skinny_f16_bytes(t->g), hipMemcpyHostToDevice);
  }
  if (e != hipSuccess) {
    wq4_tensor_destroy(t);
    return hip_fail(e, "F16 weight upload");
  }
  *out = t;
  return WQ4_OK;
}

int wq4_tensor_weight_type(const wq4_tensor* t) { return t ? t->wtype : -1; }

wq4_status wq4_tensor_raw_bytes(const wq4_tensor* t, uint8_t* host_out) {
  if (!t || !host_out) return fail(WQ4_EINVAL, "null argument");
  DeviceGuard dg(t->device);
  if (t->wtype == wq4::kWeightsF16) {  // the f16 [N, K] halves as given
    std::vector<uint16_t> frag(t->g.f16_frag_bytes() / 2);
    hipError_t e = hipMemcpy(frag.data(), t->nib, t->g.f16_frag_bytes(), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return hip_fail(e, "F16 weight read-back");
    wq4::unrepack_f16(frag.data(), t->g, reinterpret_cast<uint16_t*>(host_out));
    return WQ4_OK;
  }
  if (t->flat) {
    hipError_t e = hipMemcpy(host_out, t->raw, t->raw_bytes, hipMemcpyDeviceToHost);
    return e == hipSuccess ? WQ4_OK : hip_fail(e, "Q4Tensor read-back");
  }
  std::vector<uint8_t> nib(t->g.nib_bytes());
  std::vector<uint32_t> sc(t->g.sc_bytes() / 4);
  std::vector<float> cs(t->g.np);
  hipError_t e = hipMemcpy(nib.data(), t->nib, nib.size(), hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(sc.data(), t->sc, t->g.sc_bytes(), hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(cs.data(), t->cs, t->g.colscale_bytes(), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return hip_fail(e, "Q4Tensor read-back");
  wq4::unrepack_q4(nib.data(), sc.data(), cs.data(), t->g, host_out);
  return WQ4_OK;
}

static float f16_to_f32_host(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }

// Q4Tensor::dequantize, src/gguf/tensor.rs:88-113 (D2H, then host dequant).
wq4_status wq4_tensor_dequantize(const wq4_tensor* t, float* host_out) {
  if (!t || !host_out) return fail(WQ4_EINVAL, "null argument");
  if (t->wtype == wq4::kWeightsF16) {
    std::vector<uint16_t> h((size_t)(t->g.n * t->g.k));
    wq4_status s = wq4_tensor_raw_bytes(t, reinterpret_cast<uint8_t*>(h.data()));
    if (s != WQ4_OK) return s;
    for (size_t i = 0; i < h.size(); ++i) host_out[i] = f16_to_f32_host(h[i]);
    return WQ4_OK;
  }
  const int64_t nb = t->g.n * t->g.k / 32;
  std::vector<uint8_t> raw((size_t)nb * 18);
  wq4_status s = wq4_tensor_raw_bytes(t, raw.data());
  if (s != WQ4_OK) return s;
  for (int64_t b = 0; b < nb; ++b) {
    const uint8_t* o = raw.data() + b * 18;
    const float d = f16_to_f32_host((uint16_t)(o[0] | (o[1] << 8)));
    float* dst = host_out + b * 32;
    for (int i = 0; i < 16; ++i) {
      const float lo = (float)(o[2 + i] & 0x0f) - 8.0f;
      const float hi = (float)((o[2 + i] >> 4) & 0x0f) - 8.0f;
      dst[i] = lo * d;
      dst[i + 16] = hi * d;
    }
  }
  return WQ4_OK;
}

size_t wq4_linear_workspace_bytes(const wq4_tensor* w, int64_t rows) {
  if (!w || w->flat) return 0;
  return wq4::atiled_bytes(rows, w->g.k, 2);
}

// fc1's operand, fc2's operand and the f32 fc1 output between them.
static size_t ffn_ws_bytes(const wq4_tensor* fc1, const wq4_tensor* fc2, int64_t rows, int ns) {
  return wq4::atiled_bytes(rows, fc1->g.k, ns) + wq4::atiled_bytes(rows, fc2->g.k, ns) +
         (size_t)rows * (size_t)fc1->g.n * sizeof(float);
}

size_t wq4_ffn_workspace_bytes(const wq4_tensor* fc1, const wq4_tensor* fc2, int64_t rows) {
  if (!fc1 || !fc2 || fc1->flat || fc2->flat || rows < 0) return 0;
  return ffn_ws_bytes(fc1, fc2, rows, 2);
}

static wq4_status linear_impl(const wq4_tensor* w, const float* bias, const float* x, const float* residual,
                              float* y, int64_t rows, int64_t k, unsigned flags, wq4_precision prec, void* ws,
                              size_t ws_bytes, void* stream) {
  wq4_status s = check_gemm_tensor(w);
  if (s != WQ4_OK) return s;
  s = check_prec(prec);
  if (s != WQ4_OK) return s;
  if (k != w->g.k)  // op.rs:58-61
    return fail(WQ4_ESHAPE, "K dimension mismatch: input has " + std::to_string(k) + ", weights have " +
                                std::to_string(w->g.k));
  if (rows < 0 || rows > (1 << 24)) return fail(WQ4_ESHAPE, "bad row count " + std::to_string(rows));
  if (rows == 0) return WQ4_OK;  // empty batch: nothing to read or write
  if (!x || !y) return fail(WQ4_EINVAL, "null activation / output pointer");
  if ((flags & WQ4_EPI_RESIDUAL) && !residual) return fail(WQ4_EINVAL, "WQ4_EPI_RESIDUAL without residual");
  const int ns = ns_of(prec);
  const size_t need = wq4::atiled_bytes(rows, k, ns);
  if (!ws || ws_bytes < need) return fail(WQ4_ENOMEM, "workspace too small: need " + std::to_string(need) + " bytes");
  DeviceGuard dg(w->device);
  if (!dg.ok) return fail(WQ4_EHIP, "hipSetDevice failed");
  hipStream_t st = static_cast<hipStream_t>(stream);
  auto* at = static_cast<_Float16*>(ws);
  // the reference API takes any f32 input: the operand scale is chosen per
  // call from max |x| (device-side, stream-ordered)
  const wq4::DecodeWs* dws = nullptr;
  s = decode_ws_get(w->device, st, &dws);
  if (s != WQ4_OK) return s;
  hipError_t e = wq4::launch_act_scale(x, (int)rows, (int)k, (int)k, dws->act_scale, st);
  if (e == hipSuccess) e = wq4::launch_tile_activations(x, at, (int)rows, (int)k, (int)k, ns, st, dws->act_scale);
  if (e != hipSuccess) return hip_fail(e, "tile_activations launch");
  wq4::EpiArgs epi = make_epi(bias, (flags & WQ4_EPI_RESIDUAL) ? residual : nullptr, y, (int)w->g.n, (int)rows,
                              (int)w->g.n, (flags & WQ4_EPI_GELU) != 0);
  epi.act_inv = dws->act_scale + 1;
  const int kk = pick_kernel(w, rows, 0);
  return gemm(w, at, rows, epi, wq4::kEpiF32, ns, st, kk == 2, kk == 3);
}

wq4_status wq4_linear_forward_ws(const wq4_tensor* w, const float* bias_dev, const float* x_dev,
                                 const float* residual_dev, float* y_dev, int64_t rows, int64_t k, unsigned flags,
                                 wq4_precision prec, void* workspace, size_t ws_bytes, void* stream) {
  return linear_impl(w, bias_dev, x_dev, residual_dev, y_dev, rows, k, flags, prec, workspace, ws_bytes, stream);
}

wq4_status wq4_linear_forward(const wq4_tensor* w, const float* bias_dev, const float* x_dev, float* y_dev,
                              int64_t b, int64_t m, int64_t k, void* stream) {
  wq4_status s = check_gemm_tensor(w);
  if (s != WQ4_OK) return s;
  if (b < 0 || m < 0) return fail(WQ4_ESHAPE, "negative B or M");
  const int64_t rows = b * m;
  const wq4_precision prec = wq4_get_precision();
  void* ws = nullptr;
  const size_t need = wq4::atiled_bytes(rows, k > 0 ? k : 32, ns_of(prec));
  if (rows > 0 && k == w->g.k) {
    DeviceGuard dg(w->device);
    s = arena_get(w->device, stream, need, &ws);
    if (s != WQ4_OK) return s;
  }
  return linear_impl(w, bias_dev, x_dev, nullptr, y_dev, rows, k, 0u, prec, ws, need, stream);
}

// q4_matmul, src/gguf/op.rs:47-117.
wq4_status wq4_matmul(const wq4_tensor* w, const float* x_dev, float* y_dev, int64_t b, int64_t m, int64_t k,
                      void* stream) {
  return wq4_linear_forward(w, nullptr, x_dev, y_dev, b, m, k, stream);
}

static wq4_status ffn_impl(const wq4_tensor* fc1, const float* b1, const wq4_tensor* fc2, const float* b2,
                           const float* x, const float* residual, float* y, int64_t rows, unsigned flags,
                           wq4_precision prec, void* ws, size_t ws_bytes, void* stream) {
  wq4_status s = check_gemm_tensor(fc1);
  if (s == WQ4_OK) s = check_gemm_tensor(fc2);
  if (s != WQ4_OK) return s;
  s = check_prec(prec);
  if (s != WQ4_OK) return s;
  if (fc1->device != fc2->device) return fail(WQ4_EINVAL, "fc1 and fc2 live on different devices");
  if (fc2->g.k != fc1->g.n)
    return fail(WQ4_ESHAPE, "FFN shape mismatch: fc1 is [" + std::to_string(fc1->g.n) + ", " +
                                std::to_string(fc1->g.k) + "], fc2 is [" + std::to_string(fc2->g.n) + ", " +
                                std::to_string(fc2->g.k) + "]");
  if (rows < 0 || rows > (1 << 24)) return fail(WQ4_ESHAPE, "bad row count");
  if (rows == 0) return WQ4_OK;
  if (!x || !y) return fail(WQ4_EINVAL, "null activation / output pointer");
  if ((flags & WQ4_EPI_RESIDUAL) && !residual) return fail(WQ4_EINVAL, "WQ4_EPI_RESIDUAL without residual");
  const int ns = ns_of(prec);
  const size_t n1 = wq4::atiled_bytes(rows, fc1->g.k, ns);
  const size_t n2 = wq4::atiled_bytes(rows, fc2->g.k, ns);
  const size_t need = ffn_ws_bytes(fc1, fc2, rows, ns);
  if (!ws || ws_bytes < need) return fail(WQ4_ENOMEM, "workspace too small: need " + std::to_string(need));
  DeviceGuard dg(fc1->device);
  if (!dg.ok) return fail(WQ4_EHIP, "hipSetDevice failed");
  hipStream_t st = static_cast<hipStream_t>(stream);
  auto* a1 = static_cast<_Float16*>(ws);
  auto* a2 = reinterpret_cast<_Float16*>(static_cast<uint8_t*>(ws) + n1);
  auto* h = reinterpret_cast<float*>(static_cast<uint8_t*>(ws) + n1 + n2);
  const wq4::DecodeWs* dws = nullptr;
  s = decode_ws_get(fc1->device, st, &dws);
  if (s != WQ4_OK) return s;
  // Each GEMM's A operand is scaled by a power of two picked from ITS input's
  // max |x| (device-side, stream-ordered), so any finite f32 input and any
  // finite gelu(fc1 x) stay finite -- the reference's f32 path has no range
  // limit below FLT_MAX either.  fc1 + bias + GELU go to f32 first.
  const int n1c = (int)fc1->g.n;
  hipError_t e = wq4::launch_act_scale(x, (int)rows, (int)fc1->g.k, (int)fc1->g.k, dws->act_scale, st);
  if (e == hipSuccess)
    e = wq4::launch_tile_activations(x, a1, (int)rows, (int)fc1->g.k, (int)fc1->g.k, ns, st, dws->act_scale);
  if (e != hipSuccess) return hip_fail(e, "tile_activations launch");
  wq4::EpiArgs e1 = make_epi(b1, nullptr, h, n1c, (int)rows, n1c, true);
  e1.act_inv = dws->act_scale + 1;
  const int k1 = pick_kernel(fc1, rows, 0), k2 = pick_kernel(fc2, rows, 0);
  wq4_status s1 = gemm(fc1, a1, rows, e1, wq4::kEpiF32, ns, st, k1 == 2, k1 == 3);
  if (s1 != WQ4_OK) return s1;
  // fc2's operand scale lives in the second half of the act-scale words
  // (fc1's may still be read by its launch: stream order keeps them apart,
  // but a separate slot keeps the two scales independent for inspection)
  float* sc2 = dws->act_scale + 4;
  e = wq4::launch_act_scale(h, (int)rows, n1c, n1c, sc2, st);
  if (e == hipSuccess) e = wq4::launch_tile_activations(h, a2, (int)rows, n1c, n1c, ns, st, sc2);
  if (e != hipSuccess) return hip_fail(e, "tile_activations launch (fc2 operand)");
  wq4::EpiArgs e2 = make_epi(b2, (flags & WQ4_EPI_RESIDUAL) ? residual : nullptr, y, (int)fc2->g.n, (int)rows,
                             (int)fc2->g.n, (flags & WQ4_EPI_GELU) != 0);
  e2.act_inv = sc2 + 1;
  return gemm(fc2, a2, rows, e2, wq4::kEpiF32, ns, st, k2 == 2, k2 == 3);
}

wq4_status wq4_ffn_forward_ws(const wq4_tensor* fc1, const float* b1_dev, const wq4_tensor* fc2,
                              const float* b2_dev, const float* x_dev, const float* residual_dev, float* y_dev,
                              int64_t rows, unsigned flags, wq4_precision prec, void* workspace, size_t ws_bytes,
                              void* stream) {
  return ffn_impl(fc1, b1_dev, fc2, b2_dev, x_dev, residual_dev, y_dev, rows, flags, prec, workspace, ws_bytes,
                  stream);
}

// Q4FFN::forward, src/model/layers.rs:54-58.
wq4_status wq4_ffn_forward(const wq4_tensor* fc1, const float* b1_dev, const wq4_tensor* fc2,
                           const float* b2_dev, const float* x_dev, float* y_dev, int64_t b, int64_t m,
                           void* stream) {
  wq4_status s = check_gemm_tensor(fc1);
  if (s == WQ4_OK) s = check_gemm_tensor(fc2);
  if (s != WQ4_OK) return s;
  if (b < 0 || m < 0) return fail(WQ4_ESHAPE, "negative B or M");
  const int64_t rows = b * m;
  const wq4_precision prec = wq4_get_precision();
  const int ns = ns_of(prec);
  const size_t need = ffn_ws_bytes(fc1, fc2, rows, ns);
  void* ws = nullptr;
  if (rows > 0) {
    DeviceGuard dg(fc1->device);
    s = arena_get(fc1->device, stream, need, &ws);
    if (s != WQ4_OK) return s;
  }
  return ffn_impl(fc1, b1_dev, fc2, b2_dev, x_dev, nullptr, y_dev, rows, 0u, prec, ws, need, stream);
}

size_t wq4_atiled_bytes(int64_t rows, int64_t k, wq4_precision prec) {
  if (rows < 0 || k <= 0 || k % 32 != 0) return 0;
  return wq4::atiled_bytes(rows, k, ns_of(prec));
}

wq4_status wq4_tile_activations(const float* x_dev, int64_t rows, int64_t k, int64_t ld, wq4_precision prec,
                                void* at_dev, size_t at_bytes, void* stream) {
  wq4_status s = check_prec(prec);
  if (s != WQ4_OK) return s;
  if (rows < 0 || rows > (1 << 24) || k <= 0 || k % 32 != 0 || ld < k) return fail(WQ4_ESHAPE, "bad activation shape");
  if (!x_dev || !at_dev) return fail(WQ4_EINVAL, "null argument");
  if (at_bytes < wq4::atiled_bytes(rows, k, ns_of(prec))) return fail(WQ4_ENOMEM, "A-tiled buffer too small");
  hipError_t e = wq4::launch_tile_activations(x_dev, static_cast<_Float16*>(at_dev), (int)rows, (int)k, (int)ld,
                                              ns_of(prec), static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "tile_activations launch");
  return WQ4_OK;
}

wq4_status wq4_linear_forward_tiled(const wq4_tensor* w, const float* bias_dev, const void* at_dev,
                                    const float* residual_dev, float* y_dev, int64_t rows, unsigned flags,
                                    wq4_precision prec, void* stream) {
  wq4_status s = check_gemm_tensor(w);
  if (s != WQ4_OK) return s;
  s = check_prec(prec);
  if (s != WQ4_OK) return s;
  if (rows < 0 || rows > (1 << 24)) return fail(WQ4_ESHAPE, "bad row count");
  if (rows == 0) return WQ4_OK;
  if (!at_dev || !y_dev) return fail(WQ4_EINVAL, "null argument");
  if ((flags & WQ4_EPI_RESIDUAL) && !residual_dev) return fail(WQ4_EINVAL, "WQ4_EPI_RESIDUAL without residual");
  DeviceGuard dg(w->device);
  wq4::EpiArgs epi = make_epi(bias_dev, (flags & WQ4_EPI_RESIDUAL) ? residual_dev : nullptr, y_dev, (int)w->g.n,
                              (int)rows, (int)w->g.n, (flags & WQ4_EPI_GELU) != 0);
  return gemm(w, static_cast<const _Float16*>(at_dev), rows, epi, wq4::kEpiF32, ns_of(prec),
              static_cast<hipStream_t>(stream), pick_kernel(w, rows, 0) == 2, pick_kernel(w, rows, 0) == 3);
}

wq4_status wq4_linear_forward_tiled_out(const wq4_tensor* w, const float* bias_dev, const void* at_dev,
                                        void* at_out_dev, size_t at_out_bytes, int64_t rows, unsigned flags,
                                        wq4_precision prec, void* stream) {
  wq4_status s = check_gemm_tensor(w);
  if (s != WQ4_OK) return s;
  s = check_prec(prec);
  if (s != WQ4_OK) return s;
  if (flags & WQ4_EPI_RESIDUAL) return fail(WQ4_EUNSUPPORTED, "residual with a tiled output");
  if (rows < 0 || rows > (1 << 24)) return fail(WQ4_ESHAPE, "bad row count");
  if (w->g.n % 32 != 0) return fail(WQ4_ESHAPE, "tiled output needs N % 32 == 0");
  if (rows == 0) return WQ4_OK;
  if (!at_dev || !at_out_dev) return fail(WQ4_EINVAL, "null argument");
  if (at_out_bytes < wq4::atiled_bytes(rows, w->g.n, ns_of(prec)))
    return fail(WQ4_ENOMEM, "A-tiled output buffer too small");
  DeviceGuard dg(w->device);
  wq4::EpiArgs epi = make_epi(bias_dev, nullptr, nullptr, (int)w->g.n, (int)rows, (int)w->g.n,
                              (flags & WQ4_EPI_GELU) != 0);
  epi.out_tiled = static_cast<_Float16*>(at_out_dev);
  epi.nbp_next = (int)((w->g.n / 32 + 1) / 2);
  return gemm(w, static_cast<const _Float16*>(at_dev), rows, epi, wq4::kEpiTiled, ns_of(prec),
              static_cast<hipStream_t>(stream), pick_kernel(w, rows, 0) == 2, pick_kernel(w, rows, 0) == 3);
}

wq4_status wq4_gemm_tiled(const wq4_tensor* w, const float* bias_dev, const void* at_dev, const float* residual_dev,
                          float* y_dev, void* at_out_dev, int64_t rows, unsigned flags, wq4_precision prec,
                          int kernel, void* stream) {
  wq4_status s = check_gemm_tensor(w);
  if (s != WQ4_OK) return s;
  s = check_prec(prec);
  if (s != WQ4_OK) return s;
  if (kernel < 0 || kernel > 3) return fail(WQ4_EINVAL, "kernel must be 0, 1, 2 or 3");
  if (rows < 0 || rows > (1 << 24)) return fail(WQ4_ESHAPE, "bad row count");
  if (rows == 0) return WQ4_OK;
  const bool tiled_out = (flags & WQ4_EPI_TILED_OUT) != 0;
  if (!at_dev || (tiled_out ? !at_out_dev : !y_dev)) return fail(WQ4_EINVAL, "null argument");
  if ((flags & WQ4_EPI_RESIDUAL) && (!residual_dev || tiled_out))
    return fail(WQ4_EINVAL, "WQ4_EPI_RESIDUAL needs a residual and an f32 output");
  if (tiled_out && w->g.n % 32 != 0) return fail(WQ4_ESHAPE, "tiled output needs N % 32 == 0");
  DeviceGuard dg(w->device);
  wq4::EpiArgs epi = make_epi(bias_dev, (flags & WQ4_EPI_RESIDUAL) ? residual_dev : nullptr, y_dev, (int)w->g.n,
                              (int)rows, (int)w->g.n, (flags & WQ4_EPI_GELU) != 0);
  if (tiled_out) {
    epi.out_tiled = static_cast<_Float16*>(at_out_dev);
    epi.nbp_next = (int)((w->g.n / 32 + 1) / 2);
  }
  const int kk = pick_kernel(w, rows, kernel);
  return gemm(w, static_cast<const _Float16*>(at_dev), rows, epi, tiled_out ? wq4::kEpiTiled : wq4::kEpiF32,
              ns_of(prec), static_cast<hipStream_t>(stream), kk == 2, kk == 3);
}

wq4_status wq4_gemm_ln_tiled(const wq4_tensor* w, const float* bias_dev, const float* x_dev, const float* ln_w_dev,
                             const float* ln_b_dev, void* at_scratch_dev, const float* residual_dev, float* y_dev,
                             void* at_out_dev, int64_t rows, unsigned flags, wq4_precision prec, int kernel,
                             void* stream) {
  wq4_status s = check_gemm_tensor(w);
  if (s != WQ4_OK) return s;
  s = check_prec(prec);
  if (s != WQ4_OK) return s;
  if (kernel < 0 || kernel > 2) return fail(WQ4_EINVAL, "kernel must be 0, 1 or 2");
  if (rows < 0 || rows > (1 << 24)) return fail(WQ4_ESHAPE, "bad row count");
  if (rows == 0) return WQ4_OK;
  if (!x_dev || !ln_w_dev || !ln_b_dev || !at_scratch_dev) return fail(WQ4_EINVAL, "null argument");
  if (w->g.k % 4 != 0 || w->g.k > 2048) return fail(WQ4_ESHAPE, "LayerNorm width must be % 4 == 0 and <= 2048");
  // Measured on MI355X (decode step, 32 rows, K = 1280): building the
  // operand inside every n-tile's workgroup repeats the row statistics and
  // the normalisation N / 32 times and ran 19.5 us against 7.8 + ~6 us for
  // the two launches, so the fused form is opt-in (WQ4_EPI_LN_FUSED).
  const bool dec = kernel == 0 ? use_decode(rows) : kernel == 2;
  if ((flags & WQ4_EPI_LN_FUSED) && dec && wq4::decode_ln_supported(w->g, (int)rows)) {
    const bool tiled_out = (flags & WQ4_EPI_TILED_OUT) != 0;
    if (tiled_out ? !at_out_dev : !y_dev) return fail(WQ4_EINVAL, "null argument");
    if ((flags & WQ4_EPI_RESIDUAL) && (!residual_dev || tiled_out))
      return fail(WQ4_EINVAL, "WQ4_EPI_RESIDUAL needs a residual and an f32 output");
    if (tiled_out && w->g.n % 32 != 0) return fail(WQ4_ESHAPE, "tiled output needs N % 32 == 0");
    DeviceGuard dg(w->device);
    wq4::EpiArgs epi = make_epi(bias_dev, (flags & WQ4_EPI_RESIDUAL) ? residual_dev : nullptr, y_dev, (int)w->g.n,
                                (int)rows, (int)w->g.n, (flags & WQ4_EPI_GELU) != 0);
    if (tiled_out) {
      epi.out_tiled = static_cast<_Float16*>(at_out_dev);
      epi.nbp_next = (int)((w->g.n / 32 + 1) / 2);
    }
    epi.lnx = x_dev;
    epi.lng = ln_w_dev;
    epi.lnb = ln_b_dev;
    epi.lnd = (int)w->g.k;
    return gemm(w, nullptr, rows, epi, tiled_out ? wq4::kEpiTiled : wq4::kEpiF32, ns_of(prec),
                static_cast<hipStream_t>(stream), true);
  }
  s = wq4_layernorm(x_dev, ln_w_dev, ln_b_dev, rows, w->g.k, prec, at_scratch_dev, nullptr, stream);
  if (s != WQ4_OK) return s;
  return wq4_gemm_tiled(w, bias_dev, at_scratch_dev, residual_dev, y_dev, at_out_dev, rows,
                        flags & ~WQ4_EPI_LN_FUSED, prec, kernel, stream);
}

int wq4_lnfold_supported(const wq4_tensor* w, int64_t rows) { return lnfold_kernel(w, rows) != 0 ? 1 : 0; }

wq4_status wq4_gemm_tiled_lnfold(const wq4_tensor* w, const float* bias_dev, const void* at_dev,
                                 const float* residual_dev, float* y_dev, void* at_out_dev, int64_t rows,
                                 unsigned flags, wq4_precision prec, const wq4_ln_fold* fold, void* stream) {
  wq4_status s = check_gemm_tensor(w);
  if (s != WQ4_OK) return s;
  s = check_prec(prec);
  if (s != WQ4_OK) return s;
  if (!fold) return fail(WQ4_EINVAL, "fold is null");
  if (rows == 0) return WQ4_OK;
  const int kk = lnfold_kernel(w, rows);
  if (kk == 0)
    return fail(WQ4_ESHAPE, "LayerNorm fold needs rows <= 32 and the decode-step or 8-wave decode kernel");
  const bool tiled_out = (flags & WQ4_EPI_TILED_OUT) != 0;
  const bool producer = fold->at_out_dev != nullptr, consumer = fold->stats_in_dev != nullptr;
  if (!at_dev || (tiled_out ? !at_out_dev : !y_dev)) return fail(WQ4_EINVAL, "null argument");
  if ((flags & WQ4_EPI_RESIDUAL) && (!residual_dev || tiled_out))
    return fail(WQ4_EINVAL, "WQ4_EPI_RESIDUAL needs a residual and an f32 output");
  if (producer && (!fold->gamma_dev || !fold->stats_out_dev || tiled_out || w->g.n % 32 != 0))
    return fail(WQ4_EINVAL, "LayerNorm-fold producer needs gamma, statistics, an f32 output and N % 32 == 0");
  if (consumer && (!fold->wg_dev || w->g.k / 16 > wq4::kSkinnyMaxLnTiles))
    return fail(WQ4_EINVAL, "LayerNorm-fold consumer needs W gamma and K <= 1280");
  if (tiled_out && w->g.n % 32 != 0) return fail(WQ4_ESHAPE, "tiled output needs N % 32 == 0");
  DeviceGuard dg(w->device);
  wq4::EpiArgs epi = make_epi(bias_dev, (flags & WQ4_EPI_RESIDUAL) ? residual_dev : nullptr, y_dev, (int)w->g.n,
                              (int)rows, (int)w->g.n, (flags & WQ4_EPI_GELU) != 0);
  if (tiled_out) {
    epi.out_tiled = static_cast<_Float16*>(at_out_dev);
    epi.nbp_next = (int)((w->g.n / 32 + 1) / 2);
  }
  if (producer) {
    epi.lnf_g = fold->gamma_dev;
    epi.lnf_at = static_cast<_Float16*>(fold->at_out_dev);
    epi.lnf_stats_out = fold->stats_out_dev;
    epi.lnf_nbp = (int)((w->g.n / 32 + 1) / 2);
  }
  if (consumer) {
    epi.lnf_stats_in = fold->stats_in_dev;
    epi.lnf_wg = fold->wg_dev;
    epi.lnf_tiles = (int)(w->g.k / 16);
  }
  return gemm(w, static_cast<const _Float16*>(at_dev), rows, epi, tiled_out ? wq4::kEpiTiled : wq4::kEpiF32,
              ns_of(prec), static_cast<hipStream_t>(stream), kk == 2, kk == 3);
}

wq4_status wq4_ln_fold_vectors(const wq4_tensor* w, const float* gamma, const float* beta, const float* bias,
                               float* wg_out, float* bias_out) {
  if (!w || !gamma || !beta || !wg_out || !bias_out) return fail(WQ4_EINVAL, "null argument");
  const int64_t n = w->g.n, k = w->g.k;
  std::vector<float> wd((size_t)(n * k));
  wq4_status s = wq4_tensor_dequantize(w, wd.data());
  if (s != WQ4_OK) return s;
  for (int64_t i = 0; i < n; ++i) {
    const float* row = wd.data() + i * k;
    double sg = 0.0, sb = 0.0;
    for (int64_t j = 0; j < k; ++j) {
      sg += (double)row[j] * gamma[j];
      sb += (double)row[j] * beta[j];
    }
    wg_out[i] = (float)sg;
    bias_out[i] = (float)(sb + (bias ? (double)bias[i] : 0.0));
  }
  return WQ4_OK;
}

wq4_status wq4_prepare_stream(int device, void* stream) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return fail(WQ4_EINVAL, "bad device");
  DeviceGuard dg(device);
  const wq4::DecodeWs* ws = nullptr;
  return decode_ws_get(device, stream, &ws);
}

wq4_status wq4_layernorm(const float* x_dev, const float* w_dev, const float* b_dev, int64_t rows, int64_t d,
                         wq4_precision prec, void* at_out_dev, float* y_dev, void* stream) {
  wq4_status s = check_prec(prec);
  if (s != WQ4_OK) return s;
  if (!x_dev || !w_dev || !b_dev || (at_out_dev == nullptr) == (y_dev == nullptr))
    return fail(WQ4_EINVAL, "layernorm needs x, w, b and exactly one of at_out / y");
  if (rows < 0 || rows > (1 << 24) || d <= 0 || d % 4 != 0 || d > 2048)
    return fail(WQ4_ESHAPE, "layernorm needs d % 4 == 0, d <= 2048");
  if (rows == 0) return WQ4_OK;
  hipError_t e = wq4::launch_layernorm(x_dev, w_dev, b_dev, (int)rows, (int)d, static_cast<_Float16*>(at_out_dev),
                                       ns_of(prec), y_dev, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "layernorm launch");
  return WQ4_OK;
}

wq4_status wq4_gemm_tiled_headmajor(const wq4_tensor* w, const float* bias_dev, const void* at_dev, float* y_dev,
                                    int64_t rows, int group_rows, int d, wq4_precision prec, int kernel,
                                    void* stream) {
  wq4_status s = check_gemm_tensor(w);
  if (s != WQ4_OK) return s;
  s = check_prec(prec);
  if (s != WQ4_OK) return s;
  if (kernel < 0 || kernel > 2) return fail(WQ4_EINVAL, "kernel must be 0, 1 or 2");
  if (rows < 0 || rows > (1 << 24)) return fail(WQ4_ESHAPE, "bad row count");
  if (group_rows <= 0 || rows % group_rows != 0) return fail(WQ4_ESHAPE, "rows must be a multiple of group_rows");
  if (d <= 0 || d % 64 != 0 || w->g.n % d != 0)
    return fail(WQ4_ESHAPE, "head-major output needs d % 64 == 0 and N % d == 0");
  if (rows == 0) return WQ4_OK;
  if (!at_dev || !y_dev) return fail(WQ4_EINVAL, "null argument");
  DeviceGuard dg(w->device);
  wq4::EpiArgs epi = make_epi(bias_dev, nullptr, y_dev, (int)w->g.n, (int)rows, (int)w->g.n, false);
  epi.hm_t = group_rows;
  epi.hm_d = d;
  const bool dec = kernel == 0 ? use_decode(rows) : kernel == 2;
  return gemm(w, static_cast<const _Float16*>(at_dev), rows, epi, wq4::kEpiHeadMajor, ns_of(prec),
              static_cast<hipStream_t>(stream), dec);
}

// scripts/convert_whisper.py:33-74 (numpy 2 scalar semantics: amax, d in f32).
wq4_status wq4_quantize_q4_0(const float* x, int64_t n, uint8_t* out) {
  if (!x || !out) return fail(WQ4_EINVAL, "null argument");
  if (n < 0 || n % 32 != 0) return fail(WQ4_ESHAPE, "Element count " + std::to_string(n) + " not divisible by 32");
  for (int64_t b = 0; b < n / 32; ++b) {
    const float* blk = x + b * 32;
    float amax = 0.0f;
    for (int i = 0; i < 32; ++i) {
      const float a = std::fabs(blk[i]);
      if (a > amax || std::isnan(a)) amax = a;
    }
    const float d = amax > 0.0f ? amax / 7.0f : 0.0f;
    const uint16_t h = __builtin_bit_cast(uint16_t, (_Float16)d);
    uint8_t* o = out + b * 18;
    o[0] = (uint8_t)(h & 0xff);
    o[1] = (uint8_t)(h >> 8);
    int q[32];
    for (int i = 0; i < 32; ++i) q[i] = d > 0.0f ? (int)(int8_t)(int)std::nearbyint(blk[i] / d) : 0;
    for (int i = 0; i < 16; ++i) o[2 + i] = (uint8_t)(((q[i] + 8) & 0x0f) | (((q[i + 16] + 8) & 0x0f) << 4));
  }
  return WQ4_OK;
}

static wq4_status check_nk(int64_t n, int64_t k) {
  if (n <= 0 || k <= 0 || k % 32 != 0 || n > (1 << 24) || k > (1 << 24))
    return fail(WQ4_ESHAPE, "bad Q4_0 shape [" + std::to_string(n) + ", " + std::to_string(k) + "]");
  return WQ4_OK;
}

wq4_status wq4_debug_repacked_bytes(int64_t n, int64_t k, size_t* nib_bytes, size_t* sc_bytes, size_t* cs_bytes) {
  wq4_status s = check_nk(n, k);
  if (s != WQ4_OK) return s;
  if (!nib_bytes || !sc_bytes || !cs_bytes) return fail(WQ4_EINVAL, "null argument");
  const wq4::Q4Geom g = wq4::make_geom(n, k);
  *nib_bytes = g.nib_bytes();
  *sc_bytes = g.sc_bytes();
  *cs_bytes = g.colscale_bytes();
  return WQ4_OK;
}

wq4_status wq4_debug_repack(const uint8_t* raw, int64_t n, int64_t k, uint8_t* nib_out, uint32_t* sc_out,
                            float* colscale_out) {
  wq4_status s = check_nk(n, k);
  if (s != WQ4_OK) return s;
  if (!raw || !nib_out || !sc_out || !colscale_out) return fail(WQ4_EINVAL, "null argument");
  wq4::repack_q4(raw, wq4::make_geom(n, k), nib_out, sc_out, colscale_out);
  return WQ4_OK;
}

wq4_status wq4_debug_unrepack(const uint8_t* nib, const uint32_t* sc, const float* colscale, int64_t n, int64_t k,
                              uint8_t* raw_out) {
  wq4_status s = check_nk(n, k);
  if (s != WQ4_OK) return s;
  if (!nib || !sc || !colscale || !raw_out) return fail(WQ4_EINVAL, "null argument");
  wq4::unrepack_q4(nib, sc, colscale, wq4::make_geom(n, k), raw_out);
  return WQ4_OK;
}

}  // extern "C"
