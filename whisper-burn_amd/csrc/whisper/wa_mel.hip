// wa_mel.hip -- log-mel front-end kernels.
//
// Reference: src/audio/mel.rs:126-228 (compute_log / stft) driven by
// src/transcribe.rs:44-76.  Two launches per batch of clips:
//
//   mel_power_kernel  one workgroup per 8 frames of one clip: reflect-padded,
//                     windowed frames -> 201-bin DFT (f64 accumulation over
//                     the symmetric half, so the spectrum is the exact DFT of
//                     the f32 windowed frame rounded once to f32, i.e. at
//                     least as accurate as the reference's f32 rustfft) ->
//                     |X|^2 (f32) -> mel filterbank (f32, the reference's
//                     product/sum order) -> log10(max(v, 1e-10)), written
//                     transposed [clip][mel][frame], plus the workgroup max.
//   mel_norm_kernel   clip max = max of the 375 workgroup maxima; clamp to
//                     max - 8 and (v + 4) / 4, in place (mel.rs:136-154).
//
// Cost per 30 s clip: 3000 frames x 201 bins x 398 f64 FMA (the symmetric
// DFT) = 0.24 G FMA + 3000 x ~2 x 201 filterbank MACs; HBM traffic is 1.9 MB
// in + 2 x 1.5 MB out -- a compute-bound, sub-millisecond step next to the
// encoder.
#include <hip/hip_runtime.h>

#include <cmath>

#include "wa_mel.hpp"

namespace wa {
namespace {

constexpr int kThreads = 256;
constexpr int kHalf = kMelNfft / 2;  // 200
constexpr int kFr = kMelFramesPerWg;

// Sample p of the reflect-padded 480 400-sample signal (mel.rs:179-193) of a
// clip already padded / truncated to 480 000 samples (transcribe.rs:45-52):
// padded[p] = s[200 - p] on the left, s[p - 200] inside, s[479998 - i] at
// i = p - 480 200 on the right.  Samples at or past n are the zero padding.
__device__ __forceinline__ float padded_sample(const float* __restrict__ a, int64_t n, int p) {
  int s;
  if (p < kHalf)
    s = kHalf - p;
  else if (p < kMelChunk + kHalf)
    s = p - kHalf;
  else
    s = (kMelChunk - 2) - (p - (kMelChunk + kHalf));
  return (int64_t)s < n ? a[s] : 0.0f;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__global__ __launch_bounds__(kThreads) void mel_power_kernel(const float* __restrict__ audio, int64_t n,
                                                             int64_t ld, int n_mels,
                                                             const float* __restrict__ window,
                                                             const float* __restrict__ filters,
                                                             const int* __restrict__ range,
                                                             const double* __restrict__ twiddle,
                                                             float* __restrict__ part, float* __restrict__ out) {
  // s_j = x_j + x_{400-j}, d_j = x_j - x_{400-j} (exact in f64); s_0 = x_0,
  // s_200 = x_200.  Re X_k = s_0 + (-1)^k s_200 + sum_j s_j cos(2 pi jk/400),
  // Im X_k = -sum_j d_j sin(2 pi jk/400), j = 1..199.
  __shared__ double sx[kFr][kHalf + 1];
  __shared__ double dx[kFr][kHalf];
  __shared__ double tw[2 * kMelNfft];
  __shared__ float pw[kFr][kMelBins + 3];
  __shared__ float red[kThreads / 64];

  const int tid = threadIdx.x;
  const int b = blockIdx.y;
  const int f0 = blockIdx.x * kFr;
  const int nfr = min(kFr, kMelFrames - f0);
  const float* a = audio + (int64_t)b * ld;

  for (int i = tid; i < 2 * kMelNfft; i += kThreads) tw[i] = twiddle[i];
  for (int i = tid; i < kFr * (kHalf + 1); i += kThreads) {
    const int fr = i / (kHalf + 1), j = i - fr * (kHalf + 1);
    double s = 0.0, d = 0.0;
    if (fr < nfr) {
      const int p = (f0 + fr) * kMelHop;
      // windowed sample, one f32 multiply as mel.rs:208
      const float xj = __fmul_rn(padded_sample(a, n, p + j), window[j]);
      if (j == 0 || j == kHalf) {
        s = xj;
      } else {
        const float xm = __fmul_rn(padded_sample(a, n, p + kMelNfft - j), window[kMelNfft - j]);
        s = (double)xj + (double)xm;
        d = (double)xj - (double)xm;
      }
    }
    sx[fr][j] = s;
    if (j < kHalf) dx[fr][j] = d;
  }
  __syncthreads();

  const int k = tid;
  if (k < kMelBins) {
    double re[kFr], im[kFr];
    const double sgn = (k & 1) ? -1.0 : 1.0;
#pragma unroll
    for (int fr = 0; fr < kFr; ++fr) {
      re[fr] = sx[fr][0] + sgn * sx[fr][kHalf];
      im[fr] = 0.0;
    }
    int idx = k;  // (j * k) mod 400 at j = 1
    for (int j = 1; j < kHalf; ++j) {
      const double c = tw[idx], s = tw[kMelNfft + idx];
#pragma unroll
      for (int fr = 0; fr < kFr; ++fr) {
        re[fr] = fma(sx[fr][j], c, re[fr]);
        im[fr] = fma(dx[fr][j], s, im[fr]);
      }
      idx += k;
      if (idx >= kMelNfft) idx -= kMelNfft;
    }
#pragma unroll
    for (int fr = 0; fr < kFr; ++fr) {
      const float r = (float)re[fr], i = (float)im[fr];
      pw[fr][k] = __fadd_rn(__fmul_rn(r, r), __fmul_rn(i, i));  // norm_sqr, mel.rs:111
    }
  }
  __syncthreads();

  // filterbank: lanes 8 apart in idx share a mel, consecutive lanes write
  // consecutive frames of the transposed output
  float mx = -INFINITY;
  for (int i = tid; i < n_mels * kFr; i += kThreads) {
    const int m = i / kFr, fr = i - m * kFr;
    if (fr >= nfr) continue;
    const int lo = range[2 * m], hi = range[2 * m + 1];
    const float* f = filters + (int64_t)m * kMelBins;
    float acc = 0.0f;  // mel.rs:237, zero taps contribute exact zeros and are skipped
    for (int kk = lo; kk <= hi; ++kk) acc = __fadd_rn(acc, __fmul_rn(f[kk], pw[fr][kk]));
    // mel.rs:132; f64 log10 rounded once to f32 = the correctly rounded
    // log10f of the reference's libm (device log10f is 1 ulp off at 1e-10)
    const float v = (float)log10((double)fmaxf(acc, 1e-10f));
    out[((int64_t)b * n_mels + m) * kMelFrames + f0 + fr] = v;
    mx = fmaxf(mx, v);
  }
  mx = wave_max(mx);
  if ((tid & 63) == 0) red[tid >> 6] = mx;
  __syncthreads();
  if (tid == 0) {
    float r = red[0];
    for (int w = 1; w < kThreads / 64; ++w) r = fmaxf(r, red[w]);
    part[(int64_t)b * kMelWgPerClip + blockIdx.x] = r;
  }
}

__global__ __launch_bounds__(kThreads) void mel_norm_kernel(const float* __restrict__ part, int per_clip,
                                                            float* __restrict__ out) {
  __shared__ float smx;
  const int b = blockIdx.y;
  if (threadIdx.x < 64) {
    float m = -INFINITY;
    for (int i = threadIdx.x; i < kMelWgPerClip; i += 64) m = fmaxf(m, part[(int64_t)b * kMelWgPerClip + i]);
    m = wave_max(m);
    if (threadIdx.x == 0) smx = m;
  }
  __syncthreads();
  const float lo = smx - 8.0f;  // mel.rs:141
  const int i4 = blockIdx.x * kThreads + threadIdx.x;
  if (i4 * 4 >= per_clip) return;
  float4* p = reinterpret_cast<float4*>(out + (int64_t)b * per_clip) + i4;
  float4 v = *p;
  v.x = (fmaxf(v.x, lo) + 4.0f) / 4.0f;  // mel.rs:145, 152
  v.y = (fmaxf(v.y, lo) + 4.0f) / 4.0f;
  v.z = (fmaxf(v.z, lo) + 4.0f) / 4.0f;
  v.w = (fmaxf(v.w, lo) + 4.0f) / 4.0f;
  *p = v;
}

size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

}  // namespace

hipError_t launch_log_mel(const float* audio, int B, int64_t n_samples, int64_t ld_audio, int n_mels,
                          const uint8_t* consts, float* part, float* out, hipStream_t st) {
  const float* window = reinterpret_cast<const float*>(consts);
  size_t off = align16(kMelNfft * 4);
  const float* filters = reinterpret_cast<const float*>(consts + off);
  off += align16((size_t)n_mels * kMelBins * 4);
  const int* range = reinterpret_cast<const int*>(consts + off);
  off += align16((size_t)n_mels * 8);
  const double* twiddle = reinterpret_cast<const double*>(consts + off);
  const int64_t n = n_samples < kMelChunk ? n_samples : kMelChunk;
  hipLaunchKernelGGL(mel_power_kernel, dim3(kMelWgPerClip, B), dim3(kThreads), 0, st, audio, n, ld_audio, n_mels,
                     window, filters, range, twiddle, part, out);
  const int per_clip = n_mels * kMelFrames;
  const int g = (per_clip / 4 + kThreads - 1) / kThreads;
  hipLaunchKernelGGL(mel_norm_kernel, dim3(g, B), dim3(kThreads), 0, st, part, per_clip, out);
  return hipGetLastError();
}

}  // namespace wa
