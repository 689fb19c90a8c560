// wa_melbank.cpp -- host constants of the log-mel front-end.  Built with
// -ffp-contract=off: every expression below is the f32 (or f64 for the
// twiddles) arithmetic of src/audio/mel.rs, op for op.
#include <cmath>
#include <cstring>

#include "wa_mel.hpp"

namespace wa {
namespace {

// mel.rs:244-255 (Slaney / O'Shaughnessy)
constexpr float kFsp = 200.0f / 3.0f;
constexpr float kMinLogHz = 1000.0f;
constexpr float kMinLogMel = kMinLogHz / kFsp;
constexpr float kLogStep = 0.06875174f;

float hz_to_mel(float f) { return f < kMinLogHz ? f / kFsp : kMinLogMel + std::log(f / kMinLogHz) / kLogStep; }

// mel.rs:258-269
float mel_to_hz(float m) { return m < kMinLogMel ? m * kFsp : kMinLogHz * std::exp((m - kMinLogMel) * kLogStep); }

size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

}  // namespace

MelBank make_mel_bank(int n_mels) {
  MelBank b;
  b.n_mels = n_mels;
  // mel.rs:316-320: 0.5 * (1 - cos(2*PI*i / len)), f32
  const float two_pi = 2.0f * 3.14159265358979323846f;
  b.window.resize(kMelNfft);
  for (int i = 0; i < kMelNfft; ++i) b.window[i] = 0.5f * (1.0f - std::cos(two_pi * (float)i / (float)kMelNfft));

  // mel.rs:272-313, fmin 0, fmax sr / 2
  const float mel_min = hz_to_mel(0.0f);
  const float mel_max = hz_to_mel((float)kMelSampleRate / 2.0f);
  std::vector<float> hz(n_mels + 2);
  for (int i = 0; i <= n_mels + 1; ++i)
    hz[i] = mel_to_hz(mel_min + (mel_max - mel_min) * (float)i / (float)(n_mels + 1));
  std::vector<float> freq(kMelBins);
  for (int j = 0; j < kMelBins; ++j) freq[j] = (float)j * (float)kMelSampleRate / (float)kMelNfft;
  b.filters.assign((size_t)n_mels * kMelBins, 0.0f);
  b.range.assign((size_t)n_mels * 2, 0);
  for (int i = 0; i < n_mels; ++i) {
    const float lo = hz[i], c = hz[i + 1], hi = hz[i + 2];
    int first = -1, last = -2;
    for (int j = 0; j < kMelBins; ++j) {
      float v = 0.0f;
      const float f = freq[j];
      if (f >= lo && f <= c && c > lo)
        v = (f - lo) / (c - lo);
      else if (f > c && f <= hi && hi > c)
        v = (hi - f) / (hi - c);
      b.filters[(size_t)i * kMelBins + j] = v;
      if (v != 0.0f) {
        if (first < 0) first = j;
        last = j;
      }
    }
    b.range[2 * i] = first;
    b.range[2 * i + 1] = last;
  }

  b.twiddle.resize(2 * kMelNfft);
  for (int m = 0; m < kMelNfft; ++m) {
    const double a = 2.0 * M_PI * (double)m / (double)kMelNfft;
    b.twiddle[m] = std::cos(a);
    b.twiddle[kMelNfft + m] = std::sin(a);
  }
  return b;
}

size_t mel_const_bytes(int n_mels) {
  return align16(kMelNfft * 4) + align16((size_t)n_mels * kMelBins * 4) + align16((size_t)n_mels * 8) +
         2 * kMelNfft * 8;
}

void mel_pack_consts(const MelBank& b, uint8_t* host) {
  size_t off = 0;
  std::memcpy(host + off, b.window.data(), kMelNfft * 4);
  off += align16(kMelNfft * 4);
  std::memcpy(host + off, b.filters.data(), b.filters.size() * 4);
  off += align16(b.filters.size() * 4);
  std::memcpy(host + off, b.range.data(), b.range.size() * 4);
  off += align16(b.range.size() * 4);
  std::memcpy(host + off, b.twiddle.data(), b.twiddle.size() * 8);
}

}  // namespace wa
