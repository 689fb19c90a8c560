// wa_mel.hpp -- Whisper log-mel front-end.
//
// Behaviour of the reference's CPU path, src/transcribe.rs:44-76 +
// src/audio/mel.rs:126-320: pad/truncate each clip to 480 000 samples,
// reflect-pad 200 samples each side (mel.rs:179-193), 3000 frames of 400
// samples at hop 160, periodic Hann window (mel.rs:316-320), 201-bin power
// spectrum (mel.rs:109-112), Slaney mel filterbank without area
// normalisation (mel.rs:243-313), log10(max(v, 1e-10)), clamp to the clip's
// max - 8, (v + 4) / 4 (mel.rs:126-157), written transposed as
// [clip][n_mels][3000] (transcribe.rs:65-76).
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <vector>

namespace wa {

constexpr int kMelSampleRate = 16000;
constexpr int kMelNfft = 400;
constexpr int kMelHop = 160;
constexpr int kMelBins = kMelNfft / 2 + 1;  // 201
constexpr int kMelChunk = 480000;           // 30 s at 16 kHz (transcribe.rs:45-52)
constexpr int kMelFrames = 3000;            // (480000 + 400 - 400) / 160 (mel.rs:166-171)
constexpr int kMelFramesPerWg = 8;
constexpr int kMelWgPerClip = (kMelFrames + kMelFramesPerWg - 1) / kMelFramesPerWg;  // 375
constexpr int kMelMaxMels = 256;

// Host-side constants (wa_melbank.cpp), f32 arithmetic exactly as mel.rs.
struct MelBank {
  int n_mels = 0;
  std::vector<float> window;     // [400]  periodic Hann (mel.rs:316-320)
  std::vector<float> filters;    // [n_mels][201] (mel.rs:272-313)
  std::vector<int32_t> range;    // [n_mels][2] first / last nonzero bin (-1, -2 when empty)
  std::vector<double> twiddle;   // [2][400]  cos, sin of 2*pi*m/400
};
MelBank make_mel_bank(int n_mels);

// Device constants: window f32[400] | filters f32[n_mels*201] | range
// i32[n_mels*2] | twiddle f64[800], 16-byte aligned sections.
size_t mel_const_bytes(int n_mels);
void mel_pack_consts(const MelBank& bank, uint8_t* host);

// audio: [B] clips of n_samples f32 at stride ld_audio (samples past
// n_samples read as 0, samples past 480000 ignored).  out: [B][n_mels][3000].
// part: B * kMelWgPerClip floats of scratch (per-workgroup maxima).
hipError_t launch_log_mel(const float* audio, int B, int64_t n_samples, int64_t ld_audio, int n_mels,
                          const uint8_t* consts, float* part, float* out, hipStream_t st);

}  // namespace wa
