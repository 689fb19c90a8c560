"""numpy restatement of the reference's log-mel front-end -- TEST INFRASTRUCTURE ONLY.

Only tests/ (and bench.py's checker) import it; the product path
(whisper-burn_amd/csrc/whisper/wa_mel.hip behind wa_log_mel) never does.

Restates, op for op in float32 where the reference computes in f32:
  pad / truncate to 480 000 samples       src/transcribe.rs:45-52
  reflect padding (center=True)           src/audio/mel.rs:179-193
  frames, periodic Hann window            src/audio/mel.rs:199-214, 316-320
  power spectrum |X_k|^2, k = 0..200       src/audio/mel.rs:107-112, 216-222
  Slaney mel filterbank (no area norm)    src/audio/mel.rs:243-313
  filterbank product (f*p summed in order) src/audio/mel.rs:231-241
  log10 floor / max-8 clamp / (v+4)/4      src/audio/mel.rs:126-157
  transpose to [n_mels, 3000]             src/transcribe.rs:65-76

The reference's FFT is the third-party crate rustfft (f32, planner-chosen
mixed radix for n = 400; Cargo.toml pins rustfft 6).  It is not available
here, so the DFT is restated by its definition: numpy's float64 rfft of the
f32 windowed frame, rounded once to f32 -- the exactly-rounded spectrum that
rustfft approximates to within its own f32 rounding.  Parity pinning: the
reference holds no mel fixtures or tests, so this
restatement is pinned by known answers only -- silence -> -1.5 everywhere
(the constant SURVEY.md §8(d) uses), pure tones landing in the mel band of
their frequency, and the reflect-padding loop of mel.rs:184-193 restated
literally (reflect_pad_literal) -- "partially pinned" in DESIGN.md.
"""
from __future__ import annotations

import numpy as np

SAMPLE_RATE = 16000
N_FFT = 400
HOP = 160
N_BINS = N_FFT // 2 + 1
CHUNK = 480000  # WHISPER_CHUNK_SAMPLES, transcribe.rs:45
FRAMES = 3000  # WHISPER_MEL_FRAMES

f32 = np.float32
F_SP = f32(200.0) / f32(3.0)
MIN_LOG_HZ = f32(1000.0)
MIN_LOG_MEL = MIN_LOG_HZ / F_SP
LOGSTEP = f32(0.06875174)


def _rnd(fn, x):
    """f32 libm function as the reference's Rust f32 math calls it (glibc
    logf / expf / cosf / log10f): evaluated in f64 and rounded once to f32
    (numpy's own float32 kernels are not correctly rounded)."""
    return np.asarray(fn(np.asarray(x, np.float64)), np.float64).astype(f32)


def hz_to_mel(f: np.float32) -> np.float32:
    """mel.rs:244-255."""
    f = f32(f)
    if f < MIN_LOG_HZ:
        return f / F_SP
    return MIN_LOG_MEL + _rnd(np.log, f / MIN_LOG_HZ) / LOGSTEP


def mel_to_hz(m: np.float32) -> np.float32:
    """mel.rs:258-269."""
    m = f32(m)
    if m < MIN_LOG_MEL:
        return m * F_SP
    return MIN_LOG_HZ * _rnd(np.exp, (m - MIN_LOG_MEL) * LOGSTEP)


def mel_filterbank(n_mels: int, sample_rate: int = SAMPLE_RATE, n_fft: int = N_FFT) -> np.ndarray:
    """create_mel_filterbank (mel.rs:272-313), fmin 0, fmax sr/2 -> [n_mels, 201] f32."""
    n_freqs = n_fft // 2 + 1
    mel_min = hz_to_mel(f32(0.0))
    mel_max = hz_to_mel(f32(sample_rate) / f32(2.0))
    hz = [mel_to_hz(mel_min + (mel_max - mel_min) * f32(i) / f32(n_mels + 1)) for i in range(n_mels + 2)]
    freqs = [f32(i) * f32(sample_rate) / f32(n_fft) for i in range(n_freqs)]
    fb = np.zeros((n_mels, n_freqs), f32)
    for i in range(n_mels):
        lo, c, hi = hz[i], hz[i + 1], hz[i + 2]
        for j, fr in enumerate(freqs):
            if lo <= fr <= c and c > lo:
                fb[i, j] = (fr - lo) / (c - lo)
            elif c < fr <= hi and hi > c:
                fb[i, j] = (hi - fr) / (hi - c)
    return fb


def hann_window(length: int = N_FFT) -> np.ndarray:
    """mel.rs:316-320 (periodic), f32."""
    two_pi = f32(2.0) * f32(np.pi)
    i = np.arange(length, dtype=f32)
    return (f32(0.5) * (f32(1.0) - _rnd(np.cos, two_pi * i / f32(length)))).astype(f32)


def pad_or_truncate(samples: np.ndarray) -> np.ndarray:
    """transcribe.rs:45-52."""
    s = np.asarray(samples, f32)
    if len(s) >= CHUNK:
        return s[:CHUNK].copy()
    return np.concatenate([s, np.zeros(CHUNK - len(s), f32)])


def reflect_pad_literal(samples) -> list:
    """mel.rs:179-193 line by line (pure Python; small inputs only)."""
    pad = N_FFT // 2
    n = len(samples)
    out = []
    for i in range(pad, 0, -1):
        idx = min(i, max(n - 1, 0))
        out.append(samples[idx] if idx < n else 0.0)
    out.extend(samples)
    for i in range(pad):
        idx = max(max(n - 2, 0) - i, 0)
        out.append(samples[idx] if idx < n else 0.0)
    return out


def reflect_pad(samples: np.ndarray) -> np.ndarray:
    """Vectorised reflect_pad_literal for len(samples) > 200."""
    pad = N_FFT // 2
    s = np.asarray(samples, f32)
    n = len(s)
    assert n > pad
    left = s[np.arange(pad, 0, -1)]
    right = s[np.arange(n - 2, n - 2 - pad, -1)]
    return np.concatenate([left, s, right])


def power_spectrum(samples: np.ndarray) -> np.ndarray:
    """stft + norm_sqr (mel.rs:106-112, 174-228) -> [n_frames, 201] f32."""
    padded = reflect_pad(samples)
    n_frames = (len(padded) - N_FFT) // HOP
    idx = np.arange(n_frames)[:, None] * HOP + np.arange(N_FFT)[None, :]
    xw = (padded[idx] * hann_window()[None, :]).astype(f32)  # one f32 multiply, mel.rs:208
    X = np.fft.rfft(xw.astype(np.float64), axis=1)
    re = X.real.astype(f32)
    im = X.imag.astype(f32)
    return (re * re + im * im).astype(f32)


def apply_filterbank(power: np.ndarray, fb: np.ndarray) -> np.ndarray:
    """mel.rs:231-241: per (frame, mel) the f32 products summed in bin order."""
    acc = np.zeros((power.shape[0], fb.shape[0]), f32)
    for k in range(fb.shape[1]):
        acc = (acc + (fb[None, :, k] * power[:, k:k + 1]).astype(f32)).astype(f32)
    return acc


def log_mel(samples: np.ndarray, n_mels: int = 128, fb: np.ndarray | None = None) -> np.ndarray:
    """transcribe.rs:44-76 + compute_log (mel.rs:126-157) -> [n_mels, 3000] f32."""
    s = pad_or_truncate(samples)
    if fb is None:
        fb = mel_filterbank(n_mels)
    mel = apply_filterbank(power_spectrum(s), fb)
    lg = _rnd(np.log10, np.maximum(mel, f32(1e-10)))
    lo = f32(lg.max()) - f32(8.0)
    lg = np.maximum(lg, lo)
    lg = ((lg + f32(4.0)) / f32(4.0)).astype(f32)
    out = np.zeros((n_mels, FRAMES), f32)
    nf = min(FRAMES, lg.shape[0])
    out[:, :nf] = lg[:nf].T
    return out


def log_mel_batch(audio: np.ndarray, n_samples: int | None = None, n_mels: int = 128) -> np.ndarray:
    """[B, >= n_samples] -> [B, n_mels, 3000] (wa_log_mel semantics)."""
    audio = np.asarray(audio, f32)
    n = audio.shape[1] if n_samples is None else n_samples
    fb = mel_filterbank(n_mels)
    return np.stack([log_mel(audio[b, :n], n_mels, fb) for b in range(audio.shape[0])])


def synthetic_audio(n_clips: int, n_samples: int = CHUNK, seed: int = 0) -> np.ndarray:
    """Deterministic speech-like test audio (clip c: noise floor + two tones
    + a chirp with per-clip frequencies and a 4 Hz amplitude envelope),
    f32 in [-1, 1] -- the audio analogue of SURVEY.md §8(d)'s synthetic mel."""
    rng = np.random.default_rng(seed)
    t = np.arange(n_samples, dtype=np.float64) / SAMPLE_RATE
    out = np.empty((n_clips, n_samples), f32)
    for c in range(n_clips):
        f1, f2 = 150.0 + 37.0 * c, 1200.0 + 211.0 * c
        env = 0.5 * (1.0 + np.sin(2 * np.pi * 4.0 * t + c))
        chirp = np.sin(2 * np.pi * (300.0 * t + 60.0 * t * t))
        x = 0.3 * env * np.sin(2 * np.pi * f1 * t) + 0.15 * np.sin(2 * np.pi * f2 * t) + 0.1 * chirp
        x += 0.02 * rng.standard_normal(n_samples)
        out[c] = np.clip(x, -1.0, 1.0)
    return out
