"""GPU parity tests of the log-mel front-end (wa_log_mel).

Oracle: oracle/mel_oracle.py, the numpy restatement of src/audio/mel.rs +
transcribe.rs:44-76 (exactly-rounded DFT, f32 everywhere else).
Tolerance (stated here and in DESIGN.md "Numerics"): on the normalised
log-mel, max|gpu - oracle| <= 1e-4 and mean|gpu - oracle| <= 1e-6 -- the GPU
accumulates the DFT in f64 and rounds it once, like the oracle, so the
remaining differences are f32 rounding ties and the device log10f ulp.
Silence is bit-exact (-1.5 everywhere).
"""
from __future__ import annotations

import numpy as np
import pytest

import mel_oracle as mo
import wq4

pytestmark = pytest.mark.gpu

ATOL_MAX = 1e-4
ATOL_MEAN = 1e-6


@pytest.fixture(scope="module")
def torch():
    import torch as _t

    assert _t.cuda.is_available()
    return _t


@pytest.fixture(scope="module")
def wa():
    import whisper_amd

    return whisper_amd


def _check(gpu, ref):
    d = np.abs(gpu - ref)
    assert d.max() <= ATOL_MAX, (d.max(), np.unravel_index(d.argmax(), d.shape))
    assert d.mean() <= ATOL_MEAN, d.mean()


@pytest.mark.parametrize("n_mels", [80, 128])
def test_log_mel_matches_oracle(torch, wa, n_mels):
    audio = mo.synthetic_audio(3, seed=7)
    gpu = wa.log_mel(torch.from_numpy(audio).cuda(), n_mels).cpu().numpy()
    assert gpu.shape == (3, n_mels, 3000)
    _check(gpu, mo.log_mel_batch(audio, n_mels=n_mels))


def test_log_mel_noise_and_tones(torch, wa):
    rng = np.random.default_rng(11)
    t = np.arange(mo.CHUNK) / mo.SAMPLE_RATE
    clips = np.stack([
        (0.3 * rng.standard_normal(mo.CHUNK)).astype(np.float32),
        (0.5 * np.sin(2 * np.pi * 1000.0 * t)).astype(np.float32),
        (0.9 * np.sign(np.sin(2 * np.pi * 97.0 * t))).astype(np.float32),  # square wave: rich spectrum
        (1e-4 * rng.standard_normal(mo.CHUNK)).astype(np.float32),  # near-silent
    ])
    gpu = wa.log_mel(torch.from_numpy(clips).cuda(), 128).cpu().numpy()
    _check(gpu, mo.log_mel_batch(clips, n_mels=128))


def test_silence_exact(torch, wa):
    gpu = wa.log_mel(torch.zeros((2, 16000), device="cuda"), 80).cpu().numpy()
    assert np.all(gpu == np.float32(-1.5))


def test_short_and_strided_clips(torch, wa):
    # 100 000 valid samples per row inside rows of 120 000 (ld > n_samples):
    # zero padding to 30 s, and the tail of each row must be ignored
    audio = mo.synthetic_audio(2, 120000, seed=3)
    gpu = wa.log_mel(torch.from_numpy(audio).cuda(), 80, n_samples=100000).cpu().numpy()
    _check(gpu, mo.log_mel_batch(audio, n_samples=100000, n_mels=80))


def test_truncation_past_30s(torch, wa):
    audio = mo.synthetic_audio(1, 500000, seed=5)
    gpu = wa.log_mel(torch.from_numpy(audio).cuda(), 128).cpu().numpy()
    _check(gpu, mo.log_mel_batch(audio[:, : mo.CHUNK], n_mels=128))


def test_batch_invariance(torch, wa):
    audio = torch.from_numpy(mo.synthetic_audio(5, seed=9)).cuda()
    full = wa.log_mel(audio, 128).cpu()
    one = wa.log_mel(audio[3:4].contiguous(), 128).cpu()
    assert torch.equal(full[3:4], one)


def test_log_mel_errors(torch, wa):
    a = torch.zeros((1, 1000), device="cuda")
    with pytest.raises(wq4.WQ4Error):
        wa.log_mel(a, 0)
    with pytest.raises(wq4.WQ4Error):
        wa.log_mel(a, 80, n_samples=2000)  # n_samples > row stride


def test_audio_to_tokens_matches_oracle(torch, wa):
    """transcribe.rs:34-107 end to end on the GPU (tiny_test, 80 mels): the
    tokens from audio equal the oracle model's tokens on the same mel."""
    import whisper_oracle as wo

    audio = mo.synthetic_audio(2, seed=21)
    m = wa.WhisperModel("tiny_test", 1234, max_batch=2)
    mel = wa.log_mel(torch.from_numpy(audio).cuda(), 80)
    toks = m.transcribe_audio(torch.from_numpy(audio).cuda(), max_tokens=24, eot_stop=False)
    ref = wo.SynthWhisper("tiny_test", 1234).transcribe(mel.cpu().numpy(), max_tokens=24, eot_stop=False)
    assert toks == ref
