"""CPU tests of the log-mel front-end: the oracle
restatement of src/audio/mel.rs against known answers, and the product's
host-side constants (wa_mel_filterbank) against the restatement.

Tolerances: filterbank and window within 2 ulp-scale (rtol 1e-6, atol 1e-7)
-- the product uses glibc logf/expf/cosf as the reference's Rust f32 math
does, numpy its own float32 kernels.
"""
from __future__ import annotations

import numpy as np
import pytest

import mel_oracle as mo


def test_reflect_pad_matches_literal_restatement():
    rng = np.random.default_rng(3)
    x = rng.standard_normal(1000).astype(np.float32)
    lit = np.asarray(mo.reflect_pad_literal(list(x)), np.float32)
    np.testing.assert_array_equal(mo.reflect_pad(x), lit)
    assert len(lit) == 1400
    assert lit[0] == x[200] and lit[199] == x[1] and lit[200] == x[0]  # mel.rs:184-187
    assert lit[1200] == x[998] and lit[-1] == x[799]  # mel.rs:190-193


def test_reflect_pad_literal_short_inputs():
    # mel.rs:185 / 191 saturating index rules on inputs shorter than the pad
    assert mo.reflect_pad_literal([]) == [0.0] * 400
    one = mo.reflect_pad_literal([5.0])
    assert one == [5.0] * 401


def test_frame_count():
    # num_frames (mel.rs:166-171) for the padded 30 s chunk
    assert (mo.CHUNK + 2 * 200 - mo.N_FFT) // mo.HOP == mo.FRAMES


def test_silence_is_constant_minus_1_5():
    out = mo.log_mel(np.zeros(1000, np.float32), 80)
    assert out.shape == (80, 3000)
    assert np.all(out == np.float32(-1.5))


def test_hann_window_periodic():
    w = mo.hann_window()
    assert w[0] == 0.0 and abs(w[200] - 1.0) < 1e-7
    np.testing.assert_allclose(w[1:200], w[399:200:-1], rtol=0, atol=1e-6)


@pytest.mark.parametrize("n_mels", [80, 128])
def test_filterbank_shape_and_triangles(n_mels):
    fb = mo.mel_filterbank(n_mels)
    assert fb.shape == (n_mels, 201)
    assert fb.min() >= 0 and fb.max() <= 1.0
    peaks = fb.argmax(axis=1)
    assert np.all(np.diff(peaks) >= 0)  # centers ascend in frequency
    # no area normalisation (mel.rs:308-309): triangles of unit height
    assert fb.max() > 0.9


@pytest.mark.parametrize("freq", [250.0, 1000.0, 3000.0, 6000.0])
def test_tone_lands_in_its_mel_band(freq):
    t = np.arange(mo.CHUNK) / mo.SAMPLE_RATE
    x = (0.5 * np.sin(2 * np.pi * freq * t)).astype(np.float32)
    out = mo.log_mel(x, 128)
    fb = mo.mel_filterbank(128)
    b = int(round(freq * mo.N_FFT / mo.SAMPLE_RATE))
    band = int(np.argmax(out[:, 1500]))
    assert fb[band, b] > 0, (band, b)
    assert out[:, 1500].max() == pytest.approx(out.max(), abs=1e-3)


def test_truncation_and_zero_padding():
    x = mo.synthetic_audio(1, 500000, seed=1)[0]
    np.testing.assert_array_equal(mo.log_mel(x, 80), mo.log_mel(x[: mo.CHUNK], 80))
    short = x[:100000]
    padded = np.concatenate([short, np.zeros(mo.CHUNK - 100000, np.float32)])
    np.testing.assert_array_equal(mo.log_mel(short, 80), mo.log_mel(padded, 80))


def test_dynamic_range_clamp():
    out = mo.log_mel(mo.synthetic_audio(1, seed=2)[0], 128)
    assert out.max() - out.min() <= 2.0 + 1e-6  # 8 decades / 4
    assert out.min() >= -1.5 - 1e-6 or out.max() > -1.5


@pytest.mark.parametrize("n_mels", [80, 128])
def test_product_filterbank_matches_restatement(n_mels):
    import whisper_amd

    fb, win = whisper_amd.mel_filterbank(n_mels)
    ref = mo.mel_filterbank(n_mels)
    np.testing.assert_array_equal(fb != 0, ref != 0)
    np.testing.assert_allclose(fb, ref, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(win, mo.hann_window(), rtol=1e-6, atol=1e-7)


def test_log_mel_argument_errors():
    import wq4
    import whisper_amd

    with pytest.raises(wq4.WQ4Error):
        whisper_amd.mel_filterbank(0)
    with pytest.raises(wq4.WQ4Error):
        whisper_amd.mel_filterbank(257)
