"""Pipelined transcribes (wa_transcribe_batches, include/whisper_amd.h): the
conv stem and first encoder layers of batch i + 1 run on a CU-masked stream
beside batch i's decode, the rest of that encoder after it.  Every kernel
computes what it computes in wa_transcribe, so the tokens must EQUAL those of
one wa_transcribe per batch -- at every overlap depth (WA_ENC_OVERLAP pins
it; unset: adapted per batch), for decode groups on the encoder planes and
the few-clip cross K / V caches, explicit and auto language, EOT stop and
fixed length.  The full-size check against the oracle fixture is
tests/test_full_size_gpu.py::test_full_size_tokens_pipelined."""
from __future__ import annotations

import numpy as np
import pytest

import whisper_oracle as wo

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as _t

    assert _t.cuda.is_available()
    return _t


@pytest.fixture(scope="module")
def model():
    import whisper_amd

    return whisper_amd.WhisperModel("tiny_test", 1234, max_batch=16)


def mels(nb, b, first=0):
    return np.stack([np.stack([wo.synthetic_mel(first + i * b + c, 80) for c in range(b)]) for i in range(nb)])


@pytest.mark.parametrize("B,overlap,lang,eot", [
    (16, None, 50259, True),   # two plane groups, adaptive depth
    (16, "0", 50259, True),    # only the conv stem beside the decode
    (16, "1", None, True),     # auto language
    (16, "2", 50259, False),   # the whole encoder beside the decode, fixed length
    (3, None, 50259, True),    # few clips: the cross K / V caches
    (1, "1", None, False),
])
def test_pipelined_tokens_equal_sequential(torch, model, monkeypatch, B, overlap, lang, eot):
    x = torch.from_numpy(mels(3, B, first=7 * B)).cuda()
    seq = [model.transcribe(x[i], lang, max_tokens=24, eot_stop=eot) for i in range(3)]
    if overlap is None:
        monkeypatch.delenv("WA_ENC_OVERLAP", raising=False)
    else:
        monkeypatch.setenv("WA_ENC_OVERLAP", overlap)
    got = model.transcribe_batches(x, lang, max_tokens=24, eot_stop=eot)
    assert got == seq
    st = model.pipeline_stats()
    assert st["batches"] == 3 and st["masked_cus"] == 32
    if overlap is not None:
        assert st["overlap_layers"] == int(overlap)
    t = model.last_timings()
    assert t["decode_ms"] > 0 and (eot or t["steps"] == 24)


def test_pipelined_single_batch_and_errors(torch, model):
    import wq4

    x = torch.from_numpy(mels(1, 2)).cuda()
    assert model.transcribe_batches(x, 50259, max_tokens=16) == [model.transcribe(x[0], 50259, max_tokens=16)]
    with pytest.raises(wq4.WQ4Error):
        model.transcribe_batches(torch.from_numpy(mels(2, 17)).cuda(), 50259, max_tokens=4)
    with pytest.raises(wq4.WQ4Error):
        model.transcribe_batches(x, 50259, max_tokens=225)
