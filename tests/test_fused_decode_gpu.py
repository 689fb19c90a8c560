"""In-launch projections of the decode step (wa_headproj.hpp, VERDICT r03
item 2): in few-clip groups the decoder self-attention forms its head's q / k
/ v and the K / V cross-attention its query inside their own launches,
replacing the qkv and cq GEMM launches; in groups of up to 16 clips on the
encoder planes the cross-attention's query transform forms the query itself,
replacing the cq GEMM launch (decoder.rs:77-112, attention.rs:93-125,208-236).

The fused kernels reproduce the decode-step GEMM's arithmetic (wq4_skinny.hip)
exactly, so under kernel policy 3 (every <= 32-row GEMM on that kernel) a
transcribe with the fused launches and one with the GEMM launches give the
SAME BITS: tokens and every traced decode-step logit.  Under the default
policy the GEMM launches run the 8-wave decode kernel (another summation
order), and parity is the oracle's (test_model_gpu.py, test_full_size_gpu.py
run the product default: the GEMM launches; the in-launch forms are
diagnostics until measured faster)."""
from __future__ import annotations

import numpy as np
import pytest

import whisper_oracle as wo

pytestmark = pytest.mark.gpu

SEED = 1234


def _trace_ids(B: int, steps: int, V: int) -> np.ndarray:
    rng = np.random.default_rng(5)
    return rng.integers(0, V, size=(B, steps + 1, 16), dtype=np.int32)


def _run(m, mel, ids, lang, steps, fused: int):
    prev = m.set_fused_projections(fused)
    try:
        return m.transcribe_trace(mel, ids, lang, steps, eot_stop=False)
    finally:
        m.set_fused_projections(prev)


@pytest.mark.parametrize("variant,n_mels,B,lang,steps", [
    ("tiny_test", 80, 1, 50259, 24),   # D = 384: 3 units per subtile (padded DMA regions)
    ("tiny_test", 80, 3, None, 24),    # three clips, auto language
    ("medium", 80, 1, 50259, 16),      # D = 1024, H = 16
    ("large_v3", 128, 2, 50259, 16),   # D = 1280, H = 20: the product's one/two-clip decode
    ("tiny_test", 80, 16, 50259, 24),  # a 16-clip group on the encoder planes: the fused query transform
    ("tiny_test", 80, 11, None, 24),   # 11 rows of the 16-row tile, auto language
    ("large_v3", 128, 16, 50259, 8),   # the bench's decode-group shape
])
def test_fused_projections_bit_identical_under_policy3(variant, n_mels, B, lang, steps):
    import torch

    import whisper_amd
    import wq4

    m = whisper_amd.WhisperModel(variant, SEED, max_batch=B)
    V = m.config["n_vocab"]
    mel = torch.from_numpy(np.stack([wo.synthetic_mel(60 + c, n_mels) for c in range(B)])).cuda()
    ids = _trace_ids(B, steps, V)
    wq4.set_kernel_policy(3)
    try:
        t_gemm, l_gemm = _run(m, mel, ids, lang, steps, fused=0)
        runs = {mask: _run(m, mel, ids, lang, steps, fused=mask) for mask in (1, 2, 3, 5, 7)}
    finally:
        wq4.set_kernel_policy(0)
    for mask, (t_fused, l_fused) in runs.items():
        assert t_fused == t_gemm, mask
        assert np.array_equal(l_fused[:, 1:], l_gemm[:, 1:], equal_nan=True), \
            (mask, float(np.nanmax(np.abs(l_fused[:, 1:] - l_gemm[:, 1:]))))
    m.close()


def test_fused_default_policy_tokens_match_oracle():
    """Default kernel policy (8-wave decode GEMMs) with every in-launch
    projection on: tiny_test tokens equal the f32 oracle's, explicit and auto
    language."""
    import torch

    import whisper_amd

    m = whisper_amd.WhisperModel("tiny_test", SEED, max_batch=2)
    m.set_fused_projections(7)
    o = wo.SynthWhisper("tiny_test", SEED)
    mel_np = np.stack([wo.synthetic_mel(70 + c, 80) for c in range(2)])
    mel = torch.from_numpy(mel_np).cuda()
    for lang in (50259, None):
        got = m.transcribe(mel, lang, 32, eot_stop=False)
        ref = o.transcribe(mel_np, lang, 32, eot_stop=False)
        assert got == ref, lang
    m.close()
