"""Activation-range guard (layers.rs:12-58, wq4_device.hpp
split_act): every internal producer feeds the MFMAs f16 pairs of x * 2^4,
finite for |x| < 4094, where the reference's f32 stays finite far beyond.

Stress fixtures through the whole model (tiny_test, synthetic weights written
to a GGUF and loaded by the product's loader; the oracle gets the same bytes):
  * "residual": the decoder's attn.out / cross_attn.out / mlp.2 projections
    scaled by 3e3, so the decoder residual stream reaches ~1e3-2e4.  The
    LayerNorm fold feeds that raw stream (x * gamma) to the MFMAs and
    overflows; the model must notice (non-finite logits flag), re-run on the
    LayerNorm path (bounded operands) and return the f32 oracle's tokens.
  * "fc1": decoder layer 0's mlp.0 scaled by 5e3 -- fc1 outputs ~1e3-2e4, the
    GELU output is fc2's operand and the LayerNorm path does not bound it:
    the model must fall to range tier 2 (every FFN through the ABI's
    per-call operand scales, wq4_ffn_forward_ws) and return the oracle's
    tokens.
  * "value": decoder layer 0's attn.value scaled by 3e5 -- the self-attention
    output (a convex combination of values ~1e4) is the out projection's
    operand: tiers 1 and 2 still overflow, range tier 3 (every attention
    output in f32, the output projections through the ABI's per-call operand
    scales, wq4_linear_forward_ws) must return the oracle's tokens.
The oracle is float32 numpy (oracle/whisper_oracle.py) with a float64 run to
check the fixture has no near-ties; it also records the activation
magnitudes the fixture promises (CPU test below)."""
from __future__ import annotations

import os

import numpy as np
import pytest

import oracle
import whisper_oracle as wo

SEED = 1234
STEPS = 24
CLIPS = (0, 1)
SCALE = {"residual": 3.0e3, "fc1": 5.0e3, "value": 3.0e5}


def _scaled_names(kind: str) -> list[str]:
    if kind == "residual":
        return [f"decoder.blocks.{i}.{p}.{s}" for i in range(2) for p in ("attn.out", "cross_attn.out", "mlp.2")
                for s in ("weight", "bias")]
    if kind == "value":
        return ["decoder.blocks.0.attn.value.weight", "decoder.blocks.0.attn.value.bias"]
    return ["decoder.blocks.0.mlp.0.weight", "decoder.blocks.0.mlp.0.bias"]


def stress_tensors(kind: str) -> dict[str, np.ndarray]:
    """The synthetic tiny_test tensors (oracle generator = the product's) with
    the fixture's tensors scaled by SCALE."""
    import write_gguf

    out = {}
    scaled = set(_scaled_names(kind))
    for name, shape, lo, hi in write_gguf.synthetic_specs("tiny_test"):
        a = oracle.synth_uniform(SEED, name, int(np.prod(shape)), lo, hi).reshape(shape)
        out[name] = (a * np.float32(SCALE[kind])).astype(np.float32) if name in scaled else a
    return out


class _Recorder(wo.SynthWhisper):
    """The oracle, recording max |residual stream| (LayerNorm inputs of the
    decoder blocks) and max |fc1 output| of the decoder."""

    def __init__(self, *a, **k):
        self.max_resid = 0.0
        self.max_fc1 = 0.0
        self.max_attn = 0.0  # self-attention outputs (the out projection's operand)
        super().__init__(*a, **k)

    def layer_norm(self, x, p):
        if p.startswith("decoder.blocks."):
            self.max_resid = max(self.max_resid, float(np.max(np.abs(x))))
        return super().layer_norm(x, p)

    def linear(self, x, p, bias=True):
        if p.startswith("decoder.blocks.") and p.endswith(".attn.out") and "cross" not in p:
            self.max_attn = max(self.max_attn, float(np.max(np.abs(x))))
        y = super().linear(x, p, bias)
        if p.startswith("decoder.blocks.") and p.endswith("mlp.0"):
            self.max_fc1 = max(self.max_fc1, float(np.max(np.abs(y))))
        return y


def stress_oracle(kind: str, dtype=np.float32) -> _Recorder:
    import write_gguf

    m = _Recorder("tiny_test", SEED, dtype=dtype)
    t = stress_tensors(kind)
    for name in _scaled_names(kind):
        a = t[name]
        if write_gguf.should_quantize(name, a.shape):
            q = oracle.quantize_convert_np(a.reshape(-1))
            m.w[name] = oracle.dequantize_np(q, a.size).reshape(a.shape).astype(dtype)
        else:
            m.w[name] = a.astype(dtype)
    return m


def _mels(n_mels: int) -> np.ndarray:
    return np.stack([wo.synthetic_mel(c, n_mels) for c in CLIPS])


_CACHE: dict = {}


def oracle_run(kind: str):
    if kind not in _CACHE:
        m32 = stress_oracle(kind)
        mel = _mels(m32.cfg["n_mels"])
        t32 = m32.transcribe(mel, 50259, STEPS, eot_stop=False)
        m64 = stress_oracle(kind, np.float64)
        t64 = m64.transcribe(mel, 50259, STEPS, eot_stop=False)
        _CACHE[kind] = (t32, t64, m32.max_resid, m32.max_fc1, m32.max_attn)
    return _CACHE[kind]


@pytest.mark.parametrize("kind", ["residual", "fc1", "value"])
def test_stress_fixture_reaches_the_range(kind):
    """CPU: the fixture really drives the activations to 1e3-2e4 (beyond the
    4094 the f16 pair of x * 2^4 holds), and the f32 oracle's tokens equal the
    f64 oracle's (no near-ties: the GPU comparison below is meaningful)."""
    t32, t64, max_resid, max_fc1, max_attn = oracle_run(kind)
    print(f"{kind}: max |residual| {max_resid:.4g}, max |fc1| {max_fc1:.4g}, max |attention| {max_attn:.4g}")
    assert t32 == t64
    if kind == "residual":
        assert 4094 < max_resid <= 2e4, max_resid
        assert max_fc1 < 100, max_fc1
    elif kind == "fc1":
        assert 4094 < max_fc1 <= 2e4, max_fc1
    else:
        assert max_attn > 4094, max_attn


def _write(kind: str, tmp_path) -> str:
    import write_gguf

    p = os.path.join(str(tmp_path), f"stress_{kind}.gguf")
    write_gguf.write_gguf(p, stress_tensors(kind), f"stress-{kind}", quantize=oracle.quantize_convert_np)
    return p


@pytest.mark.gpu
def test_residual_overflow_recovers_oracle_tokens(tmp_path):
    import torch

    import whisper_amd

    t32, _, _, _, _ = oracle_run("residual")
    m = whisper_amd.WhisperModel.from_gguf(_write("residual", tmp_path), "tiny_test", max_batch=len(CLIPS))
    assert not m.wide_range
    mel = torch.from_numpy(_mels(m.config["n_mels"])).cuda()
    toks = m.transcribe(mel, 50259, STEPS, eot_stop=False)
    assert m.wide_range  # the fold overflowed and the transcribe was re-run on the LayerNorm path
    assert toks == t32
    toks2 = m.transcribe(mel, 50259, STEPS, eot_stop=False)  # sticky: straight on the LayerNorm path
    assert toks2 == t32
    m.close()


@pytest.mark.gpu
def test_fc1_overflow_recovers_oracle_tokens(tmp_path):
    """fc1 outputs beyond the f16 pair's range recover
    through range tier 2 (per-call operand scales on every FFN) and give the
    f32 oracle's tokens, as the reference's f32 path does."""
    import torch

    import whisper_amd

    t32, _, _, _, _ = oracle_run("fc1")
    m = whisper_amd.WhisperModel.from_gguf(_write("fc1", tmp_path), "tiny_test", max_batch=len(CLIPS))
    mel = torch.from_numpy(_mels(m.config["n_mels"])).cuda()
    toks = m.transcribe(mel, 50259, STEPS, eot_stop=False)
    assert m.range_tier == 2
    assert toks == t32
    toks2 = m.transcribe(mel, 50259, STEPS, eot_stop=False)  # sticky: straight on tier 2
    assert toks2 == t32 and m.range_tier == 2
    m.close()


@pytest.mark.gpu
def test_value_overflow_recovers_oracle_tokens(tmp_path):
    """an attention output past the f16 pair's range
    (attention.rs:243-298 is f32 to FLT_MAX) recovers through range tier 3 --
    f32 attention outputs, output projections on per-call operand scales --
    and gives the f32 oracle's tokens, sticky for the model."""
    import torch

    import whisper_amd

    t32, _, _, _, _ = oracle_run("value")
    m = whisper_amd.WhisperModel.from_gguf(_write("value", tmp_path), "tiny_test", max_batch=len(CLIPS))
    mel = torch.from_numpy(_mels(m.config["n_mels"])).cuda()
    toks = m.transcribe(mel, 50259, STEPS, eot_stop=False)
    assert m.range_tier == 3
    assert toks == t32
    toks2 = m.transcribe(mel, 50259, STEPS, eot_stop=False)  # sticky: straight on tier 3
    assert toks2 == t32 and m.range_tier == 3
    m.close()


@pytest.mark.gpu
def test_normal_model_never_flags():
    import torch

    import whisper_amd

    m = whisper_amd.WhisperModel("tiny_test", SEED, max_batch=2)
    mel = torch.from_numpy(_mels(m.config["n_mels"])).cuda()
    m.transcribe(mel, 50259, STEPS, eot_stop=False)
    m.transcribe(mel, None, STEPS, eot_stop=True)
    assert not m.wide_range and m.range_tier == 0
    m.close()


@pytest.mark.gpu
def test_pipelined_batches_recover_through_the_tiers(tmp_path):
    """wa_transcribe_batches on the fc1 stress model: the first batch flags in
    the pipeline, is re-run through wa_transcribe's tiers (tier 2), and every
    batch -- including those decoded after the model went to tier 2 -- gives
    the f32 oracle's tokens; the value stress model likewise through tier 3."""
    import torch

    import whisper_amd

    t32, _, _, _, _ = oracle_run("fc1")
    m = whisper_amd.WhisperModel.from_gguf(_write("fc1", tmp_path), "tiny_test", max_batch=len(CLIPS))
    mel = torch.from_numpy(_mels(m.config["n_mels"])).cuda()
    out = m.transcribe_batches(torch.stack([mel, mel, mel]), 50259, STEPS, eot_stop=False)
    assert m.range_tier == 2
    assert out == [t32, t32, t32]
    m.close()
    tv, _, _, _, _ = oracle_run("value")
    m = whisper_amd.WhisperModel.from_gguf(_write("value", tmp_path), "tiny_test", max_batch=len(CLIPS))
    out = m.transcribe_batches(torch.stack([mel, mel]), 50259, STEPS, eot_stop=False)
    assert m.range_tier == 3
    assert out == [tv, tv]
    m.close()
