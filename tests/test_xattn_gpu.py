"""GPU parity tests of the K/V-cache-free decoder cross-attention
(whisper-burn_amd/csrc/whisper/wa_xattn.hip) against the reference's
cross-attention restated in float64 numpy:

    K = enc Wk^T, V = enc Wv^T + bv        (attention.rs:204-236, key bias absent)
    out_h = softmax(q_h K_h^T / sqrt(64)) V_h   (attention.rs:243-298)

with Wk, Wv dequantized from the same Q4_0 bytes (tests.rs:60-87) or f16.
Tolerance (stated here and in DESIGN.md "Numerics"): max|gpu - ref| <=
2e-5 * max|ref| for the f16x2 precision (f32-faithful), 5e-3 for f16.
Covers the Large-V3 (H = 20: two head tiles, the second in LDS), Medium
(H = 16) and test (H = 6) shapes, Tq = 4 prompt rows, 33 clips (several
query-row groups), short T, and f16 weights.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle
import wq4

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as _t

    assert _t.cuda.is_available()
    return _t


def reference(q, wk, wv, bv, enc, Tq, H):
    B, T, D = enc.shape
    q = q.astype(np.float64).reshape(B, Tq, H, 64)
    K = (enc.astype(np.float64) @ wk.astype(np.float64).T).reshape(B, T, H, 64)
    V = (enc.astype(np.float64) @ wv.astype(np.float64).T + bv).reshape(B, T, H, 64)
    s = np.einsum("bqhd,bthd->bhqt", q, K) / 8.0
    s -= s.max(axis=-1, keepdims=True)
    p = np.exp(s)
    p /= p.sum(axis=-1, keepdims=True)
    o = np.einsum("bhqt,bthd->bqhd", p, V)
    return o.reshape(B * Tq, H * 64)


def run_case(torch, B, Tq, T, H, wtype=0, prec=wq4.PREC_F16X2, seed=0):
    import whisper_amd

    D = 64 * H
    rng = np.random.default_rng(seed)
    enc = rng.standard_normal((B, T, D)).astype(np.float32)
    q = (2.0 * rng.standard_normal((B * Tq, D))).astype(np.float32)
    wk = rng.uniform(-0.05, 0.05, (D, D)).astype(np.float32)
    wv = rng.uniform(-0.05, 0.05, (D, D)).astype(np.float32)
    bv = rng.uniform(-0.02, 0.02, D).astype(np.float32)
    if wtype == 0:
        rk, rv = wq4.quantize_q4_0(wk), wq4.quantize_q4_0(wv)
        wk_d = oracle.dequantize_np(rk, D * D).reshape(D, D)
        wv_d = oracle.dequantize_np(rv, D * D).reshape(D, D)
    else:
        hk, hv = wk.astype(np.float16), wv.astype(np.float16)
        rk, rv = hk.view(np.uint8).ravel(), hv.view(np.uint8).ravel()
        wk_d, wv_d = hk.astype(np.float32), hv.astype(np.float32)
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    got = whisper_amd.xattn_check(cu(q), cu(rk), cu(rv), cu(bv), cu(enc), Tq, H, wtype, prec).cpu().numpy()
    ref = reference(q, wk_d, wv_d, bv, enc, Tq, H)
    return got, ref


@pytest.mark.parametrize("B,Tq,T,H", [
    (3, 1, 1500, 20),   # Large-V3 decode step
    (2, 4, 1500, 20),   # Large-V3 prompt (Tq = 4)
    (2, 1, 1500, 16),   # Medium
    (5, 1, 1500, 6),    # test configuration
    (33, 1, 200, 6),    # > 32 query rows, short T
    (1, 1, 37, 20),     # T not a multiple of the 16-frame sub-chunk, one chunk per split
])
def test_xattn_matches_reference(torch, B, Tq, T, H):
    got, ref = run_case(torch, B, Tq, T, H)
    err = np.abs(got - ref).max() / np.abs(ref).max()
    assert err <= 2e-5, err


def test_xattn_f16_weights(torch):
    got, ref = run_case(torch, 2, 1, 1500, 20, wtype=1, seed=3)
    assert np.abs(got - ref).max() / np.abs(ref).max() <= 2e-5


def test_xattn_f16_precision(torch):
    got, ref = run_case(torch, 2, 1, 1500, 20, prec=wq4.PREC_F16, seed=5)
    assert np.abs(got - ref).max() / np.abs(ref).max() <= 5e-3


@pytest.mark.parametrize("B,Tq,T,H", [
    (1, 1, 1500, 20),   # Large-V3, one clip (BASELINE config 3)
    (3, 1, 1500, 20),
    (1, 4, 1500, 20),   # one clip's prompt rows
    (8, 1, 1500, 20),   # the largest split-phase batch
    (2, 1, 1500, 16),   # Medium (one head tile)
    (2, 1, 200, 6),     # test configuration (4 waves per slice)
    (1, 1, 37, 20),     # a ragged last sub-chunk, one sub-chunk per split
])
def test_xattn_small_rows_bit_identical(torch, monkeypatch, B, Tq, T, H):
    """The split-phase path for few query rows (scores / softmax / z launches,
    wa_xattn.hip) reproduces the fused kernel's partials bit for bit, so the
    output -- and a clip's tokens -- do not depend on which path its batch
    size selects; both are within the f16x2 tolerance of the reference."""
    monkeypatch.setenv("WA_XATTN_SMALL_ROWS", "0")
    fused, ref = run_case(torch, B, Tq, T, H, seed=11)
    monkeypatch.setenv("WA_XATTN_SMALL_ROWS", "8")
    split, _ = run_case(torch, B, Tq, T, H, seed=11)
    assert np.array_equal(fused, split), np.abs(fused - split).max()
    assert np.abs(split - ref).max() / np.abs(ref).max() <= 2e-5


def test_xattn_small_rows_f16_precision(torch, monkeypatch):
    monkeypatch.setenv("WA_XATTN_SMALL_ROWS", "0")
    fused, _ = run_case(torch, 2, 1, 1500, 20, prec=wq4.PREC_F16, seed=12)
    monkeypatch.setenv("WA_XATTN_SMALL_ROWS", "8")
    split, _ = run_case(torch, 2, 1, 1500, 20, prec=wq4.PREC_F16, seed=12)
    assert np.array_equal(fused, split)


def test_xattn_rows_independent(torch):
    """Each query row's result is independent of the batch it runs in."""
    import whisper_amd

    H, D, T = 20, 1280, 1500
    rng = np.random.default_rng(9)
    enc = torch.from_numpy(rng.standard_normal((4, T, D)).astype(np.float32)).cuda()
    q = torch.from_numpy(rng.standard_normal((4, D)).astype(np.float32)).cuda()
    rk = torch.from_numpy(wq4.quantize_q4_0(rng.uniform(-0.05, 0.05, (D, D)).astype(np.float32))).cuda()
    bv = torch.zeros(D, device="cuda")
    full = whisper_amd.xattn_check(q, rk, rk, bv, enc, 1, H)
    one = whisper_amd.xattn_check(q[2:3], rk, rk, bv, enc[2:3], 1, H)
    assert torch.equal(full[2:3], one)


@pytest.mark.parametrize("B,Tq,T,H", [
    (1, 1, 1500, 20),   # Large-V3, one clip (BASELINE config 3): the product's few-clip form
    (3, 1, 1500, 20),
    (1, 4, 1500, 20),   # one clip's prompt rows
    (8, 1, 1500, 16),   # Medium, the largest few-clip group
    (2, 3, 37, 6),      # short T (one split), the auto-language prompt's 3 rows
    (5, 1, 200, 6),
])
def test_xattn_kv_cache_form(torch, B, Tq, T, H):
    """The few-clip cross-attention over cached K / V (cross_attn_kv_kernel,
    attention.rs:177-236's cached form: f32 products, online softmax, split
    merge by the last arriver) against float64 softmax(q K^T / 8) V."""
    import whisper_amd

    rng = np.random.default_rng(B * 100 + Tq * 10 + H)
    D = 64 * H
    q = (2.0 * rng.standard_normal((B * Tq, D))).astype(np.float32)
    k = rng.standard_normal((B, H, T, 64)).astype(np.float32)
    v = rng.standard_normal((B, H, T, 64)).astype(np.float32)
    got = whisper_amd.xattn_kv_check(torch.from_numpy(q).cuda(), torch.from_numpy(k).cuda(),
                                     torch.from_numpy(v).cuda(), Tq).cpu().numpy()
    qh = q.astype(np.float64).reshape(B, Tq, H, 64)
    s = np.einsum("bqhd,bhtd->bhqt", qh, k.astype(np.float64)) / 8.0
    s -= s.max(axis=-1, keepdims=True)
    p = np.exp(s)
    p /= p.sum(axis=-1, keepdims=True)
    ref = np.einsum("bhqt,bhtd->bqhd", p, v.astype(np.float64)).reshape(B * Tq, D)
    # f32 products and sums over T keys, the output split into an exact-to-
    # 2^-22 f16 pair (the output projection's operand) and read back
    err = np.abs(got - ref).max() / np.abs(v).max()
    assert err <= 2e-6, err
