"""Direct parity tests of the attention and logits kernels at Whisper sizes,
through their C-ABI check entry points, against float64 numpy.

  * encoder self-attention (attention.rs:243-298, non-causal) at Large-V3's
    H = 20, D = 1280, T = 1500 and Medium's H = 16;
  * decoder self-attention with the KV cache (attention.rs:62-125) at
    kv = 0 .. 227 cached keys (+1 new: up to the 228 keys of a 224-token
    decode), H = 20 and 16, and the causal 4-token prompt;
  * the fused tied-embedding logits + greedy pick at V = 51866 with planted
    exact ties (Rust max_by keeps the LAST maximum, whisper.rs:131-138) and
    the EOT suppression of the first steps (whisper.rs:97-98,120-122).

Tolerance (written per test): every product of these kernels is an
exact-to-2^-22 f16 pair product with f32 accumulation and an f32 softmax
(DESIGN.md §3), so an attention output is within a few 2^-22 of max |v|.
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _sdpa64(q, k, v, causal_from=None):
    """softmax(q k^T / 8) v in float64; q [Tq, 64], k, v [Tk, 64].  causal_from:
    query t sees keys <= causal_from + t (attention.rs:270-287)."""
    s = (q.astype(np.float64) @ k.astype(np.float64).T) / 8.0
    if causal_from is not None:
        Tq, Tk = s.shape
        mask = np.arange(Tk)[None, :] > causal_from + np.arange(Tq)[:, None]
        s = np.where(mask, -np.inf, s)
    s = s - s.max(axis=-1, keepdims=True)
    p = np.exp(s)
    p /= p.sum(axis=-1, keepdims=True)
    return p @ v.astype(np.float64)


@pytest.mark.parametrize("H,B", [(20, 1), (16, 2), (20, 3)])  # 4-wave (few clips) and 8-wave workgroups
def test_encoder_attention_whisper_size(H, B):
    import torch

    import whisper_amd

    T, D = 1500, 64 * H
    rng = np.random.default_rng(H * 7 + B)
    qkv = rng.standard_normal((B * T, 3 * D)).astype(np.float32)
    qkv[:, :D] *= 2.0  # peaked softmax rows as well as flat ones
    out = whisper_amd.encoder_attention_check(torch.from_numpy(qkv).cuda(), T, H).cpu().numpy()
    worst = 0.0
    for b in range(B):
        x = qkv[b * T:(b + 1) * T]
        for h in range(H):
            ref = _sdpa64(x[:, h * 64:(h + 1) * 64], x[:, D + h * 64:D + (h + 1) * 64],
                          x[:, 2 * D + h * 64:2 * D + (h + 1) * 64])
            got = out[b * T:(b + 1) * T, h * 64:(h + 1) * 64]
            vmax = np.abs(x[:, 2 * D + h * 64:2 * D + (h + 1) * 64]).max()
            err = np.abs(got - ref).max()
            worst = max(worst, err / vmax)
            # f16x2 products (2^-22, operands scaled so no lo half is a flushed
            # f16 subnormal) + f32 softmax / accumulation over 1500 keys: the
            # numpy f32 restatement itself is ~6e-7 x max|v| off f64 here
            assert err <= 4e-6 * vmax, f"b {b} head {h}: {err:.3e} vs max|v| {vmax:.3e}"
    print(f"encoder attention H={H}: worst error {worst:.2e} x max|v|")


@pytest.mark.parametrize("H", [20, 16])
def test_decoder_self_attention_kv_range(H):
    import torch

    import whisper_amd

    D, ctx, B = 64 * H, 448, 3
    rng = np.random.default_rng(H)
    cache_k = rng.standard_normal((B, H, ctx, 64)).astype(np.float32)
    cache_v = rng.standard_normal((B, H, ctx, 64)).astype(np.float32)
    ck_dev, cv_dev = torch.from_numpy(cache_k).cuda(), torch.from_numpy(cache_v).cuda()
    for kv in (0, 1, 2, 15, 16, 17, 63, 64, 65, 127, 128, 200, 226, 227):
        qkv = rng.standard_normal((B, 3 * D)).astype(np.float32)
        qkv[:, :D] *= 3.0
        out = whisper_amd.self_attention_check(torch.from_numpy(qkv).cuda(), ck_dev, cv_dev, 1, H, kv).cpu().numpy()
        kc, vc = ck_dev.cpu().numpy(), cv_dev.cpu().numpy()
        for b in range(B):
            for h in range(H):
                sl = slice(h * 64, (h + 1) * 64)
                # the new key / value appended at index kv (decoder.rs:77-112)
                assert np.array_equal(kc[b, h, kv], qkv[b, D:][sl]) and np.array_equal(vc[b, h, kv], qkv[b, 2 * D:][sl])
                ref = _sdpa64(qkv[b, :D][sl][None], kc[b, h, :kv + 1], vc[b, h, :kv + 1])[0]
                err = np.abs(out[b, sl] - ref).max()
                # f32 scores and softmax, f32 accumulation over <= 228 keys
                assert err <= 2e-6 * np.abs(vc[b, h, :kv + 1]).max(), f"kv {kv} clip {b} head {h}: {err:.3e}"


def test_decoder_self_attention_prompt_causal():
    import torch

    import whisper_amd

    H, Tq, B, ctx = 20, 4, 2, 448
    D = 64 * H
    rng = np.random.default_rng(5)
    ck = torch.zeros((B, H, ctx, 64), device="cuda")
    cv = torch.zeros((B, H, ctx, 64), device="cuda")
    qkv = rng.standard_normal((B * Tq, 3 * D)).astype(np.float32)
    out = whisper_amd.self_attention_check(torch.from_numpy(qkv).cuda(), ck, cv, Tq, H, 0).cpu().numpy()
    for b in range(B):
        x = qkv[b * Tq:(b + 1) * Tq]
        for h in range(H):
            sl = slice(h * 64, (h + 1) * 64)
            ref = _sdpa64(x[:, :D][:, sl], x[:, D:2 * D][:, sl], x[:, 2 * D:][:, sl], causal_from=0)
            assert np.abs(out[b * Tq:(b + 1) * Tq, sl] - ref).max() <= 2e-6 * np.abs(x[:, 2 * D:][:, sl]).max()


@pytest.mark.parametrize("step", [0, 1, 2, 40])
def test_logits_argmax_ties_and_eot(step):
    """V = 51866 (Large-V3), D = 1280, 6 clips.  Planted: clip 0's maximum is
    an exact tie between rows 1000 and 40000 (identical embedding rows give
    identical bits) -> 40000 (the LAST maximum); clip 1's maximum is EOT
    (50257) -> masked while step + 1 < 3, picked afterwards; clip 2's maximum
    is tied between rows 7 and 51865 (the last row) -> 51865."""
    import torch

    import whisper_amd

    V, D, B = 51866, 1280, 6
    rng = np.random.default_rng(step + 11)
    emb = (rng.uniform(-1, 1, (V, D)) * 0.03).astype(np.float32)
    hid = rng.standard_normal((B, D)).astype(np.float32)
    big = hid / np.linalg.norm(hid, axis=1, keepdims=True)
    emb[1000] = emb[40000] = big[0] * 3.0
    emb[50257] = big[1] * 3.0
    emb[50100] = big[1] * 2.5  # clip 1's runner-up
    emb[7] = emb[51865] = big[2] * 3.0
    tok, lg = whisper_amd.logits_argmax_check(torch.from_numpy(hid).cuda(), torch.from_numpy(emb).cuda(), step)
    tok, lg = tok.cpu().numpy(), lg.cpu().numpy()
    ref = hid.astype(np.float64) @ emb.astype(np.float64).T
    suppress = step + 1 < 3
    if suppress:
        ref[:, 50257] = -np.inf
    for b in range(B):
        fin = np.isfinite(ref[b])
        # exact-to-2^-22 pairs, f32 accumulation over D = 1280
        assert np.abs(lg[b][fin] - ref[b][fin]).max() <= 4e-6 * np.abs(ref[b][fin]).max() + 1e-6
        assert (lg[b][~fin] == -np.inf).all()
        want = int(len(lg[b]) - 1 - np.argmax(lg[b][::-1]))  # last max of the kernel's own logits
        assert tok[b] == want, (b, tok[b], want)
    assert lg[0, 1000] == lg[0, 40000] and tok[0] == 40000
    assert tok[1] == (50100 if suppress else 50257)
    assert lg[2, 7] == lg[2, 51865] and tok[2] == 51865
