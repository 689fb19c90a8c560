"""CPU oracle vs the reference's golden vectors and known-answer tests.

The oracle (oracle/q4_oracle.c, oracle/oracle.py) is pinned here before any
GPU test trusts it:
  * quantizer bytes == scripts/convert_whisper.py:quantize_q4_0 run on the
    reference itself (tests/golden/q4_golden.npz, made by make_golden.py);
  * the assertions of src/gguf/tests.rs that need no GPU, re-expressed;
  * f16 conversion exhaustively against numpy.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle


def test_f16_to_f32_exhaustive():
    L = oracle.lib()
    bits = np.arange(65536, dtype=np.uint16)
    want = bits.view(np.float16).astype(np.float32)
    got = np.array([L.q4o_f16_to_f32(int(b)) for b in bits[::7]], np.float32)
    w = want[::7]
    nan = np.isnan(w)
    assert np.array_equal(np.isnan(got), nan)
    assert np.array_equal(got[~nan].view(np.uint32), w[~nan].view(np.uint32))


def test_f32_to_f16_matches_numpy():
    L = oracle.lib()
    rng = np.random.default_rng(1)
    # random bit patterns over the whole f32 range + the f16 subnormal / tie band
    xs = np.concatenate([
        rng.integers(0, 2**32, 20000, dtype=np.uint64).astype(np.uint32).view(np.float32),
        (rng.standard_normal(20000) * 1e-5).astype(np.float32),
        np.array([65504, 65519.99, 65520, 6.1035156e-05, 5.9604645e-08, 2.9802322e-08, 2.9802326e-08,
                  1.0 + 2**-11, 1.0 + 3 * 2**-11, 0.0, -0.0], np.float32),
    ])
    xs = xs[~np.isnan(xs)]
    with np.errstate(over="ignore"):  # overflow to +-inf is part of what is checked
        want = xs.astype(np.float16).view(np.uint16)
    got = np.array([L.q4o_f32_to_f16(float(x)) for x in xs], np.uint16)
    assert np.array_equal(got, want)


def _cases(golden):
    return sorted(k[3:] for k in golden.files if k.startswith("in/"))


def test_golden_fixture_provenance(golden):
    assert str(golden["meta/numpy_version"]).startswith("2.")
    # the survey's probe of the reference quantizer
    assert golden["q4/ramp_pm1"].tobytes().hex() == "9230819192a2a3a3b4b4c5c5d6d6e6e7f7f8"


def test_convert_quantizer_c_matches_reference_bytes(golden):
    for name in _cases(golden):
        x = golden[f"in/{name}"]
        assert np.array_equal(oracle.quantize_convert_c(x), golden[f"q4/{name}"]), name


def test_convert_quantizer_numpy_matches_reference_bytes(golden):
    for name in _cases(golden):
        x = golden[f"in/{name}"]
        assert np.array_equal(oracle.quantize_convert_np(x), golden[f"q4/{name}"]), name


def test_test_quantizer_vs_reference_quantizer(golden):
    """tests.rs:24-57 (truncating (v/d + 8.5) as u8) and convert_whisper.py
    (round half-even of v/d) agree on every golden case except exact ties."""
    for name in _cases(golden):
        x = golden[f"in/{name}"]
        t = oracle.quantize_test(x).reshape(-1, 18)
        g = golden[f"q4/{name}"].reshape(-1, 18)
        assert np.array_equal(t[:, :2], g[:, :2]), name  # identical f16 scales
        if name != "ties_d1":
            assert np.array_equal(t, g), name
    t = oracle.quantize_test(golden["in/ties_d1"]).reshape(-1, 18)
    g = golden["q4/ties_d1"].reshape(-1, 18)
    dq_t = oracle.dequantize_np(t.ravel(), 32)
    dq_g = oracle.dequantize_np(g.ravel(), 32)
    x = golden["in/ties_d1"]
    # both are within half a step of the input; they differ only at .5 ties
    assert np.all(np.abs(dq_t - x) <= 0.5) and np.all(np.abs(dq_g - x) <= 0.5)
    assert np.all((dq_t == dq_g) | (np.abs(np.abs(x - np.trunc(x)) - 0.5) < 1e-6))


def test_q4_block_dequant():
    """tests.rs:191-226."""
    original = ((np.arange(32, dtype=np.float32) - np.float32(15.5)) / np.float32(15.5)).astype(np.float32)
    q = oracle.quantize_test(original)
    assert q.size == 18
    d = q[:2].copy().view(np.float16).astype(np.float32)[0]
    assert abs(d - np.max(np.abs(original)) / np.float32(7.0)) < 0.01
    deq = oracle.dequantize_c(q, 32)
    assert np.max(np.abs(deq - original)) < 0.08


def test_q4_block_edge_cases():
    """tests.rs:229-273."""
    z = oracle.dequantize_c(oracle.quantize_test(np.zeros(32, np.float32)), 32)
    assert np.all(z == 0.0)
    u = np.full(32, 0.5, np.float32)
    assert np.max(np.abs(oracle.dequantize_c(oracle.quantize_test(u), 32) - u)) < 0.08
    large = ((np.arange(32, dtype=np.float32) - np.float32(15.5)) * np.float32(100.0)).astype(np.float32)
    dl = np.max(np.abs(large)) / np.float32(7.0)
    assert np.max(np.abs(oracle.dequantize_c(oracle.quantize_test(large), 32) - large)) < dl / 2 + 1.0


def test_dequant_c_equals_numpy(golden):
    for name in _cases(golden):
        q = golden[f"q4/{name}"]
        n = q.size // 18 * 32
        a = oracle.dequantize_c(q, n)
        b = oracle.dequantize_np(q, n)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), name


def test_roundtrip_quant_error():
    """tests.rs:695-705 quantization error bound on the roundtrip input."""
    x = oracle.closed_form(5, 32 * 64)
    deq = oracle.dequantize_c(oracle.quantize_test(x), x.size)
    assert np.max(np.abs(deq - x)) < 0.1


def test_closed_form_inputs_are_rust_f32():
    """The generators reproduce Rust's f32 evaluation (no fma, f32 sin/cos)."""
    x = oracle.closed_form(3, 5)
    assert np.array_equal(x, np.arange(5, dtype=np.float32) * np.float32(0.1))
    a = oracle.closed_form(0, 1000)
    ref = (np.sin(np.arange(1000, dtype=np.float64) * np.float64(np.float32(0.001)) ) * 0.1)
    assert np.max(np.abs(a - ref)) < 1e-7


def test_reference_matmul_vs_f64():
    rng = np.random.default_rng(3)
    m, k, n = 7, 96, 33
    a = rng.standard_normal(m * k).astype(np.float32)
    b = rng.standard_normal(n * k).astype(np.float32)
    got = oracle.reference_matmul(a, b, m, k, n)
    want = a.reshape(m, k).astype(np.float64) @ b.reshape(n, k).astype(np.float64).T
    mag = np.abs(a.reshape(m, k)).astype(np.float64) @ np.abs(b.reshape(n, k)).astype(np.float64).T
    assert np.all(np.abs(got - want) <= k * 2**-24 * mag + 1e-30)


def test_shader_order_matmul_vs_dequant_matmul():
    """shader.wgsl order (interleaved lo/hi per block) vs the tests.rs
    reference_matmul on dequantized weights: same value up to f32 rounding."""
    w = oracle.closed_form(1, 64 * 128)
    q = oracle.quantize_test(w)
    deq = oracle.dequantize_c(q, w.size)
    x = oracle.closed_form(0, 4 * 10 * 128)
    a = oracle.shader_matmul(q, x, 4, 10, 128, 64).reshape(40, 64)
    b = oracle.reference_matmul(x, deq, 40, 128, 64)
    _, mag = oracle.matmul_f64(x.reshape(40, 128), deq.reshape(64, 128))
    assert np.all(np.abs(a - b) <= 2 * 128 * 2**-24 * mag + 1e-30)
    assert np.max(np.abs(a - b)) < 1e-3  # the reference's own test_q4_matmul_batch tolerance


def test_linear_bias_and_ffn_oracle():
    """linear.rs:34-40 and layers.rs:35-58 restatements agree with numpy."""
    d, f = 64, 256
    w1 = oracle.closed_form(7, f * d)
    w2 = oracle.closed_form(7, d * f)
    q1, q2 = oracle.quantize_test(w1), oracle.quantize_test(w2)
    b1 = oracle.closed_form(8, f)
    b2 = oracle.closed_form(8, d)
    x = oracle.closed_form(0, 4 * d)
    y = oracle.ffn(q1, b1, q2, b2, x, 1, 4, d, f)
    h = x.reshape(4, d).astype(np.float64) @ oracle.dequantize_np(q1, f * d).reshape(f, d).T.astype(np.float64) + b1
    h = oracle.gelu_np(h.astype(np.float32)).astype(np.float64)
    want = h @ oracle.dequantize_np(q2, d * f).reshape(d, f).T.astype(np.float64) + b2
    assert np.max(np.abs(y.reshape(4, d) - want)) < 1e-5


def test_gelu_c_vs_numpy():
    x = np.linspace(-8, 8, 4001).astype(np.float32)
    assert np.max(np.abs(oracle.gelu_c(x) - oracle.gelu_np(x))) < 2e-6


def test_synth_generator_is_deterministic():
    a = oracle.synth_uniform(7, "encoder.blocks.0.attn.query.weight", 1000, -0.05, 0.05)
    b = oracle.synth_uniform(7, "encoder.blocks.0.attn.query.weight", 1000, -0.05, 0.05)
    c = oracle.synth_uniform(8, "encoder.blocks.0.attn.query.weight", 1000, -0.05, 0.05)
    assert np.array_equal(a, b) and not np.array_equal(a, c)
    assert a.min() >= -0.05 and a.max() < 0.05


@pytest.mark.parametrize("name", ["encoder.blocks.0.attn.query.weight", "x"])
def test_fnv(name):
    assert 0 <= oracle.fnv1a64(name) < 2**64
