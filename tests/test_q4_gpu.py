"""GPU parity tests of the fused Q4_0 dequant+GEMM (run on an MI355X).

Each of the reference's 9 GPU tests (src/gguf/tests.rs) is re-expressed with
its own inputs and tolerance, calling the HIP kernels through the C ABI, and
then tightened: every result is also compared with a float64 evaluation of
the same dequantized product, against the error bound of the f16-hi/lo
scheme (DESIGN.md "Numerics"):

    |y_gpu - y_f64| <= TOL_REL * sum_k |x_k w_k| + TOL_ABS * sum_k |w_k|

TOL_REL = 4e-6, TOL_ABS = 2^-24 for WQ4_PREC_F16X2 (x split into two f16
terms, ~22 significant bits; f32 MFMA accumulation), and TOL_REL = 6e-4 for
WQ4_PREC_F16.  For scale: the reference's own f32 loop (tests.rs:172-184) is
bounded only by K * 2^-24 * sum|x w| (6e-5 at K = 1280).
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle
import wq4

pytestmark = pytest.mark.gpu

TOL = {wq4.PREC_F16X2: (4e-6, 2.0**-24), wq4.PREC_F16: (6e-4, 2.0**-12)}


@pytest.fixture(scope="module")
def torch():
    import torch as _t

    assert _t.cuda.is_available(), "GPU tests need an MI355X"
    assert wq4.device_count() >= 1
    return _t


@pytest.fixture(autouse=True)
def _reset_modes():
    wq4.set_precision(wq4.PREC_F16X2)
    wq4.set_kernel_policy(0)
    yield
    wq4.set_precision(wq4.PREC_F16X2)
    wq4.set_kernel_policy(0)


def to_dev(torch, a, shape):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32).reshape(shape)).to("cuda:0")


def assert_q4_close(y, x2d, deq2d, prec=wq4.PREC_F16X2, bias=None, what=""):
    truth, mag = oracle.matmul_f64(x2d, deq2d)
    if bias is not None:
        truth = truth + np.asarray(bias, np.float64)[None, :]
    wabs = np.abs(np.asarray(deq2d, np.float64)).sum(axis=1)[None, :]
    rel, ab = TOL[prec]
    bound = rel * mag + ab * wabs + 1e-30 + (0 if bias is None else 2**-24 * np.abs(truth))
    err = np.abs(np.asarray(y, np.float64).reshape(truth.shape) - truth)
    worst = float(np.max(err / bound))
    assert worst <= 1.0, f"{what}: max err/bound = {worst:.3g} (max err {err.max():.3g})"
    return worst


def make_weights(n, k, kind=1):
    w = oracle.closed_form(kind, n * k)
    q = oracle.quantize_test(w)
    return q, oracle.dequantize_np(q, n * k).reshape(n, k)


# ------------------------------------------------------- reference tests --
def test_q4_dequantize_gpu(torch):
    """tests.rs:331-363 (< 1e-5; here bit-exact)."""
    x = oracle.closed_form(4, 256)
    q = oracle.quantize_test(x)
    t = wq4.Q4Tensor.from_q4_bytes(q, [16, 16])
    deq = t.dequantize()
    assert list(deq.shape) == [16, 16]
    want = oracle.dequantize_c(q, 256).reshape(16, 16)
    assert np.array_equal(deq.cpu().numpy(), want)


def test_q4_matmul_small(torch):
    """tests.rs:370-410: 32x32, act i*0.1, vs reference_matmul, < 1e-3."""
    k = n = 32
    q, deq = make_weights(n, k, kind=2)
    act = oracle.closed_form(3, k)
    expected = oracle.reference_matmul(act, deq.ravel(), 1, k, n)
    t = wq4.Q4Tensor.from_q4_bytes(q, [n, k])
    out = wq4.q4_matmul(to_dev(torch, act, (1, 1, k)), t)
    assert list(out.shape) == [1, 1, n]
    y = out.cpu().numpy().reshape(1, n)
    assert np.max(np.abs(y - expected)) < 1e-3
    assert_q4_close(y, act.reshape(1, k), deq, what="small")


SHAPES = [(1, 1, 128, 64), (1, 1, 1280, 1280), (1, 10, 1280, 1280), (1, 1, 1280, 5120), (1, 1, 5120, 1280)]


@pytest.mark.parametrize("batch,seq,k,n", SHAPES)
@pytest.mark.parametrize("policy", [0, 1, 2, 3])
def test_q4_matmul_shapes(torch, batch, seq, k, n, policy):
    """tests.rs:413-480 (tol 1e-2 vs f32 matmul), both kernels."""
    wq4.set_kernel_policy(policy)
    act = oracle.closed_form(0, batch * seq * k)
    q, deq = make_weights(n, k, kind=1)
    expected = oracle.reference_matmul(act, deq.ravel(), batch * seq, k, n)
    t = wq4.Q4Tensor.from_q4_bytes(q, [n, k])
    out = wq4.q4_matmul(to_dev(torch, act, (batch, seq, k)), t)
    assert list(out.shape) == [batch, seq, n]
    y = out.cpu().numpy().reshape(batch * seq, n)
    assert np.max(np.abs(y - expected)) < 1e-2
    assert_q4_close(y, act.reshape(-1, k), deq, what=f"{(batch, seq, k, n)} policy {policy}")


def test_q4_linear_forward_shape(torch):
    """tests.rs:487-506."""
    q, _ = make_weights(64, 128, kind=0)
    lin = wq4.Q4Linear(wq4.Q4Tensor.from_q4_bytes(q, [64, 128]), None)
    out = lin.forward(torch.zeros((2, 5, 128), dtype=torch.float32, device="cuda:0"))
    assert list(out.shape) == [2, 5, 64]
    assert torch.count_nonzero(out).item() == 0


def test_q4_linear_forward_with_bias(torch):
    """tests.rs:509-564 (< 1e-3 vs reference matmul + bias)."""
    q, deq = make_weights(32, 64, kind=0)
    bias = oracle.closed_form(8, 32)
    lin = wq4.Q4Linear(wq4.Q4Tensor.from_q4_bytes(q, [32, 64]), to_dev(torch, bias, (32,)))
    act = oracle.closed_form(3, 64)
    out = lin.forward(to_dev(torch, act, (1, 1, 64)))
    assert list(out.shape) == [1, 1, 32]
    expected = oracle.reference_matmul(act, deq.ravel(), 1, 64, 32) + bias
    y = out.cpu().numpy().reshape(1, 32)
    assert np.max(np.abs(y - expected)) < 1e-3
    assert_q4_close(y, act.reshape(1, 64), deq, bias=bias, what="bias")


def test_q4_ffn_forward_shape(torch):
    """tests.rs:571-597 (shape only, zero input) -- plus zero output."""
    d, f = 64, 256
    q1, _ = make_weights(f, d, kind=7)
    q2, _ = make_weights(d, f, kind=7)
    ffn = wq4.Q4FFN(wq4.Q4Linear(wq4.Q4Tensor.from_q4_bytes(q1, [f, d])),
                    wq4.Q4Linear(wq4.Q4Tensor.from_q4_bytes(q2, [d, f])))
    out = ffn.forward(torch.zeros((1, 4, d), dtype=torch.float32, device="cuda:0"))
    assert list(out.shape) == [1, 4, d]
    assert torch.count_nonzero(out).item() == 0  # gelu(0) = 0, no bias


def test_q4_matmul_batch(torch):
    """tests.rs:604-655: (4, 10, 128, 64), < 1e-3."""
    b, s, k, n = 4, 10, 128, 64
    act = oracle.closed_form(0, b * s * k)
    q, deq = make_weights(n, k, kind=1)
    out = wq4.q4_matmul(to_dev(torch, act, (b, s, k)), wq4.Q4Tensor.from_q4_bytes(q, [n, k]))
    y = out.cpu().numpy().reshape(b * s, n)
    expected = oracle.shader_matmul(q, act, b, s, k, n).reshape(b * s, n)
    assert np.max(np.abs(y - expected)) < 1e-3
    assert_q4_close(y, act.reshape(-1, k), deq, what="batch")


def test_q4_roundtrip_small(torch):
    """tests.rs:662-706: device dequant == CPU dequant; raw bytes survive."""
    x = oracle.closed_form(5, 32 * 64)
    q = oracle.quantize_test(x)
    t = wq4.Q4Tensor.from_q4_bytes(q, [32, 64])
    gpu = t.dequantize().cpu().numpy().ravel()
    assert np.array_equal(gpu, oracle.dequantize_c(q, x.size))
    assert np.max(np.abs(gpu - x)) < 0.1
    assert np.array_equal(t.raw_bytes(), q)
    assert t.num_blocks() == 64 and t.shape() == [32, 64]


def test_q4_matmul_encoder_shape(torch):
    """tests.rs:713-764: (1, 32, 1280, 1280), < 1e-2."""
    act = oracle.closed_form(0, 32 * 1280)
    q, deq = make_weights(1280, 1280, kind=1)
    out = wq4.q4_matmul(to_dev(torch, act, (1, 32, 1280)), wq4.Q4Tensor.from_q4_bytes(q, [1280, 1280]))
    y = out.cpu().numpy().reshape(32, 1280)
    assert np.max(np.abs(y - oracle.reference_matmul(act, deq.ravel(), 32, 1280, 1280))) < 1e-2
    assert_q4_close(y, act.reshape(32, 1280), deq, what="encoder32")


# --------------------------------------------- beyond the reference tests --
WHISPER = [  # (N, K): Large-V3 and Medium projections and FFN
    (1280, 1280), (5120, 1280), (1280, 5120), (1024, 1024), (4096, 1024), (1024, 4096)]


@pytest.mark.parametrize("n,k", WHISPER)
@pytest.mark.parametrize("m", [1, 4, 32, 1500])
def test_whisper_shapes_reference_quantizer(torch, n, k, m):
    """Real Whisper shapes (full M = 1500 encoder rows), weights quantized by
    the product quantizer (convert_whisper.py), random activations."""
    rng = np.random.default_rng(n + 3 * k + m)
    w = (rng.standard_normal(n * k) * 0.02).astype(np.float32)
    q = oracle.quantize_convert_np(w)
    deq = oracle.dequantize_np(q, n * k).reshape(n, k)
    x = rng.standard_normal(m * k).astype(np.float32)
    t = wq4.Q4Tensor.from_q4_bytes(q, [n, k])
    y = wq4.q4_matmul(to_dev(torch, x, (1, m, k)), t).cpu().numpy().reshape(m, n)
    assert_q4_close(y, x.reshape(m, k), deq, what=f"{(m, n, k)}")


@pytest.mark.parametrize("policy", [1, 2, 3])
def test_batch_invariance(torch, policy):
    """Rows of a batch-of-clips call equal the single-clip call bit for bit
    (the per-row K-reduction order never depends on M or on the tile)."""
    wq4.set_kernel_policy(policy)
    n, k = 1280, 1280
    rng = np.random.default_rng(11)
    q = oracle.quantize_convert_np((rng.standard_normal(n * k) * 0.02).astype(np.float32))
    t = wq4.Q4Tensor.from_q4_bytes(q, [n, k])
    m1 = 1500 if policy == 1 else 1
    nb = 3 if policy == 1 else 32
    x = rng.standard_normal(nb * m1 * k).astype(np.float32)
    xb = to_dev(torch, x, (nb, m1, k))
    yb = wq4.q4_matmul(xb, t).cpu().numpy()
    for i in (0, nb - 1):
        yi = wq4.q4_matmul(xb[i:i + 1].contiguous(), t).cpu().numpy()
        assert np.array_equal(yb[i:i + 1].view(np.uint32), yi.view(np.uint32))


def test_prefill_and_decode_kernels_agree(torch):
    n, k, m = 5120, 1280, 48
    rng = np.random.default_rng(5)
    q = oracle.quantize_convert_np((rng.standard_normal(n * k) * 0.02).astype(np.float32))
    t = wq4.Q4Tensor.from_q4_bytes(q, [n, k])
    x = to_dev(torch, rng.standard_normal(m * k).astype(np.float32), (1, m, k))
    wq4.set_kernel_policy(1)
    a = wq4.q4_matmul(x, t).cpu().numpy()
    wq4.set_kernel_policy(2)
    b = wq4.q4_matmul(x, t).cpu().numpy()
    deq = oracle.dequantize_np(q, n * k).reshape(n, k)
    assert_q4_close(a.reshape(m, n), x.cpu().numpy().reshape(m, k), deq, what="prefill")
    assert_q4_close(b.reshape(m, n), x.cpu().numpy().reshape(m, k), deq, what="decode")


@pytest.mark.parametrize("policy", [1, 2, 3])
def test_precision_f16_mode(torch, policy):
    wq4.set_kernel_policy(policy)
    wq4.set_precision(wq4.PREC_F16)
    n, k, m = 1280, 1280, 32 if policy == 3 else 64
    rng = np.random.default_rng(6)
    q = oracle.quantize_convert_np((rng.standard_normal(n * k) * 0.02).astype(np.float32))
    deq = oracle.dequantize_np(q, n * k).reshape(n, k)
    x = rng.standard_normal(m * k).astype(np.float32)
    y = wq4.q4_matmul(to_dev(torch, x, (1, m, k)), wq4.Q4Tensor.from_q4_bytes(q, [n, k])).cpu().numpy()
    assert_q4_close(y.reshape(m, n), x.reshape(m, k), deq, prec=wq4.PREC_F16, what="f16")


@pytest.mark.parametrize("n,k", [(32, 32), (96, 64), (64, 96), (33 * 32, 160), (100, 320)])
@pytest.mark.parametrize("m", [1, 5, 65, 130])
def test_ragged_shapes(torch, n, k, m):
    """Odd block counts, N not a multiple of 64, M not a multiple of 32/64."""
    rng = np.random.default_rng(n * k + m)
    q = oracle.quantize_convert_np(rng.uniform(-1, 1, n * k).astype(np.float32))
    deq = oracle.dequantize_np(q, n * k).reshape(n, k)
    x = rng.standard_normal(m * k).astype(np.float32)
    for policy in (1, 2):
        wq4.set_kernel_policy(policy)
        y = wq4.q4_matmul(to_dev(torch, x, (1, m, k)), wq4.Q4Tensor.from_q4_bytes(q, [n, k])).cpu().numpy()
        assert_q4_close(y.reshape(m, n), x.reshape(m, k), deq, what=f"ragged {(m, n, k)} p{policy}")


def test_activation_range_edges(torch):
    """f16 subnormal lo terms (tiny x) and large |x| (up to ~4e4)."""
    n, k, m = 256, 512, 8
    rng = np.random.default_rng(9)
    q = oracle.quantize_convert_np(rng.uniform(-1, 1, n * k).astype(np.float32))
    deq = oracle.dequantize_np(q, n * k).reshape(n, k)
    for scale in (1e-6, 1e-3, 1e4):  # f16 hi term: |x| < 65504
        x = (rng.standard_normal(m * k) * scale).astype(np.float32)
        x[::97] = 0.0
        y = wq4.q4_matmul(to_dev(torch, x, (1, m, k)), wq4.Q4Tensor.from_q4_bytes(q, [n, k])).cpu().numpy()
        assert_q4_close(y.reshape(m, n), x.reshape(m, k), deq, what=f"scale {scale}")


def test_partial_block_rows_dequantize_but_refuse_matmul(torch):
    """[16, 16]: accepted like the reference (only N*K % 32 is checked,
    tensor.rs:38-42); the GEMM needs whole blocks per row (shader.wgsl:69)."""
    x = oracle.closed_form(4, 256)
    q = oracle.quantize_test(x)
    t = wq4.Q4Tensor.from_q4_bytes(q, [16, 16])
    assert np.array_equal(t.raw_bytes(), q)
    with pytest.raises(wq4.WQ4Error, match="K % 32"):
        wq4.q4_matmul(torch.zeros((1, 1, 16), dtype=torch.float32, device="cuda:0"), t)


def test_zero_rows_is_noop(torch):
    q, _ = make_weights(64, 128)
    t = wq4.Q4Tensor.from_q4_bytes(q, [64, 128])
    out = wq4.q4_matmul(torch.zeros((0, 3, 128), dtype=torch.float32, device="cuda:0"), t)
    assert list(out.shape) == [0, 3, 64]


def test_k_mismatch_raises(torch):
    """op.rs:58-61 panics; the C ABI returns WQ4_ESHAPE with the same text."""
    q, _ = make_weights(64, 128)
    t = wq4.Q4Tensor.from_q4_bytes(q, [64, 128])
    with pytest.raises(wq4.WQ4Error, match="K dimension mismatch: input has 96, weights have 128"):
        wq4.q4_matmul(torch.zeros((1, 1, 96), dtype=torch.float32, device="cuda:0"), t)


@pytest.mark.parametrize("policy", [1, 2, 3])
def test_ffn_numerics_vs_oracle(torch, policy):
    """Q4FFN numerics -- unpinned in the reference (shape-only test); here vs
    the oracle's layers.rs:35-58 restatement in float64 with f32 GELU."""
    wq4.set_kernel_policy(policy)
    d, f, m = 1280, 5120, 32 if policy == 3 else 40
    rng = np.random.default_rng(12)
    q1 = oracle.quantize_convert_np((rng.standard_normal(f * d) * 0.02).astype(np.float32))
    q2 = oracle.quantize_convert_np((rng.standard_normal(d * f) * 0.02).astype(np.float32))
    b1 = (rng.standard_normal(f) * 0.01).astype(np.float32)
    b2 = (rng.standard_normal(d) * 0.01).astype(np.float32)
    x = rng.standard_normal(m * d).astype(np.float32)
    ffn = wq4.Q4FFN(wq4.Q4Linear(wq4.Q4Tensor.from_q4_bytes(q1, [f, d]), to_dev(torch, b1, (f,))),
                    wq4.Q4Linear(wq4.Q4Tensor.from_q4_bytes(q2, [d, f]), to_dev(torch, b2, (d,))))
    y = ffn.forward(to_dev(torch, x, (1, m, d))).cpu().numpy().reshape(m, d)
    w1 = oracle.dequantize_np(q1, f * d).reshape(f, d).astype(np.float64)
    w2 = oracle.dequantize_np(q2, d * f).reshape(d, f).astype(np.float64)
    h = x.reshape(m, d).astype(np.float64) @ w1.T + b1
    g = oracle.gelu_np(h.astype(np.float32)).astype(np.float64)
    want = g @ w2.T + b2
    mag = np.abs(g) @ np.abs(w2).T + 1.0
    err = np.abs(y - want)
    assert np.max(err / mag) < 2e-5, np.max(err / mag)


def test_linear_ws_residual_and_gelu(torch):
    """The fused epilogue flags of wq4_linear_forward_ws: y = res + gelu(xW^T+b)."""
    import ctypes

    n, k, m = 1280, 1280, 100
    rng = np.random.default_rng(13)
    q = oracle.quantize_convert_np((rng.standard_normal(n * k) * 0.02).astype(np.float32))
    deq = oracle.dequantize_np(q, n * k).reshape(n, k)
    t = wq4.Q4Tensor.from_q4_bytes(q, [n, k])
    x = to_dev(torch, rng.standard_normal(m * k).astype(np.float32), (m, k))
    b = to_dev(torch, (rng.standard_normal(n) * 0.1).astype(np.float32), (n,))
    res = to_dev(torch, rng.standard_normal(m * n).astype(np.float32), (m, n))
    y = res.clone()
    nbytes = wq4.lib().wq4_linear_workspace_bytes(t.handle, m)
    ws = torch.empty(nbytes, dtype=torch.uint8, device="cuda:0")
    wq4.check(wq4.lib().wq4_linear_forward_ws(t.handle, ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(x.data_ptr()),
                                              ctypes.c_void_p(y.data_ptr()), ctypes.c_void_p(y.data_ptr()), m, k,
                                              wq4.EPI_GELU | wq4.EPI_RESIDUAL, wq4.PREC_F16X2,
                                              ctypes.c_void_p(ws.data_ptr()), nbytes,
                                              ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    h = x.cpu().numpy().astype(np.float64) @ deq.T.astype(np.float64) + b.cpu().numpy()
    want = res.cpu().numpy() + oracle.gelu_np(h.astype(np.float32))
    assert np.max(np.abs(y.cpu().numpy() - want)) < 1e-4


def _identity_q4(n):
    """Q4_0 bytes of the n x n identity: d = 1, nibble 9 (q = 1) on the diagonal."""
    nb = n // 32
    raw = bytearray()
    for r in range(n):
        for b in range(nb):
            q = [8] * 32
            if r // 32 == b:
                q[r % 32] = 9
            raw += np.float16(1.0).tobytes() + bytes((q[i] | (q[i + 16] << 4)) for i in range(16))
    return np.frombuffer(bytes(raw), np.uint8)


@pytest.mark.parametrize("m", [16, 3000])
def test_gelu_epilogue_vs_float64(torch, m):
    """The GEMM epilogue's GELU (evaluated as x / (1 + 2^t), wq4_device.hpp)
    against float64 0.5 x (1 + tanh(sqrt(2/pi) (x + 0.044715 x^3)))
    (layers.rs:35-41) through an exact identity weight: relative error a few
    f32 ulps over x in [-12, 12], including the negative tail where the f32
    tanh form cancels (decode-size and encoder-size row counts)."""
    import ctypes

    n = 64
    t = wq4.Q4Tensor.from_q4_bytes(_identity_q4(n), [n, n])
    rng = np.random.default_rng(5)
    x = np.concatenate([np.linspace(-12.0, 12.0, m * n // 2), rng.standard_normal(m * n - m * n // 2) * 3.0])
    x = x.astype(np.float32)
    xd = to_dev(torch, x, (m, n))
    b = torch.zeros(n, device="cuda:0")
    y = torch.zeros((m, n), device="cuda:0")
    nbytes = wq4.lib().wq4_linear_workspace_bytes(t.handle, m)
    ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device="cuda:0")
    vp = ctypes.c_void_p
    wq4.check(wq4.lib().wq4_linear_forward_ws(t.handle, vp(b.data_ptr()), vp(xd.data_ptr()), None,
                                              vp(y.data_ptr()), m, n, wq4.EPI_GELU, wq4.PREC_F16X2,
                                              vp(ws.data_ptr()), nbytes,
                                              vp(torch.cuda.current_stream().cuda_stream)))
    x64 = x.astype(np.float64)
    u = 0.7978845608028654 * (x64 + 0.044715 * x64**3)
    # 0.5 x (1 + tanh u) == x / (1 + e^(-2u)); the latter has no cancellation
    # in float64 either where tanh u -> -1
    want = x64 / (1.0 + np.exp(-2.0 * u))
    tanh_form = 0.5 * x64 * (1.0 + np.tanh(u))
    ok = np.abs(want) > 1e-6
    assert np.allclose(want[ok], tanh_form[ok], rtol=1e-9, atol=0)
    got = y.cpu().numpy().reshape(-1).astype(np.float64)
    # the operand representation of include/wq4.h ("Result precision"): x to
    # 2^-22 relative (GELU's slope is <= 1.13) where |x s| >= 2^-3, 2^-11
    # relative (the lo half an f16 subnormal, flushed by the MFMA) where
    # 2^-14 <= |x s| < 2^-3, with s the per-call operand scale of this ABI
    # entry point (2^4 here: max |x| = 12) -- times GELU's slope ~1/2 near 0
    s = 2.0 ** min(4, int(np.floor(np.log2(16384.0 / float(np.max(np.abs(x)))))))
    err = np.abs(got - want)
    ax = np.abs(x64)
    bound = 2e-6 * ax + 1e-6 * np.abs(want) + np.where(ax * s < 2.0**-3, 2.0**-12 * ax, 0.0) + 1e-37
    worst = int(np.argmax(err / bound))
    assert np.all(err <= bound), (float(err[worst] / bound[worst]), float(x64[worst]), float(got[worst]),
                                  float(want[worst]))


@pytest.mark.parametrize("policy", [1, 2])
def test_gemm_headmajor_layout(torch, policy):
    """wq4_gemm_tiled_headmajor == row-major GEMM permuted to [part][g][head][t][64]."""
    import ctypes

    d, k, groups, trows = 128, 256, 2, 24  # parts = 2 (K | V), heads of 64
    n, m = 2 * d, groups * trows
    rng = np.random.default_rng(21)
    q = oracle.quantize_convert_np((rng.standard_normal(n * k) * 0.05).astype(np.float32))
    t = wq4.Q4Tensor.from_q4_bytes(q, [n, k])
    x = to_dev(torch, rng.standard_normal(m * k).astype(np.float32), (m, k))
    b = to_dev(torch, (rng.standard_normal(n) * 0.1).astype(np.float32), (n,))
    L = wq4.lib()
    atb = L.wq4_atiled_bytes(m, k, wq4.PREC_F16X2)
    at = torch.zeros(atb, dtype=torch.uint8, device="cuda:0")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    wq4.check(L.wq4_tile_activations(ctypes.c_void_p(x.data_ptr()), m, k, k, wq4.PREC_F16X2,
                                     ctypes.c_void_p(at.data_ptr()), atb, st))
    ref = torch.empty((m, n), device="cuda:0", dtype=torch.float32)
    hm = torch.empty((m * n,), device="cuda:0", dtype=torch.float32)
    wq4.check(L.wq4_gemm_tiled(t.handle, ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(at.data_ptr()), None,
                               ctypes.c_void_p(ref.data_ptr()), None, m, 0, wq4.PREC_F16X2, policy, st))
    wq4.check(L.wq4_gemm_tiled_headmajor(t.handle, ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(at.data_ptr()),
                                         ctypes.c_void_p(hm.data_ptr()), m, trows, d, wq4.PREC_F16X2, policy, st))
    want = ref.cpu().numpy().reshape(groups, trows, 2, d // 64, 64).transpose(2, 0, 3, 1, 4).ravel()
    assert np.array_equal(hm.cpu().numpy(), want)
    with pytest.raises(wq4.WQ4Error):
        wq4.check(L.wq4_gemm_tiled_headmajor(t.handle, None, ctypes.c_void_p(at.data_ptr()),
                                             ctypes.c_void_p(hm.data_ptr()), m, 25, d, wq4.PREC_F16X2, policy, st))


@pytest.mark.parametrize("clips,mode", [(1, 1), (2, 1), (2, 5), (9, 5)])
def test_gemm_headmajor_ring_kernel(torch, clips, mode):
    """The few-clip cross K / V cache GEMMs (wa_model.cpp cross_kv_forward:
    M = clips x 1500 rows, head-major output) run on the encoder ring kernel
    (wq4_enc.hip; mode 5: the wide kernel, wq4_wide.hip); their bits equal
    the prefill tile kernel's row-major result permuted to [g][head][t][64]."""
    import ctypes

    d = k = 1280
    trows, m = 1500, 1500 * clips
    rng = np.random.default_rng(1500 + clips)
    q = oracle.quantize_convert_np((rng.standard_normal(d * k) * 0.05).astype(np.float32))
    t = wq4.Q4Tensor.from_q4_bytes(q, [d, k], decode_step=False)
    x = to_dev(torch, rng.standard_normal(m * k).astype(np.float32), (m, k))
    b = to_dev(torch, (rng.standard_normal(d) * 0.1).astype(np.float32), (d,))
    L = wq4.lib()
    atb = L.wq4_atiled_bytes(m, k, wq4.PREC_F16X2)
    at = torch.zeros(atb, dtype=torch.uint8, device="cuda:0")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    wq4.check(L.wq4_tile_activations(ctypes.c_void_p(x.data_ptr()), m, k, k, wq4.PREC_F16X2,
                                     ctypes.c_void_p(at.data_ptr()), atb, st))
    ref = torch.empty((m, d), device="cuda:0", dtype=torch.float32)
    hm = torch.empty((m * d,), device="cuda:0", dtype=torch.float32)
    prev = L.wq4_debug_set_enc_kernel(0)  # the tile kernel for the row-major reference
    try:
        wq4.check(L.wq4_gemm_tiled(t.handle, ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(at.data_ptr()), None,
                                   ctypes.c_void_p(ref.data_ptr()), None, m, 0, wq4.PREC_F16X2, 1, st))
        assert L.wq4_debug_set_enc_kernel(mode) >= 0  # 1: by rows (the ring kernel at these grids)
        wq4.check(L.wq4_gemm_tiled_headmajor(t.handle, ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(at.data_ptr()),
                                             ctypes.c_void_p(hm.data_ptr()), m, trows, d, wq4.PREC_F16X2, 0, st))
        torch.cuda.synchronize()
    finally:
        L.wq4_debug_set_enc_kernel(prev)
    want = ref.cpu().numpy().reshape(clips, trows, d // 64, 64).transpose(0, 2, 1, 3).ravel()
    assert np.array_equal(hm.cpu().numpy(), want)


@pytest.mark.parametrize("wtype", ["q4_0", "f16"])
@pytest.mark.parametrize("prec", [0, 1])
@pytest.mark.parametrize("m,n,flags", [(1, 3840, 0), (17, 1280, 0), (32, 5120, 5), (100, 1280, 2), (128, 96, 0)])
def test_gemm_ln_fused_bit_exact(torch, wtype, prec, m, n, flags):
    """wq4_gemm_ln_tiled (LayerNorm built inside the decode GEMM) equals
    wq4_layernorm -> wq4_gemm_tiled bit for bit (flags: 1 GELU, 2 residual,
    4 tiled output)."""
    import ctypes

    k = 1280 if n != 96 else 160
    rng = np.random.default_rng(m * 7 + n + prec)
    if wtype == "f16":
        t = wq4.Q4Tensor.from_f16((rng.standard_normal((n, k)) * 0.03).astype(np.float16))
    else:
        t = wq4.Q4Tensor.from_q4_bytes(oracle.quantize_convert_np((rng.standard_normal(n * k) * 0.05).astype(np.float32)), [n, k])
    x = to_dev(torch, (rng.standard_normal(m * k) * 2 + 0.5).astype(np.float32), (m, k))
    g = to_dev(torch, rng.uniform(0.8, 1.2, k).astype(np.float32), (k,))
    be = to_dev(torch, rng.uniform(-0.1, 0.1, k).astype(np.float32), (k,))
    b = to_dev(torch, (rng.standard_normal(n) * 0.1).astype(np.float32), (n,))
    res = to_dev(torch, rng.standard_normal(m * n).astype(np.float32), (m, n))
    L = wq4.lib()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    p = lambda a: ctypes.c_void_p(a.data_ptr()) if a is not None else None
    atb = L.wq4_atiled_bytes(m, k, prec)
    at_ref = torch.zeros(atb, dtype=torch.uint8, device="cuda:0")
    at_scr = torch.zeros(atb, dtype=torch.uint8, device="cuda:0")
    tiled = (flags & 4) != 0
    ob = L.wq4_atiled_bytes(m, n, prec)
    outs = []
    for fused in (False, True):
        y = torch.full((m, n), 7.0, device="cuda:0") if not tiled else None
        ot = torch.zeros(ob, dtype=torch.uint8, device="cuda:0") if tiled else None
        r = res if flags & 2 else None
        if fused:
            wq4.check(L.wq4_gemm_ln_tiled(t.handle, p(b), p(x), p(g), p(be), p(at_scr), p(r), p(y), p(ot), m,
                                          flags | 8, prec, 2, st))  # WQ4_EPI_LN_FUSED
        else:
            wq4.check(L.wq4_layernorm(p(x), p(g), p(be), m, k, prec, p(at_ref), None, st))
            wq4.check(L.wq4_gemm_tiled(t.handle, p(b), p(at_ref), p(r), p(y), p(ot), m, flags, prec, 2, st))
        outs.append((y if not tiled else ot).cpu().numpy())
    assert np.array_equal(outs[0].view(np.uint32) if not tiled else outs[0], outs[1].view(np.uint32) if not tiled else outs[1])


@pytest.mark.parametrize("prec", [0, 1])
@pytest.mark.parametrize("m,d", [(1, 1280), (31, 1280), (33, 384), (100, 160), (70, 96), (40, 2048), (3000, 1280),
                                 (2049, 96), (4100, 2048), (3001, 160)])
def test_layernorm_tiled_equals_f32_then_tile(torch, prec, m, d):
    """wq4_layernorm's A-tiled output (one wave per row up to 2048 rows, then
    layernorm_tiled_kernel: rows in registers, 1 KiB fragment stores) equals
    the f32 LayerNorm rows tiled by
    wq4_tile_activations bit for bit -- including the zero rows / columns that
    pad the m-tile (m % 32 != 0) and a padded odd block count (d = 96, 160)."""
    import ctypes

    rng = np.random.default_rng(m * 3 + d + prec)
    x = to_dev(torch, (rng.standard_normal(m * d) * 3 + 0.7).astype(np.float32), (m, d))
    g = to_dev(torch, rng.uniform(0.5, 1.5, d).astype(np.float32), (d,))
    be = to_dev(torch, rng.uniform(-0.2, 0.2, d).astype(np.float32), (d,))
    L = wq4.lib()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    p = lambda a: ctypes.c_void_p(a.data_ptr())  # noqa: E731
    atb = L.wq4_atiled_bytes(m, d, prec)
    got = torch.full((atb,), 0x5A, dtype=torch.uint8, device="cuda:0")  # poisoned: every byte must be written
    wq4.check(L.wq4_layernorm(p(x), p(g), p(be), m, d, prec, p(got), None, st))
    y = torch.zeros((m, d), device="cuda:0")
    wq4.check(L.wq4_layernorm(p(x), p(g), p(be), m, d, prec, None, p(y), st))
    want = torch.zeros((atb,), dtype=torch.uint8, device="cuda:0")
    wq4.check(L.wq4_tile_activations(p(y), m, d, d, prec, p(want), atb, st))
    torch.cuda.synchronize()
    ns = 2 if prec == 0 else 1
    kbp = ((d // 32 + 1) // 2) * 2
    nmt, kb = -(-m // 32), -(-d // 32)  # m-tiles and Q4 blocks the LayerNorm writes
    gb = got.cpu().numpy().reshape(-1, kbp, 2, ns, 1024)[:nmt, :kb]
    wb = want.cpu().numpy().reshape(-1, kbp, 2, ns, 1024)[:nmt, :kb]
    assert np.array_equal(gb, wb)


# ------------------------------------------- f16 weights (BASELINE config 5) --
@pytest.mark.parametrize("policy", [1, 2, 3])
@pytest.mark.parametrize("m,n,k", [(1, 1280, 1280), (32, 5120, 1280), (100, 1280, 5120), (1500, 1280, 1280),
                                   (5, 96, 160)])
def test_f16_weights_gemm(torch, policy, m, n, k):
    """The same kernels on f16 weight fragments: x = hi + lo against the exact
    f16 w, f32 accumulation -> the f16x2 tolerance of the Q4 path."""
    rng = np.random.default_rng(41 + m + n)
    w = (rng.standard_normal((n, k)) * 0.03).astype(np.float16)
    t = wq4.Q4Tensor.from_f16(w)
    assert t.weight_type == "f16"
    assert np.array_equal(t.raw_bytes().view(np.float16).reshape(n, k), w)
    assert np.array_equal(t.dequantize_host(), w.astype(np.float32))
    x = rng.standard_normal(m * k).astype(np.float32)
    wq4.set_kernel_policy(policy)
    y = wq4.q4_matmul(to_dev(torch, x, (1, m, k)), t).cpu().numpy().reshape(m, n)
    assert_q4_close(y, x.reshape(m, k), w.astype(np.float32), what="f16 weights")


@pytest.mark.parametrize("policy", [2, 3])
def test_f16_weights_batch_invariance(torch, policy):
    n, k = 1280, 1280
    rng = np.random.default_rng(43)
    t = wq4.Q4Tensor.from_f16((rng.standard_normal((n, k)) * 0.03).astype(np.float16))
    wq4.set_kernel_policy(policy)
    xb = to_dev(torch, rng.standard_normal(32 * k).astype(np.float32), (32, 1, k))
    yb = wq4.q4_matmul(xb, t).cpu().numpy()
    y1 = wq4.q4_matmul(xb[5:6].contiguous(), t).cpu().numpy()
    assert np.array_equal(yb[5:6].view(np.uint32), y1.view(np.uint32))


# ------------------------------ LayerNorm folded into the decoder GEMMs --
@pytest.mark.parametrize("wtype", ["q4_0", "f16"])
@pytest.mark.parametrize("prec", [0, 1])
@pytest.mark.parametrize("m", [1, 7, 16, 32])
@pytest.mark.parametrize("n2,flags", [(1280, 0), (5120, 1)])
@pytest.mark.parametrize("kern", [3, 2])
def test_ln_fold_matches_layernorm_path(torch, wtype, prec, m, n2, flags, kern):
    """wq4_gemm_tiled_lnfold: a residual GEMM x = r + W1 a + b1 that also
    emits tiled(x * gamma) and 16-column tile statistics (producer; rows <=
    32: the 8-wave decode kernel, kern 2 -- the model's choice -- or the
    decode-step kernel, kern 3), then a GEMM on
    LayerNorm(x) (consumer, decoder.rs:77-112 attn_ln -> query etc.),
    against wq4_gemm_tiled -> wq4_layernorm -> wq4_gemm_tiled.  The
    producer's x is bit-identical; the consumer re-associates
    W LN(x) = (W (x gamma) - mean W gamma) / den + W beta, so it is held to
    |z - z_ref| <= 2e-5 * (1 + max|z_ref|) (f32 reference arithmetic itself
    is ~1e-6 here)."""
    import ctypes

    d = 1280
    rng = np.random.default_rng(m * 13 + n2 + prec)

    def weights(n, k, s):
        if wtype == "f16":
            return wq4.Q4Tensor.from_f16((rng.standard_normal((n, k)) * s).astype(np.float16))
        return wq4.Q4Tensor.from_q4_bytes(oracle.quantize_convert_np((rng.standard_normal(n * k) * s).astype(np.float32)),
                                          [n, k])

    w1, w2 = weights(d, d, 0.05), weights(n2, d, 0.04)
    a = to_dev(torch, rng.standard_normal(m * d).astype(np.float32), (m, d))
    res = to_dev(torch, (rng.standard_normal(m * d) * 2 + 0.7).astype(np.float32), (m, d))
    b1 = to_dev(torch, (rng.standard_normal(d) * 0.1).astype(np.float32), (d,))
    b2 = rng.standard_normal(n2).astype(np.float32) * 0.1
    g = rng.uniform(0.8, 1.2, d).astype(np.float32)
    be = rng.uniform(-0.1, 0.1, d).astype(np.float32)
    L = wq4.lib()
    wq4.set_kernel_policy(kern)
    assert L.wq4_lnfold_supported(w1.handle, m) == 1 and L.wq4_lnfold_supported(w2.handle, m) == 1
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    fp = lambda v: v.ctypes.data_as(ctypes.POINTER(ctypes.c_float))  # noqa: E731
    at_a = torch.zeros(L.wq4_atiled_bytes(m, d, prec), dtype=torch.uint8, device="cuda:0")
    wq4.check(L.wq4_tile_activations(p(a), m, d, d, prec, p(at_a), at_a.numel(), st))
    tiled = (flags & 4) != 0
    gd, bed, b2d = (to_dev(torch, v, v.shape) for v in (g, be, b2))

    # reference: residual GEMM, LayerNorm kernel, GEMM
    x_ref = res.clone()
    wq4.check(L.wq4_gemm_tiled(w1.handle, p(b1), p(at_a), p(x_ref), p(x_ref), None, m, 2, prec, kern, st))
    at_ln = torch.zeros(L.wq4_atiled_bytes(m, d, prec), dtype=torch.uint8, device="cuda:0")
    wq4.check(L.wq4_layernorm(p(x_ref), p(gd), p(bed), m, d, prec, p(at_ln), None, st))
    ob = L.wq4_atiled_bytes(m, n2, prec)
    z_ref = torch.zeros((m, n2), device="cuda:0")
    zt_ref = torch.zeros(ob, dtype=torch.uint8, device="cuda:0")
    wq4.check(L.wq4_gemm_tiled(w2.handle, p(b2d), p(at_ln), None, None if tiled else p(z_ref), p(zt_ref) if tiled else None,
                               m, flags, prec, 2, st))

    # fold: producer then consumer
    wg = np.zeros(n2, np.float32)
    b2f = np.zeros(n2, np.float32)
    wq4.check(L.wq4_ln_fold_vectors(w2.handle, fp(g), fp(be), fp(b2), fp(wg), fp(b2f)))
    wgd, b2fd = to_dev(torch, wg, wg.shape), to_dev(torch, b2f, b2f.shape)
    x = res.clone()
    at_f = torch.zeros(L.wq4_atiled_bytes(m, d, prec), dtype=torch.uint8, device="cuda:0")
    stats = torch.zeros(m * (d // 16) * 2, device="cuda:0")
    prod = wq4.LnFold(gd.data_ptr(), at_f.data_ptr(), stats.data_ptr(), None, None)
    wq4.check(L.wq4_gemm_tiled_lnfold(w1.handle, p(b1), p(at_a), p(x), p(x), None, m, 2, prec, ctypes.byref(prod), st))
    cons = wq4.LnFold(None, None, None, stats.data_ptr(), wgd.data_ptr())
    z = torch.zeros((m, n2), device="cuda:0")
    zt = torch.zeros(ob, dtype=torch.uint8, device="cuda:0")
    wq4.check(L.wq4_gemm_tiled_lnfold(w2.handle, p(b2fd), p(at_f), None, None if tiled else p(z), p(zt) if tiled else None,
                                      m, flags, prec, ctypes.byref(cons), st))
    torch.cuda.synchronize()
    assert np.array_equal(x.cpu().numpy().view(np.uint32), x_ref.cpu().numpy().view(np.uint32))
    # both paths against float64 arithmetic on the same x, held to the Q4
    # GEMM tolerance of this file (per output: c * sum_k |W[n,k] LN(x)[k]|,
    # c = 8e-6 f16x2 / 1.2e-3 f16 -- twice test_q4_linear's, as the fold
    # rounds x * gamma instead of LN(x))
    xs = x_ref.cpu().numpy().astype(np.float64)
    mu = xs.mean(axis=1, keepdims=True)
    ln = (xs - mu) / np.sqrt(((xs - mu) ** 2).mean(axis=1, keepdims=True) + 1e-5) * g + be
    w2d = w2.dequantize_host().astype(np.float64)
    z64 = ln @ w2d.T + b2
    if flags & 1:
        z64 = 0.5 * z64 * (1.0 + np.tanh(0.7978845608028654 * (z64 + 0.044715 * z64 ** 3)))
    scale = np.abs(ln) @ np.abs(w2d).T
    c = 8e-6 if prec == 0 else 1.2e-3
    for zz in (z_ref, z):
        err = np.abs(zz.cpu().numpy() - z64)
        assert np.all(err <= c * scale + 1e-6), float(np.max(err / (scale + 1e-30)))


# ------------------------------------------- range and layout edge cases --
@pytest.mark.parametrize("policy", [1, 2, 3])
def test_ffn_large_range_vs_oracle(torch, policy):
    """Q4FFN with inputs around 1e3-1e4 and fc1 outputs far beyond the
    internal operands' 2^4-scaled f16 range (|gelu(fc1 x)| up to ~1e6): each
    GEMM's operand scale comes from its own input's max |x|, so the result
    stays finite and within the f16x2 tolerance of the float64 oracle (the
    reference's f32 path has no range limit below FLT_MAX)."""
    wq4.set_kernel_policy(policy)
    d, f, m = 256, 1024, 32 if policy == 3 else 40
    rng = np.random.default_rng(77)
    q1 = oracle.quantize_convert_np((rng.standard_normal(f * d) * 0.5).astype(np.float32))
    q2 = oracle.quantize_convert_np((rng.standard_normal(d * f) * 0.05).astype(np.float32))
    b1 = (rng.standard_normal(f) * 10).astype(np.float32)
    b2 = (rng.standard_normal(d) * 0.01).astype(np.float32)
    x = (rng.standard_normal(m * d) * 3e3).astype(np.float32)
    x[::7] *= 3.0  # some |x| ~ 1e4
    ffn = wq4.Q4FFN(wq4.Q4Linear(wq4.Q4Tensor.from_q4_bytes(q1, [f, d]), to_dev(torch, b1, (f,))),
                    wq4.Q4Linear(wq4.Q4Tensor.from_q4_bytes(q2, [d, f]), to_dev(torch, b2, (d,))))
    y = ffn.forward(to_dev(torch, x, (1, m, d))).cpu().numpy().reshape(m, d)
    assert np.all(np.isfinite(y))
    w1 = oracle.dequantize_np(q1, f * d).reshape(f, d).astype(np.float64)
    w2 = oracle.dequantize_np(q2, d * f).reshape(d, f).astype(np.float64)
    h = x.reshape(m, d).astype(np.float64) @ w1.T + b1
    assert np.max(np.abs(h)) > 4094.0 * 4, "the test must exceed the old fixed operand range"
    g = oracle.gelu_np(h.astype(np.float32)).astype(np.float64)
    want = g @ w2.T + b2
    mag = np.abs(g) @ np.abs(w2).T + 1.0
    assert np.max(np.abs(y - want) / mag) < 2e-5


@pytest.mark.parametrize("kern", [3, 2])
def test_ln_fold_producer_statistics_n1312(torch, kern):
    """LayerNorm-fold producer at N = 1312 (N % 64 == 32: the last 64-column
    slab of the decode-step kernel is half padding): the 16-column tile
    statistics land in exactly rows * N / 16 slots -- a poisoned guard region
    right after them stays untouched -- and equal (mean, M2) of each tile of
    the produced x."""
    import ctypes

    n, k, m = 1312, 1280, 13
    rng = np.random.default_rng(1312 + kern)
    w = wq4.Q4Tensor.from_q4_bytes(oracle.quantize_convert_np((rng.standard_normal(n * k) * 0.05).astype(np.float32)),
                                   [n, k])
    L = wq4.lib()
    wq4.set_kernel_policy(kern)
    if L.wq4_lnfold_supported(w.handle, m) != 1:
        pytest.skip("no LayerNorm-fold kernel for this shape under this policy")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    a = to_dev(torch, rng.standard_normal(m * k).astype(np.float32), (m, k))
    at_a = torch.zeros(L.wq4_atiled_bytes(m, k, 0), dtype=torch.uint8, device="cuda:0")
    wq4.check(L.wq4_tile_activations(p(a), m, k, k, 0, p(at_a), at_a.numel(), st))
    res = to_dev(torch, rng.standard_normal(m * n).astype(np.float32), (m, n))
    b = to_dev(torch, (rng.standard_normal(n) * 0.1).astype(np.float32), (n,))
    gam = to_dev(torch, rng.uniform(0.8, 1.2, n).astype(np.float32), (n,))
    x_ref = res.clone()
    wq4.check(L.wq4_gemm_tiled(w.handle, p(b), p(at_a), p(x_ref), p(x_ref), None, m, 2, 0, kern, st))
    nslots = m * (n // 16) * 2
    stats = torch.full((nslots + 4096,), 12345.0, device="cuda:0")
    at_f = torch.zeros(L.wq4_atiled_bytes(m, n, 0), dtype=torch.uint8, device="cuda:0")
    x = res.clone()
    prod = wq4.LnFold(gam.data_ptr(), at_f.data_ptr(), stats.data_ptr(), None, None)
    wq4.check(L.wq4_gemm_tiled_lnfold(w.handle, p(b), p(at_a), p(x), p(x), None, m, 2, 0, ctypes.byref(prod), st))
    torch.cuda.synchronize()
    xs = x.cpu().numpy()
    assert np.array_equal(xs.view(np.uint32), x_ref.cpu().numpy().view(np.uint32))
    s = stats.cpu().numpy()
    assert np.all(s[nslots:] == 12345.0), "statistics written past rows * N / 16 slots"
    got = s[:nslots].reshape(m, n // 16, 2)
    tiles = xs.astype(np.float64).reshape(m, n // 16, 16)
    mean = tiles.mean(axis=2)
    m2 = ((tiles - mean[..., None]) ** 2).sum(axis=2)
    assert np.allclose(got[..., 0], mean, rtol=1e-5, atol=1e-5)
    assert np.allclose(got[..., 1], m2, rtol=1e-4, atol=1e-4)


def test_tensor_without_decode_step_layout(torch):
    """WQ4_TENSOR_NO_DECODE_STEP (encoder weights): no second weight copy,
    and <= 32-row calls fall back to the other kernels within tolerance."""
    n, k, m = 1280, 1280, 8
    rng = np.random.default_rng(5)
    q = oracle.quantize_convert_np((rng.standard_normal(n * k) * 0.05).astype(np.float32))
    deq = oracle.dequantize_np(q, n * k).reshape(n, k)
    full = wq4.Q4Tensor.from_q4_bytes(q, [n, k])
    lean = wq4.Q4Tensor.from_q4_bytes(q, [n, k], decode_step=False)
    assert full.has_decode_step and not lean.has_decode_step
    assert lean.device_bytes() < full.device_bytes()
    assert np.array_equal(lean.raw_bytes(), q)
    x = rng.standard_normal(m * k).astype(np.float32)
    for policy in (0, 3):
        wq4.set_kernel_policy(policy)
        y = wq4.q4_matmul(to_dev(torch, x, (1, m, k)), lean).cpu().numpy().reshape(m, n)
        assert_q4_close(y, x.reshape(m, k), deq, what=f"no decode-step layout, policy {policy}")


def test_f16_weights_out_of_decode_step_range(torch):
    """f16 weights with |w| >= 256 (w * 2^8 would overflow the decode-step
    kernel's f16 layout): that layout is not built and small-row GEMMs use
    the other kernels, still within the f16x2 tolerance."""
    n, k, m = 256, 512, 4
    rng = np.random.default_rng(6)
    w = (rng.standard_normal((n, k)) * 0.03).astype(np.float16)
    w[3, 17] = np.float16(300.0)
    t = wq4.Q4Tensor.from_f16(w)
    assert not t.has_decode_step
    x = rng.standard_normal(m * k).astype(np.float32)
    for policy in (0, 3):
        wq4.set_kernel_policy(policy)
        y = wq4.q4_matmul(to_dev(torch, x, (1, m, k)), t).cpu().numpy().reshape(m, n)
        assert np.all(np.isfinite(y))
        assert_q4_close(y, x.reshape(m, k), w.astype(np.float32), what=f"f16 |w| >= 256, policy {policy}")


@pytest.mark.parametrize("flags", [0, 2])
def test_enc_epilogue_past_2gib(torch, flags):
    """An f32 output past 2 GiB (M = 110000 rows x N = 5120): the tile and
    wide kernels' epilogue leaves its offset-masked buffer stores for the
    pointer path (wq4_tile_epi.hpp), the ring kernel (its own epilogue) is the
    reference -- bit-identical, with and without the in-place residual."""
    import ctypes

    m, n, k = 110000, 5120, 64
    rng = np.random.default_rng(11 + flags)
    q = oracle.quantize_convert_np((rng.standard_normal(n * k) * 0.05).astype(np.float32))
    t = wq4.Q4Tensor.from_q4_bytes(q, [n, k])
    L = wq4.lib()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    p = lambda a: ctypes.c_void_p(a.data_ptr()) if a is not None else None  # noqa: E731
    g = torch.Generator(device="cuda:0").manual_seed(5)
    x = torch.randn(m, k, device="cuda:0", generator=g)
    at = torch.zeros(L.wq4_atiled_bytes(m, k, 0), dtype=torch.uint8, device="cuda:0")
    wq4.check(L.wq4_tile_activations(p(x), m, k, k, 0, p(at), at.numel(), st))
    b = torch.randn(n, device="cuda:0", generator=g) * 0.1
    res0 = torch.randn(m, n, device="cuda:0", generator=g) if flags & 2 else None
    ref = None
    prev = L.wq4_debug_set_enc_kernel(0)
    try:
        for mode in (3, 0, 5):
            assert L.wq4_debug_set_enc_kernel(mode) >= 0
            y = res0.clone() if flags & 2 else torch.full((m, n), 7.0, device="cuda:0")
            wq4.check(L.wq4_gemm_tiled(t.handle, p(b), p(at), p(y) if flags & 2 else None, p(y), None, m, flags, 0, 1,
                                       st))
            torch.cuda.synchronize()
            if ref is None:
                ref = y
            else:
                diff = int((y.view(torch.int32) != ref.view(torch.int32)).sum().item())
                assert diff == 0, f"mode {mode}: {diff} of {y.numel()} outputs differ"
                del y
    finally:
        L.wq4_debug_set_enc_kernel(prev)


# ------------------------------- encoder GEMM: LDS-DMA ring kernel (wq4_enc.hip) --
@pytest.mark.parametrize("m,n,k,flags,prec", [(1500, 1280, 1280, 0, 0), (3000, 3840, 1280, 0, 0), (700, 5120, 1280, 5, 0),
                                              (300, 1280, 5120, 2, 0), (2049, 1280, 1280, 1, 0), (16000, 1280, 1280, 2, 0),
                                              (4500, 5120, 1280, 5, 0), (200, 96, 160, 0, 0), (1000, 1312, 1280, 4, 0),
                                              (2049, 1280, 1280, 4, 0), (1500, 1280, 5120, 3, 0), (2000, 5120, 1280, 5, 1),
                                              (300, 1312, 160, 4, 1),
                                              # K loop lengths for the wide kernel's peeled first block pair,
                                              # three-pair trips and 0-3 trailing pairs (nbp = K / 64: 1, 4, 5, 6, 7)
                                              (600, 1280, 64, 1, 0), (500, 1280, 256, 0, 0), (900, 1280, 320, 2, 0),
                                              (400, 1280, 384, 0, 1), (700, 1280, 448, 4, 0)])
def test_enc_kernel_bit_identical(torch, m, n, k, flags, prec):
    """The encoder-size GEMM kernels -- the ring kernel (its geometries: 256 x
    256 with 8 waves, 64 x 128 and 32 x 256 with 4) and the 8-wave wide
    kernel (wq4_wide.hip, mode 5) -- give the prefill tile kernel's bits
    exactly: the same per-block MFMA chain and scale FMA order, only the
    memory pipeline differs.  flags: 1 GELU, 2 residual, 4 A-tiled output
    (then compared fragment for fragment, padding included).  prec 1 (f16
    operands): the ring kernel is f16x2-only, so the tile and wide kernels."""
    import ctypes

    rng = np.random.default_rng(m + n + k + flags)
    q = oracle.quantize_convert_np((rng.standard_normal(n * k) * 0.05).astype(np.float32))
    t = wq4.Q4Tensor.from_q4_bytes(q, [n, k])
    L = wq4.lib()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    p = lambda a: ctypes.c_void_p(a.data_ptr()) if a is not None else None  # noqa: E731
    x = to_dev(torch, rng.standard_normal(m * k).astype(np.float32), (m, k))
    at = torch.zeros(L.wq4_atiled_bytes(m, k, prec), dtype=torch.uint8, device="cuda:0")
    wq4.check(L.wq4_tile_activations(p(x), m, k, k, prec, p(at), at.numel(), st))
    b = to_dev(torch, (rng.standard_normal(n) * 0.1).astype(np.float32), (n,))
    res = to_dev(torch, rng.standard_normal(m * n).astype(np.float32), (m, n))
    tiled = (flags & 4) != 0
    modes = (0, 2, 3, 4, 5, 1) if prec == 0 else (0, 5, 1)
    outs = []
    prev = L.wq4_debug_set_enc_kernel(0)
    try:
        for mode in modes:
            assert L.wq4_debug_set_enc_kernel(mode) >= 0
            y = res.clone() if flags & 2 else torch.full((m, n), 7.0, device="cuda:0")
            ot = torch.full((L.wq4_atiled_bytes(m, n, prec),), 0x5A, dtype=torch.uint8, device="cuda:0") if tiled else None
            wq4.check(L.wq4_gemm_tiled(t.handle, p(b), p(at), p(y) if flags & 2 else None, None if tiled else p(y),
                                       p(ot), m, flags, prec, 1, st))
            torch.cuda.synchronize()
            outs.append((ot if tiled else y).cpu().numpy().copy())
    finally:
        L.wq4_debug_set_enc_kernel(prev)
    ref = outs[0]
    for mode, o in zip(modes[1:], outs[1:]):
        if tiled:
            assert np.array_equal(o, ref), f"A-tiled output differs in mode {mode}"
        else:
            assert np.array_equal(o.view(np.uint32), ref.view(np.uint32)), \
                f"mode {mode}: {np.count_nonzero(o != ref)} of {o.size} outputs differ, max |d| {np.max(np.abs(o - ref))}"
