"""CPU tests: the product's synthetic-weight generator and quantizer are bit-identical
to the oracle's (numpy) statement, so the GPU model and the numpy model run on
exactly the same weights."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

import oracle
import whisper_amd
import wq4


@pytest.mark.parametrize("name,n,lo,hi", [
    ("encoder.blocks.0.attn.query.weight", 4096, -float(oracle.lin_scale(1280)), float(oracle.lin_scale(1280))),
    ("decoder.blocks.3.mlp_ln.weight", 1280, 0.9, 1.1),
    ("mel", 80 * 3000, -1.5, 1.0),
    ("decoder.positional_embedding", 448 * 384, -0.02, 0.02),
])
@pytest.mark.parametrize("seed", [1234, 0x5EED0000 + 7])
def test_cpp_generator_matches_numpy(name, n, lo, hi, seed):
    a = whisper_amd.synth_uniform(seed, name, n, lo, hi)
    b = oracle.synth_uniform(seed, name, n, lo, hi)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_product_quantizer_matches_reference_golden(golden):
    L = wq4.lib()
    L.wq4_quantize_q4_0.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    L.wq4_quantize_q4_0.restype = ctypes.c_int
    for key in golden.files:
        if not key.startswith("in/"):
            continue
        x = np.ascontiguousarray(golden[key], np.float32)
        out = np.zeros(x.size // 32 * 18, np.uint8)
        assert L.wq4_quantize_q4_0(x.ctypes.data, x.size, out.ctypes.data) == 0
        assert np.array_equal(out, golden["q4/" + key[3:]]), key


def test_product_quantizer_matches_numpy_on_synthetic_weights():
    L = wq4.lib()
    L.wq4_quantize_q4_0.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    a = float(oracle.lin_scale(5120))
    x = oracle.synth_uniform(99, "encoder.blocks.1.mlp.2.weight", 1280 * 5120 // 8, -a, a)
    out = np.zeros(x.size // 32 * 18, np.uint8)
    assert L.wq4_quantize_q4_0(x.ctypes.data, x.size, out.ctypes.data) == 0
    assert np.array_equal(out, oracle.quantize_convert_np(x))
