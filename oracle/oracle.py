"""CPU oracle for the Q4_0 dequant+GEMM path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker.  The product (whisper-burn_amd/ and its
libwq4.so) never imports, links or calls anything under oracle/.

Two layers:
  * ctypes bindings to oracle/q4_oracle.c (the loop-order-faithful C
    restatement; see that file for the reference file:line of each function);
  * numpy restatements of the same functions, vectorised, for sizes where the
    scalar C loops would be too slow (and to cross-check the C code).

Parity pinning: see q4_oracle.c header and tests/test_oracle.py.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libq4oracle.so")
_lib = None

Q4_BLOCK = 32
Q4_BYTES = 18


def build() -> str:
    """Compile q4_oracle.c with oracle/Makefile (gcc, no GPU needed)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        f32p = ctypes.POINTER(ctypes.c_float)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        i64 = ctypes.c_int64
        L.q4o_f16_to_f32.argtypes = [ctypes.c_uint16]
        L.q4o_f16_to_f32.restype = ctypes.c_float
        L.q4o_f32_to_f16.argtypes = [ctypes.c_float]
        L.q4o_f32_to_f16.restype = ctypes.c_uint16
        L.q4o_quantize_test.argtypes = [f32p, i64, u8p]
        L.q4o_quantize_convert.argtypes = [f32p, i64, u8p]
        L.q4o_dequantize.argtypes = [u8p, i64, f32p]
        L.q4o_reference_matmul.argtypes = [f32p, f32p, i64, i64, i64, f32p]
        L.q4o_shader_matmul.argtypes = [u8p, f32p, i64, i64, i64, i64, f32p]
        L.q4o_linear.argtypes = [u8p, f32p, f32p, i64, i64, i64, i64, f32p]
        L.q4o_gelu1.argtypes = [ctypes.c_float]
        L.q4o_gelu1.restype = ctypes.c_float
        L.q4o_gelu.argtypes = [f32p, i64]
        L.q4o_ffn.argtypes = [u8p, f32p, u8p, f32p, f32p, i64, i64, i64, i64, f32p, f32p]
        L.q4o_cpu_dequant_gemm.argtypes = [u8p, f32p, i64, i64, i64, f32p, f32p]
        L.q4o_closed_form.argtypes = [ctypes.c_int, i64, f32p]
        L.q4o_cpu_linear.argtypes = [u8p, f32p, f32p, i64, i64, i64, f32p, f32p, ctypes.c_int]
        L.q4o_cpu_ffn.argtypes = [u8p, f32p, u8p, f32p, f32p, i64, i64, i64, f32p, f32p, f32p, ctypes.c_int]
        _lib = L
    return _lib


def _f32p(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _u8p(a: np.ndarray):
    assert a.dtype == np.uint8 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


# ---------------------------------------------------------------- C oracle --
def closed_form(kind: int, n: int) -> np.ndarray:
    """Reference test inputs (src/gguf/tests.rs; see q4_oracle.c)."""
    out = np.empty(n, np.float32)
    lib().q4o_closed_form(kind, n, _f32p(out))
    return out


def quantize_test(x: np.ndarray) -> np.ndarray:
    """src/gguf/tests.rs:24-57 quantizer (C restatement)."""
    x = np.ascontiguousarray(x, np.float32).ravel()
    assert x.size % Q4_BLOCK == 0
    out = np.empty(x.size // Q4_BLOCK * Q4_BYTES, np.uint8)
    lib().q4o_quantize_test(_f32p(x), x.size, _u8p(out))
    return out


def quantize_convert_c(x: np.ndarray) -> np.ndarray:
    """scripts/convert_whisper.py:33-74 quantizer (C restatement)."""
    x = np.ascontiguousarray(x, np.float32).ravel()
    assert x.size % Q4_BLOCK == 0
    out = np.empty(x.size // Q4_BLOCK * Q4_BYTES, np.uint8)
    lib().q4o_quantize_convert(_f32p(x), x.size, _u8p(out))
    return out


def dequantize_c(q4: np.ndarray, n: int) -> np.ndarray:
    """src/gguf/tests.rs:60-87 (C restatement)."""
    q4 = np.ascontiguousarray(q4, np.uint8)
    out = np.empty(n, np.float32)
    lib().q4o_dequantize(_u8p(q4), n, _f32p(out))
    return out


def reference_matmul(a: np.ndarray, bt: np.ndarray, m: int, k: int, n: int) -> np.ndarray:
    """src/gguf/tests.rs:172-184 naive i-j-l f32 loop (C restatement)."""
    a = np.ascontiguousarray(a, np.float32)
    bt = np.ascontiguousarray(bt, np.float32)
    out = np.empty(m * n, np.float32)
    lib().q4o_reference_matmul(_f32p(a), _f32p(bt), m, k, n, _f32p(out))
    return out.reshape(m, n)


def shader_matmul(q4: np.ndarray, x: np.ndarray, B: int, M: int, K: int, N: int) -> np.ndarray:
    """src/gguf/shader.wgsl:51-92 arithmetic, per output, in shader order."""
    q4 = np.ascontiguousarray(q4, np.uint8)
    x = np.ascontiguousarray(x, np.float32)
    out = np.empty(B * M * N, np.float32)
    lib().q4o_shader_matmul(_u8p(q4), _f32p(x), B, M, K, N, _f32p(out))
    return out.reshape(B, M, N)


def linear(q4, bias, x, B, M, K, N) -> np.ndarray:
    """src/gguf/linear.rs:34-40."""
    q4 = np.ascontiguousarray(q4, np.uint8)
    x = np.ascontiguousarray(x, np.float32)
    out = np.empty(B * M * N, np.float32)
    bp = None if bias is None else _f32p(np.ascontiguousarray(bias, np.float32))
    lib().q4o_linear(_u8p(q4), bp, _f32p(x), B, M, K, N, _f32p(out))
    return out.reshape(B, M, N)


def gelu_c(x: np.ndarray) -> np.ndarray:
    """src/model/layers.rs:35-41."""
    y = np.array(x, np.float32, copy=True).ravel()
    lib().q4o_gelu(_f32p(y), y.size)
    return y.reshape(np.shape(x))


def ffn(fc1, b1, fc2, b2, x, B, M, D, F) -> np.ndarray:
    """src/model/layers.rs:54-58."""
    x = np.ascontiguousarray(x, np.float32)
    h = np.empty(B * M * F, np.float32)
    out = np.empty(B * M * D, np.float32)
    L = lib()
    b1p = None if b1 is None else _f32p(np.ascontiguousarray(b1, np.float32))
    b2p = None if b2 is None else _f32p(np.ascontiguousarray(b2, np.float32))
    L.q4o_ffn(_u8p(np.ascontiguousarray(fc1, np.uint8)), b1p, _u8p(np.ascontiguousarray(fc2, np.uint8)), b2p,
              _f32p(x), B, M, D, F, _f32p(h), _f32p(out))
    return out.reshape(B, M, D)


def cpu_dequant_gemm(q4: np.ndarray, x: np.ndarray, M: int, K: int, N: int) -> np.ndarray:
    """The timed CPU baseline: dequantize (tests.rs:60-87) + naive matmul (:172-184)."""
    deq = np.empty(N * K, np.float32)
    out = np.empty(M * N, np.float32)
    lib().q4o_cpu_dequant_gemm(_u8p(np.ascontiguousarray(q4, np.uint8)), _f32p(np.ascontiguousarray(x, np.float32)),
                               M, K, N, _f32p(deq), _f32p(out))
    return out.reshape(M, N)


def cpu_linear(q4, bias, x, M: int, K: int, N: int, nthreads: int = 1) -> np.ndarray:
    """SURVEY §8(d) CPU baseline: Q4Linear on the reference's CPU path
    (dequantize tests.rs:60-87 + naive matmul :172-184 + bias linear.rs:37-39);
    nthreads > 1 = OpenMP over the outputs (same bits)."""
    deq = np.empty(N * K, np.float32)
    out = np.empty(M * N, np.float32)
    bp = None if bias is None else _f32p(np.ascontiguousarray(bias, np.float32))
    lib().q4o_cpu_linear(_u8p(np.ascontiguousarray(q4, np.uint8)), bp, _f32p(np.ascontiguousarray(x, np.float32)),
                         M, K, N, _f32p(deq), _f32p(out), int(nthreads))
    return out.reshape(M, N)


def cpu_ffn(fc1, b1, fc2, b2, x, M: int, D: int, F: int, nthreads: int = 1) -> np.ndarray:
    """SURVEY §8(d) CPU baseline: Q4FFN (layers.rs:54-58) on the CPU path."""
    deq = np.empty(F * D, np.float32)
    h = np.empty(M * F, np.float32)
    out = np.empty(M * D, np.float32)
    lib().q4o_cpu_ffn(_u8p(np.ascontiguousarray(fc1, np.uint8)), _f32p(np.ascontiguousarray(b1, np.float32)),
                      _u8p(np.ascontiguousarray(fc2, np.uint8)), _f32p(np.ascontiguousarray(b2, np.float32)),
                      _f32p(np.ascontiguousarray(x, np.float32)), M, D, F, _f32p(deq), _f32p(h), _f32p(out),
                      int(nthreads))
    return out.reshape(M, D)


# ------------------------------------------------------------ numpy oracle --
def quantize_convert_np(x: np.ndarray) -> np.ndarray:
    """Vectorised scripts/convert_whisper.py:33-74 under numpy 2 semantics.

    Same arithmetic as the reference loop: amax float32 (:51), d = amax / 7.0
    float32 (:52), scale np.float16(d) (:55), np.round(block / d) half-even in
    float32 (:60), nibble (q + 8) & 0xF, low = elements 0..15 (:65-69).
    """
    flat = np.ascontiguousarray(x, np.float32).reshape(-1, Q4_BLOCK)
    amax = np.max(np.abs(flat), axis=1)
    d = np.where(amax > 0, amax / np.float32(7.0), np.float32(0.0)).astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        q = np.where(d[:, None] > 0, np.round(flat / d[:, None]), 0).astype(np.int8).astype(np.int32)
    nib = (q + 8) & 0x0F
    packed = (nib[:, :16] | (nib[:, 16:] << 4)).astype(np.uint8)
    out = np.empty((flat.shape[0], Q4_BYTES), np.uint8)
    out[:, :2] = d.astype(np.float16).view(np.uint8).reshape(-1, 2)
    out[:, 2:] = packed
    return out.ravel()


def dequantize_np(q4: np.ndarray, n: int) -> np.ndarray:
    """Vectorised src/gguf/tests.rs:60-87."""
    blk = np.ascontiguousarray(q4, np.uint8).reshape(-1, Q4_BYTES)
    assert blk.shape[0] * Q4_BLOCK == n
    d = blk[:, :2].copy().view(np.float16).astype(np.float32)  # [nb, 1]
    lo = (blk[:, 2:] & 0x0F).astype(np.float32) - np.float32(8.0)
    hi = ((blk[:, 2:] >> 4) & 0x0F).astype(np.float32) - np.float32(8.0)
    out = np.concatenate([lo * d, hi * d], axis=1)
    return out.astype(np.float32).ravel()


def gelu_np(x: np.ndarray) -> np.ndarray:
    """src/model/layers.rs:35-41 in float32."""
    x = np.asarray(x, np.float32)
    s = np.float32(0.7978845608028654)
    x3 = x * x * x
    inner = (x + x3 * np.float32(0.044715)) * s
    return (x * np.float32(0.5) * (np.tanh(inner) + np.float32(1.0))).astype(np.float32)


def matmul_f64(x: np.ndarray, w_deq: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """Exact-ish ground truth for tolerance checks: x @ W^T in float64, plus
    the per-output magnitude sum(|x|*|w|) that scales any f32 rounding error."""
    x64 = np.asarray(x, np.float64)
    w64 = np.asarray(w_deq, np.float64)
    return x64 @ w64.T, np.abs(x64) @ np.abs(w64).T


# --------------------------------------------------- synthetic data (spec) --
# The bench/test inputs are synthetic (no Whisper weights exist offline).
# This is the numpy statement of the generator; the product's C++ generator
# (whisper-burn_amd/csrc/wq4_synth.cpp) must match it bit for bit, which
# tests/test_synth.py checks.
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for ch in s.encode():
        h ^= ch
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def synth_uniform(seed: int, name: str, n: int, lo: float, hi: float) -> np.ndarray:
    """u_i = top 24 bits of splitmix64(key + i) -> lo + (hi-lo) * u_i / 2^24, f32.

    Every step is exact or a single IEEE f32 rounding, so C++ and numpy agree.
    """
    key = np.uint64((seed ^ fnv1a64(name)) & 0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        idx = np.arange(n, dtype=np.uint64) + key
    u = (splitmix64(idx) >> np.uint64(40)).astype(np.float32)  # exact: < 2^24
    unit = u * np.float32(1.0 / 16777216.0)  # exact
    lo32, hi32 = np.float32(lo), np.float32(hi)
    span = np.float32(np.float64(hi32) - np.float64(lo32))
    t = (unit * span).astype(np.float32)
    return (lo32 + t).astype(np.float32)


def lin_scale(k: int) -> np.float32:
    """Uniform half-width of a synthetic linear weight with fan-in k."""
    import math

    return np.float32(1.5 / math.sqrt(k))
