"""C-ABI library tests that need no GPU: load, exports, host logic, errors.

No compute call is made here (there is no GPU in the build container); the
shape / byte-count validation of Q4Tensor::from_q4_bytes (tensor.rs:38-48)
runs before any device work, so its error behaviour is testable on the CPU.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest

import oracle
import wq4


def test_library_loads_and_reports_abi():
    L = wq4.lib()
    assert L.wq4_abi_version() == 1


def test_every_header_function_is_exported():
    L = wq4.lib()
    names = wq4.header_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_no_oracle_symbols_in_product():
    import subprocess

    out = subprocess.run(["nm", "-D", "--defined-only", wq4.LIB_PATH], capture_output=True, text=True).stdout
    assert "q4o_" not in out  # the product never contains the checker


@pytest.mark.parametrize("n,k", [(1, 32), (32, 32), (64, 128), (96, 64), (1280, 1280), (33, 96), (5120, 160)])
def test_repack_roundtrip_lossless(n, k):
    rng = np.random.default_rng(n * 7 + k)
    raw = rng.integers(0, 256, n * k // 32 * 18, dtype=np.uint8)
    raw.reshape(-1, 18)[:, 1] &= 0x3F  # finite f16 scales of mixed magnitude (NaN/inf rows are tested below)
    nib, sc, cs = wq4.debug_repack(raw, n, k)
    assert nib.size == ((n + 63) // 64 * 2) * ((k // 32 + 1) // 2) * 1024
    back = wq4.debug_unrepack(nib, sc, cs, n, k)
    assert np.array_equal(back, raw)
    # same information content: 4.5 bits per weight + padding only
    assert nib.size + sc.size * 4 >= raw.size


def test_repack_layout_spec():
    """Spot-check wq4_layout.hpp: lane (r, h) of (n-tile, block pair) holds the
    kk=0/1 nibble words of bytes 8h..8h+7 of row 32*nt + r, blocks 2bp, 2bp+1."""
    n, k = 64, 128
    w = oracle.closed_form(1, n * k)
    raw = oracle.quantize_convert_np(w)
    nib, sc, cs = wq4.debug_repack(raw, n, k)
    nbp = 2
    words = nib.view(np.uint32).reshape(2, nbp, 64, 4)
    blocks = raw.reshape(n, k // 32, 18)
    for nt in range(2):
        for bp in range(nbp):
            for lane in (0, 5, 31, 32, 63):
                r, h = lane & 31, lane >> 5
                for bi in range(2):
                    blk = blocks[32 * nt + r, 2 * bp + bi]
                    by = blk[2 + 8 * h: 10 + 8 * h]
                    for kk in range(2):
                        q = [(b >> 4) if kk else (b & 15) for b in by]
                        want = sum(int(q[2 * i]) << (4 * i) | int(q[2 * i + 1]) << (16 + 4 * i) for i in range(4))
                        assert words[nt, bp, lane, bi * 2 + kk] == want
                    d = np.array([int(blk[0]) | int(blk[1]) << 8], np.uint16).view(np.float16)[0]
                    ds = np.array([(int(sc.reshape(2, nbp, 32)[nt, bp, r]) >> (16 * bi)) & 0xFFFF],
                                  np.uint16).view(np.float16)[0]
                    # d' = d * 2^s exactly, colscale = 2^-s, 8 * max d' <= 2^15
                    assert float(ds) * float(cs[32 * nt + r]) == float(d)
                    assert abs(float(ds)) <= 4096.0


def test_repack_extreme_scales_lossless():
    """Rows whose scales span > 2^26 (or hold inf/NaN/subnormal) keep s = 0."""
    n, k = 64, 256
    rng = np.random.default_rng(4)
    raw = rng.integers(0, 256, n * k // 32 * 18, dtype=np.uint8).reshape(n, k // 32, 18)
    def put(row, blk, val):
        raw[row, blk, :2] = np.array([val], np.float16).view(np.uint8)
    put(0, 0, 60000.0); put(0, 1, 6e-8)          # ratio 1e12
    put(1, 0, np.inf); put(2, 3, np.nan); put(3, 2, 0.0)
    for b in range(8):
        put(4, b, 3e-7)                            # all-subnormal row
    raw = raw.ravel()
    nib, sc, cs = wq4.debug_repack(raw, n, k)
    assert cs[0] == 1.0 and cs[1] == 1.0 and cs[2] == 1.0
    assert cs[4] < 1.0  # subnormal scales are shifted up into the normal range
    assert np.array_equal(wq4.debug_unrepack(nib, sc, cs, n, k), raw)


def test_deq8_arithmetic_is_exact():
    """The kernel's nibble -> f16 (q - 8) trick, in numpy f16: exact for all q."""
    q = np.arange(16, dtype=np.uint16)
    lo = (np.uint16(0x6400) | q).view(np.float16)
    hi = (np.uint16(0x6400) | (q << 4)).view(np.float16)
    a = (lo - np.float16(1032)).astype(np.float32)
    b = (hi * np.float16(0.0625) - np.float16(72)).astype(np.float32)
    assert np.array_equal(a, q.astype(np.float32) - 8) and np.array_equal(b, q.astype(np.float32) - 8)


def _create(raw, n, k):
    h = ctypes.c_void_p(None)
    st = wq4.lib().wq4_tensor_create(0, raw.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), raw.size, n, k,
                                     ctypes.byref(h))
    return st, wq4.lib().wq4_last_error().decode()


def test_create_rejects_bad_element_count():
    """tensor.rs:38-42 message."""
    raw = np.zeros(18, np.uint8)
    st, msg = _create(raw, 3, 5)
    assert st == 2 and "divisible by 32, got 15" in msg


def test_create_rejects_bad_byte_count():
    """tensor.rs:43-48 message."""
    raw = np.zeros(17, np.uint8)
    st, msg = _create(raw, 1, 32)
    assert st == 3 and "expected 18 for 1 blocks, got 17" in msg


def test_precision_and_policy_setters():
    wq4.set_precision(wq4.PREC_F16)
    assert wq4.get_precision() == wq4.PREC_F16
    wq4.set_precision(wq4.PREC_F16X2)
    with pytest.raises(wq4.WQ4Error):
        wq4.set_precision(7)
    with pytest.raises(wq4.WQ4Error):
        wq4.set_kernel_policy(9)
    wq4.set_kernel_policy(0)


def test_gemm_kernel_name_follows_rows():
    """wq4_gemm_kernel_name (bench.py's roofline label): the decode-step kernel
    at <= 32 rows, the 8-wave decode kernel to 128, the encoder ring kernel at
    one clip (M = 1500: the tile kernel's grid would leave CUs idle) and up
    to a wide grid of 170 workgroups, the 8-wave wide kernel from there (M =
    12000 at N = 1280: 235 workgroups; 32 clips, M = 48000); the prefill tile
    kernel under kernel policy 1 (and for operands the others do not take)."""
    assert wq4.gemm_kernel_name(1280, 1280, 16) == "skinny_gemm_kernel"
    assert wq4.gemm_kernel_name(1280, 1280, 100) == "q4_gemm_decode_kernel"
    assert wq4.gemm_kernel_name(1280, 1280, 1500) == "q4_gemm_enc_kernel"
    assert wq4.gemm_kernel_name(5120, 1280, 1500) == "q4_gemm_enc_kernel"
    assert wq4.gemm_kernel_name(1280, 1280, 48000) == "q4_gemm_wide_kernel"
    assert wq4.gemm_kernel_name(5120, 1280, 12000) == "q4_gemm_wide_kernel"
    assert wq4.gemm_kernel_name(1280, 1280, 12000) == "q4_gemm_wide_kernel"
    assert wq4.gemm_kernel_name(1280, 1280, 6000) == "q4_gemm_enc_kernel"
    assert wq4.gemm_kernel_name(1280, 1281, 16) == ""
    wq4.set_kernel_policy(1)
    try:
        assert wq4.gemm_kernel_name(1280, 1280, 16) == "q4_gemm_prefill_kernel"
    finally:
        wq4.set_kernel_policy(0)


def test_every_whisper_header_function_is_exported():
    import re

    import whisper_amd

    text = re.sub(r"/\*.*?\*/", "", open(whisper_amd.HEADER_PATH).read(), flags=re.S)
    names = sorted(set(re.findall(r"\b(wa_[a-z0-9_]+)\s*\(", text)))
    assert len(names) >= 20
    L = whisper_amd.lib()
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_decode_group_rows():
    """wa_decode_group_rows: the clips of the largest decode group (the row
    count of every captured decode-step launch and of bench.py's probe): one
    group below 16 clips, two from 16 on (wa_model.cpp decode_groups)."""
    import whisper_amd

    assert whisper_amd.decode_group_rows(0) == 0
    for n in range(1, 65):
        want = n if n < 16 else (n + 1) // 2
        assert whisper_amd.decode_group_rows(n) == want, n


@pytest.mark.parametrize("heads,d_model", [(20, 1280), (16, 1024)])
def test_bench_in_graph_lookup(tmp_path, monkeypatch, heads, d_model):
    """bench.in_graph_xattn sums the three cross-attention kernels at the
    group's grids from profiles/xattn_in_graph.json, only for the same
    workload; grids follow the head count and width (Large-V3 H = 20,
    Medium H = 16)."""
    import json
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    wl = {"variant": "large_v3", "weights": "q4_0", "precision": "f16x2", "clips": 32}
    (tmp_path / "profiles").mkdir()
    rows = [{"kernel": "xattn_q_mfma_kernel", "grid": [heads * 128, d_model // 64, 1], "avg_us": 5.5},
            {"kernel": "xattn_main_kernel", "grid": [4096, 16, 1], "avg_us": 38.0},
            {"kernel": "xattn_main_kernel", "grid": [4096, 32, 1], "avg_us": 48.0},
            {"kernel": "xattn_out_kernel", "grid": [heads * 512, 4, 1], "avg_us": 12.5}]
    (tmp_path / "profiles" / "xattn_in_graph.json").write_text(json.dumps({"workload": wl, "kernels": rows}))
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    assert bench.in_graph_xattn(16, heads, d_model, wl) == 5.5 + 38.0 + 12.5
    assert bench.in_graph_xattn(16, heads, d_model, dict(wl, clips=16)) is None
    assert bench.in_graph_xattn(8, heads, d_model, wl) is None  # no trace at that grid
    other = (16, 1024) if heads == 20 else (20, 1280)
    assert bench.in_graph_xattn(16, other[0], other[1], wl) is None  # another model's grids
