"""GGUF reader / writer (src/gguf/reader.rs, scripts/convert_whisper.py) on CPU.

Pinned by tests/golden/ref_writer_tiny.gguf, written with the reference's own
GGUF helpers and quantizer (tests/golden/make_gguf_golden.py)."""
import hashlib
import json
import os
import struct
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, os.path.join(REPO, "whisper-burn_amd"))
sys.path.insert(0, os.path.join(REPO, "whisper-burn_amd", "tools"))


def golden_inputs() -> dict:
    """Same function as tests/golden/make_gguf_golden.py:golden_inputs."""
    rng = np.random.default_rng(20260301)
    f = lambda *s: (rng.standard_normal(s) * 0.05).astype(np.float32)  # noqa: E731
    return {
        "encoder.blocks.0.attn.query.weight": f(256, 256),
        "encoder.blocks.0.attn.query.bias": f(256),
        "encoder.blocks.0.attn_ln.weight": f(256),
        "encoder.conv1.weight": f(8, 4, 3),
        "encoder.positional_embedding": f(6, 256),
        "decoder.blocks.0.mlp.0.weight": f(512, 256),
        "decoder.blocks.0.mlp.0.bias": f(512),
        "decoder.token_embedding.weight": f(40, 256),
    }


@pytest.fixture(scope="module")
def wa():
    import whisper_amd

    return whisper_amd


@pytest.fixture(scope="module")
def golden():
    with open(os.path.join(GOLD, "ref_writer_tiny.json")) as f:
        return json.load(f)


def test_reader_parses_reference_written_file(wa, golden):
    r = wa.GgufReader(os.path.join(GOLD, "ref_writer_tiny.gguf"))
    assert r.version == golden["version"] == 3
    got = r.tensors()
    assert [t["name"] for t in got] == [t["name"] for t in golden["tensors"]]
    for g, e in zip(got, golden["tensors"]):
        assert g["dims"] == e["dims"] and g["type"] == e["dtype"] and g["offset"] == e["offset"]
        assert g["nbytes"] == e["nbytes"]
        assert hashlib.sha256(r.tensor_data(g["name"]).tobytes()).hexdigest() == e["sha256"]


def test_reader_data_values(wa):
    r = wa.GgufReader(os.path.join(GOLD, "ref_writer_tiny.gguf"))
    inp = golden_inputs()
    b = r.tensor_data("encoder.blocks.0.attn.query.bias").view(np.float32)
    assert np.array_equal(b, inp["encoder.blocks.0.attn.query.bias"])
    conv = r.tensor_data("encoder.conv1.weight").view(np.float32)
    assert np.array_equal(conv, inp["encoder.conv1.weight"].ravel())  # [out][in][k], dims [3, 4, 8]


def test_writer_reproduces_reference_bytes(tmp_path):
    import write_gguf

    out = tmp_path / "w.gguf"
    write_gguf.write_gguf(str(out), golden_inputs(), "ref-helpers-golden")
    assert out.read_bytes() == open(os.path.join(GOLD, "ref_writer_tiny.gguf"), "rb").read()


def _header(version=3, n_t=0, n_kv=0):
    return struct.pack("<IIQQ", 0x46554747, version, n_t, n_kv)


@pytest.mark.parametrize("blob,msg", [
    (b"GGML" + b"\x00" * 40, "Invalid GGUF magic"),
    (_header(version=4) + b"\x00" * 8, "Unsupported GGUF version"),
    (_header(n_kv=1) + struct.pack("<Q", 3) + b"abc" + struct.pack("<I", 13) + b"\x00" * 16, "metadata"),
    (_header(n_t=1) + struct.pack("<Q", 1) + b"t" + struct.pack("<I", 1) + struct.pack("<Q", 32)
     + struct.pack("<IQ", 8, 0) + b"\x00" * 32, "Unsupported GGML dtype code: 8"),
    (_header(n_t=1) + struct.pack("<Q", 1) + b"t", "Failed to read ndims for tensor 0"),
])
def test_reader_errors(wa, tmp_path, blob, msg):
    p = tmp_path / "bad.gguf"
    p.write_bytes(blob)
    with pytest.raises(Exception) as ei:
        wa.GgufReader(str(p))
    assert msg in str(ei.value)


def test_reader_v2_and_metadata_skipping(wa, tmp_path):
    """Every metadata value type of reader.rs:236-283 (arrays nested) is skipped."""
    kv = b""
    kv += struct.pack("<Q", 1) + b"a" + struct.pack("<I", 0) + b"\x01"
    kv += struct.pack("<Q", 1) + b"b" + struct.pack("<I", 3) + b"\x02\x00"
    kv += struct.pack("<Q", 1) + b"c" + struct.pack("<I", 6) + struct.pack("<f", 1.5)
    kv += struct.pack("<Q", 1) + b"d" + struct.pack("<I", 8) + struct.pack("<Q", 2) + b"hi"
    kv += (struct.pack("<Q", 1) + b"e" + struct.pack("<I", 9) + struct.pack("<IQ", 9, 2)
           + struct.pack("<IQ", 4, 1) + struct.pack("<I", 7) + struct.pack("<IQ", 12, 1) + struct.pack("<d", 2.0))
    kv += struct.pack("<Q", 1) + b"f" + struct.pack("<I", 11) + struct.pack("<q", -3)
    idx = struct.pack("<Q", 1) + b"w" + struct.pack("<I", 1) + struct.pack("<Q", 4) + struct.pack("<IQ", 0, 0)
    head = _header(version=2, n_t=1, n_kv=6) + kv + idx
    pad = (-len(head)) % 32
    p = tmp_path / "v2.gguf"
    p.write_bytes(head + b"\x00" * pad + np.arange(4, dtype=np.float32).tobytes())
    r = wa.GgufReader(str(p))
    assert r.version == 2
    assert r.tensors()[0]["dims"] == [4]
    assert np.array_equal(r.tensor_data("w").view(np.float32), np.arange(4, dtype=np.float32))


def test_synthetic_gguf_layout(wa, tmp_path):
    """tools/write_gguf.py's synthetic checkpoint: Q4_0 linear weights, F32
    rest, the names load_whisper_from_gguf asks for (loader.rs:279-377)."""
    import write_gguf

    tensors = {n: np.zeros(s, np.float32) for n, s, _, _ in write_gguf.synthetic_specs("tiny_test")}
    p = tmp_path / "s.gguf"
    write_gguf.write_gguf(str(p), tensors, "layout")
    ts = {t["name"]: t for t in wa.GgufReader(str(p)).tensors()}
    assert ts["encoder.blocks.1.mlp.0.weight"]["type"] == 2 and ts["encoder.blocks.1.mlp.0.weight"]["dims"] == [384, 1536]
    assert ts["decoder.blocks.0.cross_attn.key.weight"]["type"] == 2
    assert "decoder.blocks.0.cross_attn.key.bias" not in ts and "encoder.blocks.0.attn.key.bias" not in ts
    assert ts["encoder.conv1.weight"]["dims"] == [3, 80, 384] and ts["encoder.conv1.weight"]["type"] == 0
    assert ts["decoder.token_embedding.weight"]["type"] == 0
