"""Generate tests/golden/ref_writer_tiny.gguf (+ .json) with the REFERENCE's
own GGUF helpers.

Run in the build container only (it reads /root/reference):

    python tests/golden/make_gguf_golden.py

Imports /root/reference/scripts/convert_whisper.py by path and uses its
constants and helpers -- quantize_q4_0, should_quantize, write_gguf_string,
write_gguf_metadata_kv, align_offset -- to lay out a small Whisper-named
tensor map following the steps of convert_model (convert_whisper.py:138-214;
convert_model itself loads a HuggingFace model by name and is never called).
The fixture is data: the file's bytes plus, per tensor, the expected index
entry and a SHA-256 of its data.  The inputs are regenerated from a fixed
numpy seed (tests/test_gguf.py:golden_inputs) so they need not be stored.
"""
from __future__ import annotations

import hashlib
import importlib.util
import io
import json
import os
import struct

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SCRIPT = "/root/reference/scripts/convert_whisper.py"


def golden_inputs() -> dict[str, np.ndarray]:
    """Same function as tests/test_gguf.py:golden_inputs (kept in sync)."""
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


def main() -> None:
    spec = importlib.util.spec_from_file_location("ref_convert_whisper", REF_SCRIPT)
    ref = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref)
    tensor_map = golden_inputs()
    entries, blobs, cur = [], [], 0
    for name, array in sorted(tensor_map.items()):
        if ref.should_quantize(name, array.shape):
            data, dtype = ref.quantize_q4_0(array), ref.GGML_TYPE_Q4_0
        else:
            data, dtype = array.astype(np.float32).tobytes(), ref.GGML_TYPE_F32
        aligned = ref.align_offset(cur)
        entries.append({"name": name, "dims": list(reversed(array.shape)), "dtype": dtype, "offset": aligned})
        blobs.append((aligned - cur, data))
        cur = aligned + len(data)
    metadata = {
        "general.architecture": ("whisper", 8),
        "general.name": ("ref-helpers-golden", 8),
        "whisper.encoder.layer_count": (len([n for n in tensor_map if n.startswith("encoder.blocks.")]) // 8, 4),
        "whisper.decoder.layer_count": (len([n for n in tensor_map if n.startswith("decoder.blocks.")]) // 16, 4),
    }
    f = io.BytesIO()
    f.write(struct.pack("<I", ref.GGUF_MAGIC))
    f.write(struct.pack("<I", ref.GGUF_VERSION))
    f.write(struct.pack("<Q", len(entries)))
    f.write(struct.pack("<Q", len(metadata)))
    for key, (value, vtype) in metadata.items():
        ref.write_gguf_metadata_kv(f, key, vtype, value)
    for e in entries:
        ref.write_gguf_string(f, e["name"])
        f.write(struct.pack("<I", len(e["dims"])))
        for d in e["dims"]:
            f.write(struct.pack("<Q", d))
        f.write(struct.pack("<I", e["dtype"]))
        f.write(struct.pack("<Q", e["offset"]))
    pos = f.tell()
    data_start = ref.align_offset(pos)
    f.write(b"\x00" * (data_start - pos))
    for pad, data in blobs:
        f.write(b"\x00" * pad)
        f.write(data)
    raw = f.getvalue()
    with open(os.path.join(HERE, "ref_writer_tiny.gguf"), "wb") as out:
        out.write(raw)
    for e, (_, data) in zip(entries, blobs):
        e["nbytes"] = len(data)
        e["sha256"] = hashlib.sha256(data).hexdigest()
    with open(os.path.join(HERE, "ref_writer_tiny.json"), "w") as out:
        json.dump({"version": ref.GGUF_VERSION, "data_section_offset": data_start, "file_bytes": len(raw),
                   "sha256": hashlib.sha256(raw).hexdigest(), "model_name": "ref-helpers-golden",
                   "tensors": entries}, out, indent=1)
    print(f"wrote {len(raw)} bytes, {len(entries)} tensors")


if __name__ == "__main__":
    main()
